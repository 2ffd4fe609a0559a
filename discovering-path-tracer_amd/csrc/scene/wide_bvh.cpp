// Wide BVH builder and the cull bound of the culled walk (wide_bvh.h,
// csrc/wide_walk.h).
#include "wide_bvh.h"

#include <math.h>
#include <string.h>

#include <algorithm>
#include <system_error>
#include <thread>

namespace pt {

namespace {

constexpr int32_t kEmpty = (int32_t)0x80000000;   // wide_walk.h kWideEmpty
constexpr double kMaxCoord = 1e15;                 // wide_walk.h kWideMaxCoord
constexpr double kU = 0x1p-24;                      // unit roundoff of fp32
double gam(int k) { return k * kU / (1.0 - k * kU); }

float up_f(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, INFINITY);
  return f;
}
float down_f(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -INFINITY);
  return f;
}

// bf16 bits of x >= 0 rounded up (toward +inf)
uint32_t bf16_up(float x) {
  uint32_t b;
  memcpy(&b, &x, 4);
  return (b >> 16) + ((b & 0xffffu) ? 1u : 0u);
}

// One 64-B node (wide_walk.h kWideQNodeF4) from a 32-float node: per axis a
// grid origin p (the children's least lo) and step s = 2^e (the smallest
// with fl(p + 255 s) >= the largest hi); each child's lo rounded down and hi
// rounded up onto the grid, checked with the device's own decode
// fmaf(q, s, p) (q s is exact, so this is fl(p + q s) on both sides).
// Returns false if some box cannot be enclosed (it always can: the caller
// reports it as a builder error).
bool quantize_node(const float* rec, float* q) {
  int32_t refs[4];
  memcpy(refs, rec + 24, sizeof refs);
  uint32_t packed[6] = {0, 0, 0, 0, 0, 0};   // qlo.x qhi.x qlo.y qhi.y qlo.z qhi.z
  uint32_t meta = 0;
  for (int a = 0; a < 3; ++a) {
    float pmin = INFINITY, hmax = -INFINITY;
    for (int j = 0; j < 4; ++j)
      if (refs[j] != kEmpty) {
        pmin = std::min(pmin, rec[8 * a + j]);
        hmax = std::max(hmax, rec[8 * a + 4 + j]);
      }
    if (!(pmin <= hmax)) return false;
    const float p = pmin;
    const double d = (double)hmax - (double)p;
    int e = d > 0.0 ? (int)ceil(log2(d / 255.0)) : -126;
    e = std::max(-126, std::min(127, e));
    while (e < 127 && fmaf(255.0f, ldexpf(1.0f, e), p) < hmax) ++e;
    while (e > -126 && fmaf(255.0f, ldexpf(1.0f, e - 1), p) >= hmax) --e;
    const float s = ldexpf(1.0f, e);
    if (!(fmaf(255.0f, s, p) >= hmax)) return false;
    meta |= (uint32_t)(e + 127) << (8 * a);
    q[a] = p;
    for (int j = 0; j < 4; ++j) {
      uint32_t ql = 255, qh = 0;   // empty slot: an inverted box (the walk also checks the ref)
      if (refs[j] != kEmpty) {
        const float lo = rec[8 * a + j], hi = rec[8 * a + 4 + j];
        int l = (int)std::max(0.0, std::min(255.0, floor(((double)lo - (double)p) / (double)s)));
        while (l > 0 && fmaf((float)l, s, p) > lo) --l;
        while (l < 255 && fmaf((float)(l + 1), s, p) <= lo) ++l;
        int h = (int)std::max(0.0, std::min(255.0, ceil(((double)hi - (double)p) / (double)s)));
        while (h < 255 && fmaf((float)h, s, p) < hi) ++h;
        while (h > 0 && fmaf((float)(h - 1), s, p) >= hi) --h;
        if (!(fmaf((float)l, s, p) <= lo && fmaf((float)h, s, p) >= hi)) return false;
        ql = (uint32_t)l;
        qh = (uint32_t)h;
      }
      packed[2 * a] |= ql << (8 * j);
      packed[2 * a + 1] |= qh << (8 * j);
    }
  }
  memcpy(&q[3], &meta, 4);
  memcpy(&q[4], packed, sizeof packed);
  q[10] = rec[28];   // c1 (already rounded down)
  const uint32_t e01 = bf16_up(rec[29]) | (bf16_up(rec[30]) << 16);   // E0, E1 rounded up
  memcpy(&q[11], &e01, 4);
  memcpy(&q[12], refs, sizeof refs);
  return true;
}

}  // namespace

WideCoeffs coeff_max(const WideCoeffs& a, const WideCoeffs& b) {
  return WideCoeffs{std::max(a.k1, b.k1), std::max(a.k2, b.k2), std::max(a.eps0, b.eps0), std::max(a.eps1, b.eps1)};
}

// The node's cull constants {c1, E0, E1, 0} (wide_walk.h wide_child) from the
// largest coefficients of the triangles below it: a child is culled when
// lim < th = c1 * (t_near (1 - 2^-20) - (E0 + E1 Smax) (|1/d|_max + 1)).
// Margins: the float slab's t_near is within (1+u)^3 of the exact entry;
// S <= (1 + 3u) Smax (Smax from the slab's own differences); |1/d| within 2u
// of the float reciprocal; each float op of the evaluation rounds once --
// all covered by the 2^-18 and 2^-20 factors.  The device evaluates the same
// bound with the t_near factor moved into the constants:
//   th = c1' * (t_near - (E0' + E1' Smax) (|1/d| + 1)),
//   c1' = c1 (1 - 2^-20) rounded down, E' = E / (1 - 2^-20) rounded up,
// which is c1 * (t_near (1 - 2^-20) - (E0 + E1 Smax) ...) exactly in real
// arithmetic (c1' E' = c1 E), with one float rounding fewer per axis.  A
// triangle without a bound (k1 infinite) gives c1 = 0: th = 0 culls nothing
// a hit (t > 1e-6) could need.
void node_cull_consts(const WideCoeffs& co, float* out) {
  out[3] = 0.0f;
  if (!(co.k1 <= 0.5) || !(co.eps0 < 1e30) || !(co.eps1 < 1e30) || !(co.k2 < 1e30)) {
    out[0] = out[1] = out[2] = 0.0f;
    return;
  }
  const double k = 1.0 - 0x1p-20;   // the t_near factor
  const double c1 = down_f((1.0 - co.k1) / (1.0 + gam(3)) * (1.0 - 0x1p-20));
  out[0] = (float)down_f(c1 * k);
  out[1] = up_f(co.eps0 * (1.0 + 0x1p-18) / k);
  out[2] = up_f(std::max(co.eps1, co.k2 / c1) * (1.0 + 3.0 * kU) * (1.0 + 0x1p-18) / k);
}

// Error bound of intersectTriangle (raytrace_comp.comp:114-157) as the
// kernels evaluate it (tri_test: edges e1, e2 precomputed, no contraction,
// IEEE reciprocal).  Notation: u = 2^-24, g_k = k u / (1 - k u), |x|_1 and
// |x|_inf vector norms, s = fl(o - v0), S = |s|_inf, p = fl(cross(d, e2)),
// det = fl(dot(e1, p)), q = fl(cross(s, e1)).  Let o'' = v0 + s (exact), so
// |o'' - o|_inf <= u |o - v0|_inf.  In exact arithmetic on these float
// inputs, Cramer's rule gives o'' + T d = v0 + u* e1 + v* e2 =: X with
// T = dot(e2, q*)/det*, u* = dot(s, p*)/det*, v* = dot(d, q*)/det* (starred:
// exact cross/dot).  Standard bounds (cross component g2, dot of 3 terms g3):
//   |det - det*|         <= g6 Dd,  Dd <= |d|inf D0,  D0 = sum_i |e1_i|(|e2|_1 - |e2_i|)
//   |fl(s.p) - s.p*|     <= g6 S |d|inf 2|e2|_1
//   |fl(d.q) - d.q*|     <= g6 S |d|inf 2|e1|_1
//   |fl(e2.q) - e2.q*|   <= g6 S D0
// and with the acceptance |det| >= 1e-6 (EPSILON, :127), g = g6 / 0.999e-6:
//   du = |u_b - u*| <= (2 g dm |e2|_1 S + g dm D0 + g3) / (1 - g dm D0)   (u_b in [0,1])
//   dv = |v_b - v*| <= (2 g dm |e1|_1 S + g dm D0 + g3) / (1 - g dm D0)
//   |t_b - T| <= g D0 (S + dm |T|) + g3 t_b
// (dm >= |d|_2, |d|_inf: the walk takes only rays with fl(d.d) <= 1.00002).
// X lies within rho (inf-norm) of conv(v0, v0+e1, v0+e2) -- hence of the
// triangle (|e1 - (v1 - v0)| <= u|e1|) and of any box B containing it:
//   rho = u max(|e1|inf, |e2|inf) + du |e1|inf + dv |e2|inf = rho0 + rhoS S.
// So the point o + T d lies in B grown by eps = rho + u S / (1 - u) on every
// side, and on each axis i, T >= entry_i(B) - eps / |d_i|: T is at least the
// ray's exact entry parameter into B less eps |1/d|_max.  With t_b > 1e-6
// (:153) and T > 0, t_b >= (T (1 - k1) - k2 S) / (1 + g3), k1 = g dm D0,
// k2 = g D0.  wide_walk.h evaluates the resulting threshold per child.
bool wide_tri_coeffs(const float e1f[3], const float e2f[3], WideCoeffs* out) {
  const double dm = 1.0000102;   // sqrt(1.00002 (1 + g3)) rounded up
  const double g = gam(6) / 0.999e-6;
  double n1 = 0, n2 = 0, m1 = 0, m2 = 0, D0 = 0;
  double a1[3], a2[3];
  for (int i = 0; i < 3; ++i) {
    a1[i] = fabs((double)e1f[i]);
    a2[i] = fabs((double)e2f[i]);
    n1 += a1[i];
    n2 += a2[i];
    m1 = std::max(m1, a1[i]);
    m2 = std::max(m2, a2[i]);
  }
  for (int i = 0; i < 3; ++i) D0 += a1[i] * (n2 - a2[i]);
  if (!(n1 < 1e30 && n2 < 1e30)) return false;
  const double den = 1.0 - g * dm * D0;
  if (!(den >= 0.5)) return false;
  const double alpha_u = 2.0 * g * dm * n2 / den, alpha_v = 2.0 * g * dm * n1 / den;
  const double beta = (g * dm * D0 + gam(3)) / den;
  const double rhoS = alpha_u * m1 + alpha_v * m2;
  const double rho0 = 1.01 * kU * std::max(m1, m2) + beta * (m1 + m2);
  out->k1 = g * dm * D0;
  out->k2 = g * D0;
  out->eps0 = rho0;
  out->eps1 = rhoS + kU / (1.0 - kU);
  return true;
}

namespace {

// A binary tree the wide nodes are collapsed from: the reference's own tree
// (WIDE_FROM_REFERENCE) or a binned-SAH tree over the reference's leaves
// (WIDE_SAH).  Children are stored after their parent; leaves carry the
// reference leaf node they stand for.
struct BinTree {
  std::vector<float> box;       // 6 per node: lo.xyz, hi.xyz
  std::vector<int32_t> kid;     // 2 per node: children, or {-1, reference leaf node}
  std::vector<WideCoeffs> co;   // per node: the largest coefficients over its subtree
  bool leaf(size_t v) const { return kid[2 * v] < 0; }
};

double half_area(const float* b) {
  const double dx = (double)b[3] - b[0], dy = (double)b[4] - b[1], dz = (double)b[5] - b[2];
  return dx * dy + dy * dz + dz * dx;
}

void grow(float* b, const float* c) {
  for (int a = 0; a < 3; ++a) {
    b[a] = std::min(b[a], c[a]);
    b[3 + a] = std::max(b[3 + a], c[3 + a]);
  }
}

void empty_box(float* b) {
  for (int a = 0; a < 3; ++a) {
    b[a] = INFINITY;
    b[3 + a] = -INFINITY;
  }
}

// Binned SAH over leaves [b, e) of `ids` (reference leaf nodes; their boxes in
// lbox by position), written at node `at` of T: a subtree of n leaves takes
// the 2n - 1 nodes [at, at + 2n - 1), left subtree first, so disjoint ranges
// build in parallel and the result does not depend on the thread count.
constexpr int kBins = 32;
void sah_build(BinTree& T, std::vector<int32_t>& ids, std::vector<float>& lbox, std::vector<float>& cen, size_t b,
               size_t e, size_t at, int par_depth) {
  const size_t n = e - b;
  float* nb = &T.box[6 * at];
  empty_box(nb);
  for (size_t i = b; i < e; ++i) grow(nb, &lbox[6 * i]);
  if (n == 1) {
    T.kid[2 * at] = -1;
    T.kid[2 * at + 1] = ids[b];
    return;
  }
  float cb[6];
  empty_box(cb);
  for (size_t i = b; i < e; ++i) {
    const float* c = &cen[3 * i];
    for (int a = 0; a < 3; ++a) {
      cb[a] = std::min(cb[a], c[a]);
      cb[3 + a] = std::max(cb[3 + a], c[a]);
    }
  }
  int axis = -1, split = 0;
  double best = INFINITY;
  float bin_lo[3], bin_scale[3];
  for (int a = 0; a < 3; ++a) {
    const double ext = (double)cb[3 + a] - cb[a];
    if (!(ext > 1e-30)) continue;   // (a bin scale must stay a finite float)
    bin_lo[a] = cb[a];
    bin_scale[a] = (float)(kBins / ext * (1.0 - 1e-6));
    float bbox[kBins][6];
    size_t bcnt[kBins] = {};
    for (int k = 0; k < kBins; ++k) empty_box(bbox[k]);
    for (size_t i = b; i < e; ++i) {
      int k = (int)((cen[3 * i + a] - bin_lo[a]) * bin_scale[a]);
      k = std::min(std::max(k, 0), kBins - 1);
      bcnt[k]++;
      grow(bbox[k], &lbox[6 * i]);
    }
    double right_cost[kBins];
    float acc[6];
    empty_box(acc);
    size_t cnt = 0;
    for (int k = kBins - 1; k > 0; --k) {
      grow(acc, bbox[k]);
      cnt += bcnt[k];
      right_cost[k] = cnt ? half_area(acc) * (double)cnt : 0.0;
    }
    empty_box(acc);
    cnt = 0;
    for (int k = 0; k < kBins - 1; ++k) {
      grow(acc, bbox[k]);
      cnt += bcnt[k];
      if (cnt == 0 || cnt == n) continue;
      const double cost = half_area(acc) * (double)cnt + right_cost[k + 1];
      if (cost < best) {
        best = cost;
        axis = a;
        split = k + 1;
      }
    }
  }
  size_t m;
  if (axis >= 0) {
    const float lo = bin_lo[axis], sc = bin_scale[axis];
    // partition ids, boxes and centroids together
    size_t i = b, j = e;
    auto bin_of = [&](size_t q) {
      int k = (int)((cen[3 * q + axis] - lo) * sc);
      return std::min(std::max(k, 0), kBins - 1);
    };
    while (i < j) {
      if (bin_of(i) < split) {
        ++i;
      } else {
        --j;
        std::swap(ids[i], ids[j]);
        for (int q = 0; q < 6; ++q) std::swap(lbox[6 * i + q], lbox[6 * j + q]);
        for (int q = 0; q < 3; ++q) std::swap(cen[3 * i + q], cen[3 * j + q]);
      }
    }
    m = i;
  } else {
    m = b + n / 2;   // every centroid equal: any split
  }
  if (m == b || m == e) m = b + n / 2;
  const size_t nl = m - b;
  const size_t left = at + 1, right = at + 2 * nl;
  T.kid[2 * at] = (int32_t)left;
  T.kid[2 * at + 1] = (int32_t)right;
  if (par_depth > 0 && n > 65536) {
    std::thread th;
    try {
      th = std::thread([&] { sah_build(T, ids, lbox, cen, b, m, left, par_depth - 1); });
    } catch (const std::system_error&) {   // no thread to be had: build both halves here
      sah_build(T, ids, lbox, cen, b, m, left, 0);
    }
    sah_build(T, ids, lbox, cen, m, e, right, par_depth - 1);
    if (th.joinable()) th.join();
  } else {
    sah_build(T, ids, lbox, cen, b, m, left, 0);
    sah_build(T, ids, lbox, cen, m, e, right, 0);
  }
}

}  // namespace

std::string build_wide_bvh(const float* N, size_t n, bool int_bits, const float* V, size_t n_vf,
                           const uint32_t* I, size_t n_tris, WideBVH* out, int mode) {
  *out = WideBVH();
  if (n == 0) return "no nodes";
  if (mode != WIDE_FROM_REFERENCE && mode != WIDE_SAH) return "unknown wide build mode";
  auto link = [&](size_t i, int which) -> int32_t {
    const float f = N[8 * i + (which ? 7 : 3)];
    int32_t v;
    if (int_bits) memcpy(&v, &f, 4);
    else v = (int32_t)f;
    return v;
  };
  auto leaf = [&](size_t i) { return link(i, 0) == -1; };
  auto lo = [&](size_t i, int a) { return N[8 * i + a]; };
  auto hi = [&](size_t i, int a) { return N[8 * i + 4 + a]; };
  // pre-order (right child first: the reference's visit order) and leaf ranks
  std::vector<int32_t> order, rank(n, -1);
  order.reserve(n);
  {
    std::vector<int32_t> st{0};
    while (!st.empty()) {
      const int32_t v = st.back();
      st.pop_back();
      order.push_back(v);
      if (leaf(v)) {
        rank[v] = (int32_t)out->rank_tri.size();
        out->rank_tri.push_back(link(v, 1));
      } else {
        st.push_back(link(v, 0));
        st.push_back(link(v, 1));
      }
    }
  }
  if (out->rank_tri.size() != n_tris) return "tree leaves do not cover the triangles once";
  {   // every triangle slot exactly once: the rank <-> slot maps must be bijective
    std::vector<uint8_t> seen(n_tris, 0);
    for (const int32_t t : out->rank_tri) {
      if (t < 0 || (size_t)t >= n_tris || seen[(size_t)t]) return "tree leaves do not cover the triangles once";
      seen[(size_t)t] = 1;
    }
  }
  // the walk's premises on the uploaded arrays: finite, bounded coordinates;
  // parent boxes contain their children's (so the reference tests a triangle
  // iff its leaf box passes); leaf boxes contain their triangle
  for (size_t i = 0; i < n; ++i)
    for (int a = 0; a < 3; ++a)
      if (!(fabs((double)lo(i, a)) <= kMaxCoord && fabs((double)hi(i, a)) <= kMaxCoord))
        return "node coordinates not finite or beyond 1e15";
  std::vector<WideCoeffs> lc(n);   // per reference node: the largest coefficients over its subtree
  for (size_t k = order.size(); k-- > 0;) {
    const int32_t v = order[k];
    if (leaf(v)) {
      const uint32_t t = (uint32_t)link(v, 1);
      float p[3][3];
      for (int c = 0; c < 3; ++c) {
        const uint32_t vi = I[3 * (size_t)t + c];
        if ((size_t)vi * 3 + 2 >= n_vf) return "vertex index out of range";
        for (int a = 0; a < 3; ++a) {
          p[c][a] = V[3 * (size_t)vi + a];
          if (!(p[c][a] >= lo(v, a) && p[c][a] <= hi(v, a))) return "leaf box does not contain its triangle";
        }
      }
      float e1[3], e2[3];
      for (int a = 0; a < 3; ++a) {
        e1[a] = p[1][a] - p[0][a];   // fl(v1 - v0), as setup_tris_kernel
        e2[a] = p[2][a] - p[0][a];
      }
      if (!wide_tri_coeffs(e1, e2, &lc[v])) lc[v] = WideCoeffs{INFINITY, 0.0, 0.0, 0.0};   // no culling
    } else {
      const int32_t l = link(v, 0), r = link(v, 1);
      for (int32_t ch : {l, r})
        for (int a = 0; a < 3; ++a)
          if (!(lo(v, a) <= lo(ch, a) && hi(v, a) >= hi(ch, a))) return "a parent box does not contain its child's";
      lc[v] = coeff_max(lc[l], lc[r]);
    }
  }
  // the binary tree to collapse
  BinTree T;
  if (mode == WIDE_FROM_REFERENCE) {
    T.box.resize(6 * n);
    T.kid.resize(2 * n);
    T.co = std::move(lc);
    for (size_t v = 0; v < n; ++v) {
      for (int a = 0; a < 3; ++a) {
        T.box[6 * v + a] = lo(v, a);
        T.box[6 * v + 3 + a] = hi(v, a);
      }
      if (leaf(v)) {
        T.kid[2 * v] = -1;
        T.kid[2 * v + 1] = (int32_t)v;
      } else {   // right child first, as the reference visits them
        T.kid[2 * v] = link(v, 1);
        T.kid[2 * v + 1] = link(v, 0);
      }
    }
  } else {
    std::vector<int32_t> ids;
    ids.reserve(n_tris);
    for (int32_t v : order)
      if (leaf(v)) ids.push_back(v);
    std::vector<float> lbox(6 * n_tris), cen(3 * n_tris);
    for (size_t i = 0; i < n_tris; ++i)
      for (int a = 0; a < 3; ++a) {
        const float l = lo(ids[i], a), h = hi(ids[i], a);
        lbox[6 * i + a] = l;
        lbox[6 * i + 3 + a] = h;
        cen[3 * i + a] = 0.5f * l + 0.5f * h;
      }
    const size_t nb = 2 * n_tris - 1;
    T.box.resize(6 * nb);
    T.kid.resize(2 * nb);
    sah_build(T, ids, lbox, cen, 0, n_tris, 0, 4);
    T.co.resize(nb);
    for (size_t v = nb; v-- > 0;)   // children are stored after their parent
      T.co[v] = T.leaf(v) ? lc[T.kid[2 * v + 1]] : coeff_max(T.co[T.kid[2 * v]], T.co[T.kid[2 * v + 1]]);
  }
  // wide nodes: expand the binary node's children, largest box first, until
  // four entries or all leaves
  auto area = [&](int32_t v) { return half_area(&T.box[6 * (size_t)v]); };
  std::vector<float>& W = out->nodes;
  std::vector<int32_t> n_inner;              // per wide node: inner children
  std::vector<std::vector<int32_t>> kids;    // per wide node: its inner children's wide indices
  auto alloc = [&]() {
    W.resize(W.size() + 32, 0.0f);
    n_inner.push_back(0);
    kids.emplace_back();
    return (int32_t)(n_inner.size() - 1);
  };
  std::vector<std::pair<int32_t, int32_t>> st;   // (binary node, wide node)
  st.push_back({0, alloc()});
  while (!st.empty()) {
    const auto [v, w] = st.back();
    st.pop_back();
    std::vector<int32_t> list;
    if (T.leaf(v)) {
      list.push_back(v);   // a one-triangle tree: the root leaf is the only child
    } else {
      list = {T.kid[2 * v], T.kid[2 * v + 1]};
      while (list.size() < 4) {
        int best = -1;
        double ba = -1.0;
        for (size_t j = 0; j < list.size(); ++j)
          if (!T.leaf(list[j]) && area(list[j]) > ba) {
            ba = area(list[j]);
            best = (int)j;
          }
        if (best < 0) break;
        const int32_t x = list[best];
        list[best] = T.kid[2 * x];
        list.insert(list.begin() + best + 1, T.kid[2 * x + 1]);
      }
    }
    WideCoeffs co{0.0, 0.0, 0.0, 0.0};
    float* rec = &W[32 * (size_t)w];
    for (int j = 0; j < 4; ++j) {
      int32_t ref = kEmpty;
      if (j < (int)list.size()) {
        const int32_t c = list[j];
        const float* cb = &T.box[6 * (size_t)c];
        for (int a = 0; a < 3; ++a) {
          rec[8 * a + j] = cb[a];
          rec[8 * a + 4 + j] = cb[3 + a];
        }
        co = coeff_max(co, T.co[c]);
        if (T.leaf(c)) {
          ref = ~rank[T.kid[2 * (size_t)c + 1]];
        } else {
          ref = alloc();
          rec = &W[32 * (size_t)w];   // alloc may move W
          n_inner[w]++;
          kids[w].push_back(ref);
          st.push_back({c, ref});
        }
      }
      memcpy(&rec[24 + j], &ref, 4);
    }
    node_cull_consts(co, &rec[28]);
  }
  // stack bound: a node pushes at most (inner children - 1) entries, which
  // stay until its subtree is done: the most along any root-to-node path
  const size_t nw = n_inner.size();
  std::vector<int32_t> bound(nw, 0);
  for (size_t w = nw; w-- > 0;) {   // children are allocated after their parent
    int32_t m = 0;
    for (int32_t k : kids[w]) m = std::max(m, bound[k]);
    bound[w] = std::max(0, n_inner[w] - 1) + m;
  }
  if (bound[0] > 4096) return "tree too deep for the wide walk's stack";
  // the 64-B layout of the same nodes, and the reference's leaf boxes by rank
  // (the walk over 64-B nodes tests a leaf's exact box before it accepts a hit)
  out->qnodes.assign(16 * nw, 0.0f);
  for (size_t w = 0; w < nw; ++w)
    if (!quantize_node(&W[32 * w], &out->qnodes[16 * w])) return "a wide node's boxes cannot be quantized";
  out->leaf_box.assign(8 * n_tris, 0.0f);
  for (size_t v = 0; v < n; ++v)
    if (leaf(v))
      for (int a = 0; a < 3; ++a) {
        out->leaf_box[8 * (size_t)rank[v] + a] = lo(v, a);
        out->leaf_box[8 * (size_t)rank[v] + 4 + a] = hi(v, a);
      }
  out->n_nodes = (int)nw;
  out->stack_cap = bound[0] + 1;
  return "";
}

}  // namespace pt
