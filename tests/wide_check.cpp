// Test infrastructure: runs the culled wide walk (csrc/wide_walk.h, the same
// code the GPU kernel runs, compiled for the host) over a batch of rays and
// compares every answer with the oracle's exhaustive traceRay restatement
// (oracle/pt_oracle.cpp, raytrace_comp.comp:159-204).  Built by
// tests/test_wide.py with hipcc (host code only) and linked to liboracle.so.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "scene/wide_bvh.h"
#include "wide_walk.h"

extern "C" void oracle_trace(const float* verts, const uint32_t* idx, const float* nodes, size_t n_nodes,
                             const float* o3, const float* d3, float* out, uint64_t* counters);

using namespace ptd;

namespace {
int g_mode = pt::WIDE_SAH;   // wide_set_mode
int g_node = 128;            // wide_set_variant: node bytes (64: the quantized layout with exact leaf tests)
int g_queue = 0;             // ... and 1: the queued leaf tests with per-lane flushes; 2: with the wave-wide flush's
                             // merge (flush_lexmin, the trace kernel's default)
unsigned long long g_steps = 0;   // walk steps (wide_step calls) since wide_set_variant (tools/walk_counts.py)

struct Built {
  pt::WideBVH w;
  std::vector<float4> tris;    // by rank: {v0, e1.x} {e1.yz, e2.xy} {e2.z, n}
};

std::string build(const float* V, size_t nvf, const uint32_t* I, size_t nt, const float* N, size_t nn, int int_bits,
                  Built* b) {
  std::string why = pt::build_wide_bvh(N, nn, int_bits != 0, V, nvf, I, nt, &b->w, g_mode);
  if (!why.empty()) return why;
  b->tris.resize(3 * nt);
  for (size_t r = 0; r < nt; ++r) {
    const uint32_t t = (uint32_t)b->w.rank_tri[r];
    v3 p[3];
    for (int c = 0; c < 3; ++c) {
      const uint32_t vi = I[3 * (size_t)t + c];
      p[c] = mk(V[3 * vi], V[3 * vi + 1], V[3 * vi + 2]);
    }
    const v3 e1 = sub(p[1], p[0]), e2 = sub(p[2], p[0]);
    const v3 n = normalize(cross(e1, e2));
    b->tris[3 * r] = make_float4(p[0].x, p[0].y, p[0].z, e1.x);
    b->tris[3 * r + 1] = make_float4(e1.y, e1.z, e2.x, e2.y);
    b->tris[3 * r + 2] = make_float4(e2.z, n.x, n.y, n.z);
  }
  return "";
}

// One ray's walk in the configured variant, as the trace kernel runs it:
// QUEUE: leaf hits queued (stride 64, like one lane of the kernel's LDS
// queue) and flushed when the queue cannot take another node's four leaves
// or the walk has no node left (PT_WIDE_FLUSH_T 1).
// The wave-wide flush of the trace kernel (pt_device.hip wide_flush_wave),
// restated for one lane: every queued candidate is tested (here in reverse
// queue order, as another lane of the wave could), the accepted ones reduce
// to the lexicographic least (t, rank) -- the kernel's LDS atomic min of
// (t bits << 32 | rank) -- which is merged with the ray's best by
// wide_cand's rule; a shadow ray is occluded by any accepted candidate.
template <bool QN>
bool flush_lexmin(WideRay& R, const float4* tris, const int* cand, uint32_t* cl, const float4* leaf_box) {
  const int n = R.nc;
  R.nc = 0;
  bool any = false;
  unsigned long long key = ~0ull;
  for (int i = n - 1; i >= 0; --i) {
    const int r = wide_qrank(cand[i * 64]);
    const float4* T = tris + 3 * (size_t)r;
    ++*cl;
    float t;
    if (tri_test(R.o, R.d, T[0], T[1], T[2], &t) && t < 1e30f && (R.shadow ? !(t >= R.lim) : t <= R.lim) &&
        (!QN || slab(R.o, mk(rcp_(R.d.x), rcp_(R.d.y), rcp_(R.d.z)), leaf_box[2 * (size_t)r],
                     leaf_box[2 * (size_t)r + 1]))) {
      any = true;
      const unsigned long long k = ((unsigned long long)f2u(t) << 32) | (uint32_t)r;
      if (k < key) key = k;
    }
  }
  if (!any) return false;
  if (R.shadow) {
    R.best = 1;
    return true;
  }
  const float tm = u2f((uint32_t)(key >> 32));
  const int rm = (int)(uint32_t)key;
  if (tm < R.lim || (tm == R.lim && R.best >= 0 && rm < R.best)) {
    R.lim = tm;
    R.best = rm;
  }
  return false;
}

template <bool QN, bool QUEUE>
void walk(WideRay& R, const Built& b, int2* lds, int2* ovf, bool* exact, uint32_t* cn, uint32_t* cl) {
  const float4* nodes = (const float4*)(QN ? b.w.qnodes.data() : b.w.nodes.data());
  const float4* leafbox = (const float4*)b.w.leaf_box.data();
  if (!QUEUE) {
    while (!wide_step<true, false, QN>(R, nodes, b.tris.data(), lds, 1, ovf, 1, b.w.stack_cap, exact, cn, cl, nullptr,
                                       leafbox)) {
    }
    return;
  }
  std::vector<int> cand(kWideQ * 64, -1);
  bool fin = false;
  for (;;) {
    if (!fin && ++g_steps)
      fin = wide_step<true, true, QN>(R, nodes, b.tris.data(), lds, 1, ovf, 1, b.w.stack_cap, exact, cn, cl,
                                      cand.data(), leafbox);
    if (*exact) return;
    if (R.nc > kWideQ - 4 || (fin && R.nc > 0)) {
      if (g_queue == 2 ? flush_lexmin<QN>(R, b.tris.data(), cand.data(), cl, leafbox)
                       : wide_flush<true, QN>(R, b.tris.data(), cand.data(), cl, leafbox)) {   // occluded
        fin = true;
        R.sp = 0;
        R.cur = -1;
      }
    }
    if (fin && R.nc == 0) return;
  }
}

}  // namespace

extern "C" {

// The wide builder the next calls use (pt::WideBuild).
void wide_set_mode(int mode) { g_mode = mode; }
// The walk variant the next wide_check calls run: node bytes 64 or 128,
// queued leaf tests or not.
void wide_set_variant(int node_bytes, int queue) {
  g_node = node_bytes;
  g_queue = queue;
  g_steps = 0;
}
unsigned long long wide_steps() { return g_steps; }

// info[0] wide nodes, info[1] stack bound.  Returns 0, or 1 with the reason in err.
int wide_info(const float* V, size_t nvf, const uint32_t* I, size_t nt, const float* N, size_t nn, int int_bits,
              int* info, char* err, size_t errlen) {
  Built b;
  const std::string why = build(V, nvf, I, nt, N, nn, int_bits, &b);
  if (!why.empty()) {
    snprintf(err, errlen, "%s", why.c_str());
    return 1;
  }
  info[0] = b.w.n_nodes;
  info[1] = b.w.stack_cap;
  return 0;
}

// The built wide tree itself: node floats (32 per node) into nodes (room for
// cap floats) and rank -> triangle slot into rank_tri (room for n_tris).
// Returns the float count, or -1 (err).
long long wide_dump(const float* V, size_t nvf, const uint32_t* I, size_t nt, const float* N, size_t nn, int int_bits,
                    float* nodes, size_t cap, int32_t* rank_tri, char* err, size_t errlen) {
  pt::WideBVH w;
  const std::string why = pt::build_wide_bvh(N, nn, int_bits != 0, V, nvf, I, nt, &w, g_mode);
  if (!why.empty()) {
    snprintf(err, errlen, "%s", why.c_str());
    return -1;
  }
  if (w.nodes.size() > cap || w.rank_tri.size() != nt) {
    snprintf(err, errlen, "buffer too small");
    return -1;
  }
  memcpy(nodes, w.nodes.data(), w.nodes.size() * sizeof(float));
  memcpy(rank_tri, w.rank_tri.data(), nt * sizeof(int32_t));
  return (long long)w.nodes.size();
}

// rays: n x 8 floats {o.xyz, d.xyz, kind (0 closest, 1 shadow), limit}.
// out: n x 4 {wide t|lim, wide hit/occluded (-1 exact walk needed), oracle t, oracle hit/occluded}.
// stats: [0] closest mismatches [1] shadow mismatches [2] exact hand-backs
// [3] wide nodes [4] wide triangle tests [5] oracle nodes [6] oracle leaf tests
// [7] first mismatching ray (or ~0).  Returns 0 or 1 (err).
int wide_check(const float* V, size_t nvf, const uint32_t* I, size_t nt, const float* N, size_t nn, int int_bits,
               const float* rays, size_t n, float* out, uint64_t* stats, char* err, size_t errlen) {
  Built b;
  const std::string why = build(V, nvf, I, nt, N, nn, int_bits, &b);
  if (!why.empty()) {
    snprintf(err, errlen, "%s", why.c_str());
    return 1;
  }
  std::vector<int2> lds(kWideLds), ovf((size_t)(size_t)b.w.stack_cap + 1);
  memset(stats, 0, 8 * sizeof(uint64_t));
  stats[7] = ~0ull;
  for (size_t i = 0; i < n; ++i) {
    const float* r = rays + 8 * i;
    const v3 o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
    const bool shadow = r[6] != 0.0f;
    float ref[8];
    uint64_t oc[3] = {0, 0, 0};
    oracle_trace(V, I, N, nn, r, r + 3, ref, oc);
    stats[5] += oc[1];
    stats[6] += oc[2];
    const bool ohit = ref[0] != 0.0f;
    const float lim = r[7];
    WideRay R;
    wide_start(R, o, d, shadow, lim);
    float wt = 0.0f, wres = -1.0f;
    bool exact = !wide_ray_ok(R.o, R.d, R.inv);
    uint32_t cn = 0, cl = 0;
    if (!exact) {
      if (g_node == 64)
        g_queue ? walk<true, true>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl)
                : walk<true, false>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl);
      else
        g_queue ? walk<false, true>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl)
                : walk<false, false>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl);
    }
    stats[3] += cn;
    stats[4] += cl;
    out[4 * i + 2] = ref[1];
    if (exact) {
      stats[2]++;
      out[4 * i] = 0.0f;
      out[4 * i + 1] = -1.0f;
      out[4 * i + 3] = ohit ? 1.0f : 0.0f;
      continue;
    }
    bool bad;
    if (shadow) {
      const bool occ_ref = ohit && !(ref[1] >= lim);   // :359 !hit || t >= dist - OFFSET
      wt = R.lim;
      wres = R.best ? 1.0f : 0.0f;
      out[4 * i + 3] = occ_ref ? 1.0f : 0.0f;
      bad = (R.best != 0) != occ_ref;
      if (bad) stats[1]++;
    } else {
      wt = R.lim;
      wres = R.best >= 0 ? 1.0f : 0.0f;
      out[4 * i + 3] = ohit ? 1.0f : 0.0f;
      bad = (R.best >= 0) != ohit;
      if (!bad && ohit) {
        // same t bits and the same triangle (its geometric normal, :189)
        const float4* T = &b.tris[3 * (size_t)R.best];
        const v3 e1 = mk(T[0].w, T[1].x, T[1].y), e2 = mk(T[1].z, T[1].w, T[2].x);
        const v3 nn3 = normalize(cross(e1, e2));
        bad = memcmp(&R.lim, &ref[1], 4) != 0 || memcmp(&nn3.x, &ref[5], 4) != 0 ||
              memcmp(&nn3.y, &ref[6], 4) != 0 || memcmp(&nn3.z, &ref[7], 4) != 0;
      }
      if (bad) stats[0]++;
    }
    if (bad && stats[7] == ~0ull) stats[7] = i;
    out[4 * i] = wt;
    out[4 * i + 1] = wres;
  }
  return 0;
}

// Per-ray work of the configured walk: nodes[i] node visits and tris[i]
// triangle tests of ray i (rays as for wide_check; -1 for a hand-back).
int wide_counts(const float* V, size_t nvf, const uint32_t* I, size_t nt, const float* N, size_t nn, int int_bits,
                const float* rays, size_t n, int32_t* nodes, int32_t* tris, char* err, size_t errlen) {
  Built b;
  const std::string why = build(V, nvf, I, nt, N, nn, int_bits, &b);
  if (!why.empty()) {
    snprintf(err, errlen, "%s", why.c_str());
    return 1;
  }
  std::vector<int2> lds(kWideLds), ovf((size_t)(size_t)b.w.stack_cap + 1);
  for (size_t i = 0; i < n; ++i) {
    const float* r = rays + 8 * i;
    WideRay R;
    wide_start(R, mk(r[0], r[1], r[2]), mk(r[3], r[4], r[5]), r[6] != 0.0f, r[7]);
    bool exact = !wide_ray_ok(R.o, R.d, R.inv);
    uint32_t cn = 0, cl = 0;
    if (!exact) {
      if (g_node == 64)
        g_queue ? walk<true, true>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl)
                : walk<true, false>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl);
      else
        g_queue ? walk<false, true>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl)
                : walk<false, false>(R, b, lds.data(), ovf.data(), &exact, &cn, &cl);
    }
    nodes[i] = exact ? -1 : (int32_t)cn;
    tris[i] = exact ? -1 : (int32_t)cl;
  }
  return 0;
}

// The per-triangle cull coefficients (wide_tri_coeffs) {k1, k2, eps0, eps1}
// and the node constants {c1, E0, E1, 0} a node over that one triangle gets.
int wide_coeffs(const float* e1, const float* e2, double* co, float* node) {
  pt::WideCoeffs c;
  if (!pt::wide_tri_coeffs(e1, e2, &c)) return 1;
  co[0] = c.k1;
  co[1] = c.k2;
  co[2] = c.eps0;
  co[3] = c.eps1;
  pt::node_cull_consts(c, node);
  return 0;
}

}  // extern "C"
