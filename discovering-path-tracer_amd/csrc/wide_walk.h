// wide_walk.h — culled closest-hit / any-hit walk over a 4-wide BVH built
// from the reference's tree, for scenes in device memory.
//
// Why it returns the reference's hit.  traceRay (raytrace_comp.comp:159-204)
// is an exhaustive DFS: a leaf's triangle is tested iff the leaf's box and
// every ancestor's box pass intersectAABB, and the hit is the accepted
// triangle of least t, ties going to the first visited.  For a ray whose
// invDir = 1/dir is finite on all three axes (and a finite origin and
// scene), every slab quantity (lo - o) * inv is NaN-free and monotone in lo,
// so a box B' containing B bitwise gives t_near' <= t_near and t_far' >=
// t_far, hence "B hit => B' hit".  The reference builder makes every parent
// box the componentwise min/max over its subtree (BoundingVolumeHierarchy.cpp
// :84-100), so a leaf passes its own test only if all its ancestors pass
// theirs: the triangles the reference tests are exactly those whose LEAF box
// passes.  The result is then the least t over those triangles with ties to
// the least visit rank (the leaf's position in the right-first DFS order,
// :198-199), and any walk that tests every such triangle that could still
// win -- in any order, over any grouping of the boxes -- returns it bit for
// bit.  Rays with an infinite/NaN invDir component (a zero or subnormal
// direction component), or a direction longer than the cull bound assumes,
// are handed back for the exact threaded walk (kNeedExact*); the host builds
// the wide tree only after checking the containment on the uploaded arrays.
//
// The walk visits 4-wide nodes nearest child first and skips (culls) a child
// box B when no triangle inside it can have t <= the current best t (closest
// rays) or t < limit (shadow rays).  The cull test must be exact-safe, i.e.
// hold for the t the reference's float Moller-Trumbore computes, not the
// real intersection.  wide_bvh.cpp derives from IEEE error bounds of every op
// of intersectTriangle (:114-157), under its |det| >= 1e-6 and t > 1e-6
// acceptance: an accepted t_b comes from an exact T at which the ray o + T d
// lies within eps = eps0 + eps1 S of the triangle (S = |o - v0|_inf), so T is
// at least the ray's exact entry parameter into B less eps |1/d|_max; and
// t_b >= (T (1 - k1) - k2 S) / (1 + g3).  A node stores, over the triangles
// below each child, c1 = min (1 - k1) / (1 + g3) rounded down and E0, E1
// rounded up (E1 also covering k2 / c1); a child is culled iff
//     lim < th,  th = c1 * (t_near (1 - 2^-20) - (E0 + E1 Smax) (|1/d|_max + 1))
// (evaluated per axis, with the (1 - 2^-20) folded into c1, E0, E1:
// node_cull_consts) with t_near the slab test's own entry value and Smax the largest |lo - o|,
// |hi - o| of its own differences (>= S / (1 + 3u): v0 lies in B).  The
// margins cover every rounding of this evaluation.  Culling never removes a
// triangle that could win or tie, so the answer is the reference's.
// (Round 2's first bound used the Euclidean distance to the box instead of
// the entry parameter: it culled less -- the box nearest the origin is often
// entered far along the ray -- and needed a square root per child.)
// tests/wide_check.cpp checks it against the exhaustive walk on hundreds of
// thousands of rays (grazing, axis-aligned, inside-box origins).
#pragma once
#include "pt_isect.h"

namespace ptd {

// Node: 128 B = 8 float4 (one cache line):
//   [0] lo.x[4] [1] hi.x[4] [2] lo.y[4] [3] hi.y[4] [4] lo.z[4] [5] hi.z[4]
//   [6] child refs (int bits): >= 0 node index, < 0 ~rank of a leaf,
//       kWideEmpty unused slot
//   [7] cull constants {c1 (rounded down), E0, E1 (rounded up), 0}
// Leaf boxes are the reference's leaf boxes bitwise.  Triangle records are
// stored by rank (the reference tris layout, 3 float4), with rank -> slot.
constexpr int kWideNodeF4 = 8;
constexpr int32_t kWideEmpty = (int32_t)0x80000000;
// 64-B node (QN, the default layout; wide_bvh.cpp quantize_node): 4 float4
//   [0] {p.xyz, meta}  meta byte a: biased exponent of the axis-a grid step s_a
//   [1] {qlo.x, qhi.x, qlo.y, qhi.y}   uint32 each, byte j = child j
//   [2] {qlo.z, qhi.z, c1, E0 | E1 << 16 (bf16, rounded up)}
//   [3] child refs
// Child j's box on axis a is [fma(qlo_j, s_a, p_a), fma(qhi_j, s_a, p_a)]:
// the builder rounds every box outward onto the grid and checks these exact
// float values enclose it, so the decoded box contains the 128-B node's box
// (a leaf's decoded box contains the reference's leaf box, which the walk
// then tests exactly before it accepts that leaf's hit, wide_cand).  Every
// argument above holds for any enclosing box: a larger box passes the slab
// test whenever the box it contains does, its entry parameter and Smax only
// lower the cull threshold.  Half the bytes and load instructions per node
// visit: the trace kernel is bound by its vector-memory pipeline (TD busy
// 91-97 % with 128-B nodes, profiles/r03).
constexpr int kWideQNodeF4 = 4;
PT_FN float wq_scale(uint32_t meta, int a) { return u2f(((meta >> (8 * a)) & 0xffu) << 23); }
PT_FN float wq_dec(uint32_t w, int j, float s, float p) { return fma_((float)((w >> (8 * j)) & 0xffu), s, p); }
#ifndef PT_WIDE_LDS_STACK
#define PT_WIDE_LDS_STACK 8
#endif
constexpr int kWideLds = PT_WIDE_LDS_STACK;   // stack entries per lane kept in LDS (a ring)
#ifndef PT_WIDE_PUSH
#define PT_WIDE_PUSH 1
#endif
#ifndef PT_WIDE_POP2
#define PT_WIDE_POP2 0
#endif
// PT_WIDE_QRAW: the leaf queue holds the child ref as the node stores it
// (~rank), and the flush takes the complement once per tested candidate
// instead of the walk once per child per step
#ifndef PT_WIDE_QRAW
#define PT_WIDE_QRAW 1
#endif
#ifndef PT_WIDE_POPWAIT
#define PT_WIDE_POPWAIT 1
#endif
PT_FN int wide_qput(int c) { return PT_WIDE_QRAW ? c : ~c; }
PT_FN int wide_qrank(int q) { return PT_WIDE_QRAW ? ~q : q; }
// position of stack entry i in the LDS ring
PT_FN int wide_ring(int i) { return (kWideLds & (kWideLds - 1)) == 0 ? (i & (kWideLds - 1)) : (i % kWideLds); }
// hits[] markers: the ray needs the exact threaded walk (wide_ray_ok false,
// or a stack bound violation, which the builder rules out)
constexpr int kNeedExactClosest = -2;
constexpr int kNeedExactShadow = 2;
// direction-length guard of the cull bound: |d|^2 <= 1 + 2e-5 (computed)
constexpr float kWideMaxD2 = 1.00002f;
// |1/d_i| bound: with coordinates <= 1e15 every slab t stays finite (< 1e28)
constexpr float kWideMaxInv = 0x1p40f;

struct WideRay {
  v3 o, d, inv;
  v3 ainv;      // fl(|1/d_i| + 1)
  float lim;    // closest: best t (1e30 = none yet); shadow: occlusion limit
  int best;     // closest: rank of the best triangle (-1 none); shadow: 1 once occluded
  int shadow;
  int cur;      // node to expand next, -1 = take one from the stack
  int sp, lo;   // entries on the stack; entries below lo live in the overflow area
  int nc;       // PT_WIDE_QUEUE: leaf candidates queued for the next wave-wide flush
};

// PT_WIDE_QUEUE: leaf hits are queued (their ranks, per lane in LDS) and
// tested when the wave flushes -- every lane with candidates in one loop --
// instead of in a per-node loop that runs while most lanes wait (measured:
// 14 of 64 lanes active per VALU instruction in the per-node form).  The
// candidates and their tests are the same; only the best-so-far used for
// culling may lag, which culls less, never wrongly.
#ifndef PT_WIDE_QUEUE
#define PT_WIDE_QUEUE 1   // 1080p 8 spp: displaced sphere 138 -> 131.5 ms, 10M cloud 258 -> 261, 1M cloud 231 -> 229
#endif
#ifndef PT_WIDE_QCAP
#define PT_WIDE_QCAP 8
#endif
constexpr int kWideQ = PT_WIDE_QCAP;

PT_FN bool finite_(float x) { return fabs_(x) <= 3.40282347e38f; }

// |coordinate| bound of origins and scene (the builder checks the scene):
// keeps dist^2 finite in wide_child
constexpr float kWideMaxCoord = 1e15f;

PT_FN bool wide_ray_ok(v3 o, v3 d, v3 inv) {
  return fabs_(inv.x) <= kWideMaxInv && fabs_(inv.y) <= kWideMaxInv && fabs_(inv.z) <= kWideMaxInv &&
         fabs_(o.x) <= kWideMaxCoord &&
         fabs_(o.y) <= kWideMaxCoord && fabs_(o.z) <= kWideMaxCoord && dot(d, d) <= kWideMaxD2;
}

// One child box: the reference slab test (same ops as slab()), its t_near,
// and the cull threshold th (culled iff lim < th).  kf: the node's
// {c1, E0, E1, 0}.
// PT_WIDE_AINV_REG 0: fl(|1/d_i| + 1) is recomputed per node (3 ops shared by
// the 4 children) instead of held in 3 registers across the walk
#ifndef PT_WIDE_AINV_REG
#define PT_WIDE_AINV_REG 0
#endif
PT_FN v3 wide_ainv(const WideRay& R) {
  return PT_WIDE_AINV_REG ? R.ainv : mk(fabs_(R.inv.x) + 1.0f, fabs_(R.inv.y) + 1.0f, fabs_(R.inv.z) + 1.0f);
}
PT_FN void wide_child(const WideRay& R, v3 ainv, float lx, float hx, float ly, float hy, float lz, float hz, float4 kf,
                      bool* hit, float* tn, float* th) {
  const float dlx = lx - R.o.x, dly = ly - R.o.y, dlz = lz - R.o.z;
  const float dhx = hx - R.o.x, dhy = hy - R.o.y, dhz = hz - R.o.z;
  const float t0x = dlx * R.inv.x, t0y = dly * R.inv.y, t0z = dlz * R.inv.z;
  const float t1x = dhx * R.inv.x, t1y = dhy * R.inv.y, t1z = dhz * R.inv.z;
  const float tmin = fmax_(fmax_(fmin_(t0x, t1x), fmin_(t0y, t1y)), fmin_(t0z, t1z));
  const float tmax = fmin_(fmin_(fmax_(t0x, t1x), fmax_(t0y, t1y)), fmax_(t0z, t1z));
  *hit = tmin <= tmax && tmax >= 0.0f;
  *tn = tmin;
  const float smax = fmax_(fmax_(fmax_(fabs_(dlx), fabs_(dhx)), fmax_(fabs_(dly), fabs_(dhy))),
                           fmax_(fabs_(dlz), fabs_(dhz)));
  // the (1 - 2^-20) factor of t_near is folded into the node's constants
  // (wide_bvh.cpp node_cull_consts: c1' = c1 (1 - 2^-20), E' = E / (1 - 2^-20))
  const float eps = fma_(kf.z, smax, kf.y);
  const float e0 = fma_(-eps, ainv.x, fmin_(t0x, t1x));
  const float e1 = fma_(-eps, ainv.y, fmin_(t0y, t1y));
  const float e2 = fma_(-eps, ainv.z, fmin_(t0z, t1z));
  *th = kf.x * fmax_(fmax_(e0, e1), e2);
}

// Stack: entries [lo, sp) in the lane's LDS ring, older ones in its global
// overflow area.  Pop: the entry's two words come in one 8-B LDS read, made
// unconditionally (the ring slot is always there): a select between the LDS
// and the overflow pointer made the compiler issue two dependent flat loads
// per pop (the threshold, then the node index once the threshold passed),
// each waiting on both memory counters.  The rare overflow entry is then
// re-read from the global area.
PT_FN int2 wide_pop(WideRay& R, const int2* lds, int ls, const int2* ovf, long long os) {
  --R.sp;
  const unsigned long long w = *(const unsigned long long*)&lds[wide_ring(R.sp) * ls];
  int2 e = make_int2((int)(uint32_t)w, (int)(uint32_t)(w >> 32));
  if (R.sp < R.lo) {
    R.lo = R.sp;
    e = ovf[(long long)R.sp * os];
#if PT_WIDE_POPWAIT && defined(__HIP_DEVICE_COMPILE__)
    // wait for the overflow entry here, on this rare path: otherwise the
    // join after the branch waits for every vector-memory operation of the
    // wave (vmcnt(0)), stores of hits and evicted entries included, on every pop
    __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0), expcnt and lgkmcnt unconstrained
#endif
  }
  return e;
}

PT_FN void wide_start(WideRay& R, v3 o, v3 d, bool shadow, float limit) {
  R.o = o;
  R.d = d;
  R.inv = mk(rcp_(d.x), rcp_(d.y), rcp_(d.z));
  R.ainv = mk(fabs_(R.inv.x) + 1.0f, fabs_(R.inv.y) + 1.0f, fabs_(R.inv.z) + 1.0f);
  R.shadow = shadow ? 1 : 0;
  R.lim = shadow ? limit : 1e30f;
  R.best = shadow ? 0 : -1;
  R.cur = 0;   // the root node
  R.sp = 0;
  R.lo = 0;
  R.nc = 0;
}

// Tests the queued candidates (PT_WIDE_QUEUE) with the reference's accept
// rules; true when a shadow ray is occluded (its walk is over).
// One queued candidate's test with the reference's accept rules; true when a
// shadow ray is occluded.
// QN: the candidate came from a decoded (enclosing) leaf box; the reference
// tests its triangle only if its own leaf box passes intersectAABB, so a hit
// that would count is checked against that box first (rare: accepted hits).
template <bool QN = false>
PT_FN bool wide_leaf_ok(const WideRay& R, const float4* __restrict__ leaf_box, int r) {
  return !QN || slab(R.o, R.inv, leaf_box[2 * (size_t)r], leaf_box[2 * (size_t)r + 1]);
}
// A tie in t goes to the lower rank (the reference's visit order).
template <bool QN = false>
PT_FN bool wide_cand(WideRay& R, int r, float4 A, float4 B, float4 C, const float4* __restrict__ leaf_box = nullptr) {
  float t;
  if (tri_test(R.o, R.d, A, B, C, &t)) {
    if (R.shadow) {
      if (t < 1e30f && !(t >= R.lim) && wide_leaf_ok<QN>(R, leaf_box, r)) {   // :359, :398
        R.best = 1;
        return true;
      }
    } else if ((t < R.lim || (t == R.lim && R.best >= 0 && r < R.best)) &&
               wide_leaf_ok<QN>(R, leaf_box, r)) {   // :185
      R.lim = t;   // strict '<' in visit order
      R.best = r;
    }
  }
  return false;
}

// The closest hit does not depend on the order the candidates are tested in
// (ties go to the lower rank, the reference's visit order), nor does a
// shadow ray's answer; PT_WIDE_FLUSH_BATCH candidates' records are loaded
// before the first of them is tested, so a flush waits for one round trip
// per batch instead of one per candidate.  2: sphere -3.2 %, 10M cloud
// -0.9 % (80 VGPRs, no spill); 4 spills: +26 % / +31 %.
#ifndef PT_WIDE_FLUSH_BATCH
#define PT_WIDE_FLUSH_BATCH 2
#endif
template <bool CNT, bool QN = false>
PT_FN bool wide_flush(WideRay& R, const float4* __restrict__ tris, const int* cand, uint32_t* cl,
                      const float4* __restrict__ leaf_box = nullptr) {
  const int n = R.nc;
  R.nc = 0;
  constexpr int KB = PT_WIDE_FLUSH_BATCH;
  for (int i = 0; i < n; i += KB) {
    int r[KB];
    float4 A[KB], B[KB], C[KB];
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      r[k] = wide_qrank(cand[(i + k < n ? i + k : i) * 64]);
      const float4* T = tris + 3 * (size_t)r[k];
      A[k] = T[0];
      B[k] = T[1];
      C[k] = T[2];
    }
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      if (i + k < n) {
        if (CNT) ++*cl;
        if (wide_cand<QN>(R, r[k], A[k], B[k], C[k], leaf_box)) return true;
      }
    }
  }
  return false;
}

// One node of the walk; true when the ray is finished (R.lim / R.best hold
// the answer) or must be handed to the exact walk (*exact).  stack_cap: the
// builder's bound on entries (overflow area size per lane).
template <bool CNT, bool QUEUE = false, bool QN = false>
PT_FN bool wide_step(WideRay& R, const float4* __restrict__ nodes, const float4* __restrict__ tris, int2* lds,
                     int ls, int2* ovf, long long os, int stack_cap, bool* exact, uint32_t* cn, uint32_t* cl,
                     int* cand = nullptr, const float4* __restrict__ leaf_box = nullptr) {
#if PT_WIDE_POP2
  // PT_WIDE_POP2: the top two entries are read together, so a pop whose entry
  // is culled goes on to the next one without a second LDS round trip (the
  // ring slot below the top always exists; an entry below lo is re-read from
  // the overflow area, as in wide_pop)
  while (R.cur < 0) {
    if (R.sp == 0) return true;
    const unsigned long long w1 = *(const unsigned long long*)&lds[wide_ring(R.sp - 1) * ls];
    const unsigned long long w2 = *(const unsigned long long*)&lds[wide_ring(R.sp - 2) * ls];
    --R.sp;
    int2 e = make_int2((int)(uint32_t)w1, (int)(uint32_t)(w1 >> 32));
    if (R.sp < R.lo) {
      R.lo = R.sp;
      e = ovf[(long long)R.sp * os];
    }
    if (!(R.lim < u2f((uint32_t)e.y))) {
      R.cur = e.x;
      break;
    }
    if (R.sp == 0) return true;
    --R.sp;
    e = make_int2((int)(uint32_t)w2, (int)(uint32_t)(w2 >> 32));
    if (R.sp < R.lo) {
      R.lo = R.sp;
      e = ovf[(long long)R.sp * os];
    }
    if (!(R.lim < u2f((uint32_t)e.y))) R.cur = e.x;
  }
#else
  while (R.cur < 0) {
    if (R.sp == 0) return true;
    const int2 e = wide_pop(R, lds, ls, ovf, os);
    if (!(R.lim < u2f((uint32_t)e.y))) R.cur = e.x;   // still able to hold a winner
  }
#endif
  float4 lx, hx, ly, hy, lz, hz, cf, kf;
  if (QN) {
    const float4* nd = nodes + (size_t)R.cur * kWideQNodeF4;
    const float4 q0 = nd[0], q1 = nd[1], q2 = nd[2];
    cf = nd[3];
    const uint32_t meta = f2u(q0.w);
    const float sx = wq_scale(meta, 0), sy = wq_scale(meta, 1), sz = wq_scale(meta, 2);
    const uint32_t a0 = f2u(q1.x), a1 = f2u(q1.y), a2 = f2u(q1.z), a3 = f2u(q1.w), a4 = f2u(q2.x), a5 = f2u(q2.y);
    lx = make_float4(wq_dec(a0, 0, sx, q0.x), wq_dec(a0, 1, sx, q0.x), wq_dec(a0, 2, sx, q0.x), wq_dec(a0, 3, sx, q0.x));
    hx = make_float4(wq_dec(a1, 0, sx, q0.x), wq_dec(a1, 1, sx, q0.x), wq_dec(a1, 2, sx, q0.x), wq_dec(a1, 3, sx, q0.x));
    ly = make_float4(wq_dec(a2, 0, sy, q0.y), wq_dec(a2, 1, sy, q0.y), wq_dec(a2, 2, sy, q0.y), wq_dec(a2, 3, sy, q0.y));
    hy = make_float4(wq_dec(a3, 0, sy, q0.y), wq_dec(a3, 1, sy, q0.y), wq_dec(a3, 2, sy, q0.y), wq_dec(a3, 3, sy, q0.y));
    lz = make_float4(wq_dec(a4, 0, sz, q0.z), wq_dec(a4, 1, sz, q0.z), wq_dec(a4, 2, sz, q0.z), wq_dec(a4, 3, sz, q0.z));
    hz = make_float4(wq_dec(a5, 0, sz, q0.z), wq_dec(a5, 1, sz, q0.z), wq_dec(a5, 2, sz, q0.z), wq_dec(a5, 3, sz, q0.z));
    const uint32_t e01 = f2u(q2.w);
    kf = make_float4(q2.z, u2f(e01 << 16), u2f(e01 & 0xffff0000u), 0.0f);
  } else {
    const float4* nd = nodes + (size_t)R.cur * kWideNodeF4;
    lx = nd[0]; hx = nd[1]; ly = nd[2]; hy = nd[3]; lz = nd[4]; hz = nd[5]; cf = nd[6]; kf = nd[7];
  }
  if (CNT) ++*cn;
  const v3 ainv = wide_ainv(R);
  const int c0 = (int)f2u(cf.x), c1 = (int)f2u(cf.y), c2 = (int)f2u(cf.z),
            c3 = (int)f2u(cf.w);
  bool h0, h1, h2, h3;
  float n0, n1, n2, n3, th0, th1, th2, th3;
  wide_child(R, ainv, lx.x, hx.x, ly.x, hy.x, lz.x, hz.x, kf, &h0, &n0, &th0);
  wide_child(R, ainv, lx.y, hx.y, ly.y, hy.y, lz.y, hz.y, kf, &h1, &n1, &th1);
  wide_child(R, ainv, lx.z, hx.z, ly.z, hy.z, lz.z, hz.z, kf, &h2, &n2, &th2);
  wide_child(R, ainv, lx.w, hx.w, ly.w, hy.w, lz.w, hz.w, kf, &h3, &n3, &th3);
  h0 = h0 && c0 != kWideEmpty && !(R.lim < th0);
  h1 = h1 && c1 != kWideEmpty && !(R.lim < th1);
  h2 = h2 && c2 != kWideEmpty && !(R.lim < th2);
  h3 = h3 && c3 != kWideEmpty && !(R.lim < th3);
  // leaves: test their triangles now (reference accept rules, rank tie-break)
  uint32_t lm = (h0 && c0 < 0 ? 1u : 0u) | (h1 && c1 < 0 ? 2u : 0u) | (h2 && c2 < 0 ? 4u : 0u) |
                (h3 && c3 < 0 ? 8u : 0u);
  if (QUEUE) {   // ... or queue them for the wave-wide flush
    cand[R.nc * 64] = wide_qput(c0);
    R.nc += (lm & 1u) ? 1 : 0;
    cand[R.nc * 64] = wide_qput(c1);
    R.nc += (lm & 2u) ? 1 : 0;
    cand[R.nc * 64] = wide_qput(c2);
    R.nc += (lm & 4u) ? 1 : 0;
    cand[R.nc * 64] = wide_qput(c3);
    R.nc += (lm & 8u) ? 1 : 0;
    lm = 0u;
  }
  while (lm) {
    const int j = __builtin_ctz(lm);
    lm &= lm - 1u;
    const int r = ~(j == 0 ? c0 : j == 1 ? c1 : j == 2 ? c2 : c3);
    const float thj = j == 0 ? th0 : j == 1 ? th1 : j == 2 ? th2 : th3;
    if (R.lim < thj) continue;   // culled by a hit found in this node
    if (CNT) ++*cl;
    const float4* T = tris + 3 * (size_t)r;
    if (wide_cand<QN>(R, r, T[0], T[1], T[2], leaf_box)) {   // an occluded shadow ray
      R.cur = -1;
      R.sp = 0;
      return true;
    }
  }
  // inner children still live: nearest first, the others onto the stack
  // (liveness is kept in its own mask: a live t_near may overflow to +inf)
  const uint32_t live = (h0 && c0 >= 0 && !(R.lim < th0) ? 1u : 0u) | (h1 && c1 >= 0 && !(R.lim < th1) ? 2u : 0u) |
                        (h2 && c2 >= 0 && !(R.lim < th2) ? 4u : 0u) | (h3 && c3 >= 0 && !(R.lim < th3) ? 8u : 0u);
  // Each live child's rank among the live ones by t_near (nearest 0, ties to
  // the lower slot): the nearest is expanded next, the others are written
  // straight to their stack slots, farthest deepest.  (A sorting network and
  // a push loop over the sorted slots measured 3 % slower on configs 3 and 5,
  // profiles/r04j: the same stack order, more select and branch instructions.)
  const bool l0 = live & 1u, l1 = (live >> 1) & 1u, l2 = (live >> 2) & 1u, l3 = (live >> 3) & 1u;
#if PT_WIDE_PUSH
  // Six pairwise orders instead of twelve: every t_near is finite here
  // (wide_ray_ok bounds the origin, the scene and |1/d|, so no slab product
  // is NaN), hence n_a <= n_b is exactly !(n_b < n_a) -- the same ranks.
  const bool b10 = n1 < n0, b20 = n2 < n0, b30 = n3 < n0, b21 = n2 < n1, b31 = n3 < n1, b32 = n3 < n2;
  const int r0 = (l1 && b10) + (l2 && b20) + (l3 && b30);
  const int r1 = (l0 && !b10) + (l2 && b21) + (l3 && b31);
  const int r2 = (l0 && !b20) + (l1 && !b21) + (l3 && b32);
  const int r3 = (l0 && !b30) + (l1 && !b31) + (l2 && !b32);
#else
  const int r0 = (l1 && n1 < n0) + (l2 && n2 < n0) + (l3 && n3 < n0);
  const int r1 = (l0 && n0 <= n1) + (l2 && n2 < n1) + (l3 && n3 < n1);
  const int r2 = (l0 && n0 <= n2) + (l1 && n1 <= n2) + (l3 && n3 < n2);
  const int r3 = (l0 && n0 <= n3) + (l1 && n1 <= n3) + (l2 && n2 <= n3);
#endif
  const int n_live = __builtin_popcount(live);
  R.cur = -1;
  if (n_live == 0) return false;
  if (R.sp + n_live - 1 > stack_cap) {   // cannot happen with the builder's bound; stay memory-safe
    *exact = true;
    return true;
  }
  const int top = R.sp + n_live - 1;   // stack entries after the pushes
  // PT_WIDE_PUSH 2: the ring keeps one slot free, ring(top), and every child
  // is written unconditionally -- a pushed one to its rank's slot, the
  // nearest and the dead ones to the free slot -- with no branch per child
  constexpr int kRingUse = PT_WIDE_PUSH >= 2 ? kWideLds - 1 : kWideLds;
  while (top - R.lo > kRingUse) {      // the LDS ring's oldest entries move to the overflow area
    ovf[(long long)R.lo * os] = lds[wide_ring(R.lo) * ls];
    ++R.lo;
  }
  if (PT_WIDE_PUSH >= 2) {
    lds[wide_ring(l0 && r0 > 0 ? top - r0 : top) * ls] = make_int2(c0, (int)f2u(th0));
    lds[wide_ring(l1 && r1 > 0 ? top - r1 : top) * ls] = make_int2(c1, (int)f2u(th1));
    lds[wide_ring(l2 && r2 > 0 ? top - r2 : top) * ls] = make_int2(c2, (int)f2u(th2));
    lds[wide_ring(l3 && r3 > 0 ? top - r3 : top) * ls] = make_int2(c3, (int)f2u(th3));
  } else {
    if (l0 && r0 > 0) lds[wide_ring(top - r0) * ls] = make_int2(c0, (int)f2u(th0));
    if (l1 && r1 > 0) lds[wide_ring(top - r1) * ls] = make_int2(c1, (int)f2u(th1));
    if (l2 && r2 > 0) lds[wide_ring(top - r2) * ls] = make_int2(c2, (int)f2u(th2));
    if (l3 && r3 > 0) lds[wide_ring(top - r3) * ls] = make_int2(c3, (int)f2u(th3));
  }
  R.sp = top;
  R.cur = (l0 && r0 == 0) ? c0 : (l1 && r1 == 0) ? c1 : (l2 && r2 == 0) ? c2 : c3;
  return false;
}

}  // namespace ptd
