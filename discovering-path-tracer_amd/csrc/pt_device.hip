// pt_device.hip — the CDNA4 path-tracing kernels.
//
// One thread per pixel, one 64-lane wave per 8x8 pixel tile, four waves per
// 256-thread workgroup covering a 16x16 block (the reference's workgroup
// footprint, raytrace_comp.comp:43).  Each thread runs n_batches consecutive
// samples of its pixel and folds them into the running mean in registers, so
// the accumulation buffer is read and written once per launch instead of once
// per sample; the op sequence per sample is identical to n separate 1-spp
// dispatches (raytrace_comp.comp:467-469).
//
// Traversal (raytrace_comp.comp:159-204) is the reference's exhaustive DFS,
// executed stack-free over the threaded layout documented in pt_device.h: the
// node visit sequence, the AABB tests and the strict '<' tie-break are the
// reference's, so hits are bit-identical.  Two exact shortcuts:
//   * shadow rays only need "is there a hit closer than the light"
//     (:359, :398) — any accepted triangle with t < 1e30 and !(t >= limit)
//     settles it, so traversal stops there;
//   * the light pre-pass (:319-320) traces exactly the depth-0 ray (:333), so
//     that closest hit is computed once and used for both.
// In stats mode neither shortcut is taken and every reference traceRay call
// is counted with its exhaustive node/leaf counts.
//
// Numerics: every float op is the reference's, in its order, via pt_math.h;
// the file is compiled with -ffp-contract=off and correctly rounded div/sqrt.
#include <algorithm>

#include "pt_device.h"
#include "pt_isect.h"
#include "wide_walk.h"
#include "pt_math.h"

#pragma clang fp contract(off)

namespace ptd {
using namespace ptm;

namespace {

// Per-lane counters.  STATS (reference-exhaustive mode): rays = every
// reference traceRay, nodes/leaves = its exhaustive visits.  CNT (the fast
// kernels with counters, PT_OPT_COUNT_TRACED): rays = closest-hit walks and
// srays = shadow walks actually started, nodes = nodes actually visited,
// leaves = triangle tests actually run, prim = primary rays generated.
struct Ctr {
  uint32_t rays, nodes, leaves, srays, prim;
};

// This rank's li-th tile (pt_device.h Part; slot positions in device memory:
// a kernel argument array indexed at run time would be copied to scratch).
__device__ __forceinline__ int rank_tile(const RenderParams& P, int li) {
  return (li / P.part_cnt) * P.part_m + P.part_pos[li % P.part_cnt];
}

struct Hit {
  float t;
  int tri;   // -1 = miss
};

// Leaf candidates are queued per lane (in LDS, [slot][lane] so a wave's
// stores hit 64 distinct banks) and their triangles tested after the walk:
// in a wave whose lanes pass different leaves the triangle test then runs
// max-over-lanes times instead of once per leaf any lane passed.  Candidates
// are tested in visit order with the same strict '<', so the hit is the same.
#ifndef PT_WF_PF
#define PT_WF_PF 0
#endif
#ifndef PT_REC_PF
#define PT_REC_PF 0
#endif
#ifndef PT_KCAND
#define PT_KCAND 8
#endif
#ifndef PT_WF_WAVEFLUSH
#define PT_WF_WAVEFLUSH 1   // wf_trace_kernel: wave-wide candidate flush (see there)
#endif
#ifndef PT_WF_SORT
#define PT_WF_SORT 1   // wf_shade_kernel: bin each workgroup's next rays (see there)
#endif
#ifndef PT_WF_SORT_PHASE
#define PT_WF_SORT_PHASE 1   // ... by the phase the path waits in (0: by ray kind and octant)
#endif
#ifndef PT_WF_SHADOW_QUEUE
#define PT_WF_SHADOW_QUEUE 1   // wf_trace_kernel: shadow rays queue their leaves too (see there)
#endif
// queued shadow leaves are only ever flushed by the wave-wide flush
static_assert(PT_WF_WAVEFLUSH || !PT_WF_SHADOW_QUEUE, "PT_WF_SHADOW_QUEUE needs PT_WF_WAVEFLUSH");
constexpr int kCand = PT_KCAND;

// The running mean's step (:467-469): (acc * b + c) / (b + 1).  PT_FOLD_FAST:
// where b + 1 is a power of two the quotient is a product with its exact
// reciprocal (bitwise the IEEE quotient: both round the same exact value),
// and a running value of 1 folding a colour of 1 stays 1 ((b + 1) / (b + 1),
// b + 1 < 2^24 exact) -- the alpha channel of every live pixel.
#ifndef PT_FOLD_FAST
#define PT_FOLD_FAST 1
#endif
// PT_FOLD_DIRECT: with one lane per pixel each lane folds its own sample
// (no colour hand-off through LDS).  PT_SKIP_DEAD: the last SSS step's next
// direction and the last bounce's direction, never traced, are not computed
// (their draws still advance the stream).
#ifndef PT_FOLD_DIRECT
#define PT_FOLD_DIRECT 1   // box 1080p8, driver command: with PT_SKIP_DEAD and PT_FOLD_FAST 0.2131 -> 0.2114 ms (profiles/r05b/ab_box.log)
#endif
#ifndef PT_SKIP_DEAD
#define PT_SKIP_DEAD 1
#endif

// PF (prefetch): load node k+1 while node k is being tested — it is the next
// visit whenever k is a hit internal node or a leaf (the node arrays carry one
// node of padding so k+1 is always readable).  It was worth 12 % on a
// 1M-triangle scene in the first kernel; re-measured after the candidate queue,
// paired walks and null shadow rays it costs more than it hides: wavefront 1M
// cloud 400 -> 337 ms and 10M cloud 662 -> 616 ms without it, sphere 452 ->
// 423, recursive 5K sphere -2.5 %.  Off by default (PT_WF_PF, PT_REC_PF); an
// LDS-staged walk never used it.

__device__ __forceinline__ void test_candidates(const RenderParams& P, v3 o, v3 d, const int* cand, int nc,
                                                float* best, int* bt) {
  for (int i = 0; i < nc; ++i) {
    const int tri = cand[i * 64];
    const float4* T = P.tris + 3 * tri;
    float t;
    if (tri_test(o, d, T[0], T[1], T[2], &t) && t < *best) {
      *best = t;
      *bt = tri;
    }
  }
}

// Shadow-ray candidates (PT_WF_SHADOW_QUEUE): the queued triangles in visit
// order until the first one occluded() would stop at; true if any.
__device__ __forceinline__ bool test_shadow_candidates(const RenderParams& P, v3 o, v3 d, float limit,
                                                       const int* cand, int nc) {
  for (int i = 0; i < nc; ++i) {
    const int tri = cand[i * 64];
    const float4* T = P.tris + 3 * tri;
    float t;
    if (tri_test(o, d, T[0], T[1], T[2], &t) && t < 1e30f && !(t >= limit)) return true;
  }
  return false;
}

// FLUSH_OUT: the candidate queue is tested when the walk ends or the queue is
// full, by an outer loop around the node loop, instead of by a branch inside
// it.  Device-memory walks (path_trace_fused) gain 7 % (sphere 5K tris);
// LDS walks lose 1.6 % (box), so they keep the inner branch.
template <bool STATS, bool PF, bool FLUSH_OUT = false, bool CNT = false>
__device__ Hit trace_closest(const RenderParams& P, v3 o, v3 d, Ctr& c, int* cand) {
  const v3 inv = mk(rcp_(d.x), rcp_(d.y), rcp_(d.z));
  float best = 1e30f;
  int bt = -1;
  if (STATS || CNT) c.rays++;
  int k = 0, nc = 0;
  const int n = P.n_nodes;
  float4 a = P.nodes[0], b = P.nodes[1];
  while (k < n) {
   // FLUSH_OUT: walk until the walk ends or the queue is full, then test it
   while (k < n && (!FLUSH_OUT || nc < kCand)) {
    float4 na, nb;
    if (PF) {
      na = P.nodes[2 * k + 2];
      nb = P.nodes[2 * k + 3];
    }
    if (STATS || CNT) c.nodes++;
    const int raw = __float_as_int(a.w);
    // bit 31: bounds identical to the parent's, which this ray hit -> hit
    const bool h = slab(o, inv, a, b) || (raw < 0);   // branch-free: one LDS round trip per node
    const int tri = __float_as_int(b.w);
    // slot nc is free: write it unconditionally, keep it only for a hit leaf
    cand[nc * 64] = tri;
    const bool leaf_hit = h && tri >= 0;
    if (STATS || CNT) c.leaves += leaf_hit ? 1u : 0u;
    nc += leaf_hit ? 1 : 0;
    if (!FLUSH_OUT && nc == kCand) {
      test_candidates(P, o, d, cand, nc, &best, &bt);
      nc = 0;
    }
    const int next = (h && tri < 0) ? k + 1 : (raw & 0x7fffffff);
    if (PF && next == k + 1) {
      a = na;
      b = nb;
    } else {
      a = P.nodes[2 * next];
      b = P.nodes[2 * next + 1];
    }
    k = next;
   }
   if (FLUSH_OUT && nc == kCand) {
     test_candidates(P, o, d, cand, nc, &best, &bt);
     nc = 0;
   }
  }
  test_candidates(P, o, d, cand, nc, &best, &bt);
  Hit r;
  r.t = best;
  r.tri = bt;
  return r;
}

// Shadow query for "!hit || hit.t >= limit" (:359, :398): true iff some
// triangle the reference would accept (t < 1e30) has !(t >= limit).
// Triangles are tested as soon as their leaf is reached (no candidate queue):
// the early exit is worth more than the compaction for shadow rays (queueing
// 2/4/8 candidates measured 1-15 % slower on box.obj).
template <bool STATS, bool PF, bool CNT = false>
__device__ bool occluded(const RenderParams& P, v3 o, v3 d, float limit, Ctr& c) {
  const v3 inv = mk(rcp_(d.x), rcp_(d.y), rcp_(d.z));
  bool occ = false;
  if (STATS) c.rays++;
  if (CNT) c.srays++;
  int k = 0;
  const int n = P.n_nodes;
  float4 a = P.nodes[0], b = P.nodes[1];
  while (k < n) {
    float4 na, nb;
    if (PF) {
      na = P.nodes[2 * k + 2];
      nb = P.nodes[2 * k + 3];
    }
    if (STATS || CNT) c.nodes++;
    const int raw = __float_as_int(a.w);
    // bit 31: bounds identical to the parent's, which this ray hit -> hit
    const bool h = slab(o, inv, a, b) || (raw < 0);   // branch-free: one LDS round trip per node
    const int tri = __float_as_int(b.w);
    if (h && tri >= 0) {
      if (STATS || CNT) c.leaves++;
      const float4* T = P.tris + 3 * tri;
      float t;
      if (tri_test(o, d, T[0], T[1], T[2], &t) && t < 1e30f && !(t >= limit)) {
        occ = true;
        if (!STATS) return true;
      }
    }
    const int next = (h && tri < 0) ? k + 1 : (raw & 0x7fffffff);
    if (PF && next == k + 1) {
      a = na;
      b = nb;
    } else {
      a = P.nodes[2 * next];
      b = P.nodes[2 * next + 1];
    }
    k = next;
  }
  return occ;
}

// An occlusion query S and a closest-hit walk C, interleaved one node each per
// iteration: each walker visits exactly the node sequence of occluded() /
// trace_closest() above, with the same tests, candidate queue and strict '<',
// so both results are theirs bit for bit.  Interleaving only puts two
// independent node round trips in flight per lane -- the walks are bound by
// that latency (LDS or L2), not by issue.  has_s / has_c switch a walker off
// (it starts finished).  Fast kernels only: stats mode walks one ray at a time.
template <bool CNT = false>
__device__ __forceinline__ void walk_pair(const RenderParams& P, bool has_s, v3 so, v3 sd, float limit, bool* occ,
                                          bool has_c, v3 co, v3 cd, int* cand, Hit* hit, Ctr& c) {
  const int n = P.n_nodes;
  const v3 sinv = mk(rcp_(sd.x), rcp_(sd.y), rcp_(sd.z));
  const v3 cinv = mk(rcp_(cd.x), rcp_(cd.y), rcp_(cd.z));
  int ks = has_s ? 0 : n, kc = has_c ? 0 : n;
  if (CNT) {
    c.srays += has_s ? 1u : 0u;
    c.rays += has_c ? 1u : 0u;
  }
  bool oc = false;
  float best = 1e30f;
  int bt = -1, nc = 0;
  while (ks < n || kc < n) {
    // both loads first (a finished walker re-reads node 0, unused)
    const int ls = ks < n ? ks : 0, lc = kc < n ? kc : 0;
    const float4 sa = P.nodes[2 * ls], sb = P.nodes[2 * ls + 1];
    const float4 ca = P.nodes[2 * lc], cb = P.nodes[2 * lc + 1];
    if (ks < n) {
      const int raw = __float_as_int(sa.w);
      const bool h = slab(so, sinv, sa, sb) || (raw < 0);
      const int tri = __float_as_int(sb.w);
      int next = (h && tri < 0) ? ks + 1 : (raw & 0x7fffffff);
      if (CNT) c.nodes++;
      if (h && tri >= 0) {
        if (CNT) c.leaves++;
        const float4* T = P.tris + 3 * tri;
        float t;
        if (tri_test(so, sd, T[0], T[1], T[2], &t) && t < 1e30f && !(t >= limit)) {
          oc = true;
          next = n;
        }
      }
      ks = next;
    }
    if (kc < n) {
      const int raw = __float_as_int(ca.w);
      const bool h = slab(co, cinv, ca, cb) || (raw < 0);
      const int tri = __float_as_int(cb.w);
      cand[nc * 64] = tri;
      nc += (h && tri >= 0) ? 1 : 0;
      if (CNT) {
        c.nodes++;
        c.leaves += (h && tri >= 0) ? 1u : 0u;
      }
      if (nc == kCand) {
        test_candidates(P, co, cd, cand, nc, &best, &bt);
        nc = 0;
      }
      kc = (h && tri < 0) ? kc + 1 : (raw & 0x7fffffff);
    }
  }
  test_candidates(P, co, cd, cand, nc, &best, &bt);
  *occ = oc;
  hit->t = best;
  hit->tri = bt;
}

// Lights are read-only for the whole launch and indexed by a wave-uniform
// loop counter: reading them through the constant address space lets the
// compiler use scalar loads (scalar cache, one load per wave) instead of a
// per-lane vector load whose latency every shadow ray waited on.
__device__ __forceinline__ LightDev load_light(const RenderParams& P, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) float* ConstF;
  const ConstF f = (ConstF)(P.lights + i);
  LightDev L;
  float* o = (float*)&L;
#pragma unroll
  for (int k = 0; k < (int)(sizeof(LightDev) / 4); ++k) o[k] = f[k];
  return L;
#else
  return P.lights[i];
#endif
}

// Whether a shadow ray's answer can change the image.  Its light term is
// I * diff * rcp(max(d2, 0.01)) (:352-363, :392-402).  When diff = max(dot, 0)
// is 0 and I is finite, every channel of the term is +-0, and adding +-0 to
// the running sum (direct / sssLight, which start at +0 and so are never -0)
// leaves it bitwise unchanged: occluded or not, the result is the same, so the
// fast kernels skip the walk.  (The RNG draws for the light sample are made
// before, as in the reference.)  Stats mode still walks every shadow ray.
__device__ __forceinline__ bool shadow_needed(const LightDev& L, float diff) {
  return diff != 0.0f || L.finite == 0.0f;
}

// sampleAreaLight (:255-268); the light's frame (:261-264) is precomputed per
// light by setup_lights_kernel with the same ops.
__device__ __forceinline__ v3 sample_area_light(const LightDev& L, uint32_t* rng) {
  const float u = rng_next(rng) * 2.0f - 1.0f;
  const float v = rng_next(rng) * 2.0f - 1.0f;
  const v3 right = mk(L.right[0], L.right[1], L.right[2]);
  const v3 up = mk(L.up[0], L.up[1], L.up[2]);
  const v3 pos = mk(L.pos[0], L.pos[1], L.pos[2]);
  return add(add(pos, muls(muls(muls(right, u), L.size[0]), 0.5f)), muls(muls(muls(up, v), L.size[1]), 0.5f));
}

// intersectAreaLight (:271-298)
__device__ __forceinline__ bool intersect_area_light(v3 o, v3 d, const LightDev& L, float* t) {
  const v3 n_raw = mk(L.nraw[0], L.nraw[1], L.nraw[2]);
  const v3 pos = mk(L.pos[0], L.pos[1], L.pos[2]);
  const float denom = dot(n_raw, d);
  if (fabs_(denom) < 0.0001f) return false;
  const float tt = dot(n_raw, sub(pos, o)) / denom;
  *t = tt;
  if (tt <= 0.0f) return false;
  const v3 hp = add(o, muls(d, tt));
  const v3 th = sub(hp, pos);
  const float u = dot(th, mk(L.right[0], L.right[1], L.right[2]));
  const float v = dot(th, mk(L.up[0], L.up[1], L.up[2]));
  return fabs_(u) <= L.half[0] && fabs_(v) <= L.half[1];
}

// sampleSphere (:246-253)
__device__ __forceinline__ v3 sample_sphere(uint32_t* rng) {
  const float z = 2.0f * rng_next(rng) - 1.0f;
  const float th = (2.0f * 0x1.921fb6p+1f) * rng_next(rng);
  const float r = sqrt_(1.0f - z * z);
  float sn, cs;
  sincos_(th, &sn, &cs);
  return mk(r * cs, r * sn, z);
}

// sampleHemisphere (:229-243)
__device__ __forceinline__ v3 sample_hemisphere(v3 n, uint32_t* rng) {
  const float r1 = rng_next(rng);
  const float r2 = rng_next(rng);
  const float th = acos_(sqrt_(1.0f - r1));
  const float ph = (2.0f * 0x1.921fb6p+1f) * r2;
  float st, ct, sp, cp;
  sincos_(th, &st, &ct);
  sincos_(ph, &sp, &cp);
  const v3 l = mk(st * cp, st * sp, ct);
  const v3 upv = fabs_(n.z) < 0.999f ? mk(0.0f, 0.0f, 1.0f) : mk(1.0f, 0.0f, 0.0f);
  const v3 t = normalize(cross(upv, n));
  const v3 b = cross(n, t);
  return add(add(muls(t, l.x), muls(b, l.y)), muls(n, l.z));
}

__device__ __forceinline__ v3 tri_normal(const RenderParams& P, int tri) {
  const float4 C = P.hit_tris[3 * tri + 2];
  return mk(C.y, C.z, C.w);
}

__device__ __forceinline__ void add_ctr(Ctr& a, const Ctr& b) {
  a.rays += b.rays;
  a.nodes += b.nodes;
  a.leaves += b.leaves;
  a.srays += b.srays;
  a.prim += b.prim;
}

// LDS-staged scenes park path state in LDS during walks (PT_PARK) and run 6
// waves per SIMD (80 VGPRs, 2 spilled) instead of 5 (96): box 1080p8 -3.8 %.
// 7 waves spill 19 VGPRs and gain nothing; parking at 5 waves costs +1.7 %.
#ifndef PT_PARK
#define PT_PARK 1
#endif
// Parking in the paired walks of device-memory scenes (25 instead of 35
// spilled VGPRs, at 5 waves/SIMD): sphere 5K tris -1.0 %, 20K cloud -2.0 %
// (neutral while the k+1 prefetch held 8 more registers).  4 waves without
// spills: +12 %.
#ifndef PT_PARK_FUSED
#define PT_PARK_FUSED 1
#endif
constexpr int kPark = (PT_PARK || PT_PARK_FUSED) ? 12 : 0;   // floats of path state parked in LDS around a walk
__device__ __forceinline__ void park3(float* pk, int i, v3 v) {
  pk[i * 64] = v.x;
  pk[(i + 1) * 64] = v.y;
  pk[(i + 2) * 64] = v.z;
}
__device__ __forceinline__ v3 unpark3(const float* pk, int i) {
  return mk(pk[i * 64], pk[(i + 1) * 64], pk[(i + 2) * 64]);
}
// PARK: the path state a walk does not read (throughput, radiance, hit
// point and normal) waits in this lane's LDS column during the walk, so the
// walk's registers peak lower.  The empty asm with a memory clobber keeps the
// compiler from forwarding the stored values past the walk.
#define PT_WALK2(PARK, stmt)                                                         \
  do {                                                                               \
    if (PARK) { park3(pk, 0, thr); park3(pk, 3, rad); __asm__ volatile("" ::: "memory"); } \
    stmt;                                                                            \
    if (PARK) { __asm__ volatile("" ::: "memory"); thr = unpark3(pk, 0); rad = unpark3(pk, 3); } \
  } while (0)
#define PT_WALK4(PARK, stmt)                                                         \
  do {                                                                               \
    if (PARK) {                                                                      \
      park3(pk, 0, thr); park3(pk, 3, rad); park3(pk, 6, hp); park3(pk, 9, hn);      \
      __asm__ volatile("" ::: "memory");                                             \
    }                                                                                \
    stmt;                                                                            \
    if (PARK) {                                                                      \
      __asm__ volatile("" ::: "memory");                                             \
      thr = unpark3(pk, 0); rad = unpark3(pk, 3); hp = unpark3(pk, 6); hn = unpark3(pk, 9); \
    }                                                                                \
  } while (0)

// pathTrace (:300-418)
template <bool STATS, bool PF, bool CNT = false>
__device__ v3 path_trace(const RenderParams& P, v3 ro, v3 rd, uint32_t seed, Ctr& c, int* cand) {
  constexpr bool PARK = PT_PARK && !STATS && !PF;
  float* pk = (float*)(cand + kCand * 64);
  const float OFFSET = 0.001f;
  v3 thr = mk(1.0f, 1.0f, 1.0f);
  v3 rad = mk(0.0f, 0.0f, 0.0f);
  v3 hp, hn;
  uint32_t rng = seed;                                  // :307 re-seed

  Hit h0;
  h0.t = 1e30f;
  h0.tri = -1;
  bool have_h0 = false;
  Ctr c0 = {0u, 0u, 0u, 0u, 0u};
  Ctr& cp0 = CNT ? c : c0;   // CNT: the one walk is counted once
  for (int i = 0; i < P.n_lights; ++i) {                // :311-328
    const LightDev L = load_light(P, i);
    float tl;
    if (intersect_area_light(ro, rd, L, &tl)) {
      if (!have_h0) {
        h0 = trace_closest<STATS, PF, false, CNT>(P, ro, rd, cp0, cand);
        have_h0 = true;
      }
      if (STATS) add_ctr(c, c0);
      if (h0.tri < 0 || h0.t > tl) return mk(L.inten[0], L.inten[1], L.inten[2]);
    }
  }

  for (int depth = 0; depth < P.max_depth; ++depth) {   // :331
    Hit h;
    if (depth == 0) {
      if (!have_h0) {
        h0 = trace_closest<STATS, PF, false, CNT>(P, ro, rd, cp0, cand);
        have_h0 = true;
      }
      if (STATS) add_ctr(c, c0);
      h = h0;
    } else {
      PT_WALK2(PARK, h = (trace_closest<STATS, PF, false, CNT>(P, ro, rd, c, cand)));
    }
    if (h.tri < 0) {
      rad = add(rad, mul(thr, mk(0.0f, 0.0f, 0.0f)));  // background (:336)
      break;
    }
    hp = add(ro, muls(rd, h.t));                        // :188
    hn = tri_normal(P, h.tri);                          // :189

    const v3 albedo = mk(0.8f, 0.8f, 0.8f);
    v3 direct = mk(0.0f, 0.0f, 0.0f);
    for (int i = 0; i < P.n_lights; ++i) {              // :345-366
      const LightDev L = load_light(P, i);
      const v3 lp = sample_area_light(L, &rng);
      const v3 ld = normalize(sub(lp, hp));
      const float diff = fmax_(dot(hn, ld), 0.0f);
      const float dist = length(sub(lp, hp));
      bool vis = !STATS && !shadow_needed(L, diff);
      if (!vis) PT_WALK4(PARK, vis = !(occluded<STATS, PF, CNT>(P, add(hp, muls(hn, OFFSET)), ld, dist - OFFSET, c)));
      if (vis) {
        const float d2 = dist * dist;
        const v3 contrib = muls(muls(mk(L.inten[0], L.inten[1], L.inten[2]), diff), rcp_(fmax_(d2, 0.01f)));
        direct = add(direct, mul(albedo, contrib));
      }
    }
    rad = add(rad, mul(thr, direct));

    const v3 sss_albedo = mk(1.0f, 0.2f, 0.1f);         // :371-408
    const float sss_radius = 1.0f;
    v3 sss_thr = mk(1.0f, 1.0f, 1.0f);
    v3 so = sub(hp, muls(hn, OFFSET));
    v3 sd = sample_sphere(&rng);
    for (int k = 0; k < P.sss_bounces; ++k) {
      Hit sh;
      PT_WALK4(PARK, sh = (trace_closest<STATS, PF, false, CNT>(P, so, sd, c, cand)));
      if (sh.tri < 0) break;
      const float travel = sh.t;
      const v3 cp = add(so, muls(sd, travel));
      const v3 sn = tri_normal(P, sh.tri);
      v3 sl = mk(0.0f, 0.0f, 0.0f);
      for (int i = 0; i < P.n_lights; ++i) {
        const LightDev L = load_light(P, i);
        const v3 lp = sample_area_light(L, &rng);
        const v3 ed = normalize(sub(lp, cp));
        const float ediff = fmax_(dot(sn, ed), 0.0f);
        const float edist = length(sub(lp, cp));
        bool vis = !STATS && !shadow_needed(L, ediff);
        if (!vis) PT_WALK4(PARK, vis = !(occluded<STATS, PF, CNT>(P, add(cp, muls(sn, OFFSET)), ed, edist - OFFSET, c)));
        if (vis) {
          const float d2 = edist * edist;
          sl = add(sl, muls(mul(muls(sss_albedo, ediff), mk(L.inten[0], L.inten[1], L.inten[2])),
                            rcp_(fmax_(d2, 0.01f))));
        }
      }
      rad = add(rad, muls(mul(mul(thr, sss_thr), sl), 1.0f + sss_radius * 0.5f));
      sss_thr = mul(sss_thr, muls(sss_albedo, exp_(-travel / (sss_radius * 1.5f))));
      // the last step's next direction (:406-407) is never traced: its two
      // draws only advance the stream (the same state as sample_sphere's)
      if (STATS || !PT_SKIP_DEAD || k + 1 < P.sss_bounces) {
        so = sub(cp, muls(sn, OFFSET));
        sd = sample_sphere(&rng);
      } else {
        rng_skip(&rng, 2);
      }
    }

    // the last bounce's direction (:411-414) is never traced and the stream
    // is not read again: the path ends here
    if (PT_SKIP_DEAD && !STATS && depth + 1 >= P.max_depth) break;
    const v3 bd = sample_hemisphere(hn, &rng);          // :411-414
    thr = mul(thr, muls(albedo, dot(hn, bd)));
    ro = add(hp, muls(hn, OFFSET));
    rd = bd;
  }
  return rad;
}


// pathTrace (:300-418) for the fast kernels, with every shadow ray that has an
// independent closest-hit ray next to it walked as a pair (walk_pair): the
// last light's shadow ray of the direct term with the first SSS ray, and each
// SSS step's last shadow ray with the next SSS ray.  The RNG draws, the float
// operations and their order are path_trace's: a shadow result is only used
// after the pair returns, to finish the same sums in the same order.
template <bool PF, bool CNT = false>
__device__ v3 path_trace_fused(const RenderParams& P, v3 ro, v3 rd, uint32_t seed, int* cand, Ctr& c) {
  constexpr bool PARK = PT_PARK_FUSED != 0;
  float* pk = (float*)(cand + kCand * 64);
  const float OFFSET = 0.001f;
  v3 thr = mk(1.0f, 1.0f, 1.0f);
  v3 rad = mk(0.0f, 0.0f, 0.0f);
  v3 hp, hn;
  uint32_t rng = seed;                                  // :307 re-seed
  const int NL = P.n_lights;

  Hit h0;
  h0.t = 1e30f;
  h0.tri = -1;
  bool have_h0 = false;
  for (int i = 0; i < NL; ++i) {                        // :311-328
    const LightDev L = load_light(P, i);
    float tl;
    if (intersect_area_light(ro, rd, L, &tl)) {
      if (!have_h0) {
        h0 = trace_closest<false, PF, true, CNT>(P, ro, rd, c, cand);
        have_h0 = true;
      }
      if (h0.tri < 0 || h0.t > tl) return mk(L.inten[0], L.inten[1], L.inten[2]);
    }
  }

  const v3 albedo = mk(0.8f, 0.8f, 0.8f);
  const v3 sss_albedo = mk(1.0f, 0.2f, 0.1f);           // :371-408
  const float sss_radius = 1.0f;
  for (int depth = 0; depth < P.max_depth; ++depth) {   // :331
    Hit h;
    if (depth == 0) {
      if (!have_h0) {
        h0 = trace_closest<false, PF, true, CNT>(P, ro, rd, c, cand);
        have_h0 = true;
      }
      h = h0;
    } else {
      PT_WALK2(PARK, h = (trace_closest<false, PF, true, CNT>(P, ro, rd, c, cand)));
    }
    if (h.tri < 0) {
      rad = add(rad, mul(thr, mk(0.0f, 0.0f, 0.0f)));  // background (:336)
      break;
    }
    hp = add(ro, muls(rd, h.t));                        // :188
    hn = tri_normal(P, h.tri);                          // :189

    // direct light (:345-366); the last light's shadow ray is deferred
    v3 direct = mk(0.0f, 0.0f, 0.0f);
    v3 s_o = hp, s_d = hp, s_c = hp;   // deferred shadow ray: origin, dir, contribution if visible
    float s_lim = 0.0f;
    bool s_need = false;   // the deferred shadow ray can change the image (shadow_needed)
    for (int i = 0; i < NL; ++i) {
      const LightDev L = load_light(P, i);
      const v3 lp = sample_area_light(L, &rng);
      const v3 ld = normalize(sub(lp, hp));
      const float diff = fmax_(dot(hn, ld), 0.0f);
      const float dist = length(sub(lp, hp));
      const float d2 = dist * dist;
      const v3 contrib = mul(albedo, muls(muls(mk(L.inten[0], L.inten[1], L.inten[2]), diff), rcp_(fmax_(d2, 0.01f))));
      if (i + 1 < NL) {
        if (!shadow_needed(L, diff) || !occluded<false, PF, CNT>(P, add(hp, muls(hn, OFFSET)), ld, dist - OFFSET, c))
          direct = add(direct, contrib);
      } else {
        s_need = shadow_needed(L, diff);
        s_o = add(hp, muls(hn, OFFSET));
        s_d = ld;
        s_lim = dist - OFFSET;
        s_c = contrib;
      }
    }
    v3 sss_thr = mk(1.0f, 1.0f, 1.0f);
    v3 so = sub(hp, muls(hn, OFFSET));
    v3 sd = sample_sphere(&rng);
    Hit sh;
    bool occ = false;
    PT_WALK4(PARK, walk_pair<CNT>(P, NL > 0 && s_need, s_o, s_d, s_lim, &occ, P.sss_bounces > 0, so, sd, cand, &sh, c));
    if (NL > 0 && !occ) direct = add(direct, s_c);
    rad = add(rad, mul(thr, direct));

    for (int k = 0; k < P.sss_bounces; ++k) {
      if (sh.tri < 0) break;
      const float travel = sh.t;
      const v3 cp = add(so, muls(sd, travel));
      const v3 sn = tri_normal(P, sh.tri);
      v3 sl = mk(0.0f, 0.0f, 0.0f);
      for (int i = 0; i < NL; ++i) {
        const LightDev L = load_light(P, i);
        const v3 lp = sample_area_light(L, &rng);
        const v3 ed = normalize(sub(lp, cp));
        const float ediff = fmax_(dot(sn, ed), 0.0f);
        const float edist = length(sub(lp, cp));
        const float d2 = edist * edist;
        const v3 term = muls(mul(muls(sss_albedo, ediff), mk(L.inten[0], L.inten[1], L.inten[2])),
                             rcp_(fmax_(d2, 0.01f)));
        if (i + 1 < NL) {
          if (!shadow_needed(L, ediff) || !occluded<false, PF, CNT>(P, add(cp, muls(sn, OFFSET)), ed, edist - OFFSET, c))
            sl = add(sl, term);
        } else {
          s_need = shadow_needed(L, ediff);
          s_o = add(cp, muls(sn, OFFSET));
          s_d = ed;
          s_lim = edist - OFFSET;
          s_c = term;
        }
      }
      const v3 thr_k = mul(thr, sss_thr);
      sss_thr = mul(sss_thr, muls(sss_albedo, exp_(-travel / (sss_radius * 1.5f))));
      so = sub(cp, muls(sn, OFFSET));
      sd = sample_sphere(&rng);
      PT_WALK4(PARK, walk_pair<CNT>(P, NL > 0 && s_need, s_o, s_d, s_lim, &occ, k + 1 < P.sss_bounces, so, sd, cand, &sh, c));
      if (NL > 0 && !occ) sl = add(sl, s_c);
      rad = add(rad, muls(mul(thr_k, sl), 1.0f + sss_radius * 0.5f));
    }

    const v3 bd = sample_hemisphere(hn, &rng);          // :411-414
    thr = mul(thr, muls(albedo, dot(hn, bd)));
    ro = add(hp, muls(hn, OFFSET));
    rd = bd;
  }
  return rad;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// CNT kernels: add the wave's traced-work counters to P.stats[4..8]
// (closest walks, shadow walks, nodes visited, triangle tests, primaries).
__device__ __forceinline__ void flush_traced(const RenderParams& P, const Ctr& c, int lane) {
  const unsigned long long v0 = wave_sum(c.rays), v1 = wave_sum(c.srays), v2 = wave_sum(c.nodes),
                           v3_ = wave_sum(c.leaves), v4 = wave_sum(c.prim);
  if (lane == 0) {
    atomicAdd(&P.stats[4], v0);
    atomicAdd(&P.stats[5], v1);
    atomicAdd(&P.stats[6], v2);
    atomicAdd(&P.stats[7], v3_);
    atomicAdd(&P.stats[8], v4);
  }
}

// Running mean of n_batches constant colours (0,0,0,1) over this lane's
// channels (c = j mod spl), op for op the fold below.  Closed form where it is
// exact: (acc*b + 0)/(b+1) stays +0 once acc is +-0, and a batch-0 fold of
// any finite acc gives acc*0 + 0 = +0; (acc*b + 1)/(b+1) likewise stays 1.
__device__ __forceinline__ void fold_constant(const RenderParams& P, float* acc, int spl, int j) {
  if (P.n_batches == 0) return;
#pragma unroll
  for (int ch = 0; ch < 4; ++ch) {
    if (ch % spl != j) continue;
    const float k = ch < 3 ? 0.0f : 1.0f;
    if (acc[ch] == k || (P.first_batch == 0 && __builtin_isfinite(acc[ch]))) {
      acc[ch] = k;
    } else {
      for (uint32_t t = 0; t < P.n_batches; ++t) {
        const uint32_t batch = P.first_batch + t;
        acc[ch] = (acc[ch] * (float)batch + k) / (float)(batch + 1u);
      }
    }
  }
}

// This lane's channels (c = j mod spl) of the pixel's running mean.
__device__ __forceinline__ void store_lane(float4* px, const float* acc, int spl, int j) {
  float* a = (float*)px;
#pragma unroll
  for (int ch = 0; ch < 4; ++ch)
    if (ch % spl == j) a[ch] = acc[ch];
}

// The pixel's result: into the accumulation buffer, or (pt_render_packed)
// into this workgroup's slot of the packed live-item layout, where pixels
// outside the image are zeros (acc of an inactive lane is never loaded).
__device__ __forceinline__ void emit_lane(const RenderParams& P, bool active, size_t pix, int q, const float* acc,
                                          int spl, int j) {
  if (P.pack_out)
    store_lane(P.pack_out + (size_t)blockIdx.x * (size_t)(256 / spl) + (size_t)q, acc, spl, j);
  else if (active)
    store_lane(P.accum + pix, acc, spl, j);
}

// Items (tile parts) whose every pixel is culled, listed by the host with
// their first pixel: each thread folds the constant colour (0,0,0,1) into one
// pixel's running mean, closed form where exact (fold_constant) — kPixPerFill
// pixels per thread.  Runs as the trailing workgroups of the render launch,
// so it overlaps the render tail instead of costing a launch of its own.
// An item is 256 / spl pixels (a power of two), so a pixel's item and place
// in it are a shift and a mask: the per-pixel tile arithmetic (a 64-bit
// division, the partition's and the rotated tile order's) cost more than the
// fill itself -- box 1080p8, 70 % of the pixels culled: see DESIGN A.4.
#ifndef PT_PIX_PER_FILL
#define PT_PIX_PER_FILL 8
#endif
constexpr int kPixPerFill = PT_PIX_PER_FILL;
__device__ __forceinline__ int item_shift(int spl) { return 8 - __builtin_ctz((unsigned)spl); }   // log2(256 / spl)
__device__ __forceinline__ void fill_culled(const RenderParams& P, const int2* __restrict__ org, int n, int block) {
  const int lg = item_shift(P.spl);
  const long long total = (long long)n << lg;
  for (int k = 0; k < kPixPerFill; ++k) {
    const long long g = ((long long)block * kPixPerFill + k) * 256 + threadIdx.x;
    if (g >= total) return;
    const int2 o = org[g >> lg];
    const int q = (int)g & ((1 << lg) - 1);
    const int px = o.x + (q & 15);
    const int py = o.y + (q >> 4);
    if (px >= P.width || py >= P.height) continue;
    float4* dst = P.accum + (size_t)py * (size_t)P.width + (size_t)px;
    float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (!(P.fresh && P.first_batch == 0)) {
      const float4 a = *dst;
      acc[0] = a.x; acc[1] = a.y; acc[2] = a.z; acc[3] = a.w;
    }
    fold_constant(P, acc, 1, 0);
    *dst = make_float4(acc[0], acc[1], acc[2], acc[3]);
  }
}

// Pixel q of part `part` of tile `tile` (the render kernel's mapping).
__device__ __forceinline__ bool tile_pixel(const RenderParams& P, int tile, int part, int q, size_t* pix) {
  const int spl = P.spl;
  int bx, by;
  tile_block(tile, P.blocks_x, &bx, &by);
  const int px = bx * 16 + q % 16;
  const int py = by * 16 + part * (16 / spl) + q / 16;
  *pix = (size_t)py * (size_t)P.width + (size_t)px;
  return px < P.width && py < P.height;
}

// One pixel-slot g of the gathered-frame assembly (items_unpack_kernel, and
// the trailing workgroups of a pt_render_packed launch): a live item's pixel
// from its rank's slot, a culled item's pixel as (0,0,0,1).  Table entries
// are {rank, x0, y0, slot}: the item's first pixel comes from the host, so
// a pixel costs a shift and a mask (fill_culled).
__device__ __forceinline__ void unpack_pixel(const RenderParams& P, float4* __restrict__ frame,
                                             const float4* __restrict__ src, size_t slot_f4,
                                             const int* __restrict__ table, long long g) {
  const int lg = item_shift(P.spl);
  const int4 e = ((const int4*)table)[g >> lg];
  const int q = (int)g & ((1 << lg) - 1);
  const int px = e.y + (q & 15), py = e.z + (q >> 4);
  if (px >= P.width || py >= P.height) return;
  frame[(size_t)py * (size_t)P.width + (size_t)px] =
      e.w >= 0 ? src[(size_t)e.x * slot_f4 + ((size_t)e.w << lg) + q] : make_float4(0.0f, 0.0f, 0.0f, 1.0f);
}

__device__ __forceinline__ void unpack_block(const RenderParams& P, int block) {
  const long long total = (long long)P.n_unpack * (256 / P.spl);
  for (int k = 0; k < kPixPerFill; ++k) {
    const long long g = ((long long)block * kPixPerFill + k) * 256 + threadIdx.x;
    if (g >= total) return;
    unpack_pixel(P, P.unpack_frame, P.unpack_src, (size_t)P.unpack_slot_f4, P.unpack_table, g);
  }
}

// One step of the running mean (:467-469); PT_FOLD_FAST above.
__device__ __forceinline__ float fold_one(float a, float c, uint32_t batch) {
  const float fb = (float)batch, fb1 = (float)(batch + 1u);
  if (PT_FOLD_FAST && a == 1.0f && c == 1.0f && batch < (1u << 24)) return 1.0f;
  const float x = a * fb + c;
  if (PT_FOLD_FAST && ((batch + 1u) & batch) == 0u && batch + 1u != 0u) return x * (1.0f / fb1);
  return x / fb1;
}

#ifdef PT_WG_TRACE   // probe builds only (tools/r06_wg_trace.py): per live workgroup {t0, t1, hw_id << 32 | xcc | spl << 8, x0 << 32 | y0}
constexpr int kWgTraceCap = 1 << 16;
__device__ unsigned long long g_wg_trace[kWgTraceCap][4];
#endif

// LDS=true stages the whole scene (threaded nodes + triangle records) in LDS
// once per workgroup; chosen by the host for scenes of at most a few tens of
// KB (box.obj is 1.3 KB), where every lane re-reads the same few nodes.
template <bool STATS, bool LDS, bool CNT = false>
#ifndef PT_RENDER_MIN_BLOCKS
#define PT_RENDER_MIN_BLOCKS 5
#endif
#ifndef PT_RENDER_MIN_BLOCKS_LDS
#define PT_RENDER_MIN_BLOCKS_LDS (PT_PARK ? 6 : PT_RENDER_MIN_BLOCKS)
#endif
__global__ __launch_bounds__(256, LDS && !STATS ? PT_RENDER_MIN_BLOCKS_LDS : PT_RENDER_MIN_BLOCKS) void render_kernel(
    RenderParams P) {
  const int tid = (int)threadIdx.x;
  // Work mapping.  A 16x16 pixel tile (the partition unit) is split into
  // SPL workgroups; lane l of wave w handles pixel q = w*(64/SPL) + l/SPL of
  // its workgroup and sample slot j = l % SPL, so the SPL lanes of a pixel
  // trace that pixel's samples side by side: coherent rays, and SPL times
  // finer work granularity than one pixel per thread, which is what keeps a
  // tile-split frame fast on 8 GPUs (pixels on geometry cost ~10x the others).
  // A persistent variant pulling wave-sized items from per-XCD queues was
  // measured slower at every SPL, on 1 GPU and on a 1/8 tile share.
  if ((P.items || P.pack_out) && (int)blockIdx.x >= P.n_items) {   // trailing workgroups (uniform)
    if (P.pack_out)
      unpack_block(P, (int)blockIdx.x - P.n_items);   // assemble the previous gathered frame
    else
      fill_culled(P, P.culled_org, P.n_culled_items, (int)blockIdx.x - P.n_items);
    return;
  }
  // item = (owned tile, part); with culling the host launches only items that
  // can hold a live pixel, listed in P.items.  With mixed lanes (P.mix) each
  // live item carries its own lane count: whole tiles at one lane per pixel
  // first (the cheapest per sample), parts at P.spl lanes after them (short
  // workgroups that fill the launch's drain).  Uniform per workgroup.
  // cost feedback (PT_OPT_MIXED_LANES' measured schedule): each wave adds
  // its duration on the GPU wall clock to the counter of the 16x4 part of
  // the frame its pixels lie in
  const unsigned long long cost_t0 = P.cost_out ? wall_clock64() : 0ull;
  int gx0, gy0;
  bool tile_ok = true;
  int spl = P.spl;
  if (P.items_org) {
    const int2 o = P.items_org[blockIdx.x];
    gx0 = o.x & ((1 << kMixShift) - 1);
    gy0 = o.y;
    if (P.mix) spl = 1 << (o.x >> kMixShift);
  } else {
    const int item = (int)blockIdx.x;
    const int tile = rank_tile(P, item / spl);
    int bx, by;
    tile_block(tile, P.blocks_x, &bx, &by);
    gx0 = bx * 16;
    gy0 = by * 16 + (item % spl) * (16 / spl);
    tile_ok = tile < P.blocks_total;
  }
#ifdef PT_WG_TRACE
  const unsigned long long wg_t0 = wall_clock64();
#endif
  const int wave = tid >> 6, lane = tid & 63;
  // per wave: the leaf-candidate queue, then a [slot][lane] area that holds
  // the path state parked during walks (kPark floats) and, between samples,
  // the colour hand-off (4 floats) -- never both at once
  __shared__ int cand_buf[4][kCand + (kPark > 4 ? kPark : 4)][64];
  int* cand = &cand_buf[wave][0][lane];
  float* colw = (float*)&cand_buf[wave][kCand][0];   // colour hand-off, [channel][lane]
  const int q = wave * (64 / spl) + lane / spl;       // pixel within the workgroup
  const int j = lane % spl;                           // sample slot
  const int px = gx0 + q % 16;
  const int py = gy0 + q / 16;
  const bool active = tile_ok && px < P.width && py < P.height;   // :425-428
  Ctr c = {0u, 0u, 0u, 0u, 0u};
  const int W = P.width, H = P.height;
  // Per-pixel constants of main() (:430-432, :446-447, :457), hoisted out of
  // the sample loop — same values every sample.
  const float ndcX0 = (2.0f * (float)px / (float)W) - 1.0f;
  const float ndcY0 = (2.0f * (float)py / (float)H) - 1.0f;
  // Primary-ray culling (pt_primary_cull_rects): outside every rectangle no
  // primary ray of this pixel can reach the root box or a light, so each
  // sample is (0,0,0) — the value the trace below would produce.  A workgroup
  // with no live pixel skips the scene staging and the sample loop.
  bool live = true;
  bool wg_live = true;
  if (P.n_cull >= 0) {
    const float wx0 = (2.0f * (float)gx0 / (float)W) - 1.0f, wx1 = (2.0f * (float)(gx0 + 15) / (float)W) - 1.0f;
    const float wy0 = (2.0f * (float)gy0 / (float)H) - 1.0f;
    const float wy1 = (2.0f * (float)(gy0 + 16 / spl - 1) / (float)H) - 1.0f;
    live = false;
    wg_live = false;
#pragma unroll
    for (int r = 0; r < kMaxCullRects; ++r) {   // static indices: P stays in SGPRs/kernarg
      live = live || (r < P.n_cull && ndcX0 >= P.cull[r][0] && ndcX0 <= P.cull[r][1] && ndcY0 >= P.cull[r][2] &&
                      ndcY0 <= P.cull[r][3]);
      wg_live = wg_live || (r < P.n_cull && wx1 >= P.cull[r][0] && wx0 <= P.cull[r][1] && wy1 >= P.cull[r][2] &&
                            wy0 <= P.cull[r][3]);
    }
  }
  const size_t pix = (size_t)py * (size_t)W + (size_t)px;
  uint32_t nsamp = 0;
  if (active && (uint32_t)j < P.n_batches)
    nsamp = (P.n_batches - (uint32_t)j + (uint32_t)spl - 1) / (uint32_t)spl;
  // Running mean (:467-469): lane j of a pixel folds channels c = j (mod spl)
  // of that pixel, sample by sample in batch order.
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  // fresh: a launch that starts at batch 0 begins a new accumulation from a
  // cleared (+0) image — what pt_clear_accum would have stored — without
  // reading it (PT_OPT_FRESH_BATCH0).
  if (active && !(P.fresh && P.first_batch == 0)) {
    const float* a = (const float*)&P.accum[pix];
#pragma unroll
    for (int ch = 0; ch < 4; ++ch)
      if (ch % spl == j) acc[ch] = a[ch];
  }
  // A culled pixel's colours are all (0,0,0,1): its lanes fold them without
  // the colour hand-off (fold_constant), the live pixels' lanes below.
  if (!live && active) fold_constant(P, acc, spl, j);
  if (!wg_live) {   // uniform per workgroup; stats mode never culls
    emit_lane(P, active, pix, q, acc, spl, j);
    return;
  }
  if (LDS) {
    extern __shared__ float4 lds_scene[];
    const int nn = 2 * P.n_nodes, nt = 3 * P.n_tris;
    for (int i = tid; i < nn; i += 256) lds_scene[i] = P.nodes[i];
    for (int i = tid; i < nt; i += 256) lds_scene[nn + i] = P.tris[i];
    __syncthreads();
    P.nodes = lds_scene;
    P.tris = lds_scene + nn;
    P.hit_tris = P.tris;   // no wide walk here: hits are slots
  }
  {
    const v3 cpos = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
    const v3 cdir = mk(P.cam_dir[0], P.cam_dir[1], P.cam_dir[2]);
    const float aspect = (float)W / (float)H;
    // Camera frame (:430-432): computed once on the host with the same ops.
    const v3 right = mk(P.cam_right[0], P.cam_right[1], P.cam_right[2]);
    const v3 up = mk(P.cam_upv[0], P.cam_upv[1], P.cam_upv[2]);
    const float tanFov = P.tan_fov;
    for (uint32_t base = 0; base < P.n_batches; base += (uint32_t)spl) {
     const uint32_t s = base + (uint32_t)j;
     float4 col4 = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
     if (active && live && s < P.n_batches) {
      const uint32_t batch = P.first_batch + s;
      const uint32_t seed = (batch * (uint32_t)H + (uint32_t)py) * (uint32_t)W + (uint32_t)px;   // :435
      uint32_t rng = seed;
      // randomGaussian x2 (:218-226, :445, :451)
      float u1 = fmax_(1e-38f, rng_next(&rng));
      float u2 = rng_next(&rng);
      float r = sqrt_(-2.0f * log_(u1));
      float th = (2.0f * 0x1.921fb6p+1f) * u2;
      float sn, cs;
      sincos_(th, &sn, &cs);
      const float ax = (r * cs) * 0.02f;
      const float ay = (r * sn) * 0.02f;
      const v3 origin = add(add(cpos, muls(right, ax)), muls(up, ay));   // :448
      u1 = fmax_(1e-38f, rng_next(&rng));
      u2 = rng_next(&rng);
      r = sqrt_(-2.0f * log_(u1));
      th = (2.0f * 0x1.921fb6p+1f) * u2;
      sincos_(th, &sn, &cs);
      const float jx = r * cs, jy = r * sn;
      const float ndcX = ndcX0 + (jx * 0.5f) / (float)W;                 // :453-454
      const float ndcY = ndcY0 + (jy * 0.5f) / (float)H;
      const v3 bdir = normalize(sub(add(cdir, muls(neg(right), (ndcX * tanFov) * aspect)), muls(up, ndcY * tanFov)));
      const v3 focal = add(cpos, muls(bdir, 3.0f));                       // :459
      const v3 dir = normalize(sub(focal, origin));                       // :460
      // PF (prefetch node k+1) for walks from device memory; on an LDS-staged
      // scene it measured slower at every tile share (1080p box: +7 % on a
      // whole frame, +12 % on a 1/8 share: registers)
      // Scenes walked from device memory pair each shadow ray with the next
      // closest-hit ray (path_trace_fused: two node round trips in flight,
      // sphere 20K tris -9 %); on an LDS-staged scene the round trip is short
      // and the pair's registers cost more than it hides (box +11 %).
      v3 col;
      if (CNT) c.prim++;
      if (STATS || LDS)
        col = path_trace<STATS, !LDS, CNT>(P, origin, dir, seed, c, cand);
      else
        col = path_trace_fused<PT_REC_PF != 0, CNT>(P, origin, dir, seed, cand, c);
      col4 = make_float4(col.x, col.y, col.z, 1.0f);                      // vec4(color, 1.0)
     }
     if (PT_FOLD_DIRECT && spl == 1) {   // uniform: each lane folds its own sample, no hand-off (:467-469)
      if (active && live) {
        const uint32_t batch = P.first_batch + base;   // wave-uniform
        acc[0] = fold_one(acc[0], col4.x, batch);
        acc[1] = fold_one(acc[1], col4.y, batch);
        acc[2] = fold_one(acc[2], col4.z, batch);
        acc[3] = fold_one(acc[3], col4.w, batch);
      }
      continue;
     }
     // hand the chunk's colours to the folding lanes of the same pixel
     colw[lane] = col4.x;
     colw[64 + lane] = col4.y;
     colw[128 + lane] = col4.z;
     colw[192 + lane] = col4.w;
     __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
     __builtin_amdgcn_wave_barrier();
     __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
     if (active && live) {
      const uint32_t m = min((uint32_t)spl, P.n_batches - base);
      const int first_lane = lane - j;
      for (uint32_t t = 0; t < m; ++t) {
        const uint32_t batch = P.first_batch + base + t;                    // :468
        const float* cc = colw + first_lane + (int)t;
#pragma unroll
        for (int ch = 0; ch < 4; ++ch)
          if (ch % spl == j) acc[ch] = fold_one(acc[ch], cc[ch * 64], batch);
      }
     }
     __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
     __builtin_amdgcn_wave_barrier();
     __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  emit_lane(P, active, pix, q, acc, spl, j);
  if (!STATS && P.cost_out && lane == 0) {
    // the wave's pixels lie in one 16x4 part: its first pixel row / 4
    const int part_row = (gy0 + wave * (64 / spl) / 16) >> 2;
    const unsigned long long dt = wall_clock64() - cost_t0;
    atomicAdd(&P.cost_out[part_row * P.blocks_x + (gx0 >> 4)], (unsigned)(dt < 0xffffffull ? dt : 0xffffffull));
  }
#ifdef PT_WG_TRACE
  if (!STATS && !CNT) {
    __syncthreads();
    if (tid == 0 && blockIdx.x < (unsigned)kWgTraceCap) {
      const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID: wave, SIMD, CU, SE
      const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
      g_wg_trace[blockIdx.x][0] = wg_t0;
      g_wg_trace[blockIdx.x][1] = wall_clock64();
      g_wg_trace[blockIdx.x][2] = (unsigned long long)hw << 32 | (unsigned long long)((xcc & 0xff) | (spl << 8));
      g_wg_trace[blockIdx.x][3] = (unsigned long long)(unsigned)gx0 << 32 | (unsigned)gy0;
    }
  }
#endif
  if (STATS) {
    const unsigned long long rays = wave_sum(c.rays), nodes = wave_sum(c.nodes), leaves = wave_sum(c.leaves);
    const unsigned long long smp = wave_sum((unsigned long long)nsamp);
    if (lane == 0) {
      atomicAdd(&P.stats[0], rays);
      atomicAdd(&P.stats[1], nodes);
      atomicAdd(&P.stats[2], leaves);
      atomicAdd(&P.stats[3], smp);
    }
  }
  if (CNT) flush_traced(P, c, lane);
}

__global__ __launch_bounds__(256) void setup_tris_kernel(const float* __restrict__ V, const uint32_t* __restrict__ I,
                                                         int n_tris, float4* __restrict__ out) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= n_tris) return;
  const uint32_t i0 = I[3 * t + 0] * 3u, i1 = I[3 * t + 1] * 3u, i2 = I[3 * t + 2] * 3u;
  const v3 v0 = mk(V[i0], V[i0 + 1], V[i0 + 2]);
  const v3 v1 = mk(V[i1], V[i1 + 1], V[i1 + 2]);
  const v3 v2 = mk(V[i2], V[i2 + 1], V[i2 + 2]);
  const v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
  const v3 n = normalize(cross(e1, e2));
  out[3 * t + 0] = make_float4(v0.x, v0.y, v0.z, e1.x);
  out[3 * t + 1] = make_float4(e1.y, e1.z, e2.x, e2.y);
  out[3 * t + 2] = make_float4(e2.z, n.x, n.y, n.z);
}

// Per-light constants of sampleAreaLight / intersectAreaLight (:261-264,
// :284-287, :295-296), computed with the shader's ops.
// Triangle records in leaf-rank order for the wide walk.
__global__ __launch_bounds__(256) void gather_tris_kernel(const float4* __restrict__ tris,
                                                          const int* __restrict__ tri_of, int n,
                                                          float4* __restrict__ dst) {
  const int i = (int)(blockIdx.x * 256 + threadIdx.x);
  if (i >= 3 * n) return;
  const int r = i / 3, k = i - 3 * r;
  dst[i] = tris[3 * (size_t)tri_of[r] + k];
}

__global__ __launch_bounds__(64) void setup_lights_kernel(const LightRec* __restrict__ in, int n,
                                                          LightDev* __restrict__ out) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  const LightRec L = in[i];
  const v3 nr = mk(L.normal[0], L.normal[1], L.normal[2]);
  const v3 nn = normalize(nr);
  const v3 basis = fabs_(nn.y) < 0.999f ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
  const v3 right = normalize(cross(nn, basis));
  const v3 up = cross(right, nn);
  LightDev d;
  for (int c = 0; c < 3; ++c) {
    d.pos[c] = L.position[c];
    d.nraw[c] = L.normal[c];
    d.inten[c] = L.intensity[c];
  }
  d.right[0] = right.x; d.right[1] = right.y; d.right[2] = right.z;
  d.up[0] = up.x; d.up[1] = up.y; d.up[2] = up.z;
  d.size[0] = L.size[0];
  d.size[1] = L.size[1];
  d.half[0] = L.size[0] * 0.5f;
  d.half[1] = L.size[1] * 0.5f;
  d.finite = (__builtin_isfinite(d.inten[0]) && __builtin_isfinite(d.inten[1]) && __builtin_isfinite(d.inten[2]))
                 ? 1.0f : 0.0f;
  out[i] = d;
}

__global__ __launch_bounds__(256) void clear_kernel(float4* accum, int W, int H, int m, int cnt,
                                                    const int* __restrict__ pos) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)W * (size_t)H) return;
  const int x = (int)(i % (size_t)W), y = (int)(i / (size_t)W);
  const int blocks_x = (W + 15) / 16;
  const int b = block_tile(x / 16, y / 16, blocks_x);
  bool own = false;
  for (int i = 0; i < cnt; ++i) own = own || pos[i] == b % m;
  const float z = own ? 0.0f : -0.0f;
  accum[i] = make_float4(z, z, z, z);
}

// Owned 16x16 tiles <-> a dense buffer (tile o = the rank's o-th tile, part_tile,
// 256 float4 row-major inside the tile, zeros outside the image): what a rank
// ships to the root so the frame can be assembled by a gather.
template <bool PACK>
__global__ __launch_bounds__(256) void tiles_kernel(float4* frame, float4* packed, int W, int H, int blocks_x,
                                                    int m, int cnt, const int* __restrict__ pos) {
  const int o = (int)blockIdx.x;
  const int b = (o / cnt) * m + pos[o % cnt];
  const int t = (int)threadIdx.x;
  int bx, by;
  tile_block(b, blocks_x, &bx, &by);
  const int x = bx * 16 + (t & 15), y = by * 16 + (t >> 4);
  const bool in = x < W && y < H;
  const size_t pi = (size_t)y * (size_t)W + (size_t)x;
  const size_t ti = (size_t)o * 256 + (size_t)t;
  if (PACK)
    packed[ti] = in ? frame[pi] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  else if (in)
    frame[pi] = packed[ti];
}

__global__ __launch_bounds__(256) void items_pack_kernel(RenderParams P, const float4* __restrict__ frame,
                                                         float4* __restrict__ packed, const int* __restrict__ items,
                                                         int n) {
  const int per = 256 / P.spl;
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g >= (long long)n * per) return;
  size_t pix;
  const int item = items[g / per];
  const bool in = tile_pixel(P, rank_tile(P, item / P.spl), item % P.spl, (int)(g % per), &pix);
  packed[g] = in ? frame[pix] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

__global__ __launch_bounds__(256) void items_unpack_kernel(RenderParams P, float4* __restrict__ frame,
                                                           const float4* __restrict__ src, size_t slot_f4,
                                                           const int* __restrict__ table, int n) {
  const long long g = (long long)blockIdx.x * 256 + threadIdx.x;
  if (g >= (long long)n * (256 / P.spl)) return;
  unpack_pixel(P, frame, src, slot_f4, table, g);
}

__global__ __launch_bounds__(256) void math_kernel(int fn, const float* __restrict__ x, float* __restrict__ y,
                                                   size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  float r;
  switch (fn) {
    case 0: r = log_(v); break;
    case 1: r = exp_(v); break;
    case 2: r = sin_(v); break;
    case 3: r = cos_(v); break;
    case 4: r = tan_(v); break;
    case 5: r = acos_(v); break;
    case 6: r = sqrt_(v); break;
    case 7: { uint32_t s = __float_as_uint(v); r = rng_next(&s); break; }
    case 8: r = rcp_(v); break;
    default: r = v; break;
  }
  y[i] = r;
}

// Exhaustive equivalence of the device's fast-quotient math with the IEEE
// definitions (pt_math.h): every one of the 2^32 input bit patterns.
// fn 0 rcp_ vs 1/x, 1 log_, 2 exp_, 3 acos_ (each vs its FAST=false
// form).  NaN results compare equal when both are NaN.
__global__ __launch_bounds__(256) void exhaustive_kernel(int fn, unsigned long long* bad, uint32_t* first_bad) {
  unsigned long long nbad = 0;
  uint32_t first = 0xffffffffu;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
    const float x = __uint_as_float((uint32_t)i);
    float a, b;
    switch (fn) {
      case 0: a = rcp_(x); b = 1.0f / x; break;
      case 1: a = log_(x); b = log_impl<false>(x); break;
      case 2: a = exp_(x); b = exp_impl<false>(x); break;
      default: a = acos_(x); b = acos_impl<false>(x); break;
    }
    const bool same = __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
    if (!same) {
      ++nbad;
      first = min(first, (uint32_t)i);
    }
  }
  if (nbad) {
    atomicAdd(bad, nbad);
    atomicMin(first_bad, first);
  }
}

// ===========================================================================
// pathTrace (:300-418) as a state machine over one sample -- phases PRIMARY,
// DIRECT, SSS, SSS_SHADOW, BOUNCE -- holding at most one ray in flight: the
// shading half of the wavefront pipeline and of the tail kernel below.  The
// arithmetic, RNG draws and traversal order per ray are exactly those of
// path_trace(); only the interleaving across paths differs.  (A lane
// state-machine kernel built on it, each lane running its own pixel's
// samples, measured slower than the path-recursive kernel on every scene and
// was removed in round 4.)
// ===========================================================================
enum : int { PH_BEGIN = 0, PH_PRIMARY, PH_DIRECT, PH_SSS, PH_SSS_SHADOW, PH_BOUNCE };

struct Trav {
  v3 o, d, inv;
  int k;        // next node
  float lim;    // closest: best t so far; shadow: occlusion limit
  int res;      // closest: best triangle (-1 none); shadow: 1 once occluded
  int shadow;   // 0 closest-hit, 1 shadow query
  int nc;       // queued leaf candidates (closest)
  uint32_t cn, cl;   // node visits / leaf tests of this ray (stats)
};

struct PathSt {
  uint32_t s, rng;
  int phase, depth, li, k;
  v3 thr, rad, hp, hn, acc3, pend, sss_thr, so, sd, cp, sn;
  float travel;
};

__device__ __forceinline__ void trav_start(Trav& T, v3 o, v3 d, bool shadow, float limit) {
  T.o = o;
  T.d = d;
  T.inv = mk(rcp_(d.x), rcp_(d.y), rcp_(d.z));
  T.k = 0;
  T.shadow = shadow ? 1 : 0;
  T.lim = shadow ? limit : 1e30f;
  T.res = shadow ? 0 : -1;
  T.nc = 0;
  T.cn = 0u;
  T.cl = 0u;
}

// A shadow query whose answer cannot change the image (shadow_needed): it is
// still handed out as a ray, so the path keeps its place in the ray rounds
// (the wavefront lists stay phase-aligned, neighbouring paths coherent), but
// it starts finished, unoccluded: no node is visited.  Skipping it inside
// path_step instead measured +3 % on the displaced sphere (paths drift apart)
// with the exhaustive walks; with the culled wide walk the shading kernel
// answers it itself (PT_WF_NULL_INLINE, wf_shade_kernel).
__device__ __forceinline__ void trav_null(const RenderParams& P, Trav& T) {
  T.k = P.n_nodes;
  T.shadow = 2;
}

// One node of the walk; returns true when the ray is finished.
template <bool STATS>
__device__ __forceinline__ bool trav_step(const RenderParams& P, Trav& T, int* cand) {
  if (T.k >= P.n_nodes) {
    if (!T.shadow) {
      float best = T.lim;
      int bt = T.res;
      test_candidates(P, T.o, T.d, cand, T.nc, &best, &bt);
      T.lim = best;
      T.res = bt;
      T.nc = 0;
    }
    return true;
  }
  const float4 a = P.nodes[2 * T.k];
  const float4 b = P.nodes[2 * T.k + 1];
  if (STATS) T.cn++;
  const int raw = __float_as_int(a.w);
  const bool h = raw < 0 ? true : slab(T.o, T.inv, a, b);
  const int tri = __float_as_int(b.w);
  if (h && tri >= 0) {
    if (STATS) T.cl++;
    if (T.shadow) {
      const float4* Tr = P.tris + 3 * tri;
      float t;
      if (tri_test(T.o, T.d, Tr[0], Tr[1], Tr[2], &t) && t < 1e30f && !(t >= T.lim)) {
        T.res = 1;
        if (!STATS) return true;
      }
    } else {
      cand[T.nc * 64] = tri;
      if (++T.nc == kCand) {
        float best = T.lim;
        int bt = T.res;
        test_candidates(P, T.o, T.d, cand, T.nc, &best, &bt);
        T.lim = best;
        T.res = bt;
        T.nc = 0;
      }
    }
  }
  T.k = (h && tri < 0) ? T.k + 1 : (raw & 0x7fffffff);
  return false;
}

struct CamFrame {
  v3 cpos, cdir, right, up;
  float tanFov, aspect, ndcX0, ndcY0;
  int W, H, px, py;
};

// main() ray generation (:430-460) for one sample batch.
__device__ __forceinline__ void camera_ray(const CamFrame& F, uint32_t seed, v3* origin, v3* dir) {
  uint32_t rng = seed;
  float u1 = fmax_(1e-38f, rng_next(&rng));
  float u2 = rng_next(&rng);
  float r = sqrt_(-2.0f * log_(u1));
  float th = (2.0f * 0x1.921fb6p+1f) * u2;
  float sn, cs;
  sincos_(th, &sn, &cs);
  const float ax = (r * cs) * 0.02f;
  const float ay = (r * sn) * 0.02f;
  *origin = add(add(F.cpos, muls(F.right, ax)), muls(F.up, ay));
  u1 = fmax_(1e-38f, rng_next(&rng));
  u2 = rng_next(&rng);
  r = sqrt_(-2.0f * log_(u1));
  th = (2.0f * 0x1.921fb6p+1f) * u2;
  sincos_(th, &sn, &cs);
  const float jx = r * cs, jy = r * sn;
  const float ndcX = F.ndcX0 + (jx * 0.5f) / (float)F.W;
  const float ndcY = F.ndcY0 + (jy * 0.5f) / (float)F.H;
  const v3 bdir =
      normalize(sub(add(F.cdir, muls(neg(F.right), (ndcX * F.tanFov) * F.aspect)), muls(F.up, ndcY * F.tanFov)));
  const v3 focal = add(F.cpos, muls(bdir, 3.0f));
  *dir = normalize(sub(focal, *origin));
}

// pathTrace (:300-418) as a state machine over one sample: runs shading from
// the current phase until a ray must be traced (returns true, T set up; the
// caller traces it and calls again with T.lim/T.res holding the result) or
// the sample is complete (returns false, *out = its radiance).  Shared by the
// wavefront pipeline's generation, shading and tail kernels.
template <bool STATS>
__device__ bool path_step(const RenderParams& P, const CamFrame& F, PathSt& S, Trav& T, Ctr& c, v3* out) {
  const float OFFSET = 0.001f;
  const v3 albedo = mk(0.8f, 0.8f, 0.8f);
  const v3 sss_albedo = mk(1.0f, 0.2f, 0.1f);
  const float sss_radius = 1.0f;
  v3 color = mk(0.0f, 0.0f, 0.0f);
  for (;;) {
    bool finished = false;   // sample complete, `color` holds its radiance
    switch (S.phase) {
      case PH_BEGIN: {
        const uint32_t batch = P.first_batch + S.s;
        const uint32_t seed = (batch * (uint32_t)F.H + (uint32_t)F.py) * (uint32_t)F.W + (uint32_t)F.px;   // :435
        v3 o, d;
        camera_ray(F, seed, &o, &d);
        S.rng = seed;                                                         // :307
        S.thr = mk(1.0f, 1.0f, 1.0f);
        S.rad = mk(0.0f, 0.0f, 0.0f);
        S.depth = 0;
        bool need = P.max_depth > 0;
        for (int i = 0; i < P.n_lights && !need; ++i) {
          float tl;
          need = intersect_area_light(o, d, load_light(P, i), &tl);
        }
        if (need) {
          trav_start(T, o, d, false, 0.0f);
          S.phase = PH_PRIMARY;
          return true;
        }
        finished = true;   // no light in view and max_depth 0: radiance 0
        break;
      }
      case PH_PRIMARY: {
        // light pre-pass (:311-328) on the same ray, then depth 0 (:333)
        bool lit = false;
        for (int i = 0; i < P.n_lights; ++i) {
          const LightDev L = load_light(P, i);
          float tl;
          if (intersect_area_light(T.o, T.d, L, &tl)) {
            if (STATS) { c.rays++; c.nodes += T.cn; c.leaves += T.cl; }
            if (T.res < 0 || T.lim > tl) {
              color = mk(L.inten[0], L.inten[1], L.inten[2]);
              lit = true;
              break;
            }
          }
        }
        if (lit) { finished = true; break; }
        if (P.max_depth == 0) { color = S.rad; finished = true; break; }
        if (STATS) { c.rays++; c.nodes += T.cn; c.leaves += T.cl; }
        S.phase = PH_BOUNCE;   // handled as the result of a closest-hit trace at depth S.depth
        continue;
      }
      case PH_BOUNCE: {
        if (S.depth > 0 && STATS) { c.rays++; c.nodes += T.cn; c.leaves += T.cl; }
        if (T.res < 0) {
          S.rad = add(S.rad, mul(S.thr, mk(0.0f, 0.0f, 0.0f)));   // background (:336)
          color = S.rad;
          finished = true;
          break;
        }
        S.hp = add(T.o, muls(T.d, T.lim));
        S.hn = tri_normal(P, T.res);
        S.acc3 = mk(0.0f, 0.0f, 0.0f);   // directLight
        S.li = 0;
        S.phase = PH_DIRECT;
        S.k = -1;                         // marks "no shadow ray returned yet"
        continue;
      }
      case PH_DIRECT: {
        if (S.k >= 0) {   // a shadow ray for light S.li has returned
          if (STATS) { c.rays++; c.nodes += T.cn; c.leaves += T.cl; }
          if (!T.res) S.acc3 = add(S.acc3, mul(albedo, S.pend));
          S.li++;
        }
        if (S.li < P.n_lights) {                                            // :345-366
          const LightDev L = load_light(P, S.li);
          const v3 lp = sample_area_light(L, &S.rng);
          const v3 ld = normalize(sub(lp, S.hp));
          const float diff = fmax_(dot(S.hn, ld), 0.0f);
          const float dist = length(sub(lp, S.hp));
          const float d2 = dist * dist;
          S.pend = muls(muls(mk(L.inten[0], L.inten[1], L.inten[2]), diff), rcp_(fmax_(d2, 0.01f)));
          S.k = 0;
          trav_start(T, add(S.hp, muls(S.hn, OFFSET)), ld, true, dist - OFFSET);
          if (!STATS && !shadow_needed(L, diff)) trav_null(P, T);
          return true;
        }
        S.rad = add(S.rad, mul(S.thr, S.acc3));
        // SSS walk (:371-408): the first direction is drawn even if no step runs
        S.sss_thr = mk(1.0f, 1.0f, 1.0f);
        S.so = sub(S.hp, muls(S.hn, OFFSET));
        S.sd = sample_sphere(&S.rng);
        S.k = 0;
        if (S.k < P.sss_bounces) {
          trav_start(T, S.so, S.sd, false, 0.0f);
          S.phase = PH_SSS;
          return true;
        }
        S.phase = -1;   // to the bounce
        break;
      }
      case PH_SSS: {
        if (STATS) { c.rays++; c.nodes += T.cn; c.leaves += T.cl; }
        if (T.res < 0) { S.phase = -1; break; }                           // :381 miss ends the walk
        S.travel = T.lim;
        S.cp = add(S.so, muls(S.sd, S.travel));
        S.sn = tri_normal(P, T.res);
        S.acc3 = mk(0.0f, 0.0f, 0.0f);   // sssLight
        S.li = 0;
        S.phase = PH_SSS_SHADOW;
        if (P.n_lights > 0) {
          const LightDev L = load_light(P, 0);
          const v3 lp = sample_area_light(L, &S.rng);
          const v3 ed = normalize(sub(lp, S.cp));
          const float ediff = fmax_(dot(S.sn, ed), 0.0f);
          const float edist = length(sub(lp, S.cp));
          const float d2 = edist * edist;
          S.pend = muls(mul(muls(sss_albedo, ediff), mk(L.inten[0], L.inten[1], L.inten[2])), rcp_(fmax_(d2, 0.01f)));
          trav_start(T, add(S.cp, muls(S.sn, OFFSET)), ed, true, edist - OFFSET);
          if (!STATS && !shadow_needed(L, ediff)) trav_null(P, T);
          return true;
        }
        continue;
      }
      case PH_SSS_SHADOW: {
        if (S.li < P.n_lights) {   // the shadow ray for light S.li returned
          if (STATS) { c.rays++; c.nodes += T.cn; c.leaves += T.cl; }
          if (!T.res) S.acc3 = add(S.acc3, S.pend);
          S.li++;
        }
        if (S.li < P.n_lights) {
          const LightDev L = load_light(P, S.li);
          const v3 lp = sample_area_light(L, &S.rng);
          const v3 ed = normalize(sub(lp, S.cp));
          const float ediff = fmax_(dot(S.sn, ed), 0.0f);
          const float edist = length(sub(lp, S.cp));
          const float d2 = edist * edist;
          S.pend = muls(mul(muls(sss_albedo, ediff), mk(L.inten[0], L.inten[1], L.inten[2])), rcp_(fmax_(d2, 0.01f)));
          trav_start(T, add(S.cp, muls(S.sn, OFFSET)), ed, true, edist - OFFSET);
          if (!STATS && !shadow_needed(L, ediff)) trav_null(P, T);
          return true;
        }
        S.rad = add(S.rad, muls(mul(mul(S.thr, S.sss_thr), S.acc3), 1.0f + sss_radius * 0.5f));
        S.sss_thr = mul(S.sss_thr, muls(sss_albedo, exp_(-S.travel / (sss_radius * 1.5f))));
        S.so = sub(S.cp, muls(S.sn, OFFSET));
        S.sd = sample_sphere(&S.rng);
        S.k++;
        if (S.k < P.sss_bounces) {
          trav_start(T, S.so, S.sd, false, 0.0f);
          S.phase = PH_SSS;
          return true;
        }
        S.phase = -1;
        break;
      }
      default:
        break;
    }
    if (!finished && S.phase == -1) {
      // indirect bounce (:411-414)
      const v3 bd = sample_hemisphere(S.hn, &S.rng);
      S.thr = mul(S.thr, muls(albedo, dot(S.hn, bd)));
      const v3 ro = add(S.hp, muls(S.hn, OFFSET));
      S.depth++;
      if (S.depth < P.max_depth) {
        trav_start(T, ro, bd, false, 0.0f);
        S.phase = PH_BOUNCE;
        return true;
      }
      color = S.rad;
      finished = true;
    }
    if (finished) {
      *out = color;
      return false;
    }
  }
}

// ===========================================================================
// Wavefront pipeline, for scenes too large for LDS.
//
// Measured on the 1080p displaced sphere (16.6M paths): the path-recursive
// kernel keeps 11 % of its lanes busy (VALUUtilization) with L2 hit rate 92 %
// and no memory stall — the wave waits for its longest walk.  Here every
// (pixel, sample) path lives in HBM (PathSt, 160 B) and the work is split by
// kind: a persistent traversal kernel whose lanes pull waiting paths from a
// list and refill as soon as their walk ends (uniform code, ~20 live VGPRs),
// and a shading kernel that consumes the hits with path_step() and appends
// the paths that need another ray to the next list.  Each path's arithmetic,
// RNG draws and traversal order are those of path_trace(); the colours are
// folded per pixel in batch order at the end, so the image is bit-identical.
// ===========================================================================
// A waiting path's state travels with its ray: list slot s holds both, each
// stored by component (chunk j of the state at state[list][j * cap + s]; the
// ray at rays[list][s] and rays[list][cap + s]).  A wave reads and writes
// consecutive slots, so every access instruction covers consecutive 16-B
// words.  (Indexed by path, the state of a list's sparse surviving paths
// cost 64 lines per instruction and a dependent load of the path id first;
// by path and by component it measured +2.5 % / +4 %.)
//
// Only the fields the phase the path waits in reads again are stored, in
// chunks of 4 words, a prefix per phase (the 160-B PathSt lives in registers
// only):
//   c0 {s, rng, phase, depth}       c1 {thr.xyz, rad.x}
//   c2 {rad.yz, li | sss_thr.z, k}  c3 {hp.xyz, hn.x}
//   c4 {hn.yz, acc3.xy | sss_thr.xy}
//   c5 {acc3.z, pend.xyz}           c6 {sss_thr.xyz, travel}
//   c7 {cp.xyz, sn.x}               c8 {sn.yz, -, -}
// PH_PRIMARY: c0 (thr = 1, rad = 0, depth = 0: PH_BEGIN's values); PH_BOUNCE:
// c0-c2; PH_SSS: c0-c4 with sss_thr in the li / acc3 words (li and acc3 are
// set again before they are read; the walk ray's origin and direction are
// S.so / S.sd bitwise, restored from the ray record); PH_DIRECT: c0-c5;
// PH_SSS_SHADOW: c0-c8.  With the fused shadow walks a path mostly waits in
// PH_BOUNCE / PH_SSS: 48 / 80 B stored and loaded instead of 160.
__device__ __forceinline__ int wf_state_chunks(int phase) {
  return phase == PH_PRIMARY ? 1 : phase == PH_BOUNCE ? 3 : phase == PH_SSS ? 5 : phase == PH_DIRECT ? 6 : 9;
}

__device__ __forceinline__ void wf_store_state(const WfBuffers& B, int list, long long slot, const PathSt& S) {
  float4* __restrict__ dst = B.state[list] + slot;
  const size_t cap = (size_t)B.cap;
  const bool sss = S.phase == PH_SSS;
  const int n = wf_state_chunks(S.phase);
  dst[0] = make_float4(__uint_as_float(S.s), __uint_as_float(S.rng), __int_as_float(S.phase), __int_as_float(S.depth));
  if (n > 1) {
    dst[cap] = make_float4(S.thr.x, S.thr.y, S.thr.z, S.rad.x);
    dst[2 * cap] = make_float4(S.rad.y, S.rad.z, sss ? S.sss_thr.z : __int_as_float(S.li), __int_as_float(S.k));
  }
  if (n > 3) {
    dst[3 * cap] = make_float4(S.hp.x, S.hp.y, S.hp.z, S.hn.x);
    dst[4 * cap] = sss ? make_float4(S.hn.y, S.hn.z, S.sss_thr.x, S.sss_thr.y)
                       : make_float4(S.hn.y, S.hn.z, S.acc3.x, S.acc3.y);
  }
  if (n > 5) dst[5 * cap] = make_float4(S.acc3.z, S.pend.x, S.pend.y, S.pend.z);
  if (n > 6) {
    dst[6 * cap] = make_float4(S.sss_thr.x, S.sss_thr.y, S.sss_thr.z, S.travel);
    dst[7 * cap] = make_float4(S.cp.x, S.cp.y, S.cp.z, S.sn.x);
    dst[8 * cap] = make_float4(S.sn.y, S.sn.z, 0.0f, 0.0f);
  }
}

// o, d: the path's waiting ray (PH_SSS: S.so, S.sd).  Every field is
// assigned (chunks a phase does not store read as 0), so the state stays in
// registers.
__device__ __forceinline__ void wf_load_state(const WfBuffers& B, int list, long long slot, v3 o, v3 d, PathSt* S) {
  const float4* __restrict__ src = B.state[list] + slot;
  const size_t cap = (size_t)B.cap;
  float4 c[kWfStateF4];
  c[0] = src[0];
  const int phase = __float_as_int(c[0].z);
  const int n = wf_state_chunks(phase);
#pragma unroll
  for (int j = 1; j < kWfStateF4; ++j) c[j] = j < n ? src[(size_t)j * cap] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
  const bool prim = n == 1, sss = phase == PH_SSS;
  S->s = __float_as_uint(c[0].x);
  S->rng = __float_as_uint(c[0].y);
  S->phase = phase;
  S->depth = __float_as_int(c[0].w);
  S->thr = prim ? mk(1.0f, 1.0f, 1.0f) : mk(c[1].x, c[1].y, c[1].z);
  S->rad = prim ? mk(0.0f, 0.0f, 0.0f) : mk(c[1].w, c[2].x, c[2].y);
  S->li = __float_as_int(c[2].z);
  S->k = __float_as_int(c[2].w);
  S->hp = mk(c[3].x, c[3].y, c[3].z);
  S->hn = mk(c[3].w, c[4].x, c[4].y);
  S->acc3 = mk(c[4].z, c[4].w, c[5].x);
  S->pend = mk(c[5].y, c[5].z, c[5].w);
  S->sss_thr = sss ? mk(c[4].z, c[4].w, c[2].z) : mk(c[6].x, c[6].y, c[6].z);
  S->travel = c[6].w;
  S->so = o;
  S->sd = d;
  S->cp = mk(c[7].x, c[7].y, c[7].z);
  S->sn = mk(c[7].w, c[8].x, c[8].y);
}

// bits: kRayFuse / kRayPrimary (fuse_bits); the limit word of a fused
// closest ray (whose limit is always 1e30) carries the path's RNG state
__device__ __forceinline__ void wf_store_ray(float4* __restrict__ rays, long long cap, int slot, const Trav& T,
                                             int bits = 0, uint32_t rng = 0u) {
  rays[slot] = make_float4(T.o.x, T.o.y, T.o.z, bits ? __uint_as_float(rng) : T.lim);
  rays[(size_t)cap + (size_t)slot] = make_float4(T.d.x, T.d.y, T.d.z, __int_as_float(T.shadow | bits));
}

__device__ __forceinline__ void wf_load_ray(const float4* __restrict__ rays, long long cap, int slot, float4* r0,
                                            float4* r1) {
  *r0 = rays[slot];
  *r1 = rays[(size_t)cap + (size_t)slot];
}

// A list slot for every lane with pred set (-1 for the others): one atomic
// per wave, consecutive slots in lane order.
__device__ __forceinline__ int wave_slot(int* counter, bool pred) {
  const unsigned long long m = __ballot(pred);
  if (m == 0ull) return -1;
  const int lane = (int)__lane_id();
  const int leader = __ffsll((unsigned long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(counter, (int)__popcll(m));
  base = __shfl(base, leader);
  return pred ? base + (int)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

// PT_OPT_WF_FUSE: which closest rays the trace kernel follows with the
// path's next shadow ray.  After the hit of a primary (unless the light
// pre-pass ends the path), bounce or SSS ray, pathTrace's next draws sample
// light 0 (PH_DIRECT :345-366, PH_SSS_SHADOW :383-402) from the state the
// path holds now, and the shadow ray depends only on the hit and those draws.
__device__ __forceinline__ int fuse_bits(const RenderParams& P, const PathSt& S, const Trav& T) {
  if (!P.wf_fuse || T.shadow != 0) return 0;
  if (S.phase == PH_PRIMARY) return P.max_depth > 0 ? kRayFuse | kRayPrimary : 0;
  return (S.phase == PH_BOUNCE || S.phase == PH_SSS) ? kRayFuse : 0;
}

__device__ __forceinline__ void wf_push(const WfBuffers& B, int list, int slot, int p, const Trav& T, int bits = 0,
                                        uint32_t rng = 0u) {
  B.ids[list][slot] = p;
  wf_store_ray(B.rays[list], B.cap, slot, T, bits, rng);
}

// Path g of a launch: pixel (item, q) = g / n_batches, sample g % n_batches
// (samples of a pixel adjacent, so the fold reads them contiguously).
__device__ __forceinline__ bool wf_pixel(const RenderParams& P, long long pp, int* px, int* py) {
  const int spl = P.spl, per = 256 / spl;
  const int idx = (int)(pp / per), q = (int)(pp % per);
  const int item = P.items ? P.items[idx] : idx;
  const int tile = rank_tile(P, item / spl), part = item % spl;
  int bx, by;
  tile_block(tile, P.blocks_x, &bx, &by);
  *px = bx * 16 + q % 16;
  *py = by * 16 + part * (16 / spl) + q / 16;
  return tile < P.blocks_total && *px < P.width && *py < P.height;
}

// render_kernel's per-pixel culling test, same float ops.
__device__ __forceinline__ bool pixel_live(const RenderParams& P, float ndcX0, float ndcY0) {
  if (P.n_cull < 0) return true;
  bool live = false;
#pragma unroll
  for (int r = 0; r < kMaxCullRects; ++r)
    live = live || (r < P.n_cull && ndcX0 >= P.cull[r][0] && ndcX0 <= P.cull[r][1] && ndcY0 >= P.cull[r][2] &&
                    ndcY0 <= P.cull[r][3]);
  return live;
}

#ifndef PT_WF_GEN_BLOCK_SLOTS
#define PT_WF_GEN_BLOCK_SLOTS 1
#endif
// Ray generation + shading up to the primary trace (path_step from PH_BEGIN).
template <bool CNT>
__global__ __launch_bounds__(256) void wf_gen_kernel(RenderParams P, WfBuffers B, long long n, long long g0) {
  const long long g = g0 + (long long)blockIdx.x * 256 + threadIdx.x;   // paths [g0, g0 + n)
  bool need = false, gen = false;
  Trav T;
  PathSt S;
  if (g - g0 < n) {
    const long long pp = g / (long long)P.n_batches;
    CamFrame F;
    if (wf_pixel(P, pp, &F.px, &F.py)) {
      F.W = P.width;
      F.H = P.height;
      F.cpos = mk(P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]);
      F.cdir = mk(P.cam_dir[0], P.cam_dir[1], P.cam_dir[2]);
      F.ndcX0 = (2.0f * (float)F.px / (float)F.W) - 1.0f;
      F.ndcY0 = (2.0f * (float)F.py / (float)F.H) - 1.0f;
      F.aspect = (float)F.W / (float)F.H;
      F.right = mk(P.cam_right[0], P.cam_right[1], P.cam_right[2]);
      F.up = mk(P.cam_upv[0], P.cam_upv[1], P.cam_upv[2]);
      F.tanFov = P.tan_fov;
      v3 col = mk(0.0f, 0.0f, 0.0f);
      if (pixel_live(P, F.ndcX0, F.ndcY0)) {
        gen = true;
        S.s = (uint32_t)(g - pp * (long long)P.n_batches);
        S.phase = PH_BEGIN;
        Ctr c = {0u, 0u, 0u, 0u, 0u};
        need = path_step<false>(P, F, S, T, c, &col);
      }
      if (!need) B.colors[g] = make_float4(col.x, col.y, col.z, 1.0f);
    }
  }
  // list slots: one atomic per workgroup (PT_WF_GEN_BLOCK_SLOTS) instead of
  // one per wave -- the generation is otherwise short, and every wave of the
  // launch adding to the same counter queued on that one address
  int slot;
  if (PT_WF_GEN_BLOCK_SLOTS) {
    __shared__ int wave_n[4], wave_base[4];
    const unsigned long long m = __ballot(need);
    const int w = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
    if (lane == 0) wave_n[w] = (int)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
      const int tot = wave_n[0] + wave_n[1] + wave_n[2] + wave_n[3];
      const int base = tot ? atomicAdd(&B.counters[0], tot) : 0;
      wave_base[0] = base;
      wave_base[1] = base + wave_n[0];
      wave_base[2] = base + wave_n[0] + wave_n[1];
      wave_base[3] = base + wave_n[0] + wave_n[1] + wave_n[2];
    }
    __syncthreads();
    slot = wave_base[w] + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  } else {
    slot = wave_slot(&B.counters[0], need);
  }
  if (need) {
    wf_push(B, 0, slot, (int)g, T, fuse_bits(P, S, T), S.rng);
    wf_store_state(B, 0, slot, S);
  }
  if (CNT) {
    const unsigned long long m = __ballot(gen);
    if (__lane_id() == 0 && m) atomicAdd(&P.stats[8], (unsigned long long)__popcll(m));
  }
}

// Traversal state of one lane of the persistent traversal kernel: the ray,
// the walk position and the node at it (loaded one step ahead, as in
// trace_closest).
struct WfLane {
  v3 o, d, inv;
  float4 a, b;   // node k
  int k, nc, res, shadow;
  float lim;
};

// CNT: a ray handed to the traversal kernel -- closest (kind 0) or shadow
// (kind 1) walk; a null shadow query (kind 2, trav_null) is no walk.
__device__ __forceinline__ void count_start(float4 r1, Ctr& c) {
  const int kind = __float_as_int(r1.w) & kRayKindMask;
  c.rays += kind == 0 ? 1u : 0u;
  c.srays += kind == 1 ? 1u : 0u;
}

__device__ __forceinline__ void wf_lane_start(const RenderParams& P, float4 r0, float4 r1, float4 root_a,
                                              float4 root_b, WfLane& L) {
  L.o = mk(r0.x, r0.y, r0.z);
  L.d = mk(r1.x, r1.y, r1.z);
  L.inv = mk(rcp_(L.d.x), rcp_(L.d.y), rcp_(L.d.z));
  const int kind = __float_as_int(r1.w);   // 0 closest, 1 shadow, 2 null shadow (trav_null)
  L.shadow = kind ? 1 : 0;
  L.lim = L.shadow ? r0.w : 1e30f;
  L.res = L.shadow ? 0 : -1;
  L.k = kind == 2 ? P.n_nodes : 0;
  L.nc = 0;
  L.a = root_a;
  L.b = root_b;
}

// One node of trace_closest / occluded (same visit order and tests); true
// when the ray is finished (L.lim / L.res hold the result).
template <bool PF, bool CNT = false>
__device__ __forceinline__ bool wf_lane_step(const RenderParams& P, WfLane& L, int* cand, Ctr& c) {
  if (L.k >= P.n_nodes) {
    if (!L.shadow)
      test_candidates(P, L.o, L.d, cand, L.nc, &L.lim, &L.res);
    else if (PT_WF_SHADOW_QUEUE && L.nc > 0)
      L.res = test_shadow_candidates(P, L.o, L.d, L.lim, cand, L.nc) ? 1 : L.res;
    return true;
  }
  if (CNT) c.nodes++;
  float4 na, nb;
  if (PF) {
    na = P.nodes[2 * L.k + 2];
    nb = P.nodes[2 * L.k + 3];
  }
  const int raw = __float_as_int(L.a.w);
  const bool h = slab(L.o, L.inv, L.a, L.b) || (raw < 0);
  const int tri = __float_as_int(L.b.w);
  const bool leaf_hit = h && tri >= 0;
  if (CNT) c.leaves += leaf_hit ? 1u : 0u;
  if (L.shadow && !PT_WF_SHADOW_QUEUE) {
    if (leaf_hit) {
      const float4* T = P.tris + 3 * tri;
      float t;
      if (tri_test(L.o, L.d, T[0], T[1], T[2], &t) && t < 1e30f && !(t >= L.lim)) {
        L.res = 1;
        return true;
      }
    }
  } else {
    cand[L.nc * 64] = tri;
    L.nc += leaf_hit ? 1 : 0;
    if (!PT_WF_WAVEFLUSH && !L.shadow && L.nc == kCand) {
      test_candidates(P, L.o, L.d, cand, L.nc, &L.lim, &L.res);
      L.nc = 0;
    }
  }
  const int next = (h && tri < 0) ? L.k + 1 : (raw & 0x7fffffff);
  if (PF && next == L.k + 1) {
    L.a = na;
    L.b = nb;
  } else {
    L.a = P.nodes[2 * next];
    L.b = P.nodes[2 * next + 1];
  }
  L.k = next;
  return false;
}

// Persistent traversal over list `cur`: lanes pull list slots (one atomic per
// wave) and refill once at least PT_WF_REFILL lanes are idle.
//
// PT_WF_WAVEFLUSH: closest-hit candidates are tested wave-wide -- as soon as
// one lane's queue is full, every lane with queued candidates tests them in
// the same loop -- instead of by each full lane alone while the other lanes
// of the wave wait (round-1 counters on the sphere: ~10 of 64 lanes active
// per VALU instruction in wf_trace_kernel).  Same candidates, same visit
// order, same strict '<': the same hit.  1080p8 displaced sphere 378 -> 289
// ms, 1M cloud +0.5 %.
// PT_WF_SHADOW_QUEUE: shadow rays queue their hit leaves as well instead of
// testing each at once in a branch the other lanes wait on; the wave-wide
// flush tests them in visit order and ends the walk at the first occluder.
// The answer ("some accepted triangle has !(t >= limit)") is the same; the
// walk may visit a few nodes past that occluder before the flush finds it.
// Sphere 288 -> 242 ms, 1M cloud 636 -> 602.  (With it, the counting mode's
// triangle tests and nodes of shadow walks are the queued ones.)
#ifndef PT_WF_STEPS
#define PT_WF_STEPS 8
#endif

#ifndef PT_WF_REFILL
#define PT_WF_REFILL 32   // 1080p8: sphere -3.3 %, 1M cloud -2.0 % vs 16 (with the shadow queue); 48: +1.3 % / -0.3 %
#endif
// Refill group: lanes refill in groups of G with consecutive list slots.  G
// is chosen per launch (launch_wavefront): 2 for scenes under kWfGroup4Tris
// triangles, 4 above.  Measured at 1080p 8 spp, G = 2 vs 4: displaced sphere
// (82K) -4.6 %, random clouds 100K +3.4 % and 1M (4 spp) +3 %: a coherent
// surface gains, a random cloud loses; the threshold puts the BASELINE
// configs (sphere; 10M cloud) on their better side.
constexpr int kWfGroup4Tris = 500000;
template <int G>
constexpr unsigned long long group_lead() {
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 16, "refill group: power of two");
  return G == 1 ? ~0ull : G == 2 ? 0x5555555555555555ull : G == 4 ? 0x1111111111111111ull
                                    : G == 8 ? 0x0101010101010101ull : 0x0001000100010001ull;
}
#ifndef PT_WF_MIN_BLOCKS
#define PT_WF_MIN_BLOCKS 7   // 72 VGPRs (11 spilled): sphere -7 %, 1M cloud -0.6 % vs 6; 8 spills 30 (+50 %)
#endif
template <bool LDS, int G, bool CNT = false>
__global__ __launch_bounds__(256, PT_WF_MIN_BLOCKS) void wf_trace_kernel(RenderParams P, WfBuffers B, int cur) {
  const int tid = (int)threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) B.counters[cur ^ 1] = 0;   // filled by the shading that follows
  const int count = B.counters[cur];
  if (count == 0) return;
  if (LDS) {
    extern __shared__ float4 lds_scene[];
    const int nn = 2 * P.n_nodes, nt = 3 * P.n_tris;
    for (int i = tid; i < nn; i += 256) lds_scene[i] = P.nodes[i];
    for (int i = tid; i < nt; i += 256) lds_scene[nn + i] = P.tris[i];
    __syncthreads();
    P.nodes = lds_scene;
    P.tris = lds_scene + nn;
    P.hit_tris = P.tris;   // no wide walk here: hits are slots
  }
  const int wave = tid >> 6, lane = tid & 63;
  __shared__ int cand_buf[4][kCand][64];
  int* cand = &cand_buf[wave][0][lane];
  const float4* __restrict__ rays = B.rays[cur];
  // every walk starts at node 0: held in scalar registers
  float4 root_a = P.nodes[0], root_b = P.nodes[1];
  root_a.x = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_a.x)));
  root_a.y = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_a.y)));
  root_a.z = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_a.z)));
  root_a.w = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_a.w)));
  root_b.x = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_b.x)));
  root_b.y = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_b.y)));
  root_b.z = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_b.z)));
  root_b.w = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(root_b.w)));
  int p = -1;   // list slot this lane traces
  bool more = true;
  WfLane L;
  Ctr c = {0u, 0u, 0u, 0u, 0u};
  for (;;) {
    const unsigned long long idle = __ballot(p < 0);
    // groups of G lanes refill together with consecutive list
    // slots (neighbouring paths: the same pixel's samples), so their walks
    // stay as coherent as the path-recursive kernel's sample lanes
    unsigned long long gm = idle;
#pragma unroll
    for (int sh = 1; sh < G; sh <<= 1) gm &= gm >> sh;
    gm &= group_lead<G>();
    const int ng = (int)__popcll(gm);
    if (more && ng * G >= PT_WF_REFILL) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&B.counters[2], ng * G);
      base = __shfl(base, 0);
      if (base + ng * G >= count) more = false;
      const int lead = lane & ~(G - 1);
      if ((gm >> lead) & 1ull) {
        const int slot = base + (int)__popcll(gm & ((1ull << lead) - 1ull)) * G + (lane - lead);
        if (slot < count) {
          p = slot;
          float4 r0, r1;
          wf_load_ray(rays, B.cap, slot, &r0, &r1);
          wf_lane_start(P, r0, r1, root_a, root_b, L);
          if (CNT) count_start(r1, c);
        }
      }
    }
    if (!more && __ballot(p >= 0) == 0ull) break;
    for (int it = 0; it < PT_WF_STEPS; ++it) {
      if (p >= 0 && wf_lane_step<PT_WF_PF && !LDS, CNT>(P, L, cand, c)) {
        B.hits[p] = make_float2(L.lim, __int_as_float(L.res));
        p = -1;
      }
      if (PT_WF_WAVEFLUSH && __ballot(p >= 0 && L.nc == kCand)) {   // wave-uniform
        if (p >= 0 && L.nc > 0) {
          if (!L.shadow) {
            test_candidates(P, L.o, L.d, cand, L.nc, &L.lim, &L.res);
          } else if (test_shadow_candidates(P, L.o, L.d, L.lim, cand, L.nc)) {
            L.res = 1;
            L.k = P.n_nodes;   // occluded: the walk ends (its next step reports it)
          }
          L.nc = 0;
        }
      }
    }
  }
  if (CNT) flush_traced(P, c, lane);
}

// ---------------------------------------------------------------------------
// Culled wide walk (wide_walk.h) for scenes in device memory: 4-wide nodes of
// the reference's own boxes, nearest child first, children culled once no
// triangle in them can beat (or tie) the best hit -- the same answer as the
// exhaustive DFS, far fewer node fetches (CPU harness, 1M-triangle cloud,
// camera rays: 42 wide nodes and 4.3 triangle tests per ray against 1022
// nodes and 31 leaf tests).  Per lane: the ray, the node to expand, and a
// stack of pending (node, cull threshold) entries -- the top kWideLds in LDS
// ([entry][lane], conflict-free), older ones in a per-lane global overflow
// area (P.wide_ovf, strided by lane so neighbouring lanes' spills coalesce).
// Rays the walk does not take (zero / subnormal direction components) return
// kNeedExact* and wf_shade_kernel walks them exactly (trace_closest /
// occluded).
// ---------------------------------------------------------------------------
// Refill group of the wide walk: single lanes (G = 1).  Lane census of the
// wide walk with G = 4 on the 10M cloud: 56 % of lane-steps idle while the
// list still held rays -- a lane could refill only once its whole aligned
// group of four was idle.  G = 1 vs the earlier choice (2 below 500K
// triangles, 4 above): sphere 78.0 -> 75.1 ms, 10M cloud 237 -> 206 ms;
// the refill threshold is P.wide_refill (PT_OPT_WF_REFILL; PT_WIDE_REFILL for
// the tail kernel).
#ifndef PT_WIDE_G
#define PT_WIDE_G 1
#endif
// refill threshold of the wide walk: 16 idle lanes.  Before the finished
// walks were batched at the refill check (PT_WIDE_DEFER_DONE), 24 measured
// best (sphere -0.9 %, 10M cloud -0.35 % against 32; 16 then +3 %); with
// them batched, 16 against 24: sphere -2 %, 10M cloud -1.5 % (DESIGN item
// 36); 12: +0.2 % / +4 %, 8: +7 % / +31 %.
#ifndef PT_WIDE_REFILL
#define PT_WIDE_REFILL 16
#endif
// steps between the wide walk's refill checks: 12 (with the wave-wide flush,
// item 39): 10M cloud -1.7 %, sphere -0.1 % against 8; 16: -0.5 % / +0.6 %
#ifndef PT_WIDE_STEPS
#define PT_WIDE_STEPS 12
#endif
constexpr int kWideG = PT_WIDE_G;
#ifndef PT_WIDE_DEFER_DONE
#define PT_WIDE_DEFER_DONE 1
#endif
#ifndef PT_WIDE_FLUSH_T
#define PT_WIDE_FLUSH_T 1
#endif
#ifndef PT_WIDE_MIN_BLOCKS
// 6: the LDS stack and leaf queue (96 B per lane) fit 6 workgroups per CU;
// 79 VGPRs, no spills.  8 workgroups with a 6-entry stack ring (80 B per lane,
// 64 VGPRs, 60 B spilled): sphere +6.5 %, 10M cloud +5.4 %; with 7: +1 %.
#define PT_WIDE_MIN_BLOCKS 6
#endif
// PT_OPT_WF_FUSE: the shadow ray pathTrace traces right after closest hit
// (t, rank) of ray (o, d), from the path's RNG state `rng` -- light 0's
// sample, direction, diffuse term and distance with the ops of path_step's
// PH_DIRECT / PH_SSS_SHADOW (:345-366, :383-402; the hit point o + d t is
// S.hp / S.cp, the normal the record's).  0: none (a primary ray's light
// pre-pass, :311-328, ends the path); 1: answered without a walk (its answer
// cannot change the image, shadow_needed); 2: walk (so, sd) up to lim.
__device__ __forceinline__ int fused_shadow_ray(const RenderParams& P, v3 o, v3 d, float t, int rank, bool primary,
                                                uint32_t rng, v3* so, v3* sd, float* lim) {
  if (primary) {
    for (int i = 0; i < P.n_lights; ++i) {
      float tl;
      if (intersect_area_light(o, d, load_light(P, i), &tl) && t > tl) return 0;   // lit: T.res >= 0 here
    }
  }
  const float OFFSET = 0.001f;
  const v3 hp = add(o, muls(d, t));
  const v3 hn = tri_normal(P, rank);
  const LightDev L = load_light(P, 0);
  const v3 lp = sample_area_light(L, &rng);
  const v3 ld = normalize(sub(lp, hp));
  const float diff = fmax_(dot(hn, ld), 0.0f);
  const float dist = length(sub(lp, hp));
  if (!shadow_needed(L, diff)) return 1;
  *so = add(hp, muls(hn, OFFSET));
  *sd = ld;
  *lim = dist - OFFSET;
  return 2;
}
constexpr int kFuseWalk = 16;   // lane state: walking the fused shadow ray

// PT_WIDE_FLUSH_WAVE: the wave's queued leaf candidates tested one per lane.
// wide_flush runs a lane's queue in its own lane, so a flush takes as many
// loop trips as the longest queue while the others idle: a probe of the trace
// kernel (tools/flush_probe.py) measured 67 candidates per flush on the
// displaced sphere and 38 on the 10M cloud, against a longest queue of 5.8 /
// 4.7 -- 18 % / 13 % of the flush loop's lane slots in use.  Here the
// candidates are numbered across the wave (a prefix sum of the queue
// lengths), and lane j of each window of 64 tests candidate j: it finds the
// owner by a binary search over the prefix sums, reads the rank from the
// owner's queue column, the owner's ray by lane shuffles, and runs the same
// triangle test and accept rules.  The owner's answer is a lexicographic
// minimum of (t, rank) -- an LDS atomic min of (t bits << 32 | rank), t > 0
// (tri_test accepts t > 1e-6), so its bits order as its value -- merged with
// the owner's best by wide_cand's own rule; a shadow ray is occluded if any
// of its candidates is an accepted hit below its limit.  Neither answer
// depends on the order the candidates are tested in (ties go to the lower
// rank, the reference's visit order): the same hits as wide_flush.  Call with
// every lane of the wave active; keys: the wave's 64 LDS words; returns true
// for a shadow ray found occluded.
#ifndef PT_WIDE_FLUSH_WAVE
#define PT_WIDE_FLUSH_WAVE 1
#endif
#ifndef PT_WIDE_OWNER3
#define PT_WIDE_OWNER3 0
#endif
// Inclusive prefix sum over the wave's 64 lanes (every lane active) by DPP
// row shifts within each row of 16 and row broadcasts across rows: six VALU
// steps, where __shfl_up made six dependent LDS-crossbar round trips.
__device__ __forceinline__ int wave_incl_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 into rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 into rows 2, 3
  return v;
}
template <bool CNT, bool QN>
__device__ __forceinline__ bool wide_flush_wave(WideRay& R, bool mine, const float4* __restrict__ tris, const int* cand,
                                                unsigned long long* keys, int lane, uint32_t* cl,
                                                const float4* __restrict__ leaf_box) {
  const int n = mine ? R.nc : 0;
  const int incl = wave_incl_sum(n);   // inclusive prefix sum of the queue lengths
  const int total = __builtin_amdgcn_readlane(incl, 63);
  const int off = incl - n;
  keys[lane] = ~0ull;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const int* qbase = cand - lane;   // the wave's queue: [k][lane]
#if PT_WIDE_OWNER3
  // the inclusive sums at the ends of the wave's four 16-lane blocks (the
  // last is `total`): wave-uniform, read once per flush
  const int e15 = __builtin_amdgcn_readlane(incl, 15), e31 = __builtin_amdgcn_readlane(incl, 31),
            e47 = __builtin_amdgcn_readlane(incl, 47);
#endif
  for (int base = 0; base < total; base += 64) {
    const int target = base + lane;
    int L = 0;   // the owner: lanes whose inclusive sum is <= target
#if PT_WIDE_OWNER3
    // The same count in two dependent LDS round trips instead of six (the
    // sums never decrease): whole 16-lane blocks by the uniform block ends,
    // then whole 4-lane groups inside the block, then lanes inside the group
    L = (e15 <= target ? 16 : 0) + (e31 <= target ? 16 : 0) + (e47 <= target ? 16 : 0);
    {
      const int a0 = __shfl(incl, L + 3), a1 = __shfl(incl, L + 7), a2 = __shfl(incl, L + 11);
      L += (a0 <= target ? 4 : 0) + (a1 <= target ? 4 : 0) + (a2 <= target ? 4 : 0);
      const int b0 = __shfl(incl, L), b1 = __shfl(incl, L + 1), b2 = __shfl(incl, L + 2);
      L += (b0 <= target ? 1 : 0) + (b1 <= target ? 1 : 0) + (b2 <= target ? 1 : 0);
    }
#else
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
      const int v = __shfl(incl, L + s - 1);
      if (v <= target) L += s;
    }
#endif
    L = min(L, 63);
    const int offL = __shfl(off, L);
    const v3 o = mk(__shfl(R.o.x, L), __shfl(R.o.y, L), __shfl(R.o.z, L));
    const v3 d = mk(__shfl(R.d.x, L), __shfl(R.d.y, L), __shfl(R.d.z, L));
    const float lim = __shfl(R.lim, L);
    const int shadow = __shfl(R.shadow, L);
    if (target < total) {
      const int r = wide_qrank(qbase[(target - offL) * 64 + L]);
      const float4* T = tris + 3 * (size_t)r;
      const float4 A = T[0], B = T[1], C = T[2];
      if (CNT) ++*cl;
      float t;
      // shadow: :359 / :398; closest: a hit that can still win (t == lim may
      // tie with a lower rank)
      if (tri_test(o, d, A, B, C, &t) && t < 1e30f && (shadow ? !(t >= lim) : t <= lim)) {
        bool ok = true;
        if (QN) ok = slab(o, mk(rcp_(d.x), rcp_(d.y), rcp_(d.z)), leaf_box[2 * (size_t)r], leaf_box[2 * (size_t)r + 1]);
        if (ok) atomicMin(&keys[L], shadow ? 0ull : ((unsigned long long)__float_as_uint(t) << 32) | (uint32_t)r);
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (n == 0) return false;
  R.nc = 0;
  const unsigned long long k = keys[lane];
  if (k == ~0ull) return false;
  if (R.shadow) {
    R.best = 1;
    return true;
  }
  const float tm = __uint_as_float((uint32_t)(k >> 32));
  const int rm = (int)(uint32_t)k;
  if (tm < R.lim || (tm == R.lim && R.best >= 0 && rm < R.best)) {   // wide_cand's rule
    R.lim = tm;
    R.best = rm;
  }
  return false;
}

// LAYOUT: 0 128-B 4-wide nodes, 1 64-B 4-wide nodes (QN)
template <int G, bool CNT = false, int LAYOUT = 1>
__global__ __launch_bounds__(256, PT_WIDE_MIN_BLOCKS) void wf_trace_wide_kernel(RenderParams P, WfBuffers B,
                                                                                int cur) {
  constexpr bool QN = LAYOUT >= 1;
  const int tid = (int)threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) B.counters[cur ^ 1] = 0;   // filled by the shading that follows
  const int count = B.counters[cur];
  if (count == 0 || count < P.wf_tail) return;   // PT_OPT_WF_TAIL: wf_tail_kernel finishes the list
  const int wave = tid >> 6, lane = tid & 63;
  __shared__ int2 stk[4][kWideLds][64];
  int2* lds = &stk[wave][0][lane];
  __shared__ int cq[PT_WIDE_QUEUE ? 4 : 1][PT_WIDE_QUEUE ? kWideQ : 1][64];
  int* cand = PT_WIDE_QUEUE ? &cq[wave][0][lane] : nullptr;
  constexpr bool FW = PT_WIDE_FLUSH_WAVE && PT_WIDE_QUEUE;
  __shared__ unsigned long long fkeys[FW ? 4 : 1][64];
  bool fin = false;
  const long long os = (long long)gridDim.x * 256;
  int2* ovf = P.wide_ovf + ((long long)blockIdx.x * 256 + tid);
  const float4* __restrict__ rays = B.rays[cur];
  int p = -1;   // list slot this lane traces
  bool more = true;
  WideRay R;
  R.cur = -1;
  R.sp = R.lo = 0;
  R.nc = 0;
  // PT_OPT_WF_FUSE: fz = the ray's kRayFuse / kRayPrimary bits, or kFuseWalk
  // while the lane walks the fused shadow ray; aux = the path's RNG state,
  // then the closest hit's t; cr = its rank
  int fz = 0, cr = 0;
  uint32_t aux = 0u;
  Ctr c = {0u, 0u, 0u, 0u, 0u};
  // A lane whose walk is over (fin, queue empty): its answer goes to the
  // hit list -- or, after a closest hit whose first-light shadow ray the
  // trace kernel walks (PT_OPT_WF_FUSE), that ray starts in the lane.
  auto finish = [&]() {
    float t = R.lim;
    int res = R.best;   // occluded, or the hit's rank (hit_tris = wide_tris; the record the flush just tested)
    bool done = true;
    if (fz & kFuseWalk) {   // the fused shadow ray's answer joins its closest hit
      t = __uint_as_float(aux);
      res = cr | kHitFused | (R.best ? kHitOccluded : 0);
    } else if ((fz & kRayFuse) && R.best >= 0) {
      v3 so, sd;
      float lim;
      const int k = fused_shadow_ray(P, R.o, R.d, R.lim, R.best, (fz & kRayPrimary) != 0, aux, &so, &sd, &lim);
      if (k == 1) {
        res = R.best | kHitFused;   // unoccluded without a walk
      } else if (k == 2) {
        cr = R.best;
        aux = __float_as_uint(R.lim);
        wide_start(R, so, sd, true, lim);
        if (wide_ray_ok(R.o, R.d, R.inv)) {   // walk it in this lane now
          fz = kFuseWalk;
          fin = false;
          done = false;
          if (CNT) ++c.srays;
        } else {   // the shading's next round hands it to the exact walk
          t = __uint_as_float(aux);
          res = cr;
        }
      }
    }
    if (done) {
      B.hits[p] = make_float2(t, __int_as_float(res));
      p = -1;
      fin = false;
      fz = 0;
    }
  };
  for (;;) {
    // PT_WIDE_DEFER_DONE: the lanes whose walks ended since the last check
    // finish here together, not in the step their walk ended in (where the
    // wave ran the finishing code -- the fused shadow ray's light sample,
    // normalisations and start -- for one or two lanes at a time)
    if (PT_WIDE_DEFER_DONE && p >= 0 && fin && R.nc == 0) finish();
    const unsigned long long idle = __ballot(p < 0);
    unsigned long long gm = idle;
#pragma unroll
    for (int sh = 1; sh < G; sh <<= 1) gm &= gm >> sh;
    gm &= group_lead<G>();
    const int ng = (int)__popcll(gm);
    if (more && ng * G >= P.wide_refill) {
      const int need = ng * G;
      int base = 0;
      if (lane == 0) base = atomicAdd(&B.counters[2], need);
      base = __shfl(base, 0);
      if (base + need >= count) more = false;
      const int lead = lane & ~(G - 1);
      if ((gm >> lead) & 1ull) {
        const int slot = base + (int)__popcll(gm & ((1ull << lead) - 1ull)) * G + (lane - lead);
        if (slot < count) {
          float4 r0, r1;
          wf_load_ray(rays, B.cap, slot, &r0, &r1);
          const int kbits = __float_as_int(r1.w);
          const int kind = kbits & kRayKindMask;   // 0 closest, 1 shadow, 2 null shadow (trav_null)
          if (CNT) count_start(r1, c);
          wide_start(R, mk(r0.x, r0.y, r0.z), mk(r1.x, r1.y, r1.z), kind != 0, r0.w);
          fz = kbits & (kRayFuse | kRayPrimary);
          aux = __float_as_uint(r0.w);
          if (kind == 2) {
            B.hits[slot] = make_float2(R.lim, __int_as_float(0));
          } else if (!wide_ray_ok(R.o, R.d, R.inv) || (P.wide_handback && (slot & 1))) {
            B.hits[slot] = make_float2(R.lim, __int_as_float(kind ? kNeedExactShadow : kNeedExactClosest));
          } else {
            p = slot;
          }
        }
      }
    }
    if (!more && __ballot(p >= 0) == 0ull) break;
    for (int it = 0; it < PT_WIDE_STEPS; ++it) {
      bool exact = false;
      if (!PT_WIDE_QUEUE) {
        if (p >= 0 && wide_step<CNT, false, QN>(R, P.wide, P.wide_tris, lds, 64, ovf, os, P.wide_stack, &exact,
                                                &c.nodes, &c.leaves, nullptr, P.wide_leafbox)) {
          int res;
          if (exact) res = R.shadow ? kNeedExactShadow : kNeedExactClosest;
          else if (R.shadow) res = R.best;
          else res = R.best;   // the rank (hit_tris = wide_tris)
          B.hits[p] = make_float2(R.lim, __int_as_float(res));
          p = -1;
        }
      } else {
        // fin: the walk has no node left (its queue may still hold candidates)
        if (p >= 0 && !fin)
          fin = wide_step<CNT, true, QN>(R, P.wide, P.wide_tris, lds, 64, ovf, os, P.wide_stack, &exact, &c.nodes,
                                         &c.leaves, cand, P.wide_leafbox);
        if (exact) {
          R.nc = 0;
          // a fused shadow ray the walk cannot take goes to the shading's next round
          B.hits[p] = (fz & kFuseWalk) ? make_float2(__uint_as_float(aux), __int_as_float(cr))
                                       : make_float2(R.lim, __int_as_float(R.shadow ? kNeedExactShadow
                                                                                    : kNeedExactClosest));
          p = -1;
          fin = false;
          fz = 0;
        }
        // wave-uniform flush: a queue that cannot take another node's four
        // leaves, or PT_WIDE_FLUSH_T finished walks waiting on their queue,
        // or nothing left walking
        const unsigned long long waiting = __ballot(p >= 0 && fin && R.nc > 0);
#ifdef PT_WIDE_PROBE_FLUSH
        if (lane == 0) atomicAdd(&P.stats[7], 1ull);
        if (lane == 0) atomicAdd(&P.stats[8], (unsigned long long)__popcll(__ballot(p >= 0 && !fin)));
#endif
#ifdef PT_WIDE_PROBE   // lane-state census per step (traced counters 0-4: walking, idle with rays left
                       // in the list, idle in the drain, steps, waiting on the leaf queue)
        {
          const unsigned long long walking = __ballot(p >= 0 && !fin), idle_l = __ballot(p < 0);
          if (lane == 0) {
            atomicAdd(&P.stats[4], (unsigned long long)__popcll(walking));
            atomicAdd(&P.stats[more ? 5 : 6], (unsigned long long)__popcll(idle_l));
            atomicAdd(&P.stats[7], 1ull);
            atomicAdd(&P.stats[8], (unsigned long long)__popcll(waiting));
          }
        }
#endif
        if (__ballot(p >= 0 && R.nc > kWideQ - 4) || (int)__popcll(waiting) >= PT_WIDE_FLUSH_T ||
            (waiting && __ballot(p >= 0 && !fin) == 0ull)) {
#ifdef PT_WIDE_PROBE_FLUSH   // flush loop use: [4] flushes, [5] sum of candidates, [6] sum of the largest queue, [7] steps
          {
            int mx = p >= 0 ? R.nc : 0, sm = mx;
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) {
              mx = max(mx, __shfl_xor(mx, o));
              sm += __shfl_xor(sm, o);
            }
            if (lane == 0) {
              atomicAdd(&P.stats[4], 1ull);
              atomicAdd(&P.stats[5], (unsigned long long)sm);
              atomicAdd(&P.stats[6], (unsigned long long)mx);
            }
          }
#endif
          if (FW ? wide_flush_wave<CNT, QN>(R, p >= 0, P.wide_tris, cand, fkeys[FW ? wave : 0], lane, &c.leaves,
                                            P.wide_leafbox)
                 : (p >= 0 && R.nc > 0 &&
                    wide_flush<CNT, QN>(R, P.wide_tris, cand, &c.leaves, P.wide_leafbox))) {
            fin = true;   // occluded
            R.sp = 0;
            R.cur = -1;
          }
        }
        if (!PT_WIDE_DEFER_DONE && p >= 0 && fin && R.nc == 0) finish();
        // every lane idle or done (PT_WIDE_DEFER_DONE): back to the refill check
        if (PT_WIDE_DEFER_DONE && __ballot(p >= 0 && !(fin && R.nc == 0)) == 0ull) break;
      }
    }
  }
  if (CNT) flush_traced(P, c, lane);
}

// Shading of every path in list `cur` (path_step on the returned hit);
// paths that need another ray go to list cur^1, finished ones store colour.
//
// PT_WF_SORT: a workgroup appends its next rays binned -- one atomic per
// workgroup, a counting sort in LDS -- by the phase the path waits in
// (PT_WF_SORT_PHASE; closest-hit and shadow rays apart, and the next shading
// pass runs one case of path_step per wave instead of several), or by ray
// kind and direction octant.  A ray's result does not depend on where it
// sits in the list, so the image is unchanged.  Measured at 1080p 8 spp with
// the wide walk (G = 1, null queries inline): sphere 70.7 -> 65.0 ms, 10M
// cloud 181.5 -> 158.0 ms by phase; by kind and octant 65.7 / 158.3; by
// phase and octant 65.7 / 159.1.  (With the exhaustive walks and refill
// groups of round 2's first half, kind and octant had measured sphere -0.5 %,
// 10M cloud +3.5 %; the exhaustive walk keeps the unsorted lists.)
[[maybe_unused]] __device__ __forceinline__ int ray_bin(const Trav& T) {
  const int oct = (T.d.x < 0.0f ? 1 : 0) | (T.d.y < 0.0f ? 2 : 0) | (T.d.z < 0.0f ? 4 : 0);
  return (T.shadow ? 8 : 0) | oct;
}
// PT_WF_NULL_INLINE: a null shadow query (trav_null: its answer cannot change
// the image) is answered by the shading kernel itself, with the wide walk --
// path_step runs on with "unoccluded" -- instead of taking a list slot, a refill and a lane of
// the next traversal launch (where it started finished and left its lane
// idle until the wave's next refill) and a second shading pass.  The path's
// arithmetic and draws are the same; it only reaches its next real ray a
// round earlier.  1080p 8 spp, wide walk: sphere 75.1 -> 70.6 ms, 10M cloud
// 206 -> 181 ms; with the exhaustive threaded walk (PT_OPT_WIDE 0) the 10M
// cloud measured 2799 -> 2980 ms (paths drift out of phase), so it keeps the
// null rays in its lists.
#ifndef PT_WF_NULL_INLINE
#define PT_WF_NULL_INLINE 1
#endif
#ifndef PT_WF_SHADE_MIN_BLOCKS
#define PT_WF_SHADE_MIN_BLOCKS 4
#endif
constexpr int kWfBins = 16;
__global__ __launch_bounds__(256, PT_WF_SHADE_MIN_BLOCKS) void wf_shade_kernel(RenderParams P, WfBuffers B, int cur) {
  if (blockIdx.x == 0 && threadIdx.x == 0) B.counters[2] = 0;   // the next traversal's cursor
  const int count = B.counters[cur];
  if (count < P.wf_tail) return;   // PT_OPT_WF_TAIL: wf_tail_kernel has finished these paths
  CamFrame F = {};   // camera frame: used by PH_BEGIN only
  __shared__ int bin_cnt[kWfBins], bin_base[kWfBins], wg_base;
  __shared__ int cand_buf[4][kCand][64];   // exact walks of handed-back rays
  int* cand = &cand_buf[threadIdx.x >> 6][0][threadIdx.x & 63];
  for (int base = (int)blockIdx.x * 256; base < count; base += (int)gridDim.x * 256) {
    const int i = base + (int)threadIdx.x;
    bool need = false;
    int p = -1;
    Trav T;
    PathSt S;
    if (i < count) {
      p = B.ids[cur][i];
      float4 r0, r1;
      wf_load_ray(B.rays[cur], B.cap, i, &r0, &r1);
      const float2 h = B.hits[i];
      T.o = mk(r0.x, r0.y, r0.z);
      T.d = mk(r1.x, r1.y, r1.z);
      wf_load_state(B, cur, i, T.o, T.d, &S);
      T.shadow = __float_as_int(r1.w) & kRayKindMask;
      T.lim = h.x;
      T.res = __float_as_int(h.y);
      int fused = 0;   // PT_OPT_WF_FUSE: 1 the path's next shadow ray was walked unoccluded, 2 occluded
      if (T.shadow == 0 && T.res >= 0 && (T.res & kHitFused)) {
        fused = (T.res & kHitOccluded) ? 2 : 1;
        T.res &= kHitRankMask;
      }
      T.nc = 0;
      T.cn = T.cl = 0u;
      Ctr c = {0u, 0u, 0u, 0u, 0u};
      if (T.shadow == 0 && T.res == kNeedExactClosest) {   // handed back by wf_trace_wide_kernel
        const Hit e = trace_closest<false, false, true, false>(P, T.o, T.d, c, cand);
        T.lim = e.t;
        T.res = e.tri >= 0 ? P.wide_rank_of[e.tri] : e.tri;   // a slot; hit_tris is by rank
      } else if (T.shadow == 1 && T.res == kNeedExactShadow) {
        T.res = occluded<false, false>(P, T.o, T.d, T.lim, c) ? 1 : 0;
      }
      v3 col;
      need = path_step<false>(P, F, S, T, c, &col);
      if (fused) {
        // the shading just derived the shadow ray the trace kernel walked
        // (same hit, same draws, same ops): take its answer
        if (need && T.shadow != 0) {
          T.res = T.shadow == 2 ? 0 : fused - 1;
          need = path_step<false>(P, F, S, T, c, &col);
        } else {   // cannot happen; fail loudly rather than shade wrongly
          need = false;
          col = mk(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
        }
      }
#if PT_WF_NULL_INLINE
      while (P.wide && need && T.shadow == 2) {   // a null shadow query (trav_null): unoccluded, answered here
        T.res = 0;
        need = path_step<false>(P, F, S, T, c, &col);
      }
#endif
      if (!need) B.colors[p] = make_float4(col.x, col.y, col.z, 1.0f);
    }
    if (PT_WF_SORT && P.wide) {   // uniform: every thread of the workgroup runs each iteration
      const int tid = (int)threadIdx.x;
      if (tid < kWfBins) bin_cnt[tid] = 0;
      __syncthreads();
#if PT_WF_SORT_PHASE
      const int bin = need ? (S.phase & 7) : 0;   // the phase the path waits in
#else
      const int bin = need ? ray_bin(T) : 0;
#endif
      const int rank = need ? atomicAdd(&bin_cnt[bin], 1) : 0;
      __syncthreads();
      if (tid == 0) {
        int acc = 0;
        for (int k = 0; k < kWfBins; ++k) {
          bin_base[k] = acc;
          acc += bin_cnt[k];
        }
        wg_base = acc ? atomicAdd(&B.counters[cur ^ 1], acc) : 0;
      }
      __syncthreads();
      if (need) {
        const int slot = wg_base + bin_base[bin] + rank;
        wf_push(B, cur ^ 1, slot, p, T, fuse_bits(P, S, T), S.rng);
        wf_store_state(B, cur ^ 1, slot, S);
      }
      __syncthreads();   // the bins are reused by the next iteration
    } else {
      const int slot = wave_slot(&B.counters[cur ^ 1], need);
      if (need) {
        wf_push(B, cur ^ 1, slot, p, T, fuse_bits(P, S, T), S.rng);
        wf_store_state(B, cur ^ 1, slot, S);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// PT_OPT_WF_TAIL: the last paths of a chunk in one launch.  Every ray round
// of the pipeline ends when its longest walk ends, and a path needs a round
// per ray it traces (up to 33 at MAX_DEPTH 4, 65 at 8).  Late rounds hold few
// rays -- on a 1/8 tile share only a few per traversal lane from the start --
// so each costs about one long walk's latency plus three launches while most
// of the GPU idles.  Once a round's list holds fewer than P.wf_tail rays, this
// kernel takes the whole list instead of the trace and shading kernels: each
// lane claims a waiting path (its list slot) and runs it to the end -- walk
// (the culled wide walk with the trace kernel's queued leaf tests and
// wave-wide flushes), then path_step, then the next ray's walk in the same
// lane -- and stores the path's colour; the lanes whose walks have ended
// shade together at the check every PT_WIDE_STEPS steps, as the trace kernel
// finishes its walks.  The path's state waits in its own list slot
// (wf_store_state / wf_load_state) while the lane walks, so the walk keeps
// the trace kernel's registers.  The rays, draws, float operations and their
// order per path are those of the rounds (path_step on each returned hit,
// null shadow queries answered unoccluded, rays the wide walk does not take
// walked exactly): the image is bit-identical; the trace and shading kernels
// of that round and every later round find nothing to do.  No fused shadow
// walks here: path_step derives each shadow ray itself.
#ifndef PT_WF_TAIL_MIN_BLOCKS
#define PT_WF_TAIL_MIN_BLOCKS 4
#endif
template <bool CNT, bool QN>
__global__ __launch_bounds__(256, PT_WF_TAIL_MIN_BLOCKS) void wf_tail_kernel(RenderParams P, WfBuffers B, int cur) {
  const int count = B.counters[cur];
  if (count == 0 || count >= P.wf_tail) return;
  const int tid = (int)threadIdx.x;
  const int wave = tid >> 6, lane = tid & 63;
  __shared__ int2 stk[4][kWideLds][64];
  int2* lds = &stk[wave][0][lane];
  // leaf queue; an exact walk's candidates (the queue is empty then)
  __shared__ int cq[4][kWideQ > kCand ? kWideQ : kCand][64];
  int* cand = &cq[wave][0][lane];
  __shared__ unsigned long long fkeys[PT_WIDE_FLUSH_WAVE ? 4 : 1][64];
  const long long os = (long long)gridDim.x * 256;
  int2* ovf = P.wide_ovf + ((long long)blockIdx.x * 256 + tid);
  const float4* __restrict__ rays = B.rays[cur];
  const CamFrame F = {};   // no path begins here
  int p = -1;              // list slot of the lane's path
  bool fin = false;        // the lane's walk is over (its queue may still hold candidates)
  bool more = true;
  WideRay R;
  R.cur = -1;
  R.sp = R.lo = 0;
  R.nc = 0;
  R.shadow = 0;
  R.lim = 0.0f;
  R.best = 0;
  Ctr c = {0u, 0u, 0u, 0u, 0u};
  // the reference's traversal of the lane's ray by the exact threaded walk
  // (a ray the wide walk does not take, wide_ray_ok, or a stack bound hit)
  auto exact_walk = [&]() {
    Ctr cx = {0u, 0u, 0u, 0u, 0u};
    if (!R.shadow) {
      const Hit e = trace_closest<false, false, true, false>(P, R.o, R.d, cx, cand);
      R.lim = e.t;
      R.best = e.tri >= 0 ? P.wide_rank_of[e.tri] : e.tri;   // a slot; hit_tris is by rank
    } else {
      R.best = occluded<false, false>(P, R.o, R.d, R.lim, cx) ? 1 : 0;
    }
    R.nc = 0;
    fin = true;
  };
  // the lane's next ray: kind 0 closest, 1 shadow, 2 null shadow query (its
  // answer cannot change the image: unoccluded, no walk)
  auto begin = [&](v3 o, v3 d, int kind, float lim) {
    wide_start(R, o, d, kind != 0, lim);
    fin = true;
    if (kind == 2) {
      R.best = 0;
      return;
    }
    if (CNT) {
      c.rays += kind == 0 ? 1u : 0u;
      c.srays += kind == 1 ? 1u : 0u;
    }
    if (!wide_ray_ok(R.o, R.d, R.inv)) {
      exact_walk();
      return;
    }
    fin = false;
  };
  for (;;) {
    // lanes whose walk is over shade together: path_step on the answer, then
    // the path's next ray starts in the lane, or its colour is stored
    while (p >= 0 && fin && R.nc == 0) {
      Trav T;
      T.o = R.o;
      T.d = R.d;
      T.shadow = R.shadow;
      T.lim = R.lim;
      T.res = R.best;
      T.nc = 0;
      T.cn = T.cl = 0u;
      PathSt S;
      wf_load_state(B, cur, p, R.o, R.d, &S);   // PH_SSS: the walk ray is S.so / S.sd
      v3 col;
      bool need = path_step<false>(P, F, S, T, c, &col);
      while (need && T.shadow == 2) {   // null shadow queries (trav_null)
        T.res = 0;
        need = path_step<false>(P, F, S, T, c, &col);
      }
      if (need) {
        wf_store_state(B, cur, p, S);
        begin(T.o, T.d, T.shadow, T.lim);
      } else {
        B.colors[B.ids[cur][p]] = make_float4(col.x, col.y, col.z, 1.0f);
        p = -1;
        fin = false;
      }
    }
    const unsigned long long idle = __ballot(p < 0);
    const int ng = (int)__popcll(idle);
    if (more && ng >= PT_WIDE_REFILL) {
      int base = 0;
      if (lane == 0) base = atomicAdd(&B.counters[2], ng);
      base = __shfl(base, 0);
      if (base + ng >= count) more = false;
      if (p < 0) {
        const int slot = base + (int)__popcll(idle & ((1ull << lane) - 1ull));
        if (slot < count) {
          float4 r0, r1;
          wf_load_ray(rays, B.cap, slot, &r0, &r1);
          p = slot;
          // a closest ray's limit word may carry fuse bits' RNG state: unused
          // here (wide_start ignores a closest ray's limit)
          begin(mk(r0.x, r0.y, r0.z), mk(r1.x, r1.y, r1.z), __float_as_int(r1.w) & kRayKindMask, r0.w);
        }
      }
    }
    if (!more && __ballot(p >= 0) == 0ull) break;
    if (__ballot(p >= 0 && fin && R.nc == 0)) continue;   // shade first (a walk answered at its start)
    for (int it = 0; it < PT_WIDE_STEPS; ++it) {
      bool exact = false;
      if (p >= 0 && !fin)
        fin = wide_step<CNT, true, QN>(R, P.wide, P.wide_tris, lds, 64, ovf, os, P.wide_stack, &exact, &c.nodes,
                                       &c.leaves, cand, P.wide_leafbox);
      if (exact) exact_walk();   // the builder's stack bound rules this out; stay exact anyway
      const unsigned long long waiting = __ballot(p >= 0 && fin && R.nc > 0);
      if (__ballot(p >= 0 && R.nc > kWideQ - 4) || (int)__popcll(waiting) >= PT_WIDE_FLUSH_T ||
          (waiting && __ballot(p >= 0 && !fin) == 0ull)) {
        if (PT_WIDE_FLUSH_WAVE ? wide_flush_wave<CNT, QN>(R, p >= 0, P.wide_tris, cand, fkeys[PT_WIDE_FLUSH_WAVE ? wave : 0],
                                                        lane, &c.leaves, P.wide_leafbox)
                               : (p >= 0 && R.nc > 0 && wide_flush<CNT, QN>(R, P.wide_tris, cand, &c.leaves, P.wide_leafbox))) {
          fin = true;   // occluded
          R.sp = 0;
          R.cur = -1;
        }
      }
      if (__ballot(p >= 0 && !(fin && R.nc == 0)) == 0ull) break;
    }
  }
  if (CNT) flush_traced(P, c, lane);
}

// Running mean (:467-469) of each pixel's samples, in batch order.
__global__ __launch_bounds__(256) void wf_fold_kernel(RenderParams P, WfBuffers B, long long n_pix, long long pp0) {
  const long long pp = pp0 + (long long)blockIdx.x * 256 + threadIdx.x;   // pixels [pp0, pp0 + n_pix)
  if (pp - pp0 >= n_pix) return;
  int px, py;
  if (!wf_pixel(P, pp, &px, &py)) return;
  float4* dst = P.accum + (size_t)py * (size_t)P.width + (size_t)px;
  float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  if (!(P.fresh && P.first_batch == 0)) {
    const float4 a = *dst;
    acc[0] = a.x; acc[1] = a.y; acc[2] = a.z; acc[3] = a.w;
  }
  const float4* col = B.colors + (size_t)pp * P.n_batches;
  for (uint32_t s = 0; s < P.n_batches; ++s) {
    const float4 c = col[s];
    const uint32_t batch = P.first_batch + s;
    const float fb = (float)batch, fb1 = (float)(batch + 1u);
    acc[0] = (acc[0] * fb + c.x) / fb1;
    acc[1] = (acc[1] * fb + c.y) / fb1;
    acc[2] = (acc[2] * fb + c.z) / fb1;
    acc[3] = (acc[3] * fb + 1.0f) / fb1;
  }
  *dst = make_float4(acc[0], acc[1], acc[2], acc[3]);
}

__global__ __launch_bounds__(256) void fill_culled_kernel(RenderParams P) {
  fill_culled(P, P.culled_org, P.n_culled_items, (int)blockIdx.x);
}

}  // namespace

hipError_t launch_math(int fn, const float* x, float* y, size_t n, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  math_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(fn, x, y, n);
  return hipGetLastError();
}

hipError_t launch_exhaustive(int fn, unsigned long long* bad, uint32_t* first_bad, hipStream_t stream) {
  exhaustive_kernel<<<8192, 256, 0, stream>>>(fn, bad, first_bad);
  return hipGetLastError();
}

hipError_t launch_setup_tris(const float* d_vertices, const uint32_t* d_indices, int n_tris, float4* d_tris,
                             hipStream_t stream) {
  if (n_tris <= 0) return hipSuccess;
  setup_tris_kernel<<<(n_tris + 255) / 256, 256, 0, stream>>>(d_vertices, d_indices, n_tris, d_tris);
  return hipGetLastError();
}

hipError_t launch_gather_tris(const float4* tris, const int* tri_of, int n, float4* dst, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  gather_tris_kernel<<<(unsigned)((3ll * n + 255) / 256), 256, 0, stream>>>(tris, tri_of, n, dst);
  return hipGetLastError();
}

hipError_t launch_setup_lights(const LightRec* d_in, int n, LightDev* d_out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  setup_lights_kernel<<<(n + 63) / 64, 64, 0, stream>>>(d_in, n, d_out);
  return hipGetLastError();
}

int owned_tiles(int width, int height, const Part& part) {
  return part_count(part, ((width + 15) / 16) * ((height + 15) / 16));
}

hipError_t launch_tiles(bool pack, float4* frame, float4* packed, int width, int height, const Part& part,
                        const int* d_pos, hipStream_t stream) {
  const int n = owned_tiles(width, height, part);
  if (n <= 0) return hipSuccess;
  const int bx = (width + 15) / 16;
  if (pack)
    tiles_kernel<true><<<n, 256, 0, stream>>>(frame, packed, width, height, bx, part.m, part.cnt, d_pos);
  else
    tiles_kernel<false><<<n, 256, 0, stream>>>(frame, packed, width, height, bx, part.m, part.cnt, d_pos);
  return hipGetLastError();
}

hipError_t launch_items_pack(const RenderParams& p, const float4* frame, float4* packed, const int* items, int n,
                             hipStream_t stream) {
  const long long px = (long long)n * (256 / p.spl);
  if (px == 0) return hipSuccess;
  items_pack_kernel<<<(unsigned)((px + 255) / 256), 256, 0, stream>>>(p, frame, packed, items, n);
  return hipGetLastError();
}

hipError_t launch_items_unpack(const RenderParams& p, float4* frame, const float4* src, size_t slot_f4,
                               const int* table, int n, hipStream_t stream) {
  const long long px = (long long)n * (256 / p.spl);
  if (px == 0) return hipSuccess;
  items_unpack_kernel<<<(unsigned)((px + 255) / 256), 256, 0, stream>>>(p, frame, src, slot_f4, table, n);
  return hipGetLastError();
}

hipError_t launch_clear(float4* accum, int width, int height, const Part& part, const int* d_pos, hipStream_t stream) {
  const size_t n = (size_t)width * (size_t)height;
  if (n == 0) return hipSuccess;
  clear_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(accum, width, height, part.m, part.cnt, d_pos);
  return hipGetLastError();
}

hipError_t launch_render(const RenderParams& p, bool stats, bool lds_scene, hipStream_t stream, bool cnt) {
  if (cnt && stats) return hipErrorInvalidValue;
  if (p.spl != 1 && p.spl != 2 && p.spl != 4 && p.spl != 8) return hipErrorInvalidValue;
  // owned tiles (part_tile); the recursive kernel splits each into spl workgroups
  const long long tiles = p.n_tiles;
  long long grid = tiles * p.spl;
  if (grid <= 0 || p.n_batches == 0) return hipSuccess;
  if (p.pack_out && stats) return hipErrorInvalidValue;
  if (p.pack_out) {   // live items (p.n_items), then the assembly workgroups
    const long long px = (long long)p.n_unpack * (256 / p.spl);
    grid = p.n_items + (px + 256 * kPixPerFill - 1) / (256 * kPixPerFill);
  } else if (p.items) {   // compact list of live items, then the fill workgroups
    const long long px = (long long)p.n_culled_items * (256 / p.spl);
    grid = p.n_items + (px + 256 * kPixPerFill - 1) / (256 * kPixPerFill);
  }
  if (grid > 0x7fffffffll) return hipErrorInvalidValue;
  const size_t lds = lds_scene ? scene_lds_bytes(p) : 0;
  if (lds > kMaxSceneLds) return hipErrorInvalidValue;
  void (*kern)(RenderParams);
  if (cnt)
    kern = lds_scene ? render_kernel<false, true, true> : render_kernel<false, false, true>;
  else
    kern = lds_scene ? (stats ? render_kernel<true, true> : render_kernel<false, true>)
                     : (stats ? render_kernel<true, false> : render_kernel<false, false>);
  if (grid > 0) hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(256), lds, stream, p);
  return hipGetLastError();
}

long long render_slots(size_t lds_bytes) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, render_kernel<false, true>, 256, lds_bytes) !=
      hipSuccess)
    return 0;
  return (long long)cus * per_cu;
}

long long wide_trace_lanes() {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  int most = 0;
  for (auto k : {wf_trace_wide_kernel<kWideG, false, 1>, wf_trace_wide_kernel<kWideG, true, 1>,
                 wf_trace_wide_kernel<kWideG, false, 0>, wf_trace_wide_kernel<kWideG, true, 0>}) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, 256, 0) != hipSuccess) return 0;
    most = std::max(most, per_cu);
  }
  return (long long)cus * std::max(most, 1) * 256;
}

hipError_t launch_wavefront(const RenderParams& p0, const WfBuffers& b, bool lds_scene, hipStream_t stream, bool cnt,
                            hipStream_t stream2, hipEvent_t ev_fork, hipEvent_t ev_join) {
  if (p0.spl != 1 && p0.spl != 2 && p0.spl != 4 && p0.spl != 8) return hipErrorInvalidValue;
  if (p0.n_batches == 0) return hipSuccess;
  const int per = 256 / p0.spl;
  const long long tiles = p0.n_tiles;
  const long long items = p0.items ? p0.n_items : tiles * p0.spl;
  if (p0.items && p0.n_culled_items > 0) {
    const long long px = (long long)p0.n_culled_items * per;
    fill_culled_kernel<<<(unsigned)((px + 256 * kPixPerFill - 1) / (256 * kPixPerFill)), 256, 0, stream>>>(p0);
  }
  if (items <= 0) return hipGetLastError();
  const long long px = items * per;
  if (px > b.cap || b.cap > 0x7fffffffll) return hipErrorInvalidValue;
  const size_t lds = lds_scene ? scene_lds_bytes(p0) : 0;
  if (lds > kMaxSceneLds) return hipErrorInvalidValue;
  int dev = 0, cus = 0, per_cu_t = 0, per_cu_s = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
#ifdef PT_WF_FORCE_G
  const bool g2 = PT_WF_FORCE_G == 2;
#else
  const bool g2 = p0.n_tris < kWfGroup4Tris;
#endif
  void (*trace)(RenderParams, WfBuffers, int) =
      cnt ? (lds_scene ? (g2 ? wf_trace_kernel<true, 2, true> : wf_trace_kernel<true, 4, true>)
                       : (g2 ? wf_trace_kernel<false, 2, true> : wf_trace_kernel<false, 4, true>))
          : (lds_scene ? (g2 ? wf_trace_kernel<true, 2> : wf_trace_kernel<true, 4>)
                       : (g2 ? wf_trace_kernel<false, 2> : wf_trace_kernel<false, 4>));
  const bool wide = p0.wide && !lds_scene;
  if (wide)   // culled wide walk (PT_OPT_WIDE, default)
    trace = p0.wide_qn ? (cnt ? wf_trace_wide_kernel<kWideG, true, 1> : wf_trace_wide_kernel<kWideG, false, 1>)
                       : (cnt ? wf_trace_wide_kernel<kWideG, true, 0> : wf_trace_wide_kernel<kWideG, false, 0>);
  const size_t lds_t = wide ? 0 : lds;
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_t, trace, 256, lds_t);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_s, wf_shade_kernel, 256, 0);
  // PT_OPT_WF_TAIL (the 4-wide layouts of the wide walk): wf_tail_kernel after each round's trace
  const bool tail = wide && p0.wf_tail > 0;
  void (*tailk)(RenderParams, WfBuffers, int) =
      p0.wide_qn ? (cnt ? wf_tail_kernel<true, true> : wf_tail_kernel<false, true>)
                 : (cnt ? wf_tail_kernel<true, false> : wf_tail_kernel<false, false>);
  if (p0.wf_tail > 0 && !tail) return hipErrorInvalidValue;   // the trace and shading kernels would skip its lists
  int per_cu_x = 0;
  if (e == hipSuccess && tail) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_x, tailk, 256, 0);
  if (e != hipSuccess) return e;
  unsigned grid_t = (unsigned)(cus * (per_cu_t > 0 ? per_cu_t : 1));
  unsigned grid_x = (unsigned)(cus * (per_cu_x > 0 ? per_cu_x : 1));
  // PT_OPT_WF_GRID: a smaller persistent grid gives each lane more rays per
  // round (a shorter drain relative to the round) when other frames' launches
  // fill the rest of the GPU
  if (p0.wf_grid > 0 && p0.wf_grid < 100) grid_t = std::max(1u, (unsigned)((unsigned long long)grid_t * p0.wf_grid / 100));
  if (wide) {   // every lane needs its overflow stack area
    if (p0.wide_ovf_lanes < 256) return hipErrorInvalidValue;
    grid_t = std::min<unsigned>(grid_t, (unsigned)(p0.wide_ovf_lanes / 256));
    grid_x = std::min<unsigned>(grid_x, (unsigned)(p0.wide_ovf_lanes / 256));
  }
  const unsigned grid_s = (unsigned)(cus * (per_cu_s > 0 ? per_cu_s : 1));
  const uint32_t chunk = (uint32_t)std::min<long long>((long long)p0.n_batches, b.cap / px);
  const int iters = wf_max_rays(p0);
  // Two halves of the chunk's pixels on two streams (PT_OPT_WF_STREAMS):
  // each trace launch ends in a tail where most lanes are out of rays
  // (lane census: ~50 % of lane-steps idle), which the other half's trace
  // and shading fill.  The halves share the path state (disjoint ranges)
  // and get their own lists, counters and stack overflow areas.
  const bool split = stream2 && px >= 2 * 4096;
  const int H = split ? 2 : 1;
  for (uint32_t b0 = 0; b0 < p0.n_batches; b0 += chunk) {
    RenderParams p = p0;
    p.first_batch = p0.first_batch + b0;
    p.n_batches = std::min(chunk, p0.n_batches - b0);
    RenderParams ph[2] = {p, p};
    WfBuffers bh[2] = {b, b};
    hipStream_t sh[2] = {stream, split ? stream2 : stream};
    long long px0[2] = {0, 0}, pxn[2] = {px, 0};
    if (split) {
      pxn[0] = (px / 2 + 255) / 256 * 256;
      pxn[1] = px - pxn[0];
      px0[1] = pxn[0];
      const long long sb = pxn[0] * p.n_batches;   // half 1's paths and list slots start here
      for (int k = 0; k < 2; ++k) {
        bh[1].rays[k] = b.rays[k] + sb;   // slot s of half 1: rays[sb + s], rays[cap + sb + s]
        bh[1].ids[k] = b.ids[k] + sb;
        bh[1].state[k] = b.state[k] + sb;
      }
      bh[1].hits = b.hits + sb;
      bh[1].counters = b.counters + 4;
      ph[1].wide_ovf = p.wide_ovf ? p.wide_ovf + (size_t)p.wide_ovf_lanes * (size_t)p.wide_stack : nullptr;
      e = hipEventRecord(ev_fork, stream);
      if (e == hipSuccess) e = hipStreamWaitEvent(stream2, ev_fork, 0);
      if (e != hipSuccess) return e;
    }
    for (int h = 0; h < H; ++h) {
      const long long n = pxn[h] * p.n_batches;
      e = hipMemsetAsync(bh[h].counters, 0, 3 * sizeof(int), sh[h]);
      if (e != hipSuccess) return e;
      if (cnt)
        wf_gen_kernel<true><<<(unsigned)((n + 255) / 256), 256, 0, sh[h]>>>(ph[h], bh[h], n, px0[h] * p.n_batches);
      else
        wf_gen_kernel<false><<<(unsigned)((n + 255) / 256), 256, 0, sh[h]>>>(ph[h], bh[h], n, px0[h] * p.n_batches);
    }
    int cur = 0;
    for (int it = 0; it < iters; ++it) {
      for (int h = 0; h < H; ++h) hipLaunchKernelGGL(trace, dim3(grid_t), dim3(256), lds_t, sh[h], ph[h], bh[h], cur);
      if (tail)
        for (int h = 0; h < H; ++h) hipLaunchKernelGGL(tailk, dim3(grid_x), dim3(256), 0, sh[h], ph[h], bh[h], cur);
      for (int h = 0; h < H; ++h) wf_shade_kernel<<<grid_s, 256, 0, sh[h]>>>(ph[h], bh[h], cur);
#ifdef PT_WF_ROUND_LOG   // A/B builds only: rays per round (synchronous)
      {
        int cnt2[2] = {0, 0};
        if (hipStreamSynchronize(sh[0]) == hipSuccess &&
            hipMemcpy(cnt2, bh[0].counters, 2 * sizeof(int), hipMemcpyDeviceToHost) == hipSuccess)
          fprintf(stderr, "wf_round %d traced %d next %d\n", it, cnt2[cur], cnt2[cur ^ 1]);
      }
#endif
      cur ^= 1;
    }
    for (int h = 0; h < H; ++h)
      wf_fold_kernel<<<(unsigned)((pxn[h] + 255) / 256), 256, 0, sh[h]>>>(ph[h], bh[h], pxn[h], px0[h]);
    if (split) {
      e = hipEventRecord(ev_join, stream2);
      if (e == hipSuccess) e = hipStreamWaitEvent(stream, ev_join, 0);
      if (e != hipSuccess) return e;
    }
  }
  return hipGetLastError();
}

#ifdef PT_WG_TRACE
hipError_t wg_trace_read(unsigned long long* dst, int n) {
  if (n > kWgTraceCap) n = kWgTraceCap;
  const hipError_t e = hipDeviceSynchronize();
  if (e != hipSuccess) return e;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_wg_trace), (size_t)n * 32, 0, hipMemcpyDeviceToHost);
}
#endif

}  // namespace ptd

#ifdef PT_WG_TRACE
extern "C" int pt_probe_wg_trace(unsigned long long* dst, int n) { return (int)ptd::wg_trace_read(dst, n); }
#endif
