#!/usr/bin/env python3
"""Write an instrumented copy of pt_device.hip (per-phase wave cycle counters,
s_memtime around each traceRay/shadow/shading block) for A/B diagnosis only:
  python3 tools/phase_instrument.py ab/pt_device_phase.hip
then tools/build_ab.sh phase -DPT_PHASE with SRC=ab/pt_device_phase.hip."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "discovering-path-tracer_amd/csrc/pt_device.hip")).read()


def rep(a, b, count=1, first=False):
    global src
    if first:
        assert a in src, a
        src = src.replace(a, b, 1)
        return
    assert src.count(a) == count, (a, src.count(a))
    src = src.replace(a, b)


rep("""namespace {

struct Ctr {""", """namespace {
__device__ unsigned long long g_phase[16];
__device__ __forceinline__ unsigned long long ph_t() { return __builtin_readcyclecounter(); }
__device__ __forceinline__ void ph_add(int k, unsigned long long dt) {
  if (__lane_id() == (unsigned)__builtin_amdgcn_readfirstlane(__lane_id())) atomicAdd(&g_phase[k], dt);
}
#define PH(k, stmt) do { const unsigned long long t0_ = ph_t(); stmt; ph_add(k, ph_t() - t0_); } while (0)
#define PHV(k, decl, expr) decl; do { const unsigned long long t0_ = ph_t(); decl##_v = expr; ph_add(k, ph_t() - t0_); } while (0)

struct Ctr {""")
rep("""        h0 = trace_closest<STATS, PF>(P, ro, rd, c0, cand);
        have_h0 = true;""", """        PH(1, h0 = (trace_closest<STATS, PF>(P, ro, rd, c0, cand)));
        have_h0 = true;""", 2)
rep("""      h = trace_closest<STATS, PF>(P, ro, rd, c, cand);""", """      PH(5, h = (trace_closest<STATS, PF>(P, ro, rd, c, cand)));""")
rep("""      if (!occluded<STATS, PF>(P, add(hp, muls(hn, OFFSET)), ld, dist - OFFSET, c)) {""",
    """      bool occ_;
      PH(2, occ_ = (occluded<STATS, PF>(P, add(hp, muls(hn, OFFSET)), ld, dist - OFFSET, c)));
      if (!occ_) {""")
rep("""      const Hit sh = trace_closest<STATS, PF>(P, so, sd, c, cand);""",
    """      Hit sh;
      PH(3, sh = (trace_closest<STATS, PF>(P, so, sd, c, cand)));""")
rep("""        if (!occluded<STATS, PF>(P, add(cp, muls(sn, OFFSET)), ed, edist - OFFSET, c)) {""",
    """        bool occ2_;
        PH(4, occ2_ = (occluded<STATS, PF>(P, add(cp, muls(sn, OFFSET)), ed, edist - OFFSET, c)));
        if (!occ2_) {""")
rep("""      const v3 col = path_trace<STATS, !LDS>(P, origin, dir, seed, c, cand);""",
    """      v3 col;
      PH(6, col = (path_trace<STATS, !LDS>(P, origin, dir, seed, c, cand)));""")
rep("""     if (active && live && s < P.n_batches) {""", """     const unsigned long long tg0_ = ph_t();
     if (active && live && s < P.n_batches) {""")
rep("""     // hand the chunk's colours to the folding lanes of the same pixel""",
    """     ph_add(0, ph_t() - tg0_);
     const unsigned long long tf0_ = ph_t();
     // hand the chunk's colours to the folding lanes of the same pixel""")
rep("""     __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
     __builtin_amdgcn_wave_barrier();
     __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }""", """     __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
     __builtin_amdgcn_wave_barrier();
     __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
     ph_add(7, ph_t() - tf0_);
    }
  }""")
rep("""__global__ __launch_bounds__(256, PT_RENDER_MIN_BLOCKS) void render_kernel(RenderParams P) {
  const int tid = (int)threadIdx.x;""", """__global__ __launch_bounds__(256, PT_RENDER_MIN_BLOCKS) void render_kernel(RenderParams P) {
  const unsigned long long tk0_ = ph_t();
  const int tid = (int)threadIdx.x;""")
rep("""  if (STATS) {
    const unsigned long long rays = wave_sum(c.rays)""", """  ph_add(8, ph_t() - tk0_);
  if (STATS) {
    const unsigned long long rays = wave_sum(c.rays)""", first=True)
rep("""    __syncthreads();
    P.nodes = lds_scene;""", """    __syncthreads();
    ph_add(9, ph_t() - tk0_);
    P.nodes = lds_scene;""", first=True)
rep("""    for (uint32_t base = 0; base < P.n_batches; base += (uint32_t)spl) {
     const uint32_t s = base + (uint32_t)j;""", """    ph_add(10, ph_t() - tk0_);
    for (uint32_t base = 0; base < P.n_batches; base += (uint32_t)spl) {
     const uint32_t s = base + (uint32_t)j;""")
rep("""  emit_lane(P, active, pix, q, acc, spl, j);
  ph_add(8, ph_t() - tk0_);""", """  const unsigned long long te0_ = ph_t();
  emit_lane(P, active, pix, q, acc, spl, j);
  ph_add(8, ph_t() - tk0_);""")
rep("""  ph_add(8, ph_t() - tk0_);""", """  ph_add(11, ph_t() - te0_);
  ph_add(8, ph_t() - tk0_);""")
src += """
extern "C" int pt_debug_phase(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(ptd::g_phase), sizeof(unsigned long long) * 16) != hipSuccess) return 1;
  if (reset) {
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(ptd::g_phase), z, sizeof z) != hipSuccess) return 1;
  }
  return 0;
}
"""
open(sys.argv[1], "w").write(src)
