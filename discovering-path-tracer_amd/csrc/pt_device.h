// Device-side data layout and kernel launchers (host-visible declarations).
//
// HBM layout (all 16-B aligned, built once per scene upload):
//   nodes : 2 x float4 per BVH node, renumbered in the reference traversal's
//           visiting order (right child first, raytrace_comp.comp:198-199):
//             [0] = {min.x, min.y, min.z, skip}     skip = int bits
//             [1] = {max.x, max.y, max.z, tri}      tri  = int bits, -1 internal
//           An internal node whose box is hit continues at k+1 (its right
//           child); a missed node or a leaf continues at `skip`, the node the
//           reference's stack would pop next.  Same visit sequence, no stack.
//   tris  : 3 x float4 per triangle slot (slot = the reference's triIdx, the
//           row of the BVH-reordered index buffer):
//             {v0.xyz, e1.x} {e1.yz, e2.xy} {e2.z, n.xyz}
//           e1 = v1-v0, e2 = v2-v0 and n = normalize(cross(e1,e2)) are exactly
//           the values the reference recomputes per test (:119-120, :189).
//   accum : float4[H][W], RGBA32F running mean.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptd {

struct LightRec {          // == pt_area_light / AreaLightData
  float position[4];
  float normal[4];
  float intensity[4];
  float size[4];
};

// Light with its sampling frame precomputed on the device (setup_lights_kernel).
struct LightDev {
  float pos[3], nraw[3], inten[3], right[3], up[3], size[2], half[2];
  float finite;   // 1 when every intensity channel is finite (shadow_needed)
};

// Partition order of the 16x16 blocks: tile b is block row by = b / blocks_x,
// column (b % blocks_x + by) % blocks_x -- each row rotated by its index, so
// "b % nranks == rank" deals every rank anti-diagonal stripes of the image.
// (Row-major order gives column stripes whenever blocks_x % nranks == 0, and
// a centred object then lands unevenly: box.obj 1080p at 8 ranks put 5.7 %
// more of the geometry on rank 0 than the mean; rotated, 0.1 %.)
__host__ __device__ inline void tile_block(int b, int blocks_x, int* bx, int* by) {
  *by = b / blocks_x;
  *bx = (b % blocks_x + *by % blocks_x) % blocks_x;
}
__host__ __device__ inline int block_tile(int bx, int by, int blocks_x) {
  return by * blocks_x + (bx - by % blocks_x + blocks_x) % blocks_x;
}

// A rank's tiles under a slotted partition: tiles are dealt in periods of m
// slots and a rank owns cnt of them, at the ascending positions pos[] of each
// period, i.e. tile b iff b % m is one of pos[].  One slot per rank (m =
// nranks, pos = {rank}) is "b % nranks == rank".  Unequal slot counts let the
// root, which also assembles the frame, render a smaller share
// (pt_set_partition_slots); the host spreads every rank's slots evenly over
// the period, since runs of neighbouring tiles would land unevenly on a
// centred object.
constexpr int kMaxSlots = 64;
struct Part {
  int m, cnt;
  int pos[kMaxSlots];
};
__host__ __device__ inline int part_tile(const Part& p, int li) { return (li / p.cnt) * p.m + p.pos[li % p.cnt]; }
__host__ __device__ inline int part_count(const Part& p, int total) {
  const int rem = total % p.m;
  int n = (total / p.m) * p.cnt;
  for (int i = 0; i < p.cnt; ++i) n += p.pos[i] < rem ? 1 : 0;
  return n;
}
__host__ __device__ inline bool part_owns(const Part& p, int b) {
  const int v = b % p.m;
  bool own = false;
  for (int i = 0; i < p.cnt; ++i) own = own || p.pos[i] == v;
  return own;
}

struct RenderParams {
  // culled wide walk (wide_walk.h), or null: 4-wide nodes, triangle records
  // by leaf rank, triangle slot -> rank, per-lane stack overflow areas
  // (wide_ovf_lanes lanes of wide_stack entries, lane-strided)
  const float4* hit_tris;   // the records a closest hit's index refers to: wide_tris (by rank) with the wide walk, else tris
  const float4* wide;        // 64-B nodes when wide_qn 1, else 128-B (wide_walk.h)
  int wide_qn;
  const float4* wide_leafbox;   // wide_qn: the reference's leaf box per rank, 2 float4
  const float4* wide_tris;
  const int* wide_rank_of;
  int2* wide_ovf;
  long long wide_ovf_lanes;
  int wide_stack;
  int wide_handback;        // test: hand every odd list slot to the exact walk (PT_OPT_WIDE 2)
  int wf_fuse;              // PT_OPT_WF_FUSE: the wide trace kernel also walks a closest hit's first-light shadow ray
  int wf_tail;              // PT_OPT_WF_TAIL: a list of fewer rays than this is finished by wf_tail_kernel (0: never)
  int wf_grid;              // PT_OPT_WF_GRID: the persistent traversal grid in percent of a full-occupancy grid (1-100)
  int wide_refill;          // PT_OPT_WF_REFILL: idle lanes at which a wave of the wide trace kernel refills
  const float4* nodes;
  const float4* tris;
  const LightDev* lights;
  float4* accum;
  // [0..3] rays, nodes, leaf tests, samples (stats mode); [4..8] closest walks,
  // shadow walks, nodes visited, triangle tests, primaries (counting mode)
  unsigned long long* stats;
  int n_nodes;
  int n_tris;
  int n_lights;
  int width, height;
  uint32_t first_batch, n_batches;
  int max_depth, sss_bounces;
  float cam_pos[3], cam_dir[3], cam_up[3], fov;
  // camera frame of main() (:430-432) computed on the host with pt_math.h:
  // right = normalize(cross(dir, -up)), up' = normalize(cross(right, dir)),
  // tan(radians(fov * 0.5))
  float cam_right[3], cam_upv[3], tan_fov;
  int blocks_x, blocks_total;   // 16x16-pixel blocks
  int nranks, rank;             // this rank of nranks
  // its tiles (Part on the host): the period, its slot count, its slot
  // positions in device memory (rank_tile), and how many tiles it owns
  int part_m, part_cnt, n_tiles;
  const int* part_pos;
  int spl;                      // sample lanes per pixel: 1, 2, 4 or 8
  int fresh;                    // first_batch == 0 starts from +0 without reading accum
  // primary-ray culling (pt_primary_cull_rects): -1 = trace every pixel; else
  // a pixel traces only if its NDC origin lies in one of cull[0..n_cull)
  // compact launch (host-built when culling applies): items (owned tile *
  // spl + part) that may hold a live pixel, and those that cannot
  const int* items;             // null = every item, blockIdx.x = item
  const int2* items_org;        // with items: per live item its first pixel {x, y} (host-computed)
  int n_items;
  const int2* culled_org;       // per culled item: its first pixel {x, y} (host-computed)
  int n_culled_items;
  int n_cull;
  float cull[8][4];
  // pt_render_packed: live workgroup i stores its pixels to pack_out[i*256/spl
  // + q] (the pt_items_pack layout) instead of the accumulation buffer, and no
  // culled-item fill runs; null = normal rendering
  float4* pack_out;
  // ... and, optionally, trailing workgroups that assemble a gathered frame
  // (the pt_items_unpack_all work: int4 table entries {rank, x0, y0, slot}
  // -- the item's first pixel, its slot or -1 for a culled item -- over
  // per-rank slots of unpack_slot_f4 float4s) in the same launch
  const float4* unpack_src;
  float4* unpack_frame;
  const int* unpack_table;
  int n_unpack;
  long long unpack_slot_f4;
  int item_order;   // host only: PT_OPT_ITEM_ORDER for the item lists
  // mixed sample lanes (PT_OPT_MIXED_LANES, one-rank path-recursive launches
  // with items): live item i is items_org[i] = {x | log2(spl_i) << 24, y}, a
  // whole 16x16 tile at one lane per pixel or a part at `spl` lanes; the
  // culled items keep `spl`
  int mix = 0;
  // per 16x4 part of the frame (y / 4 * blocks_x + x / 16): the summed wave
  // durations of the launch's live workgroups in GPU wall-clock ticks, or null
  unsigned* cost_out = nullptr;
};
constexpr int kMixShift = 24;
constexpr int kMaxCullRects = 8;
constexpr int kStatsWords = 9;   // RenderParams::stats

hipError_t launch_setup_tris(const float* d_vertices, const uint32_t* d_indices, int n_tris, float4* d_tris,
                             hipStream_t stream);
hipError_t launch_setup_lights(const LightRec* d_in, int n, LightDev* d_out, hipStream_t stream);
int owned_tiles(int width, int height, const Part& part);
hipError_t launch_tiles(bool pack, float4* frame, float4* packed, int width, int height, const Part& part,
                        const int* d_pos,
                        hipStream_t stream);
hipError_t launch_clear(float4* accum, int width, int height, const Part& part, const int* d_pos, hipStream_t stream);
// live-item exchange: pack this rank's listed items (256/spl pixels each) of
// frame densely; unpack int4 entries {rank, x0, y0, slot} from per-rank slots
// of slot_f4 float4s into frame, slot -1 = culled item -> (0,0,0,1)
hipError_t launch_items_pack(const RenderParams& p, const float4* frame, float4* packed, const int* items, int n,
                             hipStream_t stream);
hipError_t launch_items_unpack(const RenderParams& p, float4* frame, const float4* src, size_t slot_f4,
                               const int* table, int n, hipStream_t stream);
// Scene bytes the LDS-staged variant needs, and the largest it accepts.
constexpr size_t kMaxSceneLds = 48 * 1024;
inline size_t scene_lds_bytes(const RenderParams& p) {
  return ((size_t)2 * p.n_nodes + (size_t)3 * p.n_tris) * 16;
}
// cnt: the fast kernel with traced-work counters (PT_OPT_COUNT_TRACED)
hipError_t launch_render(const RenderParams& p, bool stats, bool lds_scene, hipStream_t stream, bool cnt = false);
// Wavefront pipeline (PT_OPT_KERNEL 3): one path per (pixel, sample) held in
// HBM; generate, then alternate a persistent traversal kernel over the list of
// paths waiting for a ray and a shading kernel that consumes the hits and
// emits the next rays; finally fold each pixel's sample colours in batch
// order.  Buffers hold `cap` paths; larger launches run in batch chunks.
struct WfBuffers {
  float4* state[2];  // per list slot: the fields of the waiting path's PathSt its phase needs, by component
                     // (chunk j of slot s at [j * cap + s], wf_store_state)
  float4* colors;    // per path radiance
  int* ids[2];       // work lists: path id per slot
  float4* rays[2];   // ... and its ray, 2 float4 per slot: {o.xyz, limit} {d.xyz, shadow}
  float2* hits;      // per slot of the list being traced: {t, tri bits / occluded}
  int* counters;     // [0],[1] list sizes, [2] trace fetch cursor ([4..6]: the second half's, two streams)
  long long cap;     // paths the buffers hold
};
constexpr int kWfStateF4 = 9;   // state chunks (float4) a waiting path stores at most
// kind word of a listed ray (rays[cap + s].w): 0 closest, 1 shadow, 2 null
// shadow query, plus (PT_OPT_WF_FUSE, closest rays) kRayFuse: the trace
// kernel walks the path's first-light shadow ray after a hit (the ray's
// limit word then holds the path's RNG state); kRayPrimary: a primary ray,
// whose light pre-pass (raytrace_comp.comp:311-328) may end the path first
constexpr int kRayKindMask = 3, kRayFuse = 4, kRayPrimary = 8;
// hits[s].y of a fused closest hit: rank | kHitFused | (kHitOccluded if the
// shadow ray was occluded)
constexpr int kHitFused = 0x40000000, kHitOccluded = 0x20000000, kHitRankMask = 0x1fffffff;
constexpr size_t kWfBytesPerPath = 2 * (size_t)kWfStateF4 * 16 + 16 + 2 * (4 + 32) + 8;
// rays a path may trace in one sample: the primary ray, then per bounce the
// light shadow rays, sss_bounces x (walk ray + light shadow rays) and the
// next bounce ray
inline int wf_max_rays(const RenderParams& p) {
  return 1 + p.max_depth * (p.n_lights + p.sss_bounces * (1 + p.n_lights) + 1);
}
// stream2 (with two events): the chunk's pixels run as two halves on stream
// and stream2 (forked from and joined back into stream); the wide walk's
// overflow area then holds two sets of wide_ovf_lanes lanes.
hipError_t launch_wavefront(const RenderParams& p, const WfBuffers& b, bool lds_scene, hipStream_t stream,
                            bool cnt = false, hipStream_t stream2 = nullptr, hipEvent_t ev_fork = nullptr,
                            hipEvent_t ev_join = nullptr);
// lanes of the wide walk's persistent grid on this device (overflow areas to allocate)
long long wide_trace_lanes();
// workgroups of the LDS-staged render kernel resident on this device at once
long long render_slots(size_t lds_bytes);
// triangle records by rank: dst[r] = tris[tri_of[r]]
hipError_t launch_gather_tris(const float4* tris, const int* tri_of, int n, float4* dst, hipStream_t stream);
hipError_t launch_math(int fn, const float* x, float* y, size_t n, hipStream_t stream);
hipError_t launch_exhaustive(int fn, unsigned long long* bad, uint32_t* first_bad, hipStream_t stream);

}  // namespace ptd
