// pt_api.cpp — the C-ABI shim (include/pathtracer.h).
//
// Replaces the Vulkan resource/dispatch seam of src/Vulkan/VulkanRayTracer.cpp:
// staging buffers + vkCmdCopyBuffer become hipMemcpyAsync, the descriptor set
// becomes a RenderParams struct passed by value, vkCmdPushConstants +
// vkCmdDispatch become one kernel launch, and the per-batch fence wait becomes
// an explicit pt_synchronize / pt_read_accum.  Scene preparation that the
// device layout needs (threading the BVH, building triangle records) happens
// here once per upload.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <rccl/rccl.h>   // types only: the functions are resolved at run time (rccl_api)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../../include/pathtracer.h"
#include "pt_device.h"
#include "pt_group.h"
#include "pt_math.h"
#include "scene/bvh.h"
#include "scene/camera.h"
#include "scene/light.h"
#include "scene/obj_loader.h"
#include "scene/wide_bvh.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define PT_HIP(call)                                                                   \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) return fail(PT_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)

template <class T>
void dev_free(T*& p) {
  if (p) (void)hipFree((void*)p);
  p = nullptr;
}

// Threads the reference node array: renumbers nodes in the order the
// reference's DFS visits them (right child first) and records, for each, the
// node visited after its subtree.  Fails on anything that is not a tree.
int thread_bvh(const pt_bvh_node* nodes, size_t n, bool int_bits, size_t n_tris, std::vector<float4>* out) {
  if (n == 0 || n > 0x7fffffffull) return fail(PT_ERR_SCENE, "BVH has no nodes or too many");
  std::vector<int32_t> left(n), right(n);
  for (size_t i = 0; i < n; ++i) {
    float lw = nodes[i].min_bounds[3], rw = nodes[i].max_bounds[3];
    int32_t l, r;
    if (int_bits) {
      memcpy(&l, &lw, 4);
      memcpy(&r, &rw, 4);
    } else {
      // int(node.minBounds.w) (raytrace_comp.comp:173-174): only exact
      // below 2^24, so refuse anything the float cannot hold exactly.
      if (!(lw == floorf(lw)) || !(rw == floorf(rw)) || fabsf(lw) >= 16777216.0f || fabsf(rw) >= 16777216.0f)
        return fail(PT_ERR_SCENE, "float-encoded BVH index is not an exact integer below 2^24 (node " +
                                      std::to_string(i) + "); rebuild with PT_NODES_INT_BITS");
      l = (int32_t)lw;
      r = (int32_t)rw;
    }
    left[i] = l;
    right[i] = r;
    if (l == -1) {
      if (r < 0 || (size_t)r >= n_tris)
        return fail(PT_ERR_SCENE, "leaf " + std::to_string(i) + " has triangle index out of range");
    } else if (l < 0 || (size_t)l >= n || r < 0 || (size_t)r >= n) {
      return fail(PT_ERR_SCENE, "node " + std::to_string(i) + " has child index out of range");
    }
  }
  std::vector<int32_t> order;
  order.reserve(n);
  std::vector<int32_t> newidx(n, -1);
  std::vector<int32_t> stack;
  stack.push_back(0);
  while (!stack.empty()) {
    const int32_t v = stack.back();
    stack.pop_back();
    if (newidx[v] != -1) return fail(PT_ERR_SCENE, "BVH node reachable twice (not a tree)");
    newidx[v] = (int32_t)order.size();
    order.push_back(v);
    if (left[v] != -1) {
      stack.push_back(left[v]);    // :198  push left
      stack.push_back(right[v]);   // :199  push right -> popped first
    }
  }
  const size_t m = order.size();
  std::vector<int32_t> size(n, 1);
  for (size_t k = m; k-- > 0;) {
    const int32_t v = order[k];
    if (left[v] != -1) size[v] = 1 + size[left[v]] + size[right[v]];
  }
  // A child whose bounds are bitwise its parent's is hit whenever it is
  // visited (it is only visited after its parent was hit by the same ray, and
  // the slab test is a pure function of ray and bounds): flag it in bit 31 of
  // `skip` so the kernel can skip recomputing the test.
  std::vector<int32_t> parent(n, -1);
  for (size_t k = 0; k < m; ++k) {
    const int32_t v = order[k];
    if (left[v] != -1) parent[left[v]] = parent[right[v]] = v;
  }
  auto same_bounds = [&](int32_t a, int32_t b) {
    return memcmp(nodes[a].min_bounds, nodes[b].min_bounds, 12) == 0 &&
           memcmp(nodes[a].max_bounds, nodes[b].max_bounds, 12) == 0;
  };
  out->assign(2 * m, make_float4(0, 0, 0, 0));
  for (size_t k = 0; k < m; ++k) {
    const int32_t v = order[k];
    const pt_bvh_node& nd = nodes[v];
    const bool implied = parent[v] >= 0 && same_bounds(v, parent[v]);
    const int32_t skip = (int32_t)(((uint32_t)k + (uint32_t)size[v]) | (implied ? 0x80000000u : 0u));
    const int32_t tri = left[v] == -1 ? right[v] : -1;
    float fs, ft;
    memcpy(&fs, &skip, 4);
    memcpy(&ft, &tri, 4);
    (*out)[2 * k] = make_float4(nd.min_bounds[0], nd.min_bounds[1], nd.min_bounds[2], fs);
    (*out)[2 * k + 1] = make_float4(nd.max_bounds[0], nd.max_bounds[1], nd.max_bounds[2], ft);
  }
  return PT_OK;
}

// Drops internal nodes flagged as implied-hit from a threaded array: such a
// node does nothing but continue at k+1, so every link into it can point at
// the next kept node instead.  The kept nodes' visit sequence (and every slab
// and triangle test) is unchanged; only the pass-through visits disappear.
// Used by the fast kernel; stats mode keeps the full array so it still counts
// the reference's node visits.
void collapse_implied(const std::vector<float4>& full, std::vector<float4>* out) {
  const size_t m = full.size() / 2;
  auto raw_skip = [&](size_t k) { int32_t s; memcpy(&s, &full[2 * k].w, 4); return s; };
  auto tri_of = [&](size_t k) { int32_t t; memcpy(&t, &full[2 * k + 1].w, 4); return t; };
  auto dropped = [&](size_t k) { return raw_skip(k) < 0 && tri_of(k) < 0; };
  std::vector<int32_t> nxt(m + 1);
  int32_t kept = 0;
  for (size_t k = 0; k < m; ++k)
    if (!dropped(k)) ++kept;
  nxt[m] = kept;
  for (size_t k = m; k-- > 0;) nxt[k] = dropped(k) ? nxt[k + 1] : --kept;
  out->clear();
  out->reserve(2 * (size_t)nxt[m]);
  for (size_t k = 0; k < m; ++k) {
    if (dropped(k)) continue;
    const int32_t raw = raw_skip(k);
    const int32_t skip = (int32_t)((uint32_t)nxt[raw & 0x7fffffff] | ((uint32_t)raw & 0x80000000u));
    float4 a = full[2 * k];
    memcpy(&a.w, &skip, 4);
    out->push_back(a);
    out->push_back(full[2 * k + 1]);
  }
}

// ---- primary-ray bundle culling -----------------------------
// Camera model of raytrace_comp.comp:430-460 in the orthonormal camera frame
// (right, up, ez = dir/|dir|) centred on the camera position, with the
// kernel's right = normalize(cross(dir, -up0)), up = normalize(cross(right, dir)):
//   origin O = (ox, oy, 0),     |ox|, |oy| <= 0.02 * Rg        (aperture, :445-448)
//   bdir ∝ (a, b, 1),  a = -ndcX*T*A/L, b = -ndcY*T/L          (:456-457)
//   ndcX = ndcX0 + jx*0.5/W,    |jx| <= Rg                     (:451-454)
//   F = 3*bdir,  dir ∝ F - O                                   (:459-460)
// where Rg bounds every Box-Muller radius sqrt(-2 log u1) with u1 >= 1e-38
// (:220): sqrt(-2 ln 1e-38) = 13.2286.  The ray reaches depth Z at slope
//   X/Z = a + ox (1/Z - 1/Fz),  Fz = 3/sqrt(1+a^2+b^2),
// so a point of depth Z > 0 with slope s is reachable from a pixel only if
// |s - a| <= 0.02 Rg max|1/Z - 1/Fz| for some a of the pixel's jittered range.
// Every object (root box corners, light rectangle corners — convex sets whose
// slope hull is the hull of the corners' slopes) therefore maps to an NDC
// rectangle of pixel origins that can reach it; outside all rectangles every
// primary ray misses the root box (so traceRay returns no hit) and every light
// (the pre-pass hits nothing), and the sample is exactly (0,0,0).  All maths
// in double with margins far above the kernel's float rounding.
constexpr double kGaussR = 13.25;

struct D3 { double x, y, z; };
D3 d3(const float* f) { return {f[0], f[1], f[2]}; }
D3 dsub(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
D3 dadd(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
D3 dmul(D3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
double ddot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 dcross(D3 a, D3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dlen(D3 a) { return sqrt(ddot(a, a)); }

// Returns the rectangle count (>= 0) or -1 when no guarantee is derived.
int cull_rects(const float cam[16], int W, int H, const float* lo, const float* hi, const pt_area_light* lights,
               int n_lights, float* rects, int max_rects) {
  if (W <= 0 || H <= 0 || n_lights < 0 || n_lights + 1 > max_rects) return -1;
  const D3 cpos = d3(cam), cdir = d3(cam + 4), cup = d3(cam + 8);
  const double fov = cam[12];
  const double L = dlen(cdir);
  if (!(L > 1e-6 && L < 1e6) || !(fov > 0.01 && fov < 170.0)) return -1;
  const D3 rx = dcross(cdir, dmul(cup, -1.0));
  const double rl = dlen(rx);
  if (!(rl > 1e-6 * L * dlen(cup))) return -1;
  const D3 right = dmul(rx, 1.0 / rl);
  const D3 ux = dcross(right, cdir);
  const D3 up = dmul(ux, 1.0 / dlen(ux));
  const D3 ez = dmul(cdir, 1.0 / L);
  const double T = tan(fov * 0.5 * M_PI / 180.0), A = (double)W / (double)H;
  const double jx = kGaussR * 0.5 / W, jy = kGaussR * 0.5 / H;              // jitter in NDC
  const double amax = (1.0 + jx) * T * A / L, bmax = (1.0 + jy) * T / L;
  const double fz_min = 3.0 / sqrt(1.0 + amax * amax + bmax * bmax), fz_max = 3.0;
  const double rho = 0.02 * kGaussR * 1.001;
  int n = 0;
  auto add_object = [&](const D3* pts, int np) -> bool {
    double sx0 = INFINITY, sx1 = -INFINITY, sy0 = INFINITY, sy1 = -INFINITY, z0 = INFINITY, z1 = -INFINITY;
    for (int i = 0; i < np; ++i) {
      const D3 r = dsub(pts[i], cpos);
      const double X = ddot(r, right), Y = ddot(r, up), Z = ddot(r, ez);
      if (!(Z > 1e-4 * (1.0 + dlen(r)))) return false;   // at or behind the camera plane (or NaN)
      sx0 = fmin(sx0, X / Z); sx1 = fmax(sx1, X / Z);
      sy0 = fmin(sy0, Y / Z); sy1 = fmax(sy1, Y / Z);
      z0 = fmin(z0, Z); z1 = fmax(z1, Z);
    }
    const double dd = fmax(fmax(fabs(1.0 / z0 - 1.0 / fz_min), fabs(1.0 / z0 - 1.0 / fz_max)),
                           fmax(fabs(1.0 / z1 - 1.0 / fz_min), fabs(1.0 / z1 - 1.0 / fz_max)));
    const double del = rho * dd;
    // slope -> NDC (the maps are decreasing), then the jitter and a margin of
    // ~1 pixel plus 1e-4 relative for the kernel's float evaluation
    double x0 = -(sx1 + del) * L / (T * A), x1 = -(sx0 - del) * L / (T * A);
    double y0 = -(sy1 + del) * L / T, y1 = -(sy0 - del) * L / T;
    const double mx = 2.0 / W + 1e-4 * (1.0 + fabs(x0) + fabs(x1)), my = 2.0 / H + 1e-4 * (1.0 + fabs(y0) + fabs(y1));
    x0 -= jx + mx; x1 += jx + mx; y0 -= jy + my; y1 += jy + my;
    if (!(x0 == x0 && x1 == x1 && y0 == y0 && y1 == y1)) return false;
    float* o = rects + 4 * n++;
    o[0] = nextafterf((float)x0, -INFINITY); o[1] = nextafterf((float)x1, INFINITY);
    o[2] = nextafterf((float)y0, -INFINITY); o[3] = nextafterf((float)y1, INFINITY);
    return true;
  };
  // root box, dilated for the slab test's float rounding
  {
    double m = 0.0;
    for (int k = 0; k < 3; ++k) m = fmax(m, fmax(fabs((double)lo[k]), fabs((double)hi[k])));
    m = 1e-4 * m + 1e-6;
    D3 pts[8];
    for (int i = 0; i < 8; ++i)
      pts[i] = {(i & 1 ? hi[0] + m : lo[0] - m), (i & 2 ? hi[1] + m : lo[1] - m), (i & 4 ? hi[2] + m : lo[2] - m)};
    if (!add_object(pts, 8)) return -1;
  }
  // light rectangles: pos ± right*half0 ± up*half1 with the frame of
  // setup_lights_kernel (:261-264), halves dilated
  for (int l = 0; l < n_lights; ++l) {
    const pt_area_light& li = lights[l];
    const D3 nr = d3(li.normal);
    const double nl = dlen(nr);
    if (!(nl > 0.0)) return -1;
    const D3 nn = dmul(nr, 1.0 / nl);
    // the kernel picks the basis from its float normalize; near the switch
    // point either basis may be taken, and the rectangle's orientation is
    // then unknown — use its circumscribed square (both orientations inside)
    const D3 basis = fabs(nn.y) < 0.999 ? D3{0, 1, 0} : D3{1, 0, 0};
    const D3 lr = dmul(dcross(nn, basis), 1.0 / dlen(dcross(nn, basis)));
    const D3 lu = dcross(lr, nn);
    double h0 = fabs((double)li.size[0]) * 0.5, h1 = fabs((double)li.size[1]) * 0.5;
    const D3 pos = d3(li.position);
    const double pm = fmax(fmax(fabs(pos.x), fabs(pos.y)), fabs(pos.z));
    if (fabs(fabs(nn.y) - 0.999) < 1e-4) h0 = h1 = fmax(h0, h1) * 1.41422;
    h0 = h0 * 1.0001 + 1e-4 * pm + 1e-6;
    h1 = h1 * 1.0001 + 1e-4 * pm + 1e-6;
    if (!(h0 < 1e30 && h1 < 1e30)) return -1;
    D3 pts[8];
    for (int i = 0; i < 4; ++i) {
      const D3 c = dadd(dadd(pos, dmul(lr, i & 1 ? h0 : -h0)), dmul(lu, i & 2 ? h1 : -h1));
      // a thin slab around the plane covers the float plane-intersection error
      const double th = 1e-4 * (pm + h0 + h1) + 1e-6;
      pts[2 * i] = dadd(c, dmul(nn, th));
      pts[2 * i + 1] = dadd(c, dmul(nn, -th));
    }
    if (!add_object(pts, 8)) return -1;
  }
  return n;
}

}  // namespace

// Native multi-GPU step loop state (pt_dist_*): an RCCL communicator of its
// own, a high-priority stream for the gathers, two render streams (frames
// alternate), and double-buffered send / receive slots.
constexpr int kDistStreams = 3;                 // render streams: frames k, k+1, .. in flight
constexpr int kDistSets = 2 * kDistStreams;     // frame k uses buffer set k % (2 D) (see pt_dist_run)
struct DistState {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  int comm_count = -1;   // ncclCommCount of the communicator (-1: not reported by the library)
  hipStream_t comm_stream = nullptr;
  hipStream_t streams[kDistStreams] = {};
  hipStream_t own[kDistStreams + 1] = {};   // created here: render streams, then the gather stream
                                            // (pt_dist_set_streams may override)
  hipEvent_t render_done[kDistSets] = {}, gather_done[kDistSets] = {};
  hipEvent_t entry[kDistStreams + 1] = {};  // pt_dist_run's entry barrier: each stream's last work
  float* send[kDistStreams] = {};        // non-root ranks: frame k's live items (k % D)
  float* recv[kDistSets] = {};           // root: one slot per rank of the partition; slot 0 its own
  float* ingest = nullptr;               // emulated root: stand-in for the other ranks' slots
  size_t slot_floats = 0, cap_floats = 0;
  std::vector<float> layout_key;         // frame_key of the layout the slots were sized for
  // root: frame buffers that hold a whole assembled frame of a layout (its
  // culled items' constant (0,0,0,1) included); later frames of that layout
  // rebuild only their live items there (the culled bytes are the same)
  std::vector<std::pair<const void*, std::vector<float>>> assembled;
  bool ready = false;
  bool caller_streams = false;           // pt_dist_set_streams gave render streams (then at most 2)
};

struct pt_context {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  float4* d_nodes = nullptr;        // threaded, implied internal nodes collapsed (fast kernel)
  int n_nodes = 0;
  float4* d_nodes_full = nullptr;   // threaded, every reference node (stats mode)
  // culled wide walk (wide_walk.h): nodes, triangle records by rank, rank ->
  // slot, per-lane stack overflow areas (grown on demand)
  float4* d_wide = nullptr;
  float4* d_wide_q = nullptr;        // the same wide nodes in the 64-B layout
  float4* d_wide_leafbox = nullptr;  // the reference's leaf boxes by rank (64-B walk)
  float4* d_wide_tris = nullptr;
  int* d_wide_rank_of = nullptr;
  // the 8-wide layout (PT_OPT_WIDE_NODE 80): nodes, triangle records and
  // leaf boxes by leaf position, position -> rank, slot -> position
  int2* d_wide_ovf = nullptr;
  long long wide_ovf_lanes = 0;
  int wide_ovf_stack = 0;   // the stack bound d_wide_ovf was sized for
  int n_wide = 0, wide_stack = 0;
  std::string wide_reason = "no scene";
  int opt_wide = 1;           // PT_OPT_WIDE
  int opt_wf_fuse = 1;        // PT_OPT_WF_FUSE
  int opt_wf_tail = -1;       // PT_OPT_WF_TAIL (-1 auto)
  int opt_wf_grid = 100;      // PT_OPT_WF_GRID (percent of a full-occupancy traversal grid)
  int opt_wf_refill = 0;      // PT_OPT_WF_REFILL (0 auto)
  int opt_wide_node = 64;     // PT_OPT_WIDE_NODE
  int n_nodes_full = 0;
  float4* d_tris = nullptr;
  int n_tris = 0;
  ptd::LightRec* d_lights = nullptr;
  ptd::LightDev* d_lights_dev = nullptr;
  int n_lights = 0;
  float4* d_accum = nullptr;
  bool own_accum = false;
  int width = 0, height = 0;
  unsigned long long* d_stats = nullptr;
  float cam[16] = {0};
  bool has_camera = false;
  bool has_scene = false;
  pt_params params{4, 3};
  int nranks = 1, rank = 0;
  std::vector<int> slots{1};    // partition slots per rank (pt_set_partition_slots)
  std::vector<ptd::Part> parts;  // every rank's share, derived from slots (ensure_parts)
  bool parts_valid = false;     // parts match slots
  bool parts_synced = false;    // d_parts holds parts
  int* d_parts = nullptr;       // every rank's slot positions, kMaxSlots ints each (rank_tile)
  size_t parts_cap = 0;
  std::vector<int> parts_key;
  bool stats_mode = false;
  int opt_scene_lds = 1;   // PT_OPT_SCENE_IN_LDS: 0 never, 1 auto, 2 always
  int opt_sample_lanes = 0;   // PT_OPT_SAMPLE_LANES: 0 auto, else 1/2/4/8
  int opt_fresh = 0;          // PT_OPT_FRESH_BATCH0
  int opt_item_order = -1;    // PT_OPT_ITEM_ORDER (-1 auto)
  int opt_mixed = -1;         // PT_OPT_MIXED_LANES: -1 auto, 0 off, k = whole tiles for k % of the resident slots
  int opt_kernel = 0;         // PT_OPT_KERNEL: 0 auto, 1 path-recursive, 3 wavefront
  int opt_cull = 1;           // PT_OPT_PRIMARY_CULL
  int opt_wf_paths = 0;       // PT_OPT_WF_PATHS (0 = 2^27)
  long long wf_fail = 0;      // wavefront paths whose allocation failed (0: none)
  int opt_count = 0;          // PT_OPT_COUNT_TRACED
  int opt_wide_build = 1;     // PT_OPT_WIDE_BUILD (pt::WideBuild; read at upload)
  int opt_wf_streams = 1;     // PT_OPT_WF_STREAMS (2 measured slower: 10M cloud +9 %, sphere -0.8 %)
  hipStream_t wf_stream2 = nullptr;           // the wavefront pipeline's second half (created on first use)
  hipEvent_t wf_fork = nullptr, wf_join = nullptr;
  int last_kernel = 0;        // kernel of the last render (1 recursive, 3 wavefront)
  // compact-launch item lists (live items, then culled ones), rebuilt when
  // the frame, partition, sample lanes or cull rectangles change
  int* d_items = nullptr;
  size_t items_cap = 0;
  int n_live_items = 0, n_culled_items = 0;   // launched live items (mixed lanes: whole tiles + parts)
  bool items_mixed = false;                    // the live origins carry per-item lane counts
  std::vector<int> block_lanes;                // lanes per 16x16 block in the current item lists (0: not launched)
  // measured mixed-lane schedule (mix_feedback)
  unsigned* d_cost = nullptr;                  // per 16x4 part: summed wave durations of a measuring launch
  unsigned* h_cost = nullptr;                  // pinned copy
  size_t cost_n = 0;                           // blocks allocated
  hipEvent_t cost_ev = nullptr;
  bool cost_pending = false, cost_stale = false, cost_measure = false, cost_ready = false;
  int cost_stable = 0, cost_frames = 0, cost_gen = 0;
  std::vector<float> cost_key, cost_scratch;
  std::vector<int> cost_lanes;                 // block_lanes of the measuring launch
  std::vector<double> block_cost;              // per 16x4 part, at one lane per pixel (averaged)
  int scene_serial = 0;                        // bumped by scene and light uploads
  int last_mix = 0;                            // pt_mixed_info: the last launch's schedule
  // What the accumulation buffer's culled items hold (render_impl): 0 not
  // known, 1 finite (+-0 after a clear), 2 (0,0,0,1) in every culled item of
  // the item layout culled_key in buffer culled_buf.  Only the library's own
  // calls are assumed to write the buffer.
  int culled_state = 0;
  std::vector<float> culled_key;
  const void* culled_buf = nullptr;
  long long render_slots = -1;                 // resident LDS render workgroups (mixed lanes' budget)
  size_t render_slots_lds = 0;                 // ... at this many bytes of staged scene
  size_t culled_org_off = 0;   // h_items / d_items: where the culled items' first pixels start
  size_t live_org_off = 0;     // ... and the live items' ones
  std::vector<int> h_items;
  std::vector<float> items_key;
  ptd::RenderParams last{};     // configuration of the last pt_render
  bool last_valid = false;
  // sparse exchange: this rank's live items, and all ranks' (root)
  int* d_pack_items = nullptr;
  size_t pack_cap = 0;
  int n_pack_items = 0;
  std::vector<float> pack_key;
  int* d_unpack = nullptr;      // per entry: rank, x0, y0, slot (-1 = culled)
  size_t unpack_cap = 0;
  int n_unpack = 0;
  int* d_unpack_live = nullptr;   // the same table without the culled items' entries
  size_t unpack_live_cap = 0;
  int n_unpack_live = 0;
  std::vector<float> unpack_key;
  std::vector<float> packed_key;   // frame parameters of the last pt_render_packed
  std::vector<float> key_scratch, items_scratch;   // per-launch keys, built without reallocating
  float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};   // root AABB of the uploaded tree
  std::vector<pt_area_light> lights_host;
  // wavefront pipeline buffers (PT_OPT_KERNEL 3), grown on demand
  ptd::WfBuffers wf{};
  void* wf_block = nullptr;
  // progressive loop (VulkanRayTracer::mainLoop, :717-865)
  float prog_cam[16] = {0};
  bool prog_has_cam = false;
  uint32_t prog_batch = 0;
  // double-buffered asynchronous readback: device snapshot -> pinned host
  struct Readback {
    float4* dev = nullptr;
    void* host = nullptr;
    size_t bytes = 0;
    hipEvent_t snap = nullptr, done = nullptr;
    int ticket = 0;        // 0 = free
    int w = 0, h = 0;
  } rb[2];
  hipStream_t copy_stream = nullptr;
  // Launches that write context-owned buffers (the accumulation buffer, the
  // wavefront path buffers) are ordered across streams: the next such launch
  // waits for the last one when it runs on another stream (order_shared).
  hipEvent_t shared_ev = nullptr;
  hipStream_t shared_stream = nullptr;
  // Every stream this context has enqueued work on that reads its buffers
  // (node/triangle arrays, item tables, accumulation and wavefront buffers),
  // with an event recorded after the last such work (note_use).  A host-side
  // rebuild of those buffers waits on these events only (quiesce), never on
  // the whole device, so it does not wait on another component's RCCL or
  // torch work sharing the GPU.
  struct Use {
    hipStream_t stream;
    hipEvent_t ev;
  };
  std::vector<Use> uses;
  int rb_next_ticket = 1;
  bool timed = false;
  // ring of event pairs, one per render launch since pt_reset_launch_times
  static constexpr int kRing = 512;
  hipEvent_t ring[kRing][2] = {};
  int ring_n = 0;
  int last_slot = 0;          // ring slot of the newest launch (pt_last_launch_ms)
  int opt_timing = 0;         // PT_OPT_LAUNCH_TIMING: event pair on every k-th launch, 0 = none (default:
                              // a pair costs the one-stream frame ~10 us, profiles/r06a)
  long long launch_n = 0;     // render launches since pt_reset_launch_times
  long long ring_launch[kRing] = {};   // launch number of each recorded pair
  DistState* dist = nullptr;           // pt_dist_init
  pt_group* group = nullptr;           // pt_create_multi: every call goes to the group (pt_group.cpp)
  bool in_dist = false;                // inside pt_dist_run: it records the use events itself
};

struct pt_scene {
  pt::ObjScene obj;
  std::vector<uint32_t> bvh_indices;
  std::vector<pt::BVHNode> nodes;
  uint32_t flags = 0;
};

// The items (owned tile x sample-lane part) the render kernel would launch,
// split by the same float test its workgroups apply (render_kernel wg_live):
// those whose pixel rectangle can touch a cull rectangle go to the render
// kernel, the rest to fill_culled_kernel.  A culled workgroup still costs a
// workgroup launch (a fully culled 1080p frame took 0.10 ms at 4 sample
// lanes), so only live ones are launched.
// Pixels of columns [g0, g0+n) (or rows) whose NDC origin (the kernel's
// ndc = 2*p/res - 1) lies in [lo, hi].
// Before a launch that writes context-owned buffers: wait for the previous
// such launch if it ran on another stream.
static int order_shared(pt_context* c) {
  if (c->shared_stream && c->shared_stream != c->stream) PT_HIP(hipStreamWaitEvent(c->stream, c->shared_ev, 0));
  return PT_OK;
}
// After enqueueing work that reads or writes context-owned buffers on
// c->stream: record it in that stream's use event (a context rarely sees more
// than a handful of streams; past kMaxUses the oldest entry is waited for and
// dropped).
constexpr size_t kMaxUses = 16;
static int note_use(pt_context* c) {
  for (auto& u : c->uses)
    if (u.stream == c->stream) {
      PT_HIP(hipEventRecord(u.ev, c->stream));
      return PT_OK;
    }
  if (c->uses.size() >= kMaxUses) {
    PT_HIP(hipEventSynchronize(c->uses.front().ev));
    PT_HIP(hipEventDestroy(c->uses.front().ev));
    c->uses.erase(c->uses.begin());
  }
  pt_context::Use u{c->stream, nullptr};
  PT_HIP(hipEventCreateWithFlags(&u.ev, hipEventDisableTiming));
  c->uses.push_back(u);
  PT_HIP(hipEventRecord(u.ev, c->stream));
  return PT_OK;
}
// After it (or after the last launch that reads those buffers back).
static int mark_shared(pt_context* c) {
  PT_HIP(hipEventRecord(c->shared_ev, c->stream));
  c->shared_stream = c->stream;
  return note_use(c);
}
// Before buffers that launches on any stream may still read are freed or
// overwritten from the host (list rebuilds, reallocation): wait for this
// context's own work on every stream it used -- not for the whole device.
static int quiesce(pt_context* c) {
  for (auto& u : c->uses) PT_HIP(hipEventSynchronize(u.ev));
  return PT_OK;
}

static int pixels_in(int g0, int n, int res, float lo, float hi) {
  int k = 0;
  for (int i = 0; i < n; ++i) {
    const float v = (2.0f * (float)(g0 + i) / (float)res) - 1.0f;
    k += (v >= lo && v <= hi) ? 1 : 0;
  }
  return k;
}

// Live items are listed heaviest first (longest-processing-time order: the
// hardware dispatches workgroups in list order, so the long ones start early
// and the short ones fill the tail).  Weight = pixels inside the root box's
// rectangle (cull[0]: full paths, ~9 rays per sample on box.obj) x 8 + pixels
// inside a light rectangle (pre-pass only).  Output does not depend on the
// order; every consumer (launch, pack, unpack table) uses this one list.
// Rank r's share of the slotted partition (pt_device.h Part): the period's
// slots ordered by (k + 1/2) / slots[rank] for each rank's k-th slot (ties by
// rank), so every rank's slots are spread evenly over the period.
static ptd::Part part_of_slots(const std::vector<int>& slots, int r) {
  std::vector<std::pair<double, int>> seq;
  for (int i = 0; i < (int)slots.size(); ++i)
    for (int k = 0; k < slots[i]; ++k) seq.push_back({(k + 0.5) / slots[i], i});
  std::stable_sort(seq.begin(), seq.end());
  ptd::Part pt{};
  pt.m = (int)seq.size();
  for (int v = 0; v < pt.m; ++v)
    if (seq[v].second == r) pt.pos[pt.cnt++] = v;
  return pt;
}
// Every rank's share, computed once per partition change (one sort of the
// period for all ranks) -- not per launch: at 8 ranks the per-call derivation
// cost ~10 us of host time per render launch.
static void ensure_parts(pt_context* c) {
  if (c->parts_valid && c->parts.size() == c->slots.size()) return;
  std::vector<std::pair<double, int>> seq;
  for (int i = 0; i < (int)c->slots.size(); ++i)
    for (int k = 0; k < c->slots[i]; ++k) seq.push_back({(k + 0.5) / c->slots[i], i});
  std::stable_sort(seq.begin(), seq.end());
  c->parts.assign(c->slots.size(), ptd::Part{});
  for (auto& pt : c->parts) pt.m = (int)seq.size();
  for (int v = 0; v < (int)seq.size(); ++v) {
    ptd::Part& pt = c->parts[seq[v].second];
    pt.pos[pt.cnt++] = v;
  }
  c->parts_valid = true;
  c->parts_synced = false;
}
static const ptd::Part& part_of(pt_context* c, int r) {
  ensure_parts(c);
  return c->parts[r];
}

// Upload every rank's slot positions when the partition changed; the device
// copy of rank r's starts at d_parts + r * kMaxSlots.
static int upload_ints_(const std::vector<int>& h, int** d, size_t* cap) {
  if (h.size() > *cap) {
    dev_free(*d);
    *cap = 0;
    PT_HIP(hipMalloc((void**)d, h.size() * sizeof(int)));
    *cap = h.size();
  }
  if (!h.empty()) PT_HIP(hipMemcpy(*d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
  return PT_OK;
}
static int sync_parts(pt_context* c) {
  ensure_parts(c);
  if (c->parts_synced && c->d_parts) return PT_OK;
  std::vector<int> all((size_t)c->nranks * ptd::kMaxSlots, 0);
  for (int r = 0; r < c->nranks; ++r) {
    const ptd::Part& pt = c->parts[r];
    for (int i = 0; i < pt.cnt; ++i) all[(size_t)r * ptd::kMaxSlots + i] = pt.pos[i];
  }
  if (all == c->parts_key && c->d_parts) {
    c->parts_synced = true;
    return PT_OK;
  }
  { const int rc_ = quiesce(c); if (rc_) return rc_; }
  const int rc = upload_ints_(all, &c->d_parts, &c->parts_cap);
  if (rc) return rc;
  c->parts_key = all;
  c->parts_synced = true;
  return PT_OK;
}

static void item_lists(const ptd::RenderParams& p, const ptd::Part& part, std::vector<int>* live,
                       std::vector<int>* culled) {
  const int W = p.width, H = p.height, spl = p.spl, rows = 16 / spl;
  const int tiles = ptd::part_count(part, p.blocks_total);
  live->clear();
  culled->clear();
  std::vector<std::pair<int, int>> weighted;   // (-weight, item)
  for (int li = 0; li < tiles; ++li) {
    const int b = ptd::part_tile(part, li);
    int bx, by;
    ptd::tile_block(b, p.blocks_x, &bx, &by);
    const int gx0 = bx * 16;
    const float wx0 = (2.0f * (float)gx0 / (float)W) - 1.0f, wx1 = (2.0f * (float)(gx0 + 15) / (float)W) - 1.0f;
    int cols[ptd::kMaxCullRects] = {};
    for (int r = 0; r < p.n_cull; ++r) cols[r] = pixels_in(gx0, 16, W, p.cull[r][0], p.cull[r][1]);
    for (int part = 0; part < spl; ++part) {
      const int gy0 = by * 16 + part * rows;
      const float wy0 = (2.0f * (float)gy0 / (float)H) - 1.0f;
      const float wy1 = (2.0f * (float)(gy0 + rows - 1) / (float)H) - 1.0f;
      bool any = p.n_cull < 0;   // no culling: every item is live
      for (int r = 0; r < p.n_cull && !any; ++r)
        any = wx1 >= p.cull[r][0] && wx0 <= p.cull[r][1] && wy1 >= p.cull[r][2] && wy0 <= p.cull[r][3];
      if (!any) {
        culled->push_back(li * spl + part);
        continue;
      }
      int w = 0;
      for (int r = 0; r < p.n_cull; ++r)
        if (cols[r]) w += (r == 0 ? 8 : 1) * cols[r] * pixels_in(gy0, rows, H, p.cull[r][2], p.cull[r][3]);
      weighted.push_back({-w, li * spl + part});
    }
  }
  if (p.item_order)
    std::stable_sort(weighted.begin(), weighted.end(),
                   [](const std::pair<int, int>& a, const std::pair<int, int>& b) { return a.first < b.first; });
  live->reserve(weighted.size());
  for (const auto& e : weighted) live->push_back(e.second);
}

// Mixed sample lanes (PT_OPT_MIXED_LANES): the first `budget` live tiles
// whose every part is live, in list order, become whole-tile items at one lane
// per pixel; every other live part keeps p.spl lanes and follows them.  The
// whole tiles are the cheapest per sample (8 samples per lane, no colour
// hand-off) but the longest workgroups, so they start first and at most one
// round of them runs; the short parts then fill the launch's drain.
static void mixed_origins(const ptd::RenderParams& p, const ptd::Part& part, const std::vector<int>& live,
                          long long budget, std::vector<int>* org) {
  const int spl = p.spl, rows = 16 / spl;
  const int tiles = ptd::part_count(part, p.blocks_total);
  std::vector<int> parts_live(tiles, 0);
  for (int it : live) parts_live[it / spl]++;
  std::vector<char> whole(tiles, 0);
  long long k = 0;
  const int lg = __builtin_ctz((unsigned)spl);
  for (int it : live) {
    const int li = it / spl;
    if (k >= budget) break;
    if (whole[li] || parts_live[li] != spl) continue;
    whole[li] = 1;
    ++k;
    int bx, by;
    ptd::tile_block(ptd::part_tile(part, li), p.blocks_x, &bx, &by);
    org->push_back(bx * 16);   // log2(1) = 0 in the lane-count bits
    org->push_back(by * 16);
  }
  for (int it : live) {
    const int li = it / spl;
    if (whole[li]) continue;
    int bx, by;
    ptd::tile_block(ptd::part_tile(part, li), p.blocks_x, &bx, &by);
    org->push_back((bx * 16) | (lg << ptd::kMixShift));
    org->push_back(by * 16 + (it % spl) * rows);
  }
}

// Per-sample cost of 1, 2, 4 and 8 lanes per pixel relative to one lane:
// the box 1080p 8-spp frame with frames in flight (no drain), 0.2037 /
// 0.2121 / 0.2385 / 0.2775 ms per frame (profiles/r06b).
static const double kLaneInfl[4] = {1.0, 0.2121 / 0.2037, 0.2385 / 0.2037, 0.2775 / 0.2037};

// The measured schedule of mixed lanes.  cost[k], k = y / 4 * blocks_x +
// x / 16: the live work of the frame's 16x4 part k at one lane per pixel
// (render_kernel's cost feedback: every wave's duration added to the part
// its pixels lie in, divided by the lane factor it ran at).  A workgroup at s
// lanes lasts about the costliest part it covers * kLaneInfl[s] / s.
// Whole-live tiles run as 16x8 halves at kWholeLanes = 2 lanes -- the least
// work per sample whose workgroups fit inside a frame: at one lane the
// costliest tiles outlast the whole frame at two -- and the live parts of
// tiles with culled parts at p.spl lanes.  Every item goes longest first
// (longest-processing-time list scheduling on the measured costs), so the
// launch ends on its lightest items.  Box 1080p 8 spp, one context
// (profiles/r06h, r06i): 0.2214 ms per frame against 0.2416 at 4 lanes in
// the same order and 0.2349 for the best static mix (whole tiles at one lane
// for half the resident workgroups); whole tiles at one lane as well lost
// (0.2620: they outlast the frame), and so did splitting the last 5-35 % of
// the work into 4-lane parts for a finer drain (+1 to +5 %).  Any item order
// and lane count gives the same image.
struct MixItem {
  int x, y;
  double dur;
};
constexpr int kWholeLanes = 2;
static void measured_origins(const ptd::RenderParams& p, const ptd::Part& part, const std::vector<int>& live,
                             const std::vector<double>& cost, std::vector<int>* org) {
  const int spl = p.spl, rows = 16 / spl, lg_base = __builtin_ctz((unsigned)spl);
  const int lanes = std::min(kWholeLanes, spl), lg_whole = __builtin_ctz((unsigned)lanes), hrows = 16 / lanes;
  const int tiles = ptd::part_count(part, p.blocks_total);
  std::vector<int> parts_live(tiles, 0);
  for (int it : live) parts_live[it / spl]++;
  auto part_cost = [&](int x, int y) {   // pixel (x, y)'s 16x4 part
    const size_t k = (size_t)(y >> 2) * p.blocks_x + (x >> 4);
    return k < cost.size() ? std::max(1.0, cost[k]) : 1.0;
  };
  auto span_cost = [&](int x, int y, int nrows) {   // the costliest 16x4 part of rows [y, y + nrows)
    double c = 0;
    for (int yy = y; yy < y + std::max(nrows, 4); yy += 4) c = std::max(c, part_cost(x, yy));
    return c;
  };
  std::vector<char> seen(tiles, 0);
  std::vector<MixItem> items;
  for (int it : live) {
    const int li = it / spl;
    int bx, by;
    ptd::tile_block(ptd::part_tile(part, li), p.blocks_x, &bx, &by);
    const int x = bx * 16, y = by * 16;
    if (parts_live[li] == spl) {   // a whole-live tile: its halves, once
      if (seen[li]) continue;
      seen[li] = 1;
      for (int h = 0; h < lanes; ++h)
        items.push_back({x | (lg_whole << ptd::kMixShift), y + h * hrows,
                         span_cost(x, y + h * hrows, hrows) * kLaneInfl[lg_whole] / lanes});
      continue;
    }
    const int yp = y + (it % spl) * rows;
    items.push_back({x | (lg_base << ptd::kMixShift), yp, span_cost(x, yp, rows) * kLaneInfl[lg_base] / spl});
  }
  std::stable_sort(items.begin(), items.end(), [](const MixItem& a, const MixItem& b) { return a.dur > b.dur; });
  for (const MixItem& m : items) {
    org->push_back(m.x);
    org->push_back(m.y);
  }
  if (const char* dump = getenv("PT_MIX_DUMP")) {   // diagnostics: the chosen schedule and its predicted durations
    if (FILE* f = fopen(dump, "w")) {
      fprintf(f, "# items %zu\n", items.size());
      for (const MixItem& m : items)
        fprintf(f, "I %d %d %d %.1f\n", m.x & ((1 << ptd::kMixShift) - 1), m.y, m.x >> ptd::kMixShift, m.dur);
      fclose(f);
    }
  }
}

// Cost feedback of the measured mixed-lane schedule (PT_OPT_MIXED_LANES -1).
// The schedule belongs to the frame's inputs (the cost key: size, batches,
// lanes, camera, params, scene and lights, culling).  Once the key has held
// for a render, one launch records its blocks' costs (render_kernel adds
// every wave's duration on the GPU wall clock to its block), copied back
// asynchronously behind an event; a later render whose event has completed
// folds them in, divided by the lane factor each block ran at, and after
// kCostFrames such launches the schedule is built from them
// (measured_origins).  The host never waits: a render whose copy has not
// landed keeps the static schedule.
constexpr int kCostFrames = 2;
static int mix_feedback(pt_context* c, const ptd::RenderParams& p, uint32_t n_batches) {
  std::vector<float>& key = c->cost_scratch;
  key.assign({(float)p.width, (float)p.height, (float)n_batches, (float)(p.first_batch == 0), (float)p.spl,
              (float)c->params.max_depth, (float)c->params.sss_bounces, (float)c->scene_serial, (float)p.n_cull,
              (float)c->opt_item_order});
  key.insert(key.end(), c->cam, c->cam + 16);
  for (int r = 0; r < p.n_cull; ++r) key.insert(key.end(), p.cull[r], p.cull[r] + 4);
  const size_t nb = (size_t)p.blocks_total;
  const size_t np4 = (size_t)p.blocks_x * (size_t)((p.height + 15) / 16) * 4;   // 16x4 parts
  if (key != c->cost_key) {
    c->cost_key = key;
    c->cost_stable = 0;
    c->cost_frames = 0;
    c->cost_ready = false;
    c->cost_measure = false;
    c->cost_stale = c->cost_pending;   // a copy in flight belongs to the old inputs
    c->block_cost.assign(np4, 0.0);
  }
  if (c->cost_pending && hipEventQuery(c->cost_ev) == hipSuccess) {
    c->cost_pending = false;
    if (!c->cost_stale && c->cost_lanes.size() == nb) {
      for (size_t k = 0; k < np4; ++k) {   // part k lies in block (k / blocks_x / 4, k % blocks_x)
        const size_t b = (k / (size_t)p.blocks_x / 4) * (size_t)p.blocks_x + k % (size_t)p.blocks_x;
        const int s = c->cost_lanes[b];
        if (s > 0) c->block_cost[k] += (double)c->h_cost[k] / kLaneInfl[__builtin_ctz((unsigned)s)];
      }
      if (++c->cost_frames >= kCostFrames) {
        for (double& x : c->block_cost) x /= c->cost_frames;
        c->cost_ready = true;
        c->cost_gen++;
      }
    }
    c->cost_stale = false;
  }
  c->cost_stable++;
  c->cost_measure = false;
  if (!c->cost_ready && !c->cost_pending && c->cost_stable >= 2) {
    if (c->cost_n < np4) {
      dev_free(c->d_cost);
      if (c->h_cost) (void)hipHostFree(c->h_cost);
      c->h_cost = nullptr;
      c->cost_n = 0;
      PT_HIP(hipMalloc((void**)&c->d_cost, np4 * sizeof(unsigned)));
      PT_HIP(hipHostMalloc((void**)&c->h_cost, np4 * sizeof(unsigned), hipHostMallocDefault));
      c->cost_n = np4;
    }
    if (!c->cost_ev) PT_HIP(hipEventCreateWithFlags(&c->cost_ev, hipEventDisableTiming));
    c->cost_measure = true;
  }
  return PT_OK;
}

// How a launch mixes lane counts (render_impl): PT_OPT_MIXED_LANES k > 0, a
// static budget of whole tiles (mixed_origins); -1, uniform lanes until the
// part costs are measured, then the measured schedule (measured_origins).
struct MixPlan {
  long long budget = 0;                       // whole tiles of the static schedule
  const std::vector<double>* cost = nullptr;  // measured part costs, or null
  int gen = 0;                                // measured schedule generation (cache key)
};

static int compact_items(pt_context* c, ptd::RenderParams* p, const MixPlan* mix = nullptr) {
  const long long mix_budget = mix ? (mix->cost ? -1 - mix->gen : mix->budget) : 0;
  const ptd::Part& pt = part_of(c, p->rank);
  // every slot position of this rank's share: two slot sets with the same
  // period, count and first position still deal different tiles
  std::vector<float>& key = c->items_scratch;
  key.assign({(float)p->width, (float)p->height, (float)pt.m, (float)pt.cnt, (float)p->rank, (float)p->spl,
              (float)p->n_cull, (float)p->item_order, (float)mix_budget});
  for (int k = 0; k < pt.cnt; ++k) key.push_back((float)pt.pos[k]);
  for (int r = 0; r < p->n_cull; ++r) key.insert(key.end(), p->cull[r], p->cull[r] + 4);
  if (key.size() != c->items_key.size() || memcmp(key.data(), c->items_key.data(), key.size() * 4) != 0) {
    std::vector<int> live, culled;
    item_lists(*p, pt, &live, &culled);
    { const int rc_ = quiesce(c); if (rc_) return rc_; }   // the previous list may still be in use
    // live items, culled items, then (8-B aligned) each culled item's first
    // pixel {x, y} for the fill (fill_culled: no tile arithmetic per pixel)
    c->h_items = live;
    c->h_items.insert(c->h_items.end(), culled.begin(), culled.end());
    if (c->h_items.size() & 1) c->h_items.push_back(0);
    const int rows = 16 / p->spl;
    auto origins = [&](const std::vector<int>& list) {
      for (int it : list) {
        int bx, by;
        ptd::tile_block(ptd::part_tile(pt, it / p->spl), p->blocks_x, &bx, &by);
        c->h_items.push_back(bx * 16);
        c->h_items.push_back(by * 16 + (it % p->spl) * rows);
      }
    };
    c->culled_org_off = c->h_items.size();
    origins(culled);
    c->live_org_off = c->h_items.size();
    int n_launch = (int)live.size();
    if (mix && (mix->cost || (p->spl > 1 && mix->budget > 0))) {
      std::vector<int> org;
      if (mix->cost)
        measured_origins(*p, pt, live, *mix->cost, &org);
      else
        mixed_origins(*p, pt, live, mix->budget, &org);
      c->h_items.insert(c->h_items.end(), org.begin(), org.end());
      n_launch = (int)(org.size() / 2);
    } else {
      origins(live);
    }
    if (c->h_items.size() > c->items_cap) {
      dev_free(c->d_items);
      c->items_cap = 0;
      PT_HIP(hipMalloc((void**)&c->d_items, c->h_items.size() * sizeof(int)));
      c->items_cap = c->h_items.size();
    }
    if (!c->h_items.empty())
      PT_HIP(hipMemcpy(c->d_items, c->h_items.data(), c->h_items.size() * sizeof(int), hipMemcpyHostToDevice));
    c->n_live_items = n_launch;
    c->n_culled_items = (int)culled.size();
    c->items_mixed = mix && (mix->cost || (p->spl > 1 && mix->budget > 0));
    // the lane count each block's workgroups run at (cost feedback)
    c->block_lanes.assign((size_t)p->blocks_total, 0);
    for (size_t k = 0; k + 1 < c->h_items.size() - c->live_org_off; k += 2) {
      const int ox = c->h_items[c->live_org_off + k], oy = c->h_items[c->live_org_off + k + 1];
      c->block_lanes[(size_t)(oy >> 4) * p->blocks_x + ((ox & ((1 << ptd::kMixShift) - 1)) >> 4)] =
          c->items_mixed ? 1 << (ox >> ptd::kMixShift) : p->spl;
    }
    c->items_key = key;
  }
  p->items = c->d_items;
  p->n_items = c->n_live_items;
  p->mix = c->items_mixed ? 1 : 0;
  p->culled_org = (const int2*)(c->d_items + c->culled_org_off);
  p->items_org = (const int2*)(c->d_items + c->live_org_off);
  p->n_culled_items = c->n_culled_items;
  return PT_OK;
}

namespace {
// The frame parameters an item layout depends on, into *key (its capacity is
// kept between launches: no allocation per launch).
void frame_key(const pt_context* c, const ptd::RenderParams& p, std::vector<float>* key) {
  key->assign({(float)p.width, (float)p.height, (float)p.nranks, (float)p.rank, (float)p.spl, (float)p.n_cull,
               (float)p.blocks_x, (float)p.blocks_total, (float)p.item_order});
  for (int r = 0; r < p.n_cull; ++r) key->insert(key->end(), p.cull[r], p.cull[r] + 4);
  for (int sl : c->slots) key->push_back((float)sl);   // every rank's share (the assembly table)
}
int upload_ints(const std::vector<int>& h, int** d, size_t* cap) {
  if (h.size() > *cap) {
    dev_free(*d);
    *cap = 0;
    PT_HIP(hipMalloc((void**)d, h.size() * sizeof(int)));
    *cap = h.size();
  }
  if (!h.empty()) PT_HIP(hipMemcpy(*d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice));
  return PT_OK;
}
// Wavefront buffers for `paths` paths in one allocation.  Up to 2^27 paths
// (416 B each: 56 GB of the 288-GB HBM) are kept per launch, so config 4's
// 4K x 16 spp frame (133M paths) runs as one chunk: every ray round has 8x
// the rays of a 2^24 chunk, and each round's drain (its longest walk) is paid
// 65 times per frame instead of 520 -- 767 -> 560 ms (2^26: 591).  More
// batches run in chunks of that size; an allocation that fails halves it.
constexpr long long kWfMaxPaths = 1ll << 27;
constexpr int kWfAutoTris = 32768;
constexpr int kWfWideAutoTris = 16384;   // ... with the culled wide walk (render_impl)
// The root's assembly table for frames rendered with params p: per rank its
// live items {rank, x0, y0, slot} and its culled items {rank, x0, y0, -1},
// (x0, y0) the item's first pixel.
int unpack_table(pt_context* c, const ptd::RenderParams& p, const std::vector<float>& key) {
  if (key == c->unpack_key) return PT_OK;
  std::vector<int> table, live, culled;
  for (int r = 0; r < p.nranks; ++r) {
    const ptd::Part pt = part_of(c, r);
    item_lists(p, pt, &live, &culled);
    // {rank, x0, y0, slot} (unpack_pixel)
    auto add = [&](int item, int slot) {
      int bx, by;
      ptd::tile_block(ptd::part_tile(pt, item / p.spl), p.blocks_x, &bx, &by);
      table.insert(table.end(), {r, bx * 16, by * 16 + (item % p.spl) * (16 / p.spl), slot});
    };
    for (size_t i = 0; i < live.size(); ++i) add(live[i], (int)i);
    for (int it : culled) add(it, -1);
  }
  std::vector<int> live_only;
  for (size_t k = 0; k + 3 < table.size(); k += 4)
    if (table[k + 3] >= 0) live_only.insert(live_only.end(), table.begin() + k, table.begin() + k + 4);
  { const int rc_ = quiesce(c); if (rc_) return rc_; }
  const int rc = upload_ints(table, &c->d_unpack, &c->unpack_cap);
  if (rc) return rc;
  const int rl = upload_ints(live_only, &c->d_unpack_live, &c->unpack_live_cap);
  if (rl) return rl;
  c->n_unpack = (int)(table.size() / 4);
  c->n_unpack_live = (int)(live_only.size() / 4);
  c->unpack_key = key;
  return PT_OK;
}
int wf_reserve(pt_context* c, long long pixels, uint32_t batches, long long* chunk_paths) {
  const long long limit = c->opt_wf_paths > 0 ? c->opt_wf_paths : kWfMaxPaths;
  long long want = std::max(pixels, std::min(pixels * (long long)batches, limit));
  if (c->wf_fail > 0) want = std::max(pixels, std::min(want, c->wf_fail / 2));   // an earlier allocation failed
  if (want > 0x7fffffffll) return fail(PT_ERR_UNSUPPORTED, "frame too large for the wavefront kernel");
  *chunk_paths = want;
  if (want <= c->wf.cap) return PT_OK;
  { const int rc_ = quiesce(c); if (rc_) return rc_; }
  dev_free(c->wf_block);
  c->wf = ptd::WfBuffers{};
  char* base = nullptr;
  size_t n = 0, b_state = 0, b_col = 0, b_rays = 0, b_ids = 0, b_hits = 0;
  for (;;) {
    n = (size_t)want;
    b_state = n * ptd::kWfStateF4 * 16, b_col = n * 16, b_rays = n * 32, b_ids = n * 4, b_hits = n * 8;
    const hipError_t e = hipMalloc((void**)&base, 2 * b_state + b_col + 2 * (b_rays + b_ids) + b_hits + 64);
    if (e == hipSuccess) break;
    (void)hipGetLastError();
    if (e != hipErrorOutOfMemory || want <= pixels) PT_HIP(e);
    c->wf_fail = want;
    want = std::max(pixels, want / 2);   // less memory than that: smaller chunks
  }
  *chunk_paths = want;
  c->wf_block = base;
  char* q = base;
  c->wf.state[0] = (float4*)q; q += b_state;
  c->wf.state[1] = (float4*)q; q += b_state;
  c->wf.colors = (float4*)q;   q += b_col;
  c->wf.rays[0] = (float4*)q;  q += b_rays;
  c->wf.rays[1] = (float4*)q;  q += b_rays;
  c->wf.hits = (float2*)q;     q += b_hits;
  c->wf.ids[0] = (int*)q;      q += b_ids;
  c->wf.ids[1] = (int*)q;      q += b_ids;
  c->wf.counters = (int*)q;
  c->wf.cap = want;
  return PT_OK;
}
}  // namespace

extern "C" int pt_items_pack(pt_context* c, void* dst);
extern "C" int pt_items_unpack_all(pt_context* c, const void* src, size_t slot_floats, void* frame);

namespace {
// pt_render / pt_render_packed (pack_out != null: fresh frame, live items
// written to pack_out in the pt_items_pack layout).
struct Assembly {   // pt_render_packed's optional gathered frame to assemble
  const void* src = nullptr;
  size_t slot_floats = 0;
  void* frame = nullptr;
};
// The parameters of a path-recursive launch as render_impl made it, so that
// pt_dist_run can launch the next frames of a run (same scene, camera,
// options and item layout; only the packed output and the frame to assemble
// change) without rebuilding them: the host cost of a frame is then the
// launch and its events (relaunch).
struct Launched {
  ptd::RenderParams p;
  bool lds = false, cnt = false, valid = false;
};
// One path-recursive launch of prepared parameters, timed as render_impl
// times its launches (PT_OPT_LAUNCH_TIMING).
int relaunch(pt_context* c, const ptd::RenderParams& p, bool lds, bool cnt) {
  const int slot = c->ring_n % pt_context::kRing;
  const bool timed = c->opt_timing > 0 && c->launch_n % c->opt_timing == 0;
  if (timed) PT_HIP(hipEventRecord(c->ring[slot][0], c->stream));
  PT_HIP(ptd::launch_render(p, false, lds, c->stream, cnt));
  if (timed) {
    PT_HIP(hipEventRecord(c->ring[slot][1], c->stream));
    c->ring_launch[slot] = c->launch_n;
    c->last_slot = slot;
    c->ring_n++;
    c->timed = true;
  }
  c->launch_n++;
  return PT_OK;
}
int render_impl(pt_context* c, uint32_t first_batch, uint32_t n_batches, float4* pack_out,
                const Assembly& as = Assembly(), Launched* launched = nullptr) {
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (!c->has_scene) return fail(PT_ERR_INVALID, "no scene uploaded");
  if (!c->has_camera) return fail(PT_ERR_INVALID, "no camera set");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer");
  ptd::RenderParams p;
  p.wide = nullptr;
  p.wide_tris = nullptr;
  p.wide_rank_of = nullptr;
  p.wide_ovf = nullptr;
  p.wide_ovf_lanes = 0;
  p.wide_stack = 0;
  p.wide_handback = 0;
  p.wf_fuse = 0;
  p.wf_tail = 0;
  p.wf_grid = c->opt_wf_grid;
  // PT_OPT_WF_REFILL auto: 16 idle lanes on a full grid, 8 on a split one
  // (more rays per lane per round; the refill's cost is shared by fewer
  // concurrent waves: profiles/r05i)
  p.wide_refill = c->opt_wf_refill > 0 ? c->opt_wf_refill : (c->opt_wf_grid < 100 ? 8 : 16);
  p.wide_qn = 0;
  p.wide_leafbox = nullptr;
  p.nodes = c->stats_mode ? c->d_nodes_full : c->d_nodes;
  p.tris = c->d_tris;
  p.hit_tris = c->d_tris;
  p.lights = c->d_lights_dev;
  p.accum = c->d_accum;
  p.stats = c->d_stats;
  p.n_nodes = c->stats_mode ? c->n_nodes_full : c->n_nodes;
  p.n_tris = c->n_tris;
  p.n_lights = c->n_lights;
  p.width = c->width;
  p.height = c->height;
  p.first_batch = first_batch;
  p.n_batches = n_batches;
  p.max_depth = c->params.max_depth;
  p.sss_bounces = c->params.sss_bounces;
  for (int i = 0; i < 3; ++i) {
    p.cam_pos[i] = c->cam[i];
    p.cam_dir[i] = c->cam[4 + i];
    p.cam_up[i] = c->cam[8 + i];
  }
  p.fov = c->cam[12];
  {
    using namespace ptm;
    const v3 cdir = mk(p.cam_dir[0], p.cam_dir[1], p.cam_dir[2]);
    const v3 cup = mk(p.cam_up[0], p.cam_up[1], p.cam_up[2]);
    const v3 right = normalize(cross(cdir, neg(cup)));
    const v3 up = normalize(cross(right, cdir));
    p.cam_right[0] = right.x; p.cam_right[1] = right.y; p.cam_right[2] = right.z;
    p.cam_upv[0] = up.x; p.cam_upv[1] = up.y; p.cam_upv[2] = up.z;
    p.tan_fov = tan_(radians_(p.fov * 0.5f));
  }
  p.blocks_x = (c->width + 15) / 16;
  p.blocks_total = p.blocks_x * ((c->height + 15) / 16);
  p.nranks = c->nranks;
  p.rank = c->rank;
  const ptd::Part& hpart = part_of(c, c->rank);
  {
    const int rc = sync_parts(c);
    if (rc) return rc;
  }
  p.part_m = hpart.m;
  p.part_cnt = hpart.cnt;
  p.part_pos = c->d_parts + (size_t)c->rank * ptd::kMaxSlots;
  p.n_tiles = ptd::part_count(hpart, p.blocks_total);
  p.fresh = pack_out ? 1 : c->opt_fresh;
  p.pack_out = nullptr;
  if (c->opt_sample_lanes) {
    p.spl = c->opt_sample_lanes;
  } else {
    // auto: 4 sample lanes per pixel for an LDS-resident scene on up to 7
    // ranks, else 8 — on a share of the frame each GPU's share shrinks while
    // its heaviest workgroup does not, and on big scenes the samples of one
    // pixel walk nearly the same nodes, so their loads coalesce.  Measured
    // at 1080p 8spp with culling and compact launch: box spl 1/2/4/8 =
    // 0.499/0.408/0.375/0.416 ms (whole frame), 0.354/0.264/0.225/0.221
    // (1/2), 0.271/0.156/0.094/0.085 (1/8); displaced sphere 828/645/582/563;
    // 1M cloud 968/930/927/923.  Never more lanes than samples.
    // With frames alternating between two streams (bench.py N > 1), the
    // 1/2 and 1/4 shares favour 4 lanes (0.187 vs 0.210, 0.101 vs 0.110 ms
    // per step) and the 1/8 share 8 (0.062 vs 0.069).  Round 3's kernels,
    // the emulated root step on the native loop (DESIGN Appendix A, round-3 share options;
    // two runs each): 1/2 share spl 2/4 = 0.1175/0.1225 ms, 1/4 share 4/8 =
    // 0.069/0.082, 1/8 share 4/8 = 0.046/0.042.  Round 5's kernels (the
    // build without the SLP vectorizer, profiles/r05zc/spl.log, 200 frames):
    // 1/2 share spl 1/2/4/8 = 0.1066/0.1067/0.118/0.1411 ms, 1/4 share
    // 0.0811/0.0594/0.0603/0.0692, 1/8 share 0.0725/0.0465/0.0348/0.0374.
    const bool small = ptd::scene_lds_bytes(p) <= ptd::kMaxSceneLds;
    int want = !small ? 8 : c->nranks >= 8 ? 4 : c->nranks >= 2 ? 2 : 4;
    while (want > 1 && (uint32_t)want > n_batches) want >>= 1;
    p.spl = want;
  }
  PT_HIP(hipSetDevice(c->device));
  const int slot = c->ring_n % pt_context::kRing;
  const bool timed = c->opt_timing > 0 && c->launch_n % c->opt_timing == 0;
  if (timed) PT_HIP(hipEventRecord(c->ring[slot][0], c->stream));
  const bool fits = ptd::scene_lds_bytes(p) <= ptd::kMaxSceneLds;
  if (c->opt_scene_lds == 2 && !fits) return fail(PT_ERR_UNSUPPORTED, "scene too large for the LDS variant");
  const bool lds = c->opt_scene_lds == 2 || (c->opt_scene_lds == 1 && fits);
  // auto: the wavefront pipeline for scenes of at least kWfAutoTris triangles
  // (not LDS-resident) when the launch holds enough paths to keep its node
  // loads in flight, the path-recursive kernel otherwise.  Measured at 1080p
  // (ms, recursive with paired walks -> wavefront): 1 spp (2M paths):
  // displaced sphere 82K tris 101 -> 108, 10M cloud 735 -> 669; 8 spp (16.6M):
  // sphere 550 -> 465, 100K cloud 113 -> 77; 1M cloud 2 spp 225 -> 236; a 1/8
  // tile share of the 10M cloud: 1 spp (259K paths) 147 -> 273, 8 spp (2M)
  // 742 -> 669; box 0.38 -> 8.4.
  // With the culled wide walk (PT_OPT_WIDE) the wavefront pipeline wins from
  // 2^20 paths on (1080p, ms recursive -> wavefront): displaced sphere 82K
  // 1 spp 89.9 -> 39.6, 8 spp 498 -> 139, its 1/8 tile share 89.0 -> 39.1;
  // 20K sphere 2 spp 29.6 -> 23.3; 1M cloud 1 spp 108 -> 47.5; a sparse 100K
  // cloud at 1 spp (most rays miss) loses 14.3 -> 15.9.
  const long long paths = (long long)p.n_tiles * 256 * n_batches;
  const bool wide_walk = c->opt_wide && c->n_wide > 0;
  const bool wf_auto = wide_walk ? c->n_tris >= kWfWideAutoTris && paths >= (1ll << 20)
                                 : c->n_tris >= kWfAutoTris && paths >= (1ll << 20) &&
                                       (c->n_tris >= (1 << 20) || paths >= (1ll << 23));
  const bool wf = c->opt_kernel == 3 || (c->opt_kernel == 0 && !lds && !c->stats_mode && wf_auto);
  if (wf && c->stats_mode) return fail(PT_ERR_UNSUPPORTED, "stats mode runs the path-recursive kernel only");
  const bool cnt = c->opt_count != 0 && !c->stats_mode;
  // PT_OPT_ITEM_ORDER auto: scan order for a whole frame on the path-recursive
  // kernel (box 1080p8 at 4 lanes, one context: 0.2403 against 0.2463 ms
  // heaviest first, profiles/r06b), heaviest first on a share of the frame
  // and on the wavefront pipeline
  p.item_order = c->opt_item_order >= 0 ? c->opt_item_order : (!wf && c->nranks == 1 ? 0 : 1);
  p.n_cull = -1;
  c->last_mix = 0;
  p.items = nullptr;
  p.culled_org = nullptr;
  p.items_org = nullptr;
  p.n_items = p.n_culled_items = 0;
  if (c->opt_cull && !c->stats_mode)
    p.n_cull = cull_rects(c->cam, c->width, c->height, c->root_lo, c->root_hi, c->lights_host.data(),
                          c->n_lights, &p.cull[0][0], ptd::kMaxCullRects);
  if (p.n_cull >= 0) {
    // mixed lanes (PT_OPT_MIXED_LANES): one rank, LDS-staged path-recursive
    // launches that render into the accumulation buffer
    MixPlan plan;
    bool mixed = false;
    // (one lane per pixel: the measured schedule only orders whole tiles)
    if (c->opt_mixed != 0 && !wf && lds && c->nranks == 1 && !pack_out && (p.spl > 1 || c->opt_mixed < 0) &&
        !cnt) {
      mixed = true;
      const size_t lds_b = ptd::scene_lds_bytes(p);
      if (c->render_slots < 0 || c->render_slots_lds != lds_b) {
        c->render_slots = ptd::render_slots(lds_b);
        c->render_slots_lds = lds_b;
      }
      // auto: every item at PT_OPT_SAMPLE_LANES until the block costs are
      // measured -- the measuring launches then run a uniform schedule, whose
      // workgroups nearly all run at full occupancy (a mixed one measured its
      // drain's parts at low occupancy, too short: profiles/r06g)
      plan.budget = c->opt_mixed > 0 ? std::max(1ll, c->render_slots * c->opt_mixed / 100) : 0;
      if (c->opt_mixed < 0) {
        const int rm = mix_feedback(c, p, n_batches);
        if (rm) return rm;
        if (c->cost_ready) {
          plan.cost = &c->block_cost;
          plan.gen = c->cost_gen;
        }
      }
    }
    const int rc = compact_items(c, &p, mixed ? &plan : nullptr);
    if (rc) return rc;
    c->last_mix = !mixed || !c->items_mixed ? 0 : plan.cost ? 2 : 1;
    if (mixed && c->opt_mixed < 0 && c->cost_measure) {
      // this launch measures its blocks' costs (mix_feedback)
      PT_HIP(hipMemsetAsync(c->d_cost, 0, (size_t)p.blocks_total * 4 * sizeof(unsigned), c->stream));
      p.cost_out = c->d_cost;
      c->cost_lanes = c->block_lanes;
    }
  }
  c->last = p;   // the item exchange (pt_items_*) follows the last rendered frame
  // Culled items written once (culled_state): a launch whose culled items
  // already hold (0,0,0,1) in this buffer under this item layout -- a fold of
  // (0,0,0,1) samples into (0,0,0,1) is (0,0,0,1), whatever the batch --
  // skips their fill workgroups (23 MB of writes per box 1080p frame).
  const bool culled_launch = p.n_cull >= 0 && p.items && !pack_out && !c->stats_mode && n_batches > 0;
  bool culled_skipped = false;
  if (culled_launch && c->culled_state == 2 && c->culled_buf == c->d_accum && c->culled_key == c->items_key) {
    p.n_culled_items = 0;
    culled_skipped = true;
  }
  c->last_kernel = wf ? 3 : 1;
  c->last_valid = true;
  p.unpack_src = nullptr;
  p.unpack_frame = nullptr;
  p.unpack_table = nullptr;
  p.n_unpack = 0;
  p.unpack_slot_f4 = 0;
  if (pack_out && as.frame == (void*)c->d_accum) c->culled_state = 0;   // the assembly writes this buffer
  if (pack_out) {
    frame_key(c, p, &c->key_scratch);
    const std::vector<float>& key = c->key_scratch;
    if (as.src && key != c->packed_key)
      return fail(PT_ERR_INVALID, "pt_render_packed: the frame to assemble has another item layout (size, partition, lanes, culling)");
    if (wf) {
      // these kernels render into the accumulation buffer: render, pack,
      // then assemble the previous frame in a launch of its own (the calls
      // below rebuild c->key_scratch: keep this frame's key)
      const std::vector<float> frame_k = key;
      if (as.src) {
        const int rc = pt_items_unpack_all(c, as.src, as.slot_floats, as.frame);
        if (rc) return rc;
      }
      const int fresh = c->opt_fresh;
      c->opt_fresh = 1;
      const int rc = render_impl(c, 0, n_batches, nullptr);
      c->opt_fresh = fresh;
      if (rc) return rc;
      c->packed_key = frame_k;
      const int rp = pt_items_pack(c, pack_out);
      if (rp) return rp;
      return mark_shared(c);   // the pack read the accumulation buffer
    }
    if (as.src) {
      const int rc = unpack_table(c, p, key);
      if (rc) return rc;
      p.unpack_src = (const float4*)as.src;
      p.unpack_frame = (float4*)as.frame;
      p.unpack_table = c->d_unpack;
      p.n_unpack = c->n_unpack;
      p.unpack_slot_f4 = (long long)(as.slot_floats / 4);
    }
    if (!p.items) p.n_items = p.n_tiles * p.spl;
    c->packed_key = key;
  }
  p.pack_out = pack_out;
  // every launch but the path-recursive render_packed writes the context's
  // accumulation buffer or wavefront buffers
  const bool shared = !pack_out || wf || c->stats_mode;
  if (shared) {
    const int ro = order_shared(c);
    if (ro) return ro;
  }
  if (wf) {
    const long long tiles = p.n_tiles;
    const long long items = p.items ? p.n_items : tiles * p.spl;
    long long chunk_paths = 0;
    const int rc = wf_reserve(c, items * (256 / p.spl), n_batches, &chunk_paths);
    if (rc) return rc;
    ptd::WfBuffers b = c->wf;
    b.cap = chunk_paths;   // paths per chunk (the allocation may be larger)
    if (c->opt_wide && c->n_wide > 0 && !lds) {
      const long long lanes = ptd::wide_trace_lanes();
      if (lanes <= 0) return fail(PT_ERR_HIP, "wide walk: occupancy query failed");
      const int stack = c->wide_stack;
      if (lanes > c->wide_ovf_lanes || stack > c->wide_ovf_stack) {   // every lane of the grid gets its area
        { const int rc_ = quiesce(c); if (rc_) return rc_; }
        dev_free(c->d_wide_ovf);
        c->wide_ovf_lanes = 0;
        // two sets: the two halves of a chunk trace concurrently (launch_wavefront)
        PT_HIP(hipMalloc((void**)&c->d_wide_ovf, 2 * (size_t)lanes * (size_t)stack * sizeof(int2)));
        c->wide_ovf_lanes = lanes;
        c->wide_ovf_stack = stack;
      }
      // closest hits come back as leaf ranks
      p.wide_qn = c->opt_wide_node == 64 ? 1 : 0;
      p.wide = p.wide_qn ? c->d_wide_q : c->d_wide;
      p.wide_leafbox = c->d_wide_leafbox;
      p.wide_tris = c->d_wide_tris;
      p.wide_rank_of = c->d_wide_rank_of;
      p.hit_tris = c->d_wide_tris;
      p.wide_ovf = c->d_wide_ovf;
      p.wide_ovf_lanes = c->wide_ovf_lanes;
      p.wide_stack = stack;
      p.wide_handback = c->opt_wide == 2 ? 1 : 0;
      // fused shadow walks: hit records carry the rank in 29 bits
      p.wf_fuse = c->opt_wf_fuse && c->n_tris <= ptd::kHitRankMask && c->n_lights > 0 ? 1 : 0;
      // wf_tail_kernel (4-wide layouts).  Auto: once a list holds fewer than
      // 400K rays (with the wave-wide flush, item 39; ab_bench device time):
      // emulated 1/8 tile shares of configs 3 / 4 / 5 13.48 -> 11.31, 64.68 ->
      // 64.26, 22.36 -> 21.91 ms; whole frames 44.28 -> 43.77, 384.41 ->
      // 384.89, 117.72 -> 117.39 ms.  (2^20: 11.17 / 65.31 / 22.39; from the
      // first list: +28-57 % on whole frames.)
      const int tail_auto = 400000;
      p.wf_tail = c->opt_wf_tail >= 0 ? c->opt_wf_tail : tail_auto;
    }
    if (c->opt_wf_streams == 2 && !c->wf_stream2) {
      PT_HIP(hipStreamCreateWithFlags(&c->wf_stream2, hipStreamNonBlocking));
      PT_HIP(hipEventCreateWithFlags(&c->wf_fork, hipEventDisableTiming));
      PT_HIP(hipEventCreateWithFlags(&c->wf_join, hipEventDisableTiming));
    }
    const bool two = c->opt_wf_streams == 2;
    PT_HIP(ptd::launch_wavefront(p, b, lds, c->stream, cnt, two ? c->wf_stream2 : nullptr, c->wf_fork, c->wf_join));
  } else {
    PT_HIP(ptd::launch_render(p, c->stats_mode, lds, c->stream, cnt));
    if (p.cost_out) {
      PT_HIP(hipMemcpyAsync(c->h_cost, c->d_cost, (size_t)p.blocks_total * 4 * sizeof(unsigned),
                            hipMemcpyDeviceToHost, c->stream));
      PT_HIP(hipEventRecord(c->cost_ev, c->stream));
      c->cost_pending = true;
      c->cost_measure = false;
    }
    if (launched && pack_out && !c->stats_mode) {
      launched->p = p;
      launched->lds = lds;
      launched->cnt = cnt;
      launched->valid = true;
    }
  }
  if (shared) {
    const int rm = mark_shared(c);
    if (rm) return rm;
  } else if (!c->in_dist) {
    const int ru = note_use(c);   // render_packed reads the scene and item tables
    if (ru) return ru;
  }
  if (timed) {
    PT_HIP(hipEventRecord(c->ring[slot][1], c->stream));
    c->ring_launch[slot] = c->launch_n;
    c->last_slot = slot;
    c->ring_n++;
    c->timed = true;
  }
  c->launch_n++;
  // the state of the culled items after this launch (culled_state)
  if (culled_launch && !culled_skipped) {
    const bool same = c->culled_state == 2 && c->culled_buf == c->d_accum && c->culled_key == c->items_key;
    const bool exact = (c->opt_fresh && first_batch == 0) || same ||
                       (first_batch == 0 && c->culled_state == 1 && c->culled_buf == c->d_accum);
    c->culled_state = exact ? 2 : 0;
    c->culled_key = c->items_key;
    c->culled_buf = c->d_accum;
  } else if (!culled_launch && !pack_out && n_batches > 0) {
    c->culled_state = 0;   // every pixel rendered (no culling, stats mode): not tracked
  }
  return PT_OK;
}

}  // namespace

int pt_fail_internal(int code, const std::string& msg) { return fail(code, msg); }
void pt_note_accum_written(pt_context* c, bool finite) {
  if (!c) return;
  c->culled_state = finite ? 1 : 0;
  c->culled_buf = c->d_accum;
}

extern "C" {

int pt_abi_version(void) { return PT_ABI_VERSION; }
const char* pt_last_error(void) { return g_err.c_str(); }

int pt_create(int device_ordinal, pt_context** out) {
  if (!out) return fail(PT_ERR_INVALID, "out is null");
  *out = nullptr;
  int n = 0;
  PT_HIP(hipGetDeviceCount(&n));
  if (device_ordinal < 0 || device_ordinal >= n)
    return fail(PT_ERR_INVALID, "device ordinal " + std::to_string(device_ordinal) + " out of range (" +
                                    std::to_string(n) + " devices)");
  PT_HIP(hipSetDevice(device_ordinal));
  hipDeviceProp_t prop;
  PT_HIP(hipGetDeviceProperties(&prop, device_ordinal));
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(PT_ERR_UNSUPPORTED, std::string("built for gfx950, device is ") + prop.gcnArchName);
  pt_context* c = new pt_context();
  c->device = device_ordinal;
  hipError_t e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc((void**)&c->d_stats, ptd::kStatsWords * sizeof(unsigned long long));
  if (e == hipSuccess) e = hipMemset(c->d_stats, 0, ptd::kStatsWords * sizeof(unsigned long long));
  for (int i = 0; i < pt_context::kRing && e == hipSuccess; ++i) {
    e = hipEventCreate(&c->ring[i][0]);
    if (e == hipSuccess) e = hipEventCreate(&c->ring[i][1]);
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->shared_ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    pt_destroy(c);
    return fail(PT_ERR_HIP, std::string("context setup: ") + hipGetErrorString(e));
  }
  c->stream = c->own_stream;
  *out = c;
  return PT_OK;
}

int pt_dist_finalize(pt_context* c);

int pt_create_multi(const int* device_ordinals, int n, pt_context** out) {
  if (!out || !device_ordinals) return fail(PT_ERR_INVALID, "null argument");
  *out = nullptr;
  pt_group* g = nullptr;
  const int rc = ptg::make(device_ordinals, n, &g);
  if (rc) return rc;
  pt_context* c = new pt_context();
  c->device = device_ordinals[0];
  c->group = g;
  *out = c;
  return PT_OK;
}

int pt_group_info(pt_context* c, int* n_devices, int* devices, int max_devices, int* peer_stores) {
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (!c->group) {
    if (n_devices) *n_devices = 1;
    if (devices && max_devices > 0) devices[0] = c->device;
    if (peer_stores) *peer_stores = 0;
    return PT_OK;
  }
  return ptg::members(c->group, n_devices, devices, max_devices, peer_stores);
}

int pt_group_check(pt_context* c, int* state, float* ms_peer, float* ms_staged) {
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (!c->group) {
    if (state) *state = -1;
    if (ms_peer) *ms_peer = 0.0f;
    if (ms_staged) *ms_staged = 0.0f;
    return PT_OK;
  }
  return ptg::check_info(c->group, state, ms_peer, ms_staged);
}

int pt_destroy(pt_context* c) {
  if (!c) return PT_OK;
  if (c->group) {   // a multi-device context: its members and buffers
    (void)ptg::destroy(c->group);
    delete c;
    return PT_OK;
  }
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->wf_stream2) (void)hipStreamSynchronize(c->wf_stream2);
  if (c->dist) (void)pt_dist_finalize(c);
  (void)quiesce(c);
  for (auto& u : c->uses) (void)hipEventDestroy(u.ev);
  c->uses.clear();
  dev_free(c->d_nodes);
  dev_free(c->d_nodes_full);
  dev_free(c->d_wide);
  dev_free(c->d_wide_q);
  dev_free(c->d_wide_leafbox);
  dev_free(c->d_wide_tris);
  dev_free(c->d_wide_rank_of);
  dev_free(c->d_wide_ovf);
  dev_free(c->d_tris);
  dev_free(c->d_lights);
  dev_free(c->d_lights_dev);
  if (c->own_accum) dev_free(c->d_accum);
  dev_free(c->d_stats);
  dev_free(c->d_items);
  dev_free(c->d_cost);
  if (c->h_cost) (void)hipHostFree(c->h_cost);
  if (c->cost_ev) (void)hipEventDestroy(c->cost_ev);
  dev_free(c->d_pack_items);
  dev_free(c->d_unpack);
  dev_free(c->d_unpack_live);
  dev_free(c->wf_block);
  for (auto& r : c->rb) {
    dev_free(r.dev);
    if (r.host) (void)hipHostFree(r.host);
    if (r.snap) (void)hipEventDestroy(r.snap);
    if (r.done) (void)hipEventDestroy(r.done);
  }
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  if (c->shared_ev) (void)hipEventDestroy(c->shared_ev);
  dev_free(c->d_parts);
  for (int i = 0; i < pt_context::kRing; ++i)
    for (int j = 0; j < 2; ++j)
      if (c->ring[i][j]) (void)hipEventDestroy(c->ring[i][j]);
  if (c->wf_stream2) (void)hipStreamDestroy(c->wf_stream2);
  if (c->wf_fork) (void)hipEventDestroy(c->wf_fork);
  if (c->wf_join) (void)hipEventDestroy(c->wf_join);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
  return PT_OK;
}

int pt_set_stream(pt_context* c, void* s) {
  if (c && c->group) return ptg::set_stream(c->group, s);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  c->stream = s ? (hipStream_t)s : c->own_stream;
  return PT_OK;
}

int pt_synchronize(pt_context* c) {
  if (c && c->group) return ptg::synchronize(c->group);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  PT_HIP(hipSetDevice(c->device));
  PT_HIP(hipStreamSynchronize(c->stream));
  if (c->dist) {   // the native step loop's streams
    for (hipStream_t s : {c->dist->streams[0], c->dist->streams[1], c->dist->comm_stream})
      if (s) PT_HIP(hipStreamSynchronize(s));
  }
  return PT_OK;
}

int pt_upload_scene(pt_context* c, const float* vertices, size_t n_vertex_floats, const uint32_t* indices,
                    size_t n_indices, const pt_bvh_node* nodes, size_t n_nodes, const float* uvs,
                    size_t n_uv_floats, const uint32_t* mat_indices, size_t n_mat, uint32_t flags) {
  if (c && c->group) return ptg::upload_scene(c->group, vertices, n_vertex_floats, indices, n_indices, nodes, n_nodes, uvs, n_uv_floats, mat_indices, n_mat, flags);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (!vertices || !indices || !nodes) return fail(PT_ERR_INVALID, "null scene array");
  if (n_vertex_floats % 3 || n_indices % 3 || n_indices == 0)
    return fail(PT_ERR_SCENE, "vertex/index array sizes must be non-zero multiples of 3");
  if (n_nodes != 2 * (n_indices / 3) - 1)
    return fail(PT_ERR_SCENE, "expected 2T-1 = " + std::to_string(2 * (n_indices / 3) - 1) + " nodes, got " +
                                  std::to_string(n_nodes));
  if ((n_uv_floats && !uvs) || (n_mat && !mat_indices)) return fail(PT_ERR_INVALID, "null uv/material array");
  if (n_indices / 3 > 0x7fffffffull) return fail(PT_ERR_UNSUPPORTED, "too many triangles");
  const size_t nv = n_vertex_floats / 3;
  for (size_t i = 0; i < n_indices; ++i)
    if (indices[i] >= nv) return fail(PT_ERR_SCENE, "vertex index out of range at " + std::to_string(i));
  std::vector<float4> threaded, collapsed;
  int rc = thread_bvh(nodes, n_nodes, (flags & PT_NODES_INT_BITS) != 0, n_indices / 3, &threaded);
  if (rc) return rc;
  collapse_implied(threaded, &collapsed);
  pt::WideBVH wide;
  const std::string wide_reason =
      pt::build_wide_bvh((const float*)nodes, n_nodes, (flags & PT_NODES_INT_BITS) != 0, vertices, n_vertex_floats,
                         indices, n_indices / 3, &wide, c->opt_wide_build);
  float lo[3] = {threaded[0].x, threaded[0].y, threaded[0].z};   // node 0 is the root
  float hi[3] = {threaded[1].x, threaded[1].y, threaded[1].z};
  PT_HIP(hipSetDevice(c->device));
  { const int rc_ = quiesce(c); if (rc_) return rc_; }
  dev_free(c->d_nodes);
  dev_free(c->d_nodes_full);
  dev_free(c->d_wide);
  dev_free(c->d_wide_q);
  dev_free(c->d_wide_leafbox);
  dev_free(c->d_wide_tris);
  dev_free(c->d_wide_rank_of);
  dev_free(c->d_tris);
  // the wide walk's overflow area is sized by the scene's stack bound: a
  // deeper tree needs a new one (it is reallocated at the next wide launch)
  dev_free(c->d_wide_ovf);
  c->wide_ovf_lanes = 0;
  c->wide_ovf_stack = 0;
  c->n_wide = 0;
  c->has_scene = false;
  const int T = (int)(n_indices / 3);
  struct Staging {   // vertex/index copies live only until the triangle records are built
    float* v = nullptr;
    uint32_t* i = nullptr;
    ~Staging() { if (v) (void)hipFree(v); if (i) (void)hipFree(i); }
  } st;
  // one zero node of padding past the end: the traversal loads node k+1
  // speculatively, also when k is the last node
  collapsed.push_back(make_float4(0, 0, 0, 0));
  collapsed.push_back(make_float4(0, 0, 0, 0));
  threaded.push_back(make_float4(0, 0, 0, 0));
  threaded.push_back(make_float4(0, 0, 0, 0));
  PT_HIP(hipMalloc((void**)&c->d_nodes, collapsed.size() * sizeof(float4)));
  PT_HIP(hipMalloc((void**)&c->d_nodes_full, threaded.size() * sizeof(float4)));
  PT_HIP(hipMalloc((void**)&c->d_tris, (size_t)T * 3 * sizeof(float4)));
  PT_HIP(hipMalloc((void**)&st.v, n_vertex_floats * sizeof(float) + 16));
  PT_HIP(hipMalloc((void**)&st.i, n_indices * sizeof(uint32_t)));
  PT_HIP(hipMemcpyAsync(c->d_nodes, collapsed.data(), collapsed.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  PT_HIP(hipMemcpyAsync(c->d_nodes_full, threaded.data(), threaded.size() * sizeof(float4), hipMemcpyHostToDevice, c->stream));
  PT_HIP(hipMemcpyAsync(st.v, vertices, n_vertex_floats * sizeof(float), hipMemcpyHostToDevice, c->stream));
  PT_HIP(hipMemcpyAsync(st.i, indices, n_indices * sizeof(uint32_t), hipMemcpyHostToDevice, c->stream));
  PT_HIP(ptd::launch_setup_tris(st.v, st.i, T, c->d_tris, c->stream));
  std::vector<int> rank_of_host(wide_reason.empty() ? (size_t)T : 0);
  if (wide_reason.empty()) {
    PT_HIP(hipMalloc((void**)&c->d_wide, wide.nodes.size() * sizeof(float)));
    PT_HIP(hipMalloc((void**)&c->d_wide_q, wide.qnodes.size() * sizeof(float)));
    PT_HIP(hipMalloc((void**)&c->d_wide_leafbox, wide.leaf_box.size() * sizeof(float)));
    PT_HIP(hipMemcpyAsync(c->d_wide_q, wide.qnodes.data(), wide.qnodes.size() * sizeof(float), hipMemcpyHostToDevice,
                          c->stream));
    PT_HIP(hipMemcpyAsync(c->d_wide_leafbox, wide.leaf_box.data(), wide.leaf_box.size() * sizeof(float),
                          hipMemcpyHostToDevice, c->stream));
    PT_HIP(hipMalloc((void**)&c->d_wide_rank_of, (size_t)T * sizeof(int)));
    PT_HIP(hipMalloc((void**)&c->d_wide_tris, (size_t)T * 3 * sizeof(float4)));
    PT_HIP(hipMemcpyAsync(c->d_wide, wide.nodes.data(), wide.nodes.size() * sizeof(float), hipMemcpyHostToDevice,
                          c->stream));
    PT_HIP(hipMemcpyAsync(c->d_wide_rank_of, wide.rank_tri.data(), (size_t)T * sizeof(int), hipMemcpyHostToDevice,
                          c->stream));
    PT_HIP(ptd::launch_gather_tris(c->d_tris, c->d_wide_rank_of, T, c->d_wide_tris, c->stream));
    // then the same buffer becomes slot -> rank (the kernels' only use of it)
    for (int r = 0; r < T; ++r) rank_of_host[wide.rank_tri[r]] = r;
    PT_HIP(hipMemcpyAsync(c->d_wide_rank_of, rank_of_host.data(), (size_t)T * sizeof(int), hipMemcpyHostToDevice,
                          c->stream));
  }
  PT_HIP(hipStreamSynchronize(c->stream));
  c->n_wide = wide_reason.empty() ? wide.n_nodes : 0;
  c->wide_stack = wide.stack_cap;
  c->wide_reason = wide_reason;
  c->n_nodes = (int)(collapsed.size() / 2) - 1;
  c->n_nodes_full = (int)(threaded.size() / 2) - 1;
  c->n_tris = T;
  memcpy(c->root_lo, lo, sizeof lo);
  memcpy(c->root_hi, hi, sizeof hi);
  c->has_scene = true;
  c->scene_serial++;
  return PT_OK;
}

int pt_upload_lights(pt_context* c, const pt_area_light* lights, size_t n) {
  if (c && c->group) return ptg::upload_lights(c->group, lights, n);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (n && !lights) return fail(PT_ERR_INVALID, "null lights");
  if (n > 1024) return fail(PT_ERR_UNSUPPORTED, "more than 1024 lights");
  PT_HIP(hipSetDevice(c->device));
  { const int rc_ = quiesce(c); if (rc_) return rc_; }
  dev_free(c->d_lights);
  dev_free(c->d_lights_dev);
  c->n_lights = 0;
  c->lights_host.clear();
  if (n) {
    PT_HIP(hipMalloc((void**)&c->d_lights, n * sizeof(ptd::LightRec)));
    PT_HIP(hipMalloc((void**)&c->d_lights_dev, n * sizeof(ptd::LightDev)));
    PT_HIP(hipMemcpyAsync(c->d_lights, lights, n * sizeof(ptd::LightRec), hipMemcpyHostToDevice, c->stream));
    PT_HIP(ptd::launch_setup_lights(c->d_lights, (int)n, c->d_lights_dev, c->stream));
    PT_HIP(hipStreamSynchronize(c->stream));
  }
  c->n_lights = (int)n;
  c->lights_host.assign(lights, lights + n);
  c->scene_serial++;
  return PT_OK;
}

int pt_set_camera(pt_context* c, const float ubo[16]) {
  if (c && c->group) return ptg::set_camera(c->group, ubo);
  if (!c || !ubo) return fail(PT_ERR_INVALID, "null argument");
  memcpy(c->cam, ubo, sizeof c->cam);
  c->has_camera = true;
  return PT_OK;
}

int pt_set_params(pt_context* c, const pt_params* p) {
  if (c && c->group) return ptg::set_params(c->group, p);
  if (!c || !p) return fail(PT_ERR_INVALID, "null argument");
  if (p->max_depth < 0 || p->max_depth > 64 || p->sss_bounces < 0 || p->sss_bounces > 64)
    return fail(PT_ERR_INVALID, "max_depth and sss_bounces must be in [0,64]");
  c->params = *p;
  return PT_OK;
}

int pt_set_partition(pt_context* c, int nranks, int rank) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_set_partition: not on a multi-device context (pt_create_multi)");
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(PT_ERR_INVALID, "bad partition");
  c->nranks = nranks;
  c->rank = rank;
  c->slots.assign((size_t)nranks, 1);
  c->parts_valid = false;
  c->items_key.clear();   // the cached item lists follow the partition
  return PT_OK;
}

int pt_set_partition_slots(pt_context* c, int nranks, int rank, const int* slots) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_set_partition_slots: not on a multi-device context (pt_create_multi)");
  if (!c || !slots) return fail(PT_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(PT_ERR_INVALID, "bad partition");
  long long m = 0;
  for (int r = 0; r < nranks; ++r) {
    if (slots[r] < 1 || slots[r] > ptd::kMaxSlots) return fail(PT_ERR_INVALID, "partition slots must be 1..64 per rank");
    m += slots[r];
  }
  if (m > 4096) return fail(PT_ERR_INVALID, "more than 4096 partition slots");
  c->nranks = nranks;
  c->rank = rank;
  c->slots.assign(slots, slots + nranks);
  c->parts_valid = false;
  c->items_key.clear();
  return PT_OK;
}

int pt_clear_accum(pt_context* c) {
  if (c && c->group) return ptg::clear_accum(c->group);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer");
  PT_HIP(hipSetDevice(c->device));
  const int ro = order_shared(c);
  if (ro) return ro;
  {
    const int rc = sync_parts(c);
    if (rc) return rc;
  }
  PT_HIP(ptd::launch_clear(c->d_accum, c->width, c->height, part_of(c, c->rank),
                           c->d_parts + (size_t)c->rank * ptd::kMaxSlots, c->stream));
  c->culled_state = 1;
  c->culled_buf = c->d_accum;
  return mark_shared(c);
}

int pt_resize_and_clear(pt_context* c, int w, int h) {
  if (c && c->group) return ptg::resize_and_clear(c->group, w, h);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (w <= 0 || h <= 0 || (long long)w * h > (1ll << 31)) return fail(PT_ERR_INVALID, "bad resolution");
  PT_HIP(hipSetDevice(c->device));
  if (!(c->own_accum && c->width == w && c->height == h)) {
    { const int rc_ = quiesce(c); if (rc_) return rc_; }
    if (c->own_accum) dev_free(c->d_accum);
    c->d_accum = nullptr;
    c->own_accum = false;
    PT_HIP(hipMalloc((void**)&c->d_accum, (size_t)w * h * sizeof(float4)));
    c->own_accum = true;
    c->width = w;
    c->height = h;
  }
  return pt_clear_accum(c);
}

int pt_bind_accum(pt_context* c, void* ptr, int w, int h) {
  if (c && c->group) return ptg::bind_accum(c->group, ptr, w, h);
  if (!c || !ptr) return fail(PT_ERR_INVALID, "null argument");
  if (w <= 0 || h <= 0) return fail(PT_ERR_INVALID, "bad resolution");
  if (((uintptr_t)ptr) & 15) return fail(PT_ERR_INVALID, "accumulation buffer must be 16-B aligned");
  PT_HIP(hipSetDevice(c->device));
  { const int rc_ = quiesce(c); if (rc_) return rc_; }
  if (c->own_accum) dev_free(c->d_accum);
  c->d_accum = (float4*)ptr;
  c->own_accum = false;
  c->width = w;
  c->height = h;
  c->culled_state = 0;   // the caller's buffer: its content is not known
  return PT_OK;
}

void* pt_accum_device_ptr(pt_context* c) {
  if (c && c->group) return ptg::accum_device_ptr(c->group);
  return c ? (void*)c->d_accum : nullptr;
}

int pt_read_accum(pt_context* c, float* rgba, size_t n) {
  if (c && c->group) return ptg::read_accum(c->group, rgba, n);
  if (!c || !rgba) return fail(PT_ERR_INVALID, "null argument");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer");
  const size_t need = (size_t)c->width * c->height * 4;
  if (n < need) return fail(PT_ERR_INVALID, "output buffer too small: need " + std::to_string(need) + " floats");
  PT_HIP(hipSetDevice(c->device));
  const int ro = order_shared(c);
  if (ro) return ro;
  PT_HIP(hipMemcpyAsync(rgba, c->d_accum, need * sizeof(float), hipMemcpyDeviceToHost, c->stream));
  PT_HIP(hipStreamSynchronize(c->stream));
  return PT_OK;
}

int pt_render(pt_context* c, uint32_t first_batch, uint32_t n_batches) {
  if (c && c->group) return ptg::render(c->group, first_batch, n_batches);
  return render_impl(c, first_batch, n_batches, nullptr);
}

// The gather step of a tile split (bench.py N>1): a fresh frame rendered from
// batch 0 whose live items go straight into the pt_items_pack layout -- one
// launch instead of render + culled fill + pack, and no accumulation-buffer
// traffic.  The accumulation buffer is neither read nor written.
int pt_render_packed(pt_context* c, uint32_t n_batches, void* packed, const void* gathered, size_t slot_floats,
                     void* frame) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_render_packed: not on a multi-device context (pt_create_multi)");
  if (!c || !packed) return fail(PT_ERR_INVALID, "null argument");
  if (((uintptr_t)packed) & 15) return fail(PT_ERR_INVALID, "packed buffer must be 16-B aligned");
  if (c->stats_mode) return fail(PT_ERR_UNSUPPORTED, "stats mode renders into the accumulation buffer");
  Assembly as;
  if (gathered) {
    if (!frame) return fail(PT_ERR_INVALID, "gathered slots without a frame");
    if ((((uintptr_t)gathered) & 15) || (((uintptr_t)frame) & 15) || (slot_floats & 3))
      return fail(PT_ERR_INVALID, "buffers must be 16-B aligned, slots whole float4s");
    as.src = gathered;
    as.slot_floats = slot_floats;
    as.frame = frame;
  }
  return render_impl(c, 0, n_batches, (float4*)packed, as);
}

int pt_dispatch(pt_context* c, uint32_t sample_batch) { return pt_render(c, sample_batch, 1); }

// ---- progressive loop + asynchronous readback -----------
// The reference's mainLoop (VulkanRayTracer.cpp:717-865) resets sampleBatch to
// 0 whenever any camera field changes (:739-754; batch 0 weights the old image
// by 0), dispatches one 1-spp batch, waits on two fences and copies the image
// out, up to 1024 batches (:719, :857).  Here a camera change resets the
// counter the same way, pending batches go out as one fused launch, and a
// readback snapshots the image on the render stream (device-to-device) and
// copies it to pinned host memory on a second stream, so rendering goes on
// while the previous frame travels over PCIe.
int pt_progressive_camera(pt_context* c, const float ubo[16], int* reset) {
  if (c && c->group) return ptg::progressive_camera(c->group, ubo, reset);
  if (!c || !ubo) return fail(PT_ERR_INVALID, "null argument");
  const bool changed = !c->prog_has_cam || memcmp(ubo, c->prog_cam, sizeof c->prog_cam) != 0;
  if (changed) {
    memcpy(c->prog_cam, ubo, sizeof c->prog_cam);
    c->prog_has_cam = true;
    c->prog_batch = 0;
    const int rc = pt_set_camera(c, ubo);
    if (rc) return rc;
  }
  if (reset) *reset = changed ? 1 : 0;
  return PT_OK;
}

int pt_progressive_advance(pt_context* c, uint32_t max_new, uint32_t limit, uint32_t* first, uint32_t* count) {
  if (c && c->group) return ptg::progressive_advance(c->group, max_new, limit, first, count);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  if (!c->prog_has_cam) return fail(PT_ERR_INVALID, "no camera (pt_progressive_camera)");
  const uint32_t room = limit > c->prog_batch ? limit - c->prog_batch : 0u;
  const uint32_t n = max_new < room ? max_new : room;
  if (first) *first = c->prog_batch;
  if (count) *count = n;
  if (n == 0) return PT_OK;
  const int rc = pt_render(c, c->prog_batch, n);
  if (rc) return rc;
  c->prog_batch += n;
  return PT_OK;
}

int pt_readback_begin(pt_context* c, int* ticket) {
  if (c && c->group) return ptg::readback_begin(c->group, ticket);
  if (!c || !ticket) return fail(PT_ERR_INVALID, "null argument");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer");
  PT_HIP(hipSetDevice(c->device));
  if (!c->copy_stream) PT_HIP(hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking));
  // the free slot, else the older one (its unread result is dropped)
  int slot = c->rb[0].ticket == 0 ? 0 : c->rb[1].ticket == 0 ? 1 : (c->rb[0].ticket < c->rb[1].ticket ? 0 : 1);
  pt_context::Readback& r = c->rb[slot];
  if (r.ticket) PT_HIP(hipEventSynchronize(r.done));
  const size_t bytes = (size_t)c->width * c->height * sizeof(float4);
  if (r.bytes != bytes) {
    dev_free(r.dev);
    if (r.host) (void)hipHostFree(r.host);
    r.host = nullptr;
    r.bytes = 0;
    PT_HIP(hipMalloc((void**)&r.dev, bytes));
    PT_HIP(hipHostMalloc(&r.host, bytes, hipHostMallocDefault));
    r.bytes = bytes;
  }
  if (!r.snap) PT_HIP(hipEventCreateWithFlags(&r.snap, hipEventDisableTiming));
  if (!r.done) PT_HIP(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
  {
    const int ro = order_shared(c);
    if (ro) return ro;
  }
  PT_HIP(hipMemcpyAsync(r.dev, c->d_accum, bytes, hipMemcpyDeviceToDevice, c->stream));
  {
    const int ru = note_use(c);
    if (ru) return ru;
  }
  PT_HIP(hipEventRecord(r.snap, c->stream));
  PT_HIP(hipStreamWaitEvent(c->copy_stream, r.snap, 0));
  PT_HIP(hipMemcpyAsync(r.host, r.dev, bytes, hipMemcpyDeviceToHost, c->copy_stream));
  PT_HIP(hipEventRecord(r.done, c->copy_stream));
  r.w = c->width;
  r.h = c->height;
  r.ticket = c->rb_next_ticket++;
  *ticket = r.ticket;
  return PT_OK;
}

int pt_readback_end(pt_context* c, int ticket, float* rgba, size_t n) {
  if (c && c->group) return ptg::readback_end(c->group, ticket, rgba, n);
  if (!c || !rgba) return fail(PT_ERR_INVALID, "null argument");
  for (auto& r : c->rb) {
    if (r.ticket != ticket || ticket == 0) continue;
    const size_t need = (size_t)r.w * r.h * 4;
    if (n < need) return fail(PT_ERR_INVALID, "output buffer too small: need " + std::to_string(need) + " floats");
    PT_HIP(hipSetDevice(c->device));
    PT_HIP(hipEventSynchronize(r.done));
    memcpy(rgba, r.host, need * sizeof(float));
    r.ticket = 0;
    return PT_OK;
  }
  return fail(PT_ERR_INVALID, "unknown or already collected readback ticket " + std::to_string(ticket));
}

int pt_last_kernel(pt_context* c, int* kernel) {
  if (c && c->group) return ptg::last_kernel(c->group, kernel);
  if (!c || !kernel) return fail(PT_ERR_INVALID, "null argument");
  *kernel = c->last_kernel;
  return PT_OK;
}

int pt_set_option(pt_context* c, int key, int value) {
  if (c && c->group) return ptg::set_option(c->group, key, value);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  switch (key) {
    case PT_OPT_KERNEL:
      if (value == 2) return fail(PT_ERR_UNSUPPORTED, "PT_OPT_KERNEL 2 (lane state machine) was removed: slower on every scene");
      if (value < 0 || value > 3) return fail(PT_ERR_INVALID, "PT_OPT_KERNEL takes 0, 1 or 3");
      c->opt_kernel = value;
      return PT_OK;
    case PT_OPT_WIDE:
      if (value < 0 || value > 2) return fail(PT_ERR_INVALID, "PT_OPT_WIDE takes 0, 1 or 2");
      c->opt_wide = value;
      return PT_OK;
    case PT_OPT_WIDE_NODE:
      if (value == 80) return fail(PT_ERR_UNSUPPORTED, "PT_OPT_WIDE_NODE 80 (8-wide nodes) was removed: slower on every scene");
      if (value != 64 && value != 128) return fail(PT_ERR_INVALID, "PT_OPT_WIDE_NODE takes 64 or 128");
      c->opt_wide_node = value;
      return PT_OK;
    case PT_OPT_WF_FUSE:
      if (value != 0 && value != 1) return fail(PT_ERR_INVALID, "PT_OPT_WF_FUSE takes 0 or 1");
      c->opt_wf_fuse = value;
      return PT_OK;
    case PT_OPT_WF_TAIL:
      if (value < -1) return fail(PT_ERR_INVALID, "PT_OPT_WF_TAIL takes -1 (auto) or a ray count >= 0");
      c->opt_wf_tail = value;
      return PT_OK;
    case PT_OPT_WF_REFILL:
      if (value < 0 || value > 64) return fail(PT_ERR_INVALID, "PT_OPT_WF_REFILL takes 0 (auto) to 64 idle lanes");
      c->opt_wf_refill = value;
      return PT_OK;
    case PT_OPT_WF_GRID:
      if (value < 1 || value > 100) return fail(PT_ERR_INVALID, "PT_OPT_WF_GRID takes 1 to 100 (percent)");
      c->opt_wf_grid = value;
      return PT_OK;
    case PT_OPT_WF_STREAMS:
      if (value != 1 && value != 2) return fail(PT_ERR_INVALID, "PT_OPT_WF_STREAMS takes 1 or 2");
      c->opt_wf_streams = value;
      return PT_OK;
    case PT_OPT_WIDE_BUILD:
      if (value != 0 && value != 1) return fail(PT_ERR_INVALID, "PT_OPT_WIDE_BUILD takes 0 or 1");
      c->opt_wide_build = value;
      return PT_OK;
    case PT_OPT_PAIRS:
      if (value == 1) return fail(PT_ERR_UNSUPPORTED, "PT_OPT_PAIRS 1 (child-pair records) was removed: slower on every scene");
      if (value != 0) return fail(PT_ERR_INVALID, "PT_OPT_PAIRS takes 0");
      return PT_OK;
    case PT_OPT_COUNT_TRACED:
      if (value != 0 && value != 1) return fail(PT_ERR_INVALID, "PT_OPT_COUNT_TRACED takes 0 or 1");
      c->opt_count = value;
      return PT_OK;
    case PT_OPT_PRIMARY_CULL:
      if (value != 0 && value != 1) return fail(PT_ERR_INVALID, "PT_OPT_PRIMARY_CULL takes 0 or 1");
      c->opt_cull = value;
      return PT_OK;
    case PT_OPT_WF_PATHS:
      if (value < 0) return fail(PT_ERR_INVALID, "PT_OPT_WF_PATHS takes 0 or a path count");
      c->opt_wf_paths = value;
      return PT_OK;
    case PT_OPT_SM_BATCH:
      return fail(PT_ERR_UNSUPPORTED, "PT_OPT_SM_BATCH: the lane state-machine kernel was removed");
    case PT_OPT_LAUNCH_TIMING:
      if (value < 0) return fail(PT_ERR_INVALID, "PT_OPT_LAUNCH_TIMING takes 0 (off) or k >= 1 (every k-th launch)");
      c->opt_timing = value;
      return PT_OK;
    case PT_OPT_MIXED_LANES:
      if (value < -1 || value > 1000) return fail(PT_ERR_INVALID, "PT_OPT_MIXED_LANES takes -1 (auto), 0 (off) or 1-1000");
      c->opt_mixed = value;
      return PT_OK;
    case PT_OPT_ITEM_ORDER:
      if (value < -1 || value > 1) return fail(PT_ERR_INVALID, "PT_OPT_ITEM_ORDER takes -1 (auto), 0 or 1");
      c->opt_item_order = value;
      return PT_OK;
    case PT_OPT_FRESH_BATCH0:
      if (value != 0 && value != 1) return fail(PT_ERR_INVALID, "PT_OPT_FRESH_BATCH0 takes 0 or 1");
      c->opt_fresh = value;
      return PT_OK;
    case PT_OPT_SAMPLE_LANES:
      if (value != 0 && value != 1 && value != 2 && value != 4 && value != 8)
        return fail(PT_ERR_INVALID, "PT_OPT_SAMPLE_LANES takes 0 (auto), 1, 2, 4 or 8");
      c->opt_sample_lanes = value;
      return PT_OK;
    case PT_OPT_SCENE_IN_LDS:
      if (value < 0 || value > 2) return fail(PT_ERR_INVALID, "PT_OPT_SCENE_IN_LDS takes 0, 1 or 2");
      c->opt_scene_lds = value;
      return PT_OK;
    case PT_OPT_GROUP_EXCHANGE:
    case PT_OPT_GROUP_CHECK:
      return fail(PT_ERR_UNSUPPORTED, "option " + std::to_string(key) + ": multi-device contexts only (pt_create_multi)");
    default:
      return fail(PT_ERR_INVALID, "unknown option " + std::to_string(key));
  }
}

int pt_tiles_owned(pt_context* c, int* n_tiles) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_tiles_owned: not on a multi-device context (pt_create_multi)");
  if (!c || !n_tiles) return fail(PT_ERR_INVALID, "null argument");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer");
  *n_tiles = ptd::owned_tiles(c->width, c->height, part_of(c, c->rank));
  return PT_OK;
}

int pt_tiles_pack(pt_context* c, void* dst) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_tiles_pack: not on a multi-device context (pt_create_multi)");
  if (!c || !dst) return fail(PT_ERR_INVALID, "null argument");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer");
  PT_HIP(hipSetDevice(c->device));
  const int ro = order_shared(c);
  if (ro) return ro;
  {
    const int rc = sync_parts(c);
    if (rc) return rc;
  }
  PT_HIP(ptd::launch_tiles(true, c->d_accum, (float4*)dst, c->width, c->height, part_of(c, c->rank),
                           c->d_parts + (size_t)c->rank * ptd::kMaxSlots, c->stream));
  return mark_shared(c);
}

int pt_tiles_unpack(pt_context* c, const void* src, int src_rank, void* frame) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_tiles_unpack: not on a multi-device context (pt_create_multi)");
  if (!c || !src || !frame) return fail(PT_ERR_INVALID, "null argument");
  if (!c->d_accum) return fail(PT_ERR_INVALID, "no accumulation buffer (it sets the frame size)");
  if (src_rank < 0 || src_rank >= c->nranks) return fail(PT_ERR_INVALID, "src_rank out of range");
  if ((((uintptr_t)src) & 15) || (((uintptr_t)frame) & 15)) return fail(PT_ERR_INVALID, "buffers must be 16-B aligned");
  PT_HIP(hipSetDevice(c->device));
  {
    const int rc = sync_parts(c);
    if (rc) return rc;
  }
  PT_HIP(ptd::launch_tiles(false, (float4*)frame, (float4*)src, c->width, c->height, part_of(c, src_rank),
                           c->d_parts + (size_t)src_rank * ptd::kMaxSlots, c->stream));
  if (frame == (void*)c->d_accum) c->culled_state = 0;
  return note_use(c);
}

// ---- sparse tile exchange (live items only) --------------------------------

int pt_items_live(pt_context* c, int rank, int* n_items, int* item_pixels) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_items_live: not on a multi-device context (pt_create_multi)");
  if (!c || !n_items || !item_pixels) return fail(PT_ERR_INVALID, "null argument");
  if (!c->last_valid) return fail(PT_ERR_INVALID, "no path-recursive pt_render yet");
  if (rank < 0 || rank >= c->last.nranks || rank >= (int)c->slots.size()) return fail(PT_ERR_INVALID, "rank out of range");
  std::vector<int> live, culled;
  item_lists(c->last, part_of(c, rank), &live, &culled);
  *n_items = (int)live.size();
  *item_pixels = 256 / c->last.spl;
  return PT_OK;
}

int pt_items_pack(pt_context* c, void* dst) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_items_pack: not on a multi-device context (pt_create_multi)");
  if (!c || !dst) return fail(PT_ERR_INVALID, "null argument");
  if (!c->last_valid || !c->d_accum) return fail(PT_ERR_INVALID, "no path-recursive pt_render yet");
  PT_HIP(hipSetDevice(c->device));
  frame_key(c, c->last, &c->key_scratch);
  const std::vector<float>& key = c->key_scratch;
  if (key != c->pack_key) {
    std::vector<int> live, culled;
    item_lists(c->last, part_of(c, c->last.rank), &live, &culled);
    { const int rc_ = quiesce(c); if (rc_) return rc_; }
    const int rc = upload_ints(live, &c->d_pack_items, &c->pack_cap);
    if (rc) return rc;
    c->n_pack_items = (int)live.size();
    c->pack_key = key;
  }
  const int ro = order_shared(c);
  if (ro) return ro;
  PT_HIP(ptd::launch_items_pack(c->last, c->d_accum, (float4*)dst, c->d_pack_items, c->n_pack_items, c->stream));
  return mark_shared(c);
}

int pt_items_unpack_all(pt_context* c, const void* src, size_t slot_floats, void* frame) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_items_unpack_all: not on a multi-device context (pt_create_multi)");
  if (!c || !src || !frame) return fail(PT_ERR_INVALID, "null argument");
  if (!c->last_valid) return fail(PT_ERR_INVALID, "no path-recursive pt_render yet");
  if (c->last.first_batch != 0)
    return fail(PT_ERR_INVALID, "sparse exchange needs a frame rendered from batch 0 (culled pixels are rebuilt)");
  if ((((uintptr_t)src) & 15) || (((uintptr_t)frame) & 15) || (slot_floats & 3))
    return fail(PT_ERR_INVALID, "buffers must be 16-B aligned, slots whole float4s");
  PT_HIP(hipSetDevice(c->device));
  frame_key(c, c->last, &c->key_scratch);
  const int rc = unpack_table(c, c->last, c->key_scratch);
  if (rc) return rc;
  PT_HIP(ptd::launch_items_unpack(c->last, (float4*)frame, (const float4*)src, slot_floats / 4, c->d_unpack,
                                  c->n_unpack, c->stream));
  if (frame == (void*)c->d_accum) c->culled_state = 0;
  return note_use(c);
}

int pt_set_stats_mode(pt_context* c, int enabled) {
  if (c && c->group) return ptg::set_stats_mode(c->group, enabled);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  c->stats_mode = enabled != 0;
  return PT_OK;
}

int pt_get_stats(pt_context* c, pt_stats* out) {
  if (c && c->group) return ptg::get_stats(c->group, out);
  if (!c || !out) return fail(PT_ERR_INVALID, "null argument");
  unsigned long long h[4];
  PT_HIP(hipSetDevice(c->device));
  PT_HIP(hipMemcpyAsync(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost, c->stream));
  PT_HIP(hipStreamSynchronize(c->stream));
  out->rays = h[0];
  out->nodes = h[1];
  out->leaf_tests = h[2];
  out->samples = h[3];
  return PT_OK;
}

int pt_wide_info(pt_context* c, int info[2]) {
  if (c && c->group) return ptg::wide_info(c->group, info);
  if (!c || !info) return fail(PT_ERR_INVALID, "null argument");
  info[0] = c->n_wide;
  info[1] = c->n_wide ? c->wide_stack : 0;
  if (!c->n_wide) g_err = c->wide_reason;
  return PT_OK;
}

int pt_mixed_info(pt_context* c, int info[3]) {
  if (!c || !info) return fail(PT_ERR_INVALID, "null argument");
  info[0] = info[1] = info[2] = 0;
  if (c->group) return PT_OK;
  info[0] = c->last_mix;
  info[1] = c->last_mix ? c->n_live_items : 0;
  info[2] = c->cost_frames;
  return PT_OK;
}

int pt_get_traced(pt_context* c, pt_traced* out) {
  if (c && c->group) return ptg::get_traced(c->group, out);
  if (!c || !out) return fail(PT_ERR_INVALID, "null argument");
  unsigned long long h[ptd::kStatsWords];
  PT_HIP(hipSetDevice(c->device));
  PT_HIP(hipMemcpyAsync(h, c->d_stats, sizeof h, hipMemcpyDeviceToHost, c->stream));
  PT_HIP(hipStreamSynchronize(c->stream));
  out->closest_walks = h[4];
  out->shadow_walks = h[5];
  out->nodes = h[6];
  out->tri_tests = h[7];
  out->primaries = h[8];
  return PT_OK;
}

int pt_reset_stats(pt_context* c) {
  if (c && c->group) return ptg::reset_stats(c->group);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  PT_HIP(hipSetDevice(c->device));
  PT_HIP(hipMemsetAsync(c->d_stats, 0, ptd::kStatsWords * sizeof(unsigned long long), c->stream));
  return note_use(c);
}

int pt_last_launch_ms(pt_context* c, float* ms) {
  if (c && c->group) return ptg::last_launch_ms(c->group, ms);
  if (!c || !ms) return fail(PT_ERR_INVALID, "null argument");
  if (!c->timed) return fail(PT_ERR_INVALID, "no launch recorded");
  PT_HIP(hipSetDevice(c->device));
  PT_HIP(hipEventSynchronize(c->ring[c->last_slot][1]));
  PT_HIP(hipEventElapsedTime(ms, c->ring[c->last_slot][0], c->ring[c->last_slot][1]));
  return PT_OK;
}

int pt_launch_times_ms(pt_context* c, float* out, size_t max_n, size_t* n_out) {
  if (c && c->group) return ptg::launch_times_ms(c->group, out, max_n, n_out);
  if (!c || !n_out) return fail(PT_ERR_INVALID, "null argument");
  const int have = c->ring_n < pt_context::kRing ? c->ring_n : pt_context::kRing;
  const int first = c->ring_n - have;
  size_t n = 0;
  PT_HIP(hipSetDevice(c->device));
  for (int k = first; k < c->ring_n && n < max_n; ++k) {
    const int slot = k % pt_context::kRing;
    PT_HIP(hipEventSynchronize(c->ring[slot][1]));
    if (out) PT_HIP(hipEventElapsedTime(&out[n], c->ring[slot][0], c->ring[slot][1]));
    ++n;
  }
  *n_out = n;
  return PT_OK;
}

// Launches may overlap (frames alternating between streams): the device time
// from the first launch's start to the last end, i.e. the busy span a
// throughput figure divides by.
int pt_launch_span_ms(pt_context* c, float* ms, size_t* n_out) {
  if (c && c->group) return ptg::launch_span_ms(c->group, ms, n_out);
  if (!c || !ms || !n_out) return fail(PT_ERR_INVALID, "null argument");
  if (c->ring_n == 0) return fail(PT_ERR_INVALID, "no launch recorded since pt_reset_launch_times");
  if (c->ring_n > pt_context::kRing) return fail(PT_ERR_UNSUPPORTED, "more launches than the event ring holds");
  PT_HIP(hipSetDevice(c->device));
  float span = 0.0f;
  for (int k = 0; k < c->ring_n; ++k) {
    float t = 0.0f;
    PT_HIP(hipEventSynchronize(c->ring[k][1]));
    PT_HIP(hipEventElapsedTime(&t, c->ring[0][0], c->ring[k][1]));
    span = t > span ? t : span;
  }
  *ms = span;
  *n_out = (size_t)(c->ring_launch[c->ring_n - 1] - c->ring_launch[0] + 1);   // launches the span covers
  return PT_OK;
}

int pt_reset_launch_times(pt_context* c) {
  if (c && c->group) return ptg::reset_launch_times(c->group);
  if (!c) return fail(PT_ERR_INVALID, "null context");
  c->ring_n = 0;
  c->launch_n = 0;
  return PT_OK;
}

int pt_selftest_math(int device, int fn, const float* x, float* y, size_t n) {
  if (!x || !y) return fail(PT_ERR_INVALID, "null argument");
  if (n == 0) return PT_OK;
  PT_HIP(hipSetDevice(device));
  float *dx = nullptr, *dy = nullptr;
  PT_HIP(hipMalloc((void**)&dx, n * sizeof(float)));
  hipError_t e = hipMalloc((void**)&dy, n * sizeof(float));
  if (e == hipSuccess) e = hipMemcpy(dx, x, n * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = ptd::launch_math(fn, dx, dy, n, nullptr);
  if (e == hipSuccess) e = hipMemcpy(y, dy, n * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(dx);
  if (dy) (void)hipFree(dy);
  if (e != hipSuccess) return fail(PT_ERR_HIP, std::string("pt_selftest_math: ") + hipGetErrorString(e));
  return PT_OK;
}

int pt_selftest_exhaustive(int device, int fn, unsigned long long* mismatches, uint32_t* first_bad) {
  if (!mismatches || !first_bad) return fail(PT_ERR_INVALID, "null argument");
  if (fn < 0 || fn > 3) return fail(PT_ERR_INVALID, "fn must be 0..3");
  PT_HIP(hipSetDevice(device));
  unsigned long long* d_bad = nullptr;
  PT_HIP(hipMalloc((void**)&d_bad, 16));
  hipError_t e = hipMemset(d_bad, 0, 8);
  if (e == hipSuccess) e = hipMemset((char*)d_bad + 8, 0xff, 4);
  if (e == hipSuccess) e = ptd::launch_exhaustive(fn, d_bad, (uint32_t*)((char*)d_bad + 8), nullptr);
  if (e == hipSuccess) e = hipMemcpy(mismatches, d_bad, 8, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(first_bad, (char*)d_bad + 8, 4, hipMemcpyDeviceToHost);
  (void)hipFree(d_bad);
  if (e != hipSuccess) return fail(PT_ERR_HIP, std::string("pt_selftest_exhaustive: ") + hipGetErrorString(e));
  return PT_OK;
}

// ---------------------------------------------------------------- scene ----

int pt_scene_load_obj(const char* path, pt_scene** out) {
  if (!path || !out) return fail(PT_ERR_INVALID, "null argument");
  pt_scene* s = new pt_scene();
  std::string err;
  if (pt::load_obj_file(path, &s->obj, &err) != 0) {
    delete s;
    return fail(PT_ERR_IO, err);
  }
  *out = s;
  return PT_OK;
}

int pt_scene_parse_obj(const char* text, size_t len, pt_scene** out) {
  if (!text || !out) return fail(PT_ERR_INVALID, "null argument");
  pt_scene* s = new pt_scene();
  std::string err;
  if (pt::parse_obj(text, len, &s->obj, &err) != 0) {
    delete s;
    return fail(PT_ERR_IO, err);
  }
  *out = s;
  return PT_OK;
}

int pt_scene_from_arrays(const float* v, size_t nvf, const uint32_t* idx, size_t ni, pt_scene** out) {
  if (!out || (nvf && !v) || (ni && !idx)) return fail(PT_ERR_INVALID, "null argument");
  if (nvf % 3 || ni % 3) return fail(PT_ERR_SCENE, "sizes must be multiples of 3");
  pt_scene* s = new pt_scene();
  s->obj.vertices.assign(v, v + nvf);
  s->obj.indices.assign(idx, idx + ni);
  s->obj.materialIds.assign(ni / 3, 0u);
  *out = s;
  return PT_OK;
}

int pt_scene_build_bvh(pt_scene* s, uint32_t flags, int threads) {
  if (!s) return fail(PT_ERR_INVALID, "null scene");
  const size_t ni = s->obj.indices.size();
  if (ni == 0 || ni % 3) return fail(PT_ERR_SCENE, "scene has no triangles");
  pt::BVHOptions o;
  o.encoding = (flags & PT_NODES_INT_BITS) ? pt::BVHEncoding::kIntBits : pt::BVHEncoding::kFloat;
  o.threads = threads;
  s->bvh_indices.assign(ni, 0);
  s->nodes.assign(2 * (ni / 3) - 1, pt::BVHNode{});
  std::string err;
  if (pt::build_bvh(s->obj.vertices.data(), s->obj.vertices.size(), s->obj.indices.data(), ni,
                    s->bvh_indices.data(), s->nodes.data(), o, &err) != 0) {
    s->bvh_indices.clear();
    s->nodes.clear();
    return fail(PT_ERR_SCENE, err);
  }
  s->flags = flags;
  return PT_OK;
}

int pt_scene_counts(const pt_scene* s, size_t* nvf, size_t* ni, size_t* nn, size_t* nuv, size_t* nmat) {
  if (!s) return fail(PT_ERR_INVALID, "null scene");
  if (nvf) *nvf = s->obj.vertices.size();
  if (ni) *ni = s->obj.indices.size();
  if (nn) *nn = s->nodes.size();
  if (nuv) *nuv = s->obj.texcoords.size();
  if (nmat) *nmat = s->obj.materialIds.size();
  return PT_OK;
}

int pt_scene_copy(const pt_scene* s, float* v, uint32_t* idx, pt_bvh_node* nodes, float* uvs, uint32_t* mat) {
  if (!s) return fail(PT_ERR_INVALID, "null scene");
  if (v) memcpy(v, s->obj.vertices.data(), s->obj.vertices.size() * 4);
  if (idx) {
    const auto& src = s->nodes.empty() ? s->obj.indices : s->bvh_indices;   // BVH order once built
    memcpy(idx, src.data(), src.size() * 4);
  }
  if (nodes) memcpy(nodes, s->nodes.data(), s->nodes.size() * sizeof(pt_bvh_node));
  if (uvs) memcpy(uvs, s->obj.texcoords.data(), s->obj.texcoords.size() * 4);
  if (mat) memcpy(mat, s->obj.materialIds.data(), s->obj.materialIds.size() * 4);
  return PT_OK;
}

int pt_scene_upload(pt_context* c, const pt_scene* s) {
  if (!c || !s) return fail(PT_ERR_INVALID, "null argument");
  if (s->nodes.empty()) return fail(PT_ERR_INVALID, "build the BVH first (pt_scene_build_bvh)");
  return pt_upload_scene(c, s->obj.vertices.data(), s->obj.vertices.size(), s->bvh_indices.data(),
                         s->bvh_indices.size(), (const pt_bvh_node*)s->nodes.data(), s->nodes.size(),
                         s->obj.texcoords.data(), s->obj.texcoords.size(), s->obj.materialIds.data(),
                         s->obj.materialIds.size(), s->flags);
}

// ---- binary scene cache ---------------------------------
// Skips OBJ parsing and the BVH build for large meshes.  Layout: "PTSCENE1",
// u32 version, u32 flags (PT_NODES_INT_BITS), u64 counts of vertex floats,
// OBJ indices, BVH-order indices, nodes, uv floats, material ids, u64 shapes,
// then the six arrays, then a u64 FNV-1a hash of everything before it (taken
// over 8-byte words, the tail bytewise).
namespace {
constexpr char kCacheMagic[8] = {'P', 'T', 'S', 'C', 'E', 'N', 'E', '1'};
constexpr uint32_t kCacheVersion = 1;

struct Fnv {
  uint64_t h = 1469598103934665603ull;
  void add(const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
      uint64_t w;
      memcpy(&w, b + i, 8);
      h = (h ^ w) * 1099511628211ull;
    }
    for (; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
  }
};
}  // namespace

int pt_scene_save(const pt_scene* s, const char* path) {
  if (!s || !path) return fail(PT_ERR_INVALID, "null argument");
  if (s->nodes.empty()) return fail(PT_ERR_INVALID, "build the BVH first (pt_scene_build_bvh)");
  FILE* f = fopen(path, "wb");
  if (!f) return fail(PT_ERR_IO, std::string("cannot create ") + path);
  Fnv h;
  bool ok = true;
  auto put = [&](const void* p, size_t n) {
    if (n && ok) ok = fwrite(p, 1, n, f) == n;
    h.add(p, n);
  };
  const uint64_t counts[7] = {s->obj.vertices.size(), s->obj.indices.size(), s->bvh_indices.size(), s->nodes.size(),
                              s->obj.texcoords.size(), s->obj.materialIds.size(), (uint64_t)s->obj.shapes};
  put(kCacheMagic, 8);
  put(&kCacheVersion, 4);
  put(&s->flags, 4);
  put(counts, sizeof counts);
  put(s->obj.vertices.data(), counts[0] * 4);
  put(s->obj.indices.data(), counts[1] * 4);
  put(s->bvh_indices.data(), counts[2] * 4);
  put(s->nodes.data(), counts[3] * sizeof(pt::BVHNode));
  put(s->obj.texcoords.data(), counts[4] * 4);
  put(s->obj.materialIds.data(), counts[5] * 4);
  const uint64_t digest = h.h;
  if (ok) ok = fwrite(&digest, 1, 8, f) == 8;
  if (fclose(f) != 0) ok = false;
  if (!ok) return fail(PT_ERR_IO, std::string("write failed: ") + path);
  return PT_OK;
}

int pt_scene_load_cache(const char* path, pt_scene** out) {
  if (!path || !out) return fail(PT_ERR_INVALID, "null argument");
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) return fail(PT_ERR_IO, std::string("cannot open ") + path);
  Fnv h;
  bool ok = true;
  auto get = [&](void* p, size_t n) {
    if (n && ok) ok = fread(p, 1, n, f) == n;
    if (ok) h.add(p, n);
  };
  char magic[8];
  uint32_t version = 0, flags = 0;
  uint64_t counts[7] = {0};
  get(magic, 8);
  get(&version, 4);
  get(&flags, 4);
  get(counts, sizeof counts);
  if (!ok || memcmp(magic, kCacheMagic, 8) != 0 || version != kCacheVersion) {
    fclose(f);
    return fail(PT_ERR_IO, std::string("not a scene cache (or another version): ") + path);
  }
  const uint64_t nt = counts[1] / 3;
  if (counts[0] % 3 || counts[1] % 3 || counts[1] == 0 || counts[2] != counts[1] || counts[3] != 2 * nt - 1 ||
      counts[5] > (1ull << 34) || counts[0] > (1ull << 36) || counts[4] > (1ull << 36)) {
    fclose(f);
    return fail(PT_ERR_IO, std::string("inconsistent scene cache header: ") + path);
  }
  pt_scene* s = new pt_scene();
  s->flags = flags;
  s->obj.vertices.resize(counts[0]);
  s->obj.indices.resize(counts[1]);
  s->bvh_indices.resize(counts[2]);
  s->nodes.resize(counts[3]);
  s->obj.texcoords.resize(counts[4]);
  s->obj.materialIds.resize(counts[5]);
  s->obj.shapes = (size_t)counts[6];
  get(s->obj.vertices.data(), counts[0] * 4);
  get(s->obj.indices.data(), counts[1] * 4);
  get(s->bvh_indices.data(), counts[2] * 4);
  get(s->nodes.data(), counts[3] * sizeof(pt::BVHNode));
  get(s->obj.texcoords.data(), counts[4] * 4);
  get(s->obj.materialIds.data(), counts[5] * 4);
  uint64_t digest = 0;
  const uint64_t want = h.h;
  if (ok) ok = fread(&digest, 1, 8, f) == 8;
  fclose(f);
  if (!ok || digest != want) {
    delete s;
    return fail(PT_ERR_IO, std::string("scene cache truncated or corrupt: ") + path);
  }
  *out = s;
  return PT_OK;
}

// ---- image output ----------------------------------------
namespace {
uint32_t crc32_update(uint32_t crc, const unsigned char* p, size_t n) {
  static uint32_t table[256];
  static bool init = false;
  if (!init) {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    init = true;
  }
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return crc;
}

void put_be32(std::vector<unsigned char>* o, uint32_t v) {
  for (int s = 24; s >= 0; s -= 8) o->push_back((unsigned char)(v >> s));
}

void png_chunk(FILE* f, const char* type, const std::vector<unsigned char>& data, bool* ok) {
  std::vector<unsigned char> buf;
  put_be32(&buf, (uint32_t)data.size());
  buf.insert(buf.end(), type, type + 4);
  buf.insert(buf.end(), data.begin(), data.end());
  const uint32_t crc = crc32_update(0xffffffffu, buf.data() + 4, buf.size() - 4) ^ 0xffffffffu;
  put_be32(&buf, crc);
  if (*ok) *ok = fwrite(buf.data(), 1, buf.size(), f) == buf.size();
}

// linear -> 8-bit sRGB after clamping to [0,1]: what an sRGB swapchain shows
// for the reference's RGBA32F image (VulkanRenderer copies it to a texture
// that color_frag.frag outputs unchanged)
unsigned char srgb8(float x) {
  if (!(x > 0.0f)) return 0;
  if (x >= 1.0f) return 255;
  const double e = x <= 0.0031308f ? 12.92 * x : 1.055 * pow((double)x, 1.0 / 2.4) - 0.055;
  return (unsigned char)(e * 255.0 + 0.5);
}
}  // namespace

int pt_write_image(const char* path, const float* rgba, int w, int h, int format) {
  if (!path || !rgba) return fail(PT_ERR_INVALID, "null argument");
  if (w <= 0 || h <= 0) return fail(PT_ERR_INVALID, "bad resolution");
  if (format != PT_IMAGE_PFM && format != PT_IMAGE_PNG) return fail(PT_ERR_INVALID, "unknown image format");
  FILE* f = fopen(path, "wb");
  if (!f) return fail(PT_ERR_IO, std::string("cannot create ") + path);
  bool ok = true;
  if (format == PT_IMAGE_PFM) {
    // rows bottom-to-top: row y = 0 of the accumulation buffer is written first
    ok = fprintf(f, "PF\n%d %d\n-1.0\n", w, h) > 0;
    std::vector<float> rgb((size_t)w * 3);
    for (int y = 0; y < h && ok; ++y) {
      for (int x = 0; x < w; ++x)
        for (int c = 0; c < 3; ++c) rgb[(size_t)x * 3 + c] = rgba[((size_t)y * w + x) * 4 + c];
      ok = fwrite(rgb.data(), 4, rgb.size(), f) == rgb.size();
    }
  } else {
    // 8-bit RGB PNG, zlib stream of stored (uncompressed) deflate blocks;
    // rows top-to-bottom, so the accumulation buffer's last row comes first
    static const unsigned char sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    ok = fwrite(sig, 1, 8, f) == 8;
    std::vector<unsigned char> ihdr;
    put_be32(&ihdr, (uint32_t)w);
    put_be32(&ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});   // 8-bit, truecolour, deflate, filter 0, no interlace
    png_chunk(f, "IHDR", ihdr, &ok);
    std::vector<unsigned char> raw;
    raw.reserve((size_t)h * (1 + 3 * (size_t)w));
    for (int y = h - 1; y >= 0; --y) {
      raw.push_back(0);   // filter: none
      for (int x = 0; x < w; ++x)
        for (int c = 0; c < 3; ++c) raw.push_back(srgb8(rgba[((size_t)y * w + x) * 4 + c]));
    }
    std::vector<unsigned char> z = {0x78, 0x01};
    uint32_t a = 1, b = 0;   // Adler-32
    for (size_t i = 0; i < raw.size(); ++i) {
      a = (a + raw[i]) % 65521u;
      b = (b + a) % 65521u;
    }
    for (size_t off = 0; off < raw.size() || off == 0; off += 65535) {
      const size_t n = std::min<size_t>(65535, raw.size() - off);
      z.push_back(off + n >= raw.size() ? 1 : 0);
      z.push_back((unsigned char)(n & 0xff));
      z.push_back((unsigned char)(n >> 8));
      z.push_back((unsigned char)(~n & 0xff));
      z.push_back((unsigned char)((~n >> 8) & 0xff));
      z.insert(z.end(), raw.begin() + (long)off, raw.begin() + (long)(off + n));
      if (raw.empty()) break;
    }
    put_be32(&z, (b << 16) | a);
    png_chunk(f, "IDAT", z, &ok);
    png_chunk(f, "IEND", {}, &ok);
  }
  if (fclose(f) != 0) ok = false;
  if (!ok) return fail(PT_ERR_IO, std::string("write failed: ") + path);
  return PT_OK;
}

int pt_scene_free(pt_scene* s) {
  delete s;
  return PT_OK;
}

int pt_pack_light(const float pos[3], const float nrm[3], const float inten[3], const float size[2],
                  pt_area_light* out) {
  if (!pos || !nrm || !inten || !size || !out) return fail(PT_ERR_INVALID, "null argument");
  pt::Light l({{pos[0], pos[1], pos[2]}}, {{nrm[0], nrm[1], nrm[2]}}, {{inten[0], inten[1], inten[2]}},
              {{size[0], size[1]}});
  memcpy(out, &l.getLights()[0], sizeof *out);
  return PT_OK;
}

int pt_primary_cull_rects(const float cam[16], int w, int h, const float root_min[3], const float root_max[3],
                          const pt_area_light* lights, int n_lights, float* rects, int max_rects, int* n_rects) {
  if (!cam || !root_min || !root_max || !rects || !n_rects || (n_lights > 0 && !lights))
    return fail(PT_ERR_INVALID, "null argument");
  if (max_rects < 1) return fail(PT_ERR_INVALID, "max_rects must be >= 1");
  *n_rects = cull_rects(cam, w, h, root_min, root_max, lights, n_lights, rects, max_rects);
  return PT_OK;
}

int pt_partition_items(int w, int h, int spl, int nranks, int rank, const int* slots, const float* cull_rects,
                       int n_cull, int item_order, int* live, size_t* n_live, int* culled, size_t* n_culled,
                       int* pixel_of) {
  if (!n_live || !n_culled) return fail(PT_ERR_INVALID, "null argument");
  if (w <= 0 || h <= 0) return fail(PT_ERR_INVALID, "bad resolution");
  if (spl != 1 && spl != 2 && spl != 4 && spl != 8) return fail(PT_ERR_INVALID, "sample lanes must be 1, 2, 4 or 8");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(PT_ERR_INVALID, "bad partition");
  if (n_cull > ptd::kMaxCullRects || (n_cull > 0 && !cull_rects)) return fail(PT_ERR_INVALID, "bad cull rectangles");
  std::vector<int> sl((size_t)nranks, 1);
  if (slots) {
    long long m = 0;
    for (int r = 0; r < nranks; ++r) {
      if (slots[r] < 1 || slots[r] > ptd::kMaxSlots) return fail(PT_ERR_INVALID, "partition slots must be 1..64");
      sl[r] = slots[r];
      m += slots[r];
    }
    if (m > 4096) return fail(PT_ERR_INVALID, "more than 4096 partition slots");
  }
  ptd::RenderParams p{};
  p.width = w;
  p.height = h;
  p.spl = spl;
  p.blocks_x = (w + 15) / 16;
  p.blocks_total = p.blocks_x * ((h + 15) / 16);
  p.n_cull = n_cull < 0 ? -1 : n_cull;
  for (int r = 0; r < n_cull; ++r)
    for (int k = 0; k < 4; ++k) p.cull[r][k] = cull_rects[4 * r + k];
  p.item_order = item_order;
  const ptd::Part pt = part_of_slots(sl, rank);
  std::vector<int> lv, cu;
  item_lists(p, pt, &lv, &cu);
  if ((live && *n_live < lv.size()) || (culled && *n_culled < cu.size()))
    return fail(PT_ERR_INVALID, "item buffers too small");
  if (live) std::copy(lv.begin(), lv.end(), live);
  if (culled) std::copy(cu.begin(), cu.end(), culled);
  if (pixel_of) {   // the kernels' item -> pixel map (tile_pixel), live items first
    const int per = 256 / spl;
    size_t o = 0;
    for (const std::vector<int>* v : {&lv, &cu})
      for (int item : *v) {
        const int tile = ptd::part_tile(pt, item / spl), part = item % spl;
        int bx, by;
        ptd::tile_block(tile, p.blocks_x, &bx, &by);
        for (int q = 0; q < per; ++q, ++o) {
          const int px = bx * 16 + q % 16, py = by * 16 + part * (16 / spl) + q / 16;
          pixel_of[o] = (tile < p.blocks_total && px < w && py < h) ? py * w + px : -1;
        }
      }
  }
  *n_live = lv.size();
  *n_culled = cu.size();
  return PT_OK;
}

int pt_default_camera(float ubo[16]) {
  if (!ubo) return fail(PT_ERR_INVALID, "null argument");
  pt::Camera cam;
  cam.toUBO(ubo);
  return PT_OK;
}

}  // extern "C"

// ===========================================================================
// Native multi-GPU step loop: the tile split's frames with the
// RCCL gather issued from C++, so a run of frames costs no Python per frame.
// bench.py's Python step (render_packed + torch.distributed.gather + stream
// switches) costs ~40-50 us of host time per frame, more than the ~40-us GPU
// step of a 1/8 box.obj share; here one frame is a render_packed launch, two
// event operations and one grouped send/recv.
// ===========================================================================
namespace {
struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommCount)(ncclComm_t, int*) = nullptr;   // optional (the tests' stand-in may lack it)
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};
// RCCL is loaded only when the multi-GPU loop is used: the one already in
// the process (torch's) if there is one, else the system's.  PT_RCCL_LIB
// names another library with the same nine entry points instead, and then
// only that one is tried (the tests' one-GPU stand-in, tests/dist_shim.cpp,
// which moves the point-to-point bytes between processes sharing a device).
const RcclApi* rccl_api() {
  static RcclApi api;
  static bool tried = false;
  if (!tried) {
    tried = true;
    const char* alt = getenv("PT_RCCL_LIB");
    void* h = nullptr;
    if (alt && *alt) {
      h = dlopen(alt, RTLD_NOW | RTLD_LOCAL);
    } else {
      h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
      if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
      if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    }
    if (h) {
      api.GetUniqueId = (decltype(api.GetUniqueId))dlsym(h, "ncclGetUniqueId");
      api.CommInitRank = (decltype(api.CommInitRank))dlsym(h, "ncclCommInitRank");
      api.CommCount = (decltype(api.CommCount))dlsym(h, "ncclCommCount");
      api.CommDestroy = (decltype(api.CommDestroy))dlsym(h, "ncclCommDestroy");
      api.CommAbort = (decltype(api.CommAbort))dlsym(h, "ncclCommAbort");
      api.GroupStart = (decltype(api.GroupStart))dlsym(h, "ncclGroupStart");
      api.GroupEnd = (decltype(api.GroupEnd))dlsym(h, "ncclGroupEnd");
      api.Send = (decltype(api.Send))dlsym(h, "ncclSend");
      api.Recv = (decltype(api.Recv))dlsym(h, "ncclRecv");
      api.GetErrorString = (decltype(api.GetErrorString))dlsym(h, "ncclGetErrorString");
      if (api.GetUniqueId && api.CommInitRank && api.CommDestroy && api.CommAbort && api.GroupStart && api.GroupEnd && api.Send &&
          api.Recv && api.GetErrorString)
        api.h = h;
    }
  }
  return api.h ? &api : nullptr;
}
#define PT_NCCL(call)                                                                                   \
  do {                                                                                                  \
    ncclResult_t r_ = (call);                                                                           \
    if (r_ != ncclSuccess) return fail(PT_ERR_HIP, std::string(#call ": ") + R->GetErrorString(r_));    \
  } while (0)

// Slot size and buffers for the layout of the last rendered frame (c->last).
int dist_layout(pt_context* c) {
  DistState* d = c->dist;
  std::vector<float> key;
  frame_key(c, c->last, &key);
  // (the root has no send slots: its layout is valid once any buffer was
  // sized for it; testing send[0] made the root rebuild every rank's item
  // lists on every call, ~0.45 ms of host time per call at N = 8)
  if (key == d->layout_key && d->cap_floats > 0) return PT_OK;
  size_t live_max = 0;
  std::vector<int> live, culled;
  for (int r = 0; r < c->nranks; ++r) {
    item_lists(c->last, part_of(c, r), &live, &culled);
    live_max = std::max(live_max, live.size());
  }
  const size_t slot = std::max<size_t>(4, live_max * (size_t)(256 / c->last.spl) * 4);
  const size_t nslots = (size_t)c->nranks;   // the partition's ranks (emulation: > d->nranks)
  if (slot > d->cap_floats) {
    for (int b = 0; b < kDistStreams; ++b)
      for (hipStream_t s : {d->streams[b], d->comm_stream}) PT_HIP(hipStreamSynchronize(s));
    for (int b = 0; b < kDistStreams; ++b) dev_free(d->send[b]);
    for (int b = 0; b < kDistSets; ++b) dev_free(d->recv[b]);
    dev_free(d->ingest);
    d->cap_floats = 0;
    for (int b = 0; b < kDistStreams && d->rank != 0; ++b) {
      PT_HIP(hipMalloc((void**)&d->send[b], slot * sizeof(float)));
      PT_HIP(hipMemset(d->send[b], 0, slot * sizeof(float)));
    }
    for (int b = 0; b < kDistSets && d->rank == 0; ++b) {
      PT_HIP(hipMalloc((void**)&d->recv[b], nslots * slot * sizeof(float)));
      PT_HIP(hipMemset(d->recv[b], 0, nslots * slot * sizeof(float)));
    }
    if (d->nranks == 1 && nslots > 1) {
      PT_HIP(hipMalloc((void**)&d->ingest, (nslots - 1) * slot * sizeof(float)));
      PT_HIP(hipMemset(d->ingest, 0, (nslots - 1) * slot * sizeof(float)));
    }
    d->cap_floats = slot;
  }
  d->slot_floats = slot;
  d->layout_key = key;
  return PT_OK;
}
}  // namespace

extern "C" {

int pt_dist_unique_id(void* id, size_t id_bytes) {
  if (!id || id_bytes < sizeof(ncclUniqueId)) return fail(PT_ERR_INVALID, "id buffer must hold 128 bytes");
  const RcclApi* R = rccl_api();
  if (!R) return fail(PT_ERR_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
  ncclUniqueId u;
  PT_NCCL(R->GetUniqueId(&u));
  memcpy(id, &u, sizeof u);
  return PT_OK;
}

int pt_dist_init(pt_context* c, const void* id, int nranks, int rank) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_init: not on a multi-device context (pt_create_multi)");
  if (!c || !id) return fail(PT_ERR_INVALID, "null argument");
  const bool emulated = nranks == 1 && rank == 0 && c->rank == 0 && c->nranks > 1;
  if (!emulated && (nranks != c->nranks || rank != c->rank))
    return fail(PT_ERR_INVALID, "pt_dist_init: set the same partition first (pt_set_partition / _slots)");
  const RcclApi* R = rccl_api();
  if (!R) return fail(PT_ERR_UNSUPPORTED, "RCCL (librccl.so.1) could not be loaded");
  if (c->dist) pt_dist_finalize(c);
  PT_HIP(hipSetDevice(c->device));
  DistState* d = new DistState();
  c->dist = d;
  d->nranks = nranks;
  d->rank = rank;
  int lo = 0, hi = 0;
  PT_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
  PT_HIP(hipStreamCreateWithPriority(&d->own[kDistStreams], hipStreamNonBlocking, hi));   // gathers take CUs first
  // the two render streams at the least priority: the HIP runtime gives each
  // priority its own pool of GPU_MAX_HW_QUEUES hardware queues, so these two
  // get a queue each instead of sharing one with the process's other streams
  // (two frames on one queue do not overlap)
  for (int b = 0; b < kDistStreams; ++b) {
    PT_HIP(hipStreamCreateWithPriority(&d->own[b], hipStreamNonBlocking, lo));
    d->streams[b] = d->own[b];
  }
  d->comm_stream = d->own[kDistStreams];
  for (int b = 0; b < kDistSets; ++b) {
    PT_HIP(hipEventCreateWithFlags(&d->render_done[b], hipEventDisableTiming));
    PT_HIP(hipEventCreateWithFlags(&d->gather_done[b], hipEventDisableTiming));
  }
  for (hipEvent_t& e : d->entry) PT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  PT_NCCL(R->CommInitRank(&d->comm, nranks, u, rank));
  if (R->CommCount) {
    int cnt = -1;
    if (R->CommCount(d->comm, &cnt) == ncclSuccess) d->comm_count = cnt;
  }
  d->ready = true;
  return PT_OK;
}

int pt_dist_info(pt_context* c, int* comm_ranks, int* nranks, int* rank) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_info: not on a multi-device context (pt_create_multi)");
  if (!c || !c->dist) return fail(PT_ERR_INVALID, "pt_dist_info: no communicator (pt_dist_init)");
  if (comm_ranks) *comm_ranks = c->dist->comm_count;
  if (nranks) *nranks = c->dist->nranks;
  if (rank) *rank = c->dist->rank;
  return PT_OK;
}

// Whether frame buffer `frame` already holds a whole assembled frame of the
// layout `key` (its culled items' constant included).
static bool dist_assembled(const DistState* d, const void* frame, const std::vector<float>& key) {
  for (const auto& e : d->assembled)
    if (e.first == frame) return e.second == key;
  return false;
}
static void dist_mark_assembled(DistState* d, const void* frame, const std::vector<float>& key) {
  for (auto& e : d->assembled)
    if (e.first == frame) {
      e.second = key;
      return;
    }
  d->assembled.push_back({frame, key});
}

int pt_dist_run(pt_context* c, uint32_t n_batches, int n_frames, int n_streams, void* frames, int n_frame_bufs) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_run: not on a multi-device context (pt_create_multi)");
  if (!c) return fail(PT_ERR_INVALID, "null context");
  DistState* d = c->dist;
  if (!d || !d->ready) return fail(PT_ERR_INVALID, "pt_dist_run: no communicator (pt_dist_init)");
  if (n_frames < 0 || n_batches == 0) return fail(PT_ERR_INVALID, "pt_dist_run: bad frame or batch count");
  if (d->rank == 0 && (!frames || n_frame_bufs < 1 || (((uintptr_t)frames) & 15)))
    return fail(PT_ERR_INVALID, "pt_dist_run: the root needs 16-B aligned frame buffers");
  if (n_streams < 1 || n_streams > kDistStreams) return fail(PT_ERR_INVALID, "pt_dist_run: 1 to 3 streams");
  if (d->caller_streams && n_streams > 2)
    return fail(PT_ERR_INVALID, "pt_dist_run: 3 streams with caller render streams (pt_dist_set_streams sets two)");
  const bool emulated = d->nranks == 1 && c->nranks > 1;
  if ((d->nranks != c->nranks && !emulated) || d->rank != c->rank)
    return fail(PT_ERR_INVALID, "partition changed since pt_dist_init");
  if (!c->last_valid) return fail(PT_ERR_INVALID, "pt_dist_run: render one frame with pt_render first (item layout)");
  const RcclApi* R = rccl_api();
  PT_HIP(hipSetDevice(c->device));
  {
    const int rc = dist_layout(c);
    if (rc) return rc;
  }
  const size_t slot = d->slot_floats;
  const size_t frame_f = (size_t)c->width * c->height * 4;
  hipStream_t saved = c->stream;
  int rc = PT_OK;
  // D = max(2, streams) frames in flight.  Frame k runs on stream k % S
  // with buffer set k % 2D.  Its launch (pt_render_packed) writes this rank's
  // live items -- on the root straight into its own slot of receive set
  // k % 2D, elsewhere into send slot k % D -- and, on the root, assembles
  // frame k-D from receive set (k-D) % 2D, after waiting for that frame's
  // gather.  Hazards: the gather of frame k (comm stream, after frame k's
  // launch) overwrites set k % 2D, which frame k-D's launch read -- earlier
  // on frame k's own stream (S divides D: S = 1 or D); a send slot is read by
  // the gather of frame k-D, which frame k's launch waits for.
  const int D = std::max(2, n_streams), nsets = 2 * D;
  // Those hazards hold within a call.  Across calls, frame k < D of this call
  // has no gather_done to wait for: a previous call's last sends (comm stream)
  // may still read send slot k % D, and its trailing assemblies (other render
  // streams) may still write the frame buffers.  So every render stream
  // starts behind every stream's last work of the previous call.
  {
    hipStream_t all[kDistStreams + 1];
    for (int s = 0; s < kDistStreams; ++s) all[s] = d->streams[s];
    all[kDistStreams] = d->comm_stream;
    for (int s = 0; s <= kDistStreams; ++s) PT_HIP(hipEventRecord(d->entry[s], all[s]));
    for (int s = 0; s < n_streams; ++s)
      for (int e = 0; e <= kDistStreams; ++e)
        if (all[e] != d->streams[s]) PT_HIP(hipStreamWaitEvent(d->streams[s], d->entry[e], 0));
  }
  c->in_dist = true;
  const bool self_p2p = emulated && getenv("PT_DIST_EMU_P2P") && atoi(getenv("PT_DIST_EMU_P2P")) == 1;
  // frames after the first of each kind (with and without an assembly) reuse
  // its launch parameters: nothing but the output and the assembled frame
  // change within a call (relaunch)
  Launched tmpl[2];
  for (int k = 0; k < n_frames && rc == PT_OK; ++k) {
    const int b = k % nsets;
    c->stream = d->streams[k % n_streams];
    Assembly as;
    if (k >= D) {
      const int pb = (k - D) % nsets;
      PT_HIP(hipStreamWaitEvent(c->stream, d->gather_done[pb], 0));
      if (d->rank == 0) {
        as.src = d->recv[pb];
        as.slot_floats = slot;
        as.frame = (float*)frames + (size_t)((k - D) % n_frame_bufs) * frame_f;
      }
    }
    float4* out = (float4*)(d->rank == 0 ? d->recv[b] : d->send[k % D]);
    Launched& t = tmpl[as.src ? 1 : 0];
    if (t.valid) {
      ptd::RenderParams p = t.p;
      p.pack_out = out;
      p.unpack_src = (const float4*)as.src;
      p.unpack_frame = (float4*)as.frame;
      if (as.src && dist_assembled(d, as.frame, c->unpack_key)) {   // live items only
        p.unpack_table = c->d_unpack_live;
        p.n_unpack = c->n_unpack_live;
      } else if (as.src) {
        p.unpack_table = c->d_unpack;
        p.n_unpack = c->n_unpack;
        dist_mark_assembled(d, as.frame, c->unpack_key);
      }
      rc = relaunch(c, p, t.lds, t.cnt);
    } else {
      rc = render_impl(c, 0, n_batches, out, as, &t);   // a whole assembly (the full table)
      if (rc == PT_OK && as.src) dist_mark_assembled(d, as.frame, c->unpack_key);
    }
    if (rc) break;
    PT_HIP(hipEventRecord(d->render_done[b], c->stream));
    PT_HIP(hipStreamWaitEvent(d->comm_stream, d->render_done[b], 0));
    if (emulated && self_p2p) {
      // measurement (PT_DIST_EMU_P2P=1): the other ranks' slots through
      // RCCL itself -- one grouped self send/recv per emulated rank, the
      // calls the root's real gather makes -- so the emulated step carries
      // RCCL's host and device cost per frame
      PT_NCCL(R->GroupStart());
      for (int r = 1; r < c->nranks; ++r) {
        PT_NCCL(R->Send(d->ingest + (size_t)(r - 1) * slot, slot, ncclFloat32, 0, d->comm, d->comm_stream));
        PT_NCCL(R->Recv(d->recv[b] + (size_t)r * slot, slot, ncclFloat32, 0, d->comm, d->comm_stream));
      }
      PT_NCCL(R->GroupEnd());
    } else if (emulated) {   // the other ranks' slots: the bytes a real gather would write here
      PT_HIP(hipMemcpyAsync(d->recv[b] + slot, d->ingest, (size_t)(c->nranks - 1) * slot * sizeof(float),
                            hipMemcpyDeviceToDevice, d->comm_stream));
    }
    if (d->nranks > 1) {
      PT_NCCL(R->GroupStart());
      if (d->rank == 0)
        for (int r = 1; r < d->nranks; ++r)
          PT_NCCL(R->Recv(d->recv[b] + (size_t)r * slot, slot, ncclFloat32, r, d->comm, d->comm_stream));
      else
        PT_NCCL(R->Send(d->send[k % D], slot, ncclFloat32, 0, d->comm, d->comm_stream));
      PT_NCCL(R->GroupEnd());
    }
    PT_HIP(hipEventRecord(d->gather_done[b], d->comm_stream));
  }
  c->in_dist = false;
  // the root assembles the last (up to) D frames in launches of their own
  if (rc == PT_OK && d->rank == 0) {
    frame_key(c, c->last, &c->key_scratch);
    rc = unpack_table(c, c->last, c->key_scratch);
    for (int k = std::max(0, n_frames - D); k < n_frames && rc == PT_OK; ++k) {
      const int b = k % nsets;
      c->stream = d->streams[k % n_streams];
      PT_HIP(hipStreamWaitEvent(c->stream, d->gather_done[b], 0));
      float4* out = (float4*)((float*)frames + (size_t)(k % n_frame_bufs) * frame_f);
      const bool live_only = dist_assembled(d, out, c->unpack_key);
      PT_HIP(ptd::launch_items_unpack(c->last, out, (const float4*)d->recv[b], slot / 4,
                                      live_only ? c->d_unpack_live : c->d_unpack,
                                      live_only ? c->n_unpack_live : c->n_unpack, c->stream));
      if (!live_only) dist_mark_assembled(d, out, c->unpack_key);
    }
  }
  // one use event per stream for the whole run (the launches above skip theirs)
  for (int sidx = 0; sidx < n_streams && rc == PT_OK; ++sidx) {
    c->stream = d->streams[sidx];
    rc = note_use(c);
  }
  c->stream = saved;
  return rc;
}

int pt_dist_set_streams(pt_context* c, void* render0, void* render1, void* comm) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_set_streams: not on a multi-device context (pt_create_multi)");
  if (!c || !c->dist) return fail(PT_ERR_INVALID, "pt_dist_set_streams: no communicator (pt_dist_init)");
  DistState* d = c->dist;
  PT_HIP(hipSetDevice(c->device));
  for (hipStream_t s : {d->streams[0], d->streams[1], d->streams[2], d->comm_stream}) PT_HIP(hipStreamSynchronize(s));
  d->streams[0] = render0 ? (hipStream_t)render0 : d->own[0];
  d->streams[1] = render1 ? (hipStream_t)render1 : d->own[1];
  d->caller_streams = render0 || render1;
  d->comm_stream = comm ? (hipStream_t)comm : d->own[kDistStreams];
  return PT_OK;
}

int pt_dist_slot_floats(pt_context* c, size_t* slot_floats) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_slot_floats: not on a multi-device context (pt_create_multi)");
  if (!c || !slot_floats) return fail(PT_ERR_INVALID, "null argument");
  if (!c->dist || !c->dist->slot_floats) return fail(PT_ERR_INVALID, "no pt_dist_run yet");
  *slot_floats = c->dist->slot_floats;
  return PT_OK;
}

int pt_dist_wait(pt_context* c, int timeout_ms) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_wait: not on a multi-device context (pt_create_multi)");
  if (!c || !c->dist) return fail(PT_ERR_INVALID, "pt_dist_wait: no communicator");
  DistState* d = c->dist;
  PT_HIP(hipSetDevice(c->device));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    bool done = true;
    for (hipStream_t s : {d->streams[0], d->streams[1], d->streams[2], d->comm_stream}) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipErrorNotReady) done = false;
      else if (q != hipSuccess) return fail(PT_ERR_HIP, std::string("pt_dist_wait: ") + hipGetErrorString(q));
    }
    if (done) return PT_OK;
    const long long ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_ms >= 0 && ms > timeout_ms) return fail(PT_ERR_HIP, "pt_dist_wait: timed out (gather not complete)");
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

int pt_dist_abort(pt_context* c) {
  if (c && c->group) return fail(PT_ERR_UNSUPPORTED, "pt_dist_abort: not on a multi-device context (pt_create_multi)");
  if (!c || !c->dist) return PT_OK;
  const RcclApi* R = rccl_api();
  if (c->dist->comm && R) (void)R->CommAbort(c->dist->comm);   // ends outstanding transfers
  c->dist->comm = nullptr;
  return pt_dist_finalize(c);
}

int pt_dist_finalize(pt_context* c) {
  if (!c) return fail(PT_ERR_INVALID, "null context");
  DistState* d = c->dist;
  if (!d) return PT_OK;
  (void)hipSetDevice(c->device);
  for (hipStream_t s : {d->streams[0], d->streams[1], d->streams[2], d->comm_stream})
    if (s) (void)hipStreamSynchronize(s);
  const RcclApi* R = rccl_api();
  if (d->comm && R) (void)R->CommDestroy(d->comm);
  dev_free(d->ingest);
  for (int b = 0; b < kDistStreams; ++b) dev_free(d->send[b]);
  for (hipStream_t s : d->own)
    if (s) (void)hipStreamDestroy(s);
  for (int b = 0; b < kDistSets; ++b) {
    dev_free(d->recv[b]);
    if (d->render_done[b]) (void)hipEventDestroy(d->render_done[b]);
    if (d->gather_done[b]) (void)hipEventDestroy(d->gather_done[b]);
  }
  for (hipEvent_t e : d->entry)
    if (e) (void)hipEventDestroy(e);
  delete d;
  c->dist = nullptr;
  return PT_OK;
}

}  // extern "C"
