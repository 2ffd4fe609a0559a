/*
 * pathtracer.h — C ABI of the MI355X-native path-tracing pixel kernel.
 *
 * This is the drop-in boundary.  The reference has no plugin/operator API:
 * its seam is the Vulkan compute interface that VulkanRayTracer builds and
 * drives (src/Vulkan/VulkanRayTracer.cpp) for the shader
 * src/shaders/raytrace_comp.comp.  Every entry point below replaces one piece
 * of that seam; the comment on each cites what it replaces.  A maintainer
 * swaps the Vulkan descriptor/dispatch code for these calls.
 *
 * Conventions (inherited from the reference):
 *   - every call returns int status: PT_OK (0) or a negative PT_ERR_*;
 *     pt_last_error() describes the last failure on the calling thread.
 *     Nothing throws across the ABI.
 *   - the caller keeps ownership of every host array; uploads copy.
 *   - the accumulation buffer is device-resident (RGBA32F, row-major,
 *     pixel (x,y) at index y*W+x) until read back.
 *   - one context per GPU, driven from one thread.  Calls are ordered on the
 *     context's HIP stream; pt_dispatch/pt_render return once the work is
 *     enqueued, pt_read_accum/pt_synchronize wait for it (the reference blocks
 *     on a fence after every dispatch, VulkanCommandBuffer.cpp:140).
 */
#ifndef PATHTRACER_H_
#define PATHTRACER_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history.  2 (round 5): pt_group_check, pt_dist_info and
 * PT_OPT_GROUP_CHECK added; option values removed since 1 now return
 * PT_ERR_UNSUPPORTED: PT_OPT_KERNEL 2, PT_OPT_SM_BATCH, PT_OPT_PAIRS 1,
 * PT_OPT_WIDE_NODE 80 (kernels measured slower on every scene).
 * 3 (round 6): pt_mixed_info and PT_OPT_MIXED_LANES added; defaults changed:
 * PT_OPT_LAUNCH_TIMING 0 (was 1), PT_OPT_ITEM_ORDER -1 auto (was 1);
 * pt_group_check state 2 (probe failed). */
#define PT_ABI_VERSION 3

enum {
  PT_OK = 0,
  PT_ERR_INVALID = -1,     /* bad argument / state */
  PT_ERR_HIP = -2,         /* HIP runtime failure */
  PT_ERR_SCENE = -3,       /* malformed scene / BVH */
  PT_ERR_IO = -4,          /* file not found / parse error */
  PT_ERR_UNSUPPORTED = -5  /* valid input this build does not handle */
};

/* BVHNode — src/BoundingVolumeHierarchy.h:8-13, std430 stride 32 B.
 * min_bounds.w = left child or -1 (leaf); max_bounds.w = right child or the
 * leaf's triangle index.  Indices are floats (reference) unless
 * PT_NODES_INT_BITS is passed, in which case they are int32 bit patterns. */
typedef struct pt_bvh_node {
  float min_bounds[4];
  float max_bounds[4];
} pt_bvh_node;

/* AreaLightData — src/Light.h:6-12, 64 B. */
typedef struct pt_area_light {
  float position[4];
  float normal[4];
  float intensity[4];
  float size[4];
} pt_area_light;

/* Tunables the reference hard-codes (raytrace_comp.comp:304,373). */
typedef struct pt_params {
  int max_depth;    /* MAX_DEPTH, reference 4 */
  int sss_bounces;  /* SSS_MAX_BOUNCES, reference 3 */
} pt_params;

/* Statistics of the reference traversal (exhaustive DFS, raytrace_comp.comp:159-204),
 * accumulated while stats mode is on: traceRay calls, BVH nodes visited,
 * leaf triangle tests, pixel-samples. */
typedef struct pt_stats {
  uint64_t rays;
  uint64_t nodes;
  uint64_t leaf_tests;
  uint64_t samples;
} pt_stats;

/* Work the fast kernels actually did while PT_OPT_COUNT_TRACED is on (they
 * skip work the reference does without changing a bit of the output: culled
 * primary rays, shadow rays whose answer cannot change the image, the
 * repeated light pre-pass ray, implied-hit nodes, leaf tests after an
 * occluder): closest-hit and shadow walks started, BVH nodes visited,
 * triangle tests, primary rays generated.  Reset by pt_reset_stats. */
typedef struct pt_traced {
  uint64_t closest_walks;
  uint64_t shadow_walks;
  uint64_t nodes;
  uint64_t tri_tests;
  uint64_t primaries;
} pt_traced;

typedef struct pt_context pt_context;

/* upload flags */
#define PT_NODES_INT_BITS 0x1u

/* ---- lifetime ---------------------------------------------------------- */
int pt_abi_version(void);
const char* pt_last_error(void);
/* Replaces VulkanWindow's device/queue selection (VulkanWindow.cpp:106-174)
 * and VulkanRayTracer::initComputePipeline's pipeline creation (:624-672). */
int pt_create(int device_ordinal, pt_context** out);
/* One context over n devices of this process (SURVEY.md §8b create(device
 * ordinals[], n)): the reference's single host thread (VulkanRenderer.cpp:
 * 643-647, mainLoop VulkanRayTracer.cpp:717-865) drives all of them through
 * the calls below exactly as it drives one.  Member r renders the 16x16
 * screen tiles of rank r of an n-way pt_set_partition; the frame lives in
 * device memory of device_ordinals[0] (pt_accum_device_ptr), where pt_read_accum,
 * pt_readback_* and pt_synchronize see every member's tiles, bit-identical to
 * a single-GPU render.  Members store their tiles into that frame directly
 * over xGMI (peer access), or -- when a member cannot map it, or with
 * PT_OPT_GROUP_EXCHANGE 1 -- ship them as packed tiles copied to the first
 * device.  Before peer stores carry a frame on members of distinct devices,
 * a probe frame checks them bit for bit against the packed copies and falls
 * back to the copies on any difference (PT_OPT_GROUP_CHECK, pt_group_check).
 * UNVERIFIED on hardware: members on distinct devices have not run in this
 * build's tests (one-GPU boxes); every group test so far put its members on
 * one device, where the bit identity is tested.  An ordinal may repeat (several members on one device: tests).
 * With three or more members, members 1..n-1 enqueue their launches from
 * threads of their own (environment PT_GROUP_THREADS=0: all on the calling
 * thread), so a render costs the caller about one member's host time.
 * Calls on a member's share (pt_set_partition*, pt_tiles_*, pt_items_*,
 * pt_render_packed, pt_dist_*) return PT_ERR_UNSUPPORTED on such a context;
 * the launch-timing calls report the first device's launches.  pt_destroy
 * frees it. */
int pt_create_multi(const int* device_ordinals, int n, pt_context** out);
/* Devices of a context (1 and its ordinal for a pt_create context) and
 * whether its members store their tiles straight into the frame (1) or ship
 * packed tiles (0). */
int pt_group_info(pt_context* ctx, int* n_devices, int* devices, int max_devices, int* peer_stores);
/* The peer-store check of a multi-device context (PT_OPT_GROUP_CHECK):
 * *state -2 armed (runs on the next render), -1 not run (members on one
 * device, staged exchange in force, or a pt_create context), 0 the probe
 * frames matched bit for bit (peer stores in force), 1 they differed (the
 * staged exchange is in force from then on), 2 the peer-store probe failed
 * (a HIP error; staged exchange from then on, the render goes on); the probe
 * frames' wall times.  The probe is read back the way a frame is consumed:
 * on the first device's stream, behind its wait for every member's
 * completion event, with no host synchronisation of the members before it.
 * The check is meant to catch a cross-device visibility failure of peer
 * stores at run time; it has not yet run on members of distinct devices
 * (every test so far ran its members on one device), so whether it does is
 * unverified. */
int pt_group_check(pt_context* ctx, int* state, float* ms_peer, float* ms_staged);
int pt_destroy(pt_context* ctx);
/* Launch on a caller-owned hipStream_t (e.g. a torch.cuda.Stream's handle);
 * NULL returns to the context's own stream — so the legacy default stream
 * (handle 0) cannot be selected: share a created stream instead. */
int pt_set_stream(pt_context* ctx, void* hip_stream);
int pt_synchronize(pt_context* ctx);

/* ---- scene upload (VulkanRayTracer.cpp:100-311, bindings 1,2,3,6,7) ---- */
/* vertices: float[3V] (binding 1); indices: uint[3T] in BVH-leaf order
 * (binding 2); nodes: BVHNode[2T-1] (binding 3); uvs (binding 6) and
 * mat_indices (binding 7) are accepted for interface parity and validated but
 * do not affect the output (raytrace_comp.comp:150-154,192 are dead). */
int pt_upload_scene(pt_context* ctx,
                    const float* vertices, size_t n_vertex_floats,
                    const uint32_t* indices, size_t n_indices,
                    const pt_bvh_node* nodes, size_t n_nodes,
                    const float* uvs, size_t n_uv_floats,
                    const uint32_t* mat_indices, size_t n_mat,
                    uint32_t flags);
/* binding 5 (VulkanRayTracer.cpp:165-176) */
int pt_upload_lights(pt_context* ctx, const pt_area_light* lights, size_t n_lights);
/* binding 4: std140 CameraBuffer — pos@0, dir@16, up@32, fov.x@48
 * (raytrace_comp.comp:67-73; written at VulkanRayTracer.cpp:761-764). */
int pt_set_camera(pt_context* ctx, const float camera_ubo[16]);
int pt_set_params(pt_context* ctx, const pt_params* params);

/* ---- accumulation image (binding 0, VulkanRayTracer.cpp:317-320) ------- */
/* Allocate (or reuse) a W x H RGBA32F buffer and zero it.  The reference
 * never clears its image (VulkanImage.cpp:71); batch 0 multiplies prev by 0. */
int pt_resize_and_clear(pt_context* ctx, int width, int height);
/* Render into caller-owned device memory of W*H*16 bytes instead (not
 * cleared; call pt_clear_accum). */
int pt_bind_accum(pt_context* ctx, void* device_ptr, int width, int height);
int pt_clear_accum(pt_context* ctx);
void* pt_accum_device_ptr(pt_context* ctx);
int pt_read_accum(pt_context* ctx, float* rgba, size_t n_floats);

/* ---- the hot path ------------------------------------------------------ */
/* One 1-spp accumulation pass with push constant sample_batch
 * (VulkanRayTracer.cpp:803-813 vkCmdPushConstants + vkCmdDispatch). */
int pt_dispatch(pt_context* ctx, uint32_t sample_batch);
/* n_batches sequential passes first_batch..first_batch+n-1 fused into one
 * launch; bit-identical to that many pt_dispatch calls. */
int pt_render(pt_context* ctx, uint32_t first_batch, uint32_t n_batches);

/* ---- progressive loop (VulkanRayTracer::mainLoop, :717-865) ------------ */
/* Sets the camera; if any of its 16 floats differs from the last one given
 * here, the sample counter restarts at 0 (:739-754 — batch 0 weights the old
 * image by 0, so no clear is needed).  *reset (optional) reports it. */
int pt_progressive_camera(pt_context* ctx, const float camera_ubo[16], int* reset);
/* Enqueues min(max_new, limit - counter) further batches as one fused launch
 * (the reference renders up to limit = 1024, :719) and advances the counter;
 * *first and *count (optional) report what was enqueued.  Bit-identical to
 * that many pt_dispatch calls. */
int pt_progressive_advance(pt_context* ctx, uint32_t max_new, uint32_t limit, uint32_t* first, uint32_t* count);
/* Asynchronous double-buffered readback (replaces the per-batch fence waits
 * and copyStorageImage, :826-846): begin snapshots the image as of the work
 * enqueued so far and copies it to pinned host memory on a second stream;
 * end waits for that copy and writes W*H*4 floats.  Two readbacks may be in
 * flight; a third begin recycles the oldest unclaimed one. */
int pt_readback_begin(pt_context* ctx, int* ticket);
int pt_readback_end(pt_context* ctx, int ticket, float* rgba, size_t n_floats);

/* ---- multi-GPU screen-space partition ------------------ */
/* Pixels are grouped into 16x16 blocks.  Block (bx, by) is tile
 * b = by*blocks_x + (bx - by) mod blocks_x (rows rotated by their index, so
 * ranks get anti-diagonal stripes, not column stripes); this context renders
 * tile b iff b % nranks == rank.  pt_clear_accum then writes +0 to
 * owned pixels and -0 (the IEEE additive identity) to the others, so a sum
 * reduction of all ranks' buffers is bit-identical to a single-GPU frame. */
int pt_set_partition(pt_context* ctx, int nranks, int rank);
/* Unequal shares: tiles are dealt in periods of sum(slots) slots, rank r
 * owning slots[r] consecutive ones (1..64 each, at most 4096 in all).
 * pt_set_partition is the case of one slot per rank.  Every rank must pass
 * the same slots.  bench.py gives the root, which also assembles the
 * gathered frame, fewer slots. */
int pt_set_partition_slots(pt_context* ctx, int nranks, int rank, const int* slots);
/* Gather-based assembly (cheaper than a full-frame sum for N > 2): a rank
 * packs the tiles it owns into a dense device buffer of
 * n_tiles * 16*16 float4 (pt_tiles_owned), ships it to the root, and the
 * root unpacks each rank's buffer into a W x H frame.  The frame size and
 * partition are the context's; all work is enqueued on its stream. */
int pt_tiles_owned(pt_context* ctx, int* n_tiles);
int pt_tiles_pack(pt_context* ctx, void* dst_device);
int pt_tiles_unpack(pt_context* ctx, const void* src_device, int src_rank, void* frame_device);
/* Sparse exchange of the last rendered frame: only the tile parts ("items",
 * 256/SPL pixels each) that can hold a live pixel under primary culling.
 * Every rank must have rendered the same frame (camera, size, partition
 * size, batches).  pt_items_live: rank's live item count and pixels per item
 * (a slot must hold n_items*item_pixels float4).  pt_items_pack: this rank's
 * live items, densely.  pt_items_unpack_all: rank r's slot at
 * src + r*slot_floats; live items are scattered into the frame, culled ones
 * written as (0,0,0,1) — their value for a frame rendered from batch 0, which
 * this call requires.  With culling off every item is live. */
int pt_items_live(pt_context* ctx, int rank, int* n_items, int* item_pixels);
int pt_items_pack(pt_context* ctx, void* dst_device);
int pt_items_unpack_all(pt_context* ctx, const void* src_device, size_t slot_floats, void* frame_device);
/* pt_render_packed: render a fresh frame (batches 0..n_batches-1, as
 * pt_clear_accum + pt_render) and write this rank's live items straight into
 * dst_device in the pt_items_pack layout — what pt_render + pt_items_pack
 * give, in one launch, without the culled-item fill.  The accumulation buffer
 * is neither read nor written.  gathered_device (optional, else null): the
 * per-rank slots of the PREVIOUS frame, which the same launch assembles into
 * frame_device exactly as pt_items_unpack_all would — the root's step of a
 * pipelined tile split is then one launch; that frame must have been
 * rendered by pt_render_packed with the same item layout — frame size,
 * partition, sample lanes, culling rectangles, item order (error otherwise).
 * Replaces, for the tile split, the reference's one dispatch per frame plus
 * image readback (VulkanRayTracer.cpp:803-865). */
int pt_render_packed(pt_context* ctx, uint32_t n_batches, void* dst_device, const void* gathered_device,
                     size_t slot_floats, void* frame_device);
/* The item tables behind pt_items_live / pt_items_pack / pt_items_unpack_all
 * and pt_render_packed, as a pure host function (no context, no GPU): rank's
 * live items (tile parts that can hold a live pixel) in launch order, its
 * culled items, and -- when pixel_of is not null -- for every listed item
 * (live first, then culled) and each of its 256/sample_lanes slots q the
 * pixel index y*W+x it carries, or -1 past the frame edge.  slots: null for
 * one slot per rank, else as pt_set_partition_slots.  cull_rects / n_cull: as
 * pt_primary_cull_rects returns them (n_cull < 0: no culling, every item is
 * live).  item_order: PT_OPT_ITEM_ORDER.  Call with null live/culled to get
 * the counts; *n_live / *n_culled give the buffer sizes on input. */
int pt_partition_items(int width, int height, int sample_lanes, int nranks, int rank, const int* slots,
                       const float* cull_rects, int n_cull, int item_order, int* live, size_t* n_live,
                       int* culled, size_t* n_culled, int* pixel_of);

/* ---- native multi-GPU step loop (RCCL) ------------------ */
/* The tile split's pipelined sparse gather with the collective issued from
 * C++: frames alternate between two internal streams; frame k's launch
 * renders this rank's live items into a send slot and, on the root, assembles
 * frame k-2 (pt_render_packed); a grouped RCCL send/recv on a high-priority
 * stream gathers every rank's slot on rank 0.  RCCL (librccl.so.1) is loaded
 * at run time -- the copy already in the process if there is one -- so the
 * single-GPU library needs none.
 * pt_dist_unique_id: rank 0 makes the communicator id (128 bytes), which the
 * caller broadcasts (e.g. over torch.distributed); pt_dist_init: every rank,
 * collectively, after setting the same partition (or, to time the root's
 * step on one GPU, nranks = 1 with an N-way partition on rank 0: the other
 * ranks' slots then arrive as a device copy of the same bytes -- an
 * emulation, not a gather); pt_dist_run: n_frames frames of n_batches
 * samples (batch 0..n-1, fresh) on 1 to 3 alternating streams (2 or 3: a
 * frame's tail overlaps the next ones' heads; max(2, n_streams) frames are
 * in flight before the root assembles one); the root writes frame j
 * to frames + (j % n_frame_bufs) * W*H*4 floats (device memory; ignored on
 * other ranks).  Every rank must have rendered the frame's configuration once
 * with pt_render (it fixes the item layout).  Work is enqueued; the frames
 * are complete after pt_synchronize.  pt_dist_finalize frees it (also done
 * by pt_destroy).  Replaces, for the tile split, the reference's
 * dispatch-and-readback per frame (VulkanRayTracer.cpp:803-865). */
#define PT_DIST_ID_BYTES 128
int pt_dist_unique_id(void* id, size_t id_bytes);
int pt_dist_init(pt_context* ctx, const void* id, int nranks, int rank);
int pt_dist_run(pt_context* ctx, uint32_t n_batches, int n_frames, int n_streams, void* frames_device,
                int n_frame_bufs);
/* Run the loop on caller-owned streams (e.g. torch streams) instead of the
 * ones it creates: the first two render streams and the gather stream (null
 * keeps the library's own).  With caller render streams pt_dist_run takes at
 * most 2 streams (PT_ERR_INVALID for 3, which would mix in a library stream
 * outside the caller's ordering).  The library creates its render streams at the least priority
 * and the gather stream at the greatest: the HIP runtime keeps a pool of
 * GPU_MAX_HW_QUEUES hardware queues per priority, so each render stream gets
 * a queue of its own. */
int pt_dist_set_streams(pt_context* ctx, void* render_stream0, void* render_stream1, void* gather_stream);
int pt_dist_slot_floats(pt_context* ctx, size_t* slot_floats);
/* Wait (polling) up to timeout_ms for the loop's streams; PT_ERR_HIP on
 * timeout.  pt_dist_abort: ncclCommAbort + free, after such a timeout. */
int pt_dist_wait(pt_context* ctx, int timeout_ms);
int pt_dist_abort(pt_context* ctx);
/* The communicator's rank count as RCCL reports it (ncclCommCount; -1 if
 * the loaded library lacks it), and the rank count / rank pt_dist_init took. */
int pt_dist_info(pt_context* ctx, int* comm_ranks, int* nranks, int* rank);
int pt_dist_finalize(pt_context* ctx);

/* ---- kernel options ---------------------------------------------------- */
/* PT_OPT_SCENE_IN_LDS: stage the scene in LDS per workgroup — 0 never,
 * 1 when it fits in 48 KB (default), 2 always (error if it does not fit).
 * Output is identical either way. */
#define PT_OPT_SCENE_IN_LDS 1
/* PT_OPT_SAMPLE_LANES: lanes that trace one pixel's samples side by side in
 * pt_render — 0 auto (scenes in device memory 8; LDS-resident scenes 4 on a
 * whole frame or a partition of 8 or more ranks, 2 on 2-7 ranks; never more
 * lanes than samples), or 1, 2, 4, 8.  Output is identical for every value. */
#define PT_OPT_SAMPLE_LANES 2
/* PT_OPT_FRESH_BATCH0: 1 = a launch whose first batch is 0 starts from a
 * cleared (+0) accumulator without reading it — bitwise what
 * pt_clear_accum + pt_render give, minus a clear and a read of the image.
 * 0 (default) = read the accumulator, as the reference does (prev * 0). */
#define PT_OPT_FRESH_BATCH0 3
/* PT_OPT_KERNEL: 0 auto (wavefront for scenes of >= 32768 triangles that
 * are not LDS-resident, else path-recursive), 1 path-recursive, 3 wavefront
 * pipeline (paths held in device memory, traversal and shading in separate
 * kernels; 416 bytes of device memory per pixel x sample, at most 2^27 paths
 * per chunk; not with stats mode; auto picks it from 16384 triangles with the
 * culled wide walk).  Output is identical for every value.  2 (a lane state
 * machine, measured slower on every scene) was removed: PT_ERR_UNSUPPORTED,
 * as is PT_OPT_SM_BATCH, its only knob. */
#define PT_OPT_KERNEL 4
#define PT_OPT_SM_BATCH 5
/* PT_OPT_PRIMARY_CULL: 1 (default) = a pixel whose every possible primary
 * ray provably misses the scene's root box and every light (outside all of
 * pt_primary_cull_rects' rectangles) is not ray-generated: each of its samples
 * is (0,0,0) exactly as the reference computes it (pre-pass misses, depth-0
 * traceRay misses, background 0).  0 = generate and trace every sample.
 * Path-recursive and wavefront kernels; output is identical either way. */
#define PT_OPT_PRIMARY_CULL 6
/* PT_OPT_WF_PATHS: wavefront kernel only — paths (pixel x sample) held in
 * device memory per chunk; 0 = 2^27 (56 GB; halved until the allocation
 * succeeds).  A launch with more runs in chunks of whole batches (at least
 * one batch of the frame per chunk).
 * Output is identical for every value. */
#define PT_OPT_WF_PATHS 7
/* PT_OPT_ITEM_ORDER: 1 = live items (tile parts) launched heaviest first by
 * a host estimate (pixels inside the root box's rectangle), so long
 * workgroups start early and short ones fill the tail; 0 = scan order; -1
 * (default) = auto: scan order for a whole frame on the path-recursive
 * kernel, heaviest first on a share of the frame and on the wavefront
 * pipeline.  The packed exchange layout follows the same order.  Output is
 * identical. */
#define PT_OPT_ITEM_ORDER 8
/* PT_OPT_LAUNCH_TIMING: record a HIP event pair around every k-th render
 * launch (0 = none, the default since ABI 3: on one stream a pair cost the box
 * frame ~10 us of its ~0.25 ms) for pt_last_launch_ms / pt_launch_times_ms /
 * pt_launch_span_ms.  Output-invariant. */
#define PT_OPT_LAUNCH_TIMING 9
/* PT_OPT_COUNT_TRACED: 1 = run the fast kernels with counters of the work
 * they actually do (pt_get_traced); slower, output identical.  Default 0. */
#define PT_OPT_COUNT_TRACED 10
/* PT_OPT_PAIRS: 0 only.  1 (child-pair records, measured slower on every
 * scene) was removed: PT_ERR_UNSUPPORTED. */
#define PT_OPT_PAIRS 11
/* PT_OPT_WIDE: 1 (default) = the wavefront pipeline walks device-memory
 * scenes over a 4-wide BVH of the reference's own boxes, nearest child first,
 * culling children that cannot hold a hit at or before the best one found
 * (the bound is exact-safe for the shader's float
 * Moller-Trumbore, so every hit is the exhaustive DFS's bit for bit).  Built
 * at upload when the tree's boxes contain their subtrees (any
 * BoundingVolumeHierarchy.cpp tree does); pt_wide_info reports it.  0 = the
 * threaded exhaustive walk; 2 = the wide walk with every odd ray of each
 * round handed to the exact walk (tests the hand-back path).  Output is
 * identical. */
#define PT_OPT_WIDE 12
/* PT_OPT_WF_STREAMS: 2 = the wavefront pipeline runs a chunk's pixels as
 * two halves on the context's stream and a second stream of its own (forked
 * from and joined back into the context's stream), so one half's trace and
 * shading can fill the other's launch tails; 1 (default; 2 measured slower
 * on the random clouds) = one stream.  Output is identical. */
#define PT_OPT_WF_STREAMS 13
/* PT_OPT_WIDE_BUILD (read by pt_upload_scene): how the culled wide walk's
 * 4-wide nodes group the reference's leaves.  1 (default) = a binned-SAH tree
 * over the reference's leaf boxes; 0 = the reference's own tree collapsed to
 * 4-wide nodes.  Every child box is a reference leaf box bitwise or contains
 * the leaf boxes below it, so the walk's answers are the same. */
#define PT_OPT_WIDE_BUILD 14
/* PT_OPT_WF_FUSE: 1 (default) = with the culled wide walk, a lane of the
 * wavefront traversal kernel that finds a closest hit for a primary, bounce
 * or SSS ray also samples the path's first light (the draws pathTrace makes
 * next, raytrace_comp.comp:345-366 / :383-402) and walks that shadow ray
 * itself, so the path skips a ray round; the shading kernel takes both
 * answers and runs the same shading.  0 = one ray per round.  Output is
 * identical. */
#define PT_OPT_WF_FUSE 15
/* PT_OPT_WIDE_NODE: byte size of the culled wide walk's nodes.  64 (default)
 * = child boxes rounded outward onto an 8-bit grid per node (half the bytes
 * and load instructions per node visit; a leaf's exact box is tested before
 * its hit counts); 128 = the boxes as floats.  Both are built at upload.
 * Output is identical.  80 (8-wide nodes, measured slower) was removed:
 * PT_ERR_UNSUPPORTED. */
#define PT_OPT_WIDE_NODE 16
/* PT_OPT_WF_TAIL: with the culled wide walk (4-wide nodes), once a ray
 * round's list holds fewer than this many rays, one persistent launch runs
 * every remaining path to its end (each lane walks a ray, shades it and walks
 * the path's next ray) instead of a trace and a shading launch per remaining
 * round; 0 = never; -1 (default) = auto (400000 rays).  Output is
 * identical. */
#define PT_OPT_WF_TAIL 17
/* PT_OPT_GROUP_EXCHANGE (pt_create_multi contexts only): 0 (default) = each
 * member stores its tiles straight into the frame on the first device (peer
 * access over xGMI) when every member can map it, else packed copies; 1 =
 * always packed copies (pt_tiles_pack, hipMemcpyPeerAsync, pt_tiles_unpack).
 * Output is identical. */
#define PT_OPT_GROUP_EXCHANGE 18
/* PT_OPT_GROUP_CHECK (pt_create_multi contexts only): before peer stores
 * carry a frame, a probe frame (16n x 32 pixels, 1 spp) is rendered once
 * through peer stores and once through the staged exchange, and the two are
 * compared bit for bit; on any difference the context falls back to the
 * staged exchange for good (pt_group_check reports it).  1 (default) = once
 * per context, when its members span distinct devices; 2 = on the first
 * render after every pt_resize_and_clear / pt_bind_accum, any devices; 3 =
 * as 2 with a mismatch forced (tests of the fallback); 0 = never. */
#define PT_OPT_GROUP_CHECK 19
/* PT_OPT_WF_GRID: wavefront traversal launches use this percentage (1-100,
 * default 100) of a full-occupancy persistent grid; with frames in flight on
 * several contexts a smaller grid gives each lane more rays per round.
 * Output is identical. */
#define PT_OPT_WF_GRID 20
/* PT_OPT_WF_REFILL: idle lanes at which a wave of the wavefront's wide
 * traversal kernel claims new rays; 0 (default) = auto: 16 with a full grid,
 * 8 with PT_OPT_WF_GRID below 100.  Output is identical. */
#define PT_OPT_WF_REFILL 21
/* PT_OPT_MIXED_LANES: one-rank path-recursive launches of LDS-resident scenes
 * (box.obj) with primary culling mix lane counts per workgroup: whole 16x16
 * tiles at one lane per pixel (all samples of a pixel in one lane: the least
 * work per sample, the longest workgroups) and tile parts at more lanes
 * (short workgroups that fill the launch's drain).  -1 (default) = measured:
 * until the frame's inputs have been measured, the first live tiles up to
 * half of the workgroups the device holds at once run whole and the rest at
 * PT_OPT_SAMPLE_LANES; render_kernel meanwhile times its blocks (two
 * launches once the inputs are unchanged for a render, copied back without
 * a host wait), and from then on every tile gets the fewest lanes that keep
 * its workgroups short enough, longest first, the lane cut chosen by a
 * simulation of the launch (pt_mixed_info reports the schedule).  A change of
 * size, batches, camera, params, scene or lights starts over.  k = 1-1000:
 * the static schedule with whole tiles for k % of the resident workgroups,
 * never measured.  0 = off (every item at PT_OPT_SAMPLE_LANES).  Output is
 * identical for every value. */
#define PT_OPT_MIXED_LANES 22
int pt_set_option(pt_context* ctx, int key, int value);
/* The kernel the last pt_render / pt_dispatch ran (PT_OPT_KERNEL values 1-3,
 * after auto selection); 0 before the first render. */
int pt_last_kernel(pt_context* ctx, int* kernel);

/* Screen regions that primary rays can reach the scene or a light from.
 * Writes up to max_rects NDC rectangles {x0, x1, y0, y1} (one per object:
 * the root box, then each light) to rects and their count to *n_rects; a
 * pixel whose (2px/W - 1, 2py/H - 1) lies outside all of them has no primary
 * ray (any aperture draw, any jitter draw — Box-Muller radii are bounded by
 * 13.23 since u1 >= 1e-38, raytrace_comp.comp:220) that hits the root box or
 * a light.  *n_rects = -1 when no such guarantee is derived (object at or
 * behind the camera plane, degenerate camera, more lights than max_rects-1):
 * every pixel is then traced.  Pure host function. */
int pt_primary_cull_rects(const float camera_ubo[16], int width, int height, const float root_min[3],
                          const float root_max[3], const pt_area_light* lights, int n_lights, float* rects,
                          int max_rects, int* n_rects);

/* ---- instrumentation --------------------------------------------------- */
/* Stats mode runs the reference-exhaustive traversal with counters (output is
 * unchanged); used for the roofline's algorithmic byte count. */
int pt_set_stats_mode(pt_context* ctx, int enabled);
int pt_get_stats(pt_context* ctx, pt_stats* out);
int pt_reset_stats(pt_context* ctx);
int pt_get_traced(pt_context* ctx, pt_traced* out);
/* The culled wide walk of the uploaded scene (PT_OPT_WIDE): info[0] = wide
 * nodes (0 = not built; pt_last_error() then says why), info[1] = the most
 * stack entries one walk can hold. */
int pt_wide_info(pt_context* ctx, int info[2]);
/* Mixed sample lanes of the last path-recursive launch (PT_OPT_MIXED_LANES):
 * info[0] = 0 uniform lanes, 1 the static mixed schedule, 2 the measured one;
 * info[1] = live workgroups it launched; info[2] = measuring launches folded
 * into the current inputs' block costs.  Multi-device contexts: zeros. */
int pt_mixed_info(pt_context* ctx, int info[3]);
/* Device time of the last pt_render/pt_dispatch launch, from HIP events
 * recorded on the launch stream. */
int pt_last_launch_ms(pt_context* ctx, float* ms);
/* Device times of every render launch since pt_reset_launch_times (the last
 * 512 at most), oldest first; waits for them to finish. */
int pt_launch_times_ms(pt_context* ctx, float* out, size_t max_n, size_t* n_out);
/* Device time from the start of the first render launch since
 * pt_reset_launch_times to the end of the last one (launches on several
 * streams overlap, so their durations do not add up); *n_out = launches.
 * Waits for them to finish; PT_ERR_UNSUPPORTED past 512 launches. */
int pt_launch_span_ms(pt_context* ctx, float* ms, size_t* n_out);
int pt_reset_launch_times(pt_context* ctx);
/* Evaluates the kernel's fp32 math on the device for bitwise checks against
 * the oracle: fn 0 log, 1 exp, 2 sin, 3 cos, 4 tan, 5 acos, 6 sqrt,
 * 7 first RNG draw from the seed given as the float's bits, 8 reciprocal. */
int pt_selftest_math(int device_ordinal, int fn, const float* x, float* y, size_t n);
/* Exhaustive check of the device's fast-quotient math against its IEEE
 * definitions over all 2^32 inputs: fn 0 rcp (1/x), 1 log, 2 exp, 3 acos.
 * Writes the number of differing inputs and the smallest such
 * input's bit pattern (0xffffffff if none). */
int pt_selftest_exhaustive(int device, int fn, unsigned long long* mismatches, uint32_t* first_bad);

/* ---- host scene layer (L1 producers: BVH, Light, OBJ ingest) ----------- */
typedef struct pt_scene pt_scene;
/* tinyobj::ObjReader::ParseFromFile + index gathering (VulkanRayTracer.cpp:64-92) */
int pt_scene_load_obj(const char* path, pt_scene** out);
int pt_scene_parse_obj(const char* text, size_t len, pt_scene** out);
/* scene from raw arrays (e.g. synthetic meshes) */
int pt_scene_from_arrays(const float* vertices, size_t n_vertex_floats,
                         const uint32_t* indices, size_t n_indices, pt_scene** out);
/* BVH bvh(objVertices, objIndices) (BoundingVolumeHierarchy.cpp:5-23);
 * flags: PT_NODES_INT_BITS; threads 0 = all cores. */
int pt_scene_build_bvh(pt_scene* scene, uint32_t flags, int threads);
int pt_scene_counts(const pt_scene* scene, size_t* n_vertex_floats, size_t* n_indices,
                    size_t* n_nodes, size_t* n_uv_floats, size_t* n_mat);
int pt_scene_copy(const pt_scene* scene, float* vertices, uint32_t* indices, pt_bvh_node* nodes,
                  float* uvs, uint32_t* mat_indices);
int pt_scene_upload(pt_context* ctx, const pt_scene* scene);
int pt_scene_free(pt_scene* scene);
/* Binary scene cache (skip OBJ parse + BVH build for large
 * meshes): everything pt_scene_copy returns, with an FNV-1a checksum.  Load
 * fails with PT_ERR_IO on a missing, foreign, truncated or corrupt file. */
int pt_scene_save(const pt_scene* scene, const char* path);
int pt_scene_load_cache(const char* path, pt_scene** out);
/* Light lights(positions, normals, intensities, sizes) packing (Light.cpp:16-33) */
int pt_pack_light(const float position[3], const float normal[3], const float intensity[3],
                  const float size[2], pt_area_light* out);
/* Writes a W x H RGBA32F accumulation image (row y = 0 first in memory) for
 * inspection: PT_IMAGE_PFM = float RGB PFM (rows
 * bottom-to-top, i.e. row 0 first); PT_IMAGE_PNG = 8-bit sRGB PNG of the
 * colours clamped to [0,1], top row = last buffer row. */
#define PT_IMAGE_PFM 0
#define PT_IMAGE_PNG 1
int pt_write_image(const char* path, const float* rgba, int width, int height, int format);
/* Camera getters for the reference's default orbit camera, as the UBO
 * (Camera.cpp:4-10, 84-106): pos (0,0,5) dir (0,0,-1) up (0,1,0) fov 60. */
int pt_default_camera(float camera_ubo[16]);

#ifdef __cplusplus
}
#endif
#endif /* PATHTRACER_H_ */
