// pt_group.cpp — one context driving several GPUs from one process
// (pt_create_multi, include/pathtracer.h).
//
// The reference drives its GPU from one detached thread of one process
// (VulkanRenderer.cpp:643-647; the loop is VulkanRayTracer::mainLoop,
// VulkanRayTracer.cpp:717-865).  A group gives that caller the tile split of
// SURVEY §8e without a launcher: member r is an ordinary context on device
// ordinals[r] owning the screen tiles b with b % n == r (pt_set_partition,
// rows rotated), and every call on the group behaves as on one device, with
// the frame in device memory of ordinals[0].
//
// Exchange.  In one process the devices of an MI355X node reach each
// other's HBM over xGMI with ordinary loads and stores once peer access is
// enabled, so no collective is needed: every member binds the frame on
// ordinals[0] as its accumulation buffer (pt_bind_accum) and its render
// kernel reads and writes its own tiles there.  The only traffic is the
// accumulator's own 16 B per owned pixel per launch (read only when the
// first batch is not 0), spread over the kernel; the tiles are disjoint, so
// no two members touch a pixel.  Where a member cannot map the first device
// (or with PT_OPT_GROUP_EXCHANGE 1) it renders into an accumulation buffer of
// its own (+0 on its tiles, -0 elsewhere) and after each launch packs its
// tiles (pt_tiles_pack), copies them to a receive buffer on the first device
// (hipMemcpyPeerAsync) and the first device scatters them into the frame
// (pt_tiles_unpack).  Either way the frame is bit-identical to a single-GPU
// render: each pixel is computed by exactly one member, by the same kernels.
//
// Ordering.  The first member's stream is the group's stream.  A render
// records an event on it that every other member's stream waits for (so the
// clear or readback before it is done), and the group's stream then waits
// for every member's completion event (so a read, clear or readback after it
// sees every tile).  Members on other devices are waited for with
// cross-device events, never with a host synchronisation.
#include "pt_group.h"

#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace {

#define G_HIP(call)                                                                             \
  do {                                                                                          \
    hipError_t e_ = (call);                                                                     \
    if (e_ != hipSuccess) return pt_fail_internal(PT_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e_)); \
  } while (0)

#define G_RC(call)            \
  do {                        \
    const int rc_ = (call);   \
    if (rc_) return rc_;      \
  } while (0)

constexpr int kOptGroupExchange = 18;   // PT_OPT_GROUP_EXCHANGE (pathtracer.h)
constexpr int kOptGroupCheck = 19;      // PT_OPT_GROUP_CHECK (pathtracer.h)
constexpr int kOptCountTraced = 10;     // PT_OPT_COUNT_TRACED (pathtracer.h)
constexpr int kOptLaunchTiming = 9;     // PT_OPT_LAUNCH_TIMING (pathtracer.h)

}  // namespace

struct pt_group {
  int n = 0;
  std::vector<int> dev;              // member r's device
  std::vector<pt_context*> m;        // member contexts
  std::vector<hipStream_t> own;      // streams created here, one per member
  std::vector<hipStream_t> s;        // the streams the members run on (s[0] may be the caller's)
  std::vector<hipEvent_t> done;      // member r's last launch (r > 0)
  hipEvent_t start = nullptr;        // the group stream's work before a render
  bool peer_ok = true;               // peer stores usable: mapped, and not refused by the exchange check
  bool peer_map_ok = true;           // every member can map the first device's memory
  int exchange = 0;                  // PT_OPT_GROUP_EXCHANGE: 0 auto, 1 staged copies
  bool staged = false;               // the exchange the current frame buffer was set up for
  // PT_OPT_GROUP_CHECK: before peer stores carry a frame whose members span
  // devices, one probe frame through peer stores and one through the staged
  // exchange are compared bit for bit (check_exchange)
  int check = 1;                     // 0 never, 1 once per group (distinct devices), 2 every binding, 3 as 2, mismatch forced (tests)
  bool check_pending = false;        // armed by setup_frame, run by the next render
  bool check_passed = false;
  int check_state = -1;              // -1 not run, 0 peer stores matched, 1 mismatch: staged copies in force,
                                     // 2 the peer-store probe failed: staged copies in force
  float check_ms[2] = {0.0f, 0.0f};  // the probe frames' wall time: peer stores, staged copies
  bool stats_mode = false;           // the members' counters (stats mode, PT_OPT_COUNT_TRACED) are off
  bool count_traced = false;         // during the probe frames and restored after
  int timing = 1;                    // PT_OPT_LAUNCH_TIMING of the members (member 0's ring is the group's):
                                     // off during the probe frames and restored after
  float* frame = nullptr;            // W x H float4 on dev[0]
  bool own_frame = false;
  int W = 0, H = 0;
  // staged exchange: member r's tiles, packed on its device and received on dev[0]
  std::vector<float*> pack_local, pack_root;
  std::vector<size_t> pack_bytes;
  // progressive loop (the group's own counter; VulkanRayTracer.cpp:739-754)
  float prog_cam[16] = {0};
  bool prog_has_cam = false;
  uint32_t prog_batch = 0;
  // Enqueue threads: with three or more members, members 1..n-1 enqueue
  // their launches from threads of their own (one per member, parked on a
  // condition variable), so a frame's host cost is one member's enqueue
  // (~10-15 us) rather than n of them; member 0 enqueues on the caller's
  // thread.
  std::vector<std::thread> workers;
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::function<int(int)> job;
  uint64_t gen = 0;
  int pending = 0;
  bool stop = false;
  std::vector<int> job_rc;
  std::vector<std::string> job_err;
};

namespace {

template <class T>
void gfree(int device, T*& p) {
  if (p) {
    (void)hipSetDevice(device);
    (void)hipFree(p);
  }
  p = nullptr;
}

// Runs f(r) for every member, concurrently when there is more than one
// device (host-side scene preparation and uploads), and returns the first
// failure with its message.
template <class F>
int each_parallel(pt_group* g, F f) {
  if (g->n == 1) return f(0);
  std::vector<int> rc((size_t)g->n, PT_OK);
  std::vector<std::string> msg((size_t)g->n);
  std::vector<std::thread> t;
  for (int r = 0; r < g->n; ++r)
    t.emplace_back([&, r] {
      rc[(size_t)r] = f(r);
      if (rc[(size_t)r]) msg[(size_t)r] = pt_last_error();
    });
  for (auto& x : t) x.join();
  for (int r = 0; r < g->n; ++r)
    if (rc[(size_t)r]) return pt_fail_internal(rc[(size_t)r], "member " + std::to_string(r) + ": " + msg[(size_t)r]);
  return PT_OK;
}

template <class F>
int each(pt_group* g, F f) {
  for (int r = 0; r < g->n; ++r) G_RC(f(r));
  return PT_OK;
}

void worker_main(pt_group* g, int r) {
  (void)hipSetDevice(g->dev[(size_t)r]);
  uint64_t seen = 0;
  for (;;) {
    std::function<int(int)> f;
    {
      std::unique_lock<std::mutex> lk(g->mu);
      g->cv_job.wait(lk, [&] { return g->stop || g->gen != seen; });
      if (g->stop) return;
      seen = g->gen;
      f = g->job;
    }
    const int rc = f(r);
    std::lock_guard<std::mutex> lk(g->mu);
    g->job_rc[(size_t)r] = rc;
    if (rc) g->job_err[(size_t)r] = pt_last_error();
    if (--g->pending == 0) g->cv_done.notify_one();
  }
}

// f(r) for every member: members 1..n-1 on their enqueue threads (when the
// group has them), member 0 on the caller's; the first failure is returned.
int each_member(pt_group* g, const std::function<int(int)>& f) {
  if (g->workers.empty()) return each(g, f);
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->job = f;
    g->pending = g->n - 1;
    std::fill(g->job_rc.begin(), g->job_rc.end(), PT_OK);
    ++g->gen;
  }
  g->cv_job.notify_all();
  const int rc0 = f(0);
  const std::string err0 = rc0 ? pt_last_error() : "";
  std::unique_lock<std::mutex> lk(g->mu);
  g->cv_done.wait(lk, [&] { return g->pending == 0; });
  if (rc0) return pt_fail_internal(rc0, err0);
  for (int r = 1; r < g->n; ++r)
    if (g->job_rc[(size_t)r])
      return pt_fail_internal(g->job_rc[(size_t)r], "member " + std::to_string(r) + ": " + g->job_err[(size_t)r]);
  return PT_OK;
}

void stop_workers(pt_group* g) {
  {
    std::lock_guard<std::mutex> lk(g->mu);
    g->stop = true;
  }
  g->cv_job.notify_all();
  for (auto& t : g->workers)
    if (t.joinable()) t.join();
  g->workers.clear();
}

void free_exchange(pt_group* g) {
  for (int r = 0; r < g->n; ++r) {
    if (r < (int)g->pack_local.size()) gfree(g->dev[(size_t)r], g->pack_local[(size_t)r]);
    if (r < (int)g->pack_root.size()) gfree(g->dev[0], g->pack_root[(size_t)r]);
  }
  g->pack_local.assign((size_t)g->n, nullptr);
  g->pack_root.assign((size_t)g->n, nullptr);
  g->pack_bytes.assign((size_t)g->n, 0);
}

int quiesce_all(pt_group* g) {
  for (int r = 0; r < g->n; ++r) {
    G_HIP(hipSetDevice(g->dev[(size_t)r]));
    G_HIP(hipStreamSynchronize(g->s[(size_t)r]));
  }
  return PT_OK;
}

bool distinct_devices(const pt_group* g) {
  for (int r = 1; r < g->n; ++r)
    if (g->dev[(size_t)r] != g->dev[0]) return true;
  return false;
}

// (Re)binds the frame of W x H on dev[0] to the members for the exchange in
// force: peer stores (every member renders into the frame) or staged copies
// (members r > 0 render into their own buffers and ship packed tiles).  A
// staged member's buffer starts as a copy of the frame, so a render that
// continues the accumulation (first batch > 0) reads the frame's history
// whichever exchange was in force before.  arm: a new binding,
// which the exchange check (PT_OPT_GROUP_CHECK) covers before it is used.
// history: the frame holds an accumulation to continue (false right after
// an allocation that a clear follows: no copy).
int setup_frame(pt_group* g, bool arm = true, bool history = true) {
  G_RC(quiesce_all(g));
  free_exchange(g);
  g->staged = g->n > 1 && (g->exchange == 1 || !g->peer_ok);
  if (g->staged && history) {   // the copies below follow the frame's last writer on s[0]
    G_HIP(hipSetDevice(g->dev[0]));
    G_HIP(hipEventRecord(g->start, g->s[0]));
  }
  for (int r = 0; r < g->n; ++r) {
    pt_context* c = g->m[(size_t)r];
    if (r == 0 || !g->staged) {
      G_RC(pt_bind_accum(c, g->frame, g->W, g->H));
      continue;
    }
    G_RC(pt_resize_and_clear(c, g->W, g->H));   // +0 on its tiles, -0 elsewhere
    const size_t frame_bytes = (size_t)g->W * g->H * 16;
    G_HIP(hipSetDevice(g->dev[(size_t)r]));
    if (history) {
      // after the clear, on the member's stream: its tiles start from the frame's content
      G_HIP(hipStreamWaitEvent(g->s[(size_t)r], g->start, 0));
      G_HIP(hipMemcpyPeerAsync(pt_accum_device_ptr(c), g->dev[(size_t)r], g->frame, g->dev[0], frame_bytes,
                               g->s[(size_t)r]));
      pt_note_accum_written(c, false);
    }
    int tiles = 0;
    G_RC(pt_tiles_owned(c, &tiles));
    const size_t bytes = (size_t)std::max(tiles, 1) * 256 * 16;
    G_HIP(hipMalloc((void**)&g->pack_local[(size_t)r], bytes));
    G_HIP(hipSetDevice(g->dev[0]));
    G_HIP(hipMalloc((void**)&g->pack_root[(size_t)r], bytes));
    g->pack_bytes[(size_t)r] = bytes;
  }
  if (arm)
    g->check_pending = !g->staged && g->n > 1 &&
                       (g->check >= 2 || (g->check == 1 && !g->check_passed && distinct_devices(g)));
  return PT_OK;
}

// One frame of every member on the group's stream ordering (render's
// events): start after s[0]'s work, s[0] waits for every member.  staged:
// members r > 0 pack their tiles, copy them to dev[0] and member 0 unpacks
// them into `frame`.
int run_members(pt_group* g, uint32_t first_batch, uint32_t n_batches, bool staged, void* frame,
                const std::vector<float*>& loc, const std::vector<float*>& root, const std::vector<size_t>& bytes,
                bool threads) {
  G_HIP(hipSetDevice(g->dev[0]));
  G_HIP(hipEventRecord(g->start, g->s[0]));
  auto one = [&](int r) -> int {
    if (r == 0) return pt_render(g->m[0], first_batch, n_batches);
    G_HIP(hipSetDevice(g->dev[(size_t)r]));
    G_HIP(hipStreamWaitEvent(g->s[(size_t)r], g->start, 0));
    G_RC(pt_render(g->m[(size_t)r], first_batch, n_batches));
    if (staged) {
      G_RC(pt_tiles_pack(g->m[(size_t)r], loc[(size_t)r]));
      G_HIP(hipSetDevice(g->dev[(size_t)r]));
      G_HIP(hipMemcpyPeerAsync(root[(size_t)r], g->dev[0], loc[(size_t)r], g->dev[(size_t)r], bytes[(size_t)r],
                               g->s[(size_t)r]));
    }
    G_HIP(hipSetDevice(g->dev[(size_t)r]));
    G_HIP(hipEventRecord(g->done[(size_t)r], g->s[(size_t)r]));
    return PT_OK;
  };
  G_RC(threads ? each_member(g, one) : each(g, one));
  G_HIP(hipSetDevice(g->dev[0]));
  for (int r = 1; r < g->n; ++r) {
    G_HIP(hipStreamWaitEvent(g->s[0], g->done[(size_t)r], 0));
    if (staged) G_RC(pt_tiles_unpack(g->m[0], root[(size_t)r], r, frame));
  }
  return PT_OK;
}

// PT_OPT_GROUP_CHECK.  Peer stores assume that a member kernel's stores into
// the first device's memory are visible there once the group's stream has
// waited for the member's completion event -- as the reference's dispatch
// result is visible when its fence returns (VulkanCommandBuffer.cpp:140).
// Before the first frame relies on that, a probe frame of 16n x 32 pixels
// (two tiles per member) at 1 spp is rendered both ways -- peer stores into
// one buffer on the first device, and the staged exchange (pack, peer copy,
// unpack) into another -- and the two are compared bit for bit on the host.
// On any difference the group falls back to the staged exchange for good.
// check == 3 (tests) flips one bit of the peer-store probe before comparing.
int check_exchange(pt_group* g) {
  g->check_pending = false;
  const int n = g->n, PW = 16 * n, PH = 32;
  const size_t fbytes = (size_t)PW * PH * 16;
  float* probe[2] = {nullptr, nullptr};   // peer stores, staged copies
  std::vector<float*> loc((size_t)n, nullptr), root((size_t)n, nullptr);
  std::vector<size_t> bytes((size_t)n, 0);
  std::vector<float> host[2];
  auto release = [&]() {
    (void)quiesce_all(g);
    for (int r = 0; r < n; ++r) {
      gfree(g->dev[(size_t)r], loc[(size_t)r]);
      gfree(g->dev[0], root[(size_t)r]);
    }
    gfree(g->dev[0], probe[0]);
    gfree(g->dev[0], probe[1]);
  };
  // the probe frames are not the caller's frames: no stats or traced counts
  // nor launch times in member 0's ring
  auto counters = [&](bool on) -> int {
    if (g->stats_mode) G_RC(each(g, [&](int r) { return pt_set_stats_mode(g->m[(size_t)r], on ? 1 : 0); }));
    if (g->count_traced)
      G_RC(each(g, [&](int r) { return pt_set_option(g->m[(size_t)r], kOptCountTraced, on ? 1 : 0); }));
    G_RC(pt_set_option(g->m[0], kOptLaunchTiming, on ? g->timing : 0));
    return PT_OK;
  };
  auto body = [&]() -> int {
    G_RC(counters(false));
    G_RC(quiesce_all(g));
    G_HIP(hipSetDevice(g->dev[0]));
    for (float*& p : probe) {
      G_HIP(hipMalloc((void**)&p, fbytes));
      G_HIP(hipMemset(p, 0, fbytes));
    }
    // peer stores: every member renders its tiles straight into probe[0]
    for (int r = 0; r < n; ++r) G_RC(pt_bind_accum(g->m[(size_t)r], probe[0], PW, PH));
    // Production ordering: a frame's consumers see the members'
    // stores only through s[0], which run_members makes wait for every
    // member's completion event -- so the probe is read back on s[0] behind
    // that wait, with no host-side synchronisation of the members first.
    for (int k = 0; k < 2; ++k) host[k].resize(fbytes / 4);
    auto t0 = std::chrono::steady_clock::now();
    G_RC(run_members(g, 0, 1, false, probe[0], loc, root, bytes, false));
    G_HIP(hipSetDevice(g->dev[0]));
    G_HIP(hipMemcpyAsync(host[0].data(), probe[0], fbytes, hipMemcpyDeviceToHost, g->s[0]));
    G_HIP(hipStreamSynchronize(g->s[0]));
    auto t1 = std::chrono::steady_clock::now();
    G_RC(quiesce_all(g));
    // staged copies into probe[1]
    G_RC(pt_bind_accum(g->m[0], probe[1], PW, PH));
    for (int r = 1; r < n; ++r) {
      pt_context* c = g->m[(size_t)r];
      G_RC(pt_resize_and_clear(c, PW, PH));
      int tiles = 0;
      G_RC(pt_tiles_owned(c, &tiles));
      bytes[(size_t)r] = (size_t)std::max(tiles, 1) * 256 * 16;
      G_HIP(hipSetDevice(g->dev[(size_t)r]));
      G_HIP(hipMalloc((void**)&loc[(size_t)r], bytes[(size_t)r]));
      G_HIP(hipSetDevice(g->dev[0]));
      G_HIP(hipMalloc((void**)&root[(size_t)r], bytes[(size_t)r]));
    }
    G_RC(quiesce_all(g));
    auto t2 = std::chrono::steady_clock::now();
    G_RC(run_members(g, 0, 1, true, probe[1], loc, root, bytes, false));
    G_HIP(hipSetDevice(g->dev[0]));
    G_HIP(hipMemcpyAsync(host[1].data(), probe[1], fbytes, hipMemcpyDeviceToHost, g->s[0]));
    G_HIP(hipStreamSynchronize(g->s[0]));
    auto t3 = std::chrono::steady_clock::now();
    G_RC(quiesce_all(g));
    g->check_ms[0] = std::chrono::duration<float, std::milli>(t1 - t0).count();
    g->check_ms[1] = std::chrono::duration<float, std::milli>(t3 - t2).count();
    return PT_OK;
  };
  int rc = body();
  release();
  const int rc2 = counters(true);
  if (!rc) rc = rc2;
  if (rc == PT_ERR_INVALID) {   // a precondition (no scene, camera or params yet): the render fails, and
                                // the check runs again on the next one
    const std::string msg = pt_last_error();
    (void)setup_frame(g, false);
    g->check_pending = true;
    return pt_fail_internal(rc, "pt_create_multi exchange check: " + msg);
  }
  if (rc) {   // the probe itself failed: staged copies for good, and the render goes on
    g->check_state = 2;
    g->check_passed = false;
    g->peer_ok = false;
    return setup_frame(g, false);
  }
  if (g->check == 3) {
    uint32_t w;
    memcpy(&w, &host[0][0], 4);
    w ^= 1u;
    memcpy(&host[0][0], &w, 4);
  }
  const bool same = memcmp(host[0].data(), host[1].data(), fbytes) == 0;
  g->check_state = same ? 0 : 1;
  g->check_passed = same;
  if (!same) g->peer_ok = false;   // staged copies from now on
  return setup_frame(g, false);
}

}  // namespace

namespace ptg {

int make(const int* ordinals, int n, pt_group** out) {
  if (!ordinals || !out) return pt_fail_internal(PT_ERR_INVALID, "null argument");
  if (n < 1 || n > 64) return pt_fail_internal(PT_ERR_INVALID, "pt_create_multi: 1 to 64 devices");
  *out = nullptr;
  int ndev = 0;
  G_HIP(hipGetDeviceCount(&ndev));
  for (int r = 0; r < n; ++r)
    if (ordinals[r] < 0 || ordinals[r] >= ndev)
      return pt_fail_internal(PT_ERR_INVALID, "device ordinal " + std::to_string(ordinals[r]) + " out of range (" +
                                                  std::to_string(ndev) + " devices)");
  pt_group* g = new pt_group();
  g->n = n;
  g->dev.assign(ordinals, ordinals + n);
  g->m.assign((size_t)n, nullptr);
  g->own.assign((size_t)n, nullptr);
  g->s.assign((size_t)n, nullptr);
  g->done.assign((size_t)n, nullptr);
  free_exchange(g);
  auto bail = [&](int rc) {
    const std::string msg = pt_last_error();
    destroy(g);
    return pt_fail_internal(rc, msg);
  };
  for (int r = 0; r < n; ++r) {
    int rc = pt_create(g->dev[(size_t)r], &g->m[(size_t)r]);
    if (!rc) rc = pt_set_partition(g->m[(size_t)r], n, r);
    if (rc) return bail(rc);
    if (hipSetDevice(g->dev[(size_t)r]) != hipSuccess ||
        hipStreamCreateWithFlags(&g->own[(size_t)r], hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&g->done[(size_t)r], hipEventDisableTiming) != hipSuccess)
      return bail(pt_fail_internal(PT_ERR_HIP, "pt_create_multi: stream/event setup failed"));
    g->s[(size_t)r] = g->own[(size_t)r];
    rc = pt_set_stream(g->m[(size_t)r], g->s[(size_t)r]);
    if (rc) return bail(rc);
    // the members' kernels store into the first device's frame over xGMI
    if (g->dev[(size_t)r] != g->dev[0]) {
      int ok = 0;
      if (hipDeviceCanAccessPeer(&ok, g->dev[(size_t)r], g->dev[0]) != hipSuccess) ok = 0;
      if (ok) {
        const hipError_t e = hipDeviceEnablePeerAccess(g->dev[0], 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) ok = 0;
        (void)hipGetLastError();
      }
      if (!ok) g->peer_ok = g->peer_map_ok = false;
    }
  }
  if (hipSetDevice(g->dev[0]) != hipSuccess ||
      hipEventCreateWithFlags(&g->start, hipEventDisableTiming) != hipSuccess)
    return bail(pt_fail_internal(PT_ERR_HIP, "pt_create_multi: event setup failed"));
  g->job_rc.assign((size_t)n, PT_OK);
  g->job_err.assign((size_t)n, std::string());
  const char* th = getenv("PT_GROUP_THREADS");   // 0: enqueue every member on the caller's thread
  if (n >= 3 && !(th && th[0] == '0'))
    for (int r = 1; r < n; ++r) g->workers.emplace_back(worker_main, g, r);
  *out = g;
  return PT_OK;
}

int destroy(pt_group* g) {
  if (!g) return PT_OK;
  stop_workers(g);
  for (int r = 0; r < g->n; ++r)
    if (g->s[(size_t)r]) {
      (void)hipSetDevice(g->dev[(size_t)r]);
      (void)hipStreamSynchronize(g->s[(size_t)r]);
    }
  for (int r = 0; r < g->n; ++r)
    if (g->m[(size_t)r]) (void)pt_destroy(g->m[(size_t)r]);
  free_exchange(g);
  if (g->own_frame) gfree(g->dev[0], g->frame);
  for (int r = 0; r < g->n; ++r) {
    (void)hipSetDevice(g->dev[(size_t)r]);
    if (g->own[(size_t)r]) (void)hipStreamDestroy(g->own[(size_t)r]);
    if (g->done[(size_t)r]) (void)hipEventDestroy(g->done[(size_t)r]);
  }
  if (g->start) {
    (void)hipSetDevice(g->dev[0]);
    (void)hipEventDestroy(g->start);
  }
  delete g;
  return PT_OK;
}

int set_stream(pt_group* g, void* s) {
  G_RC(quiesce_all(g));
  g->s[0] = s ? (hipStream_t)s : g->own[0];
  return pt_set_stream(g->m[0], g->s[0]);
}

int synchronize(pt_group* g) { return quiesce_all(g); }

int upload_scene(pt_group* g, const float* vertices, size_t n_vertex_floats, const uint32_t* indices,
                 size_t n_indices, const pt_bvh_node* nodes, size_t n_nodes, const float* uvs, size_t n_uv_floats,
                 const uint32_t* mat_indices, size_t n_mat, uint32_t flags) {
  return each_parallel(g, [&](int r) {
    return pt_upload_scene(g->m[(size_t)r], vertices, n_vertex_floats, indices, n_indices, nodes, n_nodes, uvs,
                           n_uv_floats, mat_indices, n_mat, flags);
  });
}

int upload_lights(pt_group* g, const pt_area_light* lights, size_t n) {
  return each(g, [&](int r) { return pt_upload_lights(g->m[(size_t)r], lights, n); });
}

int set_camera(pt_group* g, const float ubo[16]) {
  return each(g, [&](int r) { return pt_set_camera(g->m[(size_t)r], ubo); });
}

int set_params(pt_group* g, const pt_params* p) {
  return each(g, [&](int r) { return pt_set_params(g->m[(size_t)r], p); });
}

int clear_accum(pt_group* g) {
  if (!g->frame) return pt_fail_internal(PT_ERR_INVALID, "no accumulation buffer");
  // every pixel +0 on the group's stream, after its members' last launches
  G_HIP(hipSetDevice(g->dev[0]));
  for (int r = 1; r < g->n; ++r) G_HIP(hipStreamWaitEvent(g->s[0], g->done[(size_t)r], 0));
  G_HIP(hipMemsetAsync(g->frame, 0, (size_t)g->W * g->H * 16, g->s[0]));
  for (int r = 0; r < g->n; ++r)   // the members that render into the frame itself see it cleared
    if (r == 0 || !g->staged) pt_note_accum_written(g->m[(size_t)r], true);
  if (g->staged)
    for (int r = 1; r < g->n; ++r) G_RC(pt_clear_accum(g->m[(size_t)r]));
  return PT_OK;
}

int resize_and_clear(pt_group* g, int w, int h) {
  if (w <= 0 || h <= 0 || (long long)w * h > (1ll << 31)) return pt_fail_internal(PT_ERR_INVALID, "bad resolution");
  if (!(g->own_frame && g->W == w && g->H == h)) {
    G_RC(quiesce_all(g));
    if (g->own_frame) gfree(g->dev[0], g->frame);
    g->frame = nullptr;
    g->own_frame = false;
    G_HIP(hipSetDevice(g->dev[0]));
    G_HIP(hipMalloc((void**)&g->frame, (size_t)w * h * 16));
    g->own_frame = true;
    g->W = w;
    g->H = h;
    G_RC(setup_frame(g, true, false));   // uninitialised until the clear below: no history to copy
  }
  return clear_accum(g);
}

int bind_accum(pt_group* g, void* ptr, int w, int h) {
  if (!ptr) return pt_fail_internal(PT_ERR_INVALID, "null argument");
  if (w <= 0 || h <= 0) return pt_fail_internal(PT_ERR_INVALID, "bad resolution");
  if (((uintptr_t)ptr) & 15) return pt_fail_internal(PT_ERR_INVALID, "accumulation buffer must be 16-B aligned");
  G_RC(quiesce_all(g));
  if (g->own_frame) gfree(g->dev[0], g->frame);
  g->frame = (float*)ptr;
  g->own_frame = false;
  g->W = w;
  g->H = h;
  return setup_frame(g);
}

void* accum_device_ptr(pt_group* g) { return g->frame; }

int read_accum(pt_group* g, float* rgba, size_t n) { return pt_read_accum(g->m[0], rgba, n); }

int render(pt_group* g, uint32_t first_batch, uint32_t n_batches) {
  if (!g->frame) return pt_fail_internal(PT_ERR_INVALID, "no accumulation buffer");
  if (g->check_pending) G_RC(check_exchange(g));
  // the members start after the group stream's earlier work (clear, readback)
  return run_members(g, first_batch, n_batches, g->staged, g->frame, g->pack_local, g->pack_root, g->pack_bytes,
                     true);
}

int progressive_camera(pt_group* g, const float ubo[16], int* reset) {
  if (!ubo) return pt_fail_internal(PT_ERR_INVALID, "null argument");
  const bool changed = !g->prog_has_cam || memcmp(ubo, g->prog_cam, sizeof g->prog_cam) != 0;
  if (changed) {
    memcpy(g->prog_cam, ubo, sizeof g->prog_cam);
    g->prog_has_cam = true;
    g->prog_batch = 0;
    G_RC(set_camera(g, ubo));
  }
  if (reset) *reset = changed ? 1 : 0;
  return PT_OK;
}

int progressive_advance(pt_group* g, uint32_t max_new, uint32_t limit, uint32_t* first, uint32_t* count) {
  if (!g->prog_has_cam) return pt_fail_internal(PT_ERR_INVALID, "no camera (pt_progressive_camera)");
  const uint32_t room = limit > g->prog_batch ? limit - g->prog_batch : 0u;
  const uint32_t k = max_new < room ? max_new : room;
  if (first) *first = g->prog_batch;
  if (count) *count = k;
  if (k == 0) return PT_OK;
  G_RC(render(g, g->prog_batch, k));
  g->prog_batch += k;
  return PT_OK;
}

// the first member's readback runs on the group's stream, which has waited
// for every member's tiles
int readback_begin(pt_group* g, int* ticket) { return pt_readback_begin(g->m[0], ticket); }
int readback_end(pt_group* g, int ticket, float* rgba, size_t n) { return pt_readback_end(g->m[0], ticket, rgba, n); }

int set_option(pt_group* g, int key, int value) {
  if (key == kOptGroupExchange) {
    if (value < 0 || value > 1) return pt_fail_internal(PT_ERR_INVALID, "PT_OPT_GROUP_EXCHANGE takes 0 or 1");
    if (value == g->exchange) return PT_OK;
    g->exchange = value;
    return g->frame ? setup_frame(g) : PT_OK;
  }
  if (key == kOptGroupCheck) {
    if (value < 0 || value > 3) return pt_fail_internal(PT_ERR_INVALID, "PT_OPT_GROUP_CHECK takes 0 to 3");
    g->check = value;
    if (value >= 2) {   // a fresh check on the next render (peer stores are tried again)
      g->peer_ok = g->peer_map_ok;
      g->check_passed = false;
      return g->frame ? setup_frame(g) : PT_OK;
    }
    if (value == 0) g->check_pending = false;
    return PT_OK;
  }
  G_RC(each(g, [&](int r) { return pt_set_option(g->m[(size_t)r], key, value); }));
  if (key == kOptCountTraced) g->count_traced = value != 0;
  if (key == kOptLaunchTiming) g->timing = value;
  return PT_OK;
}

int last_kernel(pt_group* g, int* kernel) { return pt_last_kernel(g->m[0], kernel); }

int set_stats_mode(pt_group* g, int enabled) {
  G_RC(each(g, [&](int r) { return pt_set_stats_mode(g->m[(size_t)r], enabled); }));
  g->stats_mode = enabled != 0;
  return PT_OK;
}

int get_stats(pt_group* g, pt_stats* out) {
  if (!out) return pt_fail_internal(PT_ERR_INVALID, "null argument");
  pt_stats sum{};
  for (int r = 0; r < g->n; ++r) {
    pt_stats s{};
    G_RC(pt_get_stats(g->m[(size_t)r], &s));
    sum.rays += s.rays;
    sum.nodes += s.nodes;
    sum.leaf_tests += s.leaf_tests;
    sum.samples += s.samples;
  }
  *out = sum;
  return PT_OK;
}

int reset_stats(pt_group* g) { return each(g, [&](int r) { return pt_reset_stats(g->m[(size_t)r]); }); }

int get_traced(pt_group* g, pt_traced* out) {
  if (!out) return pt_fail_internal(PT_ERR_INVALID, "null argument");
  pt_traced sum{};
  for (int r = 0; r < g->n; ++r) {
    pt_traced t{};
    G_RC(pt_get_traced(g->m[(size_t)r], &t));
    sum.closest_walks += t.closest_walks;
    sum.shadow_walks += t.shadow_walks;
    sum.nodes += t.nodes;
    sum.tri_tests += t.tri_tests;
    sum.primaries += t.primaries;
  }
  *out = sum;
  return PT_OK;
}

int wide_info(pt_group* g, int info[2]) { return pt_wide_info(g->m[0], info); }
int last_launch_ms(pt_group* g, float* ms) { return pt_last_launch_ms(g->m[0], ms); }
int launch_times_ms(pt_group* g, float* out, size_t max_n, size_t* n_out) {
  return pt_launch_times_ms(g->m[0], out, max_n, n_out);
}
int launch_span_ms(pt_group* g, float* ms, size_t* n_out) { return pt_launch_span_ms(g->m[0], ms, n_out); }
int reset_launch_times(pt_group* g) {
  return each(g, [&](int r) { return pt_reset_launch_times(g->m[(size_t)r]); });
}

int members(pt_group* g, int* n, int* devices, int max_devices, int* peer) {
  if (n) *n = g->n;
  if (devices)
    for (int r = 0; r < g->n && r < max_devices; ++r) devices[r] = g->dev[(size_t)r];
  if (peer) *peer = g->n > 1 && !(g->exchange == 1 || !g->peer_ok) ? 1 : 0;
  return PT_OK;
}

int check_info(pt_group* g, int* state, float* ms_peer, float* ms_staged) {
  if (state) *state = g->check_pending ? -2 : g->check_state;
  if (ms_peer) *ms_peer = g->check_ms[0];
  if (ms_staged) *ms_staged = g->check_ms[1];
  return PT_OK;
}

}  // namespace ptg
