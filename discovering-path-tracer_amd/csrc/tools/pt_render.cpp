// pt_render — headless C++ driver: the role VulkanRayTracer::initComputePipeline
// + mainLoop (src/Vulkan/VulkanRayTracer.cpp:41-865) play in the reference,
// minus the Qt window.  Loads an OBJ, builds the BVH, uploads, renders
// `spp` progressive 1-spp batches (or one fused launch) and writes a PFM.
//
//   pt_render scene.obj [-w 1920] [-h 1080] [-spp 8] [-depth 4] [-sss 3]
//             [-fused] [-o out.pfm] [-png out.png] [-device 0 | -devices 0,1,..]
//             [-cache scene.ptscene] [-progressive N [-chunk K] [-orbit-at B]]
//
// -progressive runs the reference's interactive loop (mainLoop, :717-865)
// headless: up to N batches (cap 1024, :719) in launches of K, a readback of
// every launch overlapped with the next one (double-buffered), and, with
// -orbit-at, a camera change after B batches that restarts at batch 0.
// -cache loads/saves the built scene (pt_scene_save) next to the OBJ.
// -devices renders on several GPUs from this one thread (pt_create_multi:
// each renders its screen tiles straight into the frame on the first one);
// every other call is unchanged.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <vector>

#include "pathtracer.h"

static int check(int rc, const char* what) {
  if (rc != PT_OK) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, pt_last_error());
    exit(1);
  }
  return rc;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s scene.obj [-w W] [-h H] [-spp N] [-depth D] [-sss S] [-fused] [-o out.pfm]\n", argv[0]);
    return 2;
  }
  std::string scene_path = argv[1], out_path;
  int W = 1024, H = 1024, spp = 8, device = 0;   // VulkanRayTracer.cpp:21-22
  pt_params params{4, 3};
  bool fused = false;
  int progressive = 0, chunk = 8, orbit_at = -1;
  std::string cache_path, png_path;
  std::vector<int> devices;   // -devices: a multi-device context
  for (int i = 2; i < argc; ++i) {
    auto next = [&](void) { return (i + 1 < argc) ? argv[++i] : (char*)"0"; };
    if (!strcmp(argv[i], "-w")) W = atoi(next());
    else if (!strcmp(argv[i], "-h")) H = atoi(next());
    else if (!strcmp(argv[i], "-spp")) spp = atoi(next());
    else if (!strcmp(argv[i], "-depth")) params.max_depth = atoi(next());
    else if (!strcmp(argv[i], "-sss")) params.sss_bounces = atoi(next());
    else if (!strcmp(argv[i], "-device")) device = atoi(next());
    else if (!strcmp(argv[i], "-devices")) {
      for (const char* p = next(); *p;) {
        devices.push_back(atoi(p));
        while (*p && *p != ',') ++p;
        if (*p == ',') ++p;
      }
    }
    else if (!strcmp(argv[i], "-fused")) fused = true;
    else if (!strcmp(argv[i], "-o")) out_path = next();
    else if (!strcmp(argv[i], "-cache")) cache_path = next();
    else if (!strcmp(argv[i], "-png")) png_path = next();
    else if (!strcmp(argv[i], "-progressive")) progressive = atoi(next());
    else if (!strcmp(argv[i], "-chunk")) chunk = atoi(next());
    else if (!strcmp(argv[i], "-orbit-at")) orbit_at = atoi(next());
  }
  pt_scene* scene = nullptr;
  auto t0 = std::chrono::steady_clock::now();
  bool cached = false;
  if (!cache_path.empty() && pt_scene_load_cache(cache_path.c_str(), &scene) == PT_OK) {
    cached = true;
  } else {
    check(pt_scene_load_obj(scene_path.c_str(), &scene), "load obj");
    check(pt_scene_build_bvh(scene, 0, 0), "build bvh");
    if (!cache_path.empty()) check(pt_scene_save(scene, cache_path.c_str()), "save cache");
  }
  auto t1 = std::chrono::steady_clock::now();
  size_t nvf, ni, nn;
  pt_scene_counts(scene, &nvf, &ni, &nn, nullptr, nullptr);
  printf("scene: %zu vertices, %zu triangles, %zu nodes, %s %.3f s\n", nvf / 3, ni / 3, nn,
         cached ? "cache load" : "OBJ parse + BVH build", std::chrono::duration<double>(t1 - t0).count());

  pt_context* ctx = nullptr;
  if (devices.empty()) {
    check(pt_create(device, &ctx), "create");
  } else {
    check(pt_create_multi(devices.data(), (int)devices.size(), &ctx), "create_multi");
    int peer = 0;
    check(pt_group_info(ctx, nullptr, nullptr, 0, &peer), "group_info");
    printf("devices: %zu (%s)\n", devices.size(), peer ? "peer stores into the first device's frame" : "packed tile copies");
  }
  check(pt_scene_upload(ctx, scene), "upload scene");
  const float pos[3] = {0.0f, 2.0f, 0.0f}, nrm[3] = {0.0f, -1.0f, 0.0f}, inten[3] = {10.0f, 10.0f, 10.0f},
              size[2] = {2.5f, 2.5f};   // VulkanRayTracer.cpp:149-162
  pt_area_light light;
  pt_pack_light(pos, nrm, inten, size, &light);
  check(pt_upload_lights(ctx, &light, 1), "upload lights");
  float ubo[16];
  pt_default_camera(ubo);
  check(pt_set_camera(ctx, ubo), "camera");
  check(pt_set_params(ctx, &params), "params");
  check(pt_resize_and_clear(ctx, W, H), "resize");
  check(pt_synchronize(ctx), "sync");
  if (progressive > 0) {
    // orbit: the default camera rotated 30 degrees about +y around the origin
    float orbit[16];
    memcpy(orbit, ubo, sizeof orbit);
    const float c30 = 0.8660254f, s30 = 0.5f;
    orbit[0] = ubo[0] * c30 + ubo[2] * s30;
    orbit[2] = -ubo[0] * s30 + ubo[2] * c30;
    orbit[4] = ubo[4] * c30 + ubo[6] * s30;
    orbit[6] = -ubo[4] * s30 + ubo[6] * c30;
    std::vector<float> frame((size_t)W * H * 4);
    int pending = 0, frames = 0, done = 0;
    auto p0 = std::chrono::steady_clock::now();
    for (;;) {
      int reset = 0;
      check(pt_progressive_camera(ctx, (orbit_at >= 0 && done >= orbit_at) ? orbit : ubo, &reset), "camera");
      uint32_t first = 0, count = 0;
      const uint32_t want = (uint32_t)std::min(chunk, progressive - done);
      check(pt_progressive_advance(ctx, want, 1024, &first, &count), "advance");
      if (count == 0) break;
      done += (int)count;
      int t = 0;
      check(pt_readback_begin(ctx, &t), "readback");
      if (pending) {   // the previous launch's image, copied while this one renders
        check(pt_readback_end(ctx, pending, frame.data(), frame.size()), "readback end");
        ++frames;
      }
      pending = t;
      if (reset) printf("camera changed: restarting at batch %u\n", first);
      if (done >= progressive) break;
    }
    if (pending) {
      check(pt_readback_end(ctx, pending, frame.data(), frame.size()), "readback end");
      ++frames;
    }
    auto p1 = std::chrono::steady_clock::now();
    printf("progressive: %d batches, %d frames read back, %.3f ms\n", done, frames,
           std::chrono::duration<double, std::milli>(p1 - p0).count());
  }
  auto r0 = std::chrono::steady_clock::now();
  if (progressive > 0) {
    // the accumulation buffer already holds the progressive result
  } else if (fused) {
    check(pt_render(ctx, 0, (uint32_t)spp), "render");
  } else {
    for (int b = 0; b < spp; ++b) check(pt_dispatch(ctx, (uint32_t)b), "dispatch");   // mainLoop, 1 spp per batch
  }
  check(pt_synchronize(ctx), "sync");
  auto r1 = std::chrono::steady_clock::now();
  if (progressive == 0)
    printf("rendered %dx%d x %d spp in %.3f ms\n", W, H, spp, std::chrono::duration<double, std::milli>(r1 - r0).count());
  if (!out_path.empty() || !png_path.empty()) {
    std::vector<float> rgba((size_t)W * H * 4);
    check(pt_read_accum(ctx, rgba.data(), rgba.size()), "read");
    if (!out_path.empty()) check(pt_write_image(out_path.c_str(), rgba.data(), W, H, PT_IMAGE_PFM), "write pfm");
    if (!png_path.empty()) check(pt_write_image(png_path.c_str(), rgba.data(), W, H, PT_IMAGE_PNG), "write png");
  }
  pt_destroy(ctx);
  pt_scene_free(scene);
  return 0;
}
