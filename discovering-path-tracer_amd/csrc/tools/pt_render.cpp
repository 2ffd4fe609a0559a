// pt_render — headless C++ driver: the role VulkanRayTracer::initComputePipeline
// + mainLoop (src/Vulkan/VulkanRayTracer.cpp:41-865) play in the reference,
// minus the Qt window.  Loads an OBJ, builds the BVH, uploads, renders
// `spp` progressive 1-spp batches (or one fused launch) and writes a PFM.
//
//   pt_render scene.obj [-w 1920] [-h 1080] [-spp 8] [-depth 4] [-sss 3]
//             [-fused] [-o out.pfm] [-device 0]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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
  for (int i = 2; i < argc; ++i) {
    auto next = [&](void) { return (i + 1 < argc) ? argv[++i] : (char*)"0"; };
    if (!strcmp(argv[i], "-w")) W = atoi(next());
    else if (!strcmp(argv[i], "-h")) H = atoi(next());
    else if (!strcmp(argv[i], "-spp")) spp = atoi(next());
    else if (!strcmp(argv[i], "-depth")) params.max_depth = atoi(next());
    else if (!strcmp(argv[i], "-sss")) params.sss_bounces = atoi(next());
    else if (!strcmp(argv[i], "-device")) device = atoi(next());
    else if (!strcmp(argv[i], "-fused")) fused = true;
    else if (!strcmp(argv[i], "-o")) out_path = next();
  }
  pt_scene* scene = nullptr;
  check(pt_scene_load_obj(scene_path.c_str(), &scene), "load obj");
  auto t0 = std::chrono::steady_clock::now();
  check(pt_scene_build_bvh(scene, 0, 0), "build bvh");
  auto t1 = std::chrono::steady_clock::now();
  size_t nvf, ni, nn;
  pt_scene_counts(scene, &nvf, &ni, &nn, nullptr, nullptr);
  printf("scene: %zu vertices, %zu triangles, %zu nodes, BVH build %.3f s\n", nvf / 3, ni / 3, nn,
         std::chrono::duration<double>(t1 - t0).count());

  pt_context* ctx = nullptr;
  check(pt_create(device, &ctx), "create");
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
  auto r0 = std::chrono::steady_clock::now();
  if (fused) {
    check(pt_render(ctx, 0, (uint32_t)spp), "render");
  } else {
    for (int b = 0; b < spp; ++b) check(pt_dispatch(ctx, (uint32_t)b), "dispatch");   // mainLoop, 1 spp per batch
  }
  check(pt_synchronize(ctx), "sync");
  auto r1 = std::chrono::steady_clock::now();
  printf("rendered %dx%d x %d spp in %.3f ms\n", W, H, spp, std::chrono::duration<double, std::milli>(r1 - r0).count());
  if (!out_path.empty()) {
    std::vector<float> rgba((size_t)W * H * 4);
    check(pt_read_accum(ctx, rgba.data(), rgba.size()), "read");
    FILE* f = fopen(out_path.c_str(), "wb");
    if (!f) { perror("fopen"); return 1; }
    fprintf(f, "PF\n%d %d\n-1.0\n", W, H);   // rows bottom-to-top = row 0 first
    std::vector<float> rgb((size_t)W * 3);
    for (int y = 0; y < H; ++y) {
      for (int x = 0; x < W; ++x)
        for (int c = 0; c < 3; ++c) rgb[(size_t)x * 3 + c] = rgba[((size_t)y * W + x) * 4 + c];
      fwrite(rgb.data(), 4, rgb.size(), f);
    }
    fclose(f);
  }
  pt_destroy(ctx);
  pt_scene_free(scene);
  return 0;
}
