// TEST INFRASTRUCTURE (tests/test_integration.py): compiles the C++ snippets
// of INTEGRATION.md §2 and §3 verbatim against include/pathtracer.h, links
// them with libptamd.so, and (on the GPU) runs them on box.obj, so the
// documented drop-in binding cannot drift from the header or the library.
//
// The snippets are written against the reference's host objects
// (VulkanRayTracer::initComputePipeline / mainLoop, VulkanRayTracer.cpp:64-865).
// The stand-ins below declare only what they touch, with the reference's
// member signatures: BVH::getVertices/getIndices/getNodes
// (BoundingVolumeHierarchy.h:8-27, BVHNode = two vec4), Light::getLights
// (Light.h:6-25, AreaLightData = four vec4), plus the camera fields mainLoop
// copies into the std140 UBO (:761-764).  The arrays are filled from the
// library's own scene layer (pt_scene_*), which restates the reference's OBJ
// load and BVH build byte for byte (tests/test_host.py, test_ref_tinyobj.py).
//
//   snippet_harness <mode> <scene.obj> <W> <H> <spp> <out.raw>
//   mode: dispatch     -- §2 setup, then §3's per-batch body for batches 0..spp-1
//         progressive  -- §2 setup, then §3's progressive loop body until done
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "pathtracer.h"

struct vec4 { float x, y, z, w; };
struct BVHNode { vec4 minBounds, maxBounds; };                  // BoundingVolumeHierarchy.h:8-13
static_assert(sizeof(BVHNode) == sizeof(pt_bvh_node), "BVHNode is layout-identical to pt_bvh_node");
class BVH {
 public:
  std::vector<float> vertices;
  std::vector<uint32_t> indices;
  std::vector<BVHNode> nodes;
  const std::vector<float>& getVertices() const { return vertices; }
  const std::vector<uint32_t>& getIndices() const { return indices; }
  const std::vector<BVHNode>& getNodes() const { return nodes; }
};
struct AreaLightData { vec4 position, normal, intensity, size; };   // Light.h:6-12
class Light {
 public:
  std::vector<AreaLightData> data;
  const std::vector<AreaLightData>& getLights() const { return data; }
};

static void check(int rc) {
  if (rc != PT_OK) {
    fprintf(stderr, "pt call failed (%d): %s\n", rc, pt_last_error());
    exit(1);
  }
}

int main(int argc, char** argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s dispatch|progressive scene.obj W H spp out.raw\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1];
  const int render_width = atoi(argv[3]), render_height = atoi(argv[4]), spp = atoi(argv[5]);
  // the reference's load + build (:64-94), through the library's scene layer
  pt_scene* sc = nullptr;
  check(pt_scene_load_obj(argv[2], &sc));
  check(pt_scene_build_bvh(sc, 0, 0));
  size_t nvf = 0, ni = 0, nn = 0, nuv = 0, nmat = 0;
  check(pt_scene_counts(sc, &nvf, &ni, &nn, &nuv, &nmat));
  BVH bvh;
  bvh.vertices.resize(nvf);
  bvh.indices.resize(ni);
  bvh.nodes.resize(nn);
  std::vector<float> objUVs(nuv);
  std::vector<uint32_t> matIndices(nmat);
  check(pt_scene_copy(sc, bvh.vertices.data(), bvh.indices.data(), reinterpret_cast<pt_bvh_node*>(bvh.nodes.data()),
                      objUVs.data(), matIndices.data()));
  pt_scene_free(sc);
  Light lights;   // VulkanRayTracer.cpp:149-162
  {
    const float pos[3] = {0.0f, 2.0f, 0.0f}, nrm[3] = {0.0f, -1.0f, 0.0f}, inten[3] = {10.0f, 10.0f, 10.0f},
                size[2] = {2.5f, 2.5f};
    pt_area_light l;
    check(pt_pack_light(pos, nrm, inten, size, &l));
    AreaLightData d;
    memcpy(&d, &l, sizeof d);
    lights.data.push_back(d);
  }

  // ---- INTEGRATION.md §2, verbatim ----
#include "snippet_init.inc"
  // ------------------------------------

  // mainLoop's camera state (Camera.cpp:4-10 defaults)
  float camera_ubo[16];
  check(pt_default_camera(camera_ubo));
  float cameraPosition[3], cameraDirection[3], cameraUp[3];
  memcpy(cameraPosition, camera_ubo, 12);
  memcpy(cameraDirection, camera_ubo + 4, 12);
  memcpy(cameraUp, camera_ubo + 8, 12);
  const float cameraFov = camera_ubo[12];
  std::vector<float> hostRGBA((size_t)render_width * render_height * 4);

  if (mode == "dispatch") {
    for (uint32_t sampleBatch = 0; sampleBatch < (uint32_t)spp; ++sampleBatch) {
      const bool cameraChanged = sampleBatch == 0;
      // ---- INTEGRATION.md §3 (per batch), verbatim ----
#include "snippet_loop.inc"
      // -------------------------------------------------
    }
  } else if (mode == "progressive") {
    float ubo[16] = {0};
    memcpy(&ubo[0], &cameraPosition, 12);
    memcpy(&ubo[4], &cameraDirection, 12);
    memcpy(&ubo[8], &cameraUp, 12);
    ubo[12] = cameraFov;
    int done = 0;
    for (int guard = 0; guard < 4096 && done < spp; ++guard) {
      // ---- INTEGRATION.md §3 (progressive loop), verbatim ----
#include "snippet_progressive.inc"
      // --------------------------------------------------------
      done += (int)count;
      if (count == 0) break;
    }
    check(pt_synchronize(m_pt));
    check(pt_read_accum(m_pt, hostRGBA.data(), hostRGBA.size()));
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  FILE* f = fopen(argv[6], "wb");
  if (!f || fwrite(hostRGBA.data(), sizeof(float), hostRGBA.size(), f) != hostRGBA.size()) return 1;
  fclose(f);
  check(pt_destroy(m_pt));
  return 0;
}
