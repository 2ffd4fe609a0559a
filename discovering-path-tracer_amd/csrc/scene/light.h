// Area lights — mirrors src/Light.h:6-30 / src/Light.cpp:3-33.
#pragma once
#include <array>
#include <vector>

namespace pt {

// Light.h:6-12 — 64 B, the std430 element of the shader's AreaLight SSBO
// (raytrace_comp.comp:17-23).
struct AreaLightData {
  float position[4];   // xyz = centre
  float normal[4];     // xyz = normalized orientation
  float intensity[4];  // xyz = RGB radiance
  float size[4];       // xy = width, height
};
static_assert(sizeof(AreaLightData) == 64, "AreaLightData is 64 B");

using vec3f = std::array<float, 3>;
using vec2f = std::array<float, 2>;

class Light {
 public:
  Light(const std::vector<vec3f>& positions, const std::vector<vec3f>& normals,
        const std::vector<vec3f>& intensities, const std::vector<vec2f>& sizes);
  Light() = default;
  const std::vector<AreaLightData>& getLights() const { return lights; }

  // The scene's one light (VulkanRayTracer.cpp:149-162).
  static Light referenceDefault();

 private:
  std::vector<AreaLightData> lights;
};

}  // namespace pt
