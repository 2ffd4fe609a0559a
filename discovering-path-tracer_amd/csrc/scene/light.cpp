#include "light.h"

#include <math.h>

namespace pt {

// Light.cpp:16-33 packData: normal = glm::normalize(n) = n * (1/sqrt(dot(n,n))).
Light::Light(const std::vector<vec3f>& positions, const std::vector<vec3f>& normals,
             const std::vector<vec3f>& intensities, const std::vector<vec2f>& sizes) {
  lights.reserve(positions.size());
  for (size_t i = 0; i < positions.size(); ++i) {
    AreaLightData d{};
    const vec3f& n = normals[i];
    const float inv = 1.0f / sqrtf(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
    for (int c = 0; c < 3; ++c) {
      d.position[c] = positions[i][c];
      d.normal[c] = n[c] * inv;
      d.intensity[c] = intensities[i][c];
    }
    d.size[0] = sizes[i][0];
    d.size[1] = sizes[i][1];
    lights.push_back(d);
  }
}

Light Light::referenceDefault() {
  return Light({{0.0f, 2.0f, 0.0f}}, {{0.0f, -1.0f, 0.0f}}, {{10.0f, 10.0f, 10.0f}}, {{2.5f, 2.5f}});
}

}  // namespace pt
