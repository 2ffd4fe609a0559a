// Orbit camera — the getters the kernel consumes, mirroring src/Camera.h:10-38
// and src/Camera.cpp.  The Qt mouse/zoom handlers are out of scope; the same
// state changes are exposed as orbit()/zoom() so a headless caller can drive
// the camera and trigger the accumulation reset (VulkanRayTracer.cpp:739-754).
#pragma once
#include <array>

namespace pt {

class Camera {
 public:
  Camera();                                   // Camera.cpp:4-10: radius 5, fov 60
  std::array<float, 3> getPosition() const { return position_; }
  std::array<float, 3> getDirection() const;  // Camera.cpp:84-89 normalize(target - pos)
  std::array<float, 3> getUp() const;         // Camera.cpp:91-95 rotation * (0,1,0)
  float getFov() const { return fov_; }

  void orbit(float yaw_deg, float pitch_deg); // Camera.cpp:37-64 (absolute angles)
  void zoom(float factor);                    // Camera.cpp:66-77
  void setPose(const std::array<float, 3>& pos, const std::array<float, 3>& up, float fov);

  // std140 CameraBuffer UBO (raytrace_comp.comp:67-73): pos@0 dir@16 up@32 fov@48.
  void toUBO(float out16[16]) const;

 private:
  void refresh();
  std::array<float, 3> position_{};
  std::array<float, 4> rotation_{1.0f, 0.0f, 0.0f, 0.0f};   // quaternion w,x,y,z
  std::array<float, 3> up_override_{};
  bool has_pose_ = false;
  float fov_ = 60.0f;
  float radius_ = 5.0f;
  float yaw_ = 0.0f, pitch_ = 0.0f;
};

}  // namespace pt
