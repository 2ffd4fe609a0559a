#include "camera.h"

#include <math.h>
#include <string.h>

namespace pt {
namespace {
using q4 = std::array<float, 4>;
using v3 = std::array<float, 3>;

// QQuaternion::fromAxisAndAngle / operator* / rotatedVector, in float.
q4 axis_angle(v3 a, float deg) {
  const float h = deg * 0.5f * 3.14159265358979f / 180.0f;
  const float s = sinf(h);
  return {cosf(h), a[0] * s, a[1] * s, a[2] * s};
}
q4 qmul(q4 p, q4 q) {
  return {p[0] * q[0] - p[1] * q[1] - p[2] * q[2] - p[3] * q[3],
          p[0] * q[1] + p[1] * q[0] + p[2] * q[3] - p[3] * q[2],
          p[0] * q[2] + p[2] * q[0] + p[3] * q[1] - p[1] * q[3],
          p[0] * q[3] + p[3] * q[0] + p[1] * q[2] - p[2] * q[1]};
}
v3 qrot(q4 q, v3 v) {
  const q4 p{0.0f, v[0], v[1], v[2]};
  const q4 c{q[0], -q[1], -q[2], -q[3]};
  const q4 r = qmul(qmul(q, p), c);
  return {r[1], r[2], r[3]};
}
}  // namespace

Camera::Camera() { refresh(); }

void Camera::refresh() { position_ = qrot(rotation_, {0.0f, 0.0f, radius_}); }

std::array<float, 3> Camera::getDirection() const {
  // (target - position).normalized() with target = origin (Camera.cpp:84-89):
  // 0.0f - p keeps +0 where p is +/-0, as the reference's subtraction does.
  const double x = 0.0f - position_[0], y = 0.0f - position_[1], z = 0.0f - position_[2];
  const double len = sqrt(x * x + y * y + z * z);
  if (len == 0.0) return {0.0f, 0.0f, 0.0f};
  return {(float)(x / len), (float)(y / len), (float)(z / len)};
}

std::array<float, 3> Camera::getUp() const {
  if (has_pose_) return up_override_;
  return qrot(rotation_, {0.0f, 1.0f, 0.0f});
}

void Camera::orbit(float yaw_deg, float pitch_deg) {
  yaw_ = yaw_deg;
  pitch_ = pitch_deg;
  rotation_ = qmul(axis_angle({0, 1, 0}, yaw_), axis_angle({1, 0, 0}, pitch_));
  has_pose_ = false;
  refresh();
}

void Camera::zoom(float factor) {
  radius_ *= factor;
  has_pose_ = false;
  refresh();
}

void Camera::setPose(const std::array<float, 3>& pos, const std::array<float, 3>& up, float fov) {
  position_ = pos;
  up_override_ = up;
  fov_ = fov;
  has_pose_ = true;
}

void Camera::toUBO(float out[16]) const {
  memset(out, 0, 16 * sizeof(float));
  const v3 d = getDirection(), u = getUp();
  for (int c = 0; c < 3; ++c) {
    out[c] = position_[c];
    out[4 + c] = d[c];
    out[8 + c] = u[c];
  }
  out[12] = fov_;
}

}  // namespace pt
