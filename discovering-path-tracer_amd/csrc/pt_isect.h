// pt_isect.h — the reference's two intersection tests, shared by the device
// kernels (pt_device.hip) and host-side checks of the culled wide walk
// (wide_walk.h, tests/wide_check.cpp).  Same float ops, same order as the
// shader; compiled with -ffp-contract=off like everything in pt_math.h.
#pragma once
#include "pt_math.h"

namespace ptd {
using namespace ptm;

// intersectAABB (raytrace_comp.comp:102-112) with invDir hoisted (same value
// every node).
PT_FN bool slab(v3 o, v3 inv, float4 a, float4 b) {
  const float t0x = (a.x - o.x) * inv.x, t0y = (a.y - o.y) * inv.y, t0z = (a.z - o.z) * inv.z;
  const float t1x = (b.x - o.x) * inv.x, t1y = (b.y - o.y) * inv.y, t1z = (b.z - o.z) * inv.z;
  const float tmin = fmax_(fmax_(fmin_(t0x, t1x), fmin_(t0y, t1y)), fmin_(t0z, t1z));
  const float tmax = fmin_(fmin_(fmax_(t0x, t1x), fmax_(t0y, t1y)), fmax_(t0z, t1z));
  return tmin <= tmax && tmax >= 0.0f;
}

// intersectTriangle (:114-157), edges precomputed; UV tail is dead code.
// Record {v0.xyz, e1.x} {e1.yz, e2.xy} {e2.z, n.xyz} (pt_device.h tris).
PT_FN bool tri_test(v3 o, v3 d, float4 A, float4 B, float4 C, float* tout) {
  const float EPS = 0.000001f;
  const v3 v0 = mk(A.x, A.y, A.z);
  const v3 e1 = mk(A.w, B.x, B.y);
  const v3 e2 = mk(B.z, B.w, C.x);
  const v3 p = cross(d, e2);
  const float det = dot(e1, p);
  if (fabs_(det) < EPS) return false;
  const float inv = rcp_(det);
  const v3 s = sub(o, v0);
  const float u = inv * dot(s, p);
  if (u < 0.0f || u > 1.0f) return false;
  const v3 q = cross(s, e1);
  const float v = inv * dot(d, q);
  if (v < 0.0f || u + v > 1.0f) return false;
  const float t = inv * dot(e2, q);
  if (t <= EPS) return false;
  *tout = t;
  return true;
}

}  // namespace ptd
