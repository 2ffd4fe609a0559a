// oracle/pt_oracle.cpp — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
//
// A scalar CPU restatement of the reference hot path, used only as the parity
// checker (tests/, __graft_entry__.smoke()) and as the CPU baseline leg of
// bench.py.  Nothing under discovering-path-tracer_amd/ links or calls it.
//
// What it restates (citations are path:line in the reference tree):
//   * OBJ ingest with tinyobjloader v2.0.0's number parser and triangulation
//     (external/tiny_obj_loader.h:897-1028, 1509-1612, ear clipping 1740-1955);
//   * the median-split BVH builder (src/BoundingVolumeHierarchy.cpp:5-117),
//     with glm's min/max/division semantics spelt out (glm is an un-vendored,
//     unpinned submodule: external/glm is empty);
//   * the compute shader src/shaders/raytrace_comp.comp:90-470, op for op,
//     including its exhaustive DFS traversal with an explicit stack, the RNG
//     re-seed quirk and the running-mean accumulation.  Instrumented with the
//     per-ray counters the roofline uses (traceRay calls, nodes visited,
//     leaf triangle tests).
//
// PARITY STATUS: the reference has no tests, fixtures or golden images
//  and its kernel is GLSL for Vulkan, which cannot run in this
// pipeline (no Vulkan ICD, no glslang, MI355X is not a Vulkan target), and its
// C++ builder needs glm/Qt headers the image lacks.  This oracle is therefore
// pinned only by (a) the box.obj BVH dump recorded in SURVEY.md §8c
// (tests/golden/box_bvh.json) and (b) its own known-answer tests; the shader
// restatement itself is "parity unpinned" against a running reference.
//
// Compile: g++ -O2 -ffp-contract=off -fno-fast-math (oracle/Makefile).
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <float.h>
#include <math.h>
#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "glsl_math.h"

namespace {

struct vec3 { float x, y, z; };
static inline vec3 V(float x, float y, float z) { return vec3{x, y, z}; }
static inline vec3 operator+(vec3 a, vec3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline vec3 operator-(vec3 a, vec3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline vec3 operator*(vec3 a, vec3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline vec3 operator*(vec3 a, float s) { return V(a.x * s, a.y * s, a.z * s); }
static inline vec3 operator-(vec3 a) { return V(-a.x, -a.y, -a.z); }
static inline float dot(vec3 a, vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline vec3 cross(vec3 a, vec3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline float length(vec3 a) { return gm_sqrt(dot(a, a)); }
static inline vec3 normalize(vec3 a) { return a * (1.0f / gm_sqrt(dot(a, a))); }

// ------------------------------------------------------------------------
// OBJ ingest (tinyobjloader v2.0.0 rules)
// ------------------------------------------------------------------------

// tiny_obj_loader.h:897-1028 tryParseDouble: the mantissa is accumulated in
// double with a 0.1^k table, the decimal exponent applied as
// ldexp(m * 5^e, e); parseReal (:1030-1038) then casts to float.
static bool obj_parse_double(const char* s, const char* e, double* out) {
  if (s >= e) return false;
  double mant = 0.0;
  int exponent = 0;
  char sign = '+', esign = '+';
  const char* c = s;
  int read = 0;
  bool lead_dot = false;
  if (*c == '+' || *c == '-') {
    sign = *c++;
    if (c != e && *c == '.') lead_dot = true;
  } else if (*c >= '0' && *c <= '9') {
  } else if (*c == '.') {
    lead_dot = true;
  } else {
    return false;
  }
  bool more = (c != e);
  if (!lead_dot) {
    while (more && *c >= '0' && *c <= '9') {
      mant *= 10;
      mant += (int)(*c - '0');
      ++c; ++read;
      more = (c != e);
    }
    if (read == 0) return false;
  }
  if (!more) goto assemble;
  if (*c == '.') {
    ++c;
    read = 1;
    more = (c != e);
    static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
    while (more && *c >= '0' && *c <= '9') {
      mant += (int)(*c - '0') * (read < 8 ? lut[read] : pow(10.0, -read));
      ++read; ++c;
      more = (c != e);
    }
  } else if (*c == 'e' || *c == 'E') {
  } else {
    goto assemble;
  }
  if (!more) goto assemble;
  if (*c == 'e' || *c == 'E') {
    ++c;
    more = (c != e);
    if (more && (*c == '+' || *c == '-')) {
      esign = *c++;
    } else if (*c >= '0' && *c <= '9') {
    } else {
      return false;
    }
    read = 0;
    more = (c != e);
    while (more && *c >= '0' && *c <= '9') {
      if (exponent > 2147483647 / 10) return false;
      exponent = exponent * 10 + (int)(*c - '0');
      ++c; ++read;
      more = (c != e);
    }
    exponent *= (esign == '+' ? 1 : -1);
    if (read == 0) return false;
  }
assemble:
  *out = (sign == '+' ? 1 : -1) * (exponent ? ldexp(mant * pow(5.0, exponent), exponent) : mant);
  return true;
}

static float obj_real(const char** tok) {
  *tok += strspn(*tok, " \t");
  const char* end = *tok + strcspn(*tok, " \t\r");
  double v = 0.0;
  obj_parse_double(*tok, end, &v);
  *tok = end;
  return (float)v;
}

struct ObjOut {
  std::vector<float> v, vt;
  std::vector<uint32_t> idx, mat;
};

// Face corner "v", "v/vt", "v//vn", "v/vt/vn"; negative = relative
// (tiny_obj_loader.h fixIndex / parseTriple).
static bool obj_corner(const char** tok, int nv, int* vi) {
  const char* c = *tok;
  char* endp;
  long i = strtol(c, &endp, 10);
  if (endp == c) return false;
  if (i > 0) *vi = (int)(i - 1);
  else if (i < 0) *vi = nv + (int)i;
  else return false;
  c = endp;
  while (*c && *c != ' ' && *c != '\t' && *c != '\r' && *c != '\n') ++c;
  *tok = c;
  return true;
}

// tinyobj built-in ear clipping, faces of 5+ corners
// (external/tiny_obj_loader.h:1740-1955; pnpoly :1438-1450).  Restated loop
// for loop: axis pair from the first non-degenerate corner, ears cut at the
// guess vertex unless reflex (cross*area < 0) or containing another vertex.
static int oracle_pnpoly3(const float* vx, const float* vy, float tx, float ty) {
  int c = 0;
  for (int i = 0, j = 2; i < 3; j = i++)
    if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
  return c;
}

static void obj_earclip(const std::vector<int>& f, const std::vector<float>& v, std::vector<uint32_t>* idx,
                        std::vector<uint32_t>* mat) {
  size_t n = f.size();
  size_t axes[2] = {1, 2};
  for (size_t k = 0; k < n; ++k) {
    size_t i0 = f[k % n], i1 = f[(k + 1) % n], i2 = f[(k + 2) % n];
    float e0x = v[i1 * 3 + 0] - v[i0 * 3 + 0], e0y = v[i1 * 3 + 1] - v[i0 * 3 + 1], e0z = v[i1 * 3 + 2] - v[i0 * 3 + 2];
    float e1x = v[i2 * 3 + 0] - v[i1 * 3 + 0], e1y = v[i2 * 3 + 1] - v[i1 * 3 + 1], e1z = v[i2 * 3 + 2] - v[i1 * 3 + 2];
    float cx = fabsf(e0y * e1z - e0z * e1y), cy = fabsf(e0z * e1x - e0x * e1z), cz = fabsf(e0x * e1y - e0y * e1x);
    const float eps = FLT_EPSILON;
    if (cx > eps || cy > eps || cz > eps) {
      if (cx > cy && cx > cz) {
      } else {
        axes[0] = 0;
        if (cz > cx && cz > cy) axes[1] = 1;
      }
      break;
    }
  }
  std::vector<int> rem(f);
  size_t guess = 0, iters = n, prev_n = n;
  int ind[3];
  float vx[3], vy[3];
  while (rem.size() > 3 && iters > 0) {
    size_t np = rem.size();
    if (guess >= np) guess -= np;
    if (prev_n != np) { prev_n = np; iters = np; } else { iters--; }
    for (int k = 0; k < 3; ++k) {
      ind[k] = rem[(guess + k) % np];
      vx[k] = v[(size_t)ind[k] * 3 + axes[0]];
      vy[k] = v[(size_t)ind[k] * 3 + axes[1]];
    }
    float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
    float cross = e0x * e1y - e0y * e1x;
    float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
    if (cross * area < 0.0f) { guess += 1; continue; }
    bool overlap = false;
    for (size_t ov = 3; ov < np; ++ov) {
      size_t id = (guess + ov) % np;
      size_t ovi = (size_t)rem[id];
      if (oracle_pnpoly3(vx, vy, v[ovi * 3 + axes[0]], v[ovi * 3 + axes[1]])) { overlap = true; break; }
    }
    if (overlap) { guess += 1; continue; }
    for (int k = 0; k < 3; ++k) idx->push_back((uint32_t)ind[k]);
    mat->push_back(0);
    size_t r = (guess + 1) % np;
    while (r + 1 < np) { rem[r] = rem[r + 1]; r += 1; }
    rem.pop_back();
  }
  if (rem.size() == 3) {
    for (int k = 0; k < 3; ++k) idx->push_back((uint32_t)rem[k]);
    mat->push_back(0);
  }
}

static int obj_parse(const char* text, size_t len, ObjOut* out) {
  std::string buf(text, len);
  size_t pos = 0;
  while (pos < buf.size()) {
    size_t nl = buf.find('\n', pos);
    if (nl == std::string::npos) nl = buf.size();
    std::string line = buf.substr(pos, nl - pos);
    pos = nl + 1;
    const char* t = line.c_str();
    t += strspn(t, " \t");
    if (t[0] == 'v' && (t[1] == ' ' || t[1] == '\t')) {
      t += 2;
      float x = obj_real(&t), y = obj_real(&t), z = obj_real(&t);
      out->v.push_back(x); out->v.push_back(y); out->v.push_back(z);
    } else if (t[0] == 'v' && t[1] == 't' && (t[2] == ' ' || t[2] == '\t')) {
      t += 3;
      float u = obj_real(&t), w = obj_real(&t);
      out->vt.push_back(u); out->vt.push_back(w);
    } else if (t[0] == 'f' && (t[1] == ' ' || t[1] == '\t')) {
      t += 2;
      int nv = (int)(out->v.size() / 3);
      std::vector<int> f;
      while (true) {
        t += strspn(t, " \t");
        if (*t == 0 || *t == '\r' || *t == '\n') break;
        int vi;
        if (!obj_corner(&t, nv, &vi)) return -2;
        f.push_back(vi);
      }
      if (f.size() < 3) continue;                              // :1500-1506
      if (f.size() == 3) {
        for (int k = 0; k < 3; ++k) out->idx.push_back((uint32_t)f[k]);
        out->mat.push_back(0);
      } else if (f.size() == 4) {                              // :1509-1604
        const float* v = out->v.data();
        size_t i0 = f[0], i1 = f[1], i2 = f[2], i3 = f[3];
        float e02x = v[i2 * 3 + 0] - v[i0 * 3 + 0];
        float e02y = v[i2 * 3 + 1] - v[i0 * 3 + 1];
        float e02z = v[i2 * 3 + 2] - v[i0 * 3 + 2];
        float e13x = v[i3 * 3 + 0] - v[i1 * 3 + 0];
        float e13y = v[i3 * 3 + 1] - v[i1 * 3 + 1];
        float e13z = v[i3 * 3 + 2] - v[i1 * 3 + 2];
        float s02 = e02x * e02x + e02y * e02y + e02z * e02z;
        float s13 = e13x * e13x + e13y * e13y + e13z * e13z;
        uint32_t a[6];
        if (s02 < s13) { uint32_t t6[6] = {(uint32_t)i0, (uint32_t)i1, (uint32_t)i2, (uint32_t)i0, (uint32_t)i2, (uint32_t)i3}; memcpy(a, t6, sizeof a); }
        else { uint32_t t6[6] = {(uint32_t)i0, (uint32_t)i1, (uint32_t)i3, (uint32_t)i1, (uint32_t)i2, (uint32_t)i3}; memcpy(a, t6, sizeof a); }
        for (int k = 0; k < 6; ++k) out->idx.push_back(a[k]);
        out->mat.push_back(0); out->mat.push_back(0);
      } else {
        obj_earclip(f, out->v, &out->idx, &out->mat);   // :1740-1955
      }
    }
  }
  return 0;
}

// ------------------------------------------------------------------------
// BVH builder — src/BoundingVolumeHierarchy.cpp
// ------------------------------------------------------------------------
// glm::min(x,y) = (y < x) ? y : x ; glm::max(x,y) = (x < y) ? y : x
static inline float glm_min(float x, float y) { return (y < x) ? y : x; }
static inline float glm_max(float x, float y) { return (x < y) ? y : x; }
static inline vec3 vmin(vec3 a, vec3 b) { return V(glm_min(a.x, b.x), glm_min(a.y, b.y), glm_min(a.z, b.z)); }
static inline vec3 vmax(vec3 a, vec3 b) { return V(glm_max(a.x, b.x), glm_max(a.y, b.y), glm_max(a.z, b.z)); }

struct OracleBVH {
  const float* verts;
  std::vector<uint32_t> indices;
  float* nodes;                 // 8 floats per node: min.xyzw, max.xyzw
  vec3 vertex(uint32_t i) const {           // :113-117
    uint32_t b = indices[i] * 3;
    return V(verts[b], verts[b + 1], verts[b + 2]);
  }
  vec3 centroid(uint32_t t) const {         // :102-111
    uint32_t i = t * 3;
    vec3 a = vertex(i), b = vertex(i + 1), c = vertex(i + 2);
    vec3 s = (a + b) + c;
    return V(s.x / 3.0f, s.y / 3.0f, s.z / 3.0f);
  }
  void bounds(uint32_t s, uint32_t e, vec3* mn, vec3* mx) const {   // :84-100
    *mn = V(FLT_MAX, FLT_MAX, FLT_MAX);
    *mx = V(-FLT_MAX, -FLT_MAX, -FLT_MAX);
    for (uint32_t t = s; t < e; ++t) {
      uint32_t i = t * 3;
      vec3 a = vertex(i), b = vertex(i + 1), c = vertex(i + 2);
      *mn = vmin(*mn, vmin(a, vmin(b, c)));
      *mx = vmax(*mx, vmax(a, vmax(b, c)));
    }
  }
  void build(uint32_t s, uint32_t e, uint32_t* next) {   // :25-82
    uint32_t cur = (*next)++;
    vec3 mn, mx;
    bounds(s, e, &mn, &mx);
    float node[8] = {mn.x, mn.y, mn.z, 0.0f, mx.x, mx.y, mx.z, 0.0f};
    uint32_t cnt = e - s;
    if (cnt == 1) {
      node[3] = -1.0f;
      node[7] = (float)s;
    } else {
      std::vector<std::pair<uint32_t, vec3>> tc;
      tc.reserve(cnt);
      for (uint32_t t = s; t < e; ++t) tc.emplace_back(t, centroid(t));
      vec3 size = mx - mn;
      int axis = (size.x > size.y) ? ((size.x > size.z) ? 0 : 2) : ((size.y > size.z) ? 1 : 2);
      std::sort(tc.begin(), tc.end(), [axis](const std::pair<uint32_t, vec3>& a, const std::pair<uint32_t, vec3>& b) {
        const float ka = axis == 0 ? a.second.x : axis == 1 ? a.second.y : a.second.z;
        const float kb = axis == 0 ? b.second.x : axis == 1 ? b.second.y : b.second.z;
        return ka < kb;
      });
      std::vector<uint32_t> tmp(cnt * 3);
      for (uint32_t i = 0; i < cnt; ++i) memcpy(&tmp[i * 3], &indices[tc[i].first * 3], 12);
      memcpy(&indices[s * 3], tmp.data(), cnt * 12);
      uint32_t mid = (s + e) / 2;
      node[3] = (float)*next;
      build(s, mid, next);
      node[7] = (float)*next;
      build(mid, e, next);
    }
    memcpy(nodes + (size_t)cur * 8, node, sizeof node);
  }
};

// ------------------------------------------------------------------------
// The shader — src/shaders/raytrace_comp.comp
// ------------------------------------------------------------------------
struct Light { vec3 pos, nrm, inten; float sx, sy; };
struct Hit { float t; vec3 p, n; bool hit; };

struct Stats { uint64_t rays = 0, nodes = 0, leaves = 0; };

struct Scene {
  const float* V;
  const uint32_t* I;
  const float* N;          // BVHNode[] as 8 floats
  size_t nn;
  bool int_bits = false;   // child/triangle links stored as int32 bit patterns (PT_NODES_INT_BITS)
  std::vector<Light> lights;
  vec3 cpos, cdir, cup;
  float fov;
  int W, H, max_depth, sss_bounces;
};

static inline vec3 vtx(const Scene& s, uint32_t i) {            // :90-94
  uint32_t o = i * 3;
  return V(s.V[o], s.V[o + 1], s.V[o + 2]);
}

// :102-112 — slab test, invDir recomputed per call as the shader does.
static inline bool aabb(vec3 o, vec3 d, vec3 mn, vec3 mx) {
  vec3 inv = V(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
  vec3 t0 = (mn - o) * inv;
  vec3 t1 = (mx - o) * inv;
  vec3 tn = V(gm_fmin(t0.x, t1.x), gm_fmin(t0.y, t1.y), gm_fmin(t0.z, t1.z));
  vec3 tf = V(gm_fmax(t0.x, t1.x), gm_fmax(t0.y, t1.y), gm_fmax(t0.z, t1.z));
  float tmin = gm_fmax(gm_fmax(tn.x, tn.y), tn.z);
  float tmax = gm_fmin(gm_fmin(tf.x, tf.y), tf.z);
  return tmin <= tmax && tmax >= 0.0f;
}

// :114-157 — Möller–Trumbore; the UV tail (:150-154) has no effect on the
// output and is omitted.
static inline bool tri(vec3 o, vec3 d, vec3 v0, vec3 v1, vec3 v2, float* t) {
  const float EPS = 0.000001f;
  vec3 e1 = v1 - v0, e2 = v2 - v0;
  vec3 p = cross(d, e2);
  float det = dot(e1, p);
  if (gm_abs(det) < EPS) return false;
  float inv = 1.0f / det;
  vec3 s = o - v0;
  float u = inv * dot(s, p);
  if (u < 0.0f || u > 1.0f) return false;
  vec3 q = cross(s, e1);
  float v = inv * dot(d, q);
  if (v < 0.0f || u + v > 1.0f) return false;
  *t = inv * dot(e2, q);
  if (*t <= EPS) return false;
  return true;
}

// :159-204 — exhaustive DFS: push left then right, pop right first; strict <.
static Hit trace(const Scene& s, vec3 o, vec3 d, Stats* st) {
  Hit h{1e30f, V(0, 0, 0), V(0, 0, 0), false};
  int stack[64];
  int sp = 0;
  stack[sp++] = 0;
  st->rays++;
  while (sp > 0) {
    int ni = stack[--sp];
    const float* n = s.N + (size_t)ni * 8;
    st->nodes++;
    if (aabb(o, d, V(n[0], n[1], n[2]), V(n[4], n[5], n[6]))) {
      int l, r;
      if (s.int_bits) {
        // N >= 2^24 layout variant: the float cannot hold the index exactly
        // (BoundingVolumeHierarchy.cpp:74,77), so it travels as int32 bits
        memcpy(&l, &n[3], 4);
        memcpy(&r, &n[7], 4);
      } else {
        l = (int)n[3];                                           // :173-174
        r = (int)n[7];
      }
      if (l == -1) {
        uint32_t ti = (uint32_t)r;
        vec3 v0 = vtx(s, s.I[ti * 3 + 0]);
        vec3 v1 = vtx(s, s.I[ti * 3 + 1]);
        vec3 v2 = vtx(s, s.I[ti * 3 + 2]);
        float t;
        st->leaves++;
        if (tri(o, d, v0, v1, v2, &t) && t < h.t) {
          h.t = t;
          h.p = o + d * t;
          h.n = normalize(cross(v1 - v0, v2 - v0));
          h.hit = true;
        }
      } else {
        if (sp + 2 > 64) abort();
        stack[sp++] = l;
        stack[sp++] = r;
      }
    }
  }
  return h;
}


// :207-216 — RNG; float(result) / 4294967295.0 where the literal is a GLSL
// float, i.e. exactly 2^32.
static inline float rng_f(uint32_t* s) {
  *s = *s * 747796405u + 2891336453u;
  uint32_t r = ((*s >> ((*s >> 28u) + 4u)) ^ *s) * 277803737u;
  r = (r >> 22u) ^ r;
  return (float)r / 4294967296.0f;
}

static const float PI_F = 0x1.921fb6p+1f;    // MATH_PI as a float (:3)

// :218-226 — Box–Muller; 1e-38 is a subnormal float (denormals kept).
static inline void random_gaussian(uint32_t* s, float* gx, float* gy) {
  float u1 = gm_fmax(1e-38f, rng_f(s));
  float u2 = rng_f(s);
  float r = gm_sqrt(-2.0f * gm_log(u1));
  float th = (2.0f * PI_F) * u2;
  *gx = r * gm_cos(th);
  *gy = r * gm_sin(th);
}

// :229-243
static vec3 sample_hemisphere(vec3 n, uint32_t* s) {
  float r1 = rng_f(s);
  float r2 = rng_f(s);
  float th = gm_acos(gm_sqrt(1.0f - r1));
  float ph = (2.0f * PI_F) * r2;
  vec3 l = V(gm_sin(th) * gm_cos(ph), gm_sin(th) * gm_sin(ph), gm_cos(th));
  vec3 up = gm_abs(n.z) < 0.999f ? V(0, 0, 1) : V(1, 0, 0);
  vec3 t = normalize(cross(up, n));
  vec3 b = cross(n, t);
  return (t * l.x + b * l.y) + n * l.z;
}

// :246-253
static vec3 sample_sphere(uint32_t* s) {
  float z = 2.0f * rng_f(s) - 1.0f;
  float th = (2.0f * PI_F) * rng_f(s);
  float r = gm_sqrt(1.0f - z * z);
  return V(r * gm_cos(th), r * gm_sin(th), z);
}

// :255-268
static vec3 sample_area_light(const Light& L, uint32_t* s) {
  float u = rng_f(s) * 2.0f - 1.0f;
  float v = rng_f(s) * 2.0f - 1.0f;
  vec3 n = normalize(L.nrm);
  vec3 basis = gm_abs(n.y) < 0.999f ? V(0, 1, 0) : V(1, 0, 0);
  vec3 right = normalize(cross(n, basis));
  vec3 up = cross(right, n);
  return (L.pos + ((right * u) * L.sx) * 0.5f) + ((up * v) * L.sy) * 0.5f;
}

// :271-298
static bool intersect_area_light(vec3 o, vec3 d, const Light& L, float* t) {
  float denom = dot(L.nrm, d);
  if (gm_abs(denom) < 0.0001f) return false;
  *t = dot(L.nrm, L.pos - o) / denom;
  if (*t <= 0.0f) return false;
  vec3 hp = o + d * *t;
  vec3 n = normalize(L.nrm);
  vec3 basis = gm_abs(n.y) < 0.999f ? V(0, 1, 0) : V(1, 0, 0);
  vec3 right = normalize(cross(n, basis));
  vec3 up = cross(right, n);
  vec3 th = hp - L.pos;
  float u = dot(th, right), v = dot(th, up);
  return gm_abs(u) <= L.sx * 0.5f && gm_abs(v) <= L.sy * 0.5f;
}

// :300-418
static vec3 path_trace(const Scene& S, vec3 ro, vec3 rd, uint32_t seed, Stats* st) {
  vec3 thr = V(1, 1, 1);
  vec3 rad = V(0, 0, 0);
  const float OFFSET = 0.001f;
  uint32_t rng = seed;                                         // :307 re-seed
  for (const Light& L : S.lights) {                            // :311-328
    float t;
    if (intersect_area_light(ro, rd, L, &t)) {
      Hit sh = trace(S, ro, rd, st);
      if (!sh.hit || sh.t > t) return L.inten;
    }
  }
  for (int depth = 0; depth < S.max_depth; ++depth) {          // :331
    Hit h = trace(S, ro, rd, st);
    if (!h.hit) { rad = rad + thr * V(0, 0, 0); break; }
    const vec3 albedo = V(0.8f, 0.8f, 0.8f);
    vec3 direct = V(0, 0, 0);
    for (const Light& L : S.lights) {                          // :345-366
      vec3 lp = sample_area_light(L, &rng);
      vec3 ld = normalize(lp - h.p);
      float diff = gm_fmax(dot(h.n, ld), 0.0f);
      Hit sh = trace(S, h.p + h.n * OFFSET, ld, st);
      float dist = length(lp - h.p);
      if (!sh.hit || sh.t >= dist - OFFSET) {
        float d2 = dist * dist;
        vec3 c = (L.inten * diff) * (1.0f / gm_fmax(d2, 0.01f));
        direct = direct + albedo * c;
      }
    }
    rad = rad + thr * direct;
    const vec3 sss_albedo = V(1.0f, 0.2f, 0.1f);               // :371-408
    const float sss_radius = 1.0f;
    vec3 sss_thr = V(1, 1, 1);
    vec3 so = h.p - h.n * OFFSET;
    vec3 sd = sample_sphere(&rng);
    for (int k = 0; k < S.sss_bounces; ++k) {
      Hit sh = trace(S, so, sd, st);
      if (!sh.hit) break;
      float travel = sh.t;
      vec3 cp = so + sd * travel;
      vec3 sl = V(0, 0, 0);
      for (const Light& L : S.lights) {
        vec3 lp = sample_area_light(L, &rng);
        vec3 ed = normalize(lp - cp);
        float ediff = gm_fmax(dot(sh.n, ed), 0.0f);
        Hit eh = trace(S, cp + sh.n * OFFSET, ed, st);
        float edist = length(lp - cp);
        if (!eh.hit || eh.t >= edist - OFFSET) {
          float d2 = edist * edist;
          sl = sl + ((sss_albedo * ediff) * L.inten) * (1.0f / gm_fmax(d2, 0.01f));
        }
      }
      rad = rad + ((thr * sss_thr) * sl) * (1.0f + sss_radius * 0.5f);
      sss_thr = sss_thr * (sss_albedo * gm_exp(-travel / (sss_radius * 1.5f)));
      so = cp - sh.n * OFFSET;
      sd = sample_sphere(&rng);
    }
    vec3 bd = sample_hemisphere(h.n, &rng);                    // :411-414
    thr = thr * (albedo * dot(h.n, bd));
    ro = h.p + h.n * OFFSET;
    rd = bd;
  }
  return rad;
}

// :420-470 for one pixel and one sample batch; returns the new accumulator.
static void shade_pixel(const Scene& S, uint32_t px, uint32_t py, uint32_t batch, float* acc4, Stats* st) {
  const int W = S.W, H = S.H;
  float ndcX = (2.0f * (float)px / (float)W) - 1.0f;
  float ndcY = (2.0f * (float)py / (float)H) - 1.0f;
  float aspect = (float)W / (float)H;
  uint32_t seed = (batch * (uint32_t)H + py) * (uint32_t)W + px;
  uint32_t rng = seed;
  const float aperture = 0.02f, focal = 3.0f;
  float ax, ay;
  random_gaussian(&rng, &ax, &ay);
  ax = ax * aperture; ay = ay * aperture;
  vec3 right = normalize(cross(S.cdir, -S.cup));
  vec3 up = normalize(cross(right, S.cdir));
  vec3 no = (S.cpos + right * ax) + up * ay;
  float jx, jy;
  random_gaussian(&rng, &jx, &jy);
  const float js = 0.5f;
  ndcX = ndcX + (jx * js) / (float)W;
  ndcY = ndcY + (jy * js) / (float)H;
  float tf = gm_tan(gm_radians(S.fov * 0.5f));
  vec3 bd = normalize((S.cdir + (-right) * ((ndcX * tf) * aspect)) - up * (ndcY * tf));
  vec3 fp = S.cpos + bd * focal;
  vec3 rd = normalize(fp - no);
  vec3 c = path_trace(S, no, rd, seed, st);
  const float fb = (float)batch, fb1 = (float)(batch + 1u);
  acc4[0] = (acc4[0] * fb + c.x) / fb1;
  acc4[1] = (acc4[1] * fb + c.y) / fb1;
  acc4[2] = (acc4[2] * fb + c.z) / fb1;
  acc4[3] = (acc4[3] * fb + 1.0f) / fb1;
}

}  // namespace

extern "C" {

// Parse OBJ text with tinyobj's rules. Returns 0 on success.  Two-phase:
// call with null outputs to get the sizes, then with buffers.
int oracle_obj_parse(const char* text, size_t len, float* v_out, size_t* nv_floats,
                     uint32_t* idx_out, size_t* n_idx, float* vt_out, size_t* n_vt) {
  ObjOut o;
  int rc = obj_parse(text, len, &o);
  if (rc) return rc;
  if (v_out) memcpy(v_out, o.v.data(), o.v.size() * 4);
  if (idx_out) memcpy(idx_out, o.idx.data(), o.idx.size() * 4);
  if (vt_out) memcpy(vt_out, o.vt.data(), o.vt.size() * 4);
  *nv_floats = o.v.size();
  *n_idx = o.idx.size();
  *n_vt = o.vt.size();
  return 0;
}

// BoundingVolumeHierarchy.cpp:5-23: idx_out receives the reordered index
// buffer (3T), nodes_out 8 floats per node (2T-1 nodes).
int oracle_bvh_build(const float* verts, const uint32_t* idx_in, size_t n_idx,
                     uint32_t* idx_out, float* nodes_out) {
  if (n_idx % 3 != 0 || n_idx == 0) return -1;
  OracleBVH b;
  b.verts = verts;
  b.indices.assign(idx_in, idx_in + n_idx);
  b.nodes = nodes_out;
  uint32_t next = 0;
  b.build(0, (uint32_t)(n_idx / 3), &next);
  memcpy(idx_out, b.indices.data(), n_idx * 4);
  return 0;
}

// One or more sequential sample batches (= that many 1-spp dispatches of the
// reference) over the pixels selected by (row_stride,row_phase) and the tile
// ownership (tile, nranks, rank): pixel (x,y) is rendered iff
// y % row_stride == row_phase and tile (x/tile, y/tile) is owned: with
// tx = ceil(W/tile), block (bx, by) is tile by*tx + (bx - by) mod tx, owned iff
// that % nranks == rank.
// accum is W*H*4 floats (RGBA32F, row-major, y*W+x), read-modify-written.
// stats[0..2] += traceRay calls, nodes visited, leaf triangle tests.
// flags: ORACLE_INT_BITS = node links are int32 bit patterns.
// Threads take runs of 32 pixels of the selected rows (a row subset of a
// large scene is then balanced over the threads).
enum { ORACLE_INT_BITS = 1 };
int oracle_render_ex(const float* verts, const uint32_t* idx, const float* nodes, size_t n_nodes,
                     const float* camera16, const float* lights16, size_t n_lights,
                     int W, int H, uint32_t first_batch, uint32_t n_batches,
                     int max_depth, int sss_bounces,
                     int row_stride, int row_phase, int tile, int nranks, int rank,
                     float* accum, uint64_t* stats, int nthreads, uint32_t flags) {
  if (W <= 0 || H <= 0 || n_nodes == 0 || row_stride <= 0 || tile <= 0 || nranks <= 0) return -1;
  Scene S;
  S.V = verts; S.I = idx; S.N = nodes; S.nn = n_nodes;
  S.int_bits = (flags & ORACLE_INT_BITS) != 0;
  S.cpos = V(camera16[0], camera16[1], camera16[2]);
  S.cdir = V(camera16[4], camera16[5], camera16[6]);
  S.cup = V(camera16[8], camera16[9], camera16[10]);
  S.fov = camera16[12];
  for (size_t i = 0; i < n_lights; ++i) {
    const float* l = lights16 + i * 16;
    Light L;
    L.pos = V(l[0], l[1], l[2]);
    L.nrm = V(l[4], l[5], l[6]);
    L.inten = V(l[8], l[9], l[10]);
    L.sx = l[12]; L.sy = l[13];
    S.lights.push_back(L);
  }
  S.W = W; S.H = H; S.max_depth = max_depth; S.sss_bounces = sss_bounces;
  const int tiles_x = (W + tile - 1) / tile;
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::vector<int> rows;
  for (int y = 0; y < H; ++y)
    if (y % row_stride == row_phase) rows.push_back(y);
  constexpr int kRun = 32;
  const int runs_per_row = (W + kRun - 1) / kRun;
  const long long n_runs = (long long)rows.size() * runs_per_row;
  std::atomic<long long> next_run{0};
  std::vector<Stats> per(nthreads);
  auto work = [&](int tid) {
    Stats& st = per[tid];
    for (;;) {
      const long long j = next_run.fetch_add(1);
      if (j >= n_runs) break;
      const int y = rows[(size_t)(j / runs_per_row)];
      const int x0 = (int)(j % runs_per_row) * kRun, x1 = std::min(W, x0 + kRun);
      for (int x = x0; x < x1; ++x) {
        // partition order of the product (pt_device.h tile_block): rows rotated by their index
        const int by = y / tile, bx = x / tile;
        const int tid2 = by * tiles_x + (bx - by % tiles_x + tiles_x) % tiles_x;
        if (tid2 % nranks != rank) continue;
        float* a = accum + ((size_t)y * W + x) * 4;
        for (uint32_t b = 0; b < n_batches; ++b) shade_pixel(S, (uint32_t)x, (uint32_t)y, first_batch + b, a, &st);
      }
    }
  };
  if (nthreads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int i = 0; i < nthreads; ++i) th.emplace_back(work, i);
    for (auto& t : th) t.join();
  }
  if (stats) {
    for (auto& s : per) { stats[0] += s.rays; stats[1] += s.nodes; stats[2] += s.leaves; }
  }
  return 0;
}

// The pixels listed in pixels[0..n) (y*W+x; negative entries skipped), each
// with n_batches sequential batches, threads over runs of 32 list entries.
int oracle_render_pixels(const float* verts, const uint32_t* idx, const float* nodes, size_t n_nodes,
                         const float* camera16, const float* lights16, size_t n_lights,
                         int W, int H, uint32_t first_batch, uint32_t n_batches, int max_depth, int sss_bounces,
                         const int32_t* pixels, size_t n, float* accum, uint64_t* stats, int nthreads,
                         uint32_t flags) {
  if (W <= 0 || H <= 0 || n_nodes == 0) return -1;
  Scene S;
  S.V = verts; S.I = idx; S.N = nodes; S.nn = n_nodes;
  S.int_bits = (flags & ORACLE_INT_BITS) != 0;
  S.cpos = V(camera16[0], camera16[1], camera16[2]);
  S.cdir = V(camera16[4], camera16[5], camera16[6]);
  S.cup = V(camera16[8], camera16[9], camera16[10]);
  S.fov = camera16[12];
  for (size_t i = 0; i < n_lights; ++i) {
    const float* l = lights16 + i * 16;
    Light L;
    L.pos = V(l[0], l[1], l[2]);
    L.nrm = V(l[4], l[5], l[6]);
    L.inten = V(l[8], l[9], l[10]);
    L.sx = l[12]; L.sy = l[13];
    S.lights.push_back(L);
  }
  S.W = W; S.H = H; S.max_depth = max_depth; S.sss_bounces = sss_bounces;
  if (nthreads <= 0) nthreads = (int)std::thread::hardware_concurrency();
  if (nthreads <= 0) nthreads = 1;
  std::atomic<size_t> next{0};
  std::vector<Stats> per(nthreads);
  auto work = [&](int tid) {
    for (;;) {
      const size_t j0 = next.fetch_add(32);
      if (j0 >= n) break;
      for (size_t j = j0; j < std::min(n, j0 + 32); ++j) {
        const int32_t pix = pixels[j];
        if (pix < 0 || pix >= W * H) continue;
        float* a = accum + (size_t)pix * 4;
        for (uint32_t b = 0; b < n_batches; ++b)
          shade_pixel(S, (uint32_t)(pix % W), (uint32_t)(pix / W), first_batch + b, a, &per[tid]);
      }
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < nthreads; ++i) th.emplace_back(work, i);
  for (auto& t : th) t.join();
  if (stats) {
    for (auto& s : per) { stats[0] += s.rays; stats[1] += s.nodes; stats[2] += s.leaves; }
  }
  return 0;
}

int oracle_render(const float* verts, const uint32_t* idx, const float* nodes, size_t n_nodes,
                  const float* camera16, const float* lights16, size_t n_lights,
                  int W, int H, uint32_t first_batch, uint32_t n_batches,
                  int max_depth, int sss_bounces,
                  int row_stride, int row_phase, int tile, int nranks, int rank,
                  float* accum, uint64_t* stats, int nthreads) {
  return oracle_render_ex(verts, idx, nodes, n_nodes, camera16, lights16, n_lights, W, H, first_batch, n_batches,
                          max_depth, sss_bounces, row_stride, row_phase, tile, nranks, rank, accum, stats,
                          nthreads, 0u);
}

// Math entry points for tests/test_math.py (bitwise agreement with the
// device math and ulp distance to libm).
void oracle_math(int fn, const float* x, float* y, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    float v = x[i];
    switch (fn) {
      case 0: y[i] = gm_log(v); break;
      case 1: y[i] = gm_exp(v); break;
      case 2: y[i] = gm_sin(v); break;
      case 3: y[i] = gm_cos(v); break;
      case 4: y[i] = gm_tan(v); break;
      case 5: y[i] = gm_acos(v); break;
      case 6: y[i] = gm_sqrt(v); break;
      case 7: { uint32_t sd = gm_f2u(v); y[i] = rng_f(&sd); break; }
      case 8: y[i] = 1.0f / v; break;
      default: y[i] = v; break;
    }
  }
}

void oracle_rng(uint32_t seed, float* out, size_t n) {
  uint32_t s = seed;
  for (size_t i = 0; i < n; ++i) out[i] = rng_f(&s);
}

}  // extern "C"

extern "C" {
// Single traceRay (raytrace_comp.comp:159-204) for known-answer tests:
// out[0] = hit (0/1), out[1] = t, out[2..4] = position, out[5..7] = normal;
// counters[0..2] += rays, nodes, leaves.
void oracle_trace(const float* verts, const uint32_t* idx, const float* nodes, size_t n_nodes,
                  const float* o3, const float* d3, float* out, uint64_t* counters) {
  Scene S;
  S.V = verts; S.I = idx; S.N = nodes; S.nn = n_nodes;
  Stats st;
  Hit h = trace(S, V(o3[0], o3[1], o3[2]), V(d3[0], d3[1], d3[2]), &st);
  out[0] = h.hit ? 1.0f : 0.0f;
  out[1] = h.t;
  out[2] = h.p.x; out[3] = h.p.y; out[4] = h.p.z;
  out[5] = h.n.x; out[6] = h.n.y; out[7] = h.n.z;
  if (counters) { counters[0] += st.rays; counters[1] += st.nodes; counters[2] += st.leaves; }
}
}
