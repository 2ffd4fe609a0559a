// Host BVH builder; see bvh.h for the contract.  Algorithm restated from
// src/BoundingVolumeHierarchy.cpp:25-111 (reference), restructured so that
// per-triangle work is done once and independent subtrees run in parallel.
#include "bvh.h"

#include <float.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <system_error>
#include <thread>
#include <utility>

namespace pt {
namespace {

// glm::min / glm::max on floats: (y < x) ? y : x and (x < y) ? y : x.
// Spelt out because the order of operands decides which signed zero wins.
inline float glm_min(float x, float y) { return (y < x) ? y : x; }
inline float glm_max(float x, float y) { return (x < y) ? y : x; }

struct Key {
  float k;
  uint32_t id;
};

class Builder {
 public:
  Builder(const float* V, const uint32_t* idx, size_t T, BVHNode* nodes, BVHEncoding enc, int threads)
      : V_(V), idx_(idx), T_(T), nodes_(nodes), enc_(enc), spare_threads_(threads - 1) {}

  void run(uint32_t* idx_out) {
    perm_.resize(T_);
    tmin_.resize(T_ * 3);
    tmax_.resize(T_ * 3);
    cen_.resize(T_ * 3);
    // Per-triangle terms of computeBounds (:91-99) and computeCentroid
    // (:102-111), evaluated once per triangle in the reference's op order.
    auto prep = [&](size_t a, size_t b) {
      for (size_t t = a; t < b; ++t) {
        perm_[t] = (uint32_t)t;
        const float* v0 = V_ + (size_t)idx_[t * 3 + 0] * 3;
        const float* v1 = V_ + (size_t)idx_[t * 3 + 1] * 3;
        const float* v2 = V_ + (size_t)idx_[t * 3 + 2] * 3;
        for (int c = 0; c < 3; ++c) {
          tmin_[t * 3 + c] = glm_min(v0[c], glm_min(v1[c], v2[c]));
          tmax_[t * 3 + c] = glm_max(v0[c], glm_max(v1[c], v2[c]));
          cen_[t * 3 + c] = ((v0[c] + v1[c]) + v2[c]) / 3.0f;
        }
      }
    };
    parallel_for(T_, prep);
    build(0, (uint32_t)T_, 0);
    auto scatter = [&](size_t a, size_t b) {
      for (size_t p = a; p < b; ++p) memcpy(idx_out + p * 3, idx_ + (size_t)perm_[p] * 3, 12);
    };
    parallel_for(T_, scatter);
  }

 private:
  template <class F>
  void parallel_for(size_t n, F f) {
    int nt = std::max(1, spare_threads_.load() + 1);
    if (n < 65536 || nt == 1) { f(0, n); return; }
    std::vector<std::thread> th;
    size_t chunk = (n + nt - 1) / nt;
    for (int i = 0; i < nt; ++i) {
      size_t a = i * chunk, b = std::min(n, a + chunk);
      if (a >= b) continue;
      try {
        th.emplace_back(f, a, b);
      } catch (const std::system_error&) {   // no thread to be had: this chunk here
        f(a, b);
      }
    }
    for (auto& t : th) t.join();
  }

  float enc(uint32_t v) const {
    if (enc_ == BVHEncoding::kFloat) return (float)v;   // glm::vec4::w = uint32 (:74,77)
    float f;
    memcpy(&f, &v, 4);
    return f;
  }
  float leaf_flag() const {
    if (enc_ == BVHEncoding::kFloat) return -1.0f;
    int32_t m1 = -1;
    float f;
    memcpy(&f, &m1, 4);
    return f;
  }

  // constructBVH (:25-82) for triangle positions [s,e) rooted at node `cur`.
  void build(uint32_t s, uint32_t e, uint32_t cur) {
    // computeBounds (:84-100): fold in the current triangle order.
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (uint32_t p = s; p < e; ++p) {
      const uint32_t t = perm_[p];
      for (int c = 0; c < 3; ++c) {
        mn[c] = glm_min(mn[c], tmin_[(size_t)t * 3 + c]);
        mx[c] = glm_max(mx[c], tmax_[(size_t)t * 3 + c]);
      }
    }
    BVHNode node;
    node.minBounds[0] = mn[0]; node.minBounds[1] = mn[1]; node.minBounds[2] = mn[2];
    node.maxBounds[0] = mx[0]; node.maxBounds[1] = mx[1]; node.maxBounds[2] = mx[2];
    const uint32_t cnt = e - s;
    if (cnt == 1) {
      node.minBounds[3] = leaf_flag();
      node.maxBounds[3] = enc(s);
      nodes_[cur] = node;
      return;
    }
    const float sx = mx[0] - mn[0], sy = mx[1] - mn[1], sz = mx[2] - mn[2];
    const int axis = (sx > sy) ? ((sx > sz) ? 0 : 2) : ((sy > sz) ? 1 : 2);   // :56
    {
      std::vector<Key> keys(cnt);
      for (uint32_t i = 0; i < cnt; ++i) {
        const uint32_t t = perm_[s + i];
        keys[i].k = cen_[(size_t)t * 3 + axis];
        keys[i].id = t;
      }
      // Same comparator as :58-61 on the same key sequence -> same permutation.
      std::sort(keys.begin(), keys.end(), [](const Key& a, const Key& b) { return a.k < b.k; });
      for (uint32_t i = 0; i < cnt; ++i) perm_[s + i] = keys[i].id;
    }
    const uint32_t mid = (s + e) / 2;                                         // :72
    const uint32_t left = cur + 1;
    const uint32_t right = cur + 2 * (mid - s);          // left subtree has 2(mid-s)-1 nodes
    node.minBounds[3] = enc(left);
    node.maxBounds[3] = enc(right);
    nodes_[cur] = node;
    std::thread th;
    if (cnt >= 200000 && try_take_thread()) {
      try {
        th = std::thread([=] { build(s, mid, left); });
      } catch (const std::system_error&) {   // no thread to be had: build both halves here
        spare_threads_.fetch_add(1);
      }
    }
    if (th.joinable()) {
      build(mid, e, right);
      th.join();
      spare_threads_.fetch_add(1);
    } else {
      build(s, mid, left);
      build(mid, e, right);
    }
  }

  bool try_take_thread() {
    int v = spare_threads_.load();
    while (v > 0) {
      if (spare_threads_.compare_exchange_weak(v, v - 1)) return true;
    }
    return false;
  }

  const float* V_;
  const uint32_t* idx_;
  size_t T_;
  BVHNode* nodes_;
  BVHEncoding enc_;
  std::atomic<int> spare_threads_;
  std::vector<uint32_t> perm_;
  std::vector<float> tmin_, tmax_, cen_;
};

}  // namespace

int build_bvh(const float* vertices, size_t n_vertex_floats, const uint32_t* idx_in, size_t n_idx,
              uint32_t* idx_out, BVHNode* nodes_out, BVHOptions opts, std::string* err) {
  if (n_idx % 3 != 0) {           // :8-12
    if (err) *err = "index array size must be a multiple of 3";
    return -1;
  }
  if (n_idx == 0) {               // the reference computes 2*0-1 = 0xFFFFFFFF nodes and throws
    if (err) *err = "scene has no triangles";
    return -1;
  }
  if (n_idx / 3 > 0x7fffffffull) {
    if (err) *err = "too many triangles";
    return -1;
  }
  const size_t nv = n_vertex_floats / 3;
  for (size_t i = 0; i < n_idx; ++i) {
    if (idx_in[i] >= nv) {
      if (err) *err = "vertex index out of range";
      return -2;
    }
  }
  int threads = opts.threads > 0 ? opts.threads : (int)std::thread::hardware_concurrency();
  if (threads <= 0) threads = 1;
  Builder b(vertices, idx_in, n_idx / 3, nodes_out, opts.encoding, threads);
  b.run(idx_out);
  return 0;
}

BVH::BVH(const std::vector<float>& objVertices, const std::vector<uint32_t>& objIndices, BVHOptions opts)
    : vertices(objVertices) {
  const size_t n = objIndices.size();
  if (n == 0 || n % 3 != 0) {
    error = n == 0 ? "scene has no triangles" : "index array size must be a multiple of 3";
    return;
  }
  indices.resize(n);
  nodes.resize(2 * (n / 3) - 1);
  if (build_bvh(objVertices.data(), objVertices.size(), objIndices.data(), n, indices.data(), nodes.data(),
                opts, &error) != 0) {
    indices.clear();
    nodes.clear();
  }
}

}  // namespace pt
