// Host BVH builder — the producer of the kernel's node and index buffers.
//
// Mirrors the reference class src/BoundingVolumeHierarchy.h:15-36 (same
// constructor, same getVertices/getIndices/getNodes accessors, same flattened
// layout) and produces byte-identical output to
// src/BoundingVolumeHierarchy.cpp:5-82 whenever the reference's float-encoded
// child indices are exact (node count < 2^24):
//   * median split on the longest axis of the node bounds (strict '>' tie
//     rule, :56), std::sort by centroid[axis] (:58-61) — libstdc++'s
//     introsort, so ties resolve exactly as the reference's do;
//   * pre-order node numbering, leaf = {min.w = -1, max.w = first triangle}.
// Differences that do not change the output:
//   * per-triangle centroids and bounds are computed once, not per level;
//   * the two subtrees of a node are independent (disjoint index and node
//     ranges), so large subtrees are built on worker threads;
//   * BVHEncoding::kIntBits stores child/triangle indices as int bit
//     patterns, the fix for trees with >= 2^24 nodes,
//     where the reference's float encoding silently corrupts indices.
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace pt {

// BoundingVolumeHierarchy.h:8-13
struct BVHNode {
  float minBounds[4];   // xyz = min, w = left child index, or -1 for a leaf
  float maxBounds[4];   // xyz = max, w = right child index, or triangle index
};
static_assert(sizeof(BVHNode) == 32, "std430 stride of BVHNode is 32 B");

enum class BVHEncoding { kFloat = 0, kIntBits = 1 };

struct BVHOptions {
  BVHEncoding encoding = BVHEncoding::kFloat;
  int threads = 0;                 // 0 = hardware_concurrency
};

class BVH {
 public:
  BVH(const std::vector<float>& objVertices, const std::vector<uint32_t>& objIndices,
      BVHOptions opts = BVHOptions());

  const std::vector<float>& getVertices() const { return vertices; }
  const std::vector<uint32_t>& getIndices() const { return indices; }
  const std::vector<BVHNode>& getNodes() const { return nodes; }
  bool ok() const { return error.empty(); }
  const std::string& getError() const { return error; }

 private:
  const std::vector<float>& vertices;   // like the reference: a reference to the caller's data
  std::vector<uint32_t> indices;
  std::vector<BVHNode> nodes;
  std::string error;
};

// Flat C-style entry used by the C-ABI: builds into caller buffers.
// nodes_out has 2T-1 entries, idx_out 3T.  Returns 0 or a negative error.
int build_bvh(const float* vertices, size_t n_vertex_floats, const uint32_t* idx_in, size_t n_idx,
              uint32_t* idx_out, BVHNode* nodes_out, BVHOptions opts, std::string* err);

}  // namespace pt
