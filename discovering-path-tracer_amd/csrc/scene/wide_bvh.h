// Wide (4-ary) BVH for the culled walk of device-memory scenes
// (csrc/wide_walk.h explains why the walk returns the reference's hits).
//
// Built from the uploaded reference tree (BoundingVolumeHierarchy.cpp layout,
// already validated as a tree by thread_bvh): every wide node holds up to four
// of the reference's own nodes (their boxes bitwise), obtained by expanding a
// reference internal node's children until four or all leaves; leaves are
// numbered by the rank the reference's right-first DFS (raytrace_comp.comp
// :196-200) visits them in.  Each node also stores the cull coefficients of
// the triangles below it.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace pt {

struct WideBVH {
  std::vector<float> nodes;        // 32 floats per node, the wide_walk.h layout
  std::vector<float> qnodes;       // the same nodes, 16 floats each: child boxes on an 8-bit grid (wide_walk.h)
  std::vector<float> leaf_box;     // 8 floats per leaf rank: the reference's leaf box {lo.xyz, 0, hi.xyz, 0}
  std::vector<int32_t> rank_tri;   // leaf rank -> triangle slot (the reference's triIdx)
  int n_nodes = 0;
  int stack_cap = 0;               // most stack entries a walk can hold
};

// How the 4-wide nodes group the reference's leaves.  Either way every child
// box is a reference leaf box (bitwise) or contains the leaf boxes below it,
// which is all the walk's exactness needs (wide_walk.h).
enum WideBuild {
  WIDE_FROM_REFERENCE = 0,   // collapse the reference's own tree (its internal boxes)
  WIDE_SAH = 1,              // binned-SAH tree over the reference's leaf boxes
};

// nodes: n reference nodes, 8 floats each ({min.xyz, left}, {max.xyz, right};
// links float- or int-encoded).  Returns "" on success, else the reason the
// culled walk cannot take this scene (the caller keeps the exact walk): a
// parent box not containing a child's, a leaf box not containing its
// triangle, non-finite or huge coordinates, or a degenerate depth.
std::string build_wide_bvh(const float* nodes, size_t n, bool int_bits, const float* verts, size_t n_vertex_floats,
                           const uint32_t* idx, size_t n_tris, WideBVH* out, int mode = WIDE_SAH);

// The cull coefficients of one triangle (edges e1 = fl(v1-v0), e2 = fl(v2-v0)),
// wide_bvh.cpp: an accepted t_b and the exact T of the same test satisfy
// t_b >= (T (1 - k1) - k2 S) / (1 + g3), and o + T d lies within
// eps0 + eps1 S (inf-norm) of the triangle, S = |o - v0|_inf.  false: no
// bound (the triangle is too large for the |det| >= 1e-6 analysis).
struct WideCoeffs {
  double k1, k2, eps0, eps1;
};
bool wide_tri_coeffs(const float e1[3], const float e2[3], WideCoeffs* out);
WideCoeffs coeff_max(const WideCoeffs& a, const WideCoeffs& b);
// The 4 floats of a node's cull constants from its children's coefficients.
void node_cull_consts(const WideCoeffs& co, float* out);

}  // namespace pt
