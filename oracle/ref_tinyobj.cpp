// oracle/ref_tinyobj.cpp — TEST INFRASTRUCTURE: a C-ABI wrapper around the
// reference's own, unmodified OBJ loader, used only to pin the two OBJ
// restatements (the product's csrc/scene/obj_loader.cpp and the oracle's
// obj_parse in pt_oracle.cpp) against the real thing.
//
// The loader itself is NOT in this repository: oracle/Makefile's `ref` target
// compiles this file with -I/root/reference/external, so the header is read
// where it lies (tinyobjloader v2.0.0 as vendored by the reference,
// external/tiny_obj_loader.h: number parser :897-1028, triangulation
// :1509-1612, ear clipping :1740-1955).  Output goes to oracle/_ref/ (git-
// ignored).  tiny_obj_loader.h is dependency-free, so the build needs no
// stand-in headers.
//
// ref_obj_parse follows the reference's ingest call site
// (src/Vulkan/VulkanRayTracer.cpp:64-92): ObjReader with the default config
// (triangulate, "simple"), vertices = GetAttrib().GetVertices(), uvs =
// GetAttrib().texcoords, indices = every shape's mesh.indices[].vertex_index in
// shape order, material ids one per triangle with -1 -> 0.
#define TINYOBJLOADER_IMPLEMENTATION
#include "tiny_obj_loader.h"

#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

extern "C" {

// Two-phase like oracle_obj_parse: call with null buffers for the sizes, then
// with buffers of at least those sizes.  Returns 0, or -1 when ParseFromString
// fails.
int ref_obj_parse(const char* text, size_t len, float* v_out, size_t* nv, uint32_t* idx_out, size_t* ni,
                  float* vt_out, size_t* nvt, uint32_t* mat_out, size_t* nmat) {
  tinyobj::ObjReader reader;
  if (!reader.ParseFromString(std::string(text, len), std::string())) return -1;
  const std::vector<tinyobj::real_t>& v = reader.GetAttrib().GetVertices();
  const std::vector<tinyobj::real_t>& vt = reader.GetAttrib().texcoords;
  std::vector<uint32_t> idx, mat;
  for (const tinyobj::shape_t& s : reader.GetShapes())
    for (const tinyobj::index_t& i : s.mesh.indices) idx.push_back((uint32_t)i.vertex_index);
  for (const tinyobj::shape_t& s : reader.GetShapes())
    for (int m : s.mesh.material_ids) mat.push_back(m >= 0 ? (uint32_t)m : 0u);
  if (v_out) memcpy(v_out, v.data(), v.size() * sizeof(float));
  if (idx_out) memcpy(idx_out, idx.data(), idx.size() * sizeof(uint32_t));
  if (vt_out) memcpy(vt_out, vt.data(), vt.size() * sizeof(float));
  if (mat_out) memcpy(mat_out, mat.data(), mat.size() * sizeof(uint32_t));
  *nv = v.size();
  *ni = idx.size();
  *nvt = vt.size();
  *nmat = mat.size();
  return 0;
}

}  // extern "C"
