// OBJ scene ingest — what VulkanRayTracer.cpp:64-92 does with
// tinyobj::ObjReader::ParseFromFile (external/tiny_obj_loader.h, v2.0.0,
// triangulate=true): positions, texcoords, the vertex_index of every face
// corner of every shape in file order, and one material id per triangle
// (-1 -> 0).  Numbers are parsed with tinyobj's own algorithm (:897-1028) and
// quads are split on the shorter diagonal exactly as :1509-1604, so the
// triangle order — which the BVH builder's unstable sort depends on — is the
// reference's.  Faces with more than four corners take tinyobj's built-in
// ear-clipping path (:1740-1955), restated here (the reference build does not
// define TINYOBJLOADER_USE_MAPBOX_EARCUT).
#pragma once
#include <stdint.h>
#include <string>
#include <vector>

namespace pt {

struct ObjScene {
  std::vector<float> vertices;        // x,y,z per vertex   (attrib.vertices)
  std::vector<float> texcoords;       // u,v per texcoord   (attrib.texcoords)
  std::vector<uint32_t> indices;      // 3 per triangle     (index_t::vertex_index)
  std::vector<uint32_t> materialIds;  // 1 per triangle     (mesh.material_ids, -1 -> 0)
  size_t shapes = 0;
};

int parse_obj(const char* text, size_t len, ObjScene* out, std::string* err);
int load_obj_file(const std::string& path, ObjScene* out, std::string* err);

}  // namespace pt
