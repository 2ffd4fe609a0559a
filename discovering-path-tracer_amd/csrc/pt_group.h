// pt_group.h — internal interface between the C-ABI shim (pt_api.cpp) and
// the single-process multi-device context (pt_group.cpp, pt_create_multi).
//
// A group is a pt_context whose calls the shim forwards here.  The group
// drives one ordinary context per member device through the public C ABI,
// each owning the screen tiles of the tile partition (pt_set_partition), and
// assembles the frame on the first device.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/pathtracer.h"

struct pt_group;

// Sets pt_last_error() on the calling thread and returns code (pt_api.cpp).
int pt_fail_internal(int code, const std::string& msg);
// The group wrote a member's accumulation buffer itself (a memset, a peer
// copy): what its culled items hold is no longer what the member last wrote.
// finite: every pixel is now +-0 (a memset to zero).
void pt_note_accum_written(pt_context* c, bool finite);

namespace ptg {
int make(const int* ordinals, int n, pt_group** out);
int destroy(pt_group* g);
int set_stream(pt_group* g, void* s);
int synchronize(pt_group* g);
int upload_scene(pt_group* g, const float* vertices, size_t n_vertex_floats, const uint32_t* indices,
                 size_t n_indices, const pt_bvh_node* nodes, size_t n_nodes, const float* uvs, size_t n_uv_floats,
                 const uint32_t* mat_indices, size_t n_mat, uint32_t flags);
int upload_lights(pt_group* g, const pt_area_light* lights, size_t n);
int set_camera(pt_group* g, const float ubo[16]);
int set_params(pt_group* g, const pt_params* p);
int resize_and_clear(pt_group* g, int w, int h);
int bind_accum(pt_group* g, void* ptr, int w, int h);
int clear_accum(pt_group* g);
void* accum_device_ptr(pt_group* g);
int read_accum(pt_group* g, float* rgba, size_t n);
int render(pt_group* g, uint32_t first_batch, uint32_t n_batches);
int progressive_camera(pt_group* g, const float ubo[16], int* reset);
int progressive_advance(pt_group* g, uint32_t max_new, uint32_t limit, uint32_t* first, uint32_t* count);
int readback_begin(pt_group* g, int* ticket);
int readback_end(pt_group* g, int ticket, float* rgba, size_t n);
int set_option(pt_group* g, int key, int value);
int last_kernel(pt_group* g, int* kernel);
int set_stats_mode(pt_group* g, int enabled);
int get_stats(pt_group* g, pt_stats* out);
int reset_stats(pt_group* g);
int get_traced(pt_group* g, pt_traced* out);
int wide_info(pt_group* g, int info[2]);
int last_launch_ms(pt_group* g, float* ms);
int launch_times_ms(pt_group* g, float* out, size_t max_n, size_t* n_out);
int launch_span_ms(pt_group* g, float* ms, size_t* n_out);
int reset_launch_times(pt_group* g);
int members(pt_group* g, int* n, int* devices, int max_devices, int* peer);
int check_info(pt_group* g, int* state, float* ms_peer, float* ms_staged);
}  // namespace ptg
