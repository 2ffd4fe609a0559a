// tools/gather_roof.hip — ceilings of random small-record gathers on MI355X
// (the access pattern of BVH traversal).  Not part of the product.
//
// gather: every lane issues U independent random loads of an F4 x 16-B
// record per iteration from a table of T bytes (throughput ceiling: many
// loads in flight per lane).
// chase: every lane follows a chain of dependent loads -- the next record's
// index is read from the record just loaded -- one load in flight per lane,
// as the wide walk's node fetches are (a node's children are known only
// once it has arrived).  Run at the trace kernel's occupancy (6 workgroups
// of 256 per CU) this is the ceiling for one node fetch per lane per step:
// the "l2_gather" roofline of cache-resident trees.
// Reports records/s and useful GB/s (record bytes).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return x;
}

template <int U, int F4>
__global__ __launch_bounds__(256) void gather(const float4* __restrict__ t, uint64_t nrec, int iters, float* out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  float s = 0.0f;
  uint64_t h = mix(g + 1);
  for (int it = 0; it < iters; ++it) {
    float4 v[U][F4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      h = mix(h + u);
      const uint64_t r = h & (nrec - 1);
#pragma unroll
      for (int k = 0; k < F4; ++k) v[u][k] = t[r * F4 + k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < F4; ++k) s += v[u][k].x + v[u][k].w;
  }
  if (s == 1234.5f) out[0] = s;
}

// record r's first word: a random record index (the chain's next link)
template <int F4>
__global__ void init_links(float4* t, uint64_t nrec) {
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (r >= nrec) return;
  const uint32_t nxt = (uint32_t)(mix(r * 0x9e3779b97f4a7c15ull + 7) & (nrec - 1));
  for (int k = 0; k < F4; ++k) t[r * F4 + k] = make_float4(k == 0 ? __uint_as_float(nxt) : 0.0f, 0.0f, 0.0f, 1.0f);
}

template <int F4>
__global__ __launch_bounds__(256) void chase(const float4* __restrict__ t, uint64_t nrec, int iters, float* out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint32_t mask = (uint32_t)(nrec - 1), seed = (uint32_t)mix(g + 1);
  uint32_t r = seed & mask;
  float s = 0.0f;
  for (int it = 0; it < iters; ++it) {
    float4 v[F4];
#pragma unroll
    for (int k = 0; k < F4; ++k) v[k] = t[(uint64_t)r * F4 + k];
#pragma unroll
    for (int k = 1; k < F4; ++k) s += v[k].w;
    // the loaded link, re-scrambled per step so no chain settles into a
    // short cycle (a random mapping's cycles would end up in L1)
    r = (__float_as_uint(v[0].x) ^ (seed + (uint32_t)it * 0x9e3779b9u)) & mask;
  }
  if (s == 1234.5f || r == 0xffffffffu) out[0] = s;
}

// C independent dependent chains per lane, interleaved: C records in flight
// per lane (the wide walk's memory-level parallelism with several walks or
// a prefetch per lane), four 16-B loads per 64-B record.
template <int F4, int C>
__global__ __launch_bounds__(256) void chase_multi(const float4* __restrict__ t, uint64_t nrec, int iters,
                                                   float* out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint32_t mask = (uint32_t)(nrec - 1);
  uint32_t r[C], seed[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    seed[c] = (uint32_t)mix(g * C + c + 1);
    r[c] = seed[c] & mask;
  }
  float s = 0.0f;
  for (int it = 0; it < iters; ++it) {
    float4 v[C][F4];
#pragma unroll
    for (int c = 0; c < C; ++c)
#pragma unroll
      for (int k = 0; k < F4; ++k) v[c][k] = t[(uint64_t)r[c] * F4 + k];
#pragma unroll
    for (int c = 0; c < C; ++c) {
#pragma unroll
      for (int k = 1; k < F4; ++k) s += v[c][k].w;
      r[c] = (__float_as_uint(v[c][0].x) ^ (seed[c] + (uint32_t)it * 0x9e3779b9u)) & mask;
    }
  }
  uint32_t x = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) x ^= r[c];
  if (s == 1234.5f || x == 0xffffffffu) out[0] = s;
}

// Independent random records with a cheap 32-bit index generator (xorshift):
// U records in flight per lane, so the issue of the index arithmetic is not
// what bounds the rate (the 64-bit mix of `gather` above is).
template <int U, int F4>
__global__ __launch_bounds__(256) void gather32(const float4* __restrict__ t, uint32_t mask, int iters, float* out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint32_t h = (uint32_t)mix(g + 1) | 1u;
  float s = 0.0f;
  for (int it = 0; it < iters; ++it) {
    float4 v[U][F4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      h ^= h << 13;
      h ^= h >> 17;
      h ^= h << 5;
      const uint32_t r = h & mask;
#pragma unroll
      for (int k = 0; k < F4; ++k) v[u][k] = t[(uint64_t)r * F4 + k];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int k = 0; k < F4; ++k) s += v[u][k].x + v[u][k].w;
  }
  if (s == 1234.5f) out[0] = s;
}

template <int F4, int C>
void run_chase_multi(float4* t, uint64_t table_bytes, int blocks, int iters, float* out, const char* tag) {
  const uint64_t nrec = table_bytes / (16 * F4);
  init_links<F4><<<(unsigned)((nrec + 255) / 256), 256>>>(t, nrec);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  chase_multi<F4, C><<<blocks, 256>>>(t, nrec, 8, out);   // warm
  CK(hipEventRecord(e0));
  chase_multi<F4, C><<<blocks, 256>>>(t, nrec, iters, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double recs = (double)blocks * 256 * iters * C;
  printf("{\"case\": \"%s\", \"pattern\": \"dependent_chains\", \"chains_per_lane\": %d, \"table_MB\": %.1f, "
         "\"record_B\": %d, \"loads_per_record\": %d, \"blocks\": %d, \"iters\": %d, \"ms\": %.3f, "
         "\"Grec_per_s\": %.2f, \"useful_GBps\": %.1f}\n",
         tag, C, table_bytes / 1e6, 16 * F4, F4, blocks, iters, ms, recs / ms / 1e6, recs * 16 * F4 / ms / 1e6);
  fflush(stdout);
}

template <int U, int F4>
void run_gather32(const float4* t, uint64_t table_bytes, int blocks, int iters, float* out, const char* tag) {
  const uint64_t nrec = table_bytes / (16 * F4);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  gather32<U, F4><<<blocks, 256>>>(t, (uint32_t)(nrec - 1), 1, out);   // warm
  CK(hipEventRecord(e0));
  gather32<U, F4><<<blocks, 256>>>(t, (uint32_t)(nrec - 1), iters, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double recs = (double)blocks * 256 * iters * U;
  printf("{\"case\": \"%s\", \"pattern\": \"independent32\", \"records_in_flight_per_lane\": %d, "
         "\"table_MB\": %.1f, \"record_B\": %d, \"loads_per_record\": %d, \"blocks\": %d, \"ms\": %.3f, "
         "\"Grec_per_s\": %.2f, \"useful_GBps\": %.1f}\n",
         tag, U, table_bytes / 1e6, 16 * F4, F4, blocks, ms, recs / ms / 1e6, recs * 16 * F4 / ms / 1e6);
  fflush(stdout);
}

template <int U, int F4>
void run(const float4* t, uint64_t table_bytes, int blocks, int iters, float* out, const char* tag) {
  const uint64_t nrec = table_bytes / (16 * F4);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  gather<U, F4><<<blocks, 256>>>(t, nrec, 1, out);   // warm
  CK(hipEventRecord(e0));
  gather<U, F4><<<blocks, 256>>>(t, nrec, iters, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double recs = (double)blocks * 256 * iters * U;
  printf("{\"case\": \"%s\", \"pattern\": \"independent\", \"table_MB\": %.1f, \"record_B\": %d, \"unroll\": %d, "
         "\"blocks\": %d, \"ms\": %.3f, \"Grec_per_s\": %.2f, \"useful_GBps\": %.1f}\n",
         tag, table_bytes / 1e6, 16 * F4, U, blocks, ms, recs / ms / 1e6, recs * 16 * F4 / ms / 1e6);
  fflush(stdout);
}

template <int F4>
void run_chase(float4* t, uint64_t table_bytes, int blocks, int iters, float* out, const char* tag) {
  const uint64_t nrec = table_bytes / (16 * F4);
  init_links<F4><<<(unsigned)((nrec + 255) / 256), 256>>>(t, nrec);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  chase<F4><<<blocks, 256>>>(t, nrec, 8, out);   // warm
  CK(hipEventRecord(e0));
  chase<F4><<<blocks, 256>>>(t, nrec, iters, out);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double recs = (double)blocks * 256 * iters;
  printf("{\"case\": \"%s\", \"pattern\": \"dependent_chain\", \"table_MB\": %.1f, \"record_B\": %d, \"blocks\": %d, "
         "\"iters\": %d, \"ms\": %.3f, \"Grec_per_s\": %.2f, \"useful_GBps\": %.1f, "
         "\"latency_ns_per_load\": %.1f}\n",
         tag, table_bytes / 1e6, 16 * F4, blocks, iters, ms, recs / ms / 1e6, recs * 16 * F4 / ms / 1e6,
         ms * 1e6 / iters);
  fflush(stdout);
}

int main(int argc, char** argv) {
  // "mlp": the ceilings at the trace kernel's memory-level parallelism
  // (VERDICT r04 item 4): 4-MB and 1-GB tables of 64-B records, four 16-B
  // loads per record per lane, 1/2/4 dependent chains per lane and
  // independent records 2/4/8 in flight, at 6 workgroups of 256 per CU
  if (argc > 1 && argv[1][0] == 'm') {
    const uint64_t big = 1ull << 30;
    float4* t = nullptr;
    float* out = nullptr;
    CK(hipMalloc((void**)&t, big));
    CK(hipMalloc((void**)&out, 64));
    CK(hipMemset(t, 0, big));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = cus * 6;
    struct Tab { uint64_t bytes; const char* tag; int iters; } tabs[] = {{4ull << 20, "l2_4MB", 1024},
                                                                         {1ull << 30, "hbm1GB", 128}};
    for (const Tab& tb : tabs) {
      run_chase_multi<4, 1>(t, tb.bytes, blocks, tb.iters, out, tb.tag);
      run_chase_multi<4, 2>(t, tb.bytes, blocks, tb.iters, out, tb.tag);
      run_chase_multi<4, 4>(t, tb.bytes, blocks, tb.iters, out, tb.tag);
      run_gather32<2, 4>(t, tb.bytes, blocks, tb.iters, out, tb.tag);
      run_gather32<4, 4>(t, tb.bytes, blocks, tb.iters, out, tb.tag);
      run_gather32<8, 4>(t, tb.bytes, blocks, tb.iters / 2, out, tb.tag);
    }
    return 0;
  }
  const bool quick = argc > 1;   // only the chase cases (the l2_gather roofline)
  const uint64_t big = 4ull << 30;
  float4* t = nullptr;
  float* out = nullptr;
  CK(hipMalloc((void**)&t, big));
  CK(hipMalloc((void**)&out, 64));
  CK(hipMemset(t, 0, big));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  if (!quick) {
    for (int occ : {4, 8}) {
      const int blocks = cus * occ;
      run<1, 2>(t, big, blocks, 64, out, "hbm");
      run<8, 2>(t, big, blocks, 16, out, "hbm");
      run<8, 4>(t, big, blocks, 16, out, "hbm64B");
      run<8, 2>(t, 64ull << 20, blocks, 64, out, "mall64MB");
      run<8, 4>(t, 64ull << 20, blocks, 64, out, "mall64MB");
      run<8, 2>(t, 2ull << 20, blocks, 256, out, "l2_2MB");
      run<8, 4>(t, 2ull << 20, blocks, 256, out, "l2_2MB");
      run<8, 4>(t, 4ull << 20, blocks, 256, out, "l2_4MB");
    }
  }
  // dependent chains at the trace kernel's occupancy (6 workgroups of 256 per CU)
  const int blocks = cus * 6;
  run_chase<4>(t, 2ull << 20, blocks, 2048, out, "l2_2MB");
  run_chase<4>(t, 4ull << 20, blocks, 2048, out, "l2_4MB");
  run_chase<4>(t, 64ull << 20, blocks, 512, out, "mall64MB");
  run_chase<4>(t, 1ull << 30, blocks, 256, out, "hbm1GB");
  run_chase<2>(t, 2ull << 20, blocks, 2048, out, "l2_2MB");
  return 0;
}
