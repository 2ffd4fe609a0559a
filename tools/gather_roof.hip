// tools/gather_roof.hip — ceiling of random small-record gathers on MI355X
// (the access pattern of BVH traversal over a scene far larger than the
// caches).  Every lane issues U independent random loads of a 32-B record
// (2 x float4, the node layout) per iteration from a table of T bytes, for
// ITER iterations; reports useful GB/s (32 B per record) and the 64-B
// granule rate.  Not part of the product.
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
  printf("{\"case\": \"%s\", \"table_MB\": %.0f, \"record_B\": %d, \"unroll\": %d, \"blocks\": %d, \"ms\": %.3f, "
         "\"Grec_per_s\": %.2f, \"useful_GBps\": %.1f}\n",
         tag, table_bytes / 1e6, 16 * F4, U, blocks, ms, recs / ms / 1e6, recs * 16 * F4 / ms / 1e6);
  fflush(stdout);
}

int main() {
  const uint64_t big = 4ull << 30;
  float4* t = nullptr;
  float* out = nullptr;
  CK(hipMalloc((void**)&t, big));
  CK(hipMalloc((void**)&out, 64));
  CK(hipMemset(t, 0, big));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int occ : {4, 8}) {
    const int blocks = cus * occ;
    run<1, 2>(t, big, blocks, 64, out, "hbm");
    run<4, 2>(t, big, blocks, 32, out, "hbm");
    run<8, 2>(t, big, blocks, 16, out, "hbm");
    run<8, 4>(t, big, blocks, 16, out, "hbm64B");
    run<8, 2>(t, 64ull << 20, blocks, 16, out, "mall64MB");
    run<8, 2>(t, 2ull << 20, blocks, 16, out, "l2_2MB");
  }
  return 0;
}
