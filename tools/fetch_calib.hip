// tools/fetch_calib.hip — calibrates rocprofv3 FETCH_SIZE against known byte
// counts for the access patterns the path tracer's large-scene kernels use
// (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of the bytes of a 16-B/lane
// streaming read; "other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern").  Not part of the product.
//
//   stream16 : every lane reads consecutive float4 of a 2 GiB buffer once
//   gather32 : every lane reads one random 32-B record (2 x float4, the BVH
//              node layout) of a 4 GiB table, each record at most once
//   gather48 : the same with 48-B records (3 x float4, the triangle records)
//
// The tables are far above the 256 MiB Infinity Cache and every line is read
// at most once per launch, so the memory-side byte count should be the
// algorithmic one rounded up to the fetch granule.  Prints one JSON line per
// kernel with the algorithmic bytes; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib
// and divide.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void stream16(const float4* __restrict__ a, size_t n, float* out) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.0f) out[0] = s;
}

// record r = perm(g): a multiplicative permutation of [0, nrec) (nrec a power
// of two, odd multiplier), so every record is read at most once
template <int F4>
__global__ void gather(const float4* __restrict__ t, uint64_t nrec, uint64_t nloads, float* out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (g >= nloads) return;
  const uint64_t r = (g * 0x9E3779B97F4A7C15ull) & (nrec - 1);
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < F4; ++k) {
    const float4 v = t[r * F4 + k];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.0f) out[0] = s;
}

int main() {
  const size_t stream_bytes = 2ull << 30, table_bytes = 6ull << 30;
  float4* buf = nullptr;
  float* out = nullptr;
  CK(hipMalloc((void**)&buf, table_bytes));
  CK(hipMalloc((void**)&out, 64));
  CK(hipMemset(buf, 0, table_bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms = 0.0f;
  {
    const size_t n = stream_bytes / 16;
    CK(hipEventRecord(e0));
    stream16<<<256 * 64, 256>>>(buf, n, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"stream16\", \"bytes\": %zu, \"ms\": %.4f}\n", stream_bytes, ms);
  }
  // 32-B records: 4 GiB table = 2^27 records, read 2^25 of them (1 GiB)
  {
    const uint64_t nrec = (4ull << 30) / 32, nloads = 1ull << 25;
    CK(hipEventRecord(e0));
    gather<2><<<(unsigned)(nloads / 256), 256>>>(buf, nrec, nloads, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"gather<2>\", \"bytes\": %llu, \"ms\": %.4f}\n", (unsigned long long)(nloads * 32), ms);
  }
  // 48-B records: 2^27 records of a 6 GiB table, read 2^25
  {
    const uint64_t nrec = 1ull << 27, nloads = 1ull << 25;
    CK(hipEventRecord(e0));
    gather<3><<<(unsigned)(nloads / 256), 256>>>(buf, nrec, nloads, out);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"kernel\": \"gather<3>\", \"bytes\": %llu, \"ms\": %.4f}\n", (unsigned long long)(nloads * 48), ms);
  }
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
