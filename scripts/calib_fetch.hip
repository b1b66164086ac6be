// calib_fetch.hip -- calibrates rocprofv3's FETCH_SIZE on gfx950 per access
// shape (scripts/pmc_summary.py applies the factors).  Each kernel reads a
// known number of bytes / elements of a 1 GiB buffer (far past the 256 MiB
// Infinity Cache, so every line comes from HBM):
//   k_stream16  16 B per lane, coalesced            1 GiB
//   k_stream4    4 B per lane, coalesced            1 GiB
//   k_gather4    4 B at a random index per lane     16 Mi elements
//   k_gather8    8 B at a random index per lane     16 Mi elements
// Run under `rocprofv3 --pmc FETCH_SIZE --kernel-trace` (own pass) and divide
// each dispatch's FETCH_SIZE (KiB) by the known count.
//   hipcc --offload-arch=gfx950 -O3 -o scripts/calib_fetch scripts/calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_stream16(const uint4* __restrict__ a, size_t n, unsigned* __restrict__ out) {
  unsigned s = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;   // keeps the loads
}

__global__ void k_stream4(const unsigned* __restrict__ a, size_t n, unsigned* __restrict__ out) {
  unsigned s = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s ^= a[i];
  if (s == 0x12345678u) out[0] = s;
}

__global__ void k_gather4(const unsigned* __restrict__ a, size_t n, size_t m, unsigned* __restrict__ out) {
  unsigned s = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x)
    s ^= a[mix(i) % n];
  if (s == 0x12345678u) out[0] = s;
}

__global__ void k_gather8(const uint64_t* __restrict__ a, size_t n, size_t m, unsigned* __restrict__ out) {
  uint64_t s = 0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (size_t)gridDim.x * blockDim.x)
    s ^= a[mix(i) % n];
  if (s == 0x12345678ull) out[0] = (unsigned)s;
}

int main() {
  const size_t bytes = (size_t)1 << 30;   // 1 GiB
  const size_t gathers = (size_t)1 << 24;
  void* buf = nullptr;
  unsigned* out = nullptr;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, bytes));
  const int grid = 256 * 32, block = 256;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(block), 0, 0, (const uint4*)buf, bytes / 16, out);
    hipLaunchKernelGGL(k_stream4, dim3(grid), dim3(block), 0, 0, (const unsigned*)buf, bytes / 4, out);
    hipLaunchKernelGGL(k_gather4, dim3(grid), dim3(block), 0, 0, (const unsigned*)buf, bytes / 4, gathers, out);
    hipLaunchKernelGGL(k_gather8, dim3(grid), dim3(block), 0, 0, (const uint64_t*)buf, bytes / 8, gathers, out);
    CK(hipGetLastError());
  }
  CK(hipDeviceSynchronize());
  printf("calib_fetch: stream16/stream4 read %zu bytes, gather4/gather8 %zu elements each, 2 reps\n", bytes, gathers);
  CK(hipFree(buf));
  CK(hipFree(out));
  return 0;
}
