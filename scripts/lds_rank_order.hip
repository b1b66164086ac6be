// Probe: does ds_add_rtn_u32 (LDS atomicAdd with return) hand out the old
// values of lanes that hit one address in LANE ORDER within a wave
// instruction?  If so, an LDS atomic ranks a wave's keys by digit stably
// (radix ranking without the 8-ballot peer masks).  Counts, over many
// trials and collision patterns, lanes whose returned rank is below a
// lower-numbered lane's of the same address.  Build: hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void k_probe(unsigned long long* bad, unsigned long long* total, int trials, unsigned mask) {
  __shared__ uint32_t cnt[4][256];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  unsigned long long nbad = 0, ntot = 0;
  for (int t = 0; t < trials; t++) {
    for (int i = lane; i < 256; i += 64) cnt[w][i] = 0;
    __builtin_amdgcn_wave_barrier();
    uint32_t h = (uint32_t)(blockIdx.x * 1315423911u + t * 2654435761u + lane * 97u + w * 7919u);
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    const uint32_t d = h & mask;
    const uint32_t r = atomicAdd(&cnt[w][d], 1u);
    __builtin_amdgcn_wave_barrier();
    // every lower lane with the same digit must hold a lower rank
    for (int j = 0; j < 64; j++) {
      const uint32_t dj = __shfl(d, j, 64), rj = __shfl(r, j, 64);
      if (j < lane && dj == d) {
        ntot++;
        if (rj > r) nbad++;
      }
    }
  }
  atomicAdd(bad, nbad);
  atomicAdd(total, ntot);
}

int main() {
  unsigned long long *d, h[2];
  hipMalloc(&d, 16);
  const unsigned masks[] = {0u, 1u, 3u, 15u, 63u, 255u};
  int fails = 0;
  for (unsigned m : masks) {
    hipMemset(d, 0, 16);
    hipLaunchKernelGGL(k_probe, dim3(2048), dim3(256), 0, 0, d, d + 1, 64, m);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("mask %3u: same-address lane pairs %llu, out of lane order %llu\n", m, h[1], h[0]);
    fails += h[0] != 0;
  }
  printf(fails ? "LDS atomic ranks NOT in lane order\n" : "LDS atomic ranks in lane order\n");
  return fails;
}
