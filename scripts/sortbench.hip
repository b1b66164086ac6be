// sortbench.hip -- timing harness for the LSD radix sort in
// siddhi_amd/csrc/primitives.hip (tile shape chosen at compile time with
// -DSHD_RS_ROUNDS / -DSHD_RS_BLOCK).  Sorts n (key < kmax, row, u32 payload)
// triples like the pattern engine's key sort, checks order + stability on
// the device result, prints one JSON line.  Built by scripts/build_sortbench.sh.
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../siddhi_amd/csrc/primitives.hip"

namespace shd {
void check_launch(const char*, int) {}
}  // namespace shd

using namespace shd;

__global__ void k_gen(uint32_t* k, uint32_t* v, uint32_t* w, int64_t n, uint32_t kmax, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = seed + (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    k[i] = (uint32_t)(z % kmax);
    v[i] = (uint32_t)i;
    w[i] = (uint32_t)(z >> 32);
  }
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 50000000;
  const uint32_t kmax = argc > 2 ? (uint32_t)atoll(argv[2]) : 10000000u;
  const int iters = argc > 3 ? atoi(argv[3]) : 5;
  const bool triples = argc > 4 ? atoi(argv[4]) != 0 : true;
  int bits = 0;
  while (bits < 32 && ((kmax - 1) >> bits)) bits++;
  DevBuf k, v, w, ka, va, wa, scratch;
  k.reserve(n * 4); v.reserve(n * 4); w.reserve(n * 4);
  ka.reserve(n * 4); va.reserve(n * 4); wa.reserve(n * 4);
  hipStream_t s;
  SHD_HIP(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  SHD_HIP(hipEventCreate(&e0));
  SHD_HIP(hipEventCreate(&e1));
  float best = 1e30f, total = 0.f;
  bool in_alt = false;
  for (int it = 0; it <= iters; it++) {
    hipLaunchKernelGGL(k_gen, dim3(4096), dim3(256), 0, s, k.as<uint32_t>(), v.as<uint32_t>(), w.as<uint32_t>(), n,
                       kmax, 1234567ull + it);
    SHD_HIP(hipEventRecord(e0, s));
    if (triples)
      radix_sort_triples_u32(k.as<uint32_t>(), v.as<uint32_t>(), w.as<uint32_t>(), ka.as<uint32_t>(),
                             va.as<uint32_t>(), wa.as<uint32_t>(), n, bits, scratch, s, in_alt);
    else
      radix_sort_pairs_u32(k.as<uint32_t>(), v.as<uint32_t>(), ka.as<uint32_t>(), va.as<uint32_t>(), n, bits,
                           scratch, s, in_alt);
    SHD_HIP(hipEventRecord(e1, s));
    SHD_HIP(hipEventSynchronize(e1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, e0, e1));
    if (it > 0) {
      total += ms;
      best = ms < best ? ms : best;
    }
  }
  // verify the last sort: keys non-decreasing, rows increasing within a key,
  // payload consistent with the generator
  std::vector<uint32_t> hk(n), hv(n), hw(n);
  SHD_HIP(hipMemcpy(hk.data(), (in_alt ? ka : k).p, n * 4, hipMemcpyDeviceToHost));
  SHD_HIP(hipMemcpy(hv.data(), (in_alt ? va : v).p, n * 4, hipMemcpyDeviceToHost));
  SHD_HIP(hipMemcpy(hw.data(), (in_alt ? wa : w).p, n * 4, hipMemcpyDeviceToHost));
  std::vector<uint8_t> seen(n, 0);
  int64_t bad = 0;
  for (int64_t i = 0; i < n; i++) {
    if (hv[i] >= (uint64_t)n || seen[hv[i]]) { bad++; continue; }
    seen[hv[i]] = 1;
    if (i > 0 && (hk[i] < hk[i - 1] || (hk[i] == hk[i - 1] && hv[i] < hv[i - 1]))) bad++;
  }
  const double per_pass_bytes = (double)n * (triples ? 28.0 : 20.0);   // hist read 4 + scatter r/w
  const int passes = (bits + 7) / 8;
  printf("{\"rounds\": %d, \"block\": %d, \"n\": %lld, \"bits\": %d, \"triples\": %d, \"ms_best\": %.4f, "
         "\"ms_mean\": %.4f, \"alg_GBps\": %.1f, \"bad\": %lld, \"xcd\": %d}\n",
         kRsRounds, kRsBlock, (long long)n, bits, (int)triples, best, total / iters,
         per_pass_bytes * passes / (best * 1e6), (long long)bad, getenv("SHD_RS_NOXCD") ? 0 : 1);
  return bad ? 1 : 0;
}
