// primitives.hip -- device-wide building blocks on gfx950 (wave64):
//   * exclusive scan of u32 counts (reduce -> scan block sums -> downsweep),
//   * stable LSD radix sort of (key, u32 value[, u32 value]) tuples, 8-bit
//     digits, register-resident tiles of 4096 keys per 256-thread workgroup,
//     XCD-aware tile order, stable in-wave ranking from ballots,
//   * small helpers (iota, u64 max).
#include <cstdlib>

#include "common.h"
#include "radix_tile.h"

namespace shd {

// ============================================================ scan
constexpr int kScanItems = 4;                     // per thread
constexpr int kScanTile = kBlock * kScanItems;    // 1024

__device__ inline uint32_t wave_incl_scan(uint32_t v) {
  int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

// Block-wide exclusive scan of one value per thread; returns block total in *total.
__device__ inline uint32_t block_excl_scan(uint32_t v, uint32_t* lds4, uint32_t* total) {
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = wave_incl_scan(v);
  if (lane == 63) lds4[w] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < kBlock / 64; i++) {
    uint32_t s = lds4[i];
    if (i < w) pre += s;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + inc - v;
}

__global__ __launch_bounds__(kBlock) void k_scan_reduce(const uint32_t* in, int64_t n, uint32_t* bsum) {
  __shared__ uint32_t lds[4];
  int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; i++)
    if (base + i < n) s += in[base + i];
  uint32_t tot;
  block_excl_scan(s, lds, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_scan_down(const uint32_t* in, int64_t n, const uint32_t* boff,
                                                      uint32_t* out, uint32_t* total_dev) {
  __shared__ uint32_t lds[4];
  int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    v[i] = (base + i < n) ? in[base + i] : 0;
    s += v[i];
  }
  uint32_t tot;
  uint32_t pre = block_excl_scan(s, lds, &tot) + (boff ? boff[blockIdx.x] : 0);
#pragma unroll
  for (int i = 0; i < kScanItems; i++) {
    if (base + i < n) out[base + i] = pre;
    pre += v[i];
  }
  if (total_dev && blockIdx.x == gridDim.x - 1 && threadIdx.x == kBlock - 1) *total_dev = pre;
}

static void scan_rec(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, uint32_t* scratch,
                     hipStream_t s) {
  int64_t nb = ceil_div(n, kScanTile);
  if (nb <= 1) {
    hipLaunchKernelGGL(k_scan_down, dim3(1), dim3(kBlock), 0, s, in, n, (const uint32_t*)nullptr, out, total_dev);
    SHD_CHECK_LAUNCH();
    return;
  }
  uint32_t* bsum = scratch;
  uint32_t* boff = scratch + nb;
  hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, bsum);
  SHD_CHECK_LAUNCH();
  scan_rec(bsum, boff, nb, nullptr, scratch + 2 * nb, s);
  hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, (const uint32_t*)boff, out,
                     total_dev);
  SHD_CHECK_LAUNCH();
}

static int64_t scan_need(int64_t n) {
  // 2*nb words at each recursion level (geometric) + slack
  int64_t need = 0, m = n;
  while (m > kScanTile) {
    int64_t nb = ceil_div(m, kScanTile);
    need += 2 * nb;
    m = nb;
  }
  return need + 64;
}

static void scan_raw(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, uint32_t* scratch,
                     hipStream_t s) {
  if (n <= 0) {
    if (total_dev) SHD_HIP(hipMemsetAsync(total_dev, 0, 4, s));
    return;
  }
  scan_rec(in, out, n, total_dev, scratch, s);
}

void scan_exclusive_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev, DevBuf& scratch,
                        hipStream_t s) {
  scratch.reserve(scan_need(n) * sizeof(uint32_t));
  scan_raw(in, out, n, total_dev, scratch.as<uint32_t>(), s);
}

// ============================================================ radix sort
// (tile constants, digit helpers and the in-tile scatter: radix_tile.h)

template <class K, int R, bool H>
__global__ __launch_bounds__(kRsBlock) void k_rs_hist(const K* __restrict__ keys, int64_t n, int shift,
                                                      uint32_t* __restrict__ hist, int nb, int xcd, K kb) {
  __shared__ uint32_t h[kRsWaves][256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kRsWaves * 256; i += kRsBlock) (&h[0][0])[i] = 0;
  const int tile = xcd ? rs_tile_of(blockIdx.x, nb) : (int)blockIdx.x;
  const int64_t wb = (int64_t)tile * rs_tile(R) + (int64_t)w * 64 * R;
  bool done = false;
  if constexpr (sizeof(K) == 4 && R % 4 == 0) {
    if ((int64_t)(tile + 1) * rs_tile(R) <= n) {
      // full tile of 32-bit keys: 16-byte loads (counting needs no order)
      const uint4* kv = reinterpret_cast<const uint4*>(keys + wb);
      uint4 q[R / 4];
#pragma unroll
      for (int i = 0; i < R / 4; i++) q[i] = kv[i * 64 + lane];
      __syncthreads();
#pragma unroll
      for (int i = 0; i < R / 4; i++) {
        atomicAdd(&h[w][rs_hdigit<H>((K)q[i].x, shift, kb)], 1u);
        atomicAdd(&h[w][rs_hdigit<H>((K)q[i].y, shift, kb)], 1u);
        atomicAdd(&h[w][rs_hdigit<H>((K)q[i].z, shift, kb)], 1u);
        atomicAdd(&h[w][rs_hdigit<H>((K)q[i].w, shift, kb)], 1u);
      }
      done = true;
    }
  }
  if (!done) {
    K k[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int64_t idx = wb + r * 64 + lane;
      k[r] = keys[idx < n ? idx : n - 1];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; r++)
      if (wb + r * 64 + lane < n) atomicAdd(&h[w][rs_hdigit<H>(k[r], shift, kb)], 1u);
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < kRsWaves; i++) c += h[i][tid];
    hist[(int64_t)tid * nb + tile] = c;
  }
}

// Exclusive scan of one digit's row of per-tile counts (one workgroup per
// digit): offs[d*nb + t] = digit d's count in tiles before t, total[d] = its
// count in the whole array.  The scatter adds the exclusive prefix of the 256
// digit totals itself, so a pass is three launches (hist, row scan, scatter).
__global__ __launch_bounds__(kRsBlock) void k_rs_digit_scan(const uint32_t* __restrict__ hist, int nb,
                                                            uint32_t* __restrict__ offs, uint32_t* __restrict__ total) {
  constexpr int kRowLds = 16384;   // rows up to 16k tiles (~100M keys) are staged in LDS
  __shared__ uint32_t wsum[kRsWaves];
  __shared__ uint32_t lrow[kRowLds];
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint32_t* grow = hist + (int64_t)d * nb;
  uint32_t* orow = offs + (int64_t)d * nb;
  // coalesced copy of the row into LDS; each thread then walks a contiguous run
  const bool staged = nb <= kRowLds;
  if (staged)
    for (int t = tid; t < nb; t += kRsBlock) lrow[t] = grow[t];
  __syncthreads();
  const uint32_t* row = staged ? lrow : grow;
  const int per = (nb + kRsBlock - 1) / kRsBlock;   // contiguous run of tiles per thread
  const int a = tid * per, b = a + per < nb ? a + per : nb;
  uint32_t s = 0;
  for (int t = a; t < b; t++) s += row[t];
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(inc, o, 64);
    if (lane >= o) inc += x;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = inc - s, tot = 0;
  for (int i = 0; i < kRsWaves; i++) {
    if (i < w) pre += wsum[i];
    tot += wsum[i];
  }
  for (int t = a; t < b; t++) {
    const uint32_t c = row[t];
    orow[t] = pre;
    pre += c;
  }
  if (tid == 0) total[d] = tot;
}

template <class K, int R, bool P2, bool H>
__global__ __launch_bounds__(kRsBlock) void k_rs_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                         const uint32_t* __restrict__ win, K* __restrict__ kout,
                                                         uint32_t* __restrict__ vout, uint32_t* __restrict__ wout,
                                                         int64_t n, int shift, const uint32_t* __restrict__ hist,
                                                         const uint32_t* __restrict__ offs,
                                                         const uint32_t* __restrict__ dtotal, int nb, int xcd,
                                                         K kb) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = xcd ? rs_tile_of(blockIdx.x, nb) : (int)blockIdx.x;
  const int64_t t0 = (int64_t)tile * rs_tile(R);
  const int64_t wb = t0 + (int64_t)w * 64 * R;
  // this tile's histogram column and global digit offsets are loaded first:
  // the digit prefix then waits only for them, while the key loads issued
  // after them are still in flight (in-order vmcnt)
  const uint32_t c = tid < 256 ? hist[(int64_t)tid * nb + tile] : 0u;
  const uint32_t gr = tid < 256 ? offs[(int64_t)tid * nb + tile] : 0u;
  const uint32_t dt = tid < 256 ? dtotal[tid] : 0u;
  K k[R];
  uint32_t v[R];
  uint32_t x[P2 ? R : 1];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int64_t idx = wb + r * 64 + lane;
    const int64_t li = idx < n ? idx : n - 1;
    k[r] = kin[li];
    v[r] = vin[li];
    if (P2) x[r] = win[li];
  }
  rs_scatter_tile<K, R, P2, H>(k, v, x, n, t0, wb, shift, c, gr, dt, kb, kout, vout, wout);
}

template <class K, int R, bool P2, bool H = false>
static void radix_sort_run(K* keys, uint32_t* vals, uint32_t* w, K* keys_alt, uint32_t* vals_alt, uint32_t* w_alt,
                           int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& in_alt, K kb = 0,
                           int shift0 = 0) {
  in_alt = false;
  if (n <= 1 || bits <= 0) return;
  // k_rs_hist reads full tiles of 32-bit keys with 16-byte loads
  if ((reinterpret_cast<uintptr_t>(keys) | reinterpret_cast<uintptr_t>(keys_alt)) & 15)
    throw Error(SHD_E_ARG, "radix sort: key arrays must be 16-byte aligned");
  const int nb = (int)ceil_div(n, rs_tile(R));
  const int64_t nh = (int64_t)nb * 256;
  // scratch layout: hist[nh] | offs[nh] | digit totals[256]
  const size_t need = (size_t)(2 * nh + 256) * sizeof(uint32_t);
  scratch.reserve(need);
  uint32_t* hist = scratch.as<uint32_t>();
  uint32_t* offs = hist + nh;
  uint32_t* dtot = offs + nh;
  const int xcd = getenv("SHD_RS_NOXCD") ? 0 : 1;   // A/B switch for the tile order
  K* ki = keys; uint32_t* vi = vals; uint32_t* wi = w;
  K* ko = keys_alt; uint32_t* vo = vals_alt; uint32_t* wo = w_alt;
  for (int shift = shift0; shift < bits; shift += 8) {
    hipLaunchKernelGGL((k_rs_hist<K, R, H>), dim3(nb), dim3(kRsBlock), 0, s, (const K*)ki, n, shift, hist, nb, xcd, kb);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_rs_digit_scan, dim3(256), dim3(kRsBlock), 0, s, (const uint32_t*)hist, nb, offs, dtot);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL((k_rs_scatter<K, R, P2, H>), dim3(nb), dim3(kRsBlock), 0, s, (const K*)ki, (const uint32_t*)vi,
                       (const uint32_t*)wi, ko, vo, wo, n, shift, (const uint32_t*)hist, (const uint32_t*)offs,
                       (const uint32_t*)dtot, nb, xcd, kb);
    SHD_CHECK_LAUNCH();
    std::swap(ki, ko);
    std::swap(vi, vo);
    std::swap(wi, wo);
    in_alt = !in_alt;
  }
}

void radix_digit_scan(const uint32_t* hist, int nb, uint32_t* offs, uint32_t* dtot, hipStream_t s) {
  hipLaunchKernelGGL(k_rs_digit_scan, dim3(256), dim3(kRsBlock), 0, s, hist, nb, offs, dtot);
  SHD_CHECK_LAUNCH();
}

const uint32_t* radix_digit_totals(const DevBuf& scratch, int64_t n) {
  const int64_t nh = ceil_div(n, rs_tile(kRsRounds)) * 256;   // scratch layout of radix_sort_run
  return scratch.as<uint32_t>() + 2 * nh;
}

void radix_sort_pairs_u32(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt, int64_t n,
                          int bits, DevBuf& scratch, hipStream_t s, bool& in_alt) {
  radix_sort_run<uint32_t, kRsRounds, false>(keys, vals, nullptr, keys_alt, vals_alt, nullptr, n, bits, scratch, s,
                                             in_alt);
}

void radix_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt, int64_t n,
                          int bits, DevBuf& scratch, hipStream_t s, bool& in_alt) {
  radix_sort_run<uint64_t, kRsRounds, false>(keys, vals, nullptr, keys_alt, vals_alt, nullptr, n, bits, scratch, s,
                                             in_alt);
}

void radix_sort_triples_u32(uint32_t* keys, uint32_t* vals, uint32_t* w, uint32_t* keys_alt, uint32_t* vals_alt,
                            uint32_t* w_alt, int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& in_alt,
                            bool hashed, uint32_t kbase, int shift0) {
  if (hashed)
    radix_sort_run<uint32_t, kRsRounds, true, true>(keys, vals, w, keys_alt, vals_alt, w_alt, n, bits, scratch, s,
                                                    in_alt, 0u, shift0);
  else
    radix_sort_run<uint32_t, kRsRounds, true>(keys, vals, w, keys_alt, vals_alt, w_alt, n, bits, scratch, s, in_alt,
                                              kbase, shift0);
}

void radix_sort_triples_u64(uint64_t* keys, uint32_t* vals, uint32_t* w, uint64_t* keys_alt, uint32_t* vals_alt,
                            uint32_t* w_alt, int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& in_alt) {
  radix_sort_run<uint64_t, kRsRounds, true>(keys, vals, w, keys_alt, vals_alt, w_alt, n, bits, scratch, s, in_alt);
}

// ============================================================ helpers
__global__ void k_iota(uint32_t* out, int64_t n, uint32_t base) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = base + (uint32_t)i;
}

void fill_iota_u32(uint32_t* out, int64_t n, uint32_t base, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kBlock), 0, s, out, n, base);
  SHD_CHECK_LAUNCH();
}

__global__ __launch_bounds__(kBlock) void k_max_u64(const uint64_t* in, int64_t n, unsigned long long* out) {
  unsigned long long m = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    m = in[i] > m ? in[i] : m;
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(m, o, 64);
    m = t > m ? t : m;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(out, m);
}

void reduce_max_u64(const uint64_t* in, int64_t n, uint64_t* out_dev, hipStream_t s) {
  SHD_HIP(hipMemsetAsync(out_dev, 0, 8, s));
  if (n <= 0) return;
  hipLaunchKernelGGL(k_max_u64, dim3(grid_for(n, 4, 2048)), dim3(kBlock), 0, s, in, n,
                     (unsigned long long*)out_dev);
  SHD_CHECK_LAUNCH();
}

}  // namespace shd
