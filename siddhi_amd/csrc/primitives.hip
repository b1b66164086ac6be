// primitives.hip -- device-wide building blocks on gfx950 (wave64):
//   * exclusive scan of u32 counts (reduce -> scan block sums -> downsweep),
//   * stable LSD radix sort of (key, u32 value) pairs, 8-bit digits, tiles of
//     4096 keys per 256-thread workgroup, per-wave LDS histograms, stable
//     in-tile ranking from eight 64-bit ballots per round,
//   * small helpers (iota, u64 max).
#include "common.h"

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
constexpr int kRsRounds = 16;
constexpr int kRsTile = kBlock * kRsRounds;   // 4096 keys per workgroup

template <class K>
__global__ __launch_bounds__(kBlock) void k_rs_hist(const K* keys, int64_t n, int shift, uint32_t* hist, int nb) {
  __shared__ uint32_t h[4][256];
  int tid = threadIdx.x, w = tid >> 6;
#pragma unroll
  for (int i = 0; i < 4; i++) h[i][tid] = 0;
  __syncthreads();
  int64_t t0 = (int64_t)blockIdx.x * kRsTile;
  for (int r = 0; r < kRsRounds; r++) {
    int64_t idx = t0 + r * kBlock + tid;
    if (idx < n) {
      uint32_t d = (uint32_t)((keys[idx] >> shift) & 255u);
      atomicAdd(&h[w][d], 1u);
    }
  }
  __syncthreads();
  hist[(int64_t)tid * nb + blockIdx.x] = h[0][tid] + h[1][tid] + h[2][tid] + h[3][tid];
}

// Scatter one 4096-key tile: stable in-tile ranking (ballots), the tile is
// first reordered by digit in LDS, then written out so that consecutive lanes
// store consecutive addresses of one digit bucket (coalesced runs instead of
// one scattered dword per key).
template <class K>
__global__ __launch_bounds__(kBlock) void k_rs_scatter(const K* kin, const uint32_t* vin, K* kout, uint32_t* vout,
                                                       int64_t n, int shift, const uint32_t* hist,
                                                       const uint32_t* offs, int nb) {
  __shared__ K sk[kRsTile];
  __shared__ uint32_t sv[kRsTile];
  __shared__ uint32_t lpre[256];    // tile-local first position of each digit
  __shared__ uint32_t lbase[256];   // running tile-local position per digit
  __shared__ uint32_t gbase[256];   // global first position of this tile's digit run
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t wsum[4];
  int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int64_t t0 = (int64_t)blockIdx.x * kRsTile;
  // tile-local exclusive prefix over digits from this tile's histogram column
  {
    uint32_t c = hist[(int64_t)tid * nb + blockIdx.x];
    uint32_t inc = c;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (int i = 0; i < w; i++) pre += wsum[i];
    lpre[tid] = pre + inc - c;
    lbase[tid] = pre + inc - c;
    gbase[tid] = offs[(int64_t)tid * nb + blockIdx.x];
  }
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int r = 0; r < kRsRounds; r++) {
    int64_t idx = t0 + r * kBlock + tid;
    bool valid = idx < n;
    K k = valid ? kin[idx] : (K)0;
    uint32_t v = valid ? vin[idx] : 0u;
    uint32_t d = (uint32_t)((k >> shift) & 255u);
#pragma unroll
    for (int i = 0; i < 4; i++) wcnt[i][tid] = 0;
    __syncthreads();
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      bool bit = (d >> b) & 1u;
      uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    int rank = __popcll(peers & lt);
    if (valid && (peers & lt) == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t pos = lbase[d] + rank;
      for (int ww = 0; ww < w; ww++) pos += wcnt[ww][d];
      sk[pos] = k;
      sv[pos] = v;
    }
    __syncthreads();
    lbase[tid] += wcnt[0][tid] + wcnt[1][tid] + wcnt[2][tid] + wcnt[3][tid];
  }
  __syncthreads();
  int64_t tile_n = n - t0 < kRsTile ? n - t0 : kRsTile;
  for (int i = tid; i < tile_n; i += kBlock) {
    K k = sk[i];
    uint32_t d = (uint32_t)((k >> shift) & 255u);
    uint32_t o = gbase[d] + (uint32_t)i - lpre[d];
    kout[o] = k;
    vout[o] = sv[i];
  }
}

template <class K>
static void radix_sort_impl(K* keys, uint32_t* vals, K* keys_alt, uint32_t* vals_alt, int64_t n, int bits,
                            DevBuf& scratch, hipStream_t s, bool& in_alt) {
  in_alt = false;
  if (n <= 1 || bits <= 0) return;
  int nb = (int)ceil_div(n, kRsTile);
  int64_t nh = (int64_t)nb * 256;
  // scratch layout: hist[nh] | offs[nh] | scan scratch
  size_t need = (size_t)(2 * nh + scan_need(nh)) * sizeof(uint32_t);
  scratch.reserve(need);
  uint32_t* hist = scratch.as<uint32_t>();
  uint32_t* offs = hist + nh;
  uint32_t* sscr = offs + nh;
  K* ki = keys; uint32_t* vi = vals; K* ko = keys_alt; uint32_t* vo = vals_alt;
  for (int shift = 0; shift < bits; shift += 8) {
    hipLaunchKernelGGL(k_rs_hist<K>, dim3(nb), dim3(kBlock), 0, s, (const K*)ki, n, shift, hist, nb);
    SHD_CHECK_LAUNCH();
    scan_raw(hist, offs, nh, nullptr, sscr, s);
    hipLaunchKernelGGL(k_rs_scatter<K>, dim3(nb), dim3(kBlock), 0, s, (const K*)ki, (const uint32_t*)vi, ko, vo, n,
                       shift, (const uint32_t*)hist, (const uint32_t*)offs, nb);
    SHD_CHECK_LAUNCH();
    std::swap(ki, ko);
    std::swap(vi, vo);
    in_alt = !in_alt;
  }
}

void radix_sort_pairs_u32(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt, int64_t n,
                          int bits, DevBuf& scratch, hipStream_t s, bool& in_alt) {
  radix_sort_impl<uint32_t>(keys, vals, keys_alt, vals_alt, n, bits, scratch, s, in_alt);
}

void radix_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt, int64_t n,
                          int bits, DevBuf& scratch, hipStream_t s, bool& in_alt) {
  radix_sort_impl<uint64_t>(keys, vals, keys_alt, vals_alt, n, bits, scratch, s, in_alt);
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
