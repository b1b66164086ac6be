// route.hip -- key-owner re-route of a micro-batch across ranks.
//
// Partitioned queries keep all state per partition key (PartitionStateHolder
// .getState, C/util/snapshot/state/PartitionStateHolder.java:43-48), so a rank
// may process exactly the events whose key it owns, in the reference's per-key
// arrival order and InputHandler-call membership.  Input that arrives
// round-robin is re-routed with ONE all-to-all per micro-batch; the two device
// passes around it are here:
//
//   shd_route_bucket  stable bucket-by-owner scatter of the batch's rows into
//                     one packed send buffer (owner = fmix32(key) % world, the
//                     same hash as siddhi_amd/exchange.py), plus the per-owner
//                     row counts (the all-to-all's split sizes);
//   shd_route_merge   the received rows (one segment per sender, each in the
//                     sender's arrival order) back into global arrival order,
//                     unpacked into typed columns, with the call boundaries:
//                     the global stream's calls are consecutive runs of
//                     `block` sequence numbers, so one workgroup per call
//                     merges the (at most `block`) rows every sender holds of
//                     that call in LDS, and its output offset is the sum of the
//                     senders' row counts before it -- a single coalesced pass,
//                     no sort.
//
// Wire format (8-byte words per row): the 8-byte columns in column order, then
// the 4-byte columns two per word, the last 4-byte slot holding the event's
// sequence offset seq - seq_lo (< 2^32).
#include <algorithm>

#include "common.h"

namespace shd {
namespace {

constexpr int kRouteMaxCols = 8;
constexpr int kRouteMaxWorld = 64;
constexpr int kRouteTileIters = 16;                        // rows per thread per tile
constexpr int64_t kRouteTile = (int64_t)kBlock * kRouteTileIters;
constexpr int64_t kRouteMaxBlock = 8192;                   // LDS sequence offsets per call

struct RouteLayout {
  const void* col[kRouteMaxCols];   // bucket: source columns; merge: destination columns
  int slot[kRouteMaxCols];          // word index (8-byte) or 2 * word + half (4-byte)
  int wide[kRouteMaxCols];          // 1: 8-byte column
  int ncols;
  int nwords;
  int seq_slot;                     // 2 * word + half of the sequence offset
};

__device__ __forceinline__ uint32_t fmix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ int owner_at(const void* key, int key_wide, int64_t i, int world) {
  const uint32_t k = key_wide ? (uint32_t)((const uint64_t*)key)[i] : ((const uint32_t*)key)[i];
  return (int)(fmix32(k) % (uint32_t)world);
}

// per-tile row counts per owner, owner-major: tcount[o * ntiles + tile]
__global__ __launch_bounds__(kBlock) void k_route_hist(const void* __restrict__ key, int key_wide, int64_t n,
                                                       int world, int64_t ntiles, uint32_t* __restrict__ tcount) {
  __shared__ uint32_t c[kRouteMaxWorld];
  if (threadIdx.x < kRouteMaxWorld) c[threadIdx.x] = 0;
  __syncthreads();
  const int64_t t0 = (int64_t)blockIdx.x * kRouteTile;
  for (int it = 0; it < kRouteTileIters; it++) {
    const int64_t i = t0 + (int64_t)it * kBlock + threadIdx.x;
    if (i < n) atomicAdd(&c[owner_at(key, key_wide, i, world)], 1u);
  }
  __syncthreads();
  if ((int)threadIdx.x < world) tcount[(int64_t)threadIdx.x * ntiles + blockIdx.x] = c[threadIdx.x];
}

// exclusive prefix over the owner-major tile counts (one block), and the
// per-owner totals (the all-to-all's send counts)
__global__ __launch_bounds__(1024) void k_route_scan(uint32_t* __restrict__ tcount, int64_t len, int world,
                                                     int64_t ntiles, int64_t* __restrict__ counts) {
  __shared__ uint64_t part[1024];
  const int64_t per = (len + 1023) / 1024;
  const int64_t a = (int64_t)threadIdx.x * per;
  const int64_t b = a + per < len ? a + per : len;
  uint64_t s = 0;
  for (int64_t i = a; i < b; i++) s += tcount[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const uint64_t v = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t run = part[threadIdx.x] - s;
  for (int64_t i = a; i < b; i++) {
    const uint32_t v = tcount[i];
    tcount[i] = (uint32_t)run;
    run += v;
  }
  __syncthreads();
  if ((int)threadIdx.x < world) {
    const int64_t o = threadIdx.x;
    const uint64_t lo = tcount[o * ntiles];
    const uint64_t hi = o + 1 < world ? (uint64_t)tcount[(o + 1) * ntiles] : (uint64_t)part[1023];
    counts[o] = (int64_t)(hi - lo);
  }
}

// Stable scatter: tile rows in order (iteration, wave, lane); each wave ranks its
// rows per owner with ballots, the waves' counts are prefixed in LDS.
__global__ __launch_bounds__(kBlock) void k_route_scatter(const void* __restrict__ key, int key_wide, int64_t n,
                                                          int world, int64_t ntiles,
                                                          const uint32_t* __restrict__ toff, RouteLayout L,
                                                          const int64_t* __restrict__ seq, int64_t seq_lo,
                                                          uint64_t* __restrict__ send) {
  __shared__ uint32_t base[kRouteMaxWorld];
  __shared__ uint32_t wcnt[kBlock / 64][kRouteMaxWorld];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if ((int)threadIdx.x < world) base[threadIdx.x] = toff[(int64_t)threadIdx.x * ntiles + blockIdx.x];
  const int64_t t0 = (int64_t)blockIdx.x * kRouteTile;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int it = 0; it < kRouteTileIters; it++) {
    const int64_t i = t0 + (int64_t)it * kBlock + threadIdx.x;
    const bool in = i < n;
    const int o = in ? owner_at(key, key_wide, i, world) : -1;
    uint32_t rank = 0;
    for (int q = 0; q < world; q++) {
      const uint64_t m = __ballot(o == q);
      if (o == q) rank = (uint32_t)__popcll(m & lt);
      if (lane == 0) wcnt[w][q] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (in) {
      uint32_t at = base[o] + rank;
      for (int v = 0; v < w; v++) at += wcnt[v][o];
      uint64_t* row = send + (int64_t)at * L.nwords;
      uint64_t packed[kRouteMaxCols + 1];
#pragma unroll
      for (int j = 0; j < kRouteMaxCols + 1; j++) packed[j] = 0;
#pragma unroll
      for (int c = 0; c < kRouteMaxCols; c++) {
        if (c >= L.ncols) break;
        if (L.wide[c]) {
          const uint64_t v = ((const uint64_t*)L.col[c])[i];
#pragma unroll
          for (int j = 0; j < kRouteMaxCols + 1; j++)
            if (j == L.slot[c]) packed[j] = v;
        } else {
          const uint64_t v = ((const uint32_t*)L.col[c])[i];
          const int wj = L.slot[c] >> 1, sh = (L.slot[c] & 1) * 32;
#pragma unroll
          for (int j = 0; j < kRouteMaxCols + 1; j++)
            if (j == wj) packed[j] |= v << sh;
        }
      }
      {
        const uint64_t v = (uint32_t)(seq[i] - seq_lo);
        const int wj = L.seq_slot >> 1, sh = (L.seq_slot & 1) * 32;
#pragma unroll
        for (int j = 0; j < kRouteMaxCols + 1; j++)
          if (j == wj) packed[j] |= v << sh;
      }
#pragma unroll
      for (int j = 0; j < kRouteMaxCols + 1; j++)
        if (j < L.nwords) row[j] = packed[j];
    }
    __syncthreads();
    if ((int)threadIdx.x < world) {
      uint32_t s = 0;
      for (int v = 0; v < kBlock / 64; v++) s += wcnt[v][threadIdx.x];
      base[threadIdx.x] += s;
    }
    __syncthreads();
  }
}

__device__ __forceinline__ uint32_t seq_off_of(const uint64_t* __restrict__ recv, int nwords, int seq_slot,
                                               int64_t r) {
  const uint64_t v = recv[r * nwords + (seq_slot >> 1)];
  return (uint32_t)(v >> ((seq_slot & 1) * 32));
}

// start[b * world + s] = first row of sender s's segment whose sequence offset is
// >= b * block (b = 0 .. nblocks)
__global__ __launch_bounds__(kBlock) void k_route_starts(const uint64_t* __restrict__ recv, int nwords, int seq_slot,
                                                         const int64_t* __restrict__ seg_off, int world,
                                                         int64_t block, int64_t nblocks,
                                                         int64_t* __restrict__ start) {
  const int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (t >= (nblocks + 1) * world) return;
  const int64_t b = t / world;
  const int s = (int)(t % world);
  int64_t lo = seg_off[s], hi = seg_off[s + 1];
  const uint64_t x = (uint64_t)b * (uint64_t)block;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((uint64_t)seq_off_of(recv, nwords, seq_slot, mid) < x) lo = mid + 1;
    else hi = mid;
  }
  start[t] = lo;
}

// One workgroup per call (block of sequence numbers): the senders' rows of the
// call (each run in sequence order) are ranked by binary searches in LDS and
// written unpacked at (rows of earlier calls) + rank.  block_off[b] = output
// offset of call b; block_off[nblocks] = rows merged.  err[0] |= 1 when a row
// lies outside the calls or a call holds more rows than sequence numbers.
__global__ __launch_bounds__(kBlock) void k_route_merge(const uint64_t* __restrict__ recv, RouteLayout L,
                                                        const int64_t* __restrict__ seg_off, int world, int64_t m,
                                                        int64_t seq_lo, int64_t block, int64_t nblocks,
                                                        const int64_t* __restrict__ start,
                                                        int64_t* __restrict__ out_seq,
                                                        int64_t* __restrict__ block_off, int32_t* __restrict__ err) {
  __shared__ uint32_t sq[kRouteMaxBlock];
  __shared__ int64_t s0[kRouteMaxWorld];
  __shared__ uint32_t pre[kRouteMaxWorld + 1];
  __shared__ int64_t ob;
  const int64_t b = blockIdx.x;
  if (threadIdx.x == 0) {
    int64_t o = 0;
    uint32_t p = 0;
    for (int s = 0; s < world; s++) {
      const int64_t a = start[b * world + s], e = start[(b + 1) * world + s];
      s0[s] = a;
      pre[s] = p;
      p += (uint32_t)(e - a);
      o += a - seg_off[s];
    }
    pre[world] = p;
    ob = o;
    block_off[b] = o;
    if (b == nblocks - 1) {
      block_off[nblocks] = o + p;
      if (o + p != m) err[0] = 1;   // rows past the last call
    }
    if (p > (uint32_t)block) err[0] = 1;
  }
  __syncthreads();
  const uint32_t T = pre[world];
  if (T > (uint32_t)block) return;
  const uint32_t bb = (uint32_t)(b * block);
  for (uint32_t idx = threadIdx.x; idx < T; idx += kBlock) {
    int s = 0;
    while (idx >= pre[s + 1]) s++;
    sq[idx] = seq_off_of(recv, L.nwords, L.seq_slot, s0[s] + (idx - pre[s])) - bb;
  }
  __syncthreads();
  const int64_t o = ob;
  for (uint32_t idx = threadIdx.x; idx < T; idx += kBlock) {
    int s = 0;
    while (idx >= pre[s + 1]) s++;
    const uint32_t x = sq[idx];
    if (x >= (uint32_t)block) err[0] = 1;
    uint32_t pos = idx - pre[s];
    for (int t = 0; t < world; t++) {
      if (t == s) continue;
      uint32_t lo = pre[t], hi = pre[t + 1];
      const uint32_t base_t = lo;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (sq[mid] < x) lo = mid + 1;
        else hi = mid;
      }
      pos += lo - base_t;
    }
    const int64_t r = s0[s] + (idx - pre[s]);
    const int64_t d = o + pos;
    const uint64_t* row = recv + r * L.nwords;
#pragma unroll
    for (int c = 0; c < kRouteMaxCols; c++) {
      if (c >= L.ncols) break;
      if (L.wide[c]) {
        ((uint64_t*)L.col[c])[d] = row[L.slot[c]];
      } else {
        ((uint32_t*)L.col[c])[d] = (uint32_t)(row[L.slot[c] >> 1] >> ((L.slot[c] & 1) * 32));
      }
    }
    out_seq[d] = seq_lo + (int64_t)bb + x;
  }
}

RouteLayout layout(int ncols, const int* widths) {
  if (ncols < 0 || ncols > kRouteMaxCols) throw Error(SHD_E_ARG, "route: 0..8 columns");
  RouteLayout L{};
  L.ncols = ncols;
  int w8 = 0, n4 = 0;
  for (int c = 0; c < ncols; c++) {
    if (widths[c] != 4 && widths[c] != 8) throw Error(SHD_E_ARG, "route: column widths must be 4 or 8 bytes");
    if (widths[c] == 8) w8++;
    else n4++;
  }
  int next8 = 0, next4 = 2 * w8;
  for (int c = 0; c < ncols; c++) {
    L.wide[c] = widths[c] == 8;
    L.slot[c] = L.wide[c] ? next8++ : next4++;
  }
  L.seq_slot = next4++;
  L.nwords = w8 + (n4 + 2) / 2;
  return L;
}

}  // namespace

// per-tile owner counts of the bucket pass (caller-owned, so concurrent
// buckets on different streams never share scratch)
int64_t route_bucket_scratch(int64_t n, int world) {
  if (world < 1 || world > kRouteMaxWorld || n < 0) throw Error(SHD_E_ARG, "route: world 1..64, n >= 0");
  return std::max<int64_t>(ceil_div(n, kRouteTile) * world, 1) * (int64_t)sizeof(uint32_t);
}

int route_words(int ncols, const int* widths) { return layout(ncols, widths).nwords; }

void route_bucket(hipStream_t s, int64_t n, int world, const void* key, int key_width, int ncols,
                  const void* const* cols, const int* widths, const int64_t* seq, int64_t seq_lo, uint64_t* send,
                  int64_t* counts, uint32_t* scratch) {
  if (world < 1 || world > kRouteMaxWorld) throw Error(SHD_E_ARG, "route: world must be 1..64");
  if (key_width != 4 && key_width != 8) throw Error(SHD_E_ARG, "route: key width must be 4 or 8 bytes");
  if (n < 0 || n >= (int64_t(1) << 32)) throw Error(SHD_E_ARG, "route: batch of 0 .. 2^32-1 rows");
  if (!counts || (n > 0 && (!key || !seq || !send || !scratch))) throw Error(SHD_E_ARG, "route: null buffer");
  RouteLayout L = layout(ncols, widths);
  for (int c = 0; c < ncols; c++) {
    if (n > 0 && !cols[c]) throw Error(SHD_E_ARG, "route: null column");
    L.col[c] = cols[c];
  }
  if (n == 0) {
    SHD_HIP(hipMemsetAsync(counts, 0, sizeof(int64_t) * world, s));
    return;
  }
  const int64_t ntiles = ceil_div(n, kRouteTile);
  uint32_t* d_tc = scratch;   // [world][ntiles] (route_bucket_scratch bytes)
  hipLaunchKernelGGL(k_route_hist, dim3((unsigned)ntiles), dim3(kBlock), 0, s, key, key_width == 8 ? 1 : 0, n, world,
                     ntiles, d_tc);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, s, d_tc, ntiles * world, world, ntiles, counts);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_route_scatter, dim3((unsigned)ntiles), dim3(kBlock), 0, s, key, key_width == 8 ? 1 : 0, n,
                     world, ntiles, (const uint32_t*)d_tc, L, seq, seq_lo, send);
  SHD_CHECK_LAUNCH();
}

void route_merge(hipStream_t s, int world, const uint64_t* recv, const int64_t* seg_off, int64_t m, int64_t seq_lo,
                 int64_t block, int64_t nblocks, int ncols, void* const* out_cols, const int* widths,
                 int64_t* out_seq, int64_t* start, int64_t* block_off, int32_t* err) {
  if (world < 1 || world > kRouteMaxWorld) throw Error(SHD_E_ARG, "route: world must be 1..64");
  if (block < 1 || block > kRouteMaxBlock) throw Error(SHD_E_ARG, "route: call size must be 1..8192");
  if (nblocks < 1 || nblocks * block >= (int64_t(1) << 32)) throw Error(SHD_E_ARG, "route: 1 .. 2^32 sequence numbers");
  if (!seg_off || !start || !block_off || !err || (m > 0 && (!recv || !out_seq)))
    throw Error(SHD_E_ARG, "route: null buffer");
  RouteLayout L = layout(ncols, widths);
  for (int c = 0; c < ncols; c++) {
    if (m > 0 && !out_cols[c]) throw Error(SHD_E_ARG, "route: null column");
    L.col[c] = out_cols[c];
  }
  SHD_HIP(hipMemsetAsync(err, 0, sizeof(int32_t), s));
  const int64_t nst = (nblocks + 1) * world;
  hipLaunchKernelGGL(k_route_starts, dim3((unsigned)ceil_div(nst, kBlock)), dim3(kBlock), 0, s, recv, L.nwords,
                     L.seq_slot, seg_off, world, block, nblocks, start);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_route_merge, dim3((unsigned)nblocks), dim3(kBlock), 0, s, recv, L, seg_off, world, m, seq_lo,
                     block, nblocks, (const int64_t*)start, out_seq, block_off, err);
  SHD_CHECK_LAUNCH();
}

}  // namespace shd
