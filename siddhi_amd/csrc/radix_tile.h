// radix_tile.h -- one workgroup's tile of a stable LSD radix pass (gfx950,
// wave64): tile constants, digit helpers and the in-tile ranking / LDS
// reorder / per-digit-run write-out shared by the radix sort kernels of
// primitives.hip and the fused bucket scatter of engine_pattern.hip.
#pragma once
#include "common.h"

namespace shd {

// One workgroup (kRsBlock threads, kRsWaves waves) sorts a tile of
// R*kRsBlock keys per pass.  Wave w owns the contiguous slice
// [t0 + w*64R, t0 + (w+1)*64R) and holds its R keys per lane in registers
// (all loads issued up front).  Stable in-wave ranking from eight 64-bit
// ballots per round and a per-wave running count per digit in LDS (the wave
// executes in order, so no barrier between rounds); a tile needs four
// workgroup barriers.  The tile is reordered by digit in LDS and written out
// in per-digit runs, so consecutive lanes store consecutive addresses.
// Optional second payload: a 32-bit word per key.
#ifndef SHD_RS_ROUNDS
#define SHD_RS_ROUNDS 24
#endif
#ifndef SHD_RS_BLOCK
#define SHD_RS_BLOCK 256
#endif
constexpr int kRsRounds = SHD_RS_ROUNDS;
constexpr int kRsBlock = SHD_RS_BLOCK;
constexpr int kRsWaves = kRsBlock / 64;
static_assert(kRsBlock >= 256 && kRsBlock % 64 == 0, "one thread per digit in the digit phases");

__host__ __device__ constexpr int rs_tile(int rounds) { return kRsBlock * rounds; }

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs
// (blocks b and b+8 share one), so block b takes tile (b%8)*per + b/8: the
// tiles of one XCD are consecutive, and the per-digit runs that neighbouring
// tiles write next to each other meet in the same L2 (fewer partial-line
// write-backs).  Any bijection is correct; this one is for speed only.
__device__ __forceinline__ int rs_tile_of(int b, int nb) {
  const int per = nb >> 3, rem = nb & 7, x = b & 7, i = b >> 3;
  return x * per + (x < rem ? x : rem) + i;
}

template <class K>
__device__ __forceinline__ uint32_t rs_digit(K k, int shift) { return (uint32_t)((k >> shift) & 255u); }
// H: digits of key_bucket_mix(key) (hashed bucket sort; 32-bit keys only).
// kb: key base subtracted first (the keys of a push span [kb, kb + 2^bits)).
template <bool H, class K>
__device__ __forceinline__ uint32_t rs_hdigit(K k, int shift, K kb) {
  if constexpr (H) return (key_bucket_mix((uint32_t)k) >> shift) & 255u;
  else return rs_digit((K)(k - kb), shift);
}

// Rank the tile's keys by digit (stable: ballots inside a wave, waves in
// order), reorder them in LDS and write them out in per-digit runs.  Thread
// tid < 256 holds digit tid's count in this tile (c), the tile's global
// offset inside the digit (gr) and the digit's total (dt); wave w holds rows
// [wb, wb + 64R) of the tile starting at t0, R per lane (k, v, x; rows >= n
// are padding).
// dig(key) -> digit in [0, 256): rs_scatter_tile below takes the digits of
// (key - kb) >> shift (or of the hashed key); the fused first pass of the
// pattern engine's key sort (keyed_sort.hip) passes its own.
template <class K, int R, bool P2, class Dig>
__device__ __forceinline__ void rs_scatter_tile_fn(const K (&k)[R], const uint32_t (&v)[R],
                                                   const uint32_t (&x)[P2 ? R : 1], int64_t n, int64_t t0,
                                                   int64_t wb, const Dig& dig, uint32_t c, uint32_t gr, uint32_t dt,
                                                   K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                   uint32_t* __restrict__ wout) {
  constexpr int T = rs_tile(R);
  __shared__ K sk[T];
  __shared__ uint32_t sv[T];
  __shared__ uint32_t sw[P2 ? T : 1];
  // 16-bit tile-local counts and positions (a tile holds < 65536 keys): 2.5 KB
  // less LDS, which takes the fused first pass (keyed_sort.hip, 4096-key
  // tiles) from 55.8 to 53.0 KB, three workgroups per CU instead of two
  // (490 -> 410 us per 50 M-row pass)
  static_assert(T < 65536, "16-bit tile-local counts");
  __shared__ uint16_t lpre[256];             // tile-local first position of each digit
  __shared__ uint32_t gbase[256];            // global first position of this tile's digit run
  __shared__ uint16_t wcnt[kRsWaves][256];   // per-wave running digit counts, then per-wave digit bases
  __shared__ uint32_t wsum[4], dsum[4];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kRsWaves * 256; i += kRsBlock) (&wcnt[0][0])[i] = 0;
  {
    // tile-local exclusive prefix over digits (threads 0..255, one digit
    // each), and the global base of each digit (prefix of the digit totals)
    uint32_t inc = c, dinc = dt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      const uint32_t u = __shfl_up(dinc, o, 64);
      if (lane >= o) {
        inc += t;
        dinc += u;
      }
    }
    if (lane == 63 && w < 4) {
      wsum[w] = inc;
      dsum[w] = dinc;
    }
    __syncthreads();
    if (tid < 256) {
      uint32_t pre = 0, dpre = 0;
      for (int i = 0; i < w; i++) {
        pre += wsum[i];
        dpre += dsum[i];
      }
      lpre[tid] = (uint16_t)(pre + inc - c);
      gbase[tid] = dpre + dinc - dt + gr;
    }
  }
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint32_t lr[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const bool ok = wb + r * 64 + lane < n;
    const uint32_t d = dig(k[r]);
    uint64_t peers = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const bool bit = (d >> b) & 1u;
      const uint64_t m = __ballot(bit);
      peers &= bit ? m : ~m;
    }
    const uint64_t below = peers & lt;
    const uint32_t c = wcnt[w][d];
    lr[r] = c + (uint32_t)__popcll(below);
    __builtin_amdgcn_wave_barrier();
    if (ok && below == 0) wcnt[w][d] = (uint16_t)(c + (uint32_t)__popcll(peers));
    __builtin_amdgcn_wave_barrier();
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t acc = lpre[tid];
#pragma unroll
    for (int i = 0; i < kRsWaves; i++) {
      const uint32_t c = wcnt[i][tid];
      wcnt[i][tid] = (uint16_t)acc;
      acc += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < R; r++) {
    if (wb + r * 64 + lane < n) {
      const uint32_t pos = wcnt[w][dig(k[r])] + lr[r];
      sk[pos] = k[r];
      sv[pos] = v[r];
      if (P2) sw[pos] = x[r];
    }
  }
  __syncthreads();
  const int tile_n = n - t0 < T ? (int)(n - t0) : T;
#pragma unroll 4
  for (int i = tid; i < tile_n; i += kRsBlock) {
    const K kk = sk[i];
    const uint32_t d = dig(kk);
    const uint32_t o = gbase[d] + (uint32_t)i - lpre[d];
    kout[o] = kk;
    vout[o] = sv[i];
    if (P2) wout[o] = sw[i];
  }
}

template <class K, int R, bool P2, bool H>
__device__ __forceinline__ void rs_scatter_tile(const K (&k)[R], const uint32_t (&v)[R],
                                                const uint32_t (&x)[P2 ? R : 1], int64_t n, int64_t t0, int64_t wb,
                                                int shift, uint32_t c, uint32_t gr, uint32_t dt, K kb,
                                                K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                uint32_t* __restrict__ wout) {
  rs_scatter_tile_fn<K, R, P2>(k, v, x, n, t0, wb, [shift, kb](K kk) { return rs_hdigit<H>(kk, shift, kb); }, c, gr,
                               dt, kout, vout, wout);
}

}  // namespace shd
