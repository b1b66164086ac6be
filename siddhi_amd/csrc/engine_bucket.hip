// engine_bucket.hip -- the pattern engine's bucket walk (sparse partitioned
// pushes, config P3): see the comment at the top of the kernels below and
// DESIGN.md §4.1.  Launched from engine_pattern.hip (PatternEngine::sort_push)
// through bucket_walk_launch().
#include <cstdlib>

#include "engine.h"
#include "pattern_common.h"

namespace shd {
using namespace pat;
namespace {

// ---------------------------------------------------------------- bucket walk
// Sparse partitioned pushes (config P3: a partial rarely meets another event of
// its key inside `within`).  The key sort is cut to two radix passes over the
// low 16 bits of key_bucket_mix(key) (hashed buckets of ~n/65536 positions,
// the keys of a bucket interleaved in ext-row order), and each bucket is
// staged in LDS sorted by the top 8 bits of the mix (one stable counting-sort
// pass: sub-buckets of a few positions, each key's positions in one
// sub-bucket in ext-row order -- the mix is bijective, so within a bucket
// equal high 16 bits = equal key).  A walk steps over the later positions of
// its sub-bucket, passing those of other keys: exactly the later events of its
// own key, in ext-row order, as over a full-key sort, so the outcomes,
// counters and per-position results (pst / match_row at the bucket positions)
// are those of k_forward_scan.  A walk that reaches a B event inside `within`
// defers (PS_DEFER, match_row = its sorted slot) and k_bucket_resume evaluates
// f2 through the bucket's key-grouped order (perm).  Downstream kernels only
// need each key's positions in ext-row order, which bucket order keeps.  A
// bucket larger than the LDS stage sets *ovf: the push is then sorted by the
// full key and scanned the usual way.
constexpr int kBwBlock = 256;
constexpr int kBwWaves = kBwBlock / 64;
constexpr int kBwCap = 2048;                  // largest bucket staged in LDS
constexpr int kBwR = kBwCap / kBwBlock;       // rounds of the counting sort

__device__ __forceinline__ uint32_t bw_bucket(uint32_t k) { return key_bucket_mix(k) & kBwMask; }
// a position's key inside its bucket (the mix's high 16 bits) and its sub-bucket
__device__ __forceinline__ uint32_t bw_hh(uint32_t k) { return key_bucket_mix(k) >> 16; }
__device__ __forceinline__ uint32_t bw_sub(uint32_t hh) { return hh >> 8; }

// The hot walk over the staged, sub-bucket-sorted bucket: the same steps,
// expiry and per-key time-order check as walk_partial<DEFER = true>
// (pattern_walk.h) with every ScanArgs field it reads passed in registers
// (inside the walk loop the compiler otherwise reloads them): from the
// partial's successor slot q to the first B event of its key inside `within`
// (ST_DEFER, q at it, its step counted), or the end of its sub-bucket.
__device__ __forceinline__ uint8_t bw_hot(const uint32_t* s_pv, const int32_t* s_ts, const uint16_t* s_hh,
                                          int64_t tbase, int cnt, uint32_t k, int64_t tsi, int64_t within, int& q,
                                          uint64_t& steps, uint32_t& viol) {
  int64_t prev = tsi;
  for (; q < cnt; q++) {
    const uint32_t kq = s_hh[q];
    if (kq != k) {
      if (bw_sub(kq) != bw_sub(k)) return ST_OPEN;   // end of the sub-bucket: no later event of the key
      continue;                                       // another key of the sub-bucket
    }
    const uint32_t fq = pv_flags(s_pv[q]);
    if ((fq & F_NEW) && !(fq & F_SKIP)) {
      const int64_t tq = tbase + (int64_t)s_ts[q];
      if (within != INT64_MAX && tq < prev) {   // a per-key time regression: the push goes to the NFA engine
        viol = 1;
        return ST_OPEN;
      }
      prev = tq;
      steps++;
      if (tq - tsi > within) return ST_DEAD;   // stabilizeStates -> expireEvents
      if (fq & F_B) return ST_DEFER;
    }
  }
  return ST_OPEN;
}

// Bucket starts of the hashed sort's output: bnd[b] = first position of
// bucket b at its head (bnd is filled with 0xFF first).  Coalesced: lane i
// takes position p, its predecessor's key comes from lane i-1.
__global__ __launch_bounds__(kBlock) void k_bucket_heads(const uint32_t* __restrict__ skey, int64_t n_ext,
                                                         int64_t stride, uint32_t* __restrict__ bnd) {
  const int lane = threadIdx.x & 63;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n_ext; p += stride) {
    const uint32_t k = skey[p];
    uint32_t kp = __shfl_up(k, 1, 64);
    if (lane == 0) kp = p > 0 ? skey[p - 1] : ~k;
    const uint32_t b = bw_bucket(k);
    if (p == 0 || bw_bucket(kp) != b) bnd[b] = (uint32_t)p;
  }
}

// bnd[b] of an empty bucket = the start of the next non-empty one (suffix
// minimum), bnd[kBwMask + 1] = n_ext: bucket b is [bnd[b], bnd[b + 1]).
// One workgroup, 64 consecutive entries per thread.
__global__ __launch_bounds__(1024) void k_bucket_fill(uint32_t* __restrict__ bnd, int64_t n_ext) {
  constexpr int NB = (int)kBwMask + 1, PER = NB / 1024;
  __shared__ uint32_t tmin[1024];
  const int t = threadIdx.x;
  uint32_t v[PER];
  uint32_t m = 0xFFFFFFFFu;
#pragma unroll
  for (int i = PER - 1; i >= 0; i--) {
    v[i] = bnd[t * PER + i];
    m = v[i] < m ? v[i] : m;
    v[i] = m;
  }
  tmin[t] = m;
  __syncthreads();
  // minimum over the threads after t (their entries follow t's)
  uint32_t after = (uint32_t)n_ext;
  for (int u = t + 1; u < 1024; u++) after = tmin[u] < after ? tmin[u] : after;
#pragma unroll
  for (int i = 0; i < PER; i++) bnd[t * PER + i] = v[i] < after ? v[i] : after;
  if (t == 0) bnd[NB] = (uint32_t)n_ext;
}

// A run of consecutive buckets per workgroup ([b0, b1), contiguous
// positions).  Per bucket: the positions' loads go to registers (wave w owns
// the slots [w*64R, (w+1)*64R), R rounds of 64), one stable counting-sort pass
// by sub-bucket ranks them (64-bit ballots per round, per-wave digit counts in
// LDS: radix_tile.h's scheme) and scatters them into LDS in sorted order; one
// lane per candidate walks; outcomes go back to ext-row order through s_org
// and are written coalesced.
template <bool FAST>
__global__ __launch_bounds__(kBwBlock, 4) void k_bucket_walk(const ScanArgs* __restrict__ ap, int64_t n_ext,
                                                          const uint32_t* __restrict__ skey,
                                                          const uint32_t* __restrict__ spv,
                                                          const int32_t* __restrict__ sts,
                                                          const uint32_t* __restrict__ bnd, int per_wg,
                                                          int32_t* __restrict__ match_row,
                                                          uint8_t* __restrict__ pst, uint16_t* __restrict__ perm,
                                                          ScanOut* __restrict__ blk, uint32_t* __restrict__ ovf,
                                                          int probe) {
  const ScanArgs& a = *ap;
  __shared__ uint32_t s_pv[kBwCap];
  __shared__ int32_t s_ts[kBwCap];
  __shared__ uint16_t s_hh[kBwCap], s_org[kBwCap];
  __shared__ uint8_t s_out[kBwCap];
  __shared__ uint32_t wcnt[kBwWaves][256];
  __shared__ uint32_t wsum[kBwWaves];
  __shared__ int s_def;   // some walk of this bucket deferred
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0;
  const int64_t tbase = a.x.batch.ts[0];
  const int64_t within = a.within, t_end = a.t_end;
  const bool prune = a.prune != 0;
  const int b0 = (int)blockIdx.x * per_wg;
  const int b1 = b0 + per_wg < (int)kBwMask + 1 ? b0 + per_wg : (int)kBwMask + 1;
  for (int b = b0; b < b1; b++) {
    const int64_t h = bnd[b];
    const int cnt = (int)((int64_t)bnd[b + 1] - h);
    if (cnt > kBwCap) {   // larger than the stage: the full-key path takes this push
      if (tid == 0) atomicOr(ovf, 1u);
      return;
    }
    if (cnt == 0) continue;
    const int R = (cnt + kBwBlock - 1) / kBwBlock;
    // the bucket's base pointers are uniform: 32-bit lane offsets from them
    const uint32_t* kb = skey + h;
    const uint32_t* vb = spv + h;
    const int32_t* tb = sts + h;
    uint32_t v[kBwR], hh[kBwR], lr[kBwR];
    int32_t t[kBwR];
#pragma unroll
    for (int r = 0; r < kBwR; r++) {
      const int sl = w * 64 * R + r * 64 + lane;
      if (r < R && sl < cnt) {
        hh[r] = bw_hh(kb[sl]);
        v[r] = vb[sl];
        t[r] = tb[sl];
      }
    }
    #pragma unroll 1
    for (int i = tid; i < kBwWaves * 256; i += kBwBlock) (&wcnt[0][0])[i] = 0;
    if (tid == 0) s_def = 0;
    __syncthreads();
    // ranks within the wave's slots, by sub-bucket
#pragma unroll
    for (int r = 0; r < kBwR; r++) {
      if (r >= R) break;
      const int sl = w * 64 * R + r * 64 + lane;
      const bool ok = sl < cnt;
      const uint32_t d = ok ? bw_sub(hh[r]) : 0u;
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int bit = 0; bit < 8; bit++) {
        const bool x = (d >> bit) & 1u;
        const uint64_t m = __ballot(x);
        peers &= x ? m : ~m;
      }
      const uint64_t below = peers & lt;
      const uint32_t c = wcnt[w][d];
      lr[r] = c + (uint32_t)__popcll(below);
      __builtin_amdgcn_wave_barrier();
      if (ok && below == 0) wcnt[w][d] = c + (uint32_t)__popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // digit bases: exclusive prefix over digits (thread tid = digit), then waves
    uint32_t tot = 0;
    for (int i = 0; i < kBwWaves; i++) tot += wcnt[i][tid];
    uint32_t inc = tot;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o, 64);
      if (lane >= o) inc += y;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    {
      uint32_t acc = inc - tot;
      for (int i = 0; i < w; i++) acc += wsum[i];
      for (int i = 0; i < kBwWaves; i++) {
        const uint32_t c = wcnt[i][tid];
        wcnt[i][tid] = acc;
        acc += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < kBwR; r++) {
      if (r >= R) break;
      const int sl = w * 64 * R + r * 64 + lane;
      if (sl < cnt) {
        const int dst = (int)(wcnt[w][bw_sub(hh[r])] + lr[r]);
        s_pv[dst] = v[r];
        s_ts[dst] = t[r];
        s_hh[dst] = (uint16_t)hh[r];
        s_org[dst] = (uint16_t)sl;
      }
    }
    __syncthreads();
    #pragma unroll 1
    for (int sl = tid; sl < cnt; sl += kBwBlock) {
      const uint32_t pvp = s_pv[sl];
      uint8_t out = PS_NONE;
      if ((pv_flags(pvp) & F_CAND) && !(probe & 2)) {
        const uint32_t k = s_hh[sl];
        const int64_t tsi = tbase + (int64_t)s_ts[sl];
        int q = sl + 1;
        uint8_t st = bw_hot(s_pv, s_ts, s_hh, tbase, cnt, k, tsi, within, q, steps, viol);
        if (st == ST_OPEN && prune && t_end - tsi > within) st = ST_PRUNED;
        if (st == ST_DEFER) {   // f2 walk: k_bucket_resume, from slot q
          out = PS_DEFER;
          (match_row + h)[s_org[sl]] = q;
          s_def = 1;
        } else if (st == ST_OPEN) {
          out = PS_OPEN;
        } else if (st == ST_PRUNED) {
          pruned++;
        }
      }
      s_out[s_org[sl]] = out;
    }
    __syncthreads();
    if (!(probe & 4))
      #pragma unroll 1
      for (int i = tid; i < cnt; i += kBwBlock) (pst + h)[i] = s_out[i];
    // the bucket's key-grouped order, for the deferred walks
    if (s_def)
      #pragma unroll 1
      for (int sl = tid; sl < cnt; sl += kBwBlock) (perm + h)[sl] = s_org[sl];
    __syncthreads();
  }
  // ScanOut partial of this workgroup (the tile counts come from k_tile_count)
  for (int o = 32; o > 0; o >>= 1) {
    steps += __shfl_xor(steps, o, 64);
    pruned += __shfl_xor(pruned, o, 64);
    viol |= __shfl_xor(viol, o, 64);
  }
  __shared__ ScanOut wpart[kBwWaves];
  if ((tid & 63) == 0) wpart[tid >> 6] = ScanOut{steps, pruned, viol};
  __syncthreads();
  if (tid == 0) {
    ScanOut r = wpart[0];
    for (int w = 1; w < kBwWaves; w++) {
      r.steps += wpart[w].steps;
      r.pruned += wpart[w].pruned;
      r.violation |= wpart[w].violation;
    }
    blk[blockIdx.x] = r;
  }
}

// Deferred walks of the bucket walk (k_forward_resume MODE 0's scheme): each
// thread scans 16 outcome bytes; a PS_DEFER position p resumes at slot
// match_row[p] of its bucket, stepping through the bucket's sub-bucket order
// (perm, written by k_bucket_walk) over the sorted arrays in HBM: f2 at the
// deferral's event (FAST predicate, descriptors read through the uniform
// ScanArgs), then on over the later events of its key to its sub-bucket's end.
__global__ __launch_bounds__(kBlock) void k_bucket_resume(const ScanArgs* __restrict__ ap, int64_t n_ext,
                                                          const uint32_t* __restrict__ skey,
                                                          const uint32_t* __restrict__ spv,
                                                          const int32_t* __restrict__ sts,
                                                          const uint32_t* __restrict__ bnd,
                                                          const uint16_t* __restrict__ perm,
                                                          int32_t* __restrict__ match_row, uint8_t* __restrict__ pst,
                                                          ScanOut* __restrict__ blk) {
  const ScanArgs& a = *ap;
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0;
  const int64_t tbase = a.x.batch.ts[0];
  const int64_t within = a.within, t_end = a.t_end;
  const bool prune = a.prune != 0;
  const int64_t stride = (int64_t)gridDim.x * kBlock * 16;
  for (int64_t pb = ((int64_t)blockIdx.x * kBlock + threadIdx.x) * 16; pb < n_ext; pb += stride) {
    const uint4 raw = *reinterpret_cast<const uint4*>(pst + pb);   // pst is padded (kCompactPad)
    const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
    uint32_t hit = 0;
#pragma unroll
    for (int i = 0; i < 16; i++)
      if (((wv[i >> 2] >> ((i & 3) * 8)) & 255u) == PS_DEFER && pb + i < n_ext) hit |= 1u << i;
    while (hit) {
      const int64_t p = pb + __ffs(hit) - 1;
      hit &= hit - 1;
      const uint32_t k = skey[p];
      const uint32_t bk = bw_bucket(k);
      const int64_t h = bnd[bk];
      const int cnt = (int)((int64_t)bnd[bk + 1] - h);
      const int64_t r = pv_row(spv[p]);
      const int64_t tsi = tbase + (int64_t)sts[p];
      int q = match_row[p];
      int64_t g = h + perm[h + q];
      uint32_t pq = spv[g];
      int64_t prev = tbase + (int64_t)sts[g];
      int32_t j = -1;
      uint8_t st = ST_OPEN;
      bool f2_now = true;
      while (q < cnt) {
        if (!f2_now) {
          g = h + perm[h + q];
          const uint32_t kq = skey[g];
          pq = spv[g];
          const uint32_t fq = pv_flags(pq);
          if (kq != k) {
            if (bw_sub(bw_hh(kq)) != bw_sub(bw_hh(k))) break;   // end of the sub-bucket
            q++;
            continue;   // another key of the sub-bucket
          }
          if ((fq & F_NEW) && !(fq & F_SKIP)) {
            const int64_t tq = tbase + (int64_t)sts[g];
            if (within != INT64_MAX && tq < prev) {
              viol = 1;
              break;
            }
            prev = tq;
            steps++;
            if (tq - tsi > within) {
              st = ST_DEAD;
              break;
            }
            if (fq & F_B) f2_now = true;
          }
        }
        if (f2_now) {
          f2_now = false;
          const int64_t r2 = pv_row(pq);
          PairCtx cx{&a.x, r, r2, a.s_first};
          if (eval_fpred(a.f2.fp, cx)) {
            j = (int32_t)r2;
            st = ST_MATCH;
            break;
          }
        }
        q++;
      }
      if (st == ST_OPEN && prune && t_end - tsi > within) st = ST_PRUNED;
      uint8_t out = PS_NONE;
      if (st == ST_MATCH) {
        out = PS_MATCH;
        match_row[p] = j;
      } else if (st == ST_OPEN) {
        out = PS_OPEN | PS_PEND;   // it met a B event of its key: in the pending list now
      } else if (st == ST_PRUNED) {
        pruned++;
      }
      pst[p] = out;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    steps += __shfl_xor(steps, o, 64);
    pruned += __shfl_xor(pruned, o, 64);
    viol |= __shfl_xor(viol, o, 64);
  }
  __shared__ ScanOut wpart[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = ScanOut{steps, pruned, viol};
  __syncthreads();
  if (threadIdx.x == 0) {
    ScanOut t = wpart[0];
    for (int w = 1; w < kBlock / 64; w++) {
      t.steps += wpart[w].steps;
      t.pruned += wpart[w].pruned;
      t.violation |= wpart[w].violation;
    }
    blk[blockIdx.x] = t;
  }
}

}  // namespace

// Bucket bounds, the walk (grid of runs of per_wg buckets), the deferred
// walks (probe: timing experiments, SHD_BW_PROBE).  ovf is zeroed by the
// caller; blk takes nbw + bucket_resume_blocks(n_ext) partials (the count returned).
int pat::bucket_walk_launch(hipStream_t s, const ScanArgs* d_sa, int64_t n_ext, const uint32_t* skey, const uint32_t* spv,
                            const int32_t* sts, uint32_t* bnd, uint16_t* perm, int nblk, int32_t* match_row,
                            uint8_t* pst, ScanOut* blk, uint32_t* ovf, int per_wg) {
  const int nbk = (int)kBwMask + 1;
  const int nbw = (nbk + per_wg - 1) / per_wg;
  SHD_HIP(hipMemsetAsync(bnd, 0xFF, (size_t)(nbk + 1) * 4, s));
  hipLaunchKernelGGL(k_bucket_heads, dim3(nblk), dim3(kBlock), 0, s, skey, n_ext, (int64_t)nblk * kBlock, bnd);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_bucket_fill, dim3(1), dim3(1024), 0, s, bnd, n_ext);
  SHD_CHECK_LAUNCH();
  const int probe = getenv("SHD_BW_PROBE") ? atoi(getenv("SHD_BW_PROBE")) : 0;
  hipLaunchKernelGGL(k_bucket_walk<true>, dim3(nbw), dim3(kBwBlock), 0, s, d_sa, n_ext, skey, spv, sts,
                     (const uint32_t*)bnd, per_wg, match_row, pst, perm, blk, ovf, probe);
  SHD_CHECK_LAUNCH();
  const int nres = bucket_resume_blocks(n_ext);
  if (!(probe & 8)) {
    hipLaunchKernelGGL(k_bucket_resume, dim3(nres), dim3(kBlock), 0, s, d_sa, n_ext, skey, spv, sts,
                       (const uint32_t*)bnd, (const uint16_t*)perm, match_row, pst, blk + nbw);
    SHD_CHECK_LAUNCH();
  } else {
    SHD_HIP(hipMemsetAsync(blk + nbw, 0, (size_t)nres * sizeof(ScanOut), s));
  }
  return nbw + nres;
}

}  // namespace shd
