// keyed_sort.hip -- the pattern engine's row preparation fused into the first
// pass of its key sort (partitioned plans on a 32-bit plain key attribute:
// config P3, BASELINE.json configs[2]).
//
// The unfused push (engine_pattern.hip k_prepare + radix_sort_triples_u32)
// reads key + f1 operand + ts per extended row (20 B), writes the sort inputs
// key / (flags, row) / 32-bit ts offset (12 B), and the first LSD pass reads
// the keys again for its histogram (4 B) and the 12 B for its scatter: 48 B
// per row before the first pass has written anything.  Here:
//   k_ks_hist      reads the key (4 B; carried partials: the low word of
//                  their 8-byte key): tile-major histogram of the key's raw
//                  low byte + the key range;
//   k_ks_finish    folds the aggregates and derives the sort's key base and
//                  width exactly as the host does (engine_pattern.hip
//                  sort_push), so the first pass needs no host round trip;
//   k_ks_chunk_sum / k_ks_chunk_scan / k_ks_offsets
//                  per-tile digit offsets of the first pass, tile-major (a
//                  tile reads its 256 offsets as one 1 KB line run).  The
//                  first digit is (key - kbase) & 255 = (low byte - kbase)
//                  & 255, a rotation of the raw low-byte histogram;
//   k_ks_scatter0  reads key + f1 operand + ts (20 B), evaluates f1 and the
//                  flags (prep_row's rules), ranks the tile by the first
//                  digit and writes key / (flags, row) / ts offset sorted by
//                  it (12 B) -- the input of the remaining passes
//                  (radix_sort_triples_u32 from shift 8) -- and per tile the
//                  time aggregates (pushed rows: range, order, offset
//                  overflow; carried partials: latest time, overflow) and the
//                  candidates created;
//   k_ks_tfold     folds those into the push's PrepAgg: the host reads the
//                  key range after k_ks_finish (the remaining passes need
//                  only that) and the times after this fold, while the
//                  remaining passes run.
// 24 + 12 B per row instead of 48 + 12, and the first pass's histogram comes
// with the aggregates.  The sorted arrays are bit-identical to the unfused
// path's (same digits, same stable order), so everything downstream is
// unchanged.  Reference semantics of the row flags: PartitionStreamReceiver
// (null key -> dropped, C/partition/PartitionStreamReceiver.java:81-283),
// FilterProcessor on the start state (StreamPreStateProcessor.java:364-403).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "engine.h"
#include "radix_tile.h"
#include "pattern_common.h"

namespace shd {
namespace pat {

namespace {

constexpr int kKsRounds = 16;                 // rows per lane of the fused pass
constexpr int kKsTile = kRsBlock * kKsRounds;   // 4096 rows per workgroup
constexpr int kKsChunk = 64;                  // tiles per offsets workgroup

// Count of first-pass digit d in tile t (rotated raw low-byte histogram; a
// zero-width sort puts every row in digit 0 like the unfused path, which does
// not sort then).
__device__ __forceinline__ uint32_t ks_count(const uint32_t* __restrict__ hraw, int64_t t, int d, const KsInfo& in,
                                             int64_t n_ext) {
  if (in.bits == 0) {
    if (d) return 0u;
    const int64_t r = n_ext - t * kKsTile;
    return (uint32_t)(r < kKsTile ? r : kKsTile);
  }
  return hraw[t * 256 + ((d + (int)in.kb) & 255)];
}

// Extended row li: key word and time (carried partial: carry table, else the
// pushed batch), as one load each through a per-lane selected address.
struct KsRow {
  const uint32_t* kp;
  const int64_t* tp;
  int64_t br;   // batch row (-1: carried partial)
};
__device__ __forceinline__ KsRow ks_row(const PrepArgs& a, const uint32_t* kcol, int64_t li) {
  const int64_t C = a.x.C;
  KsRow r;
  if (li < C) {
    r.kp = reinterpret_cast<const uint32_t*>(a.carry_key) + 2 * li;   // low word of the u64 carry key
    r.tp = a.x.carry.ts + li;
    r.br = -1;
  } else {
    r.kp = kcol + (li - C);
    r.tp = a.x.batch.ts + (li - C);
    r.br = li - C;
  }
  return r;
}

template <bool KNUL>
__global__ __launch_bounds__(kRsBlock) void k_ks_hist(const PrepArgs* __restrict__ ap, int64_t n_ext,
                                                      uint32_t* __restrict__ hraw, PrepAgg* __restrict__ blk, int nb) {
  const PrepArgs& a = *ap;
  __shared__ uint32_t h[kRsWaves][256];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < kRsWaves * 256; i += kRsBlock) (&h[0][0])[i] = 0;
  const int tile = rs_tile_of(blockIdx.x, nb);
  const int64_t wb = (int64_t)tile * kKsTile + (int64_t)w * 64 * kKsRounds;
  const uint32_t* kcol = (const uint32_t*)a.x.batch.col[a.key_col];
  const uint8_t* knul = a.x.batch.nul[a.key_col];
  const int64_t C = a.x.C;
  uint32_t kk[kKsRounds];
  uint8_t kn[kKsRounds];
  // the key only (every time aggregate comes from k_ks_scatter0, which loads
  // the times anyway)
  const bool pushed = (int64_t)tile * kKsTile >= C;
  const bool carried = (int64_t)(tile + 1) * kKsTile <= C;   // every row a carried partial
  if (carried) {
    const uint32_t* ck = reinterpret_cast<const uint32_t*>(a.carry_key);
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      kk[r] = gld(ck, 2 * (wb + r * 64 + lane));   // low word of the u64 carry key
      kn[r] = 0;
    }
  } else if (pushed) {
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      const int64_t idx = wb + r * 64 + lane;
      const int64_t b0 = (idx < n_ext ? idx : n_ext - 1) - C;
      kk[r] = gld(kcol, b0);
      kn[r] = KNUL ? gld(knul, b0) : (uint8_t)0;
    }
  } else {
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      const int64_t idx = wb + r * 64 + lane;
      const int64_t li = idx < n_ext ? idx : n_ext - 1;
      const KsRow x = ks_row(a, kcol, li);
      kk[r] = gld(x.kp, 0);
      kn[r] = KNUL ? gld(knul, x.br >= 0 ? x.br : 0) : (uint8_t)0;
    }
  }
  __syncthreads();
  // key range as 32-bit keys (kmx < kmn: no keyed row in this lane)
  uint32_t kmn = 0xFFFFFFFFu, kmx = 0;
  bool any = false;
#pragma unroll
  for (int r = 0; r < kKsRounds; r++) {
    const int64_t idx = wb + r * 64 + lane;
    if (idx >= n_ext) continue;
    uint32_t k = kk[r];
    bool skip = false;
    if (idx >= C && KNUL && kn[r]) {
      if (a.null_skip) {
        skip = true;
        k = (uint32_t)idx;   // prep_row: a dropped row's key is its row index
      } else {
        k = 0;
      }
    }
    if (!skip) {
      kmx = k > kmx ? k : kmx;
      kmn = k < kmn ? k : kmn;
      any = true;
    }
    atomicAdd(&h[w][k & 255u], 1u);
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < kRsWaves; i++) c += h[i][tid];
    hraw[(int64_t)tile * 256 + tid] = c;
  }
  const bool wany = __ballot(any) != 0;
  kmn = wave_min(kmn);
  kmx = wave_max(kmx);
  __shared__ uint32_t wk[2][kRsWaves];
  __shared__ uint32_t wa[kRsWaves];
  if (lane == 0) {
    wk[0][w] = kmn;
    wk[1][w] = kmx;
    wa[w] = wany;
  }
  __syncthreads();
  if (tid == 0) {
    PrepAgg r{0, 0, LLONG_MAX, LLONG_MIN, 0, 0, LLONG_MIN, ULLONG_MAX};
    for (int i = 0; i < kRsWaves; i++) {
      if (!wa[i]) continue;
      r.kmin = wk[0][i] < r.kmin ? wk[0][i] : r.kmin;
      r.kmax = wk[1][i] > r.kmax ? wk[1][i] : r.kmax;
    }
    blk[tile] = r;
  }
}

// Per chunk of kKsChunk tiles: each raw low byte's count over the chunk, and
// the chunk's fold of the tiles' aggregates (k_ks_finish folds the chunks).
__global__ __launch_bounds__(256) void k_ks_chunk_sum(const uint32_t* __restrict__ hraw, int nb,
                                                      const PrepAgg* __restrict__ blk, uint32_t* __restrict__ csum,
                                                      PrepAgg* __restrict__ cblk) {
  const int d = threadIdx.x;
  const int64_t t0 = (int64_t)blockIdx.x * kKsChunk;
  const int64_t t1 = t0 + kKsChunk < nb ? t0 + kKsChunk : nb;
  uint32_t s = 0;
#pragma unroll 8
  for (int64_t t = t0; t < t1; t++) s += hraw[t * 256 + d];
  csum[(int64_t)blockIdx.x * 256 + d] = s;
  PrepAcc acc;
  if (t0 + d < t1) {
    const PrepAgg& b = blk[t0 + d];
    acc.ovf = b.ovf;
    acc.unmono = b.unmono;
    acc.kmin = b.kmin;
    acc.kmax = b.kmax;
    acc.tmin = b.ts_min;
    acc.tmax = b.ts_max;
    acc.ctmax = b.carry_tmax;
  }
  prep_block_reduce<256>(acc, cblk, blockIdx.x);
}

// Fold of the chunks' aggregates + the sort's key base / width
// (engine_pattern.hip sort_push: offsets from kmin when that narrows the key).
__global__ __launch_bounds__(256) void k_ks_finish(const PrepAgg* __restrict__ cblk, int nch,
                                                   PrepAgg* __restrict__ out, KsInfo* __restrict__ info) {
  PrepAcc acc;
  for (int b = threadIdx.x; b < nch; b += 256) {
    const PrepAgg& x = cblk[b];
    acc.ovf |= x.ovf;
    acc.unmono |= x.unmono;
    acc.kmin = x.kmin < acc.kmin ? x.kmin : acc.kmin;
    acc.kmax = x.kmax > acc.kmax ? x.kmax : acc.kmax;
    acc.tmin = x.ts_min < acc.tmin ? x.ts_min : acc.tmin;
    acc.tmax = x.ts_max > acc.tmax ? x.ts_max : acc.tmax;
    acc.ctmax = x.carry_tmax > acc.ctmax ? x.carry_tmax : acc.ctmax;
  }
  __shared__ PrepAgg r1[1];
  prep_block_reduce<256>(acc, r1, 0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const PrepAgg r = r1[0];
    *out = r;
    const unsigned long long kmin = r.kmin <= r.kmax ? r.kmin : 0ull, kmax = r.kmax;
    int bits = 0;
    while (bits < 64 && (kmax >> bits)) bits++;
    uint32_t kb = 0;
    int rb = 0;
    while (rb < 64 && ((kmax - kmin) >> rb)) rb++;
    if (rb < bits) {
      bits = rb > 0 ? rb : 1;
      kb = (uint32_t)kmin;
    }
    *info = KsInfo{kb, bits};
  }
}

// Count of first-pass digit d in chunk ch (rotated raw chunk sums; bits == 0:
// every row in digit 0).
__device__ __forceinline__ uint32_t ks_chunk_count(const uint32_t* __restrict__ csum, int64_t ch, int d,
                                                   const KsInfo& in, int nb, int64_t n_ext) {
  if (in.bits == 0) {
    if (d) return 0u;
    const int64_t t0 = ch * kKsChunk;
    const int64_t r = n_ext - t0 * kKsTile;
    return (uint32_t)(r < (int64_t)kKsChunk * kKsTile ? r : (int64_t)kKsChunk * kKsTile);
  }
  return csum[ch * 256 + ((d + (int)in.kb) & 255)];
}

// One workgroup per digit: exclusive prefix of its chunk counts (cpre) and
// its total (dtot).
__global__ __launch_bounds__(256) void k_ks_chunk_scan(const uint32_t* __restrict__ csum, int nch, int nb,
                                                       const KsInfo* __restrict__ info, int64_t n_ext,
                                                       uint32_t* __restrict__ cpre, uint32_t* __restrict__ dtot) {
  const KsInfo in = *info;
  const int d = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int per = (nch + 255) / 256;   // contiguous chunks per thread
  const int c0 = tid * per, c1 = c0 + per < nch ? c0 + per : nch;
  uint32_t s = 0;
  for (int c = c0; c < c1; c++) s += ks_chunk_count(csum, c, d, in, nb, n_ext);
  uint32_t inc = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  __shared__ uint32_t wsum[4];
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = inc - s, tot = 0;
  for (int i = 0; i < 4; i++) {
    if (i < w) pre += wsum[i];
    tot += wsum[i];
  }
  for (int c = c0; c < c1; c++) {
    cpre[(int64_t)c * 256 + d] = pre;
    pre += ks_chunk_count(csum, c, d, in, nb, n_ext);
  }
  if (tid == 0) dtot[d] = tot;
}

// Tile-major global offsets: offs[t][d] = first sorted position of tile t's
// rows of digit d (digit base + chunk prefix + tiles before t in the chunk).
__global__ __launch_bounds__(256) void k_ks_offsets(const uint32_t* __restrict__ hraw, int nb,
                                                    const KsInfo* __restrict__ info, int64_t n_ext,
                                                    const uint32_t* __restrict__ cpre,
                                                    const uint32_t* __restrict__ dtot, uint32_t* __restrict__ offs) {
  const KsInfo in = *info;
  const int d = threadIdx.x, lane = d & 63, w = d >> 6;
  const uint32_t tot = dtot[d];
  uint32_t inc = tot;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  __shared__ uint32_t wsum[4];
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t base = inc - tot;
  for (int i = 0; i < w; i++) base += wsum[i];
  const int64_t t0 = (int64_t)blockIdx.x * kKsChunk;
  const int64_t t1 = t0 + kKsChunk < nb ? t0 + kKsChunk : nb;
  uint32_t run = base + cpre[(int64_t)blockIdx.x * 256 + d];
  for (int64_t t = t0; t < t1; t++) {
    offs[t * 256 + d] = run;
    run += ks_count(hraw, t, d, in, n_ext);
  }
}

// Expression context of the fused pass: the row's f1 operand, loaded up front
// with the tile's other loads (BatchRowCtx semantics: state 0, index 0 /
// CURRENT; the host admits only f1 chains whose loads read attribute fattr).
struct KsCtx {
  Val v;
  __device__ __forceinline__ Val load(int st, int idx, int) const {
    if (st != 0 || !(idx == 0 || idx == SHD_IDX_CURRENT)) {
      Val n;
      n.b = 0;
      n.null = 1;
      return n;
    }
    return v;
  }
  __device__ __forceinline__ bool evnull(int st, int idx) const { return !(st == 0 && (idx == 0 || idx == SHD_IDX_CURRENT)); }
  __device__ __forceinline__ int64_t ts(int, int) const { return 0; }
  __device__ __forceinline__ Val agg(int) const {
    Val n;
    n.b = 0;
    n.null = 1;
    return n;
  }
};

// f1 pre-resolved on the host (ks_f1): kind 1 = no comparison, 2 = the
// attribute (double column) OP a constant (the constant's conversion applied
// once per workgroup); 0 = eval_fpred per row.
struct KsF1 {
  int32_t kind, op, cvt_from, cvt_to;
  uint64_t cval;
};

// FSZ: byte width of the f1 operand column (0: f1 reads no attribute or the
// pushed stream is not A); FK: KsF1::kind the kernel is specialised for.
template <int FSZ, bool KNUL, bool FNUL, int FK>
__global__ __launch_bounds__(kRsBlock) void k_ks_scatter0(const PrepArgs* __restrict__ ap, int64_t n_ext, int fattr,
                                                          const KsF1 f1, const KsInfo* __restrict__ info,
                                                          const uint32_t* __restrict__ hraw,
                                                          const uint32_t* __restrict__ offs, int nb,
                                                          uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                          uint32_t* __restrict__ wout,
                                                          PrepAgg* __restrict__ blk) {
  const PrepArgs& a = *ap;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = rs_tile_of(blockIdx.x, nb);
  const int64_t t0 = (int64_t)tile * kKsTile;
  const int64_t wb = t0 + (int64_t)w * 64 * kKsRounds;
  const KsInfo in = *info;
  const uint32_t c = ks_count(hraw, tile, tid, in, n_ext);
  const uint32_t gr = offs[(int64_t)tile * 256 + tid];
  const uint32_t* kcol = (const uint32_t*)a.x.batch.col[a.key_col];
  const uint8_t* knul = a.x.batch.nul[a.key_col];
  const void* fcol = fattr >= 0 ? a.x.batch.col[fattr] : nullptr;
  const uint8_t* fnul = fattr >= 0 ? a.x.batch.nul[fattr] : nullptr;
  const int ftype = fattr >= 0 ? a.x.batch.type[fattr] : 0;
  const int64_t tbase = a.x.batch.ts[0];
  uint32_t kk[kKsRounds];
  int64_t tt[kKsRounds];
  typedef typename std::conditional<FSZ == 8, uint64_t, uint32_t>::type FT;
  FT fv[FSZ ? kKsRounds : 1];
  uint8_t kn[kKsRounds], fn[kKsRounds];
  const int64_t C = a.x.C;
  auto load_f = [&](int r, int64_t b0) {
    if constexpr (FSZ == 8) fv[r] = gld((const uint64_t*)fcol, b0);
    else if constexpr (FSZ == 4) fv[r] = gld((const uint32_t*)fcol, b0);
    else if constexpr (FSZ == 1) fv[r] = gld((const uint8_t*)fcol, b0);
    kn[r] = KNUL ? gld(knul, b0) : (uint8_t)0;
    fn[r] = FNUL ? gld(fnul, b0) : (uint8_t)0;
  };
  if (t0 + kKsTile <= C) {
    // every row a carried partial (the first C rows): key + time, uniform bases
    const uint32_t* ck = reinterpret_cast<const uint32_t*>(a.carry_key);
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      const int64_t idx = wb + r * 64 + lane;
      kk[r] = gld(ck, 2 * idx);   // low word of the u64 carry key
      tt[r] = gld(a.x.carry.ts, idx);
      if constexpr (FSZ != 0) fv[r] = 0;
      kn[r] = 0;
      fn[r] = 0;
    }
  } else if (t0 >= C) {
    // every row of the tile is a pushed event: uniform column bases (the
    // common case; carried partials fill only the first C rows)
    const int64_t* bts = a.x.batch.ts;
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      const int64_t idx = wb + r * 64 + lane;
      const int64_t b0 = (idx < n_ext ? idx : n_ext - 1) - C;
      kk[r] = gld(kcol, b0);
      tt[r] = gld(bts, b0);
      load_f(r, b0);
    }
  } else {
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      const int64_t idx = wb + r * 64 + lane;
      const int64_t li = idx < n_ext ? idx : n_ext - 1;
      const KsRow x = ks_row(a, kcol, li);
      kk[r] = gld(x.kp, 0);
      tt[r] = gld(x.tp, 0);
      load_f(r, x.br >= 0 ? x.br : 0);
    }
  }
  // time of the pushed row before the wave's slice (lane 0); the others by shuffle
  int64_t t_before = 0;
  {
    const int64_t li = wb < n_ext ? wb : n_ext - 1;
    const int64_t pb = li - C - 1;
    if (lane == 0 && pb >= 0) t_before = gld(a.x.batch.ts, pb);
  }
  uint32_t kv[kKsRounds], pv[kKsRounds], tv[kKsRounds];
  // time aggregates (pushed rows: range, order, offset overflow; carried
  // partials: latest time, offset overflow) and the candidates created
  PrepAcc acc;
  // FK 2: f1 = (double attribute) op threshold for every row at once, the
  // operator switch outside the row loop (Java double comparison:
  // d_compare's -1 / 0 / 1 / unordered classes)
  bool pre1[FK == 2 ? kKsRounds : 1];
  if constexpr (FK == 2) {
    const double thr = v_f64(f1.cvt_to >= 0 ? d_cvt(f1.cval, f1.cvt_from, f1.cvt_to) : f1.cval);
    int cls[kKsRounds];
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) {
      const double x = v_f64((uint64_t)fv[r]);
      cls[r] = x < thr ? -1 : (x > thr ? 1 : (x == thr ? 0 : 2));
    }
    switch (f1.op) {
      case SHD_OP_GT:
#pragma unroll
        for (int r = 0; r < kKsRounds; r++) pre1[r] = cls[r] == 1;
        break;
      case SHD_OP_GE:
#pragma unroll
        for (int r = 0; r < kKsRounds; r++) pre1[r] = cls[r] == 1 || cls[r] == 0;
        break;
      case SHD_OP_LT:
#pragma unroll
        for (int r = 0; r < kKsRounds; r++) pre1[r] = cls[r] == -1;
        break;
      case SHD_OP_LE:
#pragma unroll
        for (int r = 0; r < kKsRounds; r++) pre1[r] = cls[r] == -1 || cls[r] == 0;
        break;
      case SHD_OP_EQ:
#pragma unroll
        for (int r = 0; r < kKsRounds; r++) pre1[r] = cls[r] == 0;
        break;
      default:   // NE
#pragma unroll
        for (int r = 0; r < kKsRounds; r++) pre1[r] = cls[r] != 0;
        break;
    }
#pragma unroll
    for (int r = 0; r < kKsRounds; r++) pre1[r] = pre1[r] && !(FNUL && fn[r]);
  }
#pragma unroll
  for (int r = 0; r < kKsRounds; r++) {
    const int64_t idx = wb + r * 64 + lane;
    // predecessor row idx - 1: lane - 1 of this round, lane 63 of the last
    // (shuffles with every lane active)
    const int64_t up = __shfl_up(tt[r], 1, 64);
    const int64_t prev63 = r > 0 ? __shfl(tt[r > 0 ? r - 1 : 0], 63, 64) : t_before;
    uint32_t k = kk[r];
    uint32_t f;
    if ((idx < n_ext ? idx : n_ext - 1) < a.x.C) {
      f = F_CAND;
      if (idx < n_ext) {   // carried partial: the latest one's time, offset overflow
        const long long t = (long long)tt[r];
        acc.ctmax = t > acc.ctmax ? t : acc.ctmax;
        const int64_t dt = (int64_t)t - tbase;
        acc.ovf |= dt != (int64_t)(int32_t)dt;
      }
    } else {
      f = F_NEW;
      if (idx < n_ext) {
        const long long t = (long long)tt[r];
        const long long tprev = (long long)(lane ? up : prev63);
        acc.tmin = t < acc.tmin ? t : acc.tmin;
        acc.tmax = t > acc.tmax ? t : acc.tmax;
        acc.unmono |= (idx - C > 0) && tprev > t;
        const int64_t dt = (int64_t)t - tbase;
        acc.ovf |= dt != (int64_t)(int32_t)dt;
      }
      bool p1 = false;
      if constexpr (FK == 2) {
        p1 = a.is_a && pre1[r];
      } else if constexpr (FK == 1) {
        p1 = a.is_a;
      } else if (a.is_a) {
        KsCtx cx;
        cx.v.null = 0;
        cx.v.b = 0;
        if constexpr (FSZ != 0) {
          uint64_t b = (uint64_t)fv[r];
          switch (ftype) {
            case SHD_T_INT: b = p_i32((int32_t)(uint32_t)b); break;
            case SHD_T_BOOL: b = b ? 1 : 0; break;
            default: break;
          }
          cx.v.b = b;
          if (FNUL && fn[r]) {
            cx.v.b = 0;
            cx.v.null = 1;
          }
        } else {
          cx.v.null = 1;
        }
        p1 = eval_fpred(a.f1.fp, cx);
      }
      if (KNUL && kn[r] && a.null_skip) {
        f |= F_SKIP;
        k = (uint32_t)idx;
      } else {
        if (a.is_b) f |= F_B;
        if (p1) {
          f |= F_CAND;
          acc.created += idx < n_ext ? 1u : 0u;
        }
        if (KNUL && kn[r]) k = 0;
      }
    }
    kv[r] = k;
    pv[r] = (f << kRowBits) | (uint32_t)idx;
    tv[r] = (uint32_t)(int32_t)((int64_t)tt[r] - tbase);
  }
  const bool zero = in.bits == 0;
  const uint32_t kb = in.kb;
  rs_scatter_tile_fn<uint32_t, kKsRounds, true>(
      kv, pv, tv, n_ext, t0, wb, [zero, kb](uint32_t k) { return zero ? 0u : ((k - kb) & 255u); }, c, gr, 0u, kout,
      vout, wout);
  prep_block_reduce<kRsBlock>(acc, blk, tile);
}

// Fold of k_ks_scatter0's per-tile partials into the push's PrepAgg (whose
// key range k_ks_finish wrote; n_cand 0, time fields empty): candidates
// created, pushed rows' time range / order, offset overflow, latest carried
// partial.  kKsFoldBlocks workgroups each fold a strided
// slice (one workgroup alone was bound by its own CU's load rate) and merge
// it with one atomic per field.
constexpr int kKsFoldBlocks = 64;
__global__ __launch_bounds__(256) void k_ks_tfold(const PrepAgg* __restrict__ blk, int nb, PrepAgg* __restrict__ out) {
  PrepAcc acc;
  constexpr int U = 4;   // partials per thread per round, loaded together
  const int stride = kKsFoldBlocks * 256;
  for (int b0 = blockIdx.x * 256 + threadIdx.x; b0 < nb; b0 += U * stride) {
    unsigned long long c[U], o[U], u[U];
    long long lo[U], hi[U], ch[U];
#pragma unroll
    for (int i = 0; i < U; i++) {
      const bool in = b0 + i * stride < nb;
      const PrepAgg& x = blk[in ? b0 + i * stride : b0];
      c[i] = in ? x.n_cand : 0ull;
      o[i] = x.ovf;
      u[i] = x.unmono;
      lo[i] = x.ts_min;
      hi[i] = x.ts_max;
      ch[i] = x.carry_tmax;
    }
#pragma unroll
    for (int i = 0; i < U; i++) {
      acc.created += c[i];
      acc.ovf |= o[i];
      acc.unmono |= u[i];
      acc.tmin = lo[i] < acc.tmin ? lo[i] : acc.tmin;
      acc.tmax = hi[i] > acc.tmax ? hi[i] : acc.tmax;
      acc.ctmax = ch[i] > acc.ctmax ? ch[i] : acc.ctmax;
    }
  }
  __shared__ PrepAgg r1[1];
  prep_block_reduce<256>(acc, r1, 0);
  __syncthreads();
  if (threadIdx.x == 0) {
    const PrepAgg r = r1[0];
    if (r.n_cand) atomicAdd(&out->n_cand, r.n_cand);
    if (r.ovf) atomicOr(&out->ovf, r.ovf);
    if (r.unmono) atomicOr(&out->unmono, r.unmono);
    if (r.ts_min != LLONG_MAX) atomicMin(&out->ts_min, r.ts_min);
    if (r.ts_max != LLONG_MIN) atomicMax(&out->ts_max, r.ts_max);
    if (r.carry_tmax != LLONG_MIN) atomicMax(&out->carry_tmax, r.carry_tmax);
  }
}

}  // namespace

int keyed_sort_f1_attr(const DFilters& f1, bool is_a) {
  if (!is_a) return -1;
  if (!f1.fp.ok) return -2;
  int attr = -1;
  auto atom = [&](const FAtom& x) {
    if (x.kind != FA_LOAD || x.st != 0 || !(x.idx == 0 || x.idx == SHD_IDX_CURRENT)) return true;
    if (attr >= 0 && attr != x.attr) return false;
    attr = x.attr;
    return true;
  };
  for (int i = 0; i < f1.fp.n; i++) {
    const FCmp& c = f1.fp.c[i];
    if (!atom(c.l.a) || (c.l.aop && !atom(c.l.b)) || !atom(c.r.a) || (c.r.aop && !atom(c.r.b))) return -2;
  }
  return attr;
}

static int64_t ks_tiles(int64_t n_ext) { return (n_ext + kKsTile - 1) / kKsTile; }

// scratch: hraw[nb][256] | offs[nb][256] | csum[nch][256] | cpre[nch][256] | dtot[256] |
//          PrepAgg blk[nb] | PrepAgg cblk[nch]
struct KsScratch {
  uint32_t *hraw, *offs, *csum, *cpre, *dtot;
  PrepAgg *blk, *cblk;
  int nb, nch;
};
static KsScratch ks_scratch(DevBuf& scratch, int64_t n_ext, bool reserve) {
  KsScratch k;
  k.nb = (int)ks_tiles(n_ext);
  k.nch = (k.nb + kKsChunk - 1) / kKsChunk;
  const size_t words = (size_t)2 * k.nb * 256 + (size_t)2 * k.nch * 256 + 256;
  const size_t aoff = (words * 4 + 63) & ~(size_t)63;
  if (reserve) scratch.reserve(aoff + (size_t)(k.nb + k.nch) * sizeof(PrepAgg));
  k.hraw = scratch.as<uint32_t>();
  k.offs = k.hraw + (size_t)k.nb * 256;
  k.csum = k.offs + (size_t)k.nb * 256;
  k.cpre = k.csum + (size_t)k.nch * 256;
  k.dtot = k.cpre + (size_t)k.nch * 256;
  k.blk = reinterpret_cast<PrepAgg*>(scratch.as<char>() + aoff);
  k.cblk = k.blk + k.nb;
  return k;
}

void keyed_sort_front(hipStream_t s, const PrepArgs* d_pa, const PrepArgs& pa, int64_t n_ext, DevBuf& scratch,
                      PrepAgg* d_pg, KsInfo* d_info) {
  const KsScratch k = ks_scratch(scratch, n_ext, true);
  const bool knul = pa.x.batch.nul[pa.key_col] != nullptr;
  if (knul)
    hipLaunchKernelGGL(k_ks_hist<true>, dim3(k.nb), dim3(kRsBlock), 0, s, d_pa, n_ext, k.hraw, k.blk, k.nb);
  else
    hipLaunchKernelGGL(k_ks_hist<false>, dim3(k.nb), dim3(kRsBlock), 0, s, d_pa, n_ext, k.hraw, k.blk, k.nb);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ks_chunk_sum, dim3(k.nch), dim3(256), 0, s, (const uint32_t*)k.hraw, k.nb,
                     (const PrepAgg*)k.blk, k.csum, k.cblk);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ks_finish, dim3(1), dim3(256), 0, s, (const PrepAgg*)k.cblk, k.nch, d_pg, d_info);
  SHD_CHECK_LAUNCH();
}

// f1 pre-resolved for the fused pass (KsF1): FK 1 = no comparison (true);
// FK 2 = one comparison of the attribute (a double column, no conversion)
// with a constant (converted to double once per workgroup), either side;
// FK 0 = eval_fpred per row.
static KsF1 ks_f1(const DFilters& f1, int fattr, const ColSet& cs) {
  KsF1 r{};
  r.kind = 0;
  if (fattr < 0) {
    if (f1.fp.ok && f1.fp.n == 0) r.kind = 1;
    return r;
  }
  if (!f1.fp.ok || f1.fp.n != 1 || cs.type[fattr] != SHD_T_DOUBLE) return r;
  const FCmp& c = f1.fp.c[0];
  if (c.l.aop || c.r.aop || c.type != SHD_T_DOUBLE) return r;
  auto col = [&](const FAtom& x) {
    return x.kind == FA_LOAD && x.attr == fattr && (x.cvt_to < 0 || x.cvt_to == x.cvt_from);
  };
  auto konst = [&](const FAtom& x) { return x.kind == FA_CONST; };
  int op = c.op;
  const FAtom* k = nullptr;
  if (col(c.l.a) && konst(c.r.a)) {
    k = &c.r.a;
  } else if (konst(c.l.a) && col(c.r.a)) {
    k = &c.l.a;
    switch (op) {   // a OP b == b OP' a
      case SHD_OP_GT: op = SHD_OP_LT; break;
      case SHD_OP_LT: op = SHD_OP_GT; break;
      case SHD_OP_GE: op = SHD_OP_LE; break;
      case SHD_OP_LE: op = SHD_OP_GE; break;
      default: break;
    }
  } else {
    return r;
  }
  if (op != SHD_OP_EQ && op != SHD_OP_NE && op != SHD_OP_GT && op != SHD_OP_GE && op != SHD_OP_LT &&
      op != SHD_OP_LE)
    return r;
  r.kind = 2;
  r.op = op;
  r.cval = k->cval;
  r.cvt_from = k->cvt_from;
  r.cvt_to = k->cvt_to;
  return r;
}

void keyed_sort_pass0(hipStream_t s, const PrepArgs* d_pa, const PrepArgs& pa, int fattr, int64_t n_ext,
                      DevBuf& scratch, const KsInfo* d_info, uint32_t* k32, uint32_t* pv, uint32_t* ts,
                      PrepAgg* d_pg) {
  const KsScratch k = ks_scratch(scratch, n_ext, false);
  hipLaunchKernelGGL(k_ks_chunk_scan, dim3(256), dim3(256), 0, s, (const uint32_t*)k.csum, k.nch, k.nb, d_info, n_ext,
                     k.cpre, k.dtot);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ks_offsets, dim3(k.nch), dim3(256), 0, s, (const uint32_t*)k.hraw, k.nb, d_info, n_ext,
                     (const uint32_t*)k.cpre, (const uint32_t*)k.dtot, k.offs);
  SHD_CHECK_LAUNCH();
  const bool knul = pa.x.batch.nul[pa.key_col] != nullptr;
  const bool fnul = fattr >= 0 && pa.x.batch.nul[fattr] != nullptr;
  const int fsz = fattr >= 0 ? type_size(pa.x.batch.type[fattr]) : 0;
  const KsF1 f1 = getenv("SHD_KS_GENERIC_F1") ? KsF1{} : ks_f1(pa.f1, pa.is_a ? fattr : -1, pa.x.batch);
  const int nb = k.nb;
  const uint32_t* hraw = k.hraw;
  const uint32_t* offs = k.offs;
  PrepAgg* blk = k.blk;   // k_ks_hist's partials were folded by k_ks_chunk_sum already
#define SHD_KS_LAUNCH(FSZ, KN, FN, FK)                                                                               \
  hipLaunchKernelGGL((k_ks_scatter0<FSZ, KN, FN, FK>), dim3(nb), dim3(kRsBlock), 0, s, d_pa, n_ext, fattr, f1,      \
                     d_info, hraw, offs, nb, k32, pv, ts, blk)
#define SHD_KS_LAUNCH_N(FSZ, FK)                             \
  do {                                                       \
    if (knul) {                                              \
      if (fnul) SHD_KS_LAUNCH(FSZ, true, true, FK);          \
      else SHD_KS_LAUNCH(FSZ, true, false, FK);              \
    } else {                                                 \
      if (fnul) SHD_KS_LAUNCH(FSZ, false, true, FK);         \
      else SHD_KS_LAUNCH(FSZ, false, false, FK);             \
    }                                                        \
  } while (0)
  if (f1.kind == 2) SHD_KS_LAUNCH_N(8, 2);
  else if (f1.kind == 1 && fsz == 0) SHD_KS_LAUNCH_N(0, 1);
  else {
    switch (fsz) {
      case 8: SHD_KS_LAUNCH_N(8, 0); break;
      case 4: SHD_KS_LAUNCH_N(4, 0); break;
      case 1: SHD_KS_LAUNCH_N(1, 0); break;
      default: SHD_KS_LAUNCH_N(0, 0); break;
    }
  }
#undef SHD_KS_LAUNCH_N
#undef SHD_KS_LAUNCH
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_ks_tfold, dim3(kKsFoldBlocks), dim3(256), 0, s, (const PrepAgg*)blk, nb, d_pg);
  SHD_CHECK_LAUNCH();
}


// The passes after the first (digits from shift 8 up to `bits`), on
// (k32, pv, ts) -> alternate buffers and back; in_alt: the result is in the
// alternate set.  These run on the library's radix passes: a persistent,
// software-pipelined pass kernel with tile-major offsets (the next tile's
// loads issued before the current tile's ranking) was built and measured
// slower on P3 (447 vs 300 us per 56 M-row pass).
void keyed_sort_rest(hipStream_t s, int64_t n_ext, int bits, uint32_t kb, uint32_t* k32, uint32_t* pv, uint32_t* ts,
                     uint32_t* k32_alt, uint32_t* pv_alt, uint32_t* ts_alt, DevBuf&, DevBuf& sort_scratch,
                     bool& in_alt) {
  in_alt = false;
  if (bits <= 8) return;
  radix_sort_triples_u32(k32, pv, ts, k32_alt, pv_alt, ts_alt, n_ext, bits, sort_scratch, s, in_alt, false, kb, 8);
}

}  // namespace pat
}  // namespace shd
