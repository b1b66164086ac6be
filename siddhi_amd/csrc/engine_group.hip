// engine_group.hip -- grouped LDS walk of the pattern engine (partitioned or
// implicitly grouped `every e1=A[f1] -> e2=B[f2] within W`, config P3).
//
// The extended batch (carried partials + pushed events) is stable-sorted by
// the low 16 bits of key_bucket_mix(key) -- two 8-bit hashed LSD passes
// instead of the three a full 24-bit key sort needs.  A group (one 16-bit
// hash value) then holds EVERY row of each of its keys, in arrival order
// (carried partials first), so the reference's per-key processing resolves
// inside the group alone -- no lookahead, no time horizon, nothing retired:
//   StreamPreStateProcessor.processAndReturn / expireEvents for this plan
//   shape (ST/StreamPreStateProcessor.java:118-129,326-403): a partial P_i
//   completes at the first later B event j of its key with f2(P_i, j), unless
//   an event of its key with ts - ts_i > W comes first (expiry); with neither
//   it stays open (carried to the next push).
// One workgroup per group: the group's (key, flags|row, ts32) rows are staged
// in LDS, keys are interned in an LDS hash table, each key's events are
// listed in arrival order (counting-sort layout + in-list ranks), and every
// candidate partial walks its key's later events there.  A group larger than
// the LDS capacity walks the same lists in global memory (rare: the hash
// spreads 10M keys over 65536 groups of ~760 rows).
//
// Bytes: one read of the 12-byte sorted row per position + the outcome byte
// and match row written; f2 reads e1 / e2 attributes only for same-key pairs
// inside `within`.
#include "pattern_common.h"
#include "radix_tile.h"

namespace shd {
namespace pat {

namespace {

constexpr int kGwThreads = 256;
constexpr int kGwCap = 1024;      // rows of a group staged in LDS
constexpr int kGwSlots = 2048;    // LDS key table (load <= 1/2)
constexpr uint64_t kGwEmpty = ~0ull;

__device__ __forceinline__ uint32_t gw_group(uint32_t key, int bits) {
  return key_bucket_mix(key) & ((1u << bits) - 1u);
}

// Group boundaries in the sorted order: gbeg[g] / gend[g] (both 0 for an
// empty group: the arrays are zeroed first).  Four positions per thread (one
// 16-byte load; the previous position's key from the neighbouring lane).
__global__ __launch_bounds__(kBlock) void k_group_bounds(const uint32_t* __restrict__ skey,
                                                         const uint32_t* __restrict__ spv, int64_t n, int bits,
                                                         uint32_t* __restrict__ gbeg, uint32_t* __restrict__ gend) {
  const int64_t nq = (n + 3) >> 2;
  for (int64_t qd = (int64_t)blockIdx.x * kBlock + threadIdx.x; qd < nq; qd += (int64_t)gridDim.x * kBlock) {
    const int64_t p0 = qd << 2;
    uint32_t k[4];
    if (p0 + 3 < n && ((reinterpret_cast<uintptr_t>(skey) & 15) == 0)) {
      const uint4 v = *reinterpret_cast<const uint4*>(skey + p0);
      k[0] = v.x; k[1] = v.y; k[2] = v.z; k[3] = v.w;
    } else {
      for (int j = 0; j < 4; j++) k[j] = p0 + j < n ? skey[p0 + j] : 0u;
    }
    uint32_t prev = p0 > 0 ? gw_group(skey[p0 - 1], bits) : 0xFFFFFFFFu;
    for (int j = 0; j < 4; j++) {
      const int64_t p = p0 + j;
      if (p >= n) break;
      const uint32_t g = gw_group(k[j], bits);
      if (g != prev) {
        if (p > 0) gend[prev] = (uint32_t)p;
        gbeg[g] = (uint32_t)p;
      }
      if (p == n - 1) gend[g] = (uint32_t)n;
      prev = g;
    }
  }
}

// The walk of candidate partial i over its key's later events e (ascending
// positions): the reference's outcome (expiry / match / open) and the
// (partial, event) pairs it examined.
template <bool FAST, class EvAt>
__device__ __forceinline__ uint8_t gw_walk(const ScanArgs& a, const DExprSet& es, int64_t r, int64_t tsi, int n_ev,
                                           const EvAt& ev_at, int32_t& mrow, uint64_t& steps, uint32_t& viol) {
  int64_t prev = tsi;
  uint8_t pend = 0;   // met a B event: pending list (PS_PEND)
  for (int k = 0; k < n_ev; k++) {
    uint32_t pv;
    int64_t tq;
    ev_at(k, pv, tq);
    if (a.within != INT64_MAX && tq < prev) {   // a per-key time regression: generic NFA engine
      viol = 1;
      return PS_NONE;
    }
    prev = tq;
    steps++;
    if (tq - tsi > a.within) return PS_NONE;   // stabilizeStates -> expireEvents
    if (pv_flags(pv) & F_B) {
      pend = PS_PEND;
      PairCtx cx{&a.x, r, (int64_t)pv_row(pv), a.s_first};
      if (FAST ? eval_fpred(a.f2.fp, cx) : eval_filters(es, a.f2, cx)) {
        mrow = (int32_t)pv_row(pv);
        return PS_MATCH;
      }
    }
  }
  return PS_OPEN | pend;
}

template <bool FAST>
__global__ __launch_bounds__(kGwThreads) void k_group_walk(const ScanArgs* __restrict__ ap, int ngroups, int bits,
                                                            const uint32_t* __restrict__ gbeg,
                                                            const uint32_t* __restrict__ gend,
                                                            const uint32_t* __restrict__ skey,
                                                            const uint32_t* __restrict__ spv,
                                                            const int32_t* __restrict__ sts,
                                                            int32_t* __restrict__ match_row, uint8_t* __restrict__ pst,
                                                            ScanOut* __restrict__ blk) {
  const ScanArgs& a = *ap;
  const DExprSet es = a.es;
  __shared__ uint32_t lkey[kGwCap];
  __shared__ uint32_t lpv[kGwCap];
  __shared__ int32_t lts[kGwCap];
  __shared__ uint16_t lslot[kGwCap];
  __shared__ uint16_t lidx[kGwCap];   // an event's index in its key's ordered list
  __shared__ uint16_t lst[kGwCap];    // per-key event lists (unordered fill)
  __shared__ uint16_t lsorted[kGwCap];
  __shared__ unsigned long long tkey[kGwSlots];
  __shared__ uint32_t tcnt[kGwSlots];   // events per slot, then the fill counter
  __shared__ uint16_t tbase[kGwSlots];
  __shared__ uint32_t wsum[kGwThreads / 64];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t tbase_ts = a.x.batch.ts[0];
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0;
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int64_t q0 = gbeg[g], q1 = gend[g];
    const int len = (int)(q1 - q0);
    if (len <= 0) continue;
    if (len > kGwCap) {
      // oversized group: the same lists walked in global memory (each
      // candidate scans the group forward for its key)
      for (int i = tid; i < len; i += kGwThreads) {
        const int64_t q = q0 + i;
        const uint32_t pv = spv[q];
        uint8_t out = PS_NONE;
        if (pv_flags(pv) & F_CAND) {
          const uint32_t k = skey[q];
          const int64_t tsi = tbase_ts + (int64_t)sts[q];
          // its key's events after it, in position order
          int64_t nxt = q + 1;
          auto ev_at = [&](int, uint32_t& pvo, int64_t& tq) {
            while (true) {
              const uint32_t pq = spv[nxt];
              if (skey[nxt] == k && (pv_flags(pq) & F_NEW) && !(pv_flags(pq) & F_SKIP)) {
                pvo = pq;
                tq = tbase_ts + (int64_t)sts[nxt];
                nxt++;
                return;
              }
              nxt++;
            }
          };
          int n_ev = 0;
          for (int64_t y = q + 1; y < q1; y++) {
            const uint32_t py = spv[y];
            n_ev += (skey[y] == k && (pv_flags(py) & F_NEW) && !(pv_flags(py) & F_SKIP)) ? 1 : 0;
          }
          int32_t mrow = -1;
          out = gw_walk<FAST>(a, es, (int64_t)pv_row(pv), tsi, n_ev, ev_at, mrow, steps, viol);
          if (out == PS_MATCH) match_row[q] = mrow;
          if ((out & 0x7F) == PS_OPEN && a.prune && a.t_end - tsi > a.within) {
            out = PS_NONE;
            pruned++;
          }
        }
        pst[q] = out;
      }
      continue;
    }
    // ---- stage the group (all loads issued before the LDS stores)
    {
      constexpr int kPer = kGwCap / kGwThreads;
      uint32_t rk[kPer], rp[kPer];
      int32_t rt[kPer];
#pragma unroll
      for (int j = 0; j < kPer; j++) {
        const int i = tid + j * kGwThreads;
        const int64_t q = q0 + (i < len ? i : 0);
        rk[j] = skey[q];
        rp[j] = spv[q];
        rt[j] = sts[q];
      }
      __syncthreads();   // the previous group's readers are done
#pragma unroll
      for (int j = 0; j < kPer; j++) {
        const int i = tid + j * kGwThreads;
        if (i < len) {
          lkey[i] = rk[j];
          lpv[i] = rp[j];
          lts[i] = rt[j];
        }
      }
      for (int s = tid; s < kGwSlots; s += kGwThreads) {
        tkey[s] = kGwEmpty;
        tcnt[s] = 0;
      }
    }
    __syncthreads();
    // ---- intern the keys of events and candidates; count events per key
    for (int i = tid; i < len; i += kGwThreads) {
      const uint32_t f = pv_flags(lpv[i]);
      const bool ev = (f & F_NEW) && !(f & F_SKIP);
      if (!ev && !(f & F_CAND)) continue;
      const unsigned long long k = lkey[i];
      // (every key of the group shares the low 16 bits of key_bucket_mix: the
      // table slot comes from another multiplicative hash's top bits)
      uint32_t s = (lkey[i] * 0x85EBCA6Bu) >> (32 - 11);
      static_assert(kGwSlots == 1 << 11, "slot bits");
      while (true) {
        const unsigned long long old = atomicCAS(&tkey[s], kGwEmpty, k);
        if (old == kGwEmpty || old == k) break;
        s = (s + 1) & (kGwSlots - 1);
      }
      lslot[i] = (uint16_t)s;
      if (ev) atomicAdd(&tcnt[s], 1u);
    }
    __syncthreads();
    // ---- list bases: exclusive scan of the per-slot event counts
    {
      constexpr int kPerS = kGwSlots / kGwThreads;
      uint32_t c[kPerS], sum = 0;
#pragma unroll
      for (int j = 0; j < kPerS; j++) {
        c[j] = tcnt[tid * kPerS + j];
        sum += c[j];
      }
      uint32_t inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      uint32_t pre = inc - sum;
      for (int k = 0; k < w; k++) pre += wsum[k];
#pragma unroll
      for (int j = 0; j < kPerS; j++) {
        tbase[tid * kPerS + j] = (uint16_t)pre;
        pre += c[j];
        tcnt[tid * kPerS + j] = 0;   // from here: fill counter
      }
    }
    __syncthreads();
    for (int i = tid; i < len; i += kGwThreads) {
      const uint32_t f = pv_flags(lpv[i]);
      if (!((f & F_NEW) && !(f & F_SKIP))) continue;
      const uint32_t s = lslot[i];
      lst[tbase[s] + atomicAdd(&tcnt[s], 1u)] = (uint16_t)i;
    }
    __syncthreads();
    // order each key's list by position (lists are short: rank by counting)
    for (int i = tid; i < len; i += kGwThreads) {
      const uint32_t f = pv_flags(lpv[i]);
      if (!((f & F_NEW) && !(f & F_SKIP))) continue;
      const uint32_t s = lslot[i];
      const int b = tbase[s], c = (int)tcnt[s];
      int rank = 0;
      for (int y = 0; y < c; y++) rank += lst[b + y] < i ? 1 : 0;
      lsorted[b + rank] = (uint16_t)i;
      lidx[i] = (uint16_t)(b + rank);
    }
    __syncthreads();
    // ---- every candidate walks its key's later events
    for (int i = tid; i < len; i += kGwThreads) {
      const uint32_t pv = lpv[i];
      const uint32_t f = pv_flags(pv);
      uint8_t out = PS_NONE;
      if (f & F_CAND) {
        const uint32_t s = lslot[i];
        const int b = tbase[s], end = b + (int)tcnt[s];
        // carried partials precede every event of the push (stable sort)
        const int from = ((f & F_NEW) && !(f & F_SKIP)) ? lidx[i] + 1 : b;
        auto ev_at = [&](int k, uint32_t& pvo, int64_t& tq) {
          const int e = lsorted[from + k];
          pvo = lpv[e];
          tq = tbase_ts + (int64_t)lts[e];
        };
        int32_t mrow = -1;
        const int64_t tsi = tbase_ts + (int64_t)lts[i];
        out = gw_walk<FAST>(a, es, (int64_t)pv_row(pv), tsi, end - from, ev_at, mrow, steps, viol);
        if (out == PS_MATCH) match_row[q0 + i] = mrow;
        // unpartitioned plans (implicit grouping) expire globally: the push's
        // last event expired what is older than `within` (partitioned: prune 0)
        if ((out & 0x7F) == PS_OPEN && a.prune && a.t_end - tsi > a.within) {
          out = PS_NONE;
          pruned++;
        }
      }
      pst[q0 + i] = out;
    }
  }
  // block partials of the scan counters (match / open counts: k_tile_count)
  for (int o = 32; o > 0; o >>= 1) {
    steps += __shfl_xor(steps, o, 64);
    pruned += __shfl_xor(pruned, o, 64);
    viol |= __shfl_xor(viol, o, 64);
  }
  __shared__ ScanOut wpart[kGwThreads / 64];
  if (lane == 0) wpart[w] = ScanOut{steps, pruned, viol, 0};
  __syncthreads();
  if (tid == 0) {
    ScanOut r = wpart[0];
    for (int k = 1; k < kGwThreads / 64; k++) {
      r.steps += wpart[k].steps;
      r.pruned += wpart[k].pruned;
      r.violation |= wpart[k].violation;
    }
    blk[blockIdx.x] = r;
  }
}

// ---------------------------------------------------------------- fused prepare + first hashed pass
// k_prepare's row preparation (prep_row: flags F_CAND / F_NEW / F_B / F_SKIP,
// 32-bit key, ts offset, batch aggregates) fused into the first 8-bit pass of
// the grouped walk's hashed key sort: the prepared rows go straight to their
// digit positions instead of a round trip through HBM.  Every load of a
// lane's R rows -- key, ts, the <= 2 attributes f1 reads, their null bytes --
// is issued before the first use (a row's loads, then the next row's, would
// serialise the memory round trips); f1 is a fast predicate evaluated over
// the preloaded values.  Same results as prep_row (plain 32-bit key column).
struct PreRow {
  Val v0, v1;
  int a0, a1;
  int64_t ts;
};
struct PreCtx {   // BatchRowCtx over preloaded values
  const PreRow* p;
  __device__ __forceinline__ Val load(int st, int idx, int attr) const {
    if (st != 0 || !(idx == 0 || idx == SHD_IDX_CURRENT)) {
      Val v;
      v.b = 0;
      v.null = 1;
      return v;
    }
    return attr == p->a0 ? p->v0 : p->v1;
  }
  __device__ __forceinline__ bool evnull(int st, int idx) const { return !(st == 0 && (idx == 0 || idx == SHD_IDX_CURRENT)); }
  __device__ __forceinline__ int64_t ts(int st, int idx) const { return evnull(st, idx) ? 0 : p->ts; }
  __device__ __forceinline__ Val agg(int) const {
    Val v;
    v.b = 0;
    v.null = 1;
    return v;
  }
};

template <int R>
__global__ __launch_bounds__(kRsBlock) void k_prep_scatter(const PrepArgs* __restrict__ ap, int64_t n_ext,
                                                           const uint32_t* __restrict__ hist,
                                                           const uint32_t* __restrict__ offs,
                                                           const uint32_t* __restrict__ dtotal, int nb, int a0, int a1,
                                                           uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                           uint32_t* __restrict__ tout, PrepAgg* __restrict__ blk) {
  const PrepArgs& a = *ap;
  const ExtRows& x = a.x;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int tile = rs_tile_of(blockIdx.x, nb);
  const int64_t t0 = (int64_t)tile * rs_tile(R);
  const int64_t wb = t0 + (int64_t)w * 64 * R;
  const uint32_t c = tid < 256 ? hist[(int64_t)tid * nb + tile] : 0u;
  const uint32_t gr = tid < 256 ? offs[(int64_t)tid * nb + tile] : 0u;
  const uint32_t dt = tid < 256 ? dtotal[tid] : 0u;
  const int64_t tbase = x.batch.ts[0];
  const int64_t C = x.C;
  const uint32_t* kcol = (const uint32_t*)x.batch.col[a.key_col];
  const uint8_t* knul = x.batch.nul[a.key_col];
  // ---- loads
  PreRow pr[R];
  uint32_t kk[R];
  uint8_t kn[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int64_t idx = wb + r * 64 + lane;
    const int64_t li = idx < n_ext ? idx : n_ext - 1;
    const bool isc = li < C;
    const int64_t br = isc ? 0 : li - C;
    const int64_t cr = isc ? li : 0;
    pr[r].a0 = a0;
    pr[r].a1 = a1;
    if (C > 0 && isc) {
      kk[r] = (uint32_t)a.carry_key[cr];
      kn[r] = 0;
      pr[r].ts = x.carry.ts[cr];
    } else {
      kk[r] = kcol[br];
      kn[r] = knul ? knul[br] : 0;
      pr[r].ts = x.batch.ts[br];
      pr[r].v0 = a0 >= 0 ? col_load(x.batch, br, a0) : Val{};
      pr[r].v1 = a1 >= 0 ? col_load(x.batch, br, a1) : Val{};
    }
  }
  // the row before this wave's first row (unmono: its own predecessor)
  const int64_t first = wb;
  int64_t t_before = 0;
  if (lane == 0 && first > C && first < n_ext) t_before = x.batch.ts[first - C - 1];
  // ---- prepare (prep_row semantics)
  PrepAcc acc;
  uint32_t k[R], v[R], xo[R];
  int64_t tprev_round = 0;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const int64_t idx = wb + r * 64 + lane;
    const bool ok = idx < n_ext;
    const int64_t li = ok ? idx : n_ext - 1;
    const int64_t t = pr[r].ts;
    uint32_t f;
    uint32_t key = 0;
    // predecessor row's ts: lane - 1 of this round, the previous round's lane
    // 63 for lane 0, the row before the wave for the wave's first row
    int64_t tp = __shfl_up(t, 1, 64);
    const int64_t last63 = __shfl(t, 63, 64);
    if (lane == 0) tp = r > 0 ? tprev_round : t_before;
    tprev_round = last63;
    if (li < C) {
      f = F_CAND;
      key = kk[r];
      if (ok) acc.ctmax = t > (long long)acc.ctmax ? t : acc.ctmax;
    } else {
      PreCtx cx{&pr[r]};
      const bool p1 = a.is_a && eval_fpred(a.f1.fp, cx);
      f = F_NEW;
      if (kn[r] && a.null_skip) {
        f |= F_SKIP;
        key = (uint32_t)li;   // no key: spread over the groups (passed over by every walk)
      } else {
        if (a.is_b) f |= F_B;
        if (p1) {
          f |= F_CAND;
          acc.created += ok ? 1u : 0u;
        }
        key = kn[r] ? 0u : kk[r];
      }
      if (ok) {
        acc.tmin = t < acc.tmin ? t : acc.tmin;
        acc.tmax = t > acc.tmax ? t : acc.tmax;
        const bool has_prev = li - C > 0;
        acc.unmono |= (has_prev && tp > t) ? 1ull : 0ull;
      }
    }
    if (ok && !(f & F_SKIP)) {
      acc.kmax = key > acc.kmax ? key : acc.kmax;
      acc.kmin = key < acc.kmin ? key : acc.kmin;
    }
    const int64_t d = t - tbase;
    if (ok) acc.ovf |= d != (int64_t)(int32_t)d;
    k[r] = key;
    v[r] = (f << kRowBits) | (uint32_t)li;
    xo[r] = (uint32_t)(int32_t)d;
  }
  rs_scatter_tile<uint32_t, R, true, true>(k, v, xo, n_ext, t0, wb, 0, c, gr, dt, 0u, kout, vout, tout);
  prep_block_reduce<kRsBlock>(acc, blk, tile);
}

}  // namespace

// Fused prepare + first hashed pass (bits 0..7 of key_bucket_mix), FAST plans
// with a plain 32-bit key column; f1 reads attributes a0 / a1 (-1: none).
// Writes the pass's (key, flags|row, ts32) triples to kout / vout / tout and
// one PrepAgg per tile to blk (fold with k_finish_prep).
int prep_scatter_tiles(int64_t n_ext) { return (int)((n_ext + rs_tile(kPrepRounds) - 1) / rs_tile(kPrepRounds)); }

void launch_prep_scatter(const PrepArgs* d_args, int64_t n_ext, const uint32_t* hist, const uint32_t* offs,
                         const uint32_t* dtot, int nb, int a0, int a1, uint32_t* kout, uint32_t* vout, uint32_t* tout,
                         PrepAgg* blk, hipStream_t s) {
  hipLaunchKernelGGL(k_prep_scatter<kPrepRounds>, dim3(nb), dim3(kRsBlock), 0, s, d_args, n_ext, hist, offs, dtot, nb,
                     a0, a1, kout, vout, tout, blk);
  SHD_CHECK_LAUNCH();
}

namespace {

// ---------------------------------------------------------------- sorted LDS walk
// The exact per-key order inside a hashed group: the group's rows (arrival
// order after the stable 16-bit hashed sort) are staged in LDS and binned by
// 10 more bits of key_bucket_mix(key) (1024 bins; the mix is a bijection, so
// rows of one key share a bin and a bin holds few keys): a counting pass with
// LDS atomics places them, and each row's rank among its bin's rows by arrival
// index restores arrival order inside the bin (stable).  Each candidate then
// walks the later rows of its bin in LDS, passing over other keys' rows: the
// forward scan's semantics (walk_partial: expiry at the first later event of
// the key with ts - ts_i > within, else a B event passing f2 completes it,
// else it stays open -- dormant when every later event would expire it) with
// no global loads but f2's attribute reads.  The group's rows are written back
// in bin order (per key: creation order, all the compaction tail needs) with
// the outcome byte / match row, as the forward scan writes them.
constexpr int kLwThreads = 256;
constexpr int kLwCap = 2048;
constexpr int kLwBins = 1024;
constexpr int kLwPer = kLwCap / kLwThreads;

__device__ __forceinline__ uint32_t lw_bin(uint32_t key) { return (key_bucket_mix(key) >> 16) & (kLwBins - 1); }

template <bool FAST>
__global__ __launch_bounds__(kLwThreads) void k_lds_walk(const ScanArgs* __restrict__ ap, int ngroups,
                                                          const uint32_t* __restrict__ gbeg,
                                                          const uint32_t* __restrict__ gend, uint32_t* __restrict__ skey,
                                                          uint32_t* __restrict__ spv, const int32_t* __restrict__ sts,
                                                          int32_t* __restrict__ match_row, uint8_t* __restrict__ pst,
                                                          ScanOut* __restrict__ blk) {
  const ScanArgs& a = *ap;
  const DExprSet es = a.es;
  __shared__ uint32_t lk[kLwCap];
  __shared__ uint32_t lpv[kLwCap];
  __shared__ int32_t lts[kLwCap];
  __shared__ uint16_t lbin[kLwCap];     // binned (unordered), then arrival-ordered inside each bin
  __shared__ uint16_t lord[kLwCap];
  __shared__ uint32_t cnt[kLwBins];
  __shared__ uint32_t bstart[kLwBins + 1];
  __shared__ uint32_t wsum[kLwThreads / 64];
  __shared__ uint32_t rbase, mbase, lcnt_o, lcnt_m, over_l;
  if (threadIdx.x == 0) {
    lcnt_o = 0;
    lcnt_m = 0;
    over_l = 0;
  }
  __syncthreads();
  __shared__ uint8_t lout[kLwCap];     // per position: the walk's outcome (direct mode)
  __shared__ uint32_t lmrow[kLwCap];   // per position: the match row
  __shared__ uint32_t lpre[kLwThreads];  // per 8-position chunk: (open | match << 16) before it
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t tbase = a.x.batch.ts[0];
  const int64_t W = a.within;
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0, over = 0;
  // software pipeline over this block's groups: the next group's rows are
  // loaded while this one is binned and walked in LDS
  uint32_t nk[kLwPer], np[kLwPer];
  int32_t nt[kLwPer];
  int64_t nq0 = 0, nq1 = 0;
  auto fetch = [&](int gg) {
    nq0 = gbeg[gg];
    nq1 = gend[gg];
    const int nl = (int)(nq1 - nq0);
    if (nl <= 0 || nl > kLwCap) return;
#pragma unroll
    for (int j = 0; j < kLwPer; j++) {
      const int i = tid + j * kLwThreads;
      const int64_t q = nq0 + (i < nl ? i : 0);
      nk[j] = skey[q];
      np[j] = spv[q];
      nt[j] = sts[q];
    }
  };
  if ((int)blockIdx.x < ngroups) fetch(blockIdx.x);
  for (int g = blockIdx.x; g < ngroups; g += gridDim.x) {
    const int64_t q0 = nq0, q1 = nq1;
    const int len = (int)(q1 - q0);
    uint32_t rk[kLwPer], rp[kLwPer];
    int32_t rt[kLwPer];
#pragma unroll
    for (int j = 0; j < kLwPer; j++) {
      rk[j] = nk[j];
      rp[j] = np[j];
      rt[j] = nt[j];
    }
    if (g + (int)gridDim.x < ngroups) fetch(g + gridDim.x);
    if (len <= 0) continue;
    if (len > kLwCap) {   // the host redoes this push on the full key sort
      over += tid == 0 ? 1u : 0u;
      continue;
    }
    __syncthreads();   // the previous group's readers are done
    for (int b = tid; b < kLwBins; b += kLwThreads) cnt[b] = 0;
#pragma unroll
    for (int j = 0; j < kLwPer; j++) {
      const int i = tid + j * kLwThreads;
      if (i < len) {
        lk[i] = rk[j];
        lpv[i] = rp[j];
        lts[i] = rt[j];
      }
    }
    __syncthreads();
    // ---- counting pass: a slot per row in its bin (LDS atomics: unordered)
    uint32_t slot[kLwPer];
#pragma unroll
    for (int j = 0; j < kLwPer; j++) {
      const int i = tid + j * kLwThreads;
      slot[j] = i < len ? atomicAdd(&cnt[lw_bin(rk[j])], 1u) : 0u;
    }
    __syncthreads();
    // bin starts: exclusive scan of cnt (4 bins per thread)
    {
      constexpr int kB = kLwBins / kLwThreads;
      uint32_t c[kB], sum = 0;
#pragma unroll
      for (int j = 0; j < kB; j++) {
        c[j] = cnt[tid * kB + j];
        sum += c[j];
      }
      uint32_t inc = sum;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      uint32_t pre = inc - sum;
      for (int k = 0; k < w; k++) pre += wsum[k];
#pragma unroll
      for (int j = 0; j < kB; j++) {
        bstart[tid * kB + j] = pre;
        pre += c[j];
      }
      if (tid == kLwThreads - 1) bstart[kLwBins] = pre;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kLwPer; j++) {
      const int i = tid + j * kLwThreads;
      if (i < len) lbin[bstart[lw_bin(rk[j])] + slot[j]] = (uint16_t)i;
    }
    __syncthreads();
    // arrival order inside a bin: rank by arrival index among the bin's rows
#pragma unroll
    for (int j = 0; j < kLwPer; j++) {
      const int i = tid + j * kLwThreads;
      if (i < len) {
        const uint32_t bn = lw_bin(rk[j]);
        const int b0 = (int)bstart[bn], b1 = (int)bstart[bn + 1];
        int rank = 0;
        for (int y = b0; y < b1; y++) rank += lbin[y] < (uint16_t)i ? 1 : 0;
        lord[b0 + rank] = (uint16_t)i;
      }
    }
    __syncthreads();
    // ---- walks: each candidate over the later rows of its bin (outcomes in LDS)
    for (int p = tid; p < len; p += kLwThreads) {
      const int i = lord[p];
      const uint32_t pv = lpv[i];
      const uint32_t f = pv_flags(pv);
      const uint32_t k = lk[i];
      uint8_t out = PS_NONE;
      if (f & F_CAND) {
        const int pend_end = (int)bstart[lw_bin(k) + 1];
        const int64_t tsi = tbase + (int64_t)lts[i];
        int64_t prev = tsi;
        uint8_t st = ST_OPEN;
        uint8_t pend = 0;
        int32_t mrow = -1;
        for (int q = p + 1; q < pend_end; q++) {
          const int jj = lord[q];
          if (lk[jj] != k) continue;   // another key of the bin
          const uint32_t pq = lpv[jj];
          const uint32_t fq = pv_flags(pq);
          if ((fq & F_SKIP) || !(fq & F_NEW)) continue;   // a dropped event / a carried partial: not an event
          const int64_t tq = tbase + (int64_t)lts[jj];
          if (W != INT64_MAX && tq < prev) {   // a per-key time regression: generic NFA engine
            viol = 1;
            break;
          }
          prev = tq;
          steps++;
          if (tq - tsi > W) {   // stabilizeStates -> expireEvents
            st = ST_DEAD;
            break;
          }
          if (fq & F_B) {
            pend = PS_PEND;
            PairCtx cx{&a.x, (int64_t)pv_row(pv), (int64_t)pv_row(pq), a.s_first};
            if (FAST ? eval_fpred(a.f2.fp, cx) : eval_filters(es, a.f2, cx)) {
              st = ST_MATCH;
              mrow = (int32_t)pv_row(pq);
              break;
            }
          }
        }
        if (st == ST_MATCH) {
          out = PS_MATCH;
          lmrow[p] = (uint32_t)mrow;
          if (!a.mj) match_row[q0 + p] = mrow;
        } else if (st == ST_OPEN) {
          if (a.prune && a.t_end - tsi > W) {
            pruned++;
            if (a.spill) out = PS_DORM | pend;
          } else {
            out = PS_OPEN | pend;
          }
        }
      }
      if (a.lp && (f & F_NEW) && !(f & F_SKIP)) a.lp[k - a.lp_base] = a.push_idx;
      if (a.direct) {
        lout[p] = out;
      } else {
        skey[q0 + p] = k;
        spv[q0 + p] = pv;
        pst[q0 + p] = out;
      }
    }
    if (a.direct) {
      // ---- the group's matches and carried / dormant partials, in position
      // order (per key: creation order), into this block's regions
      __syncthreads();
      constexpr int kPerT = kLwCap / kLwThreads;
      const int c0 = tid * kPerT;
      uint32_t no = 0, nm = 0;
#pragma unroll
      for (int j = 0; j < kPerT; j++) {
        const int p = c0 + j;
        const uint8_t o = p < len ? lout[p] : (uint8_t)PS_NONE;
        no += (o & 0x7Fu) == a.direct_val ? 1u : 0u;
        nm += o == PS_MATCH ? 1u : 0u;
      }
      // block exclusive scan of (no, nm) packed in one word (each < 2^16)
      const uint32_t v = no | (nm << 16);
      uint32_t inc = v;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      if (lane == 63) wsum[w] = inc;
      __syncthreads();
      uint32_t pre = inc - v, tot = 0;
      for (int kk = 0; kk < kLwThreads / 64; kk++) {
        pre += kk < w ? wsum[kk] : 0u;
        tot += wsum[kk];
      }
      const uint32_t to = tot & 0xFFFFu, tm = tot >> 16;
      const uint32_t base_o = lcnt_o, base_m = lcnt_m;
      const bool fits = base_o + to <= a.region && base_m + tm <= a.region;
      __syncthreads();   // every thread read lcnt_* / wsum
      if (tid == 0) {
        if (!fits) over_l = 1;
        else {
          lcnt_o = base_o + to;
          lcnt_m = base_m + tm;
        }
      }
      if (tid < kLwThreads) lpre[tid] = pre;   // this thread's 8-position chunk: (open, match) before it
      __syncthreads();
      if (fits && !over_l) {
        // strided: every thread takes few rows, so their random operand
        // loads are in flight together (a contiguous chunk would serialise them)
        const SpillCols& d = a.fresh;
        for (int p = tid; p < len; p += kLwThreads) {
          const uint8_t o = lout[p];
          const bool isopen = (o & 0x7Fu) == a.direct_val;
          if (o != PS_MATCH && !isopen) continue;
          uint32_t r2 = lpre[p / kPerT];
          for (int y = p & ~(kPerT - 1); y < p; y++) {
            const uint8_t oy = lout[y];
            r2 += ((oy & 0x7Fu) == a.direct_val ? 1u : 0u) | (oy == PS_MATCH ? 0x10000u : 0u);
          }
          if (o == PS_MATCH) {
            const int64_t ob = (int64_t)blockIdx.x * a.region + base_m + (r2 >> 16);
            a.mj[ob] = lmrow[p];
            a.mi[ob] = pv_row(lpv[lord[p]]);
          } else {
            const int i = lord[p];
            const int64_t ob = (int64_t)blockIdx.x * a.region + base_o + (r2 & 0xFFFFu);
            const int64_t r = (int64_t)pv_row(lpv[i]);
            const ColSet& cs = a.x.cs(r);
            const int64_t row = a.x.row(r);
            for (int c = 0; c < d.ncols; c++) {
              if (!((a.amask >> c) & 1u)) continue;
              const Val vv = col_load(cs, row, c);
              switch (d.types[c]) {
                case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: ((uint32_t*)d.col[c])[ob] = (uint32_t)vv.b; break;
                case SHD_T_LONG: case SHD_T_DOUBLE: ((uint64_t*)d.col[c])[ob] = vv.b; break;
                case SHD_T_BOOL: ((uint8_t*)d.col[c])[ob] = (uint8_t)vv.b; break;
              }
              d.nul[c][ob] = (uint8_t)vv.null;
            }
            d.ts[ob] = tbase + (int64_t)lts[i];
            d.key[ob] = lk[i];
            d.seq[ob] = a.x.seq(r);
            d.pend[ob] = (uint8_t)(((o & PS_PEND) || (r < a.x.C && a.carry_pend[r])) ? 1 : 0);
            if (d.push) d.push[ob] = a.push_idx;
          }
        }
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    steps += __shfl_xor(steps, o, 64);
    pruned += __shfl_xor(pruned, o, 64);
    viol |= __shfl_xor(viol, o, 64);
    over += __shfl_xor(over, o, 64);
  }
  __shared__ ScanOut wpart[kLwThreads / 64];
  if (lane == 0) wpart[w] = ScanOut{steps, pruned, viol, over};
  __syncthreads();
  if (tid == 0) {
    ScanOut r = wpart[0];
    for (int k = 1; k < kLwThreads / 64; k++) {
      r.steps += wpart[k].steps;
      r.pruned += wpart[k].pruned;
      r.violation |= wpart[k].violation;
      r.hbm_walks += wpart[k].hbm_walks;
    }
    if (over_l) r.hbm_walks += 1;   // a region overflowed: the host redoes the push
    blk[blockIdx.x] = r;
    if (a.blk_open) {
      a.blk_open[blockIdx.x] = lcnt_o;
      a.blk_match[blockIdx.x] = lcnt_m;
    }
  }
}

// Block regions of the sorted LDS walk -> contiguous rows: block b's count_b
// rows at [b * region, ...) move to [off_b, off_b + count_b) (one block per region).
__global__ __launch_bounds__(kBlock) void k_region_rows(SpillCols src, SpillCols dst, uint32_t amask, int64_t region,
                                                        const uint32_t* __restrict__ cnt,
                                                        const uint32_t* __restrict__ off) {
  const int b = blockIdx.x;
  const int64_t n = cnt[b];
  const int64_t s0 = (int64_t)b * region, d0 = off[b];
  for (int64_t k = threadIdx.x; k < n; k += kBlock) {
    const int64_t i = s0 + k, o = d0 + k;
    for (int c = 0; c < src.ncols; c++) {
      if (!((amask >> c) & 1u)) continue;
      switch (src.types[c]) {
        case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT:
          ((uint32_t*)dst.col[c])[o] = ((const uint32_t*)src.col[c])[i];
          break;
        case SHD_T_LONG: case SHD_T_DOUBLE: ((uint64_t*)dst.col[c])[o] = ((const uint64_t*)src.col[c])[i]; break;
        case SHD_T_BOOL: ((uint8_t*)dst.col[c])[o] = ((const uint8_t*)src.col[c])[i]; break;
      }
      dst.nul[c][o] = src.nul[c][i];
    }
    dst.ts[o] = src.ts[i];
    dst.key[o] = src.key[i];
    dst.seq[o] = src.seq[i];
    dst.pend[o] = src.pend[i];
  }
}

__global__ __launch_bounds__(kBlock) void k_region_pairs(const uint32_t* __restrict__ sj, const uint32_t* __restrict__ si,
                                                         uint32_t* __restrict__ dj, uint32_t* __restrict__ di,
                                                         int64_t region, const uint32_t* __restrict__ cnt,
                                                         const uint32_t* __restrict__ off) {
  const int b = blockIdx.x;
  const int64_t n = cnt[b];
  const int64_t s0 = (int64_t)b * region, d0 = off[b];
  for (int64_t k = threadIdx.x; k < n; k += kBlock) {
    dj[d0 + k] = sj[s0 + k];
    di[d0 + k] = si[s0 + k];
  }
}

}  // namespace

void launch_region_compact(const SpillCols& src, const SpillCols& dst, uint32_t amask, int64_t region, int nblk,
                           const uint32_t* ocnt, const uint32_t* ooff, const uint32_t* sj, const uint32_t* si,
                           uint32_t* dj, uint32_t* di, const uint32_t* mcnt, const uint32_t* moff, hipStream_t s) {
  hipLaunchKernelGGL(k_region_rows, dim3(nblk), dim3(kBlock), 0, s, src, dst, amask, region, ocnt, ooff);
  SHD_CHECK_LAUNCH();
  hipLaunchKernelGGL(k_region_pairs, dim3(nblk), dim3(kBlock), 0, s, sj, si, dj, di, region, mcnt, moff);
  SHD_CHECK_LAUNCH();
}

int group_walk_blocks(int ngroups) { return ngroups < 8192 ? ngroups : 8192; }

int lds_walk_cap() { return kLwCap; }

void launch_lds_walk(const ScanArgs* d_args, bool fast, int64_t n_ext, int bits, uint32_t* skey, uint32_t* spv,
                     const int32_t* sts, uint32_t* gbeg, uint32_t* gend, int32_t* match_row, uint8_t* pst,
                     ScanOut* blk, int nblk, hipStream_t s) {
  const int ngroups = 1 << bits;
  SHD_HIP(hipMemsetAsync(gbeg, 0, (size_t)ngroups * 4, s));
  SHD_HIP(hipMemsetAsync(gend, 0, (size_t)ngroups * 4, s));
  hipLaunchKernelGGL(k_group_bounds, dim3(grid_for(n_ext, 1, 4096)), dim3(kBlock), 0, s, skey, spv, n_ext, bits, gbeg,
                     gend);
  SHD_CHECK_LAUNCH();
  if (fast)
    hipLaunchKernelGGL(k_lds_walk<true>, dim3(nblk), dim3(kLwThreads), 0, s, d_args, ngroups, (const uint32_t*)gbeg,
                       (const uint32_t*)gend, skey, spv, sts, match_row, pst, blk);
  else
    hipLaunchKernelGGL(k_lds_walk<false>, dim3(nblk), dim3(kLwThreads), 0, s, d_args, ngroups, (const uint32_t*)gbeg,
                       (const uint32_t*)gend, skey, spv, sts, match_row, pst, blk);
  SHD_CHECK_LAUNCH();
}

void launch_group_walk(const ScanArgs* d_args, bool fast, int64_t n_ext, int bits, const uint32_t* skey,
                       const uint32_t* spv, const int32_t* sts, uint32_t* gbeg, uint32_t* gend, int32_t* match_row,
                       uint8_t* pst, ScanOut* blk, hipStream_t s) {
  const int ngroups = 1 << bits;
  SHD_HIP(hipMemsetAsync(gbeg, 0, (size_t)ngroups * 4, s));
  SHD_HIP(hipMemsetAsync(gend, 0, (size_t)ngroups * 4, s));
  hipLaunchKernelGGL(k_group_bounds, dim3(grid_for(n_ext, 1, 4096)), dim3(kBlock), 0, s, skey, spv, n_ext, bits, gbeg,
                     gend);
  SHD_CHECK_LAUNCH();
  const int nb = group_walk_blocks(ngroups);
  if (fast)
    hipLaunchKernelGGL(k_group_walk<true>, dim3(nb), dim3(kGwThreads), 0, s, d_args, ngroups, bits,
                       (const uint32_t*)gbeg, (const uint32_t*)gend, skey, spv, sts, match_row, pst, blk);
  else
    hipLaunchKernelGGL(k_group_walk<false>, dim3(nb), dim3(kGwThreads), 0, s, d_args, ngroups, bits,
                       (const uint32_t*)gbeg, (const uint32_t*)gend, skey, spv, sts, match_row, pst, blk);
  SHD_CHECK_LAUNCH();
}

}  // namespace pat
}  // namespace shd
