// engine_pattern.hip -- device engine for the two-state pattern
//     every e1=A[f1] -> e2=B[f2] (within W)        [optionally inside `partition with`]
// i.e. configs P1 and P3 (BASELINE.json configs[0], configs[2]).
//
// Reference semantics (modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/input/stream/state/StreamPreStateProcessor.java:326-403 (expire, process)
//   query/input/stream/state/StreamPostStateProcessor.java:64-83 (match, every clone)
//   query/input/stream/state/receiver/PatternMultiProcessStreamReceiver.java:31-51
//   query/input/MultiProcessStreamReceiver.java:155-183 (reverse state order,
//   deferred per-(event, state) callback chunks).
// For this plan shape the reference NFA reduces to independent partials: the
// e1 start state always holds exactly one start partial, every f1 match i
// creates one partial P_i that becomes visible to e2 from the next event of
// its key on, stays pending until it matches or expires, and never interacts
// with other partials.  With per-key non-decreasing timestamps the prefix
// expiry (break on first non-expired, :331-342) equals "alive while
// ts_j - ts_i <= W", so
//     P_i completes at the first B event j > i of its key with f2(P_i, x_j)
//     before the first event of its key with ts - ts_i > W,
// and the matches of event j come out in P_i creation order.  The kernels
// evaluate exactly that, per partial in parallel, over key-sorted micro-batches;
// open partials carry to the next push.  A per-key timestamp decrease is
// detected on device and the query continues on the generic NFA engine with
// its open partials (NeedNfa hand-over, shd_api.cpp switch_to_nfa), never
// approximated.
#include <algorithm>
#include <unordered_map>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "engine.h"
#include "pattern_common.h"

namespace shd {

using namespace pat;

namespace {

// Per extended row: key and packed (flags, row) sort payload (prep_row), for
// the key sort of the sort path.
template <bool FAST>
__global__ __launch_bounds__(kBlock) void k_prepare(const PrepArgs* __restrict__ ap, int64_t n_ext, int64_t stride,
                                                    uint32_t* __restrict__ k32, uint64_t* __restrict__ k64,
                                                    uint32_t* __restrict__ pv, int32_t* __restrict__ tso,
                                                    PrepAgg* __restrict__ blk) {
  const PrepArgs& a = *ap;
  const DExprSet es = a.es;
  PrepAcc acc;
  const int64_t tbase = a.x.batch.ts[0];
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n_ext; r += stride) {
    uint64_t k;
    uint32_t f;
    int32_t t32;
    prep_row<FAST>(a, es, r, tbase, true, k, f, t32, acc);
    if (a.partitioned) {
      if (a.key64) k64[r] = k;
      else k32[r] = (uint32_t)k;
    }
    pv[r] = (f << kRowBits) | (uint32_t)r;
    tso[r] = t32;
  }
  prep_block_reduce<kBlock>(acc, blk, blockIdx.x);
}

__global__ __launch_bounds__(kBlock) void k_finish_prep(const PrepAgg* blk, int nblk, PrepAgg* out) {
  unsigned long long c = 0, km = 0, ov = 0, um = 0, kn = ULLONG_MAX;
  long long tmin = LLONG_MAX, tmax = LLONG_MIN, ctm = LLONG_MIN;
#pragma unroll 8
  for (int b = threadIdx.x; b < nblk; b += kBlock) {
    ov |= blk[b].ovf;
    um |= blk[b].unmono;
    kn = blk[b].kmin < kn ? blk[b].kmin : kn;
    ctm = blk[b].carry_tmax > ctm ? blk[b].carry_tmax : ctm;
    c += blk[b].n_cand;
    km = blk[b].kmax > km ? blk[b].kmax : km;
    tmin = blk[b].ts_min < tmin ? blk[b].ts_min : tmin;
    tmax = blk[b].ts_max > tmax ? blk[b].ts_max : tmax;
  }
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o, 64);
    ov |= __shfl_xor(ov, o, 64);
    um |= __shfl_xor(um, o, 64);
  }
  km = wave_max(km);
  kn = wave_min(kn);
  tmin = wave_min(tmin);
  tmax = wave_max(tmax);
  ctm = wave_max(ctm);
  __shared__ PrepAgg wpart[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = PrepAgg{c, km, tmin, tmax, ov, um, ctm, kn};
  __syncthreads();
  if (threadIdx.x == 0) {
    PrepAgg r = wpart[0];
    for (int w = 1; w < kBlock / 64; w++) {
      r.ovf |= wpart[w].ovf;
      r.unmono |= wpart[w].unmono;
      r.carry_tmax = wpart[w].carry_tmax > r.carry_tmax ? wpart[w].carry_tmax : r.carry_tmax;
      r.kmin = wpart[w].kmin < r.kmin ? wpart[w].kmin : r.kmin;
      r.n_cand += wpart[w].n_cand;
      r.kmax = wpart[w].kmax > r.kmax ? wpart[w].kmax : r.kmax;
      r.ts_min = wpart[w].ts_min < r.ts_min ? wpart[w].ts_min : r.ts_min;
      r.ts_max = wpart[w].ts_max > r.ts_max ? wpart[w].ts_max : r.ts_max;
    }
    *out = r;
  }
}

__global__ void k_narrow_keys(const uint64_t* in, uint32_t* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)in[i];
}

// Overflow path (a timestamp offset does not fit in 32 bits): full event
// timestamps at sorted positions, gathered by row after the key sort.
__global__ __launch_bounds__(kBlock) void k_sorted_ts64(const ExtRows* __restrict__ xp,
                                                        const uint32_t* __restrict__ spv, int64_t n,
                                                        int64_t* __restrict__ sts64) {
  const ExtRows& x = *xp;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n; p = n) sts64[p] = x.ts(pv_row(spv[p]));
}

// d_agg layout: PrepAgg at 0, ScanOut at 64, match / open totals at 128
static_assert(sizeof(PrepAgg) <= 64 && sizeof(ScanOut) <= 64, "d_agg layout");

#include "pattern_walk.h"

// Per-block reduction of the scan counters: ScanOut partial at blk[slot] and
// the tile's match / open counts (plain store, or added for the resume pass).
__device__ __forceinline__ void scan_block_reduce(uint64_t steps, uint64_t pruned, uint32_t viol, uint32_t nm,
                                                  uint32_t no, ScanOut* blk, int slot, uint32_t* bcnt, int tile,
                                                  int ntile, bool add, uint32_t nd = 0) {
  for (int o2 = 32; o2 > 0; o2 >>= 1) {
    steps += __shfl_xor(steps, o2, 64);
    pruned += __shfl_xor(pruned, o2, 64);
    viol |= __shfl_xor(viol, o2, 64);
    nm += __shfl_xor(nm, o2, 64);
    no += __shfl_xor(no, o2, 64);
    nd += __shfl_xor(nd, o2, 64);
  }
  __shared__ ScanOut wpart[kBlock / 64];
  __shared__ uint32_t wcnt[3][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    wpart[threadIdx.x >> 6] = ScanOut{steps, pruned, viol};
    wcnt[0][threadIdx.x >> 6] = nm;
    wcnt[1][threadIdx.x >> 6] = no;
    wcnt[2][threadIdx.x >> 6] = nd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    ScanOut r = wpart[0];
    uint32_t tm = wcnt[0][0], to = wcnt[1][0], td = wcnt[2][0];
    for (int w = 1; w < kBlock / 64; w++) {
      r.steps += wpart[w].steps;
      r.pruned += wpart[w].pruned;
      r.violation |= wpart[w].violation;
      tm += wcnt[0][w];
      to += wcnt[1][w];
      td += wcnt[2][w];
    }
    blk[slot] = r;
    if (add) {
      if (tm) atomicAdd(&bcnt[tile], tm);
      if (to) atomicAdd(&bcnt[ntile + tile], to);
    } else {
      bcnt[tile] = tm;                // matches of this tile
      bcnt[ntile + tile] = to;        // still-open partials of this tile
      bcnt[2 * ntile + tile] = td;    // deferred walks of this tile (k_forward_scan)
    }
  }
}

// AND: a partial's filled-operand state as the carry stores it, match_row =
// filled operand row | fm << kRowBits (0 when no operand is filled).  A carried
// half-filled partial holds its operand event at ext row C + n + (carry row).
__device__ __forceinline__ void and_carried(const ScanArgs& a, int64_t r, uint32_t& fm, int64_t& ra, int64_t& rb) {
  fm = 0;
  ra = rb = -1;
  if (r < a.x.C) {
    fm = a.carry_half[r];
    const int64_t hr = a.x.C + a.x.batch.n + r;
    if (fm & 1u) ra = hr;
    if (fm & 2u) rb = hr;
  }
}
__device__ __forceinline__ int32_t and_code(uint32_t fm, int64_t ra, int64_t rb) {
  return fm == 0 ? 0 : (int32_t)((fm & 1u ? ra : rb) | ((int64_t)fm << kRowBits));
}
__device__ __forceinline__ int32_t and_open_code(const ScanArgs& a, int64_t r) {
  uint32_t fm;
  int64_t ra, rb;
  and_carried(a, r, fm, ra, rb);
  return and_code(fm, ra, rb);
}

// One lane per position; candidates walk forward over the later events of
// their key (sorted positions when partitioned, ext rows otherwise).  Keys,
// flags and timestamps are read at sorted positions (timestamps travel with
// the key sort), so the walk is sequential.  A walk that reaches a B event
// inside `within` is deferred to k_forward_resume (pst = PS_DEFER, resume
// position in match_row).  Writes a 1-byte outcome per position and the
// per-tile match / open counts.
// HASH: hashed-bucket positions (walks fetch 4 positions per round trip).
template <bool K64, bool TS64, bool HASH>
__global__ __launch_bounds__(kBlock) void k_forward_scan(const ScanArgs* __restrict__ ap, int64_t n_ext,
                                                         int64_t tile, const uint32_t* __restrict__ skey32,
                                                         const uint64_t* __restrict__ skey64,
                                                         const uint32_t* __restrict__ spv,
                                                         const int32_t* __restrict__ sts32,
                                                         const int64_t* __restrict__ sts64,
                                                         int32_t* __restrict__ match_row, uint8_t* __restrict__ pst,
                                                         uint32_t* __restrict__ bcnt, ScanOut* __restrict__ blk) {
  const ScanArgs& a = *ap;
  const DExprSet es{};
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0, nm = 0, no = 0, nd = 0;
  // this block's contiguous tile of positions (compaction offsets are per block)
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n_ext ? t0 + tile : n_ext;
  // sorted timestamps: 32-bit offsets from the batch's first event, or full
  // 64-bit values when some offset overflowed (separate instantiation: a
  // run-time choice merges the two loads and serialises every load after it)
  const int64_t tbase = TS64 ? 0 : a.x.batch.ts[0];
  auto visit = [&](int64_t p, const auto& ld) {
    uint32_t pvp, pq;
    int64_t tsi, tq;
    uint64_t k = 0, kq = 0;
    // the position and its first successor are loaded together before use
    const int64_t q0 = p + 1 < n_ext ? p + 1 : n_ext - 1;
    ld(p, pvp, tsi, k);
    ld(q0, pq, tq, kq);
    uint8_t out = PS_NONE;
    if (pv_flags(pvp) & F_CAND) {
      int64_t q = p + 1;
      int32_t j = -1;
      uint32_t fm = 0;
      int64_t ra = -1, rb = -1;
      const uint8_t st = walk_partial<true, false, HASH ? 4 : 1>(a, es, n_ext, ld, pv_row(pvp), k, tsi, q, pq, tq,
                                                                 kq, tsi, false, j, steps, viol, fm, ra, rb);
      if (st == ST_DEFER) {
        out = PS_DEFER;
        match_row[p] = (int32_t)q;   // resume position (< 2^28)
        nd++;
      } else if (st == ST_OPEN) {
        out = PS_OPEN;
        no++;
        if (a.logical == 2) match_row[p] = and_open_code(a, pv_row(pvp));   // carried half state unchanged
      } else if (st == ST_PRUNED) {
        pruned++;   // every later event is at or after t_end: it would expire this partial
      }
    }
    pst[p] = out;
  };
  const GlobalPos<K64, TS64> ld{skey32, skey64, spv, sts32, sts64, tbase, a.partitioned};
  for (int64_t p = t0 + threadIdx.x; p < t1; p += kBlock) visit(p, ld);
  scan_block_reduce(steps, pruned, viol, nm, no, blk, blockIdx.x, bcnt, blockIdx.x, gridDim.x, false, nd);
}

// Position-major copy of the e2-side attributes the filters read (ExtRows::bpos):
// dst column a, position p = batch row of position p (carried rows are e1
// partials, never evaluated as e2 events).
__global__ __launch_bounds__(kBlock) void k_gather_bpos(const ExtRows* __restrict__ xp, const uint32_t* spv,
                                                       int64_t n_ext) {
  const ExtRows& x = *xp;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < n_ext; p += (int64_t)gridDim.x * kBlock) {
    const int64_t r = pv_row(spv[p]);
    // carried rows are e1 partials: only their e1-side operands (apos_mask)
    const uint32_t m = r < x.C ? x.apos_mask : (x.bpos_mask | x.apos_mask);
    for (int c = 0; c < x.batch.ncols; c++) {
      if (!((m >> c) & 1u)) continue;
      const Val v = r < x.C ? col_load(x.carry, r, c) : col_load(x.batch, r - x.C, c);
      switch (x.bpos.type[c]) {
        case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: ((uint32_t*)x.bpos.col[c])[p] = (uint32_t)v.b; break;
        case SHD_T_LONG: case SHD_T_DOUBLE: ((uint64_t*)x.bpos.col[c])[p] = v.b; break;
        case SHD_T_BOOL: ((uint8_t*)x.bpos.col[c])[p] = (uint8_t)v.b; break;
      }
      ((uint8_t*)x.bpos.nul[c])[p] = (uint8_t)v.null;
    }
  }
}

// Block summaries for skipping walks (BlockSum): one wave per 64 sorted
// positions (32-bit keys and timestamps).
__global__ __launch_bounds__(kBlock) void k_block_sum(const ScanArgs* __restrict__ ap, int64_t n_ext,
                                                     const uint32_t* __restrict__ skey32,
                                                     const uint32_t* __restrict__ spv,
                                                     const int32_t* __restrict__ sts32, BlockSum* __restrict__ out) {
  const ScanArgs& a = *ap;
  const ExtRows& x = a.x;
  const int lane = threadIdx.x & 63;
  const int64_t nblk = (n_ext + 63) >> 6;
  const int64_t tbase = x.batch.ts[0];
  const int attr = a.bs_attr;
  const bool usemax = a.bs_op == SHD_OP_GT || a.bs_op == SHD_OP_GE;
  for (int64_t b = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6; b < nblk;
       b += ((int64_t)gridDim.x * kBlock) >> 6) {
    const int64_t p = (b << 6) + lane;
    const bool valid = p < n_ext;
    const uint32_t pv = valid ? spv[p] : 0u;
    const int64_t t = valid ? tbase + (int64_t)sts32[p] : 0;
    const uint32_t key = (valid && a.partitioned) ? skey32[p] : 0u;
    const uint32_t f = pv_flags(pv);
    const bool keyed = valid && !(f & F_SKIP);
    const bool nw = keyed && (f & F_NEW);
    double dv = usemax ? -__builtin_inf() : __builtin_inf();
    if (nw && (f & F_B)) {
      const int64_t r = pv_row(pv);
      const Val v = ((x.bpos_mask >> attr) & 1u) ? col_load(x.bpos, p, attr)
                    : (r < x.C ? col_load(x.carry, r, attr) : col_load(x.batch, r - x.C, attr));
      if (!v.null) {
        const double d = v_f64(v.b);
        if (d == d) dv = d;   // NaN never passes a comparison
      }
    }
    dv = usemax ? wave_max(dv) : wave_min(dv);
    const uint64_t km = __ballot(keyed), nm = __ballot(nw);
    const uint32_t k0 = km ? __shfl(key, __ffsll((unsigned long long)km) - 1, 64) : 0u;
    const bool uniform = __ballot(keyed && key != k0) == 0;
    // running max of the earlier F_NEW times: a decrease breaks monotonicity
    int64_t m = nw ? t : INT64_MIN;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = __shfl_up(m, o, 64);
      if (lane >= o) m = u > m ? u : m;
    }
    int64_t before = __shfl_up(m, 1, 64);
    if (lane == 0) before = INT64_MIN;
    const bool mono = __ballot(nw && t < before) == 0;
    const int64_t tfirst = nm ? __shfl(t, __ffsll((unsigned long long)nm) - 1, 64) : 0;
    const int64_t tlast = __shfl(m, 63, 64);
    if (lane == 0) {
      BlockSum o;
      o.key = k0;
      o.cnt = (uint16_t)__popcll(nm);
      o.flags = (uint8_t)((uniform ? 1u : 0u) | (mono ? 2u : 0u) | (km ? 0u : 4u));
      o.pad = 0;
      o.tfirst = tfirst;
      o.tlast = tlast;
      o.v = dv;
      o.newmask = nm;
      out[b] = o;
    }
  }
}

// The f2 comparison block skipping can answer from a block's max / min: a
// double comparison (> >= < <=) between a plain e2 attribute (state s2, no
// conversion) and a term free of e2.  Normalised to `e2.attr op threshold`.
static bool block_skip_term(const FPred& fp, int s2, int& ci, int& side, int& op, int& attr) {
  auto is_e2 = [&](const FTerm& t) {
    return t.aop == 0 && t.a.kind == FA_LOAD && t.a.st == s2 && (t.a.idx == 0 || t.a.idx == SHD_IDX_CURRENT) &&
           t.a.cvt_to < 0;
  };
  auto no_e2 = [&](const FTerm& t) {
    auto ok = [&](const FAtom& x) { return x.kind != FA_LOAD || x.st == 0; };
    return ok(t.a) && (t.aop == 0 || ok(t.b));
  };
  auto flip = [](int o) {
    return o == SHD_OP_GT ? SHD_OP_LT : o == SHD_OP_LT ? SHD_OP_GT : o == SHD_OP_GE ? SHD_OP_LE : SHD_OP_GE;
  };
  for (int i = 0; i < fp.n && i < 4; i++) {
    const FCmp& c = fp.c[i];
    if (c.type != SHD_T_DOUBLE) continue;
    if (c.op != SHD_OP_GT && c.op != SHD_OP_GE && c.op != SHD_OP_LT && c.op != SHD_OP_LE) continue;
    if (is_e2(c.l) && no_e2(c.r)) {
      ci = i, side = 0, op = c.op, attr = c.l.a.attr;
      return true;
    }
    if (is_e2(c.r) && no_e2(c.l)) {
      ci = i, side = 1, op = flip(c.op), attr = c.r.a.attr;
      return true;
    }
  }
  return false;
}

// Split f2 (F2Split) for the plain form: every comparison either reads no
// e2 attribute (decided once per partial) or compares one plain e2 attribute
// load (+ conversion) with a term free of e2.  False: eval_fpred per step.
static bool split_f2(const FPred& fp, int s2, const ExtRows& x, F2Split& sp) {
  sp = F2Split{};
  if (!fp.ok || fp.n > kSplitMax) return false;
  auto e2dep = [&](const FAtom& t) { return t.kind == FA_LOAD && t.st == s2; };
  auto dep = [&](const FTerm& t) { return e2dep(t.a) || (t.aop != 0 && e2dep(t.b)); };
  for (int i = 0; i < fp.n; i++) {
    const FCmp& c = fp.c[i];
    SplitCmp& o = sp.c[i];
    o.op = c.op;
    o.type = c.type;
    const bool dl = dep(c.l), dr = dep(c.r);
    if (!dl && !dr) {
      o.konst = 1;
      continue;
    }
    if (dl && dr) return false;
    const FTerm& e = dl ? c.l : c.r;
    if (e.aop != 0 || (e.a.idx != 0 && e.a.idx != SHD_IDX_CURRENT)) return false;
    const int attr = e.a.attr;
    if (attr < 0 || attr >= x.batch.ncols || attr >= kMaxCols) return false;
    o.swap = dr ? 1 : 0;
    o.pos = (x.bpos_mask >> attr) & 1u;
    const ColSet& cs = o.pos ? x.bpos : x.batch;
    o.col = cs.col[attr];
    o.nul = cs.nul[attr];
    o.ctype = cs.type[attr];
    o.cvt_from = e.a.cvt_from;
    o.cvt_to = e.a.cvt_to;
    // pre-resolved kinds (split_eval): the operator flipped so e2 is on the left
    const bool cvt = o.cvt_to >= 0 && o.cvt_to != o.cvt_from;
    const bool rel = c.op == SHD_OP_EQ || c.op == SHD_OP_NE || c.op == SHD_OP_GT || c.op == SHD_OP_GE ||
                     c.op == SHD_OP_LT || c.op == SHD_OP_LE;
    o.kind = SK_GENERIC;
    if (rel && c.type == SHD_T_DOUBLE && o.ctype == SHD_T_FLOAT && cvt && o.cvt_from == SHD_T_FLOAT &&
        o.cvt_to == SHD_T_DOUBLE)
      o.kind = SK_F32_F64;
    else if (rel && c.type == SHD_T_DOUBLE && o.ctype == SHD_T_DOUBLE && !cvt)
      o.kind = SK_F64;
    else if ((c.op == SHD_OP_EQ || c.op == SHD_OP_NE) && c.type == SHD_T_STRING && o.ctype == SHD_T_STRING && !cvt)
      o.kind = SK_STR_EQ;
    else if (rel && c.type == SHD_T_INT && o.ctype == SHD_T_INT && !cvt)
      o.kind = SK_I32;
    if (o.kind != SK_GENERIC && o.swap) {
      switch (c.op) {
        case SHD_OP_GT: o.op = SHD_OP_LT; break;
        case SHD_OP_GE: o.op = SHD_OP_LE; break;
        case SHD_OP_LT: o.op = SHD_OP_GT; break;
        case SHD_OP_LE: o.op = SHD_OP_GE; break;
      }
    }
  }
  sp.n = fp.n;
  sp.ok = 1;
  return true;
}

// Cooperative walk (resume MODE 2): the 64 lanes of a wave scan ONE deferred
// partial's later positions 64 at a time (coalesced loads, f2 evaluated for all
// of them at once) and ballot the first terminating position -- the same
// outcome as walk_partial's sequential walk: the first of {f2 match, expiry
// (ts - tsi > within), end of the key's run, end of the push, timestamp
// decrease} in position order.  A lane-per-partial walk keeps a wave busy for
// its longest walk; here a partial that completes early costs one round and
// one that never matches ceil(window / 64) rounds.  Plain and OR forms only
// (an AND partial's operand state is sequential).
template <bool FAST, bool SKIP, class Ld>
__device__ __forceinline__ void coop_resume(const ScanArgs& a, const DExprSet& es, int64_t n_ext, const Ld& ld,
                                            int64_t p, bool cont, int32_t* __restrict__ match_row,
                                            int32_t* __restrict__ match_other, uint8_t* __restrict__ pst,
                                            uint64_t& steps, uint64_t& pruned,
                                            uint32_t& viol, uint32_t& nm, uint32_t& no) {
  const int lane = threadIdx.x & 63;
  uint32_t pvp, pd;
  int64_t tsi, td;
  uint64_t k = 0, kd = 0;
  ld(p, pvp, tsi, k);
  int64_t q0 = match_row[p];
  // deferred (PS_DEFER): q0 is the B event where f2 comes first, its step
  // already counted; continued (PS_CONT): q0 is unprocessed, the last walked
  // position precedes it
  ld(cont ? q0 - 1 : q0, pd, td, kd);
  const int64_t r = pv_row(pvp);
  int64_t prev = td;   // time of the last step taken (running-order check)
  if (cont && (!(pv_flags(pd) & F_NEW) || (pv_flags(pd) & F_SKIP) || (a.partitioned && kd != k))) prev = tsi;
  bool first = !cont;
  uint8_t st = ST_OPEN;
  int32_t j = -1;
  // AND (operand filters that do not read the partner slot): each operand
  // fills at its first passing position; state carried between rounds
  uint32_t fm = 0;
  int64_t ra = -1, rb = -1;
  int32_t other = -1;
  if (a.logical == 2) and_carried(a, r, fm, ra, rb);
  // split f2: the partial's side once (the same for every lane)
  SplitThr sth;
  if (FAST && a.sp.ok && !a.logical) sth = split_prep(a, r, p);
  uint64_t wsteps = 0;
  bool wviol = false;
  bool thr_ok = false;
  Val thr;
  thr.b = 0;
  thr.null = 1;
  while (q0 < n_ext) {
    if (SKIP && !first && (q0 & 63) == 0 && q0 + 64 <= n_ext) {
      // a whole 64-position block without an outcome is skipped (block_skippable)
      if (!thr_ok) {
        thr = skip_threshold(a, r, p);
        thr_ok = true;
      }
      const BlockSum bs = a.bsum[q0 >> 6];
      if (block_skippable(a, bs, k, tsi, prev, thr)) {
        wsteps += bs.cnt;
        if (bs.cnt) prev = bs.tlast;
        q0 += 64;
        continue;
      }
    }
    // with block skipping, rounds end on 64-position block boundaries
    const int64_t qend = SKIP ? ((q0 | 63) + 1) : q0 + 64;
    const int64_t q = q0 + lane;
    const bool act = q < qend;
    const bool inb = act && q < n_ext;
    uint32_t pq = 0;
    int64_t tq = 0;
    uint64_t kq = 0;
    if (inb) ld(q, pq, tq, kq);
    const uint32_t fq = pv_flags(pq);
    const bool f0 = first && lane == 0;   // the deferred B event: f2 is evaluated there directly
    const bool skip = (fq & F_SKIP) != 0;
    const bool endkey = inb && !f0 && a.partitioned && kq != k && !skip;
    const bool isnew = inb && !f0 && !endkey && (fq & F_NEW) && !skip;
    // running maximum of the earlier steps' times (a decrease is a violation)
    int64_t m = isnew ? tq : INT64_MIN;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t t = __shfl_up(m, o, 64);
      if (lane >= o) m = t > m ? t : m;
    }
    int64_t before = __shfl_up(m, 1, 64);
    if (lane == 0) before = INT64_MIN;
    before = before > prev ? before : prev;
    const bool vio = isnew && a.within != INT64_MAX && tq < before;
    const bool expire = isnew && !vio && tq - tsi > a.within;
    const uint64_t stopm = __ballot(act && (!inb || endkey || vio || expire));
    const int sidx = stopm ? __ffsll((unsigned long long)stopm) - 1 : 64;
    bool hit = false;
    int32_t code = 0;
    if (a.logical == 2) {
      const bool cand = lane < sidx && (f0 || (isnew && (fq & F_B)));
      const int64_t r2 = pv_row(pq);
      bool ha = false, hb = false;
      if (cand && !(fm & 1u)) {
        PairCtx cx{&a.x, r, r2, a.s_first};
        cx.q2 = q;
        cx.q1 = p;
        ha = FAST ? eval_fpred(a.f2.fp, cx) : eval_filters(es, a.f2, cx);
      }
      if (cand && !(fm & 2u)) {
        PairCtx cx{&a.x, r, r2, a.s_second};
        cx.q2 = q;
        cx.q1 = p;
        hb = FAST ? eval_fpred(a.f3.fp, cx) : eval_filters(es, a.f3, cx);
      }
      const uint64_t am = __ballot(ha), bm = __ballot(hb);
      // fill positions in this round (-1: filled in an earlier round)
      int ia = (fm & 1u) ? -1 : (am ? __ffsll((unsigned long long)am) - 1 : 64);
      int ib = (fm & 2u) ? -1 : (bm ? __ffsll((unsigned long long)bm) - 1 : 64);
      if (ia >= 0 && ia < 64) {
        fm |= 1u;
        ra = __shfl(r2, ia, 64);
      }
      if (ib >= 0 && ib < 64) {
        fm |= 2u;
        rb = __shfl(r2, ib, 64);
      }
      const int term2 = fm == 3u ? (ia > ib ? ia : ib) : sidx;
      const uint64_t upto2 = term2 >= 63 ? ~0ull : ((2ull << term2) - 1ull);
      wsteps += (uint64_t)__popcll(__ballot(isnew && !vio) & upto2);
      if (fm == 3u) {
        // the processor that fills last completes it; on one event the second
        // operand's processor comes last
        const int br = ib >= ia ? 1 : 0;
        st = ST_MATCH;
        j = (int32_t)__shfl(r2, term2, 64) | (br << kRowBits);
        other = (int32_t)(br ? ra : rb);
        break;
      }
      if (sidx < 64) {
        const int kind = __shfl(vio ? 2 : (expire ? 1 : 0), sidx, 64);
        if (kind == 2) wviol = true;
        else if (kind == 1) st = ST_DEAD;
        break;
      }
      prev = __shfl(m, 63, 64) > prev ? __shfl(m, 63, 64) : prev;
      first = false;
      q0 = qend;
      continue;
    }
    if (lane < sidx && (f0 || (isnew && (fq & F_B)))) {
      const int64_t r2 = pv_row(pq);
      PairCtx cx{&a.x, r, r2, a.s_first};
      cx.q2 = q;
      cx.q1 = p;
      if (FAST && a.sp.ok && !a.logical) hit = split_eval(a.sp, sth, r2 - a.x.C, q);
      else hit = FAST ? eval_fpred(a.f2.fp, cx) : eval_filters(es, a.f2, cx);
      int32_t br = 0;
      if (!hit && a.logical) {
        cx.s2 = a.s_second;
        hit = FAST ? eval_fpred(a.f3.fp, cx) : eval_filters(es, a.f3, cx);
        br = 1;
      }
      code = (int32_t)r2 | (br << kRowBits);
    }
    const uint64_t hm = __ballot(hit);
    const int fidx = hm ? __ffsll((unsigned long long)hm) - 1 : 64;
    const int term = fidx < sidx ? fidx : sidx;
    const uint64_t upto = term >= 63 ? ~0ull : ((2ull << term) - 1ull);
    wsteps += (uint64_t)__popcll(__ballot(isnew && !vio) & upto);
    if (fidx < sidx) {
      st = ST_MATCH;
      j = __shfl(code, fidx, 64);
      break;
    }
    if (sidx < 64) {
      const int kind = __shfl(vio ? 2 : (expire ? 1 : 0), sidx, 64);
      if (kind == 2) wviol = true;
      else if (kind == 1) st = ST_DEAD;
      break;
    }
    prev = __shfl(m, 63, 64) > prev ? __shfl(m, 63, 64) : prev;
    first = false;
    q0 = qend;
  }
  if (st == ST_OPEN && a.prune && a.t_end - tsi > a.within) st = ST_PRUNED;
  if (lane == 0) {
    steps += wsteps;
    if (wviol) viol = 1;
    uint8_t out = PS_NONE;
    if (st == ST_MATCH) {
      out = PS_MATCH;
      match_row[p] = j;
      if (a.logical == 2) match_other[p] = other;
      nm++;
    } else if (st == ST_OPEN) {
      out = PS_OPEN | PS_PEND;
      no++;
      if (a.logical == 2) match_row[p] = and_code(fm, ra, rb);
    } else if (st == ST_PRUNED) {
      pruned++;
    }
    pst[p] = out;
  }
}

// Deferred walks: positions whose walk reached a B event inside `within`
// evaluate f2 there (FAST: pre-decoded predicate, else the interpreter) and
// continue.  Same tiles as k_forward_scan.  MODE 2: one wave per deferred
// partial (coop_resume); MODE 1: one position per lane per round; MODE 0: each
// thread scans 16 outcome bytes and resumes its hits in turn.
template <bool K64, bool FAST, bool TS64, int MODE, bool SKIP = false>
__global__ __launch_bounds__(kBlock) void k_forward_resume(const ScanArgs* __restrict__ ap, int64_t n_ext,
                                                           int64_t tile, const uint32_t* __restrict__ skey32,
                                                           const uint64_t* __restrict__ skey64,
                                                           const uint32_t* __restrict__ spv,
                                                           const int32_t* __restrict__ sts32,
                                                           const int64_t* __restrict__ sts64,
                                                           int32_t* __restrict__ match_row,
                                                           int32_t* __restrict__ match_other,
                                                           uint8_t* __restrict__ pst, uint32_t* __restrict__ bcnt,
                                                           ScanOut* __restrict__ blk, int slot0) {
  const ScanArgs& a = *ap;
  const DExprSet es = a.es;
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0, nm = 0, no = 0;
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n_ext ? t0 + tile : n_ext;
  const int64_t tbase = TS64 ? 0 : a.x.batch.ts[0];
  const GlobalPos<K64, TS64> ld{skey32, skey64, spv, sts32, sts64, tbase, a.partitioned};
  auto resume_one = [&](int64_t p) {
      int64_t q = match_row[p];
      uint32_t pvp, pq;
      int64_t tsi, tq;
      uint64_t k = 0, kq = 0;
      ld(p, pvp, tsi, k);
      ld(q, pq, tq, kq);
      int32_t j = -1;
      uint32_t fm = 0;
      int64_t ra = -1, rb = -1;
      if (a.logical == 2) and_carried(a, pv_row(pvp), fm, ra, rb);
      const uint8_t st = walk_partial<false, FAST, 1, GlobalPos<K64, TS64>, 0, SKIP>(a, es, n_ext, ld, pv_row(pvp), k, tsi, q, pq, tq, kq, tq, true,
                                                      j, steps, viol, fm, ra, rb, p);
      uint8_t out = PS_NONE;
      if (st == ST_MATCH) {
        out = PS_MATCH;
        match_row[p] = j;
        // AND: the partner operand's row (the completing processor is bit kRowBits)
        if (a.logical == 2) match_other[p] = (int32_t)((j >> kRowBits) ? ra : rb);
        nm++;
      } else if (st == ST_OPEN) {
        out = PS_OPEN | PS_PEND;   // it met a B event of its key: in the pending list now
        no++;
        if (a.logical == 2) match_row[p] = and_code(fm, ra, rb);
      } else if (st == ST_PRUNED) {
        pruned++;
      }
      pst[p] = out;
  };
  if constexpr (MODE == 2) {
    // one wave per deferred / continued partial, the wave's 64-position slices in turn
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int64_t base = t0 + (int64_t)w * 64; base < t1; base += kBlock) {
      const int64_t pp = base + lane;
      const uint8_t o = pp < t1 ? pst[pp] : (uint8_t)PS_NONE;
      uint64_t dm = __ballot(o == PS_DEFER || o == PS_CONT);
      const uint64_t cm = __ballot(o == PS_CONT);
      while (dm) {
        const int b = __ffsll((unsigned long long)dm) - 1;
        dm &= dm - 1;
        coop_resume<FAST, SKIP>(a, es, n_ext, ld, base + b, (cm >> b) & 1ull, match_row, match_other, pst, steps, pruned,
                          viol, nm, no);
      }
    }
  } else if constexpr (MODE == 3) {
    // lane walks capped at 64 positions; longer ones go on in the MODE 2 pass
    for (int64_t p = t0 + threadIdx.x; p < t1; p += kBlock) {
      if (pst[p] != PS_DEFER) continue;
      int64_t q = match_row[p];
      uint32_t pvp, pq;
      int64_t tsi, tq;
      uint64_t k = 0, kq = 0;
      ld(p, pvp, tsi, k);
      ld(q, pq, tq, kq);
      int32_t j = -1;
      uint32_t fm = 0;
      int64_t ra = -1, rb = -1;
      const uint8_t st = walk_partial<false, FAST, 1, GlobalPos<K64, TS64>, 64, SKIP>(
          a, es, n_ext, ld, pv_row(pvp), k, tsi, q, pq, tq, kq, tq, true, j, steps, viol, fm, ra, rb, p);
      uint8_t out = PS_NONE;
      if (st == ST_MATCH) {
        out = PS_MATCH;
        match_row[p] = j;
        nm++;
      } else if (st == ST_OPEN) {
        out = PS_OPEN | PS_PEND;
        no++;
      } else if (st == ST_PRUNED) {
        pruned++;
      } else if (st == ST_YIELD) {
        out = PS_CONT;
        match_row[p] = (int32_t)q;
      }
      pst[p] = out;
    }
  } else if constexpr (MODE == 1) {
    // one position per lane per round: when most candidates defer (walks over
    // every event of a busy key or of the whole stream) the walks of
    // neighbouring positions run side by side, not one after another in a lane
    for (int64_t p = t0 + threadIdx.x; p < t1; p += kBlock)
      if (pst[p] == PS_DEFER) resume_one(p);
  } else {
    // few deferrals (sparse keys): 16 outcome bytes per thread per 16-byte load
    for (int64_t c0 = t0; c0 < t1; c0 += kBlock * 16) {
      const int64_t pb = c0 + (int64_t)threadIdx.x * 16;
      if (pb >= t1) continue;
      const uint4 raw = *reinterpret_cast<const uint4*>(pst + pb);
      const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
      uint32_t hit = 0;
#pragma unroll
      for (int i = 0; i < 16; i++)
        if (((wv[i >> 2] >> ((i & 3) * 8)) & 255u) == PS_DEFER && pb + i < t1) hit |= 1u << i;
      while (hit) {
        const int64_t p = pb + __ffs(hit) - 1;
        hit &= hit - 1;
        resume_one(p);
      }
    }
  }
  scan_block_reduce(steps, pruned, viol, nm, no, blk, slot0 + blockIdx.x, bcnt, blockIdx.x, gridDim.x, true);
}

// Deferred walks from a list (sparse keys): the deferred positions, compacted
// in position order by k_open_list (val PS_DEFER), one lane each -- every
// lane of a wave walks, where the per-tile MODE 0 pass leaves a wave with a
// few walking lanes among outcome-byte scans.  Same walk as MODE 0/1
// (walk_partial from the deferred B event); a position's match / open counts
// go to its own tile's slots, the walk counters to ScanOut partials
// [slot0, slot0 + gridDim.x).  The list length is read on the device.
template <bool K64, bool FAST, bool TS64>
__global__ __launch_bounds__(kBlock) void k_resume_list(const ScanArgs* __restrict__ ap, int64_t n_ext, int64_t tile,
                                                        int ntile, const uint32_t* __restrict__ skey32,
                                                        const uint64_t* __restrict__ skey64,
                                                        const uint32_t* __restrict__ spv,
                                                        const int32_t* __restrict__ sts32,
                                                        const int64_t* __restrict__ sts64,
                                                        int32_t* __restrict__ match_row,
                                                        int32_t* __restrict__ match_other, uint8_t* __restrict__ pst,
                                                        uint32_t* __restrict__ bcnt, ScanOut* __restrict__ blk,
                                                        int slot0, const uint32_t* __restrict__ dlist,
                                                        const uint32_t* __restrict__ dcount) {
  const ScanArgs& a = *ap;
  const DExprSet es = a.es;
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0;
  const int64_t tbase = TS64 ? 0 : a.x.batch.ts[0];
  const GlobalPos<K64, TS64> ld{skey32, skey64, spv, sts32, sts64, tbase, a.partitioned};
  const int64_t cnt = *dcount;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < cnt; i += (int64_t)gridDim.x * kBlock) {
    const int64_t p = dlist[i];
    int64_t q = match_row[p];
    uint32_t pvp, pq;
    int64_t tsi, tq;
    uint64_t k = 0, kq = 0;
    ld(p, pvp, tsi, k);
    ld(q, pq, tq, kq);
    int32_t j = -1;
    uint32_t fm = 0;
    int64_t ra = -1, rb = -1;
    if (a.logical == 2) and_carried(a, pv_row(pvp), fm, ra, rb);
    const uint8_t st = walk_partial<false, FAST, 1, GlobalPos<K64, TS64>, 0, false>(
        a, es, n_ext, ld, pv_row(pvp), k, tsi, q, pq, tq, kq, tq, true, j, steps, viol, fm, ra, rb, p);
    uint8_t out = PS_NONE;
    const int t = (int)(p / tile);
    if (st == ST_MATCH) {
      out = PS_MATCH;
      match_row[p] = j;
      if (a.logical == 2) match_other[p] = (int32_t)((j >> kRowBits) ? ra : rb);
      atomicAdd(&bcnt[t], 1u);
    } else if (st == ST_OPEN) {
      out = PS_OPEN | PS_PEND;   // it met a B event of its key: in the pending list now
      if (a.logical == 2) match_row[p] = and_code(fm, ra, rb);
      atomicAdd(&bcnt[ntile + t], 1u);
    } else if (st == ST_PRUNED) {
      pruned++;
    }
    pst[p] = out;
  }
  scan_block_reduce(steps, pruned, viol, 0u, 0u, blk, slot0 + blockIdx.x, bcnt, 0, ntile, true);
}

// Lockstep walks (plain `e1 -> e2` form, full-key sort, pre-decoded f2): one
// lane per position as in k_forward_scan, but f2 is evaluated in the walk
// itself, so every candidate of a wave starts at its successor and all of
// them advance one position per round -- at round d lane i reads position
// base + i + d: the key / payload / time / e2-attribute loads of a wave are
// one contiguous 64-position slice per round (coalesced, and each slice
// overlaps the previous one by 63 positions in L1/L2), where the deferred
// walks start at scattered B events.  Same steps and outcomes as
// walk_partial; a walk that has met a B event and still runs after 64
// positions is handed to the wave-cooperative pass (PS_CONT, resume position
// in match_row).  Writes the per-tile counts like k_forward_scan.
template <bool TS64>
__global__ __launch_bounds__(kBlock, 8) void k_lockstep_walk(const ScanArgs* __restrict__ ap, int64_t n_ext, int64_t tile,
                                                          const uint32_t* __restrict__ skey32,
                                                          const uint32_t* __restrict__ spv,
                                                          const int32_t* __restrict__ sts32,
                                                          const int64_t* __restrict__ sts64,
                                                          int32_t* __restrict__ match_row, uint8_t* __restrict__ pst,
                                                          uint32_t* __restrict__ bcnt, ScanOut* __restrict__ blk) {
  const ScanArgs& a = *ap;
  uint64_t steps = 0, pruned = 0;
  uint32_t viol = 0, nm = 0, no = 0;
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n_ext ? t0 + tile : n_ext;
  const int64_t tbase = TS64 ? 0 : a.x.batch.ts[0];
  const GlobalPos<false, TS64> ld{skey32, nullptr, spv, sts32, sts64, tbase, a.partitioned};
  for (int64_t p = t0 + threadIdx.x; p < t1; p += kBlock) {
    uint32_t pvp;
    int64_t tsi;
    uint64_t k = 0;
    ld(p, pvp, tsi, k);
    uint8_t out = PS_NONE;
    if (pv_flags(pvp) & F_CAND) {
      const int64_t r = pv_row(pvp);
      uint8_t st = ST_OPEN;
      bool metb = false;
      // split f2: the partial's side up front (its loads overlap the first
      // position's)
      SplitThr sth;
      if (a.sp.ok) sth = split_prep(a, r, p);
      int32_t j = -1;
      int64_t prev = tsi;
      int64_t q = p + 1;
      // software pipeline: position q + 1 is loaded while q's f2 operand
      // load is in flight (one memory round trip per step, not two; two
      // deep -- q + 1's operands too -- measured slower: 11.6 vs 10.1 ms per
      // P3-dense step, the extra registers cost occupancy)
      uint32_t pn = 0;
      int64_t tn = 0;
      uint64_t kn = 0;
      if (q < n_ext) ld(q, pn, tn, kn);
      for (int d = 0; q < n_ext; q++, d++) {
        if (d >= 64 && metb) {
          st = ST_YIELD;
          break;
        }
        const uint32_t pq = pn;
        const int64_t tq = tn;
        const uint64_t kq = kn;
        if (q + 1 < n_ext) ld(q + 1, pn, tn, kn);
        const uint32_t fq = pv_flags(pq);
        if (fq & F_SKIP) continue;   // dropped (null-key) rows: passed over
        if (kq != k) break;          // end of the key's run
        if (!(fq & F_NEW)) continue;
        if (a.within != INT64_MAX && tq < prev) {
          viol = 1;
          break;
        }
        prev = tq;
        steps++;
        if (tq - tsi > a.within) {
          st = ST_DEAD;
          break;
        }
        if (fq & F_B) {
          bool hit;
          if (a.sp.ok) {
            hit = split_eval(a.sp, sth, (int64_t)pv_row(pq) - a.x.C, q);
          } else {
            PairCtx cx{&a.x, r, (int64_t)pv_row(pq), a.s_first};
            cx.q2 = q;
            cx.q1 = p;
            hit = eval_fpred(a.f2.fp, cx);
          }
          metb = true;
          if (hit) {
            st = ST_MATCH;
            j = (int32_t)pv_row(pq);
            break;
          }
        }
      }
      if (st == ST_OPEN && a.prune && a.t_end - tsi > a.within) st = ST_PRUNED;
      if (st == ST_MATCH) {
        out = PS_MATCH;
        match_row[p] = j;
        nm++;
      } else if (st == ST_OPEN) {
        out = metb ? (uint8_t)(PS_OPEN | PS_PEND) : (uint8_t)PS_OPEN;
        no++;
      } else if (st == ST_PRUNED) {
        pruned++;
      } else if (st == ST_YIELD) {
        out = PS_CONT;
        match_row[p] = (int32_t)q;
      }
    }
    pst[p] = out;
  }
  scan_block_reduce(steps, pruned, viol, nm, no, blk, blockIdx.x, bcnt, blockIdx.x, gridDim.x, false);
}

// Per-tile match / open counts of the outcome bytes (the compaction tiles of
// k_emit_pairs / k_gather_carry): 16 bytes per thread per round.
__global__ __launch_bounds__(kBlock) void k_tile_count(const uint8_t* __restrict__ pst, int64_t n, int64_t tile,
                                                       uint32_t* __restrict__ bcnt) {
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n ? t0 + tile : n;
  uint32_t nm = 0, no = 0;
  for (int64_t pb = t0 + (int64_t)threadIdx.x * 16; pb < t1; pb += kBlock * 16) {
    const uint4 raw = *reinterpret_cast<const uint4*>(pst + pb);
    const uint32_t wv[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 16; i++) {
      const uint32_t o = (wv[i >> 2] >> ((i & 3) * 8)) & 255u;
      const bool in = pb + i < t1;
      nm += (in && o == PS_MATCH) ? 1u : 0u;
      no += (in && (o & 0x7Fu) == PS_OPEN) ? 1u : 0u;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    nm += __shfl_xor(nm, o, 64);
    no += __shfl_xor(no, o, 64);
  }
  __shared__ uint32_t ws[2][kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    ws[0][threadIdx.x >> 6] = nm;
    ws[1][threadIdx.x >> 6] = no;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t a = 0, b = 0;
    for (int k = 0; k < kBlock / 64; k++) {
      a += ws[0][k];
      b += ws[1][k];
    }
    bcnt[blockIdx.x] = a;
    bcnt[gridDim.x + blockIdx.x] = b;
  }
}

// Stable compaction of one block's tile: position p with pst[p] == want gets
// output index base + (# such positions before p in the tile).  Each thread
// takes 16 consecutive outcome bytes per round (one 16-byte load; tiles start
// on 256-byte boundaries and pst is padded by kCompactPad bytes), block-wide
// exclusive scan of the per-thread counts, then emits its positions in order.
constexpr int kCompactPad = kBlock * 16;
template <class F>
__device__ __forceinline__ void tile_compact(const uint8_t* __restrict__ pst, int64_t t0, int64_t t1, uint8_t want,
                                             uint32_t base, F&& emit) {
  __shared__ uint32_t wsum[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t c0 = t0; c0 < t1; c0 += kBlock * 16) {
    const int64_t pb = c0 + (int64_t)threadIdx.x * 16;
    uint32_t wv[4] = {0u, 0u, 0u, 0u};
    if (pb < t1) {
      const uint4 raw = *reinterpret_cast<const uint4*>(pst + pb);
      wv[0] = raw.x;
      wv[1] = raw.y;
      wv[2] = raw.z;
      wv[3] = raw.w;
    }
    uint32_t hit = 0;   // bit i: position pb + i is wanted
#pragma unroll
    for (int i = 0; i < 16; i++)
      if (((wv[i >> 2] >> ((i & 3) * 8)) & 127u) == want && pb + i < t1) hit |= 1u << i;   // (PS_PEND masked)
    const uint32_t cnt = (uint32_t)__popc(hit);
    uint32_t inc = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= o) inc += t;
    }
    if (lane == 63) wsum[w] = inc;
    __syncthreads();
    uint32_t pre = base + inc - cnt, tot = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; k++) {
      if (k < w) pre += wsum[k];
      tot += wsum[k];
    }
    while (hit) {
      const int i = __ffs(hit) - 1;
      hit &= hit - 1;
      emit(pb + i, pre++);
    }
    base += tot;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_finish_scan(const ScanOut* blk, int nblk, ScanOut* out) {
  unsigned long long st = 0, pr = 0;
  uint32_t v = 0;
#pragma unroll 8
  for (int b = threadIdx.x; b < nblk; b += kBlock) {
    st += blk[b].steps;
    pr += blk[b].pruned;
    v |= blk[b].violation;
  }
  for (int o = 32; o > 0; o >>= 1) {
    st += __shfl_xor(st, o, 64);
    pr += __shfl_xor(pr, o, 64);
    v |= __shfl_xor(v, o, 64);
  }
  __shared__ ScanOut wpart[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wpart[threadIdx.x >> 6] = ScanOut{st, pr, v};
  __syncthreads();
  if (threadIdx.x == 0) {
    ScanOut r = wpart[0];
    for (int w = 1; w < kBlock / 64; w++) {
      r.steps += wpart[w].steps;
      r.pruned += wpart[w].pruned;
      r.violation |= wpart[w].violation;
    }
    *out = r;
  }
}

__global__ __launch_bounds__(kBlock) void k_emit_pairs(const uint8_t* pst, const uint32_t* boff,
                                                       const int32_t* match_row, const uint32_t* spv, int64_t n,
                                                       int64_t tile, int logical, const int32_t* match_other,
                                                       uint32_t* pj, uint32_t* pi, uint32_t* se1, int32_t* sot) {
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n ? t0 + tile : n;
  tile_compact(pst, t0, t1, PS_MATCH, boff[blockIdx.x], [&](int64_t p, uint32_t o) {
    const uint32_t mr = (uint32_t)match_row[p];
    // logical: sort key (e2 event, processor order) = row * 2 + branch
    pj[o] = logical ? ((mr & kRowMask) << 1) | (mr >> kRowBits) : mr;
    if (logical == 2) {
      // AND: the pair sort carries the match index; e1 / partner rows stay put
      pi[o] = o;
      se1[o] = pv_row(spv[p]);
      sot[o] = match_other[p];
      return;
    }
    pi[o] = pv_row(spv[p]);
  });
}

struct ProjArgs {
  ExtRows x;
  DExprSet es;
  DExpr outs[kMaxCols];
  int nout;
  int multi;            // chunk per e2 event (same stream) vs per match
  int logical;          // pj = row * 2 + branch; chunk per (event, processor)
  int s_first, s_second;
  const uint32_t* se1;  // AND: pi = match index -> e1 row / partner operand row
  const int32_t* sot;
  int64_t chunk0;
  int64_t row0;         // output buffer offset
  int fast;             // every output is a pre-decoded atom (oat): no bytecode per row
  FAtom oat[kMaxCols];
};

__global__ __launch_bounds__(kBlock) void k_project(const ProjArgs* __restrict__ ap, const uint32_t* pj,
                                                    const uint32_t* pi, int64_t m, int64_t* o_chunk, int32_t* o_type,
                                                    int64_t* o_ts, uint64_t* o_vals, uint8_t* o_nul, int64_t* o_seq,
                                                    int32_t* o_sidx) {
  const ProjArgs& a = *ap;
  const DExprSet es = a.es;
  const ExtRows& x = a.x;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < m; k = m) {
    int64_t j = pj[k], i = pi[k];
    int br = 0;
    if (a.logical) {
      br = (int)(j & 1);
      j >>= 1;
    }
    int64_t other = -1;
    if (a.logical == 2) {
      other = a.sot[i];
      i = a.se1[i];
    }
    PairCtx cx{&x, i, j, br ? a.s_second : a.s_first, true, other, br ? a.s_first : a.s_second};
    int64_t row = a.row0 + k;
    for (int c = 0; c < a.nout; c++) {
      const Val v = a.fast ? fp_atom(a.oat[c], cx) : eval_expr(es.ins + a.outs[c].off, a.outs[c].len, es.consts, cx);
      o_vals[row * a.nout + c] = v.b;
      o_nul[row * a.nout + c] = (uint8_t)v.null;
    }
    o_ts[row] = x.ts(j);
    o_type[row] = 0;
    o_seq[row] = x.seq(j);
    o_sidx[row] = br ? a.s_second : a.s_first;   // the processor that completed the partial
    // MultiProcessStreamReceiver: one callback chunk per (event, processor)
    o_chunk[row] = a.logical ? 2 * x.seq(j) + br : (a.multi ? x.seq(j) : a.chunk0 + k);
  }
}

// ---- query sharing (PatternEngine::group_emit)
// Partials of `every e1=A[f1] -> e2=B[f2] within W` evolve independently: each
// A event passing f1 opens one StateEvent and meets the later events alone
// (StreamPreStateProcessor.java:118-129,326-403; nothing a partial does depends
// on another).  A leader whose e1 filter accepts every event a member's does
// (their disjunction) therefore holds every member partial, with the member's
// outcome, and the member's matches are the leader's match pairs whose e1 row
// passes the member's own f1 -- in the leader's (e2 event, creation) order.
constexpr int kGroupMax = 64;
constexpr int kGroupWaveItems = 8;   // pairs per lane: one wave covers 512 consecutive pairs

struct GroupSelArgs {
  ExtRows x;
  int G;
  DExprSet es[kGroupMax];
  DFilters f1[kGroupMax];
};

// bit g of mask[k]: member g's f1 on the e1 row of pair k
__global__ __launch_bounds__(kBlock) void k_group_mask(const GroupSelArgs* __restrict__ ap, const uint32_t* pi,
                                                       int64_t m, uint64_t* __restrict__ mask) {
  const GroupSelArgs& a = *ap;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < m; k = m) {
    PairCtx cx{&a.x, (int64_t)pi[k], -1, 1, false, -1, -1};
    uint64_t b = 0;
    for (int g = 0; g < a.G; g++)
      if (eval_filters(a.es[g], a.f1[g], cx)) b |= 1ull << g;
    mask[k] = b;
  }
}

// cnt[g * nw + w]: member g's pairs among wave w's 512 pairs.  SCATTER: the
// same walk writes them, in pair order, from off[g * nw + w] on.
template <bool SCATTER>
__global__ __launch_bounds__(kBlock) void k_group_split(const uint64_t* __restrict__ mask, const uint32_t* pj,
                                                        const uint32_t* pi, int64_t m, int G, int64_t nw,
                                                        uint32_t* __restrict__ cnt, uint32_t* __restrict__ gpj,
                                                        uint32_t* __restrict__ gpi) {
  const int lane = threadIdx.x & 63;
  const int64_t w = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;
  if (w >= nw) return;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t mk[kGroupWaveItems];
  uint32_t vj[kGroupWaveItems], vi[kGroupWaveItems];
  for (int s = 0; s < kGroupWaveItems; s++) {
    const int64_t k = w * (64 * kGroupWaveItems) + s * 64 + lane;
    mk[s] = k < m ? mask[k] : 0ull;
    if (SCATTER) {
      vj[s] = k < m ? pj[k] : 0u;
      vi[s] = k < m ? pi[k] : 0u;
    }
  }
  for (int g = 0; g < G; g++) {
    uint32_t base = SCATTER ? cnt[(int64_t)g * nw + w] : 0u;
    for (int s = 0; s < kGroupWaveItems; s++) {
      const bool on = (mk[s] >> g) & 1ull;
      const uint64_t bal = __ballot(on);
      if (SCATTER && on) {
        const uint32_t pos = base + (uint32_t)__popcll(bal & below);
        gpj[pos] = vj[s];
        gpi[pos] = vi[s];
      }
      base += (uint32_t)__popcll(bal);
    }
    if (!SCATTER && lane == 0) cnt[(int64_t)g * nw + w] = base;
  }
}

// bases[g] = first pair of member g in the split lists, bases[G] = their total
__global__ void k_group_bases(const uint32_t* __restrict__ off, const uint32_t* __restrict__ cnt, int G, int64_t nw,
                              uint32_t* __restrict__ bases) {
  const int g = threadIdx.x;
  if (g < G) bases[g] = off[(int64_t)g * nw];
  if (g == G) bases[G] = off[(int64_t)G * nw - 1] + cnt[(int64_t)G * nw - 1];
}

struct GatherArgs {
  ExtRows x;
  int ncols;
  int partitioned;
  int key64;
  int32_t types[kMaxCols];
  void* dcol[kMaxCols];
  uint8_t* dnul[kMaxCols];
  int64_t* dts;
  uint64_t* dkey;
  int64_t* dseq;
  uint32_t amask;   // k_gather_list: stream-A columns to copy
  // k_gather_list: the partial's time from the sorted positions (32-bit
  // offsets from tbase, or 64-bit) and the stream-A attribute that IS the
  // partition key (from the sorted key; -1: none) -- only the other masked
  // attributes are row gathers
  const int32_t* sts32;
  const int64_t* sts64;
  int key_attr;
  // new-list / pending-list placement of each carried partial (export_replay)
  uint8_t* dpend;
  const uint8_t* pend_old;
  // logical AND: filled-operand bits + the held operand event (stream B)
  int and_mode;
  const int32_t* match_row;
  uint8_t* dhalf;
  int ncolsB;
  int32_t typesB[kMaxCols];
  void* dcolB[kMaxCols];
  uint8_t* dnulB[kMaxCols];
  int64_t* dtsB;
  int64_t* dseqB;
};

__device__ __forceinline__ void store_col(void* dst, int type, int64_t o, uint64_t b) {
  switch (type) {
    case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: ((uint32_t*)dst)[o] = (uint32_t)b; break;
    case SHD_T_LONG: case SHD_T_DOUBLE: ((uint64_t*)dst)[o] = b; break;
    case SHD_T_BOOL: ((uint8_t*)dst)[o] = (uint8_t)b; break;
  }
}

// Still-open partials -> next push's carry rows (position order: per key in
// creation order, which is all the stable key sort of the next push needs).
__global__ __launch_bounds__(kBlock) void k_gather_carry(const GatherArgs* __restrict__ ap, const uint8_t* pst,
                                                         const uint32_t* boff, const uint32_t* spv,
                                                         const uint32_t* skey32, const uint64_t* skey64, int64_t n,
                                                         int64_t tile) {
  const GatherArgs& a = *ap;
  const ExtRows& x = a.x;
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n ? t0 + tile : n;
  tile_compact(pst, t0, t1, PS_OPEN, boff[gridDim.x + blockIdx.x], [&](int64_t p, uint32_t o32) {
    const int64_t o = o32;
    int64_t r = pv_row(spv[p]);
    const ColSet& cs = x.cs(r);
    int64_t row = x.row(r);
    for (int c = 0; c < a.ncols; c++) {
      Val v = col_load(cs, row, c);
      switch (a.types[c]) {
        case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: ((uint32_t*)a.dcol[c])[o] = (uint32_t)v.b; break;
        case SHD_T_LONG: case SHD_T_DOUBLE: ((uint64_t*)a.dcol[c])[o] = v.b; break;
        case SHD_T_BOOL: ((uint8_t*)a.dcol[c])[o] = (uint8_t)v.b; break;
      }
      a.dnul[c][o] = (uint8_t)v.null;
    }
    a.dts[o] = x.ts(r);
    a.dkey[o] = !a.partitioned ? 0 : (a.key64 ? skey64[p] : (uint64_t)skey32[p]);
    a.dseq[o] = x.seq(r);
    a.dpend[o] = (uint8_t)(((pst[p] & PS_PEND) || (r < x.C && a.pend_old[r])) ? 1 : 0);
    if (a.and_mode) {
      const uint32_t mr = (uint32_t)a.match_row[p];
      const uint32_t fm = mr >> kRowBits;
      a.dhalf[o] = (uint8_t)fm;
      if (fm) {
        const int64_t hr = mr & kRowMask;
        const ColSet& hc = x.cs(hr);
        const int64_t hrow = x.row(hr);
        for (int c = 0; c < a.ncolsB; c++) {
          const Val v = col_load(hc, hrow, c);
          store_col(a.dcolB[c], a.typesB[c], o, v.b);
          a.dnulB[c][o] = (uint8_t)v.null;
        }
        a.dtsB[o] = x.ts(hr);
        a.dseqB[o] = x.seq(hr);
      }
    }
  });
}

// Carry gather (plain / OR forms), two kernels: k_open_list compacts the
// positions of the still-open partials in position order (one lane per
// position, wave ballots + a block prefix); k_gather_list then gives every
// open partial its own thread, so all their random row reads are in flight at
// once.  Only the e1 columns read again after the carry (amask) are copied.
__global__ __launch_bounds__(kBlock) void k_open_list(const uint8_t* __restrict__ pst, const uint32_t* __restrict__ boff,
                                                      int64_t n, int64_t tile, uint32_t* __restrict__ olist,
                                                      uint32_t val, int which) {
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n ? t0 + tile : n;
  // Each lane reads four outcome bytes as one word (positions c0 + 4 lane ..
  // + 3 of a 4 kBlock-position chunk; tiles start on 256-position boundaries
  // and pst is padded, so the word loads are aligned and in bounds), kOlU
  // chunks per round sharing one pair of barriers; a lane's hits are placed
  // by a wave prefix sum of the per-lane hit counts.
  constexpr int kOlU = 4;
  constexpr int kW = kBlock / 64;
  constexpr int kChunk = 4 * kBlock;
  __shared__ uint32_t wsum[kOlU][kW];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t base = boff[which * gridDim.x + blockIdx.x];   // offsets of count `which` (1: open, 2: deferred)
  for (int64_t c0 = t0; c0 < t1; c0 += kOlU * kChunk) {
    uint32_t word[kOlU];
#pragma unroll
    for (int u = 0; u < kOlU; u++) {
      const int64_t p = c0 + u * kChunk + 4 * threadIdx.x;
      word[u] = p < t1 ? *reinterpret_cast<const uint32_t*>(pst + p) : 0u;
    }
    uint32_t hm[kOlU], ex[kOlU];   // hit mask over the lane's 4 bytes, exclusive prefix in the wave
#pragma unroll
    for (int u = 0; u < kOlU; u++) {
      const int64_t p = c0 + u * kChunk + 4 * threadIdx.x;
      uint32_t m = 0;
#pragma unroll
      for (int b = 0; b < 4; b++)
        m |= ((((word[u] >> (8 * b)) & 0x7Fu) == val) && p + b < t1 ? 1u : 0u) << b;
      hm[u] = m;
      const uint32_t c = (uint32_t)__popc(m);
      uint32_t inc = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o, 64);
        if (lane >= o) inc += t;
      }
      ex[u] = inc - c;
      if (lane == 63) wsum[u][w] = inc;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kOlU; u++) {
      uint32_t pre = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < kW; k++) {
        pre += k < w ? wsum[u][k] : 0u;
        tot += wsum[u][k];
      }
      uint32_t o = base + pre + ex[u];
      const uint32_t p = (uint32_t)(c0 + u * kChunk + 4 * threadIdx.x);
#pragma unroll
      for (int b = 0; b < 4; b++)
        if ((hm[u] >> b) & 1u) olist[o++] = p + (uint32_t)b;
      base += tot;
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_gather_list(const GatherArgs* __restrict__ ap,
                                                        const uint32_t* __restrict__ olist, int64_t n_open,
                                                        const uint8_t* __restrict__ pst,
                                                        const uint32_t* __restrict__ spv,
                                                        const uint32_t* __restrict__ skey32,
                                                        const uint64_t* __restrict__ skey64) {
  const GatherArgs& a = *ap;
  const ExtRows& x = a.x;
  for (int64_t oi = (int64_t)blockIdx.x * kBlock + threadIdx.x; oi < n_open; oi = n_open) {
    const int64_t p = olist[oi];
    const int64_t o = oi;
    const int64_t r = pv_row(spv[p]);
    // one uniform column table per branch (carried rows / pushed rows)
    const uint64_t kk = !a.partitioned ? 0 : (a.key64 ? skey64[p] : (uint64_t)skey32[p]);
    const bool sts = a.sts32 || a.sts64;
    if (r < x.C) {
      for (int c = 0; c < a.ncols; c++) {
        if (!((a.amask >> c) & 1u)) continue;
        if (c == a.key_attr) {
          store_col(a.dcol[c], a.types[c], o, kk);
          a.dnul[c][o] = 0;
          continue;
        }
        const Val v = col_load(x.carry, r, c);
        store_col(a.dcol[c], a.types[c], o, v.b);
        a.dnul[c][o] = (uint8_t)v.null;
      }
      if (!sts) a.dts[o] = gld(x.carry.ts, r);
      a.dseq[o] = x.carry_seq[r];
    } else {
      const int64_t br = r - x.C;
      for (int c = 0; c < a.ncols; c++) {
        if (!((a.amask >> c) & 1u)) continue;
        if (c == a.key_attr) {
          store_col(a.dcol[c], a.types[c], o, kk);
          a.dnul[c][o] = 0;
          continue;
        }
        const Val v = col_load(x.batch, br, c);
        store_col(a.dcol[c], a.types[c], o, v.b);
        a.dnul[c][o] = (uint8_t)v.null;
      }
      if (!sts) a.dts[o] = gld(x.batch.ts, br);
      a.dseq[o] = x.seq0 + br;
    }
    if (sts) a.dts[o] = a.sts64 ? a.sts64[p] : gld(x.batch.ts, 0) + (int64_t)a.sts32[p];
    a.dkey[o] = kk;
    a.dpend[o] = (uint8_t)(((pst[p] & PS_PEND) || (r < x.C && a.pend_old[r])) ? 1 : 0);
  }
}

struct CarryTable {
  DevBuf col[kMaxCols], nul[kMaxCols], ts, key, seq;
  // 1: the partial met a B event of its key after it was created -- it left
  // the new list for the pending list (StreamPreStateProcessor.updateState);
  // 0: still in the new list (export_replay rebuilds the placement)
  DevBuf pend;
  // logical AND: filled-operand bits and the held operand event (stream B)
  DevBuf half, bcol[kMaxCols], bnul[kMaxCols], bts, bseq;
  void reserve_b(int64_t n, const std::vector<int>& types) {
    n = std::max<int64_t>(n, 1);
    half.reserve(n);
    for (size_t c = 0; c < types.size(); c++) {
      bcol[c].reserve(n * type_size(types[c]));
      bnul[c].reserve(n);
    }
    bts.reserve(n * 8);
    bseq.reserve(n * 8);
  }
  ColSet colset_b(const std::vector<int>& types, int64_t n) const {
    ColSet cs{};
    cs.ncols = (int)types.size();
    for (size_t c = 0; c < types.size(); c++) {
      cs.col[c] = bcol[c].p;
      cs.nul[c] = bnul[c].as<uint8_t>();
      cs.type[c] = (int32_t)types[c];
    }
    cs.ts = bts.as<int64_t>();
    cs.n = n;
    return cs;
  }
  void reserve(int64_t n, const std::vector<int>& types) {
    for (size_t c = 0; c < types.size(); c++) {
      col[c].reserve(std::max<int64_t>(n, 1) * type_size(types[c]));
      nul[c].reserve(std::max<int64_t>(n, 1));
    }
    ts.reserve(std::max<int64_t>(n, 1) * 8);
    key.reserve(std::max<int64_t>(n, 1) * 8);
    seq.reserve(std::max<int64_t>(n, 1) * 8);
    pend.reserve(std::max<int64_t>(n, 1));
  }
  ColSet colset(const std::vector<int>& types) const {
    ColSet cs{};
    cs.ncols = (int)types.size();
    for (size_t c = 0; c < types.size(); c++) {
      cs.col[c] = col[c].p;
      cs.nul[c] = nul[c].as<uint8_t>();
      cs.type[c] = (int32_t)types[c];
    }
    cs.ts = ts.as<int64_t>();
    return cs;
  }
};

// Does expression `e` only read state `st` (or constants)?
bool expr_reads_only(const Plan& p, int e, int st) {
  for (auto& in : p.exprs[e])
    if ((in.op == SHD_OP_LOAD || in.op == SHD_OP_EVNULL || in.op == SHD_OP_TS) && in.a != st) return false;
  return true;
}

int plain_load_attr(const Plan& p, int e) {
  auto& code = p.exprs[e];
  if (code.size() == 1 && code[0].op == SHD_OP_LOAD) return code[0].c & 0xFFFF;
  return -1;
}

// Does one of the e2 filters hold a top-level conjunct `e2.x == e1.y` (x, y
// attributes of the same string / int / long type, no conversion)?  Then an
// unpartitioned partial can only complete on an event with its own x value, so
// with time-ordered events the pattern runs grouped by that value exactly like
// a partitioned one (SURVEY.md §8e "sharding by symbol ... provable from the
// plan").  Returns the attribute pair (A-stream attr, B-stream attr).
bool find_key_equality(const Plan& p, const std::vector<int>& filters, int& attr_a, int& attr_b, int& type) {
  for (int e : filters) {
    const auto& code = p.exprs[e];
    // postfix -> tree (children of binary ops), then walk AND nodes from the root
    std::vector<int> st;
    std::vector<std::pair<int, int>> kid(code.size(), {-1, -1});
    bool ok = true;
    for (int i = 0; i < (int)code.size() && ok; i++) {
      const int op = code[i].op;
      if (op == SHD_OP_LOAD || op == SHD_OP_CONST || op == SHD_OP_NULL || op == SHD_OP_EVNULL || op == SHD_OP_TS ||
          op == SHD_OP_AGG) {
        st.push_back(i);
      } else if (op == SHD_OP_CVT || op == SHD_OP_NOT || op == SHD_OP_ISNULL) {
        if (st.empty()) ok = false;
        else { kid[i].first = st.back(); st.back() = i; }
      } else if (op >= SHD_OP_ADD && op <= SHD_OP_OR) {
        if (st.size() < 2) { ok = false; break; }
        kid[i] = {st[st.size() - 2], st.back()};
        st.pop_back();
        st.back() = i;
      } else if (op != SHD_OP_END) {
        ok = false;
      }
    }
    if (!ok || st.size() != 1) continue;
    std::vector<int> todo{st[0]};
    while (!todo.empty()) {
      const int n = todo.back();
      todo.pop_back();
      const Instr& in = code[n];
      if (in.op == SHD_OP_AND) {
        todo.push_back(kid[n].first);
        todo.push_back(kid[n].second);
        continue;
      }
      if (in.op != SHD_OP_EQ) continue;
      const Instr& l = code[kid[n].first];
      const Instr& r = code[kid[n].second];
      if (l.op != SHD_OP_LOAD || r.op != SHD_OP_LOAD) continue;
      auto cur = [](const Instr& x) { return x.b == 0 || x.b == SHD_IDX_CURRENT; };
      if (!cur(l) || !cur(r)) continue;
      const Instr& la = l.a == 0 ? l : r;
      const Instr& lb = l.a == 0 ? r : l;
      if (la.a != 0 || lb.a != 1) continue;
      const int ta = la.c >> 16, tb = lb.c >> 16;
      if (ta != tb || in.a != ta || !(ta == SHD_T_STRING || ta == SHD_T_INT || ta == SHD_T_LONG)) continue;
      attr_a = la.c & 0xFFFF;
      attr_b = lb.c & 0xFFFF;
      type = ta;
      return true;
    }
  }
  return false;
}


}  // namespace

struct PatternEngine : Engine {
  int sA = 0, sB = 0;
  std::vector<int> f1, f2;
  // `every e1 -> (e2 or|and e3)`: logical 1 = OR, 2 = AND; f3 = the partner's
  // filters, s_first / s_second = state ids in the order the two processors see
  // an event
  int logical = 0;
  std::vector<int> f3;
  std::vector<int> typesB;   // AND: schema of the operand events carried with half-filled partials
  bool and_indep = false;    // AND: neither operand filter reads the partner's slot
  uint32_t bpos_mask = 0;    // e2-side attributes read by the operand filters (ExtRows::bpos)
  uint32_t apos_mask = 0;    // e1-side attributes read by the operand filters (ExtRows::apos_mask)
  DevBuf d_bpos[kMaxCols], d_bpos_nul[kMaxCols];
  DevBuf d_bsum;   // k_block_sum output (long walks)
  int s_first = 1, s_second = -1;
  int64_t W = INT64_MAX;
  bool partitioned = false;
  // unpartitioned plan whose f2 holds `e2.x == e1.y`: keys written by prepare,
  // pushes with time-ordered events run grouped by that attribute
  bool implicit_key = false;
  int key_expr[2] = {-1, -1}, key_col[2] = {-1, -1}, key_type[2] = {0, 0};
  std::vector<int> outs;
  std::vector<int> typesA;
  CarryTable carry[2];
  int cur = 0;
  int64_t C = 0;
  // horizon rule: once open partials were dropped because every later event
  // (time >= horizon) would expire them, later pushes must not go back before it
  bool have_horizon = false;
  int64_t horizon = INT64_MIN;
  int64_t t_last = INT64_MIN;   // time of the last event (arrival order) of the committed pushes
  int64_t last_b_seq = -1;      // arrival index of the last B-stream event (export_replay placement)
  static constexpr int64_t kPruneMinRows = 1 << 16;
  // fused prepare + first key-sort pass (keyed_sort.hip): the host reads the
  // push aggregates while the first pass runs
  DevBuf d_kps;
  hipEvent_t ev_pg = nullptr, ev_pt = nullptr;
  // sorted times of this push's positions (finish: carried partials' times)
  const int32_t* fin_sts32 = nullptr;
  const int64_t* fin_sts64 = nullptr;
  // scratch
  DevBuf d_k32, d_k32_alt, d_k64, d_k64_alt, d_pv, d_pv_alt, d_ts, d_ts_alt, d_ts64, d_match, d_pst, d_bcnt, d_boff, d_pj,
      d_pi, d_pj_alt, d_pi_alt, d_agg, d_sort, d_scan, d_blk, d_mother, d_se1, d_sot, d_olist, d_dlist;
  // stream-A attributes read again after a partial is carried (state-0 loads
  // of f2 / f3 / the selector): only these columns are copied into the carry
  uint32_t carry_mask = ~0u;
  PinnedBuf h_agg;

  int kind() const override { return ENG_PATTERN; }

  void reset() override {
    C = 0;
    last_b_seq = -1;
    seq = 0;
    now = INT64_MIN;
    chunk_seq = 0;
    out.count = 0;
    counters = shd_counters{};
    have_horizon = false;
    horizon = INT64_MIN;
    t_last = INT64_MIN;
  }

  // Open partials as the A events that created them, in arrival order.  Each
  // was processed by the reference against every later event without
  // completing or expiring, so replaying just these events from a fresh state
  // rebuilds the same pending lists (a replayed event j meets an earlier
  // replayed partial i exactly as it did the first time: f2(i, j) false,
  // |ts_j - ts_i| <= within).  Unpartitioned plans expire globally: partials
  // further than `within` behind the latest event are already gone there.
  // Logical AND: a half-filled partial also needs the event that filled its
  // operand (LogicalPreStateProcessor: the slot keeps that event).  Replayed
  // after its partial's A event, that event fills the same operand of the same
  // partials it filled the first time -- every partial it met then either
  // still holds it (and is replayed) or is gone -- and, when its own start
  // partial is gone, it is replayed past the start state only (skip_start),
  // so it opens no partial the reference does not hold.
  void export_replay(std::vector<Replay>& parts) override {
    SHD_HIP(hipStreamSynchronize(stream));
    const CarryTable& t = carry[cur];
    std::vector<int64_t> ts(C), sq(C);
    if (C > 0) {
      SHD_HIP(hipMemcpy(ts.data(), t.ts.p, C * 8, hipMemcpyDeviceToHost));
      SHD_HIP(hipMemcpy(sq.data(), t.seq.p, C * 8, hipMemcpyDeviceToHost));
    }
    auto host_cols = [&](const std::vector<int>& types, const DevBuf* dcol, const DevBuf* dnul,
                         std::vector<std::vector<uint8_t>>& col, std::vector<std::vector<uint8_t>>& nul) {
      col.assign(types.size(), {});
      nul.assign(types.size(), {});
      for (size_t c = 0; c < types.size(); c++) {
        col[c].resize((size_t)C * type_size(types[c]));
        nul[c].resize((size_t)C);
        if (C > 0) {
          SHD_HIP(hipMemcpy(col[c].data(), dcol[c].p, col[c].size(), hipMemcpyDeviceToHost));
          SHD_HIP(hipMemcpy(nul[c].data(), dnul[c].p, (size_t)C, hipMemcpyDeviceToHost));
        }
      }
    };
    std::vector<std::vector<uint8_t>> col, nul, bcol, bnul;
    host_cols(typesA, t.col, t.nul, col, nul);
    std::vector<uint8_t> half;
    std::vector<int64_t> bts, bsq;
    if (logical == 2 && C > 0) {
      half.resize(C);
      bts.resize(C);
      bsq.resize(C);
      SHD_HIP(hipMemcpy(half.data(), t.half.p, C, hipMemcpyDeviceToHost));
      SHD_HIP(hipMemcpy(bts.data(), t.bts.p, C * 8, hipMemcpyDeviceToHost));
      SHD_HIP(hipMemcpy(bsq.data(), t.bseq.p, C * 8, hipMemcpyDeviceToHost));
      host_cols(typesB, t.bcol, t.bnul, bcol, bnul);
    }
    // New-list / pending-list placement (StreamPreStateProcessor.updateState:
    // a partial leaves the new list at the next B event of its key; expiry
    // walks the pending list only up to its first live partial but the new
    // list in full, so the placement matters once time goes back).  The
    // replayed A events place every partial but the newest of its key (each
    // later replayed event moves the earlier ones); when the newest too met a
    // later B event -- one of the events the replay leaves out -- a
    // stabilize-only replay event (skip_start 2, the newest partial's own
    // columns and time: it expires nothing that event did not) moves it.
    std::vector<uint8_t> pend(C, 0);
    if (C > 0) SHD_HIP(hipMemcpy(pend.data(), t.pend.p, C, hipMemcpyDeviceToHost));
    std::vector<uint64_t> keyv(C, 0);
    if (C > 0 && partitioned) SHD_HIP(hipMemcpy(keyv.data(), t.key.p, C * 8, hipMemcpyDeviceToHost));
    // replay events: (seq, source 0 = A row / 1 = operand row / 2 = stabilize-only, carry index)
    struct Ev { int64_t seq; int src; int64_t i; };
    std::vector<Ev> evs;
    std::unordered_map<uint64_t, int64_t> newest;   // key -> carry index of its newest exported partial
    for (int64_t i = 0; i < C; i++) {
      if (!(partitioned || W == INT64_MAX || t_last == INT64_MIN || !(t_last - ts[i] > W))) continue;
      evs.push_back({sq[i], 0, i});
      if (!half.empty() && half[i]) evs.push_back({bsq[i], 1, i});
      const uint64_t k = partitioned ? keyv[i] : 0;
      auto it = newest.find(k);
      if (it == newest.end() || sq[i] > sq[it->second]) newest[k] = i;
    }
    for (auto& kv : newest) {
      const int64_t i = kv.second;
      // unpartitioned: one global list, left by the next B event of the stream
      const bool moved = partitioned ? pend[i] != 0 : (last_b_seq >= 0 && last_b_seq > sq[i]);
      if (moved) evs.push_back({sq[i], 2, i});
    }
    std::stable_sort(evs.begin(), evs.end(), [](const Ev& a, const Ev& b) {
      return a.seq != b.seq ? a.seq < b.seq : a.src < b.src;
    });
    parts.clear();
    for (size_t k = 0; k < evs.size(); k++) {
      const Ev& e = evs[k];
      if (k > 0 && evs[k - 1].seq == e.seq && e.src != 2) continue;   // one event: A row first (it opens a partial)
      const int stream_e = e.src == 1 ? sB : sA;
      const std::vector<int>& types = e.src == 1 ? typesB : typesA;
      const auto& cc = e.src == 1 ? bcol : col;
      const auto& nn = e.src == 1 ? bnul : nul;
      if (parts.empty() || parts.back().stream != stream_e) {
        parts.emplace_back();
        Replay& r = parts.back();
        r.stream = stream_e;
        r.cols.assign(types.size(), {});
        r.nulls.assign(types.size(), {});
      }
      Replay& r = parts.back();
      r.ts.push_back(e.src == 1 ? bts[e.i] : ts[e.i]);
      for (size_t c = 0; c < types.size(); c++) {
        const int w = type_size(types[c]);
        r.cols[c].insert(r.cols[c].end(), cc[c].begin() + e.i * w, cc[c].begin() + (e.i + 1) * w);
        r.nulls[c].push_back(nn[c][e.i]);
      }
      r.skip_start.push_back((uint8_t)e.src);
      r.n++;
    }
  }

  // open partials (carry table) + horizon guard
  void save_state(SnapW& w) override {
    w.put<int64_t>(C);
    w.put<int32_t>(have_horizon ? 1 : 0);
    w.put<int64_t>(horizon);
    w.put<int64_t>(t_last);
    w.put<int64_t>(last_b_seq);
    w.put<int32_t>((int32_t)typesA.size());
    const CarryTable& t = carry[cur];
    for (size_t c = 0; c < typesA.size(); c++) {
      w.dev(t.col[c].p, (size_t)C * type_size(typesA[c]));
      w.dev(t.nul[c].p, (size_t)C);
    }
    w.dev(t.ts.p, (size_t)C * 8);
    w.dev(t.key.p, (size_t)C * 8);
    w.dev(t.seq.p, (size_t)C * 8);
    w.dev(t.pend.p, (size_t)C);
    if (logical == 2) {
      w.dev(t.half.p, (size_t)C);
      for (size_t c = 0; c < typesB.size(); c++) {
        w.dev(t.bcol[c].p, (size_t)C * type_size(typesB[c]));
        w.dev(t.bnul[c].p, (size_t)C);
      }
      w.dev(t.bts.p, (size_t)C * 8);
      w.dev(t.bseq.p, (size_t)C * 8);
    }
  }
  void load_state(SnapR& r) override {
    const int64_t c0 = r.get<int64_t>();
    have_horizon = r.get<int32_t>() != 0;
    horizon = r.get<int64_t>();
    t_last = r.get<int64_t>();
    last_b_seq = r.get<int64_t>();
    if (r.get<int32_t>() != (int32_t)typesA.size() || c0 < 0) throw Error(SHD_E_ARG, "snapshot of a different plan");
    cur = 0;
    CarryTable& t = carry[0];
    t.reserve(c0, typesA);
    for (size_t c = 0; c < typesA.size(); c++) {
      r.dev_into(t.col[c].p, (size_t)c0 * type_size(typesA[c]));
      r.dev_into(t.nul[c].p, (size_t)c0);
    }
    r.dev_into(t.ts.p, (size_t)c0 * 8);
    r.dev_into(t.key.p, (size_t)c0 * 8);
    r.dev_into(t.seq.p, (size_t)c0 * 8);
    r.dev_into(t.pend.p, (size_t)c0);
    if (logical == 2) {
      t.reserve_b(c0, typesB);
      r.dev_into(t.half.p, (size_t)c0);
      for (size_t c = 0; c < typesB.size(); c++) {
        r.dev_into(t.bcol[c].p, (size_t)c0 * type_size(typesB[c]));
        r.dev_into(t.bnul[c].p, (size_t)c0);
      }
      r.dev_into(t.bts.p, (size_t)c0 * 8);
      r.dev_into(t.bseq.p, (size_t)c0 * 8);
    }
    C = c0;
    counters.carry = C;
  }

  ColSet carry_cs() const {
    ColSet cs = carry[cur].colset(typesA);
    cs.n = C;
    return cs;
  }

  static bool type_key64(int t) { return t == SHD_T_LONG || t == SHD_T_DOUBLE || t == SHD_T_FLOAT; }

  // Key grouping by hashed buckets instead of the full key: the sort then
  // needs ceil(b/8) passes instead of ceil(key_bits/8), and a walk steps over
  // the other keys of its bucket until one is beyond `within` (valid only
  // when the pushed rows are time-ordered, every carried partial precedes
  // them, and the horizon rule is on -- see walk_partial).  b is chosen from
  // the expected number of other-key events of a bucket inside one `within`
  // span, E = n * (W+1) / (T+1) / 2^b, against the passes saved.
  // SHD_HASH_BITS=b forces b (tests), SHD_NO_HASH disables.
  int hashed_bucket_bits(const PrepAgg& pg, int64_t n_ext, int key_bits, bool prune) const {
    if (getenv("SHD_NO_HASH")) return 0;
    if (!prune || pg.unmono || (C > 0 && pg.carry_tmax > pg.ts_min) || pg.ts_max < pg.ts_min) return 0;
    if (const char* f = getenv("SHD_HASH_BITS")) {
      const int b = atoi(f);
      return b > 0 && b <= 32 ? b : 0;
    }
    const int exact_passes = (key_bits + 7) / 8;
    const double span = (double)(pg.ts_max - pg.ts_min) + 1.0;
    const double per_w = std::min((double)n_ext, (double)n_ext * ((double)W + 1.0) / span);
    double best = exact_passes;
    int best_b = 0;
    for (int p = 1; p < exact_passes; p++) {
      const double e = per_w / std::ldexp(1.0, 8 * p);
      // calibrated on MI355X (P3, 50M-event pushes): a sort pass ~0.29 ms, the
      // walks over E = 1.5 other keys per bucket ~ +0.32 ms of scan time, i.e.
      // one other-key step per walk ~ 0.7 of a pass
      const double cost = p + 0.7 * e;
      if (cost < best) {
        best = cost;
        best_b = 8 * p;
      }
    }
    return best_b;
  }

  ~PatternEngine() override {
    if (ev_pg) (void)hipEventDestroy(ev_pg);
    if (ev_pt) (void)hipEventDestroy(ev_pt);
  }

  void push(const Staged& b) override {
    if (b.n <= 0) return;
    fin_sts32 = nullptr;
    fin_sts64 = nullptr;
    sort_push(b);
  }

  void sort_push(const Staged& b) {
    const int64_t n = b.n;
    if (n <= 0) return;
    const bool isA = b.stream == sA, isB = b.stream == sB;
    const int64_t n_ext = C + n;
    if (n_ext + (logical == 2 ? C : 0) > (int64_t)kRowMask)
      throw Error(SHD_E_CAPACITY, "pattern batch + carried partials exceed 2^28 rows");
    hipStream_t s = stream;
    SHD_HIP(hipEventRecord(ev0, s));
    stage_begin();
    const int slot = isA ? 0 : 1;
    const bool keyed = partitioned || implicit_key;
    const bool key64 = keyed && type_key64(key_type[slot]);
    d_pv.reserve(n_ext * 4);
    d_ts.reserve(n_ext * 4);
    if (keyed) {
      if (key64) d_k64.reserve(n_ext * 8);
      d_k32.reserve(n_ext * 4);
    }
    d_match.reserve(n_ext * 4);
    d_pst.reserve(n_ext + kCompactPad);
    d_agg.reserve(256);
    h_agg.reserve(320);

    ExtRows x{};
    x.carry = carry_cs();
    x.batch = b.cs;
    x.C = C;
    x.seq0 = seq;
    x.carry_seq = carry[cur].seq.as<int64_t>();
    if (logical == 2) {
      carry[cur].reserve_b(C, typesB);
      x.half = carry[cur].colset_b(typesB, C);
      x.half_seq = carry[cur].bseq.as<int64_t>();
      d_mother.reserve(n_ext * 4);
    }

    PrepArgs pa{};
    pa.x = x;
    pa.es = dset();
    pa.f1 = dfilters(f1);
    pa.is_a = isA;
    pa.is_b = isB;
    pa.partitioned = keyed;
    pa.null_skip = partitioned;
    pa.key64 = key64;
    if (keyed) {
      if (key_expr[slot] >= 0) pa.key_expr = dexpr(key_expr[slot]);
      pa.key_col = key_col[slot];
      pa.key_type = key_type[slot];
    } else {
      pa.key_col = -1;
    }
    pa.carry_key = carry[cur].key.as<uint64_t>();
    PrepAgg init{0, 0, LLONG_MAX, LLONG_MIN, 0, 0, LLONG_MIN, ULLONG_MAX};
    PrepAgg* d_pa = d_agg.as<PrepAgg>();
    ScanOut* d_so = reinterpret_cast<ScanOut*>(d_agg.as<char>() + 64);
    std::memcpy(h_agg.p, &init, sizeof(init));
    std::memset(h_agg.as<char>() + 64, 0, sizeof(ScanOut));
    SHD_HIP(hipMemcpyAsync(d_agg.p, h_agg.p, 128, hipMemcpyHostToDevice, s));
    // 4096 workgroups (16 waves per SIMD at full occupancy): enough to stream
    // at full bandwidth, and the one-block folds of the per-block partials
    // (k_finish_prep / k_finish_scan) stay short
    const int nblk = grid_for(n_ext, 1, 4096);
    d_blk.reserve((size_t)3 * nblk * std::max(sizeof(PrepAgg), sizeof(ScanOut)));   // per-block partials
    const PrepArgs* d_pa_args = dev_args(pa);
    const bool fast1 = (!isA || pa.f1.fp.ok) && (!keyed || pa.key_col >= 0);
    // fused prepare + first sort pass: partitioned on a 32-bit plain key
    // attribute, f1 pre-decoded over at most one attribute, a push big enough
    // to pay for the extra launches (SHD_FUSED_SORT=0 / 1: off / on at any size)
    const char* fs_env = getenv("SHD_FUSED_SORT");
    const int fattr = keyed_sort_f1_attr(pa.f1, isA);
    const bool fused = partitioned && !key64 && pa.key_col >= 0 && fattr >= -1 &&
                       (key_type[slot] == SHD_T_STRING || key_type[slot] == SHD_T_INT) && n_ext >= 2 &&
                       (fs_env ? atoi(fs_env) != 0 : n_ext >= ((int64_t)1 << 20));
    KsInfo* d_ksi = reinterpret_cast<KsInfo*>(d_agg.as<char>() + 232);
    if (fused) {
      // the key range (ev_pg) is all the remaining passes need; the pushed
      // rows' time aggregates and the candidate count arrive with the first
      // pass (ev_pt, into h_agg + 256), read while the remaining passes run
      if (!ev_pg) SHD_HIP(hipEventCreateWithFlags(&ev_pg, hipEventDisableTiming));
      if (!ev_pt) SHD_HIP(hipEventCreateWithFlags(&ev_pt, hipEventDisableTiming));
      keyed_sort_front(s, d_pa_args, pa, n_ext, d_kps, d_pa, d_ksi);
      SHD_HIP(hipMemcpyAsync(h_agg.p, d_agg.p, 64, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipEventRecord(ev_pg, s));
      keyed_sort_pass0(s, d_pa_args, pa, fattr, n_ext, d_kps, d_ksi, d_k32.as<uint32_t>(), d_pv.as<uint32_t>(),
                       d_ts.as<uint32_t>(), d_pa);
      SHD_HIP(hipMemcpyAsync(h_agg.as<char>() + 256, d_agg.p, 64, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipEventRecord(ev_pt, s));
      SHD_HIP(hipEventSynchronize(ev_pg));
    } else if (fast1)
      hipLaunchKernelGGL(k_prepare<true>, dim3(nblk), dim3(kBlock), 0, s, d_pa_args, n_ext, (int64_t)nblk * kBlock,
                         d_k32.as<uint32_t>(), d_k64.as<uint64_t>(), d_pv.as<uint32_t>(), d_ts.as<int32_t>(),
                         d_blk.as<PrepAgg>());
    else
      hipLaunchKernelGGL(k_prepare<false>, dim3(nblk), dim3(kBlock), 0, s, d_pa_args, n_ext, (int64_t)nblk * kBlock,
                         d_k32.as<uint32_t>(), d_k64.as<uint64_t>(), d_pv.as<uint32_t>(), d_ts.as<int32_t>(),
                         d_blk.as<PrepAgg>());
    if (!fused) {
      SHD_CHECK_LAUNCH();
      hipLaunchKernelGGL(k_finish_prep, dim3(1), dim3(kBlock), 0, s, (const PrepAgg*)d_blk.as<PrepAgg>(), nblk, d_pa);
      SHD_CHECK_LAUNCH();
      SHD_HIP(hipMemcpyAsync(h_agg.p, d_agg.p, 64, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
    }
    PrepAgg pg;
    std::memcpy(&pg, h_agg.p, sizeof(pg));
    mark("prepare");
    // an unpartitioned plan retired partials that the last event of an earlier
    // push expired (global expiry: they are gone in the reference too); a push
    // going back before that time continues on the generic NFA engine with the
    // remaining open partials (partitioned plans never retire: see `prune`;
    // the fused path is partitioned, so its ts_min, not read yet, is not needed)
    if (have_horizon && (int64_t)pg.ts_min < horizon)
      throw NeedNfa("pattern engine: an event precedes the retirement horizon of an earlier push");

    // ---- key-sort the extended batch (stable: creation order within a key),
    //      carrying the packed (flags, row) payload and the event timestamp
    const uint32_t* skey32 = nullptr;
    const uint64_t* skey64 = nullptr;
    const uint32_t* spv = d_pv.as<uint32_t>();
    const int32_t* sts32 = d_ts.as<int32_t>();
    const int64_t* sts64 = nullptr;
    bool sorted64 = false;
    // Retirement of open partials that every later event would expire: exact
    // only under global expiry (unpartitioned plans: the push's last event
    // expired them, StreamPreStateProcessor.expireEvents :326-361).  A
    // partitioned partial is expired only by an event of its own key
    // (PartitionStateHolder: per-key pending lists), which may arrive in any
    // later push with any timestamp, so partitioned plans carry every open
    // partial until its key kills or completes it.
    const bool prune = n_ext >= kPruneMinRows && W != INT64_MAX && !partitioned;
    // implicit grouping needs the reference's global expiry order to be the
    // per-key one: pushed rows time-ordered, carried partials before them
    const bool grouped = partitioned || (implicit_key && !pg.unmono && (C == 0 || pg.carry_tmax <= pg.ts_min));
    uint32_t hash_mask = 0;
    counters.group_bits = 0;
    if (grouped) {
      // keys of this push span [kmin, kmax]: sort the offsets from kmin (a
      // rank owning one key slice sorts as many bits as rank 0)
      const uint64_t kmin = pg.kmin <= pg.kmax ? pg.kmin : 0;
      uint64_t kmax = pg.kmax;
      int bits = 0;
      while (bits < 64 && (kmax >> bits)) bits++;
      uint32_t kbase = 0;
      if (bits <= 32 && !type_key64(key_type[slot])) {
        int rb = 0;
        while (rb < 64 && ((kmax - kmin) >> rb)) rb++;
        if (rb < bits) {
          bits = rb > 0 ? rb : 1;
          kbase = (uint32_t)kmin;
        }
      }
      bool in_alt = false;
      if (bits <= 32) {
        const int hb = hashed_bucket_bits(pg, n_ext, bits, prune && !partitioned);
        if (hb > 0) {
          bits = hb;
          hash_mask = hb >= 32 ? 0xFFFFFFFFu : ((1u << hb) - 1u);
        }
      }
      d_pv_alt.reserve(n_ext * 4);
      d_ts_alt.reserve(n_ext * 4);
      if (key64 && bits <= 32) {
        hipLaunchKernelGGL(k_narrow_keys, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, d_k64.as<uint64_t>(),
                           d_k32.as<uint32_t>(), n_ext);
        SHD_CHECK_LAUNCH();
      }
      if (fused && (hash_mask || bits > 32))
        throw Error(SHD_E_DEVICE, "pattern engine: fused key sort on a hashed or wide key");
      if (bits <= 32) {
        d_k32_alt.reserve(n_ext * 4);
        // fused: the first pass ran already (keyed_sort_pass0, same digits);
        // the rest on keyed_sort.hip's pipelined passes
        if (fused)
          keyed_sort_rest(s, n_ext, bits, kbase, d_k32.as<uint32_t>(), d_pv.as<uint32_t>(), d_ts.as<uint32_t>(),
                          d_k32_alt.as<uint32_t>(), d_pv_alt.as<uint32_t>(), d_ts_alt.as<uint32_t>(), d_kps, d_sort,
                          in_alt);
        else
          radix_sort_triples_u32(d_k32.as<uint32_t>(), d_pv.as<uint32_t>(), d_ts.as<uint32_t>(),
                                 d_k32_alt.as<uint32_t>(), d_pv_alt.as<uint32_t>(), d_ts_alt.as<uint32_t>(), n_ext,
                                 bits, d_sort, s, in_alt, hash_mask != 0, hash_mask ? 0u : kbase);
        skey32 = in_alt ? d_k32_alt.as<uint32_t>() : d_k32.as<uint32_t>();
      } else {
        d_k64_alt.reserve(n_ext * 8);
        radix_sort_triples_u64(d_k64.as<uint64_t>(), d_pv.as<uint32_t>(), d_ts.as<uint32_t>(),
                               d_k64_alt.as<uint64_t>(), d_pv_alt.as<uint32_t>(), d_ts_alt.as<uint32_t>(), n_ext,
                               bits, d_sort, s, in_alt);
        skey64 = in_alt ? d_k64_alt.as<uint64_t>() : d_k64.as<uint64_t>();
        sorted64 = true;
      }
      spv = in_alt ? d_pv_alt.as<uint32_t>() : d_pv.as<uint32_t>();
      sts32 = in_alt ? d_ts_alt.as<int32_t>() : d_ts.as<int32_t>();
      mark("key_sort");
      counters.group_bits = bits;
    }
    if (fused) {   // the complete PrepAgg (k_ks_tfold after the first pass)
      SHD_HIP(hipEventSynchronize(ev_pt));
      std::memcpy(&pg, h_agg.as<char>() + 256, sizeof(pg));
    }
    if (pg.ovf || getenv("SHD_TS64")) {   // SHD_TS64: force the 64-bit path (tests)
      // some timestamp is more than 2^31 ms away from the batch's first event
      d_ts64.reserve(n_ext * 8);
      hipLaunchKernelGGL(k_sorted_ts64, dim3(grid_cover(n_ext)), dim3(kBlock), 0, s, dev_args(x), spv, n_ext,
                         d_ts64.as<int64_t>());
      SHD_CHECK_LAUNCH();
      sts64 = d_ts64.as<int64_t>();
    }

    // ---- forward scan, one lane per position
    ScanArgs sa{};
    sa.x = x;
    sa.es = dset();
    sa.f2 = dfilters(f2);
    sa.logical = logical;
    sa.s_first = s_first;
    sa.s_second = s_second;
    if (logical) sa.f3 = dfilters(f3);
    if (logical == 2) sa.carry_half = carry[cur].half.as<uint8_t>();
    sa.within = W;
    sa.partitioned = grouped;
    sa.prune = prune;
    sa.hash_mask = hash_mask;
    const int64_t t_end = (int64_t)pg.ts_max;   // latest event of this push
    sa.t_end = t_end;
    const bool fast2 = sa.f2.fp.ok != 0 && (!logical || sa.f3.fp.ok != 0);
    // contiguous tiles of positions per block (compaction offsets per block)
    const int64_t tile = ceil_div(ceil_div(n_ext, nblk), kBlock) * kBlock;
    const int ntile = (int)ceil_div(n_ext, tile);
    d_bcnt.reserve((size_t)3 * ntile * 4);
    d_boff.reserve((size_t)3 * ntile * 4);
    const bool ts64 = sts64 != nullptr;
    // deferred walks are dense when a partial expects another event of its key
    // inside `within` (every event, ungrouped): E = events per `within` span / keys
    bool dense = !grouped;
    double e_key = 0.0;   // expected events of a partial's key inside one `within` span
    if (grouped) {
      const double span = (double)(pg.ts_max - pg.ts_min) + 1.0;
      const double per_w = W == INT64_MAX ? (double)n_ext : std::min((double)n_ext, (double)n_ext * ((double)W + 1.0) / span);
      const double nkeys = hash_mask ? (double)hash_mask + 1.0 : (double)(pg.kmax - std::min(pg.kmin, pg.kmax)) + 1.0;
      e_key = per_w / nkeys;
      dense = e_key >= 0.25;
    }
    // dense: lane walks capped at 64 positions, the longer ones continued one
    // wave per partial (plain / OR forms, full-key grouping), else uncapped
    // lane walks; SHD_RESUME_MODE forces 0..3 (tests)
    // AND with operand filters that do not read the partner slot: one wave per
    // partial from the start (no capped lane phase: the operand state would
    // have to travel between the two passes)
    int rmode = dense ? (hash_mask ? 1 : (logical != 2 ? 3 : (and_indep ? 2 : 1))) : 0;
    if (const char* f = getenv("SHD_RESUME_MODE")) {
      const int m = atoi(f);
      if (m >= 0 && m <= 3 && !(m >= 2 && (hash_mask || (logical == 2 && (m == 3 || !and_indep))))) rmode = m;
    }
    // plain form over the full-key sort with a pre-decoded f2 and walks shorter
    // than the block-skip range: lockstep walks (k_lockstep_walk) instead of
    // the hot walk + deferred walks -- by default where the capped lane walks
    // would run (dense keys); SHD_LOCKSTEP=0 / 1 forces
    const char* ls_env = getenv("SHD_LOCKSTEP");
    const bool lockstep = grouped && !hash_mask && !sorted64 && logical == 0 && isB && fast2 && e_key < 64.0 &&
                          (ls_env ? atoi(ls_env) != 0 : rmode == 3);
    // dense grouped walks revisit each position once per partial of its key
    // inside `within`: the e2 attributes the filters read are copied into
    // position order once, so the walks load them coalesced; worth its pass
    // only when walks are long (SHD_NO_BPOS: off, SHD_BPOS: always when dense)
    if (grouped && (rmode != 0 || lockstep) && isB && bpos_mask && !getenv("SHD_NO_BPOS") && (e_key >= 8.0 || getenv("SHD_BPOS"))) {
      // e1 operands position-major too (same stream schema, columns the carry keeps)
      uint32_t apos = getenv("SHD_NO_APOS") ? 0u : (apos_mask & carry_mask);
      for (int c = 0; c < kMaxCols; c++)
        if (((apos >> c) & 1u) && (c >= b.cs.ncols || c >= (int)typesA.size() || typesA[c] != b.cs.type[c]))
          apos &= ~(1u << c);
      sa.x.bpos = b.cs;
      sa.x.bpos.n = n_ext;
      sa.x.apos_mask = apos;
      for (int c = 0; c < b.cs.ncols; c++) {
        if (!(((bpos_mask | apos) >> c) & 1u)) continue;
        d_bpos[c].reserve(n_ext * type_size(b.cs.type[c]));
        d_bpos_nul[c].reserve(n_ext);
        sa.x.bpos.col[c] = d_bpos[c].p;
        sa.x.bpos.nul[c] = d_bpos_nul[c].as<uint8_t>();
      }
      sa.x.bpos_mask = bpos_mask;
      hipLaunchKernelGGL(k_gather_bpos, dim3(grid_for(n_ext, 1, 4096)), dim3(kBlock), 0, s, dev_args(sa.x), spv, n_ext);
      SHD_CHECK_LAUNCH();
    }
    // plain form: f2 split per comparison (SHD_NO_SPLIT: eval_fpred per step)
    sa.sp = F2Split{};
    if (fast2 && logical == 0 && !getenv("SHD_NO_SPLIT")) split_f2(sa.f2.fp, s_first, sa.x, sa.sp);
    // long dense walks (a partial expects >= 64 events of its key inside
    // `within`) skip whole 64-position blocks that cannot end them
    sa.bsum = nullptr;
    const bool skip_ok = grouped && !hash_mask && !sorted64 && !ts64 && isB && logical == 0 && rmode != 0 && !lockstep &&
                         sa.f2.fp.ok && !getenv("SHD_NO_BLOCK_SKIP") && (e_key >= 64.0 || getenv("SHD_BLOCK_SKIP"));
    if (skip_ok && block_skip_term(sa.f2.fp, s_first, sa.bs_ci, sa.bs_side, sa.bs_op, sa.bs_attr)) {
      d_bsum.reserve(ceil_div(n_ext, 64) * (int64_t)sizeof(BlockSum));
      sa.bsum = d_bsum.as<BlockSum>();
    }
    const ScanArgs* d_sa = dev_args(sa);
    // sparse keys (MODE 0): the deferred walks from a compacted list
    // (k_resume_list) unless SHD_NO_RESUME_LIST
    const bool rlist = rmode == 0 && !lockstep && !sa.bsum && !sorted64 && !getenv("SHD_NO_RESUME_LIST");
    const int nlb = (int)std::max<int64_t>(1, std::min<int64_t>(1024, ceil_div(n_ext, (int64_t)64 * kBlock)));
    if (sa.bsum) {
      hipLaunchKernelGGL(k_block_sum, dim3(grid_for(ceil_div(n_ext, 64) * 64, 1, 4096)), dim3(kBlock), 0, s, d_sa,
                         n_ext, skey32, spv, sts32, d_bsum.as<BlockSum>());
      SHD_CHECK_LAUNCH();
    }
    // hot walk without f2 (deferrals), then the deferred walks with f2
#define SHD_LAUNCH_SCAN(K64, TS64, H)                                                                           \
  hipLaunchKernelGGL((k_forward_scan<K64, TS64, H>), dim3(ntile), dim3(kBlock), 0, s, d_sa, n_ext, tile, skey32,    \
                     skey64, spv, sts32, sts64, d_match.as<int32_t>(), d_pst.as<uint8_t>(), d_bcnt.as<uint32_t>(), \
                     d_blk.as<ScanOut>())
#define SHD_LAUNCH_RESUME_D(K64, FAST, TS64, D, SLOT)                                                           \
  hipLaunchKernelGGL((k_forward_resume<K64, FAST, TS64, D>), dim3(ntile), dim3(kBlock), 0, s, d_sa, n_ext, tile, \
                     skey32, skey64, spv, sts32, sts64, d_match.as<int32_t>(), d_mother.as<int32_t>(),           \
                     d_pst.as<uint8_t>(), d_bcnt.as<uint32_t>(), d_blk.as<ScanOut>(), SLOT)
#define SHD_LAUNCH_RESUME(K64, FAST, TS64)                                                                      \
  do {                                                                                                          \
    if (rmode == 3) {                                                                                           \
      SHD_LAUNCH_RESUME_D(K64, FAST, TS64, 3, ntile);                                                           \
      SHD_CHECK_LAUNCH();                                                                                       \
      SHD_LAUNCH_RESUME_D(K64, FAST, TS64, 2, 2 * ntile);                                                       \
    } else if (rmode == 2) SHD_LAUNCH_RESUME_D(K64, FAST, TS64, 2, ntile);                                      \
    else if (rmode == 1) SHD_LAUNCH_RESUME_D(K64, FAST, TS64, 1, ntile);                                        \
    else SHD_LAUNCH_RESUME_D(K64, FAST, TS64, 0, ntile);                                                        \
  } while (0)
#define SHD_LAUNCH_RESUME2(K64, FAST) \
  if (ts64) SHD_LAUNCH_RESUME(K64, FAST, true); else SHD_LAUNCH_RESUME(K64, FAST, false)
    // block skipping (sa.bsum: 32-bit keys and times, fast f2): its own instantiations
#define SHD_LAUNCH_SKIP(D, SLOT)                                                                                 \
  hipLaunchKernelGGL((k_forward_resume<false, true, false, D, true>), dim3(ntile), dim3(kBlock), 0, s, d_sa, n_ext, \
                     tile, skey32, skey64, spv, sts32, sts64, d_match.as<int32_t>(), d_mother.as<int32_t>(),      \
                     d_pst.as<uint8_t>(), d_bcnt.as<uint32_t>(), d_blk.as<ScanOut>(), SLOT)
    if (sorted64) {
      if (ts64) SHD_LAUNCH_SCAN(true, true, false); else SHD_LAUNCH_SCAN(true, false, false);
      SHD_CHECK_LAUNCH();
      if (fast2) { SHD_LAUNCH_RESUME2(true, true); }
      else { SHD_LAUNCH_RESUME2(true, false); }
    } else {
      if (lockstep) {
        // lockstep walks with f2, then the wave-cooperative pass for the
        // capped ones (PS_CONT)
        if (ts64)
          hipLaunchKernelGGL(k_lockstep_walk<true>, dim3(ntile), dim3(kBlock), 0, s, d_sa, n_ext, tile, skey32, spv,
                             sts32, sts64, d_match.as<int32_t>(), d_pst.as<uint8_t>(), d_bcnt.as<uint32_t>(),
                             d_blk.as<ScanOut>());
        else
          hipLaunchKernelGGL(k_lockstep_walk<false>, dim3(ntile), dim3(kBlock), 0, s, d_sa, n_ext, tile, skey32, spv,
                             sts32, sts64, d_match.as<int32_t>(), d_pst.as<uint8_t>(), d_bcnt.as<uint32_t>(),
                             d_blk.as<ScanOut>());
      } else if (hash_mask) {
        if (ts64) SHD_LAUNCH_SCAN(false, true, true); else SHD_LAUNCH_SCAN(false, false, true);
      } else {
        if (ts64) SHD_LAUNCH_SCAN(false, true, false); else SHD_LAUNCH_SCAN(false, false, false);
      }
      SHD_CHECK_LAUNCH();
      if (lockstep) {
        if (ts64) SHD_LAUNCH_RESUME_D(false, true, true, 2, ntile);
        else SHD_LAUNCH_RESUME_D(false, true, false, 2, ntile);
      } else if (sa.bsum) {
        if (rmode == 3) {
          SHD_LAUNCH_SKIP(3, ntile);
          SHD_CHECK_LAUNCH();
          SHD_LAUNCH_SKIP(2, 2 * ntile);
        } else if (rmode == 2) SHD_LAUNCH_SKIP(2, ntile);
        else SHD_LAUNCH_SKIP(1, ntile);
      } else if (rlist) {
        // sparse keys: the deferred positions compacted into a list (per-tile
        // counts from k_forward_scan), then one lane per deferred walk
        uint32_t* d_ndef = reinterpret_cast<uint32_t*>(d_agg.as<char>() + 240);
        scan_exclusive_u32(d_bcnt.as<uint32_t>() + 2 * ntile, d_boff.as<uint32_t>() + 2 * ntile, ntile, d_ndef, d_scan,
                           s);
        d_dlist.reserve((size_t)n_ext * 4);
        hipLaunchKernelGGL(k_open_list, dim3(ntile), dim3(kBlock), 0, s, (const uint8_t*)d_pst.as<uint8_t>(),
                           (const uint32_t*)d_boff.as<uint32_t>(), n_ext, tile, d_dlist.as<uint32_t>(),
                           (uint32_t)PS_DEFER, 2);
        SHD_CHECK_LAUNCH();
#define SHD_LAUNCH_RLIST(FAST, TS64)                                                                               \
  hipLaunchKernelGGL((k_resume_list<false, FAST, TS64>), dim3(nlb), dim3(kBlock), 0, s, d_sa, n_ext, tile, ntile,     \
                     skey32, skey64, spv, sts32, sts64, d_match.as<int32_t>(), d_mother.as<int32_t>(),              \
                     d_pst.as<uint8_t>(), d_bcnt.as<uint32_t>(), d_blk.as<ScanOut>(), ntile,                        \
                     (const uint32_t*)d_dlist.as<uint32_t>(), (const uint32_t*)d_ndef)
        if (fast2) {
          if (ts64) SHD_LAUNCH_RLIST(true, true); else SHD_LAUNCH_RLIST(true, false);
        } else {
          if (ts64) SHD_LAUNCH_RLIST(false, true); else SHD_LAUNCH_RLIST(false, false);
        }
#undef SHD_LAUNCH_RLIST
      } else if (fast2) { SHD_LAUNCH_RESUME2(false, true); }
      else { SHD_LAUNCH_RESUME2(false, false); }
    }
#undef SHD_LAUNCH_RESUME2
#undef SHD_LAUNCH_SKIP
#undef SHD_LAUNCH_RESUME_D
#undef SHD_LAUNCH_RESUME
#undef SHD_LAUNCH_SCAN
    SHD_CHECK_LAUNCH();
    // partials: [0, ntile) hot walk, [ntile, 2 ntile) deferred walks, [2 ntile, 3 ntile) continued walks
    hipLaunchKernelGGL(k_finish_scan, dim3(1), dim3(kBlock), 0, s, (const ScanOut*)d_blk.as<ScanOut>(),
                       rlist ? ntile + nlb : (rmode == 3 && !lockstep ? 3 : 2) * ntile,
                       d_so);
    SHD_CHECK_LAUNCH();
    mark("forward_scan");

    // ---- per-tile compaction offsets for matches and open partials (position order)
    uint32_t* d_mo = reinterpret_cast<uint32_t*>(d_agg.as<char>() + 128);
    scan_exclusive_u32(d_bcnt.as<uint32_t>(), d_boff.as<uint32_t>(), ntile, d_mo, d_scan, s);
    scan_exclusive_u32(d_bcnt.as<uint32_t>() + ntile, d_boff.as<uint32_t>() + ntile, ntile, d_mo + 1, d_scan, s);
    mark("compact");
    SHD_HIP(hipMemcpyAsync(h_agg.as<char>() + 64, d_agg.as<char>() + 64, 80, hipMemcpyDeviceToHost, s));
    // time of the push's last event in arrival order (NeedNfa hand-over: global expiry of unpartitioned plans)
    SHD_HIP(hipMemcpyAsync(h_agg.as<char>() + 192, b.cs.ts + (n - 1), 8, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    ScanOut so;
    std::memcpy(&so, h_agg.as<char>() + 64, sizeof(so));
    const uint32_t m = h_agg.as<uint32_t>()[32];
    const uint32_t n_open = h_agg.as<uint32_t>()[33];
    if (so.violation)   // the generic NFA engine takes over (shd_push replays the open partials)
      throw NeedNfa("pattern engine: event timestamps decrease within a key under `within`");
    if (so.pruned) {
      have_horizon = true;
      horizon = std::max(horizon, t_end);
    }
    fin_sts32 = sts32;
    fin_sts64 = sts64;
    finish(b, x, n_ext, tile, ntile, spv, skey32, skey64, sorted64, keyed, grouped, key64, m, n_open, so, t_end,
           pg.n_cand);
  }

  // Shared tail of a push: matches in (e2 event, creation) order -> projected
  // output rows; still-open partials -> the next push's carry; commit.
  void finish(const Staged& b, const ExtRows& x, int64_t n_ext, int64_t tile, int ntile, const uint32_t* spv,
              const uint32_t* skey32, const uint64_t* skey64, bool sorted64, bool keyed, bool grouped, bool key64,
              uint32_t m, uint32_t n_open, const ScanOut& so, int64_t t_end, uint64_t n_cand) {
    hipStream_t s = stream;
    const int64_t n = b.n;
    // ---- matches ordered by (e2 event, creation) -> projected output rows
    if (m > 0) {
      d_pj.reserve((int64_t)m * 4);
      d_pi.reserve((int64_t)m * 4);
      d_pj_alt.reserve((int64_t)m * 4);
      d_pi_alt.reserve((int64_t)m * 4);
      if (logical == 2) {
        d_se1.reserve((int64_t)m * 4);
        d_sot.reserve((int64_t)m * 4);
      }
      hipLaunchKernelGGL(k_emit_pairs, dim3(ntile), dim3(kBlock), 0, s, (const uint8_t*)d_pst.as<uint8_t>(),
                         (const uint32_t*)d_boff.as<uint32_t>(), (const int32_t*)d_match.as<int32_t>(), spv, n_ext,
                         tile, logical, (const int32_t*)d_mother.as<int32_t>(), d_pj.as<uint32_t>(),
                         d_pi.as<uint32_t>(), d_se1.as<uint32_t>(), d_sot.as<int32_t>());
      SHD_CHECK_LAUNCH();
      int bits = 0;
      while (bits < 32 && ((uint64_t)n_ext >> bits)) bits++;
      if (logical) bits++;   // + processor order
      bool in_alt = false;
      // pairs come out in (key, creation) order; the stable sort by j leaves the
      // partials of one e2 event in creation order (pending-list order)
      radix_sort_pairs_u32(d_pj.as<uint32_t>(), d_pi.as<uint32_t>(), d_pj_alt.as<uint32_t>(),
                           d_pi_alt.as<uint32_t>(), m, bits, d_sort, s, in_alt);
      const uint32_t* pj = in_alt ? d_pj_alt.as<uint32_t>() : d_pj.as<uint32_t>();
      const uint32_t* pi = in_alt ? d_pi_alt.as<uint32_t>() : d_pi.as<uint32_t>();
      if (!gmembers.empty()) {   // a group leader: its members' rows only
        group_emit(b, x, pj, pi, m);
        mark("order_project");
      } else {
        out.ensure(m, s);
        ProjArgs pr{};
        pr.x = x;
        pr.es = dset();
        pr.nout = (int)outs.size();
        pr.fast = 1;
        for (size_t c = 0; c < outs.size(); c++) {
          pr.outs[c] = dexpr(outs[c]);
          if (!fast_atom(outs[c], pr.oat[c])) pr.fast = 0;
        }
        pr.multi = (sA == sB);
        pr.logical = logical;
        pr.s_first = s_first;
        pr.s_second = s_second;
        pr.se1 = d_se1.as<uint32_t>();
        pr.sot = d_sot.as<int32_t>();
        pr.chunk0 = chunk_seq;
        pr.row0 = out.count;
        hipLaunchKernelGGL(k_project, dim3(grid_cover(m)), dim3(kBlock), 0, s, dev_args(pr), pj, pi, (int64_t)m,
                           out.d_chunk(), out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls(), out.d_seq(),
                           out.d_sidx());
        SHD_CHECK_LAUNCH();
        out.count += m;
        if (sA != sB && !logical) chunk_seq += m;
        mark("order_project");
      }
    }

    // ---- carry the still-open partials
    int nxt = cur ^ 1;
    carry[nxt].reserve(n_open, typesA);
    if (n_open > 0) {
      GatherArgs ga{};
      ga.x = x;
      ga.ncols = (int)typesA.size();
      ga.partitioned = keyed;
      ga.key64 = sorted64;
      for (size_t c = 0; c < typesA.size(); c++) {
        ga.types[c] = (int32_t)typesA[c];
        ga.dcol[c] = carry[nxt].col[c].p;
        ga.dnul[c] = carry[nxt].nul[c].as<uint8_t>();
      }
      ga.dts = carry[nxt].ts.as<int64_t>();
      ga.dkey = carry[nxt].key.as<uint64_t>();
      ga.dseq = carry[nxt].seq.as<int64_t>();
      carry[cur].pend.reserve(std::max<int64_t>(C, 1));
      ga.dpend = carry[nxt].pend.as<uint8_t>();
      ga.pend_old = carry[cur].pend.as<uint8_t>();
      if (logical == 2) {
        carry[nxt].reserve_b(n_open, typesB);
        ga.and_mode = 1;
        ga.match_row = d_match.as<int32_t>();
        ga.dhalf = carry[nxt].half.as<uint8_t>();
        ga.ncolsB = (int)typesB.size();
        for (size_t c = 0; c < typesB.size(); c++) {
          ga.typesB[c] = (int32_t)typesB[c];
          ga.dcolB[c] = carry[nxt].bcol[c].p;
          ga.dnulB[c] = carry[nxt].bnul[c].as<uint8_t>();
        }
        ga.dtsB = carry[nxt].bts.as<int64_t>();
        ga.dseqB = carry[nxt].bseq.as<int64_t>();
      }
      if (keyed && !grouped) {   // positions are rows: the prepare output holds each row's key
        ga.key64 = key64;
        skey32 = d_k32.as<uint32_t>();
        skey64 = d_k64.as<uint64_t>();
      }
      if (logical != 2 && !getenv("SHD_CARRY_SERIAL")) {
        ga.amask = carry_mask;
        if (grouped && !getenv("SHD_GATHER_ROWS")) {
          ga.sts32 = fin_sts32;
          ga.sts64 = fin_sts64;
          // the partition key attribute of stream A, a 32-bit plain column (sorted key == its value)
          ga.key_attr = (partitioned && !sorted64 && key_col[0] >= 0 &&
                         (key_type[0] == SHD_T_STRING || key_type[0] == SHD_T_INT)) ? key_col[0] : -1;
        } else {
          ga.key_attr = -1;
        }
        d_olist.reserve((size_t)n_open * 4);
        hipLaunchKernelGGL(k_open_list, dim3(ntile), dim3(kBlock), 0, s, (const uint8_t*)d_pst.as<uint8_t>(),
                           (const uint32_t*)d_boff.as<uint32_t>(), n_ext, tile, d_olist.as<uint32_t>(),
                           (uint32_t)PS_OPEN, 1);
        SHD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_gather_list, dim3(grid_cover((int64_t)n_open)), dim3(kBlock), 0, s, dev_args(ga),
                           (const uint32_t*)d_olist.as<uint32_t>(), (int64_t)n_open,
                           (const uint8_t*)d_pst.as<uint8_t>(), spv, skey32, skey64);
      } else {
        hipLaunchKernelGGL(k_gather_carry, dim3(ntile), dim3(kBlock), 0, s, dev_args(ga),
                           (const uint8_t*)d_pst.as<uint8_t>(), (const uint32_t*)d_boff.as<uint32_t>(), spv, skey32,
                           skey64, n_ext, tile);
      }
      SHD_CHECK_LAUNCH();
      mark("carry");
    }
    SHD_HIP(hipEventRecord(ev1, s));
    stage_end();
    SHD_HIP(hipEventSynchronize(ev1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    cur = nxt;
    C = n_open;
    if (b.stream == sB) last_b_seq = seq + n - 1;
    seq += n;
    if (b.advance_time && t_end > now) now = t_end;
    std::memcpy(&t_last, h_agg.as<char>() + 192, 8);
    counters.events += n;
    counters.matches += m;
    counters.partial_scans += (int64_t)so.steps;
    counters.carry = C;
    counters.kernel_ns = (int64_t)(ms * 1e6);
    counters.partials += (int64_t)n_cand;
    for (PatternEngine* g : gmembers) {
      g->seq = seq;
      if (b.advance_time && t_end > g->now) g->now = t_end;
      g->counters.events += n;
      g->counters.kernel_ns = 0;
    }
  }

  // ---- query sharing (shd_group_create): members whose plans differ from this
  // one only in the e1 filter (and the output names); this engine's e1 filter
  // accepts every event any member's does (the planner builds it as their
  // disjunction).  A member's own state is never used while grouped: its open
  // partials are the leader's whose A event passes its f1.
  std::vector<PatternEngine*> gmembers;
  DevBuf d_gmask, d_gcnt, d_goff, d_gscan, d_gpj, d_gpi, d_gbase;
  PinnedBuf h_gbase;

  static bool same_expr(const Plan& p, int e, const Plan& q, int f) {
    if (e < 0 || f < 0) return e == f;
    const auto& A = p.exprs[e];
    const auto& B = q.exprs[f];
    if (A.size() != B.size()) return false;
    for (size_t i = 0; i < A.size(); i++) {
      if (A[i].op != B[i].op || A[i].b != B[i].b || A[i].c != B[i].c) return false;
      if (A[i].op == SHD_OP_CONST ? p.consts[A[i].a] != q.consts[B[i].a] : A[i].a != B[i].a) return false;
    }
    return true;
  }

  void group_attach(const std::vector<Engine*>& ms) override {
    if (grouped) throw Error(SHD_E_ARG, "the leader already belongs to a group");
    if (ms.empty() || ms.size() > (size_t)kGroupMax) throw Error(SHD_E_ARG, "a group holds 1..64 member queries");
    if (logical != 0) throw Error(SHD_E_UNSUPPORTED, "query groups: logical patterns are not shared");
    if (counters.events != 0 || C != 0) throw Error(SHD_E_ARG, "the group leader must be fresh");
    std::vector<PatternEngine*> v;
    for (Engine* e : ms) {
      auto* m = dynamic_cast<PatternEngine*>(e);
      if (!m || m == this || m->grouped) throw Error(SHD_E_ARG, "group member: not a free pattern-engine query");
      for (PatternEngine* o : v)
        if (o == m) throw Error(SHD_E_ARG, "group member listed twice");
      bool ok = m->logical == 0 && m->sA == sA && m->sB == sB && m->W == W && m->partitioned == partitioned &&
                m->implicit_key == implicit_key && m->typesA == typesA && m->f2.size() == f2.size() &&
                m->plan.stream_types == plan.stream_types && (m->carry_mask & ~carry_mask) == 0;
      for (int k = 0; ok && k < 2; k++)
        ok = m->key_col[k] == key_col[k] && m->key_type[k] == key_type[k] &&
             same_expr(plan, key_expr[k], m->plan, m->key_expr[k]);
      for (size_t k = 0; ok && k < f2.size(); k++) ok = same_expr(plan, f2[k], m->plan, m->f2[k]);
      if (!ok)
        throw Error(SHD_E_ARG, "group member differs from the leader beyond the e1 filter and the selector");
      if (m->counters.events != 0 || m->C != 0 || m->out.count != 0)
        throw Error(SHD_E_ARG, "group members must be fresh (reset, no unpolled rows)");
      v.push_back(m);
    }
    gmembers = v;
    grouped = true;
    for (PatternEngine* m : gmembers) m->grouped = true;
  }

  void group_detach() override {
    for (PatternEngine* m : gmembers) m->grouped = false;
    gmembers.clear();
    grouped = false;
  }

  // this push's match pairs (sorted by e2 row, then creation) -> each member's
  // output rows
  void group_emit(const Staged& b, const ExtRows& x, const uint32_t* pj, const uint32_t* pi, uint32_t m) {
    hipStream_t s = stream;
    const int G = (int)gmembers.size();
    if ((uint64_t)m * (uint64_t)G >= (1ull << 32))
      throw Error(SHD_E_CAPACITY, "query group: too many matches in one push for 32-bit pair lists (split the batch)");
    const int64_t per_wave = 64 * kGroupWaveItems;
    const int64_t nw = ((int64_t)m + per_wave - 1) / per_wave;
    GroupSelArgs ga{};
    ga.x = x;
    ga.G = G;
    for (int g = 0; g < G; g++) {
      ga.es[g] = gmembers[g]->dset();
      ga.f1[g] = gmembers[g]->dfilters(gmembers[g]->f1);
    }
    d_gmask.reserve((size_t)m * 8);
    d_gcnt.reserve((size_t)G * nw * 4);
    d_goff.reserve((size_t)G * nw * 4);
    d_gbase.reserve((size_t)(G + 1) * 4);
    h_gbase.reserve((size_t)(G + 1) * 4);
    hipLaunchKernelGGL(k_group_mask, dim3(grid_cover(m)), dim3(kBlock), 0, s, dev_args(ga), pi, (int64_t)m,
                       d_gmask.as<uint64_t>());
    SHD_CHECK_LAUNCH();
    const int split_blocks = (int)((nw * 64 + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_group_split<false>, dim3(split_blocks), dim3(kBlock), 0, s,
                       (const uint64_t*)d_gmask.as<uint64_t>(), pj, pi, (int64_t)m, G, nw, d_gcnt.as<uint32_t>(),
                       (uint32_t*)nullptr, (uint32_t*)nullptr);
    SHD_CHECK_LAUNCH();
    scan_exclusive_u32(d_gcnt.as<uint32_t>(), d_goff.as<uint32_t>(), (int64_t)G * nw, nullptr, d_gscan, s);
    hipLaunchKernelGGL(k_group_bases, dim3(1), dim3(128), 0, s, (const uint32_t*)d_goff.as<uint32_t>(),
                       (const uint32_t*)d_gcnt.as<uint32_t>(), G, nw, d_gbase.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    SHD_HIP(hipMemcpyAsync(h_gbase.p, d_gbase.p, (size_t)(G + 1) * 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const uint32_t* base = h_gbase.as<uint32_t>();
    const uint32_t total = base[G];
    if (total == 0) return;
    d_gpj.reserve((size_t)total * 4);
    d_gpi.reserve((size_t)total * 4);
    hipLaunchKernelGGL(k_group_split<true>, dim3(split_blocks), dim3(kBlock), 0, s,
                       (const uint64_t*)d_gmask.as<uint64_t>(), pj, pi, (int64_t)m, G, nw, d_goff.as<uint32_t>(),
                       d_gpj.as<uint32_t>(), d_gpi.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    for (int g = 0; g < G; g++) {
      PatternEngine& e = *gmembers[g];
      const uint32_t mq = base[g + 1] - base[g];
      if (mq == 0) continue;
      e.out.ensure(mq, s);
      ProjArgs pr{};
      pr.x = x;
      pr.es = e.dset();
      pr.nout = (int)e.outs.size();
      pr.fast = 1;
      for (size_t c = 0; c < e.outs.size(); c++) {
        pr.outs[c] = e.dexpr(e.outs[c]);
        if (!e.fast_atom(e.outs[c], pr.oat[c])) pr.fast = 0;
      }
      pr.multi = (sA == sB);
      pr.logical = 0;
      pr.s_first = e.s_first;
      pr.s_second = e.s_second;
      pr.chunk0 = e.chunk_seq;
      pr.row0 = e.out.count;
      hipLaunchKernelGGL(k_project, dim3(grid_cover(mq)), dim3(kBlock), 0, s, dev_args(pr),
                         (const uint32_t*)d_gpj.as<uint32_t>() + base[g], (const uint32_t*)d_gpi.as<uint32_t>() + base[g],
                         (int64_t)mq, e.out.d_chunk(), e.out.d_type(), e.out.d_ts(), e.out.d_vals(), e.out.d_nulls(),
                         e.out.d_seq(), e.out.d_sidx());
      SHD_CHECK_LAUNCH();
      e.out.count += mq;
      if (sA != sB) e.chunk_seq += mq;
      e.counters.matches += mq;
    }
    (void)b;
  }
};

std::unique_ptr<Engine> finish_pattern_engine(const Plan& p, const PNode& a, const PNode& b, const PNode* c,
                                              std::string& why);

std::unique_ptr<Engine> make_pattern_engine(const Plan& p, std::string& why) {
  // shape: NEXT(EVERY(STREAM a), STREAM b), pattern type, plain stream states
  if (p.kind != SHD_KIND_STATE || p.state_type != 0) { why = "not a pattern"; return nullptr; }
  const PNode& r = p.root;
  if (r.kind != SHD_NODE_NEXT || r.kids.size() != 2) { why = "not a two-state chain"; return nullptr; }
  const PNode& ev = r.kids[0];
  const PNode& b = r.kids[1];
  if (ev.kind != SHD_NODE_EVERY || ev.kids.size() != 1 || ev.kids[0].kind != SHD_NODE_STREAM ||
      b.kind != SHD_NODE_STREAM) {
    why = "not every e1 -> e2";
    return nullptr;
  }
  const PNode& a = ev.kids[0];
  if (a.absent || b.absent || a.state_id != 0 || b.state_id != 1) { why = "absent / unexpected state ids"; return nullptr; }
  return finish_pattern_engine(p, a, b, nullptr, why);
}

// `every e1=A[f1] -> (e2=B[f2] or e3=B[f3]) (within W)`: a partial completes at
// the first B event that passes the filters of one of the two logical
// processors, tried in the order MultiProcessStreamReceiver hands them an event
// (reverse setup order: the first logical operand first,
// StateInputStreamParser.java:349-361 + LogicalInnerStateRuntime.setup); the
// partner slot stays empty (LogicalPreStateProcessor.java:113-154 drops the
// partial from the partner's pending list).
// `... -> (e2=B[f2] and e3=B[f3])`: each operand fills at the first B event
// that passes its filter (tried in the same order, the partner slot visible to
// the filter); the partial completes when both are filled, emitted by the
// processor that filled last.  A half-filled open partial carries its operand
// event to the next push (CarryTable::half / bcol, ext rows C + n + i).
std::unique_ptr<Engine> make_logical_pattern_engine(const Plan& p, std::string& why) {
  if (p.kind != SHD_KIND_STATE || p.state_type != 0) { why = "not a pattern"; return nullptr; }
  const PNode& r = p.root;
  if (r.kind != SHD_NODE_NEXT || r.kids.size() != 2) { why = "not a two-state chain"; return nullptr; }
  const PNode& ev = r.kids[0];
  const PNode& lg = r.kids[1];
  if (ev.kind != SHD_NODE_EVERY || ev.kids.size() != 1 || ev.kids[0].kind != SHD_NODE_STREAM ||
      lg.kind != SHD_NODE_LOGICAL || (lg.ltype != 0 && lg.ltype != 1) || lg.kids.size() != 2) {
    why = "not every e1 -> (e2 or|and e3)";
    return nullptr;
  }
  const PNode& a = ev.kids[0];
  const PNode& b = lg.kids[0];
  const PNode& c = lg.kids[1];
  if (b.kind != SHD_NODE_STREAM || c.kind != SHD_NODE_STREAM || a.absent || b.absent || c.absent ||
      a.state_id != 0 || b.stream != c.stream) {
    why = "logical operands: absent / different streams";
    return nullptr;
  }
  return finish_pattern_engine(p, a, b, &c, why);
}

std::unique_ptr<Engine> finish_pattern_engine(const Plan& p, const PNode& a, const PNode& b, const PNode* c,
                                              std::string& why) {
  if (!p.aggs.empty() || !p.group_by.empty() || p.having >= 0) { why = "aggregating selector"; return nullptr; }
  if (!p.current_on) { why = "pattern without current events output"; return nullptr; }
  if (p.outputs.size() > (size_t)kMaxCols || a.filters.size() > 4 || b.filters.size() > 4 ||
      (c && c->filters.size() > 4)) {
    why = "too many outputs / filters";
    return nullptr;
  }
  for (int f : a.filters)
    if (!expr_reads_only(p, f, 0)) { why = "e1 filter reads other states"; return nullptr; }
  if (p.stream_types[a.stream].size() > (size_t)kMaxCols || p.stream_types[b.stream].size() > (size_t)kMaxCols) {
    why = "too many attributes";
    return nullptr;
  }
  auto e = std::make_unique<PatternEngine>();
  e->sA = a.stream;
  e->sB = b.stream;
  e->f1 = a.filters;
  e->f2 = b.filters;
  if (c) {
    e->logical = p.root.kids[1].ltype == 1 ? 1 : 2;
    e->f3 = c->filters;
    e->typesB = p.stream_types[b.stream];
    auto reads_only = [&](const std::vector<int>& fs, int own) {
      for (int f : fs)
        for (auto& in : p.exprs[f])
          if ((in.op == SHD_OP_LOAD || in.op == SHD_OP_EVNULL || in.op == SHD_OP_TS) && in.a != 0 && in.a != own)
            return false;
      return true;
    };
    e->and_indep = reads_only(b.filters, b.state_id) && reads_only(c->filters, c->state_id);
    e->s_first = b.state_id;
    e->s_second = c->state_id;
  }
  e->W = p.within >= 0 ? p.within : INT64_MAX;
  e->typesA = p.stream_types[a.stream];
  {
    // attributes of the e2-side state(s) that the walk filters load
    auto scan = [&](const std::vector<int>& fs, int st) {
      for (int f : fs)
        for (auto& in : p.exprs[f])
          if (in.op == SHD_OP_LOAD && in.a == st && (in.c & 0xFFFF) < kMaxCols) e->bpos_mask |= 1u << (in.c & 0xFFFF);
    };
    scan(b.filters, b.state_id);
    if (c) scan(c->filters, c->state_id);
    for (const std::vector<int>* fs : {&b.filters, c ? &c->filters : nullptr})
      if (fs)
        for (int f : *fs)
          for (auto& in : p.exprs[f])
            if (in.op == SHD_OP_LOAD && in.a == 0 && (in.c & 0xFFFF) < kMaxCols) e->apos_mask |= 1u << (in.c & 0xFFFF);
  }
  for (auto& o : p.outputs) e->outs.push_back(o.second);
  e->partitioned = !p.part_keys.empty();
  if (!e->partitioned && !c && !getenv("SHD_NO_IMPLICIT_KEY")) {
    int aa, ab, t;
    // one stream playing both roles: an event has one key, so both sides must be the same attribute
    if (find_key_equality(p, b.filters, aa, ab, t) && (a.stream != b.stream || aa == ab)) {
      e->implicit_key = true;
      e->key_col[0] = aa;
      e->key_col[1] = ab;
      e->key_type[0] = e->key_type[1] = t;
    }
  }
  if (e->partitioned) {
    int cls = -1;
    for (auto& pk : p.part_keys) {
      int slot = pk.first == a.stream ? 0 : (pk.first == b.stream ? 1 : -1);
      if (slot < 0) continue;
      int t = expr_result_type(p, pk.second, {});
      if (cls >= 0 && t != cls) { why = "partition keys of different types"; return nullptr; }
      cls = t;
      e->key_expr[slot] = pk.second;
      e->key_col[slot] = plain_load_attr(p, pk.second);
      e->key_type[slot] = t;
      if (a.stream == b.stream) {
        e->key_expr[1 - slot] = pk.second;
        e->key_col[1 - slot] = e->key_col[slot];
        e->key_type[1 - slot] = t;
      }
    }
    if (e->key_expr[0] < 0 || e->key_expr[1] < 0) { why = "partition key missing for a stream"; return nullptr; }
  }
  // e1 columns read after a partial is carried: f2 / f3 / the selector, and
  // (for a hand-over replay through the generic NFA engine) f1 and the keys
  uint32_t mask = 0;
  auto add = [&](int ex) {
    if (ex < 0) return;
    for (const Instr& in : p.exprs[ex])
      if (in.op == SHD_OP_LOAD && in.a == 0) mask |= 1u << (in.c & 0xFFFF);
  };
  for (int f : e->f1) add(f);
  for (int f : e->f2) add(f);
  for (int f : e->f3) add(f);
  for (int o : e->outs) add(o);
  add(e->key_expr[0]);
  add(e->key_expr[1]);
  e->carry_mask = mask;
  return e;
}

}  // namespace shd
