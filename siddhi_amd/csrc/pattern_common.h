// pattern_common.h -- types of the pattern engine (engine_pattern.hip:
// prepare / key sort / forward scan / compaction): row flags, per-position
// outcomes, extended-batch row addressing, the pair expression context and
// the scan argument / counter blocks.  See engine_pattern.hip for the
// semantics.
#pragma once
#include "engine.h"

namespace shd {
namespace pat {

enum : uint32_t { F_CAND = 1, F_NEW = 2, F_B = 4, F_SKIP = 8 };
// Per-position scan result (positions = key-sorted order when partitioned).
enum : uint8_t { ST_NONE = 0, ST_OPEN = 1, ST_DEAD = 2, ST_MATCH = 3, ST_DEFER = 4, ST_PRUNED = 5, ST_YIELD = 6 };
// per-position outcome stored by k_forward_scan for the compaction kernels
// PS_CONT: a capped lane walk stopped before position match_row[p] (long
// walk, continued by the wave-cooperative pass)
enum : uint8_t { PS_NONE = 0, PS_OPEN = 1, PS_MATCH = 2, PS_DEFER = 3, PS_CONT = 4 };
// flag on PS_OPEN: the partial met a B event of its key after its creation,
// so it sits in the pending list, not the new list (carried as CarryTable::pend)
constexpr uint8_t PS_PEND = 0x80;

// Sort payload: row index of the extended batch (28 bits) | flags (4 bits).
constexpr int kRowBits = 28;
constexpr uint32_t kRowMask = (1u << kRowBits) - 1;
__device__ __forceinline__ uint32_t pv_row(uint32_t pv) { return pv & kRowMask; }
__device__ __forceinline__ uint32_t pv_flags(uint32_t pv) { return pv >> kRowBits; }

// Row addressing over the extended batch: rows [0, C) are carried partials
// (stream A columns), rows [C, C+n) are the pushed batch.
struct ExtRows {
  ColSet carry;   // stream A schema
  ColSet batch;   // pushed stream schema
  int64_t C;
  int64_t seq0;           // global seq of batch row 0
  const int64_t* carry_seq;
  // logical AND: rows [C + n, 2C + n) are the operand events the carried
  // half-filled partials hold (stream B schema; row C + n + i for carry row i)
  ColSet half;
  const int64_t* half_seq;
  // dense grouped walks: the e2-side attributes the filters read, copied into
  // key-sorted position order (bit a of bpos_mask: attribute a is there), so
  // the 64 positions a wave steps over load coalesced instead of one row each
  ColSet bpos;
  uint32_t bpos_mask;
  // e1-side attributes the filters read, in the same position-major columns
  // (carried rows included): a walk reads its partial's own operands at its
  // start position, coalesced, instead of one random row load per step
  uint32_t apos_mask;
  __device__ __forceinline__ const ColSet& cs(int64_t r) const { return r < C ? carry : (r < C + batch.n ? batch : half); }
  __device__ __forceinline__ int64_t row(int64_t r) const { return r < C ? r : (r < C + batch.n ? r - C : r - C - batch.n); }
  __device__ __forceinline__ int64_t ts(int64_t r) const {
#ifdef SHD_DEBUG
    if (r < 0 || r >= C + batch.n) {
      printf("SHD_DEBUG ExtRows.ts: row %lld C %lld n %lld\n", (long long)r, (long long)C, (long long)batch.n);
      return 0;
    }
#endif
    if (r < C) return gld(carry.ts, r);
    if (r < C + batch.n) return gld(batch.ts, r - C);
    return gld(half.ts, r - C - batch.n);
  }
  __device__ __forceinline__ int64_t seq(int64_t r) const {
    return r < C ? carry_seq[r] : (r < C + batch.n ? seq0 + (r - C) : half_seq[r - C - batch.n]);
  }
};

// Expression context over (e1 row, second-state row); stream-state chains
// hold one event.  s2: the state id r2 fills (1 for e1 -> e2; for the logical
// OR form the branch that matched -- the partner slot is always empty then).
struct PairCtx {
  const ExtRows* x;
  int64_t r1, r2;   // ext rows of state 0 / state s2 (-1 = empty slot)
  int s2 = 1;
  bool matched = false;   // projection of a completed partial
  int64_t r3 = -1;        // logical AND: the partner operand's row (state s3)
  int s3 = -1;
  int64_t q2 = -1;        // sorted position of r2 (walks; -1 in the projection)
  int64_t q1 = -1;        // sorted position of r1 (walks from a known start position)
  __device__ __forceinline__ int64_t slot(int st, int idx) const {
    int64_t r = st == 0 ? r1 : (st == s2 ? r2 : (st == s3 ? r3 : -1));
    if (r < 0) return -1;
    // StateEvent.getStreamEvent(int[]) on a one-event chain: index 0 / CURRENT hit it
    return (idx == 0 || idx == SHD_IDX_CURRENT) ? r : -1;
  }
  __device__ __forceinline__ Val load(int st, int idx, int attr) const {
    int64_t r = slot(st, idx);
    if (r < 0) {
      Val v;
      v.b = 0;
      v.null = 1;
      return v;
    }
    // branch on the row's table instead of selecting a per-lane ColSet
    // pointer: each branch reads a wave-uniform column table (scalar loads)
    if (st == s2 && q2 >= 0 && ((x->bpos_mask >> attr) & 1u)) return col_load(x->bpos, q2, attr);
    if (st == 0 && q1 >= 0 && ((x->apos_mask >> attr) & 1u)) return col_load(x->bpos, q1, attr);
    if (r < x->C) return col_load(x->carry, r, attr);
    if (r < x->C + x->batch.n) return col_load(x->batch, r - x->C, attr);
    return col_load(x->half, r - x->C - x->batch.n, attr);
  }
  __device__ __forceinline__ bool evnull(int st, int idx) const { return slot(st, idx) < 0; }
  // eventTimestamp() reads the StateEvent's timestamp: e1's while the e2 filters
  // run, the completing event's once matched (StreamPostStateProcessor.java:64-83
  // sets it before the selector)
  __device__ __forceinline__ int64_t ts(int, int) const { return x->ts(matched ? r2 : r1); }
  __device__ __forceinline__ Val agg(int) const {
    Val v;
    v.b = 0;
    v.null = 1;
    return v;
  }
};

// Summary of 64 sorted positions [64b, 64b + 64) for walks that skip whole
// blocks (k_block_sum): the key all non-skip positions share (flag 1; flag 4:
// no non-skip position), whether the F_NEW times are nondecreasing (flag 2),
// the first / last F_NEW time, the F_NEW count and positions, and the max (ops
// > >=) or min (< <=) of the e2 attribute the f2 comparison reads over the
// F_NEW B events.
struct BlockSum {
  uint32_t key;
  uint16_t cnt;
  uint8_t flags, pad;
  int64_t tfirst, tlast;
  double v;
  uint64_t newmask;   // bit i: position 64b + i is an F_NEW non-skip event
};

// f2 of the plain form split per comparison (split_f2, engine_pattern.hip):
// the side free of e2 is evaluated once per partial (split_prep), the e2 side
// is a plain attribute load (+ one conversion) per walk step (split_eval) --
// the same operations as eval_fpred, without re-deciding the descriptor's
// atoms, the e1 operand loads and the e1 arithmetic at every step.
struct SplitCmp {
  const void* col;          // the e2 attribute's column: position-major (bpos) when pos, else batch rows
  const uint8_t* nul;
  int32_t ctype, pos, cvt_from, cvt_to;
  int32_t op, type;
  int32_t swap;             // the e2 load is the right operand
  int32_t konst;            // no e2 operand: decided once per partial
  int32_t kind;             // SK_*: a pre-resolved load + conversion + comparison (op with e2 on the left)
};
// split comparison kinds (SK_GENERIC: col_load_raw + d_cvt + d_compare)
enum : int32_t { SK_GENERIC = 0, SK_F32_F64 = 1, SK_F64 = 2, SK_STR_EQ = 3, SK_I32 = 4 };
constexpr int kSplitMax = 3;
struct F2Split {
  int32_t ok, n;
  SplitCmp c[kSplitMax];
};

struct ScanArgs {
  ExtRows x;
  DExprSet es;
  DFilters f2;
  // logical OR second state `(e2=B[f2] or e3=B[f3])`: f2 = the filters of the
  // processor that sees an event first (state s_first), f3 = its partner's
  DFilters f3;
  int logical;          // 0: e1 -> e2, 1: OR, 2: AND
  int s_first, s_second;
  const uint8_t* carry_half;   // AND: operands already filled per carried partial (bit 0 first, bit 1 second)
  int64_t within;
  int partitioned;
  int prune;            // drop partials that can no longer match (horizon guard on later pushes)
  int64_t t_end;        // latest event time of this push
  // hashed buckets (0: positions are sorted by the full key): positions are
  // grouped by the low bits of key_bucket_mix(key), keys of one bucket
  // interleaved in input order.  Only set when the batch rows are globally
  // time-ordered, carried partials precede them in time, and prune is on.
  uint32_t hash_mask;
  // block skip (long walks): f2's comparison bs_ci reads the e2 attribute
  // bs_attr, normalised as `e2.attr bs_op threshold` with the threshold on the
  // e1 side (bs_side 0: its right term, 1: its left); bsum null: no skipping
  const BlockSum* bsum;
  int bs_ci, bs_side, bs_op, bs_attr;
  F2Split sp;           // plain form: f2 split per comparison (sp.ok = 0: eval_fpred)
};

struct ScanOut {
  unsigned long long steps;   // (partial, event) pairs examined
  unsigned long long pruned;  // open partials dropped by the horizon rule
  uint32_t violation;         // per-key timestamp decrease seen
};
// Expression context of k_prepare: the pushed event as state 0 (stream-state
// chain of one event), read from the uniform batch column table.
struct BatchRowCtx {
  const ColSet* cs;
  int64_t row;
  __device__ __forceinline__ Val load(int st, int idx, int attr) const {
    if (st != 0 || !(idx == 0 || idx == SHD_IDX_CURRENT)) {
      Val v;
      v.b = 0;
      v.null = 1;
      return v;
    }
    return col_load(*cs, row, attr);
  }
  __device__ __forceinline__ bool evnull(int st, int idx) const { return !(st == 0 && (idx == 0 || idx == SHD_IDX_CURRENT)); }
  __device__ __forceinline__ int64_t ts(int st, int idx) const { return evnull(st, idx) ? 0 : cs->ts[row]; }
  __device__ __forceinline__ Val agg(int) const {
    Val v;
    v.b = 0;
    v.null = 1;
    return v;
  }
};

__device__ __forceinline__ uint64_t canon_key(Val v, int type) {
  switch (type) {
    case SHD_T_FLOAT: return p_f64((double)v_f32(v.b));
    default: return v.b;
  }
}

// Batch-wide aggregates written by k_prepare (one 64-byte block):
//   [0] candidates created  [1] max key  [2] min batch ts  [3] max batch ts
struct PrepAgg {
  unsigned long long n_cand;
  unsigned long long kmax;
  long long ts_min;
  long long ts_max;
  unsigned long long ovf;   // some row's ts - batch.ts[0] does not fit in int32
  unsigned long long unmono;   // some batch row's ts is below its predecessor's
  long long carry_tmax;        // latest carried partial (LLONG_MIN: none)
  unsigned long long kmin;     // smallest key (rows with a key)
};

struct PrepArgs {
  ExtRows x;
  DExprSet es;
  DFilters f1;
  int is_a, is_b;           // pushed stream plays A and/or B
  int partitioned;          // write a key per row
  int null_skip;            // partition key semantics: null key -> event dropped (F_SKIP)
  int key64;                // key written as u64 (long / double / float keys)
  DExpr key_expr;           // key expression of the pushed stream
  int key_type;
  int key_col;              // >= 0: plain attribute key of the pushed stream
  const uint64_t* carry_key;
};

template <class T>
__device__ __forceinline__ T wave_max(T v) {
  for (int o = 32; o > 0; o >>= 1) {
    T t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}
template <class T>
__device__ __forceinline__ T wave_min(T v) {
  for (int o = 32; o > 0; o >>= 1) {
    T t = __shfl_xor(v, o, 64);
    v = t < v ? t : v;
  }
  return v;
}

// Running per-thread aggregates of the row preparation (PrepAgg fields).
struct PrepAcc {
  unsigned long long created = 0, kmax = 0, ovf = 0, unmono = 0, kmin = ULLONG_MAX;
  long long tmin = LLONG_MAX, tmax = LLONG_MIN, ctmax = LLONG_MIN;
};

// One extended row: key, flags (F_CAND / F_NEW / F_B / F_SKIP) and the
// timestamp as a 32-bit offset from the batch's first event (acc.ovf when it
// does not fit: the push then falls back to a 64-bit gather after the sort).
// Every load of the row is issued before the first use (ts, key, f1
// operands); the null-key test comes last.  FAST: the f1 chain is a
// pre-decoded conjunction and the key a plain column (no interpreter).
template <bool FAST>
__device__ __forceinline__ void prep_row(const PrepArgs& a, const DExprSet& es, int64_t r, int64_t tbase,
                                         bool count, uint64_t& k, uint32_t& f, int32_t& tso, PrepAcc& acc) {
  const ExtRows& x = a.x;
  long long t;
  k = 0;
  if (r < x.C) {
    k = a.partitioned ? gld(a.carry_key, r) : 0;
    f = F_CAND;
    t = (long long)gld(x.carry.ts, r);
    if (count) acc.ctmax = t > acc.ctmax ? t : acc.ctmax;
  } else {
    const int64_t br = r - x.C;
    BatchRowCtx cx{&x.batch, br};
    t = (long long)gld(x.batch.ts, br);
    const long long tprev = br > 0 ? (long long)gld(x.batch.ts, br - 1) : t;
    Val kv;
    kv.b = 0;
    kv.null = 0;
    if (a.partitioned) {
      if (FAST || a.key_col >= 0) kv = col_load(x.batch, br, a.key_col);
      else kv = eval_expr(es.ins + a.key_expr.off, a.key_expr.len, es.consts, cx);
    }
    const bool p1 = a.is_a && (FAST ? eval_fpred(a.f1.fp, cx) : eval_filters(es, a.f1, cx));
    f = F_NEW;
    if (kv.null && a.null_skip) {
      f |= F_SKIP;   // PartitionStreamReceiver drops null keys
      // no key: the row index spreads these rows over the hashed groups
      // (every walk passes over them, wherever they sort)
      k = (uint64_t)r;
    } else {
      if (a.is_b) f |= F_B;
      if (p1) {
        f |= F_CAND;
        acc.created += count ? 1u : 0u;
      }
      k = kv.null ? 0 : canon_key(kv, a.key_type);
    }
    if (count) {
      acc.tmin = t < acc.tmin ? t : acc.tmin;
      acc.tmax = t > acc.tmax ? t : acc.tmax;
      acc.unmono |= tprev > t;
    }
  }
  if (a.partitioned) {
    if (!a.key64) k = (uint32_t)k;   // 32-bit key types: the dictionary id / int bits
    if (count && !(f & F_SKIP)) {
      acc.kmax = k > acc.kmax ? k : acc.kmax;
      acc.kmin = k < acc.kmin ? k : acc.kmin;
    }
  }
  const int64_t dt = (int64_t)t - tbase;
  if (count) acc.ovf |= dt != (int64_t)(int32_t)dt;
  tso = (int32_t)dt;
}

// Per-block fold of the PrepAcc partials into blk[slot] (plain store;
// k_finish_prep folds the blocks): no same-address atomics from every wave.
template <int NT>
__device__ __forceinline__ void prep_block_reduce(PrepAcc acc, PrepAgg* blk, int slot) {
  for (int o = 32; o > 0; o >>= 1) {
    acc.created += __shfl_xor(acc.created, o, 64);
    acc.ovf |= __shfl_xor(acc.ovf, o, 64);
    acc.unmono |= __shfl_xor(acc.unmono, o, 64);
  }
  acc.kmax = wave_max(acc.kmax);
  acc.kmin = wave_min(acc.kmin);
  acc.tmin = wave_min(acc.tmin);
  acc.tmax = wave_max(acc.tmax);
  acc.ctmax = wave_max(acc.ctmax);
  __shared__ PrepAgg wpart[NT / 64];
  if ((threadIdx.x & 63) == 0)
    wpart[threadIdx.x >> 6] = PrepAgg{acc.created, acc.kmax, acc.tmin, acc.tmax, acc.ovf, acc.unmono, acc.ctmax, acc.kmin};
  __syncthreads();
  if (threadIdx.x == 0) {
    PrepAgg r = wpart[0];
    for (int w = 1; w < NT / 64; w++) {
      r.ovf |= wpart[w].ovf;
      r.unmono |= wpart[w].unmono;
      r.carry_tmax = wpart[w].carry_tmax > r.carry_tmax ? wpart[w].carry_tmax : r.carry_tmax;
      r.kmin = wpart[w].kmin < r.kmin ? wpart[w].kmin : r.kmin;
      r.n_cand += wpart[w].n_cand;
      r.kmax = wpart[w].kmax > r.kmax ? wpart[w].kmax : r.kmax;
      r.ts_min = wpart[w].ts_min < r.ts_min ? wpart[w].ts_min : r.ts_min;
      r.ts_max = wpart[w].ts_max > r.ts_max ? wpart[w].ts_max : r.ts_max;
    }
    blk[slot] = r;
  }
}

// Fused row preparation + first key-sort pass (keyed_sort.hip; partitioned
// plans on a 32-bit plain key attribute).  KsInfo: the sort's key base and
// width as sort_push derives them from the push's key range.
struct KsInfo {
  uint32_t kb;
  int32_t bits;
};
// The one attribute f1's loads read (-1: none or the pushed stream is not A;
// -2: f1 is not a pre-decoded chain over one attribute -- not fusable).
int keyed_sort_f1_attr(const DFilters& f1, bool is_a);
// hist + key range (d_pg: the push's PrepAgg with the key range only -- n_cand
// 0, time fields unset: keyed_sort_pass0 completes them -- and d_info, the
// sort's key base / width)
void keyed_sort_front(hipStream_t s, const PrepArgs* d_pa, const PrepArgs& pa, int64_t n_ext, DevBuf& scratch,
                      PrepAgg* d_pg, KsInfo* d_info);
// first pass: rows sorted by the first digit into (k32, pv, ts); completes
// d_pg (candidates created, time range / order / overflow, latest carried)
void keyed_sort_pass0(hipStream_t s, const PrepArgs* d_pa, const PrepArgs& pa, int fattr, int64_t n_ext,
                      DevBuf& scratch, const KsInfo* d_info, uint32_t* k32, uint32_t* pv, uint32_t* ts,
                      PrepAgg* d_pg);
// the remaining passes (digits from shift 8 to bits) of a fused sort
void keyed_sort_rest(hipStream_t s, int64_t n_ext, int bits, uint32_t kb, uint32_t* k32, uint32_t* pv, uint32_t* ts,
                     uint32_t* k32_alt, uint32_t* pv_alt, uint32_t* ts_alt, DevBuf& scratch, DevBuf& sort_scratch,
                     bool& in_alt);

}  // namespace pat
}  // namespace shd
