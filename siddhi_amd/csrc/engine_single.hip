// engine_single.hip -- single-stream queries on the device:
//   FILTER mode:  S[f]... select <expr> insert into   (+ optional `partition with`)
//   AGG mode:     S[f]#window.length(L)|time(T) select k, sum/avg/count group by k  (config W2)
//
// Reference semantics (modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/processor/filter/FilterProcessor.java:47-60
//   query/processor/stream/window/LengthWindowProcessor.java:105-142
//   query/processor/stream/window/TimeWindowProcessor.java:132-169 (+ Scheduler TIMERs)
//   query/selector/QuerySelector.java:161-205 (processNoGroupBy),
//     :271-313 (processInBatchNoGroupBy), :315-373 (processInBatchGroupBy)
//   query/selector/attribute/aggregator/{Sum,Avg,Count}AttributeAggregatorExecutor.java
//   stream/input/InputHandler.java:85-89 (playback: now := last ts of the call)
//
// AGG mode turns a micro-batch into the reference's operation stream: for every
// filtered event t, the window items that expire before it (FIFO order), then
// its own add.  Expiry position of item x: length -> x + L; time -> first later
// filtered event whose call time reaches ts_x + T, made FIFO-monotone with a
// prefix max.  Operations are key-sorted (stable) and each group is folded
// SEQUENTIALLY by one lane in operation order, so every double sum / avg is the
// same IEEE result the reference computes (bit-exact, no reassociation).
// Emission: one row per (call, group) with a CURRENT event, in first-seen
// order, carrying the values after the group's last event of the call.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "engine.h"
#include "gdict.h"
#include "agg.h"

namespace shd {

namespace {

constexpr uint32_t kInf = 0xFFFFFFFFu;
constexpr uint32_t kAddBit = 0x80000000u;
constexpr int64_t kMaxDenseKey = (int64_t)1 << 26;
// segmented scans only while every operand seen so far is finite and the
// non-zero magnitudes span at most 2^kSegMaxExpSpan (k_operand_stats)
constexpr uint32_t kSegMaxExpSpan = 30;
// ... and all of one sign: a window of mixed signs can cancel to far below its
// operands, where the reference's running sum keeps its rounding history
// (a difference of prefix sums does not bound that within 1e-9)
constexpr uint32_t kOpNeg = 2u, kOpPos = 4u;

// One aggregated operand into the range guard's statistics: flags (1 non-
// finite, kOpNeg, kOpPos) and the binary exponent range of the non-zero
// magnitudes.  int operands are skipped: their double running sums are exact
// (every partial sum is an integer below 2^53) in the reference and in the scans.
__device__ __forceinline__ void guard_operand(uint64_t b, int type, uint32_t& nf, uint32_t& emax, uint32_t& emin) {
  double d;
  if (type == SHD_T_INT) return;
  if (type == SHD_T_FLOAT) d = (double)__uint_as_float((uint32_t)b);
  else if (type == SHD_T_LONG) d = (double)(int64_t)b;
  else d = __longlong_as_double((long long)b);
  if (!(d - d == 0.0)) {   // Inf or NaN
    nf |= 1u;
    return;
  }
  if (d == 0.0) return;
  nf |= d < 0.0 ? kOpNeg : kOpPos;
  const uint32_t e = (uint32_t)((__double_as_longlong(d) >> 52) & 0x7FF);
  emax = e > emax ? e : emax;
  emin = e < emin ? e : emin;
}
constexpr int kMaxChan = 4;                   // distinct aggregated expressions (segmented scans)

struct RowCtx {
  const ColSet* cs;
  int64_t row;
  const uint64_t* aggv;   // [nagg] payloads for OP_AGG (may be null)
  const uint8_t* aggn;
  __device__ __forceinline__ Val load(int, int idx, int attr) const {
    (void)idx;
    return col_load(*cs, row, attr);
  }
  __device__ __forceinline__ bool evnull(int, int) const { return false; }
  __device__ __forceinline__ int64_t ts(int, int) const { return cs->ts[row]; }
  __device__ __forceinline__ Val agg(int i) const {
    Val v;
    v.b = aggv ? aggv[i] : 0;
    v.null = aggn ? aggn[i] : 1;
    return v;
  }
};

// ---------------------------------------------------------------- calls / time
// call_of[i] for every event; call_last_ts[c]
__global__ void k_call_of(const int64_t* offs, int ncalls, const int64_t* ts, int32_t* call_of, int64_t* last_ts) {
  for (int c = blockIdx.x; c < ncalls; c += gridDim.x) {
    int64_t a = offs[c], b = offs[c + 1];
    for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) call_of[i] = c;
    if (threadIdx.x == 0) last_ts[c] = b > a ? ts[b - 1] : INT64_MIN;
  }
}

// now[c] = max(now_prev, last_ts[0..c])  (TimestampGeneratorImpl only moves forward)
// only the playback time after the push: now[ncalls - 1] = max(now_prev, every last_ts)
__global__ __launch_bounds__(kBlock) void k_call_now_last(const int64_t* last_ts, int ncalls, int64_t now_prev,
                                                          int64_t* now) {
  __shared__ int64_t wmax[kBlock / 64];
  int64_t v = now_prev;
  for (int c = threadIdx.x; c < ncalls; c += kBlock) v = last_ts[c] > v ? last_ts[c] : v;
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  if ((threadIdx.x & 63) == 0) wmax[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; k++) v = wmax[k] > v ? wmax[k] : v;
    now[ncalls - 1] = v;
  }
}

__global__ __launch_bounds__(kBlock) void k_call_now(const int64_t* last_ts, int ncalls, int64_t now_prev,
                                                     int64_t* now) {
  __shared__ int64_t carry;
  __shared__ int64_t wmax[4];
  if (threadIdx.x == 0) carry = now_prev;
  __syncthreads();
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int base = 0; base < ncalls; base += kBlock) {
    int c = base + threadIdx.x;
    int64_t v = c < ncalls ? last_ts[c] : INT64_MIN;
    for (int o = 1; o < 64; o <<= 1) {
      int64_t t = __shfl_up(v, o, 64);
      if (lane >= o) v = t > v ? t : v;
    }
    if (lane == 63) wmax[w] = v;
    __syncthreads();
    int64_t pre = carry;
    for (int i = 0; i < w; i++) pre = wmax[i] > pre ? wmax[i] : pre;
    int64_t r = v > pre ? v : pre;
    if (c < ncalls) now[c] = r;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry = r;
    __syncthreads();
  }
}

// ---------------------------------------------------------------- filter
struct FilterArgs {
  ColSet cs;
  DExprSet es;
  DFilters filters;
  int partitioned;
  DExpr key;
  int key_col;
  int key_type;
};

// flags: bit0 = passes filters, bit1 = has a (non-null) partition key
__global__ __launch_bounds__(kBlock) void k_filter(const FilterArgs* __restrict__ ap, int64_t n, uint8_t* flags, uint32_t* cnt,
                                                   uint64_t* pkey) {
  const FilterArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  const DExprSet es = a.es;
  const ColSet& cs = a.cs;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    RowCtx cx{&cs, i, nullptr, nullptr};
    uint8_t f = 0;
    bool keyed = true;
    if (a.partitioned) {
      Val kv = a.key_col >= 0 ? col_load(cs, i, a.key_col)
                              : eval_expr(es.ins + a.key.off, a.key.len, es.consts, cx);
      keyed = !kv.null;
      pkey[i] = canon_key(kv, a.key_type);
    }
    if (keyed) {
      f |= 2;
      if (eval_filters(es, a.filters, cx)) f |= 1;
    }
    flags[i] = f;
    cnt[i] = (f & 3) == 3 ? 1u : 0u;
  }
}

// Partition runs (PartitionStreamReceiver.receive(Event[]) :189-214): a run
// starts at the first keyed event of a call or where the key changes from the
// previous keyed event.  run_start[i] in {0,1}; computed over keyed events.
__global__ void k_run_starts(const uint8_t* flags, const uint64_t* pkey, const int32_t* call_of, int64_t n,
                             uint32_t* start) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t s = 0;
    if (flags[i] & 2) {
      int64_t p = i - 1;
      while (p >= 0 && call_of[p] == call_of[i] && !(flags[p] & 2)) p--;
      s = (p < 0 || call_of[p] != call_of[i] || pkey[p] != pkey[i]) ? 1u : 0u;
    }
    start[i] = s;
  }
}

struct ProjArgs {
  ColSet cs;
  DExprSet es;
  DExpr outs[kMaxCols];
  int nout;
  int64_t row0;
  int64_t chunk0;
  int64_t seq0;   // arrival index of the batch's first event (shd_out.in_seq)
  int partitioned;
};

__global__ __launch_bounds__(kBlock) void k_project_rows(const ProjArgs* __restrict__ ap, int64_t n, const uint32_t* cnt,
                                                         const uint32_t* off, const int32_t* call_of,
                                                         const uint32_t* run_excl, const uint32_t* run_start,
                                                         int64_t* o_chunk, int32_t* o_type,
                                                         int64_t* o_ts, uint64_t* o_vals, uint8_t* o_nul,
                                                         int64_t* o_seq) {
  const ProjArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  const DExprSet es = a.es;
  const ColSet& cs = a.cs;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    if (!cnt[i]) continue;
    int64_t row = a.row0 + off[i];
    RowCtx cx{&cs, i, nullptr, nullptr};
    for (int c = 0; c < a.nout; c++) {
      Val v = eval_expr(es.ins + a.outs[c].off, a.outs[c].len, es.consts, cx);
      o_vals[row * a.nout + c] = v.b;
      o_nul[row * a.nout + c] = (uint8_t)v.null;
    }
    o_ts[row] = cs.ts[i];
    o_type[row] = 0;
    o_seq[row] = a.seq0 + i;
    // run of event i = inclusive start count - 1
    o_chunk[row] = a.chunk0 + (a.partitioned ? (int64_t)run_excl[i] + run_start[i] - 1 : (int64_t)call_of[i]);
  }
}

// ---------------------------------------------------------------- aggregation
struct ItemArgs {
  ColSet cs;
  DExprSet es;
  int nagg;
  DExpr agg_arg[kMaxAggs];
  int has_arg[kMaxAggs];
  int arg_col[kMaxAggs];   // >= 0: the argument is a plain attribute load (no interpreter)
  int ngroup;                 // group-by attributes (0..kMaxGroupAttrs)
  DExpr group[kMaxGroupAttrs];
  int group_col[kMaxGroupAttrs];
  int group_type[kMaxGroupAttrs];
  int dense;                  // 1: the one key value is the dense group id (string ids, bool)
  int64_t null_str_id;        // group id of a null string key (the string "null")
  // dictionary mode: per new item, the canonical key words, null mask and hash
  uint64_t* gkw;              // [ngroup][n_new]
  uint8_t* gkn;
  uint64_t* gh;
  int64_t gstride;            // words per group attribute in gkw (>= new items)
  int64_t C;
  int time_window;            // the item's time and call time are read (k_expiry) only by time windows
};

// Window item t (new item number inew = t - C) from event i.
__device__ __forceinline__ void make_item(const ItemArgs& a, int64_t i, int64_t inew, const int32_t* call_of,
                                          const int64_t* call_now, uint64_t* ikey, int64_t* its, uint64_t* iargv,
                                          uint8_t* iargn, int32_t* ievrow, int32_t* icall, int64_t* inow,
                                          int64_t cap) {
  const DExprSet es = a.es;
  const ColSet& cs = a.cs;
  const int64_t t = a.C + inew;
  RowCtx cx{&cs, i, nullptr, nullptr};
  uint64_t k = 0;
  if (a.ngroup) {
    // GroupByKeyGenerator.constructEventKey: String.valueOf of every value
    // joined -- canonical words with the same identifications (group_word)
    uint64_t h = 0x9E3779B97F4A7C15ull;
    uint8_t nm = 0;
    for (int g = 0; g < a.ngroup; g++) {
      Val kv = a.group_col[g] >= 0 ? col_load(cs, i, a.group_col[g])
                                   : eval_expr(es.ins + a.group[g].off, a.group[g].len, es.consts, cx);
      bool isnull = false;
      const uint64_t w = group_word(kv, a.group_type[g], a.null_str_id, isnull);
      if (a.dense) {
        k = isnull ? 2u : w;   // bool null: its own group (the text "null")
      } else {
        a.gkw[(int64_t)g * a.gstride + inew] = w;
        nm |= (uint8_t)((isnull ? 1u : 0u) << g);
        h = gdict_mix(h ^ gdict_mix(w + 0x632BE59BD9B4E019ull * (uint64_t)(g + 1)));
      }
    }
    if (!a.dense) {
      h = gdict_mix(h ^ ((uint64_t)nm << 56));
      a.gkn[inew] = nm;
      a.gh[inew] = h;
    }
  }
  ikey[t] = k;
  if (a.time_window) its[t] = cs.ts[i];
  for (int g = 0; g < a.nagg; g++) {
    if (!a.has_arg[g]) continue;   // count(): no operand (agg_step never reads it)
    const Val v = a.arg_col[g] >= 0 ? col_load(cs, i, a.arg_col[g])
                                    : eval_expr(es.ins + a.agg_arg[g].off, a.agg_arg[g].len, es.consts, cx);
    iargv[g * cap + t] = v.b;
    iargn[g * cap + t] = (uint8_t)v.null;
  }
  ievrow[t] = (int32_t)i;
  const int32_t c = call_of[i];
  icall[t] = c;
  if (a.time_window) inow[t] = call_now[c];
}

// New window items (one per filtered event), appended after the carried ones.
__global__ __launch_bounds__(kBlock) void k_make_items(const ItemArgs* __restrict__ ap, int64_t n, const uint32_t* cnt, const uint32_t* off,
                                                       const int32_t* call_of, const int64_t* call_now,
                                                       uint64_t* ikey, int64_t* its, uint64_t* iargv, uint8_t* iargn,
                                                       int32_t* ievrow, int32_t* icall, int64_t* inow, int64_t cap,
                                                       uint32_t* null_key_flag) {
  const ItemArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    if (!cnt[i]) continue;
    make_item(a, i, off[i], call_of, call_now, ikey, its, iargv, iargn, ievrow, icall, inow, cap);
  }
}

// Look-back status words: a device-coherent plain load (no read-modify-write:
// many workgroups poll the same words, and atomics on one line serialise in L2)
__device__ __forceinline__ uint64_t cw_status_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Filter + window items in one pass (aggregate queries outside partitions):
// tiles of kFiTile events in arrival order; a tile's passing events become
// items at the tile's offset, found by a decoupled look-back over the tiles
// (each tile publishes its count first).  Also: the first item of every
// InputHandler call (citem, for the call-window path), the largest new group
// id, and the range guard's operand statistics (k_operand_stats).
constexpr int kFiPer = 8;
constexpr int kFiTile = kBlock * kFiPer;

struct FusedArgs {
  FilterArgs f;
  ItemArgs it;
  const int32_t* call_of;
  const int64_t* call_now;
  uint64_t* ikey;
  int64_t* its;
  uint64_t* iargv;
  uint8_t* iargn;
  int32_t* ievrow;
  int32_t* icall;
  int64_t* inow;
  int64_t cap;
  uint64_t* status;     // [tiles] look-back words (zeroed)
  uint32_t* citem;      // [ncalls + 1]
  int ncalls;
  uint32_t* m_out;      // new items
  unsigned long long* kmax_out;
  int nch;              // range guard channels (0: none)
  int ch_agg[kMaxChan];
  int ch_t[kMaxChan];   // operand type of each channel
  uint32_t* opstats;    // [3]: flags (1 non-finite, kOpNeg, kOpPos), max / min binary exponent
};

__global__ __launch_bounds__(kBlock) void k_filter_items(const FusedArgs* __restrict__ ap, int64_t n) {
  const FusedArgs& a = *ap;
  const FilterArgs& fa = a.f;
  __shared__ uint32_t wcnt[kFiPer][kBlock / 64];
  __shared__ uint32_t tbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t base = (int64_t)blockIdx.x * kFiTile;
  const uint64_t below = (1ull << lane) - 1ull;
  uint64_t bal[kFiPer];
  for (int j = 0; j < kFiPer; j++) {
    const int64_t i = base + j * kBlock + threadIdx.x;
    bool pass = false;
    if (i < n) {
      RowCtx cx{&fa.cs, i, nullptr, nullptr};
      pass = eval_filters(fa.es, fa.filters, cx);
    }
    bal[j] = __ballot(pass);
    if (lane == 0) wcnt[j][w] = (uint32_t)__popcll(bal[j]);
  }
  __syncthreads();
  constexpr uint64_t kAgg = 1ull << 62, kInc = 2ull << 62, kVal = (1ull << 62) - 1;
  if (threadIdx.x < 64) {
    uint32_t local = 0;
    for (int j = 0; j < kFiPer; j++)
      for (int k = 0; k < kBlock / 64; k++) local += wcnt[j][k];
    const int c = blockIdx.x;
    if (lane == 0)
      atomicExch((unsigned long long*)&a.status[c], (unsigned long long)((c == 0 ? kInc : kAgg) | local));
    uint64_t tb = 0;
    for (int top = c - 1; top >= 0;) {
      const int j = top - lane;
      const uint64_t st = j >= 0 ? cw_status_load(&a.status[j]) : kInc;
      if (__any((st >> 62) == 0)) {   // an earlier, running workgroup has not published yet
        __builtin_amdgcn_s_sleep(4);
        continue;
      }
      const uint64_t incl = __ballot((st >> 62) == 2);
      const int stop = incl ? __ffsll((long long)incl) - 1 : 64;
      uint64_t v = lane <= stop && j >= 0 ? (st & kVal) : 0ull;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      tb += v;
      if (incl) break;
      top -= 64;
    }
    if (lane == 0) {
      if (c > 0) atomicExch((unsigned long long*)&a.status[c], (unsigned long long)(kInc | (tb + local)));
      tbase = (uint32_t)tb;
      if (base + kFiTile >= n) {   // the last tile: the push's item count, trailing empty calls
        const uint32_t m = (uint32_t)(tb + local);
        *a.m_out = m;
        const int c0 = n > 0 ? a.call_of[n - 1] + 1 : 0;
        for (int cc = c0; cc <= a.ncalls; cc++) a.citem[cc] = (uint32_t)(a.it.C + m);
      }
    }
  }
  __syncthreads();
  uint32_t pre = tbase;
  uint64_t kmax = 0;
  uint32_t nf = 0, emax = 0, emin = 0xFFFFFFFFu;
  for (int j = 0; j < kFiPer; j++) {
    uint32_t before_w = 0, tot_j = 0;
    for (int k = 0; k < kBlock / 64; k++) {
      before_w += k < w ? wcnt[j][k] : 0u;
      tot_j += wcnt[j][k];
    }
    const int64_t i = base + j * kBlock + threadIdx.x;
    const uint32_t pos = pre + before_w + (uint32_t)__popcll(bal[j] & below);   // items before event i
    if (i < n) {
      // first event of one or more calls (empty calls share their start event)
      const int32_t ci = a.call_of[i];
      const int32_t cp = i > 0 ? a.call_of[i - 1] : -1;
      for (int cc = cp + 1; cc <= ci; cc++) a.citem[cc] = (uint32_t)(a.it.C + pos);
      if ((bal[j] >> lane) & 1ull) {
        make_item(a.it, i, pos, a.call_of, a.call_now, a.ikey, a.its, a.iargv, a.iargn, a.ievrow, a.icall, a.inow,
                  a.cap);
        const int64_t t = a.it.C + pos;
        kmax = a.ikey[t] > kmax ? a.ikey[t] : kmax;
        for (int ch = 0; ch < a.nch; ch++) {
          const int g = a.ch_agg[ch];
          if (a.iargn[(int64_t)g * a.cap + t]) continue;
          guard_operand(a.iargv[(int64_t)g * a.cap + t], a.ch_t[ch], nf, emax, emin);
        }
      }
    }
    pre += tot_j;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t km = __shfl_xor(kmax, o, 64);
    kmax = km > kmax ? km : kmax;
    nf |= __shfl_xor(nf, o, 64);
    const uint32_t x = __shfl_xor(emax, o, 64), y = __shfl_xor(emin, o, 64);
    emax = x > emax ? x : emax;
    emin = y < emin ? y : emin;
  }
  // one word each for the whole push: an atomic only when this wave would
  // change it (atomics on one address serialise in L2; the words settle fast)
  if (lane == 0) {
    if (kmax > cw_status_load((const uint64_t*)a.kmax_out)) atomicMax(a.kmax_out, (unsigned long long)kmax);
    if (a.nch) {
      if (nf & ~__hip_atomic_load(&a.opstats[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicOr(&a.opstats[0], nf);
      if (emax > __hip_atomic_load(&a.opstats[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMax(&a.opstats[1], emax);
      if (emin < __hip_atomic_load(&a.opstats[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        atomicMin(&a.opstats[2], emin);
    }
  }
}

// ---------------------------------------------------------------- group dictionary (gdict.h)

// Range guard of the segmented-scan mode: over the new items' double / float
// operands of the scanned channels, flags[0] |= 1 for a non-finite value,
// flags[1] = max and flags[2] = min binary exponent of the non-zero values.
// (One atomic per block; a grid of at most 1024 blocks.)
__global__ __launch_bounds__(kBlock) void k_operand_stats(const uint64_t* argv, const uint8_t* argn, int64_t cap,
                                                          int64_t C, int64_t m, int nch, const int* ch_agg,
                                                          const int* ch_type, uint32_t* flags) {
  uint32_t nf = 0, emax = 0, emin = 0xFFFFFFFFu;
  for (int c = 0; c < nch; c++) {
    const int g = ch_agg[c];
    const int type = ch_type[c];
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < m; i += (int64_t)gridDim.x * kBlock) {
      const int64_t t = C + i;
      if (argn[(int64_t)g * cap + t]) continue;
      guard_operand(argv[(int64_t)g * cap + t], type, nf, emax, emin);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    nf |= __shfl_xor(nf, o, 64);
    const uint32_t a = __shfl_xor(emax, o, 64), b = __shfl_xor(emin, o, 64);
    emax = a > emax ? a : emax;
    emin = b < emin ? b : emin;
  }
  __shared__ uint32_t sh[3][kBlock / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[0][w] = nf;
    sh[1][w] = emax;
    sh[2][w] = emin;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kBlock / 64; k++) {
      nf |= sh[0][k];
      emax = sh[1][k] > emax ? sh[1][k] : emax;
      emin = sh[2][k] < emin ? sh[2][k] : emin;
    }
    if (nf) atomicOr(&flags[0], nf);
    atomicMax(&flags[1], emax);
    atomicMin(&flags[2], emin);
  }
}

// Expiry position of every window item.
__global__ void k_expiry(int wkind, int64_t wparam, int64_t C, int64_t total, const int64_t* its,
                         const int64_t* inow, uint32_t* e) {
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (int64_t)gridDim.x * blockDim.x) {
    uint32_t r = kInf;
    if (wkind == SHD_W_LENGTH) {
      int64_t t = x + wparam;
      if (t < total) r = (uint32_t)t;
    } else if (wkind == SHD_W_TIME) {
      // TimeWindowProcessor: expire when ts_x - now + T <= 0, checked before each later add
      int64_t lo = x + 1 > C ? x + 1 : C, hi = total;
      int64_t target = its[x] + wparam;
      while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (inow[mid] >= target) hi = mid;
        else lo = mid + 1;
      }
      if (lo < total) r = (uint32_t)lo;
    }
    e[x] = r;
  }
}

// in-place inclusive prefix max over u32 (FIFO: an item cannot leave before its predecessor)
__global__ __launch_bounds__(kBlock) void k_prefix_max_u32(uint32_t* e, int64_t n) {
  __shared__ uint32_t carry;
  __shared__ uint32_t wm[4];
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t base = 0; base < n; base += kBlock) {
    int64_t i = base + threadIdx.x;
    uint32_t v = i < n ? e[i] : 0;
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t t = __shfl_up(v, o, 64);
      if (lane >= o) v = t > v ? t : v;
    }
    if (lane == 63) wm[w] = v;
    __syncthreads();
    uint32_t pre = carry;
    for (int k = 0; k < w; k++) pre = wm[k] > pre ? wm[k] : pre;
    uint32_t r = v > pre ? v : pre;
    if (i < n) e[i] = r;
    __syncthreads();
    if (threadIdx.x == kBlock - 1) carry = r;
    __syncthreads();
  }
}

// Parallel form of k_prefix_max_u32 for large item counts: per-tile maxima,
// one-block exclusive prefix max over the tiles, then per-tile inclusive
// prefix max with the carry-in.  Tiles of kPmaxTile items (4 per thread).
constexpr int kPmaxTile = kBlock * 4;

__device__ __forceinline__ uint32_t block_max_u32(uint32_t v, uint32_t* wm) {
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t r = 0;
  for (int k = 0; k < kBlock / 64; k++) r = wm[k] > r ? wm[k] : r;
  return r;
}

__global__ __launch_bounds__(kBlock) void k_pmax_tiles(const uint32_t* e, int64_t n, uint32_t* tmax) {
  __shared__ uint32_t wm[kBlock / 64];
  const int64_t b0 = (int64_t)blockIdx.x * kPmaxTile + threadIdx.x * 4;
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 4; i++)
    if (b0 + i < n) v = e[b0 + i] > v ? e[b0 + i] : v;
  const uint32_t r = block_max_u32(v, wm);
  if (threadIdx.x == 0) tmax[blockIdx.x] = r;
}

// exclusive prefix max over the tile maxima (in place), one block
__global__ __launch_bounds__(kBlock) void k_pmax_scan(uint32_t* tmax, int64_t nt) {
  __shared__ uint32_t wm[kBlock / 64];
  __shared__ uint32_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t base = 0; base < nt; base += kBlock) {
    const int64_t i = base + threadIdx.x;
    const uint32_t x = i < nt ? tmax[i] : 0;
    uint32_t v = x;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(v, o, 64);
      if (lane >= o) v = t > v ? t : v;
    }
    if (lane == 63) wm[w] = v;
    __syncthreads();
    uint32_t pre = carry;
    for (int k = 0; k < w; k++) pre = wm[k] > pre ? wm[k] : pre;
    // exclusive: max of everything before i
    uint32_t ex = __shfl_up(v, 1, 64);
    ex = lane == 0 ? pre : (ex > pre ? ex : pre);
    const uint32_t inc = v > pre ? v : pre;
    __syncthreads();
    if (i < nt) tmax[i] = ex;
    if (threadIdx.x == kBlock - 1) carry = inc;
    __syncthreads();
  }
}

__global__ __launch_bounds__(kBlock) void k_pmax_apply(uint32_t* e, int64_t n, const uint32_t* tpre) {
  __shared__ uint32_t wm[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * kPmaxTile + threadIdx.x * 4;
  uint32_t x[4];
  uint32_t v = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    x[i] = b0 + i < n ? e[b0 + i] : 0;
    v = x[i] > v ? x[i] : v;
  }
  // exclusive prefix max of the per-thread maxima within the block
  uint32_t inc = v;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc = t > inc ? t : inc;
  }
  if (lane == 63) wm[w] = inc;
  __syncthreads();
  uint32_t pre = tpre[blockIdx.x];
  for (int k = 0; k < w; k++) pre = wm[k] > pre ? wm[k] : pre;
  uint32_t ex = __shfl_up(inc, 1, 64);
  if (lane != 0) pre = ex > pre ? ex : pre;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    pre = x[i] > pre ? x[i] : pre;
    if (b0 + i < n) e[b0 + i] = pre;
  }
}

__global__ void k_count_expired(const uint32_t* e, int64_t n, unsigned long long* cnt) {
  uint64_t c = 0;
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n; x += (int64_t)gridDim.x * blockDim.x)
    c += e[x] != kInf;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, (unsigned long long)c);
}

// number of x with e[x] <= t (e is non-decreasing)
__device__ __forceinline__ int64_t count_le(const uint32_t* e, int64_t n, uint32_t t) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    int64_t mid = (lo + hi) >> 1;
    if (e[mid] <= t) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ void k_make_ops(int64_t C, int64_t total, const uint32_t* e, const uint64_t* ikey, uint64_t* okey,
                           uint32_t* oref) {
  for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total; x += (int64_t)gridDim.x * blockDim.x) {
    if (e[x] != kInf) {   // expire op of item x, before the add of item e[x]
      int64_t idx = ((int64_t)e[x] - C) + x;
      okey[idx] = ikey[x];
      oref[idx] = (uint32_t)x;
    }
    if (x >= C) {         // add op of item x
      int64_t idx = (x - C) + count_le(e, total, (uint32_t)x);
      okey[idx] = ikey[x];
      oref[idx] = (uint32_t)x | kAddBit;
    }
  }
}

__global__ void k_narrow(const uint64_t* in, uint32_t* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)in[i];
}

__global__ void k_gather_u64(const uint64_t* src, const uint32_t* perm, uint64_t* dst, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[perm[i]];
}

__global__ void k_seg_heads(const uint32_t* skey, int64_t n, uint32_t* head) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i == 0 || skey[i] != skey[i - 1]) ? 1u : 0u;
}

__global__ void k_head_list(const uint32_t* head, const uint32_t* hoff, int64_t n, uint32_t* hl) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (head[i]) hl[hoff[i]] = (uint32_t)i;
}

struct FoldArgs {
  int nagg;
  int kind[kMaxAggs];
  int type[kMaxAggs];
  int64_t cap;               // item capacity (stride of per-agg item arrays)
  // group state tables (dense by key), [nagg][nkeys]
  double* dsum;
  int64_t* lsum;
  int64_t* cnt;
  int64_t nkeys;
};

// One lane per group segment: the reference's sequential add/remove order
// (short segments: many groups, few operations each).
__global__ __launch_bounds__(kBlock) void k_fold(const FoldArgs* __restrict__ ap, const uint32_t* heads, int64_t nheads, int64_t nops,
                                                 const uint32_t* okey_sorted, const uint32_t* oref_sorted,
                                                 const uint64_t* iargv, const uint8_t* iargn, const int32_t* ievrow,
                                                 const int32_t* call_of, uint64_t* resv, uint8_t* resn,
                                                 int64_t* resc, uint8_t* first, uint32_t* last_of) {
  const FoldArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  for (int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; h < nheads; h += (int64_t)gridDim.x * blockDim.x) {
    int64_t q0 = heads[h];
    int64_t q1 = h + 1 < nheads ? (int64_t)heads[h + 1] : nops;
    uint32_t key = okey_sorted[q0];
    double d[kMaxAggs];
    int64_t l[kMaxAggs], c[kMaxAggs];
    for (int g = 0; g < a.nagg; g++) {
      d[g] = a.dsum[g * a.nkeys + key];
      l[g] = a.lsum[g * a.nkeys + key];
      c[g] = a.cnt[g * a.nkeys + key];
    }
    int32_t cur_call = -1;
    uint32_t t_first = 0, t_prev = 0;
    for (int64_t q = q0; q < q1; q++) {
      uint32_t ref = oref_sorted[q];
      bool add = ref & kAddBit;
      uint32_t t = ref & ~kAddBit;
      for (int g = 0; g < a.nagg; g++) {
        uint64_t ob;
        bool on;
        agg_step(a.kind[g], a.type[g], add, iargv[g * a.cap + t], iargn[g * a.cap + t], d[g], l[g], c[g], ob, on);
        if (add) {
          resv[g * a.cap + t] = ob;
          resn[g * a.cap + t] = (uint8_t)on;
          if (a.kind[g] == SHD_AGG_AVG) resc[g * a.cap + t] = c[g];
        }
      }
      if (add) {
        int32_t call = call_of[ievrow[t]];
        if (call != cur_call) {
          if (cur_call >= 0) last_of[t_first] = t_prev;
          first[t] = 1;
          t_first = t;
          cur_call = call;
        }
        t_prev = t;
      }
    }
    if (cur_call >= 0) last_of[t_first] = t_prev;
    for (int g = 0; g < a.nagg; g++) {
      a.dsum[g * a.nkeys + key] = d[g];
      a.lsum[g * a.nkeys + key] = l[g];
      a.cnt[g * a.nkeys + key] = c[g];
    }
  }
}

// One WAVE per group segment (long segments: few groups, many operations --
// config W2 has 1000 groups and ~30k operations per group per push).  The
// wave loads 64 consecutive operations with coalesced loads (the gathers of
// their operands run in parallel across lanes, NCH chunks ahead of the fold),
// then folds them in order with the running state held wave-uniform: step k
// reads lane k's operands (readlane) and deposits the result in lane k.  Same
// arithmetic, same order as k_fold: bit-identical results.
template <int NA>
__global__ __launch_bounds__(kBlock) void k_fold_wave(const FoldArgs* __restrict__ ap, const uint32_t* heads,
                                                      int64_t nheads, int64_t nops, const uint32_t* okey_sorted,
                                                      const uint32_t* oref_sorted, const uint64_t* iargv,
                                                      const uint8_t* iargn, const int32_t* ievrow,
                                                      const int32_t* call_of, uint64_t* resv, uint8_t* resn,
                                                      int64_t* resc, uint8_t* first, uint32_t* last_of) {
  const FoldArgs& a = *ap;
  const int lane = threadIdx.x & 63;
  const int64_t h = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;   // one wave per head
  if (h >= nheads) return;
  const int64_t q0 = heads[h];
  const int64_t q1 = h + 1 < nheads ? (int64_t)heads[h + 1] : nops;
  const uint32_t key = okey_sorted[q0];
  double d[NA];
  int64_t l[NA], c[NA];
#pragma unroll
  for (int g = 0; g < NA; g++) {
    d[g] = a.dsum[g * a.nkeys + key];
    l[g] = a.lsum[g * a.nkeys + key];
    c[g] = a.cnt[g * a.nkeys + key];
  }
  int kind[NA], type[NA];
#pragma unroll
  for (int g = 0; g < NA; g++) {
    kind[g] = a.kind[g];
    type[g] = a.type[g];
  }
  int32_t cur_call = -1;
  uint32_t t_first = 0, t_prev = 0;
  // operands of one 64-operation chunk, lane k = operation base + k
  struct Chunk {
    uint32_t ref;
    int32_t call;
    uint64_t xb[NA];
    uint8_t xn[NA];
  };
  auto load = [&](int64_t base, Chunk& ch) {
    const int64_t q = base + lane;
    ch.ref = q < q1 ? oref_sorted[q] : 0u;
    const uint32_t t = ch.ref & ~kAddBit;
#pragma unroll
    for (int g = 0; g < NA; g++) {
      ch.xb[g] = q < q1 ? iargv[g * a.cap + t] : 0ull;
      ch.xn[g] = q < q1 ? iargn[g * a.cap + t] : (uint8_t)0;
    }
    ch.call = (q < q1 && (ch.ref & kAddBit)) ? call_of[ievrow[t]] : -1;
  };
  constexpr int NCH = 4;   // chunks in flight
  Chunk ring[NCH];
#pragma unroll
  for (int i = 0; i < NCH; i++) load(q0 + (int64_t)i * 64, ring[i]);
  for (int64_t base = q0; base < q1; base += 64 * NCH) {
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      const int64_t cb = base + (int64_t)i * 64;
      if (cb >= q1) break;
      Chunk ch = ring[i];
      load(cb + 64 * NCH, ring[i]);   // refill this slot NCH chunks ahead
      const int nk = q1 - cb < 64 ? (int)(q1 - cb) : 64;
      uint64_t ob_l[NA];
      int64_t oc_l[NA];
      uint8_t on_l[NA];
      uint8_t first_l = 0;
      for (int k = 0; k < nk; k++) {
        const uint32_t ref = (uint32_t)__builtin_amdgcn_readlane((int)ch.ref, k);
        const bool add = ref & kAddBit;
        const uint32_t t = ref & ~kAddBit;
#pragma unroll
        for (int g = 0; g < NA; g++) {
          const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ch.xb[g], k);
          const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ch.xb[g] >> 32), k);
          const bool xn = __builtin_amdgcn_readlane((int)ch.xn[g], k) != 0;
          uint64_t ob;
          bool on;
          agg_step(kind[g], type[g], add, ((uint64_t)hi << 32) | lo, xn, d[g], l[g], c[g], ob, on);
          if (lane == k) {
            ob_l[g] = ob;
            on_l[g] = (uint8_t)on;
            oc_l[g] = c[g];
          }
        }
        if (add) {
          const int32_t call = __builtin_amdgcn_readlane(ch.call, k);
          if (call != cur_call) {
            if (cur_call >= 0 && lane == 0) last_of[t_first] = t_prev;
            if (lane == k) first_l = 1;
            t_first = t;
            cur_call = call;
          }
          t_prev = t;
        }
      }
      if (lane < nk && (ch.ref & kAddBit)) {
        const uint32_t t = ch.ref & ~kAddBit;
#pragma unroll
        for (int g = 0; g < NA; g++) {
          resv[g * a.cap + t] = ob_l[g];
          resn[g * a.cap + t] = on_l[g];
          if (kind[g] == SHD_AGG_AVG) resc[g * a.cap + t] = oc_l[g];
        }
        if (first_l) first[t] = 1;
      }
    }
  }
  if (cur_call >= 0 && lane == 0) last_of[t_first] = t_prev;
  if (lane == 0) {
#pragma unroll
    for (int g = 0; g < NA; g++) {
      a.dsum[g * a.nkeys + key] = d[g];
      a.lsum[g * a.nkeys + key] = l[g];
      a.cnt[g * a.nkeys + key] = c[g];
    }
  }
}

// Wave fold specialised for the aggregators whose state is a double running
// sum plus a count -- count(), sum(double|float), avg(any numeric); config W2
// is avg(price), sum(price), count().  Branch-light: the counts after every
// operation are a wave prefix sum (integers: exact in any order); only the
// double sums run as sequential chains, one v_add_f64 per operation in
// operation order (a - b == a + (-b) in IEEE 754: identical to the reference's
// value -= x), with the operands read by v_readlane; the callback-run
// bookkeeping (first / last_of) comes from ballots.  Results are bit-identical
// to agg_step / k_fold.
__device__ __forceinline__ int wave_incl_scan_i32(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ double readlane_f64(double v, int k) {
  const uint64_t b = (uint64_t)__double_as_longlong(v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, k);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), k);
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

template <int NA>
__global__ __launch_bounds__(kBlock) void k_fold_wave_d(const FoldArgs* __restrict__ ap, const uint32_t* heads,
                                                        int64_t nheads, int64_t nops, const uint32_t* okey_sorted,
                                                        const uint32_t* oref_sorted, const uint64_t* iargv,
                                                        const uint8_t* iargn, const int32_t* ievrow,
                                                        const int32_t* call_of, uint64_t* resv, uint8_t* resn,
                                                        int64_t* resc, uint8_t* first, uint32_t* last_of) {
  const FoldArgs& a = *ap;
  const int lane = threadIdx.x & 63;
  const uint64_t below = lane ? (~0ull >> (64 - lane)) : 0ull;
  const int64_t h = ((int64_t)blockIdx.x * kBlock + threadIdx.x) >> 6;   // one wave per head
  if (h >= nheads) return;
  const int64_t q0 = heads[h];
  const int64_t q1 = h + 1 < nheads ? (int64_t)heads[h + 1] : nops;
  const uint32_t key = okey_sorted[q0];
  int kind[NA], type[NA];
  double d[NA];
  int64_t c[NA];
#pragma unroll
  for (int g = 0; g < NA; g++) {
    kind[g] = a.kind[g];
    type[g] = a.type[g];
    d[g] = a.dsum[g * a.nkeys + key];
    c[g] = a.cnt[g * a.nkeys + key];
  }
  int32_t cur_call = -1;
  uint32_t t_first = 0, t_prev = 0;
  struct Chunk {
    uint32_t ref;
    int32_t call;
    uint64_t xb[NA];
    uint8_t xn[NA];
  };
  auto load = [&](int64_t base, Chunk& ch) {
    const int64_t q = base + lane;
    ch.ref = q < q1 ? oref_sorted[q] : 0u;
    const uint32_t t = ch.ref & ~kAddBit;
#pragma unroll
    for (int g = 0; g < NA; g++) {
      ch.xb[g] = q < q1 ? iargv[g * a.cap + t] : 0ull;
      ch.xn[g] = q < q1 ? iargn[g * a.cap + t] : (uint8_t)0;
    }
    ch.call = (q < q1 && (ch.ref & kAddBit)) ? call_of[ievrow[t]] : -1;
  };
  constexpr int NCH = 4;   // chunks in flight
  Chunk ring[NCH];
#pragma unroll
  for (int i = 0; i < NCH; i++) load(q0 + (int64_t)i * 64, ring[i]);
  for (int64_t base = q0; base < q1; base += 64 * NCH) {
#pragma unroll
    for (int i = 0; i < NCH; i++) {
      const int64_t cb = base + (int64_t)i * 64;
      if (cb >= q1) break;
      const Chunk ch = ring[i];
      load(cb + 64 * NCH, ring[i]);   // refill this slot NCH chunks ahead
      const int nk = q1 - cb < 64 ? (int)(q1 - cb) : 64;
      const bool valid = lane < nk;
      const bool add = valid && (ch.ref & kAddBit);
      const uint32_t t = ch.ref & ~kAddBit;
      double x[NA], dk[NA];
      uint64_t skip[NA];
      int64_t ck[NA];
      bool xn[NA];
#pragma unroll
      for (int g = 0; g < NA; g++) {
        xn[g] = kind[g] != SHD_AGG_COUNT && ch.xn[g];
        const int dc = !valid || xn[g] ? 0 : (add ? 1 : -1);
        const int inc = wave_incl_scan_i32(dc, lane);
        ck[g] = c[g] + inc;
        c[g] += __builtin_amdgcn_readlane(inc, 63);
        double v;
        switch (type[g]) {   // Number.doubleValue() of the operand
          case SHD_T_INT: v = (double)v_i32(ch.xb[g]); break;
          case SHD_T_LONG: v = (double)(int64_t)ch.xb[g]; break;
          case SHD_T_FLOAT: v = (double)v_f32(ch.xb[g]); break;
          default: v = v_f64(ch.xb[g]);
        }
        x[g] = add ? v : -v;
        skip[g] = __ballot(!valid || xn[g] || kind[g] == SHD_AGG_COUNT);
        dk[g] = d[g];
      }
      // the sequential double chains, in operation order (independent across aggregators)
      for (int k = 0; k < nk; k++) {
#pragma unroll
        for (int g = 0; g < NA; g++) {
          const double xk = readlane_f64(x[g], k);
          if (!((skip[g] >> k) & 1ull)) d[g] = __dadd_rn(d[g], xk);
          dk[g] = lane == k ? d[g] : dk[g];
        }
      }
      // callback runs: consecutive add operations of one InputHandler call
      const uint64_t A = __ballot(add);
      const uint64_t Ab = A & below;
      const bool has_prev = Ab != 0;
      const int pl = has_prev ? 63 - __clzll(Ab) : lane;   // previous add lane
      const int32_t call_p = __shfl(ch.call, pl, 64);
      const uint32_t t_p = __shfl(t, pl, 64);
      const bool fst = add && ch.call != (has_prev ? call_p : cur_call);
      const uint64_t F = __ballot(fst);
      const uint64_t Fp = has_prev ? (F & (pl == 63 ? ~0ull : ((2ull << pl) - 1ull))) : 0ull;
      const int sl = Fp ? 63 - __clzll(Fp) : lane;          // run start at or before pl
      const uint32_t t_s = __shfl(t, sl, 64);
      if (fst) {
        if (has_prev) last_of[Fp ? t_s : t_first] = t_p;    // the run that ended at pl
        else if (cur_call >= 0) last_of[t_first] = t_prev;  // the run carried from earlier chunks
      }
      if (add) {
#pragma unroll
        for (int g = 0; g < NA; g++) {
          uint64_t ob;
          uint8_t on;
          if (kind[g] == SHD_AGG_COUNT) {
            ob = (uint64_t)ck[g];
            on = 0;
          } else {
            ob = p_f64(dk[g]);
            on = kind[g] == SHD_AGG_SUM ? (uint8_t)(xn[g] && !(type[g] == SHD_T_DOUBLE && ck[g] != 0))
                                        : (uint8_t)(ck[g] == 0);   // avg: value / count at emission
            if (on) ob = 0;
          }
          resv[g * a.cap + t] = ob;
          resn[g * a.cap + t] = on;
          if (kind[g] == SHD_AGG_AVG) resc[g * a.cap + t] = ck[g];
        }
        if (fst) first[t] = 1;
      }
      if (A) {
        const int ll = 63 - __clzll(A);
        cur_call = __builtin_amdgcn_readlane(ch.call, ll);
        t_prev = (uint32_t)__builtin_amdgcn_readlane((int)t, ll);
        if (F) t_first = (uint32_t)__builtin_amdgcn_readlane((int)t, 63 - __clzll(F));
      }
    }
  }
  if (cur_call >= 0 && lane == 0) last_of[t_first] = t_prev;
  if (lane == 0) {
#pragma unroll
    for (int g = 0; g < NA; g++) {
      a.dsum[g * a.nkeys + key] = d[g];
      a.cnt[g * a.nkeys + key] = c[g];
    }
  }
}

// ------------------------------------------------ segmented-scan aggregation
// Default mode for count / sum(double|float) / avg(any numeric) (north_star:
// "sliding-window sum/avg/count use segmented scans"; the exact sequential
// fold above stays behind the `exact_aggregates` option).  Window items are
// stably sorted by group, so a group's items are one segment in arrival order.
// A segmented inclusive scan gives every position p the group prefix S(p) of
// its channel values (double-double: hi + lo, so the prefix itself carries
// no rounding error worth the name) and of its non-null counts.  The window
// of a group right after the add of item x (sorted position p) is the
// positions [k, p] of its segment whose expiry e > x (FIFO expiry makes e
// non-decreasing along a segment, so k comes from a galloping search), and
// its aggregate is S(p) - S(k-1): the reference's running value (Java
// `sum += v; sum -= v`, SumAttributeAggregatorExecutor.java:184-198,
// AvgAttributeAggregatorExecutor.java:148-166) up to that running value's
// own rounding residue -- checked at rtol 1e-9 (tests/test_gpu_segscan.py).
// Counts are exact integers.
constexpr int kSegPer = 8;                    // positions per thread
constexpr int kSegTile = kBlock * kSegPer;    // positions per tile (workgroup)

struct DD {
  double hi, lo;
};
// error-free sum of two double-doubles (Knuth two-sum + renormalisation);
// the build has -ffp-contract=off, so no step is fused
__device__ __forceinline__ DD dd_add(DD a, DD b) {
  const double s = a.hi + b.hi;
  const double bb = s - a.hi;
  const double err = (a.hi - (s - bb)) + (b.hi - bb);
  const double lo = (a.lo + b.lo) + err;
  const double hi = s + lo;
  return DD{hi, lo - (hi - s)};
}
__device__ __forceinline__ double dd_diff(DD a, DD b) {   // round(a - b)
  const double s = a.hi - b.hi;
  const double bb = s - a.hi;
  const double err = (a.hi - (s - bb)) + (-b.hi - bb);
  return s + (err + (a.lo - b.lo));
}

template <int NC>
struct SegAcc {
  int flag;            // a segment head lies in the range
  DD s[NC];            // channel sums since the range's last head (whole range if none)
  int32_t nn[NC];      // non-null counts, likewise
};
template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_identity() {
  SegAcc<NC> r;
  r.flag = 0;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    r.s[c] = DD{0.0, 0.0};
    r.nn[c] = 0;
  }
  return r;
}
// a (earlier range) then b (later range)
template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_combine(const SegAcc<NC>& a, const SegAcc<NC>& b) {
  if (b.flag) return b;
  SegAcc<NC> r;
  r.flag = a.flag;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    r.s[c] = dd_add(a.s[c], b.s[c]);
    r.nn[c] = a.nn[c] + b.nn[c];
  }
  return r;
}
template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_shfl_up(const SegAcc<NC>& a, int o) {
  SegAcc<NC> r;
  r.flag = __shfl_up(a.flag, o, 64);
#pragma unroll
  for (int c = 0; c < NC; c++) {
    r.s[c].hi = __shfl_up(a.s[c].hi, o, 64);
    r.s[c].lo = __shfl_up(a.s[c].lo, o, 64);
    r.nn[c] = __shfl_up(a.nn[c], o, 64);
  }
  return r;
}
// inclusive segmented scan over the 64 lanes of a wave
template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_wave_scan(SegAcc<NC> v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const SegAcc<NC> t = seg_shfl_up(v, o);
    if (lane >= o) v = seg_combine(t, v);
  }
  return v;
}

struct SegArgs {
  int nch;
  int ch_agg[kMaxChan];      // first aggregator of each channel (its argument column)
  int ch_type[kMaxChan];
  int nagg;
  int kind[kMaxAggs];
  int type[kMaxAggs];
  int chan[kMaxAggs];        // channel of each aggregator (-1: count())
  int64_t cap;               // item capacity (stride of per-agg item arrays)
  int64_t C;                 // carried items [0, C)
  int64_t total;             // items [0, total)
  double* dsum;              // group tables [nagg][nkeys] (window state after the push)
  int64_t* cnt;
  int64_t nkeys;
};

// sorted-order copies of what the scan and the window search read
template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_gather(const SegArgs* __restrict__ ap, const uint32_t* sp,
                                                       const uint64_t* iargv, const uint8_t* iargn,
                                                       const uint32_t* e, const int32_t* icall, double* sval,
                                                       uint8_t* snn, uint32_t* se, int32_t* scall) {
  const SegArgs& a = *ap;
  const int64_t total = a.total;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < total; p = total) {
    const uint32_t x = sp[p];
    uint8_t m = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const int g = a.ch_agg[c];
      const uint64_t b = iargv[g * a.cap + x];
      const bool nul = iargn[g * a.cap + x] != 0;
      double v;
      switch (a.ch_type[c]) {   // Number.doubleValue() of the operand
        case SHD_T_INT: v = (double)v_i32(b); break;
        case SHD_T_LONG: v = (double)(int64_t)b; break;
        case SHD_T_FLOAT: v = (double)v_f32(b); break;
        default: v = v_f64(b);
      }
      sval[c * total + p] = nul ? 0.0 : v;
      m |= nul ? 0 : (uint8_t)(1u << c);
    }
    snn[p] = m;
    se[p] = e[x];
    scall[p] = (int64_t)x >= a.C ? icall[x] : -1;
  }
}

// Packed item records (NC <= 2): everything the sorted copies need of item x
// in one 8*NC + 8 byte record written in item order (coalesced), so the
// gather by sorted position reads one record per item instead of 2 + 2*NC
// scattered words.  w = (call + 1) | nn << 30 (calls of a push < 2^30).
template <int NC>
struct SegItem {
  double v[NC];
  uint32_t e;
  uint32_t w;
};

template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_pack(const SegArgs* __restrict__ ap, const uint64_t* iargv,
                                                     const uint8_t* iargn, const uint32_t* e, const int32_t* icall,
                                                     SegItem<NC>* items) {
  const SegArgs& a = *ap;
  const int64_t total = a.total;
  for (int64_t x = (int64_t)blockIdx.x * kBlock + threadIdx.x; x < total; x = total) {
    SegItem<NC> it;
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      const int g = a.ch_agg[c];
      const uint64_t b = iargv[g * a.cap + x];
      const bool nul = iargn[g * a.cap + x] != 0;
      double v;
      switch (a.ch_type[c]) {   // Number.doubleValue() of the operand
        case SHD_T_INT: v = (double)v_i32(b); break;
        case SHD_T_LONG: v = (double)(int64_t)b; break;
        case SHD_T_FLOAT: v = (double)v_f32(b); break;
        default: v = v_f64(b);
      }
      it.v[c] = nul ? 0.0 : v;
      m |= nul ? 0u : (1u << c);
    }
    const int32_t call = x >= a.C ? icall[x] : -1;
    it.e = e[x];
    it.w = ((uint32_t)(call + 1) & 0x3FFFFFFFu) | (m << 30);
    items[x] = it;
  }
}

template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_gather_packed(const SegArgs* __restrict__ ap, const uint32_t* sp,
                                                              const SegItem<NC>* items, double* sval, uint8_t* snn,
                                                              uint32_t* se, int32_t* scall) {
  const SegArgs& a = *ap;
  const int64_t total = a.total;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < total; p = total) {
    const SegItem<NC> it = items[sp[p]];
#pragma unroll
    for (int c = 0; c < NC; c++) sval[c * total + p] = it.v[c];
    snn[p] = (uint8_t)(it.w >> 30);
    se[p] = it.e;
    scall[p] = (int32_t)(it.w & 0x3FFFFFFFu) - 1;
  }
}

// this thread's kSegPer consecutive positions as one segmented range
template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_thread_range(int64_t p0, int64_t total, const uint32_t* sk,
                                                       const double* sval, const uint8_t* snn) {
  SegAcc<NC> acc = seg_identity<NC>();
  uint32_t prev = p0 > 0 && p0 <= total ? sk[p0 - 1] : 0xFFFFFFFFu;
#pragma unroll
  for (int i = 0; i < kSegPer; i++) {
    const int64_t p = p0 + i;
    if (p >= total) break;
    const uint32_t k = sk[p];
    const uint8_t m = snn[p];
    const bool head = p == 0 || k != prev;
    prev = k;
    if (head) acc = seg_identity<NC>(), acc.flag = 1;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      acc.s[c] = dd_add(acc.s[c], DD{sval[c * total + p], 0.0});
      acc.nn[c] += (m >> c) & 1;
    }
  }
  return acc;
}

// block-wide exclusive segmented prefix of the threads' ranges (+ carry-in);
// returns this thread's exclusive prefix, *tile_total the block's inclusive total
template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_block_exclusive(const SegAcc<NC>& mine, const SegAcc<NC>& carry,
                                                          SegAcc<NC>* wagg, SegAcc<NC>* tile_total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const SegAcc<NC> inc = seg_wave_scan(mine, lane);
  if (lane == 63) wagg[w] = inc;
  __syncthreads();
  SegAcc<NC> pre = carry;
  for (int k = 0; k < w; k++) pre = seg_combine(pre, wagg[k]);
  const SegAcc<NC> ex_w = seg_shfl_up(inc, 1);
  const SegAcc<NC> ex = lane == 0 ? pre : seg_combine(pre, ex_w);
  if (tile_total) {
    SegAcc<NC> t = carry;
    for (int k = 0; k < kBlock / 64; k++) t = seg_combine(t, wagg[k]);
    *tile_total = t;
  }
  return ex;
}

// phase 1: per-tile segmented totals
template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_tiles(int64_t total, const uint32_t* sk, const double* sval,
                                                      const uint8_t* snn, SegAcc<NC>* tagg) {
  __shared__ SegAcc<NC> wagg[kBlock / 64];
  const int64_t p0 = (int64_t)blockIdx.x * kSegTile + (int64_t)threadIdx.x * kSegPer;
  const SegAcc<NC> mine = seg_thread_range<NC>(p0, total, sk, sval, snn);
  SegAcc<NC> tot;
  seg_block_exclusive<NC>(mine, seg_identity<NC>(), wagg, &tot);
  if (threadIdx.x == 0) tagg[blockIdx.x] = tot;
}

// phase 2: exclusive segmented prefix over the tile totals (one workgroup;
// each thread folds a contiguous run of tiles)
template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_tilescan(SegAcc<NC>* tagg, int64_t nt) {
  __shared__ SegAcc<NC> wagg[kBlock / 64];
  const int64_t per = (nt + kBlock - 1) / kBlock;
  const int64_t t0 = (int64_t)threadIdx.x * per;
  const int64_t t1 = t0 + per < nt ? t0 + per : nt;
  SegAcc<NC> mine = seg_identity<NC>();
  for (int64_t t = t0; t < t1; t++) mine = seg_combine(mine, tagg[t]);
  SegAcc<NC> run = seg_block_exclusive<NC>(mine, seg_identity<NC>(), wagg, nullptr);
  for (int64_t t = t0; t < t1; t++) {
    const SegAcc<NC> v = tagg[t];
    tagg[t] = run;
    run = seg_combine(run, v);
  }
}

// phase 3: inclusive segmented prefix at every position (S, NN)
template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_apply(int64_t total, const uint32_t* sk, const double* sval,
                                                      const uint8_t* snn, const SegAcc<NC>* tcarry, DD* S,
                                                      int32_t* NN) {
  __shared__ SegAcc<NC> wagg[kBlock / 64];
  const int64_t p0 = (int64_t)blockIdx.x * kSegTile + (int64_t)threadIdx.x * kSegPer;
  const SegAcc<NC> mine = seg_thread_range<NC>(p0, total, sk, sval, snn);
  SegAcc<NC> run = seg_block_exclusive<NC>(mine, tcarry[blockIdx.x], wagg, nullptr);
  uint32_t prev = p0 > 0 && p0 <= total ? sk[p0 - 1] : 0xFFFFFFFFu;
#pragma unroll
  for (int i = 0; i < kSegPer; i++) {
    const int64_t p = p0 + i;
    if (p >= total) break;
    const uint32_t k = sk[p];
    const uint8_t m = snn[p];
    if (p == 0 || k != prev) run = seg_identity<NC>(), run.flag = 1;
    prev = k;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      run.s[c] = dd_add(run.s[c], DD{sval[c * total + p], 0.0});
      run.nn[c] += (m >> c) & 1;
      S[c * total + p] = run.s[c];
      NN[c * total + p] = run.nn[c];
    }
  }
}

// LDS-staged variants of phases 1 and 3 (NC <= 2): the tile's keys, operand
// bits and values are loaded coalesced into LDS, every thread folds its
// kSegPer consecutive positions from there, and phase 3 stages S / NN in LDS
// for coalesced stores -- the per-thread strided global accesses of the plain
// kernels touch kSegPer times more cache lines per wave instruction.
template <int NC>
struct SegTileLds {
  uint32_t k[kSegTile + 1];   // k[0]: the key before the tile
  uint8_t m[kSegTile];
  double v[NC][kSegTile];     // operands, then S.hi
  double lo[NC][kSegTile];    // S.lo (phase 3)
  int32_t nn[NC][kSegTile];   // NN (phase 3)
};

template <int NC>
__device__ __forceinline__ int seg_stage_tile(SegTileLds<NC>& L, int64_t t0, int64_t total, const uint32_t* sk,
                                              const double* sval, const uint8_t* snn) {
  const int nt = (int)(total - t0 < kSegTile ? total - t0 : kSegTile);
  for (int i = threadIdx.x; i < nt; i += kBlock) {
    L.k[i + 1] = sk[t0 + i];
    L.m[i] = snn[t0 + i];
#pragma unroll
    for (int c = 0; c < NC; c++) L.v[c][i] = sval[c * total + t0 + i];
  }
  if (threadIdx.x == 0) L.k[0] = t0 > 0 ? sk[t0 - 1] : 0xFFFFFFFFu;
  __syncthreads();
  return nt;
}

template <int NC>
__device__ __forceinline__ SegAcc<NC> seg_lds_range(const SegTileLds<NC>& L, int64_t t0, int nt) {
  SegAcc<NC> acc = seg_identity<NC>();
  const int i0 = threadIdx.x * kSegPer;
#pragma unroll
  for (int i = 0; i < kSegPer; i++) {
    const int li = i0 + i;
    if (li >= nt) break;
    const uint32_t k = L.k[li + 1];
    if (t0 + li == 0 || k != L.k[li]) acc = seg_identity<NC>(), acc.flag = 1;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      acc.s[c] = dd_add(acc.s[c], DD{L.v[c][li], 0.0});
      acc.nn[c] += (L.m[li] >> c) & 1;
    }
  }
  return acc;
}

template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_tiles_lds(int64_t total, const uint32_t* sk, const double* sval,
                                                          const uint8_t* snn, SegAcc<NC>* tagg) {
  __shared__ SegAcc<NC> wagg[kBlock / 64];
  __shared__ SegTileLds<NC> L;
  const int64_t t0 = (int64_t)blockIdx.x * kSegTile;
  const int nt = seg_stage_tile<NC>(L, t0, total, sk, sval, snn);
  const SegAcc<NC> mine = seg_lds_range<NC>(L, t0, nt);
  SegAcc<NC> tot;
  seg_block_exclusive<NC>(mine, seg_identity<NC>(), wagg, &tot);
  if (threadIdx.x == 0) tagg[blockIdx.x] = tot;
}

template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_apply_lds(int64_t total, const uint32_t* sk, const double* sval,
                                                          const uint8_t* snn, const SegAcc<NC>* tcarry, DD* S,
                                                          int32_t* NN) {
  __shared__ SegAcc<NC> wagg[kBlock / 64];
  __shared__ SegTileLds<NC> L;
  const int64_t t0 = (int64_t)blockIdx.x * kSegTile;
  const int nt = seg_stage_tile<NC>(L, t0, total, sk, sval, snn);
  const SegAcc<NC> mine = seg_lds_range<NC>(L, t0, nt);
  SegAcc<NC> run = seg_block_exclusive<NC>(mine, tcarry[blockIdx.x], wagg, nullptr);
  const int i0 = threadIdx.x * kSegPer;
#pragma unroll
  for (int i = 0; i < kSegPer; i++) {
    const int li = i0 + i;
    if (li >= nt) break;
    if (t0 + li == 0 || L.k[li + 1] != L.k[li]) run = seg_identity<NC>(), run.flag = 1;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      run.s[c] = dd_add(run.s[c], DD{L.v[c][li], 0.0});
      run.nn[c] += (L.m[li] >> c) & 1;
      L.v[c][li] = run.s[c].hi;   // each position is read before it is overwritten, by its own thread
      L.lo[c][li] = run.s[c].lo;
      L.nn[c][li] = run.nn[c];
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nt; i += kBlock) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      S[c * total + t0 + i] = DD{L.v[c][i], L.lo[c][i]};
      NN[c * total + t0 + i] = L.nn[c][i];
    }
  }
}

// smallest q in [0, p] with pred(q), where pred holds on a suffix ending at p
template <class Pred>
__device__ __forceinline__ int64_t gallop_first(int64_t p, Pred pred) {
  int64_t in = p, out = -1, step = 1;
  for (;;) {
    const int64_t q = p - step;
    if (q < 0 || !pred(q)) { out = q < 0 ? -1 : q; break; }
    in = q;
    step <<= 1;
  }
  while (in - out > 1) {
    const int64_t mid = out + ((in - out) >> 1);
    if (pred(mid)) in = mid;
    else out = mid;
  }
  return in;
}

// phase 4: window aggregates at the last add of every (group, call) run ->
// one packed emission record at the run's first item (k_emit<true> reads it
// there: last item, null mask, one 8-byte value per aggregator with avg
// already divided), so a run costs one contiguous scattered write; the group
// tables get the window state after the push at every segment end
struct RunRecHdr {
  uint32_t last;   // item of the run's last add (the emitted event)
  uint32_t nul;    // bit j: aggregator j is null
};
__host__ __device__ constexpr int64_t run_rec_words(int nagg) { return 1 + nagg; }

template <int NC>
__global__ __launch_bounds__(kBlock) void k_seg_emit(const SegArgs* __restrict__ ap, const uint32_t* sk,
                                                     const uint32_t* sp, const uint32_t* se, const int32_t* scall,
                                                     const DD* S, const int32_t* NN, const uint8_t* snn,
                                                     uint64_t* rec, uint8_t* first) {
  const SegArgs& a = *ap;
  const int64_t total = a.total;
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < total; p = total) {
    const uint32_t g = sk[p];
    const uint32_t x = sp[p];
    const bool seg_end = p + 1 == total || sk[p + 1] != g;
    const int32_t call = scall[p];
    const bool run_end = (int64_t)x >= a.C && (seg_end || scall[p + 1] != call);
    if (!seg_end && !run_end) continue;
    auto window = [&](uint32_t thr, int64_t& k, int64_t& kin) {
      // first position of the segment still in the window (expiry after thr)
      k = gallop_first(p, [&](int64_t q) { return sk[q] == g && se[q] > thr; });
      kin = k - 1 >= 0 && sk[k - 1] == g ? k - 1 : -1;   // prefix before the window, in this segment
    };
    auto chan_val = [&](int c, int64_t kin, int32_t& nnw) -> double {
      const DD sp_ = S[c * total + p];
      const DD sk_ = kin >= 0 ? S[c * total + kin] : DD{0.0, 0.0};
      nnw = NN[c * total + p] - (kin >= 0 ? NN[c * total + kin] : 0);
      return dd_diff(sp_, sk_);
    };
    if (seg_end) {   // window contents after the push (items never expired: e == kInf)
      int64_t k, kin;
      window((uint32_t)(total - 1), k, kin);
      for (int j = 0; j < a.nagg; j++) {
        const int c = a.chan[j];
        int32_t nnw = 0;
        const double v = c >= 0 ? chan_val(c, kin, nnw) : 0.0;
        a.dsum[j * a.nkeys + g] = nnw ? v : 0.0;
        a.cnt[j * a.nkeys + g] = c >= 0 ? (int64_t)nnw : p - k + 1;
      }
    }
    if (!run_end) continue;
    int64_t k, kin;
    window(x, k, kin);
    const int64_t rs = gallop_first(p, [&](int64_t q) { return sk[q] == g && scall[q] == call; });
    const uint32_t xf = sp[rs];
    uint64_t vals[kMaxAggs];
    uint32_t nul = 0;
    for (int j = 0; j < a.nagg; j++) {
      const int c = a.chan[j];
      uint64_t ob = 0;
      bool on = false;
      if (a.kind[j] == SHD_AGG_COUNT) {
        ob = (uint64_t)(p - k + 1);
      } else {
        int32_t nnw = 0;
        const double v = chan_val(c, kin, nnw);
        if (a.kind[j] == SHD_AGG_SUM) {
          // a null operand leaves the sum (null once nothing is left; float sums: null);
          // the operand's null bit travels with the sorted position (channel c)
          const bool xn = ((snn[p] >> c) & 1u) == 0;
          on = xn && !(a.type[j] == SHD_T_DOUBLE && nnw != 0);
          ob = on ? 0ull : p_f64(v);
        } else {
          // avg = value / count (AvgAttributeAggregatorExecutor: value / count as double)
          on = nnw == 0;
          ob = on ? 0ull : p_f64(__ddiv_rn(v, (double)nnw));
        }
      }
      vals[j] = ob;
      nul |= on ? 1u << j : 0u;
    }
    uint64_t* r = rec + (int64_t)xf * run_rec_words(a.nagg);
    r[0] = (uint64_t)x | ((uint64_t)nul << 32);
    for (int j = 0; j < a.nagg; j++) r[1 + j] = vals[j];
    first[xf] = 1;
  }
}

// ---------------------------------------------------------------- call windows
// Window aggregates per InputHandler call, without a global group sort (group
// by, windows no longer than a few calls -- config W2-length).  The rows a call
// emits are its groups' states after their last add of the call
// (QuerySelector.processInBatchGroupBy, QuerySelector.java:315-373); group g's
// state after item x is the set of its items q <= x that have not expired by
// x (e[q] > x; LengthWindowProcessor / TimeWindowProcessor expire in FIFO
// order before each add, so e is non-decreasing and every item of the call
// sees a window inside [lb, x] with lb = first q with e[q] > the call's first
// item).  One workgroup per call:
//   1. the call's group ids go into an LDS hash table (first / last item of
//      each group in the call);
//   2. every item q of the region [lb, call end) whose group is in the table
//      and lies in that group's window (q <= x_g, e[q] > x_g) is counted and
//      listed under its group;
//   3. one thread per group folds its listed items (double-double sums per
//      channel, non-null counts) into the run record k_emit reads -- the same
//      record k_seg_emit writes, at the run's first item.
// The region is read from L2 by ~(L + call items) / call items neighbouring
// workgroups; nothing is sorted in HBM.  Sums in double-double: within 1e-9
// relative of the reference's running `sum += v; sum -= v`
// (SumAttributeAggregatorExecutor.java:184-198), like the segmented scans.
constexpr int kCwCall = 1024;          // items (events) per call
constexpr uint32_t kCwEmpty = 0xFFFFFFFFu;

struct CwArgs {
  int nch;
  int ch_agg[kMaxChan];
  int ch_type[kMaxChan];
  int nagg;
  int kind[kMaxAggs];
  int type[kMaxAggs];
  int chan[kMaxAggs];
  int64_t cap;
  int64_t C;
  int64_t total;
  int64_t wlen;            // length window: e[q] = q + wlen (kInf past the items)
  const uint64_t* ikey;
  const uint32_t* e;
  const uint64_t* iargv;
  const uint8_t* iargn;
  const uint32_t* citem;   // [ncalls + 1]: first item of each call (absolute)
  const uint32_t* clb;     // [ncalls]: first item of the call's region
  // group tables after the push (k_cw_gtables)
  double* dsum;
  int64_t* cnt;
  int64_t nkeys;
  // direct emission (k_cw<.., EMIT>): k_emit's inputs
  ColSet cs;
  DExprSet es;
  DExpr outs[kMaxCols];
  int32_t okind[kMaxCols];
  int32_t oarg[kMaxCols];
  int nout;
  const int32_t* ievrow;
  int64_t row0, chunk0, seq0;
  int64_t* o_chunk;
  int32_t* o_type;
  int64_t* o_ts;
  uint64_t* o_vals;
  uint8_t* o_nul;
  int64_t* o_seq;
  int32_t* o_sidx;
  uint64_t* status;     // [ncalls] look-back words (zeroed before the launch)
  uint64_t* nrows;      // rows of the push (written by the last call)
};

__device__ __forceinline__ double cw_operand(const CwArgs& a, int c, int64_t q, bool& nul) {
  const int g = a.ch_agg[c];
  const uint64_t b = a.iargv[(int64_t)g * a.cap + q];
  nul = a.iargn[(int64_t)g * a.cap + q] != 0;
  switch (a.ch_type[c]) {   // Number.doubleValue() of the operand
    case SHD_T_INT: return (double)v_i32(b);
    case SHD_T_LONG: return (double)(int64_t)b;
    case SHD_T_FLOAT: return (double)v_f32(b);
    default: return v_f64(b);
  }
}

// first item of every call (from the event -> item offsets of k_filter's scan)
__global__ void k_cw_citem(const int64_t* __restrict__ offs, const uint32_t* __restrict__ off, int64_t n, int64_t m,
                           int64_t C, int ncalls, uint32_t* __restrict__ citem) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c <= ncalls; c += gridDim.x * blockDim.x) {
    const int64_t ev = offs[c];
    citem[c] = (uint32_t)(C + (ev < n ? (int64_t)off[ev] : m));
  }
}

// first item of each call's region (binary search over the non-decreasing e)
// and the largest call / region, for the host's choice of path
// (wlen > 0: a length window, e[q] = q + wlen)
__global__ void k_cw_regions(const uint32_t* __restrict__ e, int64_t wlen, const uint32_t* __restrict__ citem,
                             int ncalls, uint32_t* __restrict__ clb, uint32_t* __restrict__ maxes) {
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < ncalls; c += gridDim.x * blockDim.x) {
    const uint32_t s = citem[c], t = citem[c + 1];
    uint32_t lo = 0, hi = s;   // first q in [0, s] with e[q] > s (q = s qualifies: e[s] > s)
    if (wlen > 0) {
      lo = (int64_t)s + 1 > wlen ? (uint32_t)((int64_t)s + 1 - wlen) : 0u;
    } else {
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (e[mid] > s) hi = mid;
        else lo = mid + 1;
      }
    }
    clb[c] = lo;
    if (t - s > __hip_atomic_load(&maxes[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&maxes[0], t - s);
    if (t - lo > __hip_atomic_load(&maxes[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(&maxes[1], t - lo);
  }
}

// block-wide exclusive prefix of n <= CAP values in LDS (in place)
template <int CAP>
__device__ __forceinline__ void cw_block_exclusive(uint32_t* v, int n, uint32_t* wsum) {
  constexpr int per = CAP / kBlock;
  uint32_t x[per], run = 0;
  for (int j = 0; j < per; j++) {
    const int i = threadIdx.x * per + j;
    x[j] = i < n ? v[i] : 0u;
    run += x[j];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t inc = run;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  uint32_t pre = inc - run;
  for (int k = 0; k < w; k++) pre += wsum[k];
  for (int j = 0; j < per; j++) {
    const int i = threadIdx.x * per + j;
    if (i < n) v[i] = pre;
    pre += x[j];
  }
  __syncthreads();
}

// One (call, group) row: the group's window items (list[l0, l0 + n_in),
// region-relative) folded per channel in double-double, the aggregators'
// values after item x (k_seg_emit's formulas), the selector's outputs.
template <int NC>
__device__ __forceinline__ void cw_fold_emit(const CwArgs& a, int c, uint32_t lb, const uint16_t* list, uint32_t l0,
                                             uint32_t n_in, uint32_t x, int64_t row) {
  DD acc[NC];
  int32_t nn[NC];
#pragma unroll
  for (int ch = 0; ch < NC; ch++) {
    acc[ch] = DD{0.0, 0.0};
    nn[ch] = 0;
  }
  for (uint32_t j = 0; j < n_in; j++) {
    const int64_t q = (int64_t)lb + list[l0 + j];
#pragma unroll
    for (int ch = 0; ch < NC; ch++) {
      bool nul;
      const double v = cw_operand(a, ch, q, nul);
      if (!nul) {
        acc[ch] = dd_add(acc[ch], DD{v, 0.0});
        nn[ch]++;
      }
    }
  }
  uint64_t av[kMaxAggs];
  uint8_t an[kMaxAggs];
  for (int j = 0; j < a.nagg; j++) {
    const int ch = a.chan[j];
    uint64_t ob = 0;
    bool on = false;
    if (a.kind[j] == SHD_AGG_COUNT) {
      ob = (uint64_t)n_in;
    } else {
      double v = 0.0;
      int32_t nnw = 0;
#pragma unroll
      for (int k = 0; k < NC; k++)
        if (k == ch) {
          v = acc[k].hi;   // the double-double sum rounded (dd_add keeps hi = round(hi + lo))
          nnw = nn[k];
        }
      if (a.kind[j] == SHD_AGG_SUM) {
        // a null operand leaves the sum (null once nothing is left; float sums: null)
        bool xn;
        (void)cw_operand(a, ch, x, xn);
        on = xn && !(a.type[j] == SHD_T_DOUBLE && nnw != 0);
        ob = on ? 0ull : p_f64(v);
      } else {
        // avg = value / count (AvgAttributeAggregatorExecutor: value / count as double)
        on = nnw == 0;
        ob = on ? 0ull : p_f64(__ddiv_rn(v, (double)nnw));
      }
    }
    av[j] = ob;
    an[j] = on ? 1 : 0;
  }
  const int64_t ev = a.ievrow[x];
  RowCtx cx{&a.cs, ev, av, an};
  for (int k = 0; k < a.nout; k++) {
    Val v;
    if (a.okind[k] == 1) {
      v = col_load(a.cs, ev, a.oarg[k]);
    } else if (a.okind[k] == 2) {
      v.b = av[a.oarg[k]];
      v.null = an[a.oarg[k]];
    } else {
      v = eval_expr(a.es.ins + a.outs[k].off, a.outs[k].len, a.es.consts, cx);
    }
    a.o_vals[row * a.nout + k] = v.b;
    a.o_nul[row * a.nout + k] = (uint8_t)v.null;
  }
  a.o_ts[row] = a.cs.ts[ev];
  a.o_type[row] = 0;
  a.o_seq[row] = a.seq0 + ev;   // the group's last event of the call
  a.o_chunk[row] = a.chunk0 + c;
  a.o_sidx[row] = 0;
}

// Direct-mapped variant for small dense group ids (g < GCAP, config W2's
// symbols): per-group LDS arrays indexed by the id -- no hash table -- and the
// call's row base from k_cw_count + a scan instead of the look-back.
// k_cw_count: distinct groups of every call (an LDS bitmap per call).
template <int GCAP>
__global__ __launch_bounds__(kBlock) void k_cw_count(const CwArgs* __restrict__ ap, int ncalls, uint32_t* cnt) {
  const CwArgs& a = *ap;
  __shared__ uint32_t bits[GCAP / 32];
  __shared__ uint32_t wsum[kBlock / 64];
  const int c = blockIdx.x;
  if (c >= ncalls) return;
  const uint32_t s = a.citem[c], t = a.citem[c + 1];
  for (int i = threadIdx.x; i < GCAP / 32; i += kBlock) bits[i] = 0;
  __syncthreads();
  for (uint32_t q = s + threadIdx.x; q < t; q += kBlock) {
    const uint32_t g = (uint32_t)a.ikey[q];
    atomicOr(&bits[g >> 5], 1u << (g & 31));
  }
  __syncthreads();
  uint32_t v = 0;
  for (int i = threadIdx.x; i < GCAP / 32; i += kBlock) v += __popc(bits[i]);
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int k = 0; k < kBlock / 64; k++) tot += wsum[k];
    cnt[c] = tot;
  }
}

template <int NC, int RC, int CALLCAP, int GCAP, bool LEN>
__device__ __forceinline__ void cw_direct_call(const CwArgs& a, const int c, int ncalls,
                                               const uint32_t* __restrict__ rbase) {
  constexpr bool kStage = RC <= 2048;
  constexpr int kExpN = (kStage && !LEN) ? RC : 1;
  __shared__ uint32_t sfirst[GCAP], slast[GCAP], scnt[GCAP];
  __shared__ uint16_t qslot[RC];
  // staged group ids; after the region pass, the window lists (u16)
  __shared__ uint32_t rkey[kStage ? RC : (RC + 1) / 2];
  __shared__ uint32_t rexp[kExpN];
  __shared__ uint32_t srank[CALLCAP];   // first-seen rank of the call's items
  __shared__ uint32_t wsum[kBlock / 64];
  uint16_t* list = reinterpret_cast<uint16_t*>(rkey);
  uint32_t* soff = scnt;                // list offsets, in place of the counts (kept in registers below)
  if (c >= ncalls) return;
  const uint32_t s = a.citem[c], t = a.citem[c + 1];
  if (s == t) return;
  // (a length window: the region starts L - 1 items before the call)
  const uint32_t lb = LEN ? ((int64_t)s + 1 > a.wlen ? (uint32_t)((int64_t)s + 1 - a.wlen) : 0u) : a.clb[c];
  const int nr = (int)(t - lb);
  const int rs = (int)(s - lb);
  for (int g = threadIdx.x; g < GCAP; g += kBlock) {
    sfirst[g] = 0xFFFFFFFFu;
    slast[g] = 0;
    scnt[g] = 0;
  }
  if (kStage)
    for (int r = threadIdx.x; r < nr; r += kBlock) {
      rkey[r] = (uint32_t)a.ikey[lb + r];
      if (!LEN) rexp[r] = a.e[lb + r];
    }
  __syncthreads();
  auto key_at = [&](int r) -> uint32_t { return kStage ? rkey[r] : (uint32_t)a.ikey[lb + r]; };
  auto exp_of = [&](int r) -> uint32_t {
    const uint32_t q = lb + r;
    if (LEN) return (int64_t)q + a.wlen < a.total ? (uint32_t)(q + a.wlen) : kInf;
    return kStage ? rexp[r] : a.e[q];
  };
  for (int r = rs + threadIdx.x; r < nr; r += kBlock) {
    const uint32_t g = key_at(r);
    atomicMin(&sfirst[g], lb + r);
    atomicMax(&slast[g], lb + r);
  }
  __syncthreads();
  // region items inside their group's window; first items of the call's groups
  for (int r = threadIdx.x; r < nr; r += kBlock) {
    const uint32_t q = lb + r;
    const uint32_t g = key_at(r);
    uint16_t sl = 0xFFFF;
    const uint32_t x = slast[g];
    if (sfirst[g] != 0xFFFFFFFFu && q <= x && exp_of(r) > x) {
      sl = (uint16_t)g;
      atomicAdd(&scnt[g], 1u);
    }
    qslot[r] = sl;
    if (r >= rs) srank[r - rs] = sfirst[g] == q ? 1u : 0u;
  }
  __syncthreads();
  // the counts of the call's groups, kept by the thread of the group's first item
  uint32_t my_n[CALLCAP / kBlock];
  for (int k = 0; k < CALLCAP / kBlock; k++) {
    const int r = rs + threadIdx.x + k * kBlock;
    my_n[k] = r < nr && srank[r - rs] ? scnt[key_at(r)] : 0u;
  }
  __syncthreads();
  cw_block_exclusive<GCAP>(soff, GCAP, wsum);   // scnt -> list offsets
  cw_block_exclusive<CALLCAP>(srank, nr - rs, wsum);
  // (after the offsets: the group ids are still staged, the lists overwrite them next)
  uint32_t my_g[CALLCAP / kBlock];
  for (int k = 0; k < CALLCAP / kBlock; k++) {
    const int r = rs + threadIdx.x + k * kBlock;
    my_g[k] = r < nr ? key_at(r) : 0u;
  }
  __syncthreads();
  for (int r = threadIdx.x; r < nr; r += kBlock) {
    const uint16_t g = qslot[r];
    if (g != 0xFFFF) list[atomicAdd(&soff[g], 1u)] = (uint16_t)r;
  }
  __syncthreads();
  const int64_t base = a.row0 + (int64_t)rbase[c];
  for (int k = 0; k < CALLCAP / kBlock; k++) {
    const int r = rs + threadIdx.x + k * kBlock;
    if (r >= nr || !my_n[k]) continue;
    const uint32_t g = my_g[k];
    // soff[g] now ends the group's list
    cw_fold_emit<NC>(a, c, lb, list, soff[g] - my_n[k], my_n[k], slast[g], base + srank[r - rs]);
  }
}

template <int NC, int RC, int CALLCAP, int GCAP, bool LEN>
__global__ __launch_bounds__(kBlock) void k_cw_direct(const CwArgs* __restrict__ ap, int ncalls,
                                                      const uint32_t* __restrict__ rbase) {
  cw_direct_call<NC, RC, CALLCAP, GCAP, LEN>(*ap, blockIdx.x, ncalls, rbase);
}

// Every member of a window group in one launch (the members' CwArgs `stride`
// bytes apart): the workgroups of one call -- one per member, its region a
// suffix of the longest member's -- are dealt to the same XCD back to back
// (workgroups go round-robin over the 8 XCDs), so the call's items are read
// from HBM about once and from that XCD's L2 by the other members.
template <int NC, int RC, int CALLCAP, int GCAP, bool LEN>
__global__ __launch_bounds__(kBlock) void k_cw_direct_multi(const char* __restrict__ aps, int64_t stride, int nmem,
                                                            int ncalls, const uint32_t* __restrict__ rbase) {
  const int b = blockIdx.x, x = b & 7, i = b >> 3;
  const int m = i % nmem, c = (i / nmem) * 8 + x;
  cw_direct_call<NC, RC, CALLCAP, GCAP, LEN>(*reinterpret_cast<const CwArgs*>(aps + (int64_t)m * stride), c, ncalls,
                                             rbase);
}

// The call's rows are written here, in first-seen order, at row0 + the rows
// of all earlier calls (single-pass decoupled look-back over the calls: each
// workgroup publishes its row count as soon as its groups are known).
// CALLCAP: items per call (hash table of 2 * CALLCAP slots); RC: region items.
// LDS: 38 KB at (512, 2048) -- four workgroups per CU.
template <int NC, int RC, int CALLCAP, bool LEN>
__global__ __launch_bounds__(kBlock) void k_cw(const CwArgs* __restrict__ ap, int ncalls) {
  // small regions are staged in LDS (group id, and the expiry unless a length
  // window gives it as q + L; one coalesced pass); larger ones are read from
  // global memory (L2)
  constexpr bool kStage = RC <= 2048;
  constexpr int kStageN = kStage ? RC : 1;
  constexpr int kExpN = (kStage && !LEN) ? RC : 1;
  constexpr int kHash = 2 * CALLCAP;
  const CwArgs& a = *ap;
  __shared__ uint32_t hkey[kHash];
  __shared__ uint16_t hidx[kHash];
  // per group of the call: first / last item, items in its window, list offset
  __shared__ uint32_t sfirst[CALLCAP], slast[CALLCAP], scnt[CALLCAP], soff[CALLCAP];
  __shared__ uint16_t qslot[RC];
  // staged group ids; after the region pass, the window lists (u16)
  __shared__ uint32_t rkey[kStage ? RC : (RC + 1) / 2];
  __shared__ uint32_t rexp[kExpN];
  __shared__ uint32_t srank[CALLCAP];   // first-seen rank of the call's items
  __shared__ uint32_t nslots;
  __shared__ uint64_t sbase;
  __shared__ uint32_t wsum[kBlock / 64];
  uint16_t* list = reinterpret_cast<uint16_t*>(rkey);
  const int c = blockIdx.x;
  if (c >= ncalls) return;
  const uint32_t s = a.citem[c], t = a.citem[c + 1];
  const uint32_t lb = s == t ? s : (LEN ? ((int64_t)s + 1 > a.wlen ? (uint32_t)((int64_t)s + 1 - a.wlen) : 0u) : a.clb[c]);
  const int nr = (int)(t - lb);
  for (int h = threadIdx.x; h < kHash; h += kBlock) hkey[h] = kCwEmpty;
  if (threadIdx.x == 0) nslots = 0;
  if (kStage)
    for (int r = threadIdx.x; r < nr; r += kBlock) {
      rkey[r] = (uint32_t)a.ikey[lb + r];
      if (!LEN) rexp[r] = a.e[lb + r];
    }
  __syncthreads();
  auto exp_of = [&](int r) -> uint32_t {
    const uint32_t q = lb + r;
    if (LEN) return (int64_t)q + a.wlen < a.total ? (uint32_t)(q + a.wlen) : kInf;
    return kStage ? rexp[r] : a.e[q];
  };
  auto key_at = [&](int r) -> uint32_t { return kStage ? rkey[r] : (uint32_t)a.ikey[lb + r]; };
  auto hash = [&](uint32_t k) -> uint32_t { return key_bucket_mix(k) & (kHash - 1); };
  // 1. the call's groups: the thread that claims a hash slot numbers it
  const int rs = (int)(s - lb);
  for (int r = rs + threadIdx.x; r < nr; r += kBlock) {
    const uint32_t k = key_at(r);
    uint32_t h = hash(k);
    for (;;) {
      const uint32_t old = atomicCAS(&hkey[h], kCwEmpty, k);
      if (old == kCwEmpty) {
        const uint32_t i = atomicAdd(&nslots, 1u);
        hidx[h] = (uint16_t)i;
        sfirst[i] = 0xFFFFFFFFu;
        slast[i] = 0;
        scnt[i] = 0;
        break;
      }
      if (old == k) break;
      h = (h + 1) & (kHash - 1);
    }
  }
  __syncthreads();
  constexpr uint64_t kAgg = 1ull << 62, kInc = 2ull << 62, kVal = (1ull << 62) - 1;
  if (threadIdx.x == 0) {
    // publish this call's row count at once; the look-back for the earlier
    // calls' rows waits until the fold needs it
    const uint64_t local = nslots;
    atomicExch((unsigned long long*)&a.status[c], (unsigned long long)((c == 0 ? kInc : kAgg) | local));
  }
  // one wave reads 64 predecessors' words per step: the nearest inclusive
  // prefix ends the walk, aggregates before it add up
  auto look_back = [&]() {
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    const uint64_t local = nslots;
    uint64_t base = 0;
    for (int top = c - 1; top >= 0;) {
      const int j = top - lane;
      uint64_t st = j >= 0 ? cw_status_load(&a.status[j]) : kInc;
      if (__any((st >> 62) == 0)) {   // an earlier, running workgroup has not published yet
        __builtin_amdgcn_s_sleep(4);
        continue;
      }
      const uint64_t incl = __ballot((st >> 62) == 2);
      const int stop = incl ? __ffsll((long long)incl) - 1 : 64;   // nearest inclusive word
      uint64_t v = lane <= stop && j >= 0 ? (st & kVal) : 0ull;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      base += v;
      if (incl) break;
      top -= 64;
    }
    if (lane == 0) {
      if (c > 0) atomicExch((unsigned long long*)&a.status[c], (unsigned long long)(kInc | (base + local)));
      if (c == ncalls - 1) *a.nrows = base + local;
      sbase = base;
    }
  };
  // the look-back runs at once (short chains: every workgroup resolves its
  // prefix right after publishing its count)
  look_back();
  if (s == t) return;   // an empty call: its zero rows are published, the chain continues through it
  auto find = [&](uint32_t k) -> int {
    uint32_t h = hash(k);
    for (;;) {
      const uint32_t x = hkey[h];
      if (x == k) return hidx[h];
      if (x == kCwEmpty) return -1;
      h = (h + 1) & (kHash - 1);
    }
  };
  for (int r = rs + threadIdx.x; r < nr; r += kBlock) {
    const int i = find(key_at(r));
    atomicMin(&sfirst[i], lb + r);
    atomicMax(&slast[i], lb + r);
  }
  __syncthreads();
  // 2. region items inside their group's window
  for (int r = threadIdx.x; r < nr; r += kBlock) {
    const uint32_t q = lb + r;
    const int i = find(key_at(r));
    uint16_t sl = 0xFFFF;
    if (i >= 0) {
      const uint32_t x = slast[i];
      if (q <= x && exp_of(r) > x) {
        sl = (uint16_t)i;
        atomicAdd(&scnt[i], 1u);
      }
    }
    qslot[r] = sl;
  }
  __syncthreads();
  // first-seen order of the groups (LinkedHashMap insertion order): the rank
  // of each group's first item among the call's first items
  for (int r = threadIdx.x; r < nr - rs; r += kBlock) srank[r] = 0;
  for (int i = threadIdx.x; i < (int)nslots; i += kBlock) soff[i] = scnt[i];
  __syncthreads();
  for (int i = threadIdx.x; i < (int)nslots; i += kBlock) srank[sfirst[i] - s] = 1;
  cw_block_exclusive<CALLCAP>(soff, (int)nslots, wsum);
  cw_block_exclusive<CALLCAP>(srank, nr - rs, wsum);
  // lists: soff[i] advances to the end of group i's list
  for (int r = threadIdx.x; r < nr; r += kBlock) {
    const uint16_t i = qslot[r];
    if (i != 0xFFFF) list[atomicAdd(&soff[i], 1u)] = (uint16_t)r;
  }
  __syncthreads();
  // 3. one thread per group: fold the window, write the row
  for (int i = threadIdx.x; i < (int)nslots; i += kBlock) {
    const uint32_t xf = sfirst[i];
    cw_fold_emit<NC>(a, c, lb, list, soff[i] - scnt[i], scnt[i], slast[i],
                     a.row0 + (int64_t)sbase + srank[xf - s]);
  }
}

// group tables after the push: the groups of items [q0, q1) are reset (!ADD),
// or those items, if still in the window (never expired: e == kInf), add in
template <bool ADD>
__global__ __launch_bounds__(kBlock) void k_cw_gtables(const CwArgs* __restrict__ ap, int64_t q0, int64_t q1) {
  const CwArgs& a = *ap;
  for (int64_t q = q0 + (int64_t)blockIdx.x * kBlock + threadIdx.x; q < q1; q += (int64_t)gridDim.x * kBlock) {
    const uint32_t g = (uint32_t)a.ikey[q];
    for (int j = 0; j < a.nagg; j++) {
      const int64_t at = (int64_t)j * a.nkeys + g;
      if (!ADD) {
        a.dsum[at] = 0.0;
        a.cnt[at] = 0;
        continue;
      }
      if (a.wlen == 0 && a.e[q] != kInf) continue;   // (a length window: every item from X on stays)
      const int ch = a.chan[j];
      if (ch < 0) {
        atomicAdd((unsigned long long*)&a.cnt[at], 1ull);
        continue;
      }
      bool nul;
      const double v = cw_operand(a, ch, q, nul);
      if (nul) continue;
      atomicAdd(&a.dsum[at], v);
      atomicAdd((unsigned long long*)&a.cnt[at], 1ull);
    }
  }
}

// ---------------------------------------------------------------- chunked window walk
// Window aggregates without a global group sort (dense group ids, at most
// kWcMaxG groups).  The op stream of the push (item x added at position x;
// item i expired at position e[i], before that position's add -- the
// reference's LengthWindowProcessor / TimeWindowProcessor order) is cut into
// chunks of whole InputHandler calls (<= kWcItems adds; the carried items
// [0, C) form their own add-only chunks).  A chunk's ops are two contiguous
// item ranges: its adds and the items expiring at its positions (e is
// non-decreasing).
//   k_wc_delta: per chunk, the ops sorted by group in LDS (counting sort,
//     arrival order restored inside a group), folded per group -> the
//     chunk's change of every group's window state (sum per channel in
//     double-double, non-null count, item count);
//   k_wc_scan1..3: prefix over the chunks -> every group's state at the
//     start of every chunk (and after the push: the group tables);
//   k_wc_emit: per chunk again, each group folded from its start state; at
//     the last add of every (call, group) run the run record k_emit reads
//     (the same record k_seg_emit writes), written at the run's first item.
// A group's window state is a running sum of the items inside the window
// (the reference's `sum += v; sum -= v`, SumAttributeAggregatorExecutor.java
// :184-198) kept in double-double: within 1e-9 relative of the reference,
// like the segmented scans.
constexpr int kWcItems = 4096;          // adds per chunk (whole calls)
constexpr int kWcOps = 8192;            // adds + expires per chunk
constexpr int kWcMaxG = 2048;           // dense group ids [0, kWcMaxG)
constexpr int kWcThreads = 512;
constexpr int kWcSeg = 64;              // chunks per scan segment

template <int NC>
struct WcAcc {
  double s[NC];     // window sum per channel (double-double hi only in the table)
  int32_t nn[NC];   // non-null operands in the window
  int32_t cnt;      // items in the window
};

struct WcArgs {
  int64_t C, total;
  int G;
  int nagg;
  int kind[kMaxAggs];
  int type[kMaxAggs];
  int chan[kMaxAggs];
  const uint64_t* ikey;      // group id per item (dense)
  const uint32_t* e;         // expiry position per item (kInf: none)
  const int64_t* cp;         // chunk k: positions [cp[k], cp[k+1])
  const int64_t* ce;         // chunk k: expiring items [ce[k], ce[k+1])
  uint64_t* rec;             // run records (k_emit<true>)
  uint8_t* first;
  double* dsum;              // group tables [nagg][nkeys]: the window state after the push
  int64_t* gcnt;
  int64_t nkeys;
  unsigned int* flag;        // a chunk with more than kWcOps ops
};

// chunk item ranges: K_c carried chunks of kWcItems items, then one chunk per
// F calls (first item of a call: lower bound of its index in icall[C, total))
__global__ void k_wc_bounds(const WcArgs* __restrict__ ap, int kc, int K, int F, int ncalls, const int32_t* icall,
                            int64_t* cp, int64_t* ce) {
  const WcArgs& a = *ap;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k <= K; k += gridDim.x * blockDim.x) {
    int64_t p;
    if (k < kc) p = (int64_t)k * kWcItems;
    else if (k == K) p = a.total;
    else {
      const int c = (k - kc) * F;
      if (c >= ncalls) p = a.total;
      else {
        int64_t lo = a.C, hi = a.total;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if (icall[mid] >= c) hi = mid;
          else lo = mid + 1;
        }
        p = lo;
      }
    }
    if (k < kc && p > a.C) p = a.C;
    cp[k] = p;
    // first item expiring at or after position p
    int64_t lo = 0, hi = a.total;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)a.e[mid] >= p) hi = mid;
      else lo = mid + 1;
    }
    ce[k] = lo;
  }
}

// a chunk with more ops than fit in LDS -> flag (the host keeps the segmented scans)
__global__ void k_wc_check(const int64_t* cp, const int64_t* ce, int K, unsigned int* flag) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < K; k += gridDim.x * blockDim.x)
    if ((cp[k + 1] - cp[k]) + (ce[k + 1] - ce[k]) > kWcOps || cp[k + 1] < cp[k]) atomicOr(flag, 1u);
}

// Load chunk k's ops into LDS sorted by group (arrival order inside a group:
// position, expire before add, then item).  Returns the op count (0 and the
// flag set when it exceeds kWcOps).  sop: op codes (item | add << 31) in
// group order; gs: group starts [G + 1].
template <int NC>
__device__ int wc_load_sorted(const WcArgs& a, int k, uint32_t* op, uint32_t* ordk, uint16_t* grp, uint32_t* cnt,
                              uint32_t* gs, uint16_t* tmp, uint32_t* sop, uint32_t* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t P0 = a.cp[k], P1 = a.cp[k + 1], E0 = a.ce[k], E1 = a.ce[k + 1];
  const int na = (int)(P1 - P0), nx = (int)(E1 - E0);
  const int nops = na + nx;
  if (nops > kWcOps) {
    if (tid == 0) atomicOr(a.flag, 1u);
    return 0;
  }
  for (int g = tid; g < a.G; g += kWcThreads) cnt[g] = 0;
  __syncthreads();
  for (int i = tid; i < nops; i += kWcThreads) {
    uint32_t item, code, ord;
    if (i < nx) {   // expire of item E0 + i at position e[...]
      item = (uint32_t)(E0 + i);
      const int64_t pos = (int64_t)a.e[item];
      code = item;
      ord = ((uint32_t)(2 * (pos - P0)) << 14) | (uint32_t)i;
    } else {
      item = (uint32_t)(P0 + (i - nx));
      code = item | 0x80000000u;
      ord = ((uint32_t)(2 * (item - P0) + 1) << 14) | (uint32_t)(i - nx);
    }
    const uint32_t g = (uint32_t)a.ikey[item];
    op[i] = code;
    ordk[i] = ord;
    grp[i] = (uint16_t)g;
    tmp[i] = (uint16_t)atomicAdd(&cnt[g], 1u);
  }
  __syncthreads();
  // group starts: exclusive scan of cnt[0, G)
  {
    constexpr int kPer = kWcMaxG / kWcThreads;
    uint32_t c[kPer], sum = 0;
#pragma unroll
    for (int j = 0; j < kPer; j++) {
      const int g = tid * kPer + j;
      c[j] = g < a.G ? cnt[g] : 0u;
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
    for (int kk = 0; kk < w; kk++) pre += wsum[kk];
#pragma unroll
    for (int j = 0; j < kPer; j++) {
      const int g = tid * kPer + j;
      if (g < a.G) gs[g] = pre;
      pre += c[j];
    }
    if (tid == kWcThreads - 1) gs[a.G] = pre;
  }
  __syncthreads();
  // unordered placement, then the arrival rank inside the group
  for (int i = tid; i < nops; i += kWcThreads) sop[gs[grp[i]] + tmp[i]] = (uint32_t)i;
  __syncthreads();
  for (int i = tid; i < nops; i += kWcThreads) {
    const uint32_t g = grp[i];
    const int b0 = (int)gs[g], b1 = (int)gs[g + 1];
    const uint32_t my = ordk[i];
    int rank = 0;
    for (int y = b0; y < b1; y++) rank += ordk[sop[y]] < my ? 1 : 0;
    tmp[b0 + rank] = (uint16_t)i;   // tmp is free again: the group-ordered op indices
  }
  __syncthreads();
  return nops;
}

template <int NC>
__device__ __forceinline__ void wc_apply(const SegItem<NC>& it, bool add, DD (&s)[NC], int32_t (&nn)[NC], int32_t& cnt) {
  const uint32_t m = it.w >> 30;
#pragma unroll
  for (int c = 0; c < NC; c++) {
    if (!((m >> c) & 1u)) continue;
    s[c] = dd_add(s[c], DD{add ? it.v[c] : -it.v[c], 0.0});
    nn[c] += add ? 1 : -1;
  }
  cnt += add ? 1 : -1;
}

template <int NC>
__global__ __launch_bounds__(kWcThreads) void k_wc_delta(const WcArgs* __restrict__ ap, const SegItem<NC>* items,
                                                        WcAcc<NC>* table) {
  const WcArgs& a = *ap;
  __shared__ uint32_t op[kWcOps], ordk[kWcOps], sop[kWcOps];
  __shared__ uint16_t grp[kWcOps], tmp[kWcOps];
  __shared__ uint32_t cnt[kWcMaxG], gs[kWcMaxG + 1];
  __shared__ uint32_t wsum[kWcThreads / 64];
  const int k = blockIdx.x;
  const int nops = wc_load_sorted<NC>(a, k, op, ordk, grp, cnt, gs, tmp, sop, wsum);
  for (int g = threadIdx.x; g < a.G; g += kWcThreads) {
    DD s[NC];
    int32_t nn[NC];
    int32_t c = 0;
#pragma unroll
    for (int j = 0; j < NC; j++) {
      s[j] = DD{0.0, 0.0};
      nn[j] = 0;
    }
    if (nops) {
      for (int y = (int)gs[g]; y < (int)gs[g + 1]; y++) {
        const uint32_t code = op[tmp[y]];
        wc_apply<NC>(items[code & 0x7FFFFFFFu], (code >> 31) != 0, s, nn, c);
      }
    }
    WcAcc<NC> r;
#pragma unroll
    for (int j = 0; j < NC; j++) {
      r.s[j] = s[j].hi;
      r.nn[j] = nn[j];
    }
    r.cnt = c;
    table[(int64_t)k * a.G + g] = r;
  }
}

// prefix over the chunks: per (segment of kWcSeg chunks, group) totals; per
// group the segments' exclusive prefix (+ the state after the push -> the
// group tables); per (segment, group) the chunk-start states in place
template <int NC>
__global__ void k_wc_scan1(const WcArgs* __restrict__ ap, int K, const WcAcc<NC>* table, WcAcc<NC>* seg) {
  const WcArgs& a = *ap;
  const int nseg = (K + kWcSeg - 1) / kWcSeg;
  const int64_t nt = (int64_t)nseg * a.G;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (int64_t)gridDim.x * blockDim.x) {
    const int sg = (int)(t / a.G), g = (int)(t % a.G);
    DD s[NC];
    WcAcc<NC> r{};
#pragma unroll
    for (int j = 0; j < NC; j++) s[j] = DD{0.0, 0.0};
    const int k1 = min(K, (sg + 1) * kWcSeg);
    for (int k = sg * kWcSeg; k < k1; k++) {
      const WcAcc<NC> d = table[(int64_t)k * a.G + g];
#pragma unroll
      for (int j = 0; j < NC; j++) {
        s[j] = dd_add(s[j], DD{d.s[j], 0.0});
        r.nn[j] += d.nn[j];
      }
      r.cnt += d.cnt;
    }
#pragma unroll
    for (int j = 0; j < NC; j++) r.s[j] = s[j].hi;
    seg[t] = r;
  }
}

template <int NC>
__global__ void k_wc_scan2(const WcArgs* __restrict__ ap, int K, WcAcc<NC>* seg) {
  const WcArgs& a = *ap;
  const int nseg = (K + kWcSeg - 1) / kWcSeg;
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < a.G; g += gridDim.x * blockDim.x) {
    DD s[NC];
    int32_t nn[NC];
    int32_t c = 0;
#pragma unroll
    for (int j = 0; j < NC; j++) {
      s[j] = DD{0.0, 0.0};
      nn[j] = 0;
    }
    for (int sg = 0; sg < nseg; sg++) {
      WcAcc<NC>& x = seg[(int64_t)sg * a.G + g];
      const WcAcc<NC> d = x;
#pragma unroll
      for (int j = 0; j < NC; j++) {
        x.s[j] = s[j].hi;
        x.nn[j] = nn[j];
        s[j] = dd_add(s[j], DD{d.s[j], 0.0});
        nn[j] += d.nn[j];
      }
      x.cnt = c;
      c += d.cnt;
    }
    // the window state after the push -> group tables (as k_seg_emit's seg_end)
    for (int j = 0; j < a.nagg; j++) {
      const int ch = a.chan[j];
      const int32_t nnw = ch >= 0 ? nn[ch] : 0;
      a.dsum[j * a.nkeys + g] = (ch >= 0 && nnw) ? s[ch].hi : 0.0;
      a.gcnt[j * a.nkeys + g] = ch >= 0 ? (int64_t)nnw : (int64_t)c;
    }
  }
}

template <int NC>
__global__ void k_wc_scan3(const WcArgs* __restrict__ ap, int K, WcAcc<NC>* table, const WcAcc<NC>* seg) {
  const WcArgs& a = *ap;
  const int nseg = (K + kWcSeg - 1) / kWcSeg;
  const int64_t nt = (int64_t)nseg * a.G;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += (int64_t)gridDim.x * blockDim.x) {
    const int sg = (int)(t / a.G), g = (int)(t % a.G);
    const WcAcc<NC> b = seg[t];
    DD s[NC];
    int32_t nn[NC];
    int32_t c = b.cnt;
#pragma unroll
    for (int j = 0; j < NC; j++) {
      s[j] = DD{b.s[j], 0.0};
      nn[j] = b.nn[j];
    }
    const int k1 = min(K, (sg + 1) * kWcSeg);
    for (int k = sg * kWcSeg; k < k1; k++) {
      WcAcc<NC>& x = table[(int64_t)k * a.G + g];
      const WcAcc<NC> d = x;
#pragma unroll
      for (int j = 0; j < NC; j++) {
        x.s[j] = s[j].hi;
        x.nn[j] = nn[j];
        s[j] = dd_add(s[j], DD{d.s[j], 0.0});
        nn[j] += d.nn[j];
      }
      x.cnt = c;
      c += d.cnt;
    }
  }
}

template <int NC>
__global__ __launch_bounds__(kWcThreads) void k_wc_emit(const WcArgs* __restrict__ ap, const SegItem<NC>* items,
                                                       const WcAcc<NC>* table) {
  const WcArgs& a = *ap;
  __shared__ uint32_t op[kWcOps], ordk[kWcOps], sop[kWcOps];
  __shared__ uint16_t grp[kWcOps], tmp[kWcOps];
  __shared__ uint32_t cnt[kWcMaxG], gs[kWcMaxG + 1];
  __shared__ uint32_t wsum[kWcThreads / 64];
  const int k = blockIdx.x;
  const int nops = wc_load_sorted<NC>(a, k, op, ordk, grp, cnt, gs, tmp, sop, wsum);
  if (!nops) return;
  for (int g = threadIdx.x; g < a.G; g += kWcThreads) {
    const int y0 = (int)gs[g], y1 = (int)gs[g + 1];
    if (y0 == y1) continue;
    const WcAcc<NC> st = table[(int64_t)k * a.G + g];
    DD s[NC];
    int32_t nn[NC];
    int32_t c = st.cnt;
#pragma unroll
    for (int j = 0; j < NC; j++) {
      s[j] = DD{st.s[j], 0.0};
      nn[j] = st.nn[j];
    }
    // run ends, backwards: an add ends its (call, group) run unless the
    // group's next add has the same call (ordk: free after the sort)
    {
      uint32_t next_call = 0xFFFFFFFFu;
      for (int y = y1 - 1; y >= y0; y--) {
        const uint32_t i = tmp[y];
        const uint32_t code = op[i];
        if (!(code >> 31)) continue;
        const uint32_t call = items[code & 0x7FFFFFFFu].w & 0x3FFFFFFFu;
        ordk[i] = call != next_call ? 1u : 0u;
        next_call = call;
      }
    }
    int64_t xf = -1;      // first item of the current (call, group) run
    uint32_t rcall = 0;   // its call (+1)
    for (int y = y0; y < y1; y++) {
      const uint32_t code = op[tmp[y]];
      const uint32_t x = code & 0x7FFFFFFFu;
      const bool add = (code >> 31) != 0;
      const SegItem<NC> it = items[x];
      wc_apply<NC>(it, add, s, nn, c);
      if (!add || (int64_t)x < a.C) continue;
      const uint32_t call = it.w & 0x3FFFFFFFu;
      if (xf < 0 || call != rcall) {
        xf = x;
        rcall = call;
      }
      if (!ordk[tmp[y]]) continue;   // not the run's last add
      uint64_t vals[kMaxAggs];
      uint32_t nul = 0;
      for (int j = 0; j < a.nagg; j++) {
        const int ch = a.chan[j];
        uint64_t ob = 0;
        bool on = false;
        if (a.kind[j] == SHD_AGG_COUNT) {
          ob = (uint64_t)c;
        } else {
          const int32_t nnw = nn[ch];
          const double v = s[ch].hi;
          if (a.kind[j] == SHD_AGG_SUM) {
            const bool xn = (((it.w >> 30) >> ch) & 1u) == 0;
            on = xn && !(a.type[j] == SHD_T_DOUBLE && nnw != 0);
            ob = on ? 0ull : p_f64(v);
          } else {
            on = nnw == 0;
            ob = on ? 0ull : p_f64(__ddiv_rn(v, (double)nnw));
          }
        }
        vals[j] = ob;
        nul |= on ? 1u << j : 0u;
      }
      uint64_t* r = a.rec + xf * run_rec_words(a.nagg);
      r[0] = (uint64_t)x | ((uint64_t)nul << 32);
      for (int j = 0; j < a.nagg; j++) r[1 + j] = vals[j];
      a.first[xf] = 1;
      xf = -1;
    }
  }
}

__global__ void k_first_counts(const uint8_t* first, int64_t C, int64_t total, uint32_t* cnt) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total - C; t += (int64_t)gridDim.x * blockDim.x)
    cnt[t] = first[C + t] ? 1u : 0u;
}

struct EmitArgs {
  ColSet cs;
  DExprSet es;
  DExpr outs[kMaxCols];
  // single-instruction outputs decoded on the host: 1 = attribute load (arg =
  // attribute), 2 = aggregator (arg = index), 0 = the interpreter
  int32_t okind[kMaxCols];
  int32_t oarg[kMaxCols];
  int nout;
  int nagg;
  int kind[kMaxAggs];
  int64_t cap;
  int64_t C;
  int64_t row0;
  int64_t chunk0;
  int64_t seq0;
};

// REC: the run's values come from its packed record (segmented-scan mode)
template <bool REC>
__global__ __launch_bounds__(kBlock) void k_emit(const EmitArgs* __restrict__ ap, int64_t nnew, const uint32_t* fcnt, const uint32_t* foff,
                                                 const uint32_t* last_of, const int32_t* ievrow, const int32_t* call_of,
                                                 const uint64_t* resv, const uint8_t* resn, const int64_t* resc,
                                                 int64_t* o_chunk, int32_t* o_type, int64_t* o_ts, uint64_t* o_vals,
                                                 uint8_t* o_nul, int64_t* o_seq) {
  const EmitArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  const DExprSet es = a.es;
  const ColSet& cs = a.cs;
  for (int64_t t0 = (int64_t)blockIdx.x * kBlock + threadIdx.x; t0 < nnew; t0 = nnew) {
    if (!fcnt[t0]) continue;
    int64_t tf = a.C + t0;
    int64_t tl;
    uint64_t av[kMaxAggs];
    uint8_t an[kMaxAggs];
    if (REC) {
      const uint64_t* r = resv + tf * run_rec_words(a.nagg);
      const uint64_t h = r[0];
      tl = (int64_t)(uint32_t)h;
      for (int g = 0; g < a.nagg; g++) {
        av[g] = r[1 + g];
        an[g] = (uint8_t)((h >> (32 + g)) & 1u);
      }
    } else {
      tl = last_of[tf];
      for (int g = 0; g < a.nagg; g++) {
        av[g] = resv[g * a.cap + tl];
        an[g] = resn[g * a.cap + tl];
        // avg = value / count (AvgAttributeAggregatorExecutor: value / count as double)
        if (a.kind[g] == SHD_AGG_AVG && !an[g]) av[g] = p_f64(__ddiv_rn(v_f64(av[g]), (double)resc[g * a.cap + tl]));
      }
    }
    int64_t ev = ievrow[tl];
    RowCtx cx{&cs, ev, av, an};
    int64_t row = a.row0 + foff[t0];
    for (int c = 0; c < a.nout; c++) {
      Val v;
      if (a.okind[c] == 1) {
        v = col_load(cs, ev, a.oarg[c]);
      } else if (a.okind[c] == 2) {
        v.b = av[a.oarg[c]];
        v.null = an[a.oarg[c]];
      } else {
        v = eval_expr(es.ins + a.outs[c].off, a.outs[c].len, es.consts, cx);
      }
      o_vals[row * a.nout + c] = v.b;
      o_nul[row * a.nout + c] = (uint8_t)v.null;
    }
    o_ts[row] = cs.ts[ev];
    o_type[row] = 0;
    o_seq[row] = a.seq0 + ev;   // the group's last event of the call
    o_chunk[row] = a.chunk0 + call_of[ev];
  }
}

int plain_load_attr(const Plan& p, int e) {
  auto& code = p.exprs[e];
  if (code.size() == 1 && code[0].op == SHD_OP_LOAD) return code[0].c & 0xFFFF;
  return -1;
}

}  // namespace

struct SingleEngine : Engine {
  bool agg_mode = false;
  std::vector<int> filters;
  int wkind = 0;
  int64_t wparam = 0;
  bool partitioned = false;
  int key_expr = -1, key_col = -1, key_type = 0;
  // group by: up to kMaxGroupAttrs attributes; dense ids (one string / bool
  // attribute) or the device group dictionary (GDict) for every other key
  int ngk = 0;
  int gk_expr[kMaxGroupAttrs] = {}, gk_col[kMaxGroupAttrs] = {}, gk_type[kMaxGroupAttrs] = {};
  bool gdense = false;
  GroupDict gd;                      // group ids of non-dense keys
  DevBuf g_kw, g_kn, g_h;            // per new item: key words, null mask, hash
  std::vector<int> outs;
  std::vector<int> types;
  int nagg = 0;
  // per-batch scratch
  DevBuf d_offs, d_call_of, d_last_ts, d_now, d_flags, d_cnt, d_off, d_pkey, d_start, d_run, d_tot, d_scan, d_sort,
      d_pmax;
  PinnedBuf h_tot;
  // window items: carry [0, C) + new; double-buffered
  int64_t C = 0;
  int cur = 0;
  DevBuf ikey[2], its[2], iargv[2], iargn[2];
  int64_t icap[2] = {0, 0};
  DevBuf ievrow, icall, inow, e_exp, okey, oref, okey32, okey32_alt, oref_alt, heads, hoff, hlist, resv, resc, resn, first,
      last_of, fcnt, foff;
  // segmented-scan mode (default for count / sum(double|float) / avg)
  bool seg_ok = false, seg_mode = false;
  bool seg_unsafe = false;   // a non-finite or wide-range operand was seen: exact fold from then on
  // running operand statistics of every push since reset (k_operand_stats):
  // the window can hold items of earlier pushes, so the span covers them all
  uint32_t op_emax = 0, op_emin = 0xFFFFFFFFu;
  uint32_t op_signs = 0;     // kOpNeg / kOpPos of every operand since reset
  bool seg_pref = true;      // the mode asked for (option / default), restored by reset()
  DevBuf d_chmeta;
  PinnedBuf h_chmeta;
  int nch = 0;                       // distinct aggregated expressions (channels)
  int ch_agg[kMaxChan] = {}, ch_type[kMaxChan] = {};
  int chan_of[kMaxAggs] = {};
  DevBuf sval, snn, se, scall, tagg, segS, segNN, rec, seg_items;
  // group state (dense by key)
  DevBuf g_dsum, g_lsum, g_cnt;
  int64_t g_nkeys = 0;

  int kind() const override { return agg_mode ? ENG_WINDOW : ENG_FILTER; }

  // "exact_aggregates" = 1: the bit-exact sequential fold instead of the
  // segmented scans (any time; both keep the group tables current)
  void set_option(const std::string& key, int64_t v) override {
    if (key == "exact_aggregates") {
      seg_pref = v == 0;
      seg_mode = seg_ok && !seg_unsafe && seg_pref;
    }
    else Engine::set_option(key, v);
  }

  void reset() override {
    C = 0;
    seq = 0;
    now = INT64_MIN;
    chunk_seq = 0;
    out.count = 0;
    counters = shd_counters{};
    if (g_nkeys) {
      SHD_HIP(hipMemsetAsync(g_dsum.p, 0, g_dsum.cap, stream));
      SHD_HIP(hipMemsetAsync(g_lsum.p, 0, g_lsum.cap, stream));
      SHD_HIP(hipMemsetAsync(g_cnt.p, 0, g_cnt.cap, stream));
    }
    gd.reset(stream);
    kmax_seen = 0;
    kmax_known = true;
    seg_unsafe = false;
    op_emax = 0;
    op_emin = 0xFFFFFFFFu;
    op_signs = 0;
    seg_mode = seg_ok && seg_pref;
  }

  // Dense group ids of the m new items [C, C + m) (dictionary mode).
  void gdict_assign(int64_t m, int64_t gstride) {
    gd.nk = std::max(ngk, 1);
    gd.assign(m, g_h.as<uint64_t>(), g_kw.as<uint64_t>(), g_kn.as<uint8_t>(), gstride, ikey[cur].as<uint64_t>(), C,
              stream);
  }

  // window contents (items [0, C) of slot `cur`) + dense per-group aggregates
  void save_state(SnapW& w) override {
    w.put<int64_t>(C);
    w.put<int32_t>(nagg);
    w.put<int64_t>(g_nkeys);
    if (C > 0) {
      w.dev(ikey[cur].p, (size_t)C * 8);
      w.dev(its[cur].p, (size_t)C * 8);
      for (int g = 0; g < nagg; g++) {
        w.dev(iargv[cur].as<uint64_t>() + g * icap[cur], (size_t)C * 8);
        w.dev(iargn[cur].as<uint8_t>() + g * icap[cur], (size_t)C);
      }
    }
    if (g_nkeys > 0) {
      const size_t gb = (size_t)std::max(nagg, 1) * g_nkeys * 8;
      w.dev(g_dsum.p, gb);
      w.dev(g_lsum.p, gb);
      w.dev(g_cnt.p, gb);
    }
    w.put<int32_t>(seg_unsafe ? 1 : 0);
    w.put<uint32_t>(op_emax);
    w.put<uint32_t>(op_emin);
    w.put<uint32_t>(op_signs);
    // group dictionary (dictionary-mode group keys)
    gd.save(w);
  }
  void load_state(SnapR& r) override {
    const int64_t c0 = r.get<int64_t>();
    if (r.get<int32_t>() != nagg || c0 < 0) throw Error(SHD_E_ARG, "snapshot of a different plan");
    const int64_t nk = r.get<int64_t>();
    cur = 0;
    if (c0 > 0) {
      ensure_items(0, c0);
      r.dev_into(ikey[0].p, (size_t)c0 * 8);
      r.dev_into(its[0].p, (size_t)c0 * 8);
      for (int g = 0; g < nagg; g++) {
        r.dev_into(iargv[0].as<uint64_t>() + g * icap[0], (size_t)c0 * 8);
        r.dev_into(iargn[0].as<uint8_t>() + g * icap[0], (size_t)c0);
      }
    }
    C = c0;
    if (nk > 0) {
      const size_t gb = (size_t)std::max(nagg, 1) * nk * 8;
      g_dsum.reserve(gb);
      g_lsum.reserve(gb);
      g_cnt.reserve(gb);
      r.dev_into(g_dsum.p, gb);
      r.dev_into(g_lsum.p, gb);
      r.dev_into(g_cnt.p, gb);
    } else if (g_nkeys) {
      SHD_HIP(hipMemsetAsync(g_dsum.p, 0, g_dsum.cap, stream));
      SHD_HIP(hipMemsetAsync(g_lsum.p, 0, g_lsum.cap, stream));
      SHD_HIP(hipMemsetAsync(g_cnt.p, 0, g_cnt.cap, stream));
    }
    if (nk > 0 || !g_nkeys) g_nkeys = nk;
    seg_unsafe = r.get<int32_t>() != 0;
    op_emax = r.get<uint32_t>();
    op_emin = r.get<uint32_t>();
    op_signs = r.get<uint32_t>();
    seg_mode = seg_ok && seg_pref && !seg_unsafe;
    gd.nk = std::max(ngk, 1);
    gd.load(r, stream);
    kmax_known = false;
    counters.carry = C;
  }

  // ---- query sharing (shd_group_create): window queries that differ only in
  // the length of their length window share this engine's filter pass and
  // items (it holds the longest window); each member's rows come from its own
  // call-window fold over them.  The leader emits no rows of its own.
  std::vector<SingleEngine*> wmembers;

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
    if (ms.empty() || ms.size() > 64) throw Error(SHD_E_ARG, "a group holds 1..64 member queries");
    if (!agg_mode || !seg_mode || wkind != SHD_W_LENGTH || ngk == 0 || partitioned)
      throw Error(SHD_E_UNSUPPORTED, "query groups: only length-window group-by aggregates share items");
    if (counters.events != 0 || C != 0) throw Error(SHD_E_ARG, "the group leader must be fresh");
    std::vector<SingleEngine*> v;
    for (Engine* e : ms) {
      auto* m = dynamic_cast<SingleEngine*>(e);
      if (!m || m == this || m->grouped) throw Error(SHD_E_ARG, "group member: not a free window query");
      for (SingleEngine* o : v)
        if (o == m) throw Error(SHD_E_ARG, "group member listed twice");
      bool ok = m->agg_mode && m->seg_mode && m->wkind == SHD_W_LENGTH && m->wparam <= wparam && !m->partitioned &&
                m->plan.stream_types == plan.stream_types && m->filters.size() == filters.size() &&
                m->ngk == ngk && m->gdense == gdense && m->nagg == nagg && m->outs.size() == outs.size() &&
                m->nch == nch;
      for (size_t k = 0; ok && k < filters.size(); k++) ok = same_expr(plan, filters[k], m->plan, m->filters[k]);
      for (int k = 0; ok && k < ngk; k++)
        ok = same_expr(plan, gk_expr[k], m->plan, m->gk_expr[k]) && gk_type[k] == m->gk_type[k];
      for (int k = 0; ok && k < nagg; k++)
        ok = plan.aggs[k].kind == m->plan.aggs[k].kind && plan.aggs[k].type == m->plan.aggs[k].type &&
             same_expr(plan, plan.aggs[k].expr, m->plan, m->plan.aggs[k].expr) && chan_of[k] == m->chan_of[k];
      if (!ok)
        throw Error(SHD_E_ARG, "group member differs from the leader beyond its window length (or is longer)");
      if (m->counters.events != 0 || m->C != 0 || m->out.count != 0)
        throw Error(SHD_E_ARG, "group members must be fresh (reset, no unpolled rows)");
      v.push_back(m);
    }
    wmembers = v;
    grouped = true;
    for (SingleEngine* m : wmembers) m->grouped = true;
  }

  void group_detach() override {
    for (SingleEngine* m : wmembers) m->grouped = false;
    wmembers.clear();
    grouped = false;
  }

  // The leader hands its window over: every member's state becomes the one it
  // would hold running alone -- its length window is the last `wparam` of the
  // leader's carried items (filter passed, same group ids and operands), its
  // group tables are already current (k_cw_gtables after every push), the
  // group dictionary is the leader's, and the operand statistics carry the
  // range guard over.  The members leave the group.
  void group_dissolve() override {
    SHD_HIP(hipStreamSynchronize(stream));
    for (SingleEngine* m : wmembers) m->adopt_window(*this);
    group_detach();
  }

  void adopt_window(SingleEngine& L) {
    SHD_HIP(hipStreamSynchronize(stream));
    hipStream_t s = stream;
    const int64_t k = std::min<int64_t>(L.C, wparam);
    const int64_t from = L.C - k;
    cur = 0;
    if (k > 0) {
      ensure_items(0, k);
      SHD_HIP(hipMemcpyAsync(ikey[0].p, L.ikey[L.cur].as<uint64_t>() + from, k * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(its[0].p, L.its[L.cur].as<int64_t>() + from, k * 8, hipMemcpyDeviceToDevice, s));
      for (int g = 0; g < nagg; g++) {
        SHD_HIP(hipMemcpyAsync(iargv[0].as<uint64_t>() + g * icap[0], L.iargv[L.cur].as<uint64_t>() + g * L.icap[L.cur] +
                               from, k * 8, hipMemcpyDeviceToDevice, s));
        SHD_HIP(hipMemcpyAsync(iargn[0].as<uint8_t>() + g * icap[0], L.iargn[L.cur].as<uint8_t>() + g * L.icap[L.cur] +
                               from, k, hipMemcpyDeviceToDevice, s));
      }
    }
    C = k;
    if (!gdense) {   // hashed group ids: the leader's dictionary assigned them
      SnapW w;
      w.s = L.stream;
      L.gd.save(w);
      SnapR r;
      r.p = w.b.data();
      r.n = w.b.size();
      r.s = s;
      gd.nk = std::max(ngk, 1);
      gd.load(r, s);
    }
    op_emax = L.op_emax;
    op_emin = L.op_emin;
    op_signs = L.op_signs;
    seg_unsafe = L.seg_unsafe;
    seg_mode = seg_ok && seg_pref && !seg_unsafe;
    kmax_known = false;
    counters.carry = C;
    SHD_HIP(hipStreamSynchronize(s));
  }

  std::vector<int64_t> h_offs;   // lives until the next push (async H2D source)
  PinnedBuf h_last, h_offs_pin;

  void stage_calls(const Staged& b, int64_t& ncalls) {
    h_offs = b.call_offsets;
    if (h_offs.size() < 2) h_offs = {0, b.n};
    std::vector<int64_t>& offs = h_offs;
    ncalls = (int64_t)offs.size() - 1;
    d_offs.reserve(offs.size() * 8);
    // pinned source: the previous push ended with a stream sync, so the area is free
    h_offs_pin.reserve(offs.size() * 8);
    std::memcpy(h_offs_pin.p, offs.data(), offs.size() * 8);
    SHD_HIP(hipMemcpyAsync(d_offs.p, h_offs_pin.p, offs.size() * 8, hipMemcpyHostToDevice, stream));
    d_call_of.reserve(b.n * 4);
    d_last_ts.reserve(ncalls * 8);
    d_now.reserve(ncalls * 8);
    hipLaunchKernelGGL(k_call_of, dim3((unsigned)std::min<int64_t>(ncalls, 65535)), dim3(kBlock), 0, stream,
                       (const int64_t*)d_offs.as<int64_t>(), (int)ncalls, b.cs.ts, d_call_of.as<int32_t>(),
                       d_last_ts.as<int64_t>());
    SHD_CHECK_LAUNCH();
    // per-call times feed the time window's expiry; every other query only
    // moves the clock to the push's latest call time
    if (wkind == SHD_W_TIME)
      hipLaunchKernelGGL(k_call_now, dim3(1), dim3(kBlock), 0, stream, (const int64_t*)d_last_ts.as<int64_t>(),
                         (int)ncalls, now, d_now.as<int64_t>());
    else
      hipLaunchKernelGGL(k_call_now_last, dim3(1), dim3(kBlock), 0, stream, (const int64_t*)d_last_ts.as<int64_t>(),
                         (int)ncalls, now, d_now.as<int64_t>());
    SHD_CHECK_LAUNCH();
  }

  void push(const Staged& b) override {
    const int64_t n = b.n;
    if (n <= 0) return;
    hipStream_t s = stream;
    SHD_HIP(hipEventRecord(ev0, s));
    stage_begin();
    int64_t ncalls = 0;
    stage_calls(b, ncalls);
    d_flags.reserve(n);
    d_cnt.reserve(n * 4);
    d_off.reserve(n * 4);
    d_tot.reserve(128);
    h_tot.reserve(128);
    if (partitioned) d_pkey.reserve(n * 8);
    FilterArgs fa{};
    fa.cs = b.cs;
    fa.es = dset();
    fa.filters = dfilters(filters);
    fa.partitioned = partitioned;
    if (partitioned) {
      fa.key = dexpr(key_expr);
      fa.key_col = key_col;
      fa.key_type = key_type;
    }
    // aggregate queries (never inside a partition here: those run on the
    // keyed window engine) filter and build their items in one pass
    if (agg_mode && !partitioned && !getenv("SHD_NO_FUSED_ITEMS")) {
      push_agg_fused(b, ncalls, n, fa);
    } else {
      const FilterArgs* d_fa = dev_args(fa);
      if (std::getenv("SHD_DEBUG_ARGS")) debug_filter_args(d_fa, fa, n);
      hipLaunchKernelGGL(k_filter, dim3(grid_cover(n)), dim3(kBlock), 0, s, d_fa, n, d_flags.as<uint8_t>(),
                         d_cnt.as<uint32_t>(), d_pkey.as<uint64_t>());
      SHD_CHECK_LAUNCH();
      uint32_t* d_m = (uint32_t*)d_tot.p;
      scan_exclusive_u32(d_cnt.as<uint32_t>(), d_off.as<uint32_t>(), n, d_m, d_scan, s);
      mark("filter");
      if (!agg_mode) push_filter(b, ncalls, n);
      else push_agg(b, ncalls, n);
    }
    SHD_HIP(hipEventRecord(ev1, s));
    stage_end();
    SHD_HIP(hipEventSynchronize(ev1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    counters.kernel_ns = (int64_t)(ms * 1e6);
    counters.events += n;
    // TimestampGeneratorImpl: time moves to the last call's ts if later
    if (b.advance_time || true) {
      int64_t last = 0;
      h_last.reserve(8);
      SHD_HIP(hipMemcpyAsync(h_last.p, d_now.as<int64_t>() + (ncalls - 1), 8, hipMemcpyDeviceToHost, stream));
      SHD_HIP(hipStreamSynchronize(stream));
      last = *h_last.as<int64_t>();
      if (last > now) now = last;
    }
    seq += n;
    for (SingleEngine* q : wmembers)
      if (now > q->now) q->now = now;
  }

  // Debug hook (SHD_DEBUG_ARGS=1): read the argument block back from the
  // device, print it with the allocation each pointer belongs to, and stop
  // before the launch.
  void debug_filter_args(const FilterArgs* d_fa, const FilterArgs& fa, int64_t n) {
    SHD_HIP(hipStreamSynchronize(stream));
    FilterArgs h{};
    SHD_HIP(hipMemcpy(&h, d_fa, sizeof(h), hipMemcpyDeviceToHost));
    auto where = [](const void* p) {
      if (!p) return std::string("null");
      hipPointerAttribute_t at{};
      hipError_t e = hipPointerGetAttributes(&at, p);
      char buf[160];
      std::snprintf(buf, sizeof buf, "%p type=%d dev=%d err=%d", p, e == hipSuccess ? (int)at.type : -1,
                    e == hipSuccess ? at.device : -1, (int)e);
      (void)hipGetLastError();
      return std::string(buf);
    };
    std::fprintf(stderr, "SHD_DEBUG_ARGS k_filter n=%lld same=%d sizeof=%zu\n", (long long)n,
                 (int)(std::memcmp(&h, &fa, sizeof(h)) == 0), sizeof(h));
    std::fprintf(stderr, "  es.ins %s nins=%d consts %s nconsts=%d\n", where(h.es.ins).c_str(), h.es.nins,
                 where(h.es.consts).c_str(), h.es.nconsts);
    for (int c = 0; c < h.cs.ncols; c++)
      std::fprintf(stderr, "  col[%d] %s nul %s type=%d\n", c, where(h.cs.col[c]).c_str(), where(h.cs.nul[c]).c_str(),
                   (int)h.cs.type[c]);
    std::fprintf(stderr, "  ts %s n=%lld ncols=%d filters.n=%d f0=(%d,%d) part=%d\n", where(h.cs.ts).c_str(),
                 (long long)h.cs.n, h.cs.ncols, h.filters.n, h.filters.f[0].off, h.filters.f[0].len, h.partitioned);
    std::fprintf(stderr, "  flags %s cnt %s pkey %s argdev %s\n", where(d_flags.p).c_str(), where(d_cnt.p).c_str(),
                 where(d_pkey.p).c_str(), where(d_fa).c_str());
    std::vector<int4> ins(std::max(h.es.nins, 1));
    SHD_HIP(hipMemcpy(ins.data(), h.es.ins, h.es.nins * sizeof(int4), hipMemcpyDeviceToHost));
    for (int i = 0; i < h.es.nins; i++) std::fprintf(stderr, "  ins[%d] = %d %d %d %d\n", i, ins[i].x, ins[i].y, ins[i].z, ins[i].w);
    throw Error(SHD_E_DEVICE, "SHD_DEBUG_ARGS: stopped before k_filter");
  }

  void push_filter(const Staged& b, int64_t ncalls, int64_t n) {
    hipStream_t s = stream;
    uint32_t* d_m = (uint32_t*)d_tot.p;
    uint32_t* d_r = d_m + 1;
    if (partitioned) {
      d_start.reserve(n * 4);
      d_run.reserve(n * 4);
      hipLaunchKernelGGL(k_run_starts, dim3(grid_for(n)), dim3(kBlock), 0, s, (const uint8_t*)d_flags.as<uint8_t>(),
                         (const uint64_t*)d_pkey.as<uint64_t>(), (const int32_t*)d_call_of.as<int32_t>(), n,
                         d_start.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      // run id of event i = (#starts up to and including i) - 1
      scan_exclusive_u32(d_start.as<uint32_t>(), d_run.as<uint32_t>(), n, d_r, d_scan, s);
    }
    SHD_HIP(hipMemcpyAsync(h_tot.p, d_tot.p, 8, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    uint32_t m = h_tot.as<uint32_t>()[0];
    uint32_t nruns = h_tot.as<uint32_t>()[1];
    if (m > 0) {
      out.ensure(m, s);
      ProjArgs pa{};
      pa.cs = b.cs;
      pa.es = dset();
      pa.nout = (int)outs.size();
      for (size_t c = 0; c < outs.size(); c++) pa.outs[c] = dexpr(outs[c]);
      pa.row0 = out.count;
      // exclusive run ids: the run of event i is start-scan[i] (+0 if i is a start it is its own index)
      pa.chunk0 = chunk_seq;
      pa.seq0 = seq;
      pa.partitioned = partitioned;
      hipLaunchKernelGGL(k_project_rows, dim3(grid_cover(n)), dim3(kBlock), 0, s, dev_args(pa), n,
                         (const uint32_t*)d_cnt.as<uint32_t>(), (const uint32_t*)d_off.as<uint32_t>(),
                         (const int32_t*)d_call_of.as<int32_t>(), (const uint32_t*)d_run.as<uint32_t>(),
                         (const uint32_t*)d_start.as<uint32_t>(), out.d_chunk(), out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls(),
                         out.d_seq());
      SHD_CHECK_LAUNCH();
      SHD_HIP(hipMemsetAsync(out.d_sidx() + out.count, 0, (size_t)m * 4, s));   // no states: state_idx 0
      out.count += m;
    }
    chunk_seq += partitioned ? (int64_t)nruns : ncalls;
    counters.matches += m;
  }

  void ensure_items(int slot, int64_t cap) {
    if (icap[slot] >= cap) return;
    int64_t nc = std::max<int64_t>(cap, 1024);
    DevBuf k2, t2, v2, n2;
    k2.reserve(nc * 8);
    t2.reserve(nc * 8);
    v2.reserve(std::max(nagg, 1) * nc * 8);
    n2.reserve(std::max(nagg, 1) * nc);
    std::swap(ikey[slot].p, k2.p); std::swap(ikey[slot].cap, k2.cap);
    std::swap(its[slot].p, t2.p); std::swap(its[slot].cap, t2.cap);
    std::swap(iargv[slot].p, v2.p); std::swap(iargv[slot].cap, v2.cap);
    std::swap(iargn[slot].p, n2.p); std::swap(iargn[slot].cap, n2.cap);
    icap[slot] = nc;
    // (old contents are only needed for the carry slot, which is copied explicitly)
  }

  void ensure_groups(int64_t nkeys) {
    if (nkeys <= g_nkeys) return;
    int64_t nk = std::max<int64_t>(nkeys, g_nkeys * 2);
    nk = std::max<int64_t>(nk, 1024);
    DevBuf a, l, c;
    int na = std::max(nagg, 1);
    a.reserve(na * nk * 8);
    l.reserve(na * nk * 8);
    c.reserve(na * nk * 8);
    SHD_HIP(hipMemsetAsync(a.p, 0, na * nk * 8, stream));
    SHD_HIP(hipMemsetAsync(l.p, 0, na * nk * 8, stream));
    SHD_HIP(hipMemsetAsync(c.p, 0, na * nk * 8, stream));
    for (int g = 0; g < nagg && g_nkeys; g++) {
      SHD_HIP(hipMemcpyAsync(a.as<double>() + g * nk, g_dsum.as<double>() + g * g_nkeys, g_nkeys * 8,
                             hipMemcpyDeviceToDevice, stream));
      SHD_HIP(hipMemcpyAsync(l.as<int64_t>() + g * nk, g_lsum.as<int64_t>() + g * g_nkeys, g_nkeys * 8,
                             hipMemcpyDeviceToDevice, stream));
      SHD_HIP(hipMemcpyAsync(c.as<int64_t>() + g * nk, g_cnt.as<int64_t>() + g * g_nkeys, g_nkeys * 8,
                             hipMemcpyDeviceToDevice, stream));
    }
    SHD_HIP(hipStreamSynchronize(stream));
    std::swap(g_dsum.p, a.p); std::swap(g_dsum.cap, a.cap);
    std::swap(g_lsum.p, l.p); std::swap(g_lsum.cap, l.cap);
    std::swap(g_cnt.p, c.p); std::swap(g_cnt.cap, c.cap);
    g_nkeys = nk;
  }

  // Emission: one row per (call, group) with a CURRENT event, in first-seen
  // order, with the group's values after its last event of the call
  // (QuerySelector.processInBatchGroupBy, QuerySelector.java:315-373).
  void emit_rows(const Staged& b, int64_t m, int64_t cap) {
    hipStream_t s = stream;
    const int64_t total = C + m;
    fcnt.reserve(m * 4);
    foff.reserve(m * 4);
    hipLaunchKernelGGL(k_first_counts, dim3(grid_for(m)), dim3(kBlock), 0, s, (const uint8_t*)first.as<uint8_t>(), C,
                       total, fcnt.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    uint32_t* d_f = (uint32_t*)(d_tot.as<uint64_t>() + 4);
    scan_exclusive_u32(fcnt.as<uint32_t>(), foff.as<uint32_t>(), m, d_f, d_scan, s);
    SHD_HIP(hipMemcpyAsync(h_tot.as<uint64_t>() + 4, d_f, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t nrows = h_tot.as<uint32_t>()[8];
    if (nrows <= 0) return;
    out.ensure(nrows, s);
    EmitArgs ea{};
    ea.cs = b.cs;
    ea.es = dset();
    ea.nout = (int)outs.size();
    for (size_t c = 0; c < outs.size(); c++) {
      ea.outs[c] = dexpr(outs[c]);
      const auto& code = plan.exprs[outs[c]];
      ea.okind[c] = 0;
      if (code.size() == 1 && code[0].op == SHD_OP_LOAD) {
        ea.okind[c] = 1;
        ea.oarg[c] = code[0].c & 0xFFFF;
      } else if (code.size() == 1 && code[0].op == SHD_OP_AGG && code[0].a >= 0 && code[0].a < nagg) {
        ea.okind[c] = 2;
        ea.oarg[c] = code[0].a;
      }
      if (getenv("SHD_NO_FAST_OUT")) ea.okind[c] = 0;
    }
    ea.nagg = nagg;
    for (int g = 0; g < nagg; g++) ea.kind[g] = plan.aggs[g].kind;
    ea.cap = cap;
    ea.C = C;
    ea.row0 = out.count;
    ea.chunk0 = chunk_seq;
    ea.seq0 = seq;
    if (seg_mode)
      hipLaunchKernelGGL(k_emit<true>, dim3(grid_cover(m)), dim3(kBlock), 0, s, dev_args(ea), m,
                         (const uint32_t*)fcnt.as<uint32_t>(), (const uint32_t*)foff.as<uint32_t>(),
                         (const uint32_t*)last_of.as<uint32_t>(), (const int32_t*)ievrow.as<int32_t>(),
                         (const int32_t*)d_call_of.as<int32_t>(), (const uint64_t*)rec.as<uint64_t>(),
                         (const uint8_t*)resn.as<uint8_t>(), (const int64_t*)resc.as<int64_t>(), out.d_chunk(),
                         out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls(), out.d_seq());
    else
      hipLaunchKernelGGL(k_emit<false>, dim3(grid_cover(m)), dim3(kBlock), 0, s, dev_args(ea), m,
                         (const uint32_t*)fcnt.as<uint32_t>(), (const uint32_t*)foff.as<uint32_t>(),
                         (const uint32_t*)last_of.as<uint32_t>(), (const int32_t*)ievrow.as<int32_t>(),
                         (const int32_t*)d_call_of.as<int32_t>(), (const uint64_t*)resv.as<uint64_t>(),
                         (const uint8_t*)resn.as<uint8_t>(), (const int64_t*)resc.as<int64_t>(), out.d_chunk(),
                         out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls(), out.d_seq());
    SHD_CHECK_LAUNCH();
    SHD_HIP(hipMemsetAsync(out.d_sidx() + out.count, 0, (size_t)nrows * 4, s));   // no states: state_idx 0
    out.count += nrows;
    counters.matches += nrows;
    mark("emit");
  }

  // Segmented-scan window aggregates (see k_seg_gather .. k_seg_emit): stable
  // group sort of the window items, sorted copies, 3-phase segmented scan,
  // windowed differences at the (call, group) run ends.
  template <int NC>
  void segscan_kernels(int64_t total, const uint32_t* sk, const uint32_t* sp, const SegArgs* d_sa, int64_t cap) {
    hipStream_t s = stream;
    sval.reserve((size_t)NC * total * 8);
    snn.reserve(total);
    se.reserve(total * 4);
    scall.reserve(total * 4);
    if (NC <= 2 && !getenv("SHD_SEG_UNPACKED")) {
      constexpr int N2 = NC <= 2 ? NC : 1;
      // packed in item order (coalesced), then one record read per sorted position
      seg_items.reserve((size_t)total * sizeof(SegItem<N2>));
      hipLaunchKernelGGL(k_seg_pack<N2>, dim3(grid_cover(total)), dim3(kBlock), 0, s, d_sa,
                         (const uint64_t*)iargv[cur].as<uint64_t>(), (const uint8_t*)iargn[cur].as<uint8_t>(),
                         (const uint32_t*)e_exp.as<uint32_t>(), (const int32_t*)icall.as<int32_t>(),
                         (SegItem<N2>*)seg_items.as<char>());
      SHD_CHECK_LAUNCH();
      hipLaunchKernelGGL(k_seg_gather_packed<N2>, dim3(grid_cover(total)), dim3(kBlock), 0, s, d_sa, sp,
                         (const SegItem<N2>*)seg_items.as<char>(), sval.as<double>(), snn.as<uint8_t>(),
                         se.as<uint32_t>(), scall.as<int32_t>());
    } else {
      hipLaunchKernelGGL(k_seg_gather<NC>, dim3(grid_cover(total)), dim3(kBlock), 0, s, d_sa, sp,
                         (const uint64_t*)iargv[cur].as<uint64_t>(), (const uint8_t*)iargn[cur].as<uint8_t>(),
                         (const uint32_t*)e_exp.as<uint32_t>(), (const int32_t*)icall.as<int32_t>(), sval.as<double>(),
                         snn.as<uint8_t>(), se.as<uint32_t>(), scall.as<int32_t>());
    }
    SHD_CHECK_LAUNCH();
    mark("seg_gather");
    const int64_t nt = ceil_div(total, kSegTile);
    tagg.reserve(nt * sizeof(SegAcc<NC>));
    segS.reserve((size_t)NC * total * sizeof(DD));
    segNN.reserve((size_t)NC * total * 4);
    const bool lds = NC <= 2 && !getenv("SHD_SEG_NOLDS");
    if (lds)
      hipLaunchKernelGGL(k_seg_tiles_lds<(NC <= 2 ? NC : 1)>, dim3((unsigned)nt), dim3(kBlock), 0, s, total, sk,
                         (const double*)sval.as<double>(), (const uint8_t*)snn.as<uint8_t>(),
                         (SegAcc<(NC <= 2 ? NC : 1)>*)tagg.as<char>());
    else
      hipLaunchKernelGGL(k_seg_tiles<NC>, dim3((unsigned)nt), dim3(kBlock), 0, s, total, sk,
                         (const double*)sval.as<double>(), (const uint8_t*)snn.as<uint8_t>(), tagg.as<SegAcc<NC>>());
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_seg_tilescan<NC>, dim3(1), dim3(kBlock), 0, s, tagg.as<SegAcc<NC>>(), nt);
    SHD_CHECK_LAUNCH();
    if (lds)
      hipLaunchKernelGGL(k_seg_apply_lds<(NC <= 2 ? NC : 1)>, dim3((unsigned)nt), dim3(kBlock), 0, s, total, sk,
                         (const double*)sval.as<double>(), (const uint8_t*)snn.as<uint8_t>(),
                         (const SegAcc<(NC <= 2 ? NC : 1)>*)tagg.as<char>(), segS.as<DD>(), segNN.as<int32_t>());
    else
      hipLaunchKernelGGL(k_seg_apply<NC>, dim3((unsigned)nt), dim3(kBlock), 0, s, total, sk,
                         (const double*)sval.as<double>(), (const uint8_t*)snn.as<uint8_t>(),
                         (const SegAcc<NC>*)tagg.as<SegAcc<NC>>(), segS.as<DD>(), segNN.as<int32_t>());
    SHD_CHECK_LAUNCH();
    mark("seg_scan");
    rec.reserve((size_t)cap * run_rec_words(nagg) * 8);
    hipLaunchKernelGGL(k_seg_emit<NC>, dim3(grid_cover(total)), dim3(kBlock), 0, s, d_sa, sk, sp,
                       (const uint32_t*)se.as<uint32_t>(), (const int32_t*)scall.as<int32_t>(),
                       (const DD*)segS.as<DD>(), (const int32_t*)segNN.as<int32_t>(),
                       (const uint8_t*)snn.as<uint8_t>(), rec.as<uint64_t>(), first.as<uint8_t>());
    SHD_CHECK_LAUNCH();
    mark("seg_window");
  }

  // Chunked window walk (k_wc_*): dense group ids in [64, kWcMaxG], at most
  // two aggregated expressions, calls of at most kWcItems events.  false:
  // not this push's path (nothing written yet): the segmented scans run.
  DevBuf wc_cp, wc_ce, wc_table, wc_seg;
  template <int NC>
  bool wc_kernels(int64_t total, int G, int64_t cap, int64_t ncalls, int F, int kc, int K) {
    hipStream_t s = stream;
    SegArgs sa{};
    sa.nch = NC;
    for (int c = 0; c < NC; c++) {
      sa.ch_agg[c] = nch ? ch_agg[c] : 0;
      sa.ch_type[c] = nch ? ch_type[c] : SHD_T_DOUBLE;
    }
    sa.nagg = nagg;
    sa.cap = cap;
    sa.C = C;
    sa.total = total;
    WcArgs wa{};
    wa.C = C;
    wa.total = total;
    wa.G = G;
    wa.nagg = nagg;
    for (int g = 0; g < nagg; g++) {
      wa.kind[g] = plan.aggs[g].kind;
      wa.type[g] = plan.aggs[g].type;
      wa.chan[g] = chan_of[g];
    }
    wc_cp.reserve((size_t)(K + 1) * 8);
    wc_ce.reserve((size_t)(K + 1) * 8);
    wa.ikey = ikey[cur].as<uint64_t>();
    wa.e = e_exp.as<uint32_t>();
    wa.cp = wc_cp.as<int64_t>();
    wa.ce = wc_ce.as<int64_t>();
    rec.reserve((size_t)cap * run_rec_words(nagg) * 8);
    wa.rec = rec.as<uint64_t>();
    wa.first = first.as<uint8_t>();
    wa.dsum = g_dsum.as<double>();
    wa.gcnt = g_cnt.as<int64_t>();
    wa.nkeys = g_nkeys;
    unsigned int* d_flag = (unsigned int*)(d_tot.as<uint64_t>() + 7);
    SHD_HIP(hipMemsetAsync(d_flag, 0, 4, s));
    wa.flag = d_flag;
    const WcArgs* d_wa = dev_args(wa);
    hipLaunchKernelGGL(k_wc_bounds, dim3(grid_for(K + 1)), dim3(kBlock), 0, s, d_wa, kc, K, F, (int)ncalls,
                       (const int32_t*)icall.as<int32_t>(), wc_cp.as<int64_t>(), wc_ce.as<int64_t>());
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_wc_check, dim3(grid_for(K)), dim3(kBlock), 0, s, (const int64_t*)wc_cp.as<int64_t>(),
                       (const int64_t*)wc_ce.as<int64_t>(), K, d_flag);
    SHD_CHECK_LAUNCH();
    SHD_HIP(hipMemcpyAsync(h_tot.as<uint64_t>() + 7, d_flag, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    if (h_tot.as<uint32_t>()[14]) return false;   // a chunk beyond the LDS capacity
    seg_items.reserve((size_t)total * sizeof(SegItem<NC>));
    hipLaunchKernelGGL(k_seg_pack<NC>, dim3(grid_cover(total)), dim3(kBlock), 0, s, dev_args(sa),
                       (const uint64_t*)iargv[cur].as<uint64_t>(), (const uint8_t*)iargn[cur].as<uint8_t>(),
                       (const uint32_t*)e_exp.as<uint32_t>(), (const int32_t*)icall.as<int32_t>(),
                       (SegItem<NC>*)seg_items.as<char>());
    SHD_CHECK_LAUNCH();
    const SegItem<NC>* items = (const SegItem<NC>*)seg_items.as<char>();
    wc_table.reserve((size_t)K * G * sizeof(WcAcc<NC>));
    const int nseg = (K + kWcSeg - 1) / kWcSeg;
    wc_seg.reserve((size_t)nseg * G * sizeof(WcAcc<NC>));
    WcAcc<NC>* table = (WcAcc<NC>*)wc_table.as<char>();
    WcAcc<NC>* seg = (WcAcc<NC>*)wc_seg.as<char>();
    hipLaunchKernelGGL(k_wc_delta<NC>, dim3(K), dim3(kWcThreads), 0, s, d_wa, items, table);
    SHD_CHECK_LAUNCH();
    mark("wc_delta");
    const int64_t nt = (int64_t)nseg * G;
    hipLaunchKernelGGL(k_wc_scan1<NC>, dim3(grid_for(nt)), dim3(kBlock), 0, s, d_wa, K, (const WcAcc<NC>*)table, seg);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_wc_scan2<NC>, dim3(grid_for(G)), dim3(kBlock), 0, s, d_wa, K, seg);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_wc_scan3<NC>, dim3(grid_for(nt)), dim3(kBlock), 0, s, d_wa, K, table, (const WcAcc<NC>*)seg);
    SHD_CHECK_LAUNCH();
    mark("wc_scan");
    hipLaunchKernelGGL(k_wc_emit<NC>, dim3(K), dim3(kWcThreads), 0, s, d_wa, items, (const WcAcc<NC>*)table);
    SHD_CHECK_LAUNCH();
    mark("wc_emit");
    return true;
  }

  bool agg_chunked(int64_t total, uint64_t kmax, int64_t cap, int64_t ncalls) {
    // group ids: dense dictionary ids (string / bool attribute) or the group
    // dictionary's dense ids -- either way in [0, kmax]
    // opt-in (SHD_WCHUNK=1): on W2 the per-chunk workgroups (144 KB of LDS:
    // one per CU) are latency-bound -- r03m: 13.5 ms of delta + emit per
    // 100 M events against 10.4 ms for the group sort + segmented scans
    if (!getenv("SHD_WCHUNK") || getenv("SHD_NO_WCHUNK") || ngk == 0 || (wkind != SHD_W_LENGTH && wkind != SHD_W_TIME) ||
        nch > 2 ||
        kmax + 1 > (uint64_t)kWcMaxG || kmax + 1 < 64 || total >= (int64_t)INT32_MAX)
      return false;
    int64_t maxcall = 0;
    for (size_t c = 0; c + 1 < h_offs.size(); c++) maxcall = std::max<int64_t>(maxcall, h_offs[c + 1] - h_offs[c]);
    if (maxcall <= 0 || maxcall > kWcItems || ncalls <= 0) return false;
    const int F = (int)std::max<int64_t>(1, kWcItems / maxcall);
    const int kc = (int)ceil_div(C, kWcItems);
    const int K = kc + (int)ceil_div(ncalls, F);
    const int G = (int)kmax + 1;
    ensure_groups(G);
    return nch <= 1 ? wc_kernels<1>(total, G, cap, ncalls, F, kc, K) : wc_kernels<2>(total, G, cap, ncalls, F, kc, K);
  }

  // Call-window path (k_cw): group by, a length / time window whose region
  // per call fits the LDS lists, calls of at most kCwCall events.
  static constexpr int kCwRegionMax = 8192;
  DevBuf d_cw_citem, d_cw_clb;
  bool callwin_candidate(int64_t ncalls, int64_t total) const {
    if (!seg_mode || ngk == 0 || partitioned || nch > kMaxChan || (wkind != SHD_W_LENGTH && wkind != SHD_W_TIME) ||
        total >= (int64_t)UINT32_MAX - 1 || ncalls <= 0 || getenv("SHD_NO_CALLWIN"))
      return false;
    for (size_t c = 0; c + 1 < h_offs.size(); c++)
      if (h_offs[c + 1] - h_offs[c] > kCwCall) return false;
    return true;
  }

  template <int NC>
  void callwin_launch(const CwArgs* d_ca, int64_t ncalls, uint32_t call, uint32_t region) {
    const dim3 g((unsigned)ncalls), bl(kBlock);
    const bool len = wkind == SHD_W_LENGTH;
    if (region <= 2048 && call <= 512) {
      if (len) hipLaunchKernelGGL((k_cw<NC, 2048, 512, true>), g, bl, 0, stream, d_ca, (int)ncalls);
      else hipLaunchKernelGGL((k_cw<NC, 2048, 512, false>), g, bl, 0, stream, d_ca, (int)ncalls);
    } else if (region <= 2048) {
      if (len) hipLaunchKernelGGL((k_cw<NC, 2048, kCwCall, true>), g, bl, 0, stream, d_ca, (int)ncalls);
      else hipLaunchKernelGGL((k_cw<NC, 2048, kCwCall, false>), g, bl, 0, stream, d_ca, (int)ncalls);
    } else {
      if (len) hipLaunchKernelGGL((k_cw<NC, kCwRegionMax, kCwCall, true>), g, bl, 0, stream, d_ca, (int)ncalls);
      else hipLaunchKernelGGL((k_cw<NC, kCwRegionMax, kCwCall, false>), g, bl, 0, stream, d_ca, (int)ncalls);
    }
    SHD_CHECK_LAUNCH();
  }

  static constexpr int kCwDirectG = 1024;   // direct-mapped groups (dense ids below this)
  DevBuf d_cw_status, d_cw_cnt, d_cw_base;

  template <int NC, int RC, int CALLCAP>
  void callwin_direct_launch(const CwArgs* d_ca, int64_t ncalls) {
    const dim3 g((unsigned)ncalls), bl(kBlock);
    const uint32_t* base = d_cw_base.as<uint32_t>();
    if (wkind == SHD_W_LENGTH)
      hipLaunchKernelGGL((k_cw_direct<NC, RC, CALLCAP, kCwDirectG, true>), g, bl, 0, stream, d_ca, (int)ncalls, base);
    else
      hipLaunchKernelGGL((k_cw_direct<NC, RC, CALLCAP, kCwDirectG, false>), g, bl, 0, stream, d_ca, (int)ncalls, base);
    SHD_CHECK_LAUNCH();
  }
  template <int NC>
  void callwin_direct(const CwArgs* d_ca, int64_t ncalls, uint32_t call, uint32_t region) {
    if (region <= 2048 && call <= 512) callwin_direct_launch<NC, 2048, 512>(d_ca, ncalls);
    else if (region <= 2048) callwin_direct_launch<NC, 2048, kCwCall>(d_ca, ncalls);
    else callwin_direct_launch<NC, kCwRegionMax, kCwCall>(d_ca, ncalls);
  }
  // the call-window fold + the rows of every call (no run records / k_emit)
  void agg_callwin(const Staged& b, int64_t total, int64_t cap, int64_t ncalls, int64_t X, uint32_t call,
                   uint32_t region, uint64_t kmax) {
    callwin_rows(*this, b, total, cap, ncalls, X, call, region, kmax, true);
  }

  // The call-window rows of query `q` (this engine, or a member of its window
  // group) over this engine's items: q's window length, group tables, output
  // buffer and ids.  rows_known: k_cw_count's scan of the rows per call is
  // still current (a group's members share it: the calls' distinct groups do
  // not depend on the window).
  // defer (window groups): the direct-mapped rows kernel is not launched here;
  // the member's device arguments are appended for one k_cw_direct_multi, and
  // the row count is left for the caller (the same for every member)
  void callwin_rows(SingleEngine& q, const Staged& b, int64_t total, int64_t cap, int64_t ncalls, int64_t X,
                    uint32_t call, uint32_t region, uint64_t kmax, bool count_rows,
                    std::vector<const CwArgs*>* defer = nullptr) {
    hipStream_t s = stream;
    const int64_t m = total - C;
    q.ensure_groups((int64_t)kmax + 1);
    CwArgs ca{};
    ca.nch = std::max(q.nch, 1);
    for (int c = 0; c < ca.nch; c++) {
      ca.ch_agg[c] = q.nch ? q.ch_agg[c] : 0;
      ca.ch_type[c] = q.nch ? q.ch_type[c] : SHD_T_DOUBLE;
    }
    ca.nagg = q.nagg;
    for (int g = 0; g < q.nagg; g++) {
      ca.kind[g] = q.plan.aggs[g].kind;
      ca.type[g] = q.plan.aggs[g].type;
      ca.chan[g] = q.chan_of[g];
    }
    ca.cap = cap;
    ca.C = C;
    ca.total = total;
    ca.wlen = wkind == SHD_W_LENGTH ? q.wparam : 0;
    ca.ikey = ikey[cur].as<uint64_t>();
    ca.e = e_exp.as<uint32_t>();
    ca.iargv = iargv[cur].as<uint64_t>();
    ca.iargn = iargn[cur].as<uint8_t>();
    ca.citem = d_cw_citem.as<uint32_t>();
    ca.clb = d_cw_clb.as<uint32_t>();
    ca.dsum = q.g_dsum.as<double>();
    ca.cnt = q.g_cnt.as<int64_t>();
    ca.nkeys = q.g_nkeys;
    // rows: at most one per new item
    q.out.ensure(std::max<int64_t>(m, 1), s);
    ca.cs = b.cs;
    ca.es = q.dset();
    ca.nout = (int)q.outs.size();
    for (size_t c = 0; c < q.outs.size(); c++) {
      ca.outs[c] = q.dexpr(q.outs[c]);
      const auto& code = q.plan.exprs[q.outs[c]];
      ca.okind[c] = 0;
      if (code.size() == 1 && code[0].op == SHD_OP_LOAD) {
        ca.okind[c] = 1;
        ca.oarg[c] = code[0].c & 0xFFFF;
      } else if (code.size() == 1 && code[0].op == SHD_OP_AGG && code[0].a >= 0 && code[0].a < q.nagg) {
        ca.okind[c] = 2;
        ca.oarg[c] = code[0].a;
      }
    }
    ca.ievrow = ievrow.as<int32_t>();
    ca.row0 = q.out.count;
    ca.chunk0 = q.chunk_seq;
    ca.seq0 = q.seq;
    ca.o_chunk = q.out.d_chunk();
    ca.o_type = q.out.d_type();
    ca.o_ts = q.out.d_ts();
    ca.o_vals = q.out.d_vals();
    ca.o_nul = q.out.d_nulls();
    ca.o_seq = q.out.d_seq();
    ca.o_sidx = q.out.d_sidx();
    d_cw_status.reserve((size_t)ncalls * 8);
    SHD_HIP(hipMemsetAsync(d_cw_status.p, 0, (size_t)ncalls * 8, s));
    ca.status = d_cw_status.as<uint64_t>();
    ca.nrows = d_tot.as<uint64_t>() + 9;
    const CwArgs* d_ca = dev_args(ca);
    if (kmax < (uint64_t)kCwDirectG && !getenv("SHD_CW_HASH")) {
      // rows per call (distinct groups) -> each call's first row
      if (count_rows) {
        d_cw_cnt.reserve((size_t)ncalls * 4);
        d_cw_base.reserve((size_t)ncalls * 4);
        hipLaunchKernelGGL(k_cw_count<kCwDirectG>, dim3((unsigned)ncalls), dim3(kBlock), 0, s, d_ca, (int)ncalls,
                           d_cw_cnt.as<uint32_t>());
        SHD_CHECK_LAUNCH();
        scan_exclusive_u32(d_cw_cnt.as<uint32_t>(), d_cw_base.as<uint32_t>(), ncalls,
                           (uint32_t*)(d_tot.as<uint64_t>() + 9), d_scan, s);
        SHD_HIP(hipMemsetAsync(d_tot.as<uint32_t>() + 19, 0, 4, s));   // (the row count's high word)
      }
      if (defer) {
        defer->push_back(d_ca);
      } else {
        switch (ca.nch) {
          case 1: callwin_direct<1>(d_ca, ncalls, call, region); break;
          case 2: callwin_direct<2>(d_ca, ncalls, call, region); break;
          case 3: callwin_direct<3>(d_ca, ncalls, call, region); break;
          default: callwin_direct<4>(d_ca, ncalls, call, region); break;
        }
      }
    } else {
      switch (ca.nch) {
        case 1: callwin_launch<1>(d_ca, ncalls, call, region); break;
        case 2: callwin_launch<2>(d_ca, ncalls, call, region); break;
        case 3: callwin_launch<3>(d_ca, ncalls, call, region); break;
        default: callwin_launch<4>(d_ca, ncalls, call, region); break;
      }
    }
    SHD_HIP(hipMemcpyAsync(h_tot.as<uint64_t>() + 9, d_tot.as<uint64_t>() + 9, 8, hipMemcpyDeviceToHost, s));
    mark("call_window");
    // the group tables: the window state after the push.  Only groups of the
    // carried items (the state before the push) and of the final window can
    // hold a non-empty state: those are reset, then the final window adds in
    if (C > 0) {
      hipLaunchKernelGGL(k_cw_gtables<false>, dim3(grid_for(C)), dim3(kBlock), 0, s, d_ca, (int64_t)0, C);
      SHD_CHECK_LAUNCH();
    }
    if (total > X) {
      hipLaunchKernelGGL(k_cw_gtables<false>, dim3(grid_for(total - X)), dim3(kBlock), 0, s, d_ca, X, total);
      SHD_CHECK_LAUNCH();
    }
    if (total > X) {
      hipLaunchKernelGGL(k_cw_gtables<true>, dim3(grid_for(total - X)), dim3(kBlock), 0, s, d_ca, X, total);
      SHD_CHECK_LAUNCH();
    }
    mark("group_tables");
    if (defer && !defer->empty() && defer->back() == d_ca) return;
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t nrows = m > 0 ? (int64_t)h_tot.as<uint64_t>()[9] : 0;
    q.out.count += nrows;
    q.counters.matches += nrows;
  }

  // One launch of the direct-mapped rows kernel for a window group's members
  // (callwin_rows with `defer`): their arguments must lie at a fixed stride in
  // the argument arena (consecutive dev_args of one type).
  void callwin_direct_multi(const std::vector<const CwArgs*>& args, int nch, int64_t ncalls, uint32_t call,
                            uint32_t region) {
    const int nm = (int)args.size();
    const int64_t stride = nm > 1 ? (const char*)args[1] - (const char*)args[0] : 0;
    for (int k = 1; k < nm; k++)
      if ((const char*)args[k] - (const char*)args[0] != k * stride)
        throw Error(SHD_E_DEVICE, "window group: member arguments not at a fixed stride");
    const dim3 g((unsigned)(ceil_div(ncalls, 8) * 8 * nm)), bl(kBlock);
    const uint32_t* base = d_cw_base.as<uint32_t>();
    const char* a0 = (const char*)args[0];
#define SHD_CW_MULTI(NC, RC, CC)                                                                                    \
  hipLaunchKernelGGL((k_cw_direct_multi<NC, RC, CC, kCwDirectG, true>), g, bl, 0, stream, a0, stride, nm, (int)ncalls, \
                     base)
#define SHD_CW_MULTI_NC(NC)                                                   \
  do {                                                                        \
    if (region <= 2048 && call <= 512) SHD_CW_MULTI(NC, 2048, 512);           \
    else if (region <= 2048) SHD_CW_MULTI(NC, 2048, kCwCall);                 \
    else SHD_CW_MULTI(NC, kCwRegionMax, kCwCall);                             \
  } while (0)
    switch (nch) {
      case 1: SHD_CW_MULTI_NC(1); break;
      case 2: SHD_CW_MULTI_NC(2); break;
      case 3: SHD_CW_MULTI_NC(3); break;
      default: SHD_CW_MULTI_NC(4); break;
    }
#undef SHD_CW_MULTI_NC
#undef SHD_CW_MULTI
    SHD_CHECK_LAUNCH();
  }

  void agg_segscan(int64_t total, uint64_t kmax, int64_t cap) {
    hipStream_t s = stream;
    okey32.reserve(total * 4);
    okey32_alt.reserve(total * 4);
    oref.reserve(total * 4);
    oref_alt.reserve(total * 4);
    hipLaunchKernelGGL(k_narrow, dim3(grid_for(total)), dim3(kBlock), 0, s, (const uint64_t*)ikey[cur].as<uint64_t>(),
                       okey32.as<uint32_t>(), total);
    SHD_CHECK_LAUNCH();
    fill_iota_u32(oref.as<uint32_t>(), total, 0, s);
    int bits = 0;
    while (bits < 32 && (kmax >> bits)) bits++;
    bool in_alt = false;
    radix_sort_pairs_u32(okey32.as<uint32_t>(), oref.as<uint32_t>(), okey32_alt.as<uint32_t>(),
                         oref_alt.as<uint32_t>(), total, bits, d_sort, s, in_alt);
    const uint32_t* sk = in_alt ? okey32_alt.as<uint32_t>() : okey32.as<uint32_t>();
    const uint32_t* sp = in_alt ? oref_alt.as<uint32_t>() : oref.as<uint32_t>();
    mark("group_sort");
    SegArgs sa{};
    sa.nch = std::max(nch, 1);
    for (int c = 0; c < sa.nch; c++) {
      sa.ch_agg[c] = nch ? ch_agg[c] : 0;
      sa.ch_type[c] = nch ? ch_type[c] : SHD_T_DOUBLE;
    }
    sa.nagg = nagg;
    for (int g = 0; g < nagg; g++) {
      sa.kind[g] = plan.aggs[g].kind;
      sa.type[g] = plan.aggs[g].type;
      sa.chan[g] = chan_of[g];
    }
    sa.cap = cap;
    sa.C = C;
    sa.total = total;
    sa.dsum = g_dsum.as<double>();
    sa.cnt = g_cnt.as<int64_t>();
    sa.nkeys = g_nkeys;
    const SegArgs* d_sa = dev_args(sa);
    switch (sa.nch) {
      case 1: segscan_kernels<1>(total, sk, sp, d_sa, cap); break;
      case 2: segscan_kernels<2>(total, sk, sp, d_sa, cap); break;
      case 3: segscan_kernels<3>(total, sk, sp, d_sa, cap); break;
      default: segscan_kernels<4>(total, sk, sp, d_sa, cap); break;
    }
  }

  // the item slot `cur` holds the carry [0, C) and room for `total` items
  void grow_items(int64_t total) {
    hipStream_t s = stream;
    if (total >= (int64_t)INT32_MAX) throw Error(SHD_E_CAPACITY, "window items exceed 2^31");
    if (icap[cur] < total) {
      int old = cur, nw = cur ^ 1;
      ensure_items(nw, total);
      if (C > 0) {
        SHD_HIP(hipMemcpyAsync(ikey[nw].p, ikey[old].p, C * 8, hipMemcpyDeviceToDevice, s));
        SHD_HIP(hipMemcpyAsync(its[nw].p, its[old].p, C * 8, hipMemcpyDeviceToDevice, s));
        for (int g = 0; g < nagg; g++) {
          SHD_HIP(hipMemcpyAsync(iargv[nw].as<uint64_t>() + g * icap[nw], iargv[old].as<uint64_t>() + g * icap[old],
                                 C * 8, hipMemcpyDeviceToDevice, s));
          SHD_HIP(hipMemcpyAsync(iargn[nw].as<uint8_t>() + g * icap[nw], iargn[old].as<uint8_t>() + g * icap[old], C,
                                 hipMemcpyDeviceToDevice, s));
        }
      }
      cur = nw;
    }
    const int64_t cap = icap[cur];
    ievrow.reserve(cap * 4);
    icall.reserve(cap * 4);
    inow.reserve(cap * 8);
  }

  // gstride: words per group attribute of the dictionary-mode key arrays (>= new items)
  ItemArgs item_args(const Staged& b, int64_t gstride) {
    ItemArgs ia{};
    ia.cs = b.cs;
    ia.es = dset();
    ia.nagg = nagg;
    for (int g = 0; g < nagg; g++) {
      ia.has_arg[g] = plan.aggs[g].expr >= 0;
      ia.arg_col[g] = -1;
      if (ia.has_arg[g]) {
        ia.agg_arg[g] = dexpr(plan.aggs[g].expr);
        if (!getenv("SHD_NO_FAST_OUT")) ia.arg_col[g] = plain_load_attr(plan, plan.aggs[g].expr);
      }
    }
    ia.ngroup = ngk;
    for (int g = 0; g < ngk; g++) {
      ia.group[g] = dexpr(gk_expr[g]);
      ia.group_col[g] = gk_col[g];
      ia.group_type[g] = gk_type[g];
    }
    ia.dense = gdense;
    ia.null_str_id = plan.null_str_id;
    if (ngk && !gdense) {
      g_kw.reserve((size_t)ngk * gstride * 8);
      g_kn.reserve(gstride);
      g_h.reserve(gstride * 8);
      ia.gkw = g_kw.as<uint64_t>();
      ia.gkn = g_kn.as<uint8_t>();
      ia.gh = g_h.as<uint64_t>();
      ia.gstride = gstride;
    }
    ia.C = C;
    ia.time_window = wkind == SHD_W_TIME;
    return ia;
  }

  void push_agg(const Staged& b, int64_t ncalls, int64_t n) {
    hipStream_t s = stream;
    SHD_HIP(hipMemcpyAsync(h_tot.p, d_tot.p, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t m = h_tot.as<uint32_t>()[0];
    SHD_HIP(hipMemsetAsync(d_tot.as<uint64_t>() + 5, 0, 8, s));
    SHD_HIP(hipMemsetAsync(d_tot.as<uint64_t>() + 6, 0xFF, 8, s));
    // items: carry slot `cur` already holds [0, C); build the new item set in slot `cur`
    grow_items(C + m);
    const int64_t cap = icap[cur];
    const ItemArgs ia = item_args(b, std::max<int64_t>(m, 1));
    hipLaunchKernelGGL(k_make_items, dim3(grid_cover(n)), dim3(kBlock), 0, s, dev_args(ia), n,
                       (const uint32_t*)d_cnt.as<uint32_t>(), (const uint32_t*)d_off.as<uint32_t>(),
                       (const int32_t*)d_call_of.as<int32_t>(), (const int64_t*)d_now.as<int64_t>(),
                       ikey[cur].as<uint64_t>(), its[cur].as<int64_t>(), iargv[cur].as<uint64_t>(),
                       iargn[cur].as<uint8_t>(), ievrow.as<int32_t>(), icall.as<int32_t>(), inow.as<int64_t>(), cap,
                       (uint32_t*)(d_tot.as<uint64_t>() + 5));
    SHD_CHECK_LAUNCH();
    if (ngk && !gdense) gdict_assign(m, std::max<int64_t>(m, 1));
    mark("window_items");
    push_agg_tail(b, ncalls, n, m, false);
  }

  // filter + items in one pass (k_filter_items); the item arrays are sized
  // for every event passing
  DevBuf d_fi_status;
  void push_agg_fused(const Staged& b, int64_t ncalls, int64_t n, const FilterArgs& fa) {
    hipStream_t s = stream;
    grow_items(C + n);
    const int64_t cap = icap[cur];
    FusedArgs fu{};
    fu.f = fa;
    fu.it = item_args(b, std::max<int64_t>(n, 1));
    fu.call_of = d_call_of.as<int32_t>();
    fu.call_now = d_now.as<int64_t>();
    fu.ikey = ikey[cur].as<uint64_t>();
    fu.its = its[cur].as<int64_t>();
    fu.iargv = iargv[cur].as<uint64_t>();
    fu.iargn = iargn[cur].as<uint8_t>();
    fu.ievrow = ievrow.as<int32_t>();
    fu.icall = icall.as<int32_t>();
    fu.inow = inow.as<int64_t>();
    fu.cap = cap;
    const int64_t ntiles = ceil_div(n, kFiTile);
    d_fi_status.reserve((size_t)ntiles * 8);
    SHD_HIP(hipMemsetAsync(d_fi_status.p, 0, (size_t)ntiles * 8, s));
    fu.status = d_fi_status.as<uint64_t>();
    d_cw_citem.reserve((size_t)(ncalls + 1) * 4);
    fu.citem = d_cw_citem.as<uint32_t>();
    fu.ncalls = (int)ncalls;
    fu.m_out = (uint32_t*)d_tot.p;
    SHD_HIP(hipMemsetAsync(d_tot.as<uint64_t>() + 2, 0, 8, s));
    fu.kmax_out = (unsigned long long*)(d_tot.as<uint64_t>() + 2);
    SHD_HIP(hipMemsetAsync(d_tot.as<uint64_t>() + 5, 0, 8, s));
    SHD_HIP(hipMemsetAsync(d_tot.as<uint64_t>() + 6, 0xFF, 8, s));
    fu.nch = seg_mode ? nch : 0;
    for (int c = 0; c < nch; c++) {
      fu.ch_agg[c] = ch_agg[c];
      fu.ch_t[c] = ch_type[c];
    }
    fu.opstats = (uint32_t*)(d_tot.as<uint64_t>() + 5);
    hipLaunchKernelGGL(k_filter_items, dim3((unsigned)ntiles), dim3(kBlock), 0, s, dev_args(fu), n);
    SHD_CHECK_LAUNCH();
    SHD_HIP(hipMemcpyAsync(h_tot.p, d_tot.p, 24, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t m = h_tot.as<uint32_t>()[0];
    fused_kmax = h_tot.as<uint64_t>()[2];
    if (ngk && !gdense) gdict_assign(m, std::max<int64_t>(n, 1));
    mark("filter_items");
    push_agg_tail(b, ncalls, n, m, true);
  }
  uint64_t fused_kmax = 0;     // largest group id of the push's new items (dense ids)
  uint64_t kmax_seen = 0;      // largest dense group id since reset (an upper bound of the carried ones)
  bool kmax_known = true;      // false after a restore: one reduction over the items

  void push_agg_tail(const Staged& b, int64_t ncalls, int64_t n, int64_t m, bool fused) {
    hipStream_t s = stream;
    const int64_t total = C + m;
    const int64_t cap = icap[cur];
    // expiry positions.  A length window's are x + L (kInf past the items):
    // X = max(0, total - L) expire, and e is only materialised for the paths
    // that read it (not the call-window path)
    e_exp.reserve(std::max<int64_t>(total, 1) * 4);
    const bool len_win = wkind == SHD_W_LENGTH;
    bool e_ready = false;
    auto make_expiry = [&]() {
      hipLaunchKernelGGL(k_expiry, dim3(grid_for(total)), dim3(kBlock), 0, s, wkind, wparam, C, total,
                         (const int64_t*)its[cur].as<int64_t>(), (const int64_t*)inow.as<int64_t>(),
                         e_exp.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      if (wkind == SHD_W_TIME) {
        if (total <= (int64_t)kPmaxTile * 8) {
          hipLaunchKernelGGL(k_prefix_max_u32, dim3(1), dim3(kBlock), 0, s, e_exp.as<uint32_t>(), total);
          SHD_CHECK_LAUNCH();
        } else {
          const int64_t nt = ceil_div(total, kPmaxTile);
          d_pmax.reserve(nt * 4);
          hipLaunchKernelGGL(k_pmax_tiles, dim3((unsigned)nt), dim3(kBlock), 0, s,
                             (const uint32_t*)e_exp.as<uint32_t>(), total, d_pmax.as<uint32_t>());
          SHD_CHECK_LAUNCH();
          hipLaunchKernelGGL(k_pmax_scan, dim3(1), dim3(kBlock), 0, s, d_pmax.as<uint32_t>(), nt);
          SHD_CHECK_LAUNCH();
          hipLaunchKernelGGL(k_pmax_apply, dim3((unsigned)nt), dim3(kBlock), 0, s, e_exp.as<uint32_t>(), total,
                             (const uint32_t*)d_pmax.as<uint32_t>());
          SHD_CHECK_LAUNCH();
        }
      }
      e_ready = true;
    };
    unsigned long long* d_x = (unsigned long long*)(d_tot.as<uint64_t>() + 1);
    uint64_t* d_kmax = d_tot.as<uint64_t>() + 2;
    if (!len_win) {
      make_expiry();
      SHD_HIP(hipMemsetAsync(d_x, 0, 8, s));
      hipLaunchKernelGGL(k_count_expired, dim3(grid_for(total, 4, 2048)), dim3(kBlock), 0, s,
                         (const uint32_t*)e_exp.as<uint32_t>(), total, d_x);
      SHD_CHECK_LAUNCH();
    }
    // the largest group id: dense ids of a fused push come from k_filter_items
    // (carried ids are bounded by the running maximum)
    const bool kmax_fused = fused && (gdense || ngk == 0) && kmax_known;
    if (!kmax_fused) reduce_max_u64(ikey[cur].as<uint64_t>(), total, d_kmax, s);
    const bool guard = seg_mode && nch > 0 && m > 0;
    if (guard && !fused) {
      d_chmeta.reserve(2 * kMaxChan * sizeof(int));
      int meta[2 * kMaxChan];
      for (int c = 0; c < nch; c++) {
        meta[c] = ch_agg[c];
        meta[kMaxChan + c] = ch_type[c];
      }
      h_chmeta.reserve(sizeof(meta));
      std::memcpy(h_chmeta.p, meta, sizeof(meta));
      SHD_HIP(hipMemcpyAsync(d_chmeta.p, h_chmeta.p, sizeof(meta), hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_operand_stats, dim3((unsigned)std::min<int64_t>(1024, ceil_div(m, kBlock))), dim3(kBlock), 0,
                         s, (const uint64_t*)iargv[cur].as<uint64_t>(), (const uint8_t*)iargn[cur].as<uint8_t>(), cap,
                         C, m, nch, (const int*)d_chmeta.as<int>(), (const int*)d_chmeta.as<int>() + kMaxChan,
                         (uint32_t*)(d_tot.as<uint64_t>() + 5));
      SHD_CHECK_LAUNCH();
    }
    const bool cw_cand = callwin_candidate(ncalls, total);
    if (cw_cand) {
      d_cw_citem.reserve((size_t)(ncalls + 1) * 4);
      d_cw_clb.reserve((size_t)std::max<int64_t>(ncalls, 1) * 4);
      SHD_HIP(hipMemsetAsync(d_tot.as<uint64_t>() + 8, 0, 8, s));
      if (!fused) {   // (k_filter_items wrote them)
        hipLaunchKernelGGL(k_cw_citem, dim3(grid_for(ncalls + 1)), dim3(kBlock), 0, s,
                           (const int64_t*)d_offs.as<int64_t>(), (const uint32_t*)d_off.as<uint32_t>(), n, m, C,
                           (int)ncalls, d_cw_citem.as<uint32_t>());
        SHD_CHECK_LAUNCH();
      }
      hipLaunchKernelGGL(k_cw_regions, dim3(grid_for(ncalls)), dim3(kBlock), 0, s,
                         (const uint32_t*)e_exp.as<uint32_t>(), len_win ? wparam : (int64_t)0,
                         (const uint32_t*)d_cw_citem.as<uint32_t>(), (int)ncalls, d_cw_clb.as<uint32_t>(),
                         (uint32_t*)(d_tot.as<uint64_t>() + 8));
      SHD_CHECK_LAUNCH();
    }
    SHD_HIP(hipMemcpyAsync(h_tot.p, d_tot.p, 72, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t X = len_win ? std::max<int64_t>(0, total - wparam) : (int64_t)h_tot.as<uint64_t>()[1];
    uint64_t kmax = h_tot.as<uint64_t>()[2];
    if (kmax_fused) kmax = std::max(kmax_seen, fused_kmax);
    kmax_seen = std::max(kmax_seen, kmax);
    kmax_known = true;
    const uint32_t cw_call = cw_cand ? h_tot.as<uint32_t>()[16] : 0u;
    const uint32_t cw_region = cw_cand ? h_tot.as<uint32_t>()[17] : 0u;
    if (guard) {
      // Segmented scans reassociate the reference's running `sum += v; sum -= v`
      // (SumAttributeAggregatorExecutor.java:184-198).  With a non-finite
      // operand the reference's sum stays Inf / NaN for good (Inf - Inf), and
      // over a wide magnitude range its rounding history shows in the result
      // (1e20 + 1 - 1e20 = 0), as it does when operands of both signs cancel
      // (1e6 + 1e-3 - 1e6): from the first such push on, this query keeps the
      // bit-exact sequential fold (the group tables carry over).
      // the span and the signs are over every operand since reset (window
      // items of earlier pushes included), not just this push's
      const uint32_t* fl = h_tot.as<uint32_t>() + 10;
      op_emax = std::max(op_emax, fl[1]);
      op_emin = std::min(op_emin, fl[2]);
      op_signs |= fl[0] & (kOpNeg | kOpPos);
      const bool wide = op_emin != 0xFFFFFFFFu && op_emax > op_emin + kSegMaxExpSpan;
      const bool mixed = (op_signs & (kOpNeg | kOpPos)) == (kOpNeg | kOpPos);
      if ((fl[0] & 1u) || wide || mixed) {
        seg_mode = false;
        seg_unsafe = true;
      }
    }
    if ((int64_t)kmax >= kMaxDenseKey)   // dense string ids: more than 2^26 distinct strings
      throw Error(SHD_E_CAPACITY, "more than 2^26 group-by keys in the dense group tables");
    ensure_groups((int64_t)kmax + 1);
    const int64_t nops = m + X;
    if (!wmembers.empty()) {   // a window group's leader: its members' rows from these items, no rows of its own
      // the shared call-window pass needs the segmented scans' operand range
      // and the call-window shape; otherwise the group dissolves before this
      // push changes anything the members read: each member takes its window
      // (a suffix of the carried items) and runs this push and every later
      // one alone (shd_group_push, group_dissolve)
      if (!seg_mode)
        throw NeedDissolve("query group: an operand outside the segmented scans' range (non-finite, magnitudes "
                           "spanning more than 2^30, or of both signs)");
      if (!(cw_cand && cw_call <= (uint32_t)kCwCall && cw_region <= (uint32_t)kCwRegionMax))
        throw NeedDissolve("query group: a call above 1024 events or a window beyond the call-window path");
      // direct-mapped group ids: one rows kernel for all members (they share
      // the calls' row counts); hashed ids: a launch per member
      const bool multi = kmax < (uint64_t)kCwDirectG && !getenv("SHD_CW_HASH") && !getenv("SHD_CW_NO_MULTI") &&
                         wkind == SHD_W_LENGTH;
      std::vector<const CwArgs*> margs;
      int mnch = 1;
      for (size_t k = 0; k < wmembers.size(); k++) {
        SingleEngine& q = *wmembers[k];
        const int64_t Xq = std::max<int64_t>(0, total - q.wparam);
        callwin_rows(q, b, total, cap, ncalls, Xq, cw_call, cw_region, kmax, k == 0, multi ? &margs : nullptr);
        mnch = std::max(mnch, std::max(q.nch, 1));
        q.counters.events += n;
        q.counters.carry = total - Xq;
        q.chunk_seq += ncalls;
        q.seq += n;
      }
      if (multi && !margs.empty()) {
        callwin_direct_multi(margs, mnch, ncalls, cw_call, cw_region);
        SHD_HIP(hipStreamSynchronize(stream));
        const int64_t nrows = m > 0 ? (int64_t)h_tot.as<uint64_t>()[9] : 0;
        for (auto* qp : wmembers) {
          qp->out.count += nrows;
          qp->counters.matches += nrows;
        }
      }
      mark("members");
      commit_carry(total, X, nops, ncalls);
      return;
    }
    if (!seg_mode) {   // (segmented-scan mode: packed run records instead)
      resv.reserve(std::max(nagg, 1) * cap * 8);
      resc.reserve(std::max(nagg, 1) * cap * 8);
      resn.reserve(std::max(nagg, 1) * cap);
      last_of.reserve(cap * 4);
    }
    // (a range-guard trip above cleared seg_mode: that push folds exactly)
    const bool use_cw = seg_mode && total > 0 && cw_cand && cw_call <= (uint32_t)kCwCall &&
                        cw_region <= (uint32_t)kCwRegionMax;
    bool emitted = false;
    if (!use_cw && !e_ready) make_expiry();
    first.reserve(cap);
    if (total > 0 && !use_cw) SHD_HIP(hipMemsetAsync(first.p, 0, total, s));
    if (use_cw) {
      agg_callwin(b, total, cap, ncalls, X, cw_call, cw_region, kmax);
      emitted = true;
    } else if (seg_mode && total > 0) {
      if (!agg_chunked(total, kmax, cap, ncalls)) agg_segscan(total, kmax, cap);
    } else if (nops > 0) {
      okey.reserve(nops * 8);
      oref.reserve(nops * 4);
      hipLaunchKernelGGL(k_make_ops, dim3(grid_for(total)), dim3(kBlock), 0, s, C, total,
                         (const uint32_t*)e_exp.as<uint32_t>(), (const uint64_t*)ikey[cur].as<uint64_t>(),
                         okey.as<uint64_t>(), oref.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      // stable key sort of the operation stream (op order kept inside a group)
      okey32.reserve(nops * 4);
      okey32_alt.reserve(nops * 4);
      oref_alt.reserve(nops * 4);
      hipLaunchKernelGGL(k_narrow, dim3(grid_for(nops)), dim3(kBlock), 0, s, (const uint64_t*)okey.as<uint64_t>(),
                         okey32.as<uint32_t>(), nops);
      SHD_CHECK_LAUNCH();
      int bits = 0;
      while (bits < 32 && (kmax >> bits)) bits++;
      bool in_alt = false;
      radix_sort_pairs_u32(okey32.as<uint32_t>(), oref.as<uint32_t>(), okey32_alt.as<uint32_t>(),
                           oref_alt.as<uint32_t>(), nops, bits, d_sort, s, in_alt);
      const uint32_t* sk = in_alt ? okey32_alt.as<uint32_t>() : okey32.as<uint32_t>();
      const uint32_t* sr = in_alt ? oref_alt.as<uint32_t>() : oref.as<uint32_t>();
      mark("group_sort");
      heads.reserve(nops * 4);
      hoff.reserve(nops * 4);
      hipLaunchKernelGGL(k_seg_heads, dim3(grid_for(nops)), dim3(kBlock), 0, s, sk, nops, heads.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      uint32_t* d_h = (uint32_t*)(d_tot.as<uint64_t>() + 3);
      scan_exclusive_u32(heads.as<uint32_t>(), hoff.as<uint32_t>(), nops, d_h, d_scan, s);
      SHD_HIP(hipMemcpyAsync(h_tot.as<uint64_t>() + 3, d_h, 4, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
      const int64_t nheads = h_tot.as<uint32_t>()[6];
      hlist.reserve(std::max<int64_t>(nheads, 1) * 4);
      hipLaunchKernelGGL(k_head_list, dim3(grid_for(nops)), dim3(kBlock), 0, s, (const uint32_t*)heads.as<uint32_t>(),
                         (const uint32_t*)hoff.as<uint32_t>(), nops, hlist.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      FoldArgs fo{};
      fo.nagg = nagg;
      for (int g = 0; g < nagg; g++) {
        fo.kind[g] = plan.aggs[g].kind;
        fo.type[g] = plan.aggs[g].type;
      }
      fo.cap = cap;
      fo.dsum = g_dsum.as<double>();
      fo.lsum = g_lsum.as<int64_t>();
      fo.cnt = g_cnt.as<int64_t>();
      fo.nkeys = g_nkeys;
      const FoldArgs* d_fo = dev_args(fo);
      // long group segments: one wave per group (coalesced operand loads,
      // wave-uniform fold); short ones: one lane per group
      const bool wave = nops >= 256 * nheads && !getenv("SHD_FOLD_LANE");
#define SHD_FOLD_ARGS                                                                                           \
  d_fo, (const uint32_t*)hlist.as<uint32_t>(), nheads, nops, sk, sr, (const uint64_t*)iargv[cur].as<uint64_t>(), \
      (const uint8_t*)iargn[cur].as<uint8_t>(), (const int32_t*)ievrow.as<int32_t>(),                            \
      (const int32_t*)d_call_of.as<int32_t>(), resv.as<uint64_t>(), resn.as<uint8_t>(), resc.as<int64_t>(),     \
      first.as<uint8_t>(), last_of.as<uint32_t>()
      // aggregators with a double running sum + count only: the branch-light fold
      bool dfam = nagg >= 1 && nagg <= 4 && !getenv("SHD_FOLD_GENERIC");
      for (int g = 0; g < nagg; g++) {
        const int k = plan.aggs[g].kind, t = plan.aggs[g].type;
        dfam = dfam && (k == SHD_AGG_COUNT || k == SHD_AGG_AVG ||
                        (k == SHD_AGG_SUM && (t == SHD_T_DOUBLE || t == SHD_T_FLOAT)));
      }
      if (wave && dfam) {
        const dim3 gw((unsigned)ceil_div(nheads * 64, kBlock));
        switch (nagg) {
          case 1: hipLaunchKernelGGL(k_fold_wave_d<1>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          case 2: hipLaunchKernelGGL(k_fold_wave_d<2>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          case 3: hipLaunchKernelGGL(k_fold_wave_d<3>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          default: hipLaunchKernelGGL(k_fold_wave_d<4>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
        }
      } else if (wave) {
        const dim3 gw((unsigned)ceil_div(nheads * 64, kBlock));
        switch (nagg) {
          case 1: hipLaunchKernelGGL(k_fold_wave<1>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          case 2: hipLaunchKernelGGL(k_fold_wave<2>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          case 3: hipLaunchKernelGGL(k_fold_wave<3>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          case 4: hipLaunchKernelGGL(k_fold_wave<4>, gw, dim3(kBlock), 0, s, SHD_FOLD_ARGS); break;
          default:
            hipLaunchKernelGGL(k_fold, dim3(grid_for(nheads)), dim3(kBlock), 0, s, SHD_FOLD_ARGS);
        }
      } else {
        hipLaunchKernelGGL(k_fold, dim3(grid_for(nheads)), dim3(kBlock), 0, s, SHD_FOLD_ARGS);
      }
#undef SHD_FOLD_ARGS
      SHD_CHECK_LAUNCH();
      mark("group_fold");
    }
    // emission: first-seen (call, group) rows in event order
    if (m > 0 && !emitted) emit_rows(b, m, cap);
    commit_carry(total, X, nops, ncalls);
  }

  // carry: the unexpired suffix [X, total) becomes the new window contents
  void commit_carry(int64_t total, int64_t X, int64_t nops, int64_t ncalls) {
    hipStream_t s = stream;
    int64_t keep = wkind == 0 ? 0 : total - X;
    if (keep > 0 && X > 0) {
      int nw = cur ^ 1;
      ensure_items(nw, keep);
      SHD_HIP(hipMemcpyAsync(ikey[nw].p, ikey[cur].as<uint64_t>() + X, keep * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(its[nw].p, its[cur].as<int64_t>() + X, keep * 8, hipMemcpyDeviceToDevice, s));
      for (int g = 0; g < nagg; g++) {
        SHD_HIP(hipMemcpyAsync(iargv[nw].as<uint64_t>() + g * icap[nw], iargv[cur].as<uint64_t>() + g * icap[cur] + X,
                               keep * 8, hipMemcpyDeviceToDevice, s));
        SHD_HIP(hipMemcpyAsync(iargn[nw].as<uint8_t>() + g * icap[nw], iargn[cur].as<uint8_t>() + g * icap[cur] + X,
                               keep, hipMemcpyDeviceToDevice, s));
      }
      cur = nw;
    }
    C = keep;
    counters.carry = C;
    counters.partial_scans += nops;
    chunk_seq += ncalls;
  }
};

std::unique_ptr<Engine> make_single_engine(const Plan& p, std::string& why) {
  if (p.kind != SHD_KIND_SINGLE) { why = "not a single-stream query"; return nullptr; }
  auto e = std::make_unique<SingleEngine>();
  e->types = p.stream_types[p.single_stream];
  if (e->types.size() > (size_t)kMaxCols) { why = "too many attributes"; return nullptr; }
  bool seen_window = false;
  for (auto& h : p.handlers) {
    if (h.kind == SHD_H_FILTER) {
      if (seen_window) { why = "filter after window"; return nullptr; }
      e->filters.push_back(h.expr);
    } else {
      seen_window = true;
      e->wkind = h.wkind;
      e->wparam = h.param;
    }
  }
  if (e->filters.size() > 4) { why = "too many filters"; return nullptr; }
  for (auto& o : p.outputs) e->outs.push_back(o.second);
  if (e->outs.size() > (size_t)kMaxCols) { why = "too many outputs"; return nullptr; }
  e->nagg = (int)p.aggs.size();
  if (e->nagg > kMaxAggs) { why = "too many aggregators"; return nullptr; }
  e->partitioned = !p.part_keys.empty();
  bool needs_agg = e->nagg > 0 || !p.group_by.empty();
  // batch windows (flush chunks with RESET) and timeLength: the window-x engine
  if (e->wkind == SHD_W_LENGTH_BATCH || e->wkind == SHD_W_TIME_BATCH || e->wkind == SHD_W_TIME_LENGTH ||
      e->wkind == SHD_W_EXTERNAL_TIME || e->wkind == SHD_W_TIME_BATCH_STREAM)
    return make_window_x_engine(p, why);
  // EXPIRED output, `having`, no CURRENT output, aggregation inside a
  // partition: the keyed exact window engine (engine_window.hip)
  if ((p.expired_on && (needs_agg || e->wkind != 0)) || p.having >= 0 || !p.current_on ||
      (!p.part_keys.empty() && (needs_agg || (e->wkind != 0 && p.expired_on))))
    return make_window_x_engine(p, why);
  if (e->wkind != 0 && e->wparam <= 0 && e->wkind == SHD_W_LENGTH) { why = "length(0) window"; return nullptr; }
  e->agg_mode = needs_agg;
  // segmented-scan aggregation: count(), sum(double|float), avg(numeric); one
  // channel per distinct argument expression (avg(price) and sum(price) share one)
  bool seg = e->agg_mode && e->nagg >= 1;
  for (int g = 0; g < e->nagg && seg; g++) {
    const auto& a = p.aggs[g];
    if (a.kind == SHD_AGG_COUNT) { e->chan_of[g] = -1; continue; }
    if (a.kind == SHD_AGG_SUM && a.type != SHD_T_DOUBLE && a.type != SHD_T_FLOAT) { seg = false; break; }
    if (a.kind != SHD_AGG_SUM && a.kind != SHD_AGG_AVG) { seg = false; break; }
    if (a.expr < 0) { seg = false; break; }
    int c = -1;
    for (int k = 0; k < e->nch && c < 0; k++) {
      const auto& x = p.exprs[p.aggs[e->ch_agg[k]].expr];
      const auto& y = p.exprs[a.expr];
      bool same = x.size() == y.size() && e->ch_type[k] == a.type;
      for (size_t i = 0; same && i < x.size(); i++)
        same = x[i].op == y[i].op && x[i].a == y[i].a && x[i].b == y[i].b && x[i].c == y[i].c;
      if (same) c = k;
    }
    if (c < 0) {
      if (e->nch == kMaxChan) { seg = false; break; }
      c = e->nch++;
      e->ch_agg[c] = g;
      e->ch_type[c] = a.type;
    }
    e->chan_of[g] = c;
  }
  e->seg_ok = seg;
  e->seg_pref = !getenv("SHD_EXACT_AGGREGATES");
  e->seg_mode = seg && e->seg_pref;
  if (e->partitioned) {
    e->key_expr = p.part_keys[0].second;
    e->key_col = plain_load_attr(p, e->key_expr);
    e->key_type = expr_result_type(p, e->key_expr, {});
  }
  if (p.group_by.size() > (size_t)kMaxGroupAttrs) { why = "more than 4 group-by attributes"; return nullptr; }
  e->ngk = (int)p.group_by.size();
  for (int g = 0; g < e->ngk; g++) {
    e->gk_expr[g] = p.group_by[g];
    e->gk_col[g] = plain_load_attr(p, e->gk_expr[g]);
    e->gk_type[g] = expr_result_type(p, e->gk_expr[g], {});
  }
  // dense ids: one string attribute (dictionary ids; null = the id of "null")
  // or one bool attribute (0, 1, null = 2); the group dictionary otherwise
  e->gdense = e->ngk == 1 && ((e->gk_type[0] == SHD_T_STRING && p.null_str_id >= 0) || e->gk_type[0] == SHD_T_BOOL);
  if (getenv("SHD_GROUP_DICT")) e->gdense = false;   // tests: dictionary path for every key
  return e;
}

}  // namespace shd
