// engine_window.hip -- keyed exact window engine ("window-x").
//
// Single-stream queries the segmented-scan engine (engine_single.hip) does
// not take: windows whose selector emits EXPIRED events (`insert all events` /
// `insert expired events`), and window / aggregate queries inside a
// `partition with (...)` block.  Reference semantics
// (modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/processor/stream/window/LengthWindowProcessor.java:105-142
//   query/processor/stream/window/TimeWindowProcessor.java:132-169 (+ state :196-222)
//   util/Scheduler.java:71-104,113-209 (TIMER events in playback: onTimeChange)
//   query/selector/QuerySelector.java:76-99 (process), :161-205 (processNoGroupBy),
//     :271-313 (processInBatchNoGroupBy), :315-373 (processInBatchGroupBy)
//   query/selector/attribute/aggregator/{Sum,Avg,Count}AttributeAggregatorExecutor.java
//   partition/PartitionStreamReceiver.java:175-216 (same-key runs = chunks)
//   util/snapshot/state/PartitionStateHolder.java:43-69 (state per (partition key,
//     group key); a window state is dropped when its queue empties)
//
// Formulation: every window item (a filtered, keyed event) lives in its
// partition key's FIFO.  Items of a push -- the carried FIFOs first, then the
// new items in arrival order -- are stable-sorted by partition key, so each key
// is one contiguous segment in FIFO order.  Each item gets its EXPIRY
// OPPORTUNITY: the add of a later item of its key (length: the L-th next item;
// time: the first later item whose call clock reaches ts + T) or a TIMER of its
// key at a time change; FIFO order makes the opportunities non-decreasing along
// a segment.  The reference's operation stream of one key -- at each
// opportunity its expirations (FIFO), then the add -- then has a closed-form
// position for every operation (counting by binary search inside the segment),
// so all operations of the push are written in key-major order in one pass.
// Aggregator states (dense ids of (partition key, group key), device group
// dictionary) are folded SEQUENTIALLY in that order (bit-exact add / remove,
// agg.h); output rows are the selector's per-chunk picks, ordered by (chunk,
// position) with a radix sort.
//
// Time windows with expired output need the Scheduler's TIMER events: a key's
// notify queue holds ts + T of every item that raised the key's last time
// (state.lastTimestamp); at a time change to `now` every key whose queue head
// is <= now gets one TIMER chunk that expires its FIFO prefix with ts + T <= now
// (emitted as its own callback chunk, before the call's events).  That part is
// inherently sequential per key: one lane per key segment walks its items and
// the push's clock moves (k_xw_time_lane); everything else is data-parallel.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <deque>
#include <cstdlib>

#include "engine.h"
#include "gdict.h"
#include "agg.h"

namespace shd {

namespace {

constexpr uint64_t kNoOpp = ~0ull;        // item does not expire in this push
constexpr uint32_t kNoTimer = 0xFFFFFFFFu;

// ---------------------------------------------------------------- contexts
// An event of the batch (filters, keys, aggregator arguments).
struct BatchCtx {
  const ColSet* cs;
  int64_t row;
  __device__ __forceinline__ Val load(int, int, int attr) const { return col_load(*cs, row, attr); }
  __device__ __forceinline__ bool evnull(int, int) const { return false; }
  __device__ __forceinline__ int64_t ts(int, int) const { return cs->ts[row]; }
  __device__ __forceinline__ Val agg(int) const { return Val{0, 1}; }
};

// A window item (attributes as 64-bit payloads) with the row's timestamp and
// aggregator values: selector outputs and `having`.
struct ItemCtx {
  const uint64_t* attr;   // [ncols][cap]
  const uint8_t* nul;
  int64_t cap;
  int64_t item;
  int ncols;
  int64_t tsv;            // the output event's timestamp (EXPIRED: the expiry time)
  const uint64_t* aggv;
  const uint8_t* aggn;
  __device__ __forceinline__ Val load(int, int, int a) const {
    if ((unsigned)a >= (unsigned)ncols) return Val{0, 1};
    return Val{attr[(int64_t)a * cap + item], (int)nul[(int64_t)a * cap + item]};
  }
  __device__ __forceinline__ bool evnull(int, int) const { return false; }
  __device__ __forceinline__ int64_t ts(int, int) const { return tsv; }
  __device__ __forceinline__ Val agg(int i) const { return Val{aggv[i], (int)aggn[i]}; }
};

__device__ __forceinline__ int64_t lower_bound_i64(const int64_t* a, int64_t lo, int64_t hi, int64_t v) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// ---------------------------------------------------------------- calls
// call_of[i] for every event; last_ts[c] (INT64_MIN for an empty call)
__global__ void k_xw_calls(const int64_t* offs, int ncalls, const int64_t* ts, int32_t* call_of, int64_t* last_ts) {
  const int c = blockIdx.x;
  if (c >= ncalls) return;
  const int64_t a = offs[c], b = offs[c + 1];
  for (int64_t i = a + threadIdx.x; i < b; i += kBlock) call_of[i] = c;
  if (threadIdx.x == 0) last_ts[c] = b > a ? ts[b - 1] : INT64_MIN;
}

// ---------------------------------------------------------------- items
struct XwArgs {
  ColSet cs;
  DExprSet es;
  DFilters filters;
  int partitioned;
  DExpr key;
  int key_col, key_type;
  int ngk;                          // group-by attributes
  DExpr group[kMaxGroupAttrs];
  int group_col[kMaxGroupAttrs];
  int group_type[kMaxGroupAttrs];
  int64_t null_str_id;
  int nagg;
  DExpr agg_arg[kMaxAggs];
  int has_arg[kMaxAggs];
  int ncols;
  int nw;                           // state key words (partition key + group words), 0 = one state
  int64_t C, cap, seq0;
};

// flags[i]: bit0 passes the filters, bit1 has a (non-null) partition key
__global__ __launch_bounds__(kBlock) void k_xw_filter(const XwArgs* __restrict__ ap, int64_t n, uint8_t* flags,
                                                      uint32_t* cnt, uint64_t* pkey) {
  const XwArgs& a = *ap;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    BatchCtx cx{&a.cs, i};
    uint8_t f = 0;
    uint64_t k = 0;
    bool keyed = true;
    if (a.partitioned) {
      Val kv = a.key_col >= 0 ? col_load(a.cs, i, a.key_col)
                              : eval_expr(a.es.ins + a.key.off, a.key.len, a.es.consts, cx);
      keyed = !kv.null;
      k = canon_key(kv, a.key_type);
    }
    if (keyed) {
      f |= 2;
      if (eval_filters(a.es, a.filters, cx)) f |= 1;
    }
    flags[i] = f;
    pkey[i] = k;
    cnt[i] = f == 3 ? 1u : 0u;
  }
}

// Partition runs (PartitionStreamReceiver.receive(Event[]) :189-214): a run
// starts at the first keyed event of a call or where the key changes.
__global__ __launch_bounds__(kBlock) void k_xw_run_starts(const uint8_t* flags, const uint64_t* pkey,
                                                          const int32_t* call_of, int64_t n, uint32_t* start) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    uint32_t s = 0;
    if (flags[i] & 2) {
      int64_t p = i - 1;
      while (p >= 0 && call_of[p] == call_of[i] && !(flags[p] & 2)) p--;
      s = (p < 0 || call_of[p] != call_of[i] || pkey[p] != pkey[i]) ? 1u : 0u;
    }
    start[i] = s;
  }
}

struct ItemOut {
  uint64_t* pk;
  int64_t* ts;
  int64_t* seq;
  int32_t* call;
  int32_t* row;
  uint64_t* attr;   // [ncols][cap]
  uint8_t* nul;
  uint64_t* argv;   // [nagg][cap]
  uint8_t* argn;
  uint64_t* kw;     // [nw][m] state key words of the new items
  uint8_t* kn;
  uint64_t* kh;
};

// New window items [C, C + m): one per passing event.
__global__ __launch_bounds__(kBlock) void k_xw_items(const XwArgs* __restrict__ ap, const ItemOut* __restrict__ op,
                                                     int64_t n, const uint32_t* cnt, const uint32_t* off,
                                                     const uint64_t* pkey, const int32_t* call_of, int64_t m) {
  const XwArgs& a = *ap;
  const ItemOut& o = *op;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    if (!cnt[i]) continue;
    const int64_t j = off[i];
    const int64_t t = a.C + j;
    BatchCtx cx{&a.cs, i};
    o.pk[t] = pkey[i];
    o.ts[t] = a.cs.ts[i];
    o.seq[t] = a.seq0 + i;
    o.call[t] = call_of[i];
    o.row[t] = (int32_t)i;
    for (int c = 0; c < a.ncols; c++) {
      Val v = col_load(a.cs, i, c);
      o.attr[(int64_t)c * a.cap + t] = v.b;
      o.nul[(int64_t)c * a.cap + t] = (uint8_t)v.null;
    }
    for (int g = 0; g < a.nagg; g++) {
      Val v{0, 1};
      if (a.has_arg[g]) v = eval_expr(a.es.ins + a.agg_arg[g].off, a.agg_arg[g].len, a.es.consts, cx);
      o.argv[(int64_t)g * a.cap + t] = v.b;
      o.argn[(int64_t)g * a.cap + t] = (uint8_t)v.null;
    }
    if (a.nw > 0) {
      // state key: (partition key, GroupByKeyGenerator words) -- gdict.h
      uint64_t h = kGdictSeed;
      uint8_t nm = 0;
      int w = 0;
      if (a.partitioned) {
        o.kw[j] = pkey[i];
        h = gdict_hash_step(h, pkey[i], w);
        w++;
      }
      for (int g = 0; g < a.ngk; g++, w++) {
        Val kv = a.group_col[g] >= 0 ? col_load(a.cs, i, a.group_col[g])
                                     : eval_expr(a.es.ins + a.group[g].off, a.group[g].len, a.es.consts, cx);
        bool isnull = false;
        const uint64_t gw = group_word(kv, a.group_type[g], a.null_str_id, isnull);
        o.kw[(int64_t)w * m + j] = gw;
        nm |= (uint8_t)((isnull ? 1u : 0u) << w);
        h = gdict_hash_step(h, gw, w);
      }
      h = gdict_hash_final(h, nm);
      o.kn[j] = nm;
      o.kh[j] = h;
    }
  }
}

// ---------------------------------------------------------------- segments
__global__ __launch_bounds__(kBlock) void k_xw_seg_heads(const uint64_t* spk, int64_t total, uint32_t* head) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total)
    head[j] = (j == 0 || spk[j] != spk[j - 1]) ? 1u : 0u;
}

// segS[k] = first sorted position of segment k; segid[j]
__global__ __launch_bounds__(kBlock) void k_xw_seg_list(const uint32_t* head, const uint32_t* hscan, int64_t total,
                                                        int64_t* segS, uint32_t* segid) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total) {
    const uint32_t k = hscan[j] + head[j] - 1;
    segid[j] = k;
    if (head[j]) segS[k] = j;
    if (j == total - 1) segS[k + 1] = total;
  }
}

// inclusive partition-run id of every keyed event, in place over the starts
__global__ __launch_bounds__(kBlock) void k_xw_run_ids(int64_t n, const uint32_t* run_excl, uint32_t* start_to_id) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n)
    start_to_id[i] = run_excl[i] + start_to_id[i] - 1u;
}

__global__ __launch_bounds__(kBlock) void k_xw_widen(const uint8_t* f, int64_t n, uint32_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) out[i] = f[i];
}

// Per segment: carried items at its front (ck), its pending notify entries
// [pA, pB) (pending keys sorted), the output room of its pending entries.
__global__ __launch_bounds__(kBlock) void k_xw_seg_info(int64_t nseg, const int64_t* segS, const uint32_t* sp,
                                                        int64_t C, const uint64_t* ipk, const uint64_t* ppk, int64_t np,
                                                        int64_t* segCk, int64_t* pA, int64_t* pB, uint32_t* proom) {
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < nseg; k = nseg) {
    const int64_t s = segS[k], e = segS[k + 1];
    int64_t lo = s, hi = e;   // first position holding a new item
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (sp[mid] < (uint32_t)C) lo = mid + 1;
      else hi = mid;
    }
    segCk[k] = lo - s;
    const uint64_t pk = ipk[sp[s]];
    int64_t a = 0, b = np;
    while (a < b) {
      const int64_t mid = (a + b) >> 1;
      if (ppk[mid] < pk) a = mid + 1;
      else b = mid;
    }
    int64_t c = a, d = np;
    while (c < d) {
      const int64_t mid = (c + d) >> 1;
      if (ppk[mid] <= pk) c = mid + 1;
      else d = mid;
    }
    pA[k] = a;
    pB[k] = c;
    proom[k] = (uint32_t)((c - a) + (e - s - (lo - s)));
  }
}

// ---------------------------------------------------------------- expiry
// length(L): item at segment rank r leaves at the add of rank r + L
// (LengthWindowProcessor :105-142; a carried FIFO holds at most L items).
__global__ __launch_bounds__(kBlock) void k_xw_len_expiry(int64_t total, int64_t L, const int64_t* segS,
                                                          const uint32_t* segid, const uint32_t* sp,
                                                          const int32_t* irow, uint64_t* eopp, uint32_t* etid) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total) {
    const int64_t e = segS[segid[j] + 1];
    uint64_t o = kNoOpp;
    if (j + L < e) o = 2ull * (uint64_t)irow[sp[j + L]] + 1ull;
    eopp[j] = o;
    etid[j] = kNoTimer;
  }
}

struct LaneArgs {
  int64_t nseg;
  const int64_t* segS;
  const int64_t* segCk;
  const int64_t* pA;
  const int64_t* pB;
  const uint32_t* proom_off;   // exclusive scan of the per-segment pending room
  const uint32_t* sp;
  const uint64_t* ipk;
  const int64_t* its;
  const int32_t* icall;
  const int32_t* irow;
  const int64_t* ilast;
  const int64_t* call_now;
  const int64_t* offs;
  const int32_t* F;            // firing calls (clock moves), ascending
  const int64_t* fnow;
  int nf;
  int64_t T;
  int64_t L;                   // timeLength: the length bound (0: time window)
  int ext_col;                 // externalTime: the item attribute holding its time (-1: the clock)
  const uint64_t* iattr;       // [ncols][cap]
  int64_t cap;
  int partitioned;
  int64_t last_global;         // unpartitioned: the window's lastTimestamp
  const int64_t* pv;           // pending notify values (sorted by key, then value)
  // outputs
  uint64_t* eopp;
  uint32_t* etid;
  uint8_t* rec;
  unsigned int* ntimer;
  int32_t* tF;
  int64_t* tHead;
  uint32_t* tSeg;
  uint64_t* pout_pk;
  int64_t* pout_v;
  uint32_t* pcnt;
  int64_t* last_out;
};

__device__ __forceinline__ int upper_bound_call(const int32_t* F, int lo, int hi, int32_t c) {
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (F[mid] <= c) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// One lane per key segment: TimeWindowProcessor.process over the key's items
// in arrival order, interleaved with the push's clock moves (Scheduler
// onTimeChange -> sendTimerEvents for the key when its notify head <= now).
__global__ __launch_bounds__(kBlock) void k_xw_time_lane(const LaneArgs* __restrict__ ap) {
  const LaneArgs& a = *ap;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < a.nseg; k = a.nseg) {
    const int64_t s = a.segS[k], e = a.segS[k + 1], ck = a.segCk[k];
    const int64_t pB = a.pB[k];
    int64_t pc = a.pA[k];
    const uint64_t pk = a.ipk[a.sp[s]];
    int64_t lastTs = a.partitioned ? (ck > 0 ? a.ilast[a.sp[s]] : INT64_MIN) : a.last_global;
    int64_t h = s;          // FIFO head
    int64_t rnext = -1;     // oldest unconsumed new notify entry (a record position)
    int fi = 0;
    for (int64_t j = s; j < s + ck; j++) a.rec[j] = 0;
    for (int64_t y = s + ck;; y++) {
      const int32_t cy = y < e ? a.icall[a.sp[y]] : 0x7FFFFFFF;
      // clock moves before item y (its call's setCurrentTimestamp comes first)
      while (fi < a.nf && a.F[fi] <= cy) {
        const int fe = upper_bound_call(a.F, fi, a.nf, cy);
        int64_t hv;
        if (pc < pB) hv = a.pv[pc];
        else if (rnext >= 0) hv = a.its[a.sp[rnext]] + a.T;
        else {
          fi = fe;
          break;
        }
        int lo = fi, hi = fe;   // first clock move reaching the head
        while (lo < hi) {
          const int mid = (lo + hi) >> 1;
          if (a.fnow[mid] < hv) lo = mid + 1;
          else hi = mid;
        }
        if (lo == fe) {
          fi = fe;
          break;
        }
        const int32_t f = a.F[lo];
        const int64_t nowf = a.fnow[lo];
        // sendTimerEvents: the notify queue (a FIFO, Scheduler.SchedulerState
        // toNotifyQueue) is polled while its head is <= now
        while (pc < pB && a.pv[pc] <= nowf) pc++;
        while (pc == pB && rnext >= 0 && a.its[a.sp[rnext]] + a.T <= nowf) {
          a.rec[rnext] = 2;
          int64_t q = rnext + 1;
          while (q < y && a.rec[q] != 1) q++;
          rnext = q < y ? q : -1;
        }
        const uint32_t tid = atomicAdd(a.ntimer, 1u);
        a.tF[tid] = f;
        a.tHead[tid] = hv;
        a.tSeg[tid] = (uint32_t)k;
        // the TIMER chunk: FIFO prefix with ts - now + T <= 0 (:141-151)
        const uint64_t o = 2ull * (uint64_t)a.offs[f];
        while (h < y && a.its[a.sp[h]] + a.T <= nowf) {
          a.eopp[h] = o;
          a.etid[h] = tid;
          h++;
        }
        // PartitionStateHolder.returnState: an empty window state is dropped
        if (a.partitioned && h == y) lastTs = INT64_MIN;
        fi = lo + 1;
      }
      if (y >= e) break;
      // externalTime (ExternalTimeWindowProcessor.java:128-149): each event's
      // own time attribute is the clock, items expire by theirs
      const int64_t nowy = a.ext_col >= 0 ? (int64_t)a.iattr[(int64_t)a.ext_col * a.cap + a.sp[y]] : a.call_now[cy];
      const uint64_t oy = 2ull * (uint64_t)a.irow[a.sp[y]] + 1ull;
      while (h < y && (a.ext_col >= 0 ? (int64_t)a.iattr[(int64_t)a.ext_col * a.cap + a.sp[h]] : a.its[a.sp[h]]) + a.T <=
                          nowy) {
        a.eopp[h] = oy;
        a.etid[h] = kNoTimer;
        h++;
      }
      // timeLength (TimeLengthWindowProcessor.java:160-178): a full window
      // gives up its head to the add
      if (a.L > 0 && y - h >= a.L) {
        a.eopp[h] = oy;
        a.etid[h] = kNoTimer;
        h++;
      }
      const int64_t tsy = a.its[a.sp[y]];
      // scheduler.notifyAt(ts + T): the time window when its lastTimestamp
      // rises (TimeWindowProcessor :156-159), timeLength for every add (:177)
      if (a.ext_col < 0 && (a.L > 0 || lastTs < tsy)) {
        a.rec[y] = 1;
        lastTs = tsy;
        if (rnext < 0) rnext = y;
      } else {
        a.rec[y] = 0;
      }
    }
    for (int64_t j = h; j < e; j++) {
      a.eopp[j] = kNoOpp;
      a.etid[j] = kNoTimer;
    }
    // notify entries still queued for the next push
    const int64_t o0 = a.proom_off[k];
    int64_t c = 0;
    for (; pc < pB; pc++, c++) {
      a.pout_pk[o0 + c] = pk;
      a.pout_v[o0 + c] = a.pv[pc];
    }
    if (rnext >= 0)
      for (int64_t j = rnext; j < e; j++)
        if (a.rec[j] == 1) {
          a.pout_pk[o0 + c] = pk;
          a.pout_v[o0 + c] = a.its[a.sp[j]] + a.T;
          c++;
        }
    a.pcnt[k] = (uint32_t)c;
    a.last_out[k] = lastTs;
  }
}

// Pending entries of keys without items: a clock move of the push reaching
// them consumes them (their TIMER chunk finds an empty window: no rows).
__global__ __launch_bounds__(kBlock) void k_xw_orphans(int64_t np, const uint64_t* ppk, const int64_t* pv,
                                                       int64_t nseg, const uint64_t* seg_pk, int nf,
                                                       const int64_t* fnow, uint32_t* keep) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < np; p = np) {
    int64_t lo = 0, hi = nseg;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (seg_pk[mid] < ppk[p]) lo = mid + 1;
      else hi = mid;
    }
    const bool has_seg = lo < nseg && seg_pk[lo] == ppk[p];
    // the key's FIFO is polled while its head <= now: entry p is gone when it
    // and every earlier entry of its key are <= the push's last clock
    bool consumed = nf > 0 && fnow[nf - 1] >= pv[p];
    for (int64_t q = p - 1; consumed && q >= 0 && ppk[q] == ppk[p]; q--) consumed = fnow[nf - 1] >= pv[q];
    keep[p] = (!has_seg && !consumed) ? 1u : 0u;
  }
}

__global__ __launch_bounds__(kBlock) void k_xw_seg_pk(int64_t nseg, const int64_t* segS, const uint32_t* sp,
                                                      const uint64_t* ipk, uint64_t* seg_pk) {
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < nseg; k = nseg) seg_pk[k] = ipk[sp[segS[k]]];
}

// ---------------------------------------------------------------- operations
__global__ __launch_bounds__(kBlock) void k_xw_nops(int64_t total, int64_t C, const uint32_t* sp,
                                                    const uint64_t* eopp, uint32_t* nops) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total)
    nops[j] = (sp[j] >= (uint32_t)C ? 1u : 0u) + (eopp[j] != kNoOpp ? 1u : 0u);
}

struct OpArgs {
  int64_t total, C;
  const uint32_t* sp;
  const uint32_t* segid;
  const int64_t* segS;
  const int64_t* segCk;
  const uint64_t* eopp;
  const uint32_t* etid;
  const uint32_t* opscan;     // exclusive scan of k_xw_nops
  const int32_t* irow;
  const int64_t* iseq;
  const int32_t* call_of;     // per batch row
  const int64_t* call_now;    // per call
  const uint32_t* run_of;     // per batch row: partition run id (partitioned)
  const int64_t* offs;
  const int64_t* fnow_of_call;   // per call: clock after its move (timers)
  const uint32_t* trank;      // timer id -> rank in (call, head, key) order
  const int32_t* sF;          // sorted timers' calls
  int64_t nt;
  const uint64_t* runs_before;   // per call: partition runs in earlier calls
  const int64_t* row_now;     // externalTime: per batch row its time attribute (null: the call's clock)
  int partitioned;
  int current_on, expired_on;
  int64_t seq0;
  // outputs [nops]
  uint32_t* op_item;
  uint8_t* op_add;
  uint8_t* op_on;
  uint32_t* op_chunk;         // chunk ordinal of the push
  int64_t* op_now;            // EXPIRED rows: the expiry time (currentTime)
  int64_t* op_seq;            // shd_out.in_seq of a row emitted at this op
};

__device__ __forceinline__ int64_t upper_bound_i32(const int32_t* a, int64_t lo, int64_t hi, int32_t v) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// chunk ordinal of an item opportunity at batch row r: the event chunks (calls
// or partition runs) and timer chunks interleave per call, timers first
__device__ __forceinline__ uint32_t event_ordinal(const OpArgs& a, int64_t r) {
  const int32_t c = a.call_of[r];
  const int64_t ev = a.partitioned ? (int64_t)a.run_of[r] : (int64_t)c;
  return (uint32_t)(ev + upper_bound_i32(a.sF, 0, a.nt, c));
}

__global__ __launch_bounds__(kBlock) void k_xw_ops(const OpArgs* __restrict__ ap) {
  const OpArgs& a = *ap;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.total; j = a.total) {
    const uint32_t k = a.segid[j];
    const int64_t s = a.segS[k], e = a.segS[k + 1], ck = a.segCk[k];
    const int64_t base = a.opscan[s];
    const uint32_t it = a.sp[j];
    if (it >= (uint32_t)a.C) {   // the add (CURRENT) of a new item
      const int64_t r = a.irow[it];
      const uint64_t oy = 2ull * (uint64_t)r + 1ull;
      int64_t lo = s, hi = j;    // expirations of this key at or before the opportunity
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.eopp[mid] <= oy) lo = mid + 1;
        else hi = mid;
      }
      const int64_t q = base + (j - s - ck) + (lo - s);
      a.op_item[q] = it;
      a.op_add[q] = 1;
      a.op_on[q] = (uint8_t)a.current_on;
      a.op_chunk[q] = event_ordinal(a, r);
      a.op_now[q] = a.call_now[a.call_of[r]];
      a.op_seq[q] = a.iseq[it];
    }
    const uint64_t o = a.eopp[j];
    if (o != kNoOpp) {           // the EXPIRED event of item j
      int64_t lo = s + ck, hi = e;   // adds of this key before the opportunity
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (2ull * (uint64_t)a.irow[a.sp[mid]] + 1ull < o) lo = mid + 1;
        else hi = mid;
      }
      const int64_t q = base + (j - s) + (lo - s - ck);
      a.op_item[q] = it;
      a.op_add[q] = 0;
      a.op_on[q] = (uint8_t)a.expired_on;
      const uint32_t tid = a.etid[j];
      if (tid == kNoTimer) {
        const int64_t r = (int64_t)((o - 1) >> 1);
        a.op_chunk[q] = event_ordinal(a, r);
        a.op_now[q] = a.row_now ? a.row_now[r] : a.call_now[a.call_of[r]];
        a.op_seq[q] = a.seq0 + r;
      } else {
        const uint32_t t = a.trank[tid];
        const int32_t f = a.sF[t];
        const int64_t ev = a.partitioned ? (int64_t)a.runs_before[f] : (int64_t)f;
        a.op_chunk[q] = (uint32_t)(t + ev);
        a.op_now[q] = a.fnow_of_call[f];
        a.op_seq[q] = a.seq0 + a.offs[f];
      }
    }
  }
}

// runs_before[c]: partition runs that start in calls before c
__global__ __launch_bounds__(kBlock) void k_xw_runs_before(int ncalls, const int64_t* offs, int64_t n,
                                                           const uint32_t* run_excl, uint64_t total_runs,
                                                           uint64_t* out) {
  for (int64_t c = (int64_t)blockIdx.x * kBlock + threadIdx.x; c < ncalls; c = ncalls) {
    const int64_t r = offs[c];
    out[c] = r < n ? (uint64_t)run_excl[r] : total_runs;
  }
}

// ---------------------------------------------------------------- selector
struct FoldArgsX {
  int nagg;
  int kind[kMaxAggs];
  int type[kMaxAggs];
  int group;          // processInBatchGroupBy: row at the first pick, values of the last
  int64_t cap, nops, nstates;
  const uint64_t* argv;
  const uint8_t* argn;
  const uint32_t* op_item;
  const uint8_t* op_add;
  const uint8_t* op_on;
  const uint32_t* op_chunk;
  const int64_t* op_now;
  const int64_t* its;
  const uint64_t* attr;
  const uint8_t* nul;
  int ncols;
  DExprSet es;
  int has_having;
  DExpr having;
  double* dsum;
  int64_t* lsum;
  int64_t* cnt;
  // batch windows: the chunk of a state's last RESET-started add (RESET clears
  // every group state of the partition; applied when the state is next added to)
  int64_t* epoch;     // [nstates], null: no batch window
  const int64_t* op_epoch;   // per add: the RESET epoch it folds in
  uint64_t* resv;     // [nagg][nops]
  uint8_t* resn;
  uint8_t* rowflag;   // [nops]
  uint32_t* rowsrc;
};

// Aggregated value of one aggregator after a step (avg divided here).
__device__ __forceinline__ void agg_value(int kind, uint64_t ob, bool on, int64_t c, uint64_t& v, uint8_t& vn) {
  v = ob;
  vn = (uint8_t)on;
  if (kind == SHD_AGG_AVG && !on) v = p_f64(__ddiv_rn(v_f64(ob), (double)c));
}

// One lane per aggregator state (a (partition key, group key) pair): the
// state's operations in the reference's order.  The selector's pick per chunk
// is tracked on the fly: a run = the state's consecutive operations of one
// chunk; its first and last selected ("on") operations decide the row.
__global__ __launch_bounds__(kBlock) void k_xw_fold(const FoldArgsX* __restrict__ ap, const uint32_t* heads,
                                                    int64_t nheads, const uint32_t* ssid, const uint32_t* sq) {
  const FoldArgsX& a = *ap;
  for (int64_t hh = (int64_t)blockIdx.x * kBlock + threadIdx.x; hh < nheads; hh = nheads) {
    const int64_t q0 = heads[hh];
    const int64_t q1 = hh + 1 < nheads ? (int64_t)heads[hh + 1] : a.nops;
    const uint32_t sid = ssid[q0];
    double d[kMaxAggs];
    int64_t l[kMaxAggs], c[kMaxAggs];
    for (int g = 0; g < a.nagg; g++) {
      d[g] = a.dsum[(int64_t)g * a.nstates + sid];
      l[g] = a.lsum[(int64_t)g * a.nstates + sid];
      c[g] = a.cnt[(int64_t)g * a.nstates + sid];
    }
    int64_t ep = a.epoch ? a.epoch[sid] : 0;
    uint32_t cur = 0xFFFFFFFFu;
    int64_t first = -1, last = -1;
    for (int64_t p = q0; p < q1; p++) {
      const uint32_t q = sq[p];
      const uint32_t it = a.op_item[q];
      const bool add = a.op_add[q];
      if (a.epoch && add && ep != a.op_epoch[q]) {
        // a RESET came after this state's last operation
        ep = a.op_epoch[q];
        for (int g = 0; g < a.nagg; g++) {
          d[g] = 0.0;
          l[g] = 0;
          c[g] = 0;
        }
      }
      uint64_t vv[kMaxAggs];
      uint8_t vn[kMaxAggs];
      for (int g = 0; g < a.nagg; g++) {
        uint64_t ob;
        bool on;
        agg_step(a.kind[g], a.type[g], add, a.argv[(int64_t)g * a.cap + it], a.argn[(int64_t)g * a.cap + it] != 0,
                 d[g], l[g], c[g], ob, on);
        agg_value(a.kind[g], ob, on, c[g], vv[g], vn[g]);
      }
      bool sel = a.op_on[q] != 0;
      if (sel && a.has_having) {
        ItemCtx cx{a.attr, a.nul, a.cap, (int64_t)it, a.ncols, add ? a.its[it] : a.op_now[q], vv, vn};
        sel = eval_bool(a.es.ins + a.having.off, a.having.len, a.es.consts, cx);
      }
      if (!sel) continue;
      for (int g = 0; g < a.nagg; g++) {
        a.resv[(int64_t)g * a.nops + q] = vv[g];
        a.resn[(int64_t)g * a.nops + q] = vn[g];
      }
      const uint32_t ch = a.op_chunk[q];
      if (ch != cur) {
        if (first >= 0) {
          const int64_t at = a.group ? first : last;
          a.rowflag[at] = 1;
          a.rowsrc[at] = (uint32_t)last;
        }
        cur = ch;
        first = q;
      }
      last = q;
    }
    if (first >= 0) {
      const int64_t at = a.group ? first : last;
      a.rowflag[at] = 1;
      a.rowsrc[at] = (uint32_t)last;
    }
    for (int g = 0; g < a.nagg; g++) {
      a.dsum[(int64_t)g * a.nstates + sid] = d[g];
      a.lsum[(int64_t)g * a.nstates + sid] = l[g];
      a.cnt[(int64_t)g * a.nstates + sid] = c[g];
    }
    if (a.epoch) a.epoch[sid] = ep;
  }
}

// processNoGroupBy: every selected operation is a row.
__global__ __launch_bounds__(kBlock) void k_xw_plain_rows(const FoldArgsX* __restrict__ ap) {
  const FoldArgsX& a = *ap;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < a.nops; q = a.nops) {
    bool sel = a.op_on[q] != 0;
    if (sel && a.has_having) {
      const uint32_t it = a.op_item[q];
      ItemCtx cx{a.attr, a.nul, a.cap, (int64_t)it, a.ncols, a.op_add[q] ? a.its[it] : a.op_now[q], nullptr, nullptr};
      sel = eval_bool(a.es.ins + a.having.off, a.having.len, a.es.consts, cx);
    }
    a.rowflag[q] = sel ? 1 : 0;
    a.rowsrc[q] = (uint32_t)q;
  }
}

__global__ __launch_bounds__(kBlock) void k_xw_row_keys(int64_t nops, const uint8_t* rowflag, const uint32_t* roff,
                                                        const uint32_t* op_chunk, uint64_t* rkey, uint32_t* rq) {
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nops; q = nops) {
    if (!rowflag[q]) continue;
    rkey[roff[q]] = ((uint64_t)op_chunk[q] << 32) | (uint64_t)q;
    rq[roff[q]] = (uint32_t)q;
  }
}

struct EmitArgsX {
  DExprSet es;
  DExpr outs[kMaxCols];
  int nout, nagg, ncols;
  int64_t cap, nops, row0, chunk0;
  const uint32_t* rowsrc;
  const uint32_t* op_item;
  const uint8_t* op_add;
  const uint32_t* op_chunk;
  const int64_t* op_now;
  const int64_t* op_seq;
  const int64_t* its;
  const uint64_t* attr;
  const uint8_t* nul;
  const uint64_t* resv;
  const uint8_t* resn;
};

__global__ __launch_bounds__(kBlock) void k_xw_emit(const EmitArgsX* __restrict__ ap, int64_t nrows, const uint32_t* rq,
                                                    int64_t* o_chunk, int32_t* o_type, int64_t* o_ts, uint64_t* o_vals,
                                                    uint8_t* o_nul, int64_t* o_seq, int32_t* o_sidx) {
  const EmitArgsX& a = *ap;
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < nrows; r = nrows) {
    const uint32_t q = rq[r];
    const uint32_t src = a.rowsrc[q];
    const uint32_t it = a.op_item[src];
    const bool add = a.op_add[src];
    uint64_t vv[kMaxAggs];
    uint8_t vn[kMaxAggs];
    for (int g = 0; g < a.nagg; g++) {
      vv[g] = a.resv[(int64_t)g * a.nops + src];
      vn[g] = a.resn[(int64_t)g * a.nops + src];
    }
    const int64_t ts = add ? a.its[it] : a.op_now[src];
    ItemCtx cx{a.attr, a.nul, a.cap, (int64_t)it, a.ncols, ts, vv, vn};
    const int64_t row = a.row0 + r;
    for (int c = 0; c < a.nout; c++) {
      Val v = eval_expr(a.es.ins + a.outs[c].off, a.outs[c].len, a.es.consts, cx);
      o_vals[row * a.nout + c] = v.b;
      o_nul[row * a.nout + c] = (uint8_t)v.null;
    }
    o_ts[row] = ts;
    o_type[row] = add ? 0 : 1;
    o_chunk[row] = a.chunk0 + (int64_t)a.op_chunk[q];
    o_seq[row] = a.op_seq[src];
    o_sidx[row] = 0;
  }
}

// ---------------------------------------------------------------- carry / misc
__global__ __launch_bounds__(kBlock) void k_xw_keep(int64_t total, const uint64_t* eopp, int window, uint32_t* keep) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total)
    keep[j] = (window && eopp[j] == kNoOpp) ? 1u : 0u;
}

struct CarryArgs {
  int64_t total, cap_src, cap_dst;
  int ncols, nagg;
  const uint32_t* sp;
  const uint32_t* keep;
  const uint32_t* koff;
  const uint32_t* segid;
  const int64_t* last_out;   // per segment (time windows), may be null
  const int64_t* last_j;     // batch windows: per sorted position, its ilast in the carry
  const uint64_t* pk; const int64_t* ts; const int64_t* seq; const uint64_t* sid;
  const uint64_t* attr; const uint8_t* nul; const uint64_t* argv; const uint8_t* argn;
  uint64_t* d_pk; int64_t* d_ts; int64_t* d_seq; uint64_t* d_sid; int64_t* d_last; int32_t* d_call; int32_t* d_row;
  uint64_t* d_attr; uint8_t* d_nul; uint64_t* d_argv; uint8_t* d_argn;
};

// The kept items, in sorted (key, FIFO) order, become the next push's carry.
__global__ __launch_bounds__(kBlock) void k_xw_carry(const CarryArgs* __restrict__ ap) {
  const CarryArgs& a = *ap;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.total; j = a.total) {
    if (!a.keep[j]) continue;
    const int64_t t = a.koff[j];
    const uint32_t it = a.sp[j];
    a.d_pk[t] = a.pk[it];
    a.d_ts[t] = a.ts[it];
    a.d_seq[t] = a.seq[it];
    a.d_sid[t] = a.sid[it];
    a.d_last[t] = a.last_j ? a.last_j[j] : (a.last_out ? a.last_out[a.segid[j]] : INT64_MIN);
    a.d_call[t] = -1;
    a.d_row[t] = -1;
    for (int c = 0; c < a.ncols; c++) {
      a.d_attr[(int64_t)c * a.cap_dst + t] = a.attr[(int64_t)c * a.cap_src + it];
      a.d_nul[(int64_t)c * a.cap_dst + t] = a.nul[(int64_t)c * a.cap_src + it];
    }
    for (int g = 0; g < a.nagg; g++) {
      a.d_argv[(int64_t)g * a.cap_dst + t] = a.argv[(int64_t)g * a.cap_src + it];
      a.d_argn[(int64_t)g * a.cap_dst + t] = a.argn[(int64_t)g * a.cap_src + it];
    }
  }
}

// new pending list = the segments' remaining entries + the kept orphans
__global__ __launch_bounds__(kBlock) void k_xw_pend_gather(int64_t nseg, const uint32_t* proom_off, const uint32_t* pcnt,
                                                           const uint32_t* pcnt_off, const uint64_t* spk,
                                                           const int64_t* sv, uint64_t* dpk, int64_t* dv) {
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < nseg; k = nseg) {
    const int64_t o = proom_off[k], d = pcnt_off[k];
    for (uint32_t i = 0; i < pcnt[k]; i++) {
      dpk[d + i] = spk[o + i];
      dv[d + i] = sv[o + i];
    }
  }
}

__global__ __launch_bounds__(kBlock) void k_xw_pend_orphan_copy(int64_t np, const uint32_t* keep, const uint32_t* koff,
                                                                int64_t base, const uint64_t* ppk, const int64_t* pv,
                                                                uint64_t* dpk, int64_t* dv) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < np; p = np) {
    if (!keep[p]) continue;
    dpk[base + koff[p]] = ppk[p];
    dv[base + koff[p]] = pv[p];
  }
}

__global__ __launch_bounds__(kBlock) void k_xw_gather_u64(const uint64_t* src, const uint32_t* perm, uint64_t* dst,
                                                          int64_t n, uint64_t flip) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) dst[i] = src[perm[i]] ^ flip;
}
__global__ __launch_bounds__(kBlock) void k_xw_gather_u32(const uint32_t* src, const uint32_t* perm, uint32_t* dst,
                                                          int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) dst[i] = src[perm[i]];
}
__global__ __launch_bounds__(kBlock) void k_xw_timer_rank(const uint32_t* perm, const int32_t* tF, int64_t nt,
                                                          uint32_t* rank, int32_t* sF) {
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < nt; t = nt) {
    rank[perm[t]] = (uint32_t)t;
    sF[t] = tF[perm[t]];
  }
}
__global__ __launch_bounds__(kBlock) void k_xw_narrow(const uint64_t* in, uint32_t* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) out[i] = (uint32_t)in[i];
}
__global__ __launch_bounds__(kBlock) void k_xw_op_sid(int64_t nops, const uint32_t* op_item, const uint64_t* isid,
                                                      uint32_t* out) {
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nops; q = nops) out[q] = (uint32_t)isid[op_item[q]];
}
__global__ __launch_bounds__(kBlock) void k_xw_heads_u32(const uint32_t* k, int64_t n, uint32_t* head) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n)
    head[i] = (i == 0 || k[i] != k[i - 1]) ? 1u : 0u;
}
__global__ __launch_bounds__(kBlock) void k_xw_head_list(const uint32_t* head, const uint32_t* hoff, int64_t n,
                                                         uint32_t* hl) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n)
    if (head[i]) hl[hoff[i]] = (uint32_t)i;
}
__global__ __launch_bounds__(kBlock) void k_xw_fill_u64(uint64_t* p, int64_t n, uint64_t v) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) p[i] = v;
}

// ---------------------------------------------------------------- batch windows
// lengthBatch / timeBatch in full-batch mode (LengthBatchWindowProcessor.java:
// 206-243, TimeBatchWindowProcessor.java:279-366).  A flush F of a key emits
// one chunk: the previous batch's items as EXPIRED (when the query outputs
// expired events), RESET, the batch's items as CURRENT.  Items of a key
// segment in FIFO order: [a carried items already added, awaiting expiry]
// [carried items of the open batch] [new items]; each item's add and expiry
// opportunities are flushes (2F + 1, expiry before add at one flush), both
// non-decreasing along the segment, so the operations of a key keep
// k_xw_ops' closed-form positions.  RESET (every group state of the partition
// cleared, PartitionStateHolder.cleanGroupByStates) is applied lazily by the
// fold: a state's first add of a flush starts it from zero (k_xw_fold epochs).

// added_j[j]: the item at sorted position j was added at an earlier flush
__global__ __launch_bounds__(kBlock) void k_xb_added(int64_t total, int64_t C, const uint32_t* sp, const int64_t* ilast,
                                                     uint8_t* added_j) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total) {
    const uint32_t it = sp[j];
    added_j[j] = (it < (uint32_t)C && ilast[it] == 1) ? 1 : 0;
  }
}

// carried items of the segment [s, s + ck) already added: a prefix (FIFO)
__device__ __forceinline__ int64_t xb_added_count(const uint8_t* added_j, int64_t s, int64_t ck) {
  int64_t lo = s, hi = s + ck;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (added_j[mid]) lo = mid + 1;
    else hi = mid;
  }
  return lo - s;
}

struct XbArgs {
  int64_t total, C, L;
  int expired_on;
  const uint32_t* sp;
  const uint32_t* segid;
  const int64_t* segS;
  const int64_t* segCk;
  const uint8_t* added_j;
  const int32_t* irow;
  const int32_t* icall;
  const uint32_t* fr;        // lengthBatch: flush rank of each batch row (exclusive scan of the triggers)
  const int32_t* bflush;     // timeBatch: per call, the flush its events join (-1: none in this push)
  int64_t nf;                // timeBatch: flushes of this push
  // stream.current.event timeBatch: per call its chunk, the first flush at or
  // after it and its RESET epoch; the push's first flush (carried items)
  const int32_t* cchunk;
  const int32_t* cflush;
  const int64_t* cepoch;
  int64_t first_flush;
  const int64_t* ilast;      // carried items' ilast (lengthBatch stream mode: their batch epoch)
  int64_t chunk0;            // global id of the push's first chunk
  uint64_t* aopp;
  uint64_t* eopp;
  int64_t* epoch_j;          // per sorted position: the RESET epoch its add folds in
  uint8_t* keep_j;           // carried to the next push
  int64_t* last_j;           // its ilast there
};

// batch window modes (WindowXEngine::bmode)
enum : int { XB_FULL_LEN = 0, XB_FULL_TIME = 1, XB_STREAM_LEN = 2, XB_ZERO_LEN = 3, XB_STREAM_TIME = 4 };

// lengthBatch triggers: the new item whose open-batch ordinal completes a batch
__global__ __launch_bounds__(kBlock) void k_xb_len_trig(const XbArgs* __restrict__ ap, uint32_t* trig) {
  const XbArgs& a = *ap;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.total; j = a.total) {
    const uint32_t k = a.segid[j];
    const int64_t s = a.segS[k], ck = a.segCk[k];
    const int64_t na = xb_added_count(a.added_j, s, ck);
    const int64_t o = j - s - na;
    const uint32_t it = a.sp[j];
    if (o >= 0 && (o + 1) % a.L == 0 && it >= (uint32_t)a.C) trig[a.irow[it]] = 1u;
  }
}

// per flush (lengthBatch): its clock and in_seq, from the trigger row
__global__ __launch_bounds__(kBlock) void k_xb_len_flushes(int64_t n, const uint32_t* trig, const uint32_t* fr,
                                                           const int32_t* call_of, const int64_t* call_now, int64_t seq0,
                                                           int64_t* fnow, int64_t* fseq) {
  for (int64_t r = (int64_t)blockIdx.x * kBlock + threadIdx.x; r < n; r = n) {
    if (!trig[r]) continue;
    fnow[fr[r]] = call_now[call_of[r]];
    fseq[fr[r]] = seq0 + r;
  }
}

// Each item's add / expiry opportunities (op positions: 2 * chunk + 1 when
// expirations come first in the chunk, 2 * chunk for an add before them),
// the epoch of its add and what is carried.
__global__ __launch_bounds__(kBlock) void k_xb_opp(const XbArgs* __restrict__ ap, int mode) {
  const XbArgs& a = *ap;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.total; j = a.total) {
    const uint32_t k = a.segid[j];
    const int64_t s = a.segS[k], e = a.segS[k + 1], ck = a.segCk[k];
    const uint32_t it = a.sp[j];
    uint64_t ao = kNoOpp, eo = kNoOpp;
    int64_t ep = -1, last = 0;
    bool keep = false;
    if (mode == XB_FULL_LEN || mode == XB_FULL_TIME) {
      // full batches: [expired previous batch] RESET [batch] at each flush
      const int64_t na = xb_added_count(a.added_j, s, ck);
      if (mode == XB_FULL_LEN) {
        const int64_t tot = e - s - na;             // open batch + new items
        const int64_t nb = tot / a.L;               // batches completed in this push
        // flush of batch b: the trigger at ordinal (b + 1) L - 1
        auto flush_of = [&](int64_t b) -> uint64_t {
          return (uint64_t)a.fr[a.irow[a.sp[s + na + (b + 1) * a.L - 1]]];
        };
        if (j - s < na) {
          if (a.expired_on && nb >= 1) eo = 2 * flush_of(0) + 1;
        } else {
          const int64_t b = (j - s - na) / a.L;
          if (b < nb) ao = 2 * flush_of(b) + 1;
          if (a.expired_on && b + 1 < nb) eo = 2 * flush_of(b + 1) + 1;
        }
      } else {
        if (j - s < na) {
          if (a.expired_on && a.nf >= 1) eo = 1;
        } else {
          const int64_t f = it < (uint32_t)a.C ? (a.nf >= 1 ? 0 : -1) : (int64_t)a.bflush[a.icall[it]];
          if (f >= 0) {
            ao = 2 * (uint64_t)f + 1;
            if (a.expired_on && f + 1 < a.nf) eo = 2 * (uint64_t)(f + 1) + 1;
          }
        }
      }
      if (ao != kNoOpp) ep = a.chunk0 + (int64_t)(ao >> 1);   // the flush's RESET precedes its adds
      const bool added = a.added_j[j] || ao != kNoOpp;
      keep = !added || (a.expired_on && eo == kNoOpp);
      last = added ? 1 : 0;
    } else if (mode == XB_STREAM_LEN) {
      // processStreamCurrentEvents: every event its own chunk (a new item's
      // rank); batch b of the key = ordinals [bL, (b+1)L) with the carried open
      // batch first; the first item of batch b + 1 expires batch b and RESETs
      // before its own add
      const int64_t o = j - s, bl = (e - s - 1) / a.L, b = o / a.L;
      if (o >= ck) ao = 2 * (uint64_t)(it - (uint32_t)a.C) + 1;
      if (a.expired_on && b < bl) eo = 2 * (uint64_t)(a.sp[s + (b + 1) * a.L] - (uint32_t)a.C) + 1;
      const int64_t f = s + b * a.L;   // the batch's first item
      ep = f < s + ck ? a.ilast[a.sp[f]] : a.chunk0 + (int64_t)(a.sp[f] - (uint32_t)a.C);
      keep = b == bl;
      last = ep;
    } else if (mode == XB_ZERO_LEN) {
      // processLengthZeroBatch: the event, its EXPIRED copy, RESET -- one chunk
      const uint64_t c = (uint64_t)(it - (uint32_t)a.C);
      ao = 2 * c;
      if (a.expired_on) eo = 2 * c + 1;
      ep = a.chunk0 + (int64_t)c;
    } else {
      // stream.current.event timeBatch: a call's events in its chunk, then at a
      // flush (that chunk or a later TIMER) every event since the last flush
      // as EXPIRED, then RESET
      if (it < (uint32_t)a.C) {
        if (a.expired_on && a.first_flush >= 0) eo = 2 * (uint64_t)a.first_flush + 1;
      } else {
        const int32_t c = a.icall[it];
        ao = 2 * (uint64_t)a.cchunk[c];
        if (a.expired_on && a.cflush[c] >= 0) eo = 2 * (uint64_t)a.cflush[c] + 1;
        ep = a.cepoch[c];
      }
      keep = a.expired_on && eo == kNoOpp;
    }
    a.aopp[j] = ao;
    a.eopp[j] = eo;
    a.epoch_j[j] = ep;
    a.keep_j[j] = keep ? 1 : 0;
    a.last_j[j] = last;
  }
}

// per chunk of a new item (lengthBatch stream / zero modes): its clock and in_seq
__global__ __launch_bounds__(kBlock) void k_xb_item_chunks(int64_t C, int64_t m, const int32_t* icall,
                                                           const int32_t* irow, const int64_t* call_now, int64_t seq0,
                                                           int64_t* fnow, int64_t* fseq) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < m; j = m) {
    fnow[j] = call_now[icall[C + j]];
    fseq[j] = seq0 + irow[C + j];
  }
}

__global__ __launch_bounds__(kBlock) void k_xb_nops(int64_t total, const uint64_t* aopp, const uint64_t* eopp,
                                                    uint32_t* nops) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < total; j = total)
    nops[j] = (aopp[j] != kNoOpp ? 1u : 0u) + (eopp[j] != kNoOpp ? 1u : 0u);
}

struct XbOpArgs {
  int64_t total;
  const uint32_t* sp;
  const uint32_t* segid;
  const int64_t* segS;
  const int64_t* segCk;
  const uint8_t* added_j;
  const uint64_t* aopp;
  const uint64_t* eopp;
  const int64_t* epoch_j;
  int full;                   // full-batch modes: carried items awaiting expiry precede the adds
  const uint32_t* opscan;
  const int64_t* fnow;
  const int64_t* fseq;
  int current_on, expired_on;
  int64_t* op_epoch;
  uint32_t* op_item;
  uint8_t* op_add;
  uint8_t* op_on;
  uint32_t* op_chunk;
  int64_t* op_now;
  int64_t* op_seq;
};

// Operations of a key in the reference's order: per flush its expirations
// (FIFO), then its adds (FIFO).  Adds occupy the contiguous positions
// [s + a, ...), expirations a prefix [s, ...) of the segment.
__global__ __launch_bounds__(kBlock) void k_xb_ops(const XbOpArgs* __restrict__ ap) {
  const XbOpArgs& a = *ap;
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < a.total; j = a.total) {
    const uint32_t k = a.segid[j];
    const int64_t s = a.segS[k], e = a.segS[k + 1], ck = a.segCk[k];
    const int64_t base = a.opscan[s];
    // adds occupy [s + na, ...): after the carried items awaiting expiry (full
    // batches), after every carried item (stream modes: carried items were added)
    const int64_t na = a.full ? xb_added_count(a.added_j, s, ck) : ck;
    const uint32_t it = a.sp[j];
    const uint64_t ao = a.aopp[j], eo = a.eopp[j];
    if (ao != kNoOpp) {
      int64_t lo = s, hi = e;   // expirations at or before this flush
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.eopp[mid] <= ao) lo = mid + 1;
        else hi = mid;
      }
      const int64_t q = base + (j - s - na) + (lo - s);
      const uint32_t f = (uint32_t)(ao >> 1);
      a.op_item[q] = it;
      a.op_add[q] = 1;
      a.op_on[q] = (uint8_t)a.current_on;
      a.op_chunk[q] = f;
      a.op_now[q] = a.fnow[f];
      a.op_seq[q] = a.fseq[f];
      a.op_epoch[q] = a.epoch_j[j];
    }
    if (eo != kNoOpp) {
      int64_t lo = s + na, hi = e;   // adds at earlier flushes
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a.aopp[mid] < eo) lo = mid + 1;
        else hi = mid;
      }
      const int64_t q = base + (j - s) + (lo - s - na);
      const uint32_t f = (uint32_t)(eo >> 1);
      a.op_item[q] = it;
      a.op_add[q] = 0;
      a.op_on[q] = (uint8_t)a.expired_on;
      a.op_chunk[q] = f;
      a.op_now[q] = a.fnow[f];
      a.op_seq[q] = a.fseq[f];
    }
  }
}

// timeBatch: per call its passing items and the in_seq of its last one
__global__ __launch_bounds__(kBlock) void k_xb_call_items(int64_t C, int64_t m, const int32_t* icall,
                                                          const int32_t* irow, int64_t seq0, uint32_t* ccount,
                                                          int64_t* clast_seq) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < m; j = m) {
    const int32_t c = icall[C + j];
    atomicAdd(ccount + c, 1u);
    if (j + 1 == m || icall[C + j + 1] != c) clast_seq[c] = seq0 + irow[C + j];
  }
}

int bits_for(uint64_t v) {
  int b = 0;
  while (b < 64 && (v >> b)) b++;
  return std::max(b, 1);
}

}  // namespace

// ====================================================================== host
struct WindowXEngine : Engine {
  std::vector<int> filters;
  int wkind = 0;
  int64_t wparam = 0;
  bool partitioned = false;
  int key_expr = -1, key_col = -1, key_type = 0;
  int ngk = 0;
  int gk_expr[kMaxGroupAttrs] = {}, gk_col[kMaxGroupAttrs] = {}, gk_type[kMaxGroupAttrs] = {};
  int nagg = 0, ncols = 0, nw = 0;
  bool group = false, plain = false;
  GroupDict gd;
  // window items, double-buffered: [0, C) carried (key-sorted, FIFO inside a key)
  int64_t C = 0;
  int cur = 0;
  int64_t icap[2] = {0, 0};
  DevBuf ipk[2], its[2], iseq[2], isid[2], ilast[2], icall[2], irow[2], iattr[2], inul[2], iargv[2], iargn[2];
  // pending notify entries (time windows with timers): grouped by key (sorted),
  // each key's entries in queue (FIFO) order
  int64_t np = 0;
  DevBuf ppk, pv, ppk2, pv2;
  int64_t last_global = INT64_MIN;   // unpartitioned time window: state.lastTimestamp
  // aggregator states [nagg][nstates]
  DevBuf g_dsum, g_lsum, g_cnt;
  int64_t nstates = 0;
  // batch windows: per state its RESET epoch (k_xw_fold); timeBatch's
  // processor-level nextEmitTime and the Scheduler's notify queue (FIFO)
  bool batch = false;
  int64_t wparam2 = 0;
  DevBuf g_epoch;
  int64_t tb_next = -1;
  std::deque<int64_t> tb_notify;
  int bmode = 0;   // XB_* (k_xb_opp)
  DevBuf xb_added, xb_aopp, xb_trig, xb_fr, xb_fnow, xb_fseq, xb_bflush, xb_ccount, xb_clast, xb_epoch, xb_keep,
      xb_last, xb_cchunk, xb_cflush, xb_cepoch, op_epoch;
  int64_t tb_epoch = -1;   // stream.current.event timeBatch: global chunk id of the last flush
  // per-push scratch
  DevBuf d_offs, d_call_of, d_last, d_call_now, d_F, d_fnow, d_flags, d_cnt, d_off, d_pkey, d_start,
      d_run, d_runs_before, d_tot, d_scan, d_sort, kw, kn, kh, spk, spk2, sp, sp2, head, hscan, segS, segid, segCk,
      pA, pB, proom, proom_off, eopp, etid, rec, tF, tHead, tSeg, ntimer, pout_pk, pout_v, pcnt, pcnt_off, last_out,
      seg_pk, okeep, okoff, tperm, tperm2, tk32, tk32b, tk64, tk64b, trank, sF, nops_b, opscan, op_item, op_add, op_on,
      op_chunk, op_now, op_seq, osid, osid2, oq, oq2, ohead, ohoff, ohl, resv, resn, rowflag, rowsrc, roff, rkey, rkey2,
      rq, rq2, keep, koff, pend_tmp_pk, pend_tmp_v, pend_idx, pend_idx2, pend_key2;
  PinnedBuf h_tot, h_last, h_pin;
  std::vector<int64_t> h_offs, h_now;
  std::vector<int32_t> h_F;
  std::vector<int64_t> h_fnow;

  int kind() const override { return ENG_WINDOW; }
  // sliding windows with timers: time, timeLength
  bool time_like() const { return timed() || wkind == SHD_W_EXTERNAL_TIME; }
  // with Scheduler TIMER chunks
  bool timed() const { return wkind == SHD_W_TIME || wkind == SHD_W_TIME_LENGTH; }

  // aggregates here always fold sequentially (bit-exact): the option is a no-op
  void set_option(const std::string& key, int64_t v) override {
    if (key == "exact_aggregates") return;
    Engine::set_option(key, v);
  }

  void reset() override {
    C = 0;
    np = 0;
    seq = 0;
    now = INT64_MIN;
    chunk_seq = 0;
    out.count = 0;
    counters = shd_counters{};
    last_global = INT64_MIN;
    tb_next = -1;
    tb_epoch = -1;
    tb_notify.clear();
    gd.reset(stream);
    if (nstates) {
      SHD_HIP(hipMemsetAsync(g_dsum.p, 0, g_dsum.cap, stream));
      SHD_HIP(hipMemsetAsync(g_lsum.p, 0, g_lsum.cap, stream));
      SHD_HIP(hipMemsetAsync(g_cnt.p, 0, g_cnt.cap, stream));
      if (g_epoch.p) SHD_HIP(hipMemsetAsync(g_epoch.p, 0xFF, g_epoch.cap, stream));
    }
  }

  // ---- storage
  void alloc_slot(int s, int64_t cap) {
    const int64_t nc = std::max(ncols, 1), na = std::max(nagg, 1);
    ipk[s].reserve(cap * 8);
    its[s].reserve(cap * 8);
    iseq[s].reserve(cap * 8);
    isid[s].reserve(cap * 8);
    ilast[s].reserve(cap * 8);
    icall[s].reserve(cap * 4);
    irow[s].reserve(cap * 4);
    iattr[s].reserve(nc * cap * 8);
    inul[s].reserve(nc * cap);
    iargv[s].reserve(na * cap * 8);
    iargn[s].reserve(na * cap);
    icap[s] = cap;
  }
  // slot `cur` with room for `need` items, its [0, C) preserved
  void ensure_items(int64_t need) {
    if (icap[cur] >= need) return;
    const int nw_ = cur ^ 1;
    const int64_t cap = std::max<int64_t>(need, std::max<int64_t>(1024, icap[cur] * 2));
    alloc_slot(nw_, cap);
    hipStream_t s = stream;
    if (C > 0) {
      SHD_HIP(hipMemcpyAsync(ipk[nw_].p, ipk[cur].p, C * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(its[nw_].p, its[cur].p, C * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(iseq[nw_].p, iseq[cur].p, C * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(isid[nw_].p, isid[cur].p, C * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(ilast[nw_].p, ilast[cur].p, C * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(icall[nw_].p, icall[cur].p, C * 4, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(irow[nw_].p, irow[cur].p, C * 4, hipMemcpyDeviceToDevice, s));
      for (int c = 0; c < ncols; c++) {
        SHD_HIP(hipMemcpyAsync(iattr[nw_].as<uint64_t>() + c * cap, iattr[cur].as<uint64_t>() + c * icap[cur], C * 8,
                               hipMemcpyDeviceToDevice, s));
        SHD_HIP(hipMemcpyAsync(inul[nw_].as<uint8_t>() + c * cap, inul[cur].as<uint8_t>() + c * icap[cur], C,
                               hipMemcpyDeviceToDevice, s));
      }
      for (int g = 0; g < nagg; g++) {
        SHD_HIP(hipMemcpyAsync(iargv[nw_].as<uint64_t>() + g * cap, iargv[cur].as<uint64_t>() + g * icap[cur], C * 8,
                               hipMemcpyDeviceToDevice, s));
        SHD_HIP(hipMemcpyAsync(iargn[nw_].as<uint8_t>() + g * cap, iargn[cur].as<uint8_t>() + g * icap[cur], C,
                               hipMemcpyDeviceToDevice, s));
      }
    }
    cur = nw_;
  }
  void ensure_states(int64_t n) {
    if (n <= nstates || nagg == 0) {
      if (nagg == 0) nstates = std::max(nstates, n);
      return;
    }
    const int64_t ns = std::max<int64_t>(n, std::max<int64_t>(1024, nstates * 2));
    DevBuf a, l, c;
    a.reserve((size_t)nagg * ns * 8);
    l.reserve((size_t)nagg * ns * 8);
    c.reserve((size_t)nagg * ns * 8);
    SHD_HIP(hipMemsetAsync(a.p, 0, (size_t)nagg * ns * 8, stream));
    SHD_HIP(hipMemsetAsync(l.p, 0, (size_t)nagg * ns * 8, stream));
    SHD_HIP(hipMemsetAsync(c.p, 0, (size_t)nagg * ns * 8, stream));
    for (int g = 0; g < nagg && nstates; g++) {
      SHD_HIP(hipMemcpyAsync(a.as<double>() + g * ns, g_dsum.as<double>() + g * nstates, nstates * 8,
                             hipMemcpyDeviceToDevice, stream));
      SHD_HIP(hipMemcpyAsync(l.as<int64_t>() + g * ns, g_lsum.as<int64_t>() + g * nstates, nstates * 8,
                             hipMemcpyDeviceToDevice, stream));
      SHD_HIP(hipMemcpyAsync(c.as<int64_t>() + g * ns, g_cnt.as<int64_t>() + g * nstates, nstates * 8,
                             hipMemcpyDeviceToDevice, stream));
    }
    SHD_HIP(hipStreamSynchronize(stream));
    if (batch) {
      DevBuf ep;
      ep.reserve((size_t)ns * 8);
      SHD_HIP(hipMemsetAsync(ep.p, 0xFF, (size_t)ns * 8, stream));
      if (nstates) SHD_HIP(hipMemcpyAsync(ep.p, g_epoch.p, nstates * 8, hipMemcpyDeviceToDevice, stream));
      SHD_HIP(hipStreamSynchronize(stream));
      std::swap(g_epoch.p, ep.p); std::swap(g_epoch.cap, ep.cap);
    }
    std::swap(g_dsum.p, a.p); std::swap(g_dsum.cap, a.cap);
    std::swap(g_lsum.p, l.p); std::swap(g_lsum.cap, l.cap);
    std::swap(g_cnt.p, c.p); std::swap(g_cnt.cap, c.cap);
    nstates = ns;
  }

  template <class T> void upload(DevBuf& d, const std::vector<T>& v) {
    d.reserve(std::max<size_t>(v.size(), 1) * sizeof(T));
    if (v.empty()) return;
    h_pin.reserve(v.size() * sizeof(T));
    SHD_HIP(hipStreamSynchronize(stream));   // the pinned staging area is free again
    std::memcpy(h_pin.p, v.data(), v.size() * sizeof(T));
    SHD_HIP(hipMemcpyAsync(d.p, h_pin.p, v.size() * sizeof(T), hipMemcpyHostToDevice, stream));
    SHD_HIP(hipStreamSynchronize(stream));
  }
  uint32_t read_u32(const void* dev) {
    h_tot.reserve(64);
    SHD_HIP(hipMemcpyAsync(h_tot.p, dev, 4, hipMemcpyDeviceToHost, stream));
    SHD_HIP(hipStreamSynchronize(stream));
    return h_tot.as<uint32_t>()[0];
  }
  // exclusive scan; returns the total
  uint32_t scan(const uint32_t* in, uint32_t* outp, int64_t n) {
    if (n <= 0) return 0;
    d_tot.reserve(64);
    scan_exclusive_u32(in, outp, n, d_tot.as<uint32_t>(), d_scan, stream);
    return read_u32(d_tot.p);
  }

  // ---- push
  // ncalls InputHandler calls over n events; clock moves per call when `advance`;
  // `extra_move`: one clock move to `extra_t` with no events (shd_set_time).
  void push(const Staged& b) override { run(b, false, 0); }

  void set_time(int64_t t) override {
    if (t < now) return;
    if ((timed() && plan.expired_on) ||
        ((wkind == SHD_W_TIME_BATCH || wkind == SHD_W_TIME_BATCH_STREAM) && !tb_notify.empty() &&
         tb_notify.front() <= t)) {
      Staged z;
      z.n = 0;
      z.call_offsets = {0, 0};
      z.advance_time = true;
      run(z, true, t);
    } else {
      now = t;
    }
  }

  void run(const Staged& b, bool extra_move, int64_t extra_t) {
    hipStream_t s = stream;
    const int64_t n = b.n;
    SHD_HIP(hipEventRecord(ev0, s));
    stage_begin();
    // ---- calls and clock moves (TimestampGeneratorImpl.setCurrentTimestamp per call, playback)
    h_offs = b.call_offsets;
    if (h_offs.size() < 2) h_offs = {0, n};
    const int ncalls = (int)h_offs.size() - 1;
    upload(d_offs, h_offs);
    d_call_of.reserve(std::max<int64_t>(n, 1) * 4);
    d_last.reserve((size_t)ncalls * 8);
    if (n > 0) {
      hipLaunchKernelGGL(k_xw_calls, dim3((unsigned)ncalls), dim3(kBlock), 0, s, (const int64_t*)d_offs.as<int64_t>(),
                         ncalls, b.cs.ts, d_call_of.as<int32_t>(), d_last.as<int64_t>());
      SHD_CHECK_LAUNCH();
    }
    std::vector<int64_t> last(ncalls, INT64_MIN);
    if (n > 0) {
      h_last.reserve((size_t)ncalls * 8);
      SHD_HIP(hipMemcpyAsync(h_last.p, d_last.p, (size_t)ncalls * 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
      std::memcpy(last.data(), h_last.p, (size_t)ncalls * 8);
    }
    h_now.assign(ncalls, now);
    h_F.clear();
    h_fnow.clear();
    int64_t clk = now;
    std::vector<char> moved(ncalls, 0);
    for (int c = 0; c < ncalls; c++) {
      int64_t t = INT64_MIN;
      bool move = false;
      if (extra_move && c == 0) {
        t = extra_t;
        move = true;
      } else if (b.advance_time && h_offs[c + 1] > h_offs[c]) {
        t = last[c];
        move = true;   // InputHandler.send(Event[]) with events
      }
      if (move && t >= clk) {
        clk = t;
        h_F.push_back(c);
        h_fnow.push_back(t);
        moved[c] = 1;
      }
      h_now[c] = clk;
    }
    const bool timers = timed() && plan.expired_on;
    if (!timers) {   // clock moves only matter to the TIMER chunks
      h_F.clear();
      h_fnow.clear();
    }
    upload(d_call_now, h_now);
    upload(d_F, h_F);
    upload(d_fnow, h_fnow);
    const int nf = (int)h_F.size();
    // ---- filter, partition key, runs
    d_flags.reserve(std::max<int64_t>(n, 1));
    d_cnt.reserve(std::max<int64_t>(n, 1) * 4);
    d_off.reserve(std::max<int64_t>(n, 1) * 4);
    d_pkey.reserve(std::max<int64_t>(n, 1) * 8);
    XwArgs xa{};
    xa.cs = b.cs;
    xa.es = dset();
    xa.filters = dfilters(filters);
    xa.partitioned = partitioned;
    if (partitioned) {
      xa.key = dexpr(key_expr);
      xa.key_col = key_col;
      xa.key_type = key_type;
    }
    xa.ngk = ngk;
    for (int g = 0; g < ngk; g++) {
      xa.group[g] = dexpr(gk_expr[g]);
      xa.group_col[g] = gk_col[g];
      xa.group_type[g] = gk_type[g];
    }
    xa.null_str_id = plan.null_str_id;
    xa.nagg = nagg;
    for (int g = 0; g < nagg; g++) {
      xa.has_arg[g] = plan.aggs[g].expr >= 0;
      if (xa.has_arg[g]) xa.agg_arg[g] = dexpr(plan.aggs[g].expr);
    }
    xa.ncols = ncols;
    xa.nw = nw;
    xa.C = C;
    xa.seq0 = seq;
    int64_t m = 0;
    uint32_t nruns = 0;
    const XwArgs* d_xa = nullptr;
    if (n > 0) {
      d_xa = dev_args(xa);
      hipLaunchKernelGGL(k_xw_filter, dim3(grid_cover(n)), dim3(kBlock), 0, s, d_xa, n, d_flags.as<uint8_t>(),
                         d_cnt.as<uint32_t>(), d_pkey.as<uint64_t>());
      SHD_CHECK_LAUNCH();
      m = scan(d_cnt.as<uint32_t>(), d_off.as<uint32_t>(), n);
      if (partitioned) {
        d_start.reserve(n * 4);
        d_run.reserve(n * 4);
        hipLaunchKernelGGL(k_xw_run_starts, dim3(grid_cover(n)), dim3(kBlock), 0, s, (const uint8_t*)d_flags.as<uint8_t>(),
                           (const uint64_t*)d_pkey.as<uint64_t>(), (const int32_t*)d_call_of.as<int32_t>(), n,
                           d_start.as<uint32_t>());
        SHD_CHECK_LAUNCH();
        nruns = scan(d_start.as<uint32_t>(), d_run.as<uint32_t>(), n);
        // run id of event i = exclusive count + own start - 1: k_xw_ops reads the
        // exclusive count at a run's events; fix it up to the inclusive id
      }
    }
    mark("filter");
    const int64_t total = C + m;
    if (total >= (int64_t)INT32_MAX) throw Error(SHD_E_CAPACITY, "window items exceed 2^31");
    // ---- new items
    ensure_items(std::max<int64_t>(total, 1));
    const int64_t cap = icap[cur];
    xa.cap = cap;
    if (m > 0) {
      kw.reserve((size_t)std::max(nw, 1) * m * 8);
      kn.reserve(m);
      kh.reserve(m * 8);
      ItemOut io{ipk[cur].as<uint64_t>(), its[cur].as<int64_t>(), iseq[cur].as<int64_t>(), icall[cur].as<int32_t>(),
                 irow[cur].as<int32_t>(), iattr[cur].as<uint64_t>(), inul[cur].as<uint8_t>(),
                 iargv[cur].as<uint64_t>(), iargn[cur].as<uint8_t>(), kw.as<uint64_t>(), kn.as<uint8_t>(),
                 kh.as<uint64_t>()};
      d_xa = dev_args(xa);
      hipLaunchKernelGGL(k_xw_items, dim3(grid_cover(n)), dim3(kBlock), 0, s, d_xa, dev_args(io), n,
                         (const uint32_t*)d_cnt.as<uint32_t>(), (const uint32_t*)d_off.as<uint32_t>(),
                         (const uint64_t*)d_pkey.as<uint64_t>(), (const int32_t*)d_call_of.as<int32_t>(), m);
      SHD_CHECK_LAUNCH();
      if (nw > 0) {
        gd.nk = nw;
        gd.assign(m, kh.as<uint64_t>(), kw.as<uint64_t>(), kn.as<uint8_t>(), m, isid[cur].as<uint64_t>(), C, s);
      } else {
        hipLaunchKernelGGL(k_xw_fill_u64, dim3(grid_cover(m)), dim3(kBlock), 0, s, isid[cur].as<uint64_t>() + C, m,
                           (uint64_t)0);
        SHD_CHECK_LAUNCH();
      }
    }
    ensure_states(nw > 0 ? std::max<int64_t>(gd.count, 1) : 1);
    mark("window_items");
    // ---- key segments: stable sort by partition key (carried first, FIFO kept)
    sp.reserve(std::max<int64_t>(total, 1) * 4);
    int64_t nseg = 0;
    if (total > 0) {
      fill_iota_u32(sp.as<uint32_t>(), total, 0, s);
      spk.reserve(total * 8);
      SHD_HIP(hipMemcpyAsync(spk.p, ipk[cur].p, total * 8, hipMemcpyDeviceToDevice, s));
      const uint32_t* spv = sp.as<uint32_t>();
      const uint64_t* spkv = spk.as<uint64_t>();
      if (partitioned) {
        d_tot.reserve(64);
        reduce_max_u64(ipk[cur].as<uint64_t>(), total, d_tot.as<uint64_t>() + 1, s);
        h_tot.reserve(64);
        SHD_HIP(hipMemcpyAsync(h_tot.p, d_tot.as<uint64_t>() + 1, 8, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipStreamSynchronize(s));
        const uint64_t kmax = h_tot.as<uint64_t>()[0];
        spk2.reserve(total * 8);
        sp2.reserve(total * 4);
        bool alt = false;
        radix_sort_pairs_u64(spk.as<uint64_t>(), sp.as<uint32_t>(), spk2.as<uint64_t>(), sp2.as<uint32_t>(), total,
                             bits_for(kmax), d_sort, s, alt);
        spv = alt ? sp2.as<uint32_t>() : sp.as<uint32_t>();
        spkv = alt ? spk2.as<uint64_t>() : spk.as<uint64_t>();
      }
      head.reserve(total * 4);
      hscan.reserve(total * 4);
      hipLaunchKernelGGL(k_xw_seg_heads, dim3(grid_cover(total)), dim3(kBlock), 0, s, spkv, total, head.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      nseg = scan(head.as<uint32_t>(), hscan.as<uint32_t>(), total);
      segS.reserve((nseg + 1) * 8);
      segid.reserve(total * 4);
      hipLaunchKernelGGL(k_xw_seg_list, dim3(grid_cover(total)), dim3(kBlock), 0, s, (const uint32_t*)head.as<uint32_t>(),
                         (const uint32_t*)hscan.as<uint32_t>(), total, segS.as<int64_t>(), segid.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      if (spv != sp.as<uint32_t>()) SHD_HIP(hipMemcpyAsync(sp.p, spv, total * 4, hipMemcpyDeviceToDevice, s));
    }
    const uint32_t* SP = sp.as<uint32_t>();
    segCk.reserve((nseg + 1) * 8);
    pA.reserve((nseg + 1) * 8);
    pB.reserve((nseg + 1) * 8);
    proom.reserve((nseg + 1) * 4);
    proom_off.reserve((nseg + 1) * 4);
    if (nseg > 0) {
      hipLaunchKernelGGL(k_xw_seg_info, dim3(grid_cover(nseg)), dim3(kBlock), 0, s, nseg,
                         (const int64_t*)segS.as<int64_t>(), SP, C, (const uint64_t*)ipk[cur].as<uint64_t>(),
                         (const uint64_t*)ppk.as<uint64_t>(), np, segCk.as<int64_t>(), pA.as<int64_t>(),
                         pB.as<int64_t>(), proom.as<uint32_t>());
      SHD_CHECK_LAUNCH();
    }
    mark("segments");
    int64_t nt = 0, nflush = 0, nops = 0;
    bool lane_ran = false;
    if (batch) {
      // ---- batch windows: flushes, opportunities, operations
      nops = batch_operations(n, m, total, ncalls, moved, SP, nflush);
      mark("operations");
    } else {
    // ---- expiry opportunities
    eopp.reserve(std::max<int64_t>(total, 1) * 8);
    etid.reserve(std::max<int64_t>(total, 1) * 4);
    if (total > 0 && wkind == SHD_W_LENGTH) {
      hipLaunchKernelGGL(k_xw_len_expiry, dim3(grid_cover(total)), dim3(kBlock), 0, s, total, wparam,
                         (const int64_t*)segS.as<int64_t>(), (const uint32_t*)segid.as<uint32_t>(), SP,
                         (const int32_t*)irow[cur].as<int32_t>(), eopp.as<uint64_t>(), etid.as<uint32_t>());
      SHD_CHECK_LAUNCH();
    } else if (total > 0 && time_like()) {
      const uint32_t room = nseg > 0 ? scan(proom.as<uint32_t>(), proom_off.as<uint32_t>(), nseg) : 0;
      rec.reserve(total);
      tF.reserve((np + m + 1) * 4);
      tHead.reserve((np + m + 1) * 8);
      tSeg.reserve((np + m + 1) * 4);
      ntimer.reserve(64);
      pout_pk.reserve(std::max<uint32_t>(room, 1) * 8);
      pout_v.reserve(std::max<uint32_t>(room, 1) * 8);
      pcnt.reserve((nseg + 1) * 4);
      pcnt_off.reserve((nseg + 1) * 4);
      last_out.reserve((nseg + 1) * 8);
      SHD_HIP(hipMemsetAsync(ntimer.p, 0, 4, s));
      LaneArgs la{};
      la.nseg = nseg;
      la.segS = segS.as<int64_t>();
      la.segCk = segCk.as<int64_t>();
      la.pA = pA.as<int64_t>();
      la.pB = pB.as<int64_t>();
      la.proom_off = proom_off.as<uint32_t>();
      la.sp = SP;
      la.ipk = ipk[cur].as<uint64_t>();
      la.its = its[cur].as<int64_t>();
      la.icall = icall[cur].as<int32_t>();
      la.irow = irow[cur].as<int32_t>();
      la.ilast = ilast[cur].as<int64_t>();
      la.call_now = d_call_now.as<int64_t>();
      la.offs = d_offs.as<int64_t>();
      la.F = d_F.as<int32_t>();
      la.fnow = d_fnow.as<int64_t>();
      la.nf = nf;
      la.T = wparam;
      la.L = wkind == SHD_W_TIME_LENGTH ? wparam2 : 0;
      la.ext_col = wkind == SHD_W_EXTERNAL_TIME ? (int)wparam2 : -1;
      la.iattr = iattr[cur].as<uint64_t>();
      la.cap = cap;
      la.partitioned = partitioned;
      la.last_global = last_global;
      la.pv = pv.as<int64_t>();
      la.eopp = eopp.as<uint64_t>();
      la.etid = etid.as<uint32_t>();
      la.rec = rec.as<uint8_t>();
      la.ntimer = ntimer.as<unsigned int>();
      la.tF = tF.as<int32_t>();
      la.tHead = tHead.as<int64_t>();
      la.tSeg = tSeg.as<uint32_t>();
      la.pout_pk = pout_pk.as<uint64_t>();
      la.pout_v = pout_v.as<int64_t>();
      la.pcnt = pcnt.as<uint32_t>();
      la.last_out = last_out.as<int64_t>();
      hipLaunchKernelGGL(k_xw_time_lane, dim3(grid_cover(nseg)), dim3(kBlock), 0, s, dev_args(la));
      SHD_CHECK_LAUNCH();
      nt = read_u32(ntimer.p);
      lane_ran = true;
    } else if (total > 0) {   // no window: items never expire
      hipLaunchKernelGGL(k_xw_fill_u64, dim3(grid_cover(total)), dim3(kBlock), 0, s, eopp.as<uint64_t>(), total, kNoOpp);
      SHD_CHECK_LAUNCH();
      SHD_HIP(hipMemsetAsync(etid.p, 0xFF, total * 4, s));
    }
    mark("expiry");
    // ---- timers in (call, notify head, key) order: the TIMER chunks' order
    //      (Scheduler.onTimeChange: sortedExpires by time; ties by key order)
    trank.reserve(std::max<int64_t>(nt, 1) * 4);
    sF.reserve(std::max<int64_t>(nt, 1) * 4);
    if (nt > 0) {
      tperm.reserve(nt * 4);
      tperm2.reserve(nt * 4);
      tk32.reserve(nt * 4);
      tk32b.reserve(nt * 4);
      tk64.reserve(nt * 8);
      tk64b.reserve(nt * 8);
      fill_iota_u32(tperm.as<uint32_t>(), nt, 0, s);
      // 1) by segment (key order)
      SHD_HIP(hipMemcpyAsync(tk32.p, tSeg.p, nt * 4, hipMemcpyDeviceToDevice, s));
      bool alt = false;
      radix_sort_pairs_u32(tk32.as<uint32_t>(), tperm.as<uint32_t>(), tk32b.as<uint32_t>(), tperm2.as<uint32_t>(), nt,
                           bits_for((uint64_t)nseg), d_sort, s, alt);
      if (alt) SHD_HIP(hipMemcpyAsync(tperm.p, tperm2.p, nt * 4, hipMemcpyDeviceToDevice, s));
      // 2) by notify head (signed -> order-preserving unsigned)
      hipLaunchKernelGGL(k_xw_gather_u64, dim3(grid_cover(nt)), dim3(kBlock), 0, s, (const uint64_t*)tHead.as<uint64_t>(),
                         (const uint32_t*)tperm.as<uint32_t>(), tk64.as<uint64_t>(), nt, 0x8000000000000000ull);
      SHD_CHECK_LAUNCH();
      alt = false;
      radix_sort_pairs_u64(tk64.as<uint64_t>(), tperm.as<uint32_t>(), tk64b.as<uint64_t>(), tperm2.as<uint32_t>(), nt,
                           64, d_sort, s, alt);
      if (alt) SHD_HIP(hipMemcpyAsync(tperm.p, tperm2.p, nt * 4, hipMemcpyDeviceToDevice, s));
      // 3) by call
      hipLaunchKernelGGL(k_xw_gather_u32, dim3(grid_cover(nt)), dim3(kBlock), 0, s, (const uint32_t*)tF.as<uint32_t>(),
                         (const uint32_t*)tperm.as<uint32_t>(), tk32.as<uint32_t>(), nt);
      SHD_CHECK_LAUNCH();
      alt = false;
      radix_sort_pairs_u32(tk32.as<uint32_t>(), tperm.as<uint32_t>(), tk32b.as<uint32_t>(), tperm2.as<uint32_t>(), nt,
                           bits_for((uint64_t)ncalls), d_sort, s, alt);
      if (alt) SHD_HIP(hipMemcpyAsync(tperm.p, tperm2.p, nt * 4, hipMemcpyDeviceToDevice, s));
      hipLaunchKernelGGL(k_xw_timer_rank, dim3(grid_cover(nt)), dim3(kBlock), 0, s, (const uint32_t*)tperm.as<uint32_t>(),
                         (const int32_t*)tF.as<int32_t>(), nt, trank.as<uint32_t>(), sF.as<int32_t>());
      SHD_CHECK_LAUNCH();
    }
    // partition runs before each call (chunk ordinals of timer chunks)
    d_runs_before.reserve((size_t)ncalls * 8);
    if (partitioned && n > 0) {
      hipLaunchKernelGGL(k_xw_runs_before, dim3(grid_cover(ncalls)), dim3(kBlock), 0, s, ncalls,
                         (const int64_t*)d_offs.as<int64_t>(), n, (const uint32_t*)d_run.as<uint32_t>(),
                         (uint64_t)nruns, d_runs_before.as<uint64_t>());
      SHD_CHECK_LAUNCH();
    } else if (partitioned) {
      SHD_HIP(hipMemsetAsync(d_runs_before.p, 0, (size_t)ncalls * 8, s));
    }
    // ---- operations in key-major order
    nops_b.reserve(std::max<int64_t>(total, 1) * 4);
    opscan.reserve(std::max<int64_t>(total, 1) * 4);
    if (total > 0) {
      hipLaunchKernelGGL(k_xw_nops, dim3(grid_cover(total)), dim3(kBlock), 0, s, total, C, SP,
                         (const uint64_t*)eopp.as<uint64_t>(), nops_b.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      nops = scan(nops_b.as<uint32_t>(), opscan.as<uint32_t>(), total);
    }
    if (partitioned && n > 0 && nruns > 0) {
      // run id (inclusive) of every keyed event: exclusive count + start - 1
      d_start.reserve(n * 4);
      run_ids(n);
    }
    reserve_ops(nops);
    if (nops > 0) {
      OpArgs oa{};
      oa.total = total;
      oa.C = C;
      oa.sp = SP;
      oa.segid = segid.as<uint32_t>();
      oa.segS = segS.as<int64_t>();
      oa.segCk = segCk.as<int64_t>();
      oa.eopp = eopp.as<uint64_t>();
      oa.etid = etid.as<uint32_t>();
      oa.opscan = opscan.as<uint32_t>();
      oa.irow = irow[cur].as<int32_t>();
      oa.iseq = iseq[cur].as<int64_t>();
      oa.call_of = d_call_of.as<int32_t>();
      oa.call_now = d_call_now.as<int64_t>();
      oa.run_of = partitioned ? d_start.as<uint32_t>() : nullptr;
      oa.offs = d_offs.as<int64_t>();
      oa.fnow_of_call = d_call_now.as<int64_t>();
      oa.trank = trank.as<uint32_t>();
      oa.sF = sF.as<int32_t>();
      oa.nt = nt;
      oa.runs_before = d_runs_before.as<uint64_t>();
      oa.partitioned = partitioned;
      oa.row_now = wkind == SHD_W_EXTERNAL_TIME ? reinterpret_cast<const int64_t*>(b.cs.col[wparam2]) : nullptr;
      oa.current_on = plan.current_on;
      oa.expired_on = plan.expired_on;
      oa.seq0 = seq;
      oa.op_item = op_item.as<uint32_t>();
      oa.op_add = op_add.as<uint8_t>();
      oa.op_on = op_on.as<uint8_t>();
      oa.op_chunk = op_chunk.as<uint32_t>();
      oa.op_now = op_now.as<int64_t>();
      oa.op_seq = op_seq.as<int64_t>();
      hipLaunchKernelGGL(k_xw_ops, dim3(grid_cover(total)), dim3(kBlock), 0, s, dev_args(oa));
      SHD_CHECK_LAUNCH();
    }
    mark("operations");
    }
    const int64_t nop_alloc = std::max<int64_t>(nops, 1);
    // ---- selector: aggregator folds and the rows each chunk emits
    const int na = std::max(nagg, 1);
    rowflag.reserve(nop_alloc);
    rowsrc.reserve(nop_alloc * 4);
    resv.reserve((size_t)na * nop_alloc * 8);
    resn.reserve((size_t)na * nop_alloc);
    FoldArgsX fa{};
    fa.nagg = nagg;
    for (int g = 0; g < nagg; g++) {
      fa.kind[g] = plan.aggs[g].kind;
      fa.type[g] = plan.aggs[g].type;
    }
    fa.group = group;
    fa.cap = cap;
    fa.nops = nops;
    fa.nstates = nstates;
    fa.argv = iargv[cur].as<uint64_t>();
    fa.argn = iargn[cur].as<uint8_t>();
    fa.op_item = op_item.as<uint32_t>();
    fa.op_add = op_add.as<uint8_t>();
    fa.op_on = op_on.as<uint8_t>();
    fa.op_chunk = op_chunk.as<uint32_t>();
    fa.op_now = op_now.as<int64_t>();
    fa.its = its[cur].as<int64_t>();
    fa.attr = iattr[cur].as<uint64_t>();
    fa.nul = inul[cur].as<uint8_t>();
    fa.ncols = ncols;
    fa.es = dset();
    fa.has_having = plan.having >= 0;
    if (fa.has_having) fa.having = dexpr(plan.having);
    fa.dsum = g_dsum.as<double>();
    fa.lsum = g_lsum.as<int64_t>();
    fa.cnt = g_cnt.as<int64_t>();
    fa.epoch = (batch && nagg > 0) ? g_epoch.as<int64_t>() : nullptr;
    fa.op_epoch = op_epoch.as<int64_t>();
    fa.resv = resv.as<uint64_t>();
    fa.resn = resn.as<uint8_t>();
    fa.rowflag = rowflag.as<uint8_t>();
    fa.rowsrc = rowsrc.as<uint32_t>();
    int64_t nrows = 0;
    if (nops > 0) {
      const FoldArgsX* d_fa = dev_args(fa);
      if (plain) {
        hipLaunchKernelGGL(k_xw_plain_rows, dim3(grid_cover(nops)), dim3(kBlock), 0, s, d_fa);
        SHD_CHECK_LAUNCH();
      } else {
        SHD_HIP(hipMemsetAsync(rowflag.p, 0, nops, s));
        osid.reserve(nops * 4);
        osid2.reserve(nops * 4);
        oq.reserve(nops * 4);
        oq2.reserve(nops * 4);
        hipLaunchKernelGGL(k_xw_op_sid, dim3(grid_cover(nops)), dim3(kBlock), 0, s, nops,
                           (const uint32_t*)op_item.as<uint32_t>(), (const uint64_t*)isid[cur].as<uint64_t>(),
                           osid.as<uint32_t>());
        SHD_CHECK_LAUNCH();
        fill_iota_u32(oq.as<uint32_t>(), nops, 0, s);
        bool alt = false;
        radix_sort_pairs_u32(osid.as<uint32_t>(), oq.as<uint32_t>(), osid2.as<uint32_t>(), oq2.as<uint32_t>(), nops,
                             bits_for((uint64_t)std::max<int64_t>(gd.count, 1)), d_sort, s, alt);
        const uint32_t* ssid = alt ? osid2.as<uint32_t>() : osid.as<uint32_t>();
        const uint32_t* sq = alt ? oq2.as<uint32_t>() : oq.as<uint32_t>();
        ohead.reserve(nops * 4);
        ohoff.reserve(nops * 4);
        hipLaunchKernelGGL(k_xw_heads_u32, dim3(grid_cover(nops)), dim3(kBlock), 0, s, ssid, nops, ohead.as<uint32_t>());
        SHD_CHECK_LAUNCH();
        const int64_t nheads = scan(ohead.as<uint32_t>(), ohoff.as<uint32_t>(), nops);
        ohl.reserve(std::max<int64_t>(nheads, 1) * 4);
        hipLaunchKernelGGL(k_xw_head_list, dim3(grid_cover(nops)), dim3(kBlock), 0, s,
                           (const uint32_t*)ohead.as<uint32_t>(), (const uint32_t*)ohoff.as<uint32_t>(), nops,
                           ohl.as<uint32_t>());
        SHD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_xw_fold, dim3(grid_cover(nheads)), dim3(kBlock), 0, s, d_fa,
                           (const uint32_t*)ohl.as<uint32_t>(), nheads, ssid, sq);
        SHD_CHECK_LAUNCH();
      }
      mark("fold");
      roff.reserve(nops * 4);
      nrows = scan_u8_flags(rowflag.as<uint8_t>(), nops);
    }
    // ---- rows in (chunk, position) order
    if (nrows > 0) {
      rkey.reserve(nrows * 8);
      rkey2.reserve(nrows * 8);
      rq.reserve(nrows * 4);
      rq2.reserve(nrows * 4);
      hipLaunchKernelGGL(k_xw_row_keys, dim3(grid_cover(nops)), dim3(kBlock), 0, s, nops,
                         (const uint8_t*)rowflag.as<uint8_t>(), (const uint32_t*)roff.as<uint32_t>(),
                         (const uint32_t*)op_chunk.as<uint32_t>(), rkey.as<uint64_t>(), rq.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      const int64_t nchunks = batch ? nflush : nt + (partitioned ? (int64_t)nruns : (int64_t)ncalls);
      bool alt = false;
      radix_sort_pairs_u64(rkey.as<uint64_t>(), rq.as<uint32_t>(), rkey2.as<uint64_t>(), rq2.as<uint32_t>(), nrows,
                           32 + bits_for((uint64_t)nchunks), d_sort, s, alt);
      const uint32_t* RQ = alt ? rq2.as<uint32_t>() : rq.as<uint32_t>();
      out.ensure(nrows, s);
      EmitArgsX ea{};
      ea.es = dset();
      ea.nout = (int)plan.outputs.size();
      for (int c = 0; c < ea.nout; c++) ea.outs[c] = dexpr(plan.outputs[c].second);
      ea.nagg = nagg;
      ea.ncols = ncols;
      ea.cap = cap;
      ea.nops = nops;
      ea.row0 = out.count;
      ea.chunk0 = chunk_seq;
      ea.rowsrc = rowsrc.as<uint32_t>();
      ea.op_item = op_item.as<uint32_t>();
      ea.op_add = op_add.as<uint8_t>();
      ea.op_chunk = op_chunk.as<uint32_t>();
      ea.op_now = op_now.as<int64_t>();
      ea.op_seq = op_seq.as<int64_t>();
      ea.its = its[cur].as<int64_t>();
      ea.attr = iattr[cur].as<uint64_t>();
      ea.nul = inul[cur].as<uint8_t>();
      ea.resv = resv.as<uint64_t>();
      ea.resn = resn.as<uint8_t>();
      hipLaunchKernelGGL(k_xw_emit, dim3(grid_cover(nrows)), dim3(kBlock), 0, s, dev_args(ea), nrows, RQ, out.d_chunk(),
                         out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls(), out.d_seq(), out.d_sidx());
      SHD_CHECK_LAUNCH();
      out.count += nrows;
    }
    mark("emit");
    // ---- carry: unexpired items (no window: nothing is kept; states persist)
    int64_t kept = 0;
    const int oth = cur ^ 1;
    if (total > 0) {
      keep.reserve(total * 4);
      koff.reserve(total * 4);
      if (batch) {
        hipLaunchKernelGGL(k_xw_widen, dim3(grid_cover(total)), dim3(kBlock), 0, s,
                           (const uint8_t*)xb_keep.as<uint8_t>(), total, keep.as<uint32_t>());
      } else {
        hipLaunchKernelGGL(k_xw_keep, dim3(grid_cover(total)), dim3(kBlock), 0, s, total,
                           (const uint64_t*)eopp.as<uint64_t>(), wkind != 0 ? 1 : 0, keep.as<uint32_t>());
      }
      SHD_CHECK_LAUNCH();
      kept = scan(keep.as<uint32_t>(), koff.as<uint32_t>(), total);
    }
    if (kept > 0) {
      if (icap[oth] < std::max<int64_t>(kept, 1024)) alloc_slot(oth, std::max<int64_t>(kept * 2, 1024));
      CarryArgs ca{};
      ca.total = total;
      ca.cap_src = cap;
      ca.cap_dst = icap[oth];
      ca.ncols = ncols;
      ca.nagg = nagg;
      ca.sp = SP;
      ca.keep = keep.as<uint32_t>();
      ca.koff = koff.as<uint32_t>();
      ca.segid = segid.as<uint32_t>();
      ca.last_out = lane_ran ? last_out.as<int64_t>() : nullptr;
      ca.last_j = batch ? xb_last.as<int64_t>() : nullptr;
      ca.pk = ipk[cur].as<uint64_t>(); ca.ts = its[cur].as<int64_t>(); ca.seq = iseq[cur].as<int64_t>();
      ca.sid = isid[cur].as<uint64_t>();
      ca.attr = iattr[cur].as<uint64_t>(); ca.nul = inul[cur].as<uint8_t>();
      ca.argv = iargv[cur].as<uint64_t>(); ca.argn = iargn[cur].as<uint8_t>();
      ca.d_pk = ipk[oth].as<uint64_t>(); ca.d_ts = its[oth].as<int64_t>(); ca.d_seq = iseq[oth].as<int64_t>();
      ca.d_sid = isid[oth].as<uint64_t>(); ca.d_last = ilast[oth].as<int64_t>();
      ca.d_call = icall[oth].as<int32_t>(); ca.d_row = irow[oth].as<int32_t>();
      ca.d_attr = iattr[oth].as<uint64_t>(); ca.d_nul = inul[oth].as<uint8_t>();
      ca.d_argv = iargv[oth].as<uint64_t>(); ca.d_argn = iargn[oth].as<uint8_t>();
      hipLaunchKernelGGL(k_xw_carry, dim3(grid_cover(total)), dim3(kBlock), 0, s, dev_args(ca));
      SHD_CHECK_LAUNCH();
    }
    // time windows: notify entries still queued, the window's last time
    if (time_like() && timers) update_pending(nseg, nf, lane_ran);
    if (time_like() && !partitioned && lane_ran && nseg > 0) {
      h_tot.reserve(64);
      SHD_HIP(hipMemcpyAsync(h_tot.p, last_out.p, 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
      last_global = h_tot.as<int64_t>()[0];
    }
    cur = oth;
    C = kept;
    mark("carry");
    SHD_HIP(hipEventRecord(ev1, s));
    stage_end();
    SHD_HIP(hipEventSynchronize(ev1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    counters.kernel_ns = (int64_t)(ms * 1e6);
    counters.kernel_ns_total += counters.kernel_ns;
    counters.events += n;
    counters.matches += nrows;
    counters.carry = C;
    counters.partial_scans += nops;
    chunk_seq += batch ? nflush : nt + (partitioned ? (int64_t)nruns : (int64_t)ncalls);
    now = clk;
    seq += n;
  }

  void reserve_ops(int64_t nops) {
    const int64_t nop_alloc = std::max<int64_t>(nops, 1);
    op_item.reserve(nop_alloc * 4);
    op_add.reserve(nop_alloc);
    op_on.reserve(nop_alloc);
    op_chunk.reserve(nop_alloc * 4);
    op_now.reserve(nop_alloc * 8);
    op_seq.reserve(nop_alloc * 8);
  }

  // TimeBatchWindowProcessor.process (:279-366) for one chunk at clock t:
  // nextEmitTime set up by the first chunk; a flush when t reached it
  bool tb_process(int64_t t) {
    const int64_t T = wparam;
    if (tb_next == -1) {
      if (wparam2 != INT64_MIN) tb_next = t + (T - (t - wparam2) % T);   // getNextEmitTime (:368-373)
      else tb_next = t + T;
      tb_notify.push_back(tb_next);
    }
    if (t >= tb_next) {
      tb_next += T;
      tb_notify.push_back(tb_next);
      return true;
    }
    return false;
  }

  // Batch windows: the push's output chunks (ordinals 0..nflush-1 in output
  // order: flushes, or every event / call in the stream modes), each item's
  // add / expiry chunk and RESET epoch, the operations in key-major order
  // (k_xb_ops).  Returns the operation count.
  int64_t batch_operations(int64_t n, int64_t m, int64_t total, int ncalls, const std::vector<char>& moved,
                           const uint32_t* SP, int64_t& nflush) {
    hipStream_t s = stream;
    const int64_t ta = std::max<int64_t>(total, 1);
    xb_added.reserve(ta);
    xb_aopp.reserve(ta * 8);
    eopp.reserve(ta * 8);
    xb_epoch.reserve(ta * 8);
    xb_keep.reserve(ta);
    xb_last.reserve(ta * 8);
    if (total > 0) {
      hipLaunchKernelGGL(k_xb_added, dim3(grid_cover(total)), dim3(kBlock), 0, s, total, C, SP,
                         (const int64_t*)ilast[cur].as<int64_t>(), xb_added.as<uint8_t>());
      SHD_CHECK_LAUNCH();
    }
    XbArgs xb{};
    xb.total = total;
    xb.C = C;
    xb.L = std::max<int64_t>(wparam, 1);
    xb.expired_on = plan.expired_on;
    xb.sp = SP;
    xb.segid = segid.as<uint32_t>();
    xb.segS = segS.as<int64_t>();
    xb.segCk = segCk.as<int64_t>();
    xb.added_j = xb_added.as<uint8_t>();
    xb.irow = irow[cur].as<int32_t>();
    xb.icall = icall[cur].as<int32_t>();
    xb.ilast = ilast[cur].as<int64_t>();
    xb.chunk0 = chunk_seq;
    xb.first_flush = -1;
    xb.aopp = xb_aopp.as<uint64_t>();
    xb.eopp = eopp.as<uint64_t>();
    xb.epoch_j = xb_epoch.as<int64_t>();
    xb.keep_j = xb_keep.as<uint8_t>();
    xb.last_j = xb_last.as<int64_t>();
    nflush = 0;
    if (bmode == XB_FULL_LEN) {
      // lengthBatch: a flush per completed batch, ranked by its trigger row
      xb_trig.reserve(std::max<int64_t>(n, 1) * 4);
      xb_fr.reserve(std::max<int64_t>(n, 1) * 4);
      if (n > 0) SHD_HIP(hipMemsetAsync(xb_trig.p, 0, n * 4, s));
      if (total > 0) {
        hipLaunchKernelGGL(k_xb_len_trig, dim3(grid_cover(total)), dim3(kBlock), 0, s, dev_args(xb),
                           xb_trig.as<uint32_t>());
        SHD_CHECK_LAUNCH();
      }
      nflush = n > 0 ? scan(xb_trig.as<uint32_t>(), xb_fr.as<uint32_t>(), n) : 0;
      xb_fnow.reserve(std::max<int64_t>(nflush, 1) * 8);
      xb_fseq.reserve(std::max<int64_t>(nflush, 1) * 8);
      if (nflush > 0) {
        hipLaunchKernelGGL(k_xb_len_flushes, dim3(grid_cover(n)), dim3(kBlock), 0, s, n,
                           (const uint32_t*)xb_trig.as<uint32_t>(), (const uint32_t*)xb_fr.as<uint32_t>(),
                           (const int32_t*)d_call_of.as<int32_t>(), (const int64_t*)d_call_now.as<int64_t>(), seq,
                           xb_fnow.as<int64_t>(), xb_fseq.as<int64_t>());
        SHD_CHECK_LAUNCH();
      }
      xb.fr = xb_fr.as<uint32_t>();
    } else if (bmode == XB_STREAM_LEN || bmode == XB_ZERO_LEN) {
      // an output chunk per event (its rank among the push's new items)
      nflush = m;
      xb_fnow.reserve(std::max<int64_t>(m, 1) * 8);
      xb_fseq.reserve(std::max<int64_t>(m, 1) * 8);
      if (m > 0) {
        hipLaunchKernelGGL(k_xb_item_chunks, dim3(grid_cover(m)), dim3(kBlock), 0, s, C, m,
                           (const int32_t*)icall[cur].as<int32_t>(), (const int32_t*)irow[cur].as<int32_t>(),
                           (const int64_t*)d_call_now.as<int64_t>(), seq, xb_fnow.as<int64_t>(),
                           xb_fseq.as<int64_t>());
        SHD_CHECK_LAUNCH();
      }
    } else {
      // timeBatch: the flush schedule is sequential in the chunks (calls and
      // TIMER chunks), not in the events: run it on the host per call
      xb_ccount.reserve((size_t)ncalls * 4);
      xb_clast.reserve((size_t)ncalls * 8);
      SHD_HIP(hipMemsetAsync(xb_ccount.p, 0, (size_t)ncalls * 4, s));
      if (m > 0) {
        hipLaunchKernelGGL(k_xb_call_items, dim3(grid_cover(m)), dim3(kBlock), 0, s, C, m,
                           (const int32_t*)icall[cur].as<int32_t>(), (const int32_t*)irow[cur].as<int32_t>(), seq,
                           xb_ccount.as<uint32_t>(), xb_clast.as<int64_t>());
        SHD_CHECK_LAUNCH();
      }
      std::vector<uint32_t> cc(ncalls);
      std::vector<int64_t> cl(ncalls);
      h_pin.reserve((size_t)ncalls * 12);
      SHD_HIP(hipMemcpyAsync(h_pin.p, xb_ccount.p, (size_t)ncalls * 4, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipMemcpyAsync(h_pin.as<char>() + (size_t)ncalls * 4, xb_clast.p, (size_t)ncalls * 8,
                             hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
      std::memcpy(cc.data(), h_pin.p, (size_t)ncalls * 4);
      std::memcpy(cl.data(), h_pin.as<char>() + (size_t)ncalls * 4, (size_t)ncalls * 8);
      const bool stream_cur = bmode == XB_STREAM_TIME;
      // per call: full batches -- the flush its events join; stream mode -- its
      // chunk, the first flush at or after it, its RESET epoch
      std::vector<int32_t> bfl(ncalls, -1), cch(ncalls, -1), cfl(ncalls, -1);
      std::vector<int64_t> cep(ncalls, -1), fn, fs;
      std::vector<int> pending;
      auto flush_here = [&](int64_t t, int64_t sq) {   // a flush ends the current chunk list
        const int32_t f = (int32_t)fn.size();
        for (int pc : pending) (stream_cur ? cfl : bfl)[pc] = f;
        pending.clear();
        fn.push_back(t);
        fs.push_back(sq);
        if (stream_cur) tb_epoch = chunk_seq + f;   // RESET after this chunk's expirations
      };
      for (int c = 0; c < ncalls; c++) {
        if (moved[c]) {
          // Scheduler.sendTimerEvents (C/util/Scheduler.java:190-220): TIMER
          // chunks while the queue head is due, each through the window
          const int64_t t = h_now[c];
          while (!tb_notify.empty() && tb_notify.front() <= t) {
            tb_notify.pop_front();
            if (tb_process(t)) {
              if (xb.first_flush < 0) xb.first_flush = (int64_t)fn.size();
              flush_here(t, seq + h_offs[c]);
            }
          }
        }
        if (cc[c] > 0) {   // a chunk of events reaches the window
          pending.push_back(c);
          const bool send = tb_process(h_now[c]);
          if (stream_cur) {   // the call is a chunk of its own (its events stay in it)
            cch[c] = (int32_t)fn.size();
            cep[c] = tb_epoch;
            fn.push_back(h_now[c]);
            fs.push_back(cl[c]);
            if (send) {   // expirations appended to the same chunk
              for (int pc : pending) cfl[pc] = cch[c];
              pending.clear();
              if (xb.first_flush < 0) xb.first_flush = cch[c];
              tb_epoch = chunk_seq + cch[c];
            }
          } else if (send) {
            flush_here(h_now[c], cl[c]);
          }
        }
      }
      nflush = (int64_t)fn.size();
      upload(xb_fnow, fn);
      upload(xb_fseq, fs);
      if (stream_cur) {
        upload(xb_cchunk, cch);
        upload(xb_cflush, cfl);
        upload(xb_cepoch, cep);
        xb.cchunk = xb_cchunk.as<int32_t>();
        xb.cflush = xb_cflush.as<int32_t>();
        xb.cepoch = xb_cepoch.as<int64_t>();
      } else {
        upload(xb_bflush, bfl);
        xb.bflush = xb_bflush.as<int32_t>();
        xb.nf = nflush;
      }
    }
    if (total > 0) {
      hipLaunchKernelGGL(k_xb_opp, dim3(grid_cover(total)), dim3(kBlock), 0, s, dev_args(xb), bmode);
      SHD_CHECK_LAUNCH();
    }
    int64_t nops = 0;
    nops_b.reserve(ta * 4);
    opscan.reserve(ta * 4);
    if (total > 0) {
      hipLaunchKernelGGL(k_xb_nops, dim3(grid_cover(total)), dim3(kBlock), 0, s, total,
                         (const uint64_t*)xb_aopp.as<uint64_t>(), (const uint64_t*)eopp.as<uint64_t>(),
                         nops_b.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      nops = scan(nops_b.as<uint32_t>(), opscan.as<uint32_t>(), total);
    }
    reserve_ops(nops);
    op_epoch.reserve(std::max<int64_t>(nops, 1) * 8);
    if (nops > 0) {
      XbOpArgs oa{};
      oa.total = total;
      oa.sp = SP;
      oa.segid = segid.as<uint32_t>();
      oa.segS = segS.as<int64_t>();
      oa.segCk = segCk.as<int64_t>();
      oa.added_j = xb_added.as<uint8_t>();
      oa.aopp = xb_aopp.as<uint64_t>();
      oa.eopp = eopp.as<uint64_t>();
      oa.epoch_j = xb_epoch.as<int64_t>();
      oa.full = bmode == XB_FULL_LEN || bmode == XB_FULL_TIME;
      oa.opscan = opscan.as<uint32_t>();
      oa.fnow = xb_fnow.as<int64_t>();
      oa.fseq = xb_fseq.as<int64_t>();
      oa.current_on = plan.current_on;
      oa.expired_on = plan.expired_on;
      oa.op_epoch = op_epoch.as<int64_t>();
      oa.op_item = op_item.as<uint32_t>();
      oa.op_add = op_add.as<uint8_t>();
      oa.op_on = op_on.as<uint8_t>();
      oa.op_chunk = op_chunk.as<uint32_t>();
      oa.op_now = op_now.as<int64_t>();
      oa.op_seq = op_seq.as<int64_t>();
      hipLaunchKernelGGL(k_xb_ops, dim3(grid_cover(total)), dim3(kBlock), 0, s, dev_args(oa));
      SHD_CHECK_LAUNCH();
    }
    return nops;
  }

  // inclusive run id of each keyed event into d_start (k_xw_ops' run_of)
  void run_ids(int64_t n) {
    hipLaunchKernelGGL(k_xw_run_ids, dim3(grid_cover(n)), dim3(kBlock), 0, stream, n,
                       (const uint32_t*)d_run.as<uint32_t>(), d_start.as<uint32_t>());
    SHD_CHECK_LAUNCH();
  }

  int64_t scan_u8_flags(const uint8_t* f, int64_t n) {
    nops_b.reserve(n * 4);
    hipLaunchKernelGGL(k_xw_widen, dim3(grid_cover(n)), dim3(kBlock), 0, stream, f, n, nops_b.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    return scan(nops_b.as<uint32_t>(), roff.as<uint32_t>(), n);
  }

  void update_pending(int64_t nseg, int nf, bool lane_ran) {
    hipStream_t s = stream;
    int64_t nseg_out = 0;
    if (lane_ran && nseg > 0) {
      nseg_out = scan(pcnt.as<uint32_t>(), pcnt_off.as<uint32_t>(), nseg);
    }
    // orphans: queued entries of keys without items in this push
    okeep.reserve(std::max<int64_t>(np, 1) * 4);
    okoff.reserve(std::max<int64_t>(np, 1) * 4);
    seg_pk.reserve(std::max<int64_t>(nseg, 1) * 8);
    int64_t nork = 0;
    if (np > 0) {
      if (nseg > 0) {
        hipLaunchKernelGGL(k_xw_seg_pk, dim3(grid_cover(nseg)), dim3(kBlock), 0, s, nseg,
                           (const int64_t*)segS.as<int64_t>(), (const uint32_t*)sp.as<uint32_t>(),
                           (const uint64_t*)ipk[cur].as<uint64_t>(), seg_pk.as<uint64_t>());
        SHD_CHECK_LAUNCH();
      }
      hipLaunchKernelGGL(k_xw_orphans, dim3(grid_cover(np)), dim3(kBlock), 0, s, np, (const uint64_t*)ppk.as<uint64_t>(),
                         (const int64_t*)pv.as<int64_t>(), nseg, (const uint64_t*)seg_pk.as<uint64_t>(), nf,
                         (const int64_t*)d_fnow.as<int64_t>(), okeep.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      nork = scan(okeep.as<uint32_t>(), okoff.as<uint32_t>(), np);
    }
    const int64_t nn = nseg_out + nork;
    ppk2.reserve(std::max<int64_t>(nn, 1) * 8);
    pv2.reserve(std::max<int64_t>(nn, 1) * 8);
    if (nseg_out > 0)
      hipLaunchKernelGGL(k_xw_pend_gather, dim3(grid_cover(nseg)), dim3(kBlock), 0, s, nseg,
                         (const uint32_t*)proom_off.as<uint32_t>(), (const uint32_t*)pcnt.as<uint32_t>(),
                         (const uint32_t*)pcnt_off.as<uint32_t>(), (const uint64_t*)pout_pk.as<uint64_t>(),
                         (const int64_t*)pout_v.as<int64_t>(), ppk2.as<uint64_t>(), pv2.as<int64_t>());
    if (nork > 0)
      hipLaunchKernelGGL(k_xw_pend_orphan_copy, dim3(grid_cover(np)), dim3(kBlock), 0, s, np,
                         (const uint32_t*)okeep.as<uint32_t>(), (const uint32_t*)okoff.as<uint32_t>(), nseg_out,
                         (const uint64_t*)ppk.as<uint64_t>(), (const int64_t*)pv.as<int64_t>(), ppk2.as<uint64_t>(),
                         pv2.as<int64_t>());
    SHD_CHECK_LAUNCH();
    // both parts are key-sorted: one stable key sort merges them (values stay
    // in order inside a key: a key is in one part only)
    if (nseg_out > 0 && nork > 0) {
      pend_idx.reserve(nn * 4);
      pend_idx2.reserve(nn * 4);
      pend_key2.reserve(nn * 8);
      pend_tmp_pk.reserve(nn * 8);
      pend_tmp_v.reserve(nn * 8);
      fill_iota_u32(pend_idx.as<uint32_t>(), nn, 0, s);
      SHD_HIP(hipMemcpyAsync(pend_tmp_pk.p, ppk2.p, nn * 8, hipMemcpyDeviceToDevice, s));
      bool alt = false;
      radix_sort_pairs_u64(pend_tmp_pk.as<uint64_t>(), pend_idx.as<uint32_t>(), pend_key2.as<uint64_t>(),
                           pend_idx2.as<uint32_t>(), nn, 64, d_sort, s, alt);
      const uint32_t* perm = alt ? pend_idx2.as<uint32_t>() : pend_idx.as<uint32_t>();
      hipLaunchKernelGGL(k_xw_gather_u64, dim3(grid_cover(nn)), dim3(kBlock), 0, s, (const uint64_t*)ppk2.as<uint64_t>(),
                         perm, pend_tmp_pk.as<uint64_t>(), nn, 0ull);
      hipLaunchKernelGGL(k_xw_gather_u64, dim3(grid_cover(nn)), dim3(kBlock), 0, s, (const uint64_t*)pv2.as<uint64_t>(),
                         perm, pend_tmp_v.as<uint64_t>(), nn, 0ull);
      SHD_CHECK_LAUNCH();
      std::swap(ppk2.p, pend_tmp_pk.p); std::swap(ppk2.cap, pend_tmp_pk.cap);
      std::swap(pv2.p, pend_tmp_v.p); std::swap(pv2.cap, pend_tmp_v.cap);
    }
    SHD_HIP(hipStreamSynchronize(s));
    std::swap(ppk.p, ppk2.p); std::swap(ppk.cap, ppk2.cap);
    std::swap(pv.p, pv2.p); std::swap(pv.cap, pv2.cap);
    np = nn;
  }

  // ---- snapshot: window items, notify queue, aggregator states, dictionary
  void save_state(SnapW& w) override {
    w.put<int64_t>(C);
    w.put<int32_t>(ncols);
    w.put<int32_t>(nagg);
    w.put<int64_t>(np);
    w.put<int64_t>(last_global);
    w.put<int64_t>(nstates);
    if (C > 0) {
      w.dev(ipk[cur].p, C * 8);
      w.dev(its[cur].p, C * 8);
      w.dev(iseq[cur].p, C * 8);
      w.dev(isid[cur].p, C * 8);
      w.dev(ilast[cur].p, C * 8);
      for (int c = 0; c < ncols; c++) {
        w.dev(iattr[cur].as<uint64_t>() + c * icap[cur], C * 8);
        w.dev(inul[cur].as<uint8_t>() + c * icap[cur], C);
      }
      for (int g = 0; g < nagg; g++) {
        w.dev(iargv[cur].as<uint64_t>() + g * icap[cur], C * 8);
        w.dev(iargn[cur].as<uint8_t>() + g * icap[cur], C);
      }
    }
    if (np > 0) {
      w.dev(ppk.p, np * 8);
      w.dev(pv.p, np * 8);
    }
    if (nagg > 0 && nstates > 0) {
      w.dev(g_dsum.p, (size_t)nagg * nstates * 8);
      w.dev(g_lsum.p, (size_t)nagg * nstates * 8);
      w.dev(g_cnt.p, (size_t)nagg * nstates * 8);
    }
    gd.save(w);
    // batch windows: RESET epochs, timeBatch's nextEmitTime and notify queue
    w.put<int64_t>(tb_next);
    w.put<int64_t>(tb_epoch);
    w.put<int64_t>((int64_t)tb_notify.size());
    for (int64_t t : tb_notify) w.put<int64_t>(t);
    if (batch && nagg > 0 && nstates > 0) w.dev(g_epoch.p, (size_t)nstates * 8);
  }
  void load_state(SnapR& r) override {
    const int64_t c0 = r.get<int64_t>();
    if (r.get<int32_t>() != ncols || r.get<int32_t>() != nagg || c0 < 0)
      throw Error(SHD_E_ARG, "snapshot of a different plan");
    const int64_t np0 = r.get<int64_t>();
    last_global = r.get<int64_t>();
    const int64_t ns = r.get<int64_t>();
    C = 0;
    cur = 0;
    if (c0 > 0) {
      if (icap[0] < c0) alloc_slot(0, std::max<int64_t>(c0, 1024));
      r.dev_into(ipk[0].p, c0 * 8);
      r.dev_into(its[0].p, c0 * 8);
      r.dev_into(iseq[0].p, c0 * 8);
      r.dev_into(isid[0].p, c0 * 8);
      r.dev_into(ilast[0].p, c0 * 8);
      for (int c = 0; c < ncols; c++) {
        r.dev_into(iattr[0].as<uint64_t>() + c * icap[0], c0 * 8);
        r.dev_into(inul[0].as<uint8_t>() + c * icap[0], c0);
      }
      for (int g = 0; g < nagg; g++) {
        r.dev_into(iargv[0].as<uint64_t>() + g * icap[0], c0 * 8);
        r.dev_into(iargn[0].as<uint8_t>() + g * icap[0], c0);
      }
      SHD_HIP(hipMemsetAsync(icall[0].p, 0xFF, c0 * 4, stream));
      SHD_HIP(hipMemsetAsync(irow[0].p, 0xFF, c0 * 4, stream));
    }
    C = c0;
    np = np0;
    if (np > 0) {
      ppk.reserve(np * 8);
      pv.reserve(np * 8);
      r.dev_into(ppk.p, np * 8);
      r.dev_into(pv.p, np * 8);
    }
    if (nagg > 0 && ns > 0) {
      nstates = 0;
      ensure_states(ns);
      if (nstates != ns) {   // restore into tables of exactly the saved size
        g_dsum.release(); g_lsum.release(); g_cnt.release();
        g_dsum.reserve((size_t)nagg * ns * 8);
        g_lsum.reserve((size_t)nagg * ns * 8);
        g_cnt.reserve((size_t)nagg * ns * 8);
        if (batch) {
          g_epoch.release();
          g_epoch.reserve((size_t)ns * 8);
        }
        nstates = ns;
      }
      r.dev_into(g_dsum.p, (size_t)nagg * ns * 8);
      r.dev_into(g_lsum.p, (size_t)nagg * ns * 8);
      r.dev_into(g_cnt.p, (size_t)nagg * ns * 8);
    } else {
      nstates = ns;
    }
    gd.nk = std::max(nw, 1);
    gd.load(r, stream);
    tb_next = r.get<int64_t>();
    tb_epoch = r.get<int64_t>();
    tb_notify.clear();
    const int64_t nn = r.get<int64_t>();
    for (int64_t i = 0; i < nn; i++) tb_notify.push_back(r.get<int64_t>());
    if (batch && nagg > 0 && nstates > 0) r.dev_into(g_epoch.p, (size_t)nstates * 8);
    counters.carry = C;
  }
};

std::unique_ptr<Engine> make_window_x_engine(const Plan& p, std::string& why) {
  if (p.kind != SHD_KIND_SINGLE) { why = "not a single-stream query"; return nullptr; }
  auto e = std::make_unique<WindowXEngine>();
  const auto& types = p.stream_types[p.single_stream];
  if (types.size() > (size_t)kMaxCols) { why = "too many attributes"; return nullptr; }
  e->ncols = (int)types.size();
  bool seen_window = false;
  for (auto& h : p.handlers) {
    if (h.kind == SHD_H_FILTER) {
      if (seen_window) { why = "filter after window"; return nullptr; }
      e->filters.push_back(h.expr);
    } else {
      seen_window = true;
      e->wkind = h.wkind;
      e->wparam = h.param;
      e->wparam2 = h.param2;
    }
  }
  if (e->filters.size() > 4) { why = "too many filters"; return nullptr; }
  if (e->wkind == SHD_W_LENGTH && e->wparam <= 0) { why = "length(0) window"; return nullptr; }
  e->batch = e->wkind == SHD_W_LENGTH_BATCH || e->wkind == SHD_W_TIME_BATCH || e->wkind == SHD_W_TIME_BATCH_STREAM;
  if (e->wkind == SHD_W_LENGTH_BATCH)
    e->bmode = e->wparam == 0 ? XB_ZERO_LEN : ((e->wparam2 & 1) ? XB_STREAM_LEN : XB_FULL_LEN);
  else if (e->wkind == SHD_W_TIME_BATCH)
    e->bmode = XB_FULL_TIME;
  else if (e->wkind == SHD_W_TIME_BATCH_STREAM)
    e->bmode = XB_STREAM_TIME;
  if (e->wkind == SHD_W_EXTERNAL_TIME && (e->wparam2 < 0 || e->wparam2 >= e->ncols)) {
    why = "externalTime attribute";
    return nullptr;
  }
  if (e->wkind == SHD_W_TIME_LENGTH && (e->wparam2 <= 0 || e->wparam < 0)) {
    why = "timeLength window of length 0";
    return nullptr;
  }
  if (e->batch && e->wparam <= 0 && e->bmode != XB_ZERO_LEN) { why = "batch window of time 0"; return nullptr; }
  if (e->wkind == SHD_W_TIME && e->wparam < 0) { why = "negative time window"; return nullptr; }
  if (p.outputs.size() > (size_t)kMaxCols) { why = "too many outputs"; return nullptr; }
  e->nagg = (int)p.aggs.size();
  if (e->nagg > kMaxAggs) { why = "too many aggregators"; return nullptr; }
  e->partitioned = !p.part_keys.empty();
  if (e->partitioned) {
    e->key_expr = p.part_keys[0].second;
    const auto& code = p.exprs[e->key_expr];
    e->key_col = (code.size() == 1 && code[0].op == SHD_OP_LOAD) ? (code[0].c & 0xFFFF) : -1;
    e->key_type = expr_result_type(p, e->key_expr, {});
  }
  if (p.group_by.size() > (size_t)kMaxGroupAttrs) { why = "more than 4 group-by attributes"; return nullptr; }
  e->ngk = (int)p.group_by.size();
  for (int g = 0; g < e->ngk; g++) {
    e->gk_expr[g] = p.group_by[g];
    const auto& code = p.exprs[e->gk_expr[g]];
    e->gk_col[g] = (code.size() == 1 && code[0].op == SHD_OP_LOAD) ? (code[0].c & 0xFFFF) : -1;
    e->gk_type[g] = expr_result_type(p, e->gk_expr[g], {});
  }
  e->group = e->ngk > 0;
  e->plain = e->ngk == 0 && e->nagg == 0;
  // state key words: (partition key, group words); none for one global state
  e->nw = e->plain ? 0 : (e->partitioned ? 1 : 0) + e->ngk;
  e->gd.nk = std::max(e->nw, 1);
  return e;
}

}  // namespace shd
