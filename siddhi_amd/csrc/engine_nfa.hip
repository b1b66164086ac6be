// engine_nfa.hip -- generic per-key NFA engine: every pattern / sequence plan
// the pattern forward-scan engine does not take (config S4: count <m:n> states
// with e2[last] chains, logical and/or, absent `not X for t`, sequences,
// multi-state chains), optionally inside `partition with`.
//
// Reference semantics restated here (modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/input/stream/state/StreamPreStateProcessor.java:118-403   (init/addState/
//       addEveryState/resetState/updateState/expireEvents/processAndReturn)
//   query/input/stream/state/StreamPostStateProcessor.java:64-83
//   query/input/stream/state/CountPreStateProcessor.java:52-193, CountPostStateProcessor.java:39-89
//   query/input/stream/state/LogicalPreStateProcessor.java:43-201, LogicalPostStateProcessor.java:59-129
//   query/input/stream/state/AbsentStreamPreStateProcessor.java:67-308 (+ AbsentStreamPostStateProcessor)
//   query/input/stream/state/runtime/*InnerStateRuntime.java  (init / reset / update order)
//   query/input/stream/state/receiver/*.java, query/input/{Single,Multi,StateMulti}ProcessStreamReceiver.java
//       (stabilizeStates, reverse state order, deferred callback chunks)
//   util/parser/StateInputStreamParser.java:148-408 (processor wiring, restated on the host below)
//   partition/PartitionStreamReceiver.java:175-283 (same-key runs, first-sight seeding)
//   util/Scheduler.java:71-209 (playback TIMERs for absent states)
//
// MI355X mapping.  All NFA state of one partition key lives in an HBM "key
// block": pending / newAndEvery lists of StateEvent handles per pre-processor,
// a StateEvent pool (one event-chain head per state slot), a StreamEvent
// clone pool (chain links) and an event-record pool (the attributes of every
// event a partial still references), plus flags and scheduler queues.  Blocks
// are interleaved 64 keys wide (element e of key k sits at e*64 + k%64), so
// the lanes of a wave that walk their keys through the same processor touch
// consecutive words.  One lane advances one key through its key-sorted events
// in arrival order (the reference serialises a key the same way); keys run in
// parallel.  Object identity (the reference shares StateEvent / StreamEvent
// objects between lists) is kept with handles; unreachable objects are
// reclaimed by a per-key mark-sweep between events.  Output rows are staged
// with (event seq, timer time, key) ordering tags and sorted into the
// reference's callback order on the device.
#include <algorithm>
#include <functional>
#include <cstddef>
#include <cstdio>
#include <cstdlib>

#include "engine.h"

namespace shd {

namespace {

constexpr int kNP = 16;        // pre/post processors per plan
constexpr int kNS = 16;        // StateEvent slots
constexpr int kNStream = 8;    // plan streams
constexpr int kNSched = 8;     // absent-state schedulers
constexpr uint16_t NIL = 0xFFFF;
constexpr int kLaneBlock = 64;

enum : int { PK_STREAM = 0, PK_COUNT = 1, PK_LOGICAL = 2, PK_ABSENT = 3, PK_ABSENT_LOGICAL = 4 };
enum : uint8_t { FL_CHANGED = 1, FL_INIT = 2, FL_STARTED = 4, FL_SUCCESS = 8, FL_SSRESET = 16, FL_INACTIVE = 32 };
enum : uint32_t {
  OV_LIST = 1, OV_SE = 2, OV_EV = 4, OV_REC = 8, OV_SCHED = 16, OV_RET = 32, OV_WORK = 64, OV_ROWS = 128,
  OV_MULTI = 256   // list arena of multi-value outputs
};
enum : int {
  MISC_SEEDED = 0, MISC_EVRET = 1, MISC_WKN = 2, MISC_RETN = 3, MISC_TMPN = 4,
  MISC_FREE_SE = 5, MISC_FREE_EV = 6, MISC_FREE_REC = 7, MISC_HINT_SE = 8, MISC_HINT_EV = 9, MISC_HINT_REC = 10,
  MISC_HSTAMP = 11, MISC_N = 12
};

struct DPre {
  int kind, stateId, isStart, stream, thisPost, thisLast, withinEvery, partner, sched, minC, maxC, ltype;
  int64_t waiting;
  DFilters filters;
};

struct DPost {
  int kind, pre, stateId, nextPre, nextEvery, callbackPre, partnerPre, partnerPost, minC, maxC, ltype, hasSelector;
};

// The processor graph of one plan (StateInputStreamParser output), uniform over keys.
struct NfaProg {
  int npre, nstates, nsched, seq, nstart, nout, current_on, expired_on;
  uint32_t multi_mask;            // outputs that are SHD_OP_MULTI lists
  int64_t within;                 // -1: no `within`
  int startIds[kNP];
  DPre pre[kNP];
  DPost post[kNP];
  int nall, allPre[kNP];          // allStateProcessors (expireEvents order)
  int ninit, initSeq[kNP];        // InnerStateRuntime.init order
  int nreset, resetSeq[kNP];      // InnerStateRuntime.reset order (sequences)
  int nupd, updSeq[kNP];          // InnerStateRuntime.update order (sequences)
  int nsp[kNStream], streamPres[kNStream][kNP];
  int schedPre[kNSched];
  DExpr outs[kMaxCols];
};

// Byte offsets of the per-key fields inside one 64-key block.
struct NfaLayout {
  int L, SC, EC, RC, QC, RETC, WK;   // capacities
  int ncols, nstates, npre, nsched;
  int sew, evw, recw;                // bitmap words
  int64_t o_pend, o_pend_n, o_new, o_new_n, o_flags, o_lst, o_sq, o_sq_n;
  int64_t o_se_ev, o_se_ts, o_se_type, o_se_free, o_se_mark;
  int64_t o_ev_rec, o_ev_next, o_ev_free, o_ev_mark;
  int64_t o_rec_ts, o_rec_val, o_rec_nul, o_rec_free, o_rec_mark;
  int64_t o_ret, o_tmp, o_wk, o_key, o_misc;
  int64_t o_cse, o_cev;              // canonical ids (window-lane state hashes)
  int64_t blk;   // bytes of one block of W key states
  int W;         // key states interleaved per block: 64 (lock-step keys) or 1 (one key contiguous)
  // field table (one key's state = these fields, lane-interleaved): lane copies
  static constexpr int kMaxFields = 40;
  int nf;
  int f_sz[kMaxFields];
  int64_t f_off[kMaxFields], f_cnt[kMaxFields];
};

// SHD_NFA_PROF builds: per-phase shader-clock totals over all lanes (ctl->prof)
#ifdef SHD_NFA_PROF
#define NFA_PROF_T0(v) const uint64_t v = __builtin_amdgcn_s_memtime()
#define NFA_PROF_ADD(k, v) prof[k] += __builtin_amdgcn_s_memtime() - v
#define NFA_PROF_ADDL(o, k, v) o.prof[k] += __builtin_amdgcn_s_memtime() - v
#else
#define NFA_PROF_ADDL(o, k, v)
#define NFA_PROF_T0(v)
#define NFA_PROF_ADD(k, v)
#endif
constexpr int kProfN = 8;

struct NfaCtl {
  unsigned long long prof[kProfN];
  unsigned long long rows;
  unsigned long long partials;
  unsigned long long scans;
  unsigned long long live;
  unsigned long long kmax;
  unsigned int overflow;
  unsigned int count;   // scan totals / slot counter
  unsigned long long lrows;   // list arena entries written (multi-value outputs)
};

struct NfaRunArgs {
  ColSet batch;
  int stream;
  int partitioned;
  int lanes_over_slots;
  int ncalls;
  int64_t n_keyed;      // events handed to lanes (rows[] length)
  int64_t nlanes;
  int64_t seq0;
  int64_t start_time;   // app start (seed of unpartitioned plans)
  const uint8_t* skip_start;   // hand-over replay: rows the start state does not see (Replay::skip_start)
  // window-lane mode (unpartitioned every-started plans): lane c owns the
  // events [c*chunk_len, (c+1)*chunk_len); lanes c < c_exact start at row 0
  // from a copy of the carried state (exact), the others replay the `warm`
  // events before their chunk from a fresh state, output suppressed
  int64_t chunk_len;
  int64_t warm;
  int64_t c_exact;
  uint64_t* hash_w;   // per lane: state hashes after the warm-up (= before the first owned event), 2 words
  uint64_t* hash_e;   // per lane: state hashes after the last owned event, 2 words
  int hash1_zero;     // debug hook (SHD_NFA_HASH1_ZERO): the first hash always collides
  const int32_t* call_of;
  const int64_t* call_now;
  const uint8_t* call_changed;
  const int64_t* call_first;   // global seq of each call's first event
  const uint32_t* run_id;
  const uint32_t* rows;        // key-sorted event rows (nullptr: identity)
  const uint32_t* seg_start;   // [nseg]
  const uint32_t* seg_slot;    // [nseg]
  const int32_t* slot_seg;     // [nslots] (-1: no events this push)
  int64_t nseg;
  char* state;
  DExprSet es;
  // staged output rows
  int64_t R;
  uint64_t *st_tag, *st_p, *st_s, *st_t;
  int32_t* st_sidx;
  int64_t* st_ts;
  int32_t* st_type;
  uint64_t* st_vals;
  uint8_t* st_nul;
  int64_t LR;          // list arena capacity (entries)
  uint64_t* st_lv;     // list arena values
  uint8_t* st_ln;      // list arena null flags
  NfaCtl* ctl;
};

struct KS {
  char* b;
  int l;
  int w;   // interleave width of the block (NfaLayout::W)
  template <class T>
  __device__ __forceinline__ T& at(int64_t off, int64_t e) const {
    return *reinterpret_cast<T*>(b + off + (e * w + l) * (int64_t)sizeof(T));
  }
};

struct Lane;

// Expression context over one StateEvent (StateEvent.getStreamEvent(int[]),
// C/event/state/StateEvent.java:138-182).
struct SECtx {
  Lane* L;
  uint16_t se;
  __device__ Val load(int st, int idx, int attr) const;
  __device__ bool evnull(int st, int idx) const;
  __device__ int64_t ts(int st, int idx) const;
  __device__ Val agg(int) const {
    Val v;
    v.b = 0;
    v.null = 1;
    return v;
  }
};

struct Lane {
  const NfaProg& P;
  const NfaLayout& Y;
  const NfaRunArgs& A;
  DExprSet es;
  KS ks;
  int64_t slot;
  uint64_t key;
  uint32_t evret;
  uint32_t ovf;
  unsigned long long partials, scans;
  uint32_t tagc;
  uint64_t t_prim, t_sec, t_ter;
  int32_t cur_state = 0;   // state id of the processor whose rows emit() stages (shd_out.state_idx)
  int32_t ret_state = 0;   // single-receiver runs: the state of the returned events
  int64_t last_seq;
  bool quiet;   // window lanes: warm-up events (no output)
#ifdef SHD_NFA_PROF
  uint64_t prof[kProfN] = {};
#endif
  int cdone;

  __device__ Lane(const NfaProg& p, const NfaLayout& y, const NfaRunArgs& a, DExprSet e)
      : P(p), Y(y), A(a), es(e) {}

  // ---------------------------------------------------------------- fields
  __device__ __forceinline__ uint8_t& fl(int p) { return ks.at<uint8_t>(Y.o_flags, p); }
  __device__ __forceinline__ int64_t& lst(int p) { return ks.at<int64_t>(Y.o_lst, p); }
  __device__ __forceinline__ uint16_t& pend(int p, int i) { return ks.at<uint16_t>(Y.o_pend, (int64_t)p * (Y.L + 1) + i); }
  __device__ __forceinline__ uint16_t& pn(int p) { return ks.at<uint16_t>(Y.o_pend_n, p); }
  __device__ __forceinline__ uint16_t& nw(int p, int i) { return ks.at<uint16_t>(Y.o_new, (int64_t)p * (Y.L + 1) + i); }
  __device__ __forceinline__ uint16_t& nn(int p) { return ks.at<uint16_t>(Y.o_new_n, p); }
  __device__ __forceinline__ uint16_t& sev(int s, int st) { return ks.at<uint16_t>(Y.o_se_ev, (int64_t)s * Y.nstates + st); }
  __device__ __forceinline__ int64_t& sts(int s) { return ks.at<int64_t>(Y.o_se_ts, s); }
  __device__ __forceinline__ uint8_t& stype(int s) { return ks.at<uint8_t>(Y.o_se_type, s); }
  __device__ __forceinline__ uint16_t& erec(int e) { return ks.at<uint16_t>(Y.o_ev_rec, e); }
  __device__ __forceinline__ uint16_t& enext(int e) { return ks.at<uint16_t>(Y.o_ev_next, e); }
  __device__ __forceinline__ int64_t& rts(int r) { return ks.at<int64_t>(Y.o_rec_ts, r); }
  __device__ __forceinline__ uint64_t& rval(int r, int c) { return ks.at<uint64_t>(Y.o_rec_val, (int64_t)r * Y.ncols + c); }
  __device__ __forceinline__ uint32_t& rnul(int r) { return ks.at<uint32_t>(Y.o_rec_nul, r); }
  __device__ __forceinline__ int64_t& sq(int sc, int i) { return ks.at<int64_t>(Y.o_sq, (int64_t)sc * Y.QC + i); }
  __device__ __forceinline__ uint16_t& sqn(int sc) { return ks.at<uint16_t>(Y.o_sq_n, sc); }
  __device__ __forceinline__ uint16_t& retl(int i) { return ks.at<uint16_t>(Y.o_ret, i); }
  __device__ __forceinline__ uint16_t& tmpl(int i) { return ks.at<uint16_t>(Y.o_tmp, i); }
  __device__ __forceinline__ uint32_t& wk(int i) { return ks.at<uint32_t>(Y.o_wk, i); }
  __device__ __forceinline__ uint32_t& misc(int i) { return ks.at<uint32_t>(Y.o_misc, i); }
  __device__ __forceinline__ uint64_t& bits(int64_t off, int w) { return ks.at<uint64_t>(off, w); }

  // ---------------------------------------------------------------- window lanes
  // Canonical hash of the key's NFA state (pending / new lists in order, each
  // StateEvent by content -- timestamp, type, event chains by event record --
  // with object identity kept: a StateEvent or StreamEvent seen before hashes
  // as its first-visit index, so shared objects (count-state aliasing) and
  // equal copies differ).  Two lanes whose states hash equal continue equally.
  // canonical ids carry the hash call's stamp in the high half (no clearing)
  __device__ uint32_t& cse(int i) { return ks.at<uint32_t>(Y.o_cse, i); }
  __device__ uint32_t& cev(int i) { return ks.at<uint32_t>(Y.o_cev, i); }
  // Two independent 64-bit hashes over the same canonical walk (an FNV-style
  // xor-multiply and a splitmix-style add-multiply-xorshift with other
  // constants): a lane is accepted only when both agree, so a wrong warm-up
  // state slips through only if it collides in both.
  __device__ uint64_t state_hash(uint64_t& h2) {
    uint64_t h = 1469598103934665603ull;
    uint64_t g = 0x6A09E667F3BCC909ull;
    auto mix = [&](uint64_t x) {
      h ^= x;
      h *= 1099511628211ull;
      h ^= h >> 29;
      g += x + 0x9E3779B97F4A7C15ull;
      g *= 0xBF58476D1CE4E5B9ull;
      g ^= g >> 31;
    };
    uint32_t stamp = (misc(MISC_HSTAMP) + 1) & 0xFFFFu;
    if (stamp == 0) {   // wrapped: clear once
      for (int i = 0; i <= Y.SC; i++) cse(i) = 0;
      for (int i = 0; i <= Y.EC; i++) cev(i) = 0;
      stamp = 1;
    }
    misc(MISC_HSTAMP) = stamp;
    const uint32_t hi = stamp << 16;
    uint32_t nse = 0, nev = 0;
    auto hse = [&](uint16_t s) {
      if (s > Y.SC) return;
      if ((cse(s) & 0xFFFF0000u) == hi) {
        mix(0xA0000ull + (cse(s) & 0xFFFFu));
        return;
      }
      cse(s) = hi | nse++;
      mix(0xB0000ull);
      mix((uint64_t)sts(s));
      mix(stype(s));
      for (int st = 0; st < Y.nstates; st++) {
        mix(0xC0000ull + st);
        for (uint16_t e = sev(s, st); e != NIL && e < Y.EC; e = enext(e)) {
          if ((cev(e) & 0xFFFF0000u) == hi) {
            mix(0xD0000ull + (cev(e) & 0xFFFFu));
            break;
          }
          cev(e) = hi | nev++;
          const uint16_t r = erec(e);
          if (r >= Y.RC) continue;
          mix((uint64_t)rts(r));
          for (int c = 0; c < Y.ncols; c++) mix(rval(r, c));
          mix(rnul(r));
        }
      }
    };
    for (int p = 0; p < P.npre; p++) {
      mix(fl(p));
      mix((uint64_t)lst(p));
      const int a = pn(p), b = nn(p);
      mix(0xE0000ull + a);
      for (int i = 0; i < a; i++) hse(pend(p, i));
      mix(0xF0000ull + b);
      for (int i = 0; i < b; i++) hse(nw(p, i));
    }
    const int rn = misc(MISC_RETN);
    mix(0x100000ull + rn);
    for (int i = 0; i < rn; i++) hse(retl(i));
    for (int sc = 0; sc < P.nsched; sc++) {
      const int n = sqn(sc);
      mix(0x110000ull + n);
      for (int i = 0; i < n; i++) mix((uint64_t)sq(sc, i));
    }
    mix(evret);
    mix(misc(MISC_SEEDED) != 0);
    h2 = g;
    return h;
  }

  // ---------------------------------------------------------------- pools
  // first free handle at or after the hint word (wrapping); cap = sink on exhaustion
  __device__ int alloc_bit(int64_t off, int words, int cap, uint32_t ov, int mfree, int mhint) {
    int h = (int)misc(mhint);
    if (h >= words) h = 0;
    for (int k = 0; k < words; k++) {
      int w = h + k < words ? h + k : h + k - words;
      uint64_t& f = bits(off, w);
      uint64_t v = f;
      if (v) {
        int b = __builtin_ctzll(v);
        f = v & (v - 1);
        misc(mhint) = (uint32_t)w;
        misc(mfree) -= 1;
        return w * 64 + b;
      }
    }
    ovf |= ov;
    return cap;   // sink element (never referenced as live)
  }
  __device__ void fill_free(int64_t off, int words, int cap) {
    for (int w = 0; w < words; w++) {
      int valid = cap - w * 64;
      bits(off, w) = valid >= 64 ? ~0ull : (valid <= 0 ? 0ull : ((1ull << valid) - 1));
    }
  }

  __device__ uint16_t new_se() {
    int s = alloc_bit(Y.o_se_free, Y.sew, Y.SC, OV_SE, MISC_FREE_SE, MISC_HINT_SE);
    for (int i = 0; i < Y.nstates; i++) sev(s, i) = NIL;
    sts(s) = -1;
    stype(s) = SHD_EV_CURRENT;
    partials++;
    return (uint16_t)s;
  }
  __device__ uint16_t clone_se(uint16_t o) {   // StateEventCloner.copyStateEvent
    int s = alloc_bit(Y.o_se_free, Y.sew, Y.SC, OV_SE, MISC_FREE_SE, MISC_HINT_SE);
    for (int i = 0; i < Y.nstates; i++) sev(s, i) = sev(o, i);
    sts(s) = sts(o);
    stype(s) = stype(o);
    partials++;
    return (uint16_t)s;
  }
  __device__ uint16_t new_ev(uint16_t rec) {   // StreamEventCloner.copyStreamEvent
    int e = alloc_bit(Y.o_ev_free, Y.evw, Y.EC, OV_EV, MISC_FREE_EV, MISC_HINT_EV);
    erec(e) = rec;
    enext(e) = NIL;
    return (uint16_t)e;
  }
  // a clone that was never linked anywhere else (its filter failed) goes straight back
  __device__ void free_ev(uint16_t e) {
    if (e >= Y.EC) return;
    bits(Y.o_ev_free, e >> 6) |= 1ull << (e & 63);
    misc(MISC_FREE_EV) += 1;
  }

  // list helpers (capacity L, element L is the overflow sink)
  __device__ void push_new(int p, uint16_t s) {
    uint16_t n = nn(p);
    if (n >= Y.L) {
      ovf |= OV_LIST;
      return;
    }
    nw(p, n) = s;
    nn(p) = n + 1;
  }
  __device__ void push_tmp(uint16_t s) {
    uint32_t n = misc(MISC_TMPN);
    if ((int)n >= Y.RETC) {
      ovf |= OV_RET;
      return;
    }
    tmpl(n) = s;
    misc(MISC_TMPN) = n + 1;
  }
  __device__ void push_ret(uint16_t s) {
    uint32_t n = misc(MISC_RETN);
    if ((int)n >= Y.RETC) {
      ovf |= OV_RET;
      return;
    }
    retl(n) = s;
    misc(MISC_RETN) = n + 1;
  }

  // Scheduler.notifyAt: toNotifyQueue is a priority queue (duplicates kept)
  __device__ void notifyAt(int sc, int64_t t) {
    if (sc < 0) return;
    int n = sqn(sc);
    if (n >= Y.QC) {
      ovf |= OV_SCHED;
      return;
    }
    int i = n;
    while (i > 0 && sq(sc, i - 1) > t) {
      sq(sc, i) = sq(sc, i - 1);
      i--;
    }
    sq(sc, i) = t;
    sqn(sc) = (uint16_t)(n + 1);
  }

  // ---------------------------------------------------------------- chains
  // StateEvent.getStreamEvent(int[]) over one slot's chain (StateEvent.java:138-182)
  __device__ uint16_t chain_get(uint16_t e, int idx) {
    if (e == NIL) return NIL;
    if (idx >= 0) {
      for (int i = 1; i <= idx; i++) {
        e = enext(e);
        if (e == NIL) return NIL;
      }
      return e;
    }
    if (idx == SHD_IDX_CURRENT) {
      while (enext(e) != NIL) e = enext(e);
      return e;
    }
    if (idx == SHD_IDX_LAST) {
      if (enext(e) == NIL) return NIL;
      while (enext(enext(e)) != NIL) e = enext(e);
      return e;
    }
    int len = 0;
    for (uint16_t x = e; x != NIL; x = enext(x)) len++;
    int k = len + idx;
    if (k < 0) return NIL;
    for (int i = 0; i < k; i++) e = enext(e);
    return e;
  }
  __device__ int64_t ev_ts(uint16_t e) { return rts(erec(e)); }

  // ---------------------------------------------------------------- GC
  __device__ bool mark(int64_t off, int h) {
    uint64_t& w = bits(off, h >> 6);
    uint64_t m = 1ull << (h & 63);
    if (w & m) return false;
    w |= m;
    return true;
  }
  __device__ void mark_se(uint16_t s) {
    if (s >= Y.SC) return;
    if (!mark(Y.o_se_mark, s)) return;
    for (int st = 0; st < Y.nstates; st++) {
      for (uint16_t e = sev(s, st); e != NIL && e < Y.EC; e = enext(e)) {
        if (!mark(Y.o_ev_mark, e)) break;   // shared tail already marked
        uint16_t r = erec(e);
        if (r < Y.RC) mark(Y.o_rec_mark, r);
      }
    }
  }
  __device__ int sweep(int64_t off_free, int64_t off_mark, int words, int cap) {
    int n = 0;
    for (int w = 0; w < words; w++) {
      int valid = cap - w * 64;
      uint64_t vm = valid >= 64 ? ~0ull : (valid <= 0 ? 0ull : ((1ull << valid) - 1));
      uint64_t f = ~bits(off_mark, w) & vm;
      bits(off_free, w) = f;
      n += __popcll(f);
    }
    return n;
  }
  __device__ void gc() {
    for (int w = 0; w < Y.sew; w++) bits(Y.o_se_mark, w) = 0;
    for (int w = 0; w < Y.evw; w++) bits(Y.o_ev_mark, w) = 0;
    for (int w = 0; w < Y.recw; w++) bits(Y.o_rec_mark, w) = 0;
    for (int p = 0; p < P.npre; p++) {
      int a = pn(p), b = nn(p);
      for (int i = 0; i < a; i++) mark_se(pend(p, i));
      for (int i = 0; i < b; i++) mark_se(nw(p, i));
    }
    int rn = misc(MISC_RETN), tn = misc(MISC_TMPN);
    for (int i = 0; i < rn; i++) mark_se(retl(i));
    for (int i = 0; i < tn; i++) mark_se(tmpl(i));
    misc(MISC_FREE_SE) = (uint32_t)sweep(Y.o_se_free, Y.o_se_mark, Y.sew, Y.SC);
    misc(MISC_FREE_EV) = (uint32_t)sweep(Y.o_ev_free, Y.o_ev_mark, Y.evw, Y.EC);
    misc(MISC_FREE_REC) = (uint32_t)sweep(Y.o_rec_free, Y.o_rec_mark, Y.recw, Y.RC);
    misc(MISC_HINT_SE) = misc(MISC_HINT_EV) = misc(MISC_HINT_REC) = 0;
  }
  __device__ void maybe_gc() {
    if ((int)misc(MISC_FREE_SE) * 4 < Y.SC || (int)misc(MISC_FREE_EV) * 4 < Y.EC ||
        (int)misc(MISC_FREE_REC) * 4 < Y.RC)
      gc();
  }

  // ---------------------------------------------------------------- StreamPreStateProcessor
  __device__ bool isExpired(uint16_t s, int64_t t) {   // :118-129
    if (P.within < 0) return false;
    for (int i = 0; i < P.nstart; i++) {
      uint16_t e = sev(s, P.startIds[i]);
      if (e != NIL) {
        int64_t d = ev_ts(e) - t;
        if (d < 0) d = -d;
        if (d > P.within) return true;
      }
    }
    return false;
  }

  __device__ void init_pre(int p) {   // :178-194
    const DPre& pr = P.pre[p];
    const DPost& ps = P.post[pr.thisPost];
    if (pr.isStart &&
        (!(fl(p) & FL_INIT) || ps.nextEvery >= 0 ||
         (P.seq && ps.nextPre >= 0 &&
          (P.pre[ps.nextPre].kind == PK_ABSENT || P.pre[ps.nextPre].kind == PK_ABSENT_LOGICAL)))) {
      uint16_t s = new_se();
      addState(p, s);
      fl(p) |= FL_INIT;
    }
  }

  // addState with the CountPreStateProcessor min-count-0 forwarding
  // (:126-137 -> CountPostStateProcessor.processMinCountReached) unrolled
  // onto a per-key work stack (depth-first, same order as the recursion).
  __device__ void wk_push(uint32_t v) {
    uint32_t n = misc(MISC_WKN);
    if ((int)n >= Y.WK) {
      ovf |= OV_WORK;
      return;
    }
    wk(n) = v;
    misc(MISC_WKN) = n + 1;
  }
  __device__ void addState(int p0, uint16_t s0) {
    const uint32_t base = misc(MISC_WKN);
    wk_push(((uint32_t)p0 << 16) | s0);
    while (misc(MISC_WKN) > base) {
      uint32_t n = misc(MISC_WKN) - 1;
      uint32_t v = wk(n);
      misc(MISC_WKN) = n;
      int p = (v >> 16) & 0x7FFF;
      uint16_t s = (uint16_t)(v & 0xFFFF);
      if (v >> 31) {
        addEveryState(p, s);
        continue;
      }
      const DPre& pr = P.pre[p];
      switch (pr.kind) {
        case PK_STREAM:
          if (P.seq) {
            if (nn(p) == 0) push_new(p, s);
          } else {
            push_new(p, s);
          }
          break;
        case PK_COUNT: {
          if (P.seq) {
            if (nn(p) == 0) push_new(p, s);
          } else {
            push_new(p, s);
          }
          if (pr.minC == 0 && sev(s, pr.stateId) == NIL) {
            const DPost& ps = P.post[pr.thisPost];
            if (ps.hasSelector) {
              fl(p) |= FL_CHANGED;
              evret |= 1u << pr.thisPost;
            }
            if (ps.nextEvery >= 0) wk_push((1u << 31) | ((uint32_t)ps.nextEvery << 16) | s);
            if (ps.nextPre >= 0) wk_push(((uint32_t)ps.nextPre << 16) | s);
          }
          break;
        }
        case PK_LOGICAL:
        case PK_ABSENT_LOGICAL: {   // LogicalPreStateProcessor.addState :43-63
          // AbsentLogicalPreStateProcessor.addState (:77-99): inactive -> dropped;
          // a non-start absent operand (and an absent partner) is scheduled
          if (pr.kind == PK_ABSENT_LOGICAL && (fl(p) & FL_INACTIVE)) break;
          if (pr.isStart || P.seq) {
            if (nn(p) == 0) push_new(p, s);
            if (pr.partner >= 0 && nn(pr.partner) == 0) push_new(pr.partner, s);
          } else {
            push_new(p, s);
            if (pr.partner >= 0) push_new(pr.partner, s);
          }
          if (pr.kind == PK_ABSENT_LOGICAL && !pr.isStart && pr.waiting != -1) {
            notifyAt(pr.sched, sts(s) + pr.waiting);
            const DPre& pp = P.pre[pr.partner];
            if (pp.kind == PK_ABSENT_LOGICAL) notifyAt(pp.sched, sts(s) + pp.waiting);
          }
          break;
        }
        case PK_ABSENT: {    // AbsentStreamPreStateProcessor.addState :67-88
          if (fl(p) & FL_INACTIVE) break;
          if (P.seq) {
            nn(p) = 0;
            push_new(p, s);
          } else {
            push_new(p, s);
          }
          if (!pr.isStart) {
            lst(p) = sts(s) + pr.waiting;
            notifyAt(pr.sched, lst(p));
          }
          break;
        }
      }
    }
  }

  __device__ void addEveryState(int p, uint16_t s) {   // :230-247
    const DPre& pr = P.pre[p];
    uint16_t c = clone_se(s);
    stype(c) = SHD_EV_CURRENT;
    if (pr.kind == PK_ABSENT_LOGICAL) {
      // AbsentLogicalPreStateProcessor.addEveryState (:101-119): the clone takes the
      // time of the event this processor saw; only the pair's slots clear
      if (sev(c, pr.stateId) != NIL) sts(c) = ev_ts(sev(c, pr.stateId));
      sev(c, pr.stateId) = NIL;
      sev(c, P.pre[pr.partner].stateId) = NIL;
      push_new(p, c);
      push_new(pr.partner, c);
      return;
    }
    for (int i = pr.stateId; i < Y.nstates; i++) sev(c, i) = NIL;
    if (pr.kind == PK_LOGICAL) {
      push_new(p, c);
      if (pr.partner >= 0) {
        sev(c, P.pre[pr.partner].stateId) = NIL;
        push_new(pr.partner, c);
      }
      return;
    }
    push_new(p, c);
    if (pr.kind == PK_ABSENT) {
      lst(p) = sts(s) + pr.waiting;
      notifyAt(pr.sched, lst(p));
    }
  }

  __device__ bool seq_hold(int p) {
    // sequence without every: the start state is not re-armed while the next state waits
    const DPost& ps = P.post[P.pre[p].thisPost];
    return P.seq && ps.nextEvery < 0 && ps.nextPre >= 0 && pn(ps.nextPre) != 0;
  }

  __device__ void resetState(int p) {   // :288-305 and the Logical / Absent overrides
    const DPre& pr = P.pre[p];
    switch (pr.kind) {
      case PK_STREAM:
      case PK_COUNT:
        pn(p) = 0;
        if (pr.isStart && nn(p) == 0) {
          if (seq_hold(p)) return;
          init_pre(p);
        }
        break;
      case PK_LOGICAL:
      case PK_ABSENT_LOGICAL:
        if (pr.ltype == 1 || pn(p) == pn(pr.partner)) {
          pn(p) = 0;
          pn(pr.partner) = 0;
          if (pr.isStart && nn(p) == 0) {
            if (seq_hold(p)) return;
            init_pre(p);
          }
        }
        break;
      case PK_ABSENT:
        pn(p) = 0;
        if (pr.isStart) {
          if (seq_hold(p)) return;
          init_pre(p);
        }
        break;
    }
  }

  __device__ bool ts_less(uint16_t a, uint16_t b) {   // eventTimeComparator, -1 last
    int64_t ta = sts(a), tb = sts(b);
    if (ta == -1) return false;
    if (tb == -1) return true;
    return ta < tb;
  }

  __device__ void merge_new(int p) {
    int n = nn(p);
    for (int i = 1; i < n; i++) {   // stable insertion sort (List.sort)
      uint16_t x = nw(p, i);
      int j = i - 1;
      while (j >= 0 && ts_less(x, nw(p, j))) {
        nw(p, j + 1) = nw(p, j);
        j--;
      }
      nw(p, j + 1) = x;
    }
    int m = pn(p);
    for (int i = 0; i < n; i++) {
      if (m >= Y.L) {
        ovf |= OV_LIST;
        break;
      }
      pend(p, m++) = nw(p, i);
    }
    pn(p) = (uint16_t)m;
    nn(p) = 0;
  }

  __device__ void updateState(int p) {   // :308-323
    const DPre& pr = P.pre[p];
    if (pr.kind == PK_COUNT && (fl(p) & FL_SSRESET)) {
      fl(p) &= (uint8_t)~FL_SSRESET;
      init_pre(p);
    }
    merge_new(p);
    if (pr.kind == PK_LOGICAL || pr.kind == PK_ABSENT_LOGICAL) merge_new(pr.partner);
  }

  __device__ void expireEvents(int p, int64_t t) {   // :326-361
    const DPre& pr = P.pre[p];
    uint16_t expired = NIL;
    int n = pn(p), k = 0;
    while (k < n) {
      uint16_t s = pend(p, k);
      if (!isExpired(s, t)) break;
      if (stype(s) != SHD_EV_EXPIRED) {
        stype(s) = SHD_EV_EXPIRED;
        expired = s;
      }
      k++;
    }
    if (k > 0) {
      for (int i = k; i < n; i++) pend(p, i - k) = pend(p, i);
      pn(p) = (uint16_t)(n - k);
    }
    int m = nn(p), w = 0;
    for (int i = 0; i < m; i++) {
      uint16_t s = nw(p, i);
      if (isExpired(s, t)) {
        if (stype(s) != SHD_EV_EXPIRED) {
          stype(s) = SHD_EV_EXPIRED;
          expired = s;
        }
      } else {
        nw(p, w++) = s;
      }
    }
    nn(p) = (uint16_t)w;
    if (expired != NIL && pr.withinEvery >= 0) {
      addEveryState(pr.withinEvery, expired);
      updateState(pr.withinEvery);
    }
  }

  __device__ void countStartStateReset(int p) {   // CountPreStateProcessor.startStateReset
    for (int guard = 0; p >= 0 && guard < kNP; guard++) {
      fl(p) |= FL_SSRESET;
      p = P.post[P.pre[p].thisPost].callbackPre;
    }
  }

  // ---------------------------------------------------------------- post processors
  __device__ void streamPost(int post, uint16_t s) {   // StreamPostStateProcessor.process :64-83
    const DPost& ps = P.post[post];
    fl(ps.pre) |= FL_CHANGED;
    uint16_t e = sev(s, ps.stateId);
    sts(s) = ev_ts(e);
    if (ps.hasSelector) evret |= 1u << post;
    if (ps.nextPre >= 0) addState(ps.nextPre, s);
    if (ps.nextEvery >= 0) addEveryState(ps.nextEvery, s);
    if (ps.callbackPre >= 0) countStartStateReset(ps.callbackPre);
  }

  __device__ void countMinReached(int post, uint16_t s) {   // CountPostStateProcessor.processMinCountReached
    const DPost& ps = P.post[post];
    if (ps.hasSelector) {
      fl(ps.pre) |= FL_CHANGED;
      evret |= 1u << post;
    }
    if (ps.nextPre >= 0) addState(ps.nextPre, s);
    if (ps.nextEvery >= 0) addEveryState(ps.nextEvery, s);
  }

  __device__ void countPost(int post, uint16_t s) {   // CountPostStateProcessor.process :39-67
    const DPost& ps = P.post[post];
    uint16_t e = sev(s, ps.stateId);
    int n = 1;
    while (enext(e) != NIL) {
      n++;
      e = enext(e);
    }
    fl(ps.pre) |= FL_SUCCESS;
    sts(s) = ev_ts(e);
    if (n >= ps.minC) {
      if (P.seq) {
        if (ps.nextPre >= 0) addState(ps.nextPre, s);
        if (n != ps.maxC) addState(ps.pre, s);
      } else if (n == ps.minC) {
        countMinReached(post, s);
      }
      if (n == ps.maxC) fl(ps.pre) |= FL_CHANGED;
    }
  }

  __device__ void logicalPost(int post, uint16_t s) {   // LogicalPostStateProcessor.process :59-86
    const DPost& ps = P.post[post];
    if (ps.ltype == 0) {
      const bool proceed = P.pre[ps.partnerPre].kind == PK_ABSENT_LOGICAL
                               ? partnerCanProceed(ps.partnerPre, s)
                               : sev(s, P.pre[ps.partnerPre].stateId) != NIL;
      if (proceed) streamPost(post, s);
      else fl(ps.pre) |= FL_CHANGED;
    } else {
      streamPost(post, s);
      const DPost& pp = P.post[ps.partnerPost];
      if (pp.hasSelector && P.pre[ps.pre].thisLast == ps.partnerPost) evret |= 1u << ps.partnerPost;
    }
  }

  __device__ void absentPost(int post, uint16_t s) {   // AbsentStreamPostStateProcessor.process
    const DPost& ps = P.post[post];
    const DPre& pr = P.pre[ps.pre];
    fl(ps.pre) |= FL_CHANGED;
    uint16_t e = sev(s, ps.stateId);
    sts(s) = ev_ts(e);
    evret |= 1u << post;
    if (pr.isStart && ps.nextEvery >= 0 && ps.nextEvery == ps.pre) addEveryState(ps.nextEvery, s);
    lst(ps.pre) = ev_ts(e) + pr.waiting;
    notifyAt(pr.sched, lst(ps.pre));
  }

  // AbsentLogicalPostStateProcessor.process: state changed, event returned,
  // updateLastArrivalTime (lst = LogicalStreamPreState.lastArrivalTime) -- no partner check
  __device__ void absentLogicalPost(int post, uint16_t s) {
    const DPost& ps = P.post[post];
    fl(ps.pre) |= FL_CHANGED;
    evret |= 1u << post;
    lst(ps.pre) = ev_ts(sev(s, ps.stateId));
  }

  // AbsentLogicalPreStateProcessor.partnerCanProceed (:353-388), p = the absent operand
  __device__ bool partnerCanProceed(int p, uint16_t s) {
    const DPre& pr = P.pre[p];
    const DPost& tp = P.post[pr.thisPost];
    if (P.seq && tp.nextEvery < 0 && lst(p) > 0) return false;
    if (pr.waiting == -1) {
      if (tp.nextEvery < 0) return sev(s, pr.stateId) == NIL;
      if (lst(p) > 0) {
        lst(p) = 0;
        init_pre(p);
        return false;
      }
      return true;
    }
    return sev(s, pr.stateId) != NIL;
  }

  __device__ void postProcess(int post, uint16_t s) {
    switch (P.post[post].kind) {
      case PK_STREAM: streamPost(post, s); break;
      case PK_COUNT: countPost(post, s); break;
      case PK_LOGICAL: logicalPost(post, s); break;
      case PK_ABSENT: absentPost(post, s); break;
      case PK_ABSENT_LOGICAL: absentLogicalPost(post, s); break;
    }
  }

  // StreamPreStateProcessor.process(stateEvent): filter chain, then the post processor.
  // Returns false when a filter rejected the state event (no post processing ran).
  __device__ bool processChain(int p, uint16_t s) {
    const DPre& pr = P.pre[p];
    fl(p) &= (uint8_t)~FL_CHANGED;
    SECtx cx{this, s};
    if (pr.filters.n == 1 && pr.filters.fp.ok) {
      // one filter pre-decoded on the host (compile_fast_pred): straight-line
      // comparisons, no bytecode fetched and dispatched per state event
      scans++;
      if (!eval_fpred(pr.filters.fp, cx)) return false;
    } else {
      for (int i = 0; i < pr.filters.n; i++) {
        scans++;
        if (!eval_bool(es.ins + pr.filters.f[i].off, pr.filters.f[i].len, es.consts, cx)) return false;
      }
    }
    postProcess(pr.thisPost, s);
    return true;
  }

  __device__ bool take_ret(int thisLast) {
    uint32_t b = 1u << thisLast;
    if (evret & b) {
      evret &= ~b;
      return true;
    }
    return false;
  }

  // ---------------------------------------------------------------- processAndReturn
  __device__ void streamPAR(int p, uint16_t rec, bool removeOnNoChangeSeq, bool collect) {   // :364-403
    const DPre& pr = P.pre[p];
    int n = pn(p), w = 0;
    for (int r = 0; r < n; r++) {
      uint16_t s = pend(p, r);
      uint16_t c = new_ev(rec);
      sev(s, pr.stateId) = c;
      bool passed = processChain(p, s);
      if (take_ret(pr.thisLast) && collect) push_tmp(s);
      if (fl(p) & FL_CHANGED) continue;   // removed
      if (!passed && sev(s, pr.stateId) == c) free_ev(c);
      sev(s, pr.stateId) = NIL;
      if (P.seq) {
        const DPost& tp = P.post[pr.thisPost];
        if (tp.callbackPre >= 0) countStartStateReset(tp.callbackPre);
        if (removeOnNoChangeSeq) continue;
      }
      pend(p, w++) = s;
    }
    pn(p) = (uint16_t)w;
  }

  __device__ void removeLastEvent(uint16_t s, int sid, bool release) {   // StateEvent.removeLastEvent :224-236
    uint16_t x = sev(s, sid);
    if (x == NIL) return;
    while (enext(x) != NIL) {
      uint16_t nx = enext(x);
      if (enext(nx) == NIL) {
        enext(x) = NIL;
        if (release) free_ev(nx);
        return;
      }
      x = nx;
    }
    sev(s, sid) = NIL;
    if (release) free_ev(x);
  }

  __device__ void countPAR(int p, uint16_t rec) {   // CountPreStateProcessor.processAndReturn :52-94
    const DPre& pr = P.pre[p];
    int n = pn(p), w = 0;
    for (int r = 0; r < n; r++) {
      uint16_t s = pend(p, r);
      if ((pr.stateId + 1 < Y.nstates && sev(s, pr.stateId + 1) != NIL) ||
          (pr.stateId + 2 < Y.nstates && sev(s, pr.stateId + 2) != NIL))
        continue;   // the next state already took this partial
      uint16_t c = new_ev(rec);
      if (ovf) return;   // pool exhausted: never link the sink element into a chain
      uint16_t h = sev(s, pr.stateId);
      if (h == NIL) {
        sev(s, pr.stateId) = c;
      } else {
        while (enext(h) != NIL) h = enext(h);
        enext(h) = c;
      }
      fl(p) &= (uint8_t)~FL_SUCCESS;
      bool passed = processChain(p, s);
      if (take_ret(pr.thisLast)) push_tmp(s);
      bool erased = (fl(p) & FL_CHANGED) != 0;
      if (!(fl(p) & FL_SUCCESS)) {
        removeLastEvent(s, pr.stateId, !passed);
        if (P.seq) erased = true;
      }
      if (!erased) pend(p, w++) = s;
    }
    pn(p) = (uint16_t)w;
  }

  __device__ void logicalPAR(int p, uint16_t rec) {   // LogicalPreStateProcessor.processAndReturn :113-154
    const DPre& pr = P.pre[p];
    int n = pn(p), w = 0;
    for (int r = 0; r < n; r++) {
      uint16_t s = pend(p, r);
      if (pr.ltype == 1 && sev(s, P.pre[pr.partner].stateId) != NIL) continue;
      uint16_t c = new_ev(rec);
      sev(s, pr.stateId) = c;
      bool passed = processChain(p, s);
      if (take_ret(pr.thisLast)) push_tmp(s);
      if (fl(p) & FL_CHANGED) continue;
      if (!passed && sev(s, pr.stateId) == c) free_ev(c);
      sev(s, pr.stateId) = NIL;
      if (P.seq) continue;
      pend(p, w++) = s;
    }
    pn(p) = (uint16_t)w;
  }

  // AbsentLogicalPreStateProcessor.processAndReturn (:243-296): an X arrival
  // takes the partials it passes out of this processor's pending list; never
  // returns events itself
  __device__ void absentLogicalPAR(int p, uint16_t rec) {
    const DPre& pr = P.pre[p];
    if (fl(p) & FL_INACTIVE) return;
    const DPost& tp = P.post[pr.thisPost];
    const int psid = P.pre[pr.partner].stateId;
    const bool restore = pr.waiting != -1 || (P.seq && pr.ltype == 0 && tp.nextEvery >= 0);
    int n = pn(p), w = 0;
    for (int r = 0; r < n; r++) {
      uint16_t s = pend(p, r);
      if (pr.ltype == 1 && sev(s, psid) != NIL) continue;
      const uint16_t cur = sev(s, pr.stateId);
      const uint16_t c = new_ev(rec);
      sev(s, pr.stateId) = c;
      processChain(p, s);
      if (restore) sev(s, pr.stateId) = cur;
      bool erased = false;
      if (take_ret(pr.thisLast)) {
        erased = true;
        if (P.seq) {   // also out of the partner's pending list
          const int q = pr.partner;
          int m = pn(q), k = 0;
          for (int i = 0; i < m; i++)
            if (pend(q, i) != s) pend(q, k++) = pend(q, i);
          pn(q) = (uint16_t)k;
        }
      }
      if (!(fl(p) & FL_CHANGED)) {
        sev(s, pr.stateId) = cur;
        if (P.seq) erased = true;
      }
      if (sev(s, pr.stateId) != c) free_ev(c);
      if (!erased) pend(p, w++) = s;
    }
    pn(p) = (uint16_t)w;
  }

  __device__ void processAndReturn(int p, uint16_t rec) {
    if (ovf) return;   // capacity exceeded: the push fails with SHD_E_CAPACITY
    switch (P.pre[p].kind) {
      case PK_ABSENT_LOGICAL: absentLogicalPAR(p, rec); break;
      case PK_STREAM: streamPAR(p, rec, true, true); break;
      case PK_COUNT: countPAR(p, rec); break;
      case PK_LOGICAL: logicalPAR(p, rec); break;
      case PK_ABSENT:   // AbsentStreamPreStateProcessor.processAndReturn :257-274: nothing is returned
        if (!(fl(p) & FL_INACTIVE)) streamPAR(p, rec, false, false);
        break;
    }
  }

  // ---------------------------------------------------------------- absent timers
  __device__ void absentSendEvent(int p, uint16_t s) {   // AbsentStreamPreStateProcessor.sendEvent
    const DPre& pr = P.pre[p];
    const DPost& tp = P.post[pr.thisPost];
    cur_state = pr.stateId;
    if (tp.hasSelector && accepts(s)) emit(s, new_tag());
    if (tp.nextPre >= 0) addState(tp.nextPre, s);
    if (tp.nextEvery >= 0) addEveryState(tp.nextEvery, s);
    else if (pr.isStart) fl(p) |= FL_INACTIVE;
    if (tp.callbackPre >= 0) countStartStateReset(tp.callbackPre);
  }

  // AbsentStreamPreStateProcessor.process(ComplexEventChunk) on a TIMER (:150-227)
  __device__ void absentTimer(int p, int64_t currentTime, int64_t nowt) {
    const DPre& pr = P.pre[p];
    if (fl(p) & FL_INACTIVE) return;
    const DPost& tp = P.post[pr.thisPost];
    bool initialize = pr.isStart && nn(p) == 0 && pn(p) == 0;
    if (initialize && P.seq && tp.nextEvery < 0 && lst(p) > 0) initialize = false;
    if (initialize) {
      uint16_t s = new_se();
      addState(p, s);
    } else if (P.seq && nn(p) != 0) {
      resetState(p);
    }
    updateState(p);
    misc(MISC_TMPN) = 0;
    int n = pn(p), w = 0;
    for (int r = 0; r < n; r++) {
      uint16_t s = pend(p, r);
      if (isExpired(s, currentTime)) {
        if (pr.withinEvery >= 0 && tp.nextEvery != p && tp.nextEvery >= 0) addEveryState(tp.nextEvery, s);
        continue;
      }
      if ((sts(s) == -1 && currentTime >= lst(p)) || (sts(s) != -1 && currentTime >= sts(s) + pr.waiting)) {
        sts(s) = currentTime;
        push_tmp(s);
        continue;
      }
      pend(p, w++) = s;
    }
    pn(p) = (uint16_t)w;
    if (pr.withinEvery >= 0) updateState(pr.withinEvery);
    int nret = misc(MISC_TMPN);
    bool notProcessed = nret == 0;
    for (int i = 0; i < nret; i++) absentSendEvent(p, tmpl(i));
    misc(MISC_TMPN) = 0;
    if (nowt > pr.waiting + currentTime) lst(p) = nowt + pr.waiting;
    if (notProcessed && lst(p) < currentTime) {
      lst(p) = currentTime + pr.waiting;
      notifyAt(pr.sched, lst(p));
    }
  }

  // a fresh StreamEvent (streamEventFactory.newInstance(): ts -1, no data)
  __device__ uint16_t empty_ev() {
    const int r = alloc_bit(Y.o_rec_free, Y.recw, Y.RC, OV_REC, MISC_FREE_REC, MISC_HINT_REC);
    rts(r) = -1;
    for (int c = 0; c < Y.ncols; c++) rval(r, c) = 0;
    rnul(r) = 0xFFFFFFFFu;
    return new_ev((uint16_t)r);
  }
  __device__ void add_event(uint16_t s, int sid, uint16_t e) {   // StateEvent.addEvent
    if (ovf) return;
    uint16_t h = sev(s, sid);
    if (h == NIL) {
      sev(s, sid) = e;
      return;
    }
    while (enext(h) != NIL) h = enext(h);
    enext(h) = e;
  }

  __device__ void absentLogicalSendEvent(int p, uint16_t s) {   // AbsentLogicalPreStateProcessor.sendEvent
    const DPre& pr = P.pre[p];
    const DPost& tp = P.post[pr.thisPost];
    cur_state = pr.stateId;
    if (tp.hasSelector && accepts(s)) emit(s, new_tag());
    if (tp.nextPre >= 0) addState(tp.nextPre, s);
    if (tp.nextEvery >= 0) {
      addEveryState(tp.nextEvery, s);
    } else if (pr.isStart) {
      fl(p) |= FL_INACTIVE;
      if (pr.ltype == 1 && P.pre[pr.partner].kind == PK_ABSENT_LOGICAL) fl(pr.partner) |= FL_INACTIVE;
    }
    if (tp.callbackPre >= 0) countStartStateReset(tp.callbackPre);
  }

  // AbsentLogicalPreStateProcessor.process(ComplexEventChunk) on a TIMER (:122-218)
  __device__ void absentLogicalTimer(int p, int64_t currentTime, int64_t nowt) {
    const DPre& pr = P.pre[p];
    if (fl(p) & FL_INACTIVE) return;
    const DPost& tp = P.post[pr.thisPost];
    const int psid = P.pre[pr.partner].stateId;
    bool notProcessed = true;
    if (currentTime >= lst(p) + pr.waiting) {
      if (pr.isStart && P.seq && nn(p) == 0 && pn(p) == 0) addState(p, new_se());
      else if (P.seq && nn(p) != 0) resetState(p);
      updateState(p);
      uint16_t expired = NIL;
      misc(MISC_TMPN) = 0;
      int n = pn(p), w = 0;
      for (int r = 0; r < n; r++) {
        uint16_t s = pend(p, r);
        if (isExpired(s, currentTime)) {
          expired = s;
          continue;
        }
        const uint16_t own = sev(s, pr.stateId);
        const bool passed = own == NIL ? currentTime >= sts(s) + pr.waiting : currentTime >= ev_ts(own) + pr.waiting;
        if (passed) {
          if (pr.ltype == 1 && sev(s, psid) == NIL) {          // OR: partner not received
            add_event(s, pr.stateId, empty_ev());
            push_tmp(s);
          } else if (pr.ltype == 0 && sev(s, psid) != NIL) {   // AND: partner received, not sent
            push_tmp(s);
          } else if (pr.ltype == 0) {                          // AND: let the partner proceed
            add_event(s, pr.stateId, empty_ev());
          }
          continue;
        }
        pend(p, w++) = s;
      }
      pn(p) = (uint16_t)w;
      if (expired != NIL && pr.withinEvery >= 0) {
        addEveryState(pr.withinEvery, expired);
        updateState(pr.withinEvery);
      }
      const int nret = misc(MISC_TMPN);
      notProcessed = nret == 0;
      for (int i = 0; i < nret; i++) {
        const uint16_t s = tmpl(i);
        sts(s) = currentTime;
        absentLogicalSendEvent(p, s);
      }
      misc(MISC_TMPN) = 0;
      lst(p) = 0;
    }
    if (tp.nextEvery >= 0 || (notProcessed && pr.isStart))
      notifyAt(pr.sched, (lst(p) == 0 ? nowt : lst(p)) + pr.waiting);
  }

  // ---------------------------------------------------------------- selector / output
  __device__ bool accepts(uint16_t s) {   // QuerySelector.processNoGroupBy event-type filter
    uint8_t t = stype(s);
    if (t == SHD_EV_CURRENT) return P.current_on;
    if (t == SHD_EV_EXPIRED) return P.expired_on;
    return false;
  }
  // one list per multi-value output: the attribute of every event of state
  // st's chain, in chain order, into the list arena; returns the handle
  // (offset | count << 40, offsets relative to this push's arena)
  __device__ uint64_t emit_list(uint16_t s, int4 in) {
    const uint16_t head = sev(s, in.y);
    const int attr = in.w & 0xFFFF;
    int len = 0;
    for (uint16_t x = head; x != NIL; x = enext(x)) len++;
    if (len == 0) return 0;
    const unsigned long long base = atomicAdd(&A.ctl->lrows, (unsigned long long)len);
    if ((int64_t)(base + len) > A.LR) {
      ovf |= OV_MULTI;
      return 0;
    }
    int i = 0;
    for (uint16_t x = head; x != NIL; x = enext(x), i++) {
      const uint16_t r = erec(x);
      const bool z = (rnul(r) >> attr) & 1u;
      A.st_lv[base + i] = z ? 0 : rval(r, attr);
      A.st_ln[base + i] = z ? 1 : 0;
    }
    return (uint64_t)base | ((uint64_t)len << 40);
  }
  __device__ uint64_t new_tag() { return ((uint64_t)slot << 24) | (uint64_t)(tagc++ & 0xFFFFFF); }
  __device__ void emit(uint16_t s, uint64_t tag) {
    if (quiet) return;   // warm-up event of a window lane
    NFA_PROF_T0(t4);
    unsigned long long idx = atomicAdd(&A.ctl->rows, 1ull);
    if ((int64_t)idx >= A.R) {
      ovf |= OV_ROWS;
      return;
    }
    SECtx cx{this, s};
    for (int c = 0; c < P.nout; c++) {
      if ((P.multi_mask >> c) & 1u) {   // MultiValueVariableFunctionExecutor.execute: the chain from its head
        A.st_vals[idx * P.nout + c] = emit_list(s, es.ins[P.outs[c].off]);
        A.st_nul[idx * P.nout + c] = 0;
        continue;
      }
      Val v = eval_expr(es.ins + P.outs[c].off, P.outs[c].len, es.consts, cx);
      A.st_vals[idx * P.nout + c] = v.b;
      A.st_nul[idx * P.nout + c] = (uint8_t)v.null;
    }
    A.st_ts[idx] = sts(s);
    A.st_type[idx] = stype(s);
    A.st_tag[idx] = tag;
    A.st_p[idx] = t_prim;
    A.st_s[idx] = t_sec;
    A.st_t[idx] = t_ter;
    A.st_sidx[idx] = cur_state;
    NFA_PROF_ADD(4, t4);
  }

  // ---------------------------------------------------------------- key lifecycle
  __device__ void seed(int64_t now_seed) {   // StateStreamRuntime.initPartition
    for (int p = 0; p < P.npre; p++) {
      pn(p) = 0;
      nn(p) = 0;
      fl(p) = 0;
      lst(p) = 0;
    }
    for (int sc = 0; sc < P.nsched; sc++) sqn(sc) = 0;
    fill_free(Y.o_se_free, Y.sew, Y.SC);
    fill_free(Y.o_ev_free, Y.evw, Y.EC);
    fill_free(Y.o_rec_free, Y.recw, Y.RC);
    for (int i = 0; i < MISC_N; i++)
      if (i != MISC_HSTAMP) misc(i) = 0;   // the hash stamp outlives reseeding (stale canonical ids)
    misc(MISC_FREE_SE) = (uint32_t)Y.SC;
    misc(MISC_FREE_EV) = (uint32_t)Y.EC;
    misc(MISC_FREE_REC) = (uint32_t)Y.RC;
    evret = 0;
    for (int i = 0; i < P.ninit; i++) init_pre(P.initSeq[i]);
    for (int p = 0; p < P.npre; p++) {   // partitionCreated for absent processors
      const DPre& pr = P.pre[p];
      if ((pr.kind != PK_ABSENT && pr.kind != PK_ABSENT_LOGICAL) || (fl(p) & FL_STARTED)) continue;
      fl(p) |= FL_STARTED;
      if (pr.isStart && pr.waiting != -1 && !(fl(p) & FL_INACTIVE)) {
        if (pr.kind == PK_ABSENT) {
          lst(p) = now_seed + pr.waiting;
          notifyAt(pr.sched, lst(p));
        } else {   // AbsentLogicalPreStateProcessor.partitionCreated (:318-335)
          notifyAt(pr.sched, now_seed + pr.waiting);
        }
      }
    }
    misc(MISC_SEEDED) = 1;
  }

  __device__ void stabilize(int si, int64_t t) {   // PatternMulti/SequenceMulti receivers' stabilizeStates
    for (int i = 0; i < P.nall; i++) expireEvents(P.allPre[i], t);
    if (!P.seq) {
      int np = P.nsp[si];
      if (np > 1) {
        for (int k = 0; k < np; k++) updateState(P.streamPres[si][k]);
      } else if (np == 1) {
        updateState(P.streamPres[si][0]);
      }
    } else {   // StateStreamRuntime.resetAndUpdate
      for (int i = 0; i < P.nreset; i++) resetState(P.resetSeq[i]);
      for (int i = 0; i < P.nupd; i++) updateState(P.updSeq[i]);
    }
  }

  __device__ uint16_t make_rec(int64_t row, int64_t ts) {
    int r = alloc_bit(Y.o_rec_free, Y.recw, Y.RC, OV_REC, MISC_FREE_REC, MISC_HINT_REC);
    rts(r) = ts;
    uint32_t nm = 0;
    const ColSet& cs = A.batch;
    for (int c = 0; c < cs.ncols; c++) {
      Val v = col_load(cs, row, c);
      rval(r, c) = v.b;
      if (v.null) nm |= 1u << c;
    }
    rnul(r) = nm;
    return (uint16_t)r;
  }

  __device__ void process_event(int64_t row) {
    NFA_PROF_T0(t0);
    maybe_gc();
    NFA_PROF_ADD(0, t0);
    NFA_PROF_T0(t1);
    const int si = A.stream;
    const int64_t ts = A.batch.ts[row];
    const uint16_t rec = make_rec(row, ts);
    NFA_PROF_ADD(1, t1);
    NFA_PROF_T0(t2);
    stabilize(si, ts);
    NFA_PROF_ADD(2, t2);
    // hand-over replay: a stabilize-only event (Replay::skip_start 2)
    if (A.skip_start && A.skip_start[row] == 2) return;
    NFA_PROF_T0(t3);
    const int np = P.nsp[si];
    last_seq = A.seq0 + row;
    if (np > 1) {
      // MultiProcessStreamReceiver: states in reverse order, one callback chunk
      // per (event, state) that returned events
      t_prim = 2 * (uint64_t)last_seq + 1;
      t_sec = 0;
      t_ter = 0;
      for (int k = np - 1; k >= 0; k--) {
        misc(MISC_TMPN) = 0;
        if (A.skip_start && A.skip_start[row] && P.pre[P.streamPres[si][k]].isStart) continue;
        cur_state = P.pre[P.streamPres[si][k]].stateId;
        processAndReturn(P.streamPres[si][k], rec);
        uint64_t tag = ~0ull;
        int nret = misc(MISC_TMPN);
        for (int i = 0; i < nret; i++) {
          uint16_t s = tmpl(i);
          if (!accepts(s)) continue;
          if (tag == ~0ull) tag = new_tag();
          emit(s, tag);
        }
        misc(MISC_TMPN) = 0;
      }
    } else if (np == 1) {
      // SingleProcessStreamReceiver: returned events are selected when the run ends
      misc(MISC_TMPN) = 0;
      ret_state = P.pre[P.streamPres[si][0]].stateId;
      if (!(A.skip_start && A.skip_start[row] && P.pre[P.streamPres[si][0]].isStart))
        processAndReturn(P.streamPres[si][0], rec);
      int nret = misc(MISC_TMPN);
      for (int i = 0; i < nret; i++) push_ret(tmpl(i));
      misc(MISC_TMPN) = 0;
    }
    NFA_PROF_ADD(3, t3);
    NFA_PROF_ADD(7, t0);
  }

  __device__ void flush_run() {
    int n = misc(MISC_RETN);
    if (n == 0) return;
    cur_state = ret_state;
    t_prim = 2 * (uint64_t)last_seq + 1;
    t_sec = 0;
    t_ter = 0;
    for (int i = 0; i < n; i++) {
      uint16_t s = retl(i);
      if (accepts(s)) emit(s, new_tag());
    }
    misc(MISC_RETN) = 0;
  }

  __device__ int64_t next_due() {
    int64_t m = INT64_MAX;
    for (int sc = 0; sc < P.nsched; sc++)
      if (sqn(sc) > 0 && sq(sc, 0) < m) m = sq(sc, 0);
    return m;
  }

  // Scheduler.onTimeChange for this key at call cc (playback time now[cc])
  __device__ void on_time_change(int cc) {
    const int64_t tnow = A.call_now[cc];
    t_prim = 2 * (uint64_t)A.call_first[cc];
    t_ter = key;
    for (int sc = 0; sc < P.nsched; sc++) {
      if (sqn(sc) == 0 || sq(sc, 0) > tnow) continue;
      const uint64_t head = (uint64_t)(sq(sc, 0) + ((int64_t)1 << 57)) & (((uint64_t)1 << 58) - 1);
      t_sec = ((uint64_t)sc << 58) | head;
      while (sqn(sc) > 0 && sq(sc, 0) - tnow <= 0) {
        int64_t nt = sq(sc, 0);
        int n = sqn(sc);
        for (int i = 1; i < n; i++) sq(sc, i - 1) = sq(sc, i);
        sqn(sc) = (uint16_t)(n - 1);
        maybe_gc();
        if (P.pre[P.schedPre[sc]].kind == PK_ABSENT_LOGICAL) absentLogicalTimer(P.schedPre[sc], nt, tnow);
        else absentTimer(P.schedPre[sc], nt, tnow);
        if (ovf) return;
      }
    }
  }

  // apply the time changes of calls (cdone, c]
  __device__ void fire_upto(int c) {
    if (P.nsched == 0) {
      if (c > cdone) cdone = c;
      return;
    }
    while (cdone < c && !ovf) {
      int64_t nd = next_due();
      if (nd == INT64_MAX || nd > A.call_now[c]) {
        cdone = c;
        return;
      }
      int lo = cdone + 1, hi = c;   // first call in [lo, c] with now >= nd
      while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (A.call_now[mid] >= nd) hi = mid;
        else lo = mid + 1;
      }
      if (A.call_changed[lo]) on_time_change(lo);
      cdone = lo;
    }
  }
};

__device__ Val SECtx::load(int st, int idx, int attr) const {
  Val v;
  v.b = 0;
  v.null = 1;
  uint16_t e = L->chain_get(L->sev(se, st), idx);
  if (e == NIL) return v;
  uint16_t r = L->erec(e);
  if ((L->rnul(r) >> attr) & 1u) return v;
  v.b = L->rval(r, attr);
  v.null = 0;
  return v;
}
__device__ bool SECtx::evnull(int st, int idx) const { return L->chain_get(L->sev(se, st), idx) == NIL; }
__device__ int64_t SECtx::ts(int, int) const { return L->sts(se); }

// One lane = one partition key (or the single unpartitioned key).
__global__ __launch_bounds__(kLaneBlock) void k_nfa_run(const NfaProg* __restrict__ gprog,
                                                        const NfaLayout* __restrict__ glay,
                                                        const NfaRunArgs* __restrict__ ap) {
  __shared__ NfaProg sprog;
  __shared__ NfaLayout slay;
  {
    const int* src = reinterpret_cast<const int*>(gprog);
    int* dst = reinterpret_cast<int*>(&sprog);
    for (int i = threadIdx.x; i < (int)(sizeof(NfaProg) / 4); i += kLaneBlock) dst[i] = src[i];
    const int* s2 = reinterpret_cast<const int*>(glay);
    int* d2 = reinterpret_cast<int*>(&slay);
    for (int i = threadIdx.x; i < (int)(sizeof(NfaLayout) / 4); i += kLaneBlock) d2[i] = s2[i];
  }
  const NfaRunArgs& a = *ap;
  __syncthreads();   // the program / layout copies above are complete
  const DExprSet es = a.es;
  const int64_t lane_id = (int64_t)blockIdx.x * kLaneBlock + threadIdx.x;
  if (lane_id >= a.nlanes) return;
  int64_t seg, slot;
  if (a.lanes_over_slots) {
    slot = lane_id;
    seg = a.slot_seg ? (int64_t)a.slot_seg[slot] : -1;
  } else {
    seg = lane_id;
    // window lane c works in slot c + 1 (slot 0 holds the carried state, read
    // by lane 0); the unpartitioned one-lane plan runs in slot 0
    slot = a.seg_slot ? (int64_t)a.seg_slot[seg] : (a.chunk_len > 0 ? lane_id + 1 : 0);
  }
  Lane L(sprog, slay, a, es);
  L.slot = slot;
  L.ks.b = a.state + (slot / slay.W) * slay.blk;
  L.ks.l = (int)(slot % slay.W);
  L.ks.w = slay.W;
  L.ovf = 0;
  L.partials = 0;
  L.scans = 0;
  L.tagc = 0;
  L.t_prim = L.t_sec = L.t_ter = 0;
  L.cdone = -1;
  L.last_seq = a.seq0;
  L.quiet = false;
  if (a.chunk_len > 0) {
    // Window lane.  Lanes c < c_exact start at row 0 from a copy of the carried
    // state (slot 0, copied by k_lane_copy) and replay the one-lane run
    // exactly; lane c >= c_exact starts fresh `warm` events before its chunk
    // (output suppressed) and is valid when its state before its first owned
    // event equals lane c-1's state after its last (hash_w[c] == hash_e[c-1],
    // k_win_check; on a mismatch the host reruns the push with longer warm-ups).
    // Calls' timers fire and single-receiver runs flush before the row that
    // follows them, so they belong to the lane that owns that row.
    const int64_t ob = lane_id * a.chunk_len;
    const int64_t oe = ob + a.chunk_len < a.n_keyed ? ob + a.chunk_len : a.n_keyed;
    const bool exact = lane_id < a.c_exact;
    L.key = 0;
    int64_t wb;
    uint32_t cur_run;
    if (exact) {
      if (L.misc(MISC_SEEDED) == 0) L.seed(a.start_time);
      L.evret = L.misc(MISC_EVRET);
      wb = 0;
      cur_run = 0xFFFFFFFFu;
    } else {
      L.evret = 0;
      L.seed(a.start_time);
      wb = ob - a.warm;
      const int c0 = a.call_of[wb];
      L.cdone = (wb > 0 && a.call_of[wb - 1] == c0) ? c0 : c0 - 1;
      cur_run = a.run_id[wb];
    }
    for (int64_t row = wb; row < oe && !L.ovf; row++) {
      if (row == ob) {
        L.quiet = false;
        NFA_PROF_T0(th);
        if (!exact) {
          uint64_t h2;
          const uint64_t h1 = L.state_hash(h2);
          a.hash_w[2 * lane_id] = a.hash1_zero ? 0ull : h1;
          a.hash_w[2 * lane_id + 1] = h2;
        }
        NFA_PROF_ADDL(L, 5, th);
      } else if (row == wb) {
        L.quiet = true;
      }
      NFA_PROF_T0(tf);
      const uint32_t run = a.run_id[row];
      if (run != cur_run) {
        L.flush_run();
        cur_run = run;
      }
      L.fire_upto(a.call_of[row]);
      NFA_PROF_ADDL(L, 6, tf);
      L.process_event(row);
    }
    L.quiet = false;
    if (oe == a.n_keyed) {   // the push's last lane closes it like the one-lane run
      if (!L.ovf) L.flush_run();
      if (!L.ovf) L.fire_upto(a.ncalls - 1);
    }
    L.misc(MISC_EVRET) = L.evret;
    {
      uint64_t h2;
      const uint64_t h1 = L.state_hash(h2);
      a.hash_e[2 * lane_id] = a.hash1_zero ? 0ull : h1;
      a.hash_e[2 * lane_id + 1] = h2;
    }
#ifdef SHD_NFA_PROF
    for (int k = 0; k < kProfN; k++) atomicAdd(&a.ctl->prof[k], (unsigned long long)L.prof[k]);
#endif
    if (L.ovf) atomicOr(&a.ctl->overflow, L.ovf);
    if (L.partials) atomicAdd(&a.ctl->partials, L.partials);
    if (L.scans) atomicAdd(&a.ctl->scans, L.scans);
    return;
  }
  bool seeded = L.misc(MISC_SEEDED) != 0;
  L.key = L.ks.at<uint64_t>(slay.o_key, 0);   // written by k_store_keys (0 when unpartitioned)
  L.evret = seeded ? L.misc(MISC_EVRET) : 0;
  int64_t b = 0, e = 0;
  if (!a.partitioned) {
    e = a.n_keyed;
  } else if (seg >= 0) {
    b = a.seg_start[seg];
    e = seg + 1 < a.nseg ? (int64_t)a.seg_start[seg + 1] : a.n_keyed;
  }
  if (!seeded && !a.partitioned) {   // unpartitioned queries start with the app
    L.seed(a.start_time);
    seeded = true;
  }
  uint32_t cur_run = 0xFFFFFFFFu;
  for (int64_t i = b; i < e && !L.ovf; i++) {
    const int64_t row = a.rows ? (int64_t)a.rows[i] : i;
    const int c = a.call_of[row];
    const uint32_t run = a.run_id[row];
    if (run != cur_run) {
      L.flush_run();
      cur_run = run;
    }
    L.fire_upto(c);
    if (!seeded) {   // first sight of the key: PartitionStreamReceiver.send -> initPartition
      L.seed(a.call_now[c]);
      seeded = true;
    }
    L.process_event(row);
  }
  if (!L.ovf) L.flush_run();
  if (!L.ovf && seeded) L.fire_upto(a.ncalls - 1);
  unsigned long long live = 0;
  if (seeded) {
    L.misc(MISC_EVRET) = L.evret;
    for (int p = 0; p < sprog.npre; p++) live += L.pn(p) + L.nn(p);
  }
  if (L.ovf) atomicOr(&a.ctl->overflow, L.ovf);
  if (L.partials) atomicAdd(&a.ctl->partials, L.partials);
  if (L.scans) atomicAdd(&a.ctl->scans, L.scans);
  if (live) atomicAdd(&a.ctl->live, live);
}

// window lanes: lane c >= c_exact is valid iff its warm-up state equals lane c-1's end state
__global__ void k_win_check(const uint64_t* hw, const uint64_t* he, int64_t c0, int64_t nl, unsigned int* bad) {
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + (c0 > 1 ? c0 : 1); c < nl;
       c += (int64_t)gridDim.x * blockDim.x)
    if (hw[2 * c] != he[2 * (c - 1)] || hw[2 * c + 1] != he[2 * (c - 1) + 1]) atomicAdd(bad, 1u);
}

// ---------------------------------------------------------------- growth
// One field of a layout change (grow on capacity overflow): elements (r, c) of
// the old field, r < rows, c < cols, move to the same (r, c) of the new field
// (element r * cols_old + c -> r * cols_new + c, lane-interleaved).  kind 1: a
// free bitmap (the new handles [lo, hi) start free), 2: a mark bitmap (zero),
// 3: the misc words (free-handle counters grow with their pools).
struct RelayField {
  int64_t off_old, off_new, rows, cols, cols_old, cols_new, words_old, lo, hi;
  int sz, kind;
};
struct RelayArgs {
  int nfield;
  RelayField f[NfaLayout::kMaxFields];
  int64_t blk_old, blk_new, nblocks;
  int W;
  int32_t dSE, dEV, dREC;
};

__global__ __launch_bounds__(kBlock) void k_nfa_relayout(const RelayArgs* __restrict__ ap, const char* __restrict__ src,
                                                         char* __restrict__ dst) {
  const RelayArgs& a = *ap;
  const int64_t total = a.nblocks * a.W;
  for (int64_t t = (int64_t)blockIdx.x * kBlock + threadIdx.x; t < total; t = total) {
    const int64_t b = t / a.W, k = t % a.W;
    const char* sb = src + b * a.blk_old;
    char* db = dst + b * a.blk_new;
    for (int fi = 0; fi < a.nfield; fi++) {
      const RelayField& f = a.f[fi];
      if (f.kind == 2) continue;   // mark bitmaps: zero (the destination is zeroed)
      if (f.kind == 1) {           // free bitmap: old words, then the new handles free
        for (int64_t w = 0; w < f.cols_new; w++) {
          uint64_t v = w < f.words_old ? *(const uint64_t*)(sb + f.off_old + (w * a.W + k) * 8) : 0ull;
          const int64_t w0 = w * 64;
          for (int bit = 0; bit < 64; bit++)
            if (w0 + bit >= f.lo && w0 + bit < f.hi) v |= 1ull << bit;
          *(uint64_t*)(db + f.off_new + (w * a.W + k) * 8) = v;
        }
        continue;
      }
      for (int64_t r = 0; r < f.rows; r++)
        for (int64_t c = 0; c < f.cols; c++) {
          const char* sp = sb + f.off_old + ((r * f.cols_old + c) * a.W + k) * f.sz;
          char* dp = db + f.off_new + ((r * f.cols_new + c) * a.W + k) * f.sz;
          for (int x = 0; x < f.sz; x++) dp[x] = sp[x];
        }
      if (f.kind == 3) {
        uint32_t* m = (uint32_t*)(db + f.off_new);
        m[MISC_FREE_SE * a.W + k] += (uint32_t)a.dSE;
        m[MISC_FREE_EV * a.W + k] += (uint32_t)a.dEV;
        m[MISC_FREE_REC * a.W + k] += (uint32_t)a.dREC;
      }
    }
  }
}

// one key's state (every field of slot src) into slots [dst0, dst0 + ndst):
// blockIdx.y = field, x over (element, destination); consecutive threads write
// consecutive lanes of one element
__global__ void k_lane_copy(const NfaLayout* __restrict__ glay, char* __restrict__ state, int64_t src,
                            int64_t dst0, int64_t ndst) {
  const NfaLayout& Y = *glay;
  const int f = blockIdx.y;
  const int sz = Y.f_sz[f];
  const int64_t total = Y.f_cnt[f] * ndst;
  const int W = Y.W;
  const char* sb = state + (src / W) * Y.blk + Y.f_off[f];
  const int sl = (int)(src % W);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i / ndst, d = dst0 + i % ndst;
    const char* sp = sb + (e * W + sl) * sz;
    char* dp = state + (d / W) * Y.blk + Y.f_off[f] + (e * W + d % W) * sz;
    switch (sz) {
      case 8: *reinterpret_cast<uint64_t*>(dp) = *reinterpret_cast<const uint64_t*>(sp); break;
      case 4: *reinterpret_cast<uint32_t*>(dp) = *reinterpret_cast<const uint32_t*>(sp); break;
      case 2: *reinterpret_cast<uint16_t*>(dp) = *reinterpret_cast<const uint16_t*>(sp); break;
      default: *dp = *sp;
    }
  }
}

// ---------------------------------------------------------------- batch preparation
struct BatchCtx {
  const ColSet* cs;
  int64_t row;
  __device__ Val load(int, int, int attr) const { return col_load(*cs, row, attr); }
  __device__ bool evnull(int, int) const { return false; }
  __device__ int64_t ts(int, int) const { return cs->ts[row]; }
  __device__ Val agg(int) const {
    Val v;
    v.b = 0;
    v.null = 1;
    return v;
  }
};

struct KeyArgs {
  ColSet batch;
  DExprSet es;
  DExpr key_expr;
  int key_col;
  int key_type;
};

__device__ __forceinline__ uint64_t canon_key(Val v, int type) {
  if (type == SHD_T_FLOAT) return p_f64((double)v_f32(v.b));
  return v.b;
}

// partition key per event (ValuePartitionExecutor; null key -> event dropped)
__global__ __launch_bounds__(kBlock) void k_nfa_keys(const KeyArgs* __restrict__ ap, int64_t n, int64_t stride,
                                                     uint64_t* key, uint32_t* keyed, unsigned long long* kmax) {
  const KeyArgs& a = *ap;
  const DExprSet es = a.es;
  unsigned long long m = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    BatchCtx cx{&a.batch, i};
    Val kv = a.key_col >= 0 ? col_load(a.batch, i, a.key_col)
                            : eval_expr(es.ins + a.key_expr.off, a.key_expr.len, es.consts, cx);
    uint64_t k = kv.null ? 0 : canon_key(kv, a.key_type);
    key[i] = k;
    keyed[i] = kv.null ? 0u : 1u;
    if (!kv.null && k > m) m = k;
  }
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long t = __shfl_xor(m, o, 64);
    m = t > m ? t : m;
  }
  __shared__ unsigned long long wm[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {   // one atomic per block (the grid is capped by grid_for)
    for (int w = 1; w < kBlock / 64; w++) m = wm[w] > m ? wm[w] : m;
    if (m) atomicMax(kmax, m);
  }
}

// Same-key runs of one call (PartitionStreamReceiver.receive(Event[]) :189-214)
__global__ void k_nfa_run_starts(const uint32_t* keyed, const uint64_t* key, const int32_t* call_of, int64_t n,
                                 uint32_t* start) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint32_t s = 0;
    if (keyed[i]) {
      int64_t p = i - 1;
      while (p >= 0 && call_of[p] == call_of[i] && !keyed[p]) p--;
      s = (p < 0 || call_of[p] != call_of[i] || key[p] != key[i]) ? 1u : 0u;
    }
    start[i] = s;
  }
}

__global__ void k_add_u32(const uint32_t* a, const uint32_t* b, int64_t n, uint32_t* out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = a[i] + b[i];
}

__global__ void k_call_run(const int32_t* call_of, int64_t n, uint32_t* run) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    run[i] = (uint32_t)call_of[i];
}

// compact keyed events: (key, row) in arrival order
__global__ void k_nfa_compact(const uint32_t* keyed, const uint32_t* pos, const uint64_t* key, int64_t n,
                              uint64_t* ck64, uint32_t* ck32, uint32_t* crow, int narrow) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!keyed[i]) continue;
    uint32_t o = pos[i];
    if (narrow) ck32[o] = (uint32_t)key[i];
    else ck64[o] = key[i];
    crow[o] = (uint32_t)i;
  }
}

template <class K>
__global__ void k_seg_heads(const K* sk, int64_t n, uint32_t* head) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i == 0 || sk[i] != sk[i - 1]) ? 1u : 0u;
}

template <class K>
__global__ void k_seg_write(const K* sk, const uint32_t* head, const uint32_t* hpos, int64_t n, uint32_t* seg_start,
                            uint64_t* seg_key) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!head[i]) continue;
    seg_start[hpos[i]] = (uint32_t)i;
    seg_key[hpos[i]] = (uint64_t)sk[i];
  }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Key directory: open-addressing table key -> slot.  Every inserting lane
// holds a distinct key (one lane per key segment), so a bucket claimed in
// this launch (state == epoch) never holds the probing lane's key.
__global__ void k_slot_lookup(const uint64_t* seg_key, int64_t nseg, uint32_t* ht_state, uint64_t* ht_key,
                              uint32_t* ht_slot, uint64_t mask, uint32_t epoch, unsigned int* nslots,
                              uint32_t* seg_slot, int32_t* slot_seg) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nseg; g += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = seg_key[g];
    uint64_t h = mix64(k) & mask;
    uint32_t slot = 0xFFFFFFFFu;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      uint32_t st = *reinterpret_cast<volatile uint32_t*>(&ht_state[h]);
      if (st == 0) {
        uint32_t old = atomicCAS(&ht_state[h], 0u, epoch);
        if (old == 0) {
          ht_key[h] = k;
          slot = atomicAdd(nslots, 1u);
          ht_slot[h] = slot;
          break;
        }
        st = old;
      }
      if (st != epoch && ht_key[h] == k) {
        slot = ht_slot[h];
        break;
      }
      h = (h + 1) & mask;
    }
    seg_slot[g] = slot;
    if (slot_seg && slot != 0xFFFFFFFFu) slot_seg[slot] = (int32_t)g;
  }
}

// rebuild the directory from the key blocks (after growth)
__global__ void k_slot_rebuild(const char* state, int64_t blk, int W, int64_t o_key, int64_t nslots,
                               uint32_t* ht_state, uint64_t* ht_key, uint32_t* ht_slot, uint64_t mask, uint32_t epoch) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nslots; s += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = *reinterpret_cast<const uint64_t*>(state + (s / W) * blk + o_key + (s % W) * 8);
    uint64_t h = mix64(k) & mask;
    for (uint64_t probe = 0; probe <= mask; probe++) {
      if (atomicCAS(&ht_state[h], 0u, epoch) == 0) {
        ht_key[h] = k;
        ht_slot[h] = (uint32_t)s;
        break;
      }
      h = (h + 1) & mask;
    }
  }
}

__global__ void k_store_keys(char* state, int64_t blk, int W, int64_t o_key, const uint64_t* seg_key,
                             const uint32_t* seg_slot, int64_t nseg) {
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < nseg; g += (int64_t)gridDim.x * blockDim.x) {
    uint32_t s = seg_slot[g];
    if (s == 0xFFFFFFFFu) continue;
    *reinterpret_cast<uint64_t*>(state + (s / W) * blk + o_key + (s % W) * 8) = seg_key[g];
  }
}

// call bookkeeping: call_of, per-call playback time, time-change flags, first seq
__global__ void k_nfa_calls(const int64_t* offs, int ncalls, const int64_t* ts, int32_t* call_of, int64_t* last_ts) {
  for (int c = blockIdx.x; c < ncalls; c += gridDim.x) {
    int64_t a = offs[c], b = offs[c + 1];
    for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) call_of[i] = c;
    if (threadIdx.x == 0) last_ts[c] = b > a ? ts[b - 1] : INT64_MIN;
  }
}

// TimestampGeneratorImpl.setCurrentTimestamp per call: only moves forward, and
// Scheduler.onTimeChange runs when t >= now.  Sequential over calls (one
// thread; calls are ~1/1000 of the events).
// Playback time per call (one workgroup): now[c] = the running max of the
// non-empty calls' last timestamps (InputHandler.send -> setCurrentTimestamp,
// time never goes back), changed[c] = call c moved (or met) the clock.  A
// block-wide max scan over 1024-call chunks (the one-thread loop it replaces
// took ~270 us per 1 M-event push).
__global__ __launch_bounds__(1024) void k_nfa_now(const int64_t* last_ts, const int64_t* offs, int ncalls,
                                                 int64_t now_prev, int64_t seq0, int advance, int64_t* now,
                                                 uint8_t* changed, int64_t* first) {
  __shared__ int64_t wmax[16];
  __shared__ int64_t carry_s;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (tid == 0) carry_s = now_prev;
  __syncthreads();
  for (int c0 = 0; c0 < ncalls; c0 += 1024) {
    const int c = c0 + tid;
    const bool in = c < ncalls;
    const bool live = in && advance && offs[c + 1] > offs[c];
    const int64_t t = live ? last_ts[c] : INT64_MIN;
    // inclusive max over the wave, then over the waves
    int64_t inc = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int64_t u = __shfl_up(inc, o, 64);
      if (lane >= o) inc = u > inc ? u : inc;
    }
    if (lane == 63) wmax[w] = inc;
    __syncthreads();
    const int64_t carry = carry_s;
    int64_t before = carry;   // max of now_prev and every earlier call's time
    for (int i = 0; i < w; i++) before = wmax[i] > before ? wmax[i] : before;
    int64_t excl = __shfl_up(inc, 1, 64);
    if (lane == 0) excl = INT64_MIN;
    excl = excl > before ? excl : before;
    if (in) {
      const bool ch = live && t >= excl;
      now[c] = ch ? t : excl;
      changed[c] = ch ? 1 : 0;
      first[c] = seq0 + offs[c];
    }
    __syncthreads();
    if (tid == 1023) {
      int64_t m = carry;
      for (int i = 0; i < 16; i++) m = wmax[i] > m ? wmax[i] : m;
      carry_s = m;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------- output ordering
__global__ void k_iota_u32(uint32_t* o, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    o[i] = (uint32_t)i;
}
__global__ void k_gather_keys(const uint64_t* src, const uint32_t* perm, int64_t n, uint64_t* dst) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[perm[i]];
}
__global__ void k_tag_heads(const uint64_t* tag, const uint32_t* perm, int64_t n, uint32_t* head) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    head[i] = (i == 0 || tag[perm[i]] != tag[perm[i - 1]]) ? 1u : 0u;
}
__global__ void k_out_rows(const uint32_t* perm, const uint32_t* hpos, const uint32_t* head, int64_t n, int nout,
                           int64_t chunk0, int64_t row0, const int64_t* sts, const int32_t* stype,
                           const uint64_t* svals, const uint8_t* snul, const uint64_t* sprim,
                           const int32_t* ssidx, int64_t* o_chunk, int32_t* o_type, int64_t* o_ts,
                           uint64_t* o_vals, uint8_t* o_nul, int64_t* o_seq, int32_t* o_sidx, uint32_t multi_mask,
                           int64_t lbase) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = perm[i];
    const int64_t r = row0 + i;
    o_chunk[r] = chunk0 + (int64_t)hpos[i] + (int64_t)head[i] - 1;
    o_type[r] = stype[j];
    o_ts[r] = sts[j];
    // primary tag: 2 * seq + 1 for an event's rows, 2 * (first seq of the call) for timer rows
    o_seq[r] = (int64_t)(sprim[j] >> 1);
    o_sidx[r] = ssidx[j];
    for (int c = 0; c < nout; c++) {
      const uint64_t v = svals[j * nout + c];
      // list handles: this push's arena lands at lbase of the output arena
      o_vals[r * nout + c] = (((multi_mask >> c) & 1u) && (v >> 40) != 0) ? v + (uint64_t)lbase : v;
      o_nul[r * nout + c] = snul[j * nout + c];
    }
  }
}

// ====================================================================== host: processor graph
struct HPre {
  int kind = PK_STREAM, stateId = -1, isStart = 0, stream = 0, thisPost = -1, thisLast = -1, withinEvery = -1,
      partner = -1, sched = -1, minC = 0, maxC = 0, ltype = 0;
  int64_t waiting = -1;
  std::vector<int> filters;
};
struct HPost {
  int kind = PK_STREAM, pre = -1, stateId = 0, nextPre = -1, nextEvery = -1, callbackPre = -1, partnerPre = -1,
      partnerPost = -1, minC = 0, maxC = 0, ltype = 0, hasSelector = 0;
};
struct HRt {
  int kind = 0, first = -1;
  std::vector<HRt> kids;
};

// Restates StateInputStreamParser.parse (C/util/parser/StateInputStreamParser.java:148-408)
// and the InnerStateRuntime setup / init / reset / update recursions.
struct GraphBuilder {
  const Plan& p;
  std::vector<HPre> pres;
  std::vector<HPost> posts;
  int n_sched = 0;
  std::vector<int> sched_pre;
  std::string err;
  explicit GraphBuilder(const Plan& pl) : p(pl) {}

  struct Res {
    int first, last;
    HRt rt;
  };

  Res parse(const PNode& n, int preIn, int postIn, bool isStart, std::vector<int>& preList) {
    switch (n.kind) {
      case SHD_NODE_STREAM: {
        int pi = preIn, po = postIn;
        if (pi < 0) {
          HPre pr;
          pr.kind = n.absent ? PK_ABSENT : PK_STREAM;
          if (n.absent) {
            pr.waiting = n.waiting;
            pr.sched = n_sched++;
            sched_pre.push_back((int)pres.size());
          }
          pres.push_back(pr);
          pi = (int)pres.size() - 1;
        }
        pres[pi].stateId = n.state_id;
        pres[pi].isStart = isStart;
        pres[pi].stream = n.stream;
        pres[pi].filters = n.filters;
        if (po < 0) {
          HPost ps;
          ps.kind = n.absent ? PK_ABSENT : PK_STREAM;
          posts.push_back(ps);
          po = (int)posts.size() - 1;
        }
        posts[po].stateId = n.state_id;
        posts[po].pre = pi;
        pres[pi].thisPost = po;
        pres[pi].thisLast = po;
        preList.push_back(pi);
        HRt rt;
        rt.kind = SHD_NODE_STREAM;
        rt.first = pi;
        return {pi, po, rt};
      }
      case SHD_NODE_NEXT: {
        Res a = parse(n.kids[0], preIn, postIn, isStart, preList);
        if (!err.empty()) return a;
        Res b = parse(n.kids[1], preIn, postIn, false, preList);
        if (!err.empty()) return b;
        set_next_pre(a.last, b.first);
        HRt rt;
        rt.kind = SHD_NODE_NEXT;
        rt.first = a.first;
        rt.kids.push_back(a.rt);
        rt.kids.push_back(b.rt);
        return {a.first, b.last, rt};
      }
      case SHD_NODE_EVERY: {
        std::vector<int> withinEvery;
        Res a = parse(n.kids[0], preIn, postIn, isStart, withinEvery);
        if (!err.empty()) return a;
        set_next_every(a.last, a.first);
        for (int x : withinEvery) pres[x].withinEvery = a.first;
        preList.insert(preList.end(), withinEvery.begin(), withinEvery.end());
        HRt rt;
        rt.kind = SHD_NODE_EVERY;
        rt.first = a.first;
        rt.kids.push_back(a.rt);
        return {a.first, a.last, rt};
      }
      case SHD_NODE_LOGICAL: {
        if (n.kids.size() != 2 || n.kids[0].kind != SHD_NODE_STREAM || n.kids[1].kind != SHD_NODE_STREAM) {
          err = "logical children must be stream states";
          return {-1, -1, HRt()};
        }
        const PNode& s1 = n.kids[0];
        const PNode& s2 = n.kids[1];
        // absent operands: AbsentLogicalPre/PostStateProcessor, with a scheduler each
        auto mk = [&](const PNode& sn) {
          HPre pr;
          pr.kind = sn.absent ? PK_ABSENT_LOGICAL : PK_LOGICAL;
          pr.ltype = n.ltype;
          if (sn.absent) {
            pr.waiting = sn.waiting;
            pr.sched = n_sched++;
            sched_pre.push_back((int)pres.size());
          }
          pres.push_back(pr);
          HPost ps;
          ps.kind = sn.absent ? PK_ABSENT_LOGICAL : PK_LOGICAL;
          ps.ltype = n.ltype;
          posts.push_back(ps);
          return std::make_pair((int)pres.size() - 1, (int)posts.size() - 1);
        };
        auto p1 = mk(s1);
        auto p2 = mk(s2);
        posts[p1.second].partnerPre = p2.first;
        posts[p2.second].partnerPre = p1.first;
        posts[p1.second].partnerPost = p2.second;
        posts[p2.second].partnerPost = p1.second;
        pres[p1.first].partner = p2.first;
        pres[p2.first].partner = p1.first;
        Res r2 = parse(s2, p2.first, p2.second, isStart, preList);
        Res r1 = parse(s1, p1.first, p1.second, isStart, preList);
        HRt rt;
        rt.kind = SHD_NODE_LOGICAL;
        rt.first = r1.first;
        rt.kids.push_back(r1.rt);
        rt.kids.push_back(r2.rt);
        return {r1.first, r2.last, rt};
      }
      case SHD_NODE_COUNT: {
        if (n.kids.size() != 1 || n.kids[0].kind != SHD_NODE_STREAM) {
          err = "count state over a non-stream state";
          return {-1, -1, HRt()};
        }
        int mn = n.min == -1 ? 0 : n.min;
        int mx = n.max == -1 ? INT32_MAX : n.max;
        HPre pr;
        pr.kind = PK_COUNT;
        pr.minC = mn;
        pr.maxC = mx;
        pres.push_back(pr);
        int pi = (int)pres.size() - 1;
        HPost ps;
        ps.kind = PK_COUNT;
        ps.minC = mn;
        ps.maxC = mx;
        posts.push_back(ps);
        int po = (int)posts.size() - 1;
        Res r = parse(n.kids[0], pi, po, isStart, preList);
        r.rt.kind = SHD_NODE_COUNT;
        return r;
      }
    }
    err = "bad node";
    return {-1, -1, HRt()};
  }

  void set_next_pre(int post, int pre) {
    if (post < 0 || pre < 0) return;
    HPost& ps = posts[post];
    ps.nextPre = pre;
    if (ps.kind == PK_LOGICAL || ps.kind == PK_ABSENT_LOGICAL) posts[ps.partnerPost].nextPre = pre;
    if (ps.kind == PK_COUNT) {   // CountPostStateProcessor.java:79-87
      if (pres[ps.pre].isStart && p.state_type == 1 && ps.minC == 0) posts[pres[pre].thisPost].callbackPre = ps.pre;
    }
  }
  void set_next_every(int post, int pre) {
    if (post < 0 || pre < 0) return;
    HPost& ps = posts[post];
    ps.nextEvery = pre;
    if (ps.kind == PK_LOGICAL || ps.kind == PK_ABSENT_LOGICAL) posts[ps.partnerPost].nextEvery = pre;
  }

  void setup(const HRt& r, std::vector<std::vector<int>>& streamPres) {
    switch (r.kind) {
      case SHD_NODE_STREAM:
      case SHD_NODE_COUNT: streamPres[pres[r.first].stream].push_back(r.first); break;
      case SHD_NODE_NEXT: setup(r.kids[0], streamPres); setup(r.kids[1], streamPres); break;
      case SHD_NODE_EVERY: setup(r.kids[0], streamPres); break;
      case SHD_NODE_LOGICAL: setup(r.kids[1], streamPres); setup(r.kids[0], streamPres); break;
    }
  }
  void set_selector(const HRt& r) {
    switch (r.kind) {
      case SHD_NODE_STREAM:
      case SHD_NODE_COUNT: posts[pres[r.first].thisPost].hasSelector = 1; break;
      case SHD_NODE_NEXT: set_selector(r.kids[1]); break;
      case SHD_NODE_EVERY: set_selector(r.kids[0]); break;
      case SHD_NODE_LOGICAL: set_selector(r.kids[1]); set_selector(r.kids[0]); break;
    }
  }
  void seq_init(const HRt& r, std::vector<int>& o) {
    switch (r.kind) {
      case SHD_NODE_STREAM:
      case SHD_NODE_COUNT: o.push_back(r.first); break;
      case SHD_NODE_NEXT: seq_init(r.kids[0], o); seq_init(r.kids[1], o); break;
      case SHD_NODE_EVERY: seq_init(r.kids[0], o); break;
      case SHD_NODE_LOGICAL: seq_init(r.kids[1], o); seq_init(r.kids[0], o); break;
    }
  }
  void seq_reset(const HRt& r, std::vector<int>& o) {
    switch (r.kind) {
      case SHD_NODE_STREAM:
      case SHD_NODE_COUNT:
      case SHD_NODE_EVERY: o.push_back(r.first); break;
      case SHD_NODE_NEXT: seq_reset(r.kids[1], o); seq_reset(r.kids[0], o); break;
      case SHD_NODE_LOGICAL: seq_reset(r.kids[1], o); break;
    }
  }
  void seq_update(const HRt& r, std::vector<int>& o) {
    switch (r.kind) {
      case SHD_NODE_STREAM:
      case SHD_NODE_COUNT:
      case SHD_NODE_EVERY: o.push_back(r.first); break;
      case SHD_NODE_NEXT: seq_update(r.kids[0], o); seq_update(r.kids[1], o); break;
      case SHD_NODE_LOGICAL: seq_update(r.kids[1], o); break;
    }
  }
};

int env_int(const char* name, int def) {
  const char* v = std::getenv(name);
  if (!v || !*v) return def;
  int x = std::atoi(v);
  return x > 0 ? x : def;
}

}  // namespace

void layout_offsets(NfaLayout& Y);

// Thrown by a push whose keys outgrew the per-key capacities (flags: OV_*):
// the engine grows its layout from the pre-push state and runs the push again.
struct NfaOverflow : Error {
  unsigned flags;
  int64_t rows, lrows;
  NfaOverflow(unsigned f, int64_t r, const std::string& m, int64_t lr = 0)
      : Error(SHD_E_CAPACITY, m), flags(f), rows(r), lrows(lr) {}
};

struct NfaEngine : Engine {
  NfaProg prog{};
  NfaLayout lay{};
  std::vector<std::vector<int>> pre_filters;
  // Window lanes (unpartitioned sequences whose partials span at most `span`
  // events, every-started, one stream): a sequence partial survives an event
  // only by advancing on it (StateStreamRuntime.resetAndUpdate clears every
  // non-start pending list, ST/StateStreamRuntime.java:81-84), so the state
  // after event j depends on events (j-span, j] alone.  The push is cut into
  // chunks, one lane each, every lane replaying `warm` >= span events before
  // its chunk from a fresh state (output suppressed); the last `warm` events
  // carry to the next push (prefix) instead of key blocks.
  bool windowed = false;
  int64_t win_warm = 0;
  int64_t win_span = 0;      // sequences: events a partial can span (0: unbounded)
  int64_t win_horizon = 0;   // patterns: longest within / for time (0: none)
  DevBuf d_hash;
  int64_t win_fallbacks = 0;   // window passes rerun with longer warm-ups
  const bool win_debug = getenv("SHD_NFA_DEBUG") != nullptr;
  bool partitioned = false;
  int key_expr[kNStream], key_col[kNStream], key_type[kNStream];
  // key blocks
  DevBuf state;
  int64_t slot_cap = 0;   // slots with memory (multiple of 64)
  int64_t nslots = 0;
  // key directory
  DevBuf ht_state, ht_key, ht_slot;
  int64_t ht_cap = 0;
  uint32_t epoch = 0;
  // scratch
  DevBuf d_offs, d_call_of, d_last, d_now, d_changed, d_first, d_key, d_keyed, d_pos, d_runs, d_run, d_ck64,
      d_ck64_alt, d_ck32, d_ck32_alt, d_crow, d_crow_alt, d_head, d_hpos, d_seg_start, d_seg_key, d_seg_slot,
      d_slot_seg, d_ctl, d_scan, d_sort;
  DevBuf st_sidx, st_tag, st_p, st_s, st_t, st_ts, st_type, st_vals, st_nul, d_perm, d_perm_alt, d_skey, d_skey_alt, d_thead,
      d_thpos;
  int64_t R = 0;
  PinnedBuf h_ctl, h_up;
  size_t h_up_used = 0;

  int kind() const override { return ENG_NFA; }

  void on_loaded() override {
    // expression handles exist once the plan's expression table is uploaded
    for (int i = 0; i < prog.npre; i++) prog.pre[i].filters = dfilters(pre_filters[i]);
    for (int c = 0; c < prog.nout; c++) prog.outs[c] = dexpr(plan.outputs[c].second);
  }

  void reset() override {
    if (stream) SHD_HIP(hipStreamSynchronize(stream));
    seq = 0;
    now = 0;   // TimestampGeneratorImpl starts at 0 (playback)
    chunk_seq = 0;
    out.count = 0;
    counters = shd_counters{};
    nslots = 0;
    epoch = 0;
    if (state.p && slot_cap > 0) SHD_HIP(hipMemset(state.p, 0, (size_t)(slot_cap / lay.W) * lay.blk));
    if (ht_state.p && ht_cap > 0) SHD_HIP(hipMemset(ht_state.p, 0, (size_t)ht_cap * 4));
    SHD_HIP(hipDeviceSynchronize());
  }

  // key blocks (all per-key NFA state) + key directory, byte for byte
  void save_caps(SnapW& w) const {
    w.put<int32_t>(lay.L); w.put<int32_t>(lay.SC); w.put<int32_t>(lay.EC); w.put<int32_t>(lay.RC);
    w.put<int32_t>(lay.QC); w.put<int32_t>(lay.RETC); w.put<int32_t>(lay.WK);
  }
  // a snapshot taken after growth carries its (larger) capacities: adopt them
  void load_caps(SnapR& r) {
    NfaLayout ny = lay;
    ny.L = r.get<int32_t>(); ny.SC = r.get<int32_t>(); ny.EC = r.get<int32_t>(); ny.RC = r.get<int32_t>();
    ny.QC = r.get<int32_t>(); ny.RETC = r.get<int32_t>(); ny.WK = r.get<int32_t>();
    if (ny.L < 1 || ny.L >= 65000 || ny.SC < 1 || ny.SC > 32768 || ny.EC < 1 || ny.EC > 65000 || ny.RC < 1 ||
        ny.RC > 65000 || ny.QC < 1 || ny.QC >= 65000 || ny.RETC < 1 || ny.RETC > 65000 || ny.WK < 1)
      throw Error(SHD_E_ARG, "snapshot of a different plan");
    layout_offsets(ny);
    if (ny.blk != lay.blk) {
      state.release();
      slot_cap = 0;
    }
    lay = ny;
  }
  void save_state(SnapW& w) override {
    save_caps(w);
    if (windowed) {   // the carried state: slot 0's block (+ the learned warm-up)
      w.put<int64_t>(win_warm);
      w.put<int64_t>(slot_cap > 0 ? 1 : 0);
      if (slot_cap > 0) w.dev(state.p, (size_t)lay.blk);
      return;
    }
    w.put<int64_t>(slot_cap);
    w.put<int64_t>(nslots);
    w.put<int64_t>(ht_cap);
    w.put<uint32_t>(epoch);
    w.put<int64_t>((int64_t)lay.blk);
    w.dev(state.p, (size_t)(slot_cap / lay.W) * lay.blk);
    w.dev(ht_state.p, (size_t)ht_cap * 4);
    w.dev(ht_key.p, (size_t)ht_cap * 8);
    w.dev(ht_slot.p, (size_t)ht_cap * 4);
  }
  void load_state(SnapR& r) override {
    load_caps(r);
    if (windowed) {
      const int64_t ww = r.get<int64_t>();
      if (ww < 0 || ww > ((int64_t)1 << 40)) throw Error(SHD_E_ARG, "snapshot of a different plan");
      if (r.get<int64_t>() != 0) {
        ensure_slots(kLaneBlock);
        r.dev_into(state.p, (size_t)lay.blk);
        nslots = 1;
      }
      win_warm = ww;
      return;
    }
    const int64_t sc = r.get<int64_t>(), ns = r.get<int64_t>(), hc = r.get<int64_t>();
    const uint32_t ep = r.get<uint32_t>();
    if (r.get<int64_t>() != (int64_t)lay.blk || sc < 0 || ns < 0 || ns > sc || hc < 0 || sc % kLaneBlock)
      throw Error(SHD_E_ARG, "snapshot of a different plan");
    const size_t sb = (size_t)(sc / lay.W) * lay.blk;
    state.reserve(std::max<size_t>(sb, 1));
    r.dev_into(state.p, sb);
    ht_state.reserve(std::max<int64_t>(hc, 1) * 4);
    ht_key.reserve(std::max<int64_t>(hc, 1) * 8);
    ht_slot.reserve(std::max<int64_t>(hc, 1) * 4);
    r.dev_into(ht_state.p, (size_t)hc * 4);
    r.dev_into(ht_key.p, (size_t)hc * 8);
    r.dev_into(ht_slot.p, (size_t)hc * 4);
    slot_cap = sc;
    nslots = ns;
    ht_cap = hc;
    epoch = ep;
  }

  void set_time(int64_t t) override {
    // shd_set_time: a time change without events (Scheduler TIMERs still fire)
    if (t < now) return;
    if (prog.nsched == 0) {
      now = t;
      return;
    }
    run_push(nullptr, t);
  }

  // host -> device through library-owned pinned memory (stream ordered)
  void upload(void* dst, const void* src, size_t bytes) {
    size_t need = (bytes + 63) & ~size_t(63);
    if (!h_up.p || h_up_used + need > h_up.cap) {
      SHD_HIP(hipStreamSynchronize(stream));
      h_up.reserve(std::max<size_t>(need + 4096, h_up.cap * 2));
      h_up_used = 0;
    }
    std::memcpy(h_up.as<char>() + h_up_used, src, bytes);
    SHD_HIP(hipMemcpyAsync(dst, h_up.as<char>() + h_up_used, bytes, hipMemcpyHostToDevice, stream));
    h_up_used += need;
  }

  NfaCtl read_ctl() {
    SHD_HIP(hipMemcpyAsync(h_ctl.p, d_ctl.p, sizeof(NfaCtl), hipMemcpyDeviceToHost, stream));
    SHD_HIP(hipStreamSynchronize(stream));
    NfaCtl c;
    std::memcpy(&c, h_ctl.p, sizeof(c));
    return c;
  }

  void ensure_slots(int64_t need) {
    if (need <= slot_cap) return;
    int64_t nc = std::max<int64_t>(need, slot_cap * 2);
    nc = (nc + kLaneBlock - 1) / kLaneBlock * kLaneBlock;
    DevBuf nb;
    nb.reserve((size_t)(nc / lay.W) * lay.blk);
    size_t old = (size_t)(slot_cap / lay.W) * lay.blk;
    if (old) SHD_HIP(hipMemcpyAsync(nb.p, state.p, old, hipMemcpyDeviceToDevice, stream));
    SHD_HIP(hipMemsetAsync((char*)nb.p + old, 0, (size_t)(nc / lay.W) * lay.blk - old, stream));
    SHD_HIP(hipStreamSynchronize(stream));
    std::swap(state.p, nb.p);
    std::swap(state.cap, nb.cap);
    slot_cap = nc;
  }

  void ensure_directory(int64_t keys) {
    int64_t want = 64;
    while (want < 2 * keys + 64) want <<= 1;
    if (want <= ht_cap) return;
    ht_state.reserve(want * 4);
    ht_key.reserve(want * 8);
    ht_slot.reserve(want * 4);
    ht_cap = want;
    SHD_HIP(hipMemsetAsync(ht_state.p, 0, want * 4, stream));
    if (nslots > 0) {
      epoch++;
      hipLaunchKernelGGL(k_slot_rebuild, dim3(grid_for(nslots)), dim3(kBlock), 0, stream, (const char*)state.p,
                         lay.blk, lay.W, lay.o_key, nslots, ht_state.as<uint32_t>(), ht_key.as<uint64_t>(),
                         ht_slot.as<uint32_t>(), (uint64_t)(ht_cap - 1), epoch);
      SHD_CHECK_LAUNCH();
    }
  }

  void ensure_staging(int64_t rows) {
    if (rows <= R) return;
    int nout = std::max(prog.nout, 1);
    st_tag.reserve(rows * 8);
    st_p.reserve(rows * 8);
    st_s.reserve(rows * 8);
    st_t.reserve(rows * 8);
    st_sidx.reserve(rows * 4);
    st_ts.reserve(rows * 8);
    st_type.reserve(rows * 4);
    st_vals.reserve(rows * nout * 8);
    st_nul.reserve(rows * nout);
    R = rows;
  }

  // list arena of multi-value outputs (entries)
  DevBuf st_lv, st_ln;
  int64_t LR = 0;
  void ensure_lists(int64_t n) {
    if (n <= LR) return;
    st_lv.reserve(n * 8);
    st_ln.reserve(n);
    LR = n;
  }

  void push(const Staged& b) override { run_push(&b, 0); }

  // Key-sort the keyed events of a partitioned push, map keys to slots.
  // Returns the number of key segments; fills ra.rows / seg arrays.
  int64_t route_keys(const Staged& b, NfaRunArgs& ra, int64_t& n_keyed, bool timers) {
    hipStream_t s = stream;
    const int64_t n = b.n;
    const int si = b.stream;
    d_key.reserve(n * 8);
    d_keyed.reserve(n * 4);
    d_pos.reserve(n * 4);
    d_runs.reserve(n * 4);
    KeyArgs ka{};
    ka.batch = b.cs;
    ka.es = dset();
    ka.key_expr = dexpr(key_expr[si]);
    ka.key_col = key_col[si];
    ka.key_type = key_type[si];
    SHD_HIP(hipMemsetAsync(d_ctl.p, 0, sizeof(NfaCtl), s));
    const int nblk = grid_for(n);
    hipLaunchKernelGGL(k_nfa_keys, dim3(nblk), dim3(kBlock), 0, s, dev_args(ka), n, (int64_t)nblk * kBlock,
                       d_key.as<uint64_t>(), d_keyed.as<uint32_t>(), &d_ctl.as<NfaCtl>()->kmax);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_nfa_run_starts, dim3(grid_for(n)), dim3(kBlock), 0, s, (const uint32_t*)d_keyed.as<uint32_t>(),
                       (const uint64_t*)d_key.as<uint64_t>(), (const int32_t*)d_call_of.as<int32_t>(), n,
                       d_runs.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    // run id = inclusive scan of run starts
    scan_exclusive_u32(d_runs.as<uint32_t>(), d_run.as<uint32_t>(), n, nullptr, d_scan, s);
    hipLaunchKernelGGL(k_add_u32, dim3(grid_for(n)), dim3(kBlock), 0, s, (const uint32_t*)d_run.as<uint32_t>(),
                       (const uint32_t*)d_runs.as<uint32_t>(), n, d_run.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    scan_exclusive_u32(d_keyed.as<uint32_t>(), d_pos.as<uint32_t>(), n, &d_ctl.as<NfaCtl>()->count, d_scan, s);
    NfaCtl hc = read_ctl();
    n_keyed = hc.count;
    const unsigned long long kmax = hc.kmax;
    mark("keys");
    if (n_keyed == 0) return 0;
    int bits = 0;
    while (bits < 64 && (kmax >> bits)) bits++;
    const bool narrow = bits <= 32;
    d_crow.reserve(n_keyed * 4);
    d_crow_alt.reserve(n_keyed * 4);
    d_ck32.reserve(n_keyed * 4);
    d_ck32_alt.reserve(n_keyed * 4);
    if (!narrow) {
      d_ck64.reserve(n_keyed * 8);
      d_ck64_alt.reserve(n_keyed * 8);
    }
    hipLaunchKernelGGL(k_nfa_compact, dim3(grid_for(n)), dim3(kBlock), 0, s, (const uint32_t*)d_keyed.as<uint32_t>(),
                       (const uint32_t*)d_pos.as<uint32_t>(), (const uint64_t*)d_key.as<uint64_t>(), n,
                       d_ck64.as<uint64_t>(), d_ck32.as<uint32_t>(), d_crow.as<uint32_t>(), narrow ? 1 : 0);
    SHD_CHECK_LAUNCH();
    bool in_alt = false;
    if (narrow)
      radix_sort_pairs_u32(d_ck32.as<uint32_t>(), d_crow.as<uint32_t>(), d_ck32_alt.as<uint32_t>(),
                           d_crow_alt.as<uint32_t>(), n_keyed, bits, d_sort, s, in_alt);
    else
      radix_sort_pairs_u64(d_ck64.as<uint64_t>(), d_crow.as<uint32_t>(), d_ck64_alt.as<uint64_t>(),
                           d_crow_alt.as<uint32_t>(), n_keyed, bits, d_sort, s, in_alt);
    ra.rows = in_alt ? d_crow_alt.as<uint32_t>() : d_crow.as<uint32_t>();
    d_head.reserve(n_keyed * 4);
    d_hpos.reserve(n_keyed * 4);
    d_seg_start.reserve(n_keyed * 4);
    d_seg_key.reserve(n_keyed * 8);
    SHD_HIP(hipMemsetAsync(d_ctl.p, 0, sizeof(NfaCtl), s));
    unsigned int* d_cnt = &d_ctl.as<NfaCtl>()->count;
    if (narrow) {
      const uint32_t* sk = in_alt ? d_ck32_alt.as<uint32_t>() : d_ck32.as<uint32_t>();
      hipLaunchKernelGGL(k_seg_heads<uint32_t>, dim3(grid_for(n_keyed)), dim3(kBlock), 0, s, sk, n_keyed,
                         d_head.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      scan_exclusive_u32(d_head.as<uint32_t>(), d_hpos.as<uint32_t>(), n_keyed, d_cnt, d_scan, s);
      hipLaunchKernelGGL(k_seg_write<uint32_t>, dim3(grid_for(n_keyed)), dim3(kBlock), 0, s, sk,
                         (const uint32_t*)d_head.as<uint32_t>(), (const uint32_t*)d_hpos.as<uint32_t>(), n_keyed,
                         d_seg_start.as<uint32_t>(), d_seg_key.as<uint64_t>());
    } else {
      const uint64_t* sk = in_alt ? d_ck64_alt.as<uint64_t>() : d_ck64.as<uint64_t>();
      hipLaunchKernelGGL(k_seg_heads<uint64_t>, dim3(grid_for(n_keyed)), dim3(kBlock), 0, s, sk, n_keyed,
                         d_head.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      scan_exclusive_u32(d_head.as<uint32_t>(), d_hpos.as<uint32_t>(), n_keyed, d_cnt, d_scan, s);
      hipLaunchKernelGGL(k_seg_write<uint64_t>, dim3(grid_for(n_keyed)), dim3(kBlock), 0, s, sk,
                         (const uint32_t*)d_head.as<uint32_t>(), (const uint32_t*)d_hpos.as<uint32_t>(), n_keyed,
                         d_seg_start.as<uint32_t>(), d_seg_key.as<uint64_t>());
    }
    SHD_CHECK_LAUNCH();
    hc = read_ctl();
    const int64_t nseg = hc.count;
    // ---- key directory lookup / insert
    ensure_slots(nslots + nseg);
    ensure_directory(nslots + nseg);
    d_seg_slot.reserve(nseg * 4);
    if (timers) {
      d_slot_seg.reserve(slot_cap * 4);
      SHD_HIP(hipMemsetAsync(d_slot_seg.p, 0xFF, slot_cap * 4, s));
    }
    NfaCtl init{};
    init.count = (unsigned int)nslots;
    upload(d_ctl.p, &init, sizeof(init));
    epoch++;
    hipLaunchKernelGGL(k_slot_lookup, dim3(grid_for(nseg)), dim3(kBlock), 0, s, (const uint64_t*)d_seg_key.as<uint64_t>(),
                       nseg, ht_state.as<uint32_t>(), ht_key.as<uint64_t>(), ht_slot.as<uint32_t>(),
                       (uint64_t)(ht_cap - 1), epoch, &d_ctl.as<NfaCtl>()->count, d_seg_slot.as<uint32_t>(),
                       timers ? d_slot_seg.as<int32_t>() : nullptr);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_store_keys, dim3(grid_for(nseg)), dim3(kBlock), 0, s, state.as<char>(), lay.blk, lay.W, lay.o_key,
                       (const uint64_t*)d_seg_key.as<uint64_t>(), (const uint32_t*)d_seg_slot.as<uint32_t>(), nseg);
    SHD_CHECK_LAUNCH();
    hc = read_ctl();
    nslots = hc.count;
    mark("key_sort");
    return nseg;
  }

  // copy slot src's state into slots [dst0, dst0 + ndst)
  void lane_copy(int64_t src, int64_t dst0, int64_t ndst) {
    if (ndst <= 0) return;
    int64_t mx = 1;
    for (int f = 0; f < lay.nf; f++) mx = std::max<int64_t>(mx, lay.f_cnt[f]);
    const unsigned gx = (unsigned)std::min<int64_t>(1024, ceil_div(mx * ndst, kBlock));
    hipLaunchKernelGGL(k_lane_copy, dim3(gx, (unsigned)lay.nf), dim3(kBlock), 0, stream, dev_args(lay), state.as<char>(),
                       src, dst0, ndst);
    SHD_CHECK_LAUNCH();
  }

  // Warm-up length for window lanes: a sequence partial lives at most `span`
  // events; a pattern partial bounded by `within` / `for` time H lives about
  // H / (mean event spacing) events of this push (verification catches the rest)
  int64_t win_warm_hint(const Staged& b) {
    if (win_span > 0) return 2 * win_span + 2;
    if (win_horizon <= 0 || b.n < 2) return 64;
    int64_t t2[2];
    SHD_HIP(hipMemcpyAsync(&t2[0], b.cs.ts, 8, hipMemcpyDeviceToHost, stream));
    SHD_HIP(hipMemcpyAsync(&t2[1], b.cs.ts + (b.n - 1), 8, hipMemcpyDeviceToHost, stream));
    SHD_HIP(hipStreamSynchronize(stream));
    const double dt = (double)(t2[1] - t2[0]) / (double)(b.n - 1);
    if (!(dt > 0)) return 64;
    // timers fire at call boundaries: a partial outlives its time by up to a call
    int64_t call_max = 0;
    for (size_t c = 0; c + 1 < b.call_offsets.size(); c++)
      call_max = std::max<int64_t>(call_max, b.call_offsets[c + 1] - b.call_offsets[c]);
    if (prog.nsched == 0) call_max = 0;
    return (int64_t)std::min<double>(1e9, 1.25 * ((double)win_horizon / dt + (double)call_max) + 64);
  }

  // One push (b != nullptr) or one time change (b == nullptr, time t).
  // SHD_E_CAPACITY never reaches the caller while the handle space (16-bit
  // handles) allows growth: a push that overflows a key's lists / pools is
  // rerun from the pre-push state with the overflowed capacities doubled
  // (the key blocks re-laid out on the device, k_nfa_relayout).
  DevBuf backup;
  int64_t backup_blocks = 0, backup_nslots = 0;
  int64_t grows = 0;
  void run_push(const Staged* b, int64_t t_only) {
    // the pre-push key blocks (window lanes: the carried state, slot 0's block)
    backup_nslots = nslots;
    const int64_t used = windowed ? std::min<int64_t>(slot_cap, 1) : nslots;
    backup_blocks = used > 0 ? ceil_div(used, lay.W) : 0;
    if (backup_blocks > 0) {
      backup.reserve((size_t)backup_blocks * lay.blk);
      SHD_HIP(hipMemcpyAsync(backup.p, state.p, (size_t)backup_blocks * lay.blk, hipMemcpyDeviceToDevice, stream));
    }
    for (;;) {
      try {
        run_push_once(b, t_only);
        return;
      } catch (NfaOverflow& o) {
        if (o.flags & OV_MULTI) ensure_lists(2 * std::max(LR, o.lrows));
        grow(o.flags & ~(unsigned)OV_MULTI, o.rows, o.what(), (o.flags & OV_MULTI) != 0);
      }
    }
  }

  void grow(unsigned ovf, int64_t rows, const char* msg, bool lists_grown = false) {
    args_begin();   // the failed attempt's argument blocks are no longer read
    NfaLayout ny = lay;
    bool changed = lists_grown;
    auto dbl = [&](int& v, int mx) {
      const int nv = std::min(2 * v, mx);
      if (nv > v) {
        v = nv;
        changed = true;
      }
    };
    if (ovf & OV_LIST) {
      dbl(ny.L, 64999);
      ny.RETC = std::max(ny.RETC, std::min(ny.L * std::max(ny.npre, 1), 65000));
    }
    if (ovf & OV_SE) dbl(ny.SC, 32768);
    if (ovf & OV_EV) dbl(ny.EC, 65000);
    if (ovf & OV_REC) dbl(ny.RC, 65000);
    if (ovf & OV_SCHED) dbl(ny.QC, 64999);
    if (ovf & OV_RET) dbl(ny.RETC, 65000);
    if (ovf & OV_WORK) dbl(ny.WK, 1 << 20);
    if (rows > R) {
      ensure_staging(2 * rows);
      changed = true;
    }
    if (!changed) throw Error(SHD_E_CAPACITY, std::string(msg) + " (at the largest per-key capacities)");
    grows++;
    if (ny.L != lay.L || ny.SC != lay.SC || ny.EC != lay.EC || ny.RC != lay.RC || ny.QC != lay.QC ||
        ny.RETC != lay.RETC || ny.WK != lay.WK) {
      layout_offsets(ny);
      relayout(ny);
    } else if (backup_blocks > 0) {   // same layout (staging grew): back to the pre-push blocks
      SHD_HIP(hipMemcpyAsync(state.p, backup.p, (size_t)backup_blocks * lay.blk, hipMemcpyDeviceToDevice, stream));
    }
    // keys first seen by the failed attempt are forgotten: the directory is
    // rebuilt from the pre-push slots, the retry inserts them again
    if (!windowed && partitioned && (nslots != backup_nslots || backup_blocks > 0)) {
      nslots = backup_nslots;
      if (ht_cap > 0) {
        SHD_HIP(hipMemsetAsync(ht_state.p, 0, (size_t)ht_cap * 4, stream));
        epoch++;
        if (nslots > 0) {
          hipLaunchKernelGGL(k_slot_rebuild, dim3(grid_for(nslots)), dim3(kBlock), 0, stream, (const char*)state.p,
                             lay.blk, lay.W, lay.o_key, nslots, ht_state.as<uint32_t>(), ht_key.as<uint64_t>(),
                             ht_slot.as<uint32_t>(), (uint64_t)(ht_cap - 1), epoch);
          SHD_CHECK_LAUNCH();
        }
      }
      // blocks of the forgotten slots start unseeded again
      const int64_t keep_b = ceil_div(nslots, lay.W);
      const size_t keep = (size_t)keep_b * lay.blk, all = (size_t)(slot_cap / lay.W) * lay.blk;
      if (all > keep && backup_blocks == keep_b) {
        // the pre-push blocks hold nslots slots; the partial block's later slots were unseeded before the push
        SHD_HIP(hipMemsetAsync(state.as<char>() + keep, 0, all - keep, stream));
      }
    }
    SHD_HIP(hipStreamSynchronize(stream));
  }

  // the pre-push blocks (backup) re-laid out for `ny` into a fresh state
  // array; slots beyond them start zero (unseeded)
  void relayout(const NfaLayout& ny) {
    const NfaLayout& o = lay;
    RelayArgs ra{};
    auto add = [&](int64_t oo, int64_t on, int64_t rows, int64_t cols, int64_t cold, int64_t cnew, int sz, int kind,
                   int64_t wold = 0, int64_t lo = 0, int64_t hi = 0) {
      RelayField& f = ra.f[ra.nfield++];
      f.off_old = oo; f.off_new = on; f.rows = rows; f.cols = cols; f.cols_old = cold; f.cols_new = cnew;
      f.sz = sz; f.kind = kind; f.words_old = wold; f.lo = lo; f.hi = hi;
    };
    const int64_t nsch = std::max(o.nsched, 1);
    add(o.o_pend, ny.o_pend, o.npre, o.L, o.L + 1, ny.L + 1, 2, 0);
    add(o.o_pend_n, ny.o_pend_n, 1, o.npre, o.npre, ny.npre, 2, 0);
    add(o.o_new, ny.o_new, o.npre, o.L, o.L + 1, ny.L + 1, 2, 0);
    add(o.o_new_n, ny.o_new_n, 1, o.npre, o.npre, ny.npre, 2, 0);
    add(o.o_flags, ny.o_flags, 1, o.npre, o.npre, ny.npre, 1, 0);
    add(o.o_lst, ny.o_lst, 1, o.npre, o.npre, ny.npre, 8, 0);
    add(o.o_sq, ny.o_sq, nsch, o.QC, o.QC, ny.QC, 8, 0);
    add(o.o_sq_n, ny.o_sq_n, 1, nsch, nsch, nsch, 2, 0);
    add(o.o_se_ev, ny.o_se_ev, o.SC, o.nstates, o.nstates, ny.nstates, 2, 0);
    add(o.o_se_ts, ny.o_se_ts, 1, o.SC, o.SC + 1, ny.SC + 1, 8, 0);
    add(o.o_se_type, ny.o_se_type, 1, o.SC, o.SC + 1, ny.SC + 1, 1, 0);
    add(o.o_se_free, ny.o_se_free, 0, 0, o.sew, ny.sew, 8, 1, o.sew, o.SC, ny.SC);
    add(o.o_se_mark, ny.o_se_mark, 0, 0, o.sew, ny.sew, 8, 2);
    add(o.o_ev_rec, ny.o_ev_rec, 1, o.EC, o.EC + 1, ny.EC + 1, 2, 0);
    add(o.o_ev_next, ny.o_ev_next, 1, o.EC, o.EC + 1, ny.EC + 1, 2, 0);
    add(o.o_ev_free, ny.o_ev_free, 0, 0, o.evw, ny.evw, 8, 1, o.evw, o.EC, ny.EC);
    add(o.o_ev_mark, ny.o_ev_mark, 0, 0, o.evw, ny.evw, 8, 2);
    add(o.o_rec_ts, ny.o_rec_ts, 1, o.RC, o.RC + 1, ny.RC + 1, 8, 0);
    add(o.o_rec_val, ny.o_rec_val, o.RC, o.ncols, o.ncols, ny.ncols, 8, 0);
    add(o.o_rec_nul, ny.o_rec_nul, 1, o.RC, o.RC + 1, ny.RC + 1, 4, 0);
    add(o.o_rec_free, ny.o_rec_free, 0, 0, o.recw, ny.recw, 8, 1, o.recw, o.RC, ny.RC);
    add(o.o_rec_mark, ny.o_rec_mark, 0, 0, o.recw, ny.recw, 8, 2);
    add(o.o_ret, ny.o_ret, 1, o.RETC, o.RETC + 1, ny.RETC + 1, 2, 0);
    add(o.o_tmp, ny.o_tmp, 1, o.RETC, o.RETC + 1, ny.RETC + 1, 2, 0);
    add(o.o_wk, ny.o_wk, 1, o.WK + 1, o.WK + 1, ny.WK + 1, 4, 0);
    add(o.o_key, ny.o_key, 1, 1, 1, 1, 8, 0);
    add(o.o_misc, ny.o_misc, 1, MISC_N, MISC_N, MISC_N, 4, 3);
    add(o.o_cse, ny.o_cse, 1, o.SC + 1, o.SC + 1, ny.SC + 1, 4, 0);
    add(o.o_cev, ny.o_cev, 1, o.EC + 1, o.EC + 1, ny.EC + 1, 4, 0);
    ra.blk_old = o.blk;
    ra.blk_new = ny.blk;
    ra.nblocks = backup_blocks;
    ra.W = o.W;
    ra.dSE = ny.SC - o.SC;
    ra.dEV = ny.EC - o.EC;
    ra.dREC = ny.RC - o.RC;
    const size_t bytes = (size_t)(slot_cap / o.W) * ny.blk;
    DevBuf nb;
    nb.reserve(std::max<size_t>(bytes, 1));
    SHD_HIP(hipMemsetAsync(nb.p, 0, bytes, stream));
    if (backup_blocks > 0) {
      hipLaunchKernelGGL(k_nfa_relayout, dim3(grid_cover(backup_blocks * o.W)), dim3(kBlock), 0, stream,
                         dev_args(ra), (const char*)backup.p, nb.as<char>());
      SHD_CHECK_LAUNCH();
      // the new layout's backup: a later overflow of the same push starts from it
      DevBuf bk;
      bk.reserve((size_t)backup_blocks * ny.blk);
      SHD_HIP(hipMemcpyAsync(bk.p, nb.p, (size_t)backup_blocks * ny.blk, hipMemcpyDeviceToDevice, stream));
      SHD_HIP(hipStreamSynchronize(stream));
      std::swap(backup.p, bk.p);
      std::swap(backup.cap, bk.cap);
    }
    SHD_HIP(hipStreamSynchronize(stream));
    std::swap(state.p, nb.p);
    std::swap(state.cap, nb.cap);
    lay = ny;
  }

  void run_push_once(const Staged* b, int64_t t_only) {
    hipStream_t s = stream;
    h_up_used = 0;
    SHD_HIP(hipEventRecord(ev0, s));
    stage_begin();
    const int64_t n = b ? b->n : 0;
    const int si = b ? b->stream : 0;
    std::vector<int64_t> offs = b ? b->call_offsets : std::vector<int64_t>{0, 1};
    const int ncalls = (int)offs.size() - 1;
    const int64_t n1 = std::max<int64_t>(n, 1);
    d_offs.reserve((ncalls + 1) * 8);
    d_call_of.reserve(n1 * 4);
    d_last.reserve(ncalls * 8);
    d_now.reserve(ncalls * 8);
    d_changed.reserve(ncalls);
    d_first.reserve(ncalls * 8);
    d_run.reserve(n1 * 4);
    d_ctl.reserve(sizeof(NfaCtl));
    h_ctl.reserve(256);
    upload(d_offs.p, offs.data(), (ncalls + 1) * 8);
    if (b) {
      hipLaunchKernelGGL(k_nfa_calls, dim3(std::min(ncalls, 4096)), dim3(kBlock), 0, s,
                         (const int64_t*)d_offs.as<int64_t>(), ncalls, b->cs.ts, d_call_of.as<int32_t>(),
                         d_last.as<int64_t>());
      SHD_CHECK_LAUNCH();
    } else {
      upload(d_last.p, &t_only, 8);
    }
    hipLaunchKernelGGL(k_nfa_now, dim3(1), dim3(1024), 0, s, (const int64_t*)d_last.as<int64_t>(),
                       (const int64_t*)d_offs.as<int64_t>(), ncalls, now, seq, (b ? (int)b->advance_time : 1),
                       d_now.as<int64_t>(), d_changed.as<uint8_t>(), d_first.as<int64_t>());
    SHD_CHECK_LAUNCH();
    mark("calls");

    NfaRunArgs ra{};
    if (b) ra.batch = b->cs;
    ra.skip_start = b ? b->skip_start : nullptr;
    ra.stream = si;
    ra.partitioned = partitioned;
    ra.ncalls = ncalls;
    ra.seq0 = seq;
    ra.start_time = start_time;
    ra.call_of = d_call_of.as<int32_t>();
    ra.call_now = d_now.as<int64_t>();
    ra.call_changed = d_changed.as<uint8_t>();
    ra.call_first = d_first.as<int64_t>();
    ra.es = dset();
    const bool timers = prog.nsched > 0;
    int64_t nseg = 0, n_keyed = n;
    const bool win = windowed && b && n > 0;
    bool win_one = false;   // window push rerun on one lane

    if (win) {
      ensure_slots(1);
      nslots = 1;
      ra.lanes_over_slots = 0;
      if (n > 0) {
        hipLaunchKernelGGL(k_call_run, dim3(grid_for(n)), dim3(kBlock), 0, s, (const int32_t*)d_call_of.as<int32_t>(),
                           n, d_run.as<uint32_t>());
        SHD_CHECK_LAUNCH();
      }
    } else if (!partitioned) {
      ensure_slots(1);
      nslots = 1;
      if (n > 0) {
        hipLaunchKernelGGL(k_call_run, dim3(grid_for(n)), dim3(kBlock), 0, s, (const int32_t*)d_call_of.as<int32_t>(),
                           n, d_run.as<uint32_t>());
        SHD_CHECK_LAUNCH();
      }
      ra.lanes_over_slots = 0;
      ra.nlanes = 1;
      ra.nseg = 1;
    } else {
      if (n > 0) nseg = route_keys(*b, ra, n_keyed, timers);
      ra.seg_start = d_seg_start.as<uint32_t>();
      ra.seg_slot = d_seg_slot.as<uint32_t>();
      ra.nseg = nseg;
      if (timers) {
        if (nseg == 0 && slot_cap > 0) {
          d_slot_seg.reserve(slot_cap * 4);
          SHD_HIP(hipMemsetAsync(d_slot_seg.p, 0xFF, slot_cap * 4, s));
        }
        ra.lanes_over_slots = 1;
        ra.slot_seg = d_slot_seg.as<int32_t>();
        ra.nlanes = nslots;
      } else {
        ra.lanes_over_slots = 0;
        ra.nlanes = nseg;
      }
    }
    ra.n_keyed = n_keyed;
    ra.run_id = d_run.as<uint32_t>();
    ra.state = state.as<char>();
    ensure_staging(std::max<int64_t>(1 << 16, 4 * n_keyed + 4 * (timers ? nslots : 0)));
    ra.R = R;
    ra.st_tag = st_tag.as<uint64_t>();
    ra.st_p = st_p.as<uint64_t>();
    ra.st_s = st_s.as<uint64_t>();
    ra.st_t = st_t.as<uint64_t>();
    ra.st_sidx = st_sidx.as<int32_t>();
    ra.st_ts = st_ts.as<int64_t>();
    ra.st_type = st_type.as<int32_t>();
    ra.st_vals = st_vals.as<uint64_t>();
    ra.st_nul = st_nul.as<uint8_t>();
    if (prog.multi_mask) ensure_lists(1 << 16);
    ra.LR = LR;
    ra.st_lv = st_lv.as<uint64_t>();
    ra.st_ln = st_ln.as<uint8_t>();
    ra.ctl = d_ctl.as<NfaCtl>();
    NfaCtl hc{};
    const NfaProg* dp = dev_args(prog);
    const NfaLayout* dl = dev_args(lay);
    if (win) {
      // window lanes; a failed verification reruns the push with doubled
      // warm-ups, down to the one-lane run once a warm-up spans most of it
      int64_t warm = std::max<int64_t>(win_warm, win_warm_hint(*b));
      for (;;) {
        if (4 * warm >= n) {
          win_one = true;
          break;
        }
        // lanes of >= 32 events, enough of them to fill the chip, and a
        // warm-up of at most 4 chunks
        int64_t chunk = std::max<int64_t>({32, std::min<int64_t>(1024, n / 16384), ceil_div(warm, 4)});
        if (const char* e = getenv("SHD_NFA_CHUNK")) chunk = std::max(1, atoi(e));
        const int64_t nl = ceil_div(n, chunk);
        const int64_t c0 = std::min<int64_t>(nl, warm / chunk + 1);   // lanes with ob <= warm
        ensure_slots(nl + 1);   // may move the key blocks
        ra.state = state.as<char>();
        d_hash.reserve(4 * nl * 8);
        ra.hash_w = d_hash.as<uint64_t>();
        ra.hash_e = d_hash.as<uint64_t>() + 2 * nl;
        ra.hash1_zero = getenv("SHD_NFA_HASH1_ZERO") != nullptr;
        ra.chunk_len = chunk;
        ra.warm = warm;
        ra.c_exact = c0;
        ra.nlanes = nl;
        ra.nseg = nl;
        lane_copy(0, 1, c0);
        SHD_HIP(hipMemsetAsync(d_ctl.p, 0, sizeof(NfaCtl), s));
        hipLaunchKernelGGL(k_nfa_run, dim3((unsigned)ceil_div(nl, kLaneBlock)), dim3(kLaneBlock), 0, s, dp, dl,
                           dev_args(ra));
        SHD_CHECK_LAUNCH();
        if (nl > c0)
          hipLaunchKernelGGL(k_win_check, dim3(grid_for(nl)), dim3(kBlock), 0, s, (const uint64_t*)ra.hash_w,
                             (const uint64_t*)ra.hash_e, c0, nl, &d_ctl.as<NfaCtl>()->count);
        hc = read_ctl();
        if (win_debug) {
          std::fprintf(stderr, "[shd nfa window] n=%lld warm=%lld chunk=%lld lanes=%lld exact=%lld bad=%u ovf=0x%x\n",
                       (long long)n, (long long)warm, (long long)chunk, (long long)nl, (long long)c0, hc.count,
                       hc.overflow);
#ifdef SHD_NFA_PROF
          std::fprintf(stderr, "[shd nfa prof] per lane-event clocks: gc %.0f rec %.0f stabilize %.0f process %.0f "
                       "emit %.0f hash/lane %.0f fire %.0f event %.0f\n",
                       hc.prof[0] / (double)(n + nl * warm), hc.prof[1] / (double)(n + nl * warm),
                       hc.prof[2] / (double)(n + nl * warm), hc.prof[3] / (double)(n + nl * warm),
                       hc.prof[4] / (double)(n + nl * warm), hc.prof[5] / (double)nl,
                       hc.prof[6] / (double)(n + nl * warm), hc.prof[7] / (double)(n + nl * warm));
#endif
        }
        if (hc.overflow || hc.count == 0) {
          if (!hc.overflow) lane_copy(nl, 0, 1);   // the last lane's end state is carried
          win_warm = warm;
          break;
        }
        win_fallbacks++;
        warm *= 2;
      }
      if (win_one) {
        ra.chunk_len = 0;
        ra.nlanes = 1;
        ra.nseg = 1;
      }
    }
    if (ra.nlanes > 0 && (!win || win_one)) {
      SHD_HIP(hipMemsetAsync(d_ctl.p, 0, sizeof(NfaCtl), s));
      hipLaunchKernelGGL(k_nfa_run, dim3((unsigned)ceil_div(ra.nlanes, kLaneBlock)), dim3(kLaneBlock), 0, s, dp, dl,
                         dev_args(ra));
      SHD_CHECK_LAUNCH();
      hc = read_ctl();
    }
    mark("nfa");
    if (hc.overflow || (int64_t)hc.rows > R) {
      char msg[320];
      std::snprintf(msg, sizeof msg,
                    "NFA per-key capacity exceeded (flags 0x%x; lists %d, partials %d, events %d, records %d, "
                    "timers %d, returned %d, rows %lld/%lld); raise SHD_NFA_LIST / SHD_NFA_PARTIALS / "
                    "SHD_NFA_EVENTS / SHD_NFA_RECORDS / SHD_NFA_TIMERS and reset the query",
                    hc.overflow, lay.L, lay.SC, lay.EC, lay.RC, lay.QC, lay.RETC, (long long)hc.rows, (long long)R);
      throw NfaOverflow(hc.overflow, (int64_t)hc.rows, msg, (int64_t)hc.lrows);
    }
    const int64_t m = (int64_t)hc.rows;
    if (m > 0) order_rows(m, partitioned || (win && !win_one), timers, n, (int64_t)hc.lrows);   // window lanes: merge by event order
    SHD_HIP(hipEventRecord(ev1, s));
    stage_end();
    SHD_HIP(hipEventSynchronize(ev1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    // host mirror of the playback clock: the last call's time
    int64_t last = now;
    SHD_HIP(hipMemcpyAsync(h_ctl.as<char>() + 128, d_now.as<int64_t>() + (ncalls - 1), 8, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    std::memcpy(&last, h_ctl.as<char>() + 128, 8);
    if (last > now) now = last;
    if (b) {
      seq += n;
      counters.events += n;
    }
    counters.matches += m;
    counters.partials += (int64_t)hc.partials;
    counters.partial_scans += (int64_t)hc.scans;
    counters.carry = (int64_t)hc.live;
    counters.kernel_ns = (int64_t)(ms * 1e6);
  }

  // staged rows -> reference order -> output arena
  void order_rows(int64_t m, bool sort, bool timers, int64_t n, int64_t nlist = 0) {
    hipStream_t s = stream;
    d_perm.reserve(m * 4);
    d_perm_alt.reserve(m * 4);
    d_thead.reserve(m * 4);
    d_thpos.reserve(m * 4);
    hipLaunchKernelGGL(k_iota_u32, dim3(grid_for(m)), dim3(kBlock), 0, s, d_perm.as<uint32_t>(), m);
    SHD_CHECK_LAUNCH();
    uint32_t* perm = d_perm.as<uint32_t>();
    if (sort) {
      d_skey.reserve(m * 8);
      d_skey_alt.reserve(m * 8);
      // stable LSD over (tertiary, secondary, primary): least significant field first
      const uint64_t pmax = 2 * (uint64_t)(seq + n) + 2;
      int pbits = 0;
      while (pbits < 64 && (pmax >> pbits)) pbits++;
      struct F {
        const uint64_t* k;
        int bits;
      };
      std::vector<F> fields;
      if (timers) {
        fields.push_back({st_t.as<uint64_t>(), 64});
        fields.push_back({st_s.as<uint64_t>(), 64});
      }
      fields.push_back({st_p.as<uint64_t>(), pbits});
      uint32_t* palt = d_perm_alt.as<uint32_t>();
      for (auto& f : fields) {
        hipLaunchKernelGGL(k_gather_keys, dim3(grid_for(m)), dim3(kBlock), 0, s, f.k, (const uint32_t*)perm, m,
                           d_skey.as<uint64_t>());
        SHD_CHECK_LAUNCH();
        bool in_alt = false;
        radix_sort_pairs_u64(d_skey.as<uint64_t>(), perm, d_skey_alt.as<uint64_t>(), palt, m, f.bits, d_sort, s,
                             in_alt);
        if (in_alt) std::swap(perm, palt);
      }
    }
    hipLaunchKernelGGL(k_tag_heads, dim3(grid_for(m)), dim3(kBlock), 0, s, (const uint64_t*)st_tag.as<uint64_t>(),
                       (const uint32_t*)perm, m, d_thead.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    scan_exclusive_u32(d_thead.as<uint32_t>(), d_thpos.as<uint32_t>(), m, nullptr, d_scan, s);
    out.ensure(m, s);
    const int64_t lbase = out.lcount;
    if (nlist > 0) {   // this push's list arena after the unpolled rows' lists
      out.ensure_list(nlist, s);
      SHD_HIP(hipMemcpyAsync(out.lvals.as<uint64_t>() + lbase, st_lv.p, (size_t)nlist * 8, hipMemcpyDeviceToDevice, s));
      SHD_HIP(hipMemcpyAsync(out.lnul.as<uint8_t>() + lbase, st_ln.p, (size_t)nlist, hipMemcpyDeviceToDevice, s));
      out.lcount += nlist;
    }
    hipLaunchKernelGGL(k_out_rows, dim3(grid_for(m)), dim3(kBlock), 0, s, (const uint32_t*)perm,
                       (const uint32_t*)d_thpos.as<uint32_t>(), (const uint32_t*)d_thead.as<uint32_t>(), m, prog.nout,
                       chunk_seq, out.count, (const int64_t*)st_ts.as<int64_t>(),
                       (const int32_t*)st_type.as<int32_t>(), (const uint64_t*)st_vals.as<uint64_t>(),
                       (const uint8_t*)st_nul.as<uint8_t>(), (const uint64_t*)st_p.as<uint64_t>(),
                       (const int32_t*)st_sidx.as<int32_t>(), out.d_chunk(), out.d_type(), out.d_ts(), out.d_vals(),
                       out.d_nulls(), out.d_seq(), out.d_sidx(), prog.multi_mask, lbase);
    SHD_CHECK_LAUNCH();
    // chunk ids consumed = number of distinct tags
    SHD_HIP(hipMemcpyAsync(h_ctl.as<char>() + 64, d_thpos.as<uint32_t>() + (m - 1), 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipMemcpyAsync(h_ctl.as<char>() + 68, d_thead.as<uint32_t>() + (m - 1), 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    uint32_t last_pos = 0, last_head = 0;
    std::memcpy(&last_pos, h_ctl.as<char>() + 64, 4);
    std::memcpy(&last_head, h_ctl.as<char>() + 68, 4);
    chunk_seq += (int64_t)last_pos + last_head;
    out.count += m;
    mark("order");
  }
};

std::unique_ptr<Engine> make_nfa_engine(const Plan& p, std::string& why) { return make_nfa_engine(p, why, 0); }

// Field offsets of a layout from its capacities (lane-interleaved blocks).
void layout_offsets(NfaLayout& Y) {
  Y.sew = (Y.SC + 1 + 63) / 64;
  Y.evw = (Y.EC + 1 + 63) / 64;
  Y.recw = (Y.RC + 1 + 63) / 64;
  // 64 key states interleaved per block; SHD_NFA_INTERLEAVE=0 keeps one key
  // state contiguous (measured slower on window lanes too: S4-seq 158 vs 182 M
  // events/s, S4P-seqplus 190 vs 199 M)
  Y.W = kLaneBlock;
  if (const char* w = getenv("SHD_NFA_INTERLEAVE")) Y.W = w[0] == '0' ? 1 : kLaneBlock;
  const int64_t falign = Y.W == 1 ? 16 : 256;
  int64_t off = 0;
  Y.nf = 0;
  auto field = [&](int64_t count, int sz) {
    int64_t o = off;
    off += (count * Y.W * sz + falign - 1) & ~(falign - 1);
    Y.f_off[Y.nf] = o;
    Y.f_cnt[Y.nf] = count;
    Y.f_sz[Y.nf] = sz;
    Y.nf++;
    return o;
  };
  Y.o_pend = field((int64_t)Y.npre * (Y.L + 1), 2);
  Y.o_pend_n = field(Y.npre, 2);
  Y.o_new = field((int64_t)Y.npre * (Y.L + 1), 2);
  Y.o_new_n = field(Y.npre, 2);
  Y.o_flags = field(Y.npre, 1);
  Y.o_lst = field(Y.npre, 8);
  Y.o_sq = field((int64_t)std::max(Y.nsched, 1) * Y.QC, 8);
  Y.o_sq_n = field(std::max(Y.nsched, 1), 2);
  Y.o_se_ev = field((int64_t)(Y.SC + 1) * Y.nstates, 2);
  Y.o_se_ts = field(Y.SC + 1, 8);
  Y.o_se_type = field(Y.SC + 1, 1);
  Y.o_se_free = field(Y.sew, 8);
  Y.o_se_mark = field(Y.sew, 8);
  Y.o_ev_rec = field(Y.EC + 1, 2);
  Y.o_ev_next = field(Y.EC + 1, 2);
  Y.o_ev_free = field(Y.evw, 8);
  Y.o_ev_mark = field(Y.evw, 8);
  Y.o_rec_ts = field(Y.RC + 1, 8);
  Y.o_rec_val = field((int64_t)(Y.RC + 1) * Y.ncols, 8);
  Y.o_rec_nul = field(Y.RC + 1, 4);
  Y.o_rec_free = field(Y.recw, 8);
  Y.o_rec_mark = field(Y.recw, 8);
  Y.o_ret = field(Y.RETC + 1, 2);
  Y.o_tmp = field(Y.RETC + 1, 2);
  Y.o_wk = field(Y.WK + 1, 4);
  Y.o_key = field(1, 8);
  Y.o_misc = field(MISC_N, 4);
  Y.o_cse = field(Y.SC + 1, 4);
  Y.o_cev = field(Y.EC + 1, 4);
  Y.blk = off;
}

std::unique_ptr<Engine> make_nfa_engine(const Plan& p, std::string& why, int64_t list_hint) {
  if (p.kind != SHD_KIND_STATE) {
    why = "not a state plan";
    return nullptr;
  }
  if (!p.aggs.empty() || !p.group_by.empty() || p.having >= 0) {
    why = "aggregating selector over a pattern";
    return nullptr;
  }
  if ((int)p.outputs.size() > kMaxCols) {
    why = "too many outputs";
    return nullptr;
  }
  if ((int)p.stream_types.size() > kNStream || p.n_states > kNS || p.n_states <= 0) {
    why = "too many streams / states";
    return nullptr;
  }
  for (auto& t : p.stream_types)
    if ((int)t.size() > kMaxCols) {
      why = "too many attributes";
      return nullptr;
    }
  GraphBuilder g(p);
  std::vector<int> preList;
  GraphBuilder::Res r = g.parse(p.root, -1, -1, true, preList);
  if (!g.err.empty()) {
    why = g.err;
    return nullptr;
  }
  const int npre = (int)g.pres.size();
  if (npre > kNP || (int)g.posts.size() != npre || g.n_sched > kNSched || (int)preList.size() > kNP) {
    why = "processor graph too large for the device NFA";
    return nullptr;
  }
  g.pres[r.first].thisLast = r.last;   // StateInputStreamParser.java:142-143
  std::vector<std::vector<int>> streamPres(p.stream_types.size());
  g.set_selector(r.rt);
  g.setup(r.rt, streamPres);
  std::vector<int> initSeq, resetSeq, updSeq;
  g.seq_init(r.rt, initSeq);
  g.seq_reset(r.rt, resetSeq);
  g.seq_update(r.rt, updSeq);
  if ((int)initSeq.size() > kNP || (int)resetSeq.size() > kNP || (int)updSeq.size() > kNP) {
    why = "processor graph too large for the device NFA";
    return nullptr;
  }
  for (auto& sp : streamPres)
    if ((int)sp.size() > kNP) {
      why = "processor graph too large for the device NFA";
      return nullptr;
    }

  auto e = std::make_unique<NfaEngine>();
  e->layout_hint = list_hint;   // recorded in snapshots (the restore rebuilds the same layout)
  NfaProg& P = e->prog;
  P.npre = npre;
  P.nstates = p.n_states;
  P.nsched = g.n_sched;
  P.seq = p.state_type == 1;
  P.within = p.within >= 0 ? p.within : -1;
  P.nstart = 0;
  if (p.within >= 0)
    for (int x : preList)
      if (g.pres[x].isStart && P.nstart < kNP) P.startIds[P.nstart++] = g.pres[x].stateId;
  for (int i = 0; i < npre; i++) {
    const HPre& h = g.pres[i];
    DPre& d = P.pre[i];
    if (h.filters.size() > 4) {
      why = "more than 4 filters on one state";
      return nullptr;
    }
    if (h.stateId < 0 || h.stateId >= p.n_states || h.thisPost < 0 || h.stream < 0 ||
        h.stream >= (int)p.stream_types.size()) {
      why = "inconsistent processor graph";
      return nullptr;
    }
    d.kind = h.kind;
    d.stateId = h.stateId;
    d.isStart = h.isStart;
    d.stream = h.stream;
    d.thisPost = h.thisPost;
    d.thisLast = h.thisLast;
    d.withinEvery = h.withinEvery;
    d.partner = h.partner;
    d.sched = h.sched;
    d.minC = h.minC;
    d.maxC = h.maxC;
    d.ltype = h.ltype;
    d.waiting = h.waiting;
    e->pre_filters.push_back(h.filters);
    const HPost& hp = g.posts[i];
    DPost& q = P.post[i];
    q.kind = hp.kind;
    q.pre = hp.pre;
    q.stateId = hp.stateId;
    q.nextPre = hp.nextPre;
    q.nextEvery = hp.nextEvery;
    q.callbackPre = hp.callbackPre;
    q.partnerPre = hp.partnerPre;
    q.partnerPost = hp.partnerPost;
    q.minC = hp.minC;
    q.maxC = hp.maxC;
    q.ltype = hp.ltype;
    q.hasSelector = hp.hasSelector;
  }
  P.nall = (int)preList.size();
  for (int i = 0; i < P.nall; i++) P.allPre[i] = preList[i];
  P.ninit = (int)initSeq.size();
  for (int i = 0; i < P.ninit; i++) P.initSeq[i] = initSeq[i];
  P.nreset = (int)resetSeq.size();
  for (int i = 0; i < P.nreset; i++) P.resetSeq[i] = resetSeq[i];
  P.nupd = (int)updSeq.size();
  for (int i = 0; i < P.nupd; i++) P.updSeq[i] = updSeq[i];
  for (size_t s = 0; s < streamPres.size(); s++) {
    P.nsp[s] = (int)streamPres[s].size();
    for (size_t k = 0; k < streamPres[s].size(); k++) P.streamPres[s][k] = streamPres[s][k];
  }
  for (int i = 0; i < g.n_sched; i++) P.schedPre[i] = g.sched_pre[i];
  P.current_on = p.current_on;
  P.expired_on = p.expired_on;
  P.nout = (int)p.outputs.size();
  P.multi_mask = 0;
  for (int c = 0; c < P.nout && c < 32; c++) {
    const auto& code = p.exprs[p.outputs[c].second];
    if (code.size() == 1 && code[0].op == SHD_OP_MULTI) P.multi_mask |= 1u << c;
  }

  // partition keys (ValuePartitionExecutor: one key class per query)
  e->partitioned = !p.part_keys.empty();
  for (int s = 0; s < kNStream; s++) {
    e->key_expr[s] = -1;
    e->key_col[s] = -1;
    e->key_type[s] = 0;
  }
  if (e->partitioned) {
    int cls = -1;
    for (auto& pk : p.part_keys) {
      if (pk.first < 0 || pk.first >= (int)p.stream_types.size()) continue;
      int t = expr_result_type(p, pk.second, {});
      int c = (t == SHD_T_INT || t == SHD_T_LONG) ? 1 : (t == SHD_T_FLOAT || t == SHD_T_DOUBLE) ? 2 : t + 10;
      if (cls >= 0 && c != cls) {
        why = "partition keys of different types";
        return nullptr;
      }
      cls = c;
      e->key_expr[pk.first] = pk.second;
      auto& code = p.exprs[pk.second];
      e->key_col[pk.first] = (code.size() == 1 && code[0].op == SHD_OP_LOAD) ? (code[0].c & 0xFFFF) : -1;
      e->key_type[pk.first] = t;
    }
    for (size_t s = 0; s < p.stream_types.size(); s++)
      if (P.nsp[s] > 0 && e->key_expr[s] < 0) {
        why = "partition key missing for a stream";
        return nullptr;
      }
  }

  // window lanes: unpartitioned, every-started, and partials bounded -- a
  // sequence (a partial survives an event only by advancing on it) or a
  // pattern with `within` / `for` times; the span / horizon sizes the warm-up
  {
    std::function<int64_t(const PNode&)> span = [&](const PNode& n) -> int64_t {
      switch (n.kind) {
        case SHD_NODE_STREAM: return n.absent ? -1 : 1;
        case SHD_NODE_NEXT: {
          const int64_t x = span(n.kids[0]), y = span(n.kids[1]);
          return x < 0 || y < 0 ? -1 : x + y;
        }
        case SHD_NODE_EVERY: return span(n.kids[0]);
        case SHD_NODE_LOGICAL: return n.kids[0].absent || n.kids[1].absent ? -1 : 2;
        case SHD_NODE_COUNT: return n.max < 0 ? -1 : n.max;
      }
      return -1;
    };
    bool every_start = false;
    for (int i = 0; i < npre; i++)
      if (g.pres[i].isStart && g.posts[g.pres[i].thisPost].nextEvery >= 0) every_start = true;
    // (an absent operand of `and` / `or` keeps partials past its time: not bounded)
    int64_t horizon = std::max<int64_t>(P.within, 0);
    bool absent_logical = false;
    for (int i = 0; i < npre; i++) {
      if (P.pre[i].waiting > 0) horizon = std::max<int64_t>(horizon, P.pre[i].waiting);
      if (P.pre[i].kind == PK_ABSENT_LOGICAL) absent_logical = true;
    }
    if (absent_logical && !(p.state_type == 1)) horizon = 0;
    const bool seq = p.state_type == 1;
    const char* wenv = getenv("SHD_NFA_WINDOW");
    if (!e->partitioned && every_start && (seq || horizon > 0) && !(wenv && wenv[0] == '0') && list_hint == 0) {
      e->windowed = true;
      const int64_t sp = span(p.root);
      e->win_span = seq && sp > 0 ? sp : 0;
      e->win_horizon = seq ? 0 : horizon;
    }
  }

  // per-key capacities: one key (unpartitioned) gets deep lists, many keys get lean blocks
  NfaLayout& Y = e->lay;
  const bool many = e->partitioned;
  // list_hint (a pattern query handing its open partials over): the one key of
  // an unpartitioned plan must hold about that many partials at once (window
  // lanes too: each holds the one key's whole state; sequence lanes less)
  int L0 = many ? 32 : 2048, S0 = many ? 128 : 8192;
  if (e->windowed && e->win_horizon == 0) {   // sequence lanes: partials die unless they advance
    L0 = 128;
    S0 = 512;
  }
  if (!many && list_hint > 0) {
    while (L0 < 2 * list_hint && L0 < 32768) L0 *= 2;
    S0 = std::max(S0, std::min(2 * L0, 32768));
  }
  Y.L = env_int("SHD_NFA_LIST", L0);
  Y.SC = std::min(env_int("SHD_NFA_PARTIALS", S0), 32768);
  Y.EC = std::min(env_int("SHD_NFA_EVENTS", 2 * Y.SC), 65000);
  Y.RC = std::min(env_int("SHD_NFA_RECORDS", S0), 65000);
  Y.QC = env_int("SHD_NFA_TIMERS", many ? 32 : 1024);
  Y.RETC = std::min(Y.L * std::max(npre, 1), 65000);
  Y.WK = 4 * kNP;
  if (Y.L >= 65000 || Y.QC >= 65000) {
    why = "NFA list capacities must stay below 65000";
    return nullptr;
  }
  Y.ncols = 1;
  for (auto& t : p.stream_types) Y.ncols = std::max<int>(Y.ncols, (int)t.size());
  Y.nstates = p.n_states;
  Y.npre = npre;
  Y.nsched = g.n_sched;
  layout_offsets(Y);
  return e;
}

}  // namespace shd
