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
// detected on device and rejected (SHD_E_UNSUPPORTED), never approximated.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "engine.h"

namespace shd {

namespace {

enum : uint8_t { F_CAND = 1, F_NEW = 2, F_B = 4, F_SKIP = 8 };
enum : uint8_t { ST_OPEN = 0, ST_DEAD = 1, ST_MATCH = 2 };

// Row addressing over the extended batch: rows [0, C) are carried partials
// (stream A columns), rows [C, C+n) are the pushed batch.
struct ExtRows {
  ColSet carry;   // stream A schema
  ColSet batch;   // pushed stream schema
  int64_t C;
  int64_t seq0;           // global seq of batch row 0
  const int64_t* carry_seq;
  __device__ __forceinline__ const ColSet& cs(int64_t r) const { return r < C ? carry : batch; }
  __device__ __forceinline__ int64_t row(int64_t r) const { return r < C ? r : r - C; }
  __device__ __forceinline__ int64_t ts(int64_t r) const {
#ifdef SHD_DEBUG
    if (r < 0 || r >= C + batch.n) {
      printf("SHD_DEBUG ExtRows.ts: row %lld C %lld n %lld\n", (long long)r, (long long)C, (long long)batch.n);
      return 0;
    }
#endif
    return r < C ? carry.ts[r] : batch.ts[r - C];
  }
  __device__ __forceinline__ int64_t seq(int64_t r) const { return r < C ? carry_seq[r] : seq0 + (r - C); }
};

// Expression context over (e1 row, e2 row); stream-state chains hold one event.
struct PairCtx {
  const ExtRows* x;
  int64_t r1, r2;   // ext rows of state 0 / state 1 (-1 = empty slot)
  __device__ __forceinline__ int64_t slot(int st, int idx) const {
    int64_t r = st == 0 ? r1 : (st == 1 ? r2 : -1);
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
    return col_load(x->cs(r), x->row(r), attr);
  }
  __device__ __forceinline__ bool evnull(int st, int idx) const { return slot(st, idx) < 0; }
  __device__ __forceinline__ int64_t ts(int st, int idx) const {
    int64_t r = slot(st, idx);
    return r < 0 ? 0 : x->ts(r);
  }
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

struct PrepArgs {
  ExtRows x;
  DExprSet es;
  DFilters f1;
  int is_a, is_b;           // pushed stream plays A and/or B
  int partitioned;
  DExpr key_carry_unused;
  DExpr key_expr;           // key expression of the pushed stream
  int key_type;
  int key_col;              // >= 0: plain attribute key of the pushed stream
  const uint64_t* carry_key;
};

// Per extended row: key, flags (candidate / new / B / skip).
__global__ __launch_bounds__(kBlock) void k_prepare(const PrepArgs* __restrict__ ap, int64_t n_ext, uint64_t* key, uint8_t* flags,
                                                    unsigned long long* n_new_cand) {
  const PrepArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  uint64_t created = 0;
  // kernel arguments live in the read-only kernarg segment: work on a private
  // copy before taking addresses
  const ExtRows& x = a.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_ext; r += (int64_t)gridDim.x * blockDim.x) {
    if (r < x.C) {
      key[r] = a.partitioned ? a.carry_key[r] : 0;
      flags[r] = F_CAND;
      continue;
    }
    PairCtx cx{&x, r, -1};
    uint8_t f = F_NEW;
    uint64_t k = 0;
    if (a.partitioned) {
      Val kv;
      if (a.key_col >= 0) kv = col_load(x.batch, r - x.C, a.key_col);
      else kv = eval_expr(a.es.ins + a.key_expr.off, a.key_expr.len, a.es.consts, cx);
      if (kv.null) f |= F_SKIP;   // PartitionStreamReceiver drops null keys
      k = canon_key(kv, a.key_type);
    }
    if (!(f & F_SKIP)) {
      if (a.is_b) f |= F_B;
      if (a.is_a && eval_filters(a.es, a.f1, cx)) {
        f |= F_CAND;
        created++;
      }
    }
    key[r] = k;
    flags[r] = f;
  }
  for (int o = 32; o > 0; o >>= 1) created += __shfl_xor(created, o, 64);
  if ((threadIdx.x & 63) == 0 && created) atomicAdd(n_new_cand, (unsigned long long)created);
}


// ---- fault bisection variants (SHD_PROBE=variants): same loop as k_prepare
// with progressively more of the expression machinery switched on.
struct ConstCtx {
  __device__ __forceinline__ Val load(int, int, int) const { Val v; v.b = 0x42c80000u; v.null = 0; return v; }
  __device__ __forceinline__ bool evnull(int, int) const { return false; }
  __device__ __forceinline__ int64_t ts(int, int) const { return 0; }
  __device__ __forceinline__ Val agg(int) const { Val v; v.b = 0; v.null = 1; return v; }
};
struct RawCtx {
  const ExtRows* x;
  int64_t r1;
  __device__ __forceinline__ Val load(int st, int idx, int attr) const {
    Val v; v.b = 0; v.null = 1;
    if (st != 0 || (unsigned)attr >= (unsigned)x->batch.ncols) return v;
    v.null = 0;
    v.b = ((const uint32_t*)x->batch.col[attr])[r1 - x->C];
    return v;
  }
  __device__ __forceinline__ bool evnull(int, int) const { return false; }
  __device__ __forceinline__ int64_t ts(int, int) const { return 0; }
  __device__ __forceinline__ Val agg(int) const { Val v; v.b = 0; v.null = 1; return v; }
};
template <int V>
__global__ __launch_bounds__(kBlock) void k_prepare_v(const PrepArgs* __restrict__ ap, int64_t n_ext, uint64_t* key, uint8_t* flags,
                                                      unsigned long long* n_new_cand) {
  const PrepArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  uint64_t created = 0;
  const ExtRows& x = a.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_ext; r += (int64_t)gridDim.x * blockDim.x) {
    if (r < x.C) { key[r] = 0; flags[r] = F_CAND; continue; }
    uint8_t f = F_NEW;
    bool pass = false;
    if (V == 0) pass = a.is_a;
    if (V == 1) { ConstCtx c; pass = a.is_a && eval_filters(a.es, a.f1, c); }
    if (V == 2) { RawCtx c{&x, r}; pass = a.is_a && eval_filters(a.es, a.f1, c); }
    if (V == 3) { PairCtx c{&x, r, -1}; pass = a.is_a && eval_filters(a.es, a.f1, c); }
    if (V == 4) { PairCtx c{&x, r, -1}; Val v = c.load(0, -1, 1); pass = a.is_a && !v.null && v.b != 0; }
    if (pass) { f |= F_CAND; created++; }
    key[r] = 0;
    flags[r] = f;
  }
  for (int o = 32; o > 0; o >>= 1) created += __shfl_xor(created, o, 64);
  if ((threadIdx.x & 63) == 0 && created) atomicAdd(n_new_cand, (unsigned long long)created);
}

// Diagnostic (SHD_PROBE env): print the kernel's view of its arguments without
// dereferencing any column pointer (stage 1), then the bytecode (stage 2).
__global__ void k_probe(const PrepArgs* __restrict__ ap, int64_t n_ext, int stage) {
  const PrepArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (stage == 1) {
    printf("probe dev: n_ext %lld C %lld ncols %d ts %p is_a %d is_b %d part %d key_col %d f1.n %d ins %p consts %p\n",
           (long long)n_ext, (long long)a.x.C, a.x.batch.ncols, (const void*)a.x.batch.ts, a.is_a, a.is_b,
           a.partitioned, a.key_col, a.f1.n, (const void*)a.es.ins, (const void*)a.es.consts);
    for (int c = 0; c < a.x.batch.ncols && c < kMaxCols; c++)
      printf("probe dev: col %d %p nul %p type %d\n", c, a.x.batch.col[c], (const void*)a.x.batch.nul[c],
             (int)a.x.batch.type[c]);
    for (int i = 0; i < a.f1.n && i < 4; i++) printf("probe dev: f1[%d] off %d len %d\n", i, a.f1.f[i].off, a.f1.f[i].len);
  } else {
    auto sane = [](const void* q) { return q != nullptr && ((uintptr_t)q >> 47) == 0; };
    if (!sane(a.es.ins) || !sane(a.x.batch.ts)) { printf("probe dev: insane pointer, skipping loads\n"); return; }
    for (int i = 0; i < a.f1.n && i < 4; i++)
      for (int k = 0; k < a.f1.f[i].len && k < 16; k++) {
        int4 in = a.es.ins[a.f1.f[i].off + k];
        printf("probe dev: f1[%d][%d] op %d a %d b %d c %d\n", i, k, in.x, in.y, in.z, in.w);
      }
    if (n_ext > a.x.C) printf("probe dev: ts[0] %lld\n", (long long)a.x.batch.ts[0]);
  }
}

__global__ void k_narrow_keys(const uint64_t* in, uint32_t* out, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = (uint32_t)in[i];
}

struct ScanArgs {
  ExtRows x;
  DExprSet es;
  DFilters f2;
  int64_t within;
  int partitioned;
};

// One lane per candidate partial: forward walk over the later events of its key.
__global__ __launch_bounds__(kBlock) void k_forward_scan(const ScanArgs* __restrict__ ap, int64_t n_ext, const uint32_t* perm,
                                                         const uint64_t* key, const uint8_t* flags,
                                                         int32_t* match_j, uint8_t* status,
                                                         unsigned long long* steps_total, uint32_t* violation) {
  const ScanArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  uint64_t steps = 0;
  const ExtRows& x = a.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n_ext;
       p += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = perm ? (int64_t)perm[p] : p;
    uint8_t fr = flags[r];
    if (!(fr & F_CAND)) continue;
    uint64_t k = key[r];
    int64_t tsi = x.ts(r);
    int64_t prev = tsi;
    uint8_t st = ST_OPEN;
    int32_t j = -1;
    for (int64_t q = p + 1; q < n_ext; q++) {
      int64_t r2 = perm ? (int64_t)perm[q] : q;
      if (a.partitioned && key[r2] != k) break;
      uint8_t f2 = flags[r2];
      if (!(f2 & F_NEW) || (f2 & F_SKIP)) continue;
      int64_t t2 = x.ts(r2);
      if (t2 < prev) {
        atomicOr(violation, 1u);
        break;
      }
      prev = t2;
      steps++;
      // stabilizeStates -> expireEvents: |ts_i - t| > within
      if (t2 - tsi > a.within) {
        st = ST_DEAD;
        break;
      }
      if (f2 & F_B) {
        PairCtx cx{&x, r, r2};
        if (eval_filters(a.es, a.f2, cx)) {
          st = ST_MATCH;
          j = (int32_t)r2;
          break;
        }
      }
    }
    match_j[r] = j;
    status[r] = st;
  }
  // one atomic per wave
  for (int o = 32; o > 0; o >>= 1) steps += __shfl_xor(steps, o, 64);
  if ((threadIdx.x & 63) == 0 && steps) atomicAdd(steps_total, (unsigned long long)steps);
}

// counts for compaction: matches and still-open partials, in ext (= creation) order
__global__ void k_flags_to_counts(const uint8_t* flags, const uint8_t* status, int64_t n, uint32_t* cm,
                                  uint32_t* co) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    bool c = flags[r] & F_CAND;
    cm[r] = (c && status[r] == ST_MATCH) ? 1u : 0u;
    co[r] = (c && status[r] == ST_OPEN) ? 1u : 0u;
  }
}

__global__ void k_emit_pairs(const uint32_t* cm, const uint32_t* om, const int32_t* match_j, int64_t n,
                             uint32_t* pj, uint32_t* pi) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (cm[r]) {
      uint32_t o = om[r];
      pj[o] = (uint32_t)match_j[r];
      pi[o] = (uint32_t)r;
    }
  }
}

struct ProjArgs {
  ExtRows x;
  DExprSet es;
  DExpr outs[kMaxCols];
  int nout;
  int multi;            // chunk per e2 event (same stream) vs per match
  int64_t chunk0;
  int64_t row0;         // output buffer offset
};

__global__ __launch_bounds__(kBlock) void k_project(const ProjArgs* __restrict__ ap, const uint32_t* pj, const uint32_t* pi, int64_t m,
                                                    int64_t* o_chunk, int32_t* o_type, int64_t* o_ts,
                                                    uint64_t* o_vals, uint8_t* o_nul) {
  const ProjArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  const ExtRows& x = a.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += (int64_t)gridDim.x * blockDim.x) {
    int64_t j = pj[k], i = pi[k];
    PairCtx cx{&x, i, j};
    int64_t row = a.row0 + k;
    for (int c = 0; c < a.nout; c++) {
      Val v = eval_expr(a.es.ins + a.outs[c].off, a.outs[c].len, a.es.consts, cx);
      o_vals[row * a.nout + c] = v.b;
      o_nul[row * a.nout + c] = (uint8_t)v.null;
    }
    o_ts[row] = x.ts(j);
    o_type[row] = 0;
    o_chunk[row] = a.multi ? x.seq(j) : a.chunk0 + k;
  }
}

struct GatherArgs {
  ExtRows x;
  int ncols;
  int8_t types[kMaxCols];
  void* dcol[kMaxCols];
  uint8_t* dnul[kMaxCols];
  int64_t* dts;
  uint64_t* dkey;
  int64_t* dseq;
};

__global__ void k_gather_carry(const GatherArgs* __restrict__ ap, const uint32_t* co, const uint32_t* oo, const uint64_t* key, int64_t n) {
  const GatherArgs& a = *ap;   // args live in device memory (Engine::dev_args)
  const ExtRows& x = a.x;
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (int64_t)gridDim.x * blockDim.x) {
    if (!co[r]) continue;
    int64_t o = oo[r];
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
    a.dkey[o] = key[r];
    a.dseq[o] = x.seq(r);
  }
}

struct CarryTable {
  DevBuf col[kMaxCols], nul[kMaxCols], ts, key, seq;
  void reserve(int64_t n, const std::vector<int>& types) {
    for (size_t c = 0; c < types.size(); c++) {
      col[c].reserve(std::max<int64_t>(n, 1) * type_size(types[c]));
      nul[c].reserve(std::max<int64_t>(n, 1));
    }
    ts.reserve(std::max<int64_t>(n, 1) * 8);
    key.reserve(std::max<int64_t>(n, 1) * 8);
    seq.reserve(std::max<int64_t>(n, 1) * 8);
  }
  ColSet colset(const std::vector<int>& types) const {
    ColSet cs{};
    cs.ncols = (int)types.size();
    for (size_t c = 0; c < types.size(); c++) {
      cs.col[c] = col[c].p;
      cs.nul[c] = nul[c].as<uint8_t>();
      cs.type[c] = (int8_t)types[c];
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

int key_class(int t) {
  switch (t) {
    case SHD_T_INT: case SHD_T_LONG: return 1;
    case SHD_T_FLOAT: case SHD_T_DOUBLE: return 2;
    case SHD_T_BOOL: return 3;
  }
  return 4;
}

}  // namespace

struct PatternEngine : Engine {
  int sA = 0, sB = 0;
  std::vector<int> f1, f2;
  int64_t W = INT64_MAX;
  bool partitioned = false;
  int key_expr[2] = {-1, -1}, key_col[2] = {-1, -1}, key_type[2] = {0, 0};
  std::vector<int> outs;
  std::vector<int> typesA;
  CarryTable carry[2];
  int cur = 0;
  int64_t C = 0;
  // scratch
  DevBuf d_key, d_flags, d_perm, d_perm_alt, d_k32, d_k32_alt, d_k64_alt, d_match, d_status, d_cm, d_co, d_om,
      d_oo, d_pj, d_pi, d_pj_alt, d_pi_alt, d_tot, d_sort, d_scan;
  PinnedBuf h_tot;

  int kind() const override { return ENG_PATTERN; }

  void reset() override {
    C = 0;
    seq = 0;
    now = INT64_MIN;
    chunk_seq = 0;
    out.count = 0;
    counters = shd_counters{};
  }

  ColSet carry_cs() const {
    ColSet cs = carry[cur].colset(typesA);
    cs.n = C;
    return cs;
  }

  void push(const Staged& b) override {
    if (b.advance_time) {
      for (size_t c = 0; c + 1 < b.call_offsets.size(); c++) {
        // last ts of each call: time only matters for expiry (event ts), kept for set_time parity
      }
    }
    const int64_t n = b.n;
    if (n <= 0) return;
    const bool isA = b.stream == sA, isB = b.stream == sB;
    const int64_t n_ext = C + n;
    if (n_ext >= (int64_t)INT32_MAX) throw Error(SHD_E_CAPACITY, "pattern batch + carry exceeds 2^31 rows");
    hipStream_t s = stream;
    SHD_HIP(hipEventRecord(ev0, s));
    stage_begin();
    d_key.reserve(n_ext * 8);
    d_flags.reserve(n_ext);
    d_match.reserve(n_ext * 4);
    d_status.reserve(n_ext);
    d_cm.reserve(n_ext * 4);
    d_co.reserve(n_ext * 4);
    d_om.reserve(n_ext * 4);
    d_oo.reserve(n_ext * 4);
    d_tot.reserve(64);
    h_tot.reserve(64);

    ExtRows x{};
    x.carry = carry_cs();
    x.batch = b.cs;
    x.C = C;
    x.seq0 = seq;
    x.carry_seq = carry[cur].seq.as<int64_t>();

    PrepArgs pa{};
    pa.x = x;
    pa.es = dset();
    pa.f1 = dfilters(f1);
    pa.is_a = isA;
    pa.is_b = isB;
    pa.partitioned = partitioned;
    int slot = isA ? 0 : 1;
    if (partitioned) {
      pa.key_expr = dexpr(key_expr[slot]);
      pa.key_col = key_col[slot];
      pa.key_type = key_type[slot];
    } else {
      pa.key_col = -1;
    }
    pa.carry_key = carry[cur].key.as<uint64_t>();
    SHD_HIP(hipMemsetAsync(d_tot.p, 0, 64, s));
    if (const char* pr = std::getenv("SHD_PROBE")) {
      fprintf(stderr, "probe host: n_ext %lld C %lld ncols %d ts %p is_a %d f1.n %d ins %p consts %p sizeof(PrepArgs) %zu\n",
              (long long)n_ext, (long long)pa.x.C, pa.x.batch.ncols, (const void*)pa.x.batch.ts, pa.is_a, pa.f1.n,
              (const void*)pa.es.ins, (const void*)pa.es.consts, sizeof(PrepArgs));
      for (int c = 0; c < pa.x.batch.ncols; c++)
        fprintf(stderr, "probe host: col %d %p nul %p type %d\n", c, pa.x.batch.col[c], (const void*)pa.x.batch.nul[c],
                (int)pa.x.batch.type[c]);
      SHD_HIP(hipStreamSynchronize(s));
      hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s, dev_args(pa), n_ext, 1);
      SHD_HIP(hipStreamSynchronize(s));
      hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s, dev_args(pa), n_ext, 2);
      SHD_HIP(hipStreamSynchronize(s));
      fflush(stdout);
      if (pr[0] == 'v') {
        auto chk = [&](int v) {
          SHD_HIP(hipStreamSynchronize(s));
          fprintf(stderr, "probe: variant %d ok\n", v);
          fflush(stderr);
        };
        unsigned long long* nc = (unsigned long long*)(d_tot.as<uint64_t>() + 6);
        hipLaunchKernelGGL(k_prepare_v<0>, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(pa), n_ext, d_key.as<uint64_t>(), d_flags.as<uint8_t>(), nc);
        chk(0);
        hipLaunchKernelGGL(k_prepare_v<1>, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(pa), n_ext, d_key.as<uint64_t>(), d_flags.as<uint8_t>(), nc);
        chk(1);
        hipLaunchKernelGGL(k_prepare_v<2>, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(pa), n_ext, d_key.as<uint64_t>(), d_flags.as<uint8_t>(), nc);
        chk(2);
        hipLaunchKernelGGL(k_prepare_v<4>, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(pa), n_ext, d_key.as<uint64_t>(), d_flags.as<uint8_t>(), nc);
        chk(4);
        hipLaunchKernelGGL(k_prepare_v<3>, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(pa), n_ext, d_key.as<uint64_t>(), d_flags.as<uint8_t>(), nc);
        chk(3);
        throw Error(SHD_E_UNSUPPORTED, "SHD_PROBE: variants done");
      }
      if (pr[0] != 'r') throw Error(SHD_E_UNSUPPORTED, "SHD_PROBE: stopped before k_prepare");
    }
    hipLaunchKernelGGL(k_prepare, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(pa), n_ext, d_key.as<uint64_t>(),
                       d_flags.as<uint8_t>(), (unsigned long long*)(d_tot.as<uint64_t>() + 6));
    SHD_CHECK_LAUNCH();
    mark("prepare");

    // ---- key-sort the extended batch (stable: creation order within a key)
    const uint32_t* perm = nullptr;
    if (partitioned) {
      uint64_t* dmax = d_tot.as<uint64_t>() + 4;
      reduce_max_u64(d_key.as<uint64_t>(), n_ext, dmax, s);
      SHD_HIP(hipMemcpyAsync(h_tot.as<uint64_t>() + 4, dmax, 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
      uint64_t kmax = h_tot.as<uint64_t>()[4];
      int bits = 0;
      while (bits < 64 && (kmax >> bits)) bits++;
      d_perm.reserve(n_ext * 4);
      d_perm_alt.reserve(n_ext * 4);
      fill_iota_u32(d_perm.as<uint32_t>(), n_ext, 0, s);
      bool in_alt = false;
      if (bits <= 32) {
        d_k32.reserve(n_ext * 4);
        d_k32_alt.reserve(n_ext * 4);
        hipLaunchKernelGGL(k_narrow_keys, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, d_key.as<uint64_t>(),
                           d_k32.as<uint32_t>(), n_ext);
        SHD_CHECK_LAUNCH();
        radix_sort_pairs_u32(d_k32.as<uint32_t>(), d_perm.as<uint32_t>(), d_k32_alt.as<uint32_t>(),
                             d_perm_alt.as<uint32_t>(), n_ext, bits, d_sort, s, in_alt);
      } else {
        d_k64_alt.reserve(n_ext * 8);
        DevBuf k64;
        k64.reserve(n_ext * 8);
        SHD_HIP(hipMemcpyAsync(k64.p, d_key.p, n_ext * 8, hipMemcpyDeviceToDevice, s));
        radix_sort_pairs_u64(k64.as<uint64_t>(), d_perm.as<uint32_t>(), d_k64_alt.as<uint64_t>(),
                             d_perm_alt.as<uint32_t>(), n_ext, bits, d_sort, s, in_alt);
        SHD_HIP(hipStreamSynchronize(s));
      }
      perm = in_alt ? d_perm_alt.as<uint32_t>() : d_perm.as<uint32_t>();
      mark("key_sort");
    }

    // ---- forward scan, one lane per candidate partial
    SHD_HIP(hipMemsetAsync(d_tot.p, 0, 32, s));   // keeps the candidate count at word 6
    ScanArgs sa{};
    sa.x = x;
    sa.es = dset();
    sa.f2 = dfilters(f2);
    sa.within = W;
    sa.partitioned = partitioned;
    unsigned long long* d_steps = (unsigned long long*)d_tot.as<uint64_t>();
    uint32_t* d_viol = (uint32_t*)(d_tot.as<uint64_t>() + 1);
    hipLaunchKernelGGL(k_forward_scan, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(sa), n_ext, perm,
                       (const uint64_t*)d_key.as<uint64_t>(), (const uint8_t*)d_flags.as<uint8_t>(),
                       d_match.as<int32_t>(), d_status.as<uint8_t>(), d_steps, d_viol);
    SHD_CHECK_LAUNCH();
    mark("forward_scan");

    // ---- compaction offsets for matches (ordered by creation) and open partials
    hipLaunchKernelGGL(k_flags_to_counts, dim3(grid_for(n_ext)), dim3(kBlock), 0, s,
                       (const uint8_t*)d_flags.as<uint8_t>(), (const uint8_t*)d_status.as<uint8_t>(), n_ext,
                       d_cm.as<uint32_t>(), d_co.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    uint32_t* d_m = (uint32_t*)(d_tot.as<uint64_t>() + 2);
    uint32_t* d_o = d_m + 1;
    scan_exclusive_u32(d_cm.as<uint32_t>(), d_om.as<uint32_t>(), n_ext, d_m, d_scan, s);
    scan_exclusive_u32(d_co.as<uint32_t>(), d_oo.as<uint32_t>(), n_ext, d_o, d_scan, s);
    mark("compact");
    SHD_HIP(hipMemcpyAsync(h_tot.p, d_tot.p, 56, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    uint64_t steps = h_tot.as<uint64_t>()[0];
    counters.partials += (int64_t)h_tot.as<uint64_t>()[6];
    uint32_t viol = (uint32_t)h_tot.as<uint64_t>()[1];
    uint32_t m = h_tot.as<uint32_t>()[4];
    uint32_t n_open = h_tot.as<uint32_t>()[5];
    if (viol)
      throw Error(SHD_E_UNSUPPORTED,
                  "pattern engine: event timestamps decrease within a key; the forward-scan formulation "
                  "requires per-key non-decreasing timestamps");

    // ---- matches ordered by (e2 event, creation) -> projected output rows
    if (m > 0) {
      d_pj.reserve((int64_t)m * 4);
      d_pi.reserve((int64_t)m * 4);
      d_pj_alt.reserve((int64_t)m * 4);
      d_pi_alt.reserve((int64_t)m * 4);
      hipLaunchKernelGGL(k_emit_pairs, dim3(grid_for(n_ext)), dim3(kBlock), 0, s,
                         (const uint32_t*)d_cm.as<uint32_t>(), (const uint32_t*)d_om.as<uint32_t>(),
                         (const int32_t*)d_match.as<int32_t>(), n_ext, d_pj.as<uint32_t>(), d_pi.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      int bits = 0;
      while (bits < 32 && ((uint64_t)n_ext >> bits)) bits++;
      bool in_alt = false;
      radix_sort_pairs_u32(d_pj.as<uint32_t>(), d_pi.as<uint32_t>(), d_pj_alt.as<uint32_t>(),
                           d_pi_alt.as<uint32_t>(), m, bits, d_sort, s, in_alt);
      const uint32_t* pj = in_alt ? d_pj_alt.as<uint32_t>() : d_pj.as<uint32_t>();
      const uint32_t* pi = in_alt ? d_pi_alt.as<uint32_t>() : d_pi.as<uint32_t>();
      out.ensure(m, s);
      ProjArgs pr{};
      pr.x = x;
      pr.es = dset();
      pr.nout = (int)outs.size();
      for (size_t c = 0; c < outs.size(); c++) pr.outs[c] = dexpr(outs[c]);
      pr.multi = (sA == sB);
      pr.chunk0 = chunk_seq;
      pr.row0 = out.count;
      hipLaunchKernelGGL(k_project, dim3(grid_for(m)), dim3(kBlock), 0, s, dev_args(pr), pj, pi, (int64_t)m, out.d_chunk(),
                         out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls());
      SHD_CHECK_LAUNCH();
      out.count += m;
      if (sA != sB) chunk_seq += m;
      mark("order_project");
    }

    // ---- carry the still-open partials (in creation order)
    int nxt = cur ^ 1;
    carry[nxt].reserve(n_open, typesA);
    if (n_open > 0) {
      GatherArgs ga{};
      ga.x = x;
      ga.ncols = (int)typesA.size();
      for (size_t c = 0; c < typesA.size(); c++) {
        ga.types[c] = (int8_t)typesA[c];
        ga.dcol[c] = carry[nxt].col[c].p;
        ga.dnul[c] = carry[nxt].nul[c].as<uint8_t>();
      }
      ga.dts = carry[nxt].ts.as<int64_t>();
      ga.dkey = carry[nxt].key.as<uint64_t>();
      ga.dseq = carry[nxt].seq.as<int64_t>();
      hipLaunchKernelGGL(k_gather_carry, dim3(grid_for(n_ext)), dim3(kBlock), 0, s, dev_args(ga),
                         (const uint32_t*)d_co.as<uint32_t>(), (const uint32_t*)d_oo.as<uint32_t>(),
                         (const uint64_t*)d_key.as<uint64_t>(), n_ext);
      SHD_CHECK_LAUNCH();
      mark("carry");
    }
    SHD_HIP(hipEventRecord(ev1, s));
    stage_end();
    SHD_HIP(hipEventSynchronize(ev1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    cur = nxt;
    int64_t created = 0;
    (void)created;
    C = n_open;
    seq += n;
    counters.events += n;
    counters.matches += m;
    counters.partial_scans += (int64_t)steps;
    counters.carry = C;
    counters.kernel_ns = (int64_t)(ms * 1e6);
  }
};

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
  if (!p.aggs.empty() || !p.group_by.empty() || p.having >= 0) { why = "aggregating selector"; return nullptr; }
  if (!p.current_on) { why = "pattern without current events output"; return nullptr; }
  if (p.outputs.size() > (size_t)kMaxCols || a.filters.size() > 4 || b.filters.size() > 4) {
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
  e->W = p.within >= 0 ? p.within : INT64_MAX;
  e->typesA = p.stream_types[a.stream];
  for (auto& o : p.outputs) e->outs.push_back(o.second);
  e->partitioned = !p.part_keys.empty();
  if (e->partitioned) {
    int cls = -1;
    for (auto& pk : p.part_keys) {
      int slot = pk.first == a.stream ? 0 : (pk.first == b.stream ? 1 : -1);
      if (slot < 0) continue;
      int t = expr_result_type(p, pk.second, {});
      if (cls >= 0 && key_class(t) != cls) { why = "partition keys of different types"; return nullptr; }
      cls = key_class(t);
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
  return e;
}

}  // namespace shd
