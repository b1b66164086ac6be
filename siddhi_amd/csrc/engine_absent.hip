// engine_absent.hip -- forward-scan engine for the absent pattern
//   from every e1=A[f1] -> not A[fx] for T select <e1 attributes>
// (config S4 `not ... for`, unpartitioned, one stream).
//
// Reference semantics (ST/AbsentStreamPreStateProcessor.java, restated in
// oracle/oracle.cpp absentAddState / absentTimer / absentPost):
//   * an event passing f1 opens partial P_i (ts_i) at the absent state, which
//     schedules a timer at d_i = ts_i + T (addState :67-88);
//   * every later event j is first offered to the absent state (reverse state
//     order, MultiProcessStreamReceiver): fx(P_i, j) true removes P_i from the
//     pending list (processAndReturn :257-274 -> the post kills it);
//   * InputHandler.send (playback) sets the clock to the call's last event
//     time before the call's events (TimestampGeneratorImpl: only forward);
//     every effective clock move fires the timers due, in ascending time: the
//     timer at d emits every pending partial with d_i <= d (process :150-227),
//     in pending-list order, one callback chunk each, with timestamp d_i.
// So P_i is emitted at the first effective clock move after its creation call
// that reaches d_i, unless an event between its creation and that moment
// passes fx; else it stays open.  Each candidate resolves independently: one
// lane walks the events after it (fx) up to its firing point.  With
// time-ordered events (checked on device; else the query hands over to the
// generic NFA engine) the emission order is the creation order.
#include "engine.h"
#include "pattern_common.h"

namespace shd {

namespace {

using pat::ExtRows;
using pat::PairCtx;
using pat::BatchRowCtx;

enum : uint8_t { AS_NONE = 0, AS_FIRED = 1, AS_OPEN = 2 };

struct AbsArgs {
  ExtRows x;              // rows [0, C) carried partials, [C, C+n) the batch
  DExprSet es;
  DFilters f1, fx;
  int is_a;               // the pushed stream opens partials
  int sx;                 // state id of the absent state
  int64_t T;
  // the push's effective clock moves, ascending: first batch row of the call
  // whose send moved the clock, and the clock after it (non-decreasing)
  const int64_t* e_off;
  const int64_t* e_now;
  int ne;
};

struct AbsOut {
  unsigned long long steps;     // (partial, event) pairs examined
  unsigned long long created;   // partials opened by this push
  unsigned int unmono;          // some ext row's time is below its predecessor's
  unsigned int pad;
};

__device__ __forceinline__ int first_off_after(const AbsArgs& a, int64_t b) {
  int lo = 0, hi = a.ne;   // first e with e_off[e] > b
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a.e_off[mid] > b) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}
__device__ __forceinline__ int first_now_reaching(const AbsArgs& a, int lo, int64_t d) {
  int hi = a.ne;   // first e >= lo with e_now[e] >= d (e_now non-decreasing)
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a.e_now[mid] >= d) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// One lane per extended row: candidates (carried partials, batch events
// passing f1) walk the batch events after them up to their firing point.
template <bool FAST>
__global__ __launch_bounds__(kBlock) void k_abs_scan(const AbsArgs* __restrict__ ap, int64_t n_ext,
                                                     uint8_t* __restrict__ st, int32_t* __restrict__ fe,
                                                     uint32_t* __restrict__ bcnt, AbsOut* __restrict__ blk,
                                                     int64_t tile) {
  const AbsArgs& a = *ap;
  const ExtRows& x = a.x;
  const DExprSet es = a.es;
  const int64_t C = x.C, n = x.batch.n;
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n_ext ? t0 + tile : n_ext;
  uint64_t steps = 0, created = 0;
  uint32_t unmono = 0, nf = 0, no = 0;
  for (int64_t r = t0 + threadIdx.x; r < t1; r += kBlock) {
    const int64_t tr = x.ts(r);
    if (r > 0 && x.ts(r - 1) > tr) unmono = 1;
    bool cand;
    int64_t b;   // batch row of the creating event (-1: carried)
    if (r < C) {
      cand = true;
      b = -1;
    } else {
      b = r - C;
      BatchRowCtx cx{&x.batch, b};
      cand = a.is_a && (FAST ? eval_fpred(a.f1.fp, cx) : eval_filters(es, a.f1, cx));
      created += cand ? 1u : 0u;
    }
    uint8_t out = AS_NONE;
    if (cand) {
      const int64_t d = tr + a.T;
      const int ef = first_now_reaching(a, first_off_after(a, b), d);
      const int64_t lim = ef < a.ne ? a.e_off[ef] : n;
      bool killed = false;
      for (int64_t j = b + 1; j < lim; j++) {
        steps++;
        PairCtx cx{&x, r, C + j, a.sx};
        if (FAST ? eval_fpred(a.fx.fp, cx) : eval_filters(es, a.fx, cx)) {
          killed = true;
          break;
        }
      }
      if (!killed) {
        if (ef < a.ne) {
          out = AS_FIRED;
          fe[r] = ef;
          nf++;
        } else {
          out = AS_OPEN;
          no++;
        }
      }
    }
    st[r] = out;
  }
  for (int o = 32; o > 0; o >>= 1) {
    steps += __shfl_xor(steps, o, 64);
    created += __shfl_xor(created, o, 64);
    unmono |= __shfl_xor(unmono, o, 64);
    nf += __shfl_xor(nf, o, 64);
    no += __shfl_xor(no, o, 64);
  }
  __shared__ AbsOut wpart[kBlock / 64];
  __shared__ uint32_t wc[2][kBlock / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    wpart[w] = AbsOut{steps, created, unmono, 0};
    wc[0][w] = nf;
    wc[1][w] = no;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    AbsOut r = wpart[0];
    uint32_t a0 = wc[0][0], a1 = wc[1][0];
    for (int k = 1; k < kBlock / 64; k++) {
      r.steps += wpart[k].steps;
      r.created += wpart[k].created;
      r.unmono |= wpart[k].unmono;
      a0 += wc[0][k];
      a1 += wc[1][k];
    }
    blk[blockIdx.x] = r;
    bcnt[blockIdx.x] = a0;
    bcnt[gridDim.x + blockIdx.x] = a1;
  }
}

__global__ void k_abs_fold(const AbsOut* __restrict__ blk, int nb, AbsOut* __restrict__ out) {
  AbsOut r{0, 0, 0, 0};
  for (int i = threadIdx.x; i < nb; i += kBlock) {
    r.steps += blk[i].steps;
    r.created += blk[i].created;
    r.unmono |= blk[i].unmono;
  }
  for (int o = 32; o > 0; o >>= 1) {
    r.steps += __shfl_xor(r.steps, o, 64);
    r.created += __shfl_xor(r.created, o, 64);
    r.unmono |= __shfl_xor(r.unmono, o, 64);
  }
  __shared__ AbsOut wp[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wp[threadIdx.x >> 6] = r;
  __syncthreads();
  if (threadIdx.x == 0) {
    AbsOut t = wp[0];
    for (int k = 1; k < kBlock / 64; k++) {
      t.steps += wp[k].steps;
      t.created += wp[k].created;
      t.unmono |= wp[k].unmono;
    }
    *out = t;
  }
}

// Rows of one outcome, in row order: list[boff[tile] + rank] = row.
__global__ __launch_bounds__(kBlock) void k_abs_list(const uint8_t* __restrict__ st, int64_t n, int64_t tile,
                                                     uint8_t val, const uint32_t* __restrict__ boff,
                                                     uint32_t* __restrict__ list) {
  const int64_t t0 = (int64_t)blockIdx.x * tile;
  const int64_t t1 = t0 + tile < n ? t0 + tile : n;
  __shared__ uint32_t wsum[kBlock / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t base = boff[blockIdx.x];
  const uint64_t lt = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int64_t c0 = t0; c0 < t1; c0 += kBlock) {
    const int64_t r = c0 + threadIdx.x;
    const bool hit = r < t1 && st[r] == val;
    const uint64_t m = __ballot(hit);
    if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kBlock / 64; k++) {
      pre += k < w ? wsum[k] : 0u;
      tot += wsum[k];
    }
    if (hit) list[base + pre + (uint32_t)__popcll(m & lt)] = (uint32_t)r;
    base += tot;
    __syncthreads();
  }
}

struct AbsProj {
  ExtRows x;
  DExprSet es;
  DExpr outs[kMaxCols];
  int nout;
  int sx;
  int64_t T;
  const int32_t* fe;       // firing clock move per row (null: fired by shd_set_time)
  const int64_t* e_off;
  int64_t seq_fire;        // in_seq of rows fired by shd_set_time (the next event's index)
  int64_t chunk0, row0;
};

// Fired partials -> output rows (one callback chunk each, timestamp d_i,
// in_seq = the first event of the call whose clock move fired it).
__global__ __launch_bounds__(kBlock) void k_abs_project(const AbsProj* __restrict__ ap, const uint32_t* __restrict__ list,
                                                        int64_t m, int64_t* o_chunk, int32_t* o_type, int64_t* o_ts,
                                                        uint64_t* o_vals, uint8_t* o_nul, int64_t* o_seq,
                                                        int32_t* o_sidx) {
  const AbsProj& a = *ap;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < m; k += (int64_t)gridDim.x * kBlock) {
    const int64_t r = list ? (int64_t)list[k] : k;
    PairCtx cx{&a.x, r, -1, a.sx, true};
    const int64_t row = a.row0 + k;
    for (int c = 0; c < a.nout; c++) {
      const Val v = eval_expr(a.es.ins + a.outs[c].off, a.outs[c].len, a.es.consts, cx);
      o_vals[row * a.nout + c] = v.b;
      o_nul[row * a.nout + c] = (uint8_t)v.null;
    }
    o_ts[row] = a.x.ts(r) + a.T;
    o_type[row] = 0;
    o_seq[row] = a.fe ? a.x.seq0 + a.e_off[a.fe[r]] : a.seq_fire;
    o_sidx[row] = a.sx;
    o_chunk[row] = a.chunk0 + k;
  }
}

// Open partials -> the next push's carry rows (carry_mask columns, ts, seq).
struct AbsCarryArgs {
  ExtRows x;
  int ncols;
  uint32_t amask;
  int32_t types[kMaxCols];
  void* dcol[kMaxCols];
  uint8_t* dnul[kMaxCols];
  int64_t* dts;
  int64_t* dseq;
};

__device__ __forceinline__ void abs_store(void* dst, int type, int64_t o, uint64_t b) {
  switch (type) {
    case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: ((uint32_t*)dst)[o] = (uint32_t)b; break;
    case SHD_T_LONG: case SHD_T_DOUBLE: ((uint64_t*)dst)[o] = b; break;
    case SHD_T_BOOL: ((uint8_t*)dst)[o] = (uint8_t)b; break;
  }
}

__global__ __launch_bounds__(kBlock) void k_abs_carry(const AbsCarryArgs* __restrict__ ap,
                                                      const uint32_t* __restrict__ list, int64_t m, int64_t from) {
  const AbsCarryArgs& a = *ap;
  for (int64_t k = (int64_t)blockIdx.x * kBlock + threadIdx.x; k < m; k += (int64_t)gridDim.x * kBlock) {
    const int64_t r = list ? (int64_t)list[k] : from + k;
    const ColSet& cs = a.x.cs(r);
    const int64_t row = a.x.row(r);
    for (int c = 0; c < a.ncols; c++) {
      if (!((a.amask >> c) & 1u)) continue;
      const Val v = col_load(cs, row, c);
      abs_store(a.dcol[c], a.types[c], k, v.b);
      a.dnul[c][k] = (uint8_t)v.null;
    }
    a.dts[k] = a.x.ts(r);
    a.dseq[k] = a.x.seq(r);
  }
}

// carried partials are time-ordered: how many have d_i <= t
__global__ void k_abs_due(const int64_t* __restrict__ ts, int64_t C, int64_t T, int64_t t,
                          unsigned long long* __restrict__ out) {
  unsigned long long c = 0;
  for (int64_t i = threadIdx.x; i < C; i += kBlock) c += (ts[i] + T <= t) ? 1ull : 0ull;
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  __shared__ unsigned long long wp[kBlock / 64];
  if ((threadIdx.x & 63) == 0) wp[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long s = 0;
    for (int k = 0; k < kBlock / 64; k++) s += wp[k];
    *out = s;
  }
}

// last event time of every call (INT64_MIN for an empty call: nothing is read)
__global__ void k_call_last_ts(const int64_t* __restrict__ ts, const int64_t* __restrict__ offs, int nc,
                               int64_t* __restrict__ out) {
  for (int c = blockIdx.x * kBlock + threadIdx.x; c < nc; c += gridDim.x * kBlock) {
    const int64_t a = offs[c], b = offs[c + 1];
    out[c] = b > a ? ts[b - 1] : INT64_MIN;
  }
}

struct AbsTable {
  DevBuf col[kMaxCols], nul[kMaxCols], ts, seq;
  void reserve(int64_t n, const std::vector<int>& types) {
    n = std::max<int64_t>(n, 1);
    for (size_t c = 0; c < types.size(); c++) {
      col[c].reserve(n * type_size(types[c]));
      nul[c].reserve(n);
    }
    ts.reserve(n * 8);
    seq.reserve(n * 8);
  }
  ColSet colset(const std::vector<int>& types, int64_t n) const {
    ColSet cs{};
    cs.ncols = (int)types.size();
    for (size_t c = 0; c < types.size(); c++) {
      cs.col[c] = col[c].p;
      cs.nul[c] = nul[c].as<uint8_t>();
      cs.type[c] = (int32_t)types[c];
    }
    cs.ts = ts.as<int64_t>();
    cs.n = n;
    return cs;
  }
};

}  // namespace

struct AbsentEngine : Engine {
  int sA = 0;
  int sx = 1;
  std::vector<int> f1, fx, outs, typesA;
  int64_t T = 0;
  uint32_t carry_mask = 0;
  AbsTable carry[2];
  int cur = 0;
  int64_t C = 0;
  DevBuf d_st, d_fe, d_bcnt, d_boff, d_blk, d_agg, d_list, d_scan, d_eoff, d_enow, d_ends, d_last;
  PinnedBuf h_agg, h_last;

  int kind() const override { return ENG_PATTERN; }

  void reset() override {
    C = 0;
    seq = 0;
    now = INT64_MIN;
    chunk_seq = 0;
    out.count = 0;
    counters = shd_counters{};
  }

  ExtRows ext(const ColSet* batch) const {
    ExtRows x{};
    x.carry = carry[cur].colset(typesA, C);
    if (batch) x.batch = *batch;
    x.C = C;
    x.seq0 = seq;
    x.carry_seq = carry[cur].seq.as<int64_t>();
    return x;
  }

  // open partials [from, from + m) of the carry (or the listed ext rows) -> carry[nxt]
  void carry_rows(const ExtRows& x, const uint32_t* list, int64_t m, int64_t from) {
    const int nxt = cur ^ 1;
    carry[nxt].reserve(m, typesA);
    if (m > 0) {
      AbsCarryArgs ca{};
      ca.x = x;
      ca.ncols = (int)typesA.size();
      ca.amask = carry_mask;
      for (size_t c = 0; c < typesA.size(); c++) {
        ca.types[c] = (int32_t)typesA[c];
        ca.dcol[c] = carry[nxt].col[c].p;
        ca.dnul[c] = carry[nxt].nul[c].as<uint8_t>();
      }
      ca.dts = carry[nxt].ts.as<int64_t>();
      ca.dseq = carry[nxt].seq.as<int64_t>();
      hipLaunchKernelGGL(k_abs_carry, dim3(grid_for(m, 1, 4096)), dim3(kBlock), 0, stream, dev_args(ca), list, m, from);
      SHD_CHECK_LAUNCH();
    }
    cur = nxt;
    C = m;
  }

  void project(const ExtRows& x, const uint32_t* list, int64_t m, const int32_t* fe, const int64_t* e_off,
               int64_t seq_fire) {
    if (m <= 0) return;
    out.ensure(m, stream);
    AbsProj pr{};
    pr.x = x;
    pr.es = dset();
    pr.nout = (int)outs.size();
    for (size_t c = 0; c < outs.size(); c++) pr.outs[c] = dexpr(outs[c]);
    pr.sx = sx;
    pr.T = T;
    pr.fe = fe;
    pr.e_off = e_off;
    pr.seq_fire = seq_fire;
    pr.chunk0 = chunk_seq;
    pr.row0 = out.count;
    hipLaunchKernelGGL(k_abs_project, dim3(grid_for(m, 1, 4096)), dim3(kBlock), 0, stream, dev_args(pr), list, m,
                       out.d_chunk(), out.d_type(), out.d_ts(), out.d_vals(), out.d_nulls(), out.d_seq(), out.d_sidx());
    SHD_CHECK_LAUNCH();
    out.count += m;
    chunk_seq += m;
    counters.matches += m;
  }

  // shd_set_time: a clock move fires the carried partials it reaches (they
  // are time-ordered: a prefix of the carry), before the next event.
  void set_time(int64_t t) override {
    if (t < now) return;
    now = t;
    if (C == 0) return;
    d_agg.reserve(64);
    h_agg.reserve(64);
    hipLaunchKernelGGL(k_abs_due, dim3(1), dim3(kBlock), 0, stream, carry[cur].ts.as<int64_t>(), C, T, t,
                       d_agg.as<unsigned long long>());
    SHD_CHECK_LAUNCH();
    SHD_HIP(hipMemcpyAsync(h_agg.p, d_agg.p, 8, hipMemcpyDeviceToHost, stream));
    SHD_HIP(hipStreamSynchronize(stream));
    const int64_t f = (int64_t)h_agg.as<unsigned long long>()[0];
    if (f == 0) return;
    const ExtRows x = ext(nullptr);
    project(x, nullptr, f, nullptr, nullptr, seq);
    carry_rows(x, nullptr, C - f, f);
    SHD_HIP(hipStreamSynchronize(stream));
    counters.carry = C;
  }

  void push(const Staged& b) override {
    const int64_t n = b.n;
    if (n <= 0) return;
    hipStream_t s = stream;
    SHD_HIP(hipEventRecord(ev0, s));
    stage_begin();
    const bool isA = b.stream == sA;
    const int64_t n_ext = C + n;
    // the push's clock moves (InputHandler.send of each call, playback)
    std::vector<int64_t> e_off, e_now;
    int64_t now_after = now;
    if (b.advance_time) {
      const int nc = (int)b.call_offsets.size() - 1;
      d_ends.reserve((size_t)(nc + 1) * 8);
      d_last.reserve((size_t)nc * 8);
      h_last.reserve((size_t)nc * 8);
      SHD_HIP(hipMemcpyAsync(d_ends.p, b.call_offsets.data(), (size_t)(nc + 1) * 8, hipMemcpyHostToDevice, s));
      hipLaunchKernelGGL(k_call_last_ts, dim3(grid_for(nc)), dim3(kBlock), 0, s, b.cs.ts,
                         (const int64_t*)d_ends.as<int64_t>(), nc, d_last.as<int64_t>());
      SHD_CHECK_LAUNCH();
      SHD_HIP(hipMemcpyAsync(h_last.p, d_last.p, (size_t)nc * 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
      const int64_t* last = h_last.as<int64_t>();
      for (int c = 0; c < nc; c++) {
        if (b.call_offsets[c + 1] <= b.call_offsets[c]) continue;
        if (last[c] >= now_after) {   // TimestampGeneratorImpl: the clock only moves forward
          now_after = last[c];
          e_off.push_back(b.call_offsets[c]);
          e_now.push_back(now_after);
        }
      }
    }
    const int ne = (int)e_off.size();
    d_eoff.reserve((size_t)std::max(ne, 1) * 8);
    d_enow.reserve((size_t)std::max(ne, 1) * 8);
    if (ne) {
      SHD_HIP(hipMemcpyAsync(d_eoff.p, e_off.data(), (size_t)ne * 8, hipMemcpyHostToDevice, s));
      SHD_HIP(hipMemcpyAsync(d_enow.p, e_now.data(), (size_t)ne * 8, hipMemcpyHostToDevice, s));
    }
    const ExtRows x = ext(&b.cs);
    AbsArgs aa{};
    aa.x = x;
    aa.es = dset();
    aa.f1 = dfilters(f1);
    aa.fx = dfilters(fx);
    aa.is_a = isA;
    aa.sx = sx;
    aa.T = T;
    aa.e_off = d_eoff.as<int64_t>();
    aa.e_now = d_enow.as<int64_t>();
    aa.ne = ne;
    const int nblk = grid_for(n_ext, 1, 4096);
    const int64_t tile = ceil_div(ceil_div(n_ext, nblk), kBlock) * kBlock;
    const int ntile = (int)ceil_div(n_ext, tile);
    d_st.reserve(n_ext);
    d_fe.reserve(n_ext * 4);
    d_bcnt.reserve((size_t)2 * ntile * 4);
    d_boff.reserve((size_t)2 * ntile * 4);
    d_blk.reserve((size_t)ntile * sizeof(AbsOut));
    d_agg.reserve(64);
    h_agg.reserve(64);
    const AbsArgs* d_aa = dev_args(aa);
    if (aa.f1.fp.ok && aa.fx.fp.ok)
      hipLaunchKernelGGL(k_abs_scan<true>, dim3(ntile), dim3(kBlock), 0, s, d_aa, n_ext, d_st.as<uint8_t>(),
                         d_fe.as<int32_t>(), d_bcnt.as<uint32_t>(), d_blk.as<AbsOut>(), tile);
    else
      hipLaunchKernelGGL(k_abs_scan<false>, dim3(ntile), dim3(kBlock), 0, s, d_aa, n_ext, d_st.as<uint8_t>(),
                         d_fe.as<int32_t>(), d_bcnt.as<uint32_t>(), d_blk.as<AbsOut>(), tile);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_abs_fold, dim3(1), dim3(kBlock), 0, s, (const AbsOut*)d_blk.as<AbsOut>(), ntile,
                       d_agg.as<AbsOut>());
    SHD_CHECK_LAUNCH();
    uint32_t* d_tot = reinterpret_cast<uint32_t*>(d_agg.as<char>() + 32);
    scan_exclusive_u32(d_bcnt.as<uint32_t>(), d_boff.as<uint32_t>(), ntile, d_tot, d_scan, s);
    scan_exclusive_u32(d_bcnt.as<uint32_t>() + ntile, d_boff.as<uint32_t>() + ntile, ntile, d_tot + 1, d_scan, s);
    SHD_HIP(hipMemcpyAsync(h_agg.p, d_agg.p, 40, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    mark("absent_scan");
    AbsOut so;
    std::memcpy(&so, h_agg.p, sizeof(so));
    const uint32_t n_fired = h_agg.as<uint32_t>()[8], n_open = h_agg.as<uint32_t>()[9];
    if (so.unmono)   // emission order is the creation order only for time-ordered rows
      throw NeedNfa("absent pattern engine: event timestamps decrease");
    d_list.reserve((size_t)std::max<uint32_t>(std::max(n_fired, n_open), 1) * 4);
    if (n_fired) {
      hipLaunchKernelGGL(k_abs_list, dim3(ntile), dim3(kBlock), 0, s, (const uint8_t*)d_st.as<uint8_t>(), n_ext, tile,
                         (uint8_t)AS_FIRED, (const uint32_t*)d_boff.as<uint32_t>(), d_list.as<uint32_t>());
      SHD_CHECK_LAUNCH();
      project(x, d_list.as<uint32_t>(), n_fired, d_fe.as<int32_t>(), d_eoff.as<int64_t>(), 0);
    }
    if (n_open) {
      hipLaunchKernelGGL(k_abs_list, dim3(ntile), dim3(kBlock), 0, s, (const uint8_t*)d_st.as<uint8_t>(), n_ext, tile,
                         (uint8_t)AS_OPEN, (const uint32_t*)d_boff.as<uint32_t>() + ntile, d_list.as<uint32_t>());
      SHD_CHECK_LAUNCH();
    }
    carry_rows(x, d_list.as<uint32_t>(), n_open, 0);
    mark("emit_carry");
    SHD_HIP(hipEventRecord(ev1, s));
    stage_end();
    SHD_HIP(hipEventSynchronize(ev1));
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, ev0, ev1));
    seq += n;
    now = now_after;
    counters.events += n;
    counters.partials += (int64_t)so.created;
    counters.partial_scans += (int64_t)so.steps;
    counters.carry = C;
    counters.kernel_ns = (int64_t)(ms * 1e6);
  }

  // the open partials as the A events that opened them (arrival order): each
  // met every later event without fx passing and no clock move reached its
  // deadline, so a replay from a fresh state (no clock moves) rebuilds them
  void export_replay(std::vector<Replay>& parts) override {
    SHD_HIP(hipStreamSynchronize(stream));
    parts.clear();
    if (C == 0) return;
    Replay r;
    r.stream = sA;
    r.n = C;
    r.ts.resize(C);
    SHD_HIP(hipMemcpy(r.ts.data(), carry[cur].ts.p, C * 8, hipMemcpyDeviceToHost));
    r.cols.assign(typesA.size(), {});
    r.nulls.assign(typesA.size(), {});
    for (size_t c = 0; c < typesA.size(); c++) {
      r.cols[c].resize((size_t)C * type_size(typesA[c]));
      r.nulls[c].resize((size_t)C);
      SHD_HIP(hipMemcpy(r.cols[c].data(), carry[cur].col[c].p, r.cols[c].size(), hipMemcpyDeviceToHost));
      SHD_HIP(hipMemcpy(r.nulls[c].data(), carry[cur].nul[c].p, (size_t)C, hipMemcpyDeviceToHost));
    }
    parts.push_back(std::move(r));
  }

  void save_state(SnapW& w) override {
    w.put<int64_t>(C);
    w.put<int32_t>((int32_t)typesA.size());
    const AbsTable& t = carry[cur];
    for (size_t c = 0; c < typesA.size(); c++) {
      w.dev(t.col[c].p, (size_t)C * type_size(typesA[c]));
      w.dev(t.nul[c].p, (size_t)C);
    }
    w.dev(t.ts.p, (size_t)C * 8);
    w.dev(t.seq.p, (size_t)C * 8);
  }
  void load_state(SnapR& r) override {
    const int64_t c0 = r.get<int64_t>();
    if (r.get<int32_t>() != (int32_t)typesA.size() || c0 < 0) throw Error(SHD_E_ARG, "snapshot of a different plan");
    cur = 0;
    AbsTable& t = carry[0];
    t.reserve(c0, typesA);
    for (size_t c = 0; c < typesA.size(); c++) {
      r.dev_into(t.col[c].p, (size_t)c0 * type_size(typesA[c]));
      r.dev_into(t.nul[c].p, (size_t)c0);
    }
    r.dev_into(t.ts.p, (size_t)c0 * 8);
    r.dev_into(t.seq.p, (size_t)c0 * 8);
    C = c0;
    counters.carry = C;
  }
};

static bool reads_states(const Plan& p, int e, int a, int b) {
  for (auto& in : p.exprs[e]) {
    if (in.op == SHD_OP_TS) return false;   // eventTimestamp(): the StateEvent's time (not restated here)
    if ((in.op == SHD_OP_LOAD || in.op == SHD_OP_EVNULL) && in.a != a && in.a != b) return false;
    if (in.op == SHD_OP_AGG) return false;
  }
  return true;
}

std::unique_ptr<Engine> make_absent_engine(const Plan& p, std::string& why) {
  if (p.kind != SHD_KIND_STATE || p.state_type != 0) { why = "not a pattern"; return nullptr; }
  const PNode& r = p.root;
  if (r.kind != SHD_NODE_NEXT || r.kids.size() != 2) { why = "not a two-state chain"; return nullptr; }
  const PNode& ev = r.kids[0];
  const PNode& b = r.kids[1];
  if (ev.kind != SHD_NODE_EVERY || ev.kids.size() != 1 || ev.kids[0].kind != SHD_NODE_STREAM ||
      b.kind != SHD_NODE_STREAM) {
    why = "not every e1 -> not X for t";
    return nullptr;
  }
  const PNode& a = ev.kids[0];
  if (a.absent || !b.absent || b.waiting <= 0 || a.state_id != 0 || a.stream != b.stream) {
    why = "not every e1=A -> not A for t";
    return nullptr;
  }
  if (!p.part_keys.empty() || p.within >= 0) { why = "partitioned / within"; return nullptr; }
  if (!p.aggs.empty() || !p.group_by.empty() || p.having >= 0 || !p.current_on) { why = "aggregating selector"; return nullptr; }
  if (p.outputs.size() > (size_t)kMaxCols || a.filters.size() > 4 || b.filters.size() > 4) {
    why = "too many outputs / filters";
    return nullptr;
  }
  if (p.stream_types[a.stream].size() > (size_t)kMaxCols) { why = "too many attributes"; return nullptr; }
  for (int f : a.filters)
    if (!reads_states(p, f, 0, 0)) { why = "e1 filter reads other states"; return nullptr; }
  for (int f : b.filters)
    if (!reads_states(p, f, 0, b.state_id)) { why = "absent filter reads other states"; return nullptr; }
  for (auto& o : p.outputs)
    if (!reads_states(p, o.second, 0, b.state_id)) { why = "selector reads event time / other states"; return nullptr; }
  auto e = std::make_unique<AbsentEngine>();
  e->sA = a.stream;
  e->sx = b.state_id;
  e->f1 = a.filters;
  e->fx = b.filters;
  e->T = b.waiting;
  e->typesA = p.stream_types[a.stream];
  for (auto& o : p.outputs) e->outs.push_back(o.second);
  uint32_t mask = 0;
  auto add = [&](int ex) {
    for (const Instr& in : p.exprs[ex])
      if (in.op == SHD_OP_LOAD && in.a == 0) mask |= 1u << (in.c & 0xFFFF);
  };
  for (int f : e->f1) add(f);
  for (int f : e->fx) add(f);
  for (int o : e->outs) add(o);
  e->carry_mask = mask;
  return e;
}

}  // namespace shd
