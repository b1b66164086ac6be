// engine.h -- query engines behind the C-ABI (one per loaded plan).
#pragma once
#include <algorithm>
#include <cstring>
#include <memory>
#include <vector>

#include "common.h"
#include "dev_expr.h"

namespace shd {

enum EngineKind { ENG_PATTERN = 1, ENG_WINDOW = 2, ENG_FILTER = 3, ENG_NFA = 4 };

// Device output arena: rows accumulate across pushes until polled.
struct OutputBuffer {
  int ncols = 0;
  int64_t count = 0, cap = 0;
  DevBuf chunk, type, ts, vals, nulls, seq, sidx;
  void init(int nc) { ncols = nc; }
  // Make room for `extra` more rows (copies existing rows on growth).
  void ensure(int64_t extra, hipStream_t s);
  int64_t* d_chunk() { return chunk.as<int64_t>(); }
  int32_t* d_type() { return type.as<int32_t>(); }
  int64_t* d_ts() { return ts.as<int64_t>(); }
  uint64_t* d_vals() { return vals.as<uint64_t>(); }
  uint8_t* d_nulls() { return nulls.as<uint8_t>(); }
  int64_t* d_seq() { return seq.as<int64_t>(); }   // shd_out.in_seq
  int32_t* d_sidx() { return sidx.as<int32_t>(); }  // shd_out.state_idx
  // list arena of SHD_T_OBJECT outputs (multi-value selections): values and
  // null flags; a row's list handle = offset | count << 40
  DevBuf lvals, lnul;
  int64_t lcount = 0, lcap = 0;
  void ensure_list(int64_t extra, hipStream_t s);
};

// A batch staged on the device (columns either borrowed device pointers or
// copies of host buffers).
struct Staged {
  int stream = 0;
  int64_t n = 0;
  ColSet cs{};
  std::vector<int64_t> call_offsets;   // host, ncalls+1
  bool advance_time = false;
  const uint8_t* skip_start = nullptr;   // device [n] or null: hand-over replays only (Replay::skip_start)
};

// Snapshot streams (shd_snapshot / shd_restore): a flat little-endian byte
// image of an engine's cross-push state.  Device buffers are copied with
// synchronous hipMemcpy on the query's stream after it drained.
struct SnapW {
  std::vector<uint8_t> b;
  hipStream_t s = nullptr;
  template <class T> void put(const T& v) {
    const size_t o = b.size();
    b.resize(o + sizeof(T));
    std::memcpy(b.data() + o, &v, sizeof(T));
  }
  void bytes(const void* src, size_t n) {
    const size_t o = b.size();
    b.resize(o + n);
    if (n) std::memcpy(b.data() + o, src, n);
  }
  // n bytes of device memory at p
  void dev(const void* p, size_t n) {
    put<uint64_t>(n);
    const size_t o = b.size();
    b.resize(o + n);
    if (n) {
      SHD_HIP(hipMemcpyAsync(b.data() + o, p, n, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipStreamSynchronize(s));
    }
  }
};

struct SnapR {
  const uint8_t* p = nullptr;
  size_t n = 0, at = 0;
  hipStream_t s = nullptr;
  void need(size_t k) const {
    if (at + k > n) throw Error(SHD_E_ARG, "snapshot truncated or from a different plan");
  }
  template <class T> T get() {
    need(sizeof(T));
    T v;
    std::memcpy(&v, p + at, sizeof(T));
    at += sizeof(T);
    return v;
  }
  // device section into buf (reserved to at least its size); returns its size
  size_t dev(DevBuf& buf, size_t extra_cap = 0) {
    const size_t k = (size_t)get<uint64_t>();
    need(k);
    buf.reserve(std::max<size_t>(k, extra_cap));
    if (k) {
      SHD_HIP(hipMemcpyAsync(buf.p, p + at, k, hipMemcpyHostToDevice, s));
      SHD_HIP(hipStreamSynchronize(s));
    }
    at += k;
    return k;
  }
  // device section into p (exactly `expect` bytes)
  void dev_into(void* dst, size_t expect) {
    const size_t k = (size_t)get<uint64_t>();
    if (k != expect) throw Error(SHD_E_ARG, "snapshot section size mismatch");
    need(k);
    if (k) {
      SHD_HIP(hipMemcpyAsync(dst, p + at, k, hipMemcpyHostToDevice, s));
      SHD_HIP(hipStreamSynchronize(s));
    }
    at += k;
  }
};

// Thrown by an engine whose formulation cannot continue on a valid input
// (e.g. the pattern forward scan when timestamps go back inside a key) but
// whose cross-push state the generic NFA engine can take over: shd_push then
// replays the open partials (Engine::export_replay) into a fresh NFA engine
// and runs the push there.  Never surfaces through the C-ABI.
struct NeedNfa : Error {
  explicit NeedNfa(const std::string& m) : Error(SHD_E_UNSUPPORTED, m) {}
};

// Thrown by a query group's leader whose shared pass cannot take a push (a
// window group's operand range or call shape): shd_group_push dissolves the
// group (Engine::group_dissolve) and each member takes the push alone.
struct NeedDissolve : NeedNfa {
  explicit NeedDissolve(const std::string& m) : NeedNfa(m) {}
};

// Host image of a query's open partial matches as the events whose replay
// rebuilds them, in arrival order: one part per run of same-stream events
// (typed columns as in shd_batch).  skip_start[i] = 1: event i is replayed
// only for the partials it belongs to (an operand event of a half-filled
// logical AND partial whose own start partial is gone) -- the start state does
// not see it; 2: event i only stabilises its key's states (expiry + the
// new-list -> pending-list move, StreamPreStateProcessor.updateState) and no
// state processes it.
struct Replay {
  int stream = 0;
  int64_t n = 0;
  std::vector<int64_t> ts;
  std::vector<std::vector<uint8_t>> cols, nulls;   // [ncols] typed bytes / null bytes
  std::vector<uint8_t> skip_start;                 // [n] (empty: none skipped)
};

struct Engine {
  Plan plan;
  DevExprTable ex;
  hipStream_t stream = nullptr;
  OutputBuffer out;
  shd_counters counters{};
  int64_t seq = 0;                         // global arrival index of the next event
  int64_t now = INT64_MIN;                 // playback time (TimestampGeneratorImpl.lastEventTimestamp)
  int64_t chunk_seq = 0;                   // next callback-chunk id
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  // stage timing (profiling hook): events recorded around each kernel stage
  static constexpr int kMaxStages = 16;
  hipEvent_t sev[kMaxStages + 1] = {};
  const char* stage_name[kMaxStages] = {};
  int n_stages = 0;
  int64_t stage_ns[kMaxStages] = {};
  void stage_begin() { n_stages = 0; mark(nullptr); }
  void mark(const char* name_of_finished_stage);
  void stage_end();

  virtual ~Engine();
  virtual int kind() const = 0;
  virtual void push(const Staged& b) = 0;
  virtual void set_time(int64_t t) {
    if (t >= now) now = t;
  }
  virtual void reset() = 0;
  // shd_set_option: named engine options (unknown names -> SHD_E_ARG).
  // "start_time": the app's clock when SiddhiAppRuntime.start() ran (wall-clock
  // apps: System.currentTimeMillis(); playback: 0, TimestampGeneratorImpl's
  // initial lastEventTimestamp) -- unpartitioned state queries seed their
  // absent start states with it (AbsentStreamPreStateProcessor.partitionCreated
  // :291-303 reads currentTime()).
  int64_t start_time = 0;
  // construction hint of the engine's state layout (generic NFA engine: the
  // list_hint of make_nfa_engine); snapshots carry it so that a restore builds
  // the same layout
  int64_t layout_hint = 0;
  virtual void set_option(const std::string& key, int64_t v) {
    if (key == "start_time") {
      start_time = v;
      if (v > now) now = v;
      return;
    }
    throw Error(SHD_E_ARG, "unknown option '" + key + "' for this query");
  }
  // called once the plan's expression table is on the device
  virtual void on_loaded() {}
  // Cross-push state (partial-match tables, window contents, aggregates) for
  // SiddhiAppRuntime.snapshot()/restore() (C/SiddhiAppRuntimeImpl.java:695-717,
  // SnapshotService.fullSnapshot/restore C/util/snapshot/SnapshotService.java:90,333,
  // the per-processor State.snapshot/restore maps, e.g.
  // ST/StreamPreStateProcessor.java:450-469).  The common fields (seq, time,
  // chunk ids, counters) are written by shd_snapshot itself.
  virtual void save_state(SnapW&) { throw Error(SHD_E_UNSUPPORTED, "engine has no snapshot support"); }
  virtual void load_state(SnapR&) { throw Error(SHD_E_UNSUPPORTED, "engine has no snapshot support"); }
  // Events whose replay through the reference algorithm (from a fresh state)
  // rebuilds exactly this engine's open partial matches (NeedNfa hand-over).
  virtual void export_replay(std::vector<Replay>&) {
    throw Error(SHD_E_UNSUPPORTED, "engine state cannot be handed over");
  }
  // Query sharing (shd_group_*, the junction fan-out of StreamJunction.java:146-272
  // to queries that differ only in their start-state filter): this engine
  // becomes the leader of `members`, whose rows it derives from its own
  // per-push results.  grouped: a leader or member -- pushes, resets and
  // snapshots go through the group.
  bool grouped = false;
  virtual void group_attach(const std::vector<Engine*>&) {
    throw Error(SHD_E_UNSUPPORTED, "this query's engine cannot lead a query group");
  }
  virtual void group_detach() {}
  // leader: hand each member the state it would hold running alone, detach
  virtual void group_dissolve() { throw Error(SHD_E_UNSUPPORTED, "this group cannot dissolve"); }

  // Kernel argument blocks (column tables, expression handles) are placed in
  // device memory and kernels receive a pointer: the kernels index column
  // tables with lane-dependent values, and vector loads from the kernarg
  // segment fault on the MI355X boxes (HSA aperture violation, see DESIGN.md
  // "kernel arguments").  Bump arena, reset at the start of each push.
  static constexpr size_t kArgArena = size_t(1) << 20;
  DevBuf arg_dev;
  PinnedBuf arg_host;
  size_t arg_used = 0;
  void args_begin() {
    if (!arg_dev.p) {
      arg_dev.reserve(kArgArena);
      arg_host.reserve(kArgArena);
    }
    SHD_HIP(hipStreamSynchronize(stream));   // previous push's argument copies have landed
    arg_used = 0;
  }
  template <class T> const T* dev_args(const T& a) {
    size_t off = (arg_used + 255) & ~size_t(255);
    if (!arg_dev.p || off + sizeof(T) > kArgArena) throw Error(SHD_E_CAPACITY, "kernel argument arena exhausted");
    std::memcpy(arg_host.as<char>() + off, &a, sizeof(T));
    SHD_HIP(hipMemcpyAsync(arg_dev.as<char>() + off, arg_host.as<char>() + off, sizeof(T), hipMemcpyHostToDevice,
                           stream));
    arg_used = off + sizeof(T);
    return reinterpret_cast<const T*>(arg_dev.as<char>() + off);
  }

  DExpr dexpr(int e) const { return DExpr{ex.off[e], ex.len[e]}; }
  DExprSet dset() const { return DExprSet{ex.ins.as<int4>(), ex.consts.as<uint64_t>(), ex.nins, ex.nconsts}; }
  DFilters dfilters(const std::vector<int>& ids) const;
  // An output / operand expression that is one LOAD / CONST / NULL, optionally
  // followed by one CVT, pre-decoded as an FAtom (fp_atom: no bytecode per row).
  bool fast_atom(int expr_id, FAtom& out) const;
};

std::unique_ptr<Engine> make_pattern_engine(const Plan& p, std::string& why);
std::unique_ptr<Engine> make_logical_pattern_engine(const Plan& p, std::string& why);
// `every e1=A[f1] -> not A[fx] for T` (engine_absent.hip)
std::unique_ptr<Engine> make_absent_engine(const Plan& p, std::string& why);
std::unique_ptr<Engine> make_single_engine(const Plan& p, std::string& why);
// keyed exact window engine: EXPIRED output, `having`, partitioned windows /
// aggregates (engine_window.hip)
std::unique_ptr<Engine> make_window_x_engine(const Plan& p, std::string& why);
std::unique_ptr<Engine> make_nfa_engine(const Plan& p, std::string& why);
// list_hint: expected partials per key at once (sizes the per-key lists of an
// unpartitioned plan; 0 = defaults)
std::unique_ptr<Engine> make_nfa_engine(const Plan& p, std::string& why, int64_t list_hint);
// Engine setup shared by shd_plan_load and the engine switches (expression
// table upload, output arena, stream and events, reset).
void init_engine(Engine& e, const Plan& p);

}  // namespace shd
