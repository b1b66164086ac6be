// oracle/oracle.cpp -- CPU restatement of Siddhi's pattern/sequence/window hot path.
//
// TEST INFRASTRUCTURE ONLY.  This file is the parity checker for
// libsiddhi_hip: only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.  The product path never calls it.
//
// It restates, single-threaded and object-for-object, the reference control
// flow (paths relative to modules/siddhi-core/src/main/java/io/siddhi/core/):
//   query/input/stream/state/StreamPreStateProcessor.java      (StreamPre*)
//   query/input/stream/state/StreamPostStateProcessor.java     (StreamPost*)
//   query/input/stream/state/CountPre/PostStateProcessor.java  (Count*)
//   query/input/stream/state/LogicalPre/PostStateProcessor.java(Logical*)
//   query/input/stream/state/AbsentStreamPre/PostStateProcessor.java (Absent*)
//   query/input/stream/state/runtime/*InnerStateRuntime.java   (Runtime*)
//   query/input/stream/state/receiver/*.java + query/input/{Single,Multi,
//     StateMulti}ProcessStreamReceiver.java                    (receive_*)
//   util/parser/StateInputStreamParser.java:76-408              (build_state)
//   executor/condition/**, executor/math/**                     (eval)
//   query/processor/stream/window/{Length,Time}WindowProcessor  (window_*)
//   query/selector/QuerySelector.java + aggregator/*             (selector_*)
//   partition/PartitionStreamReceiver.java:175-283               (push)
//   util/Scheduler.java:71-209, util/timestamp/TimestampGeneratorImpl.java
//
// Object identity matters (shared StateEvent / StreamEvent chains between
// clones, StateEventCloner.java:47-58), so the restatement keeps real object
// graphs in an arena instead of value copies.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../include/siddhi_ir.h"

namespace {

constexpr int64_t UNKNOWN = -1;
constexpr int CURRENT = 0, EXPIRED = 1, TIMER = 2, RESET = 3;

// ------------------------------------------------------------------ IR decode
struct Instr { int32_t op, a, b, c; };

struct Node {
  int kind = 0;
  // stream
  int state_id = -1, stream = -1, absent = 0;
  int64_t waiting = -1;
  std::vector<int> filters;
  // logical
  int ltype = 0;
  // count
  int min = 0, max = 0;
  std::vector<std::unique_ptr<Node>> kids;
};

struct Plan {
  int kind = 0;
  std::vector<std::vector<int>> stream_types;
  std::vector<uint64_t> consts;
  std::vector<std::vector<Instr>> exprs;
  std::vector<std::pair<int, int>> part_keys;
  // state
  int state_type = 0;  // 0 pattern, 1 sequence
  int64_t within = -1;
  int n_states = 0;
  std::unique_ptr<Node> root;
  // single
  int single_stream = 0;
  struct Handler { int kind; int expr; int wkind; int64_t param, param2; };
  std::vector<Handler> handlers;
  // selector
  bool current_on = true, expired_on = false;
  struct Agg { int kind, expr, type; };
  std::vector<Agg> aggs;
  std::vector<int> group_by;
  int64_t null_str_id = -1;   // dictionary id of "null" (string group keys)
  int having = -1;
  std::vector<std::pair<int, int>> outputs;  // (type, expr)
};

struct Reader {
  const int32_t* w; int64_t n, i = 0;
  int32_t next() {
    if (i >= n) throw std::runtime_error("plan IR truncated");
    return w[i++];
  }
  int64_t next64() {
    uint32_t lo = (uint32_t)next();
    uint32_t hi = (uint32_t)next();
    return (int64_t)(((uint64_t)hi << 32) | lo);
  }
};

std::unique_ptr<Node> read_node(Reader& r) {
  auto n = std::make_unique<Node>();
  n->kind = r.next();
  switch (n->kind) {
    case SHD_NODE_STREAM: {
      n->state_id = r.next();
      n->stream = r.next();
      n->absent = r.next();
      n->waiting = r.next64();
      int nf = r.next();
      for (int i = 0; i < nf; i++) n->filters.push_back(r.next());
      break;
    }
    case SHD_NODE_NEXT:
      n->kids.push_back(read_node(r));
      n->kids.push_back(read_node(r));
      break;
    case SHD_NODE_EVERY:
      n->kids.push_back(read_node(r));
      break;
    case SHD_NODE_LOGICAL:
      n->ltype = r.next();
      n->kids.push_back(read_node(r));
      n->kids.push_back(read_node(r));
      break;
    case SHD_NODE_COUNT:
      n->min = r.next();
      n->max = r.next();
      n->kids.push_back(read_node(r));
      break;
    default:
      throw std::runtime_error("bad node kind");
  }
  return n;
}

Plan decode(const int32_t* w, int64_t n) {
  Reader r{w, n};
  Plan p;
  if (r.next() != (int32_t)SHD_IR_MAGIC) throw std::runtime_error("bad plan magic");
  if (r.next() != SHD_IR_VERSION) throw std::runtime_error("bad plan version");
  p.kind = r.next();
  int ns = r.next();
  for (int s = 0; s < ns; s++) {
    int na = r.next();
    std::vector<int> t;
    for (int a = 0; a < na; a++) t.push_back(r.next());
    p.stream_types.push_back(t);
  }
  int nc = r.next();
  for (int i = 0; i < nc; i++) p.consts.push_back((uint64_t)r.next64());
  int ne = r.next();
  for (int i = 0; i < ne; i++) {
    int ni = r.next();
    std::vector<Instr> code;
    for (int k = 0; k < ni; k++) {
      Instr in;
      in.op = r.next(); in.a = r.next(); in.b = r.next(); in.c = r.next();
      code.push_back(in);
    }
    p.exprs.push_back(code);
  }
  int nk = r.next();
  for (int i = 0; i < nk; i++) {
    int s = r.next();
    int e = r.next();
    p.part_keys.push_back({s, e});
  }
  if (p.kind == SHD_KIND_STATE) {
    p.state_type = r.next();
    p.within = r.next64();
    p.n_states = r.next();
    p.root = read_node(r);
  } else {
    p.single_stream = r.next();
    int nh = r.next();
    for (int i = 0; i < nh; i++) {
      Plan::Handler h{};
      h.kind = r.next();
      if (h.kind == SHD_H_FILTER) {
        h.expr = r.next();
      } else {
        h.wkind = r.next();
        h.param = r.next64();
        h.param2 = r.next64();
      }
      p.handlers.push_back(h);
    }
  }
  p.current_on = r.next();
  p.expired_on = r.next();
  int na = r.next();
  for (int i = 0; i < na; i++) {
    Plan::Agg a;
    a.kind = r.next(); a.expr = r.next(); a.type = r.next();
    p.aggs.push_back(a);
  }
  int ng = r.next();
  for (int i = 0; i < ng; i++) p.group_by.push_back(r.next());
  p.having = r.next();
  int no = r.next();
  for (int i = 0; i < no; i++) {
    int t = r.next();
    int e = r.next();
    p.outputs.push_back({t, e});
  }
  // optional trailing section: dictionary id of the string "null" (group keys)
  if (r.i + 2 <= r.n) p.null_str_id = r.next64();
  return p;
}

// ------------------------------------------------------------------ events
// StreamEvent (C/event/stream/StreamEvent.java): payload points at the
// immutable input row; clones share it (copyStreamEvent copies the arrays,
// which are never mutated on this path).
struct Ev {
  int64_t ts = 0;
  int type = CURRENT;
  const uint64_t* data = nullptr;
  const uint8_t* nul = nullptr;
  int64_t seq = -1;   // global arrival index of the input row
  Ev* next = nullptr;
};

// StateEvent (C/event/state/StateEvent.java:42-258)
struct SE {
  std::vector<Ev*> ev;
  int64_t ts = -1;
  int type = CURRENT;
  SE* next = nullptr;
};

template <class T>
struct Arena {
  std::deque<std::unique_ptr<T[]>> blocks;
  size_t used = 1 << 16;
  std::vector<T*> free_list;
  T* get() {
    if (!free_list.empty()) {
      T* t = free_list.back();
      free_list.pop_back();
      return t;
    }
    if (used == (1u << 16)) {
      blocks.emplace_back(new T[1 << 16]);
      used = 0;
    }
    return &blocks.back()[used++];
  }
  void put(T* t) { free_list.push_back(t); }
};

// StateEvent.getStreamEvent(int[] position) (StateEvent.java:138-182)
Ev* chain_get(Ev* e, int idx) {
  if (!e) return nullptr;
  if (idx >= 0) {
    for (int i = 1; i <= idx; i++) {
      e = e->next;
      if (!e) return nullptr;
    }
    return e;
  }
  if (idx == SHD_IDX_CURRENT) {
    while (e->next) e = e->next;
    return e;
  }
  if (idx == SHD_IDX_LAST) {
    if (!e->next) return nullptr;
    while (e->next->next) e = e->next;
    return e;
  }
  std::vector<Ev*> all;
  while (e) { all.push_back(e); e = e->next; }
  int64_t k = (int64_t)all.size() + idx;
  if (k < 0) return nullptr;
  return all[k];
}

// ------------------------------------------------------------------ values
struct Val { uint64_t b = 0; bool null = true; };

inline int32_t as_i32(uint64_t b) { return (int32_t)(uint32_t)b; }
inline int64_t as_i64(uint64_t b) { return (int64_t)b; }
inline float as_f32(uint64_t b) { float f; uint32_t u = (uint32_t)b; memcpy(&f, &u, 4); return f; }
inline double as_f64(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
inline uint64_t of_i32(int32_t v) { return (uint64_t)(int64_t)v; }
inline uint64_t of_i64(int64_t v) { return (uint64_t)v; }
inline uint64_t of_f32(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
inline uint64_t of_f64(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

// Number.xValue() conversions used by the math/compare executors.
uint64_t cvt(uint64_t b, int from, int to) {
  if (from == to) return b;
  double d = 0; float f = 0; int64_t l = 0;
  switch (from) {
    case SHD_T_INT: l = as_i32(b); d = (double)as_i32(b); f = (float)as_i32(b); break;
    case SHD_T_LONG: l = as_i64(b); d = (double)as_i64(b); f = (float)as_i64(b); break;
    case SHD_T_FLOAT: d = (double)as_f32(b); f = as_f32(b); l = (int64_t)as_f32(b); break;
    case SHD_T_DOUBLE: d = as_f64(b); f = (float)as_f64(b); l = (int64_t)as_f64(b); break;
    default: throw std::runtime_error("bad cvt");
  }
  switch (to) {
    case SHD_T_INT: return of_i32((int32_t)l);
    case SHD_T_LONG: return of_i64(l);
    case SHD_T_FLOAT: return of_f32(f);
    case SHD_T_DOUBLE: return of_f64(d);
  }
  throw std::runtime_error("bad cvt target");
}

Val arith(int op, int t, Val l, Val r) {
  Val o;
  if (l.null || r.null) return o;  // math executors return null on a null operand
  o.null = false;
  switch (t) {
    case SHD_T_INT: {
      int32_t a = as_i32(l.b), b = as_i32(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = of_i32((int32_t)((uint32_t)a + (uint32_t)b)); break;
        case SHD_OP_SUB: o.b = of_i32((int32_t)((uint32_t)a - (uint32_t)b)); break;
        case SHD_OP_MUL: o.b = of_i32((int32_t)((uint32_t)a * (uint32_t)b)); break;
        case SHD_OP_DIV:
          if (b == 0) { o.null = true; break; }
          o.b = of_i32((a == INT32_MIN && b == -1) ? INT32_MIN : a / b);
          break;
        case SHD_OP_MOD:
          if (b == 0) { o.null = true; break; }
          o.b = of_i32(b == -1 ? 0 : a % b);
          break;
      }
      break;
    }
    case SHD_T_LONG: {
      int64_t a = as_i64(l.b), b = as_i64(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = (uint64_t)a + (uint64_t)b; break;
        case SHD_OP_SUB: o.b = (uint64_t)a - (uint64_t)b; break;
        case SHD_OP_MUL: o.b = (uint64_t)a * (uint64_t)b; break;
        case SHD_OP_DIV:
          if (b == 0) { o.null = true; break; }
          o.b = of_i64((a == INT64_MIN && b == -1) ? INT64_MIN : a / b);
          break;
        case SHD_OP_MOD:
          if (b == 0) { o.null = true; break; }
          o.b = of_i64(b == -1 ? 0 : a % b);
          break;
      }
      break;
    }
    case SHD_T_FLOAT: {
      float a = as_f32(l.b), b = as_f32(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = of_f32(a + b); break;
        case SHD_OP_SUB: o.b = of_f32(a - b); break;
        case SHD_OP_MUL: o.b = of_f32(a * b); break;
        case SHD_OP_DIV:
          if (b == 0.0f) { o.null = true; break; }
          o.b = of_f32(a / b);
          break;
        case SHD_OP_MOD:
          if (b == 0.0f) { o.null = true; break; }
          o.b = of_f32(std::fmod(a, b));
          break;
      }
      break;
    }
    case SHD_T_DOUBLE: {
      double a = as_f64(l.b), b = as_f64(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = of_f64(a + b); break;
        case SHD_OP_SUB: o.b = of_f64(a - b); break;
        case SHD_OP_MUL: o.b = of_f64(a * b); break;
        case SHD_OP_DIV:
          if (b == 0.0) { o.null = true; break; }
          o.b = of_f64(a / b);
          break;
        case SHD_OP_MOD:
          if (b == 0.0) { o.null = true; break; }
          o.b = of_f64(std::fmod(a, b));
          break;
      }
      break;
    }
  }
  return o;
}

bool compare(int op, int t, uint64_t l, uint64_t r) {
  int c;  // -2 = unordered (NaN)
  switch (t) {
    case SHD_T_STRING: case SHD_T_BOOL:
      c = (l == r) ? 0 : 1;
      if (op == SHD_OP_EQ) return c == 0;
      if (op == SHD_OP_NE) return c != 0;
      throw std::runtime_error("ordering compare on string/bool");
    case SHD_T_INT: { int32_t a = as_i32(l), b = as_i32(r); c = a < b ? -1 : (a > b ? 1 : 0); break; }
    case SHD_T_LONG: { int64_t a = as_i64(l), b = as_i64(r); c = a < b ? -1 : (a > b ? 1 : 0); break; }
    case SHD_T_FLOAT: { float a = as_f32(l), b = as_f32(r);
      c = (a < b) ? -1 : (a > b) ? 1 : (a == b) ? 0 : -2; break; }
    case SHD_T_DOUBLE: { double a = as_f64(l), b = as_f64(r);
      c = (a < b) ? -1 : (a > b) ? 1 : (a == b) ? 0 : -2; break; }
    default: throw std::runtime_error("bad compare type");
  }
  switch (op) {
    case SHD_OP_EQ: return c == 0;
    case SHD_OP_NE: return c != 0;
    case SHD_OP_GT: return c == 1;
    case SHD_OP_GE: return c == 1 || c == 0;
    case SHD_OP_LT: return c == -1;
    case SHD_OP_LE: return c == -1 || c == 0;
  }
  return false;
}

struct EvalCtx {
  SE* se = nullptr;        // state queries
  Ev* ev = nullptr;        // single-stream queries
  const std::vector<Val>* aggs = nullptr;
};

Val load_attr(Ev* e, int attr) {
  Val v;
  if (!e) return v;
  v.null = e->nul[attr] != 0;
  v.b = v.null ? 0 : e->data[attr];
  return v;
}

Val eval(const Plan& p, int expr, const EvalCtx& cx) {
  Val st[64];
  int sp = 0;
  for (const Instr& in : p.exprs[expr]) {
    switch (in.op) {
      case SHD_OP_CONST: st[sp].b = p.consts[in.a]; st[sp].null = false; sp++; break;
      case SHD_OP_NULL: st[sp].b = 0; st[sp].null = true; sp++; break;
      case SHD_OP_LOAD: {
        Ev* e = cx.se ? chain_get(cx.se->ev[in.a], in.b) : cx.ev;
        st[sp++] = load_attr(e, in.c & 0xFFFF);
        break;
      }
      case SHD_OP_EVNULL: {
        Ev* e = cx.se ? chain_get(cx.se->ev[in.a], in.b) : cx.ev;
        st[sp].b = e == nullptr; st[sp].null = false; sp++;
        break;
      }
      case SHD_OP_TS: {
        Ev* e = cx.se ? chain_get(cx.se->ev[in.a], in.b) : cx.ev;
        if (cx.se) {
          st[sp].b = of_i64(cx.se->ts); st[sp].null = false;
        } else {
          st[sp].b = e ? of_i64(e->ts) : 0; st[sp].null = e == nullptr;
        }
        sp++;
        break;
      }
      case SHD_OP_CVT:
        if (!st[sp - 1].null) st[sp - 1].b = cvt(st[sp - 1].b, in.a, in.b);
        break;
      case SHD_OP_ADD: case SHD_OP_SUB: case SHD_OP_MUL: case SHD_OP_DIV: case SHD_OP_MOD: {
        Val r = st[--sp], l = st[--sp];
        st[sp++] = arith(in.op, in.a, l, r);
        break;
      }
      case SHD_OP_EQ: case SHD_OP_NE: case SHD_OP_GT: case SHD_OP_GE: case SHD_OP_LT: case SHD_OP_LE: {
        Val r = st[--sp], l = st[--sp];
        // CompareConditionExpressionExecutor.java:38-42: null operand -> false
        bool res = !(l.null || r.null) && compare(in.op, in.a, l.b, r.b);
        st[sp].b = res; st[sp].null = false; sp++;
        break;
      }
      case SHD_OP_AND: {
        Val r = st[--sp], l = st[--sp];
        bool res = (!l.null && l.b) && (!r.null && r.b);
        st[sp].b = res; st[sp].null = false; sp++;
        break;
      }
      case SHD_OP_OR: {
        Val r = st[--sp], l = st[--sp];
        bool res = (!l.null && l.b) || (!r.null && r.b);
        st[sp].b = res; st[sp].null = false; sp++;
        break;
      }
      case SHD_OP_NOT: {
        Val x = st[--sp];
        st[sp].b = (!x.null && x.b) ? 0 : 1; st[sp].null = false; sp++;
        break;
      }
      case SHD_OP_ISNULL: {
        Val x = st[--sp];
        st[sp].b = x.null; st[sp].null = false; sp++;
        break;
      }
      case SHD_OP_AGG:
        st[sp++] = (*cx.aggs)[in.a];
        break;
      case SHD_OP_IFELSE: {
        // IfThenElseFunctionExecutor.execute(Object[]): Boolean.TRUE.equals(data[0]) ? data[1] : data[2]
        Val e = st[--sp], t = st[--sp], c = st[--sp];
        st[sp++] = (!c.null && c.b) ? t : e;
        break;
      }
      default:
        throw std::runtime_error("bad opcode");
    }
  }
  return sp ? st[sp - 1] : Val{};
}

bool eval_bool(const Plan& p, int expr, const EvalCtx& cx) {
  Val v = eval(p, expr, cx);
  return !v.null && v.b;
}

// ------------------------------------------------------------------ keys
struct Key {
  uint64_t bits = 0;
  int cls = 0;
  bool operator==(const Key& o) const { return bits == o.bits && cls == o.cls; }
  bool operator<(const Key& o) const { return cls != o.cls ? cls < o.cls : bits < o.bits; }
};
struct KeyHash { size_t operator()(const Key& k) const { return std::hash<uint64_t>()(k.bits * 31 + k.cls); } };

// String form identity of a value (ValuePartitionExecutor: toString()).
Key key_of(const Val& v, int type) {
  Key k;
  switch (type) {
    case SHD_T_INT: k.bits = (uint64_t)(int64_t)as_i32(v.b); k.cls = 1; break;
    case SHD_T_LONG: k.bits = v.b; k.cls = 1; break;
    case SHD_T_FLOAT: k.bits = of_f64((double)as_f32(v.b)); k.cls = 2; break;
    case SHD_T_DOUBLE: k.bits = v.b; k.cls = 2; break;
    case SHD_T_BOOL: k.bits = v.b; k.cls = 3; break;
    default: k.bits = v.b; k.cls = 4; break;
  }
  return k;
}

int expr_type(const Plan& p, int expr);

// ------------------------------------------------------------------ outputs
struct OutRow {
  int64_t chunk;
  int type;
  int64_t ts;
  int64_t seq = -1;   // arrival index of the emitting input event (shd_out.in_seq)
  std::vector<uint64_t> vals;
  std::vector<uint8_t> nul;
};

// ====================================================================== NFA
enum PreKind { PK_STREAM = 0, PK_COUNT = 1, PK_LOGICAL = 2, PK_ABSENT = 3, PK_ABSENT_LOGICAL = 4 };

struct Pre {
  int kind = PK_STREAM;
  int stateId = 0;
  bool isStart = false;
  int stream = 0;
  std::vector<int> filters;
  int thisPost = -1;          // thisStatePostProcessor
  int thisLast = -1;          // thisLastProcessor
  int withinEvery = -1;
  int64_t within = UNKNOWN;
  std::vector<int> startStateIds;
  int minC = 0, maxC = 0;     // count
  int ltype = 0;              // logical: 0 AND, 1 OR
  int partner = -1;           // logical partner pre
  int64_t waiting = -1;       // absent
  int sched = -1;             // scheduler index (absent)
};

struct Post {
  int kind = PK_STREAM;
  int pre = -1;               // thisStatePreProcessor
  int stateId = 0;
  int nextPre = -1, nextEvery = -1;
  bool hasSelector = false;   // nextProcessor != null
  int callbackPre = -1;
  int minC = 0, maxC = 0;
  int ltype = 0;
  int partnerPre = -1, partnerPost = -1;
  bool isEventReturned = false;   // field on the (shared) processor object
};

struct PreState {
  std::list<SE*> pending, newEvery;
  bool stateChanged = false, initialized = false, started = false;
  bool successCondition = false, startStateReset = false;   // count
  int64_t lastScheduledTime = 0;                              // absent
  bool active = true;                                         // absent
  int64_t lastArrivalTime = 0;                                // absent logical (LogicalStreamPreState)
};

// Runtime tree (query/input/stream/state/runtime/*InnerStateRuntime.java)
struct Rt {
  int kind;           // NODE_*
  int first;          // first pre
  std::vector<std::unique_ptr<Rt>> kids;
};

struct SchedState {            // Scheduler.SchedulerState
  std::multiset<int64_t> q;    // toNotifyQueue (PriorityBlockingQueue)
};

struct KeyNFA {
  std::vector<PreState> st;
  std::vector<SchedState> sched;
};

struct Engine;

// ====================================================================== engine
struct Engine {
  Plan p;
  std::string err;
  std::vector<OutRow> rows;
  // list arena of SHD_T_OBJECT outputs (handles: offset | count << 40)
  std::vector<uint64_t> lists;
  std::vector<uint8_t> list_nul;
  int64_t chunk_counter = 0;
  int64_t now = 0;            // TimestampGeneratorImpl.lastEventTimestamp (playback)
  int64_t seq = 0;
  std::deque<std::vector<uint64_t>> data_store;
  std::deque<std::vector<uint8_t>> null_store;
  Arena<Ev> ev_arena;
  Arena<SE> se_arena;
  // 0 events, 1 filter evaluations, 2 partials created (start-state matches),
  // 3 matches, 4 out rows, 5 partials expired (`within`)
  int64_t counters[8] = {0};

  // ---- state query structure
  std::vector<Pre> pres;
  std::vector<Post> posts;
  std::unique_ptr<Rt> root;
  std::vector<int> allPre;                          // allStateProcessors (parse order)
  std::vector<std::vector<int>> streamPres;         // receiver -> nextProcessors (setup order)
  std::vector<int> streamCount;
  int n_sched = 0;
  std::vector<int> sched_pre;                       // scheduler -> pre (absent)

  // ---- per-key state
  std::map<Key, std::unique_ptr<KeyNFA>> nfa_keys;  // partitioned
  std::unique_ptr<KeyNFA> nfa_global;
  std::vector<Key> key_order;                       // first-seen order of partition keys
  KeyNFA* cur = nullptr;
  Key cur_key;
  bool partitioned = false;

  // output deferral (MultiProcessStreamReceiver.ReturnEventHolder)
  std::vector<SE*>* holder = nullptr;

  // ================= construction =================
  void build() {
    partitioned = !p.part_keys.empty();
    if (p.kind == SHD_KIND_STATE) build_state();
    else build_single();
    if (!partitioned) {
      start_partition();   // QueryRuntimeImpl.start -> initPartition
    }
  }

  // StateInputStreamParser.parse (C/util/parser/StateInputStreamParser.java:148-408)
  struct ParseRes { int first; int last; std::unique_ptr<Rt> rt; };

  ParseRes parse(Node* n, int preIn, int postIn, bool isStart, std::vector<int>& preList) {
    switch (n->kind) {
      case SHD_NODE_STREAM: {
        int pi = preIn, po = postIn;
        if (pi < 0) {
          Pre pr;
          pr.kind = n->absent ? PK_ABSENT : PK_STREAM;
          if (n->absent) {
            pr.waiting = n->waiting;
            pr.sched = n_sched++;
            sched_pre.push_back((int)pres.size());
          }
          pres.push_back(pr);
          pi = (int)pres.size() - 1;
        }
        pres[pi].stateId = n->state_id;
        pres[pi].isStart = isStart;
        pres[pi].stream = n->stream;
        pres[pi].filters = n->filters;
        if (po < 0) {
          Post ps;
          ps.kind = n->absent ? PK_ABSENT : PK_STREAM;
          posts.push_back(ps);
          po = (int)posts.size() - 1;
        }
        posts[po].stateId = n->state_id;
        posts[po].pre = pi;
        pres[pi].thisPost = po;
        pres[pi].thisLast = po;
        preList.push_back(pi);
        auto rt = std::make_unique<Rt>();
        rt->kind = SHD_NODE_STREAM;
        rt->first = pi;
        return {pi, po, std::move(rt)};
      }
      case SHD_NODE_NEXT: {
        ParseRes a = parse(n->kids[0].get(), preIn, postIn, isStart, preList);
        ParseRes b = parse(n->kids[1].get(), preIn, postIn, false, preList);
        set_next_pre(a.last, b.first);
        auto rt = std::make_unique<Rt>();
        rt->kind = SHD_NODE_NEXT;
        rt->first = a.first;
        rt->kids.push_back(std::move(a.rt));
        rt->kids.push_back(std::move(b.rt));
        return {a.first, b.last, std::move(rt)};
      }
      case SHD_NODE_EVERY: {
        std::vector<int> withinEvery;
        ParseRes a = parse(n->kids[0].get(), preIn, postIn, isStart, withinEvery);
        set_next_every(a.last, a.first);
        for (int x : withinEvery) pres[x].withinEvery = a.first;
        preList.insert(preList.end(), withinEvery.begin(), withinEvery.end());
        auto rt = std::make_unique<Rt>();
        rt->kind = SHD_NODE_EVERY;
        rt->first = a.first;
        rt->kids.push_back(std::move(a.rt));
        return {a.first, a.last, std::move(rt)};
      }
      case SHD_NODE_LOGICAL: {
        Node* s1 = n->kids[0].get();
        Node* s2 = n->kids[1].get();
        if (s1->kind != SHD_NODE_STREAM || s2->kind != SHD_NODE_STREAM)
          throw std::runtime_error("logical children must be streams");
        auto mk = [&](Node* s) {
          Pre pr;
          pr.kind = s->absent ? PK_ABSENT_LOGICAL : PK_LOGICAL;
          pr.ltype = n->ltype;
          if (s->absent) {
            pr.waiting = s->waiting;
            pr.sched = n_sched++;
            sched_pre.push_back((int)pres.size());
          }
          pres.push_back(pr);
          int pi = (int)pres.size() - 1;
          Post ps;
          ps.kind = s->absent ? PK_ABSENT_LOGICAL : PK_LOGICAL;
          ps.ltype = n->ltype;
          posts.push_back(ps);
          return std::make_pair(pi, (int)posts.size() - 1);
        };
        auto p1 = mk(s1);
        auto p2 = mk(s2);
        posts[p1.second].partnerPre = p2.first;
        posts[p2.second].partnerPre = p1.first;
        posts[p1.second].partnerPost = p2.second;
        posts[p2.second].partnerPost = p1.second;
        pres[p1.first].partner = p2.first;
        pres[p2.first].partner = p1.first;
        ParseRes r2 = parse(s2, p2.first, p2.second, isStart, preList);
        ParseRes r1 = parse(s1, p1.first, p1.second, isStart, preList);
        auto rt = std::make_unique<Rt>();
        rt->kind = SHD_NODE_LOGICAL;
        rt->first = r1.first;
        rt->kids.push_back(std::move(r1.rt));
        rt->kids.push_back(std::move(r2.rt));
        return {r1.first, r2.last, std::move(rt)};
      }
      case SHD_NODE_COUNT: {
        int mn = n->min == -1 ? 0 : n->min;
        int mx = n->max == -1 ? INT32_MAX : n->max;
        Pre pr;
        pr.kind = PK_COUNT;
        pr.minC = mn; pr.maxC = mx;
        pres.push_back(pr);
        int pi = (int)pres.size() - 1;
        Post ps;
        ps.kind = PK_COUNT;
        ps.minC = mn; ps.maxC = mx;
        posts.push_back(ps);
        int po = (int)posts.size() - 1;
        ParseRes r = parse(n->kids[0].get(), pi, po, isStart, preList);
        r.rt->kind = SHD_NODE_COUNT;
        return r;
      }
    }
    throw std::runtime_error("bad node");
  }

  void set_next_pre(int post, int pre) {
    // StreamPostStateProcessor / LogicalPostStateProcessor / CountPostStateProcessor.setNextStatePreProcessor
    Post& ps = posts[post];
    ps.nextPre = pre;
    if (ps.kind == PK_LOGICAL || ps.kind == PK_ABSENT_LOGICAL) posts[ps.partnerPost].nextPre = pre;
    if (ps.kind == PK_COUNT) {
      // CountPostStateProcessor.java:79-87
      Pre& me = pres[ps.pre];
      if (me.isStart && p.state_type == 1 && ps.minC == 0) posts[pres[pre].thisPost].callbackPre = ps.pre;
    }
  }

  void set_next_every(int post, int pre) {
    Post& ps = posts[post];
    ps.nextEvery = pre;
    if (ps.kind == PK_LOGICAL || ps.kind == PK_ABSENT_LOGICAL) posts[ps.partnerPost].nextEvery = pre;
  }

  void setup(Rt* r) {
    // InnerStateRuntime.setup(): receiver.setNext(first) + addStatefulProcessorForStream(first)
    switch (r->kind) {
      case SHD_NODE_STREAM: case SHD_NODE_COUNT:
        streamPres[pres[r->first].stream].push_back(r->first);
        break;
      case SHD_NODE_NEXT:
        setup(r->kids[0].get());
        setup(r->kids[1].get());
        break;
      case SHD_NODE_EVERY:
        setup(r->kids[0].get());
        break;
      case SHD_NODE_LOGICAL:
        setup(r->kids[1].get());
        setup(r->kids[0].get());
        break;
    }
  }

  void set_selector(Rt* r) {
    // InnerStateRuntime.setQuerySelector
    switch (r->kind) {
      case SHD_NODE_STREAM: case SHD_NODE_COUNT:
        posts[pres[r->first].thisPost].hasSelector = true;
        break;
      case SHD_NODE_NEXT: set_selector(r->kids[1].get()); break;
      case SHD_NODE_EVERY: set_selector(r->kids[0].get()); break;
      case SHD_NODE_LOGICAL:
        set_selector(r->kids[1].get());
        set_selector(r->kids[0].get());
        break;
    }
  }

  void build_state() {
    std::vector<int> preList;
    ParseRes r = parse(p.root.get(), -1, -1, true, preList);
    root = std::move(r.rt);
    allPre = preList;
    if (p.within >= 0) {
      std::vector<int> starts;
      for (int x : allPre) if (pres[x].isStart) starts.push_back(pres[x].stateId);
      for (int x : allPre) { pres[x].startStateIds = starts; pres[x].within = p.within; }
    }
    pres[r.first].thisLast = r.last;   // StateInputStreamParser.java:142-143
    streamPres.assign(p.stream_types.size(), {});
    set_selector(root.get());
    setup(root.get());
  }

  KeyNFA* new_key_nfa() {
    auto k = new KeyNFA();
    k->st.resize(pres.size());
    k->sched.resize(n_sched);
    return k;
  }

  PreState& S(int pre) { return cur->st[pre]; }

  SE* new_se() {
    SE* s = se_arena.get();
    s->ev.assign(p.n_states, nullptr);
    s->ts = -1;
    s->type = CURRENT;
    s->next = nullptr;
    return s;
  }

  SE* clone_se(SE* o) {   // StateEventCloner.copyStateEvent
    SE* s = se_arena.get();
    s->ev = o->ev;
    s->ts = o->ts;
    s->type = o->type;
    s->next = nullptr;
    return s;
  }

  Ev* clone_ev(Ev* o) {   // StreamEventCloner.copyStreamEvent
    Ev* e = ev_arena.get();
    *e = *o;
    e->next = nullptr;
    return e;
  }

  // ---------------- StreamPreStateProcessor ----------------
  bool isExpired(int pre, SE* s, int64_t t) {
    Pre& pr = pres[pre];
    if (pr.within != UNKNOWN) {
      for (int sid : pr.startStateIds) {
        Ev* e = s->ev[sid];
        if (e != nullptr && std::llabs(e->ts - t) > pr.within) return true;
      }
    }
    return false;
  }

  void init_pre(int pre) {
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    Post& ps = posts[pr.thisPost];
    if (pr.isStart && (!st.initialized || ps.nextEvery >= 0 ||
                       (p.state_type == 1 && ps.nextPre >= 0 &&
                        (pres[ps.nextPre].kind == PK_ABSENT || pres[ps.nextPre].kind == PK_ABSENT_LOGICAL)))) {
      SE* s = new_se();
      addState(pre, s);
      st.initialized = true;
    }
  }

  void addState(int pre, SE* s) {
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    switch (pr.kind) {
      case PK_STREAM:
        if (p.state_type == 1) {
          if (st.newEvery.empty()) st.newEvery.push_back(s);
        } else {
          st.newEvery.push_back(s);
        }
        break;
      case PK_COUNT: {
        if (p.state_type == 1) {
          if (st.newEvery.empty()) st.newEvery.push_back(s);
        } else {
          st.newEvery.push_back(s);
        }
        if (pr.minC == 0 && s->ev[pr.stateId] == nullptr) {
          // CountPreStateProcessor.addState :126-137
          countProcessMinCountReached(pr.thisPost, s);
        }
        break;
      }
      case PK_LOGICAL:
        logicalAddState(pre, s);
        break;
      case PK_ABSENT_LOGICAL:
        // AbsentLogicalPreStateProcessor.addState (:77-99): inactive -> dropped
        if (!S(pre).active) break;
        logicalAddState(pre, s);
        break;
      case PK_ABSENT:
        absentAddState(pre, s);
        break;
    }
  }

  void addEveryState(int pre, SE* s) {
    Pre& pr = pres[pre];
    SE* c = clone_se(s);
    c->type = CURRENT;
    if (pr.kind == PK_ABSENT_LOGICAL) {
      // AbsentLogicalPreStateProcessor.addEveryState (:101-119): the clone takes
      // the time of the event this processor saw; only the pair's slots clear
      if (c->ev[pr.stateId] != nullptr) c->ts = c->ev[pr.stateId]->ts;
      c->ev[pr.stateId] = nullptr;
      c->ev[pres[pr.partner].stateId] = nullptr;
      S(pre).newEvery.push_back(c);
      S(pr.partner).newEvery.push_back(c);
      return;
    }
    if (pr.kind == PK_LOGICAL) {
      c->ev[pr.stateId] = nullptr;
      for (int i = pr.stateId; i < (int)c->ev.size(); i++) c->ev[i] = nullptr;
      S(pre).newEvery.push_back(c);
      if (pr.partner >= 0) {
        c->ev[pres[pr.partner].stateId] = nullptr;
        S(pr.partner).newEvery.push_back(c);
      }
      return;
    }
    for (int i = pr.stateId; i < (int)c->ev.size(); i++) c->ev[i] = nullptr;
    S(pre).newEvery.push_back(c);
    if (pr.kind == PK_ABSENT) {
      PreState& st = S(pre);
      st.lastScheduledTime = s->ts + pr.waiting;
      notifyAt(pr.sched, st.lastScheduledTime);
    }
  }

  void stateChanged(int pre) { S(pre).stateChanged = true; }

  void resetState(int pre) {
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    switch (pr.kind) {
      case PK_STREAM: case PK_COUNT: {
        st.pending.clear();
        if (pr.isStart && st.newEvery.empty()) {
          Post& ps = posts[pr.thisPost];
          if (p.state_type == 1 && ps.nextEvery < 0 && ps.nextPre >= 0 && !S(ps.nextPre).pending.empty())
            return;
          init_pre(pre);
        }
        break;
      }
      case PK_LOGICAL: case PK_ABSENT_LOGICAL: {
        if (pr.ltype == 1 || st.pending.size() == S(pr.partner).pending.size()) {
          st.pending.clear();
          S(pr.partner).pending.clear();
          if (pr.isStart && st.newEvery.empty()) {
            Post& ps = posts[pr.thisPost];
            if (p.state_type == 1 && ps.nextEvery < 0 && ps.nextPre >= 0 && !S(ps.nextPre).pending.empty())
              return;
            init_pre(pre);
          }
        }
        break;
      }
      case PK_ABSENT: {
        st.pending.clear();
        if (pr.isStart) {
          Post& ps = posts[pr.thisPost];
          if (p.state_type == 1 && ps.nextEvery < 0 && ps.nextPre >= 0 && !S(ps.nextPre).pending.empty())
            return;
          init_pre(pre);
        }
        break;
      }
    }
  }

  static void stable_sort_ts(std::list<SE*>& l) {
    // StreamPreStateProcessor.eventTimeComparator (-1 sorts last); List.sort is stable.
    l.sort([](SE* a, SE* b) {
      if (a->ts == -1) return false;
      if (b->ts == -1) return true;
      return a->ts < b->ts;
    });
  }

  void updateState(int pre) {
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (pr.kind == PK_COUNT && st.startStateReset) {
      st.startStateReset = false;
      init_pre(pre);
    }
    stable_sort_ts(st.newEvery);
    st.pending.splice(st.pending.end(), st.newEvery);
    if (pr.kind == PK_LOGICAL || pr.kind == PK_ABSENT_LOGICAL) {
      PreState& ps = S(pr.partner);
      stable_sort_ts(ps.newEvery);
      ps.pending.splice(ps.pending.end(), ps.newEvery);
    }
  }

  void expireEvents(int pre, int64_t t) {
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    SE* expired = nullptr;
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      SE* s = *it;
      if (isExpired(pre, s, t)) {
        it = st.pending.erase(it);
        counters[5]++;
        if (s->type != EXPIRED) { s->type = EXPIRED; expired = s; }
      } else {
        break;
      }
    }
    for (auto it = st.newEvery.begin(); it != st.newEvery.end();) {
      SE* s = *it;
      if (isExpired(pre, s, t)) {
        it = st.newEvery.erase(it);
        counters[5]++;
        if (s->type != EXPIRED) { s->type = EXPIRED; expired = s; }
      } else {
        ++it;
      }
    }
    if (expired && pr.withinEvery >= 0) {
      addEveryState(pr.withinEvery, expired);
      updateState(pr.withinEvery);
    }
  }

  // process(stateEvent): filter chain then post processor (StreamPreStateProcessor.java:131-142)
  void processChain(int pre, SE* s) {
    Pre& pr = pres[pre];
    S(pre).stateChanged = false;
    EvalCtx cx;
    cx.se = s;
    for (int f : pr.filters) {
      counters[1]++;
      if (!eval_bool(p, f, cx)) return;
    }
    if (pr.isStart) counters[2]++;
    postProcess(pr.thisPost, s);
  }

  // ---------------- Post processors ----------------
  void postProcess(int post, SE* s) {
    Post& ps = posts[post];
    switch (ps.kind) {
      case PK_STREAM: streamPost(post, s); break;
      case PK_COUNT: countPost(post, s); break;
      case PK_LOGICAL: logicalPost(post, s); break;
      case PK_ABSENT_LOGICAL: absentLogicalPost(post, s); break;
      case PK_ABSENT: absentPost(post, s); break;
    }
  }

  void streamPost(int post, SE* s) {
    // StreamPostStateProcessor.process (StreamPostStateProcessor.java:64-83)
    Post& ps = posts[post];
    stateChanged(ps.pre);
    Ev* e = s->ev[ps.stateId];
    s->ts = e->ts;
    if (ps.hasSelector) ps.isEventReturned = true;
    if (ps.nextPre >= 0) addState(ps.nextPre, s);
    if (ps.nextEvery >= 0) addEveryState(ps.nextEvery, s);
    if (ps.callbackPre >= 0) countStartStateReset(ps.callbackPre);
  }

  void countPost(int post, SE* s) {
    // CountPostStateProcessor.process (CountPostStateProcessor.java:39-67)
    Post& ps = posts[post];
    Ev* e = s->ev[ps.stateId];
    int n = 1;
    while (e->next) { n++; e = e->next; }
    S(ps.pre).successCondition = true;
    s->ts = e->ts;
    if (n >= ps.minC) {
      if (p.state_type == 1) {
        if (ps.nextPre >= 0) addState(ps.nextPre, s);
        if (n != ps.maxC) addState(ps.pre, s);
      } else if (n == ps.minC) {
        countProcessMinCountReached(post, s);
      }
      if (n == ps.maxC) stateChanged(ps.pre);
    }
  }

  void countProcessMinCountReached(int post, SE* s) {
    Post& ps = posts[post];
    if (ps.hasSelector) {
      stateChanged(ps.pre);
      ps.isEventReturned = true;
    }
    if (ps.nextPre >= 0) addState(ps.nextPre, s);
    if (ps.nextEvery >= 0) addEveryState(ps.nextEvery, s);
  }

  void countStartStateReset(int pre) {
    // CountPreStateProcessor.startStateReset
    S(pre).startStateReset = true;
    Post& ps = posts[pres[pre].thisPost];
    if (ps.callbackPre >= 0) countStartStateReset(posts[pres[pre].thisPost].pre);
  }

  void logicalPost(int post, SE* s) {
    // LogicalPostStateProcessor.process (LogicalPostStateProcessor.java:59-86);
    // the post of an absent operand is absentLogicalPost
    Post& ps = posts[post];
    if (ps.ltype == 0) {
      bool proceed = false;
      if (pres[ps.partnerPre].kind == PK_ABSENT_LOGICAL) {
        proceed = absentPartnerCanProceed(ps.partnerPre, s);
      } else if (s->ev[pres[ps.partnerPre].stateId] != nullptr) {
        proceed = true;
      }
      if (proceed) {
        streamPost(post, s);
      } else {
        stateChanged(ps.pre);
      }
    } else {
      streamPost(post, s);
      Post& pp = posts[ps.partnerPost];
      if (pp.hasSelector && pres[ps.pre].thisLast == ps.partnerPost) pp.isEventReturned = true;
    }
  }

  // ---------------- processAndReturn ----------------
  std::vector<SE*> processAndReturn(int pre, Ev* ev) {
    Pre& pr = pres[pre];
    switch (pr.kind) {
      case PK_STREAM: return streamProcessAndReturn(pre, ev, true);
      case PK_COUNT: return countProcessAndReturn(pre, ev);
      case PK_LOGICAL: return logicalProcessAndReturn(pre, ev);
      case PK_ABSENT: {
        if (!S(pre).active) return {};
        auto r = streamProcessAndReturn(pre, ev, false);
        return {};   // always empty (AbsentStreamPreStateProcessor.java:257-274)
      }
      case PK_ABSENT_LOGICAL: return absentLogicalProcessAndReturn(pre, ev);
    }
    return {};
  }

  std::vector<SE*> streamProcessAndReturn(int pre, Ev* ev, bool removeOnNoChangeSeq) {
    // StreamPreStateProcessor.processAndReturn (:364-403)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    std::vector<SE*> ret;
    Post& last = posts[pr.thisLast];
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      SE* s = *it;
      Ev* c = clone_ev(ev);
      s->ev[pr.stateId] = c;
      processChain(pre, s);
      if (last.isEventReturned) {
        last.isEventReturned = false;
        ret.push_back(s);
      }
      if (st.stateChanged) {
        it = st.pending.erase(it);
      } else {
        if (s->ev[pr.stateId] == c) { s->ev[pr.stateId] = nullptr; ev_arena.put(c); }
        else s->ev[pr.stateId] = nullptr;
        if (p.state_type == 1) {
          if (removeOnNoChangeSeq) it = st.pending.erase(it);
          else ++it;
          Post& tp = posts[pr.thisPost];
          if (tp.callbackPre >= 0) countStartStateReset(tp.callbackPre);
        } else {
          ++it;
        }
      }
    }
    return ret;
  }

  std::vector<SE*> countProcessAndReturn(int pre, Ev* ev) {
    // CountPreStateProcessor.processAndReturn (:52-94)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    std::vector<SE*> ret;
    Post& last = posts[pr.thisLast];
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      SE* s = *it;
      bool removed = false;
      for (int pos : {pr.stateId + 1, pr.stateId + 2}) {
        if ((int)s->ev.size() > pos && s->ev[pos] != nullptr) {
          it = st.pending.erase(it);
          removed = true;
          break;
        }
      }
      if (removed) continue;
      Ev* c = clone_ev(ev);
      // StateEvent.addEvent
      if (s->ev[pr.stateId] == nullptr) s->ev[pr.stateId] = c;
      else { Ev* x = s->ev[pr.stateId]; while (x->next) x = x->next; x->next = c; }
      st.successCondition = false;
      processChain(pre, s);
      if (last.isEventReturned) {
        last.isEventReturned = false;
        ret.push_back(s);
      }
      bool erased = false;
      if (st.stateChanged) {
        it = st.pending.erase(it);
        erased = true;
      }
      if (!st.successCondition) {
        // StateEvent.removeLastEvent
        Ev* x = s->ev[pr.stateId];
        if (x) {
          bool done = false;
          while (x->next) {
            if (x->next->next == nullptr) { x->next = nullptr; done = true; break; }
            x = x->next;
          }
          if (!done) s->ev[pr.stateId] = nullptr;
        }
        if (p.state_type == 1 && !erased) {
          it = st.pending.erase(it);
          erased = true;
        }
      }
      if (!erased) ++it;
    }
    return ret;
  }

  // ---------------- Logical ----------------
  void logicalAddState(int pre, SE* s) {
    // LogicalPreStateProcessor.addState (:43-63)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (pr.isStart || p.state_type == 1) {
      if (st.newEvery.empty()) st.newEvery.push_back(s);
      if (pr.partner >= 0 && S(pr.partner).newEvery.empty()) S(pr.partner).newEvery.push_back(s);
    } else {
      st.newEvery.push_back(s);
      if (pr.partner >= 0) S(pr.partner).newEvery.push_back(s);
    }
    if (pr.kind == PK_ABSENT_LOGICAL && !pr.isStart && pr.waiting != -1) {
      // AbsentLogicalPreStateProcessor.addState: schedule this processor (and an
      // absent partner) at the partial's time + waiting
      notifyAt(pr.sched, s->ts + pr.waiting);
      const Pre& pp = pres[pr.partner];
      if (pp.kind == PK_ABSENT_LOGICAL) notifyAt(pp.sched, s->ts + pp.waiting);
    }
  }

  std::vector<SE*> logicalProcessAndReturn(int pre, Ev* ev) {
    // LogicalPreStateProcessor.processAndReturn (:113-154)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    std::vector<SE*> ret;
    Post& last = posts[pr.thisLast];
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      SE* s = *it;
      if (pr.ltype == 1 && s->ev[pres[pr.partner].stateId] != nullptr) {
        it = st.pending.erase(it);
        continue;
      }
      Ev* c = clone_ev(ev);
      s->ev[pr.stateId] = c;
      processChain(pre, s);
      if (last.isEventReturned) {
        last.isEventReturned = false;
        ret.push_back(s);
      }
      if (st.stateChanged) {
        it = st.pending.erase(it);
      } else {
        s->ev[pr.stateId] = nullptr;
        if (p.state_type == 1) it = st.pending.erase(it);
        else ++it;
      }
    }
    return ret;
  }

  // ---------------- Absent (stream) ----------------
  void absentAddState(int pre, SE* s) {
    // AbsentStreamPreStateProcessor.addState (:67-88)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (!st.active) return;
    if (p.state_type == 1) {
      st.newEvery.clear();
      st.newEvery.push_back(s);
    } else {
      st.newEvery.push_back(s);
    }
    if (!pr.isStart) {
      st.lastScheduledTime = s->ts + pr.waiting;
      notifyAt(pr.sched, st.lastScheduledTime);
    }
  }

  void absentPost(int post, SE* s) {
    // AbsentStreamPostStateProcessor.process
    Post& ps = posts[post];
    stateChanged(ps.pre);
    Ev* e = s->ev[ps.stateId];
    s->ts = e->ts;
    ps.isEventReturned = true;
    Pre& pr = pres[ps.pre];
    if (pr.isStart && ps.nextEvery >= 0 && ps.nextEvery == ps.pre) addEveryState(ps.nextEvery, s);
    // updateLastArrivalTime
    PreState& st = S(ps.pre);
    st.lastScheduledTime = e->ts + pr.waiting;
    notifyAt(pr.sched, st.lastScheduledTime);
  }

  void absentTimer(int pre, int64_t currentTime) {
    // AbsentStreamPreStateProcessor.process(ComplexEventChunk) on a TIMER (:150-227)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (!st.active) return;
    std::vector<SE*> ret;
    Post& tp = posts[pr.thisPost];
    bool initialize = pr.isStart && st.newEvery.empty() && st.pending.empty();
    if (initialize && p.state_type == 1 && tp.nextEvery < 0 && st.lastScheduledTime > 0) initialize = false;
    if (initialize) {
      SE* s = new_se();
      addState(pre, s);
    } else if (p.state_type == 1 && !st.newEvery.empty()) {
      resetState(pre);
    }
    updateState(pre);
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      SE* s = *it;
      if (isExpired(pre, s, currentTime)) {
        it = st.pending.erase(it);
        if (pr.withinEvery >= 0 && tp.nextEvery != pre) addEveryState(tp.nextEvery, s);
        continue;
      }
      if ((s->ts == -1 && currentTime >= st.lastScheduledTime) ||
          (s->ts != -1 && currentTime >= s->ts + pr.waiting)) {
        it = st.pending.erase(it);
        s->ts = currentTime;
        ret.push_back(s);
        continue;
      }
      ++it;
    }
    if (pr.withinEvery >= 0) updateState(pr.withinEvery);
    bool notProcessed = ret.empty();
    for (SE* s : ret) absentSendEvent(pre, s);
    int64_t actual = now;
    if (actual > pr.waiting + currentTime) st.lastScheduledTime = actual + pr.waiting;
    if (notProcessed && st.lastScheduledTime < currentTime) {
      st.lastScheduledTime = currentTime + pr.waiting;
      notifyAt(pr.sched, st.lastScheduledTime);
    }
  }

  void absentSendEvent(int pre, SE* s) {
    Pre& pr = pres[pre];
    Post& tp = posts[pr.thisPost];
    PreState& st = S(pre);
    if (tp.hasSelector) selectorEmitImmediate(s);
    if (tp.nextPre >= 0) addState(tp.nextPre, s);
    if (tp.nextEvery >= 0) addEveryState(tp.nextEvery, s);
    else if (pr.isStart) st.active = false;
    if (tp.callbackPre >= 0) countStartStateReset(tp.callbackPre);
  }

  void partitionCreatedAbsent(int pre) {
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (!st.started) {
      st.started = true;
      if (pr.kind == PK_ABSENT) {
        if (pr.isStart && pr.waiting != -1 && st.active) {
          st.lastScheduledTime = now + pr.waiting;
          notifyAt(pr.sched, st.lastScheduledTime);
        }
      } else {
        absentLogicalPartitionCreated(pre);
      }
    }
  }

  // ---------------- Absent logical (not X [for t] and|or Y) ----------------
  // AbsentLogicalPreStateProcessor (ST/AbsentLogicalPreStateProcessor.java:65-388)
  // and AbsentLogicalPostStateProcessor.

  // a fresh StreamEvent (streamEventFactory.newInstance(): ts -1, no data)
  Ev* empty_ev() {
    static const uint64_t zeros[64] = {0};
    static const uint8_t ones[64] = {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1};
    Ev* e = ev_arena.get();
    *e = Ev();
    e->ts = -1;
    e->data = zeros;
    e->nul = ones;
    return e;
  }

  static void add_event(SE* s, int sid, Ev* e) {   // StateEvent.addEvent
    if (s->ev[sid] == nullptr) { s->ev[sid] = e; return; }
    Ev* x = s->ev[sid];
    while (x->next) x = x->next;
    x->next = e;
  }

  void absentLogicalPost(int post, SE* s) {
    // AbsentLogicalPostStateProcessor.process: state changed, event returned,
    // updateLastArrivalTime (:36-50) -- no partner check
    Post& ps = posts[post];
    stateChanged(ps.pre);
    ps.isEventReturned = true;
    S(ps.pre).lastArrivalTime = s->ev[ps.stateId]->ts;
  }

  std::vector<SE*> absentLogicalProcessAndReturn(int pre, Ev* ev) {
    // AbsentLogicalPreStateProcessor.processAndReturn (:243-296): an X arrival
    // takes the partials it passes out of this processor's pending list; never
    // returns events itself
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (!st.active) return {};
    Post& last = posts[pr.thisLast];
    Post& tp = posts[pr.thisPost];
    const int psid = pres[pr.partner].stateId;
    for (auto it = st.pending.begin(); it != st.pending.end();) {
      SE* s = *it;
      if (pr.ltype == 1 && s->ev[psid] != nullptr) {
        it = st.pending.erase(it);
        continue;
      }
      Ev* curEv = s->ev[pr.stateId];
      s->ev[pr.stateId] = clone_ev(ev);
      processChain(pre, s);
      if (pr.waiting != -1 || (p.state_type == 1 && pr.ltype == 0 && tp.nextEvery >= 0)) s->ev[pr.stateId] = curEv;
      bool erased = false;
      if (last.isEventReturned) {
        last.isEventReturned = false;
        it = st.pending.erase(it);
        erased = true;
        if (p.state_type == 1) S(pr.partner).pending.remove(s);
      }
      if (!st.stateChanged) {
        s->ev[pr.stateId] = curEv;
        if (p.state_type == 1 && !erased) {
          it = st.pending.erase(it);
          erased = true;
        }
      }
      if (!erased) ++it;
    }
    return {};
  }

  bool absentPartnerCanProceed(int pre, SE* s) {
    // AbsentLogicalPreStateProcessor.partnerCanProceed (:353-388)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    Post& tp = posts[pr.thisPost];
    if (p.state_type == 1 && tp.nextEvery < 0 && st.lastArrivalTime > 0) return false;
    if (pr.waiting == -1) {
      if (tp.nextEvery < 0) return s->ev[pr.stateId] == nullptr;
      if (st.lastArrivalTime > 0) {
        st.lastArrivalTime = 0;
        init_pre(pre);
        return false;
      }
      return true;
    }
    return s->ev[pr.stateId] != nullptr;
  }

  void absentLogicalSendEvent(int pre, SE* s) {
    // AbsentLogicalPreStateProcessor.sendEvent (:231-253)
    Pre& pr = pres[pre];
    Post& tp = posts[pr.thisPost];
    if (tp.hasSelector) selectorEmitImmediate(s);
    if (tp.nextPre >= 0) addState(tp.nextPre, s);
    if (tp.nextEvery >= 0) {
      addEveryState(tp.nextEvery, s);
    } else if (pr.isStart) {
      S(pre).active = false;
      if (pr.ltype == 1 && pres[pr.partner].kind == PK_ABSENT_LOGICAL) S(pr.partner).active = false;
    }
    if (tp.callbackPre >= 0) countStartStateReset(tp.callbackPre);
  }

  void absentLogicalTimer(int pre, int64_t currentTime) {
    // AbsentLogicalPreStateProcessor.process(ComplexEventChunk) on a TIMER (:122-218)
    Pre& pr = pres[pre];
    PreState& st = S(pre);
    if (!st.active) return;
    Post& tp = posts[pr.thisPost];
    const int psid = pres[pr.partner].stateId;
    bool notProcessed = true;
    if (currentTime >= st.lastArrivalTime + pr.waiting) {
      if (pr.isStart && p.state_type == 1 && st.newEvery.empty() && st.pending.empty()) {
        addState(pre, new_se());
      } else if (p.state_type == 1 && !st.newEvery.empty()) {
        resetState(pre);
      }
      updateState(pre);
      SE* expired = nullptr;
      std::vector<SE*> ret;
      for (auto it = st.pending.begin(); it != st.pending.end();) {
        SE* s = *it;
        if (isExpired(pre, s, currentTime)) {
          expired = s;
          it = st.pending.erase(it);
          continue;
        }
        Ev* own = s->ev[pr.stateId];
        const bool passed = own == nullptr ? currentTime >= s->ts + pr.waiting : currentTime >= own->ts + pr.waiting;
        if (passed) {
          it = st.pending.erase(it);
          if (pr.ltype == 1 && s->ev[psid] == nullptr) {          // OR: partner not received
            add_event(s, pr.stateId, empty_ev());
            ret.push_back(s);
          } else if (pr.ltype == 0 && s->ev[psid] != nullptr) {   // AND: partner received, not sent
            ret.push_back(s);
          } else if (pr.ltype == 0) {                              // AND: let the partner proceed
            add_event(s, pr.stateId, empty_ev());
          }
          continue;
        }
        ++it;
      }
      if (expired && pr.withinEvery >= 0) {
        addEveryState(pr.withinEvery, expired);
        updateState(pr.withinEvery);
      }
      notProcessed = ret.empty();
      for (SE* s : ret) {
        s->ts = currentTime;
        absentLogicalSendEvent(pre, s);
      }
      st.lastArrivalTime = 0;
    }
    if (tp.nextEvery >= 0 || (notProcessed && pr.isStart)) {
      const int64_t nextBreak = st.lastArrivalTime == 0 ? now + pr.waiting : st.lastArrivalTime + pr.waiting;
      notifyAt(pr.sched, nextBreak);
    }
  }

  void absentLogicalPartitionCreated(int pre) {
    // AbsentLogicalPreStateProcessor.partitionCreated (:318-335)
    Pre& pr = pres[pre];
    if (pr.isStart && pr.waiting != -1 && S(pre).active) notifyAt(pr.sched, now + pr.waiting);
  }

  // ---------------- runtimes ----------------
  void rt_init(Rt* r) {
    switch (r->kind) {
      case SHD_NODE_STREAM: case SHD_NODE_COUNT: init_pre(r->first); break;
      case SHD_NODE_NEXT: rt_init(r->kids[0].get()); rt_init(r->kids[1].get()); break;
      case SHD_NODE_EVERY: rt_init(r->kids[0].get()); break;
      case SHD_NODE_LOGICAL: rt_init(r->kids[1].get()); rt_init(r->kids[0].get()); break;
    }
  }
  void rt_reset(Rt* r) {
    switch (r->kind) {
      case SHD_NODE_STREAM: case SHD_NODE_COUNT: case SHD_NODE_EVERY: resetState(r->first); break;
      case SHD_NODE_NEXT: rt_reset(r->kids[1].get()); rt_reset(r->kids[0].get()); break;
      case SHD_NODE_LOGICAL: rt_reset(r->kids[1].get()); break;
    }
  }
  void rt_update(Rt* r) {
    switch (r->kind) {
      case SHD_NODE_STREAM: case SHD_NODE_COUNT: case SHD_NODE_EVERY: updateState(r->first); break;
      case SHD_NODE_NEXT: rt_update(r->kids[0].get()); rt_update(r->kids[1].get()); break;
      case SHD_NODE_LOGICAL: rt_update(r->kids[1].get()); break;
    }
  }

  // StateStreamRuntime.initPartition
  void start_partition() {
    if (p.kind != SHD_KIND_STATE) return;
    if (partitioned) {
      // called with cur set
    } else {
      nfa_global.reset(new_key_nfa());
      cur = nfa_global.get();
    }
    rt_init(root.get());
    for (int i = 0; i < (int)pres.size(); i++)
      if (pres[i].kind == PK_ABSENT || pres[i].kind == PK_ABSENT_LOGICAL) partitionCreatedAbsent(i);
  }

  // ---------------- receivers ----------------
  void stabilize(int stream, int64_t ts) {
    for (int x : allPre) expireEvents(x, ts);
    if (p.state_type == 0) {
      if (streamCountOf(stream) > 1) {
        for (int x : streamPres[stream]) updateState(x);
      } else if (!streamPres[stream].empty()) {
        updateState(streamPres[stream][0]);
      }
    } else {
      rt_reset(root.get());
      rt_update(root.get());
    }
  }

  int streamCountOf(int stream) { return (int)streamPres[stream].size(); }

  // Process one run of events of one stream under the current key state.
  void state_run(int stream, const std::vector<Ev*>& evs) {
    auto& procs = streamPres[stream];
    if (procs.empty()) return;
    if (procs.size() > 1) {
      // MultiProcessStreamReceiver.receive: per event, states in reverse order;
      // outputs deferred per (event, state) holder until the run ends.
      std::vector<std::vector<OutRow>> holders;
      for (Ev* e : evs) {
        counters[0]++;
        cur_seq = e->seq;
        stabilize(stream, e->ts);
        for (int k = (int)procs.size() - 1; k >= 0; k--) {
          Ev* ce = clone_ev(e);
          std::vector<SE*> r = processAndReturn(procs[k], ce);
          // StateMultiProcessStreamReceiver.processAndClear: the selector runs
          // now (output data is populated at match time), the callback later.
          std::vector<OutRow> h;
          for (SE* s : r) {
            OutRow row;
            if (select_row(s, row)) h.push_back(std::move(row));
          }
          if (!h.empty()) holders.push_back(std::move(h));
        }
      }
      for (auto& h : holders) {
        int64_t cid = chunk_counter++;
        for (auto& row : h) { row.chunk = cid; rows.push_back(std::move(row)); counters[3]++; }
      }
    } else {
      // SingleProcessStreamReceiver.processAndClear: whole chunk, then one
      // selector call (and callback) per returned event.
      std::vector<SE*> ret;
      for (Ev* e : evs) {
        counters[0]++;
        cur_seq = e->seq;
        stabilize(stream, e->ts);
        Ev* ce = clone_ev(e);
        std::vector<SE*> r = processAndReturn(procs[0], ce);
        ret.insert(ret.end(), r.begin(), r.end());
      }
      for (SE* s : ret) emitChunk({s});
    }
  }

  int64_t cur_seq = 0;   // the event being processed (timers: the next event's index)

  // QuerySelector.process over a chunk of ONE StateEvent: the receivers hand
  // every returned StateEvent to the selector on its own
  // (StateMultiProcessStreamReceiver.processAndClear, C/query/input/
  // StateMultiProcessStreamReceiver.java:47-68; SingleProcessStreamReceiver
  // .java:48-72; AbsentStreamPreStateProcessor.java:240).  isBatch() is always
  // true (C/event/ComplexEventChunk.java:265-270), so: group by ->
  // processInBatchGroupBy, aggregators -> processInBatchNoGroupBy, else
  // processNoGroupBy (QuerySelector.java:76-99).  For one event all three keep
  // it iff, after the aggregators folded it in (CURRENT adds, EXPIRED
  // removes), `having` holds and its type is selected (:161-205, :271-373).
  bool select_row(SE* s, OutRow& r) {
    if (s->type != CURRENT && s->type != EXPIRED) return false;   // TIMER / RESET
    EvalCtx cx;
    cx.se = s;
    if (!p.aggs.empty()) {
      run_aggs_ctx(state_aggs, cx, s->type);
      cx.aggs = &agg_vals;
    }
    r = OutRow();
    r.seq = cur_seq;
    r.chunk = -1;
    r.type = s->type;
    r.ts = s->ts;
    for (auto& o : p.outputs) {
      const auto& code = p.exprs[o.second];
      if (code.size() == 1 && code[0].op == SHD_OP_MULTI) {
        // MultiValueVariableFunctionExecutor.execute (C/executor/
        // MultiValueVariableFunctionExecutor.java:64-72): getStreamEvent(position)
        // (index 0: the chain head), then every getNext(), into a List
        const uint64_t off = lists.size();
        uint64_t cnt = 0;
        for (Ev* x = s->ev[code[0].a]; x; x = x->next, cnt++) {
          Val v = load_attr(x, code[0].c & 0xFFFF);
          lists.push_back(v.b);
          list_nul.push_back(v.null);
        }
        r.vals.push_back(cnt ? (off | (cnt << 40)) : 0);
        r.nul.push_back(0);
        continue;
      }
      Val v = eval(p, o.second, cx);
      r.vals.push_back(v.b);
      r.nul.push_back(v.null);
    }
    if (p.having >= 0 && !eval_bool(p, p.having, cx)) return false;
    if (s->type == CURRENT) return p.current_on;
    return p.expired_on;
  }

  // one callback chunk of the selected rows (none: no callback)
  void emitChunk(const std::vector<SE*>& ss) {
    std::vector<OutRow> sel;
    for (SE* s : ss) {
      OutRow r;
      if (select_row(s, r)) sel.push_back(std::move(r));
    }
    if (sel.empty()) return;
    int64_t cid = chunk_counter++;
    for (auto& r : sel) {
      r.chunk = cid;
      rows.push_back(std::move(r));
      counters[3]++;
    }
  }

  void selectorEmitImmediate(SE* s) { emitChunk({s}); }

  // ---------------- scheduler (playback) ----------------
  void notifyAt(int sched, int64_t t) {
    cur->sched[sched].q.insert(t);
    sched_keys_dirty = true;
  }
  bool sched_keys_dirty = false;

  // Scheduler.onTimeChange for every scheduler of the query, in creation order.
  void onTimeChange(int64_t t) {
    if (p.kind == SHD_KIND_STATE) {
      for (int sc = 0; sc < n_sched; sc++) {
        // collect (time, key) with head <= t, sorted by time
        std::vector<std::pair<int64_t, KeyNFA*>> due;
        std::vector<Key> dkeys;
        if (partitioned) {
          for (auto& kv : nfa_keys) {
            auto& q = kv.second->sched[sc].q;
            if (!q.empty() && *q.begin() <= t) due.push_back({*q.begin(), kv.second.get()});
          }
        } else if (nfa_global) {
          auto& q = nfa_global->sched[sc].q;
          if (!q.empty() && *q.begin() <= t) due.push_back({*q.begin(), nfa_global.get()});
        }
        std::stable_sort(due.begin(), due.end(), [](auto& a, auto& b) { return a.first < b.first; });
        for (auto& d : due) {
          cur = d.second;
          auto& q = cur->sched[sc].q;
          while (!q.empty() && *q.begin() - now <= 0) {
            int64_t nt = *q.begin();
            q.erase(q.begin());
            if (pres[sched_pre[sc]].kind == PK_ABSENT_LOGICAL) absentLogicalTimer(sched_pre[sc], nt);
            else absentTimer(sched_pre[sc], nt);
          }
        }
      }
    } else {
      single_on_time_change(t);
    }
  }

  void set_time(int64_t t) {
    // TimestampGeneratorImpl.setCurrentTimestamp: only moves forward.
    cur_seq = seq;   // timer rows: before the next event
    if (t >= now) {
      now = t;
      onTimeChange(t);
    }
  }

  // ================= single-stream queries =================
  struct AggState { double dsum = 0; int64_t lsum = 0; int64_t count = 0; };
  struct GroupAgg { std::vector<AggState> a; };
  struct KeySingle {
    // LengthWindowProcessor / TimeWindowProcessor state
    int64_t count = 0;
    std::deque<Ev*> q;
    int64_t lastTimestamp = INT64_MIN;
    // Scheduler.SchedulerState.toNotifyQueue: a FIFO (LinkedBlockingQueue),
    // peeked / polled at its head (C/util/Scheduler.java:113-209,330-332)
    std::deque<int64_t> notify;
    // LengthBatch / TimeBatch WindowProcessor.WindowState (full-batch mode):
    // currentEventQueue, expiredEventQueue, resetEvent != null
    std::deque<Ev*> cur_q, exp_q;
    bool reset_pending = false;
    // aggregator states per group key
    std::map<std::vector<std::pair<uint64_t, uint8_t>>, GroupAgg> groups;
  };
  std::map<Key, std::unique_ptr<KeySingle>> single_keys;
  std::unique_ptr<KeySingle> single_global;
  // Aggregator states of a state query's selector: one group table per
  // partition key (PartitionStateHolder, C/util/snapshot/state/
  // PartitionStateHolder.java:43-69; the planner refuses aggregation inside a
  // partition, so only the unpartitioned table is used).
  KeySingle state_aggs;
  int window_kind = 0;
  int64_t window_param = 0, window_param2 = 0;
  int window_pos = -1;
  // TimeBatchWindowProcessor.nextEmitTime: a field of the processor, not of a
  // partition's state (:136, :283-300)
  int64_t next_emit = -1;
  // in_seq of the rows of a batch window's flush chunk (the emitting event)
  int64_t flush_seq = -1;
  bool batch_window() const {
    return window_kind == SHD_W_LENGTH_BATCH || window_kind == SHD_W_TIME_BATCH ||
           window_kind == SHD_W_TIME_BATCH_STREAM;
  }

  void build_single() {
    for (int i = 0; i < (int)p.handlers.size(); i++) {
      if (p.handlers[i].kind == SHD_H_WINDOW) {
        window_kind = p.handlers[i].wkind;
        window_param = p.handlers[i].param;
        window_param2 = p.handlers[i].param2;
        window_pos = i;
      }
    }
    if (!partitioned) single_global.reset(new KeySingle());
  }

  std::vector<Val> agg_vals;

  // GroupByKeyGenerator.constructEventKey (C/query/selector/GroupByKeyGenerator.java:63-73):
  // the key is the concatenation of String.valueOf of every group-by value, so
  // two values build one key exactly when their texts agree: a null string and
  // the string "null" both print "null"; every NaN prints "NaN"; 0.0 and -0.0
  // differ.  Canonical (value, null) pairs with those identifications (a value
  // containing the ":-:" delimiter is not identified across attributes).
  std::vector<std::pair<uint64_t, uint8_t>> group_key(const EvalCtx& cx) {
    std::vector<std::pair<uint64_t, uint8_t>> gk;
    for (int g : p.group_by) {
      Val v = eval(p, g, cx);
      const int t = expr_type(p, g);
      if (v.null && t == SHD_T_STRING && p.null_str_id >= 0) {
        gk.push_back({(uint64_t)p.null_str_id, 0});
        continue;
      }
      if (v.null) {
        gk.push_back({0, 1});
        continue;
      }
      uint64_t b = v.b;
      if (t == SHD_T_FLOAT) {
        const float f = as_f32(b);
        b = f != f ? 0x7fc00000ull : (uint64_t)(uint32_t)b;
      } else if (t == SHD_T_DOUBLE) {
        double d;
        memcpy(&d, &b, 8);
        if (d != d) b = 0x7ff8000000000000ull;
      } else if (t == SHD_T_INT || t == SHD_T_BOOL) {
        b = (uint64_t)(uint32_t)b;
      }
      gk.push_back({b, 0});
    }
    return gk;
  }

  // AttributeAggregatorExecutor.execute for each aggregator (plan order)
  void run_aggs(KeySingle* ks, Ev* e) {
    EvalCtx cx;
    cx.ev = e;
    run_aggs_ctx(*ks, cx, e->type);
  }

  // the aggregators of the event in cx (a StreamEvent of a single-stream
  // query or a StateEvent) under its group key; agg_vals = their results
  void run_aggs_ctx(KeySingle& kst, const EvalCtx& cx, int etype) {
    KeySingle* ks = &kst;
    agg_vals.assign(p.aggs.size(), Val{});
    if (p.aggs.empty()) return;
    struct { int type; } ev_t{etype};
    auto* e = &ev_t;
    std::vector<std::pair<uint64_t, uint8_t>> gk = group_key(cx);
    GroupAgg& ga = ks->groups[gk];
    if (ga.a.size() != p.aggs.size()) ga.a.resize(p.aggs.size());
    for (size_t i = 0; i < p.aggs.size(); i++) {
      const Plan::Agg& ag = p.aggs[i];
      AggState& s = ga.a[i];
      Val arg;
      if (ag.expr >= 0) arg = eval(p, ag.expr, cx);
      Val out;
      bool add = e->type == CURRENT;
      if (e->type != CURRENT && e->type != EXPIRED) { agg_vals[i] = out; continue; }
      switch (ag.kind) {
        case SHD_AGG_COUNT:
          // CountAttributeAggregatorExecutor: +-1 regardless of argument
          s.count += add ? 1 : -1;
          out.b = of_i64(s.count); out.null = false;
          break;
        case SHD_AGG_SUM:
          if (ag.type == SHD_T_INT || ag.type == SHD_T_LONG) {
            if (arg.null) {  // currentValue()
              if (s.count != 0) { out.b = of_i64(s.lsum); out.null = false; }
              break;
            }
            int64_t x = ag.type == SHD_T_INT ? (int64_t)as_i32(arg.b) : as_i64(arg.b);
            if (add) {
              s.lsum = (int64_t)((uint64_t)s.lsum + (uint64_t)x); s.count++;
              out.b = of_i64(s.lsum); out.null = false;
            } else {
              // AggregatorStateLong.processRemove(double): sum -= data with long<-double narrowing
              double r = (double)s.lsum - (double)x;
              s.lsum = java_d2l(r);
              s.count--;
              if (s.count != 0) { out.b = of_i64(s.lsum); out.null = false; }
            }
          } else {
            if (arg.null) {
              if (ag.type == SHD_T_FLOAT) break;   // AggregatorStateFloat returns null
              if (s.count != 0) { out.b = of_f64(s.dsum); out.null = false; }
              break;
            }
            double x = ag.type == SHD_T_FLOAT ? (double)as_f32(arg.b) : as_f64(arg.b);
            if (add) {
              s.dsum += x; s.count++;
              out.b = of_f64(s.dsum); out.null = false;
            } else {
              s.dsum -= x; s.count--;
              if (s.count != 0) { out.b = of_f64(s.dsum); out.null = false; }
            }
          }
          break;
        case SHD_AGG_AVG: {
          if (arg.null) {
            if (s.count != 0) { out.b = of_f64(s.dsum / (double)s.count); out.null = false; }
            break;
          }
          double x;
          switch (ag.type) {
            case SHD_T_INT: x = (double)as_i32(arg.b); break;
            case SHD_T_LONG: x = (double)as_i64(arg.b); break;
            case SHD_T_FLOAT: x = (double)as_f32(arg.b); break;
            default: x = as_f64(arg.b);
          }
          if (add) { s.count++; s.dsum += x; }
          else { s.count--; s.dsum -= x; }
          if (s.count != 0) { out.b = of_f64(s.dsum / (double)s.count); out.null = false; }
          break;
        }
      }
      agg_vals[i] = out;
    }
  }

  static int64_t java_d2l(double d) {
    if (std::isnan(d)) return 0;
    if (d >= 9.2233720368547758e18) return INT64_MAX;
    if (d <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)d;
  }

  // Window + selector over one chunk (list of events, CURRENT/EXPIRED/TIMER)
  void single_chunk(KeySingle* ks, std::vector<Ev*> chunk, int from_handler) {
    // filters / window in handler order
    for (int hi = from_handler; hi < (int)p.handlers.size(); hi++) {
      auto& h = p.handlers[hi];
      if (h.kind == SHD_H_FILTER) {
        std::vector<Ev*> out;
        EvalCtx cx;
        for (Ev* e : chunk) {
          if (e->type == TIMER) { out.push_back(e); continue; }
          cx.ev = e;
          counters[1]++;
          if (eval_bool(p, h.expr, cx)) out.push_back(e);
        }
        chunk.swap(out);
      } else if (batch_window()) {
        // one output chunk per flush (LengthBatchWindowProcessor.process :154-187:
        // each flush's chunk goes to the next processor on its own)
        std::vector<std::pair<std::vector<Ev*>, int64_t>> flushes = batch_process(ks, chunk);
        for (auto& f : flushes) {
          flush_seq = f.second;
          single_chunk(ks, f.first, hi + 1);
          flush_seq = -1;
        }
        return;
      } else {
        chunk = window_process(ks, chunk);
      }
    }
    selector_process(ks, chunk);
  }

  Ev* reset_event() {
    Ev* r = ev_arena.get();
    *r = Ev();
    r->type = RESET;
    return r;
  }

  // A flush of a batch window's WindowState: [expired events of the previous
  // batch, timestamp currentTime] + RESET + [the batch's current events] (the
  // current events become the next flush's expired events when the query
  // outputs expired events: outputExpectsExpiredEvents).
  std::vector<Ev*> batch_flush(KeySingle* ks, int64_t currentTime) {
    std::vector<Ev*> out;
    if (p.expired_on && !ks->exp_q.empty()) {
      for (Ev* x : ks->exp_q) {
        x->ts = currentTime;
        out.push_back(x);
      }
      ks->exp_q.clear();
    }
    if (ks->reset_pending) {
      out.push_back(reset_event());
      ks->reset_pending = false;
    }
    if (!ks->cur_q.empty()) {
      for (Ev* c : ks->cur_q) {
        if (p.expired_on) {
          Ev* x = clone_ev(c);
          x->type = EXPIRED;
          ks->exp_q.push_back(x);
        }
        out.push_back(c);
      }
      ks->cur_q.clear();
    }
    return out;
  }

  // Batch windows over one input chunk: the flush chunks, each with the
  // in_seq of its emitting event.
  std::vector<std::pair<std::vector<Ev*>, int64_t>> batch_process(KeySingle* ks, const std::vector<Ev*>& in) {
    std::vector<std::pair<std::vector<Ev*>, int64_t>> res;
    const int64_t currentTime = now;
    if (window_kind == SHD_W_LENGTH_BATCH && window_param == 0) {
      // processLengthZeroBatch (:189-204): every event its own chunk -- the
      // event, its EXPIRED copy, RESET
      for (Ev* e : in) {
        std::vector<Ev*> out{e};
        if (p.expired_on) {
          Ev* x = clone_ev(e);
          x->type = EXPIRED;
          x->ts = currentTime;
          out.push_back(x);
        }
        out.push_back(reset_event());
        res.push_back({out, e->seq});
      }
      return res;
    }
    if (window_kind == SHD_W_LENGTH_BATCH && (window_param2 & 1)) {
      // processStreamCurrentEvents (:245-274): each event passes at once (its
      // own chunk); the (length+1)-th expires the previous batch and RESETs first
      for (Ev* e : in) {
        ks->reset_pending = true;
        ks->count++;
        std::vector<Ev*> out;
        if (ks->count == window_param + 1) {
          if (p.expired_on && !ks->exp_q.empty()) {
            for (Ev* x : ks->exp_q) {
              x->ts = currentTime;
              out.push_back(x);
            }
            ks->exp_q.clear();
          }
          if (ks->reset_pending) {
            out.push_back(reset_event());
            ks->reset_pending = false;
          }
          ks->count = 1;
        }
        out.push_back(e);
        if (p.expired_on) {
          Ev* x = clone_ev(e);
          x->type = EXPIRED;
          ks->exp_q.push_back(x);
        }
        res.push_back({out, e->seq});
      }
      return res;
    }
    if (window_kind == SHD_W_LENGTH_BATCH) {
      // LengthBatchWindowProcessor.processFullBatchEvents (:206-243), length >= 1
      for (Ev* e : in) {
        ks->reset_pending = true;   // resetEvent: a copy of the first event after a flush
        ks->cur_q.push_back(clone_ev(e));
        ks->count++;
        if (ks->count == window_param) {
          std::vector<Ev*> out = batch_flush(ks, currentTime);
          ks->count = 0;
          if (!out.empty()) res.push_back({out, e->seq});
        }
      }
      return res;
    }
    // TimeBatchWindowProcessor.process (:279-366), full-batch mode
    if (next_emit == -1) {
      if (window_param2 != INT64_MIN) {
        // getNextEmitTime (:368-373): aligned to start.time
        const int64_t elapsed = (currentTime - window_param2) % window_param;
        next_emit = currentTime + (window_param - elapsed);
      } else {
        next_emit = currentTime + window_param;
      }
      ks->notify.push_back(next_emit);
    }
    bool send = false;
    if (currentTime >= next_emit) {
      next_emit += window_param;
      ks->notify.push_back(next_emit);
      send = true;
    }
    int64_t last_seq = cur_seq;
    if (window_kind == SHD_W_TIME_BATCH_STREAM) {
      // stream.current.event: the chunk's events stay in it (CURRENT); a flush
      // appends every event since the last one as EXPIRED, then RESET
      std::vector<Ev*> out;
      for (Ev* e : in) {
        if (e->type != CURRENT) continue;
        ks->reset_pending = true;
        if (p.expired_on) {
          Ev* x = clone_ev(e);
          x->type = EXPIRED;
          ks->exp_q.push_back(x);
        }
        out.push_back(e);
        last_seq = e->seq;
      }
      if (send) {
        if (p.expired_on && !ks->exp_q.empty()) {
          for (Ev* x : ks->exp_q) {
            x->ts = currentTime;
            out.push_back(x);
          }
          ks->exp_q.clear();
        }
        if (ks->reset_pending) {
          out.push_back(reset_event());
          ks->reset_pending = false;
        }
      }
      if (!out.empty()) res.push_back({out, last_seq});
      return res;
    }
    for (Ev* e : in) {
      if (e->type != CURRENT) continue;
      ks->reset_pending = true;
      ks->cur_q.push_back(clone_ev(e));
      last_seq = e->seq;
    }
    if (send) {
      std::vector<Ev*> out = batch_flush(ks, currentTime);
      if (!out.empty()) res.push_back({out, last_seq});
    }
    return res;
  }

  std::vector<Ev*> window_process(KeySingle* ks, const std::vector<Ev*>& in) {
    std::vector<Ev*> out;
    if (window_kind == SHD_W_LENGTH) {
      // LengthWindowProcessor.process (:105-142)
      int64_t currentTime = now;
      for (Ev* e : in) {
        if (e->type == TIMER) { out.push_back(e); continue; }
        Ev* c = clone_ev(e);
        c->type = EXPIRED;
        if (ks->count < window_param) {
          ks->count++;
          ks->q.push_back(c);
          out.push_back(e);
        } else {
          if (!ks->q.empty()) {
            Ev* f = ks->q.front();
            ks->q.pop_front();
            f->ts = currentTime;
            out.push_back(f);
            out.push_back(e);
            ks->q.push_back(c);
          } else {
            throw std::runtime_error("length(0) window (RESET path) outside the hot path");
          }
        }
      }
    } else if (window_kind == SHD_W_EXTERNAL_TIME) {
      // ExternalTimeWindowProcessor.process (:124-158): the clock is each
      // event's own LONG timestamp attribute; no scheduler
      const int col = (int)window_param2;
      const int64_t T = window_param;
      for (Ev* e : in) {
        if (e->type == TIMER) continue;
        const int64_t currentTime = (int64_t)e->data[col];
        while (!ks->q.empty()) {
          Ev* x = ks->q.front();
          if ((int64_t)x->data[col] - currentTime + T <= 0) {
            ks->q.pop_front();
            x->ts = currentTime;
            out.push_back(x);
          } else {
            break;
          }
        }
        if (e->type == CURRENT) {
          Ev* c = clone_ev(e);
          c->type = EXPIRED;
          ks->q.push_back(c);
        }
        out.push_back(e);
      }
    } else if (window_kind == SHD_W_TIME_LENGTH) {
      // TimeLengthWindowProcessor.process (:139-188): time expiry before each
      // event (TIMER events only expire), then the length bound; every added
      // event schedules ts + time
      const int64_t T = window_param, L = window_param2;
      const int64_t currentTime = now;
      for (Ev* e : in) {
        while (!ks->q.empty()) {
          Ev* x = ks->q.front();
          if (x->ts - currentTime + T <= 0) {
            ks->q.pop_front();
            ks->count--;
            x->ts = currentTime;
            out.push_back(x);
          } else {
            break;
          }
        }
        if (e->type != CURRENT) continue;
        Ev* c = clone_ev(e);
        c->type = EXPIRED;
        if (ks->count < L) {
          ks->count++;
          ks->q.push_back(c);
        } else if (!ks->q.empty()) {
          Ev* f = ks->q.front();
          ks->q.pop_front();
          f->ts = currentTime;
          out.push_back(f);
          ks->q.push_back(c);
        }
        ks->notify.push_back(c->ts + T);
        out.push_back(e);
      }
    } else {
      // TimeWindowProcessor.process (:132-169)
      for (Ev* e : in) {
        int64_t currentTime = now;
        while (!ks->q.empty()) {
          Ev* x = ks->q.front();
          if (x->ts - currentTime + window_param <= 0) {
            ks->q.pop_front();
            x->ts = currentTime;
            out.push_back(x);
          } else {
            break;
          }
        }
        if (e->type == CURRENT) {
          Ev* c = clone_ev(e);
          c->type = EXPIRED;
          ks->q.push_back(c);
          if (ks->lastTimestamp < c->ts) {
            ks->notify.push_back(c->ts + window_param);
            ks->lastTimestamp = c->ts;
          }
          out.push_back(e);
        }
      }
      // PartitionStateHolder.returnState (C/util/snapshot/state/PartitionStateHolder.java:50-69):
      // a partition's window state whose queue emptied is dropped, so its
      // lastTimestamp starts over (TimeWindowProcessor.WindowState.canDestroy :219-221)
      if (partitioned && ks->q.empty()) ks->lastTimestamp = INT64_MIN;
    }
    return out;
  }

  void selector_process(KeySingle* ks, const std::vector<Ev*>& chunk) {
    bool has_agg = !p.aggs.empty();
    bool group = !p.group_by.empty();
    std::vector<std::pair<Ev*, OutRow>> keep;
    // group-by: LinkedHashMap<String, event> (first-seen order, last value)
    std::vector<std::vector<std::pair<uint64_t, uint8_t>>> gorder;
    std::map<std::vector<std::pair<uint64_t, uint8_t>>, OutRow> gmap;
    OutRow last;
    bool have_last = false;
    for (Ev* e : chunk) {
      // RESET: every aggregator's cleanGroupByStates -- all group states of
      // this partition (AttributeAggregatorExecutor.processReset :144-150,
      // PartitionStateHolder.cleanGroupByStates :92-99)
      if (e->type == RESET) {
        ks->groups.clear();
        continue;
      }
      if (e->type != CURRENT && e->type != EXPIRED) continue;   // TIMER
      run_aggs(ks, e);
      OutRow r;
      r.type = e->type;
      r.ts = e->ts;
      r.seq = flush_seq >= 0 ? flush_seq : e->seq;
      EvalCtx cx;
      cx.ev = e;
      cx.aggs = &agg_vals;
      for (auto& o : p.outputs) {
        Val v = eval(p, o.second, cx);
        r.vals.push_back(v.b);
        r.nul.push_back(v.null);
      }
      bool on = (e->type == CURRENT && p.current_on) || (e->type == EXPIRED && p.expired_on);
      // havingConditionExecutor (QuerySelector.java:176-178,292-293,338-339): over
      // the event with its aggregator values, before the type check
      if (on && p.having >= 0 && !eval_bool(p, p.having, cx)) on = false;
      if (!on) continue;
      if (group) {
        std::vector<std::pair<uint64_t, uint8_t>> gk = group_key(cx);
        auto it = gmap.find(gk);
        if (it == gmap.end()) { gorder.push_back(gk); gmap[gk] = r; }
        else it->second = r;
      } else if (has_agg) {
        last = r;
        have_last = true;
      } else {
        keep.push_back({e, r});
      }
    }
    std::vector<OutRow> outs;
    if (group) {
      for (auto& gk : gorder) outs.push_back(gmap[gk]);
    } else if (has_agg) {
      if (have_last) outs.push_back(last);
    } else {
      for (auto& k : keep) outs.push_back(k.second);
    }
    if (outs.empty()) return;
    int64_t cid = chunk_counter++;
    for (auto& r : outs) {
      r.chunk = cid;
      rows.push_back(r);
      counters[3]++;
    }
  }

  void single_on_time_change(int64_t t) {
    if (window_kind != SHD_W_TIME && window_kind != SHD_W_TIME_BATCH && window_kind != SHD_W_TIME_LENGTH &&
        window_kind != SHD_W_TIME_BATCH_STREAM)
      return;
    // Scheduler.onTimeChange: states with head notify <= t, sorted by time.
    std::vector<std::pair<int64_t, KeySingle*>> due;
    if (partitioned) {
      for (auto& kv : single_keys)
        if (!kv.second->notify.empty() && kv.second->notify.front() <= t)
          due.push_back({kv.second->notify.front(), kv.second.get()});
    } else if (single_global && !single_global->notify.empty() && single_global->notify.front() <= t) {
      due.push_back({single_global->notify.front(), single_global.get()});
    }
    std::stable_sort(due.begin(), due.end(), [](auto& a, auto& b) { return a.first < b.first; });
    for (auto& d : due) {
      KeySingle* ks = d.second;
      while (!ks->notify.empty() && ks->notify.front() - now <= 0) {
        int64_t nt = ks->notify.front();
        ks->notify.pop_front();
        Ev* te = ev_arena.get();
        *te = Ev();
        te->type = TIMER;
        te->ts = nt;
        // the scheduler's entry valve sits right before the window
        single_chunk(ks, {te}, window_pos);
      }
    }
  }

  // ================= input =================
  Key partition_key(int stream, Ev* e, bool& ok) {
    for (auto& pk : p.part_keys) {
      if (pk.first != stream) continue;
      EvalCtx cx;
      cx.ev = e;
      Val v = eval(p, pk.second, cx);
      if (v.null) { ok = false; return Key(); }
      ok = true;
      return key_of(v, expr_type(p, pk.second));
    }
    ok = false;
    return Key();
  }

  void push(int stream, int64_t n, const int64_t* ts, const uint64_t* vals, const uint8_t* nulls, bool advance) {
    if (n <= 0) return;
    int na = (int)p.stream_types[stream].size();
    data_store.emplace_back(vals, vals + n * na);
    null_store.emplace_back(nulls, nulls + n * na);
    const uint64_t* D = data_store.back().data();
    const uint8_t* N = null_store.back().data();
    std::vector<Ev*> evs;
    for (int64_t i = 0; i < n; i++) {
      Ev* e = ev_arena.get();
      *e = Ev();
      e->ts = ts[i];
      e->data = D + i * na;
      e->nul = N + i * na;
      e->seq = seq++;
      evs.push_back(e);
    }
    // InputHandler.send(Event[]) (playback): time := last event's ts, timers first.
    if (advance) set_time(ts[n - 1]);
    if (!partitioned) {
      if (p.kind == SHD_KIND_STATE) {
        cur = nfa_global.get();
        state_run(stream, evs);
      } else {
        single_chunk(single_global.get(), evs, 0);
      }
      return;
    }
    // PartitionStreamReceiver.receive(Event[]) (:175-216): consecutive same-key runs.
    std::vector<Ev*> run;
    Key rk;
    bool have = false;
    for (Ev* e : evs) {
      bool ok;
      Key k = partition_key(stream, e, ok);
      if (!ok) continue;
      if (!have) { rk = k; have = true; run.push_back(e); }
      else if (!(k == rk)) { send_run(stream, rk, run); run.clear(); rk = k; run.push_back(e); }
      else run.push_back(e);
    }
    if (have) send_run(stream, rk, run);
  }

  void send_run(int stream, const Key& k, const std::vector<Ev*>& run) {
    // PartitionStreamReceiver.send -> PartitionRuntimeImpl.initPartition (first sight seeds state)
    if (p.kind == SHD_KIND_STATE) {
      auto it = nfa_keys.find(k);
      if (it == nfa_keys.end()) {
        nfa_keys[k].reset(new_key_nfa());
        cur = nfa_keys[k].get();
        start_partition();
      }
      cur = nfa_keys[k].get();
      state_run(stream, run);
    } else {
      auto it = single_keys.find(k);
      if (it == single_keys.end()) single_keys[k].reset(new KeySingle());
      single_chunk(single_keys[k].get(), run, 0);
    }
  }
};

int expr_type(const Plan& p, int expr) {
  // Result type of an expression: re-derived from its last instruction.
  const auto& code = p.exprs[expr];
  std::vector<int> st;
  for (auto& in : code) {
    switch (in.op) {
      case SHD_OP_CONST: st.push_back(in.b); break;
      case SHD_OP_NULL: st.push_back(in.b); break;
      case SHD_OP_LOAD: st.push_back(in.c >> 16); break;
      case SHD_OP_EVNULL: st.push_back(SHD_T_BOOL); break;
      case SHD_OP_TS: st.push_back(SHD_T_LONG); break;
      case SHD_OP_CVT: st.back() = in.b; break;
      case SHD_OP_ADD: case SHD_OP_SUB: case SHD_OP_MUL: case SHD_OP_DIV: case SHD_OP_MOD:
        st.pop_back(); st.back() = in.a; break;
      case SHD_OP_EQ: case SHD_OP_NE: case SHD_OP_GT: case SHD_OP_GE: case SHD_OP_LT: case SHD_OP_LE:
      case SHD_OP_AND: case SHD_OP_OR:
        st.pop_back(); st.back() = SHD_T_BOOL; break;
      case SHD_OP_NOT: case SHD_OP_ISNULL: st.back() = SHD_T_BOOL; break;
      case SHD_OP_AGG: st.push_back(SHD_T_DOUBLE); break;
      case SHD_OP_MULTI: st.push_back(SHD_T_OBJECT); break;
      case SHD_OP_IFELSE: { int t = st[st.size() - 2]; st.pop_back(); st.pop_back(); st.back() = t; break; }
    }
  }
  return st.empty() ? SHD_T_LONG : st.back();
}

thread_local std::string g_err;

}  // namespace

// ====================================================================== C API
extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }

void* orc_create(const int32_t* ir, int64_t nwords) {
  try {
    auto* e = new Engine();
    e->p = decode(ir, nwords);
    e->build();
    return e;
  } catch (std::exception& ex) {
    g_err = ex.what();
    return nullptr;
  }
}

void orc_destroy(void* h) { delete (Engine*)h; }

int orc_push(void* h, int32_t stream, int64_t n, const int64_t* ts, const uint64_t* vals, const uint8_t* nulls,
             int32_t advance_time) {
  try {
    ((Engine*)h)->push(stream, n, ts, vals, nulls, advance_time != 0);
    return 0;
  } catch (std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

// SiddhiAppRuntime.start() at app time t (wall-clock apps: the clock at start;
// playback: 0): unpartitioned state queries are (re)initialised at t
// (QueryRuntimeImpl.start -> initPartition, AbsentStreamPreStateProcessor.partitionCreated :291-303).
int orc_start(void* h, int64_t t) {
  try {
    Engine* e = (Engine*)h;
    if (t > e->now) e->now = t;
    if (!e->partitioned && e->p.kind == SHD_KIND_STATE) e->start_partition();
    return 0;
  } catch (std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int orc_set_time(void* h, int64_t t) {
  try {
    ((Engine*)h)->set_time(t);
    return 0;
  } catch (std::exception& ex) {
    g_err = ex.what();
    return -1;
  }
}

int64_t orc_num_rows(void* h) { return (int64_t)((Engine*)h)->rows.size(); }

int32_t orc_num_outputs(void* h) { return (int32_t)((Engine*)h)->p.outputs.size(); }

int64_t orc_num_list(void* h) { return (int64_t)((Engine*)h)->lists.size(); }

void orc_get_list(void* h, uint64_t* vals, uint8_t* nulls) {
  Engine* e = (Engine*)h;
  for (size_t i = 0; i < e->lists.size(); i++) {
    vals[i] = e->lists[i];
    nulls[i] = e->list_nul[i];
  }
}

void orc_get_rows(void* h, int64_t* chunk, int32_t* type, int64_t* ts, uint64_t* vals, uint8_t* nulls) {
  Engine* e = (Engine*)h;
  size_t no = e->p.outputs.size();
  for (size_t i = 0; i < e->rows.size(); i++) {
    const OutRow& r = e->rows[i];
    chunk[i] = r.chunk;
    type[i] = r.type;
    ts[i] = r.ts;
    for (size_t k = 0; k < no; k++) {
      vals[i * no + k] = r.vals[k];
      nulls[i * no + k] = r.nul[k];
    }
  }
}

void orc_get_rows_seq(void* h, int64_t* seq) {
  Engine* e = (Engine*)h;
  for (size_t i = 0; i < e->rows.size(); i++) seq[i] = e->rows[i].seq;
}

void orc_clear_rows(void* h) {
  Engine* e = (Engine*)h;
  e->rows.clear();
  e->lists.clear();
  e->list_nul.clear();
}

void orc_counters(void* h, int64_t* out) {
  for (int i = 0; i < 8; i++) out[i] = ((Engine*)h)->counters[i];
}

}  // extern "C"
