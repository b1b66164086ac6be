// shd_api.cpp -- the C-ABI of libsiddhi_hip (include/siddhi_hip.h): plan
// decoding, engine selection, batch staging, output polling.
#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "engine.h"

namespace shd {

void check_launch(const char* file, int line) {
  static const bool sync = [] {
    const char* v = std::getenv("SHD_SYNC_CHECK");
    return v && *v && *v != '0';
  }();
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && sync) e = hipDeviceSynchronize();
  if (e != hipSuccess)
    throw Error(e == hipErrorOutOfMemory ? SHD_E_OOM : SHD_E_DEVICE,
                std::string("kernel launched at ") + file + ":" + std::to_string(line) + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------------ plan decode
namespace {
struct Reader {
  const int32_t* w;
  int64_t n, i = 0;
  int32_t next() {
    if (i >= n) throw Error(SHD_E_INVALID_PLAN, "plan IR truncated");
    return w[i++];
  }
  int64_t next64() {
    uint32_t lo = (uint32_t)next();
    uint32_t hi = (uint32_t)next();
    return (int64_t)(((uint64_t)hi << 32) | lo);
  }
};

PNode read_node(Reader& r, int depth) {
  if (depth > 64) throw Error(SHD_E_INVALID_PLAN, "plan tree too deep");
  PNode n;
  n.kind = r.next();
  switch (n.kind) {
    case SHD_NODE_STREAM: {
      n.state_id = r.next();
      n.stream = r.next();
      n.absent = r.next();
      n.waiting = r.next64();
      int nf = r.next();
      if (nf < 0 || nf > 64) throw Error(SHD_E_INVALID_PLAN, "bad filter count");
      for (int i = 0; i < nf; i++) n.filters.push_back(r.next());
      break;
    }
    case SHD_NODE_NEXT:
      n.kids.push_back(read_node(r, depth + 1));
      n.kids.push_back(read_node(r, depth + 1));
      break;
    case SHD_NODE_EVERY:
      n.kids.push_back(read_node(r, depth + 1));
      break;
    case SHD_NODE_LOGICAL:
      n.ltype = r.next();
      n.kids.push_back(read_node(r, depth + 1));
      n.kids.push_back(read_node(r, depth + 1));
      break;
    case SHD_NODE_COUNT:
      n.min = r.next();
      n.max = r.next();
      n.kids.push_back(read_node(r, depth + 1));
      break;
    default:
      throw Error(SHD_E_INVALID_PLAN, "bad node kind");
  }
  return n;
}
}  // namespace

Plan decode_plan(const int32_t* w, int64_t n) {
  Reader r{w, n};
  Plan p;
  if (r.next() != (int32_t)SHD_IR_MAGIC) throw Error(SHD_E_INVALID_PLAN, "bad plan magic");
  if (r.next() != SHD_IR_VERSION) throw Error(SHD_E_INVALID_PLAN, "unsupported plan version");
  p.kind = r.next();
  int ns = r.next();
  if (ns < 0 || ns > 64) throw Error(SHD_E_INVALID_PLAN, "bad stream count");
  for (int s = 0; s < ns; s++) {
    int na = r.next();
    if (na < 0 || na > 1024) throw Error(SHD_E_INVALID_PLAN, "bad attribute count");
    std::vector<int> t;
    for (int a = 0; a < na; a++) t.push_back(r.next());
    p.stream_types.push_back(t);
  }
  int nc = r.next();
  if (nc < 0) throw Error(SHD_E_INVALID_PLAN, "bad const count");
  for (int i = 0; i < nc; i++) p.consts.push_back((uint64_t)r.next64());
  int ne = r.next();
  if (ne < 0) throw Error(SHD_E_INVALID_PLAN, "bad expression count");
  for (int i = 0; i < ne; i++) {
    int ni = r.next();
    if (ni < 0 || ni > 4096) throw Error(SHD_E_INVALID_PLAN, "bad instruction count");
    std::vector<Instr> code;
    for (int k = 0; k < ni; k++) {
      Instr in;
      in.op = r.next();
      in.a = r.next();
      in.b = r.next();
      in.c = r.next();
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
    p.root = read_node(r, 0);
  } else if (p.kind == SHD_KIND_SINGLE) {
    p.single_stream = r.next();
    int nh = r.next();
    for (int i = 0; i < nh; i++) {
      Plan::Handler h{};
      h.kind = r.next();
      if (h.kind == SHD_H_FILTER) h.expr = r.next();
      else {
        h.wkind = r.next();
        h.param = r.next64();
        h.param2 = r.next64();
      }
      p.handlers.push_back(h);
    }
  } else {
    throw Error(SHD_E_INVALID_PLAN, "bad plan kind");
  }
  p.current_on = r.next();
  p.expired_on = r.next();
  int na = r.next();
  for (int i = 0; i < na; i++) {
    Plan::Agg a;
    a.kind = r.next();
    a.expr = r.next();
    a.type = r.next();
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
  // optional trailing sections: dictionary id of the string "null" (group
  // keys), then the POST section of a state plan's selector (siddhi_ir.h)
  if (r.i + 2 <= r.n) p.null_str_id = r.next64();
  if (r.i < r.n) {
    if (p.kind != SHD_KIND_STATE || r.next() != (int32_t)SHD_IR_POST_MAGIC)
      throw Error(SHD_E_INVALID_PLAN, "unknown trailing plan section");
    const int nb = r.next();
    if (nb < 0 || nb > kMaxCols) throw Error(SHD_E_UNSUPPORTED, "too many selector base values");
    for (int i = 0; i < nb; i++) {
      const int t = r.next();
      const int e = r.next();
      p.post_base.push_back({t, e});
    }
    const int nw = r.next();
    if (nw < 0 || r.i + nw > r.n) throw Error(SHD_E_INVALID_PLAN, "POST section truncated");
    p.post = std::make_shared<Plan>(decode_plan(r.w + r.i, nw));
    r.i += nw;
    if (p.post->kind != SHD_KIND_SINGLE || p.post->stream_types.size() != 1 ||
        p.post->stream_types[0].size() != (size_t)nb)
      throw Error(SHD_E_INVALID_PLAN, "POST selector plan does not match its base values");
    for (int i = 0; i < nb; i++)
      if (p.post->stream_types[0][i] != p.post_base[i].first) throw Error(SHD_E_INVALID_PLAN, "POST base type");
    if (r.i != r.n) throw Error(SHD_E_INVALID_PLAN, "trailing words after the POST section");
  }
  // validation: expression ids, stack depth, constants
  auto check_expr = [&](int e) {
    if (e < 0 || e >= (int)p.exprs.size()) throw Error(SHD_E_INVALID_PLAN, "bad expression id");
    if (expr_max_depth(p, e) > kMaxStack) throw Error(SHD_E_UNSUPPORTED, "expression stack too deep");
    for (auto& in : p.exprs[e])
      if (in.op == SHD_OP_CONST && (in.a < 0 || in.a >= (int)p.consts.size()))
        throw Error(SHD_E_INVALID_PLAN, "bad constant index");
  };
  for (size_t e = 0; e < p.exprs.size(); e++) check_expr((int)e);
  for (auto& o : p.outputs) check_expr(o.second);
  for (auto& o : p.post_base) check_expr(o.second);
  return p;
}

int expr_max_depth(const Plan& p, int expr) {
  int sp = 0, mx = 0;
  for (auto& in : p.exprs[expr]) {
    switch (in.op) {
      case SHD_OP_CONST: case SHD_OP_NULL: case SHD_OP_LOAD: case SHD_OP_EVNULL: case SHD_OP_TS: case SHD_OP_AGG:
      case SHD_OP_MULTI:
        sp++;
        break;
      case SHD_OP_ADD: case SHD_OP_SUB: case SHD_OP_MUL: case SHD_OP_DIV: case SHD_OP_MOD: case SHD_OP_EQ:
      case SHD_OP_NE: case SHD_OP_GT: case SHD_OP_GE: case SHD_OP_LT: case SHD_OP_LE: case SHD_OP_AND:
      case SHD_OP_OR:
        sp--;
        break;
      case SHD_OP_IFELSE:
        sp -= 2;
        break;
      default:
        break;
    }
    if (sp < 0) throw Error(SHD_E_INVALID_PLAN, "expression stack underflow");
    mx = std::max(mx, sp);
  }
  return mx;
}

int expr_result_type(const Plan& p, int expr, const std::vector<int>&) {
  std::vector<int> st;
  for (auto& in : p.exprs[expr]) {
    switch (in.op) {
      case SHD_OP_CONST: case SHD_OP_NULL: st.push_back(in.b); break;
      case SHD_OP_LOAD: st.push_back(in.c >> 16); break;
      case SHD_OP_EVNULL: st.push_back(SHD_T_BOOL); break;
      case SHD_OP_TS: st.push_back(SHD_T_LONG); break;
      case SHD_OP_CVT: if (!st.empty()) st.back() = in.b; break;
      case SHD_OP_ADD: case SHD_OP_SUB: case SHD_OP_MUL: case SHD_OP_DIV: case SHD_OP_MOD:
        if (st.size() >= 2) { st.pop_back(); st.back() = in.a; }
        break;
      case SHD_OP_EQ: case SHD_OP_NE: case SHD_OP_GT: case SHD_OP_GE: case SHD_OP_LT: case SHD_OP_LE:
      case SHD_OP_AND: case SHD_OP_OR:
        if (st.size() >= 2) { st.pop_back(); st.back() = SHD_T_BOOL; }
        break;
      case SHD_OP_NOT: case SHD_OP_ISNULL: if (!st.empty()) st.back() = SHD_T_BOOL; break;
      case SHD_OP_AGG: st.push_back(SHD_T_DOUBLE); break;
      case SHD_OP_MULTI: st.push_back(SHD_T_OBJECT); break;
      case SHD_OP_IFELSE:
        if (st.size() >= 3) { const int t = st[st.size() - 2]; st.pop_back(); st.pop_back(); st.back() = t; }
        break;
    }
  }
  return st.empty() ? SHD_T_LONG : st.back();
}

void DevExprTable::upload(const Plan& p) {
  std::vector<int4> all;
  off.clear();
  len.clear();
  for (auto& code : p.exprs) {
    off.push_back((int)all.size());
    len.push_back((int)code.size());
    for (auto& in : code) all.push_back(make_int4(in.op, in.a, in.b, in.c));
  }
  if (all.size() > (size_t)kLdsIns || p.consts.size() > (size_t)kLdsConsts)
    throw Error(SHD_E_UNSUPPORTED, "expression program larger than the device LDS program store");
  nins = (int)all.size();
  nconsts = (int)p.consts.size();
  ins.reserve(std::max<size_t>(all.size(), 1) * sizeof(int4));
  consts.reserve(std::max<size_t>(p.consts.size(), 1) * 8);
  if (!all.empty()) SHD_HIP(hipMemcpy(ins.p, all.data(), all.size() * sizeof(int4), hipMemcpyHostToDevice));
  if (!p.consts.empty()) SHD_HIP(hipMemcpy(consts.p, p.consts.data(), p.consts.size() * 8, hipMemcpyHostToDevice));
  // hipMemcpy from pageable memory may return before the DMA lands, and the
  // engines run on non-blocking streams that do not order after the null
  // stream: wait here so no kernel can read a half-written program.
  SHD_HIP(hipDeviceSynchronize());
}

void OutputBuffer::ensure(int64_t extra, hipStream_t s) {
  int64_t need = count + extra;
  if (need <= cap) return;
  int64_t nc = std::max<int64_t>(need, std::max<int64_t>(cap * 2, 4096));
  int w = std::max(ncols, 1);
  DevBuf c2, t2, ts2, v2, n2, q2, x2;
  q2.reserve(nc * 8);
  x2.reserve(nc * 4);
  c2.reserve(nc * 8);
  t2.reserve(nc * 4);
  ts2.reserve(nc * 8);
  v2.reserve(nc * w * 8);
  n2.reserve(nc * w);
  if (count > 0) {
    SHD_HIP(hipMemcpyAsync(c2.p, chunk.p, count * 8, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(t2.p, type.p, count * 4, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(ts2.p, ts.p, count * 8, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(v2.p, vals.p, count * w * 8, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(n2.p, nulls.p, count * w, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(q2.p, seq.p, count * 8, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(x2.p, sidx.p, count * 4, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipStreamSynchronize(s));
  }
  std::swap(chunk.p, c2.p); std::swap(chunk.cap, c2.cap);
  std::swap(type.p, t2.p); std::swap(type.cap, t2.cap);
  std::swap(ts.p, ts2.p); std::swap(ts.cap, ts2.cap);
  std::swap(vals.p, v2.p); std::swap(vals.cap, v2.cap);
  std::swap(nulls.p, n2.p); std::swap(nulls.cap, n2.cap);
  std::swap(sidx.p, x2.p); std::swap(sidx.cap, x2.cap);
  std::swap(seq.p, q2.p); std::swap(seq.cap, q2.cap);
  cap = nc;
}

void OutputBuffer::ensure_list(int64_t extra, hipStream_t s) {
  const int64_t need = lcount + extra;
  if (need <= lcap) return;
  const int64_t nc = std::max<int64_t>(need, std::max<int64_t>(lcap * 2, 4096));
  DevBuf v2, n2;
  v2.reserve(nc * 8);
  n2.reserve(nc);
  if (lcount > 0) {
    SHD_HIP(hipMemcpyAsync(v2.p, lvals.p, lcount * 8, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipMemcpyAsync(n2.p, lnul.p, lcount, hipMemcpyDeviceToDevice, s));
    SHD_HIP(hipStreamSynchronize(s));
  }
  std::swap(lvals.p, v2.p); std::swap(lvals.cap, v2.cap);
  std::swap(lnul.p, n2.p); std::swap(lnul.cap, n2.cap);
  lcap = nc;
}

void Engine::mark(const char* name) {
  if (!sev[0]) {
    for (int i = 0; i <= kMaxStages; i++) SHD_HIP(hipEventCreate(&sev[i]));
  }
  if (name == nullptr) {
    SHD_HIP(hipEventRecord(sev[0], stream));
    return;
  }
  if (n_stages >= kMaxStages) return;
  stage_name[n_stages] = name;
  SHD_HIP(hipEventRecord(sev[n_stages + 1], stream));
  n_stages++;
}

void Engine::stage_end() {
  if (n_stages == 0) return;
  SHD_HIP(hipEventSynchronize(sev[n_stages]));
  for (int i = 0; i < n_stages; i++) {
    float ms = 0.f;
    SHD_HIP(hipEventElapsedTime(&ms, sev[i], sev[i + 1]));
    stage_ns[i] = (int64_t)((double)ms * 1e6);
  }
}

Engine::~Engine() {
  for (int i = 0; i <= kMaxStages; i++)
    if (sev[i]) (void)hipEventDestroy(sev[i]);
  if (ev0) (void)hipEventDestroy(ev0);
  if (ev1) (void)hipEventDestroy(ev1);
  if (stream) (void)hipStreamDestroy(stream);
}

// Pre-decode a filter chain into a fixed-shape conjunction (dev_expr.h,
// "fast predicates"); returns false when any expression has another shape.
bool compile_fast_pred(const Plan& p, const std::vector<int>& ids, FPred& out) {
  out = FPred{};
  enum { N_ATOM, N_TERM, N_CMP, N_AND };
  struct Node {
    int kind;
    FAtom atom;
    FTerm term;
    std::vector<FCmp> cmps;
  };
  auto no_atom = [] {
    FAtom a{};
    a.kind = FA_NONE;
    a.cvt_from = a.cvt_to = -1;
    return a;
  };
  auto as_term = [&](const Node& n, FTerm& t) {
    t = FTerm{};
    if (n.kind == N_ATOM) {
      t.a = n.atom;
      t.b = no_atom();
      t.aop = 0;
      return true;
    }
    if (n.kind == N_TERM) {
      t = n.term;
      return true;
    }
    return false;
  };
  std::vector<FCmp> all;
  for (int e : ids) {
    std::vector<Node> st;
    for (const Instr& in : p.exprs[e]) {
      switch (in.op) {
        case SHD_OP_LOAD: case SHD_OP_CONST: case SHD_OP_NULL: {
          Node n{};
          n.kind = N_ATOM;
          n.atom = no_atom();
          if (in.op == SHD_OP_LOAD) {
            if (in.b < -2 || in.b > 127 || in.a < 0 || in.a > 127) return false;
            n.atom.kind = FA_LOAD;
            n.atom.st = (int8_t)in.a;
            n.atom.idx = (int8_t)in.b;
            n.atom.attr = (int16_t)(in.c & 0xFFFF);
          } else if (in.op == SHD_OP_CONST) {
            n.atom.kind = FA_CONST;
            n.atom.cval = p.consts[in.a];
          } else {
            n.atom.kind = FA_NULL;
          }
          st.push_back(n);
          break;
        }
        case SHD_OP_CVT:
          if (st.empty() || st.back().kind != N_ATOM || st.back().atom.cvt_to >= 0) return false;
          st.back().atom.cvt_from = (int8_t)in.a;
          st.back().atom.cvt_to = (int8_t)in.b;
          break;
        case SHD_OP_ADD: case SHD_OP_SUB: case SHD_OP_MUL: case SHD_OP_DIV: case SHD_OP_MOD: {
          if (st.size() < 2) return false;
          Node r = st.back();
          st.pop_back();
          Node l = st.back();
          st.pop_back();
          if (l.kind != N_ATOM || r.kind != N_ATOM) return false;
          Node n{};
          n.kind = N_TERM;
          n.term.a = l.atom;
          n.term.b = r.atom;
          n.term.aop = (int8_t)in.op;
          n.term.atype = (int8_t)in.a;
          st.push_back(n);
          break;
        }
        case SHD_OP_EQ: case SHD_OP_NE: case SHD_OP_GT: case SHD_OP_GE: case SHD_OP_LT: case SHD_OP_LE: {
          if (st.size() < 2) return false;
          Node r = st.back();
          st.pop_back();
          Node l = st.back();
          st.pop_back();
          FCmp c{};
          if (!as_term(l, c.l) || !as_term(r, c.r)) return false;
          c.op = (int8_t)in.op;
          c.type = (int8_t)in.a;
          Node n{};
          n.kind = N_CMP;
          n.cmps.push_back(c);
          st.push_back(n);
          break;
        }
        case SHD_OP_AND: {
          if (st.size() < 2) return false;
          Node r = st.back();
          st.pop_back();
          Node l = st.back();
          st.pop_back();
          if ((l.kind != N_CMP && l.kind != N_AND) || (r.kind != N_CMP && r.kind != N_AND)) return false;
          Node n{};
          n.kind = N_AND;
          n.cmps = l.cmps;
          n.cmps.insert(n.cmps.end(), r.cmps.begin(), r.cmps.end());
          st.push_back(n);
          break;
        }
        default:
          return false;
      }
    }
    if (st.size() != 1 || (st[0].kind != N_CMP && st[0].kind != N_AND)) return false;
    all.insert(all.end(), st[0].cmps.begin(), st[0].cmps.end());
  }
  if (all.size() > 4) return false;
  out.ok = 1;
  out.n = (int)all.size();
  for (size_t i = 0; i < all.size(); i++) out.c[i] = all[i];
  return true;
}

void init_engine(Engine& e, const Plan& p) {
  e.plan = p;
  e.ex.upload(p);
  e.out.init((int)p.outputs.size());
  e.on_loaded();
  SHD_HIP(hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking));
  SHD_HIP(hipEventCreate(&e.ev0));
  SHD_HIP(hipEventCreate(&e.ev1));
  e.reset();
}

DFilters Engine::dfilters(const std::vector<int>& ids) const {
  DFilters f{};
  f.n = (int)ids.size();
  if (f.n > 4) throw Error(SHD_E_UNSUPPORTED, "more than 4 filters on one state");
  for (int i = 0; i < f.n; i++) f.f[i] = dexpr(ids[i]);
  const char* nf = std::getenv("SHD_NO_FAST_PRED");   // interpreter only (cross-check in tests)
  const bool no_fast = nf && *nf && *nf != '0';
  if (no_fast || !compile_fast_pred(plan, ids, f.fp)) f.fp.ok = 0;
  return f;
}

bool Engine::fast_atom(int expr_id, FAtom& out) const {
  out = FAtom{};
  out.kind = FA_NONE;
  out.cvt_from = out.cvt_to = -1;
  const char* nf = std::getenv("SHD_NO_FAST_PRED");
  if ((nf && *nf && *nf != '0') || expr_id < 0 || expr_id >= (int)plan.exprs.size()) return false;
  const std::vector<Instr>& code = plan.exprs[expr_id];
  if (code.empty() || code.size() > 2) return false;
  const Instr& in = code[0];
  if (in.op == SHD_OP_LOAD) {
    if (in.b < -2 || in.b > 127 || in.a < 0 || in.a > 127) return false;
    out.kind = FA_LOAD;
    out.st = in.a;
    out.idx = in.b;
    out.attr = in.c & 0xFFFF;
  } else if (in.op == SHD_OP_CONST) {
    if (in.a < 0 || in.a >= (int)plan.consts.size()) return false;
    out.kind = FA_CONST;
    out.cval = plan.consts[in.a];
  } else if (in.op == SHD_OP_NULL) {
    out.kind = FA_NULL;
  } else {
    return false;
  }
  if (code.size() == 2) {
    if (code[1].op != SHD_OP_CVT) return false;
    out.cvt_from = code[1].a;
    out.cvt_to = code[1].b;
  }
  return true;
}

}  // namespace shd

// ====================================================================== C-ABI
using namespace shd;

struct shd_ctx {
  int device = 0;
};

struct shd_query {
  shd_ctx* ctx = nullptr;
  std::unique_ptr<Engine> eng;
  // state plans with an aggregating / `having` selector (IR POST section):
  // eng projects the selector's base values per match, post runs the
  // selector over those rows (one call per row) and holds the query's output
  std::unique_ptr<Engine> post;
  DevBuf post_col[kMaxCols], post_nul[kMaxCols];
  Engine& out_eng() { return post ? *post : *eng; }
  // host staging for SHD_MEM_HOST batches
  DevBuf stage_ts, stage_col[kMaxCols], stage_nul[kMaxCols];
  PinnedBuf pin;   // host staging for SHD_MEM_HOST batches
  // poll buffers (host)
  std::vector<int64_t> h_chunk, h_ts, h_seq;
  std::vector<int32_t> h_sidx;
  std::vector<int32_t> h_type;
  std::vector<uint64_t> h_vals, h_lvals;
  std::vector<uint8_t> h_nulls, h_lnul;
  uint64_t plan_hash = 0;         // FNV-1a of the plan IR (snapshot compatibility)
  std::vector<uint8_t> snap;      // last shd_snapshot image (library-owned)
};

namespace {
thread_local std::string g_err;

int fail(int code, const std::string& m) {
  g_err = m;
  return code;
}

template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (Error& e) {
    return fail(e.code, e.what());
  } catch (std::bad_alloc&) {
    return fail(SHD_E_OOM, "host allocation failed");
  } catch (std::exception& e) {
    return fail(SHD_E_DEVICE, e.what());
  }
}
}  // namespace

namespace {

// Copy host columns of one stream into device buffers (stream ordered, through
// pinned memory); the caller's buffers may be pageable and are only valid for
// the duration of the call.
void stage_host(hipStream_t s, PinnedBuf& pin, DevBuf& dts, DevBuf* dcol, DevBuf* dnul, const shd_batch* b,
                const std::vector<int>& types, Staged& st) {
  SHD_HIP(hipStreamSynchronize(s));   // the previous use of the pinned area has drained
  size_t total = (size_t)b->n * 8;
  for (int c = 0; c < b->ncols; c++) {
    total += (size_t)b->n * type_size(types[c]) + 64;
    if (b->nulls && b->nulls[c]) total += (size_t)b->n + 64;
  }
  pin.reserve(total + 64);
  char* hp = pin.as<char>();
  size_t used = 0;
  auto stage = [&](DevBuf& dst, const void* src, size_t bytes) -> void* {
    dst.reserve(bytes);
    std::memcpy(hp + used, src, bytes);
    SHD_HIP(hipMemcpyAsync(dst.p, hp + used, bytes, hipMemcpyHostToDevice, s));
    used += (bytes + 63) & ~size_t(63);
    return dst.p;
  };
  st.cs.ts = (const int64_t*)stage(dts, b->ts, (size_t)b->n * 8);
  for (int c = 0; c < b->ncols; c++) {
    st.cs.col[c] = stage(dcol[c], b->cols[c], (size_t)b->n * type_size(types[c]));
    st.cs.type[c] = (int8_t)types[c];
    st.cs.nul[c] = (b->nulls && b->nulls[c]) ? (const uint8_t*)stage(dnul[c], b->nulls[c], (size_t)b->n) : nullptr;
  }
}

// ---- selector over a state query's rows (IR POST section)
struct PostXArgs {
  int nc;
  int32_t type[kMaxCols];
  void* col[kMaxCols];
  uint8_t* nul[kMaxCols];
};

// row-major 64-bit payloads of the state engine's rows -> typed columns of
// the selector stream (one thread per row)
__global__ __launch_bounds__(kBlock) void k_post_cols(const PostXArgs* __restrict__ ap, const uint64_t* vals,
                                                      const uint8_t* nulls, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= n) return;
  const int nc = ap->nc;
  for (int c = 0; c < nc; c++) {
    const uint64_t b = vals[i * nc + c];
    const uint8_t z = nulls[i * nc + c];
    ap->nul[c][i] = z;
    switch (ap->type[c]) {
      case SHD_T_BOOL: ((uint8_t*)ap->col[c])[i] = (uint8_t)b; break;
      case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: ((uint32_t*)ap->col[c])[i] = (uint32_t)b; break;
      default: ((uint64_t*)ap->col[c])[i] = b; break;
    }
  }
}

// selector rows [r0, r0 + m): back to the state rows that emitted them (the
// selector stream's arrival index - seq0 = the state row): callback chunk,
// in_seq and state index of that row
__global__ __launch_bounds__(kBlock) void k_post_remap(int64_t* chunk, int64_t* seq, int32_t* sidx, int64_t r0,
                                                       int64_t m, int64_t seq0, const int64_t* a_chunk,
                                                       const int64_t* a_seq, const int32_t* a_sidx) {
  const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (i >= m) return;
  const int64_t a = seq[r0 + i] - seq0;
  chunk[r0 + i] = a_chunk[a];
  seq[r0 + i] = a_seq[a];
  sidx[r0 + i] = a_sidx[a];
}

// The reference's selector sees one StateEvent per chunk
// (StateMultiProcessStreamReceiver.processAndClear, C/query/input/
// StateMultiProcessStreamReceiver.java:47-68), so the state rows pushed since
// the last call are fed to the selector engine in emission order, one
// InputHandler call per row; its rows then take the callback chunks, in_seq
// and state indices of the state rows they came from.
void run_post(shd_query* q) {
  if (!q->post) return;
  Engine& a = *q->eng;
  Engine& b = *q->post;
  const int64_t n = a.out.count;
  if (n <= 0) return;
  SHD_HIP(hipStreamSynchronize(a.stream));
  hipStream_t s = b.stream;
  const auto& types = b.plan.stream_types[0];
  const int nc = (int)types.size();
  if (nc != a.out.ncols) throw Error(SHD_E_DEVICE, "internal: selector base columns");
  b.args_begin();
  PostXArgs xa{};
  xa.nc = nc;
  Staged st;
  st.stream = 0;
  st.n = n;
  st.advance_time = false;
  st.cs.ncols = nc;
  st.cs.n = n;
  st.cs.ts = a.out.d_ts();
  for (int c = 0; c < nc; c++) {
    q->post_col[c].reserve((size_t)n * type_size(types[c]));
    q->post_nul[c].reserve((size_t)n);
    xa.type[c] = types[c];
    xa.col[c] = q->post_col[c].p;
    xa.nul[c] = q->post_nul[c].as<uint8_t>();
    st.cs.col[c] = q->post_col[c].p;
    st.cs.nul[c] = q->post_nul[c].as<uint8_t>();
    st.cs.type[c] = (int8_t)types[c];
  }
  if (nc > 0) {
    hipLaunchKernelGGL(k_post_cols, dim3(grid_cover(n)), dim3(kBlock), 0, s, b.dev_args(xa), a.out.d_vals(),
                       a.out.d_nulls(), n);
    SHD_CHECK_LAUNCH();
  }
  st.call_offsets.resize((size_t)n + 1);
  for (int64_t i = 0; i <= n; i++) st.call_offsets[(size_t)i] = i;
  const int64_t seq0 = b.seq, r0 = b.out.count;
  b.push(st);
  const int64_t m = b.out.count - r0;
  if (m > 0) {
    hipLaunchKernelGGL(k_post_remap, dim3(grid_cover(m)), dim3(kBlock), 0, s, b.out.d_chunk(), b.out.d_seq(),
                       b.out.d_sidx(), r0, m, seq0, (const int64_t*)a.out.d_chunk(), (const int64_t*)a.out.d_seq(),
                       (const int32_t*)a.out.d_sidx());
    SHD_CHECK_LAUNCH();
  }
  SHD_HIP(hipStreamSynchronize(s));
  a.out.count = 0;
}

// The running engine hit a valid input its formulation cannot process
// (NeedNfa): rebuild its open partial matches in a fresh generic NFA engine
// by replaying the events that created them, carry over unpolled output and
// the query's counters, then run the push there.  The query stays on the NFA
// engine from then on.
// given: the open partials to replay (a dissolving query group hands its
// leader's to every member); null: q's own engine exports them
void switch_to_nfa(shd_query* q, const Staged& st, const shd_counters& before, const std::string& why,
                   const std::vector<Replay>* given = nullptr) {
  Engine& old = *q->eng;
  std::vector<Replay> own;
  if (!given) old.export_replay(own);
  const std::vector<Replay>& parts = given ? *given : own;
  int64_t nrep = 0;
  for (auto& r : parts) nrep += r.n;
  std::string w2;
  std::unique_ptr<Engine> ne = make_nfa_engine(old.plan, w2, nrep + st.n);
  if (!ne) throw Error(SHD_E_UNSUPPORTED, why + "; the generic NFA engine does not take this plan: " + w2);
  init_engine(*ne, old.plan);
  ne->start_time = old.start_time;
  for (auto& r : parts) {
    if (r.n <= 0) continue;
    const auto& types = old.plan.stream_types[r.stream];
    std::vector<const void*> cp(types.size());
    std::vector<const uint8_t*> np(types.size());
    for (size_t c = 0; c < types.size(); c++) {
      cp[c] = r.cols[c].data();
      np[c] = r.nulls[c].data();
    }
    shd_batch rb{};
    rb.stream = r.stream;
    rb.mem = SHD_MEM_HOST;
    rb.n = r.n;
    rb.ts = r.ts.data();
    rb.ncols = (int32_t)types.size();
    rb.cols = cp.data();
    rb.nulls = np.data();
    Staged rs;
    rs.stream = r.stream;
    rs.n = r.n;
    rs.call_offsets = {0, r.n};
    rs.advance_time = false;
    rs.cs.ncols = rb.ncols;
    rs.cs.n = r.n;
    PinnedBuf pin;
    DevBuf dts, dcol[kMaxCols], dnul[kMaxCols], dskip;
    stage_host(ne->stream, pin, dts, dcol, dnul, &rb, types, rs);
    if (!r.skip_start.empty()) {
      dskip.reserve((size_t)r.n);
      SHD_HIP(hipMemcpyAsync(dskip.p, r.skip_start.data(), (size_t)r.n, hipMemcpyHostToDevice, ne->stream));
      rs.skip_start = dskip.as<uint8_t>();
    }
    ne->args_begin();
    ne->push(rs);
    SHD_HIP(hipStreamSynchronize(ne->stream));
    if (ne->out.count != 0) throw Error(SHD_E_DEVICE, "internal: replaying the open partials produced output");
  }
  // unpolled rows of earlier pushes stay ahead of this push's rows
  if (old.out.count > 0) {
    const int64_t m = old.out.count;
    const int w = std::max(old.out.ncols, 1);
    ne->out.ensure(m, ne->stream);
    SHD_HIP(hipMemcpyAsync(ne->out.chunk.p, old.out.chunk.p, m * 8, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipMemcpyAsync(ne->out.type.p, old.out.type.p, m * 4, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipMemcpyAsync(ne->out.ts.p, old.out.ts.p, m * 8, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipMemcpyAsync(ne->out.vals.p, old.out.vals.p, m * w * 8, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipMemcpyAsync(ne->out.nulls.p, old.out.nulls.p, m * w, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipMemcpyAsync(ne->out.seq.p, old.out.seq.p, m * 8, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipMemcpyAsync(ne->out.sidx.p, old.out.sidx.p, m * 4, hipMemcpyDeviceToDevice, ne->stream));
    SHD_HIP(hipStreamSynchronize(ne->stream));
    ne->out.count = m;
  }
  ne->seq = old.seq;
  ne->now = old.now;
  ne->chunk_seq = old.chunk_seq;
  const int64_t carry = ne->counters.carry;
  ne->counters = before;
  ne->counters.carry = carry;
  q->eng = std::move(ne);
  q->eng->args_begin();
  q->eng->push(st);
}

}  // namespace

namespace shd {
int route_words(int ncols, const int* widths);
int64_t route_bucket_scratch(int64_t n, int world);
void route_bucket(hipStream_t s, int64_t n, int world, const void* key, int key_width, int ncols,
                  const void* const* cols, const int* widths, const int64_t* seq, int64_t seq_lo, uint64_t* send,
                  int64_t* counts, uint32_t* scratch);
void route_merge(hipStream_t s, int world, const uint64_t* recv, const int64_t* seg_off, int64_t m, int64_t seq_lo,
                 int64_t block, int64_t nblocks, int ncols, void* const* out_cols, const int* widths,
                 int64_t* out_seq, int64_t* start, int64_t* block_off, int32_t* err);
}  // namespace shd

extern "C" {

const char* shd_last_error(void) { return g_err.c_str(); }

int shd_device_count(int* n) {
  return guarded([&]() -> int {
    if (!n) return fail(SHD_E_ARG, "null pointer");
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    *n = (e == hipSuccess) ? c : 0;
    return SHD_OK;
  });
}

int shd_ctx_create(const int* device_ids, int n, shd_ctx** out) {
  return guarded([&]() -> int {
    if (!out) return fail(SHD_E_ARG, "null out");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(SHD_E_DEVICE, "no HIP device available");
    if (n > 1) return fail(SHD_E_ARG, "one device per context (one process per GPU; keys shard across processes)");
    auto* c = new shd_ctx();
    c->device = (device_ids && n > 0) ? device_ids[0] : 0;
    if (c->device < 0 || c->device >= count) {
      delete c;
      return fail(SHD_E_ARG, "bad device id");
    }
    SHD_HIP(hipSetDevice(c->device));
    *out = c;
    return SHD_OK;
  });
}

int shd_ctx_destroy(shd_ctx* ctx) {
  delete ctx;
  return SHD_OK;
}

int shd_route_words(int ncols, const int* widths, int* words) {
  return guarded([&]() -> int {
    if (!words || (ncols > 0 && !widths)) return fail(SHD_E_ARG, "null pointer");
    *words = route_words(ncols, widths);
    return SHD_OK;
  });
}

int shd_route_bucket_scratch(int64_t n, int world, size_t* bytes) {
  return guarded([&]() -> int {
    if (!bytes) return fail(SHD_E_ARG, "null pointer");
    *bytes = (size_t)route_bucket_scratch(n, world);
    return SHD_OK;
  });
}

int shd_route_bucket(shd_ctx* ctx, void* stream, int64_t n, int world, const void* key, int key_width, int ncols,
                     const void* const* cols, const int* widths, const int64_t* seq, int64_t seq_lo, uint64_t* send,
                     int64_t* counts, void* scratch) {
  return guarded([&]() -> int {
    if (!ctx || (ncols > 0 && (!cols || !widths))) return fail(SHD_E_ARG, "null pointer");
    SHD_HIP(hipSetDevice(ctx->device));
    route_bucket((hipStream_t)stream, n, world, key, key_width, ncols, cols, widths, seq, seq_lo, send, counts,
                 (uint32_t*)scratch);
    return SHD_OK;
  });
}

int shd_route_merge(shd_ctx* ctx, void* stream, int world, const uint64_t* recv, const int64_t* seg_off, int64_t m,
                    int64_t seq_lo, int64_t block, int64_t nblocks, int ncols, void* const* out_cols,
                    const int* widths, int64_t* out_seq, int64_t* start, int64_t* block_off, int32_t* err) {
  return guarded([&]() -> int {
    if (!ctx || (ncols > 0 && (!out_cols || !widths))) return fail(SHD_E_ARG, "null pointer");
    SHD_HIP(hipSetDevice(ctx->device));
    route_merge((hipStream_t)stream, world, recv, seg_off, m, seq_lo, block, nblocks, ncols, out_cols, widths,
                out_seq, start, block_off, err);
    return SHD_OK;
  });
}

int shd_plan_load(shd_ctx* ctx, const void* ir, size_t len, shd_query** out) {
  return guarded([&]() -> int {
    if (!ctx || !ir || !out || (len % 4) != 0) return fail(SHD_E_ARG, "bad arguments");
    SHD_HIP(hipSetDevice(ctx->device));
    Plan full = decode_plan((const int32_t*)ir, (int64_t)(len / 4));
    // a POST selector: the state engine projects the base values instead
    Plan p = full;
    if (full.post) {
      p.outputs = full.post_base;
      p.aggs.clear();
      p.group_by.clear();
      p.having = -1;
      p.post.reset();
      p.post_base.clear();
    }
    std::string why1, why2;
    std::unique_ptr<Engine> e;
    if (p.kind == SHD_KIND_STATE) {
      // the 2-state every-pattern shape (P1/P3) has a dedicated forward-scan
      // engine; every other state plan runs on the generic per-key NFA
      // SHD_FORCE_NFA: the generic engine for every state plan (tests, diagnostics)
      if (!getenv("SHD_FORCE_NFA")) e = make_pattern_engine(p, why1);
      // SHD_NO_LOGICAL_SCAN: leave `every e1 -> (e2 or e3)` to the generic NFA engine (tests)
      if (!e && !getenv("SHD_NO_LOGICAL_SCAN") && !getenv("SHD_FORCE_NFA")) e = make_logical_pattern_engine(p, why1);
      // SHD_NO_ABSENT_SCAN: leave `every e1 -> not X for t` to the generic NFA engine (tests)
      if (!e && !getenv("SHD_NO_ABSENT_SCAN") && !getenv("SHD_FORCE_NFA")) e = make_absent_engine(p, why1);
      if (!e) e = make_nfa_engine(p, why2);
      if (!e) why1 += "; ";
    } else {
      e = make_single_engine(p, why2);
    }
    if (!e) return fail(SHD_E_UNSUPPORTED, "plan outside the device path: " + why1 + why2);
    std::unique_ptr<Engine> post;
    if (full.post) {
      std::string why3;
      post = make_window_x_engine(*full.post, why3);
      if (!post) return fail(SHD_E_UNSUPPORTED, "selector over state output: " + why3);
      init_engine(*post, *full.post);
    }
    init_engine(*e, p);
    auto* q = new shd_query();
    q->ctx = ctx;
    q->eng = std::move(e);
    q->post = std::move(post);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < len; i++) h = (h ^ ((const uint8_t*)ir)[i]) * 1099511628211ull;
    q->plan_hash = h;
    *out = q;
    return SHD_OK;
  });
}

int shd_plan_free(shd_query* q) {
  if (q && q->eng && q->eng->grouped) return fail(SHD_E_ARG, "query belongs to a group: free the group first");
  if (q) {
    if (q->eng && q->eng->stream) (void)hipStreamSynchronize(q->eng->stream);
    delete q;
  }
  return SHD_OK;
}

int shd_plan_engine(shd_query* q, int* engine) {
  if (!q || !engine) return fail(SHD_E_ARG, "null");
  *engine = q->eng->kind();
  return SHD_OK;
}

int shd_query_stream(shd_query* q, void** stream) {
  if (!q || !stream) return fail(SHD_E_ARG, "null");
  *stream = (void*)q->eng->stream;
  return SHD_OK;
}

int shd_set_time(shd_query* q, int64_t ts) {
  return guarded([&]() -> int {
    if (!q) return fail(SHD_E_ARG, "null query");
    q->eng->args_begin();
    q->eng->set_time(ts);
    run_post(q);
    return SHD_OK;
  });
}

}  // extern "C"

namespace {
// shd_push's body: validate b against q's schema, stage it (host batches into
// q's pinned staging + H2D on q's stream), push; a NeedNfa from the engine goes
// to on_need_nfa with the staged batch and the counters before the push.
template <class OnNfa>
int push_batch(shd_query* q, const shd_batch* b, OnNfa&& on_need_nfa) {
  Engine& e = *q->eng;
  if (b->stream < 0 || b->stream >= (int)e.plan.stream_types.size()) return fail(SHD_E_ARG, "bad stream index");
  const auto& types = e.plan.stream_types[b->stream];
  if (b->ncols != (int)types.size()) return fail(SHD_E_ARG, "column count does not match the stream schema");
  if ((int)types.size() > kMaxCols) return fail(SHD_E_UNSUPPORTED, "too many attributes");
  if (b->n < 0 || (b->n > 0 && (!b->ts || !b->cols))) return fail(SHD_E_ARG, "bad batch");
  if (b->n == 0) return SHD_OK;
  // every column carries n value slots, null rows included (device kernels
  // load the value and the null byte together)
  for (int c = 0; c < b->ncols; c++)
    if (!b->cols[c]) return fail(SHD_E_ARG, "null column pointer (null rows still need a value slot)");
  SHD_HIP(hipSetDevice(q->ctx->device));
  Staged st;
  st.stream = b->stream;
  st.n = b->n;
  st.advance_time = b->advance_time != 0;
  if (b->ncalls > 0 && b->call_offsets) {
    st.call_offsets.assign(b->call_offsets, b->call_offsets + b->ncalls + 1);
    if (st.call_offsets.front() != 0 || st.call_offsets.back() != b->n) return fail(SHD_E_ARG, "bad call offsets");
  } else {
    st.call_offsets = {0, b->n};
  }
  st.cs.ncols = b->ncols;
  st.cs.n = b->n;
  if (b->mem == SHD_MEM_DEVICE) {
    st.cs.ts = b->ts;
    for (int c = 0; c < b->ncols; c++) {
      st.cs.col[c] = b->cols[c];
      st.cs.nul[c] = b->nulls ? b->nulls[c] : nullptr;
      st.cs.type[c] = (int8_t)types[c];
    }
  } else {
    // Host batches: copy into library-owned pinned memory, then H2D on the
    // query's stream.
    stage_host(e.stream, q->pin, q->stage_ts, q->stage_col, q->stage_nul, b, types, st);
  }
  if (b->use_base_seq) {
    if (b->base_seq < e.seq) return fail(SHD_E_ARG, "base_seq precedes events already pushed");
    e.seq = b->base_seq;   // in_seq of this batch's rows = base_seq + row
  }
  const shd_counters before = e.counters;
  e.args_begin();
  try {
    e.push(st);
  } catch (NeedNfa& nf) {
    on_need_nfa(st, before, nf);
  }
  q->eng->counters.kernel_ns_total += q->eng->counters.kernel_ns;
  return SHD_OK;
}
}  // namespace

extern "C" {

int shd_push(shd_query* q, const shd_batch* b) {
  return guarded([&]() -> int {
    if (!q || !b) return fail(SHD_E_ARG, "null argument");
    if (q->eng->grouped) return fail(SHD_E_ARG, "query belongs to a group: push through shd_group_push");
    const int rc = push_batch(q, b, [&](const Staged& st, const shd_counters& before, const NeedNfa& nf) {
      switch_to_nfa(q, st, before, nf.what());
    });
    if (rc == SHD_OK) run_post(q);
    return rc;
  });
}

int shd_set_option(shd_query* q, const char* key, int64_t value) {
  return guarded([&]() -> int {
    if (!q || !key) return fail(SHD_E_ARG, "null argument");
    SHD_HIP(hipStreamSynchronize(q->eng->stream));
    q->eng->set_option(key, value);
    return SHD_OK;
  });
}

int shd_flush(shd_query* q) {
  return guarded([&]() -> int {
    if (!q) return fail(SHD_E_ARG, "null query");
    SHD_HIP(hipStreamSynchronize(q->eng->stream));
    return SHD_OK;
  });
}

int shd_poll(shd_query* q, shd_out* out) {
  return guarded([&]() -> int {
    if (!q || !out) return fail(SHD_E_ARG, "null argument");
    Engine& e = q->out_eng();
    hipStream_t s = e.stream;
    int64_t n = e.out.count;
    int nc = e.out.ncols;
    q->h_chunk.resize(std::max<int64_t>(n, 1));
    q->h_type.resize(std::max<int64_t>(n, 1));
    q->h_ts.resize(std::max<int64_t>(n, 1));
    q->h_seq.resize(std::max<int64_t>(n, 1));
    q->h_sidx.resize(std::max<int64_t>(n, 1));
    q->h_vals.resize(std::max<int64_t>(n * nc, 1));
    q->h_nulls.resize(std::max<int64_t>(n * nc, 1));
    if (n > 0) {
      SHD_HIP(hipMemcpyAsync(q->h_chunk.data(), e.out.chunk.p, n * 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipMemcpyAsync(q->h_type.data(), e.out.type.p, n * 4, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipMemcpyAsync(q->h_ts.data(), e.out.ts.p, n * 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipMemcpyAsync(q->h_seq.data(), e.out.seq.p, n * 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipMemcpyAsync(q->h_sidx.data(), e.out.sidx.p, n * 4, hipMemcpyDeviceToHost, s));
      if (nc > 0) {
        SHD_HIP(hipMemcpyAsync(q->h_vals.data(), e.out.vals.p, n * nc * 8, hipMemcpyDeviceToHost, s));
        SHD_HIP(hipMemcpyAsync(q->h_nulls.data(), e.out.nulls.p, n * nc, hipMemcpyDeviceToHost, s));
      }
    }
    const int64_t nl = e.out.lcount;
    q->h_lvals.resize(std::max<int64_t>(nl, 1));
    q->h_lnul.resize(std::max<int64_t>(nl, 1));
    if (nl > 0) {
      SHD_HIP(hipMemcpyAsync(q->h_lvals.data(), e.out.lvals.p, nl * 8, hipMemcpyDeviceToHost, s));
      SHD_HIP(hipMemcpyAsync(q->h_lnul.data(), e.out.lnul.p, nl, hipMemcpyDeviceToHost, s));
    }
    SHD_HIP(hipStreamSynchronize(s));
    e.out.count = 0;
    e.out.lcount = 0;
    out->n_list = nl;
    out->list_values = q->h_lvals.data();
    out->list_nulls = q->h_lnul.data();
    out->n_rows = n;
    out->n_cols = nc;
    out->chunk = q->h_chunk.data();
    out->type = q->h_type.data();
    out->ts = q->h_ts.data();
    out->values = q->h_vals.data();
    out->nulls = q->h_nulls.data();
    out->in_seq = q->h_seq.data();
    out->state_idx = q->h_sidx.data();
    return SHD_OK;
  });
}

int shd_discard_output(shd_query* q) {
  if (!q) return fail(SHD_E_ARG, "null query");
  q->eng->out.count = 0;
  q->eng->out.lcount = 0;
  if (q->post) q->post->out.count = 0;
  return SHD_OK;
}

int shd_reset(shd_query* q) {
  return guarded([&]() -> int {
    if (!q) return fail(SHD_E_ARG, "null query");
    if (q->eng->grouped) return fail(SHD_E_ARG, "query belongs to a group: reset through shd_group_reset");
    SHD_HIP(hipStreamSynchronize(q->eng->stream));
    q->eng->reset();
    if (q->post) {
      SHD_HIP(hipStreamSynchronize(q->post->stream));
      q->post->reset();
    }
    return SHD_OK;
  });
}

int shd_stage_times(shd_query* q, int64_t* ns, const char** names, int max, int* n) {
  if (!q || !n) return fail(SHD_E_ARG, "null argument");
  Engine& e = *q->eng;
  int k = std::min(e.n_stages, max);
  for (int i = 0; i < k; i++) {
    if (ns) ns[i] = e.stage_ns[i];
    if (names) names[i] = e.stage_name[i];
  }
  *n = k;
  return SHD_OK;
}

// Snapshot image: magic, version, engine kind, plan hash, the Engine's common
// fields (arrival seq, playback time, next chunk id, counters), then the
// engine's own section (Engine::save_state).  Pending output rows must have
// been polled (the runtime drains after every push).
static void save_post(Engine& b, SnapW& w);
static constexpr uint32_t kSnapMagic = 0x53444853u;   // "SHDS"
static constexpr uint32_t kSnapVersion = 2;   // 2: + layout hint and start time

int shd_snapshot(shd_query* q, const void** data, size_t* len) {
  return guarded([&]() -> int {
    if (!q || !data || !len) return fail(SHD_E_ARG, "null argument");
    Engine& e = *q->eng;
    if (e.grouped) return fail(SHD_E_UNSUPPORTED, "a grouped query has no state of its own to snapshot");
    SHD_HIP(hipStreamSynchronize(e.stream));
    if (e.out.count > 0 || q->out_eng().out.count > 0) return fail(SHD_E_ARG, "snapshot with unpolled output rows");
    SnapW w;
    w.s = e.stream;
    w.put<uint32_t>(kSnapMagic);
    w.put<uint32_t>(kSnapVersion);
    w.put<int32_t>(e.kind());
    w.put<int64_t>(e.layout_hint);
    w.put<int64_t>(e.start_time);
    w.put<uint64_t>(q->plan_hash);
    w.put<int64_t>(e.seq);
    w.put<int64_t>(e.now);
    w.put<int64_t>(e.chunk_seq);
    w.put<shd_counters>(e.counters);
    e.save_state(w);
    if (q->post) save_post(*q->post, w);
    q->snap.swap(w.b);
    *data = q->snap.data();
    *len = q->snap.size();
    return SHD_OK;
  });
}

// The selector engine of a POST plan (its aggregator tables): common fields
// + its own section, after the state engine's.
static void save_post(Engine& b, SnapW& w) {
  SHD_HIP(hipStreamSynchronize(b.stream));
  w.s = b.stream;
  w.put<int64_t>(b.seq);
  w.put<int64_t>(b.now);
  w.put<int64_t>(b.chunk_seq);
  b.save_state(w);
}

static void load_post(Engine& b, SnapR& r) {
  b.reset();
  const int64_t seq = r.get<int64_t>(), now = r.get<int64_t>(), chunk = r.get<int64_t>();
  r.s = b.stream;
  b.load_state(r);
  b.seq = seq;
  b.now = now;
  b.chunk_seq = chunk;
  b.out.count = 0;
}

// Common fields + engine section of an image, from after the header
// (post: the query's selector engine, whose section follows).
static void load_image(Engine& e, SnapR& r, Engine* post = nullptr) {
  e.reset();
  const int64_t seq = r.get<int64_t>(), now = r.get<int64_t>(), chunk = r.get<int64_t>();
  const shd_counters c = r.get<shd_counters>();
  e.load_state(r);
  if (post) load_post(*post, r);
  if (r.at != r.n) throw Error(SHD_E_ARG, "trailing bytes in snapshot");
  e.seq = seq;
  e.now = now;
  e.chunk_seq = chunk;
  e.counters = c;
  e.out.count = 0;
}

int shd_restore(shd_query* q, const void* data, size_t len) {
  return guarded([&]() -> int {
    if (!q || (!data && len)) return fail(SHD_E_ARG, "null argument");
    Engine& cur = *q->eng;
    if (cur.grouped) return fail(SHD_E_ARG, "query belongs to a group: free the group before restoring it");
    SHD_HIP(hipStreamSynchronize(cur.stream));
    SnapR r;
    r.p = (const uint8_t*)data;
    r.n = len;
    r.s = cur.stream;
    if (r.get<uint32_t>() != kSnapMagic || r.get<uint32_t>() != kSnapVersion)
      return fail(SHD_E_ARG, "not a libsiddhi_hip snapshot (or another version)");
    const int kind = r.get<int32_t>();
    const int64_t hint = r.get<int64_t>();
    const int64_t start = r.get<int64_t>();
    if (r.get<uint64_t>() != q->plan_hash) return fail(SHD_E_ARG, "snapshot was taken from a different plan");
    if (kind != cur.kind() || hint != cur.layout_hint) {
      // the image comes from the other engine of this plan (a pattern query
      // that switched to the generic NFA engine, or the reverse) or from an
      // NFA engine built with another layout (a hand-over sizes its lists from
      // the replay): restore into a fresh engine of that kind and layout; a bad
      // image leaves q untouched
      std::string why;
      std::unique_ptr<Engine> fresh;
      if (kind == ENG_NFA) fresh = make_nfa_engine(cur.plan, why, hint);
      else if (kind == ENG_PATTERN) {
        fresh = make_pattern_engine(cur.plan, why);
        if (!fresh) fresh = make_logical_pattern_engine(cur.plan, why);
        if (!fresh) fresh = make_absent_engine(cur.plan, why);
      }
      if (!fresh || fresh->kind() != kind) return fail(SHD_E_ARG, "snapshot of an engine this plan cannot run on");
      init_engine(*fresh, cur.plan);
      fresh->start_time = start;
      r.s = fresh->stream;
      load_image(*fresh, r, q->post.get());
      q->eng = std::move(fresh);
      return SHD_OK;
    }
    // in place: keep an image of the current state, so that a truncated or
    // mismatched snapshot leaves the query as it was
    SnapW bk;
    bk.s = cur.stream;
    bk.put<int64_t>(cur.seq);
    bk.put<int64_t>(cur.now);
    bk.put<int64_t>(cur.chunk_seq);
    bk.put<shd_counters>(cur.counters);
    cur.save_state(bk);
    if (q->post) save_post(*q->post, bk);
    try {
      load_image(cur, r, q->post.get());
      cur.start_time = start;
    } catch (...) {
      SnapR br;
      br.p = bk.b.data();
      br.n = bk.b.size();
      br.s = cur.stream;
      load_image(cur, br, q->post.get());
      throw;
    }
    return SHD_OK;
  });
}

int shd_get_counters(shd_query* q, shd_counters* c) {
  if (!q || !c) return fail(SHD_E_ARG, "null argument");
  *c = q->eng->counters;
  return SHD_OK;
}

// ---- query groups (include/siddhi_hip.h)
struct shd_group {
  shd_query* leader = nullptr;          // owned: loaded from the leader IR
  std::vector<shd_query*> members;      // caller-owned
  bool dissolved = false;               // members run alone (after a NeedNfa hand-over)
};

int shd_group_create(shd_ctx* ctx, const void* leader_ir, size_t len, shd_query* const* members, int n,
                     shd_group** out) {
  return guarded([&]() -> int {
    if (!ctx || !leader_ir || !members || n <= 0 || !out) return fail(SHD_E_ARG, "bad arguments");
    shd_query* lq = nullptr;
    int rc = shd_plan_load(ctx, leader_ir, len, &lq);
    if (rc != SHD_OK) return rc;
    std::unique_ptr<shd_query> own(lq);
    std::vector<Engine*> es;
    if (lq->post) return fail(SHD_E_UNSUPPORTED, "a query with an aggregating / having selector cannot lead a group");
    for (int i = 0; i < n; i++) {
      if (!members[i]) return fail(SHD_E_ARG, "null member");
      if (members[i]->post) return fail(SHD_E_UNSUPPORTED, "group member with an aggregating / having selector");
      if (members[i]->ctx->device != ctx->device) return fail(SHD_E_ARG, "group member on another device");
      SHD_HIP(hipStreamSynchronize(members[i]->eng->stream));
      es.push_back(members[i]->eng.get());
    }
    lq->eng->group_attach(es);
    auto* g = new shd_group();
    g->leader = own.release();
    g->members.assign(members, members + n);
    *out = g;
    return SHD_OK;
  });
}

int shd_group_push(shd_group* g, const shd_batch* b) {
  return guarded([&]() -> int {
    if (!g || !b) return fail(SHD_E_ARG, "null argument");
    // dissolved: every member alone; members stay marked grouped (shd_push /
    // shd_plan_free refuse them) until shd_group_free
    auto push_members = [&]() -> int {
      for (shd_query* q : g->members) {
        int rc = push_batch(q, b, [&](const Staged& st, const shd_counters& before, const NeedNfa& nf) {
          switch_to_nfa(q, st, before, nf.what());
        });
        q->eng->grouped = true;
        if (rc != SHD_OK) return rc;
      }
      return SHD_OK;
    };
    if (g->dissolved) return push_members();
    shd_query* lq = g->leader;
    return push_batch(lq, b, [&](const Staged& st, const shd_counters&, const NeedNfa& nf) {
      if (dynamic_cast<const NeedDissolve*>(&nf)) {
        // window group: members adopt the leader's window, then take this
        // push (and all later ones) alone
        lq->eng->group_dissolve();
        g->dissolved = true;
        for (shd_query* q : g->members) q->eng->grouped = true;
        const int rc = push_members();
        if (rc != SHD_OK) throw Error(rc, g_err);
        return;
      }
      // the leader's open partials, replayed into each member's generic NFA
      // engine, rebuild exactly that member's (its f1 re-selects them); each
      // member then takes this batch on its own and the group runs dissolved
      SHD_HIP(hipStreamSynchronize(lq->eng->stream));
      std::vector<Replay> parts;
      lq->eng->export_replay(parts);
      const int64_t seq = lq->eng->seq;
      lq->eng->group_detach();
      g->dissolved = true;
      for (shd_query* q : g->members) {
        q->eng->seq = seq;
        const shd_counters before = q->eng->counters;
        switch_to_nfa(q, st, before, nf.what(), &parts);
        q->eng->counters.kernel_ns_total += q->eng->counters.kernel_ns;
        q->eng->grouped = true;   // the new engine stays in the (dissolved) group
      }
    });
  });
}

int shd_group_reset(shd_group* g) {
  return guarded([&]() -> int {
    if (!g) return fail(SHD_E_ARG, "null group");
    SHD_HIP(hipStreamSynchronize(g->leader->eng->stream));
    g->leader->eng->reset();
    for (shd_query* q : g->members) {
      SHD_HIP(hipStreamSynchronize(q->eng->stream));
      q->eng->reset();
    }
    return SHD_OK;
  });
}

int shd_group_leader(shd_group* g, shd_query** leader) {
  if (!g || !leader) return fail(SHD_E_ARG, "null argument");
  *leader = g->leader;
  return SHD_OK;
}

int shd_group_free(shd_group* g) {
  if (!g) return SHD_OK;
  (void)hipStreamSynchronize(g->leader->eng->stream);
  g->leader->eng->group_detach();
  for (shd_query* q : g->members) {
    q->eng->grouped = false;
    q->eng->reset();
  }
  delete g->leader;
  delete g;
  return SHD_OK;
}

}  // extern "C"

