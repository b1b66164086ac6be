// dev_expr.h -- per-lane interpreter for the filter / projection bytecode
// (include/siddhi_ir.h), one expression evaluation per lane.
//
// Semantics restate the reference executors (paths under
// modules/siddhi-core/src/main/java/io/siddhi/core/executor/):
//   compare: condition/compare/CompareConditionExpressionExecutor.java:38-42 (null -> false)
//            and the per-type subclasses (operands pre-converted by the planner)
//   and/or/not/isnull: condition/{And,Or,Not,IsNull}ConditionExpressionExecutor.java
//   + - * / %: math/*/*ExpressionExecutor{Int,Long,Float,Double}.java
//            (null operand -> null; / and % by zero -> null; int wrap-around)
// Compiled with -ffp-contract=off so float/double ops round exactly like Java.
#pragma once
#include "common.h"

namespace shd {

struct Val {
  uint64_t b;
  int null;
};

__device__ __forceinline__ int32_t v_i32(uint64_t b) { return (int32_t)(uint32_t)b; }
__device__ __forceinline__ int64_t v_i64(uint64_t b) { return (int64_t)b; }
__device__ __forceinline__ float v_f32(uint64_t b) { return __uint_as_float((uint32_t)b); }
__device__ __forceinline__ double v_f64(uint64_t b) { return __longlong_as_double((long long)b); }
__device__ __forceinline__ uint64_t p_i32(int32_t v) { return (uint64_t)(int64_t)v; }
__device__ __forceinline__ uint64_t p_f32(float f) { return (uint64_t)__float_as_uint(f); }
__device__ __forceinline__ uint64_t p_f64(double d) { return (uint64_t)__double_as_longlong(d); }

// Typed column element -> 64-bit payload.
__device__ __forceinline__ Val col_load(const ColSet& cs, int64_t row, int attr) {
  Val v;
#ifdef SHD_DEBUG
  if (attr < 0 || attr >= cs.ncols || row < 0 || row >= cs.n || cs.col[attr] == nullptr ||
      ((uintptr_t)cs.col[attr] >> 47) != 0 || ((uintptr_t)cs.nul[attr] >> 47) != 0) {
    printf("SHD_DEBUG col_load: attr %d ncols %d row %lld n %lld col %p\n", attr, cs.ncols, (long long)row,
           (long long)cs.n,
           attr >= 0 && attr < kMaxCols ? cs.col[attr] : nullptr);
    v.b = 0;
    v.null = 1;
    return v;
  }
#endif
  if ((unsigned)attr >= (unsigned)cs.ncols) {   // plan validated at load; never index past the column table
    v.b = 0;
    v.null = 1;
    return v;
  }
  // value and null byte are loaded together (a null row still has a value
  // slot), so the two loads overlap instead of costing two round trips
  const uint8_t* nm = cs.nul[attr];
  v.null = 0;
  switch (cs.type[attr]) {
    case SHD_T_STRING: v.b = gld((const uint32_t*)cs.col[attr], row); break;
    case SHD_T_INT: v.b = p_i32(gld((const int32_t*)cs.col[attr], row)); break;
    case SHD_T_LONG: v.b = (uint64_t)gld((const int64_t*)cs.col[attr], row); break;
    case SHD_T_FLOAT: v.b = (uint64_t)gld((const uint32_t*)cs.col[attr], row); break;
    case SHD_T_DOUBLE: v.b = gld((const uint64_t*)cs.col[attr], row); break;
    case SHD_T_BOOL: v.b = gld((const uint8_t*)cs.col[attr], row) ? 1 : 0; break;
    default: v.b = 0; v.null = 1;
  }
  if (nm && gld(nm, row)) {
    v.b = 0;
    v.null = 1;
  }
  return v;
}

// col_load of one column given by its pointers and type (pre-resolved
// descriptors: no column-table lookups per call).
__device__ __forceinline__ Val col_load_raw(const void* col, const uint8_t* nm, int type, int64_t row) {
  Val v;
  v.null = 0;
  switch (type) {
    case SHD_T_STRING: v.b = gld((const uint32_t*)col, row); break;
    case SHD_T_INT: v.b = p_i32(gld((const int32_t*)col, row)); break;
    case SHD_T_LONG: v.b = (uint64_t)gld((const int64_t*)col, row); break;
    case SHD_T_FLOAT: v.b = (uint64_t)gld((const uint32_t*)col, row); break;
    case SHD_T_DOUBLE: v.b = gld((const uint64_t*)col, row); break;
    case SHD_T_BOOL: v.b = gld((const uint8_t*)col, row) ? 1 : 0; break;
    default: v.b = 0; v.null = 1;
  }
  if (nm && gld(nm, row)) {
    v.b = 0;
    v.null = 1;
  }
  return v;
}

// Number.xValue() widening used by the planner's CVT ops.
__device__ __forceinline__ uint64_t d_cvt(uint64_t b, int from, int to) {
  if (from == to) return b;
  double d = 0.0;
  float f = 0.f;
  int64_t l = 0;
  switch (from) {
    case SHD_T_INT: l = v_i32(b); d = (double)v_i32(b); f = (float)v_i32(b); break;
    case SHD_T_LONG: l = v_i64(b); d = (double)v_i64(b); f = (float)v_i64(b); break;
    case SHD_T_FLOAT: d = (double)v_f32(b); f = v_f32(b); l = (int64_t)v_f32(b); break;
    case SHD_T_DOUBLE: d = v_f64(b); f = (float)v_f64(b); l = (int64_t)v_f64(b); break;
  }
  switch (to) {
    case SHD_T_INT: return p_i32((int32_t)l);
    case SHD_T_LONG: return (uint64_t)l;
    case SHD_T_FLOAT: return p_f32(f);
    case SHD_T_DOUBLE: return p_f64(d);
  }
  return b;
}

__device__ inline Val d_arith(int op, int t, Val l, Val r) {
  Val o;
  o.b = 0;
  o.null = 1;
  if (l.null || r.null) return o;
  o.null = 0;
  switch (t) {
    case SHD_T_INT: {
      int32_t a = v_i32(l.b), b = v_i32(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = p_i32((int32_t)((uint32_t)a + (uint32_t)b)); break;
        case SHD_OP_SUB: o.b = p_i32((int32_t)((uint32_t)a - (uint32_t)b)); break;
        case SHD_OP_MUL: o.b = p_i32((int32_t)((uint32_t)a * (uint32_t)b)); break;
        case SHD_OP_DIV:
          if (b == 0) o.null = 1;
          else o.b = p_i32((a == INT32_MIN && b == -1) ? INT32_MIN : a / b);
          break;
        case SHD_OP_MOD:
          if (b == 0) o.null = 1;
          else o.b = p_i32(b == -1 ? 0 : a % b);
          break;
      }
      break;
    }
    case SHD_T_LONG: {
      int64_t a = v_i64(l.b), b = v_i64(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = (uint64_t)a + (uint64_t)b; break;
        case SHD_OP_SUB: o.b = (uint64_t)a - (uint64_t)b; break;
        case SHD_OP_MUL: o.b = (uint64_t)a * (uint64_t)b; break;
        case SHD_OP_DIV:
          if (b == 0) o.null = 1;
          else o.b = (uint64_t)((a == INT64_MIN && b == -1) ? INT64_MIN : a / b);
          break;
        case SHD_OP_MOD:
          if (b == 0) o.null = 1;
          else o.b = (uint64_t)(b == -1 ? 0 : a % b);
          break;
      }
      break;
    }
    case SHD_T_FLOAT: {
      float a = v_f32(l.b), b = v_f32(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = p_f32(__fadd_rn(a, b)); break;
        case SHD_OP_SUB: o.b = p_f32(__fsub_rn(a, b)); break;
        case SHD_OP_MUL: o.b = p_f32(__fmul_rn(a, b)); break;
        case SHD_OP_DIV:
          if (b == 0.0f) o.null = 1;
          else o.b = p_f32(__fdiv_rn(a, b));
          break;
        case SHD_OP_MOD:
          if (b == 0.0f) o.null = 1;
          else o.b = p_f32(fmodf(a, b));
          break;
      }
      break;
    }
    case SHD_T_DOUBLE: {
      double a = v_f64(l.b), b = v_f64(r.b);
      switch (op) {
        case SHD_OP_ADD: o.b = p_f64(__dadd_rn(a, b)); break;
        case SHD_OP_SUB: o.b = p_f64(__dsub_rn(a, b)); break;
        case SHD_OP_MUL: o.b = p_f64(__dmul_rn(a, b)); break;
        case SHD_OP_DIV:
          if (b == 0.0) o.null = 1;
          else o.b = p_f64(__ddiv_rn(a, b));
          break;
        case SHD_OP_MOD:
          if (b == 0.0) o.null = 1;
          else o.b = p_f64(fmod(a, b));
          break;
      }
      break;
    }
  }
  return o;
}

__device__ inline bool d_compare(int op, int t, uint64_t l, uint64_t r) {
  int c;  // -1 lt, 0 eq, 1 gt, 2 unordered / not-equal
  switch (t) {
    case SHD_T_STRING:
    case SHD_T_BOOL:
      c = (l == r) ? 0 : 2;
      break;
    case SHD_T_INT: {
      int32_t a = v_i32(l), b = v_i32(r);
      c = a < b ? -1 : (a > b ? 1 : 0);
      break;
    }
    case SHD_T_LONG: {
      int64_t a = v_i64(l), b = v_i64(r);
      c = a < b ? -1 : (a > b ? 1 : 0);
      break;
    }
    case SHD_T_FLOAT: {
      float a = v_f32(l), b = v_f32(r);
      c = (a < b) ? -1 : (a > b) ? 1 : (a == b) ? 0 : 2;
      break;
    }
    default: {
      double a = v_f64(l), b = v_f64(r);
      c = (a < b) ? -1 : (a > b) ? 1 : (a == b) ? 0 : 2;
      break;
    }
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

// Evaluate one expression. Ctx provides:
//   Val load(int state, int idx, int attr) const;  bool evnull(int state, int idx) const;
//   int64_t ts(int state, int idx) const;          Val agg(int i) const;
// Value stack of the interpreter.  Slots live in named registers and are
// addressed through unrolled selects (slot indices are wave-uniform), so the
// evaluation never touches scratch memory: no dynamically indexed private
// array exists for the compiler to spill or to speculate out of bounds.
struct VStack {
  uint64_t r[kMaxStack];
  uint32_t nul;   // bit i = slot i is null
  __device__ __forceinline__ uint64_t get(int i) const {
    uint64_t v = 0;
#pragma unroll
    for (int j = 0; j < kMaxStack; j++)
      if (j == i) v = r[j];
    return v;
  }
  __device__ __forceinline__ void set(int i, uint64_t v, int null) {
#pragma unroll
    for (int j = 0; j < kMaxStack; j++)
      if (j == i) r[j] = v;
    nul = null ? (nul | (1u << i)) : (nul & ~(1u << i));
  }
  __device__ __forceinline__ int isnull(int i) const { return (nul >> i) & 1u; }
  __device__ __forceinline__ Val val(int i) const {
    Val v;
    v.b = get(i);
    v.null = isnull(i);
    return v;
  }
};

// Evaluate one expression.  The host validated every expression of the plan
// (stack depth <= kMaxStack, no underflow: shd_api.cpp decode_plan), so sp
// stays inside [0, kMaxStack].
template <class Ctx>
__device__ inline Val eval_expr(const int4* code, int len, const uint64_t* consts, const Ctx& cx) {
  VStack st;
#pragma unroll
  for (int j = 0; j < kMaxStack; j++) st.r[j] = 0;
  st.nul = 0;
  int sp = 0;
  for (int k = 0; k < len; k++) {
    const int4 in = code[k];
    switch (in.x) {
      case SHD_OP_CONST: st.set(sp++, consts[in.y], 0); break;
      case SHD_OP_NULL: st.set(sp++, 0, 1); break;
      case SHD_OP_LOAD: {
        Val v = cx.load(in.y, in.z, in.w & 0xFFFF);
        st.set(sp++, v.b, v.null);
        break;
      }
      case SHD_OP_EVNULL: st.set(sp++, cx.evnull(in.y, in.z) ? 1 : 0, 0); break;
      case SHD_OP_TS: st.set(sp++, (uint64_t)cx.ts(in.y, in.z), 0); break;
      case SHD_OP_CVT:
        if (sp > 0 && !st.isnull(sp - 1)) st.set(sp - 1, d_cvt(st.get(sp - 1), in.y, in.z), 0);
        break;
      case SHD_OP_ADD: case SHD_OP_SUB: case SHD_OP_MUL: case SHD_OP_DIV: case SHD_OP_MOD: {
        if (sp < 2) break;
        Val r = st.val(sp - 1);
        Val l = st.val(sp - 2);
        Val o = d_arith(in.x, in.y, l, r);
        sp -= 2;
        st.set(sp++, o.b, o.null);
        break;
      }
      case SHD_OP_EQ: case SHD_OP_NE: case SHD_OP_GT: case SHD_OP_GE: case SHD_OP_LT: case SHD_OP_LE: {
        if (sp < 2) break;
        Val r = st.val(sp - 1);
        Val l = st.val(sp - 2);
        sp -= 2;
        st.set(sp++, (!(l.null || r.null) && d_compare(in.x, in.y, l.b, r.b)) ? 1 : 0, 0);
        break;
      }
      case SHD_OP_AND: case SHD_OP_OR: {
        if (sp < 2) break;
        Val r = st.val(sp - 1);
        Val l = st.val(sp - 2);
        bool lt = !l.null && l.b, rt = !r.null && r.b;
        sp -= 2;
        st.set(sp++, (in.x == SHD_OP_AND ? (lt && rt) : (lt || rt)) ? 1 : 0, 0);
        break;
      }
      case SHD_OP_NOT:
        if (sp > 0) st.set(sp - 1, (!st.isnull(sp - 1) && st.get(sp - 1)) ? 0 : 1, 0);
        break;
      case SHD_OP_ISNULL:
        if (sp > 0) st.set(sp - 1, st.isnull(sp - 1) ? 1 : 0, 0);
        break;
      case SHD_OP_AGG: {
        Val v = cx.agg(in.y);
        st.set(sp++, v.b, v.null);
        break;
      }
      case SHD_OP_IFELSE: {   // IfThenElseFunctionExecutor: Boolean.TRUE.equals(cond) ? then : else
        if (sp < 3) break;
        const Val e = st.val(sp - 1), t = st.val(sp - 2), c = st.val(sp - 3);
        const Val o = (!c.null && c.b) ? t : e;
        sp -= 3;
        st.set(sp++, o.b, o.null);
        break;
      }
      default:
        break;
    }
    if (sp > kMaxStack) sp = kMaxStack;
  }
  if (sp == 0) {
    Val z;
    z.b = 0;
    z.null = 1;
    return z;
  }
  return st.val(sp - 1);
}

template <class Ctx>
__device__ __forceinline__ bool eval_bool(const int4* code, int len, const uint64_t* consts, const Ctx& cx) {
  Val v = eval_expr(code, len, consts, cx);
  return !v.null && v.b;
}

// Expression handle passed to kernels (offset/length into the plan's table).
struct DExpr {
  int off;
  int len;
};

struct DExprSet {
  const int4* ins;
  const uint64_t* consts;
  int nins, nconsts;
};

// Expression program placement: the program stays in global memory (the
// uniform instruction reads are served by the scalar / L1 caches).  Staging
// it into LDS at kernel start was measured to fault on the MI355X pool in the
// single-stream kernels (k_filter: memory aperture violation for any batch
// size, while the identical kernels reading the program from global memory
// pass: scripts/probe_filter.py, DESIGN.md "LDS program staging").  Plans
// larger than kLdsIns / kLdsConsts are still rejected at load
// (DevExprTable::upload).
constexpr int kLdsIns = 256;
constexpr int kLdsConsts = 64;

// ---------------------------------------------------------------- fast predicates
// Filter chains whose bytecode is a conjunction of comparisons between simple
// terms are pre-decoded on the host (compile_fast_pred, shd_api.cpp) into a
// fixed-shape descriptor evaluated as straight-line code: no instruction
// fetch per event.  The descriptor is wave-uniform (it sits in the kernel's
// argument block), so every branch below is a scalar branch.  It applies the
// same operations as the interpreter in the same order (d_cvt / d_arith /
// d_compare, null propagation), so results are identical; any other bytecode
// shape falls back to eval_expr.
//   atom := LOAD | CONST | NULL, optionally followed by one CVT
//   term := atom | atom atom ARITH
//   cmp  := term term COMPARE          pred := cmp (AND cmp)*   (<= 4 cmps)
enum : int32_t { FA_NONE = 0, FA_LOAD = 1, FA_CONST = 2, FA_NULL = 3 };
// All fields are 32/64-bit: the descriptor is wave-uniform and must load with
// s_load_dword (sub-dword fields would become vector loads + vmcnt waits).
struct FAtom {
  int32_t kind, st, idx, cvt_from, cvt_to, attr;
  uint64_t cval;
};
struct FTerm {
  FAtom a, b;
  int32_t aop, atype;
};
struct FCmp {
  FTerm l, r;
  int32_t op, type;
};
struct FPred {
  int32_t ok;     // 1: the filter chain is this conjunction
  int32_t n;      // comparisons
  FCmp c[4];
};

template <class Ctx>
__device__ __forceinline__ Val fp_atom(const FAtom& a, const Ctx& cx) {
  Val v;
  v.b = 0;
  v.null = 1;
  if (a.kind == FA_LOAD) v = cx.load(a.st, a.idx, a.attr);
  else if (a.kind == FA_CONST) {
    v.b = a.cval;
    v.null = 0;
  }
  if (a.cvt_to >= 0 && !v.null) v.b = d_cvt(v.b, a.cvt_from, a.cvt_to);
  return v;
}

template <class Ctx>
__device__ __forceinline__ Val fp_term(const FTerm& t, const Ctx& cx) {
  Val l = fp_atom(t.a, cx);
  if (t.aop == 0) return l;
  Val r = fp_atom(t.b, cx);
  return d_arith(t.aop, t.atype, l, r);
}

template <class Ctx>
__device__ __forceinline__ bool eval_fpred(const FPred& p, const Ctx& cx) {
  for (int i = 0; i < p.n; i++) {
    const FCmp& c = p.c[i];
    Val l = fp_term(c.l, cx);
    Val r = fp_term(c.r, cx);
    if (l.null || r.null || !d_compare(c.op, c.type, l.b, r.b)) return false;
  }
  return true;
}

// Conjunction of up to 4 filter expressions (FilterProcessor chain).
struct DFilters {
  DExpr f[4];
  int n;
  FPred fp;
};

template <class Ctx>
__device__ __forceinline__ bool eval_filters(const DExprSet& es, const DFilters& fs, const Ctx& cx) {
  if (fs.fp.ok) return eval_fpred(fs.fp, cx);
  for (int i = 0; i < fs.n; i++)
    if (!eval_bool(es.ins + fs.f[i].off, fs.f[i].len, es.consts, cx)) return false;
  return true;
}

}  // namespace shd
