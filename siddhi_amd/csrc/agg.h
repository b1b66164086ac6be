// agg.h -- the reference's incremental aggregator steps on the device.
//
// Sum / Avg / Count AttributeAggregatorExecutor (C/query/selector/attribute/
// aggregator/*.java: processAdd / processRemove): one CURRENT (add) or EXPIRED
// (remove) operand at a time, in the reference's order, so every double sum is
// the same IEEE result (built with -ffp-contract=off).
#pragma once
#include "engine.h"

namespace shd {
namespace {

__device__ __forceinline__ int64_t java_d2l(double d) {
  if (d != d) return 0;
  if (d >= 9.2233720368547758e18) return INT64_MAX;
  if (d <= -9.2233720368547758e18) return INT64_MIN;
  return (int64_t)d;
}

// One aggregator step on a CURRENT (add) or EXPIRED (remove) event: the
// reference's incremental executors, Sum/Avg/CountAttributeAggregatorExecutor
// (.../selector/attribute/aggregator/*.java: processAdd / processRemove).
// ob/on: the aggregator's value after the step (on = null).  avg: ob is the
// running sum and the count is the state c; the division value / count happens
// at emission (k_emit) for the rows that are emitted, not in the sequential fold.
__device__ __forceinline__ void agg_step(int kind, int type, bool add, uint64_t xb, bool xn, double& d, int64_t& l,
                                         int64_t& c, uint64_t& ob, bool& on) {
  ob = 0;
  on = true;
  switch (kind) {
    case SHD_AGG_COUNT:
      c += add ? 1 : -1;
      ob = (uint64_t)c;
      on = false;
      break;
    case SHD_AGG_SUM:
      if (type == SHD_T_INT || type == SHD_T_LONG) {
        if (xn) {
          if (c != 0) { ob = (uint64_t)l; on = false; }
          break;
        }
        int64_t x = type == SHD_T_INT ? (int64_t)v_i32(xb) : (int64_t)xb;
        if (add) {
          l = (int64_t)((uint64_t)l + (uint64_t)x);
          c++;
          ob = (uint64_t)l;
          on = false;
        } else {
          l = java_d2l(__dsub_rn((double)l, (double)x));
          c--;
          if (c != 0) { ob = (uint64_t)l; on = false; }
        }
      } else {
        if (xn) {
          if (type == SHD_T_DOUBLE && c != 0) { ob = p_f64(d); on = false; }
          break;
        }
        double x = type == SHD_T_FLOAT ? (double)v_f32(xb) : v_f64(xb);
        if (add) {
          d = __dadd_rn(d, x);
          c++;
          ob = p_f64(d);
          on = false;
        } else {
          d = __dsub_rn(d, x);
          c--;
          if (c != 0) { ob = p_f64(d); on = false; }
        }
      }
      break;
    case SHD_AGG_AVG: {
      if (xn) {
        if (c != 0) { ob = p_f64(d); on = false; }
        break;
      }
      double x;
      switch (type) {
        case SHD_T_INT: x = (double)v_i32(xb); break;
        case SHD_T_LONG: x = (double)(int64_t)xb; break;
        case SHD_T_FLOAT: x = (double)v_f32(xb); break;
        default: x = v_f64(xb);
      }
      if (add) { c++; d = __dadd_rn(d, x); }
      else { c--; d = __dsub_rn(d, x); }
      if (c != 0) { ob = p_f64(d); on = false; }
      break;
    }
  }
}

}  // namespace
}  // namespace shd
