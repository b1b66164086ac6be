/*
 * siddhi_ir.h -- the versioned plan IR shared by the host planner
 * (siddhi_amd/planner.py), libsiddhi_hip (siddhi_amd/csrc) and the CPU
 * oracle (oracle/).  Constants only: every consumer has its own decoder.
 *
 * A plan is a little-endian array of int32 words:
 *
 *   magic 'SHDP', version, kind (1 = STATE, 2 = SINGLE)
 *   n_streams, { n_attrs, type[n_attrs] } * n_streams      (plan-local streams)
 *   n_consts,  { lo, hi } * n_consts                         (64-bit bit patterns)
 *   n_exprs,   { n_instr, { op, a, b, c } * n_instr } * n_exprs
 *   partition: n_keys, { stream, expr } * n_keys             (n_keys = 0: unpartitioned)
 *   STATE:  state_type, within_lo, within_hi, n_states, node tree (prefix order)
 *   SINGLE: stream, n_handlers, { FILTER expr | WINDOW kind p_lo p_hi q_lo q_hi } * n_handlers
 *     (p = the window's first parameter, q = its second: see shd_window)
 *   selector: current_on, expired_on, n_aggs { kind, arg_expr, arg_type } ,
 *             n_group { expr }, having_expr, n_out { type, expr }
 *   optional trailing words:
 *     null_lo, null_hi       dictionary id of the string "null" (string group keys)
 *     POST section (STATE plans whose selector aggregates or has `having`):
 *       SHD_IR_POST_MAGIC, n_base, { type, expr } * n_base, n_words, <SINGLE plan words>
 *     The selector runs on one StateEvent per chunk
 *     (StateMultiProcessStreamReceiver.processAndClear, C/query/input/
 *     StateMultiProcessStreamReceiver.java:47-68; SingleProcessStreamReceiver
 *     :48-72), so over a state query's output rows it is a sequential fold in
 *     emission order: the base expressions are the state variables the
 *     selector reads, projected per match; the nested SINGLE plan is the same
 *     selector restated over a stream whose attributes are those base values
 *     (attribute k = base k).  The oracle evaluates the selector fields above
 *     directly on StateEvents and ignores this section; libsiddhi_hip runs
 *     the state plan with the base expressions as outputs, then the nested
 *     plan over its rows with one InputHandler call per row.
 *
 * Node tree (StateInputStreamParser.parse, C/util/parser/StateInputStreamParser.java:148-408):
 *   NODE_STREAM  state_id stream absent waiting_lo waiting_hi n_filters expr*
 *   NODE_NEXT    <a> <b>
 *   NODE_EVERY   <inner>
 *   NODE_LOGICAL type(0 and, 1 or) <stream1> <stream2>
 *   NODE_COUNT   min max <stream>
 */
#ifndef SIDDHI_IR_H
#define SIDDHI_IR_H

#define SHD_IR_MAGIC 0x50444853 /* 'SHDP' */
#define SHD_IR_VERSION 1
#define SHD_IR_POST_MAGIC 0x54534F50 /* 'POST' */

enum shd_kind { SHD_KIND_STATE = 1, SHD_KIND_SINGLE = 2 };

/* Attribute types (io.siddhi.query.api.definition.Attribute.Type). STRING is
 * a host dictionary id (u32); BOOL is a byte. */
enum shd_type {
  SHD_T_STRING = 0,
  SHD_T_INT = 1,
  SHD_T_LONG = 2,
  SHD_T_FLOAT = 3,
  SHD_T_DOUBLE = 4,
  SHD_T_BOOL = 5,
  /* output only: a list (java.util.List) of values of one attribute over a
   * count state's event chain (MultiValueVariableFunctionExecutor); the
   * 64-bit payload is a handle into shd_out's list arena:
   * offset | count << 40 (SHD_LIST_*) */
  SHD_T_OBJECT = 6
};
#define SHD_LIST_OFFSET(h) ((h) & 0xFFFFFFFFFFull)
#define SHD_LIST_COUNT(h) ((h) >> 40)

/* Expression bytecode: fixed 4-word instructions {op, a, b, c} over a value
 * stack of (64-bit payload, null flag). Semantics follow
 * C/executor/{condition,math}/ (see oracle/oracle.cpp for the restatement). */
enum shd_op {
  SHD_OP_END = 0,
  SHD_OP_CONST = 1,   /* a = const index, b = type                         */
  SHD_OP_NULL = 2,    /* b = type                                          */
  SHD_OP_LOAD = 3,    /* a = state, b = chain index, c = attr | type << 16  */
  SHD_OP_EVNULL = 4,  /* a = state, b = chain index : stream event is null  */
  SHD_OP_CVT = 5,     /* a = from type, b = to type (Number.xValue())       */
  SHD_OP_ADD = 6,     /* a = type                                          */
  SHD_OP_SUB = 7,
  SHD_OP_MUL = 8,
  SHD_OP_DIV = 9,     /* divisor 0 -> null                                 */
  SHD_OP_MOD = 10,    /* divisor 0 -> null                                 */
  SHD_OP_EQ = 11,     /* a = operand type; null operand -> false           */
  SHD_OP_NE = 12,
  SHD_OP_GT = 13,
  SHD_OP_GE = 14,
  SHD_OP_LT = 15,
  SHD_OP_LE = 16,
  SHD_OP_AND = 17,    /* null -> false                                     */
  SHD_OP_OR = 18,
  SHD_OP_NOT = 19,    /* NOT(null) -> true                                 */
  SHD_OP_ISNULL = 20,
  SHD_OP_AGG = 21,    /* a = aggregator index (selector only)              */
  SHD_OP_TS = 22,     /* a = state, b = chain index : event timestamp      */
  SHD_OP_IFELSE = 23, /* a = result type; pops else, then, cond: cond true -> then, else (null cond too)
                         (C/executor/function/IfThenElseFunctionExecutor.java) */
  SHD_OP_MULTI = 24   /* a = state, c = attr | elem type << 16: the attribute over the state's
                         whole event chain, first to last, as a list (SHD_T_OBJECT); only as a
                         whole selector output (C/executor/MultiValueVariableFunctionExecutor.java,
                         wired at C/util/parser/ExpressionParser.java:1386-1437) */
};

/* Chain indices (SiddhiConstants.CURRENT / LAST, C/util/SiddhiConstants.java:89-92). */
#define SHD_IDX_CURRENT (-1)
#define SHD_IDX_LAST (-2)

enum shd_node { SHD_NODE_STREAM = 1, SHD_NODE_NEXT = 2, SHD_NODE_EVERY = 3,
                SHD_NODE_LOGICAL = 4, SHD_NODE_COUNT = 5 };

enum shd_handler { SHD_H_FILTER = 1, SHD_H_WINDOW = 2 };
/* Windows (C/query/processor/stream/window/): p = length or time (ms); q:
 *   LENGTH_BATCH  q = 1: stream.current.event, else 0 (LengthBatchWindowProcessor.java:153-274;
 *                 p = 0: processLengthZeroBatch)
 *   TIME_BATCH    q = start.time, or INT64_MIN when absent (TimeBatchWindowProcessor.java:279-366)
 *   TIME_BATCH_STREAM  the same with stream.current.event
 *   TIME_LENGTH   q = window.length (TimeLengthWindowProcessor.java:139-188)
 *   EXTERNAL_TIME q = the LONG attribute holding the event time (ExternalTimeWindowProcessor.java:124-158)
 *   LENGTH / TIME q = 0 */
enum shd_window { SHD_W_LENGTH = 1, SHD_W_TIME = 2, SHD_W_LENGTH_BATCH = 3, SHD_W_TIME_BATCH = 4,
                  SHD_W_TIME_LENGTH = 5, SHD_W_EXTERNAL_TIME = 6, SHD_W_TIME_BATCH_STREAM = 7 };
enum shd_agg { SHD_AGG_SUM = 1, SHD_AGG_AVG = 2, SHD_AGG_COUNT = 3 };

/* Output / input event types (ComplexEvent.Type). */
enum shd_evtype { SHD_EV_CURRENT = 0, SHD_EV_EXPIRED = 1, SHD_EV_TIMER = 2, SHD_EV_RESET = 3 };

#endif
