/*
 * siddhi_hip.h -- C-ABI of libsiddhi_hip, the MI355X (gfx950) implementation of
 * Siddhi's pattern / sequence / sliding-window hot path.
 *
 * This is the drop-in boundary.  The reference has no FFI; each
 * entry point replaces an in-JVM interface on the hot path:
 *
 *   shd_plan_load   <- QueryParser.parse / StateInputStreamParser.parseInputStream
 *                      (modules/siddhi-core/src/main/java/io/siddhi/core/util/parser/
 *                       QueryParser.java:94-283, StateInputStreamParser.java:76-146):
 *                      the host planner hands over a compiled plan (include/siddhi_ir.h)
 *                      instead of building Processor objects.
 *   shd_push        <- StreamJunction.Receiver.receive(Event[])
 *                      (C/stream/StreamJunction.java:443-456, reached from
 *                       InputHandler.send(Event[]), C/stream/input/InputHandler.java:85-95)
 *                      and PartitionStreamReceiver.receive(Event[])
 *                      (C/partition/PartitionStreamReceiver.java:175-216).
 *   shd_set_time    <- TimestampGeneratorImpl.setCurrentTimestamp -> Scheduler.onTimeChange
 *                      (C/util/timestamp/TimestampGeneratorImpl.java:58-76,
 *                       C/util/Scheduler.java:71-104), playback mode.
 *   shd_poll        <- OutputRateLimiter.sendToCallBacks -> QueryCallback.receiveStreamEvent /
 *                      InsertIntoStreamCallback.send
 *                      (C/query/output/ratelimit/OutputRateLimiter.java:64-107).
 *   shd_plan_free   <- QueryRuntime stop / SiddhiAppRuntime.shutdown.
 *   shd_snapshot /  <- SiddhiAppRuntime.snapshot()/restore(byte[]) -> SnapshotService.fullSnapshot/restore
 *   shd_restore        (C/SiddhiAppRuntimeImpl.java:695-717, C/util/snapshot/SnapshotService.java:90,333)
 *                      for this query's element states (State.snapshot/restore, e.g.
 *                       ST/StreamPreStateProcessor.java:450-469, LengthWindowProcessor.java:171-196).
 *
 * Conventions: every function returns an int status (0 = OK, < 0 = shd_status);
 * no exception crosses the ABI; shd_last_error() returns a thread-local message.
 * One shd_query is driven by one host thread at a time (the reference serialises
 * a query with patternSyncObject + LockWrapper, MultiProcessStreamReceiver.java:97,
 * QueryParser.java:155-215); different queries may be driven concurrently.
 */
#ifndef SIDDHI_HIP_H
#define SIDDHI_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct shd_ctx shd_ctx;
typedef struct shd_query shd_query;
typedef struct shd_group shd_group;

enum shd_status {
  SHD_OK = 0,
  SHD_E_INVALID_PLAN = -1, /* malformed IR                                      */
  SHD_E_UNSUPPORTED = -2,  /* valid plan/data outside the device path           */
  SHD_E_OOM = -3,          /* device allocation failed                          */
  SHD_E_DEVICE = -4,       /* HIP runtime error / no device                     */
  SHD_E_CAPACITY = -5,     /* a bounded table overflowed (never silently drops)  */
  SHD_E_ARG = -6           /* bad argument                                      */
};

enum shd_mem { SHD_MEM_HOST = 0, SHD_MEM_DEVICE = 1 };

/* One columnar micro-batch of ONE plan stream (the plan's stream index). */
typedef struct shd_batch {
  int32_t stream;               /* plan-local stream index                       */
  int32_t mem;                  /* SHD_MEM_HOST or SHD_MEM_DEVICE (all pointers)  */
  int64_t n;                    /* number of events                             */
  const int64_t* ts;            /* [n] event timestamps (ms)                     */
  int32_t ncols;                /* == number of attributes of the stream        */
  const void* const* cols;      /* [ncols] typed columns: string=u32 dictionary id,
                                   int=i32, long=i64, float=f32, double=f64, bool=u8;
                                   never NULL: null rows keep a (any) value slot */
  const uint8_t* const* nulls;  /* [ncols] NULL or [n] bytes, 1 = null; may be NULL */
  int32_t ncalls;               /* InputHandler.send calls in this batch (>= 1)  */
  const int64_t* call_offsets;  /* host array [ncalls+1]; NULL = one call        */
  int32_t advance_time;         /* playback: set app time to each call's last ts */
  int32_t use_base_seq;         /* 1: base_seq is given (0, the zero-initialised
                                   default: the query continues its own count) */
  int64_t base_seq;             /* arrival index of the batch's first event in the
                                   whole stream when the batch is a CONTIGUOUS
                                   slice of it: shd_out.in_seq = base_seq + row
                                   is then global; must not go back (SHD_E_ARG).
                                   Rows re-routed by key (shd_route_merge) are not
                                   contiguous: map in_seq through out_seq
                                   (exchange.merge_outputs)                    */
} shd_batch;

/* Output rows of a query since the last poll, in reference order.  Rows with
 * the same chunk id form one callback invocation (one ComplexEventChunk). */
typedef struct shd_out {
  int64_t n_rows;
  int32_t n_cols;
  const int64_t* chunk;         /* [n_rows]                                      */
  const int32_t* type;          /* [n_rows] 0 = CURRENT, 1 = EXPIRED             */
  const int64_t* ts;            /* [n_rows]                                      */
  const uint64_t* values;       /* [n_rows * n_cols] 64-bit payloads (row-major)  */
  const uint8_t* nulls;         /* [n_rows * n_cols]                             */
  const int64_t* in_seq;        /* [n_rows] arrival index (0-based, over every event
                                   pushed to this query) of the input event whose
                                   processing emitted the row -- the completing
                                   event of a match, the last event of a group-by
                                   row, the first event of the call whose time
                                   change fired a timer row.  Rows are in
                                   (in_seq, processor, pending-list) order, so the
                                   outputs of key-sharded queries merge by the
                                   global sequence of in_seq. */
  const int32_t* state_idx;     /* [n_rows] state id of the pre-processor whose
                                   processing emitted the row (the completing
                                   state of a pattern / sequence match, the
                                   absent state of a timer row); 0 for
                                   single-stream (filter / window) queries   */
  /* list arena of SHD_T_OBJECT columns (multi-value selection of a count
     state without an index, `select e1.price` over `e1=S[..]<m:n>`: the
     reference's MultiValueVariableFunctionExecutor returns a java.util.List,
     C/executor/MultiValueVariableFunctionExecutor.java:64-72).  An OBJECT
     cell's payload is offset | count << 40 into these arrays
     (SHD_LIST_OFFSET / SHD_LIST_COUNT, siddhi_ir.h).                        */
  int64_t n_list;
  const uint64_t* list_values;  /* [n_list] element payloads (element type of the column) */
  const uint8_t* list_nulls;    /* [n_list] element null flags                   */
} shd_out;

typedef struct shd_counters {
  int64_t events;               /* events ingested                               */
  int64_t matches;              /* output rows produced                          */
  int64_t partials;             /* partial matches created                       */
  int64_t partial_scans;        /* (partial, event) pairs examined               */
  int64_t bytes_touched;        /* algorithmic bytes             */
  int64_t kernel_ns;            /* device time of the last push                  */
  int64_t carry;                /* open partials / window items carried          */
  int64_t group_bits;           /* pattern engine: sort bits of the last push's key
                                   grouping (hashed buckets when below the key
                                   width), 0 when not partitioned              */
  int64_t kernel_ns_total;      /* device time of every push since load / reset  */
} shd_counters;

int shd_device_count(int* n);
/* One context drives ONE device (n == 1; one host process per GPU, the
 * multi-GPU layer shards keys across processes over RCCL -- SURVEY.md §8e);
 * n > 1 returns SHD_E_ARG. */
int shd_ctx_create(const int* device_ids, int n, shd_ctx** out);
int shd_ctx_destroy(shd_ctx* ctx);

int shd_plan_load(shd_ctx* ctx, const void* ir, size_t len, shd_query** out);
int shd_plan_free(shd_query* q);
/* Engine the plan runs on: 1 = pattern forward-scan, 2 = window/aggregate,
 * 3 = filter/projection, 4 = generic per-key NFA. */
int shd_plan_engine(shd_query* q, int* engine);

int shd_set_time(shd_query* q, int64_t ts);
/* Named per-query options (SHD_E_ARG for an unknown name):
 *   "exact_aggregates" (window/aggregate engine): 1 = the bit-exact sequential
 *     per-group fold (Java's `sum += v; sum -= v` order, AttributeAggregator
 *     executors); 0 (default) = segmented scans (double-double prefix sums),
 *     double aggregates within 1e-9 relative of that fold (BASELINE.json
 *     north_star) while the operands are finite and their non-zero
 *     magnitudes span at most 2^30; the first push that brings a non-finite
 *     or wider-ranged operand switches the query to the exact fold for good
 *     (the reference's running sum keeps Inf / NaN and its rounding history).
 *     A mixed-sign window -- operands of both signs since the aggregate's last
 *     reset, which can cancel to far below its operands -- is caught by the
 *     guard's sign channel and also takes the exact fold (int operands are
 *     exempt: their sums are exact; long operands by value), so the default
 *     needs no option for it. */
int shd_set_option(shd_query* q, const char* key, int64_t value);
int shd_push(shd_query* q, const shd_batch* batch);
int shd_flush(shd_query* q);                  /* wait for queued device work      */
int shd_poll(shd_query* q, shd_out* out);      /* buffers valid until next call    */
int shd_discard_output(shd_query* q);          /* drop pending rows (benchmarks)   */
int shd_reset(shd_query* q);                   /* back to freshly-started state   */
int shd_get_counters(shd_query* q, shd_counters* c);
/* Opaque image of the query's device state (open partial matches, NFA key
 * blocks, window contents, aggregates) plus its arrival / time / chunk
 * counters.  The image is library-owned and valid until the next
 * shd_snapshot on q; pending output must have been polled.  shd_restore
 * replaces the query's state with an image taken from a query loaded with
 * the same plan IR (SHD_E_ARG otherwise). */
int shd_snapshot(shd_query* q, const void** data, size_t* len);
int shd_restore(shd_query* q, const void* data, size_t len);
/* Optional: the HIP stream (hipStream_t) a query launches on, for event timing. */
int shd_query_stream(shd_query* q, void** stream);
/* Profiling hook: per-stage device time of the last push, measured with HIP
 * events on the query's stream around each kernel stage.  Writes up to `max`
 * entries of ns[] and stage names (static strings) to names[]; *n = count. */
int shd_stage_times(shd_query* q, int64_t* ns, const char** names, int max, int* n);

/* Key-owner re-route of a micro-batch across ranks (replaces the
 * reference's in-process PartitionStreamReceiver.send fan-out to per-key state,
 * C/partition/PartitionStreamReceiver.java:262-283, when keys are sharded over
 * GPUs).  All buffers are device memory, all work is queued on `stream`
 * (hipStream_t), nothing synchronises.  Rows travel packed: the 8-byte columns,
 * then the 4-byte columns two per 8-byte word, the last 4-byte slot holding
 * seq - seq_lo; shd_route_words gives the words per row.  Scratch is
 * caller-owned (device memory): calls on different streams may overlap.
 *
 * shd_route_bucket: owner(i) = fmix32(low 32 bits of key[i]) % world; rows are
 * written to send[] grouped by owner, each group in batch order (stable), and
 * counts[o] (device int64[world]) = rows for owner o.  cols[c] holds
 * widths[c] (4 or 8) bytes per row; seq[i] - seq_lo must lie in [0, 2^32).
 * scratch: device buffer of shd_route_bucket_scratch(n, world) bytes.
 *
 * shd_route_merge: recv[] holds the rows of `world` senders, sender s's rows at
 * [seg_off[s], seg_off[s+1]) (device int64[world+1], seg_off[world] = m), each
 * in its sender's order.  The global stream's InputHandler calls are the
 * blocks of `block` sequence numbers from seq_lo (seq_lo a multiple of block
 * in the global numbering); every row must fall in one of the `nblocks`
 * blocks.  Writes the rows in increasing sequence order to out_cols (widths as
 * sent) and out_seq (int64), block_off[b] (device int64[nblocks+1]) = first
 * output row of block b (block_off[nblocks] = m), and err[0] (device int32) = 1
 * when a row is outside the blocks or a block holds more rows than sequence
 * numbers.  start: device scratch of (nblocks + 1) * world int64. */
int shd_route_words(int ncols, const int* widths, int* words);
int shd_route_bucket_scratch(int64_t n, int world, size_t* bytes);
int shd_route_bucket(shd_ctx* ctx, void* stream, int64_t n, int world, const void* key, int key_width, int ncols,
                     const void* const* cols, const int* widths, const int64_t* seq, int64_t seq_lo, uint64_t* send,
                     int64_t* counts, void* scratch);
int shd_route_merge(shd_ctx* ctx, void* stream, int world, const uint64_t* recv, const int64_t* seg_off, int64_t m,
                    int64_t seq_lo, int64_t block, int64_t nblocks, int ncols, void* const* out_cols,
                    const int* widths, int64_t* out_seq, int64_t* start, int64_t* block_off, int32_t* err);

/* Query groups: the queries a StreamJunction fans one stream out to
 * (C/stream/StreamJunction.java:146-272) that differ only in the start
 * state's filter -- `every e1=A[f1_g] -> e2=B[f2] within W` with the same f2,
 * W, streams and partitioning -- run ONE forward scan.  Each partial of such a
 * pattern meets the later events alone (ST/StreamPreStateProcessor.java:118-129,
 * 326-403), so a leader plan whose e1 filter accepts every event any member's
 * does (the host planner builds it as their disjunction) holds every member's
 * partials with the member's outcome; a member's rows are the leader's matches
 * whose e1 event passes the member's own f1, in the leader's order.
 *
 * shd_group_create: loads the leader IR on ctx and attaches 1..64 fresh member
 * queries (pattern-engine plans; SHD_E_ARG when one differs from the leader in
 * more than its e1 filter and its selector, or reads an e1 attribute the
 * leader does not carry).  While grouped, members refuse shd_push / shd_reset /
 * shd_snapshot / shd_restore / shd_plan_free; shd_poll, shd_get_counters
 * (events and matches of the member; the shared scan's counters are the
 * leader's) and shd_set_time work as usual.
 * shd_group_push: one batch into every member (as shd_push on each would).
 * When the leader has to hand over to the generic NFA engine (time going back
 * inside a key), each member takes over the leader's open partials through its
 * own NFA engine and the group runs its members one by one from then on.
 * shd_group_leader: the leader query (counters, stage times; not pushable).
 * shd_group_free: detaches and resets the members, frees the leader. */
int shd_group_create(shd_ctx* ctx, const void* leader_ir, size_t len, shd_query* const* members, int n,
                     shd_group** out);
int shd_group_push(shd_group* g, const shd_batch* batch);
int shd_group_reset(shd_group* g);
int shd_group_leader(shd_group* g, shd_query** leader);
int shd_group_free(shd_group* g);

const char* shd_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
