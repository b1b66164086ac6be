// common.h -- shared host/device infrastructure for libsiddhi_hip (gfx950).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/siddhi_hip.h"
#include "../../include/siddhi_ir.h"

namespace shd {

// ------------------------------------------------------------------ errors
struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define SHD_HIP(call)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess)                                                              \
      throw ::shd::Error(e_ == hipErrorOutOfMemory ? SHD_E_OOM : SHD_E_DEVICE,        \
                         std::string(#call) + ": " + hipGetErrorString(e_));           \
  } while (0)

// Launch check.  With SHD_SYNC_CHECK=1 in the environment every launch is
// also synchronised, so a faulting kernel is reported at its own launch site.
void check_launch(const char* file, int line);
#define SHD_CHECK_LAUNCH() ::shd::check_launch(__FILE__, __LINE__)

constexpr int kBlock = 256;
constexpr int kMaxCols = 16;      // attributes per stream handled on device
constexpr int kMaxStack = 8;      // expression stack depth (validated at plan load)
constexpr int kMaxAggs = 8;

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int grid_for(int64_t n, int per_thread = 1, int cap = 256 * 64) {
  int64_t g = ceil_div(n, (int64_t)kBlock * per_thread);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

// One thread per element, no grid-stride loop.  Kernels that stage their
// expression program in LDS use this form: their loops then never read the
// hidden launch-geometry kernel arguments (hipcc reads gridDim.x with a vector
// load from the kernarg segment when it is used below divergent staging loops,
// and vector loads from the kernarg segment fault on the MI355X pool; the ISA
// test tests/test_kernel_isa.py enforces this).  Body: `for (i = blockIdx.x *
// kBlock + threadIdx.x; i < n; i = n)` -- a loop that runs at most once, so
// `continue` keeps working.
inline unsigned grid_cover(int64_t n) {
  int64_t g = ceil_div(n, kBlock);
  return (unsigned)(g < 1 ? 1 : g);
}

// ------------------------------------------------------------------ device buffers
// Grow-only device allocation owned by an engine (allocated outside launch
// sequences so push() can be captured into a hipGraph later).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  void release() {
    // a kernel still queued on a query stream may hold the old pointer
    if (p) { (void)hipDeviceSynchronize(); (void)hipFree(p); }
    p = nullptr;
    cap = 0;
  }
  void reserve(size_t bytes) {
    if (bytes <= cap) return;
    release();
    size_t b = bytes < 256 ? 256 : bytes;
    b = (b + 255) & ~size_t(255);
    SHD_HIP(hipMalloc(&p, b));
    cap = b;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  ~PinnedBuf() { if (p) (void)hipHostFree(p); }
  void reserve(size_t bytes) {
    if (bytes <= cap) return;
    if (p) { (void)hipDeviceSynchronize(); (void)hipHostFree(p); }
    p = nullptr;
    size_t b = bytes < 256 ? 256 : bytes;
    SHD_HIP(hipHostMalloc(&p, b, hipHostMallocDefault));
    cap = b;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// ------------------------------------------------------------------ plan (host decode)
struct Instr { int32_t op, a, b, c; };

struct PNode {
  int kind = 0;
  int state_id = -1, stream = -1, absent = 0;
  int64_t waiting = -1;
  std::vector<int> filters;
  int ltype = 0;
  int min = 0, max = 0;
  std::vector<PNode> kids;
};

struct Plan {
  int kind = 0;
  std::vector<std::vector<int>> stream_types;
  std::vector<uint64_t> consts;
  std::vector<std::vector<Instr>> exprs;
  std::vector<std::pair<int, int>> part_keys;
  int state_type = 0;
  int64_t within = -1;
  int n_states = 0;
  PNode root;
  int single_stream = 0;
  struct Handler { int kind; int expr; int wkind; int64_t param, param2; };
  std::vector<Handler> handlers;
  bool current_on = true, expired_on = false;
  struct Agg { int kind, expr, type; };
  std::vector<Agg> aggs;
  std::vector<int> group_by;
  int64_t null_str_id = -1;   // dictionary id of "null" (string group keys, GroupByKeyGenerator)
  int having = -1;
  std::vector<std::pair<int, int>> outputs;  // (type, expr)
  // IR POST section (an aggregating / `having` selector of a STATE plan):
  // base outputs (type, expr) the state engine projects per match, and the
  // selector restated as a SINGLE plan over a stream of those values
  std::vector<std::pair<int, int>> post_base;
  std::shared_ptr<Plan> post;
};

Plan decode_plan(const int32_t* w, int64_t n);
int expr_result_type(const Plan& p, int expr, const std::vector<int>& agg_types);
int expr_max_depth(const Plan& p, int expr);

// Flattened device copy of all expressions of a plan.
struct DevExprTable {
  DevBuf ins;      // int4 per instruction
  DevBuf consts;   // u64
  std::vector<int> off, len;
  int nins = 0, nconsts = 0;
  void upload(const Plan& p);
};

// ------------------------------------------------------------------ columns
// A set of typed device columns (one stream's batch, or a carry table).
// Load element i of a device array through a global-address-space pointer.
// Column pointers read from argument structs are generic to the compiler and
// would become flat loads, which also count against lgkmcnt: every scalar
// load of the next column pointer then waits for all vector loads in flight.
template <class T>
__device__ __forceinline__ T gld(const T* p, int64_t i) {
  typedef __attribute__((address_space(1))) const T* GP;
  return ((GP)p)[i];
}

struct ColSet {
  const void* col[kMaxCols];
  const uint8_t* nul[kMaxCols];
  int32_t type[kMaxCols];   // 32-bit: uniform fields load through the scalar cache (gfx9 has no s_load_byte)
  int32_t ncols;
  const int64_t* ts;
  int64_t n;        // rows (bounds checks in SHD_DEBUG builds)
};

inline int type_size(int t) {
  switch (t) {
    case SHD_T_STRING: case SHD_T_INT: case SHD_T_FLOAT: return 4;
    case SHD_T_LONG: case SHD_T_DOUBLE: return 8;
    case SHD_T_BOOL: return 1;
  }
  return 8;
}

// Bijective 32-bit mix (odd multiply, then xor-shift by half the width):
// equal keys map to equal values, and the low bits depend on every key bit,
// so its low bits make well-spread buckets for any key distribution.
__host__ __device__ __forceinline__ uint32_t key_bucket_mix(uint32_t k) {
  const uint32_t h = k * 0x9E3779B1u;
  return h ^ (h >> 16);
}

// ------------------------------------------------------------------ primitives (primitives.hip)
// Exclusive scan of u32 counts -> u32 offsets; returns nothing (total read from out[n-1]+in[n-1]).
void scan_exclusive_u32(const uint32_t* in, uint32_t* out, int64_t n, uint32_t* total_dev,
                        DevBuf& scratch, hipStream_t s);
// Stable LSD radix sort of (key, value) pairs over key bits [0, bits).
void radix_sort_pairs_u32(uint32_t* keys, uint32_t* vals, uint32_t* keys_alt, uint32_t* vals_alt,
                          int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& result_in_alt);
void radix_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt,
                          int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& result_in_alt);
// Device-wide max of u64 keys (result to dev ptr).
// Same, carrying a second 32-bit payload word per key.
// kbase: digits of (key - kbase) (keys of the sort span [kbase, kbase + 2^bits)).
// hashed: digits are taken from key_bucket_mix(key) instead of the key, so
// bits < 32 groups equal keys into 2^bits buckets (stable: input order inside
// a bucket) while the array still carries the raw keys.
// shift0: the passes start at digit bit shift0 (the lower digits were sorted
// already, e.g. by a fused prepare + first pass).
void radix_sort_triples_u32(uint32_t* keys, uint32_t* vals, uint32_t* w, uint32_t* keys_alt, uint32_t* vals_alt,
                            uint32_t* w_alt, int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& in_alt,
                            bool hashed = false, uint32_t kbase = 0, int shift0 = 0);
void radix_sort_triples_u64(uint64_t* keys, uint32_t* vals, uint32_t* w, uint64_t* keys_alt, uint32_t* vals_alt,
                            uint32_t* w_alt, int64_t n, int bits, DevBuf& scratch, hipStream_t s, bool& in_alt);
// Digit totals (256 per pass, u32) of the last radix pass run with `scratch`
// over n keys (radix_sort_triples_u32 / _pairs_u32): the bucket sizes of a
// one-pass hashed bucket sort.
const uint32_t* radix_digit_totals(const DevBuf& scratch, int64_t n);
// Row scans of a [256][nb] per-tile digit histogram: offs[d*nb + t] = digit
// d's count in tiles before t, dtot[d] = digit d's total (one pass's offsets).
void radix_digit_scan(const uint32_t* hist, int nb, uint32_t* offs, uint32_t* dtot, hipStream_t s);
void reduce_max_u64(const uint64_t* in, int64_t n, uint64_t* out_dev, hipStream_t s);
void fill_iota_u32(uint32_t* out, int64_t n, uint32_t base, hipStream_t s);

}  // namespace shd
