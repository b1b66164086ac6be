// gdict.h -- device group dictionary: dense ids for multi-word keys.
//
// The reference keys per-group state by the text of the key values
// (GroupByKeyGenerator.constructEventKey, C/query/selector/GroupByKeyGenerator.java:63-73)
// and per-partition state by the partition key (PartitionStateHolder.getState,
// C/util/snapshot/state/PartitionStateHolder.java:43-48).  On the device a key
// is `nk` canonical 64-bit words plus a null mask; this open-addressing table
// maps it to a dense u32 id (ids 0, 1, 2, ... in first-insert order), so state
// tables are plain arrays indexed by id.
//
// Entry: tag (64-bit hash with bit 63 set, 0 = empty; its low bits are the home
// slot), id, the key words [nk][cap] and null mask.  Look-ups are read-only; a
// batch with unseen keys inserts them in a second phase (misses compacted,
// sorted by hash, one leader per distinct key, CAS insertion of distinct keys:
// no thread ever waits on another), then looks the misses up again.
//
// Included by the engines that need it; the kernels live in an anonymous
// namespace (one copy per translation unit).
#pragma once
#include <algorithm>

#include "engine.h"

namespace shd {
namespace {

constexpr uint64_t kTagBit = 1ull << 63;
constexpr int kMaxGroupAttrs = 4;   // group-by attributes of one query on the device

__host__ __device__ __forceinline__ uint64_t gdict_mix(uint64_t z) {   // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Hash of key words (word g folded with its position) and the null mask.
__device__ __forceinline__ uint64_t gdict_hash_step(uint64_t h, uint64_t w, int g) {
  return gdict_mix(h ^ gdict_mix(w + 0x632BE59BD9B4E019ull * (uint64_t)(g + 1)));
}
__device__ __forceinline__ uint64_t gdict_hash_final(uint64_t h, uint8_t nulls) {
  return gdict_mix(h ^ ((uint64_t)nulls << 56));
}
constexpr uint64_t kGdictSeed = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t canon_key(Val v, int type) {
  if (type == SHD_T_FLOAT) return p_f64((double)v_f32(v.b));
  return v.b;
}

// One group-by value as a canonical word: two values share a word exactly
// when String.valueOf prints them alike (the reference's group key is that
// text, C/query/selector/GroupByKeyGenerator.java:63-73): a null string is the
// string "null" (its dictionary id), every NaN is one NaN, 0.0 and -0.0 stay
// apart; other nulls set isnull (word 0).
__device__ __forceinline__ uint64_t group_word(Val v, int type, int64_t null_str_id, bool& isnull) {
  isnull = false;
  if (v.null) {
    if (type == SHD_T_STRING && null_str_id >= 0) return (uint64_t)null_str_id;
    isnull = true;
    return 0;
  }
  switch (type) {
    case SHD_T_FLOAT: {
      const float f = v_f32(v.b);
      return f != f ? 0x7fc00000ull : (uint64_t)(uint32_t)v.b;
    }
    case SHD_T_DOUBLE: {
      const double d = __longlong_as_double((long long)v.b);
      return d != d ? 0x7ff8000000000000ull : v.b;
    }
    case SHD_T_INT:
    case SHD_T_BOOL:
    case SHD_T_STRING: return (uint64_t)(uint32_t)v.b;
    default: return v.b;
  }
}


struct GDict {
  unsigned long long* tag;
  uint32_t* id;
  uint64_t* kw;     // [nk][cap]
  uint8_t* kn;
  uint64_t cap;     // power of two
  int nk;
};

__device__ __forceinline__ bool gdict_find(const GDict& d, uint64_t h, const uint64_t* key, int64_t kstride,
                                           int64_t ki, uint8_t nul, uint32_t& id) {
  const unsigned long long tg = (unsigned long long)(h | kTagBit);
  uint64_t slot = h & (d.cap - 1);
  for (uint64_t probe = 0; probe < d.cap; probe++) {
    const unsigned long long t = d.tag[slot];
    if (t == 0ull) return false;
    if (t == tg && d.kn[slot] == nul) {
      bool eq = true;
      for (int g = 0; g < d.nk; g++) eq = eq && d.kw[(uint64_t)g * d.cap + slot] == key[(int64_t)g * kstride + ki];
      if (eq) {
        id = d.id[slot];
        return true;
      }
    }
    slot = (slot + 1) & (d.cap - 1);
  }
  return false;
}

// Id of key i (or a miss flag): out[off + i].
__global__ __launch_bounds__(kBlock) void k_gdict_lookup(GDict d, int64_t n, const uint64_t* gh, const uint64_t* gkw,
                                                         const uint8_t* gkn, int64_t gstride, int64_t off,
                                                         uint64_t* out, uint32_t* miss) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    uint32_t id;
    const bool hit = gdict_find(d, gh[i], gkw, gstride, i, gkn[i], id);
    if (hit) out[off + i] = id;
    miss[i] = hit ? 0u : 1u;
  }
}

// Second look-up over the compacted misses (all present after the insert).
__global__ __launch_bounds__(kBlock) void k_gdict_relookup(GDict d, int64_t nm, const uint32_t* midx, const uint64_t* gh,
                                                           const uint64_t* gkw, const uint8_t* gkn, int64_t gstride,
                                                           int64_t off, uint64_t* out) {
  for (int64_t j = (int64_t)blockIdx.x * kBlock + threadIdx.x; j < nm; j = nm) {
    const int64_t i = midx[j];
    uint32_t id = 0xFFFFFFFFu;
    gdict_find(d, gh[i], gkw, gstride, i, gkn[i], id);
    out[off + i] = id;
  }
}

__global__ __launch_bounds__(kBlock) void k_gdict_compact(const uint32_t* miss, const uint32_t* moff, int64_t n,
                                                          const uint64_t* gh, uint32_t* midx, uint64_t* mh) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i = n) {
    if (!miss[i]) continue;
    midx[moff[i]] = (uint32_t)i;
    mh[moff[i]] = gh[i];
  }
}

// Leaders among the hash-sorted misses: the first of each distinct key (an
// equal-hash run is searched back for an equal key; such runs hold one key
// unless 64-bit hashes collide).
__global__ __launch_bounds__(kBlock) void k_gdict_leaders(int64_t nm, const uint64_t* sh, const uint32_t* sidx,
                                                          const uint64_t* gkw, const uint8_t* gkn, int64_t gstride,
                                                          int nk, uint32_t* lead) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < nm; p = nm) {
    const int64_t i = sidx[p];
    bool leader = true;
    for (int64_t q = p - 1; q >= 0 && sh[q] == sh[p]; q--) {
      const int64_t j = sidx[q];
      bool eq = gkn[j] == gkn[i];
      for (int g = 0; g < nk && eq; g++) eq = gkw[(int64_t)g * gstride + j] == gkw[(int64_t)g * gstride + i];
      if (eq) {
        leader = false;
        break;
      }
    }
    lead[p] = leader ? 1u : 0u;
  }
}

// CAS insertion of distinct keys (the leaders): ids base + leader rank.
__global__ __launch_bounds__(kBlock) void k_gdict_insert(GDict d, int64_t nm, const uint64_t* sh, const uint32_t* sidx,
                                                         const uint32_t* lead, const uint32_t* lrank,
                                                         const uint64_t* gkw, const uint8_t* gkn, int64_t gstride,
                                                         uint32_t base) {
  for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < nm; p = nm) {
    if (!lead[p]) continue;
    const int64_t i = sidx[p];
    const uint64_t h = sh[p];
    const unsigned long long tg = (unsigned long long)(h | kTagBit);
    uint64_t slot = h & (d.cap - 1);
    while (atomicCAS(&d.tag[slot], 0ull, tg) != 0ull) slot = (slot + 1) & (d.cap - 1);
    d.id[slot] = base + lrank[p];
    d.kn[slot] = gkn[i];
    for (int g = 0; g < d.nk; g++) d.kw[(uint64_t)g * d.cap + slot] = gkw[(int64_t)g * gstride + i];
  }
}

// Table growth: re-insert every entry of `o` into the empty table `d`.
__global__ __launch_bounds__(kBlock) void k_gdict_rehash(GDict o, GDict d) {
  for (uint64_t s = (uint64_t)blockIdx.x * kBlock + threadIdx.x; s < o.cap; s = o.cap) {
    const unsigned long long tg = o.tag[s];
    if (tg == 0ull) continue;
    uint64_t slot = (uint64_t)tg & (d.cap - 1);
    while (atomicCAS(&d.tag[slot], 0ull, tg) != 0ull) slot = (slot + 1) & (d.cap - 1);
    d.id[slot] = o.id[s];
    d.kn[slot] = o.kn[s];
    for (int g = 0; g < d.nk; g++) d.kw[(uint64_t)g * d.cap + slot] = o.kw[(uint64_t)g * o.cap + s];
  }
}

// Host side of one dictionary (owned by an engine, used on its stream).
struct GroupDict {
  int nk = 1;                 // key words per entry (>= 1)
  DevBuf tag, id, kw, kn;
  uint64_t cap = 0;
  int64_t count = 0;          // ids handed out so far
  DevBuf miss, moff, midx, mh, midx_alt, mh_alt, lead, lrank, ctr, scan, sort;
  PinnedBuf hctr;

  GDict view() const {
    return GDict{tag.as<unsigned long long>(), id.as<uint32_t>(), kw.as<uint64_t>(), kn.as<uint8_t>(), cap, nk};
  }

  void reset(hipStream_t s) {
    count = 0;
    if (cap) SHD_HIP(hipMemsetAsync(tag.p, 0, cap * 8, s));
  }

  // Table with room for `need` entries at load <= 1/2 (rehash on growth).
  void reserve(int64_t need, hipStream_t s) {
    uint64_t c = cap ? cap : 1024;
    while ((int64_t)(c / 2) < need) c *= 2;
    if (c == cap) return;
    DevBuf t, i, k, n;
    t.reserve(c * 8);
    i.reserve(c * 4);
    k.reserve((size_t)nk * c * 8);
    n.reserve(c);
    SHD_HIP(hipMemsetAsync(t.p, 0, c * 8, s));
    GDict nd{t.as<unsigned long long>(), i.as<uint32_t>(), k.as<uint64_t>(), n.as<uint8_t>(), c, nk};
    if (cap && count) {
      hipLaunchKernelGGL(k_gdict_rehash, dim3(grid_cover((int64_t)cap)), dim3(kBlock), 0, s, view(), nd);
      SHD_CHECK_LAUNCH();
    }
    SHD_HIP(hipStreamSynchronize(s));
    std::swap(tag.p, t.p); std::swap(tag.cap, t.cap);
    std::swap(id.p, i.p); std::swap(id.cap, i.cap);
    std::swap(kw.p, k.p); std::swap(kw.cap, k.cap);
    std::swap(kn.p, n.p); std::swap(kn.cap, n.cap);
    cap = c;
  }

  // Dense ids of m keys (words gkw[nk][gstride], null masks gkn, hashes gh):
  // out[off + i] = id of key i; keys never seen before get new ids.
  void assign(int64_t m, const uint64_t* gh, const uint64_t* gkw, const uint8_t* gkn, int64_t gstride, uint64_t* out,
              int64_t off, hipStream_t s) {
    if (m <= 0) return;
    reserve(1, s);
    miss.reserve(m * 4);
    moff.reserve(m * 4);
    ctr.reserve(64);
    hctr.reserve(64);
    hipLaunchKernelGGL(k_gdict_lookup, dim3(grid_cover(m)), dim3(kBlock), 0, s, view(), m, gh, gkw, gkn, gstride, off,
                       out, miss.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    scan_exclusive_u32(miss.as<uint32_t>(), moff.as<uint32_t>(), m, ctr.as<uint32_t>(), scan, s);
    SHD_HIP(hipMemcpyAsync(hctr.p, ctr.p, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t nm = hctr.as<uint32_t>()[0];
    if (nm == 0) return;
    midx.reserve(nm * 4);
    mh.reserve(nm * 8);
    midx_alt.reserve(nm * 4);
    mh_alt.reserve(nm * 8);
    hipLaunchKernelGGL(k_gdict_compact, dim3(grid_cover(m)), dim3(kBlock), 0, s, (const uint32_t*)miss.as<uint32_t>(),
                       (const uint32_t*)moff.as<uint32_t>(), m, gh, midx.as<uint32_t>(), mh.as<uint64_t>());
    SHD_CHECK_LAUNCH();
    bool in_alt = false;
    radix_sort_pairs_u64(mh.as<uint64_t>(), midx.as<uint32_t>(), mh_alt.as<uint64_t>(), midx_alt.as<uint32_t>(), nm, 64,
                         sort, s, in_alt);
    const uint64_t* sh = in_alt ? mh_alt.as<uint64_t>() : mh.as<uint64_t>();
    const uint32_t* sidx = in_alt ? midx_alt.as<uint32_t>() : midx.as<uint32_t>();
    lead.reserve(nm * 4);
    lrank.reserve(nm * 4);
    hipLaunchKernelGGL(k_gdict_leaders, dim3(grid_cover(nm)), dim3(kBlock), 0, s, nm, sh, sidx, gkw, gkn, gstride, nk,
                       lead.as<uint32_t>());
    SHD_CHECK_LAUNCH();
    scan_exclusive_u32(lead.as<uint32_t>(), lrank.as<uint32_t>(), nm, ctr.as<uint32_t>() + 1, scan, s);
    SHD_HIP(hipMemcpyAsync(hctr.as<uint32_t>() + 1, ctr.as<uint32_t>() + 1, 4, hipMemcpyDeviceToHost, s));
    SHD_HIP(hipStreamSynchronize(s));
    const int64_t nu = hctr.as<uint32_t>()[1];
    if (count + nu >= (int64_t)0xFFFFFFF0ll) throw Error(SHD_E_CAPACITY, "more than 2^32 distinct keys");
    reserve(count + nu, s);
    hipLaunchKernelGGL(k_gdict_insert, dim3(grid_cover(nm)), dim3(kBlock), 0, s, view(), nm, sh, sidx,
                       (const uint32_t*)lead.as<uint32_t>(), (const uint32_t*)lrank.as<uint32_t>(), gkw, gkn, gstride,
                       (uint32_t)count);
    SHD_CHECK_LAUNCH();
    hipLaunchKernelGGL(k_gdict_relookup, dim3(grid_cover(nm)), dim3(kBlock), 0, s, view(), nm, sidx, gh, gkw, gkn,
                       gstride, off, out);
    SHD_CHECK_LAUNCH();
    count += nu;
  }

  void save(SnapW& w) const {
    w.put<uint64_t>(cap);
    w.put<int64_t>(count);
    if (cap) {
      w.dev(tag.p, cap * 8);
      w.dev(id.p, cap * 4);
      w.dev(kw.p, (size_t)nk * cap * 8);
      w.dev(kn.p, cap);
    }
  }
  void load(SnapR& r, hipStream_t s) {
    const uint64_t dcap = r.get<uint64_t>();
    const int64_t dcount = r.get<int64_t>();
    if (dcap & (dcap - 1)) throw Error(SHD_E_ARG, "snapshot of a different plan");
    reset(s);
    if (dcap) {
      tag.reserve(dcap * 8);
      id.reserve(dcap * 4);
      kw.reserve((size_t)nk * dcap * 8);
      kn.reserve(dcap);
      r.dev_into(tag.p, dcap * 8);
      r.dev_into(id.p, dcap * 4);
      r.dev_into(kw.p, (size_t)nk * dcap * 8);
      r.dev_into(kn.p, dcap);
      cap = dcap;
      count = dcount;
    }
  }
};

}  // namespace
}  // namespace shd
