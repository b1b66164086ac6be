// pattern_walk.h -- the per-partial walk of the pattern engine (the
// StreamPreStateProcessor step for `every e1=A[f1] -> e2=B[f2] within W`),
// used by the sort-path kernels of engine_pattern.hip.  Included inside
// namespace shd::(anonymous) with shd::pat in scope.
#pragma once

// Walk of one candidate partial P (row r, key k, timestamp tsi) over the
// later events of its key, starting at position q whose pv / ts / key are
// already loaded (pq, tq, kq).  StreamPreStateProcessor.processAndReturn for
// this plan shape: expire when ts - tsi > within, complete at the first
// B event with f2(P, event).
//   DEFER: f2 is not evaluated here; the walk stops at the first B event
//          inside `within` and returns ST_DEFER with q at that event (the
//          step is already counted).  Keeps the hot kernel free of the f2
//          code (its registers and instruction footprint).
//   f2_first: resume at a deferred event: evaluate f2 at q first.
// Position loads (flags/row, timestamp, key at sorted position q) from global memory.
template <bool K64, bool TS64>
struct GlobalPos {
  const uint32_t* __restrict__ skey32;
  const uint64_t* __restrict__ skey64;
  const uint32_t* __restrict__ spv;
  const int32_t* __restrict__ sts32;
  const int64_t* __restrict__ sts64;
  int64_t tbase;
  int partitioned;
  __device__ __forceinline__ void operator()(int64_t q, uint32_t& pq, int64_t& tq, uint64_t& kq) const {
    pq = spv[q];
    tq = TS64 ? sts64[q] : tbase + (int64_t)sts32[q];
    if (partitioned) kq = K64 ? skey64[q] : skey32[q];
  }
};

// Split f2 (F2Split): the per-partial side of every comparison, and the
// step's evaluation against an e2 event (batch row r2b = ext row - C, sorted
// position q2).  Same result as eval_fpred(a.f2.fp, PairCtx{r, r2}).
struct SplitThr {
  Val t[kSplitMax];
  bool never;   // a comparison free of e2 fails: f2 never passes for this partial
};
__device__ __forceinline__ SplitThr split_prep(const ScanArgs& a, int64_t r, int64_t q1) {
  SplitThr th;
  th.never = false;
  PairCtx cx{&a.x, r, -1, a.s_first};
  cx.q1 = q1;
#pragma unroll
  for (int i = 0; i < kSplitMax; i++) {
    th.t[i].b = 0;
    th.t[i].null = 1;
    if (i >= a.sp.n) continue;
    const FCmp& c = a.f2.fp.c[i];
    if (a.sp.c[i].konst) {
      const Val l = fp_term(c.l, cx), rr = fp_term(c.r, cx);
      if (l.null || rr.null || !d_compare(c.op, c.type, l.b, rr.b)) th.never = true;
    } else {
      th.t[i] = fp_term(a.sp.c[i].swap ? c.l : c.r, cx);
      if (th.t[i].null) th.never = true;   // a null operand fails the comparison at every step
    }
  }
  return th;
}
// The step in two halves, so a walk can issue the next event's operand
// loads before it tests the current one: split_fetch loads the e2 operands
// (one typed load per comparison, null bits), split_test compares them.
struct SplitRaw {
  uint64_t v[kSplitMax];
  uint32_t nul;   // bit i: comparison i's e2 operand is null
};
__device__ __forceinline__ SplitRaw split_fetch(const F2Split& sp, int64_t r2b, int64_t q2) {
  SplitRaw w;
  w.nul = 0;
#pragma unroll
  for (int i = 0; i < kSplitMax; i++) {
    w.v[i] = 0;
    if (i >= sp.n) break;
    const SplitCmp& c = sp.c[i];
    if (c.konst) continue;
    const int64_t row = c.pos ? q2 : r2b;
    switch (c.kind) {
      case SK_F32_F64: case SK_STR_EQ: case SK_I32: w.v[i] = gld((const uint32_t*)c.col, row); break;
      case SK_F64: w.v[i] = gld((const uint64_t*)c.col, row); break;
      default: {
        const Val v = col_load_raw(c.col, c.nul, c.ctype, row);
        w.v[i] = v.b;
        if (v.null) w.nul |= 1u << i;
        continue;
      }
    }
    if (c.nul && gld(c.nul, row)) w.nul |= 1u << i;
  }
  return w;
}
__device__ __forceinline__ bool split_test(const F2Split& sp, const SplitThr& th, const SplitRaw& w) {
  if (th.never) return false;
#pragma unroll
  for (int i = 0; i < kSplitMax; i++) {
    if (i >= sp.n) break;
    const SplitCmp& c = sp.c[i];
    if (c.konst) continue;
    if ((w.nul >> i) & 1u) return false;
    const uint64_t t = th.t[i].b;
    // the common kinds: the comparison with e2 on the left (the host flipped
    // the operator of a swapped comparison)
    int cc;
    switch (c.kind) {
      case SK_F32_F64: {
        const double x = (double)__uint_as_float((uint32_t)w.v[i]), y = v_f64(t);
        cc = (x < y) ? -1 : (x > y) ? 1 : (x == y) ? 0 : 2;
        break;
      }
      case SK_F64: {
        const double x = v_f64(w.v[i]), y = v_f64(t);
        cc = (x < y) ? -1 : (x > y) ? 1 : (x == y) ? 0 : 2;
        break;
      }
      case SK_STR_EQ:
        cc = (w.v[i] == t) ? 0 : 2;
        break;
      case SK_I32: {
        const int32_t x = v_i32(w.v[i]), y = v_i32(t);
        cc = x < y ? -1 : (x > y ? 1 : 0);
        break;
      }
      default: {
        uint64_t b = w.v[i];
        if (c.cvt_to >= 0) b = d_cvt(b, c.cvt_from, c.cvt_to);
        if (!d_compare(c.op, c.type, c.swap ? t : b, c.swap ? b : t)) return false;
        continue;
      }
    }
    bool ok;
    switch (c.op) {
      case SHD_OP_EQ: ok = cc == 0; break;
      case SHD_OP_NE: ok = cc != 0; break;
      case SHD_OP_GT: ok = cc == 1; break;
      case SHD_OP_GE: ok = cc == 1 || cc == 0; break;
      case SHD_OP_LT: ok = cc == -1; break;
      case SHD_OP_LE: ok = cc == -1 || cc == 0; break;
      default: ok = false;
    }
    if (!ok) return false;
  }
  return true;
}
__device__ __forceinline__ bool split_eval(const F2Split& sp, const SplitThr& th, int64_t r2b, int64_t q2) {
  if (th.never) return false;
  return split_test(sp, th, split_fetch(sp, r2b, q2));
}

// Block skip: f2's threshold for partial (row r, sorted position q1) -- the
// e1 side of comparison bs_ci (null: f2 can never pass).
__device__ __forceinline__ Val skip_threshold(const ScanArgs& a, int64_t r, int64_t q1) {
  const FCmp& c = a.f2.fp.c[a.bs_ci];
  PairCtx cx{&a.x, r, -1, a.s_first};
  cx.q1 = q1;
  return fp_term(a.bs_side == 0 ? c.r : c.l, cx);
}

// True when a walk of key k (created at tsi, last step at prev) passes the
// whole block without an outcome: every non-skip position is of key k, no
// F_NEW event expires it or goes back in time, and no B event can pass f2.
__device__ __forceinline__ bool block_skippable(const ScanArgs& a, const BlockSum& b, uint64_t k, int64_t tsi,
                                                int64_t prev, Val thr) {
  if (a.partitioned && !(b.flags & 4u) && (!(b.flags & 1u) || b.key != (uint32_t)k)) return false;
  if (b.cnt && a.within != INT64_MAX) {
    if (!(b.flags & 2u) || b.tfirst < prev || b.tlast - tsi > a.within) return false;
  }
  if (thr.null) return true;
  const double t = v_f64(thr.b), v = b.v;
  switch (a.bs_op) {
    case SHD_OP_GT: return v <= t;
    case SHD_OP_GE: return v < t;
    case SHD_OP_LT: return v >= t;
    case SHD_OP_LE: return v > t;
  }
  return false;
}

// WIN: positions are loaded WIN at a time (one round trip for WIN steps);
// walks over hashed buckets step over a few other keys, and a wave waits for
// its longest walk, so they fetch ahead.
template <bool DEFER, bool FAST, int WIN, class Ld, int CAP = 0, bool SKIP = false>
__device__ __forceinline__ uint8_t walk_partial(const ScanArgs& a, const DExprSet& es, int64_t n_ext, const Ld& ld,
                                                int64_t r, uint64_t k, int64_t tsi, int64_t& q, uint32_t pq,
                                                int64_t tq, uint64_t kq, int64_t prev, bool f2_now, int32_t& j,
                                                uint64_t& steps, uint32_t& viol, uint32_t& fm, int64_t& ra,
                                                int64_t& rb, int64_t q1 = -1) {
  uint8_t st = ST_OPEN;
  bool stop = false, first = true;
  int it = 0;
  bool thr_ok = false;
  Val thr;
  thr.b = 0;
  thr.null = 1;
  SplitThr sth;            // split f2: the partial's side, prepared at its first B event
  bool th_ok = false;
  int64_t tried = -1;      // block whose skip was last tried
  int64_t last_new = q;    // position of the walk's last F_NEW step (the resume point's time is prev)
  while (!stop && q < n_ext) {
    if constexpr (CAP > 0) {
      // CAP positions walked: yield before position q (nothing of it processed)
      if (!f2_now && it >= CAP) {
        st = ST_YIELD;
        break;
      }
      it += WIN;
    }
    if constexpr (!DEFER && SKIP) {
      // long walks skip the rest of a 64-position block when none of it can
      // end them: from a block boundary (block_skippable), or from inside the
      // block once per block -- then the whole block's summary must allow it
      // and, for the times, the walk's last step lies in this block (the
      // block's times are nondecreasing, so the rest is no earlier than it)
      const int64_t blk = q >> 6;
      if (!first && !f2_now && blk != tried && (blk << 6) + 64 <= n_ext) {
        tried = blk;
        if (!thr_ok) {
          thr = skip_threshold(a, r, q1);
          thr_ok = true;
        }
        const BlockSum bs = a.bsum[blk];
        const int off = (int)(q & 63);
        // the last step inside this block: the block's nondecreasing times
        // after it are >= prev (block_skippable then only checks monotonicity)
        const int64_t after = (off != 0 && last_new >= (blk << 6)) ? INT64_MIN : prev;
        if (block_skippable(a, bs, k, tsi, after, thr)) {
          const uint32_t c = (uint32_t)__popcll(bs.newmask >> off);
          steps += c;
          if (c) {
            prev = bs.tlast;
            last_new = (blk << 6) + 63;
          }
          q = (blk << 6) + 64;
          continue;
        }
      }
    }
    uint32_t wp[WIN];
    int64_t wt[WIN];
    uint64_t wk[WIN];
#pragma unroll
    for (int i = 0; i < WIN; i++) {
      wk[i] = 0;
      if (i == 0 && first) {
        wp[0] = pq;
        wt[0] = tq;
        wk[0] = kq;
      } else {
        const int64_t qi = q + i < n_ext ? q + i : n_ext - 1;
        ld(qi, wp[i], wt[i], wk[i]);
      }
    }
    first = false;
#pragma unroll
    for (int i = 0; i < WIN; i++) {
      if (q >= n_ext) {
        stop = true;
        break;
      }
      pq = wp[i];
      tq = wt[i];
      kq = wk[i];
      // rows of dropped (null-key) events carry no usable key: passed over
    if (!f2_now && a.partitioned && kq != k && !(pv_flags(pq) & F_SKIP)) {
        stop = true;
        if (!a.hash_mask) break;   // end of the key's run
        if ((key_bucket_mix((uint32_t)kq) ^ key_bucket_mix((uint32_t)k)) & a.hash_mask) break;   // end of the bucket
        // another key of the bucket: pushed rows are time-ordered, so once one is
        // beyond `within` every later event of this key is too -- the partial
        // can no longer match (OPEN here; the horizon rule below retires it,
        // t_end >= tq > tsi + within)
        if (pv_row(pq) >= (uint32_t)a.x.C && tq - tsi > a.within) break;
        stop = false;
      } else if (!f2_now) {
        const uint32_t fq = pv_flags(pq);
        if ((fq & F_NEW) && !(fq & F_SKIP)) {
          // a per-key time regression only matters under `within` (expiry);
          // without it the outcome of every partial is time-independent
          if (a.within != INT64_MAX && tq < prev) {
            viol = 1;
            stop = true;
            break;
          }
          prev = tq;
          last_new = q;
          steps++;
          // stabilizeStates -> expireEvents: |ts_i - t| > within
          if (tq - tsi > a.within) {
            st = ST_DEAD;
            stop = true;
            break;
          }
          if (fq & F_B) {
            if (DEFER) {
              st = ST_DEFER;
              stop = true;
              break;
            }
            f2_now = true;
          }
        }
      }
      if constexpr (!DEFER) {
        if (f2_now) {
          f2_now = false;
          const int64_t r2 = pv_row(pq);
          if (a.logical == 2) {
            // LogicalPre/PostStateProcessor (AND): an operand that passes fills
            // its slot and leaves its processor's pending list; the partial
            // completes when the partner slot is filled too -- possibly by the
            // partner processor on this same event (LogicalPostStateProcessor.java:59-86)
            int32_t br = -1;
            if (!(fm & 1u)) {
              PairCtx cx{&a.x, r, r2, a.s_first, false, (fm & 2u) ? rb : -1, a.s_second, q, q1};
              if (FAST ? eval_fpred(a.f2.fp, cx) : eval_filters(es, a.f2, cx)) {
                fm |= 1u;
                ra = r2;
                if (fm == 3u) br = 0;
              }
            }
            if (br < 0 && !(fm & 2u)) {
              PairCtx cx{&a.x, r, r2, a.s_second, false, (fm & 1u) ? ra : -1, a.s_first, q, q1};
              if (FAST ? eval_fpred(a.f3.fp, cx) : eval_filters(es, a.f3, cx)) {
                fm |= 2u;
                rb = r2;
                if (fm == 3u) br = 1;
              }
            }
            if (br >= 0) {
              st = ST_MATCH;
              j = (int32_t)r2 | (br << kRowBits);
              stop = true;
              break;
            }
            q++;
            continue;
          }
          PairCtx cx{&a.x, r, r2, a.s_first};
          cx.q2 = q;
          cx.q1 = q1;
          bool hit;
          if (FAST && a.sp.ok && !a.logical) {
            if (!th_ok) {
              sth = split_prep(a, r, q1);
              th_ok = true;
            }
            hit = split_eval(a.sp, sth, r2 - a.x.C, q);
          } else {
            hit = FAST ? eval_fpred(a.f2.fp, cx) : eval_filters(es, a.f2, cx);
          }
          int32_t br = 0;
          if (!hit && a.logical) {
            // LogicalPreStateProcessor (OR): the partner processor sees the
            // same event next (LogicalPreStateProcessor.java:113-154)
            cx.s2 = a.s_second;
            hit = FAST ? eval_fpred(a.f3.fp, cx) : eval_filters(es, a.f3, cx);
            br = 1;
          }
          if (hit) {
            st = ST_MATCH;
            j = (int32_t)r2 | (br << kRowBits);   // matched branch above the row bits
            stop = true;
            break;
          }
        }
      }
      q++;
    }
  }
  if (st == ST_OPEN && a.prune && a.t_end - tsi > a.within) st = ST_PRUNED;
  return st;
}

