"""Benchmark: partitioned 2-state pattern (config P3) on MI355X via libsiddhi_hip.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config P3|P3-dense|P1|W2-length|W2-time]

Workload (BASELINE.json configs[2]): P1's query
`every e1=StockStream[price>70] -> e2=StockStream[symbol==e1.symbol and
price>e1.price*1.05] within 1 sec` inside `partition with (symbol of StockStream)`,
synthetic seeded StockStream, 100M events per GPU over 10M keys per GPU,
delta = 0.01 ms, InputHandler calls of 1024 events.

One step = one pass of the hot path over the whole 100M-event stream from a
freshly started query state, pushed as micro-batches (state carried between
them); inputs are resident in HBM before the timed region.  Multi-GPU: one
process per GPU, keys hash-sharded (each rank owns a disjoint 10M-key slice
with its own 100M events: weak scaling, no data-path collective).  `value` =
events of all ranks / max-over-ranks time.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: 8 TB/s HBM3E peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="P3")
    ap.add_argument("--events", type=int, default=0, help="override events per GPU")
    ap.add_argument("--keys", type=int, default=0, help="override keys per GPU")
    ap.add_argument("--batch", type=int, default=50_000_000, help="micro-batch size (events)")
    ap.add_argument("--no-share", action="store_true", help="M5: every query scans alone (no shd_group)")
    ap.add_argument("--m5-direct", action="store_true",
                    help="M5 parity: every query against its own oracle run over the prefix (no leader lemma)")
    ap.add_argument("--cpu-sample", type=int, default=-1, help="oracle sample size for cpu_baseline (0=skip)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads of the per-key parallel CPU baseline (partitioned configs; 0=skip)")
    ap.add_argument("--key-base", type=int, default=-1,
                    help="first key id of this rank's slice (default rank * keys; diagnostics)")
    ap.add_argument("--sweep-batches", default="", help="comma list of micro-batch sizes to time first (stderr lines)")
    ap.add_argument("--e2e", action="store_true",
                    help="end-to-end line instead: host columns -> SiddhiManager -> InputHandler.send_batch -> "
                         "QueryCallback (SURVEY.md section 8d, reported separately from the engine number)")
    ap.add_argument("--e2e-batch", type=int, default=5_000_000, help="events per send_batch call (--e2e)")
    ap.add_argument("--input", default="auto", choices=["auto", "prepartitioned", "roundrobin", "slices"],
                    help="roundrobin: every rank holds a round-robin share of the global stream and events are "
                         "re-routed to their key's owner with one RCCL all-to-all per micro-batch; slices "
                         "(window configs): rank r holds slice r of one global stream and primes its query "
                         "with the previous slice's tail (one RCCL send/recv per step); prepartitioned: "
                         "independent per-rank streams, no data-path collective (default at N=1)")
    return ap.parse_args()


def gen_device_columns(torch, n, keys, delta, seed_offset, key_base, dev, start=0):
    """Events [start, start + n) of the seeded StockStream, resident in HBM."""
    from siddhi_amd import workloads as wl
    sym = torch.empty(n, dtype=torch.int32, device=dev)
    price = torch.empty(n, dtype=torch.float64, device=dev)
    vol = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty(n, dtype=torch.int64, device=dev)
    chunk = 5_000_000
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        s, p, v, t = wl.stock_stream(b - a, keys, delta, seed_offset=seed_offset, start=start + a)
        sym[a:b] = torch.from_numpy((s.astype(np.int64) + key_base).astype(np.int32))
        price[a:b] = torch.from_numpy(p)
        vol[a:b] = torch.from_numpy(v)
        ts[a:b] = torch.from_numpy(t)
    return sym, price, vol, ts


def gen_roundrobin_columns(torch, n, keys_total, delta, rank, world, dev):
    """Rank `rank`'s round-robin share (global events rank, rank+world, ...) of one
    global StockStream over keys_total keys, resident in HBM, with global seq."""
    from siddhi_amd import workloads as wl
    sym = torch.empty(n, dtype=torch.int32, device=dev)
    price = torch.empty(n, dtype=torch.float64, device=dev)
    vol = torch.empty(n, dtype=torch.int64, device=dev)
    ts = torch.empty(n, dtype=torch.int64, device=dev)
    seq = torch.empty(n, dtype=torch.int64, device=dev)
    chunk = 5_000_000
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        idx = np.arange(a, b, dtype=np.int64) * world + rank
        s_, p_, v_, t_ = wl.stock_stream_at(idx, keys_total, delta, seed_offset=0)
        sym[a:b] = torch.from_numpy(s_.astype(np.int32))
        price[a:b] = torch.from_numpy(p_)
        vol[a:b] = torch.from_numpy(v_)
        ts[a:b] = torch.from_numpy(t_)
        seq[a:b] = torch.from_numpy(idx)
    return sym, price, vol, ts, seq


def align_calls(batch, n, call=1024):
    """Micro-batch size for n events in as many pushes as `batch` gives, each
    push whole InputHandler calls of `call` events (a cut inside a call would
    make two calls of it)."""
    if n <= call or batch >= n:
        return max(1, min(batch, n))
    k = -(-n // max(1, batch))          # pushes
    b = -(-n // k)
    return min(n, -(-b // call) * call)


def align_rr(batch, world, call=1024):
    """Largest micro-batch <= batch (at least one unit) whose cuts a * world are
    multiples of the call size: round-robin micro-batches then hold whole
    InputHandler calls (a call split over two pushes would see two clock moves)."""
    import math
    unit = call // math.gcd(call, world)
    return max(unit, batch // unit * unit)


def alg_bytes_pattern(c, n):
    """B_ev = 20 + 16*P + 24*f_new + 32*m per event."""
    P = c["partial_scans"] / max(n, 1)
    f_new = c["partials"] / max(n, 1)
    m = c["matches"] / max(n, 1)
    return (20 + 16 * P + 24 * f_new + 32 * m) * n, dict(P_bar=P, f_new=f_new, m_bar=m)


def alg_bytes_window(c, n, n_out):
    """B_ev = 20 (in) + 12 (re-read at expiry) + 36*o per event."""
    o = c["matches"] / max(n, 1)
    return (20 + 12 + 36 * o) * n, dict(o=o)


def pmc_summary(cfg_name):
    """Newest committed rocprofv3 PMC summary of this config (profiles/rNN_pmc_<config>.json,
    written by scripts/pmc_summary.py from separate FETCH_SIZE / WRITE_SIZE passes with the
    gfx950 corrections): per-kernel HBM bytes and times of one push.  Only a summary
    taken on the running sources (its "build" = buildinfo.source_hash()) is used;
    otherwise (None, reason) and the line's traffic stays null."""
    import glob
    from siddhi_amd.buildinfo import source_hash
    want = source_hash()
    newest = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_%s.json" % cfg_name)), reverse=True):
        d = json.load(open(f))
        if "push" not in d or "kernels" not in d:
            continue
        rel = os.path.relpath(f, ROOT)
        if d.get("build") == want:
            return d, rel
        newest = newest or rel
    return None, ("no PMC summary of build %s (newest %s is of other sources)" % (want, newest) if newest
                  else "no PMC summary of build %s" % want)


def cpu_baseline(cfg_name, app, keys, delta, sample):
    """CPU oracle (C++ restatement, 1 core) on the first `sample` events of the same
    stream; also returns its output rows (the parity_prefix check)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_engine import OracleQueryEngine
    from parity import compile_single_query, concat_rows
    from siddhi_amd import workloads as wl
    qp, _ = compile_single_query(app)
    eng = OracleQueryEngine(qp, None)
    s, p, v, t = wl.stock_stream(sample, keys, delta, seed_offset=0)
    vals = np.stack([s.astype(np.uint64), p.view(np.uint64), v.view(np.uint64)], axis=1)
    nul = np.zeros_like(vals, dtype=np.uint8)
    offs = wl.call_offsets(sample)
    lib = eng.lib
    nout = eng.n_out
    parts = []
    t0 = time.perf_counter()
    for c in range(len(offs) - 1):
        a, b = int(offs[c]), int(offs[c + 1])
        vv = np.ascontiguousarray(vals[a:b])
        nn = np.ascontiguousarray(nul[a:b])
        tt = np.ascontiguousarray(t[a:b])
        lib.orc_push(eng.h, 0, b - a, tt.ctypes.data, vv.ctypes.data, nn.ctypes.data, 1)
        m = lib.orc_num_rows(eng.h)
        if m:   # QueryCallback: the rows of this call
            ch, ty, ts_ = np.empty(m, np.int64), np.empty(m, np.int32), np.empty(m, np.int64)
            va, nu = np.empty((m, max(nout, 1)), np.uint64), np.empty((m, max(nout, 1)), np.uint8)
            lib.orc_get_rows(eng.h, ch.ctypes.data, ty.ctypes.data, ts_.ctypes.data, va.ctypes.data, nu.ctypes.data)
            parts.append((ch + 1_000_000 * c, ty, ts_, va[:, :nout], nu[:, :nout]))
        lib.orc_clear_rows(eng.h)
    dt = time.perf_counter() - t0
    oc = eng.counters()
    eng.close()
    ora_counters = {"events": int(oc[0]), "filter_evals": int(oc[1]), "partials": int(oc[2]), "matches": int(oc[3]),
                    "expired": int(oc[5])}
    return ({"value": sample / dt, "unit": "events/s", "cores": 1, "kind": "port",
             "sample": "first %d events of the %s stream (%d keys, delta %g ms), C++ restatement of the "
                       "reference NFA (oracle/oracle.cpp), 1 thread" % (sample, cfg_name, keys, delta)},
            concat_rows(parts), qp, ora_counters)


def cpu_baseline_parallel(cfg_name, app, keys, delta, sample, threads):
    """SURVEY.md §8d's per-key CPU variant: the oracle on `threads` host threads,
    thread t owning the partition keys with key % threads == t (a partitioned
    query's keys are independent: PartitionStreamReceiver), each fed its keys'
    events of every InputHandler call in arrival order.  ctypes releases the GIL
    inside orc_push, so the threads run in parallel."""
    import threading
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_engine import OracleQueryEngine
    from parity import compile_single_query
    from siddhi_amd import workloads as wl
    qp, _ = compile_single_query(app)
    s, p, v, t = wl.stock_stream(sample, keys, delta, seed_offset=0)
    offs = wl.call_offsets(sample)
    shard = s.astype(np.int64) % threads
    work = []
    for w in range(threads):
        idx = np.nonzero(shard == w)[0]
        vals = np.ascontiguousarray(np.stack([s[idx].astype(np.uint64), p[idx].view(np.uint64),
                                              v[idx].view(np.uint64)], axis=1))
        nul = np.zeros_like(vals, dtype=np.uint8)
        tt = np.ascontiguousarray(t[idx])
        cuts = np.searchsorted(idx, offs)   # this shard's slice of every call
        work.append((vals, nul, tt, cuts))
    engines = [OracleQueryEngine(qp, None) for _ in range(threads)]

    def run(w):
        vals, nul, tt, cuts = work[w]
        eng = engines[w]
        lib = eng.lib
        for c in range(len(cuts) - 1):
            a, b = int(cuts[c]), int(cuts[c + 1])
            if b > a:
                lib.orc_push(eng.h, 0, b - a, tt[a:].ctypes.data, vals[a:].ctypes.data, nul[a:].ctypes.data, 1)
                lib.orc_clear_rows(eng.h)

    ths = [threading.Thread(target=run, args=(w,)) for w in range(threads)]
    t0 = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    for e in engines:
        e.close()
    return {"value": sample / dt, "unit": "events/s", "cores": threads, "kind": "port",
            "sample": "first %d events of the %s stream, keys sharded over %d host threads (key %% %d), one oracle "
                      "engine per thread (oracle/oracle.cpp)" % (sample, cfg_name, threads, threads)}


def call_offsets_of(offs_all, a, b, cache=None):
    """InputHandler call boundaries inside micro-batch [a, b), relative to a
    (push_raw's call_offsets).  Input metadata like the columns themselves:
    with `cache` the arrays are built once, before the timed region (a
    50 M-event micro-batch has ~49 k calls, ~0.2-0.5 ms of NumPy per push)."""
    if cache is not None and (a, b) in cache:
        return cache[(a, b)]
    lo, hi = np.searchsorted(offs_all, a), np.searchsorted(offs_all, b)
    co = (np.concatenate([[a], offs_all[lo:hi][offs_all[lo:hi] > a], [b]]) - a).astype(np.int64)
    if cache is not None:
        cache[(a, b)] = co
    return co


def parity_prefix(torch, he, qp, cols, ts, offs_all, prefix, ora_rows, window, batch):
    """The device path on the first `prefix` events of the benchmark stream (one
    fresh query, the bench's micro-batch size, polled, outside the timed region)
    against the oracle's rows: bit-exact for patterns; window aggregates with
    doubles within 1e-9 relative (the default segmented scans).  Also returns
    the device's counters over the prefix (the derived P-bar / f_new / m-bar
    cross-check)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from parity import assert_rows_agg, assert_same_rows, concat_rows
    dq = he.DeviceQuery(qp.ir)
    try:
        parts = []
        for a in range(0, prefix, batch):
            b = min(prefix, a + batch)
            lo, hi = np.searchsorted(offs_all, a), np.searchsorted(offs_all, b)
            co = np.concatenate([[a], offs_all[lo:hi][offs_all[lo:hi] > a], [b]]) - a
            dq.push_raw(0, b - a, ts.data_ptr() + 8 * a, [c.data_ptr() + c.element_size() * a for c in cols],
                        [0] * len(cols), he.SHD_MEM_DEVICE, co.astype(np.int64), True)
            r = dq.poll()
            if r is not None:
                parts.append(r)
        dev = concat_rows(parts)
        if window:
            assert_rows_agg(dev, ora_rows, qp, exact=False)
        else:
            assert_same_rows(dev, ora_rows)
        pushes = -(-prefix // batch)
        return "equal (%d events in %d pushes of %d, %d rows%s)" % (
            prefix, pushes, batch, len(dev[2]), ", doubles within 1e-9" if window else ""), dq.counters()
    except AssertionError as e:
        return "DIFFERENT: %s" % str(e).splitlines()[0], dq.counters()
    finally:
        dq.close()


def run_multi(args, torch, dist, rank, world, local, dev):
    """Config M5: every query of a multi-query app on one StockStream junction
    (StreamJunction fan-out, C/stream/StreamJunction.java:146-272).
    Query-parallel: rank r runs the queries with index % world == r over the
    whole stream (broadcast input: each rank holds it in its own HBM);
    value = stream events / max-over-ranks time ("strong": the total work,
    all queries over the stream, is fixed as N grows)."""
    from siddhi_amd import workloads as wl
    from siddhi_amd import hip_engine as he
    from siddhi_amd.planner import StringDictionary, plan_query, plan_shared_leader, share_groups
    from siddhi_amd import query_compiler as qc

    app, n_def, k_def, delta = wl.CONFIGS[args.config]
    n = args.events or n_def
    keys = args.keys or k_def
    qa = qc.parse(app)
    d = StringDictionary()
    wl.register_symbols(d, keys)
    queries = list(qa.execution_order)
    plans = [plan_query(qa, item, d) for item in queries]
    mine = [i for i in range(len(plans)) if i % world == rank]
    sym, price, vol, ts = gen_device_columns(torch, n, keys, delta, seed_offset=0, key_base=0, dev=dev)
    torch.cuda.synchronize()
    he.context(local)
    dqs = {i: he.DeviceQuery(plans[i].ir, device=local) for i in mine}
    # query sharing: the P1 variants (same f2 / within, e1 threshold 60..84.5)
    # run one forward scan per rank (shd_group_*); every other query alone
    units = []      # (DeviceGroup | None, [query index])
    grouped = set()
    if not args.no_share:
        for g in share_groups([queries[i] for i in mine]):
            idx = [mine[k] for k in g]
            lead = plan_shared_leader(qa, [queries[i] for i in idx], d)
            units.append((he.DeviceGroup(lead.ir, [dqs[i] for i in idx], device=local), idx))
            grouped.update(idx)
    units += [(None, [i]) for i in mine if i not in grouped]
    # 100 queries each keep their own scratch: 10M-event micro-batches by default
    batch = align_calls(min(args.batch if args.batch != 50_000_000 else 10_000_000, n), n)
    cuts = list(range(0, n, batch)) + [n]
    offs_all = wl.call_offsets(n)

    co_cache = {}
    for a, b in zip(cuts[:-1], cuts[1:]):
        call_offsets_of(offs_all, a, b, co_cache)

    def run_step(collect=None):
        for grp, idx in units:
            if grp is not None:
                grp.reset()
            else:
                dqs[idx[0]].reset()
        tot = {}
        for a, b in zip(cuts[:-1], cuts[1:]):
            co = call_offsets_of(offs_all, a, b, co_cache)
            cols = [sym.data_ptr() + 4 * a, price.data_ptr() + 8 * a, vol.data_ptr() + 8 * a]
            for grp, idx in units:   # junction fan-out
                tgt = grp if grp is not None else dqs[idx[0]]
                tgt.push_raw(0, b - a, ts.data_ptr() + 8 * a, cols, [0, 0, 0], he.SHD_MEM_DEVICE, co, True)
                for i in idx:
                    dqs[i].discard()
                if collect is not None:
                    for k, v in tgt.stage_times().items():
                        tot[k] = tot.get(k, 0) + v
        if collect is not None:
            collect.append(tot)

    tw = time.perf_counter()
    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    if rank == 0:
        print("M5: warmup %.1f s (%d units, %d shared scans)" % (time.perf_counter() - tw, len(units),
              sum(1 for g, _ in units if g is not None)), file=sys.stderr, flush=True)
    if dist:
        dist.barrier()
    stage_runs = []
    t0 = time.perf_counter()
    for k in range(args.steps):
        run_step(stage_runs)
        if rank == 0:
            print("M5: step %d done at %.1f s" % (k, time.perf_counter() - t0), file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # algorithmic bytes (SURVEY.md §8d formulas): a shared scan counts the input
    # record and its partial-match traffic once (the leader's P and f_new) plus
    # every member's 32-byte output rows; a query alone counts its own formula
    bytes_step, matches = 0.0, 0
    for grp, idx in units:
        if grp is not None:
            c = grp.counters()
            mc = [dqs[i].counters() for i in idx]
            mem_matches = sum(x["matches"] for x in mc)
            if grp.leader_engine_kind() == 2:
                # shared windows: the input record once, each member's expiry re-read and rows
                bytes_step += 20 * c["events"] + sum(alg_bytes_window(x, x["events"], 0)[0] - 20 * x["events"]
                                                     for x in mc)
            else:
                b_lead, _ = alg_bytes_pattern(dict(c, matches=0), c["events"])
                bytes_step += b_lead + 32 * mem_matches
            matches += mem_matches
            continue
        dq = dqs[idx[0]]
        c = dq.counters()
        matches += c["matches"]
        if dq.engine_kind in (1, 4):
            bytes_step += alg_bytes_pattern(c, c["events"])[0]
        else:
            bytes_step += alg_bytes_window(c, c["events"], 0)[0]
    stages = {}
    for r in stage_runs:
        for k, v in r.items():
            stages[k] = stages.get(k, 0) + v / len(stage_runs)
    vals = torch.tensor([bytes_step, float(matches)], dtype=torch.float64, device=dev)
    if dist:
        dist.all_reduce(vals)
    bytes_all, matches_all = float(vals[0].item()), float(vals[1].item())
    roof = None
    if stages:
        # frac as on the P3 line: the path's algorithmic bytes per step / the wall
        # time of a step; device_*: / the HIP-event time of every push
        ach = bytes_step / (elapsed / args.steps) / 1e9
        dev_ach = bytes_step / (sum(stages.values()) * 1e-9) / 1e9
        # HBM bytes of the whole fan-out (every unit's kernels per stream
        # micro-batch, PMC summary of this build) x micro-batches per step
        pmc, psrc = pmc_summary("M5")
        traffic = round(pmc["push"]["hbm_bytes_per_event"] * n) if pmc else None
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_ratio": round(traffic / bytes_step, 3) if traffic else None,
                "alg_bytes_per_event": round(bytes_step / n, 2),
                "scope": "whole fan-out per step (wall clock), rank 0",
                "device_achieved": round(dev_ach, 1), "device_frac": round(dev_ach / HBM_PEAK_GBS, 4),
                "stage_top": max(stages, key=stages.get),
                "pmc_source": psrc if pmc else None, "pmc_note": None if pmc else psrc}
    if rank == 0:
        line = {
            "metric": "events/sec ingested + matches/sec (partitioned pattern, 1–8 GPU); % HBM peak",
            "value": round(n * args.steps / elapsed, 1), "unit": "events/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (seeded SplitMix64 StockStream, BASELINE.md)",
            "build": __import__("siddhi_amd.buildinfo", fromlist=["source_hash"]).source_hash(),
            "config": {"workload": "M5", "queries": len(plans), "events": n, "keys": keys, "delta_ms": delta,
                       "micro_batch": batch, "call_size": 1024,
                       "parallelism": "query-parallel x%d (broadcast input)" % world,
                       "shared_scans": [len(idx) for grp, idx in units if grp is not None]},
            "query_events_per_s": round(n * len(plans) * args.steps / elapsed, 1),
            "matches_per_s": round(matches_all * args.steps / elapsed, 1),
            "algorithmic_bytes_per_step": round(bytes_all),
            "stage_ms_per_step_rank0": {k: round(v / 1e6, 3) for k, v in stages.items()},
            "roofline": roof,
            "cpu_baseline": None,
        }
    for grp, _ in units:
        if grp is not None:
            grp.close()
    for dq in dqs.values():
        dq.close()
    if rank == 0 and args.cpu_sample != 0:
        sample = min(n, args.cpu_sample if args.cpu_sample > 0 else 200_000)
        line["parity_prefix"], line["cpu_baseline"] = m5_parity_prefix(
            he, qa, queries, plans, d, sym, price, vol, ts, sample, keys, delta, not args.no_share, args.m5_direct)
        print(json.dumps(line))
    elif rank == 0:
        print(json.dumps(line))


def m5_parity_prefix(he, qa, queries, plans, d, sym, price, vol, ts, prefix, keys, delta, share, direct_all=False):
    """Every M5 query on the first `prefix` events of the benchmark stream, run
    the way the timed loop runs it (the shared scans of shd_group included, one
    push), against the CPU oracle on the same events: pattern rows bit-exact,
    window rows with doubles within 1e-9 relative.

    The oracle scans every pending partial per event (the reference's
    StreamPreStateProcessor loop), which at M5's density is quadratic: one P1
    variant over 200 k events costs minutes.  So each group of shareable
    queries is checked through its leader plan, run once in the oracle: a
    member's expected rows are the leader's whose e1 passes the member's
    threshold (planner.share_groups' lemma, pinned on the oracle itself by
    tests/test_share_plan.py), and the group's first, middle and last members
    also run in the oracle directly.  direct_all (--m5-direct): every member
    against its own oracle run instead.  Oracle runs go to a thread pool (ctypes
    drops the GIL in the C++ oracle).

    cpu_baseline: all queries of the app through the oracle, one after the
    other on one core, over the first 10 k events (CPU seconds per thread)."""
    import concurrent.futures as cf
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_engine import OracleQueryEngine
    from parity import assert_rows_agg, assert_same_rows, concat_rows
    from siddhi_amd import query_compiler as qc
    from siddhi_amd import workloads as wl
    from siddhi_amd.planner import _e1_site, _threshold, plan_shared_leader, share_groups
    from siddhi_amd.runtime import ColumnBatch
    s, p, v, t = wl.stock_stream(prefix, keys, delta, seed_offset=0)
    offs = wl.call_offsets(prefix)
    groups = share_groups(queries)
    dqs = [he.DeviceQuery(qp.ir) for qp in plans]
    dgroups = []
    grouped = set()
    if share:
        for g in groups:
            dgroups.append(he.DeviceGroup(plan_shared_leader(qa, [queries[i] for i in g], d).ir, [dqs[i] for i in g]))
            grouped.update(g)
    cols = [sym.data_ptr(), price.data_ptr(), vol.data_ptr()]
    for tgt in dgroups + [dqs[i] for i in range(len(dqs)) if i not in grouped]:
        tgt.push_raw(0, prefix, ts.data_ptr(), cols, [0, 0, 0], he.SHD_MEM_DEVICE, offs.astype(np.int64), True)
    devs = []
    for dq in dqs:
        r = dq.poll()
        devs.append((concat_rows([r] if r is not None else []), dq.engine_kind == 2))
    for g in dgroups:
        g.close()
    for dq in dqs:
        dq.close()

    def oracle(qp, n):
        eng = OracleQueryEngine(qp, None)
        parts = []
        cid = 0
        t0 = time.thread_time()
        for c in range(len(offs) - 1):
            a, b = int(offs[c]), int(offs[c + 1])
            if a >= n:
                break
            b = min(b, n)
            sub = ColumnBatch(t[a:b], [s[a:b].astype(np.uint32), p[a:b], v[a:b]], [None, None, None])
            for ch in eng.set_time(int(t[b - 1])) + eng.push(0, sub):
                k = len(ch.ts)
                parts.append((np.full(k, cid, np.int64), ch.types, ch.ts, ch.values, ch.nulls))
                cid += 1
        cpu = time.thread_time() - t0
        eng.close()
        return concat_rows(parts), cpu

    def member_mask(q, qp, lead_rows):
        """Rows of the leader whose e1 passes q's threshold, or None when q's
        f1 is not a threshold on an attribute the selector projects as e1.<attr>."""
        th = _threshold(_e1_site(q).filters)
        if th is None:
            return None
        op, var, const = th
        ref = _e1_site(q).ref
        for c, oa in enumerate(q.selector.attrs):
            if isinstance(oa.expr, qc.Var) and oa.expr.attr == var.attr and oa.expr.stream == ref:
                col = lead_rows[3][:, c]
                vals = col.view(np.float64) if qp.output_types[c] == 4 else col.view(np.int64)
                return {">": vals > const.value, ">=": vals >= const.value, "<": vals < const.value,
                        "<=": vals <= const.value}[op]
        return None

    direct = set(range(len(plans)))
    leaders = []
    for g in groups:
        if direct_all or _e1_site(queries[g[0]]) is None:   # every member against its own oracle run
            continue
        lead = plan_shared_leader(qa, [queries[i] for i in g], d)
        spot = {g[0], g[len(g) // 2], g[-1]}
        leaders.append((g, lead, spot))
        direct -= set(g) - spot
    rows = 0
    checked_direct, checked_lemma = 0, 0
    try:
        with cf.ThreadPoolExecutor(max_workers=16) as ex:
            fut_direct = {i: ex.submit(oracle, plans[i], prefix) for i in sorted(direct)}
            fut_lead = [ex.submit(oracle, lead, prefix) for _, lead, _ in leaders]
            for i, f in fut_direct.items():
                ora, _ = f.result()
                dev, window = devs[i]
                if window:
                    assert_rows_agg(dev, ora, plans[i], exact=False)
                else:
                    assert_same_rows(dev, ora)
                rows += len(dev[2])
                checked_direct += 1
                if checked_direct % 5 == 0:
                    print("M5 parity: %d / %d direct checks" % (checked_direct, len(fut_direct)), file=sys.stderr,
                          flush=True)
            print("M5 parity: %d queries checked directly" % checked_direct, file=sys.stderr, flush=True)
            for (g, lead, spot), f in zip(leaders, fut_lead):
                lead_rows, _ = f.result()
                for i in g:
                    if i in spot:
                        continue
                    keep = member_mask(queries[i], plans[i], lead_rows)
                    if keep is None:
                        ora, _ = oracle(plans[i], prefix)
                    else:
                        # the leader's chunk ids: one callback chunk per completing event
                        ora = tuple(x[keep] for x in lead_rows)
                        checked_lemma += 1
                    dev = devs[i][0]
                    assert_same_rows(dev, ora)
                    rows += len(dev[2])
        verdict = ("equal (%d queries, %d through shared passes; %d checked against their own oracle run, %d "
                   "against the oracle leader's rows passing their e1 threshold; %d events, %d rows)"
                   % (len(plans), len(grouped), checked_direct, checked_lemma, prefix, rows))
    except AssertionError as e:
        verdict = "DIFFERENT: %s" % str(e).splitlines()[0]
    cpu_n = min(prefix, 10_000)
    cpu_s = sum(oracle(qp, cpu_n)[1] for qp in plans)
    cpu = {"value": round(cpu_n / cpu_s, 1) if cpu_s > 0 else None, "unit": "events/s", "cores": 1,
           "kind": "port",
           "sample": "the first %d stream events through all %d queries, one after the other (oracle C++ "
                     "restatement, CPU seconds of one thread, polled per InputHandler call; the pattern "
                     "queries' pending-list scans grow with the sample)" % (cpu_n, len(plans))}
    return verdict, cpu


def run_e2e(args):
    """SURVEY.md section 8d "End-to-end InputHandler throughput is reported
    separately": the config's app through the public API
    (SiddhiManager.createSiddhiAppRuntime -> InputHandler.send_batch of host
    SoA columns in InputHandler calls of 1024 events -> QueryCallback.receive
    with decoded Event[] rows), timed from the first send to the last
    callback; plus InputHandler.send(Event[]) per call on a sample (the
    per-event API, rows converted on the host).  The rows the callbacks saw
    are checked against a DeviceQuery fed the same events directly.
    Reference: C/stream/input/InputHandler.java:85-95,
    C/query/output/callback/QueryCallback.java:61-91."""
    from siddhi_amd import workloads as wl
    from siddhi_amd import hip_engine as he
    from siddhi_amd.runtime import SiddhiManager, QueryCallback, ColumnBatch, Event
    app, n_def, k_def, delta = wl.CONFIGS[args.config]
    n = args.events or 20_000_000
    keys = args.keys or k_def
    sym, price, vol, ts = wl.stock_stream(n, keys, delta)

    class Count(QueryCallback):
        def __init__(self):
            self.rows = 0
            self.calls = 0
            self.t_last = None

        def receive(self, timestamp, inEvents, removeEvents):  # noqa: N802,N803
            self.calls += 1
            self.rows += (len(inEvents) if inEvents else 0) + (len(removeEvents) if removeEvents else 0)
            self.t_last = time.perf_counter()

    def run(n_ev, per_event=False, steady=False):
        sm = SiddhiManager()
        rt = sm.createSiddhiAppRuntime(app)
        # the first query of the config app (P3: the partitioned pattern, W2: the window)
        cb = Count()
        rt.addCallback(rt.queries[0].name, cb)
        ih = rt.getInputHandler("StockStream")
        rt.start()
        # the symbol column as dictionary ids of "S%07d" strings
        d = rt.dictionary
        if per_event:
            names = ["S%07d" % i for i in range(keys)]
            calls = []
            for a in range(0, n_ev, 1024):
                b = min(a + 1024, n_ev)
                calls.append([Event(int(ts[i]), [names[int(sym[i])], float(price[i]), int(vol[i])])
                              for i in range(a, b)])
            t0 = time.perf_counter()
            timed_from = 0
            for c in calls:
                ih.send(c)
        else:
            for i in range(keys):
                d.id("S%07d" % i)
            t0 = None
            timed_from = 0
            t_send = time.perf_counter()
            for a in range(0, n_ev, args.e2e_batch):
                b = min(a + args.e2e_batch, n_ev)
                offs = np.append(np.arange(0, b - a, 1024, dtype=np.int64), np.int64(b - a))
                ih.send_batch(ColumnBatch(ts[a:b], [sym[a:b], price[a:b], vol[a:b]], [None, None, None], offs))
                if t0 is None and steady and b < n_ev:
                    # steady state: the runtime's first send_batch sizes its
                    # pinned staging and device buffers (hipHostMalloc /
                    # hipMalloc of the batch's size), once per runtime
                    t0, timed_from = time.perf_counter(), b
            if t0 is None:
                t0 = t_send
        t1 = time.perf_counter()
        name = rt.queries[0].engine.engine_name
        rt.shutdown()
        return (t1 - t0), cb, name, n_ev - timed_from
    he.load_library()
    run(min(n, 2_000_000))   # warm-up (library, device context, first allocations)
    el_cold, cb, engine, _ = run(n)
    el, cb_s, _, n_timed = run(n, steady=True)
    assert cb_s.rows == cb.rows
    sample = min(n, 200_000)
    el_ev, cb_ev, _, _ = run(sample, per_event=True)
    # the same events straight into the engine (no runtime): its row count
    dq = he.DeviceQuery(__import__("siddhi_amd.planner", fromlist=["x"]).plan_query(
        *_first_query(app)).ir)
    rows = 0
    for a in range(0, n, args.e2e_batch):
        b = min(a + args.e2e_batch, n)
        offs = np.append(np.arange(0, b - a, 1024, dtype=np.int64), np.int64(b - a))
        dq.push_raw(0, b - a, ts[a:b].ctypes.data, [sym[a:b].ctypes.data, price[a:b].ctypes.data,
                                                    vol[a:b].ctypes.data], [0, 0, 0], he.SHD_MEM_HOST, offs, True)
        r = dq.poll()
        rows += 0 if r is None else len(r[0])
    dq.close()
    from siddhi_amd.buildinfo import source_hash
    print(json.dumps({
        "metric": "end-to-end InputHandler events/s (host SoA columns -> SiddhiManager -> InputHandler.send_batch "
                  "-> QueryCallback Event[])",
        "value": round(n_timed / el, 1), "unit": "events/s", "n_gpus": 1, "higher_is_better": True,
        "build": source_hash(),
        "config": {"workload": args.config, "events": n, "keys": keys, "delta_ms": delta,
                   "send_batch_events": args.e2e_batch, "call_size": 1024, "engine": engine},
        "timed": "steady state: the send_batch calls after the runtime's first (which sizes its pinned staging "
                 "and device buffers once); %d of %d events" % (n_timed, n),
        "seconds": round(el, 3),
        "cold_start": {"value": round(n / el_cold, 1), "unit": "events/s",
                       "note": "a fresh runtime, every send_batch timed (first-use allocations included)"},
        "callback_rows": cb.rows, "callback_invocations": cb.calls,
        "rows_equal_engine_direct": cb.rows == rows,
        "per_event_api": {"value": round(sample / el_ev, 1), "unit": "events/s", "events": sample,
                          "note": "InputHandler.send(Event[]) of 1024-event calls (Python objects -> SoA on the "
                                  "host, one push per call)", "callback_rows": cb_ev.rows},
        "note": "PCIe-inclusive: columns pushed from host memory (SHD_MEM_HOST); never the engine `value`"}))


def _first_query(app):
    from siddhi_amd.planner import StringDictionary
    from siddhi_amd import query_compiler as qc
    qa = qc.parse(app)
    item = qa.execution_order[0]
    if isinstance(item, qc.Partition):
        return qa, item.queries[0], StringDictionary(), item
    return qa, item, StringDictionary(), None


def main():
    args = parse()
    if args.e2e:
        run_e2e(args)
        return
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(local)
    if args.config == "M5":
        run_multi(args, torch, dist, rank, world, local, dev)
        if dist:
            dist.destroy_process_group()
        return

    from siddhi_amd import workloads as wl
    from siddhi_amd import hip_engine as he
    from siddhi_amd.planner import StringDictionary, plan_query
    from siddhi_amd import query_compiler as qc

    app, n_def, k_def, delta = wl.CONFIGS[args.config]
    n = args.events or n_def
    keys = args.keys or k_def
    pattern = not args.config.startswith("W")   # P1 / P3 / S4: pattern formula of §8d
    qa = qc.parse(app)
    item = qa.execution_order[0]
    if isinstance(item, qc.Partition):
        qp = plan_query(qa, item.queries[0], StringDictionary(), item)
    else:
        qp = plan_query(qa, item, StringDictionary())

    # Config 3: at N > 1 the headline is one global stream over
    # 10 M keys held round-robin by the ranks and re-routed to the key owners
    # with an RCCL all-to-all per micro-batch; the prepartitioned measurement
    # (events arrive at their owner, keys_per_gpu each, no data-path
    # collective) runs alongside.  N = 1 is prepartitioned (nothing to route).
    # Window configs (unpartitioned: one window over the whole stream) split the
    # global stream by time instead: rank r holds slice r and primes its query with
    # the previous slice's tail (exchange.py, "time slices with a halo").
    mode = args.input if args.input != "auto" else (
        "prepartitioned" if world == 1 else ("roundrobin" if pattern else "slices"))
    if mode == "roundrobin" and not pattern:
        raise SystemExit("--input roundrobin re-routes by partition key; window configs use --input slices")
    if mode == "slices" and pattern:
        raise SystemExit("--input slices is for the (unpartitioned) window configs")

    def measure(mode):
        kb = None
        # inputs resident in HBM before the timed region
        if mode == "prepartitioned":
            # rank r owns key slice r and its own events (no data-path collective)
            kb = args.key_base if args.key_base >= 0 else rank * keys
            sym, price, vol, ts = gen_device_columns(torch, n, keys, delta, seed_offset=rank, key_base=kb, dev=dev)
            seqs = None
        elif mode == "slices":
            # rank r holds events [r * n, (r + 1) * n) of ONE global stream over `keys` keys
            kb = 0
            sym, price, vol, ts = gen_device_columns(torch, n, keys, delta, seed_offset=0, key_base=0, dev=dev,
                                                     start=rank * n)
            seqs = None
        else:
            # one global stream over `keys` keys in all, held round-robin; re-routed per micro-batch
            sym, price, vol, ts, seqs = gen_roundrobin_columns(torch, n, keys, delta, rank, world, dev)
        torch.cuda.synchronize()
        from siddhi_amd import exchange as ex
        he.context(local)
        dq = he.DeviceQuery(qp.ir, device=local)
        batch = align_calls(min(args.batch, n), n)   # micro-batches of whole InputHandler calls
        if seqs is not None:
            # a micro-batch [a, b) of this rank's round-robin share spans global
            # seqs [a * world, b * world): cut on InputHandler call boundaries
            # (multiples of 1024 global seqs), so no call straddles two pushes
            batch = align_rr(batch, world)
        cuts = list(range(0, n, batch)) + [n]
        offs_all = wl.call_offsets(n)

        routed_total = [0]
        take = [0]
        pipe = ex.RoutePipeline(local) if seqs is not None else None
        cols4 = [sym, price, vol, ts]

        def push_halo(halo):
            """Prime the fresh query with the previous slice's tail; its rows are dropped."""
            torch.cuda.current_stream().synchronize()   # received columns complete before the engine reads them
            m = halo[3].numel()
            dq.push_raw(0, m, halo[3].data_ptr(), [halo[0].data_ptr(), halo[1].data_ptr(), halo[2].data_ptr()],
                        [0, 0, 0], he.SHD_MEM_DEVICE, wl.call_offsets(m), True)
            dq.discard()

        if mode == "slices" and world > 1:
            window = ex.window_of(qp)
            first_ts = int(ts[0].item())

            def prime(halo):
                dq.reset()
                push_halo(halo)
                return ex.halo_covers(window, dq.counters()["carry"], halo[3], first_ts)
            take[0] = ex.halo_take(window, n, lambda k: ex.exchange_tail(cols4, k, rank, world), prime, device=dev)

        co_cache = {}   # call offsets per micro-batch, built before the timed region
        if seqs is None:
            for a, b in zip(cuts[:-1], cuts[1:]):
                call_offsets_of(offs_all, a, b, co_cache)

        def run_step(collect=None, cuts=cuts):
            dq.reset()
            tot = {}
            if take[0]:
                # the halo: one RCCL send/recv pair per rank and step, inside the timed region
                halo = ex.exchange_tail(cols4, take[0], rank, world)
                if halo is not None:
                    push_halo(halo)
            routed_iter = None
            if seqs is not None and not os.environ.get("SHD_ROUTE_TORCH") and not os.environ.get("SHD_ROUTE_SYNC"):
                # micro-batch k+1 routed on a side stream while k is pushed
                # (exchange.RoutePipeline.run_staged: bucket + counts exchange of
                # k+2 before the data exchange + merge of k+1, host copies one
                # micro-batch ahead -- no blocking device-to-host read)
                def job(a, b):
                    lo = (a * world) // 1024 * 1024
                    nb = -(-(b * world - lo) // 1024)
                    return (lambda: ex.route_stage_a([sym[a:b], price[a:b], vol[a:b], ts[a:b]], sym[a:b], seqs[a:b],
                                                     world, lo, device=local),
                            lambda st: ex.route_stage_b(st, 1024, nb))
                routed_iter = pipe.run_staged([job(a, b) for a, b in zip(cuts[:-1], cuts[1:])])
                engine_stream = torch.cuda.ExternalStream(dq.stream_handle(), device=dev)
            held = None   # the previous micro-batch's routed tensors (RoutePipeline: lifetime)
            for a, b in zip(cuts[:-1], cuts[1:]):
                if routed_iter is not None:
                    routed = next(routed_iter)
                    (rs, rp, rv, rt), rseq, co, _ = routed
                    m = rs.numel()
                    routed_total[0] += m
                    if m > 0:
                        engine_stream.wait_event(co.event)   # the merge done before the engine reads its rows
                        dq.push_raw(0, m, rt.data_ptr(), [rs.data_ptr(), rp.data_ptr(), rv.data_ptr()], [0, 0, 0],
                                    he.SHD_MEM_DEVICE, co.get().astype(np.int64), True)
                    held = routed   # released after the next push has returned
                elif seqs is None:
                    # InputHandler calls of 1024 events inside the micro-batch
                    co = call_offsets_of(offs_all, a, b, co_cache)
                    cols = [sym.data_ptr() + 4 * a, price.data_ptr() + 8 * a, vol.data_ptr() + 8 * a]
                    dq.push_raw(0, b - a, ts.data_ptr() + 8 * a, cols, [0, 0, 0], he.SHD_MEM_DEVICE, co, True)
                else:
                    # RCCL all-to-all: every event to its key's owner, arrival order restored by seq
                    if os.environ.get("SHD_ROUTE_TORCH"):
                        # round-2 routing (torch owner sort + sequence sort), for comparison
                        (rs, rp, rv, rt), rseq, _ = ex.route([sym[a:b], price[a:b], vol[a:b], ts[a:b]], sym[a:b],
                                                             seqs[a:b], world)
                        co = ex.call_offsets_from_seq(rseq, 1024).numpy() if rs.numel() else None
                    else:
                        # HIP bucket scatter -> all-to-all -> per-call merge (csrc/route.hip); the
                        # micro-batch spans global seqs [a * world, b * world) (round-robin shares)
                        lo = (a * world) // 1024 * 1024
                        nb = -(-(b * world - lo) // 1024)
                        (rs, rp, rv, rt), rseq, co, _ = ex.route_device(
                            [sym[a:b], price[a:b], vol[a:b], ts[a:b]], sym[a:b], seqs[a:b], world, lo, 1024, nb,
                            device=local)
                    m = rs.numel()
                    routed_total[0] += m
                    if m == 0:
                        continue
                    torch.cuda.current_stream().synchronize()   # routed columns complete before the engine's stream reads them
                    dq.push_raw(0, m, rt.data_ptr(), [rs.data_ptr(), rp.data_ptr(), rv.data_ptr()], [0, 0, 0],
                                he.SHD_MEM_DEVICE, co.astype(np.int64), True)
                dq.discard()
                if collect is not None:
                    for k, v in dq.stage_times().items():
                        tot[k] = tot.get(k, 0) + v
            if collect is not None:
                collect.append(tot)
            return dq.counters()

        for sb in [int(x) for x in args.sweep_batches.split(",") if x]:
            # micro-batch size sweep (diagnostic): same data, same query
            if seqs is not None:
                sb = align_rr(sb, world)
            sc = list(range(0, n, sb)) + [n]
            run_step(cuts=sc)
            torch.cuda.synchronize()
            sr = []
            t0 = time.perf_counter()
            for _ in range(max(args.steps, 1)):
                run_step(sr, cuts=sc)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / max(args.steps, 1)
            st = {k: round(sum(r.get(k, 0) for r in sr) / len(sr) / 1e6, 3) for k in sr[0]} if sr else {}
            if rank == 0:
                print(json.dumps({"sweep_batch": sb, "ms_per_step": round(dt * 1e3, 3),
                                  "events_per_s": round(n * world / dt, 1), "stage_ms_per_step": st}),
                      file=sys.stderr, flush=True)

        # SURVEY.md §8d algorithmic bytes need the reference's pending-scan counts
        # (P-bar: (partial, event) pairs its pending lists visit): the walks count
        # exactly those, taken from one untimed calibration step.
        calib = run_step() if pattern else None
        for _ in range(args.warmup):
            run_step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        stage_runs = []
        t0 = time.perf_counter()
        counters = None
        for _ in range(args.steps):
            counters = run_step(stage_runs)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if dist:
            t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        ms_per_step = elapsed / args.steps * 1e3
        total_events = n * world * args.steps
        value = total_events / elapsed
        return dict(sym=sym, price=price, vol=vol, ts=ts, seqs=seqs, kb=kb, dq=dq, calib=calib, counters=counters,
                    halo=take[0],
                    stage_runs=stage_runs, elapsed=elapsed, ms_per_step=ms_per_step, value=value, batch=batch,
                    offs_all=offs_all, total_events=total_events)

    M = measure(mode)
    sym, price, vol, ts, seqs, kb, dq, calib = (M[k] for k in ("sym", "price", "vol", "ts", "seqs", "kb", "dq", "calib"))
    counters, stage_runs, elapsed, ms_per_step, value = (M[k] for k in ("counters", "stage_runs", "elapsed",
                                                                        "ms_per_step", "value"))
    batch, offs_all, total_events = M["batch"], M["offs_all"], M["total_events"]
    alongside = None
    if world > 1 and mode == "roundrobin" and args.input == "auto":
        A = measure("prepartitioned")
        A["dq"].close()
        alongside = {"input": "prepartitioned", "keys_per_gpu": keys, "value": round(A["value"], 1),
                     "ms_per_step": round(A["ms_per_step"], 3), "matches": A["counters"]["matches"] * world}
        del A

    # per-stage device times (HIP events on the query's stream), averaged per step
    stages = {}
    for r in stage_runs:
        for k, v in r.items():
            stages[k] = stages.get(k, 0) + v / len(stage_runs)
    step_dev_ns = sum(stages.values())
    if pattern:
        bytes_step, derived = alg_bytes_pattern(calib, calib["events"])
    else:
        bytes_step, derived = alg_bytes_window(counters, counters["events"], len(qp.output_names))
    roof = None
    if stages:
        # frac: the path's algorithmic bytes per step / the wall time of a step
        # (recomputable from this line: alg_bytes_per_event * events / ms_per_step);
        # device_*: / the HIP-event time of the push pipeline; kernels: each
        # kernel's own HBM bytes (PMC) / its rocprof duration, from profiles/
        ach = bytes_step / (elapsed / args.steps) / 1e9
        dev_ach = bytes_step / (step_dev_ns * 1e-9) / 1e9
        pmc, psrc = pmc_summary(args.config)
        traffic = None
        kern = None
        pmc_note = None
        if not pmc:
            pmc_note, psrc = psrc, None
        if pmc:
            traffic = round(pmc["push"]["hbm_bytes_per_event"] * n)
            top = sorted(pmc["kernels"].items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["dispatches_per_push"])[:5]
            kern = {k: {"avg_us": v["avg_us"], "per_push": v["dispatches_per_push"],
                        "hbm_bytes_per_event": v["hbm_bytes_per_event"], "hbm_frac": v["hbm_frac"]}
                    for k, v in top}
        roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_ratio": round(traffic / bytes_step, 3) if traffic else None,
                "alg_bytes_per_event": round(bytes_step / n, 2),
                "scope": "whole push pipeline per step (wall clock)",
                "device_achieved": round(dev_ach, 1), "device_frac": round(dev_ach / HBM_PEAK_GBS, 4),
                "pmc_source": psrc, "pmc_note": pmc_note, "kernels": kern}
    matches_per_s = counters["matches"] * world * args.steps / elapsed

    cpu = None
    cpu_mt = None
    prefix = None
    derived_check = None
    if rank == 0 and world == 1 and args.cpu_sample != 0:
        sample = args.cpu_sample if args.cpu_sample > 0 else (4_000_000 if pattern else 2_000_000)
        sample = min(sample, n)
        cpu, ora_rows, _, oc = cpu_baseline(args.config, app, keys, delta, sample)
        if mode == "prepartitioned" and kb == 0:
            # at least two pushes: the prefix cut like the timed stream is, in
            # micro-batches, so the state carried between pushes is compared
            # (at most half the prefix per push)
            # (at most half the prefix per push, whole InputHandler calls: a push
            # cut inside a call would make two calls of it)
            pb = align_calls(max(1, min(batch, sample // 2)), sample)
            prefix, pc = parity_prefix(torch, he, qp, [sym, price, vol], ts, offs_all, sample, ora_rows,
                                       not pattern, pb)
            if args.config in ("P1", "P3", "P3-dense"):
                # the §8d counts two ways on the same prefix: the device's walks
                # ((partial, event) pairs visited, the expiring visit included) and
                # the oracle's filter evaluations minus the start state's f1 per
                # event, plus the partials its expireEvents removed
                dev_d = alg_bytes_pattern(pc, pc["events"])[1]
                ora_pairs = oc["filter_evals"] - oc["events"] + oc["expired"]
                ora_d = dict(P_bar=ora_pairs / sample, f_new=oc["partials"] / sample, m_bar=oc["matches"] / sample)
                derived_check = {"prefix_events": sample,
                                 "device": {k: round(v, 6) for k, v in dev_d.items()},
                                 "oracle": {k: round(v, 6) for k, v in ora_d.items()}}
                same = ["P_bar", "f_new", "m_bar"]
                if not isinstance(item, qc.Partition):
                    # unpartitioned (P1): the reference's one pending list holds every
                    # symbol's partials and each event's filter runs over all of them;
                    # the device groups by the e2 filter's symbol equality (§4.1) and
                    # visits same-symbol partials only, so only f_new and m_bar compare
                    same = ["f_new", "m_bar"]
                    derived_check["P_bar_scope"] = ("device: same-symbol partials visited; oracle: the "
                                                    "global pending list scanned per event")
                derived_check["compared"] = same
                derived_check["equal"] = all(abs(dev_d[k] - ora_d[k]) < 1e-12 for k in same)
        if pattern and isinstance(item, qc.Partition) and args.cpu_threads > 0:
            cpu_mt = cpu_baseline_parallel(args.config, app, keys, delta, min(4 * sample, n), args.cpu_threads)

    from siddhi_amd.buildinfo import source_hash
    build_id = source_hash()
    if rank == 0:
        line = {
            "metric": "events/sec ingested + matches/sec (partitioned pattern, 1\u20138 GPU); % HBM peak",
            "value": round(value, 1),
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded SplitMix64 StockStream, BASELINE.md)",
            "build": build_id,
            "config": {"workload": args.config, "events_per_gpu": n,
                       ("keys_total" if mode in ("roundrobin", "slices") else "keys_per_gpu"): keys,
                       "delta_ms": delta, "micro_batch": batch, "call_size": 1024,
                       "parallelism": ("time-sliced x%d" if mode == "slices" else "key-sharded x%d") % world,
                       "input": mode + {"roundrobin": " (RCCL all-to-all re-route)",
                                        "slices": " (one global stream; RCCL send/recv of a %d-event halo per "
                                                  "rank and step)" % M["halo"]}.get(mode, "")},
            "matches_per_s": round(matches_per_s, 1),
            "counters": {k: counters[k] for k in ("events", "matches", "partials", "partial_scans", "carry")},
            "derived": {k: round(v, 4) for k, v in derived.items()},
            "stage_ms_per_step": {k: round(v / 1e6, 3) for k, v in stages.items()},
            "roofline": roof,
            "cpu_baseline": cpu,
            "cpu_baseline_parallel": cpu_mt,
            "parity_prefix": prefix,
            "derived_check": derived_check,
        }
        if alongside:
            line["alongside"] = alongside
        print(json.dumps(line))
    dq.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
