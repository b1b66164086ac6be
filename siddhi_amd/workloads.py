"""Seeded synthetic StockStream workloads of BASELINE.md / SURVEY.md §8d.

    define stream StockStream (symbol string, price double, volume long);

SplitMix64 (seed 20261015 + per-config offset); symbol uniform over K keys
(dictionary ids 0..K-1, string "S%07d"); price = 50 + 50*U[0,1); volume
uniform in [1, 1000]; ts = T0 + floor(i * delta) ms; InputHandler calls of
1024 events.
"""
from __future__ import annotations

import numpy as np

SEED = 20261015
T0 = 1_700_000_000_000
STOCK_DEF = "define stream StockStream (symbol string, price double, volume long);"

P1_QUERY = ("@info(name='q') from every e1=StockStream[price>70] -> "
            "e2=StockStream[symbol==e1.symbol and price>e1.price*1.05] within 1 sec "
            "select e1.symbol as symbol, e1.price as p1, e2.price as p2 insert into Alert;")

P1_APP = "@app:playback " + STOCK_DEF + " " + P1_QUERY
P3_APP = ("@app:playback " + STOCK_DEF + " partition with (symbol of StockStream) begin " + P1_QUERY + " end;")
W2_LENGTH_APP = ("@app:playback " + STOCK_DEF + " @info(name='q') from StockStream[price>60]#window.length(1000) "
                 "select symbol, avg(price) as a, sum(price) as s, count() as c group by symbol insert into O1;")
W2_TIME_APP = ("@app:playback " + STOCK_DEF + " @info(name='q') from StockStream[price>60]#window.time(10 sec) "
               "select symbol, avg(price) as a, sum(price) as s, count() as c group by symbol insert into O2;")

# config S4: counting sequence with e2[last], logical and/or,
# absent `not ... for`
S4_SEQ_QUERY = ("@info(name='q') from every e1=StockStream, e2=StockStream[price>e1.price]<2:5>, "
                "e3=StockStream[price<e2[last].price] "
                "select e1.price as p1, e2[0].price as p2a, e2[last].price as p2z, e3.price as p3 insert into O;")
# S4-seq's `<2:5>` is the config text; a SEQUENCE count state is re-added only
# at count >= min (CountPostStateProcessor.java:49-57), so `<2:5>` dies at the
# next event's resetAndUpdate and emits nothing on this stream.  `<1:4>` is
# the measured variant that emits rows (same engine, same lane machine).
S4_SEQ14_QUERY = S4_SEQ_QUERY.replace("<2:5>", "<1:4>")
S4_SEQPLUS_QUERY = ("@info(name='q') from every e1=StockStream, e2=StockStream[price>e1.price]+, "
                    "e3=StockStream[price<e2[last].price] "
                    "select e1.price as p1, e2[0].price as p2a, e2[last].price as p2z, e3.price as p3 insert into O;")
S4_OR_QUERY = ("@info(name='q') from every e1=StockStream[price>70] -> "
               "(e2=StockStream[price>e1.price] or e3=StockStream[price<e1.price*0.9]) "
               "select e1.price as p1, e2.price as p2, e3.price as p3 insert into O;")
S4_AND_QUERY = ("@info(name='q') from every e1=StockStream[price>70] -> "
                "e2=StockStream[price>e1.price*1.2] and e3=StockStream[price<e1.price*0.8] within 1 sec "
                "select e1.price as p1, e2.price as p2, e3.price as p3 insert into O;")
S4_NOT_QUERY = ("@info(name='q') from every e1=StockStream[price>98] -> "
                "not StockStream[price>e1.price] for 1 sec "
                "select e1.symbol as symbol, e1.price as p1 insert into O;")
S4_BARE_QUERY = ("@info(name='q') from e1=StockStream, e2=StockStream[price>e1.price]<2:5>, "
                 "e3=StockStream[price<e2[last].price] "
                 "select e1.price as p1, e2[last].price as p2z, e3.price as p3 insert into O;")
S4_APPS = {k: "@app:playback " + STOCK_DEF + " " + q for k, q in
           (("seq", S4_SEQ_QUERY), ("seq14", S4_SEQ14_QUERY), ("seqplus", S4_SEQPLUS_QUERY), ("or", S4_OR_QUERY),
            ("and", S4_AND_QUERY), ("not", S4_NOT_QUERY), ("bare", S4_BARE_QUERY))}
S4_PART_APPS = {k: "@app:playback " + STOCK_DEF + " partition with (symbol of StockStream) begin " + q + " end;"
                for k, q in (("seq", S4_SEQ_QUERY), ("seqplus", S4_SEQPLUS_QUERY), ("or", S4_OR_QUERY), ("and", S4_AND_QUERY),
                             ("not", S4_NOT_QUERY))}

# config M5: 100 queries on one StockStream junction -- 50
# variants of P1 (e1 threshold 60..84.5, step 0.5) and 50 of W2-length
# (length 100..5000, step 100)
M5_PATTERN_THRESHOLDS = [60.0 + 0.5 * i for i in range(50)]
M5_WINDOW_LENGTHS = [100 * (i + 1) for i in range(50)]


def m5_app(n_pattern: int = 50, n_window: int = 50) -> str:
    qs = []
    for i, th in enumerate(M5_PATTERN_THRESHOLDS[:n_pattern]):
        qs.append("@info(name='p%02d') from every e1=StockStream[price>%s] -> "
                  "e2=StockStream[symbol==e1.symbol and price>e1.price*1.05] within 1 sec "
                  "select e1.symbol as symbol, e1.price as p1, e2.price as p2 insert into AlertP%02d;" % (i, repr(th), i))
    for i, ln in enumerate(M5_WINDOW_LENGTHS[:n_window]):
        qs.append("@info(name='w%02d') from StockStream[price>60]#window.length(%d) "
                  "select symbol, avg(price) as a, sum(price) as s, count() as c group by symbol "
                  "insert into OutW%02d;" % (i, ln, i))
    return "@app:playback " + STOCK_DEF + " " + " ".join(qs)


M5_APP = m5_app()

CONFIGS = {
    # name: (app, n_events, n_keys, delta_ms)
    "P1": (P1_APP, 1_000_000, 1_000, 1.0),
    "W2-length": (W2_LENGTH_APP, 100_000_000, 1_000, 0.1),
    "W2-time": (W2_TIME_APP, 100_000_000, 1_000, 0.1),
    "P3": (P3_APP, 100_000_000, 10_000_000, 0.01),
    "P3-dense": (P3_APP, 100_000_000, 10_000_000, 1e-5),
    "S4-seq": (S4_APPS["seq"], 1_000_000, 1_000, 1.0),
    "S4-seq14": (S4_APPS["seq14"], 1_000_000, 1_000, 1.0),
    "S4-or": (S4_APPS["or"], 1_000_000, 1_000, 1.0),
    "S4-and": (S4_APPS["and"], 1_000_000, 1_000, 1.0),
    "S4-not": (S4_APPS["not"], 1_000_000, 1_000, 1.0),
    "S4-seqplus": (S4_APPS["seqplus"], 1_000_000, 1_000, 1.0),
    "S4P-seqplus": (S4_PART_APPS["seqplus"], 10_000_000, 100_000, 0.01),
    # 1B events in SURVEY.md §8d; the bench default is a bounded 100M-event pass
    "M5": (M5_APP, 100_000_000, 1_000, 0.001),
}


def splitmix64(state: np.uint64, n: int) -> np.ndarray:
    """n successive SplitMix64 outputs starting from `state` (vectorised)."""
    with np.errstate(over="ignore"):
        z = (np.arange(1, n + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)) + np.uint64(state)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def stock_stream(n: int, n_keys: int, delta_ms: float, seed_offset: int = 0, start: int = 0):
    """Columns (symbol u32 ids, price f64, volume i64, ts i64) for events [start, start+n)."""
    base = np.uint64(SEED + seed_offset)
    with np.errstate(over="ignore"):
        st = base + np.uint64(3 * start) * np.uint64(0x9E3779B97F4A7C15)
    r = splitmix64(st, 3 * n).reshape(n, 3)
    symbol = (r[:, 0] % np.uint64(n_keys)).astype(np.uint32)
    price = 50.0 + 50.0 * ((r[:, 1] >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53)))
    volume = (r[:, 2] % np.uint64(1000)).astype(np.int64) + 1
    idx = np.arange(start, start + n, dtype=np.float64)
    ts = (T0 + np.floor(idx * delta_ms)).astype(np.int64)
    return symbol, price, volume, ts


def stock_stream_at(idx: np.ndarray, n_keys: int, delta_ms: float, seed_offset: int = 0):
    """The same columns as stock_stream for an arbitrary set of global event
    indices (the generator is counter based: event g, column j draws output
    3*g + j + 1 of the SplitMix64 sequence)."""
    idx = np.asarray(idx, dtype=np.uint64)
    base = np.uint64(SEED + seed_offset)
    g = np.uint64(0x9E3779B97F4A7C15)
    with np.errstate(over="ignore"):
        cols = []
        for j in range(3):
            z = (np.uint64(3) * idx + np.uint64(j + 1)) * g + base
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            cols.append(z ^ (z >> np.uint64(31)))
    symbol = (cols[0] % np.uint64(n_keys)).astype(np.uint32)
    price = 50.0 + 50.0 * ((cols[1] >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53)))
    volume = (cols[2] % np.uint64(1000)).astype(np.int64) + 1
    ts = (T0 + np.floor(idx.astype(np.float64) * delta_ms)).astype(np.int64)
    return symbol, price, volume, ts


def call_offsets(n: int, call_size: int = 1024) -> np.ndarray:
    offs = np.arange(0, n, call_size, dtype=np.int64)
    return np.append(offs, np.int64(n))


def symbol_name(i: int) -> str:
    return "S%07d" % i


def register_symbols(dictionary, n_keys: int):
    """Make dictionary id i == symbol i (the generator's u32 ids)."""
    for i in range(len(dictionary.strings), n_keys):
        assert dictionary.id(symbol_name(i)) == i
