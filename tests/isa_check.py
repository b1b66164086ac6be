"""Flag vector-memory accesses whose address derives from the kernarg segment pointer.

Vector loads from the kernarg segment fault on the MI355X pool (DESIGN.md,
"kernel arguments"); kernels must read argument blocks through a device
pointer instead.  Linear (control-flow-insensitive) scan of hipcc -S output:
taint starts at s[0:1] (the kernarg segment pointer), flows through scalar
copies/adds into SGPRs and through v_mov / v_lshl_add_u64 into VGPRs; any
global_/flat_/buffer_ access whose address operands are tainted is reported.
"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"([sv])\[(\d+):(\d+)\]", tok)
    if m:
        return [(m.group(1), r) for r in range(int(m.group(2)), int(m.group(3)) + 1)]
    m = re.fullmatch(r"([sv])(\d+)", tok)
    return [(m.group(1), int(m.group(2)))] if m else []


def scan(path):
    bad = []
    kern = None
    tainted = set()
    for ln, line in enumerate(open(path), 1):
        if re.match(r"^_Z\w+:", line):
            kern = line.split(":")[0]
            tainted = {("s", 0), ("s", 1)}
            continue
        if kern is None:
            continue
        parts = line.strip().split(None, 1)
        if not parts or parts[0].startswith((".", ";")):
            continue
        op = parts[0]
        args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
        toks = [regs(a.split()[0]) if a else [] for a in args]
        srcs = set(r for t in toks[1:] for r in t)
        if op.startswith(("global_", "flat_", "buffer_")):
            # address operands: everything except the data register of a store / the dst of a load
            addr = set(r for t in (toks[1:] if "load" in op or "atomic" in op else toks[:1] + toks[2:]) for r in t)
            if "store" in op:
                addr = set(r for t in toks[:1] + toks[2:] for r in t)
            if addr & tainted:
                bad.append((kern, ln, line.strip()))
            if "load" in op and toks:
                tainted.difference_update(toks[0])
            continue
        # VOP3b forms (v_mad_u64_u32, v_*_co_*) also write an SGPR carry-out as operand 1
        if len(toks) > 1 and (op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")) or "_co_" in op or op.endswith("_co")):
            tainted.difference_update(toks[1])
            srcs = set(r for t in toks[2:] for r in t)
        if not toks:
            continue
        dst = toks[0]
        if not dst:
            continue
        propagates = (op.startswith(("s_add_u32", "s_addc_u32", "s_mov_b64", "s_mov_b32", "s_add_i32",
                                     "v_mov_b32", "v_mov_b64", "v_lshl_add_u64", "v_add_co_u32", "v_addc_co_u32",
                                     "v_add_u32", "v_add_nc_u32", "v_cndmask_b32", "v_readfirstlane_b32"))
                      and bool(srcs & tainted))
        if propagates:
            tainted.update(dst)
        else:
            tainted.difference_update(dst)
    return bad


if __name__ == "__main__":
    n = 0
    for p in sys.argv[1:]:
        for k, ln, l in scan(p):
            print("%s:%d %s  [%s]" % (p, ln, l, k[:60]))
            n += 1
    sys.exit(1 if n else 0)
