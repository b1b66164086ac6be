"""Flag vector-memory accesses whose address derives from the kernarg segment pointer.

Vector loads from the kernarg segment fault on the MI355X pool (DESIGN.md,
"kernel arguments"); kernels must read argument blocks through a device
pointer instead.  Linear (control-flow-insensitive) scan of hipcc -S output.
"""
import re
import sys


def regs(tok):
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.fullmatch(r"s(\d+)", tok)
    return [int(m.group(1))] if m else []


def scan(path):
    bad = []
    kern = None
    tainted = set()
    for ln, line in enumerate(open(path), 1):
        if re.match(r"^_Z\w+:", line):
            kern = line.split(":")[0]
            tainted = {0, 1}
            continue
        if kern is None:
            continue
        parts = line.strip().split(None, 1)
        if not parts or parts[0].startswith((".", ";")):
            continue
        op = parts[0]
        args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
        srcs = set()
        for a in args[1:]:
            srcs.update(regs(a.split()[0]) if a else [])
        if op.startswith(("global_", "flat_", "buffer_")):
            for a in args:
                r = regs(a.split()[0]) if a else []
                if r and set(r) & tainted:
                    bad.append((kern, ln, line.strip()))
            continue
        if op.startswith("v_") and set(srcs) & tainted and "lshl_add_u64" in op:
            bad.append((kern, ln, line.strip()))
        # VOP3b forms (v_mad_u64_u32, v_*_co_*) also write an SGPR carry-out as operand 1
        if len(args) > 1 and (op.startswith(("v_mad_u64_u32", "v_mad_i64_i32")) or "_co_" in op or op.endswith("_co")):
            tainted.difference_update(regs(args[1].split()[0]))
        if args:
            dst = regs(args[0])
            if dst:
                if op.startswith(("s_add_u32", "s_addc_u32", "s_mov_b64", "s_mov_b32")) and srcs & tainted:
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
