"""Kernel statistics (calls, total/avg us, %) from a rocprofv3 rocpd SQLite database."""
import glob
import sqlite3
import sys


def stats(db):
    con = sqlite3.connect(db)
    cur = con.cursor()
    tabs = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [t for t in tabs if t.startswith("rocpd_kernel_dispatch")][0]
    ks = [t for t in tabs if t.startswith("rocpd_info_kernel_symbol")][0]
    cols = [r[1] for r in cur.execute("pragma table_info(%s)" % ks)]
    name_col = "kernel_name" if "kernel_name" in cols else ("display_name" if "display_name" in cols else cols[1])
    rows = cur.execute("select s.%s, count(*), sum(d.end - d.start) from %s d join %s s on d.kernel_id = s.id "
                       "group by s.%s" % (name_col, kd, ks, name_col)).fetchall()
    tot = sum(r[2] for r in rows) or 1
    out = []
    for name, n, t in sorted(rows, key=lambda r: -r[2]):
        out.append((name, n, t / 1e3, t / 1e3 / n, 100.0 * t / tot))
    return out


if __name__ == "__main__":
    db = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
    if not db.endswith(".db"):   # a directory: its (first) database
        db = sorted(glob.glob(db + "/**/*.db", recursive=True))[0]
    print("kernel,calls,total_us,avg_us,percent")
    for name, n, t, a, pc in stats(db):
        print('"%s",%d,%.3f,%.3f,%.3f' % (name, n, t, a, pc))
