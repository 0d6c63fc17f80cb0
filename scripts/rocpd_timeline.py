"""Print a rocpd kernel timeline (start/end relative to the first kernel of
interest, in us) to see what sits between consecutive dispatches of a kernel.

    python scripts/rocpd_timeline.py gpurun_out/r5p_kt_g4 k_unmask_run 6
(the 6 steps after the first 10 dispatches of the named kernel)
"""
import glob
import os
import sqlite3
import sys

from rocpd_stats import short


def main() -> None:
    root, key = sys.argv[1], sys.argv[2]
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    dbs = [root] if root.endswith(".db") else glob.glob(os.path.join(root, "**", "*.db"), recursive=True)
    rows = []
    for db in dbs:
        c = sqlite3.connect(db)
        rows += [(s, e, short(n), q) for s, e, n, q in c.execute("select start, end, name, queue_id from kernels")]
    rows.sort()
    idx = [i for i, r in enumerate(rows) if r[2].startswith(key)]
    if len(idx) < 12:
        print("too few dispatches of", key)
        return
    a, b = idx[10], idx[min(10 + nsteps, len(idx) - 1)]
    t0 = rows[a][0]
    for s, e, n, q in rows[a:b + 1]:
        print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:7.1f}  q{q}  {n}")


if __name__ == "__main__":
    main()
