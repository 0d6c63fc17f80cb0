"""Summarise a rocprofv3 rocpd database (`--kernel-trace --stats` without a csv format).

Prints markdown: per-kernel stats (calls, total, avg, share, min, max) over all
dispatches, and per-(kernel, grid) rows for the kernels named on the command line.

    python scripts/rocpd_stats.py gpurun_out/r1H/prof k_unmask k_build k_stream_xor
"""
import glob
import os
import sqlite3
import sys


def short(name: str) -> str:
    """`void hvws::k_unmask<256, 4, true>(unsigned char*, ...)` -> `k_unmask<256, 4, true>`"""
    name = name.split("(")[0]
    if name.startswith("void "):
        name = name[5:]
    return name.replace("hvws::", "")


def main() -> None:
    root = sys.argv[1]
    focus = sys.argv[2:]
    dbs = [root] if root.endswith(".db") else glob.glob(os.path.join(root, "**", "*.db"), recursive=True)
    rows = []
    for db in dbs:
        c = sqlite3.connect(db)
        rows += [(short(n), g, d) for n, g, d in
                 c.execute("select name, grid_x * grid_y * grid_z, duration from kernels")]
    per = {}
    for name, grid, dur in rows:
        per.setdefault(name, []).append(dur / 1000.0)
    total = sum(sum(v) for v in per.values())
    print("| kernel | calls | total ms | avg us | % | min us | max us |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        print(f"| `{name}` | {len(v)} | {s / 1000:.3f} | {s / len(v):.1f} | {100 * s / total:.1f} | "
              f"{min(v):.1f} | {max(v):.1f} |")
    if not focus:
        return
    grids = {}
    for name, grid, dur in rows:
        if any(name.startswith(f) for f in focus):
            grids.setdefault((name, grid), []).append(dur / 1000.0)
    print()
    print("| kernel | grid (work-items) | dispatches | avg us | min us | max us |")
    print("|---|---:|---:|---:|---:|---:|")
    for (name, grid), v in sorted(grids.items(), key=lambda kv: (-kv[0][1], kv[0][0])):
        if sum(v) / len(v) < 1000:   # only the batch-sized grids
            continue
        print(f"| `{name}` | {grid} | {len(v)} | {sum(v) / len(v):.1f} | {min(v):.1f} | {max(v):.1f} |")


if __name__ == "__main__":
    main()
