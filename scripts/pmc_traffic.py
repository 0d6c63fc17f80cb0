#!/usr/bin/env python3
"""Per-launch HBM traffic of each kernel from two separate rocprofv3 --pmc
passes (FETCH_SIZE, WRITE_SIZE), corrected as MI355X_MICROARCH.md's HBM
section prescribes: both counters are in KiB; on gfx950 FETCH_SIZE counts
exactly half of the bytes of a 16-B-per-lane coalesced streaming read, so
read bytes = 2 x FETCH_SIZE x 1024, write bytes = WRITE_SIZE x 1024.

  scripts/pmc_traffic.py FETCH_DIR WRITE_DIR --rx-bytes N --config NAME [--out profiles/traffic.json]
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict


def load(d, counter):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter:
                    out[r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hvws::", "")].append(
                        float(r["Counter_Value"]))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--rx-bytes", type=int, required=True)
    ap.add_argument("--config", required=True)
    ap.add_argument("--out", default="profiles/traffic.json")
    a = ap.parse_args()
    fetch, write = load(a.fetch_dir, "FETCH_SIZE"), load(a.write_dir, "WRITE_SIZE")
    db = json.load(open(a.out)) if os.path.exists(a.out) else {}
    for k in sorted(set(fetch) & set(write)):
        if not (k.startswith("k_unmask") or k.startswith("k_stream_xor") or k.startswith("k_build")):
            continue
        # a launch split in two (grids past 2^32 work-items) leaves a tail
        # dispatch of a few tiles: medians over the whole-batch dispatches
        fw = [v for v in write[k] if v >= 0.1 * max(write[k])]
        ff = [v for v, w in zip(fetch[k], write[k]) if w >= 0.1 * max(write[k])] if len(fetch[k]) == len(write[k]) \
            else [v for v in fetch[k] if v >= 0.1 * max(fetch[k])]
        rd = 2 * statistics.median(ff) * 1024
        wr = statistics.median(fw) * 1024
        name = k.replace(" ", "")
        if name.startswith("k_build<"):   # hvws_last_build_kernel spelling: k_build<TxU> / <TxU,lean>
            parts = name[len("k_build<"):-1].split(",")
            if len(parts) == 6:
                name = f"k_build<{parts[0]}x{parts[1]}" + {"2": ",lean", "0": ",wide"}.get(parts[5], "") + ">"
        elif name.startswith("k_unmask_run<"):   # hvws_run_kernel_name spelling: <T,U> / <T,U,lds>
            parts = name[len("k_unmask_run<"):-1].split(",")
            name = "k_unmask_run<" + ",".join(parts[:2]) + (",lds" if parts[2:] == ["true"] else "") + ">"
        elif not name.startswith("k_build"):   # hvws_unmask_kernel_name spelling
            name = name.replace("true", "xcd").replace("false", "linear")
        db.setdefault(name, {})[str(a.rx_bytes)] = {
            "config": a.config, "read_bytes": int(rd), "write_bytes": int(wr), "hbm_bytes": int(rd + wr),
            "dispatches": len(fw),
            "method": "median per dispatch; read = 2 x FETCH_SIZE x 1024 (gfx950 16-B/lane correction), "
                      "write = WRITE_SIZE x 1024; separate --pmc passes",
        }
        print(name, a.rx_bytes, int(rd + wr))
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(db, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
