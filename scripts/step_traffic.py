#!/usr/bin/env python3
"""HBM bytes per pipelined step from two rocprofv3 --pmc passes of the same
bench command (FETCH_SIZE, WRITE_SIZE): every dispatch except the bench's own
setup kernels (synth, verify, stream ceiling) is summed and divided by the
number of k_unmask dispatches (one per step).  Read bytes = 2 x FETCH_SIZE x
1024 (gfx950: FETCH_SIZE counts half of a 16-B/lane streaming read, the
access of k_unmask and k_sieve_count, MI355X_MICROARCH.md HBM section),
write bytes = WRITE_SIZE x 1024.

  scripts/step_traffic.py FETCH_DIR WRITE_DIR --alg-bytes N [--out FILE]
      [--steps-by k_unmask_run --drop k_unmask<,k_walk,...]

--steps-by counts steps by the dispatches of one unmask kernel (a RUN run's
first steps take the exact path); --drop leaves out the kernels of those
other steps (name prefixes).
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

SETUP = ("k_synth", "k_stream_xor", "k_digest", "k_frame_sizes")   # the bench's own setup and checks


def load(d, counter, steps_by="k_unmask", drop=()):
    per = defaultdict(float)
    n_unmask = 0
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("hvws::", "")
            if name.startswith(steps_by):
                n_unmask += 1
            if any(s in name for s in SETUP) or any(name.startswith(p) for p in drop):
                continue
            per[name] += float(r["Counter_Value"])
    return per, n_unmask


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--alg-bytes", type=float, required=True)
    ap.add_argument("--out")
    ap.add_argument("--steps-by", default="k_unmask")
    ap.add_argument("--drop", default="", help="comma-separated kernel name prefixes left out")
    a = ap.parse_args()
    drop = tuple(x for x in a.drop.split(",") if x)
    fe, nu_f = load(a.fetch_dir, "FETCH_SIZE", a.steps_by, drop)
    wr, nu_w = load(a.write_dir, "WRITE_SIZE", a.steps_by, drop)
    steps = max(nu_f, 1)
    rd = {k: 2 * v * 1024 / steps for k, v in fe.items()}
    wb = {k: v * 1024 / max(nu_w, 1) for k, v in wr.items()}
    tot = sum(rd.values()) + sum(wb.values())
    out = {"steps": steps, "read_bytes_per_step": sum(rd.values()), "write_bytes_per_step": sum(wb.values()),
           "bytes_per_step": tot, "alg_bytes_per_step": a.alg_bytes, "ratio": tot / a.alg_bytes,
           "per_kernel_GB": {k: round((rd.get(k, 0) + wb.get(k, 0)) / 1e9, 4)
                             for k in sorted(set(rd) | set(wb), key=lambda k: -(rd.get(k, 0) + wb.get(k, 0)))}}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
