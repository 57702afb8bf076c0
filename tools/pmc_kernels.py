#!/usr/bin/env python3
"""Median counter value per kernel (short name) from the rocprofv3 --pmc passes of a tools/*_pmc.sh run,
and the kernel-trace mean duration.  FETCH_SIZE x2 and KiB x1024 (MI355X_MICROARCH.md §HBM).
    python tools/pmc_kernels.py gpurun_out/r06k [--match k_wire,k_encode]"""
import argparse
import collections
import csv
import glob
import json
import os
import statistics


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--match", default="k_")
    a = ap.parse_args()
    keep = a.match.split(",")
    out = collections.defaultdict(dict)
    kt = glob.glob(os.path.join(a.dir, "kt", "*kernel_stats.csv"))
    if kt:
        for r in csv.DictReader(open(kt[0])):
            k = short(r["Name"])
            if any(m in k for m in keep):
                out[k]["us_mean"] = round(float(r["AverageNs"]) / 1e3, 2)
    for f in glob.glob(os.path.join(a.dir, "pmc_*", "pmc_counter_collection.csv")):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if any(m in k for m in keep):
                vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            x = statistics.median(v)
            if c == "FETCH_SIZE":
                x = round(2 * x * 1024 / 1e6, 2)
                c = "FETCH_MB"
            elif c == "WRITE_SIZE":
                x = round(x * 1024 / 1e6, 2)
                c = "WRITE_MB"
            out[k][c] = x
    for k, d in out.items():
        if d.get("SQ_WAVES"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM"):
                if c in d:
                    d[c + "_per_wave"] = round(d[c] / d["SQ_WAVES"], 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
