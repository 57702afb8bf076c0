#!/usr/bin/env python3
"""Summarise tools/pmc_encode_paths.sh: per variant and kernel, the median FETCH_SIZE / WRITE_SIZE per
launch (KiB x 1024; raw -- not the x2 streaming correction, which does not hold for scattered 64-B reads),
and the encode's total per call summed over its kernels (the reference launch of path 1 excluded).
    python tools/pmc_encode_paths.py gpurun_out/r05g --algorithmic 12020875264"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--algorithmic", type=float, default=0.0)
    a = ap.parse_args()
    out = {}
    for d in sorted(glob.glob(os.path.join(a.dir, "pmc_*_FETCH_SIZE"))):
        case = os.path.basename(d)[4:-len("_FETCH_SIZE")]
        rec = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            f = glob.glob(os.path.join(a.dir, f"pmc_{case}_{ctr}", "**", "*counter_collection.csv"), recursive=True)
            by = {}
            for fn in f:
                for r in csv.DictReader(open(fn)):
                    if r["Counter_Name"] == ctr and "k_encode" in r["Kernel_Name"]:
                        k = r["Kernel_Name"].split("(")[0]
                        by.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0)
            for k, vals in by.items():
                rec.setdefault(k, {})[ctr] = {"median_bytes": statistics.median(vals), "launches": len(vals)}
        tot = {"FETCH_SIZE": 0.0, "WRITE_SIZE": 0.0}
        for k, v in rec.items():
            if "k_encode<" in k:
                continue  # the path-1 reference launch of enc_paths_ab.py (the per-set kernel)
            for ctr in tot:
                tot[ctr] += v.get(ctr, {}).get("median_bytes", 0.0)
        rec["encode_total_raw"] = tot
        if a.algorithmic:
            rec["encode_total_raw"]["raw_sum_over_algorithmic"] = round(
                (tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / a.algorithmic, 4)
        out[case] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
