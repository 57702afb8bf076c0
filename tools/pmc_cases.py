#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from rocprofv3 --pmc runs laid out as
<dir>/pmc_<case>_FETCH_SIZE and <dir>/pmc_<case>_WRITE_SIZE (tools/_box scripts: one pass per
counter, MI355X_MICROARCH.md §HBM: FETCH_SIZE x2 for wide coalesced streams, KiB x1024).
    python tools/pmc_cases.py gpurun_out/r03d --kernel k_encode< --algorithmic 1528521696"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_encode<")
    ap.add_argument("--algorithmic", type=float, default=0.0)
    a = ap.parse_args()
    res = {}
    for d in sorted(glob.glob(os.path.join(a.dir, "pmc_*_FETCH_SIZE"))):
        case = os.path.basename(d)[4:-len("_FETCH_SIZE")]
        v = {}
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            f = os.path.join(a.dir, f"pmc_{case}_{ctr}", "pmc_counter_collection.csv")
            vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
                    if r["Counter_Name"] == ctr and a.kernel in r["Kernel_Name"]]
            v[ctr] = statistics.median(vals) if vals else float("nan")
        rd, wr = 2.0 * v["FETCH_SIZE"] * 1024.0, v["WRITE_SIZE"] * 1024.0
        rec = {"read_bytes": rd, "write_bytes": wr, "bytes": rd + wr}
        if a.algorithmic:
            rec["ratio_to_algorithmic"] = round((rd + wr) / a.algorithmic, 4)
        res[case] = rec
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
