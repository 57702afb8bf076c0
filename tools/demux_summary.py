#!/usr/bin/env python3
"""Per-kernel summary of a tools/demux_prof.sh run: each demux call of the trace (a k_dm_flags_prep and
the kernels after it, the fill before it), grouped by the number of non-empty radix passes (C3: 2,
64 connections: 3), with the median duration per kernel and, from the FETCH_SIZE / WRITE_SIZE passes,
the median HBM bytes per launch (FETCH x2 and KiB x1024, as tools/pmc_traffic.py).
    python tools/demux_summary.py gpurun_out/r05dmf [--out profiles/r05_demux_kernels_c3.json]"""
import argparse
import collections
import csv
import json
import os
import statistics


def name(s):
    s = s.replace("void ", "").replace("(anonymous namespace)::", "")
    return s.split("(")[0].split("<")[0]


def calls(rows, key_start, key_end, val):
    """Split rows (sorted by start) into demux calls; yields lists of (kernel, value)."""
    out, cur = [], None
    for i, r in enumerate(rows):
        k = name(r["Kernel_Name"])
        if k == "k_dm_flags_prep":
            cur = []
            out.append(cur)
            if i and name(rows[i - 1]["Kernel_Name"]).startswith("__amd_rocclr_fill"):
                cur.append(("fill", val(rows[i - 1])))
        if cur is not None and k.startswith("k_dm"):
            cur.append((k, val(r)))
    return out


def group(cs, durs):
    """Label each call's kernels (repeats numbered) and group by the number of non-empty onesweeps."""
    g = collections.defaultdict(lambda: collections.defaultdict(list))
    for c, d in zip(cs, durs):
        passes = sum(1 for k, v in d if k == "k_dm_onesweep" and v > 8.0)
        seen = collections.Counter()
        for k, v in c:
            g[passes][f"{k}#{seen[k]}" if seen[k] else k].append(v)
            seen[k] += 1
    return {p: {k: statistics.median(v) for k, v in m.items()} for p, m in g.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    kt = sorted(csv.DictReader(open(os.path.join(a.dir, "kt", "kt_kernel_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0  # noqa: E731
    kc = calls(kt, 0, 0, dur)
    res = {"source": a.dir, "calls": len(kc), "us": {str(p): {k: round(v, 1) for k, v in m.items()}
                                                       for p, m in group(kc, kc).items()}}
    for cnt, fn, scale in (("FETCH_SIZE", "pmc_fetch", 2.0), ("WRITE_SIZE", "pmc_write", 1.0)):
        path = os.path.join(a.dir, fn, "pmc_counter_collection.csv")
        if not os.path.exists(path):
            continue
        by = collections.defaultdict(float)
        meta = {}
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == cnt:
                by[r["Dispatch_Id"]] += float(r["Counter_Value"])
                meta[r["Dispatch_Id"]] = r
        rows = sorted(meta.values(), key=lambda r: int(r["Start_Timestamp"]))
        pc = calls(rows, 0, 0, lambda r: by[r["Dispatch_Id"]] * 1024.0 * scale / 1e6)
        # group PMC calls by the kernel-trace call shapes (same command, same order of calls)
        shapes = [d for d in kc][: len(pc)]
        res[f"{cnt}_MB"] = {str(p): {k: round(v, 2) for k, v in m.items()} for p, m in group(pc, shapes).items()}
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
