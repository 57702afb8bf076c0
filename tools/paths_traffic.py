#!/usr/bin/env python3
"""Per-kernel HBM traffic from tools/paths_pmc.sh's two PMC passes: median FETCH_SIZE (x2, gfx950)
and WRITE_SIZE (both KiB) per dispatch, in bytes per launch and per packet.
    python tools/paths_traffic.py gpurun_out/ppmc --packets 4194304 [--out profiles/r01_paths_traffic_c3.json]"""
import argparse
import csv
import json
import os
import re
import statistics


def load(path, counter):
    d = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = re.sub(r"^.*::", "", r["Kernel_Name"].split("(")[0]).strip()
        d.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--packets", type=int, default=4194304)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    f = load(os.path.join(a.dir, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    w = load(os.path.join(a.dir, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    rows = {}
    for k in sorted(set(f) & set(w)):
        rd, wr = 2.0 * statistics.median(f[k]), statistics.median(w[k])
        if rd + wr < 1e6:
            continue
        rows[k] = {"dispatches": len(f[k]), "read_bytes_x2": rd, "write_bytes": wr,
                   "read_B_per_pkt_raw": round(rd / 2 / a.packets, 1), "read_B_per_pkt_x2": round(rd / a.packets, 1),
                   "write_B_per_pkt": round(wr / a.packets, 1)}
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes ({a.dir}), median per dispatch",
           "note": "FETCH_SIZE counts 64 B per memory read request. Wide streaming reads are issued as 128-B "
                   "requests, so the x2 figure is the byte count for streaming kernels (encode, wire, "
                   "tcpinfo). Scattered header reads (decode, parse, filter, syncinput) are fetched as 64-B "
                   "sectors (the filter's 80-B windows cost 2.8 requests per packet), so raw is their byte "
                   "count. Kernel names are truncated (-T): k_encode_wire mixes the flat half and A/B "
                   "variants; k_encode_wire_w4 is the default per-packet half (RAW4 and Ethernet).",
           "packets": a.packets, "kernels": rows}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        open(a.out, "w").write(s + "\n")


if __name__ == "__main__":
    main()
