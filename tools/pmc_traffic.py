#!/usr/bin/env python3
"""Turns rocprofv3 --pmc CSVs (FETCH_SIZE and WRITE_SIZE, collected in separate passes by
tools/profile_box.sh) into per-launch HBM bytes for a kernel, with the gfx950 corrections of
MI355X_MICROARCH.md §HBM: both counters are in KiB; FETCH_SIZE reads half the bytes of a wide
coalesced stream, so it is doubled (the kernel's dominant reads are 16-B/lane streams); WRITE_SIZE
is exact for 16-B/lane stores.
    python tools/pmc_traffic.py gpurun_out/r01 --kernel k_encode --config c3 --packets 4194304 --frame-pitch 1440 \
        [--out profiles/traffic.json]
"""
import argparse
import csv
import json
import os
import statistics


def base_name(k):
    return k.split("(")[0].split("<")[0].strip()


def per_launch(path, kernel, counter):
    """Median per launch of each kernel named in `kernel` (comma list of names, template and argument
    lists ignored), summed over them: the encode step is one kernel (k_encode) or two
    (k_encode_heads,k_encode_copy: the two-pass form)."""
    names = set(kernel.split(","))
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter and base_name(r["Kernel_Name"]) in names:
            vals.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return sum(statistics.median(v) for v in vals.values()), {k: len(v) for k, v in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="k_encode", help="kernel name, or a comma list summed per launch")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--packets", type=int, default=4194304)
    ap.add_argument("--algorithmic", type=float, default=0.0, help="algorithmic bytes per launch")
    ap.add_argument("--frame-pitch", type=int, required=True, help="frame slot pitch of the profiled run")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    f, nf = per_launch(os.path.join(a.dir, "pmc_fetch", "pmc_counter_collection.csv"), a.kernel, "FETCH_SIZE")
    w, nw = per_launch(os.path.join(a.dir, "pmc_write", "pmc_counter_collection.csv"), a.kernel, "WRITE_SIZE")
    read_b = 2.0 * f * 1024.0
    write_b = w * 1024.0
    rec = {
        "kernel": a.kernel, "config": a.config, "packets": a.packets, "frame_pitch": a.frame_pitch,
        "fetch_size_kib_raw": f, "write_size_kib_raw": w, "launches": [nf, nw],
        "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
        "bytes_per_launch": read_b + write_b,
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE separate passes ({a.dir}); FETCH x2 (gfx950), KiB x1024",
    }
    if a.algorithmic:
        rec["ratio_to_algorithmic"] = round((read_b + write_b) / a.algorithmic, 4)
    s = json.dumps(rec, indent=1)
    print(s)
    if a.out:
        # one record per (config, packets): profiles/traffic.json maps "c3:4194304" -> record
        table = {}
        if os.path.exists(a.out):
            old = json.load(open(a.out))
            table = {f"{old['config']}:{old['packets']}": old} if "config" in old else old
        table[f"{a.config}:{a.packets}"] = rec
        open(a.out, "w").write(json.dumps(table, indent=1) + "\n")


if __name__ == "__main__":
    main()
