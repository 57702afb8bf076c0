#!/usr/bin/env python3
"""Runs tools/libhbm_probe.so kernels over a large buffer and prints achieved GB/s per pattern
(bytes counted: read + write).  python tools/hbm_probe.py [--gib 6] [--grids 2048,8192,65536]"""
import argparse
import ctypes
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=6.0)
    ap.add_argument("--grids", default="2048,8192,65536")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tiles", default="1024,16384,92160,1048576")
    args = ap.parse_args()
    L = ctypes.CDLL(os.path.join(HERE, "libhbm_probe.so"))
    L.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    nbytes = int(args.gib * 2**30) // 4096 * 4096
    src = torch.randint(0, 255, (nbytes + 4096,), dtype=torch.uint8, device="cuda")
    dst = torch.empty(nbytes + 4096, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    names = ["copy16", "read16", "write16", "shift2ld", "shiftdpp"]
    moved = {0: 2, 1: 1, 2: 1, 3: 2, 4: 2}
    res = {}
    for g in [int(x) for x in args.grids.split(",")]:
        for k, nm in enumerate(names):
            assert L.probe_run(k, src.data_ptr(), dst.data_ptr(), nbytes, g, s.cuda_stream) == 0
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                L.probe_run(k, src.data_ptr(), dst.data_ptr(), nbytes, g, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            res[f"{nm}@{g}"] = round(moved[k] * nbytes / (ms * 1e-3) / 1e9, 1)
    L.probe_tile.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                             ctypes.c_void_p]
    for unroll in (1, 4):
        for tile in [int(x) for x in args.tiles.split(",")]:
            L.probe_tile(unroll, src.data_ptr(), dst.data_ptr(), nbytes, tile, s.cuda_stream)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                L.probe_tile(unroll, src.data_ptr(), dst.data_ptr(), nbytes, tile, s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            res[f"tilecopy_u{unroll}@{tile}"] = round(2 * nbytes / (ms * 1e-3) / 1e9, 1)
    # check shiftdpp == shift2ld output on a prefix
    L.probe_run(3, src.data_ptr(), dst.data_ptr(), 1 << 20, 256, s.cuda_stream)
    a = dst[: (1 << 20) - 64 * 16].clone()
    L.probe_run(4, src.data_ptr(), dst.data_ptr(), 1 << 20, 256, s.cuda_stream)
    torch.cuda.synchronize()
    res["dpp_matches_2ld"] = bool(torch.equal(a[: (1 << 20) - 128 * 16], dst[: (1 << 20) - 128 * 16]))
    print(json.dumps({"GBps": res, "bytes": nbytes}))


if __name__ == "__main__":
    main()
