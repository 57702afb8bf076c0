#!/usr/bin/env python3
"""C4's encode ceiling, device-resident, HIP events, one process:
  gather   every 16-B chunk the C4 encode writes (frames in 1536-B slots up to their PAD128 end) copied
           from the payload chunk whose bytes land there, as ONE grid-stride gather over a precomputed
           chunk list (plain aligned loads / stores, no funnel, header or MD5: wrong bytes; the list's 2 x 4 B
           per chunk are extra reads, reported separately)
  dense    a contiguous copy of the same number of 16-B chunks (no slots at all)
  encode   rsk_encode_batch on the same batch, per path (1 = per-set kernel, 2:k = two-pass, k packets per copy wave)
Rates are the encode's algorithmic bytes (2P + 66 per packet) over each time, so the rows compare directly.
    python tools/c4_ceiling.py [--packets 1048576] [--reps 20] [--grids 8192,65536]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--grids", default="8192,32768,131072")
    ap.add_argument("--paths", default="1,2:1,2:2,2:4")
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = args.packets or workload.CONFIGS["c4"][1]
    d = workload.describe("c4", 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    P = d.pay_len.astype(np.int64)
    fo = d.frame_off.astype(np.int64)
    po = d.pay_off.astype(np.int64)
    nst = ((31 + P + 127) // 128 * 128) // 16  # frame chunks to the PAD128 end (slots are 128-B aligned)
    assert (fo % 16 == 0).all()
    tot = int(nst.sum())
    pk = np.repeat(np.arange(n), nst)
    k = np.arange(tot) - np.repeat(np.cumsum(nst) - nst, nst)
    didx = (fo[pk] // 16 + k).astype(np.uint32)
    sidx = np.where(k >= 2, (po[pk] + 16 * (k - 2)) // 16, po[pk] // 16)
    sidx = np.minimum(sidx, (po[pk] + np.maximum(P[pk] - 1, 0)) // 16).astype(np.uint32)
    alg = int((2 * P + 66).sum())
    L = ctypes.CDLL(os.path.join(HERE, "libhbm_probe.so"))
    L.probe_gather.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    L.probe_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
    di, si = torch.from_numpy(didx).to(dev), torch.from_numpy(sidx).to(dev)
    s = torch.cuda.current_stream()
    dense_src = torch.empty(16 * tot, dtype=torch.uint8, device=dev)
    dense_dst = torch.empty(16 * tot, dtype=torch.uint8, device=dev)

    def timeit(fn):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.reps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps

    out = {"config": "c4", "packets": n, "chunks_written": tot, "algorithmic_bytes": alg,
           "list_bytes": 8 * tot, "rows": {}}
    for g in [int(x) for x in args.grids.split(",")]:
        ms = timeit(lambda: L.probe_gather(w.payload.data_ptr(), w.frame.data_ptr(), di.data_ptr(), si.data_ptr(),
                                           tot, g, s.cuda_stream))
        out["rows"][f"gather@{g}"] = {"ms": round(ms, 4), "alg_TBs": round(alg / ms / 1e9, 3),
                                      "with_list_TBs": round((alg + 8 * tot) / ms / 1e9, 3)}
        ms = timeit(lambda: L.probe_run(0, dense_src.data_ptr(), dense_dst.data_ptr(), 16 * tot, g, s.cuda_stream))
        out["rows"][f"dense@{g}"] = {"ms": round(ms, 4), "alg_TBs": round(alg / ms / 1e9, 3),
                                     "copy_TBs": round(2 * 16 * tot / ms / 1e9, 3)}
    cx = rc.Codec(b"hello135", 0)
    for v in args.paths.split(","):
        f = [int(x) for x in v.split(":")]
        cx.set_encode_path(f[0])
        cx.set_copy_k(f[1] if len(f) > 1 else 0)
        ms = timeit(lambda: cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame,
                                            w.frame_off, w.status, id_uniform=workload.ID_UNIFORM, pad128=True))
        out["rows"][f"encode_path{v}"] = {"ms": round(ms, 4), "alg_TBs": round(alg / ms / 1e9, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
