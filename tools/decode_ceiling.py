#!/usr/bin/env python3
"""The ceiling of the isolated-read kernels (round 5): k_decode reads each frame's
first 32 B at the frame pitch (plus streamed descriptors and dense outputs), k_encode_heads each
payload's first bytes at the payload pitch and writes a 32-B record per packet.  Times, in one
process with HIP events, the probe `probe_strided` (tools/hbm_probe.hip: one lane per item, isolated
16- / 32-B reads at a pitch, optionally a dense 16-B record per item) at the configs' pitches, next to
k_decode (+ k_compact) and the two-pass header pass on the same workload.
    python tools/decode_ceiling.py [--config c3] [--reps 20]"""
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
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    L = ctypes.CDLL(os.path.join(HERE, "libhbm_probe.so"))
    L.probe_strided.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int,
                                ctypes.c_int, ctypes.c_void_p]
    n = workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    s = torch.cuda.current_stream()
    pad = dict(pad16=d.pad == 16, pad128=d.pad == 128)
    enc = lambda: cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame,  # noqa: E731
                                  w.frame_off, w.status, id_uniform=workload.ID_UNIFORM, **pad)
    enc()
    dec = rc.DecodeBuffers.alloc(n, dev)
    decode = lambda: cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, dec)  # noqa: E731
    rec = torch.empty(n * 16 + 4096, dtype=torch.uint8, device=dev)

    def probe(buf, pitch, nb, write):
        def f():
            r = L.probe_strided(ctypes.c_void_p(buf.data_ptr()), ctypes.c_void_p(rec.data_ptr()), n, pitch, nb,
                                write, ctypes.c_void_p(s.cuda_stream))
            assert r == 0, r
        return f

    ops = {
        "k_decode+k_compact": decode,
        "probe: 32 B at the frame pitch": probe(w.frame, d.frame_pitch, 2, 0),
        "probe: 16 B at the frame pitch": probe(w.frame, d.frame_pitch, 1, 0),
        "probe: 16 B at the payload pitch + 16-B record": probe(w.payload, d.pay_pitch, 1, 1),
        "probe: 16 B at the payload pitch": probe(w.payload, d.pay_pitch, 1, 0),
    }
    res = {}
    for r in range(3):
        for k, f in ops.items():
            f()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            for e0, e1 in ev:
                e0.record(s)
                f()
                e1.record(s)
            s.synchronize()
            res.setdefault(k, []).append(float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev])))
    torch.cuda.synchronize()
    out = {"config": args.config, "packets": n, "frame_pitch": d.frame_pitch, "pay_pitch": d.pay_pitch,
           "ms": {k: round(float(np.median(v)), 4) for k, v in res.items()}}
    out["items_per_s_G"] = {k: round(n / (v * 1e-3) / 1e9, 2) for k, v in out["ms"].items()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
