#!/usr/bin/env python3
"""Where the two-pass encode starts to pay (rsk_encode_batch's kTwoPassMinPayload): encode time of
both paths (rsk_set_encode_path 1 = per-set kernel, 2 = two-pass) on synthetic batches of uniform
and mixed payload lengths, device-resident, HIP events, interleaved rounds in one process.  Frames
of both paths are compared byte for byte before timing.
    python tools/path_threshold.py [--packets 2097152] [--rounds 4] [--reps 5]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (pmin, pmax): uniform lengths, then mixed ranges (pmin < pmax: uniform in [pmin, pmax])
CASES = [(400, 400), (600, 600), (800, 800), (900, 900), (1000, 1000), (1100, 1100), (1200, 1200),
         (1400, 1400), (700, 1400), (900, 1400), (1, 1469)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from bench import enc_bytes_per_pkt
    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    cx = rc.Codec(b"hello135", 0)
    s = torch.cuda.current_stream()
    out = {}
    for k, (pmin, pmax) in enumerate(CASES):
        name = f"t{pmin}_{pmax}"
        workload.CONFIGS[name] = (20 + k, args.packets, pmin, pmax, 1, False, 0)
        d = workload.describe(name, 0, args.packets, n=args.packets)
        w = workload.DeviceWorkload(d, dev)

        def enc():
            cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                            w.status, id_uniform=workload.ID_UNIFORM, pad16=d.pad == 16, pad128=d.pad == 128,
                            stream=s)

        frames = []
        for p in (1, 2):
            cx.set_encode_path(p)
            w.frame.zero_()
            enc()
            torch.cuda.synchronize()
            frames.append(w.frame.clone())
        if not torch.equal(frames[0], frames[1]):
            raise SystemExit(f"{name}: the two paths' frames differ")
        del frames
        t = {1: [], 2: []}
        for _ in range(args.rounds):
            for p in (1, 2):
                cx.set_encode_path(p)
                enc()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(args.reps):
                    enc()
                e1.record(s)
                torch.cuda.synchronize()
                t[p].append(e0.elapsed_time(e1) / args.reps)
        byts = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
        m1, m2 = float(np.median(t[1])), float(np.median(t[2]))
        out[name] = {"mean_payload": round(float(d.pay_len.mean()), 1), "frame_pitch": d.frame_pitch,
                     "per_set_ms": round(m1, 4), "two_pass_ms": round(m2, 4), "two_pass_over_per_set": round(m2 / m1, 4),
                     "per_set_frac": round(byts / (m1 * 1e-3) / 8e12, 4), "two_pass_frac": round(byts / (m2 * 1e-3) / 8e12, 4)}
        del w
        torch.cuda.empty_cache()
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    cx.set_encode_path(0)
    print(json.dumps({"packets": args.packets, "cases": out}))


if __name__ == "__main__":
    main()
