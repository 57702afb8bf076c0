#!/usr/bin/env python3
"""Where each encode path pays (rsk_encode_batch's thresholds): encode time of the per-set kernel
(path 1), the short-frame kernel (3) and the two-pass form with k packets per copy wave (2:k) on
synthetic batches of uniform and mixed payload lengths, device-resident, HIP events, interleaved rounds
in one process.  Every variant's frames are compared with path 1's byte for byte before timing.
    python tools/path_threshold.py [--packets 2097152] [--rounds 4] [--reps 5] [--variants 1,2:1,2:4]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (pmin, pmax): uniform lengths, then mixed ranges (pmin < pmax: uniform in [pmin, pmax])
CASES = [(100, 100), (160, 160), (200, 200), (300, 300), (400, 400), (600, 600), (800, 800), (900, 900),
         (1000, 1000), (1100, 1100), (1200, 1200), (1400, 1400), (64, 1400), (700, 1400), (900, 1400), (1, 1469),
         (64, 64), (128, 128), (250, 250), (350, 350), (450, 450), (500, 500), (1, 600), (1, 900), (100, 700),
         (256, 700), (1, 300)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=1 << 21)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="1,3,2:1,2:2,2:4")
    ap.add_argument("--cases", default="", help="subset of CASES as pmin_pmax,... (default: all)")
    ap.add_argument("--wire", default="", choices=["", "raw4", "eth"],
                    help="time rsk_encode_wire_batch (RAW4 / Ethernet wire packets) instead of rsk_encode_batch")
    args = ap.parse_args()
    variants = [tuple(int(x) for x in v.split(":")) for v in args.variants.split(",")]
    vname = lambda v: ":".join(map(str, v))  # noqa: E731
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
        if args.cases and f"{pmin}_{pmax}" not in args.cases.split(","):
            continue
        workload.CONFIGS[name] = (20 + k, args.packets, pmin, pmax, 1, False, 0)
        d = workload.describe(name, 0, args.packets, n=args.packets)
        w = workload.DeviceWorkload(d, dev)
        if args.wire:
            # wire packets in slots of the frame slot rule over the wire length (link + IPv4 + TCP + frame)
            L = (14 if args.wire == "eth" else 0) + 40
            al = 128 if d.pad == 128 else 16
            wp = (L + 31 + pmax + al - 1) // al * al
            g = torch.Generator(device=dev)
            g.manual_seed(k)
            n_ = args.packets
            ri = lambda hi, dt: torch.randint(0, hi, (n_,), device=dev, generator=g, dtype=torch.int64).to(dt)  # noqa
            wf = [ri(2**31, torch.int32), ri(2**31, torch.int32), ri(2**15, torch.int16) + 1, ri(2**15, torch.int16) + 1,
                  ri(2**31, torch.int32), ri(2**31, torch.int32), torch.full((n_,), 0x18, dtype=torch.uint8, device=dev),
                  ri(2**15, torch.int16)]
            w.frame = torch.empty(n_ * wp, dtype=torch.uint8, device=dev)
            w.frame_off = torch.arange(n_, device=dev, dtype=torch.int64) * wp
            eth = bytes(range(14)) if args.wire == "eth" else None

        def enc():
            if args.wire:
                cx.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, *wf, w.frame,
                                     w.frame_off, w.status, eth=eth, id_uniform=workload.ID_UNIFORM,
                                     pad16=d.pad == 16, pad128=d.pad == 128, stream=s)
                return
            cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                            w.status, id_uniform=workload.ID_UNIFORM, pad16=d.pad == 16, pad128=d.pad == 128,
                            stream=s)

        def setv(v):
            cx.set_encode_path(v[0])
            cx.set_copy_k(v[1] if len(v) > 1 else 0)

        setv((1,))
        w.frame.zero_()
        enc()
        torch.cuda.synchronize()
        ref = w.frame.clone()
        for v in variants:
            setv(v)
            w.frame.zero_()
            enc()
            torch.cuda.synchronize()
            if not torch.equal(ref, w.frame):
                raise SystemExit(f"{name}: variant {vname(v)} frames differ from the per-set kernel's")
        del ref
        t = {v: [] for v in variants}
        for _ in range(args.rounds):
            for v in variants:
                setv(v)
                enc()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(args.reps):
                    enc()
                e1.record(s)
                torch.cuda.synchronize()
                t[v].append(e0.elapsed_time(e1) / args.reps)
        byts = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
        if args.wire:  # + the IPv4/TCP (+ link) header and the 23 B of wire fields per packet
            byts += args.packets * ((14 if args.wire == "eth" else 0) + 40 + 23)
        out[name] = {"mean_payload": round(float(d.pay_len.mean()), 1), "frame_pitch": d.frame_pitch,
                     "ms": {vname(v): round(float(np.median(t[v])), 4) for v in variants}}
        out[name]["frac_8TBs"] = {k: round(byts / (ms * 1e-3) / 8e12, 4) for k, ms in out[name]["ms"].items()}
        out[name]["best"] = min(out[name]["ms"], key=out[name]["ms"].get)
        del w
        torch.cuda.empty_cache()
        print(json.dumps({name: out[name]}), file=sys.stderr, flush=True)
    cx.set_encode_path(0)
    cx.set_copy_k(0)
    print(json.dumps({"packets": args.packets, "variants": [vname(v) for v in variants], "cases": out}))


if __name__ == "__main__":
    main()
