#!/usr/bin/env python3
"""k_encode under payload-arena x frame-arena layouts (and encode variants of the A/B build),
device-resident, HIP events on the launch stream, interleaved rounds in one process:
  payload layouts  slots     the workload's slots (pitch round16(P_max); 1408 B = 11 lines for C3/C4)
                   packed16  payloads back to back at 16-B granularity (pay_off = prefix sum of
                             round16(P)), the bytes of each payload identical to its slot's
  frame layouts    slots     the workload's slots (C4: 1536-B, RSK_ENC_ZERO_PAD128)
                   packed16  frames back to back at 16-B granularity, RSK_ENC_ZERO_PAD16
                   packed128 frames back to back at 128-B granularity, RSK_ENC_ZERO_PAD128
Every case's frames are checked against the first case's, frame by frame, before timing.
    python tools/enc_layout_ab.py [--config c4] [--cases slots/slots,packed16/packed16] [--variants 0]
    python tools/enc_layout_ab.py --config c4 --cases packed16/packed16 --only --reps 3   # for rocprofv3 --pmc
(variants other than 0 need RSK_LIB=librsk_ab.so)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def prefix(x):
    return np.concatenate([[0], np.cumsum(x)[:-1]]).astype(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--cases", default="slots/slots,slots/packed16,packed16/packed16,packed16/packed128",
                    help="payload_layout/frame_layout pairs")
    ap.add_argument("--variants", default="0")
    ap.add_argument("--only", action="store_true", help="run each case `reps` times, no timing (PMC passes)")
    args = ap.parse_args()
    import torch

    from bench import enc_bytes_per_pkt
    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = args.packets or workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    s = torch.cuda.current_stream()
    plen = d.pay_len.astype(np.int64)
    flen = d.frame_len.astype(np.int64)
    r16p, r16f, r128f = (plen + 15) // 16 * 16, (flen + 15) // 16 * 16, (flen + 127) // 128 * 128
    pays = {"slots": (w.payload, w.pay_off)}
    po = prefix(r16p)
    pk = torch.zeros(int(po[-1] + r16p[-1]) + 64, dtype=torch.uint8, device=dev)
    src_off = torch.from_numpy(d.pay_off.astype(np.int64)).to(dev)
    dst_off = torch.from_numpy(po).to(dev)
    pl = torch.from_numpy(plen).to(dev)
    idx = torch.arange(1408, device=dev)
    for lo in range(0, n, 1 << 15):  # copy every payload into its packed place
        hi = min(n, lo + (1 << 15))
        m = idx.view(1, -1) < pl[lo:hi].view(-1, 1)
        sidx = (src_off[lo:hi].view(-1, 1) + idx.view(1, -1))[m]
        didx = (dst_off[lo:hi].view(-1, 1) + idx.view(1, -1))[m]
        pk[didx] = w.payload[sidx]
    pays["packed16"] = (pk, dst_off)
    frames = {"slots": (d.frame_off.astype(np.int64), d.pad), "packed16": (prefix(r16f), 16),
              "packed128": (prefix(r128f), 128)}
    cases = []
    for c in args.cases.split(","):
        pl_, fl_ = c.split("/")
        for v in args.variants.split(","):
            cases.append((pl_, fl_, int(v)))
    arenas = {}
    for pl_, fl_, v in cases:
        if (pl_, fl_) in arenas:
            continue
        fo, pad = frames[fl_]
        arenas[(pl_, fl_)] = (torch.zeros(int(fo[-1]) + 1664, dtype=torch.uint8, device=dev),
                              torch.from_numpy(fo).to(dev), torch.empty(n, dtype=torch.int32, device=dev), pad)

    def run(case):
        pl_, fl_, v = case
        if v:
            cx.set_encode_variant(v)
        pay, pof = pays[pl_]
        fr, fo, st, pad = arenas[(pl_, fl_)]
        cx.output_batch(pay, pof, w.pay_len, w.cmd, w.conv, w.conn_key, fr, fo, st, id_uniform=workload.ID_UNIFORM,
                        pad16=pad == 16, pad128=pad == 128, stream=s)
        if v:
            cx.set_encode_variant(0)

    if args.only:
        for case in cases:
            for _ in range(args.reps):
                run(case)
        torch.cuda.synchronize()
        print(json.dumps({"config": args.config, "cases": [list(c) for c in cases], "reps": args.reps}))
        return
    ref = None
    fl = torch.from_numpy(flen).to(dev)
    idx = torch.arange(1600, device=dev)
    for case in cases:
        run(case)
        torch.cuda.synchronize()
        fr, fo, _, _ = arenas[case[:2]]
        rows = []
        for lo in range(0, n, 1 << 15):
            hi = min(n, lo + (1 << 15))
            m = idx.view(1, -1) < fl[lo:hi].view(-1, 1)
            rows.append(fr[(fo[lo:hi].view(-1, 1) + idx.view(1, -1)).clamp(max=fr.numel() - 1)] * m)
        if ref is None:
            ref = rows
        elif not all(torch.equal(a, b) for a, b in zip(ref, rows)):
            raise SystemExit(f"case {case}: frames differ from case {cases[0]}")
    del ref
    times = {c: [] for c in cases}
    for _ in range(args.rounds):
        for c in cases:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                run(c)
            e1.record(s)
            torch.cuda.synchronize()
            times[c].append(e0.elapsed_time(e1) / args.reps)
    alg = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
    out = {}
    for c, t in times.items():
        ms = float(np.median(t))
        out[f"{c[0]}/{c[1]}/v{c[2]}"] = {"ms": round(ms, 4), "frac_of_8TBps": round(alg / ms / 8e9, 4)}
    print(json.dumps({"config": args.config, "packets": n, "algorithmic_bytes": alg, "cases": out}))


if __name__ == "__main__":
    main()
