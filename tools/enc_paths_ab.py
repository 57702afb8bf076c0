#!/usr/bin/env python3
"""In-process A/B of rsk_encode_batch's paths on one config (device-resident, HIP events on the launch
stream, interleaved rounds): each variant = (encode path, two-pass packets per copy wave k, two-pass chunk,
sub-batches): sub-batches > 1 issues the batch as that many consecutive slices alternating over two
streams forked from and joined back to the timing stream (the header pass of one slice beside the copy
of another).  Every variant's frames and statuses are compared with the per-set kernel's before timing.
    python tools/enc_paths_ab.py --config c3 [--variants 1,2:1,2:4,2:1:1048576,2:4:0:2] [--rounds 6] [--reps 10]
                                 [--layout slots|packed|odd] [--pad 16|128|0]
One JSON line: per variant the median over rounds of the mean encode time, and its fraction of 8 TB/s
by the algorithmic bytes (2P + 66 per packet)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse_variant(v):
    """path[:k[:chunk[:sub]]] -- k packets per copy wave (path 2; 0 = chosen by the library), chunk packets
    per heads / copy pair (path 2; 0 = the whole batch), sub-batches over two streams (0 / 1 = one call)"""
    f = [int(x) for x in v.split(":")] + [0, 0, 0]
    return (f[0], f[1], f[2], max(f[3], 1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--variants", default="1,2:1,2:4")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--layout", default="slots", choices=["slots", "packed", "odd"],
                    help="frame layout: the workload's slots, frames packed at byte granularity, or slots + 5 B")
    ap.add_argument("--pad", type=int, default=-1, help="zero pad 0/16/128 (default: the workload's)")
    ap.add_argument("--tag", default="md5")
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = args.packets or workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    pad = d.pad if args.pad < 0 else args.pad
    plen = d.pay_len.astype(np.int64)
    if args.layout == "packed":
        fl = plen + 31
        off = np.concatenate([[0], np.cumsum(fl)[:-1]]).astype(np.int64)
        pad = 0
    elif args.layout == "odd":
        off = np.arange(n, dtype=np.int64) * d.frame_pitch + 5
        pad = 0
    else:
        off = None
    if off is not None:
        w.frame_off = torch.from_numpy(off).to(dev)
        w.frame = torch.zeros(int(off[-1]) + 2048, dtype=torch.uint8, device=dev)
    cx = rc.Codec(b"hello135", 0, tag_mode=args.tag)
    s = torch.cuda.Stream(dev)
    s2 = torch.cuda.Stream(dev)
    variants = [parse_variant(v) for v in args.variants.split(",")]

    def run(v):
        p, k, chunk, sub = v
        cx.set_encode_path(p)
        cx.set_copy_k(k)
        cx.set_two_pass_chunk(chunk)
        if sub == 1:
            cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                            w.status, id_uniform=workload.ID_UNIFORM, pad16=pad == 16, pad128=pad == 128, stream=s)
            return
        fork = torch.cuda.Event()
        fork.record(s)
        s2.wait_event(fork)
        for q in range(sub):
            lo, hi = n * q // sub, n * (q + 1) // sub
            sl = slice(lo, hi)
            cx.output_batch(w.payload, w.pay_off[sl], w.pay_len[sl], w.cmd[sl], w.conv[sl], w.conn_key[sl], w.frame,
                            w.frame_off[sl], w.status[sl], id_uniform=workload.ID_UNIFORM, pad16=pad == 16,
                            pad128=pad == 128, stream=s if q % 2 == 0 else s2)
        join = torch.cuda.Event()
        join.record(s2)
        s.wait_event(join)

    with torch.cuda.stream(s):
        w.frame.zero_()
        run((1, 0, 0, 1))
        s.synchronize()
        ref_f, ref_s = w.frame.clone(), w.status.clone()
        for v in variants:
            w.frame.zero_()
            w.status.fill_(-7)
            run(v)
            s.synchronize()
            assert cx.last_encode_path == v[0], (v, cx.last_encode_path)
            assert torch.equal(w.frame, ref_f) and torch.equal(w.status, ref_s), f"variant {v}: bytes differ"
        del ref_f
    alg = int((2 * plen + 66).sum())
    times = {v: [] for v in variants}
    for r in range(args.rounds):
        for v in variants:
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.reps)]
            with torch.cuda.stream(s):
                run(v)
                for e0, e1 in evs:
                    e0.record(s)
                    run(v)
                    e1.record(s)
            s.synchronize()
            times[v].append(float(np.mean([e0.elapsed_time(e1) for e0, e1 in evs])))
    out = {"config": args.config, "packets": n, "layout": args.layout, "pad": pad, "tag": args.tag,
           "algorithmic_bytes": alg, "variants": {}}
    for v in variants:
        ms = float(np.median(times[v]))
        out["variants"][":".join(map(str, v))] = {"ms": round(ms, 4), "min_ms": round(min(times[v]), 4),
                                                 "frac_8TBs": round(alg / (ms * 1e-3) / 8e12, 4),
                                                 "rounds_ms": [round(t, 4) for t in times[v]]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
