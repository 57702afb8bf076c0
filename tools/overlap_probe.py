#!/usr/bin/env python3
"""Probe: encode of batch k+1 (stream 1) overlapped with decode of batch k (stream 2) on double-
buffered frame arenas — the send and receive directions of a duplex tunnel run concurrently —
against the serial encode -> decode step of bench.py.  Every step still encodes and decodes its
whole batch.  One JSON line.   python tools/overlap_probe.py [--config c3] [--steps 30]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    cx.reserve(n)
    cx2 = rc.Codec(b"hello135", 0)  # its own compaction workspace for the second stream
    cx2.reserve(n)
    frames = [w.frame, torch.empty_like(w.frame)]
    decs = [w.dec, rc.DecodeBuffers.alloc(n, dev)]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def enc(buf, s):
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, frames[buf], w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)

    def dec(buf, s, c):
        c.onrecv_batch(frames[buf], w.frame_off, w.frame_len, decs[buf], stream=s)

    def serial(K):
        for _ in range(K):
            enc(0, s1)
            dec(0, s1, cx)

    def overlapped(K):
        done = [None, None]
        for k in range(K):
            b = k & 1
            if done[b] is not None:
                s1.wait_event(done[b])  # decode of batch k-2 finished with this arena
            enc(b, s1)
            e = torch.cuda.Event()
            e.record(s1)
            s2.wait_event(e)
            dec(b, s2, cx2)
            done[b] = torch.cuda.Event()
            done[b].record(s2)

    out = {}
    for name, f in (("serial", serial), ("overlapped", overlapped), ("serial2", serial), ("overlapped2", overlapped)):
        f(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        f(args.steps)
        torch.cuda.synchronize()
        out[name] = round(n * args.steps / (time.perf_counter() - t0) / 1e6, 1)
    assert int(decs[0].n_valid.item()) == n and int(decs[1].n_valid.item()) == n
    print(json.dumps({"config": args.config, "packets": n, "Mpkt_s": out}))


if __name__ == "__main__":
    main()
