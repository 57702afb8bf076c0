#!/usr/bin/env python3
"""Probe: per-step time of bench.py's C3 step replayed from a hipGraph, for the first and a second
graph captured in one process, against eager launches (why bench.py's first timed graph region ran
~90 us per step slower than the same step timed later in the process).
    python tools/graph_probe.py [--steps 50]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--order", default="eager,graph,graph,eager,graph")
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    d = workload.describe(args.config)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    stream = torch.cuda.Stream(dev)
    cx.reserve(d.n, stream=stream)

    def step():
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                        id_uniform=workload.ID_UNIFORM, pad16=d.pad == 16, pad128=d.pad == 128, stream=stream)
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=stream)

    def t_eager():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            for _ in range(args.steps):
                step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps * 1e3

    def t_graph(on_stream=False):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=stream):
            step()
        g.replay()
        torch.cuda.synchronize()
        res = []
        for _ in range(3):
            t0 = time.perf_counter()
            if on_stream:  # replays on the capture stream instead of the current (null) stream
                with torch.cuda.stream(stream):
                    for _ in range(args.steps):
                        g.replay()
            else:
                for _ in range(args.steps):
                    g.replay()
            torch.cuda.synchronize()
            res.append((time.perf_counter() - t0) / args.steps * 1e3)
        del g
        return res

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
    out = {}
    for k, what in enumerate(args.order.split(",")):
        out[f"{k}_{what}"] = t_eager() if what == "eager" else t_graph(what == "sgraph")
    print(json.dumps({k: ([round(x, 4) for x in v] if isinstance(v, list) else round(v, 4)) for k, v in out.items()}))


if __name__ == "__main__":
    main()
