#!/usr/bin/env python3
"""Host-resident pcap receive rate (PCIe-inclusive): captured Ethernet packets sit in a pinned host
capture buffer (the pcap ring RawTcp::RawInput reads, conn/RawTcp.cpp:138-244); per chunk they go
H2D -> parse + decode + compaction -> the TcpInfo, decode fields and VALID list D2H, chunked over
several streams.  Two forms:
  whole  the whole captured packets cross PCIe (rsk_parse_decode_batch)
  slots  only the first `slot` bytes of each packet, staged by rsk_stage_capture_slots on the host
         (rsk_parse_decode_slots_batch); the payloads stay in the capture buffer for delivery
Reported in DESIGN.md §6.4; never bench.py's `value`.

  python tools/bench_pcap_host.py [--config c3] [--slot 96] [--chunk 262144] [--streams 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--slot", type=int, default=96)
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import torch

    from rsock_amd import _abi
    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = args.packets or workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    # the capture: Ethernet wire packets built on the GPU (rsk_encode_wire_batch), as a peer sends them
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    ri = lambda hi, dt: torch.randint(0, hi, (n,), device=dev, generator=g, dtype=torch.int64).to(dt)  # noqa: E731
    pmax = workload.CONFIGS[args.config][3]
    cp = (54 + 31 + pmax + 15) // 16 * 16
    cap = torch.empty(n * cp, dtype=torch.uint8, device=dev)
    cap_off = torch.arange(n, device=dev, dtype=torch.int64) * cp
    wl = torch.empty(n, dtype=torch.int32, device=dev)
    cx.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, ri(2**31, torch.int32),
                         ri(2**31, torch.int32), ri(2**15, torch.int16) + 1, ri(2**15, torch.int16) + 1,
                         ri(2**31, torch.int32), ri(2**31, torch.int32),
                         torch.full((n,), 0x18, dtype=torch.uint8, device=dev), ri(2**15, torch.int16), cap, cap_off,
                         wl, eth=bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2, 8, 0]), id_uniform=workload.ID_UNIFORM,
                         pad16=True)
    torch.cuda.synchronize()
    h_cap = cap.cpu().pin_memory()
    h_wl = wl.cpu().pin_memory()
    h_cl = h_wl.clone().pin_memory()
    del w, cap
    torch.cuda.empty_cache()
    S, C, slot = args.streams, min(args.chunk, n), args.slot
    h_slots = torch.empty(n * slot, dtype=torch.uint8).pin_memory()
    # outputs a receive loop consumes, back in pinned host memory
    outs = {k: torch.empty(n, dtype=dt).pin_memory() for k, dt in (
        ("parse_status", torch.int8), ("src", torch.int32), ("dst", torch.int32), ("sp", torch.int16),
        ("dp", torch.int16), ("seq", torch.int32), ("ack", torch.int32), ("flag", torch.uint8),
        ("cap_pay_off", torch.int16), ("cap_pay_len", torch.int16), ("status", torch.int8), ("hlen", torch.uint8),
        ("cmd", torch.uint8), ("conv", torch.int32), ("conn_key", torch.int64), ("pay_off", torch.int16),
        ("pay_len", torch.int16), ("valid_idx", torch.int32))}
    outs["id"] = torch.empty(8 * n, dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream() for _ in range(S)]
    bufs = []
    for _ in range(S):
        b = {"cap": torch.empty(C * cp, dtype=torch.uint8, device=dev),
             "slots": torch.empty(C * slot, dtype=torch.uint8, device=dev),
             "off": torch.arange(C, device=dev, dtype=torch.int64) * cp,
             "wl": torch.empty(C, dtype=torch.int32, device=dev), "cl": torch.empty(C, dtype=torch.int32, device=dev),
             "tcp": rc.TcpInfoBuffers.alloc(C, dev), "dec": rc.DecodeBuffers.alloc(C, dev),
             "cx": rc.Codec(b"hello135", 0)}
        b["cx"].reserve(C)
        bufs.append(b)

    def run(mode):
        for c0 in range(0, n, C):
            k = (c0 // C) % S
            s, b = streams[k], bufs[k]
            m = min(C, n - c0)
            with torch.cuda.stream(s):
                b["wl"][:m].copy_(h_wl[c0: c0 + m], non_blocking=True)
                b["cl"][:m].copy_(h_cl[c0: c0 + m], non_blocking=True)
                if mode == "whole":
                    b["cap"][: m * cp].copy_(h_cap[c0 * cp: (c0 + m) * cp], non_blocking=True)
                    b["cx"].rawinput_batch(b["cap"], b["off"][:m], b["wl"][:m], b["cl"][:m], 1, 0, b["tcp"], b["dec"],
                                           stream=s)
                else:
                    b["slots"][: m * slot].copy_(h_slots[c0 * slot: (c0 + m) * slot], non_blocking=True)
                    b["cx"].rawinput_slots_batch(b["slots"], slot, b["wl"][:m], b["cl"][:m], 1, 0, b["tcp"], b["dec"],
                                                 stream=s)
                for key, t in outs.items():
                    src = getattr(b["tcp"], key, None)
                    if src is None:
                        src = getattr(b["dec"], key)
                    q = 8 if key == "id" else 1
                    t[q * c0: q * (c0 + m)].copy_(src[: q * m], non_blocking=True)

    # host staging of the slots from the capture buffer (16 threads = the pod's CPU share)
    lib = _abi.load()
    capn = h_cap.numpy()
    offn = (np.arange(n, dtype=np.uint64) * cp)
    cln = h_cl.numpy().view(np.uint32)
    slotn = h_slots.numpy()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        assert lib.rsk_stage_capture_slots(n, capn.ctypes.data, offn.ctypes.data, cln.ctypes.data, slot,
                                           slotn.ctypes.data, 16) == 0
    stage_rate = n * args.reps / (time.perf_counter() - t0) / 1e6
    res, ref = {}, None
    for mode in ("whole", "slots"):
        run(mode)
        torch.cuda.synchronize()
        snap = {k: v.clone() for k, v in outs.items()}
        if ref is None:
            ref = snap
        else:
            for k in ref:
                assert torch.equal(ref[k], snap[k]), f"{mode}: {k} differs from the whole-capture path"
        t0 = time.perf_counter()
        for _ in range(args.reps):
            run(mode)
        torch.cuda.synchronize()
        res[mode] = round(n / ((time.perf_counter() - t0) / args.reps) / 1e6, 2)
    assert bool((ref["parse_status"] == _abi.PARSE_DELIVER).all()) and bool((ref["status"] == 1).all())
    print(json.dumps({"config": args.config, "packets": n, "capture_pitch": cp, "slot": slot, "chunk": C, "streams": S,
                      "host_resident_parse_decode_Mpkt_s": res,
                      "host_stage_slots_16_threads_Mpkt_s": round(stage_rate, 1),
                      "pcie_bytes_per_pkt": {"whole": {"h2d": cp + 8, "d2h": 57}, "slots": {"h2d": slot + 8, "d2h": 57}}}))


if __name__ == "__main__":
    main()
