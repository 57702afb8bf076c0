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
    nchunk = (n + C - 1) // C
    h_lens = torch.zeros(nchunk, 2, C, dtype=torch.int32)  # per chunk: wire_len row, cap_len row
    for ci in range(nchunk):
        m = min(C, n - ci * C)
        h_lens[ci, 0, :m] = h_wl[ci * C: ci * C + m]
        h_lens[ci, 1, :m] = h_cl[ci * C: ci * C + m]
    h_lens = h_lens.pin_memory()
    # every output a receive loop consumes, carved out of ONE device block per stream so a chunk
    # returns with a single D2H copy (per-field copies cost more than the bytes)
    FIELDS = (("parse_status", torch.int8, 1), ("src", torch.int32, 1), ("dst", torch.int32, 1),
              ("sp", torch.int16, 1), ("dp", torch.int16, 1), ("seq", torch.int32, 1), ("ack", torch.int32, 1),
              ("flag", torch.uint8, 1), ("cap_pay_off", torch.int16, 1), ("cap_pay_len", torch.int16, 1),
              ("status", torch.int8, 1), ("hlen", torch.uint8, 1), ("cmd", torch.uint8, 1), ("id", torch.uint8, 8),
              ("conv", torch.int32, 1), ("conn_key", torch.int64, 1), ("pay_off", torch.int16, 1),
              ("pay_len", torch.int16, 1), ("valid_idx", torch.int32, 1), ("n_valid", torch.int32, 0))

    def layout(m):
        o, offs = 0, {}
        for k, dt, q in FIELDS:
            nb = (q * m if q else 1) * torch.empty(0, dtype=dt).element_size()
            offs[k] = (o, nb, dt)
            o += (nb + 15) // 16 * 16
        return offs, o

    def carve(blk, m):
        return {k: blk[o: o + nb].view(dt) for k, (o, nb, dt) in layout(m)[0].items()}

    out_bytes = layout(C)[1]
    h_out = torch.empty(nchunk * out_bytes, dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream() for _ in range(S)]
    bufs = []
    for _ in range(S):
        blk = torch.zeros(out_bytes, dtype=torch.uint8, device=dev)
        v = carve(blk, C)
        b = {"cap": torch.empty(C * cp, dtype=torch.uint8, device=dev),
             "slots": torch.empty(C * slot, dtype=torch.uint8, device=dev),
             "off": torch.arange(C, device=dev, dtype=torch.int64) * cp,
             "lens": torch.empty(2, C, dtype=torch.int32, device=dev), "blk": blk,
             "tcp": rc.TcpInfoBuffers(**{k: v[k] for k in ("src", "dst", "sp", "dp", "seq", "ack", "flag", "parse_status",
                                                           "cap_pay_off", "cap_pay_len")}),
             "dec": rc.DecodeBuffers(**{k: v[k] for k in ("hlen", "cmd", "id", "conv", "conn_key", "pay_off", "pay_len",
                                                          "status", "valid_idx", "n_valid")}),
             "cx": rc.Codec(b"hello135", 0)}
        b["cx"].reserve(C)
        bufs.append(b)

    def run(mode):
        for c0 in range(0, n, C):
            ci = c0 // C
            k = ci % S
            s, b = streams[k], bufs[k]
            m = min(C, n - c0)
            with torch.cuda.stream(s):
                b["lens"].copy_(h_lens[ci], non_blocking=True)
                wl_d, cl_d = b["lens"][0, :m], b["lens"][1, :m]
                if mode == "whole":
                    b["cap"][: m * cp].copy_(h_cap[c0 * cp: (c0 + m) * cp], non_blocking=True)
                    b["cx"].rawinput_batch(b["cap"], b["off"][:m], wl_d, cl_d, 1, 0, b["tcp"], b["dec"], stream=s)
                else:
                    b["slots"][: m * slot].copy_(h_slots[c0 * slot: (c0 + m) * slot], non_blocking=True)
                    b["cx"].rawinput_slots_batch(b["slots"], slot, wl_d, cl_d, 1, 0, b["tcp"], b["dec"], stream=s)
                h_out[ci * out_bytes: (ci + 1) * out_bytes].copy_(b["blk"], non_blocking=True)

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
        snap = h_out.clone()
        if ref is None:
            ref = snap
        else:
            assert torch.equal(ref, snap), f"{mode}: outputs differ from the whole-capture path"
        t0 = time.perf_counter()
        for _ in range(args.reps):
            run(mode)
        torch.cuda.synchronize()
        res[mode] = round(n / ((time.perf_counter() - t0) / args.reps) / 1e6, 2)
    for ci in range((n + C - 1) // C):  # every packet delivered and verified
        m = min(C, n - ci * C)
        v = carve(ref[ci * out_bytes: (ci + 1) * out_bytes], C)
        assert bool((v["parse_status"][:m] == _abi.PARSE_DELIVER).all()) and bool((v["status"][:m] == 1).all())
    print(json.dumps({"config": args.config, "packets": n, "capture_pitch": cp, "slot": slot, "chunk": C, "streams": S,
                      "host_resident_parse_decode_Mpkt_s": res,
                      "host_stage_slots_16_threads_Mpkt_s": round(stage_rate, 1),
                      "pcie_bytes_per_pkt": {"whole": {"h2d": cp + 8, "d2h": round(out_bytes / C, 1)},
                                             "slots": {"h2d": slot + 8, "d2h": round(out_bytes / C, 1)}},
                      "copies_per_chunk": {"h2d": 2, "d2h": 1}}))


if __name__ == "__main__":
    main()
