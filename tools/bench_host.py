#!/usr/bin/env python3
"""Host-resident (PCIe-inclusive) codec rate — the path starts and ends in host memory
(BASELINE north_star: pcap buffer in, libnet buffer out), so this measures pinned host arenas ->
hipMemcpyAsync H2D -> kernels -> hipMemcpyAsync D2H, chunked over several streams so copies in both
directions overlap the kernels.  Reported in DESIGN.md §6.4; never bench.py's `value`.

  python tools/bench_host.py [--config c3] [--packets 4194304] [--chunk 262144] [--streams 3]

Modes (one JSON line each):
  encode   host payloads + descriptors -> frames back to host               (send path)
  decode   host frames -> verify + compact -> fields / valid_idx to host    (receive path)
  both     both directions per chunk
  encode_hdr / decode_hdr / both_hdr   header-only (rsk_encode_headers_batch / rsk_decode_headers_batch):
           payload[0] + descriptors in, 32-B header slots + status out; staged 32-B frame-header slots
           in, fields out — the payload never crosses PCIe (it stays in host memory for an iovec send /
           in the capture buffer for delivery)
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
    ap.add_argument("--chunk", type=int, default=262144)
    ap.add_argument("--streams", type=int, default=3)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--modes", default="encode,decode,both,encode_hdr,decode_hdr,both_hdr")
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = args.packets or workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    C = min(args.chunk, n)
    pin = lambda a: torch.from_numpy(a).pin_memory()  # noqa: E731
    # host-resident inputs (pinned), generated on the device once and copied out
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                    id_uniform=workload.ID_UNIFORM, pad16=True)
    torch.cuda.synchronize()
    h_pay = w.payload.cpu().pin_memory()
    h_frames_in = w.frame.cpu().pin_memory()  # "captured" frames for the receive path
    h_len = w.pay_len.cpu().pin_memory()
    h_cmd, h_conv, h_key = w.cmd.cpu().pin_memory(), w.conv.cpu().pin_memory(), w.conn_key.cpu().pin_memory()
    h_flen = w.frame_len.cpu().pin_memory()
    h_frames_out = torch.empty_like(h_frames_in).pin_memory()
    # header-only inputs: payload[0] per packet; staged decode slots of the captured frames
    h_b0 = w.payload[w.pay_off].cpu().pin_memory()
    h_slots = torch.from_numpy(rc.stage_decode_headers(h_frames_in.numpy(), w.frame_off.cpu().numpy(),
                                                       h_flen.numpy().astype(np.int32) & 0xFFFF).reshape(-1)).pin_memory()
    h_hdr_out = torch.empty(32 * n, dtype=torch.uint8).pin_memory()
    w_frame_off = w.frame_off.cpu().numpy().astype(np.uint64)
    w_pay_off = w.pay_off.cpu().numpy().astype(np.uint64)
    h_status = torch.empty(n, dtype=torch.int32).pin_memory()
    h_dstat = torch.empty(n, dtype=torch.int8).pin_memory()
    h_dconv = torch.empty(n, dtype=torch.int32).pin_memory()
    h_dkey = torch.empty(n, dtype=torch.int64).pin_memory()
    h_vidx = torch.empty(n, dtype=torch.int32).pin_memory()
    del w
    torch.cuda.empty_cache()

    S = args.streams
    streams = [torch.cuda.Stream() for _ in range(S)]
    pp, fp = d.pay_pitch, d.frame_pitch
    # per-stream device chunk buffers
    bufs = []
    for _ in range(S):
        b = {
            "pay": torch.empty(C * pp, dtype=torch.uint8, device=dev),
            "frame": torch.empty(C * fp, dtype=torch.uint8, device=dev),
            "frame_in": torch.empty(C * fp, dtype=torch.uint8, device=dev),
            "len": torch.empty(C, dtype=torch.int16, device=dev),
            "flen": torch.empty(C, dtype=torch.int16, device=dev),
            "cmd": torch.empty(C, dtype=torch.uint8, device=dev),
            "conv": torch.empty(C, dtype=torch.int32, device=dev),
            "key": torch.empty(C, dtype=torch.int64, device=dev),
            "status": torch.empty(C, dtype=torch.int32, device=dev),
            "pay_off": torch.arange(C, device=dev, dtype=torch.int64) * pp,
            "frame_off": torch.arange(C, device=dev, dtype=torch.int64) * fp,
            "dec": rc.DecodeBuffers.alloc(C, dev),
            "b0": torch.empty(C, dtype=torch.uint8, device=dev),
            "hdr": torch.empty(32 * C, dtype=torch.uint8, device=dev),
            "slots": torch.empty(32 * C, dtype=torch.uint8, device=dev),
            "cx": rc.Codec(b"hello135", 0),
        }
        b["cx"].reserve(C)
        bufs.append(b)

    def run(mode):
        for c0 in range(0, n, C):
            k = (c0 // C) % S
            s, b = streams[k], bufs[k]
            m = min(C, n - c0)
            with torch.cuda.stream(s):
                if mode in ("encode", "both"):
                    b["pay"][: m * pp].copy_(h_pay[c0 * pp: (c0 + m) * pp], non_blocking=True)
                    b["len"][:m].copy_(h_len[c0: c0 + m], non_blocking=True)
                    b["cmd"][:m].copy_(h_cmd[c0: c0 + m], non_blocking=True)
                    b["conv"][:m].copy_(h_conv[c0: c0 + m], non_blocking=True)
                    b["key"][:m].copy_(h_key[c0: c0 + m], non_blocking=True)
                    b["cx"].output_batch(b["pay"], b["pay_off"][:m], b["len"][:m], b["cmd"][:m], b["conv"][:m],
                                         b["key"][:m], b["frame"], b["frame_off"][:m], b["status"][:m],
                                         id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
                    h_frames_out[c0 * fp: (c0 + m) * fp].copy_(b["frame"][: m * fp], non_blocking=True)
                    h_status[c0: c0 + m].copy_(b["status"][:m], non_blocking=True)
                if mode in ("encode_hdr", "both_hdr"):
                    b["b0"][:m].copy_(h_b0[c0: c0 + m], non_blocking=True)
                    b["len"][:m].copy_(h_len[c0: c0 + m], non_blocking=True)
                    b["cmd"][:m].copy_(h_cmd[c0: c0 + m], non_blocking=True)
                    b["conv"][:m].copy_(h_conv[c0: c0 + m], non_blocking=True)
                    b["key"][:m].copy_(h_key[c0: c0 + m], non_blocking=True)
                    b["cx"].output_headers_batch(b["b0"][:m], b["len"][:m], b["cmd"][:m], b["conv"][:m], b["key"][:m],
                                                 b["hdr"], b["status"][:m], id_uniform=workload.ID_UNIFORM, stream=s)
                    h_hdr_out[32 * c0: 32 * (c0 + m)].copy_(b["hdr"][: 32 * m], non_blocking=True)
                    h_status[c0: c0 + m].copy_(b["status"][:m], non_blocking=True)
                if mode in ("decode_hdr", "both_hdr"):
                    b["slots"][: 32 * m].copy_(h_slots[32 * c0: 32 * (c0 + m)], non_blocking=True)
                    b["flen"][:m].copy_(h_flen[c0: c0 + m], non_blocking=True)
                    dec = b["dec"]
                    b["cx"].onrecv_headers_batch(b["slots"], b["flen"][:m], dec, stream=s)
                    h_dstat[c0: c0 + m].copy_(dec.status[:m], non_blocking=True)
                    h_dconv[c0: c0 + m].copy_(dec.conv[:m], non_blocking=True)
                    h_dkey[c0: c0 + m].copy_(dec.conn_key[:m], non_blocking=True)
                    h_vidx[c0: c0 + m].copy_(dec.valid_idx[:m], non_blocking=True)
                if mode in ("decode", "both"):
                    b["frame_in"][: m * fp].copy_(h_frames_in[c0 * fp: (c0 + m) * fp], non_blocking=True)
                    b["flen"][:m].copy_(h_flen[c0: c0 + m], non_blocking=True)
                    dec = b["dec"]
                    b["cx"].onrecv_batch(b["frame_in"], b["frame_off"][:m], b["flen"][:m], dec, stream=s)
                    h_dstat[c0: c0 + m].copy_(dec.status[:m], non_blocking=True)
                    h_dconv[c0: c0 + m].copy_(dec.conv[:m], non_blocking=True)
                    h_dkey[c0: c0 + m].copy_(dec.conn_key[:m], non_blocking=True)
                    h_vidx[c0: c0 + m].copy_(dec.valid_idx[:m], non_blocking=True)

    out = {}
    for mode in args.modes.split(","):
        run(mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            run(mode)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / args.reps
        out[mode] = round(n / el / 1e6, 2)
    # host side of the header-only path, on this box's host cores (16 threads, the pod's CPU share):
    # staging the 32-B decode slots from the captured frames, and assembling contiguous frames from
    # header slots + payloads (the memcpy RConn::Output makes; an iovec send skips it)
    import ctypes

    from rsock_amd import _abi
    lib = _abi.load()
    host = {}
    if any(m.endswith("_hdr") for m in out):
        fin = h_frames_in.numpy()
        foff = w_frame_off
        flen = h_flen.numpy().view(np.uint16)
        slots = np.empty(32 * n, np.uint8)
        t0 = time.perf_counter()
        assert lib.rsk_stage_decode_headers(n, fin.ctypes.data, foff.ctypes.data, flen.ctypes.data, slots.ctypes.data,
                                            16) == 0
        host["stage_decode_slots_Mpkt_s"] = round(n / (time.perf_counter() - t0) / 1e6, 1)
        assert np.array_equal(slots, h_slots.numpy())
        if "encode_hdr" in out or "both_hdr" in out:
            fout = np.empty_like(fin)
            pay = h_pay.numpy()
            t0 = time.perf_counter()
            assert lib.rsk_assemble_frames(n, h_hdr_out.numpy().ctypes.data, h_status.numpy().ctypes.data,
                                           pay.ctypes.data, w_pay_off.ctypes.data, fout.ctypes.data, foff.ctypes.data,
                                           16) == 0
            host["assemble_frames_Mpkt_s"] = round(n / (time.perf_counter() - t0) / 1e6, 1)
            assert np.array_equal(fout.reshape(n, fp)[:, :1431], fin.reshape(n, fp)[:, :1431]) or args.config != "c3"
    # sanity: host outputs equal the device-resident results
    assert bool((h_status == (h_len.to(torch.int32) & 0xFFFF) + 31).all())
    assert torch.equal(h_frames_out.view(n, fp)[:, :1431], h_frames_in.view(n, fp)[:, :1431]) or args.config != "c3"
    assert bool((h_dstat == 1).all())
    if "encode_hdr" in out or "both_hdr" in out:
        assert torch.equal(h_hdr_out.view(n, 32)[:, :31], h_frames_in.view(n, fp)[:, :31])
    print(json.dumps({"host_resident_Mpkt_s": out, "host_side_16_threads": host, "config": args.config, "packets": n, "chunk": C, "streams": S,
                      "pcie_bytes_per_pkt": {"encode": {"h2d": pp + 15, "d2h": fp + 4},
                                             "decode": {"h2d": fp + 2, "d2h": 1 + 4 + 8 + 4},
                                             "encode_hdr": {"h2d": 16, "d2h": 36},
                                             "decode_hdr": {"h2d": 34, "d2h": 1 + 4 + 8 + 4}}}))


if __name__ == "__main__":
    main()
