#!/usr/bin/env python3
"""k_encode on one config under several frame-arena layouts (device-resident, HIP events on the
launch stream, interleaved rounds in one process):
  slots        the workload's 16-B-aligned slots of pitch round16(31 + P_max) (bench.py's layout)
  packed16     frames back to back at 16-B granularity (frame_off = prefix sum of round16(31 + P))
  packed       frames back to back at byte granularity (most frames unaligned)
  odd_frames   the slots shifted by 5 bytes (every frame unaligned)
Payload arenas stay the workload's slots.  Every layout's frames are checked against the slots
layout's bytes (frame by frame) before timing.
    python tools/bench_layouts.py [--config c4] [--rounds 5] [--reps 10] [--pad16]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--pad16", action="store_true", help="RSK_ENC_ZERO_PAD16 (not for the byte-packed layout)")
    ap.add_argument("--probe", action="store_true",
                    help="also time tools/libhbm_probe.so probe_frames per layout: the encode's write pattern "
                         "(one wave per frame, payload chunks to the frame's chunks) with byte-exact edge "
                         "stores (exact) and with whole-chunk stores (whole)")
    ap.add_argument("--layouts", default="", help="comma list: time only these layouts (slots is always built)")
    ap.add_argument("--copy-k", type=int, default=0,
                    help="rsk__set_copy_k for the two-pass form: 1 / 2 / 4 packets per copy wave, -1 the "
                         "output-stationary copy, 0 chosen per call")
    ap.add_argument("--encode-path", type=int, default=0,
                    help="rsk_set_encode_path: 0 chosen per call, 1 per-set kernel, 2 two-pass")
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
    if args.encode_path:
        cx.set_encode_path(args.encode_path)
    if args.copy_k:
        cx.set_copy_k(args.copy_k)
    s = torch.cuda.current_stream()
    flen = d.frame_len.astype(np.int64)
    r16 = (flen + 15) // 16 * 16
    offs = {
        "slots": d.frame_off.astype(np.int64),
        "packed16": np.concatenate([[0], np.cumsum(r16)[:-1]]),
        "packed": np.concatenate([[0], np.cumsum(flen)[:-1]]),
        # shifted by 5 B; padded runs need 16 B more room per slot (the pad may not reach the next frame)
        "odd_frames": np.arange(n, dtype=np.int64) * (d.frame_pitch + (16 if args.pad16 else 0)) + 5,
    }
    if args.pad16:
        offs.pop("packed")
    arenas = {}
    for k, o in offs.items():
        size = int(o[-1]) + 1600
        arenas[k] = (torch.zeros(size, dtype=torch.uint8, device=dev), torch.from_numpy(o).to(dev),
                     torch.empty(n, dtype=torch.int32, device=dev))

    def run(k):
        fr, fo, st = arenas[k]
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, fr, fo, st,
                        id_uniform=workload.ID_UNIFORM, pad16=args.pad16, stream=s)

    for k in arenas:
        run(k)
    torch.cuda.synchronize()
    # correctness: every layout holds the slots layout's frames
    ref_fr, ref_fo, _ = arenas["slots"]
    idx = torch.arange(1600, device=dev)
    fl = torch.from_numpy(flen).to(dev)
    for k, (fr, fo, st) in arenas.items():
        for lo in range(0, n, 1 << 16):
            hi = min(n, lo + (1 << 16))
            m = idx.view(1, -1) < fl[lo:hi].view(-1, 1)
            a = fr[(fo[lo:hi].view(-1, 1) + idx.view(1, -1)).clamp(max=fr.numel() - 1)] * m
            b = ref_fr[(ref_fo[lo:hi].view(-1, 1) + idx.view(1, -1)).clamp(max=ref_fr.numel() - 1)] * m
            if not torch.equal(a, b):
                raise SystemExit(f"layout {k}: frames differ from the slots layout in [{lo}, {hi})")
    keep = args.layouts.split(",") if args.layouts else list(arenas)
    runs = {k: (lambda k=k: run(k)) for k in arenas if k in keep}
    if args.probe:
        import ctypes
        L = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhbm_probe.so"))
        L.probe_frames.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_uint64, ctypes.c_int, ctypes.c_void_p]
        sp = ctypes.c_void_p(s.cuda_stream)

        def probe(k, exact):
            fr, fo, _ = arenas[k]
            r = L.probe_frames(w.payload.data_ptr(), fr.data_ptr(), w.pay_off.data_ptr(), fo.data_ptr(),
                               w.pay_len.data_ptr(), n, exact, sp)
            assert r == 0

        for k in list(arenas):
            runs[f"probe_exact:{k}"] = (lambda k=k: probe(k, 1))
            runs[f"probe_whole:{k}"] = (lambda k=k: probe(k, 0))
    times = {k: [] for k in runs}
    for _ in range(args.rounds):
        for k, f in runs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                f()
            e1.record(s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.reps)
    alg = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
    out = {}
    for k, t in times.items():
        ms = float(np.median(t))
        out[k] = {"ms": round(ms, 4), "GBps_alg": round(alg / ms / 1e6, 1), "frac_of_8TBps": round(alg / ms / 8e9, 4)}
    print(json.dumps({"config": args.config, "packets": n, "pad16": args.pad16, "algorithmic_bytes": alg,
                      "layouts": out}))


if __name__ == "__main__":
    main()
