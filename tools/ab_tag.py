#!/usr/bin/env python3
"""A/B of the tag computation on k_encode and k_decode (interleaved rounds in one process):
   python tools/ab_tag.py [--config c3] [--rounds 10] [--reps 10] [--modes md5,table]
With the shipped library (default RSK_LIB=librsk.so): md5 = RSK_TAG_MD5 (MD5 per lane, round
constants as instruction immediates: the headline), table = RSK_TAG_TABLE (the key's 256 tags staged
in LDS, one ds_read_b64 per packet).  With RSK_LIB=librsk_md5lds.so (make -C rsock_amd md5lds), md5 = the MD5
per lane with its 64 round constants read from an LDS copy staged per block (the north star's "MD5
round constants ... staged in LDS"); run the two libraries back to back in separate processes.
Checks that every mode's frame arena and decode outputs are byte-identical, then prints per-mode
median / min kernel ms and the encode's fraction of 8 TB/s (algorithmic bytes)."""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--packets", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--modes", default="md5,table")
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
    modes = args.modes.split(",")
    s = torch.cuda.current_stream()

    def enc():
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM, pad16=d.pad == 16, pad128=d.pad == 128, stream=s)

    def dec():
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=s)

    ref = None
    for m in modes:  # correctness: identical frames and decode outputs in every mode
        cx.set_tag_mode(m)
        w.frame.zero_()
        enc()
        dec()
        torch.cuda.synchronize()
        h = (w.frame.clone(), w.dec.status.clone(), w.dec.conn_key.clone(), w.dec.valid_idx.clone(),
             w.dec.n_valid.clone())
        if ref is None:
            ref = h
        elif not all(torch.equal(a, b) for a, b in zip(ref, h)):
            raise SystemExit(f"tag mode {m}: outputs differ from mode {modes[0]}")
    del ref
    times = {(m, k): [] for m in modes for k in ("enc", "dec")}
    for _ in range(args.rounds):
        for m in modes:
            cx.set_tag_mode(m)
            for k, fn in (("enc", enc), ("dec", dec)):
                fn()
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(s)
                for _ in range(args.reps):
                    fn()
                ev[1].record(s)
                torch.cuda.synchronize()
                times[(m, k)].append(ev[0].elapsed_time(ev[1]) / args.reps)
    byts = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
    lib = os.path.basename(rc._abi.LIB_PATH)
    names = {"md5": "md5_consts_in_lds" if "md5lds" in lib else "md5_immediates", "table": "tag_table_lds"}
    out = {}
    for m in modes:
        te, td = np.array(times[(m, "enc")]), np.array(times[(m, "dec")])
        out[names.get(m, str(m))] = {
            "k_encode_median_ms": round(float(np.median(te)), 4), "k_encode_min_ms": round(float(te.min()), 4),
            "k_encode_frac": round(byts / (np.median(te) * 1e-3) / 1e9 / 8000.0, 4),
            "decode_median_ms": round(float(np.median(td)), 4), "decode_min_ms": round(float(td.min()), 4)}
    print(json.dumps({"config": args.config, "lib": lib, "packets": d.n, "frame_pitch": d.frame_pitch, "modes": out}))


if __name__ == "__main__":
    main()
