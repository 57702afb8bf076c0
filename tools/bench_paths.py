#!/usr/bin/env python3
"""Per-path kernel timings on one config (device-resident, HIP events, interleaved rounds in one
process): encode (framing), encode_wire RAW4 / Ethernet (framing + IPv4/TCP build + checksums),
decode (verify + compaction), parse_decode (pcap parse of the Ethernet wire packets + verify).
    python tools/bench_paths.py [--config c3] [--rounds 5] [--reps 10]"""
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
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--wire-align", type=int, default=0,
                    help="wire packet pitch alignment (bytes); 0 = the frame slot rule (128 with PAD128 for "
                         "mixed lengths, else 16)")
    ap.add_argument("--only", default="", help="time only these paths (comma list), e.g. demux,demux_64conn")
    ap.add_argument("--encode-path", type=int, default=0,
                    help="rsk_set_encode_path for the encode paths: 0 chosen per call, 1 k_encode, 2 two-pass, 3 short")
    args = ap.parse_args()
    import torch

    from rsock_amd import codec as rc
    from rsock_amd import workload

    dev = torch.device("cuda:0")
    n = args.packets or workload.CONFIGS[args.config][1]
    d = workload.describe(args.config, 0, n, n=n)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", 0)
    if args.encode_path:
        cx.set_encode_path(args.encode_path)
    cx.reserve(n)
    s = torch.cuda.current_stream()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    ri = lambda hi, dt: torch.randint(0, hi, (n,), device=dev, generator=g, dtype=torch.int64).to(dt)  # noqa: E731
    src, dst, seq, ack = ri(2**31, torch.int32), ri(2**31, torch.int32), ri(2**31, torch.int32), ri(2**31, torch.int32)
    sp, dp, ipid = ri(2**15, torch.int16) + 1, ri(2**15, torch.int16) + 1, ri(2**15, torch.int16)
    flag = torch.full((n,), 0x18, dtype=torch.uint8, device=dev)
    pmax = workload.CONFIGS[args.config][3]
    al = args.wire_align or (128 if d.pad == 128 else 16)
    wpad = dict(pad16=al != 128, pad128=al == 128)
    p4, pe = (40 + 31 + pmax + al - 1) // al * al, (54 + 31 + pmax + al - 1) // al * al
    wire4 = torch.empty(n * p4, dtype=torch.uint8, device=dev)
    wiree = torch.empty(n * pe, dtype=torch.uint8, device=dev)
    off4 = torch.arange(n, device=dev, dtype=torch.int64) * p4
    offe = torch.arange(n, device=dev, dtype=torch.int64) * pe
    st4 = torch.empty(n, dtype=torch.int32, device=dev)
    ste = torch.empty(n, dtype=torch.int32, device=dev)
    eth = bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2, 8, 0])
    tcp = rc.TcpInfoBuffers.alloc(n, dev)
    pdec = rc.DecodeBuffers.alloc(n, dev)
    common = (w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key)
    ops = {
        "encode": lambda: cx.output_batch(*common, w.frame, w.frame_off, w.status, id_uniform=workload.ID_UNIFORM,
                                          pad16=d.pad == 16, pad128=d.pad == 128, stream=s),
        "encode_wire_raw4": lambda: cx.output_wire_batch(*common, src, dst, sp, dp, seq, ack, flag, ipid, wire4, off4,
                                                         st4, id_uniform=workload.ID_UNIFORM, stream=s, **wpad),
        "encode_wire_eth": lambda: cx.output_wire_batch(*common, src, dst, sp, dp, seq, ack, flag, ipid, wiree, offe,
                                                        ste, eth=eth, id_uniform=workload.ID_UNIFORM, stream=s,
                                                        **wpad),
        # the per-set wire kernels held (round 6: AUTO takes the two-pass wire build for long frames)
        "encode_wire_raw4_perset": lambda: (cx.set_encode_path(1), cx.output_wire_batch(
            *common, src, dst, sp, dp, seq, ack, flag, ipid, wire4, off4, st4, id_uniform=workload.ID_UNIFORM,
            stream=s, **wpad), cx.set_encode_path(0)),
        "encode_wire_eth_perset": lambda: (cx.set_encode_path(1), cx.output_wire_batch(
            *common, src, dst, sp, dp, seq, ack, flag, ipid, wiree, offe, ste, eth=eth, id_uniform=workload.ID_UNIFORM,
            stream=s, **wpad), cx.set_encode_path(0)),
        "decode": lambda: cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=s),
        "parse_decode": lambda: cx.rawinput_batch(wiree, offe, ste, ste, 1, 0, tcp, pdec, stream=s),
    }
    # fake-TCP connection state: seq / IP id of a send batch over 64 connections, ack of a receive batch
    conn64 = (torch.arange(n, device=dev, dtype=torch.int64) % 64).to(torch.int32)
    cseq, cack = torch.zeros(64, dtype=torch.int32, device=dev), torch.zeros(64, dtype=torch.int32, device=dev)
    ipn = torch.zeros(1, dtype=torch.int16, device=dev)
    sq_seq, sq_ip = torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int16, device=dev)
    deliv = torch.ones(n, dtype=torch.uint8, device=dev)
    ops["tcp_send_seq"] = lambda: cx.tcp_send_seq_batch(conn64, w.status, cseq, ipn, sq_seq, sq_ip, stream=s)
    ops["tcp_send_seq_groupby"] = lambda: (cx.set_send_seq_groupby(1), cx.tcp_send_seq_batch(
        conn64, w.status, cseq, ipn, sq_seq, sq_ip, stream=s), cx.set_send_seq_groupby(0))
    ops["tcp_send_seq_scan1"] = lambda: (cx.set_send_seq_groupby(2), cx.tcp_send_seq_batch(
        conn64, w.status, cseq, ipn, sq_seq, sq_ip, stream=s), cx.set_send_seq_groupby(0))
    conn2k = (torch.arange(n, device=dev, dtype=torch.int64) * 7919 % 2047).to(torch.int32)
    cseq2k = torch.zeros(2047, dtype=torch.int32, device=dev)
    ops["tcp_send_seq_2047conn"] = lambda: cx.tcp_send_seq_batch(conn2k, w.status, cseq2k, ipn, sq_seq, sq_ip,
                                                                 stream=s)
    ops["tcp_recv_ack"] = lambda: cx.tcp_recv_ack_batch(conn64, deliv, sq_seq, cack, stream=s)
    # receive demux on the decoded fields (frames of this config; C4 marks 1/16 corrupted, 5% control)
    w.corrupt_frames()
    dmx = rc.DemuxBuffers.alloc(n, dev)
    dfields = rc._abi.DEMUX_ID | rc._abi.DEMUX_CONN_KEY | rc._abi.DEMUX_CMD_BARRIER
    # each demux shape on a context of its own: a context sizes its key table from its previous call
    # (steady traffic); one context alternating between shapes is tests/test_gpu_demux.py's business
    cx_dm = {k: rc.Codec(b"hello135", 0) for k in ("demux", "demux_64conn", "demux_server", "demux_server_group")}
    ops["demux"] = lambda: cx_dm["demux"].demux_batch(w.dec.status, w.dec.cmd, dfields, dmx, id=w.dec.id,
                                                      conv=w.dec.conv, conn_key=w.dec.conn_key, stream=s)
    # capture filter (server form) over the Ethernet wire packets: a 4M-packet capture batch
    fmatch = torch.empty(n, dtype=torch.uint8, device=dev)
    fidx = torch.empty(n, dtype=torch.int32, device=dev)
    fnm = torch.empty(1, dtype=torch.int32, device=dev)
    filt = rc.make_filter(dst_singles=[10001, 10002], dst_ranges=[(20000, 30000)], is_server=True)
    ops["capture_filter"] = lambda: cx.capture_filter_batch(wiree, offe, ste, 1, filt, fmatch, fidx, fnm, stream=s)
    tcp2, pdec2 = rc.TcpInfoBuffers.alloc(n, dev), rc.DecodeBuffers.alloc(n, dev)
    ops["filter_parse_decode"] = lambda: cx.filter_rawinput_batch(wiree, offe, ste, ste, 1, 0, filt, fmatch, tcp2,
                                                                  pdec2, stream=s)
    # header-only kernels: contiguous 32-B slots (no dependent offset load, no scattered headers)
    slots = w.frame[w.frame_off.view(-1, 1) + torch.arange(32, device=dev).view(1, -1)].reshape(-1).contiguous()
    hdec = rc.DecodeBuffers.alloc(n, dev)
    b0 = w.payload[w.pay_off].contiguous()
    hslot = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    hst = torch.empty(n, dtype=torch.int32, device=dev)
    ops["decode_hdr"] = lambda: cx.onrecv_headers_batch(slots, w.frame_len, hdec, stream=s)
    ops["encode_hdr"] = lambda: cx.output_headers_batch(b0, w.pay_len, w.cmd, w.conv, w.conn_key, hslot, hst,
                                                        id_uniform=workload.ID_UNIFORM, stream=s)
    # realistic connection counts: 64 conns, 0.1% control packets, every packet VALID
    gk = torch.Generator(device=dev)
    gk.manual_seed(7)
    k_st = torch.ones(n, dtype=torch.int8, device=dev)
    k_cmd = (torch.rand(n, device=dev, generator=gk) < 0.001).to(torch.uint8) * 3
    k_key = torch.randint(0, 64, (n,), device=dev, generator=gk, dtype=torch.int64) * 0x10001 + 0x10000000
    k_id = torch.zeros(n * 8, dtype=torch.uint8, device=dev)
    dmx64 = rc.DemuxBuffers.alloc(n, dev)
    ops["demux_64conn"] = lambda: cx_dm["demux_64conn"].demux_batch(k_st, k_cmd, dfields, dmx64, id=k_id,
                                                                    conn_key=k_key, stream=s)
    # the server's leaf key (tests/demux_ref.py): 64 clients (IdBuf, dst) x 64 convs,
    # 0.1 % control packets, every packet VALID -- 4096 SConns
    A = rc._abi
    sfields = A.DEMUX_ID | A.DEMUX_DST | A.DEMUX_CONV | A.DEMUX_CMD_BARRIER
    grp = torch.randint(0, 64, (n,), device=dev, generator=gk, dtype=torch.int64)
    s_id = torch.randint(0, 256, (64, 8), device=dev, generator=gk, dtype=torch.int64).to(torch.uint8)[grp].reshape(-1)
    s_dst = (0x0a000000 + grp).to(torch.int32)
    s_conv = torch.randint(1, 65, (n,), device=dev, generator=gk, dtype=torch.int64).to(torch.int32)
    dmxs = rc.DemuxBuffers.alloc(n, dev)
    ops["demux_server"] = lambda: cx_dm["demux_server"].demux_batch(k_st, k_cmd, sfields, dmxs, id=s_id,
                                                                    conv=s_conv, dst=s_dst, stream=s)
    # the same batch with the IdBuf-scoped barrier (RSK_DEMUX_GROUP_BARRIER: ServerGroup routes a
    # control packet to its own IdBuf's SubGroup only): two group-by passes, ~1 segment per SConn
    gfields = A.DEMUX_ID | A.DEMUX_DST | A.DEMUX_CONV | A.DEMUX_GROUP_BARRIER
    dmxg = rc.DemuxBuffers.alloc(n, dev)
    ops["demux_server_group"] = lambda: cx_dm["demux_server_group"].demux_batch(k_st, k_cmd, gfields, dmxg, id=s_id,
                                                                                conv=s_conv, dst=s_dst, stream=s)
    for k, f in ops.items():
        if k == "demux":
            cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=s)
        f()
    torch.cuda.synchronize()
    assert bool((pdec.status == 1).all()) and int(pdec.n_valid.item()) == n
    ops.pop("decode")  # decode now sees the corrupted frames; time it on them too
    ops["decode"] = lambda: cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=s)
    # syncInput hand-off records: 21-B TcpInfo (from the parse above) + the frame, one per slot
    fp = d.frame_pitch
    rp = (21 + fp + 15) // 16 * 16
    hand = torch.zeros(n * rp, dtype=torch.uint8, device=dev)
    h2 = hand.view(n, rp)
    h2[:, 21:21 + fp] = w.frame[: n * fp].view(n, fp)
    hrec = torch.empty(n * 21, dtype=torch.uint8, device=dev)
    cx.tcpinfo_encode_batch(tcp.src, tcp.dst, tcp.sp, tcp.dp, tcp.seq, tcp.ack, tcp.flag, hrec, stream=s)
    h2[:, :21] = hrec.view(n, 21)
    hoff = torch.arange(n, device=dev, dtype=torch.int64) * rp
    hlen = w.frame_len.to(torch.int32) + 21
    tcp3, sdec = rc.TcpInfoBuffers.alloc(n, dev), rc.DecodeBuffers.alloc(n, dev)
    ops["syncinput_decode"] = lambda: cx.syncinput_batch(hand, hoff, hlen, tcp3, sdec, stream=s)
    nseg = [int(dmx.n_seg.item()), int(dmx64.n_seg.item()), int(dmxs.n_seg.item()), int(dmxg.n_seg.item())]
    if args.only:
        keep = args.only.split(",")
        ops = {k: f for k, f in ops.items() if k in keep}
    times = {k: [] for k in ops}
    for _ in range(args.rounds):
        for k, f in ops.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(args.reps):
                f()
            e1.record(s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / args.reps)
    p = float(d.pay_len.astype(np.float64).mean())
    alg = {  # algorithmic bytes per packet
        "encode": 2 * p + 66,
        "encode_wire_raw4": 2 * p + 66 + 40 + 23,
        "encode_wire_eth": 2 * p + 66 + 54 + 23,
        "encode_wire_raw4_pkt": 2 * p + 66 + 40 + 23,
        "encode_wire_raw4_flat": 2 * p + 66 + 40 + 23,
        "encode_wire_raw4_hyb1": 2 * p + 66 + 40 + 23,
        "decode": 73,
        "parse_decode": 54 + 32 + 16 + 21 + 4 + 73 - 42,
        "demux": 1 + 1 + 8 + 8 + 4,  # status, cmd, id, conn_key in; perm out (+ per-segment words)
        "demux_64conn": 1 + 1 + 8 + 8 + 4,
        "demux_server": 1 + 1 + 8 + 4 + 4 + 4,  # status, cmd, id, conv, dst in; perm out
        "demux_server_group": 1 + 1 + 8 + 4 + 4 + 4,
        "capture_filter": 8 + 4 + 64 + 16 + 1 + 4,  # cap_off, cap_len, header windows, match, match_idx
        "filter_parse_decode": 8 + 4 + 64 + 16 + 1 + 54 + 32 + 16 + 21 + 4 + 73 - 42,
        "decode_hdr": 32 + 2 + 27 + 4,
        "encode_hdr": 1 + 2 + 1 + 4 + 8 + 32 + 4,
        "tcp_send_seq": 4 + 4 + 4 + 2,  # conn, status in; seq, ip_id out
        "tcp_send_seq_groupby": 4 + 4 + 4 + 2,
        "tcp_send_seq_scan1": 4 + 4 + 4 + 2,
        "tcp_send_seq_2047conn": 4 + 4 + 4 + 2,
        "tcp_recv_ack": 4 + 1 + 4,      # conn, delivered, seq in
        # record bytes [0, 53) + rec_off + nread in; TcpInfo (26) + decode fields (27) + valid_idx out
        "syncinput_decode": 53 + 8 + 4 + 26 + 27 + 4,
    }
    cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=s)
    torch.cuda.synchronize()
    if "syncinput_decode" in ops:
        assert torch.equal(sdec.status, w.dec.status) and torch.equal(sdec.n_valid, w.dec.n_valid)
    out = {}
    for k, t in times.items():
        m = float(np.median(t))
        a = alg.get(k, alg["encode_wire_eth" if "_eth_" in k else "encode_wire_raw4"])
        out[k] = {"ms": round(m, 4), "Mpkt_s": round(n / m / 1e3, 1), "GBps_alg": round(n * a / m / 1e6, 1)}
    print(json.dumps({"config": args.config, "packets": n, "wire_pitch": [p4, pe], "demux_segments": nseg,
                      "paths": out}))


if __name__ == "__main__":
    main()
