"""GPU: rsk_encode_wire_batch (RConn::Output + RawTcp::SendRawTcp / libnet build)
against the oracle, byte for byte, for both link layouts, odd payload offsets, unaligned packet
offsets (every offset r in a 16-B chunk, and packets back to back at byte granularity) and the
zero-pad modes; every packet's IPv4 and TCP checksums re-verified."""
from __future__ import annotations

import struct

import numpy as np
import pytest

from rsock_amd import workload
from tests.test_gpu_parity import dev
from tests.test_wire_oracle import py_csum

pytestmark = pytest.mark.gpu
KEY = b"hello135"


@pytest.mark.parametrize("eth", [False, True])
@pytest.mark.parametrize("layout", ["aligned", "odd_payload", "odd_wire", "any_wire", "packed_wire"])
@pytest.mark.parametrize("pad", [0, 16, 128])
@pytest.mark.parametrize("mix", ["mixed", "short", "bimodal", "long"])
# the wire build's paths, each held (rsk_set_encode_path) and asserted after the call: the per-set wire
# kernels, and the two-pass form (round 6) with 1, 2 and 4 packets per copy wave
@pytest.mark.parametrize("wpath", [(1, 0), (2, 1), (2, 2), (2, 4)], ids=["perset", "two_pass_k1", "two_pass_k2",
                                                                          "two_pass_k4"])
def test_wire_batch(codec, gpu, oracle, eth, layout, pad, mix, wpath):
    import torch

    if layout == "packed_wire" and pad:
        pytest.skip("back-to-back packets leave no room for the zero pad")
    rng = np.random.default_rng(hash((eth, layout, pad, mix)) & 0xFFFF)
    lens = [0, 1, 2, 8, 9, 10, 11, 12, 15, 16, 17, 31, 32, 33, 100, 1000, 1400, 1468, 1469, 1470] + \
        list(rng.integers(1200 if mix == "long" else 1, 1470 if mix in ("mixed", "long") else 160, 400))
    # "long": every set's mean frame >= 1024 B, so the deferred-tag copy also meets the 20 edge lengths
    if mix == "bimodal":  # short sets then long sets: both launches of the split hybrid in one batch
        lens = lens[:20] + list(rng.integers(1, 160, 236)) + list(rng.integers(1000, 1470, 200))
    n = len(lens)
    plen = np.array(lens, np.uint16)
    pitch_p = 1504
    pay_off = (np.arange(n) * pitch_p + (np.arange(n) % 13 if layout == "odd_payload" else 0)).astype(np.uint64)
    payload = rng.integers(0, 256, n * pitch_p + 64, dtype=np.uint8)
    pitch_w = 1664 if pad == 128 else 1600  # PAD128 needs every slot's padded end inside the slot
    wire_off = (np.arange(n) * pitch_w + (5 if layout == "odd_wire" else 0)).astype(np.uint64)
    if layout == "any_wire":  # every offset r = 0..15 within a 16-B chunk
        wire_off = (np.arange(n) * pitch_w + (np.arange(n) * 7) % 16).astype(np.uint64)
    elif layout == "packed_wire":  # back to back at byte granularity, 0-3 byte gaps (must survive)
        wl = np.where((plen > 0) & (plen <= 1469), (14 if eth else 0) + 40 + 31 + plen.astype(np.int64), 0)
        wire_off = np.concatenate([[3], np.cumsum(wl + rng.integers(0, 4, n))[:-1] + 3]).astype(np.uint64)
    cmd = rng.integers(0, 5, n).astype(np.uint8)
    conv = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ckey = rng.integers(0, 2**63, n, dtype=np.uint64)
    src = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    dst = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    sp = rng.integers(1, 65536, n).astype(np.uint16)
    dp = rng.integers(1, 65536, n).astype(np.uint16)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ack = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    flag = rng.integers(0, 256, n).astype(np.uint8)
    ipid = rng.integers(0, 65536, n).astype(np.uint16)
    ethb = bytes(rng.integers(0, 256, 14, dtype=np.uint8)) if eth else None
    fill = rng.integers(0, 256, n * pitch_w + 64, dtype=np.uint8)
    wire = dev(fill, gpu)
    status = torch.empty(n, dtype=torch.int32, device=gpu)
    codec.set_encode_path(wpath[0])
    codec.set_copy_k(wpath[1])
    codec.output_wire_batch(dev(payload, gpu), dev(pay_off, gpu, np.int64), dev(plen, gpu, np.int16), dev(cmd, gpu),
                            dev(conv, gpu, np.int32), dev(ckey, gpu, np.int64), dev(src, gpu, np.int32),
                            dev(dst, gpu, np.int32), dev(sp, gpu, np.int16), dev(dp, gpu, np.int16),
                            dev(seq, gpu, np.int32), dev(ack, gpu, np.int32), dev(flag, gpu), dev(ipid, gpu, np.int16),
                            wire, dev(wire_off, gpu, np.int64), status, eth=ethb, id_uniform=workload.ID_UNIFORM,
                            pad16=pad == 16, pad128=pad == 128)
    took = (codec.last_encode_path, codec.last_copy_k if wpath[0] == 2 else 0)
    codec.set_encode_path(0)
    codec.set_copy_k(0)
    assert took == wpath, f"wire build held to {wpath} ran {took}"
    torch.cuda.synchronize()
    got, st = wire.cpu().numpy(), status.cpu().numpy()
    exp = fill.copy()
    L = 14 if eth else 0
    for i in range(n):
        p = payload[int(pay_off[i]): int(pay_off[i]) + int(plen[i])].tobytes()
        fst, frame = oracle.rconn_output(KEY, p, int(cmd[i]), workload.ID_UNIFORM, int(conv[i]), int(ckey[i]))
        if fst <= 0:
            assert st[i] == fst
            continue
        w = oracle.build_wire(frame, int(src[i]), int(dst[i]), int(sp[i]), int(dp[i]), int(seq[i]), int(ack[i]),
                              int(flag[i]), int(ipid[i]), eth=ethb)
        assert st[i] == len(w), i
        o = int(wire_off[i])
        exp[o: o + len(w)] = np.frombuffer(w, np.uint8)
        if pad:
            e = o + len(w)
            exp[e: (e + pad - 1) // pad * pad] = 0
        g = got[o: o + len(w)].tobytes()
        assert py_csum(g[L: L + 20]) == 0, i                      # IPv4 header checksum verifies
        pseudo = g[L + 12: L + 20] + struct.pack("!BBH", 0, 6, len(w) - L - 20)
        assert py_csum(pseudo + g[L + 20:]) == 0, i               # TCP checksum verifies
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


def test_wire_to_parse_loop(codec, gpu):
    """Send path -> receive path on the device: Ethernet wire packets built by rsk_encode_wire_batch
    are exactly what pcap captures, so rsk_parse_decode_batch must DELIVER and verify every one and
    hand back the TcpInfo (reversed "self" view) and the EncHead fields."""
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers

    d = workload.describe("c4", 0, 20000, n=20000)
    w = workload.DeviceWorkload(d, gpu)
    n = d.n
    g = torch.Generator(device=gpu)
    g.manual_seed(5)
    ri = lambda hi, dt: torch.randint(0, hi, (n,), device=gpu, generator=g, dtype=torch.int64).to(dt)  # noqa: E731
    src, dst = ri(2**31, torch.int32), ri(2**31, torch.int32)
    sp, dp = ri(2**15, torch.int16) + 1, ri(2**15, torch.int16) + 1
    seq, ack, ipid = ri(2**31, torch.int32), ri(2**31, torch.int32), ri(2**15, torch.int16)
    flag = torch.full((n,), 0x18, dtype=torch.uint8, device=gpu)
    pitch = 1488
    wire = torch.zeros(n * pitch, dtype=torch.uint8, device=gpu)
    woff = torch.arange(n, device=gpu, dtype=torch.int64) * pitch
    st = torch.empty(n, dtype=torch.int32, device=gpu)
    eth = bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2, 8, 0])
    codec.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, src, dst, sp, dp, seq, ack,
                            flag, ipid, wire, woff, st, eth=eth, id_uniform=workload.ID_UNIFORM)
    tcp, out = TcpInfoBuffers.alloc(n, gpu), DecodeBuffers.alloc(n, gpu)
    codec.rawinput_batch(wire, woff, st, st, 1, 0, tcp, out)
    torch.cuda.synchronize()
    assert bool((tcp.parse_status == 1).all()) and bool((out.status == 1).all())
    assert int(out.n_valid.item()) == n
    assert torch.equal(tcp.src, dst) and torch.equal(tcp.dst, src)          # reversed view (RawTcp.cpp:213-216)
    assert torch.equal(tcp.sp, dp) and torch.equal(tcp.dp, sp)
    plen = (w.pay_len.to(torch.int64) & 0xFFFF) + 31
    assert torch.equal((tcp.seq.to(torch.int64) & 0xFFFFFFFF), ((seq.to(torch.int64) & 0xFFFFFFFF) + plen) & 0xFFFFFFFF)
    assert torch.equal(tcp.cap_pay_off.to(torch.int64), torch.full_like(plen, 54))
    assert torch.equal(out.conv, w.conv) and torch.equal(out.conn_key, w.conn_key) and torch.equal(out.cmd, w.cmd)
    assert torch.equal(out.pay_len.to(torch.int64) & 0xFFFF, plen - 31)


@pytest.mark.parametrize("eth", [False, True])
def test_wire_two_pass_chunks_equal_per_set(codec, gpu, eth):
    """The two-pass wire build runs its header pass and copy per chunk of 2^20 packets (records stay in
    the Infinity Cache): a batch of 2^20 + 4097 C4 packets (two chunks, the second ragged) built on the
    two-pass path with 1, 2 and 4 packets per copy wave equals the per-set kernels' packets byte for
    byte, and every status is the wire length."""
    import torch

    n = (1 << 20) + 4097
    d = workload.describe("c4", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    g = torch.Generator(device=gpu)
    g.manual_seed(9)
    ri = lambda hi, dt: torch.randint(0, hi, (n,), device=gpu, generator=g, dtype=torch.int64).to(dt)  # noqa: E731
    fields = [ri(2**31, torch.int32), ri(2**31, torch.int32), ri(2**15, torch.int16) + 1, ri(2**15, torch.int16) + 1,
              ri(2**31, torch.int32), ri(2**31, torch.int32), ri(256, torch.uint8), ri(2**15, torch.int16)]
    pitch = 1536
    woff = torch.arange(n, device=gpu, dtype=torch.int64) * pitch
    ethb = bytes(range(14)) if eth else None
    outs = {}
    try:
        for path, k in [(1, 0), (2, 1), (2, 2), (2, 4)]:
            codec.set_encode_path(path)
            codec.set_copy_k(k)
            wire = torch.zeros(n * pitch, dtype=torch.uint8, device=gpu)
            st = torch.empty(n, dtype=torch.int32, device=gpu)
            codec.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, *fields, wire, woff, st,
                                    eth=ethb, id_uniform=workload.ID_UNIFORM, pad128=True)
            assert codec.last_encode_path == path
            torch.cuda.synchronize()
            outs[(path, k)] = (wire, st)
            if path == 2:
                ref_w, ref_s = outs[(1, 0)]
                assert torch.equal(st, ref_s), (path, k)
                assert torch.equal(wire, ref_w), (path, k)
                del outs[(path, k)]
        plen = w.pay_len.to(torch.int64) & 0xFFFF
        exp = torch.where((plen >= 1) & (plen <= 1469), plen + 31 + 40 + (14 if eth else 0), outs[(1, 0)][1].to(torch.int64))
        assert torch.equal(outs[(1, 0)][1].to(torch.int64), exp)
    finally:
        codec.set_encode_path(0)
        codec.set_copy_k(0)


@pytest.mark.parametrize("cfg,eth,exp", [("c4", False, (2, 4)), ("c4", True, (2, 4)), ("c3", False, (2, 2)),
                                          ("c3", True, (1, 0)), ("c2", False, (1, 0)), ("c2", True, (1, 0))])
def test_wire_auto_path(gpu, cfg, eth, exp):
    """AUTO's wire table (rsk_kernels.hip wire_path / wire_k, profiles/r06_wire_paths.json): the per-set
    wire kernels for short frames (C2) and for Ethernet packets of 1400-B payloads (C3), the two-pass
    form with 4 packets per copy wave for mid-length frames (C4) and 2 for RAW4 packets of 1400 B --
    from a fresh context's first call (it samples its own batch) on."""
    import torch

    from rsock_amd.codec import Codec

    n = 40_000
    d = workload.describe(cfg, 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    z = lambda dt: torch.ones(n, dtype=dt, device=gpu)  # noqa: E731
    pitch = 1536
    wire = torch.zeros(n * pitch, dtype=torch.uint8, device=gpu)
    woff = torch.arange(n, device=gpu, dtype=torch.int64) * pitch
    st = torch.empty(n, dtype=torch.int32, device=gpu)
    cx = Codec(KEY, 0)
    s = torch.cuda.Stream(gpu)  # (on the legacy NULL stream a fresh context's first call does not wait)
    torch.cuda.synchronize()
    try:
        for _ in range(2):
            cx.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, z(torch.int32),
                                 z(torch.int32), z(torch.int16), z(torch.int16), z(torch.int32), z(torch.int32),
                                 z(torch.uint8), z(torch.int16), wire, woff, st, eth=bytes(14) if eth else None,
                                 id_uniform=workload.ID_UNIFORM, pad128=True, stream=s)
            got = (cx.last_encode_path, cx.last_copy_k if cx.last_encode_path == 2 else 0)
            assert got == exp, (cfg, eth, got)
        torch.cuda.synchronize()
    finally:
        cx.close()
