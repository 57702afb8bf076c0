"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit-exact.

Sizes here are what the oracle finishes in seconds; the full BASELINE sizes are covered by
size-independent properties in test_gpu_fullsize.py.
"""
from __future__ import annotations

import zlib

import numpy as np
import pytest

from rsock_amd import workload
from tests import pkt as P
from tests.enc_paths import ENC_PATHS, held, path_id

pytestmark = pytest.mark.gpu

KEY = b"hello135"


def dev(a: np.ndarray, gpu, dt=None):
    import torch

    a = np.ascontiguousarray(a)
    if dt is not None:
        a = a.view(dt)
    return torch.from_numpy(a.copy()).to(gpu)


def run_encode(codec, gpu, payload, pay_off, pay_len, cmd, conv, ckey, frame_off, frame_bytes,
               idarr=None, id_uniform=workload.ID_UNIFORM, frame_init=None, pad16=False, pad128=False):
    import torch

    n = len(pay_len)
    frame = (torch.zeros(frame_bytes, dtype=torch.uint8, device=gpu) if frame_init is None
             else dev(frame_init, gpu))
    status = torch.empty(n, dtype=torch.int32, device=gpu)
    codec.output_batch(dev(payload, gpu), dev(pay_off.astype(np.uint64), gpu, np.int64),
                       dev(pay_len.astype(np.uint16), gpu, np.int16), dev(cmd.astype(np.uint8), gpu),
                       dev(conv.astype(np.uint32), gpu, np.int32), dev(ckey.astype(np.uint64), gpu, np.int64),
                       frame, dev(frame_off.astype(np.uint64), gpu, np.int64), status,
                       id=None if idarr is None else dev(idarr, gpu), id_uniform=id_uniform, pad16=pad16,
                       pad128=pad128)
    torch.cuda.synchronize()
    return frame.cpu().numpy(), status.cpu().numpy()


def run_decode(codec, gpu, frames, frame_off, frame_len, close=None):
    import torch

    from rsock_amd.codec import DecodeBuffers

    n = len(frame_len)
    out = DecodeBuffers.alloc(n, gpu)
    codec.onrecv_batch(dev(frames, gpu), dev(frame_off.astype(np.uint64), gpu, np.int64),
                       dev(frame_len.astype(np.uint16), gpu, np.int16), out,
                       is_tcp_close=None if close is None else dev(close.astype(np.uint8), gpu))
    torch.cuda.synchronize()
    return out.to_host()


DEC_VIEWS = {"hlen": np.uint8, "cmd": np.uint8, "id": np.uint8, "conv": np.uint32, "conn_key": np.uint64,
             "pay_off": np.uint16, "pay_len": np.uint16, "status": np.int8}


def assert_dec_equal(got: dict, exp: dict):
    for k, dt in DEC_VIEWS.items():
        g = got[k].view(dt)
        bad = np.nonzero(g != exp[k])[0]
        assert bad.size == 0, f"field {k}: {bad.size} mismatches, first at {bad[:5]}: got {g[bad[:5]]} exp {exp[k][bad[:5]]}"
    nv = int(got["n_valid"][0])
    assert nv == exp["n_valid"]
    assert np.array_equal(got["valid_idx"][:nv].view(np.uint32), exp["valid_idx"][:nv])


# ---- configs (reduced n) ----------------------------------------------------------------------
# the last three sizes are past two super-blocks (65,536 packets each) and end in a partial one, so
# k_encode's last waves own fewer than 64 packets: C3 / C4 long-frame sets, C2 flat sets, C4 both
@pytest.mark.parametrize("cfg,n", [("c2", 100_000), ("c3", 20_000), ("c4", 50_000),
                                   ("c3", 170_001), ("c4", 196_613), ("c2", 200_003)])
def test_config_roundtrip_bitexact(vcodec, gpu, oracle, cfg, n):
    codec = vcodec
    d = workload.describe(cfg, 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM)
    w.corrupt_frames()
    codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec)
    import torch

    torch.cuda.synchronize()
    payload = w.payload.cpu().numpy()
    assert np.array_equal(payload, workload.payload_bytes_np(d)), "device payload generator != host generator"
    exp_frames, exp_status = oracle.encode_batch(KEY, payload, d, workload.ID_UNIFORM)
    assert np.array_equal(w.status.cpu().numpy(), exp_status)
    for i in np.nonzero(d.corrupt)[0]:
        exp_frames[int(d.frame_off[i])] ^= 1
    got_frames = w.frame.cpu().numpy()
    bad = np.nonzero(got_frames != exp_frames)[0]
    assert bad.size == 0, f"{bad.size} frame bytes differ, first at {bad[:8]}"
    exp = oracle.decode_batch(KEY, exp_frames, d.frame_off, d.frame_len)
    assert_dec_equal(w.dec.to_host(), exp)
    if cfg == "c4":
        assert exp["n_valid"] == n - int(d.corrupt.sum())


# ---- encode edge cases --------------------------------------------------------------------------
def _rand_fields(rng, n):
    return (rng.integers(0, 5, n).astype(np.uint8), rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
            rng.integers(0, 2**63, n, dtype=np.uint64) * 2 + rng.integers(0, 2, n, dtype=np.uint64))


@pytest.fixture(params=ENC_PATHS, ids=path_id)
def vcodec(request, codec):
    """The codec held to one encode path (tests/enc_paths.py): each encode asserts the path it took."""
    with held(codec, *request.param) as c:
        yield c


@pytest.mark.parametrize("layout,pad", [("slots16", 0), ("packed", 0), ("odd_frames", 0), ("odd_payloads", 0),
                                        ("slots16", 16), ("odd_frames", 16), ("odd_payloads", 16),
                                        ("slots16", 128), ("odd_frames", 128)])
def test_encode_edge_lengths_and_layouts(vcodec, gpu, oracle, layout, pad):
    codec = vcodec
    rng = np.random.default_rng(7)
    lens = [0, 1, 2, 3, 4, 7, 8, 15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 1000, 1023, 1024, 1025, 1400,
            1468, 1469, 1470, 1500, 4000, 65535]
    lens += list(rng.integers(1, 1470, 300))
    n = len(lens)
    plen = np.array(lens, np.uint32)
    pay_cap = np.minimum(plen, 1500)
    # payload layout
    if layout == "odd_payloads":
        pay_off = np.cumsum(np.concatenate([[3], pay_cap[:-1] + 1 + rng.integers(0, 5, n - 1)])).astype(np.uint64)
    else:
        pay_off = (np.arange(n) * 1504).astype(np.uint64)
    payload = rng.integers(0, 256, int(pay_off[-1]) + 1600, dtype=np.uint8)
    # frame layout
    flen = np.where((plen >= 1) & (plen <= 1469), plen + 31, 0).astype(np.uint64)
    if layout == "packed":
        frame_off = np.concatenate([[0], np.cumsum(flen)[:-1]]).astype(np.uint64)
    elif layout == "odd_frames":
        # pad16's contract: bytes up to the 16-B boundary after a frame belong to no other frame,
        # so padded runs need a gap >= 15 B after the longest (1500-B) frame
        frame_off = (np.arange(n) * {0: 1509, 16: 1521, 128: 1664}[pad] + 5).astype(np.uint64)
    else:
        frame_off = (np.arange(n) * (1664 if pad == 128 else 1504)).astype(np.uint64)
    frame_bytes = int(frame_off[-1]) + 1600
    cmd, conv, ckey = _rand_fields(rng, n)
    # pay_len is u16 in the ABI: 65535 stays representable, oversize statuses must come back -1
    pl16 = np.minimum(plen, 65535).astype(np.uint16)

    class D:  # minimal descriptor for the oracle batch helper
        pass

    d = D()
    d.n, d.pay_off, d.pay_len, d.cmd, d.conv, d.conn_key, d.frame_off = n, pay_off, pl16, cmd, conv, ckey, frame_off
    fill = rng.integers(0, 256, frame_bytes, dtype=np.uint8)  # pre-existing bytes must survive
    exp_frames = fill.copy()
    got_frames, got_status = run_encode(codec, gpu, payload, pay_off, pl16, cmd, conv, ckey, frame_off,
                                        frame_bytes, frame_init=fill, pad16=pad == 16, pad128=pad == 128)
    ef, es = oracle.encode_batch(KEY, payload, d, workload.ID_UNIFORM, frame_bytes=frame_bytes)
    assert np.array_equal(got_status, es)
    for i in range(n):
        if es[i] > 0:
            o = int(frame_off[i])
            exp_frames[o:o + es[i]] = ef[o:o + es[i]]
            if pad:  # RSK_ENC_ZERO_PAD16/128: zeros up to the next pad boundary (arena is 256-B aligned)
                e = o + int(es[i])
                exp_frames[e:(e + pad - 1) // pad * pad] = 0
    bad = np.nonzero(got_frames != exp_frames)[0]
    assert bad.size == 0, f"{layout}: {bad.size} bytes differ, first at {bad[:8]}"


def test_encode_per_packet_ids(vcodec, gpu, oracle):
    codec = vcodec
    rng = np.random.default_rng(11)
    n = 777
    plen = rng.integers(1, 1470, n).astype(np.uint16)
    pay_off = (np.arange(n) * 1472).astype(np.uint64)
    frame_off = (np.arange(n) * 1504).astype(np.uint64)
    payload = rng.integers(0, 256, n * 1472 + 64, dtype=np.uint8)
    cmd, conv, ckey = _rand_fields(rng, n)
    ids = rng.integers(0, 256, 8 * n, dtype=np.uint8)
    got_frames, got_status = run_encode(codec, gpu, payload, pay_off, plen, cmd, conv, ckey, frame_off,
                                        n * 1504 + 64, idarr=ids)

    class D:
        pass

    d = D()
    d.n, d.pay_off, d.pay_len, d.cmd, d.conv, d.conn_key, d.frame_off = n, pay_off, plen, cmd, conv, ckey, frame_off
    ef, es = oracle.encode_batch(KEY, payload, d, b"\0" * 8, frame_bytes=n * 1504 + 64, idarr=ids)
    assert np.array_equal(got_status, es)
    assert np.array_equal(got_frames, ef)


# ---- decode edge cases --------------------------------------------------------------------------
def _edge_frames(oracle, rng):
    frames = []
    close = []
    for ln in (0, 1, 8, 22, 23, 24, 30, 100, 255):  # EncHead len byte variants
        for extra in (0, 1, 2, 50):
            st, f = oracle.rconn_output(KEY, bytes(rng.integers(0, 256, 40, dtype=np.uint8)), 0, b"abcdefgh", 5, 9)
            f = bytearray(f)
            f[8] = ln
            body = bytes(f[:31]) + bytes(rng.integers(0, 256, extra + max(0, ln - 23), dtype=np.uint8))
            # re-tag for the byte the decoder will hash (so len-shifted frames can verify)
            nread = len(body)
            if 8 + ln < nread:
                body = oracle.tag(KEY, body[8 + ln]) + body[8:]
            frames.append(body)
            close.append(False)
    for nread in (0, 1, 8, 30, 31, 32, 33):
        for c in (False, True):
            st, f = oracle.rconn_output(KEY, bytes(rng.integers(0, 256, 10, dtype=np.uint8)), 2, b"zzzzzzzz", 1, 2)
            frames.append(f[:nread])
            close.append(c)
    for k in range(200):  # random valid / corrupted / truncated frames
        p = bytes(rng.integers(0, 256, int(rng.integers(1, 1470)), dtype=np.uint8))
        st, f = oracle.rconn_output(KEY, p, int(rng.integers(0, 5)), bytes(rng.integers(0, 256, 8, dtype=np.uint8)),
                                    int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)))
        f = bytearray(f)
        m = k % 5
        if m == 1:
            f[int(rng.integers(0, 8))] ^= 1 << int(rng.integers(0, 8))  # corrupt tag
        elif m == 2:
            f[31] ^= 0x40  # corrupt payload[0]
        elif m == 3:
            f[-1] ^= 0xFF  # corrupt the last byte: still verifies (only payload[0] is hashed)
        elif m == 4:
            f = f[: int(rng.integers(0, len(f) + 1))]
        frames.append(bytes(f))
        close.append(bool(k & 1))
    return frames, np.array(close, np.uint8)


@pytest.mark.parametrize("align", [16, 1, 4])
def test_decode_edge_cases(codec, gpu, oracle, align):
    rng = np.random.default_rng(3)
    frames, close = _edge_frames(oracle, rng)
    arena, offs, lens = P.pack_records(frames, align=align, base_pad=0 if align == 16 else 3)
    got = run_decode(codec, gpu, arena, offs, lens.astype(np.uint16), close)
    exp = oracle.decode_batch(KEY, arena, offs, lens, close)
    assert_dec_equal(got, exp)
    # spot-check semantics: truncated frames (<=31) with close flag -> CLOSE, else DROP
    st = got["status"].view(np.int8)
    for i, f in enumerate(frames):
        if len(f) <= 31:
            assert st[i] == (0 if close[i] else -1)


def test_all_first_bytes(codec, gpu, oracle):
    """Tags for every payload[0] value (there are only 256 per key)."""
    n = 256
    payload = np.arange(256, dtype=np.uint8).repeat(16)
    pay_off = (np.arange(n) * 16).astype(np.uint64)
    plen = np.full(n, 16, np.uint16)
    frame_off = (np.arange(n) * 48).astype(np.uint64)
    z = np.zeros(n, np.uint8)
    fr, st = run_encode(codec, gpu, payload, pay_off, plen, z, z.astype(np.uint32), z.astype(np.uint64),
                        frame_off, n * 48)
    for b in range(256):
        assert fr[b * 48: b * 48 + 8].tobytes() == oracle.tag(KEY, b)


def test_tag_tables_per_context(gpu, oracle, tag_mode):
    """Each context frames with its own key (schedule and tag table), with several contexts alive at
    once, and a context whose mode differs from the others' in the middle."""
    from rsock_amd.codec import Codec

    keys = [b"", b"k", b"hello135", bytes(range(60)), bytes(range(100, 230))]
    other = "table" if tag_mode == "md5" else "md5"
    cxs = [Codec(k, 0, tag_mode=other if j == 2 else tag_mode) for j, k in enumerate(keys)]
    try:
        n = 256
        payload = np.arange(256, dtype=np.uint8).repeat(16)
        pay_off = (np.arange(n) * 16).astype(np.uint64)
        plen = np.full(n, 16, np.uint16)
        frame_off = (np.arange(n) * 48).astype(np.uint64)
        z = np.zeros(n, np.uint8)
        for k, cx in reversed(list(zip(keys, cxs))):
            fr, _ = run_encode(cx, gpu, payload, pay_off, plen, z, z.astype(np.uint32), z.astype(np.uint64),
                               frame_off, n * 48)
            for b in (0, 1, 127, 128, 255):
                assert fr[b * 48: b * 48 + 8].tobytes() == oracle.tag(k, b)
    finally:
        for cx in cxs:
            cx.close()


@pytest.mark.parametrize("klen", [0, 1, 7, 8, 9, 53, 54, 55, 56, 62, 63, 64, 65, 100, 118, 119, 120, 127, 128, 200])
def test_key_lengths(gpu, oracle, klen, tag_mode):
    """1-block, 2-block and midstate key schedules (util/rhash.cpp hashes key || payload[0])."""
    from rsock_amd.codec import Codec

    key = bytes((np.arange(klen) * 37 + 11) % 256) if klen else b""
    cx = Codec(key, 0, tag_mode=tag_mode)
    try:
        n = 300
        rng = np.random.default_rng(klen)
        plen = rng.integers(1, 200, n).astype(np.uint16)
        pay_off = (np.arange(n) * 208).astype(np.uint64)
        frame_off = (np.arange(n) * 240).astype(np.uint64)
        payload = rng.integers(0, 256, n * 208, dtype=np.uint8)
        payload[pay_off.astype(np.int64)] = np.arange(n) % 256  # every tag-table entry of this key
        cmd, conv, ckey = _rand_fields(rng, n)
        fr, st = run_encode(cx, gpu, payload, pay_off, plen, cmd, conv, ckey, frame_off, n * 240)

        class D:
            pass

        d = D()
        d.n, d.pay_off, d.pay_len, d.cmd, d.conv, d.conn_key, d.frame_off = n, pay_off, plen, cmd, conv, ckey, frame_off
        ef, es = oracle.encode_batch(key, payload, d, workload.ID_UNIFORM, frame_bytes=n * 240)
        assert np.array_equal(st, es) and np.array_equal(fr, ef)
        got = run_decode(cx, gpu, fr, frame_off, (plen + 31).astype(np.uint16))
        assert_dec_equal(got, oracle.decode_batch(key, ef, frame_off, (plen + 31).astype(np.uint16)))
        assert int(got["n_valid"][0]) == n
    finally:
        cx.close()


# ---- parse + decode -----------------------------------------------------------------------------
def _parse_cases(oracle, rng):
    pk = []
    meta = []  # (wire_len, cap_len)
    src, dst = "10.0.0.1", "10.0.0.2"

    def frame(plen=40, cmd=0):
        st, f = oracle.rconn_output(KEY, bytes(rng.integers(0, 256, plen, dtype=np.uint8)), cmd, b"abcdefgh",
                                    int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)))
        return f

    add = lambda p, wl=None, cl=None: (pk.append(p), meta.append((len(p) if wl is None else wl, len(p) if cl is None else cl)))  # noqa: E731
    for dl in (1, 0):
        for ihl in (5, 6, 15):
            for thl in (5, 8, 15):
                for flags in (0x18, 0x10, 0x11, 0x14, 0x02, 0x12):
                    add(P.ipv4_tcp(src, 10001, dst, 43932, 256, 512, flags, frame(int(rng.integers(1, 300))),
                                   ihl, thl, datalink=dl))
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(1400), datalink=dl))  # 1431-B frame
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(1437), datalink=dl))  # payload_len 1468 (max)
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(1438), datalink=dl))  # 1469 -> cap2uv drop
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, b"x" * 8, datalink=dl))   # payload < 9 -> drop
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x11, b"x" * 8, datalink=dl))   # FIN small -> deliver/close
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x04, b"", datalink=dl))        # RST empty (44/54 B)
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x14, b"", ip_len=30, datalink=dl))  # negative payload_len
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x14, b"", ip_len=5, datalink=dl))   # < -32 -> drop
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(50), proto=17, datalink=dl))  # UDP -> drop
        add(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(50), datalink=dl, ethertype=0x86DD, null_family=24))
        p = P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(50), datalink=dl)
        add(p, wl=43)                       # wire len < 44 -> drop
        add(p, cl=30)                       # truncated capture -> malformed
        add(p, cl=len(p) - 5)               # payload runs past cap_len -> malformed
        add(p, wl=len(p) + 1000)            # wire_len > cap (snaplen) but payload present
        bad = bytearray(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(60), datalink=dl))
        bad[-5] ^= 1
        add(bytes(bad))
        bad = bytearray(P.ipv4_tcp(src, 1, dst, 2, 3, 4, 0x10, frame(60), datalink=dl))
        bad[-60 - 31] ^= 1                  # tag byte
        add(bytes(bad))
    return pk, meta


@pytest.mark.parametrize("flags", [0, 1, 3])
@pytest.mark.parametrize("align", [1, 16])
def test_parse_decode(codec, gpu, oracle, flags, align):
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers

    rng = np.random.default_rng(5)
    pk, meta = _parse_cases(oracle, rng)
    for dl in (1, 0):
        sel = [i for i, p in enumerate(pk) if (p[12:14] in (b"\x08\x00", b"\x86\xdd")) == (dl == 1)]
        recs = [pk[i] for i in sel]
        wl = np.array([meta[i][0] for i in sel], np.uint32)
        cl = np.array([meta[i][1] for i in sel], np.uint32)
        arena, offs, _ = P.pack_records(recs, align=align, base_pad=0 if align == 16 else 1)
        n = len(recs)
        tcp = TcpInfoBuffers.alloc(n, gpu)
        out = DecodeBuffers.alloc(n, gpu)
        codec.rawinput_batch(dev(arena, gpu), dev(offs, gpu, np.int64), dev(wl, gpu, np.int32),
                             dev(cl, gpu, np.int32), dl, flags, tcp, out)
        torch.cuda.synchronize()
        exp = oracle.parse_decode_batch(KEY, arena, offs, wl, cl, dl, flags)
        th = tcp.to_host()
        for k, dt in (("src", np.uint32), ("dst", np.uint32), ("sp", np.uint16), ("dp", np.uint16),
                      ("seq", np.uint32), ("ack", np.uint32), ("flag", np.uint8), ("parse_status", np.int8),
                      ("cap_pay_off", np.uint16), ("cap_pay_len", np.uint16)):
            assert np.array_equal(th[k].view(dt), exp[k]), (dl, k, th[k].view(dt), exp[k])
        assert_dec_equal(out.to_host(), exp)
        assert (exp["parse_status"] == 1).any() and (exp["status"] == 1).any()


def test_tcpinfo_records(codec, gpu, oracle):
    import torch

    from tests.oracle_lib import OrcTcpInfo

    rng = np.random.default_rng(9)
    for n in (1, 255, 256, 257, 1000):
        f = {k: rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) for k in ("src", "dst", "seq", "ack")}
        sp = rng.integers(0, 65536, n).astype(np.uint16)
        dp = rng.integers(0, 65536, n).astype(np.uint16)
        fl = rng.integers(0, 256, n).astype(np.uint8)
        rec = torch.zeros(21 * n + 5, dtype=torch.uint8, device=gpu)
        codec.tcpinfo_encode_batch(dev(f["src"], gpu, np.int32), dev(f["dst"], gpu, np.int32), dev(sp, gpu, np.int16),
                                   dev(dp, gpu, np.int16), dev(f["seq"], gpu, np.int32), dev(f["ack"], gpu, np.int32),
                                   dev(fl, gpu), rec)
        got = rec.cpu().numpy()
        for i in range(n):
            t = OrcTcpInfo(int(f["src"][i]), int(f["dst"][i]), int(sp[i]), int(dp[i]), int(f["seq"][i]),
                           int(f["ack"][i]), int(fl[i]), 0, 0, 0)
            assert got[21 * i: 21 * i + 21].tobytes() == oracle.tcpinfo_encode(t)
        assert not got[21 * n:].any()


# ---- single-call shims with the reference signatures ---------------------------------------------
def test_shims(codec, oracle):
    for b in (0, 3, 0x68, 0xFF):
        assert codec.compute_hash(bytes([b, 1, 2])) == oracle.tag(KEY, b)
        assert codec.hash_equal(oracle.tag(KEY, b), bytes([b]))
        assert not codec.hash_equal(oracle.tag(KEY, b ^ 1), bytes([b]))
    assert codec.compute_hash(b"") is None
    assert not codec.hash_equal(oracle.tag(KEY, 0), b"")
    h = codec.enc2buf(3, b"abcdefgh", 0xDEADBEEF, 0x0123456789ABCDEF)
    assert h == oracle.enchead_encode(1492, 3, b"abcdefgh", 0xDEADBEEF, 0x0123456789ABCDEF)
    assert codec.enc2buf(3, b"abcdefgh", 1, 2, buf_len=22) is None
    assert codec.decodebuf(h) == oracle.enchead_decode(h, 23)
    hb = bytes([200]) + h[1:]
    assert codec.decodebuf(hb, 100) is None and oracle.enchead_decode(hb, 100) is None
    assert codec.decodebuf(hb, 200) == oracle.enchead_decode(hb, 200)
    assert codec.decodebuf(h, 22) is None


# ---- parse + decode on host-staged header slots (rsk_parse_decode_slots_batch) -------------------
def _slot_short(p, wl, cl, dl, slot, flags):
    """The kernel's RSK_PARSE_SLOT_SHORT rule restated over the reference's parse order
    (RawTcp.cpp:138-244): True when the whole-capture path would read a byte past the slot."""
    av = min(cl, slot)
    L = 14 if dl == 1 else 4
    if wl < 44 or cl < L:
        return False
    if dl == 1 and p[12:14] != b"\x08\x00":
        return False
    if dl == 0 and int.from_bytes(p[0:4], "little") != 2:
        return False
    if cl < L + 20 or p[L + 9] != 6:
        return False
    ihl = (p[L] & 15) * 4
    tcpo = L + ihl
    if cl < tcpo + 20:
        return False
    if ihl != 20 and tcpo + 16 > av:
        return True
    thl = (p[tcpo + 12] >> 4) * 4
    payo = tcpo + thl
    plen = int.from_bytes(p[L + 2:L + 4], "big") - (ihl + thl)
    fl = p[tcpo + 13]
    if (fl & 0x02) and (flags & 1):
        return False
    close = (fl & 0x05) != 0
    if (plen < 9 and not close) or plen < 0 or plen + 32 > 1500 or payo + plen > cl:
        return False
    if plen > 31:
        if payo + 32 > av:
            return True
        ln = p[payo + 8]
        if ln != 23 and ln < plen - 8 and payo + 9 + ln > av:
            return True
    return False


@pytest.mark.parametrize("slot", [64, 96, 128, 2048])
@pytest.mark.parametrize("flags", [0, 3])
def test_parse_decode_slots(codec, gpu, oracle, slot, flags):
    """Host-resident receive: slots of the first min(cap_len, slot) bytes give the whole-capture
    outputs (oracle) for every packet whose parse/decode stays inside its slot, and SLOT_SHORT with
    zero outputs exactly for the others; rsock's own packets (IHL 5, data offset 5, len 23) fit 96 B."""
    import torch

    from rsock_amd import _abi
    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers, stage_capture_slots

    rng = np.random.default_rng(5)
    pk, meta = _parse_cases(oracle, rng)
    # a len-byte variant whose hashed byte sits past 96 B (must come back SLOT_SHORT at small slots)
    st, f = oracle.rconn_output(KEY, bytes(rng.integers(0, 256, 200, dtype=np.uint8)), 0, b"abcdefgh", 1, 2)
    f = bytearray(f)
    f[8] = 100
    f[:8] = oracle.tag(KEY, f[8 + 100])
    p = P.ipv4_tcp("10.0.0.1", 1, "10.0.0.2", 2, 3, 4, 0x18, bytes(f))
    pk.append(p)
    meta.append((len(p), len(p)))
    for dl in (1, 0):
        sel = [i for i, p in enumerate(pk) if (p[12:14] in (b"\x08\x00", b"\x86\xdd")) == (dl == 1)]
        recs = [pk[i] for i in sel]
        wl = np.array([meta[i][0] for i in sel], np.uint32)
        cl = np.array([meta[i][1] for i in sel], np.uint32)
        arena, offs, _ = P.pack_records(recs, align=16)
        n = len(recs)
        slots = stage_capture_slots(arena, offs, cl, slot)
        tcp = TcpInfoBuffers.alloc(n, gpu)
        out = DecodeBuffers.alloc(n, gpu)
        codec.rawinput_slots_batch(dev(slots.reshape(-1), gpu), slot, dev(wl, gpu, np.int32), dev(cl, gpu, np.int32),
                                   dl, flags, tcp, out)
        torch.cuda.synchronize()
        exp = oracle.parse_decode_batch(KEY, arena, offs, wl, cl, dl, flags)
        short = np.array([_slot_short(r, int(w_), int(c_), dl, slot, flags) for r, w_, c_ in zip(recs, wl, cl)])
        th = tcp.to_host()
        ps = th["parse_status"].view(np.int8)
        assert np.array_equal(ps == _abi.PARSE_SLOT_SHORT, short), (slot, dl, np.nonzero((ps == 4) != short))
        if slot >= 2048:
            assert not short.any()
        keep = ~short
        for k, dt in (("src", np.uint32), ("dst", np.uint32), ("sp", np.uint16), ("dp", np.uint16),
                      ("seq", np.uint32), ("ack", np.uint32), ("flag", np.uint8), ("parse_status", np.int8),
                      ("cap_pay_off", np.uint16), ("cap_pay_len", np.uint16)):
            g = th[k].view(dt)
            assert np.array_equal(g[keep], exp[k][keep]), (slot, dl, k)
            if k != "parse_status":
                assert not g[short].any(), (slot, dl, k)
        got = out.to_host()
        for k, dt in DEC_VIEWS.items():
            g = got[k].view(dt)
            if k == "id":
                g8, e8 = g.reshape(n, 8), exp[k].reshape(n, 8)
                assert np.array_equal(g8[keep], e8[keep]) and not g8[short].any()
            else:
                assert np.array_equal(g[keep], exp[k][keep]), (slot, dl, k)
        assert (got["status"].view(np.int8)[short] == -1).all()
        ev = exp["valid_idx"][:exp["n_valid"]]
        ev = ev[keep[ev]]
        nv = int(got["n_valid"][0])
        assert nv == len(ev) and np.array_equal(got["valid_idx"][:nv].view(np.uint32), ev)
        # rsock's own packets: IHL 5, data offset 5, EncHead len 23 -> never short at 96 B
        if slot >= 96:
            L = 14 if dl == 1 else 4
            plain = np.array([r[L] == 0x45 and (r[L + 32] >> 4) == 5 and (len(r) < L + 49 or r[L + 48] == 23)
                              for r in recs])
            assert plain.any() and not (short & plain).any()
        if slot == 64:
            assert short.any()


@pytest.mark.parametrize("mix", ["short", "mixed", "long", "bimodal"])
@pytest.mark.parametrize("layout,pad", [("packed_bytes", 0), ("rand_r", 0), ("rand_r", 16), ("every_r", 0),
                                        ("every_r", 16)])
@pytest.mark.parametrize("odd_payloads", [False, True])
def test_encode_any_frame_alignment(vcodec, gpu, oracle, mix, layout, pad, odd_payloads):
    """k_encode's vector paths at every destination offset r = frame_off mod 16:
    flat path (short sets), per-packet path (mixed), per-packet with the tag in the copy loop (long),
    frames packed back to back at byte granularity; bytes outside the frames must survive.  The same
    for the two-pass form (every frame one wave, header chunks from the records)."""
    codec = vcodec
    rng = np.random.default_rng(zlib.crc32(repr((mix, layout, pad, odd_payloads)).encode()))
    nset = 24
    n = 64 * nset
    if mix == "short":
        plen = rng.integers(1, 120, n)
    elif mix == "long":
        plen = rng.integers(1100, 1470, n)
    elif mix == "mixed":
        plen = rng.integers(1, 1470, n)
    else:  # alternate sets of short and long frames
        plen = np.where((np.arange(n) // 64) % 2 == 0, rng.integers(1, 80, n), rng.integers(1200, 1470, n))
    plen = plen.astype(np.uint16)
    plen[rng.integers(0, n, 5)] = 0  # resets in the middle of sets
    if odd_payloads:
        pay_off = np.cumsum(np.concatenate([[7], plen[:-1].astype(np.int64) + rng.integers(0, 19, n - 1)]))
    else:
        pay_off = np.arange(n) * 1472
    pay_off = pay_off.astype(np.uint64)
    payload = rng.integers(0, 256, int(pay_off[-1]) + 1600, dtype=np.uint8)
    flen = np.where(plen >= 1, plen.astype(np.int64) + 31, 0)
    if layout == "packed_bytes":
        frame_off = 3 + np.concatenate([[0], np.cumsum(flen)[:-1]])
    elif layout == "rand_r":
        frame_off = np.arange(n) * 1536 + rng.integers(0, 16, n)
    else:  # every r in turn, so each set holds all 16 offsets
        frame_off = np.arange(n) * 1536 + np.arange(n) % 16
    frame_off = frame_off.astype(np.uint64)
    frame_bytes = int(frame_off[-1]) + 1600
    cmd, conv, ckey = _rand_fields(rng, n)

    class D:
        pass

    d = D()
    d.n, d.pay_off, d.pay_len, d.cmd, d.conv, d.conn_key, d.frame_off = n, pay_off, plen, cmd, conv, ckey, frame_off
    fill = rng.integers(0, 256, frame_bytes, dtype=np.uint8)
    got_frames, got_status = run_encode(codec, gpu, payload, pay_off, plen, cmd, conv, ckey, frame_off,
                                        frame_bytes, frame_init=fill, pad16=pad == 16)
    ef, es = oracle.encode_batch(KEY, payload, d, workload.ID_UNIFORM, frame_bytes=frame_bytes)
    assert np.array_equal(got_status, es)
    exp_frames = fill.copy()
    for i in range(n):
        if es[i] > 0:
            o = int(frame_off[i])
            exp_frames[o:o + es[i]] = ef[o:o + es[i]]
            if pad:
                e = o + int(es[i])
                exp_frames[e:(e + pad - 1) // pad * pad] = 0
    bad = np.nonzero(got_frames != exp_frames)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]} (frame {np.searchsorted(frame_off, bad[0], 'right') - 1})"
