"""CPU: the oracle's RawTcp::syncInput -> TcpInfo::Decode -> RConn::OnRecv (orc_syncinput) on
hand-off records (21-B TcpInfo + frame), pinned two ways: against a Python restatement over the
oracle's own OnRecv (always), and against the reference's TcpInfo::Decode and RConn::OnRecv compiled
from /root/reference (oracle/_ref, when built).  Records: valid frames, tampered tags, FIN/RST with
short frames, and every record length around the 12 / 21 / 52-byte boundaries."""
from __future__ import annotations

import ctypes
import struct

import numpy as np
import pytest

KEY = b"hello135"
FIN, RST = 0x01, 0x04


def records(oracle, seed: int = 3):
    """[(record bytes padded to >= 64, nread)]"""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(120):
        plen = int(rng.choice([1, 2, 23, 100, 700, 1400, 1469]))
        st, frame = oracle.rconn_output(KEY, bytes(rng.integers(0, 256, plen, dtype=np.uint8)),
                                        int(rng.integers(0, 5)), b"abcdefgh", int(rng.integers(0, 2**32)),
                                        int(rng.integers(0, 2**63)))
        assert st > 0
        flag = int(rng.choice([0x10, 0x18, 0x11, 0x14, 0x02, 0x00]))
        hdr = struct.pack("<IIHHIIB", *(int(x) for x in rng.integers(0, 2**32, 2, dtype=np.uint64)), int(rng.integers(1, 65536)),
                          int(rng.integers(1, 65536)), int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), flag)
        rec = bytearray(hdr + frame)
        nread = len(rec)
        if k % 7 == 3:
            rec[21 + int(rng.integers(0, 8))] ^= 0x40            # tampered tag
        if k % 11 == 5:
            nread = int(rng.integers(21, 53))                    # frame cut to <= 31 bytes
        out.append((bytes(rec) + bytes(64), nread))
    base = out[0][0]
    for nread in (-5, 0, 1, 11, 12, 13, 20, 21, 22, 51, 52, 53):  # around the boundaries
        for flag in (0x10, 0x11, 0x04):
            rec = bytearray(base)
            rec[20] = flag
            out.append((bytes(rec), nread))
    return out


def _py_syncinput(oracle, rec: bytes, nread: int):
    """Restatement: syncInput returns early for nread <= 0 and for a failed Decode (here: < 21)."""
    if nread < 21:
        return None, None
    src, dst, sp, dp, seq, ack, flag = struct.unpack_from("<IIHHIIB", rec)
    d = oracle.rconn_onrecv(KEY, rec[21:], nread - 21, bool(flag & (FIN | RST)))
    return (src, dst, sp, dp, seq, ack, flag), d


def test_syncinput_restatement(oracle):
    for rec, nread in records(oracle):
        t, d = oracle.syncinput(KEY, rec, nread)
        et, ed = _py_syncinput(oracle, rec, nread)
        if et is None:
            assert t.parse_status == 0 and d.status == -1 and t.src == t.flag == 0
            continue
        assert t.parse_status == 1 and t.cap_pay_off == 21 and t.cap_pay_len == nread - 21
        assert (t.src, t.dst, t.sp, t.dp, t.seq, t.ack, t.flag) == et
        assert (d.status, d.hlen, d.cmd, bytes(d.id), d.conv, d.conn_key, d.pay_off, d.pay_len) == \
            (ed.status, ed.hlen, ed.cmd, bytes(ed.id), ed.conv, ed.conn_key, ed.pay_off, ed.pay_len)


def test_syncinput_vs_reference(oracle, refo):
    L = refo.L
    seen_close = seen_valid = 0
    for rec, nread in records(oracle, seed=9):
        t, d = oracle.syncinput(KEY, rec, nread)
        o7 = (ctypes.c_uint32 * 7)()
        r = L.ref_tcpinfo_decode(rec, nread, o7) if nread > 0 else -1   # syncInput: nread > 0 only
        if nread < 12:
            assert r == -1 and t.parse_status == 0 and d.status == -1
            continue
        assert r == 21                      # the reference's Decode always consumes 21 bytes
        if nread < 21:                      # ... reading past nread: the documented deviation
            assert t.parse_status == 0 and d.status == -1
            continue
        assert (t.src, t.dst, t.sp, t.dp, t.seq, t.ack, t.flag) == tuple(o7)
        hlen, cmd, conv, ckey = ctypes.c_uint8(), ctypes.c_uint8(), ctypes.c_uint32(), ctypes.c_uint64()
        idb = ctypes.create_string_buffer(8)
        po, pl = ctypes.c_int(), ctypes.c_int()
        st = L.ref_rconn_onrecv(KEY, len(KEY), rec[21:], nread - 21, int(bool(o7[6] & (FIN | RST))),
                                ctypes.byref(hlen), ctypes.byref(cmd), idb, ctypes.byref(conv), ctypes.byref(ckey),
                                ctypes.byref(po), ctypes.byref(pl))
        assert d.status == st
        if st == 1:
            seen_valid += 1
            assert (d.hlen, d.cmd, bytes(d.id), d.conv, d.conn_key, d.pay_off, d.pay_len) == \
                (hlen.value, cmd.value, idb.raw, conv.value, ckey.value, po.value, pl.value)
        seen_close += st == 0
    assert seen_valid > 50 and seen_close > 0
