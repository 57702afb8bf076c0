"""CPU: the oracle (oracle/rsk_oracle.c) pinned against the reference's own outputs (tests/golden,
made from oracle/_ref by tests/golden/make_golden.py), RFC 1321 and the SURVEY's live-capture
known answers.  No GPU needed."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from tests import pkt as P

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEY = b"hello135"


def gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


# ---- MD5 ----------------------------------------------------------------------------------------
RFC1321 = [  # RFC 1321 appendix A.5 test suite
    (b"", "d41d8cd98f00b204e9800998ecf8427e"),
    (b"a", "0cc175b9c0f1b6a831c399e269772661"),
    (b"abc", "900150983cd24fb0d6963f7d28e17f72"),
    (b"message digest", "f96b697d7cb7938d525a2f31aaf161d0"),
    (b"abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"),
    (b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789", "d174ab98d277d9f5a5611c2c9f419d9f"),
    (b"1234567890" * 8, "57edf4a22be3c955ac49da2e2107b67a"),
]


@pytest.mark.parametrize("msg,hexd", RFC1321)
def test_md5_rfc1321(oracle, msg, hexd):
    assert oracle.md5(msg).hex() == hexd


def test_md5_lengths_vs_hashlib(oracle):
    rng = np.random.default_rng(1)
    for ln in list(range(0, 200)) + [255, 256, 1000, 4097]:
        m = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        assert oracle.md5(m) == hashlib.md5(m).digest(), ln


# ---- SURVEY known answers (live loopback capture) ----------------
@pytest.mark.parametrize("b,tag", [(0x00, "f268b10bd0083eed"), (0x03, "2f02fe3129eff088"),
                                   (0x68, "e71bb9862f843799"), (0xFF, "96260db9013111bc")])
def test_known_tags(oracle, b, tag):
    assert oracle.tag(KEY, b).hex() == tag


def test_known_frame_prefix(oracle):
    payload = bytes((i * 7 + 3) & 0xFF for i in range(64))
    st, f = oracle.rconn_output(KEY, payload, 0, b"abcdefgh", 2, 0x3711D431)
    assert st == 95 and len(f) == 95
    assert f[:31].hex() == "2f02fe3129eff088" "17" "00" "6162636465666768" "02000000" "31d4113700000000" "00"
    assert f[31:] == payload
    assert oracle.key_for_tcp(54321, 10001) == 0x3711D431
    # flipping payload[0] fails verification; flipping the LAST byte still verifies
    assert oracle.rconn_onrecv(KEY, f).status == 1
    g = bytearray(f); g[31] ^= 1
    assert oracle.rconn_onrecv(KEY, bytes(g)).status == -1
    g = bytearray(f); g[-1] ^= 1
    assert oracle.rconn_onrecv(KEY, bytes(g)).status == 1


def test_known_parse_vector(oracle):
    """10.0.0.1:10001 -> 10.0.0.2:43932, seq 256, ack 512, flags 0x18, 40-B payload
    parses to src=0x0200000a sp=43932 dst=0x0100000a dp=10001 seq=296 ack=512 flag=0x18 len=40."""
    p = P.ipv4_tcp("10.0.0.1", 10001, "10.0.0.2", 43932, 256, 512, 0x18, bytes(40))
    t = oracle.rawinput(p, len(p), len(p), 1, 0)
    assert t.parse_status == 1
    assert (t.src, t.sp, t.dst, t.dp, t.seq, t.ack, t.flag, t.cap_pay_len) == (
        0x0200000A, 43932, 0x0100000A, 10001, 296, 512, 0x18, 40)
    assert t.cap_pay_off == 54


# ---- golden fixtures from the reference build ------------------------------------------------------
def test_golden_tags(oracle):
    g = gold("tags.npz")
    kb, ko, kl = g["key_bytes"], g["key_off"], g["key_len"]
    for k in range(len(kl)):
        key = kb[int(ko[k]): int(ko[k]) + int(kl[k])].tobytes()
        for b in range(256):
            assert oracle.tag(key, b) == g["tags"][k, b].tobytes(), (len(key), b)


def test_golden_frames(oracle):
    g = gold("frames.npz")
    n = len(g["status"])
    for i in range(n):
        p = g["payload"][int(g["pay_off"][i]): int(g["pay_off"][i]) + int(g["pay_len"][i])].tobytes()
        st, f = oracle.rconn_output(KEY, p, int(g["cmd"][i]), g["id"][8 * i: 8 * i + 8].tobytes(),
                                    int(g["conv"][i]), int(g["conn_key"][i]))
        assert st == g["status"][i], i
        exp = g["frames"][int(g["frame_off"][i]): int(g["frame_off"][i]) + int(g["frame_len"][i])].tobytes()
        assert f == exp, i


def test_golden_onrecv(oracle):
    g = gold("onrecv.npz")
    frames = g["frames"]
    exp = {k: g[k] for k in ("status", "hlen", "cmd", "id", "conv", "conn_key", "pay_off", "pay_len")}
    got = oracle.decode_batch(KEY, frames, g["frame_off"], g["frame_len"], g["close"])
    for k, v in exp.items():
        assert np.array_equal(got[k], v), k
    assert got["n_valid"] == int((exp["status"] == 1).sum())
    assert (exp["status"] == 1).sum() > 50 and (exp["status"] == 0).sum() > 10 and (exp["status"] == -1).sum() > 50


def test_golden_enchead(oracle):
    g = gold("enchead.npz")
    for i in range(len(g["enc_buf_len"])):
        h = oracle.enchead_encode(int(g["enc_buf_len"][i]), int(g["enc_cmd"][i]), g["enc_id"][8 * i: 8 * i + 8].tobytes(),
                                  int(g["enc_conv"][i]), int(g["enc_key"][i]))
        if g["enc_ok"][i]:
            assert h == g["enc_out"][23 * i: 23 * i + 23].tobytes()
        else:
            assert h is None
    for i in range(len(g["dec_buf_len"])):
        r = oracle.enchead_decode(g["dec_in"][23 * i: 23 * i + 23].tobytes(), int(g["dec_buf_len"][i]))
        assert (r is not None) == bool(g["dec_ok"][i]), i
        if r is not None:
            assert r[1:] == (int(g["dec_cmd"][i]), g["dec_id"][8 * i: 8 * i + 8].tobytes(), int(g["dec_conv"][i]),
                             int(g["dec_key"][i]))


def test_golden_tcpinfo_and_keys(oracle):
    from tests.oracle_lib import OrcTcpInfo

    g = gold("tcpinfo_keys.npz")
    for i in range(len(g["src"])):
        t = OrcTcpInfo(int(g["src"][i]), int(g["dst"][i]), int(g["sp"][i]), int(g["dp"][i]), int(g["seq"][i]),
                       int(g["ack"][i]), int(g["flag"][i]), 0, 0, 0)
        assert oracle.tcpinfo_encode(t) == g["records"][21 * i: 21 * i + 21].tobytes()
    for a, b, kt, ku in zip(g["key_sp"], g["key_dp"], g["key_tcp"], g["key_udp"]):
        assert oracle.key_for_tcp(int(a), int(b)) == int(kt)
        assert oracle.key_for_udp(int(a), int(b)) == int(ku)


# ---- live cross-check against the reference build (only where /root/reference was compiled) --------
def test_live_reference_random(oracle, refo):
    rng = np.random.default_rng(99)
    for k in range(300):
        key = rng.integers(0, 256, int(rng.integers(0, 130)), dtype=np.uint8).tobytes()
        p = rng.integers(0, 256, int(rng.integers(0, 1480)), dtype=np.uint8).tobytes()
        args = (int(rng.integers(0, 256)), rng.integers(0, 256, 8, dtype=np.uint8).tobytes(),
                int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)))
        assert oracle.rconn_output(key, p, *args) == refo.rconn_output(key, p, *args)
        st, f = oracle.rconn_output(key, p, *args)
        if st > 0:
            g = bytearray(f)
            if k % 3 == 1:
                g[int(rng.integers(0, len(g)))] ^= 0xFF
            if k % 5 == 2:
                g[8] = int(rng.integers(0, 256))
            d = oracle.rconn_onrecv(key, bytes(g), close=bool(k & 1))
            rs, rf = refo.rconn_onrecv(key, bytes(g), close=bool(k & 1))
            assert d.status == rs
            if rs == 1:
                assert (d.hlen, d.cmd, bytes(d.id), d.conv, d.conn_key, d.pay_off, d.pay_len) == rf


# ---- parse semantics (RawTcp.cpp:138-244) on hand-built packets -------------------------------------
def test_parse_rules(oracle):
    mk = lambda **kw: P.ipv4_tcp("1.2.3.4", 1111, "5.6.7.8", 2222, 1000, 2000, kw.pop("flags", 0x18),  # noqa: E731
                                 kw.pop("payload", bytes(40)), **kw)
    t = oracle.rawinput(mk(), 94, 94, 1, 0)
    assert t.parse_status == 1 and t.seq == 1040 and t.cap_pay_len == 40
    t = oracle.rawinput(mk(ihl_words=15, thl_words=15), 174, 174, 1, 0)
    assert t.parse_status == 1 and t.cap_pay_off == 14 + 60 + 60
    assert oracle.rawinput(mk(), 43, 94, 1, 0).parse_status == 0            # wire len < 44
    assert oracle.rawinput(mk(ethertype=0x86DD), 94, 94, 1, 0).parse_status == 0
    assert oracle.rawinput(mk(proto=17), 94, 94, 1, 0).parse_status == 0
    p = mk(flags=0x02)
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 1       # SYN, no ack pool
    t = oracle.rawinput(p, len(p), len(p), 1, 1)
    assert t.parse_status == 2 and (t.src, t.sp, t.seq) == (0x08070605, 2222, 1000)
    t = oracle.rawinput(p, len(p), len(p), 1, 3)                            # server: Reverse()
    assert t.parse_status == 2 and (t.src, t.sp, t.seq, t.ack) == (0x04030201, 1111, 2000, 1000)
    p = mk(payload=b"12345678")
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 0       # < 9 bytes, no FIN/RST
    p = mk(payload=b"12345678", flags=0x11)
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 1
    p = mk(payload=bytes(1469))
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 0       # cap2uv: 1469 + 32 > 1500
    p = mk(payload=bytes(1468))
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 1
    p = mk(payload=b"", flags=0x14, ip_len=30)                              # payload_len -10 with RST
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 3
    p = mk(payload=b"", flags=0x14, ip_len=5)                               # -35: size_t wrap -> drop
    assert oracle.rawinput(p, len(p), len(p), 1, 0).parse_status == 0
    p = mk(datalink=0)
    assert oracle.rawinput(p, len(p), len(p), 0, 0).parse_status == 1
    p = mk(datalink=0, null_family=24)
    assert oracle.rawinput(p, len(p), len(p), 0, 0).parse_status == 0
    p = mk()
    assert oracle.rawinput(p, len(p), 30, 1, 0).parse_status == 3          # truncated capture
