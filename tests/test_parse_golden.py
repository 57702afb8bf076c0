"""RawTcp::RawInput parity pinned to the REFERENCE's own parse (conn/RawTcp.cpp:138-237 compiled in
oracle/_ref/librsk_ref_parse.so): tests/golden/parse.npz (tests/golden/make_parse_golden.py) against
the oracle's restatement, plus live random packets against the reference where it is built."""
from __future__ import annotations

import os

import numpy as np
import pytest

from tests import pkt as P

HERE = os.path.dirname(os.path.abspath(__file__))
FIELDS = ("src", "dst", "sp", "dp", "seq", "ack", "flag")


def load():
    return dict(np.load(os.path.join(HERE, "golden", "parse.npz")))


def test_fixture_coverage():
    g = load()
    st = g["status"]
    for s in (0, 1, 2, 3):  # DROP, DELIVER, SYN, MALFORMED all pinned
        assert (st == s).sum() >= 20, s
    assert g["syn_refused"].any()
    assert set(np.unique(g["datalink"]).tolist()) == {0, 1}
    assert (g["wire_len"] < 44).any()


def test_oracle_matches_reference_fixture(oracle):
    g = load()
    for i in range(len(g["off"])):
        o, n = int(g["off"][i]), int(g["cap_len"][i])
        pkt = g["arena"][o:o + n].tobytes()
        for j, fl in enumerate(g["flags"]):
            t = oracle.rawinput(pkt, int(g["wire_len"][i]), n, int(g["datalink"][i]), int(fl))
            es = int(g["status"][i, j])
            if g["syn_refused"][i, j]:
                assert t.parse_status == 2, (i, fl)
                continue
            assert t.parse_status == es, (i, fl, t.parse_status, es)
            if es in (1, 2):
                got = tuple(int(getattr(t, k)) for k in FIELDS)
                exp = tuple(int(g[k][i, j]) for k in FIELDS)
                assert got == exp, (i, fl, got, exp)
            if es == 1:
                assert (t.cap_pay_off, t.cap_pay_len) == (int(g["pay_off"][i, j]), int(g["pay_len"][i, j])), i


def test_oracle_matches_live_reference_random(oracle):
    from tests.oracle_lib import RefParse, ref_parse_available

    if not ref_parse_available():
        pytest.skip("oracle/_ref/librsk_ref_parse.so not built (needs /root/reference)")
    from tests.golden.make_parse_golden import expected, is_tcp_syn

    ref = RefParse()
    rng = np.random.default_rng(1234)
    for k in range(1500):
        dl = int(rng.integers(0, 2))
        plen = int(rng.choice([int(rng.integers(0, 16)), int(rng.integers(0, 1600))]))
        ihl, thl = int(rng.integers(5, 16)), int(rng.integers(5, 16))
        # a well-formed capture: the IPv4 total length never runs past the captured bytes (the
        # reference reads there without looking at caplen; this build calls that MALFORMED)
        ipl = None if rng.random() < 0.8 else int(rng.integers(0, 4 * (ihl + thl) + plen + 1))
        p = P.ipv4_tcp(f"10.{rng.integers(256)}.0.1", int(rng.integers(0, 65536)), "192.168.0.2",
                       int(rng.integers(0, 65536)), int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)),
                       int(rng.integers(0, 256)), bytes(rng.integers(0, 256, plen, dtype=np.uint8)),
                       ihl_words=ihl, thl_words=thl, ip_len=ipl, datalink=dl)
        wl = len(p) if rng.random() < 0.95 else int(rng.integers(0, 60))
        fl = int(rng.choice([0, 1, 3]))
        r = ref.rawinput(p, wl, len(p), dl, bool(fl & 2), bool(fl & 1))
        e = expected(r)
        t = oracle.rawinput(p, wl, len(p), dl, fl)
        if (fl & 1) and e[0] == 0 and is_tcp_syn(p, dl, wl):
            assert t.parse_status == 2, k
            continue
        assert t.parse_status == e[0], (k, t.parse_status, e)
        if e[0] in (1, 2):
            assert tuple(int(getattr(t, f)) for f in FIELDS) == e[1:8], k
