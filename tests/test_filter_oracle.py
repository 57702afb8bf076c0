"""CPU: the capture filter.  BuildFilterStr (cap/cap_util.cpp:67-144) is restated
three times (oracle C, librsk's rsk_filter_str, a Python transcription here) and must agree
character for character; the predicate is checked by evaluating that STRING with an independent
pcap-filter interpreter (primitive meanings as libpcap 1.7.4 gencode compiles them; libpcap itself
exists only as the reference's prebuilt .a, so parity is pinned to the published filter
semantics, not to libpcap output) against the oracle's structured predicate."""
from __future__ import annotations

import re
import struct

import numpy as np
import pytest

from rsock_amd import codec as rc
from tests.pkt import rand_capture

DLT_NULL, DLT_EN10MB = 0, 1


# ---- BuildFilterStr, transcribed -------------------------------------------------------------
def py_filter_str(src_ip, dst_ip, src_singles, src_ranges, dst_singles, dst_ranges, is_server):
    out = "tcp"
    for ip, word in ((src_ip, "src"), (dst_ip, "dst")):
        if ip:
            out += " and " + f" (ip {word} " + ip + ")"
    for singles, ranges, word in ((src_singles, src_ranges, "src"), (dst_singles, dst_ranges, "dst")):
        if singles or ranges:
            out += " and "
            s = "("
            for p in singles:
                s += f" or {word} port {p}"
            for a, b in ranges:
                s += f" or {word} portrange {a}-{b}"
            s += " )"
            pos = s.find("or")
            s = s[:pos] + s[pos + 2:]
            out += s
    if is_server:
        s = out.replace("dst", "src")
        return f"((tcp[tcpflags] & tcp-syn != 0) and {s}) or ({out}and (tcp[tcpflags] & (tcp-syn) == 0))"
    return out


# ---- pcap-filter interpreter for the subset BuildFilterStr emits ------------------------------
class Reject(Exception):
    """A field read past cap_len: the BPF program returns 0 for the packet."""


class Pkt:
    def __init__(self, data: bytes, cl: int, dl: int):
        self.d, self.cl, self.L = data, cl, 14 if dl == DLT_EN10MB else 4
        self.dl = dl

    def need(self, n):
        if n > self.cl:
            raise Reject()

    def byte(self, k):
        self.need(k + 1)
        return self.d[k]

    def be16(self, k):
        self.need(k + 2)
        return struct.unpack_from("!H", self.d, k)[0]

    def net(self):  # "ether proto ip/ip6" / DLT_NULL family
        if self.dl == DLT_EN10MB:
            et = self.be16(12)
            return 4 if et == 0x0800 else 6 if et == 0x86DD else 0
        self.need(4)
        fam = struct.unpack_from("<I", self.d, 0)[0]
        return 4 if fam == 2 else 6 if fam in (24, 28, 30) else 0

    def v4_first_frag(self):
        return (self.be16(self.L + 6) & 0x1FFF) == 0


def prim_tcp(p):
    v = p.net()
    if v == 4:
        return p.byte(p.L + 9) == 6
    if v == 6:
        nxt = p.byte(p.L + 6)
        return nxt == 6 or (nxt == 44 and p.byte(p.L + 40) == 6)
    return False


def prim_host(p, which, ip):
    if p.net() != 4:
        return False
    off = p.L + (12 if which == "src" else 16)
    p.need(off + 4)
    return bytes(p.d[off:off + 4]) == bytes(int(x) for x in ip.split("."))


def prim_port(p, which, lo, hi):
    v = p.net()
    d = 0 if which == "src" else 2
    if v == 4:
        if p.byte(p.L + 9) in (6, 17, 132) and p.v4_first_frag():
            return lo <= p.be16(p.L + 4 * (p.byte(p.L) & 15) + d) <= hi
        return False
    if v == 6:
        if p.byte(p.L + 6) in (6, 17, 132):
            return lo <= p.be16(p.L + 40 + d) <= hi
        return False
    return False


def prim_syn(p, want):
    if p.net() != 4 or p.byte(p.L + 9) != 6 or not p.v4_first_frag():
        return False
    syn = (p.byte(p.L + 4 * (p.byte(p.L) & 15) + 13) & 2) != 0
    return syn if want else not syn


TOKEN = re.compile(r"\s*(tcp\[tcpflags\] & tcp-syn != 0|tcp\[tcpflags\] & \(tcp-syn\) == 0|\(|\)|and|or|"
                   r"ip (?:src|dst) [\d.]+|(?:src|dst) portrange \d+-\d+|(?:src|dst) port \d+|tcp)")


def tokenize(s):
    out, pos = [], 0
    while pos < len(s):
        m = TOKEN.match(s, pos)
        assert m, f"cannot tokenize at {s[pos:]!r}"
        out.append(m.group(1))
        pos = m.end()
        while pos < len(s) and s[pos] == " ":
            pos += 1
    return out


def compile_filter(s):
    """-> callable(pkt) -> bool.  pcap precedence: `and` and `or` equal, left-associative."""
    toks = tokenize(s)
    i = 0

    def atom():
        nonlocal i
        t = toks[i]
        i += 1
        if t == "(":
            e = expr()
            assert toks[i] == ")"
            i += 1
            return e
        if t == "tcp":
            return prim_tcp
        if t.startswith("ip "):
            _, w, ip = t.split()
            return lambda p: prim_host(p, w, ip)
        if "portrange" in t:
            w, _, r = t.split()
            lo, hi = map(int, r.split("-"))
            return lambda p: prim_port(p, w, lo, hi)
        if " port " in t:
            w, _, v = t.split()
            return lambda p: prim_port(p, w, int(v), int(v))
        if "!=" in t:
            return lambda p: prim_syn(p, True)
        if "==" in t:
            return lambda p: prim_syn(p, False)
        raise AssertionError(t)

    def expr():
        nonlocal i
        e = atom()
        while i < len(toks) and toks[i] in ("and", "or"):
            op = toks[i]
            i += 1
            r = atom()
            e = (lambda a, b: lambda p: a(p) and b(p))(e, r) if op == "and" else \
                (lambda a, b: lambda p: a(p) or b(p))(e, r)
        return e

    f = expr()
    assert i == len(toks)

    def run(p):
        try:
            return bool(f(p))
        except Reject:
            return False
    return run


def pools_for(a, rng):
    """Per-field pools that make a filter's clauses hit often (either direction, so a server's
    primed branch is exercised too), plus values that miss."""
    def ports(singles, ranges):
        return list(singles) + [x for r in ranges for x in (r[0], r[1], (r[0] + r[1]) // 2)]
    sp, dp = ports(a["src_singles"], a["src_ranges"]), ports(a["dst_singles"], a["dst_ranges"])
    if rng.random() < 0.5 and a["is_server"]:
        sp = sp + dp
    extra = [9, 40011]
    ips = [x for x in (a["src_ip"], a["dst_ip"]) if x]
    return dict(sports=tuple(sp + extra), dports=tuple(dp + extra),
                srcs=tuple(([a["src_ip"]] if a["src_ip"] else ips) + ["172.16.0.9"]),
                dsts=tuple(([a["dst_ip"]] if a["dst_ip"] else ips) + ["172.16.0.9"]))


def rand_filter_args(rng):
    pick = lambda k, pool: [int(x) for x in rng.choice(pool, size=k)]  # noqa: E731
    ports = [10001, 10002, 10003, 443, 53, 40000, 40001]
    mk_ranges = lambda k: [tuple(sorted(rng.choice(np.arange(1, 65535), 2, replace=False).tolist())) for _ in range(k)]  # noqa: E731
    return dict(
        src_ip=str(rng.choice(["10.0.0.1", "192.168.1.7"])) if rng.random() < 0.4 else None,
        dst_ip=str(rng.choice(["10.0.0.2", "10.0.0.1"])) if rng.random() < 0.5 else None,
        src_singles=pick(int(rng.integers(0, 3)), ports) if rng.random() < 0.4 else [],
        src_ranges=mk_ranges(int(rng.integers(0, 2))) if rng.random() < 0.3 else [],
        dst_singles=pick(int(rng.integers(0, 4)), ports) if rng.random() < 0.7 else [],
        dst_ranges=[(40000, 40010)] + mk_ranges(int(rng.integers(0, 2))) if rng.random() < 0.4 else [],
        is_server=bool(rng.random() < 0.5),
    )


@pytest.mark.parametrize("seed", range(40))
def test_filter_str_three_ways(oracle, seed):
    rng = np.random.default_rng(seed)
    a = rand_filter_args(rng)
    f = rc.make_filter(**a)
    exp = py_filter_str(a["src_ip"], a["dst_ip"], a["src_singles"], a["src_ranges"], a["dst_singles"],
                        a["dst_ranges"], a["is_server"])
    assert oracle.filter_str(f) == exp
    assert rc.filter_str(f) == exp


def test_filter_str_known():
    f = rc.make_filter(dst_ip="10.0.0.2", dst_singles=[10001], dst_ranges=[(10010, 10020)], is_server=True)
    assert rc.filter_str(f) == (
        "((tcp[tcpflags] & tcp-syn != 0) and tcp and  (ip src 10.0.0.2) and (  src port 10001 or src portrange "
        "10010-10020 )) or (tcp and  (ip dst 10.0.0.2) and (  dst port 10001 or dst portrange 10010-10020 )and "
        "(tcp[tcpflags] & (tcp-syn) == 0))")
    assert rc.filter_str(rc.make_filter()) == "tcp"


@pytest.mark.parametrize("dl", [DLT_EN10MB, DLT_NULL])
@pytest.mark.parametrize("seed", range(12))
def test_predicate_vs_filter_string(oracle, dl, seed):
    rng = np.random.default_rng(1000 * dl + seed)
    a = rand_filter_args(rng)
    f = rc.make_filter(**a)
    run = compile_filter(py_filter_str(a["src_ip"], a["dst_ip"], a["src_singles"], a["src_ranges"],
                                       a["dst_singles"], a["dst_ranges"], a["is_server"]))
    pools = pools_for(a, rng)
    hits = 0
    for _ in range(800):
        pkt, cl = rand_capture(rng, dl, **pools)
        exp = run(Pkt(pkt, cl, dl))
        got = oracle.capture_filter(pkt, dl, f, cap_len=cl)
        assert got == exp, (pkt.hex(), cl)
        hits += exp
    assert hits >= 3  # the comparison covers matches, not only rejections
