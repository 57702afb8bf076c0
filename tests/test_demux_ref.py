"""CPU: the receive demux pinned to the REFERENCE's own routing code.

oracle/_ref/librsk_ref_demux.so runs rsock's ServerGroup / SubGroup / ClientGroup / IAppGroup /
INetGroup (compiled from /root/reference, oracle/ref_demux_harness.cpp).  Three things are shown:
  1. routing the VALID packets through the reference in the order the oracle's segments give
     (orc_demux_batch with the fields of tests/demux_ref.py) changes nothing the reference can
     observe: every leaf conn (SConn / CConn) receives the same packets in the same order, leaves
     and groups are created in the same order, control packets and conv resets fall at the same
     places, every packet gets the same return; the levels in between (the IdBuf groups, the
     fake-TCP conns) receive the same packets, whose order they cannot observe (counters, max ack);
  2. keying the server's demux by connKey (the round-5 INTEGRATION.md recipe) reorders a conv's
     packets when the conv travels over several fake-TCP conns, which rsock does for every conv;
  3. tests/golden/demux.npz (the reference's per-packet outcomes, tests/golden/make_demux_golden.py)
     still matches the reference, and the oracle's segments pass tests/demux_ref.check_segments
     against it — the same check the GPU test runs on rsk_demux_batch.
1 and 2 need oracle/_ref (built in the build container from /root/reference); 3's oracle half
needs only the fixture.
"""
from __future__ import annotations

import os

import numpy as np
import pytest

from rsock_amd import _abi as A
from tests import demux_ref as D
from tests.oracle_lib import RefDemux, ref_demux_available

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "demux.npz")
needs_ref = pytest.mark.skipif(not ref_demux_available(), reason="oracle/_ref not built (no /root/reference)")


@pytest.fixture(scope="module")
def refdemux():
    return RefDemux()


def golden_cases():
    z = np.load(GOLDEN)
    out = []
    for ci, name in enumerate(z["names"].tolist()):
        p = f"c{ci}_"
        c = {k[len(p):]: z[k] for k in z.files if k.startswith(p)}
        stack, fields, n = (int(x) for x in c["meta"])
        c.update(stack=stack, fields=fields, n=n, name=name)
        out.append(c)
    return out


def _ordered_trace(T):
    """The reference trace, split into what order matters for and what it does not."""
    per = T["per_conn"]
    leaf = {k: v for k, v in per.items() if k[-1][0] == RefDemux.LV_LEAF}
    other = {k: sorted(v) for k, v in per.items() if k[-1][0] != RefDemux.LV_LEAF}
    created = {lv: (v if lv != RefDemux.LV_NET else sorted(v)) for lv, v in T["created"].items()}
    ev = T["events"]
    ctrl = [e for e in ev if e[0] in (RefDemux.EV_RST_IN, RefDemux.EV_KA_IN)]
    conv_rst = {}
    for kind, pkt, aux in ev:
        if kind == RefDemux.EV_CONV_RST:
            conv_rst.setdefault(aux, []).append(pkt)
    order_free = sorted(e for e in ev if e[0] in (RefDemux.EV_NETCONN_RST, RefDemux.EV_DEFAULT_IN))
    return leaf, other, created, ctrl, conv_rst, order_free, T["ret"].tolist()


def _known(rng, ckey, n_conv):
    keys = np.unique(ckey)
    return keys[rng.random(len(keys)) < 0.8], np.arange(1, n_conv + 1)[rng.random(n_conv) < 0.75]


SHAPES = [  # n, groups, nets, convs, p_ctrl, p_valid, p_bad_cmd
    (1500, 3, 4, 6, 0.01, 0.9, 0.0), (4000, 20, 6, 30, 0.003, 0.8, 0.002), (800, 2, 3, 3, 0.25, 0.9, 0.05),
    (5000, 1, 16, 1, 0.001, 1.0, 0.0), (300, 4, 2, 2, 0.0, 0.0, 0.0), (2000, 1, 8, 40, 0.0, 1.0, 0.0)]


@needs_ref
@pytest.mark.parametrize("stack,fields", [(D.SERVER, D.SERVER_FIELDS), (D.SERVER, D.SERVER_GROUP_FIELDS),
                                          (D.CLIENT, D.CLIENT_FIELDS)])
@pytest.mark.parametrize("shape", SHAPES)
def test_reference_unchanged_by_segment_order(refdemux, oracle, stack, fields, shape):
    n, ng, nn, nc, pc, pv, pb = shape
    rng = np.random.default_rng(n * 7 + stack * 1000 + ng)
    status, cmd, ids, conv, ckey, dst = D.rsock_case(rng, n, ng, nn, nc, pc, pv, pb)
    kk, kc = _known(rng, ckey, nc) if stack == D.CLIENT else ((), ())
    segs, nv = oracle.demux_batch(status, cmd, fields, ids, conv, ckey, dst)
    assert nv == int((status == A.RECV_VALID).sum())
    perm = [p for _f, pk in segs for p in pk]
    t_arr = RefDemux.trace(refdemux.run(stack, status, cmd, ids, conv, ckey, dst, known_keys=kk, known_convs=kc))
    t_seg = RefDemux.trace(refdemux.run(stack, status, cmd, ids, conv, ckey, dst, order=perm, known_keys=kk,
                                        known_convs=kc))
    a, b = _ordered_trace(t_arr), _ordered_trace(t_seg)
    for what, x, y in zip(("leaf sequences", "group / fake-TCP multisets", "creation order", "control events",
                           "conv resets", "net resets", "returns"), a, b):
        assert x == y, what
    if ((status == A.RECV_VALID) & (cmd == A.CMD_DATA)).any() and stack == D.SERVER:
        assert a[0], "no leaf received anything"


@needs_ref
def test_connkey_segments_reorder_a_conv(refdemux, oracle):
    """Server batches keyed by (IdBuf, connKey) hand a conv's packets to its SConn out of arrival
    order as soon as the conv uses two fake-TCP conns: the demux key is the leaf's."""
    rng = np.random.default_rng(11)
    status, cmd, ids, conv, ckey, dst = D.rsock_case(rng, 400, 1, 4, 3, 0.0, 1.0)
    old = A.DEMUX_ID | A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER
    segs, _ = oracle.demux_batch(status, cmd, old, ids, conv, ckey, dst)
    perm = [p for _f, pk in segs for p in pk]
    t_arr = RefDemux.trace(refdemux.run(D.SERVER, status, cmd, ids, conv, ckey, dst))
    t_old = RefDemux.trace(refdemux.run(D.SERVER, status, cmd, ids, conv, ckey, dst, order=perm))
    assert _ordered_trace(t_arr)[0] != _ordered_trace(t_old)[0]
    assert _ordered_trace(t_arr)[1] == _ordered_trace(t_old)[1]  # the levels above see the same packets


@needs_ref
def test_golden_is_the_reference(refdemux):
    for c in golden_cases():
        log = refdemux.run(c["stack"], c["status"], c["cmd"], c["id"], c["conv"], c["conn_key"], c["dst"],
                           known_keys=c["known_keys"], known_convs=c["known_convs"])
        o = D.outcomes(RefDemux, log, c["n"])
        for k, v in o.items():
            assert np.array_equal(v, c[k]), (c["name"], k)


@pytest.mark.parametrize("ci", range(len(golden_cases())))
def test_oracle_segments_against_golden(oracle, ci):
    c = golden_cases()[ci]
    segs, nv = oracle.demux_batch(c["status"], c["cmd"], c["fields"], c["id"], c["conv"], c["conn_key"], c["dst"])
    assert nv == int((c["status"] == A.RECV_VALID).sum())
    D.check_segments(segs, c["status"], c["cmd"], c, c["stack"] == D.SERVER)
    if c["stack"] == D.SERVER:  # the server's IdBuf-scoped barrier against the same reference outcomes
        segs, _ = oracle.demux_batch(c["status"], c["cmd"], D.SERVER_GROUP_FIELDS, c["id"], c["conv"],
                                     c["conn_key"], c["dst"])
        D.check_segments(segs, c["status"], c["cmd"], c, True, id=c["id"])


def test_check_segments_rejects_arrival_order_violations(oracle):
    """The checker is not vacuous: swapping two packets of one leaf, or moving a control packet,
    fails it."""
    c = [c for c in golden_cases() if c["name"] == "server_small"][0]
    segs, _ = oracle.demux_batch(c["status"], c["cmd"], c["fields"], c["id"], c["conv"], c["conn_key"], c["dst"])
    big = max(range(len(segs)), key=lambda s: len(segs[s][1]))
    f, pk = segs[big]
    bad = list(segs)
    bad[big] = (f, [pk[0], pk[2], pk[1]] + pk[3:])
    with pytest.raises(AssertionError):
        D.check_segments(bad, c["status"], c["cmd"], c, True)
    ctrl = [s for s, (f, _pk) in enumerate(segs) if c["cmd"][f] != 0]
    s = ctrl[len(ctrl) // 2]
    moved = segs[:s - 1] + [segs[s], segs[s - 1]] + segs[s + 1:]
    with pytest.raises(AssertionError):
        D.check_segments(moved, c["status"], c["cmd"], c, True)
    # group barrier: the batch-wide segments (a stricter order) pass the IdBuf-scoped check, and a
    # leaf's first segment after a control packet of its IdBuf, merged into the leaf's segment before
    # it (leaf order and segment order stay intact), fails it
    D.check_segments(segs, c["status"], c["cmd"], c, True, id=c["id"])
    gs, _ = oracle.demux_batch(c["status"], c["cmd"], D.SERVER_GROUP_FIELDS, c["id"], c["conv"], c["conn_key"],
                               c["dst"])
    D.check_segments(gs, c["status"], c["cmd"], c, True, id=c["id"])
    leaf, gid = c["leaf"], c["id"].reshape(-1, 8).view(np.uint64).ravel()
    bad = None
    for k, (f, _pk) in enumerate(gs):
        if c["cmd"][f] == 0:
            continue
        lf = [e for e, (f2, _p) in enumerate(gs[:k]) if c["cmd"][f2] == 0 and leaf[f2] >= 0 and gid[f2] == gid[f]]
        for e in reversed(lf):  # the leaf's next segment lies after the barrier
            m = next((m for m in range(e + 1, len(gs)) if c["cmd"][gs[m][0]] == 0 and leaf[gs[m][0]] == leaf[gs[e][0]]),
                     None)
            if m is not None and m > k:
                bad = list(gs)
                bad[e] = (gs[e][0], gs[e][1] + gs[m][1])
                del bad[m]
                break
        if bad:
            break
    assert bad is not None
    with pytest.raises(AssertionError, match="moved inside its IdBuf"):
        D.check_segments(bad, c["status"], c["cmd"], c, True, id=c["id"])
