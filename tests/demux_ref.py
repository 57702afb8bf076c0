"""TEST INFRASTRUCTURE: rsock-shaped receive batches for the demux pin and the checks
that tie a segment order to the reference's own routing.

The reference routes one packet at a time (oracle/ref_demux_harness.cpp runs its code):
  server  ServerGroup::OnRecv by IdBuf (server/ServerGroup.cpp:44-63) -> IAppGroup::Input by cmd
          (conn/IAppGroup.cpp:76-96) -> INetGroup::Input by connKey (conn/INetGroup.cpp:57-83) ->
          SubGroup::OnRecv by BuildConvKey(dst, conv) (server/SubGroup.cpp:31-51) -> SConn
  client  IAppGroup::Input by cmd -> INetGroup::Input by connKey (known conns only) ->
          ClientGroup::OnRecv by conv (client/ClientGroup.cpp:65-80) -> CConn, or SendConvRst
The conn whose packet ORDER is observable is the leaf (SConn / CConn: it forwards datagrams to the
target in the order it receives them).  The levels above it keep only order-free state: the groups'
DataStat counters (conn/IConn.cpp) and the fake-TCP ack, a max (conn/FakeTcp.cpp:52-66).  One conv's
packets travel over every fake-TCP conn of its group (INetGroup::doSend picks one at random per
packet, conn/INetGroup.cpp:111-127), so the demux key has to be the leaf's key, not the connKey:
  server  RSK_DEMUX_ID | RSK_DEMUX_DST | RSK_DEMUX_CONV | RSK_DEMUX_CMD_BARRIER
  client  RSK_DEMUX_CONV | RSK_DEMUX_CMD_BARRIER
Control packets (cmd != DATA: IReset / keep-alive input, or "unrecognized") are barriers.  On the
server a control packet only reaches its own IdBuf's SubGroup, so RSK_DEMUX_GROUP_BARRIER (a barrier
for its IdBuf's packets alone) is enough there: SERVER_GROUP_FIELDS.
"""
from __future__ import annotations

import numpy as np

from rsock_amd import _abi as A

SERVER_FIELDS = A.DEMUX_ID | A.DEMUX_DST | A.DEMUX_CONV | A.DEMUX_CMD_BARRIER
SERVER_GROUP_FIELDS = A.DEMUX_ID | A.DEMUX_DST | A.DEMUX_CONV | A.DEMUX_GROUP_BARRIER
CLIENT_FIELDS = A.DEMUX_CONV | A.DEMUX_CMD_BARRIER
SERVER, CLIENT = 0, 1


def key_for_tcp(sp, dp):
    """KeyGenerator::KeyForTcp (src/util/KeyGenerator.cpp:16-24), vectorised."""
    return (np.uint64(0x10000000) | (np.asarray(dp, np.uint64) << np.uint64(16)) | np.asarray(sp, np.uint64))


def rsock_case(rng, n, n_groups, n_net, n_conv, p_ctrl, p_valid, p_bad_cmd=0.0, ctrl_at=()):
    """A receive batch shaped like rsock traffic: n_groups clients (IdBuf + address), each with
    n_net fake-TCP conns (connKey = KeyForTcp(sp, dp), dp over 10001-10010) and n_conv convs; every
    packet of a conv leaves on a random conn of its group.  Control packets (cmd 1-4) with
    probability p_ctrl and at the indices ctrl_at, unknown cmds (5-255) with p_bad_cmd; DROP /
    CLOSE_NOTIFY with probability 1 - p_valid."""
    g = rng.integers(0, n_groups, n)
    ids_tab = rng.integers(0, 256, (n_groups, 8), dtype=np.uint8)
    dst_tab = (0x0a000000 + rng.integers(1, max(2, n_groups // 2 + 1), n_groups)).astype(np.uint32)
    net = rng.integers(0, n_net, n)
    sp = 32768 + (g * n_net + net) % 28000
    ckey = key_for_tcp(sp, 10001 + (g * n_net + net) % 10)
    conv = (1 + rng.integers(0, n_conv, n)).astype(np.uint32)
    cmd = np.zeros(n, np.uint8)
    r = rng.random(n)
    cmd[r < p_ctrl] = rng.integers(1, 5, int((r < p_ctrl).sum()))
    bad = (r >= p_ctrl) & (r < p_ctrl + p_bad_cmd)
    cmd[bad] = rng.integers(5, 256, int(bad.sum()))
    for i in ctrl_at:
        if i < n:
            cmd[i] = 1 + i % 4
    status = np.where(rng.random(n) < p_valid, A.RECV_VALID,
                      rng.choice([A.RECV_DROP, A.RECV_CLOSE], n)).astype(np.int8)
    return status, cmd, ids_tab[g].reshape(-1).copy(), conv, ckey.astype(np.uint64), dst_tab[g].copy()


def outcomes(ref_cls, log, n):
    """Per packet, from one reference run in arrival order: the leaf it reached (numbered in the
    order the leaves were created / listed; -1 none), its group (server; -1 none), whether it was a
    control packet (IReset / keep-alive input or an unrecognized cmd), the conv a SendConvRst named
    for it (-1 none), and the top-level return."""
    leaf = np.full(n, -1, np.int32)
    group = np.full(n, -1, np.int32)
    ctrl = np.zeros(n, np.int8)
    rst_conv = np.full(n, -1, np.int64)
    conns = log["conns"]
    leaf_no, group_no = {}, {}
    for c, (lv, _par, _k) in enumerate(conns):  # conns are listed in creation order
        if lv == ref_cls.LV_LEAF:
            leaf_no[c] = len(leaf_no)
        elif lv == ref_cls.LV_GROUP:
            group_no[c] = len(group_no)
    for kind, c, pkt, aux in log["ev"].tolist():
        if kind == ref_cls.EV_DELIVER and c in leaf_no:
            leaf[pkt] = leaf_no[c]
        elif kind == ref_cls.EV_DELIVER and c in group_no:
            group[pkt] = group_no[c]
        elif kind in (ref_cls.EV_RST_IN, ref_cls.EV_KA_IN):
            ctrl[pkt] = 1
        elif kind == ref_cls.EV_CONV_RST:
            rst_conv[pkt] = aux
    return {"leaf": leaf, "group": group, "ctrl": ctrl, "rst_conv": rst_conv, "ret": log["ret"].copy()}


def check_segments(segs, status, cmd, out, server: bool, id=None):
    """Delivering `segs` (list of (first, [packets])) segment by segment hands every leaf the same
    packet sequence the reference gave it, creates leaves and groups in the same order, keeps every
    control packet exactly where it was relative to the rest (with `id`, the IdBuf bytes: relative
    to the rest of its own IdBuf, the group barrier's promise), and needs one conn lookup per
    segment.  `out` = outcomes() of the reference run."""
    valid = np.nonzero(status == A.RECV_VALID)[0]
    perm = np.array([p for _f, pk in segs for p in pk], np.int64)
    assert sorted(perm.tolist()) == valid.tolist(), "perm is not the VALID packets"
    firsts = [f for f, _pk in segs]
    assert all(pk and pk[0] == f for f, pk in segs)
    assert firsts == sorted(firsts), "segments not ordered by first packet"
    pos = np.empty(len(status), np.int64)
    pos[perm] = np.arange(len(perm))
    # control packets (barriers): alone, and every VALID packet before them is delivered first
    is_ctrl = (status == A.RECV_VALID) & (cmd != A.CMD_DATA)
    assert np.array_equal(is_ctrl, (status == A.RECV_VALID) & ((out["ctrl"] == 1) | (cmd > 4))), \
        "the reference's control packets are the cmd != DATA ones"
    if id is None:
        rank = np.cumsum(status == A.RECV_VALID) - 1
        for i in np.nonzero(is_ctrl)[0]:
            assert pos[i] == rank[i], f"control packet {i} moved"
    else:
        gid = np.asarray(id, np.uint8).reshape(-1, 8).view(np.uint64).ravel()
        for g in np.unique(gid[valid]):
            mine = valid[gid[valid] == g]  # this IdBuf's VALID packets in arrival order
            pm = pos[mine]
            for k in np.nonzero(is_ctrl[mine])[0]:
                assert (pm[:k] < pm[k]).all() and (pm[k + 1:] > pm[k]).all(), \
                    f"control packet {mine[k]} moved inside its IdBuf"
    for f, pk in segs:
        if is_ctrl[f]:
            assert pk == [f]
    # one lookup per segment: its packets reach one leaf (or name one unknown conv)
    for f, pk in segs:
        targets = {("leaf", int(out["leaf"][p])) if out["leaf"][p] >= 0 else ("rst", int(out["rst_conv"][p]))
                   for p in pk if out["leaf"][p] >= 0 or out["rst_conv"][p] >= 0}
        assert len(targets) <= 1, f"segment {f} needs {len(targets)} lookups"
    # per-leaf and per-conv-reset sequences in arrival order; leaves / groups created in order
    for col in ("leaf", "rst_conv"):
        v = out[col][perm]
        for t in np.unique(v[v >= 0]):
            idx = perm[v == t]
            assert np.all(np.diff(idx) > 0), f"{col} {t} receives its packets out of order"
    for col in ("leaf", "group") if server else ():
        v = out[col][perm]
        seen = v[v >= 0]
        _, first = np.unique(seen, return_index=True)
        order = seen[np.sort(first)]
        assert np.array_equal(order, np.arange(len(order))), f"{col}s created in another order"
