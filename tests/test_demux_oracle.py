"""CPU: the receive-demux oracle (orc_demux_batch) against an independent restatement
of the reference's per-packet routing, and the property that makes batching legal: delivering the
segments in order hands every conn the same packet sequence, and creates conns in the same order,
as the reference's loop (INetGroup.cpp:57-83 connKey map, IAppGroup.cpp:76-96 cmd dispatch,
ServerGroup.cpp:44-60 IdBuf map, SubGroup.cpp:31-50 (dst, conv) map, ClientGroup.cpp:66-80 conv map).
Reference-side pinning: the reference has no batch demux and no tests for these lookups; the
semantics restated here are the per-packet lookups cited above ("parity unpinned" by fixtures)."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import _abi as A

ALL = A.DEMUX_ID | A.DEMUX_CONN_KEY | A.DEMUX_CONV | A.DEMUX_DST
BARRIERS = A.DEMUX_CMD_BARRIER | A.DEMUX_GROUP_BARRIER


def key_of(i, fields, id, conv, ckey, dst):
    return (bytes(id[8 * i: 8 * i + 8]) if fields & A.DEMUX_ID else None,
            int(ckey[i]) if fields & A.DEMUX_CONN_KEY else None,
            int(conv[i]) if fields & A.DEMUX_CONV else None,
            int(dst[i]) if fields & A.DEMUX_DST else None)


def group_of(i, fields, id):
    """The scope a control packet is a barrier for: the whole batch (CMD_BARRIER) or its IdBuf."""
    return bytes(id[8 * i: 8 * i + 8]) if fields & A.DEMUX_GROUP_BARRIER else None


def py_demux(status, cmd, fields, id, conv, ckey, dst):
    """Restatement: walk VALID packets; a control packet (barrier) is alone and closes the epoch of
    its scope (group_of)."""
    segs, where, epoch = [], {}, {}
    for i in range(len(status)):
        if status[i] != A.RECV_VALID:
            continue
        g = group_of(i, fields, id)
        if fields & BARRIERS and cmd[i] != A.CMD_DATA:
            segs.append((i, [i]))
            epoch[g] = epoch.get(g, 0) + 1
            continue
        k = (epoch.get(g, 0),) + key_of(i, fields, id, conv, ckey, dst)
        if k not in where:
            where[k] = len(segs)
            segs.append((i, []))
        segs[where[k]][1].append(i)
    return segs


def reference_routing(status, cmd, fields, id, conv, ckey, dst):
    """The reference's observable effect: per-key delivery sequences + conn creation order, with
    control packets as ordered events (each seeing the conns of its scope created so far)."""
    conns, created, events = {}, [], []
    for i in range(len(status)):
        if status[i] != A.RECV_VALID:
            continue
        if fields & BARRIERS and cmd[i] != A.CMD_DATA:
            g = group_of(i, fields, id)
            events.append(("ctrl", i, sum(1 for k in created if g is None or k[0] == g)))
            continue
        k = key_of(i, fields, id, conv, ckey, dst)
        if k not in conns:
            conns[k] = []
            created.append(k)
        conns[k].append(i)
    return conns, created, events


def segment_routing(segs, cmd, fields, id, conv, ckey, dst):
    conns, created, events = {}, [], []
    for first, pk in segs:
        if fields & BARRIERS and cmd[first] != A.CMD_DATA:
            g = group_of(first, fields, id)
            events.append(("ctrl", first, sum(1 for k in created if g is None or k[0] == g)))
            continue
        k = key_of(first, fields, id, conv, ckey, dst)
        assert all(key_of(i, fields, id, conv, ckey, dst) == k for i in pk)
        if k not in conns:
            conns[k] = []
            created.append(k)
        conns[k].extend(pk)
    return conns, created, events


def make_case(rng, n, nkeys, p_ctrl, p_valid):
    status = np.where(rng.random(n) < p_valid, A.RECV_VALID,
                      rng.choice([A.RECV_DROP, A.RECV_CLOSE], n)).astype(np.int8)
    cmd = np.where(rng.random(n) < p_ctrl, rng.integers(1, 5, n), 0).astype(np.uint8)
    pick = rng.integers(0, nkeys, n)
    ids = rng.integers(0, 256, (nkeys, 8), dtype=np.uint8)[pick % max(1, nkeys // 3 + 1)].reshape(-1)
    conv = rng.integers(0, 4, nkeys).astype(np.uint32)[pick]
    ckey = (rng.integers(0, 2**40, nkeys, dtype=np.uint64))[pick]
    dst = rng.integers(0, 3, nkeys).astype(np.uint32)[pick]
    return status, cmd, ids, conv, ckey, dst


@pytest.mark.parametrize("fields", [ALL, A.DEMUX_CONN_KEY, A.DEMUX_ID | A.DEMUX_CONV | A.DEMUX_DST, A.DEMUX_CONV,
                                    0, ALL | A.DEMUX_CMD_BARRIER, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER,
                                    A.DEMUX_CMD_BARRIER, ALL | A.DEMUX_GROUP_BARRIER,
                                    A.DEMUX_ID | A.DEMUX_GROUP_BARRIER])
@pytest.mark.parametrize("shape", [(0, 1, 0.0, 1.0), (1, 1, 0.0, 1.0), (500, 3, 0.05, 0.9), (3000, 40, 0.01, 0.7),
                                   (2000, 2000, 0.0, 1.0), (800, 5, 0.5, 1.0), (300, 4, 0.0, 0.0), (400, 7, 1.0, 1.0)])
def test_oracle_vs_restatement(oracle, fields, shape):
    n, nkeys, p_ctrl, p_valid = shape
    rng = np.random.default_rng(n * 31 + nkeys + fields)
    status, cmd, ids, conv, ckey, dst = make_case(rng, n, nkeys, p_ctrl, p_valid)
    got, nv = oracle.demux_batch(status, cmd, fields, ids, conv, ckey, dst)
    exp = py_demux(status, cmd, fields, ids, conv, ckey, dst)
    assert got == exp
    assert nv == int((status == A.RECV_VALID).sum())
    # batching preserves the reference's per-conn sequences, creation order and control-event order
    assert segment_routing(got, cmd, fields, ids, conv, ckey, dst) == \
        reference_routing(status, cmd, fields, ids, conv, ckey, dst)


def test_oracle_null_unselected_fields(oracle):
    rng = np.random.default_rng(3)
    status, cmd, ids, conv, ckey, dst = make_case(rng, 200, 6, 0.1, 0.8)
    got, _ = oracle.demux_batch(status, cmd, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER, conn_key=ckey)
    assert got == py_demux(status, cmd, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER, ids, conv, ckey, dst)


def test_group_barrier_fewer_segments(oracle):
    """A control packet splits only its own IdBuf's conns: with many IdBufs the group barrier leaves
    far fewer segments than the batch-wide barrier, and both satisfy the reference's routing."""
    rng = np.random.default_rng(5)
    status, cmd, ids, conv, ckey, dst = make_case(rng, 6000, 60, 0.05, 1.0)
    nb = len(oracle.demux_batch(status, cmd, ALL | A.DEMUX_CMD_BARRIER, ids, conv, ckey, dst)[0])
    ng = len(oracle.demux_batch(status, cmd, ALL | A.DEMUX_GROUP_BARRIER, ids, conv, ckey, dst)[0])
    assert ng < nb // 2, (ng, nb)

