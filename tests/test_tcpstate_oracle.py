"""CPU: the fake-TCP connection-state restatement (oracle orc_tcp_send_seq_batch /
orc_tcp_recv_ack_batch) against an independent Python walk of FakeTcp::Output / RawTcp::Output /
FakeTcp::OnRecv (conn/FakeTcp.cpp:43-66, conn/RawTcp.cpp:111-121), packet by packet."""
from __future__ import annotations

import numpy as np
import pytest


def py_send(conn, status, conn_seq, ip_next):
    conn_seq = [int(x) for x in conn_seq]
    seq, ipid = [], []
    for c, st in zip(conn, status):
        if st <= 0:                      # RConn::Output did not frame it: nothing reaches RawTcp
            seq.append(0)
            ipid.append(0)
            continue
        ipid.append(ip_next)             # SendRawTcp(..., mIpId++, ...)
        ip_next = (ip_next + 1) & 0xFFFF
        if c >= len(conn_seq):
            seq.append(0)
            continue
        seq.append(conn_seq[c])          # the packet carries mInfo.seq ...
        conn_seq[c] = (conn_seq[c] + int(st)) & 0xFFFFFFFF  # ... then UpdateSeq(seq + 31 + nread)
    return seq, ipid, conn_seq, ip_next


@pytest.mark.parametrize("n_conn", [1, 7, 300])
def test_send_seq_matches_reference_walk(oracle, n_conn):
    rng = np.random.default_rng(n_conn)
    n = 5000
    conn = rng.integers(0, n_conn + 2, n).astype(np.uint32)   # a few ids past n_conn
    status = np.where(rng.random(n) < 0.9, rng.integers(32, 1501, n), rng.choice([0, -1], n)).astype(np.int32)
    conn_seq = rng.integers(0, 2**32, n_conn, dtype=np.uint64).astype(np.uint32)
    conn_seq[0] = 0xFFFFFF00  # wraps inside the batch
    ip0 = 65530                # wraps inside the batch
    seq, ipid, cs, ipn = oracle.tcp_send_seq_batch(conn, status, conn_seq, ip0)
    es, ei, ecs, eipn = py_send(conn.tolist(), status.tolist(), conn_seq.tolist(), ip0)
    assert seq.tolist() == es and ipid.tolist() == ei and cs.tolist() == ecs and ipn == eipn


def test_recv_ack_is_running_max(oracle):
    rng = np.random.default_rng(3)
    n, n_conn = 4000, 50
    conn = rng.integers(0, n_conn + 1, n).astype(np.uint32)
    dl = (rng.random(n) < 0.8).astype(np.uint8)
    seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    ack0 = rng.integers(0, 2**32, n_conn, dtype=np.uint64).astype(np.uint32)
    got = oracle.tcp_recv_ack_batch(conn, dl, seq, ack0)
    exp = [int(x) for x in ack0]
    for c, d, s in zip(conn.tolist(), dl.tolist(), seq.tolist()):
        if d and c < n_conn and exp[c] < s:   # FakeTcp.cpp:60-64
            exp[c] = s
    assert got.tolist() == exp
