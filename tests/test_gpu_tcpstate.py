"""GPU: rsk_tcp_send_seq_batch / rsk_tcp_recv_ack_batch (FakeTcp::Output's seq advance and
RawTcp::Output's mIpId++, FakeTcp::OnRecv's ack; conn/FakeTcp.cpp:43-66, conn/RawTcp.cpp:111-121)
against the oracle's sequential walk: random connection mixes, unframed packets, connection ids past
n_conn, 32-bit seq and 16-bit IP id wrap-around, state carried over consecutive batches, and the
send chain encode -> seq/ip_id -> wire build -> parse back to the same TcpInfo seq."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import workload

pytestmark = pytest.mark.gpu


def _dev(a, gpu, dt):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu)


# n_conn + 1 <= 2048 takes the per-tile table path (k_sqt_*), larger ones the demux group-by; groupby=1
# forces the group-by for every case so both paths stay pinned to the oracle (2: the one-kernel column scan)
@pytest.mark.parametrize("groupby", [0, 1, 2])
@pytest.mark.parametrize("n,n_conn", [(1, 1), (777, 1), (5000, 7), (70_000, 300), (300_000, 70_000), (1, 0),
                                      (100_000, 0), (513, 64), (1_000_003, 64), (200_000, 511), (200_000, 512),
                                      (250_001, 2047), (250_001, 2048), (70_000, 1)])
def test_send_seq_matches_oracle(codec, gpu, oracle, n, n_conn, groupby):
    import torch

    codec.set_send_seq_groupby(groupby)
    rng = np.random.default_rng(n + n_conn)
    conn_seq0 = rng.integers(0, 2**32, n_conn, dtype=np.uint64).astype(np.uint32)
    if n_conn:
        conn_seq0[0] = 0xFFFFF000
    d_cs = _dev(conn_seq0, gpu, np.int32)
    ipn = np.array([65000], np.uint16)
    d_ipn = _dev(ipn, gpu, np.int16)
    cs_host, ip_host = conn_seq0.copy(), int(ipn[0])
    for batch in range(3):  # state carries over
        conn = rng.integers(0, n_conn + 3, n).astype(np.uint32)
        status = np.where(rng.random(n) < 0.9, rng.integers(32, 1501, n), rng.choice([0, -1], n)).astype(np.int32)
        seq = torch.empty(n, dtype=torch.int32, device=gpu)
        ipid = torch.empty(n, dtype=torch.int16, device=gpu)
        codec.tcp_send_seq_batch(_dev(conn, gpu, np.int32), _dev(status, gpu, np.int32), d_cs, d_ipn, seq, ipid)
        torch.cuda.synchronize()
        es, ei, cs_host, ip_host = oracle.tcp_send_seq_batch(conn, status, cs_host, ip_host)
        assert np.array_equal(seq.cpu().numpy().view(np.uint32), es), batch
        assert np.array_equal(ipid.cpu().numpy().view(np.uint16), ei), batch
        assert np.array_equal(d_cs.cpu().numpy().view(np.uint32), cs_host), batch
        assert int(d_ipn.cpu().numpy().view(np.uint16)[0]) == ip_host, batch
    codec.set_send_seq_groupby(0)


# BASELINE C3 size (4M packets) with bursty traffic: runs of 1-200 packets of one connection, as a
# sender drains one connection's queue at a time, so rounds of 64 lanes hold long same-connection runs
@pytest.mark.parametrize("n_conn", [1, 64, 2047])
def test_send_seq_fullsize_bursts(codec, gpu, oracle, n_conn):
    import torch

    n = 4 * 1024 * 1024
    rng = np.random.default_rng(n_conn)
    runs = rng.integers(1, 201, n // 50 + 1)
    owner = rng.integers(0, n_conn, runs.size)
    conn = np.repeat(owner, runs)[:n].astype(np.uint32)
    status = np.where(rng.random(n) < 0.97, 31 + 1400, 0).astype(np.int32)
    cs0 = rng.integers(0, 2**32, n_conn, dtype=np.uint64).astype(np.uint32)
    d_cs = _dev(cs0, gpu, np.int32)
    d_ipn = _dev(np.array([123], np.uint16), gpu, np.int16)
    seq = torch.empty(n, dtype=torch.int32, device=gpu)
    ipid = torch.empty(n, dtype=torch.int16, device=gpu)
    codec.tcp_send_seq_batch(_dev(conn, gpu, np.int32), _dev(status, gpu, np.int32), d_cs, d_ipn, seq, ipid)
    torch.cuda.synchronize()
    es, ei, cs_host, ip_host = oracle.tcp_send_seq_batch(conn, status, cs0, 123)
    assert np.array_equal(seq.cpu().numpy().view(np.uint32), es)
    assert np.array_equal(ipid.cpu().numpy().view(np.uint16), ei)
    assert np.array_equal(d_cs.cpu().numpy().view(np.uint32), cs_host)
    assert int(d_ipn.cpu().numpy().view(np.uint16)[0]) == ip_host


def test_recv_ack_matches_oracle(codec, gpu, oracle):
    import torch

    rng = np.random.default_rng(9)
    for n, n_conn in ((1000, 3), (200_000, 5000), (300_000, 8192), (300_000, 8193), (100_000, 50_000)):
        conn = rng.integers(0, n_conn + 1, n).astype(np.uint32)
        dl = (rng.random(n) < 0.8).astype(np.uint8)
        seq = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        ack0 = rng.integers(0, 2**32, n_conn, dtype=np.uint64).astype(np.uint32)
        d_ack = _dev(ack0, gpu, np.int32)
        codec.tcp_recv_ack_batch(_dev(conn, gpu, np.int32), _dev(dl, gpu, np.uint8), _dev(seq, gpu, np.int32), d_ack)
        torch.cuda.synchronize()
        assert np.array_equal(d_ack.cpu().numpy().view(np.uint32), oracle.tcp_recv_ack_batch(conn, dl, seq, ack0))


def test_send_chain_wire_parse(codec, gpu, oracle):
    """C4 packets of 10 connections: encode -> seq / ip_id -> wire packets -> parse: every delivered
    packet's TcpInfo seq is its send seq + payload_len (RawTcp.cpp:235), IP ids are consecutive."""
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers

    n, n_conn = 4096, 10
    d = workload.describe("c4", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                       id_uniform=workload.ID_UNIFORM)
    conn = (np.arange(n) % n_conn).astype(np.uint32)
    d_cs = torch.zeros(n_conn, dtype=torch.int32, device=gpu)
    d_ipn = torch.zeros(1, dtype=torch.int16, device=gpu)
    seq = torch.empty(n, dtype=torch.int32, device=gpu)
    ipid = torch.empty(n, dtype=torch.int16, device=gpu)
    codec.tcp_send_seq_batch(_dev(conn, gpu, np.int32), w.status, d_cs, d_ipn, seq, ipid)
    pitch = 16 * ((54 + 1500 + 15) // 16)
    wire = torch.zeros(n * pitch, dtype=torch.uint8, device=gpu)
    woff = torch.arange(n, device=gpu, dtype=torch.int64) * pitch
    wst = torch.empty(n, dtype=torch.int32, device=gpu)
    e = lambda v, dt: torch.full((n,), v, dtype=dt, device=gpu)  # noqa: E731
    codec.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, e(0x0200000A, torch.int32),
                            e(0x0100000A, torch.int32), e(43932 - 65536, torch.int16), e(10001, torch.int16), seq,
                            e(7, torch.int32), e(0x18, torch.uint8), ipid, wire, woff, wst,
                            eth=bytes([2, 0, 0, 0, 0, 1, 2, 0, 0, 0, 0, 2, 8, 0]), id_uniform=workload.ID_UNIFORM)
    tcp = TcpInfoBuffers.alloc(n, gpu)
    out = DecodeBuffers.alloc(n, gpu)
    codec.rawinput_batch(wire, woff, wst, wst, 1, 0, tcp, out)
    torch.cuda.synchronize()
    st = w.status.cpu().numpy()
    framed = st > 0
    s = seq.cpu().numpy().view(np.uint32)
    th = tcp.to_host()
    ps = th["parse_status"].view(np.int8)
    assert (ps[framed] == 1).all()
    plen = st[framed].astype(np.uint32)
    assert np.array_equal(th["seq"].view(np.uint32)[framed], s[framed] + plen)  # RawTcp.cpp:235
    ip = ipid.cpu().numpy().view(np.uint16)
    assert np.array_equal(ip[framed], np.arange(int(framed.sum()), dtype=np.uint16))
    exp_cs = np.zeros(n_conn, np.uint64)
    np.add.at(exp_cs, conn[framed], st[framed].astype(np.uint64))
    assert np.array_equal(d_cs.cpu().numpy().view(np.uint32), exp_cs.astype(np.uint32))
