"""GPU: rsk_demux_batch against the oracle (orc_demux_batch), segment for segment:
random batches over every field selection, control-packet barriers, all-invalid / all-control /
single-key / all-distinct batches (1, 2 and 3 radix passes), ragged sizes, and the decoded output
of the real receive path (C4 frames through rsk_decode_batch, demuxed on the device)."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import _abi as A
from rsock_amd import workload
from tests.test_demux_oracle import ALL, make_case

pytestmark = pytest.mark.gpu


def run_gpu(codec, gpu, status, cmd, fields, ids, conv, ckey, dst):
    import torch

    from rsock_amd.codec import DemuxBuffers

    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu)  # noqa: E731
    n = len(status)
    out = DemuxBuffers.alloc(n, gpu)
    codec.demux_batch(t(status, np.int8), t(cmd, np.uint8), fields, out, id=t(ids, np.uint8),
                      conv=t(conv, np.int32), conn_key=t(ckey, np.int64), dst=t(dst, np.int32))
    torch.cuda.synchronize()
    return out.segments(), int(out.n_valid.item())


FIELDS = [ALL, A.DEMUX_CONN_KEY, A.DEMUX_ID | A.DEMUX_CONV | A.DEMUX_DST, A.DEMUX_CONV, 0,
          ALL | A.DEMUX_CMD_BARRIER, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER, A.DEMUX_CMD_BARRIER,
          ALL | A.DEMUX_GROUP_BARRIER, A.DEMUX_ID | A.DEMUX_GROUP_BARRIER]
SHAPES = [(1, 1, 0.0, 1.0), (63, 3, 0.1, 0.9), (500, 3, 0.05, 0.9), (4097, 40, 0.01, 0.7), (3000, 3000, 0.0, 1.0),
          (800, 5, 0.5, 1.0), (300, 4, 0.0, 0.0), (400, 7, 1.0, 1.0), (70000, 300, 0.002, 0.8)]


@pytest.mark.parametrize("fields", FIELDS)
@pytest.mark.parametrize("shape", SHAPES)
def test_demux_random(codec, gpu, oracle, fields, shape):
    n, nkeys, p_ctrl, p_valid = shape
    rng = np.random.default_rng(n * 31 + nkeys + fields)
    case = make_case(rng, n, nkeys, p_ctrl, p_valid)
    got = run_gpu(codec, gpu, *case[:2], fields, *case[2:])
    exp = oracle.demux_batch(case[0], case[1], fields, *case[2:])
    assert got[1] == exp[1]
    assert got[0] == exp[0]


@pytest.mark.parametrize("n,fields", [(300000, ALL), (200000, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER),
                                      (65537, A.DEMUX_CONV), (200000, ALL | A.DEMUX_GROUP_BARRIER)])
def test_demux_many_segments(codec, gpu, oracle, n, fields):
    """Every packet its own key (segments = n_valid: 3 radix passes at 300K), and dense barriers."""
    rng = np.random.default_rng(n)
    status = np.where(rng.random(n) < 0.95, 1, -1).astype(np.int8)
    cmd = np.where(rng.random(n) < (0.3 if fields & A.DEMUX_CMD_BARRIER else 0.0), 3, 0).astype(np.uint8)
    ids = rng.integers(0, 256, 8 * n, dtype=np.uint8)
    conv = np.arange(n, dtype=np.uint32)
    ckey = rng.permutation(n).astype(np.uint64) * 7919
    dst = rng.integers(0, 2, n).astype(np.uint32)
    got = run_gpu(codec, gpu, status, cmd, fields, ids, conv, ckey, dst)
    exp = oracle.demux_batch(status, cmd, fields, ids, conv, ckey, dst)
    assert got[1] == exp[1] and len(got[0]) == len(exp[0])
    assert got[0] == exp[0]


@pytest.mark.parametrize("n_follow", [0, 1, 17, 1023, 1024, 1025, 5000])
@pytest.mark.parametrize("fields", [A.DEMUX_CONN_KEY, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER])
def test_demux_follower_counts(codec, gpu, oracle, n_follow, fields):
    """Distinct keys plus exactly `n_follow` repeats of earlier keys (near and far back, across the
    insert kernel's 1024-packet tiles): the one-block sort of <= 1024 followers, the radix passes
    above it, and no followers at all."""
    n = 30000
    rng = np.random.default_rng(n_follow * 7 + fields)
    status = np.ones(n, np.int8)
    cmd = np.zeros(n, np.uint8)
    ckey = (rng.permutation(n).astype(np.uint64) + 1) * 0x9E3779B1
    rep = np.sort(rng.choice(np.arange(1, n), n_follow, replace=False))
    for i in rep:  # a follower of a key seen up to 3000 packets earlier
        ckey[i] = ckey[max(0, i - 1 - int(rng.integers(0, 3000)))]
    if fields & A.DEMUX_CMD_BARRIER:  # sparse barriers: epochs of ~2000 packets cross the tiles
        cmd[rng.choice(n, 15, replace=False)] = 3
    ids = np.zeros(8 * n, np.uint8)
    conv = np.zeros(n, np.uint32)
    dst = np.zeros(n, np.uint32)
    got = run_gpu(codec, gpu, status, cmd, fields, ids, conv, ckey, dst)
    exp = oracle.demux_batch(status, cmd, fields, ids, conv, ckey, dst)
    assert got[1] == exp[1] and len(got[0]) == len(exp[0])
    assert got[0] == exp[0]


@pytest.mark.parametrize("shape", [(50000, 20000, 0.05, 0.95), (50000, 500, 0.05, 0.95), (200000, 50, 0.01, 0.9),
                                   (100000, 3, 0.3, 1.0)])
def test_demux_epoch_local(codec, gpu, oracle, shape):
    """Dense barriers (C4-like 5 % control packets and denser): keys whose epoch lies inside one
    insert tile never reach the global table; the tiles' first and last epochs do."""
    n, nkeys, p_ctrl, p_valid = shape
    rng = np.random.default_rng(n + nkeys)
    case = make_case(rng, n, nkeys, p_ctrl, p_valid)
    for fields in (ALL | A.DEMUX_CMD_BARRIER, A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER):
        got = run_gpu(codec, gpu, *case[:2], fields, *case[2:])
        exp = oracle.demux_batch(case[0], case[1], fields, *case[2:])
        assert got[1] == exp[1]
        assert got[0] == exp[0]


def test_demux_empty_and_errors(codec, gpu):
    import torch

    from rsock_amd.codec import DemuxBuffers, RskError

    out = DemuxBuffers.alloc(0, gpu)
    e = torch.empty(0, dtype=torch.int8, device=gpu)
    codec.demux_batch(e, e.view(torch.uint8), ALL, out, id=e.view(torch.uint8), conv=e, conn_key=e, dst=e)
    torch.cuda.synchronize()
    assert int(out.n_seg.item()) == 0 and int(out.n_valid.item()) == 0 and int(out.seg_off[0].item()) == 0
    st = torch.ones(8, dtype=torch.int8, device=gpu)
    with pytest.raises(RskError):
        codec.demux_batch(st, st.view(torch.uint8), 0x40, DemuxBuffers.alloc(8, gpu))  # unknown field bit
    with pytest.raises(RskError):
        codec.demux_batch(st, st.view(torch.uint8), A.DEMUX_CONN_KEY, DemuxBuffers.alloc(8, gpu))  # key missing
    ids = torch.zeros(64, dtype=torch.uint8, device=gpu)
    for bad in (A.DEMUX_CONV | A.DEMUX_GROUP_BARRIER,  # group barrier without the IdBuf
                A.DEMUX_ID | A.DEMUX_GROUP_BARRIER | A.DEMUX_CMD_BARRIER):  # both barriers
        with pytest.raises(RskError):
            codec.demux_batch(st, st.view(torch.uint8), bad, DemuxBuffers.alloc(8, gpu), id=ids,
                              conv=st.view(torch.uint8).to(torch.int32))


def test_demux_decoded_c4(codec, gpu, oracle):
    """The receive path end to end on the device: C4 frames (1/16 corrupted, 5% control cmds) ->
    rsk_decode_batch -> rsk_demux_batch on the decoded fields, vs the oracle on the same fields."""
    import torch

    from rsock_amd.codec import DecodeBuffers, DemuxBuffers

    d = workload.describe("c4", 0, 50000, n=50000)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                       id_uniform=workload.ID_UNIFORM)
    w.corrupt_frames()
    dec = DecodeBuffers.alloc(d.n, gpu)
    codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, dec)
    fields = A.DEMUX_ID | A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER
    out = DemuxBuffers.alloc(d.n, gpu)
    codec.demux_batch(dec.status, dec.cmd, fields, out, id=dec.id, conv=dec.conv, conn_key=dec.conn_key)
    torch.cuda.synchronize()
    h = lambda x, dt: x.cpu().numpy().view(dt)  # noqa: E731
    st = h(dec.status, np.int8)
    assert 0 < (st == 1).sum() < d.n
    exp = oracle.demux_batch(st, h(dec.cmd, np.uint8), fields, h(dec.id, np.uint8), h(dec.conv, np.uint32),
                             h(dec.conn_key, np.uint64), None)
    assert out.segments() == exp[0]


@pytest.mark.parametrize("shape,fields", [((1 << 20, 7000, 0.0, 0.97), A.DEMUX_ID | A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER),
                                          ((1 << 20, 64, 0.001, 1.0), A.DEMUX_ID | A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER),
                                          ((1 << 20, 7000, 0.0, 0.8), A.DEMUX_CONN_KEY)])
def test_demux_bench_shapes(codec, gpu, oracle, shape, fields):
    """The bench's demux shapes at 1M packets (tools/bench_paths.py: C3-like thousands of keys spread over
    every tile -- every packet probes the global table, whose slots name packet indices and are lowered
    by CAS across concurrent tiles; 64 connections with 0.1 % control packets -- epochs by packet index,
    2-3 radix passes), with invalid packets between the valid ones, against the oracle."""
    n, nkeys, p_ctrl, p_valid = shape
    rng = np.random.default_rng(nkeys + int(p_valid * 100))
    case = make_case(rng, n, nkeys, p_ctrl, p_valid)
    got = run_gpu(codec, gpu, *case[:2], fields, *case[2:])
    exp = oracle.demux_batch(case[0], case[1], fields, *case[2:])
    assert got[1] == exp[1] and len(got[0]) == len(exp[0])
    assert got[0] == exp[0]


def _golden():
    from tests.test_demux_ref import golden_cases

    return golden_cases()


@pytest.mark.parametrize("ci", range(10))
def test_demux_golden_reference_routing(codec, gpu, oracle, ci):
    """rsk_demux_batch against the REFERENCE's own routing (tests/golden/demux.npz: what rsock's
    ServerGroup / SubGroup / ClientGroup / IAppGroup / INetGroup did with each packet, in arrival
    order; tests/golden/make_demux_golden.py): delivering the GPU's segments in order gives every
    leaf conn its packets in the reference's order, creates leaves and groups in its order, keeps
    control packets in place and needs one lookup per segment (tests/demux_ref.check_segments)."""
    from tests import demux_ref as D

    cases = _golden()
    assert len(cases) == 10
    c = cases[ci]
    got, nv = run_gpu(codec, gpu, c["status"], c["cmd"], c["fields"], c["id"], c["conv"], c["conn_key"], c["dst"])
    assert nv == int((c["status"] == A.RECV_VALID).sum())
    D.check_segments(got, c["status"], c["cmd"], c, c["stack"] == D.SERVER)
    exp = oracle.demux_batch(c["status"], c["cmd"], c["fields"], c["id"], c["conv"], c["conn_key"], c["dst"])
    assert got == exp[0]
    if c["stack"] == D.SERVER:  # the IdBuf-scoped barrier (two passes on the device)
        f = D.SERVER_GROUP_FIELDS
        got, nv = run_gpu(codec, gpu, c["status"], c["cmd"], f, c["id"], c["conv"], c["conn_key"], c["dst"])
        D.check_segments(got, c["status"], c["cmd"], c, True, id=c["id"])
        assert got == oracle.demux_batch(c["status"], c["cmd"], f, c["id"], c["conv"], c["conn_key"], c["dst"])[0]


@pytest.mark.parametrize("fields", [A.DEMUX_ID | A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER,
                                    A.DEMUX_CONN_KEY | A.DEMUX_CMD_BARRIER, ALL | A.DEMUX_CMD_BARRIER,
                                    ALL | A.DEMUX_GROUP_BARRIER])
def test_demux_epoch_edges_same_key(codec, gpu, oracle, fields):
    """The same (IdBuf, connKey) on both sides of control packets placed at insert / look-back tile
    edges (511/512, 1023/1024, 4095/4096/4097, 8191/8192), one epoch spanning several tiles, and
    back-to-back barriers — the owner-epoch range test of the insert kernel."""
    n = 20000
    status = np.ones(n, np.int8)
    cmd = np.zeros(n, np.uint8)
    for i in (511, 512, 1023, 1024, 4095, 4096, 4097, 8191, 8192, 8193, 8194):
        cmd[i] = 1 + i % 4
    ids = np.tile(np.frombuffer(b"ABCDEFGH", np.uint8), n)
    ckey = np.where(np.arange(n) % 3 == 0, 0x27111000, 0x27128001).astype(np.uint64)
    conv = (np.arange(n) % 2).astype(np.uint32)
    dst = np.full(n, 0x0200000a, np.uint32)
    got = run_gpu(codec, gpu, status, cmd, fields, ids, conv, ckey, dst)
    exp = oracle.demux_batch(status, cmd, fields, ids, conv, ckey, dst)
    assert got[1] == exp[1]
    assert got[0] == exp[0]



@pytest.mark.parametrize("n,groups,p_ctrl", [(1 << 20, 64, 0.002), (1 << 20, 64, 0.05), (300000, 5000, 0.01),
                                             (100000, 2, 0.3)])
def test_demux_group_barrier_server_shapes(codec, gpu, oracle, n, groups, p_ctrl):
    """Server batches (tests/demux_ref.rsock_case: IdBuf groups, convs over several fake-TCP conns)
    under the IdBuf-scoped barrier: the device's two passes against the oracle's walk, with far fewer
    segments than the batch-wide barrier once there are many groups."""
    from tests import demux_ref as D

    rng = np.random.default_rng(n + groups)
    status, cmd, ids, conv, ckey, dst = D.rsock_case(rng, n, groups, 4, 8, p_ctrl, 0.95, 0.001)
    got, nv = run_gpu(codec, gpu, status, cmd, D.SERVER_GROUP_FIELDS, ids, conv, ckey, dst)
    exp = oracle.demux_batch(status, cmd, D.SERVER_GROUP_FIELDS, ids, conv, ckey, dst)
    assert nv == exp[1] and len(got) == len(exp[0])
    assert got == exp[0]
    if groups >= 64 and p_ctrl >= 0.002:
        assert len(got) < len(oracle.demux_batch(status, cmd, D.SERVER_FIELDS, ids, conv, ckey, dst)[0]) // 2


def test_demux_table_reuse(codec, gpu, oracle):
    """The key table is filled only when it is not known clean: every call clears the slots its keys
    claimed (k_dm_final), so back-to-back calls reuse it.  Same size with other keys, a larger batch
    (the table moves in the scratch), the first size again, and the group barrier's two passes in
    between: every result equals the oracle."""
    seq = [(70000, 300, ALL), (70000, 5000, ALL | A.DEMUX_CMD_BARRIER), (70000, 70000, A.DEMUX_CONN_KEY),
           (150000, 40, ALL | A.DEMUX_GROUP_BARRIER), (70000, 300, ALL), (1000, 10, A.DEMUX_CONV),
           (70000, 2000, ALL | A.DEMUX_CMD_BARRIER)]
    for k, (n, nkeys, fields) in enumerate(seq):
        rng = np.random.default_rng(100 + k)
        case = make_case(rng, n, nkeys, 0.02, 0.9)
        got = run_gpu(codec, gpu, *case[:2], fields, *case[2:])
        exp = oracle.demux_batch(case[0], case[1], fields, *case[2:])
        assert got[1] == exp[1] and got[0] == exp[0], (k, n, fields)
