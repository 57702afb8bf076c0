"""GPU: rsk_filter_parse_decode_batch (capture filter + RawTcp::RawInput + RConn::OnRecv in one
pass) equals the two separate steps: match = the oracle's pcap predicate; for matched packets the
parse + decode outputs equal the oracle's on the whole batch, for rejected ones RSK_PARSE_DROP with
zero outputs; the VALID list is the matched-and-verified packets in order.  Inputs: the parse edge
cases of test_gpu_parity (IHL / data offset variants, SYN, FIN/RST, truncation, oversize) and
Ethernet packets from rsk_encode_wire_batch with ports in and out of the filter's set."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import codec as rc
from tests import pkt as P
from tests.test_gpu_parity import DEC_VIEWS, KEY, _parse_cases, dev

pytestmark = pytest.mark.gpu

TCP_FIELDS = (("src", np.uint32), ("dst", np.uint32), ("sp", np.uint16), ("dp", np.uint16), ("seq", np.uint32),
              ("ack", np.uint32), ("flag", np.uint8), ("parse_status", np.int8), ("cap_pay_off", np.uint16),
              ("cap_pay_len", np.uint16))


def _check(codec, gpu, oracle, recs, wl, cl, dl, flags, f):
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers

    arena, offs, _ = P.pack_records(recs, align=1, base_pad=3)
    n = len(recs)
    tcp = TcpInfoBuffers.alloc(n, gpu)
    out = DecodeBuffers.alloc(n, gpu)
    match = torch.empty(n, dtype=torch.uint8, device=gpu)
    codec.filter_rawinput_batch(dev(arena, gpu), dev(offs, gpu, np.int64), dev(wl, gpu, np.int32),
                                dev(cl, gpu, np.int32), dl, flags, f, match, tcp, out)
    torch.cuda.synchronize()
    m_exp = np.array([oracle.capture_filter(arena[int(o):int(o) + int(c)].tobytes(), dl, f, cap_len=int(c))
                      for o, c in zip(offs, cl)], np.uint8)
    assert np.array_equal(match.cpu().numpy(), m_exp)
    exp = oracle.parse_decode_batch(KEY, arena, offs, wl, cl, dl, flags)
    keep = m_exp.astype(bool)
    th = tcp.to_host()
    for k, dt in TCP_FIELDS:
        g = th[k].view(dt)
        assert np.array_equal(g[keep], exp[k][keep]), k
        assert not g[~keep].any(), k
    got = out.to_host()
    for k, dt in DEC_VIEWS.items():
        g = got[k].view(dt)
        if k == "id":
            g8, e8 = g.reshape(n, 8), exp[k].reshape(n, 8)
            assert np.array_equal(g8[keep], e8[keep]) and not g8[~keep].any()
        elif k == "status":
            assert np.array_equal(g[keep], exp[k][keep]) and (g[~keep] == -1).all()
        else:
            assert np.array_equal(g[keep], exp[k][keep]), k
            assert not g[~keep].any(), k
    ev = exp["valid_idx"][:exp["n_valid"]]
    ev = ev[keep[ev]]
    nv = int(got["n_valid"][0])
    assert nv == len(ev) and np.array_equal(got["valid_idx"][:nv].view(np.uint32), ev)
    return keep


@pytest.mark.parametrize("flags", [0, 3])
@pytest.mark.parametrize("server", [False, True])
def test_filter_parse_edge_cases(codec, gpu, oracle, flags, server):
    rng = np.random.default_rng(5)
    pk, meta = _parse_cases(oracle, rng)
    # ports 1..2 / 10001 / 43932 appear in the cases; the filter passes some and rejects others
    f = rc.make_filter(dst_singles=[2, 43932], src_ranges=[(1, 10001)], is_server=server)
    for dl in (1, 0):
        sel = [i for i, p in enumerate(pk) if (p[12:14] in (b"\x08\x00", b"\x86\xdd")) == (dl == 1)]
        recs = [pk[i] for i in sel]
        wl = np.array([meta[i][0] for i in sel], np.uint32)
        cl = np.array([meta[i][1] for i in sel], np.uint32)
        keep = _check(codec, gpu, oracle, recs, wl, cl, dl, flags, f)
        assert keep.any()


def test_filter_parse_wire_packets(codec, gpu, oracle):
    """rsk_encode_wire_batch packets to dport 10001..10012: the filter passes 10001..10010 only."""
    import torch

    from rsock_amd import workload

    n = 3000
    d = workload.describe("c4", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    src = torch.full((n,), rc.ip_u32("10.0.0.1"), dtype=torch.int64, device=gpu).to(torch.int32)
    dst = torch.full((n,), rc.ip_u32("10.0.0.2"), dtype=torch.int64, device=gpu).to(torch.int32)
    sp = torch.full((n,), 43000, dtype=torch.int32, device=gpu).to(torch.int16)
    dp = (10001 + torch.arange(n, device=gpu) % 12).to(torch.int16)
    z32 = torch.zeros(n, dtype=torch.int32, device=gpu)
    flag = torch.full((n,), 0x18, dtype=torch.uint8, device=gpu)
    pitch = 1488
    wire = torch.zeros(n * pitch, dtype=torch.uint8, device=gpu)
    woff = torch.arange(n, device=gpu, dtype=torch.int64) * pitch
    st = torch.empty(n, dtype=torch.int32, device=gpu)
    codec.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, src, dst, sp, dp, z32, z32,
                            flag, z32.to(torch.int16), wire, woff, st, eth=bytes(12) + b"\x08\x00",
                            id_uniform=workload.ID_UNIFORM)
    torch.cuda.synchronize()
    h, sts = wire.cpu().numpy(), st.cpu().numpy()
    ok = np.nonzero(sts > 0)[0]
    recs = [h[i * pitch: i * pitch + sts[i]].tobytes() for i in ok]
    ln = sts[ok].astype(np.uint32)
    f = rc.make_filter(dst_ip="10.0.0.2", dst_singles=[10001, 10002], dst_ranges=[(10003, 10010)])
    keep = _check(codec, gpu, oracle, recs, ln, ln, 1, 0, f)
    dpn = (dp.cpu().numpy().astype(np.int32) & 0xFFFF)[ok]
    assert np.array_equal(keep, dpn <= 10010)
