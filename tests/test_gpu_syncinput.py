"""GPU: rsk_syncinput_decode_batch (RawTcp::syncInput -> TcpInfo::Decode -> RConn::OnRecv) against
the oracle record by record — every length around the 12 / 21 / 52-byte boundaries, tampered tags,
FIN/RST, records at odd offsets — and the hand-off chain: RawInput's TcpInfo -> rsk_tcpinfo_encode_batch
-> records of TcpInfo + payload (what cap2uv sends) -> rsk_syncinput_decode_batch gives the same
decode as rsk_parse_decode_batch on the captures."""
from __future__ import annotations

import numpy as np
import pytest

from tests import pkt as P
from tests.test_gpu_parity import DEC_VIEWS, KEY, _parse_cases, dev
from tests.test_syncinput_oracle import records

pytestmark = pytest.mark.gpu


def _run(codec, gpu, recs, nread, base_pad=0, align=1):
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers

    arena, offs, _ = P.pack_records(recs, align=align, base_pad=base_pad)
    n = len(recs)
    tcp = TcpInfoBuffers.alloc(n, gpu)
    out = DecodeBuffers.alloc(n, gpu)
    codec.syncinput_batch(dev(arena, gpu), dev(offs, gpu, np.int64), dev(np.asarray(nread, np.int32), gpu), tcp, out)
    torch.cuda.synchronize()
    return tcp.to_host(), out.to_host()


@pytest.mark.parametrize("base_pad", [0, 3])
def test_syncinput_vs_oracle(codec, gpu, oracle, base_pad):
    rs = records(oracle, seed=11)
    recs, nread = [r for r, _ in rs], [n for _, n in rs]
    th, got = _run(codec, gpu, recs, nread, base_pad=base_pad)
    valid = []
    for i, (rec, nr) in enumerate(rs):
        t, d = oracle.syncinput(KEY, rec, nr)
        assert th["parse_status"][i] == t.parse_status, i
        assert (th["src"].view(np.uint32)[i], th["dst"].view(np.uint32)[i], th["sp"].view(np.uint16)[i],
                th["dp"].view(np.uint16)[i], th["seq"].view(np.uint32)[i], th["ack"].view(np.uint32)[i],
                th["flag"][i]) == (t.src, t.dst, t.sp, t.dp, t.seq, t.ack, t.flag), i
        assert th["cap_pay_off"].view(np.uint16)[i] == t.cap_pay_off and \
            th["cap_pay_len"].view(np.uint16)[i] == t.cap_pay_len, i
        assert got["status"][i] == d.status, i
        assert (got["hlen"][i], got["cmd"][i], got["id"].reshape(-1, 8)[i].tobytes(),
                got["conv"].view(np.uint32)[i], got["conn_key"].view(np.uint64)[i],
                got["pay_off"].view(np.uint16)[i], got["pay_len"].view(np.uint16)[i]) == \
            (d.hlen, d.cmd, bytes(d.id), d.conv, d.conn_key, d.pay_off, d.pay_len), i
        if d.status == 1:
            valid.append(i)
    nv = int(got["n_valid"][0])
    assert nv == len(valid) > 50 and np.array_equal(got["valid_idx"][:nv].view(np.uint32), valid)
    assert (got["status"] == 0).any()       # CLOSE_NOTIFY reached through the record's flag


def test_handoff_chain_equals_rawinput(codec, gpu, oracle):
    """cap2uv (RawTcp.cpp:239-260) -> syncInput (:262-276) == the fused parse + decode."""
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers

    rng = np.random.default_rng(21)
    pk, meta = _parse_cases(oracle, rng)
    sel = [i for i, p in enumerate(pk) if p[12:14] == b"\x08\x00"]   # EN10MB IPv4 cases
    recs = [pk[i] for i in sel]
    wl = np.array([meta[i][0] for i in sel], np.uint32)
    cl = np.array([meta[i][1] for i in sel], np.uint32)
    arena, offs, _ = P.pack_records(recs, align=1, base_pad=1)
    n = len(recs)
    tcp = TcpInfoBuffers.alloc(n, gpu)
    out = DecodeBuffers.alloc(n, gpu)
    codec.rawinput_batch(dev(arena, gpu), dev(offs, gpu, np.int64), dev(wl, gpu, np.int32), dev(cl, gpu, np.int32),
                         1, 0, tcp, out)
    hrec = torch.empty(n * 21, dtype=torch.uint8, device=gpu)
    codec.tcpinfo_encode_batch(tcp.src, tcp.dst, tcp.sp, tcp.dp, tcp.seq, tcp.ack, tcp.flag, hrec)
    torch.cuda.synchronize()
    th, exp = tcp.to_host(), out.to_host()
    hr = hrec.cpu().numpy().reshape(n, 21)
    deliver = np.nonzero(th["parse_status"] == 1)[0]
    assert len(deliver) > 5
    # the records cap2uv would send: TcpInfo + payload (cap_pay_len bytes at cap_pay_off)
    hand, nread = [], []
    for i in deliver:
        po, pl = int(th["cap_pay_off"].view(np.uint16)[i]), int(th["cap_pay_len"].view(np.uint16)[i])
        pay = arena[int(offs[i]) + po: int(offs[i]) + po + pl].tobytes()
        hand.append(hr[i].tobytes() + pay)
        nread.append(21 + pl)
    th2, got = _run(codec, gpu, hand, nread, base_pad=5)
    for k, dt in DEC_VIEWS.items():
        g, e = got[k].view(dt), exp[k].view(dt)
        if k == "id":
            g, e = g.reshape(-1, 8), e.reshape(-1, 8)
        assert np.array_equal(g, e[deliver]), k
    for k in ("src", "dst", "sp", "dp", "seq", "ack", "flag"):
        assert np.array_equal(th2[k], th[k][deliver]), k
