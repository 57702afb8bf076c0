"""GPU: header-only batches (rsk_encode_headers_batch / rsk_decode_headers_batch) for host-resident
deployments.  Encode slots must equal the first 32 bytes of the reference's frames (golden
frames.npz from oracle/_ref) and of rsk_encode_batch's frames on the C4 workload; decode on staged
slots must equal the reference's OnRecv outputs (golden onrecv.npz: len-byte variants, nread
0..33, FIN/RST, corrupted tags) and rsk_decode_batch on the whole frames."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import codec as rc
from rsock_amd import workload
from tests.test_gpu_golden import gold
from tests.test_gpu_parity import DEC_VIEWS, dev

pytestmark = pytest.mark.gpu


def run_hdr_encode(codec, gpu, b0, plen, cmd, conv, ckey, idarr=None, id_uniform=b"abcdefgh"):
    import torch

    n = len(plen)
    hdr = torch.full((32 * n,), 0xEE, dtype=torch.uint8, device=gpu)
    st = torch.empty(n, dtype=torch.int32, device=gpu)
    codec.output_headers_batch(dev(b0, gpu), dev(plen, gpu, np.int16), dev(cmd, gpu), dev(conv, gpu, np.int32),
                               dev(ckey, gpu, np.int64), hdr, st, id=None if idarr is None else dev(idarr, gpu),
                               id_uniform=id_uniform)
    torch.cuda.synchronize()
    return hdr.cpu().numpy().reshape(n, 32), st.cpu().numpy()


def test_encode_headers_match_reference_frames(codec, gpu):
    g = gold("frames.npz")
    n = len(g["status"])
    plen = np.minimum(g["pay_len"], 65535).astype(np.uint16)
    po = g["pay_off"].astype(np.int64)
    b0 = np.where(plen > 0, g["payload"][np.minimum(po, len(g["payload"]) - 1)], 0).astype(np.uint8)
    hdr, st = run_hdr_encode(codec, gpu, b0, plen, g["cmd"], g["conv"], g["conn_key"], idarr=g["id"])
    assert np.array_equal(st, g["status"])
    for i in range(n):
        if st[i] > 0:
            o = int(g["frame_off"][i])
            assert hdr[i].tobytes() == g["frames"][o: o + 32].tobytes(), i
        else:
            assert not hdr[i].any()


def test_encode_headers_match_full_encode_c4(codec, gpu):
    import torch

    d = workload.describe("c4", 0, 100000, n=100000)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                       id_uniform=workload.ID_UNIFORM)
    b0 = w.payload[w.pay_off]
    hdr = torch.empty(32 * d.n, dtype=torch.uint8, device=gpu)
    st = torch.empty(d.n, dtype=torch.int32, device=gpu)
    codec.output_headers_batch(b0, w.pay_len, w.cmd, w.conv, w.conn_key, hdr, st, id_uniform=workload.ID_UNIFORM)
    torch.cuda.synchronize()
    assert torch.equal(st, w.status)
    idx = w.frame_off.view(-1, 1) + torch.arange(32, device=gpu).view(1, -1)
    assert torch.equal(hdr.view(-1, 32), w.frame[idx])


def test_decode_headers_match_reference_onrecv(codec, gpu):
    import torch

    from rsock_amd.codec import DecodeBuffers

    g = gold("onrecv.npz")
    n = len(g["status"])
    slots = rc.stage_decode_headers(g["frames"], g["frame_off"], g["frame_len"])
    out = DecodeBuffers.alloc(n, gpu)
    codec.onrecv_headers_batch(dev(slots.reshape(-1), gpu), dev(g["frame_len"].astype(np.uint16), gpu, np.int16), out,
                               is_tcp_close=dev(g["close"].astype(np.uint8), gpu))
    torch.cuda.synchronize()
    got = {k: getattr(out, k).cpu().numpy() for k in DEC_VIEWS}
    for k, dt in DEC_VIEWS.items():
        assert np.array_equal(got[k].view(dt), g[k]), k
    nv = int(out.n_valid.item())
    assert nv == int((g["status"] == 1).sum())
    assert np.array_equal(out.valid_idx[:nv].cpu().numpy().view(np.uint32),
                          np.nonzero(g["status"] == 1)[0].astype(np.uint32))


def test_decode_headers_match_full_decode_c4(codec, gpu):
    import torch

    from rsock_amd.codec import DecodeBuffers

    d = workload.describe("c4", 0, 100000, n=100000)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                       id_uniform=workload.ID_UNIFORM)
    w.corrupt_frames()
    codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec)
    slots = rc.stage_decode_headers(w.frame.cpu().numpy(), w.frame_off.cpu().numpy(), w.frame_len.cpu().numpy()
                                    .astype(np.int32) & 0xFFFF)
    out = DecodeBuffers.alloc(d.n, gpu)
    codec.onrecv_headers_batch(dev(slots.reshape(-1), gpu), w.frame_len, out)
    torch.cuda.synchronize()
    for k in DEC_VIEWS:
        assert torch.equal(getattr(out, k), getattr(w.dec, k)), k
    assert int(out.n_valid.item()) == int(w.dec.n_valid.item())
