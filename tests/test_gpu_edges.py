"""GPU: empty batches and argument errors of every batch entry point (include/rsk_codec.h).
An empty batch is a no-op that may pass null arrays and zeroes a given count; a non-empty batch with
a missing array, a bad link type or a misaligned buffer is rejected with RSK_EINVAL before any
launch, and the context stays usable."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import _abi
from rsock_amd import codec as rc
from rsock_amd import workload

pytestmark = pytest.mark.gpu
KEY = b"hello135"


def _e(gpu, dt):
    import torch

    return torch.empty(0, dtype=dt, device=gpu)


def _poisoned_count(gpu):
    import torch

    return torch.full((1,), 12345, dtype=torch.int32, device=gpu)


def test_empty_batches_are_noops(codec, gpu):
    import torch

    u8, i16, i32, i64 = (_e(gpu, t) for t in (torch.uint8, torch.int16, torch.int32, torch.int64))
    codec.output_batch(u8, i64, i16, u8, i32, i64, u8, i64, i32)
    codec.output_wire_batch(u8, i64, i16, u8, i32, i64, i32, i32, i16, i16, i32, i32, u8, i16, u8, i64, i32)
    codec.output_headers_batch(u8, i16, u8, i32, i64, u8, i32)
    codec.tcpinfo_encode_batch(i32, i32, i16, i16, i32, i32, u8, u8)
    dec = rc.DecodeBuffers(hlen=u8, cmd=u8, id=u8, conv=i32, conn_key=i64, pay_off=i16, pay_len=i16,
                           status=_e(gpu, torch.int8), valid_idx=i32, n_valid=_poisoned_count(gpu))
    codec.onrecv_batch(u8, i64, i16, dec)
    torch.cuda.synchronize()
    assert int(dec.n_valid.item()) == 0
    dec.n_valid.fill_(7)
    codec.onrecv_headers_batch(u8, i16, dec)
    torch.cuda.synchronize()
    assert int(dec.n_valid.item()) == 0
    tcp = rc.TcpInfoBuffers(src=i32, dst=i32, sp=i16, dp=i16, seq=i32, ack=i32, flag=u8,
                            parse_status=_e(gpu, torch.int8), cap_pay_off=i16, cap_pay_len=i16)
    for dl in (0, 1):
        dec.n_valid.fill_(7)
        codec.rawinput_batch(u8, i64, i32, i32, dl, 0, tcp, dec)
        torch.cuda.synchronize()
        assert int(dec.n_valid.item()) == 0
        dec.n_valid.fill_(7)
        codec.rawinput_slots_batch(u8, 96, i32, i32, dl, 3, tcp, dec)
        torch.cuda.synchronize()
        assert int(dec.n_valid.item()) == 0
    dec.n_valid.fill_(7)
    codec.syncinput_batch(u8, i64, i32, tcp, dec)
    torch.cuda.synchronize()
    assert int(dec.n_valid.item()) == 0
    nm = _poisoned_count(gpu)
    codec.capture_filter_batch(u8, i64, i32, 1, rc.make_filter(dst_singles=[10001]), u8, i32, nm)
    torch.cuda.synchronize()
    assert int(nm.item()) == 0
    # the context still works afterwards
    d = workload.describe("c2", 0, 300, n=300)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM)
    codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec)
    torch.cuda.synchronize()
    assert int(w.dec.n_valid.item()) == 300


def _lib_and_ctx(codec):
    return rc.lib(), codec._ctx


def test_missing_arrays_and_bad_arguments_rejected(codec, gpu):
    import ctypes

    import torch

    lib, ctx = _lib_and_ctx(codec)
    n = 64
    buf = torch.zeros(1 << 16, dtype=torch.uint8, device=gpu)
    p = buf.data_ptr()
    # decode: a missing frame_len
    dout = rc.DecodeBuffers.alloc(n, gpu)
    assert lib.rsk_decode_batch(ctx, n, p, p, None, None, ctypes.byref(dout.abi()), None) == _abi.EINVAL
    # decode: misaligned id output (8-B alignment)
    bad = dout.abi()
    bad.id = p + 1
    assert lib.rsk_decode_batch(ctx, n, p, p, p, None, ctypes.byref(bad), None) == _abi.EINVAL
    # decode_headers: slots must be 16-B aligned
    assert lib.rsk_decode_headers_batch(ctx, n, p + 8, p, None, ctypes.byref(dout.abi()), None) == _abi.EINVAL
    # parse: bad datalink (RawTcp.cpp:161-164 accepts EN10MB and NULL only), missing TcpInfo array
    tcp = rc.TcpInfoBuffers.alloc(n, gpu)
    for dl in (2, 105, -1):
        assert lib.rsk_parse_decode_batch(ctx, n, p, p, p, p, dl, 0, ctypes.byref(tcp.abi()),
                                          ctypes.byref(dout.abi()), None) == _abi.EINVAL
    t = tcp.abi()
    t.seq = None
    assert lib.rsk_parse_decode_batch(ctx, n, p, p, p, p, 1, 0, ctypes.byref(t), ctypes.byref(dout.abi()),
                                      None) == _abi.EINVAL
    # slots: below the minimum, not a multiple of 16, misaligned slot arena
    for slot, base in ((48, p), (72, p), (96, p + 4)):
        assert lib.rsk_parse_decode_slots_batch(ctx, n, base, slot, p, p, 1, 0, ctypes.byref(tcp.abi()),
                                                ctypes.byref(dout.abi()), None) == _abi.EINVAL
    # encode: misaligned per-packet IdBuf array
    ein = _abi.EncodeIn(p, p, p, p, p, p, p + 3, (ctypes.c_uint8 * 8)())
    eout = _abi.EncodeOut(p, p, p, 0)
    assert lib.rsk_encode_batch(ctx, n, ctypes.byref(ein), ctypes.byref(eout), None) == _abi.EINVAL
    # syncinput: missing nread, missing TcpInfo array
    assert lib.rsk_syncinput_decode_batch(ctx, n, p, p, None, ctypes.byref(tcp.abi()), ctypes.byref(dout.abi()),
                                          None) == _abi.EINVAL
    assert lib.rsk_syncinput_decode_batch(ctx, n, p, p, p, ctypes.byref(t), ctypes.byref(dout.abi()),
                                          None) == _abi.EINVAL
    # tcpinfo: a missing field array
    assert lib.rsk_tcpinfo_encode_batch(ctx, n, p, p, p, p, p, None, p, p, None) == _abi.EINVAL
    # null context everywhere
    assert lib.rsk_decode_batch(None, 0, None, None, None, None, ctypes.byref(dout.abi()), None) == _abi.EINVAL
    assert lib.rsk_tcpinfo_encode_batch(None, 0, None, None, None, None, None, None, None, None, None) == _abi.EINVAL
    torch.cuda.synchronize()
    # still usable
    d = workload.describe("c4", 0, 500, n=500)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM)
    torch.cuda.synchronize()
    assert np.array_equal(w.status.cpu().numpy(), d.pay_len.astype(np.int32) + 31)
