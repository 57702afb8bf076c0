"""GPU: the overlapped two-pass encode (round 6): the batch in chunks, each chunk's copy on the caller's
stream while the next chunk's header pass runs on the context's second stream, records double-buffered
(rsk__set_two_pass_overlap).  Bytes equal the per-set kernel's, eagerly and replayed from a captured
graph."""
from __future__ import annotations

import pytest

from rsock_amd import workload

pytestmark = pytest.mark.gpu


def _enc(cx, w, d, stream=None):
    cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off, w.status,
                    id_uniform=workload.ID_UNIFORM, pad16=d.pad == 16, pad128=d.pad == 128, stream=stream)


@pytest.mark.parametrize("cfg,n,chunk,k", [("c3", 300_000, 1 << 16, 1), ("c4", 200_000, 1 << 15, 4),
                                           ("c4", 100_001, 40_000, 2), ("c3", 70_000, 1 << 16, 2)])
def test_overlap_equals_per_set(gpu, cfg, n, chunk, k):
    import torch

    from rsock_amd.codec import Codec

    d = workload.describe(cfg, 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        cx.set_encode_path(1)
        w.frame.zero_()
        _enc(cx, w, d)
        torch.cuda.synchronize()
        ref_f, ref_s = w.frame.clone(), w.status.clone()
        cx.set_encode_path(2)
        cx.set_copy_k(k)
        cx.set_two_pass_overlap(chunk)
        for _ in range(2):
            w.frame.zero_()
            w.status.zero_()
            _enc(cx, w, d)
            assert (cx.last_encode_path, cx.last_copy_k) == (2, k)
            torch.cuda.synchronize()
            assert torch.equal(w.status, ref_s)
            assert torch.equal(w.frame, ref_f)
    finally:
        cx.close()


def test_overlap_in_a_captured_graph(gpu):
    """The fork to the second stream and the joins are recorded into the graph: a replay writes the
    same bytes, and the stream stays usable afterwards."""
    import torch

    from rsock_amd.codec import Codec

    n = 262_144
    d = workload.describe("c3", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        cx.set_encode_path(1)
        _enc(cx, w, d)
        torch.cuda.synchronize()
        ref = w.frame.clone()
        cx.set_encode_path(2)
        cx.set_two_pass_overlap(1 << 16)
        s = torch.cuda.Stream(gpu)
        cx.reserve(n, stream=s)
        with torch.cuda.stream(s):
            _enc(cx, w, d, stream=s)  # eager: creates the second stream, sizes the records
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            _enc(cx, w, d, stream=s)
        w.frame.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(w.frame, ref)
        del g
        w.frame.zero_()
        with torch.cuda.stream(s):
            _enc(cx, w, d, stream=s)
        torch.cuda.synchronize()
        assert torch.equal(w.frame, ref)
    finally:
        cx.close()
