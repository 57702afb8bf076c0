"""GPU: one context driven from two streams at once.  The compaction scratch (ballot masks, block
counts, offsets) is per stream (rsk_ctx.h stream_ws), so two compacting decodes issued back to back
on different streams — overlapping on the device — each give their own batch's VALID list
(include/rsk_codec.h, "Streams")."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import workload

pytestmark = pytest.mark.gpu


def test_two_streams_one_ctx_compacting_decode(codec, gpu):
    import torch

    from rsock_amd.codec import DecodeBuffers

    n = 1 << 20
    da = workload.describe("c4", 0, n, n=2 * n)
    db = workload.describe("c4", n, 2 * n, n=2 * n)
    wa, wb = workload.DeviceWorkload(da, gpu), workload.DeviceWorkload(db, gpu)
    for w in (wa, wb):
        codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                           w.status, id_uniform=workload.ID_UNIFORM)
    torch.cuda.synchronize()
    wa.corrupt_frames()
    wb.corrupt_frames()
    # batch B: also every 5th frame corrupted, so the two VALID lists differ everywhere
    extra = np.nonzero(np.arange(n) % 5 == 3)[0]
    pos = wb.frame_off[torch.from_numpy(extra).to(gpu)]
    wb.frame[pos] ^= 2
    keep_a = ~da.corrupt
    keep_b = ~db.corrupt & (np.arange(n) % 5 != 3)
    sa, sb = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    ev = torch.cuda.Event()
    ev.record()
    sa.wait_event(ev)
    sb.wait_event(ev)
    outs_a = [DecodeBuffers.alloc(n, gpu) for _ in range(3)]
    outs_b = [DecodeBuffers.alloc(n, gpu) for _ in range(3)]
    for k in range(3):
        first, second = ((wa, outs_a[k], sa), (wb, outs_b[k], sb)) if k % 2 == 0 else \
            ((wb, outs_b[k], sb), (wa, outs_a[k], sa))
        for w, o, s in (first, second):
            codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s)
    torch.cuda.synchronize()
    for outs, keep in ((outs_a, keep_a), (outs_b, keep_b)):
        exp = np.nonzero(keep)[0].astype(np.int32)
        for o in outs:
            nv = int(o.n_valid.item())
            assert nv == exp.size
            assert np.array_equal(o.valid_idx[:nv].cpu().numpy(), exp)
            assert np.array_equal(o.status.cpu().numpy() == 1, keep)


def test_reserve_stream(codec, gpu):
    import torch

    s = torch.cuda.Stream(gpu)
    codec.reserve(1 << 16, stream=s)
    codec.reserve(1 << 10)
