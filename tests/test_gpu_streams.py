"""GPU: one context driven from two streams at once.  The compaction's look-back state is per
stream (rsk_ctx.h stream_compact), so two compacting decodes issued back to back on different
streams — overlapping on the device — each give their own batch's VALID list (include/rsk_codec.h,
"Streams").  The state words carry a per-call epoch instead of being reset per call; the epoch
wraps after 65535 calls (the state is zeroed then)."""
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


def test_compaction_epochs_wrap(codec, gpu):
    """65 540 compacting decodes on one stream: two batches alternate (different VALID lists and
    block counts), so a state word left by the previous call that were taken as this call's would
    show up as a wrong prefix; checked around the epoch wrap (call 65 535 -> zeroed state)."""
    import torch

    from rsock_amd.codec import DecodeBuffers

    n = 5000  # 20 blocks, the last one partial
    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM)
    torch.cuda.synchronize()
    good = w.frame.clone()
    bad_rows = np.nonzero(np.arange(n) % 3 == 1)[0]
    w.frame[w.frame_off[torch.from_numpy(bad_rows).to(gpu)]] ^= 1
    bad = w.frame.clone()
    keep = [np.ones(n, bool), np.arange(n) % 3 != 1]
    exp = [np.nonzero(k)[0].astype(np.int32) for k in keep]
    s = torch.cuda.Stream(gpu)
    outs = [DecodeBuffers.alloc(n, gpu) for _ in range(2)]
    frames = [good, bad]
    checked = 0
    with torch.cuda.stream(s):
        for call in range(65540):
            k = call & 1
            codec.onrecv_batch(frames[k], w.frame_off, w.frame_len, outs[k], stream=s)
            if call in (0, 1, 9, 65533, 65534, 65535, 65536, 65537, 65539):
                s.synchronize()
                nv = int(outs[k].n_valid.item())
                assert nv == exp[k].size, call
                assert np.array_equal(outs[k].valid_idx[:nv].cpu().numpy(), exp[k]), call
                checked += 1
    assert checked == 9
