"""GPU: one context driven from two streams at once.  The compaction's look-back state is per
stream (rsk_ctx.h stream_compact), so two compacting decodes issued back to back on different
streams — overlapping on the device — each give their own batch's VALID list (include/rsk_codec.h,
"Streams").  The look-back words carry a per-call epoch kept on the device instead of being reset
per call, which also makes a captured graph replay correctly."""
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


def _alt_batches(codec, gpu, n):
    import torch

    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM)
    torch.cuda.synchronize()
    good = w.frame.clone()
    bad_rows = np.nonzero(np.arange(n) % 3 == 1)[0]
    w.frame[w.frame_off[torch.from_numpy(bad_rows).to(gpu)]] ^= 1
    bad = w.frame.clone()
    exp = [np.arange(n, dtype=np.int32), np.nonzero(np.arange(n) % 3 != 1)[0].astype(np.int32)]
    return w, [good, bad], exp


def _check(out, exp, what):
    nv = int(out.n_valid.item())
    assert nv == exp.size, what
    assert np.array_equal(out.valid_idx[:nv].cpu().numpy(), exp), what


def test_compaction_state_across_calls(codec, gpu):
    """Compaction look-back words are tagged with a device-side call epoch, never reset per call:
    batches of two sizes (different tile counts) and two VALID patterns alternate on one stream, so
    a word left by an earlier call taken as this call's would show up as a wrong prefix."""
    import torch

    from rsock_amd.codec import DecodeBuffers

    wa, fa, ea = _alt_batches(codec, gpu, 300_000)  # 74 tiles
    wb, fb, eb = _alt_batches(codec, gpu, 5000)     # 2 tiles, the last partial
    s = torch.cuda.Stream(gpu)
    oa, ob = DecodeBuffers.alloc(300_000, gpu), DecodeBuffers.alloc(5000, gpu)
    with torch.cuda.stream(s):
        for call in range(400):
            k = (call >> 1) & 1
            if call & 1:
                codec.onrecv_batch(fb[k], wb.frame_off, wb.frame_len, ob, stream=s)
            else:
                codec.onrecv_batch(fa[k], wa.frame_off, wa.frame_len, oa, stream=s)
            if call % 37 in (0, 1):
                s.synchronize()
                _check(ob if call & 1 else oa, (eb if call & 1 else ea)[k], call)


def test_compaction_in_captured_graph(codec, gpu):
    """A compacting decode captured in a HIP graph and replayed: the epoch advances on the device, so
    every replay's VALID list is right while the frames alternate between two patterns."""
    import torch

    from rsock_amd.codec import DecodeBuffers

    n = 100_000
    w, frames, exp = _alt_batches(codec, gpu, n)
    out = DecodeBuffers.alloc(n, gpu)
    s = torch.cuda.Stream(gpu)
    with torch.cuda.stream(s):
        codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, out, stream=s)  # workspace sized before capture
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, out, stream=torch.cuda.current_stream())
    for r in range(12):
        k = r % 2 if r < 8 else 1
        w.frame.copy_(frames[k])
        out.n_valid.zero_()
        g.replay()
        torch.cuda.synchronize()
        _check(out, exp[k], r)


def test_compaction_stall_is_flagged_and_recovered(gpu):
    """a look-back that gives up must not go unnoticed.  Tile 1 of one k_compact launch is
    made to publish nothing (rsk__inject_compact_stall, a tile that never runs); tile 2 times out (after
    ~4M polls, no hang), the context's sticky RSK_DEVERR_LOOKBACK flag is raised and
    rsk_check_device_errors reports it once; the next call on the same stream (state re-initialised)
    gives the right VALID list again."""
    import ctypes

    import torch

    from rsock_amd import _abi
    from rsock_amd.codec import Codec, DecodeBuffers, RskError, lib

    n = 64 * 4096  # 64 compaction tiles
    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM)
        w.corrupt_frames()
        keep = np.nonzero(~d.corrupt)[0].astype(np.int32)
        s = torch.cuda.Stream(gpu)
        o = DecodeBuffers.alloc(n, gpu)

        def decode_and_check():
            cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s)
            torch.cuda.synchronize()
            nv = int(o.n_valid.item())
            return nv == keep.size and np.array_equal(o.valid_idx[:nv].cpu().numpy(), keep)

        assert decode_and_check() and cx.check_device_errors() == 0
        fn = lib().rsk__inject_compact_stall
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        assert fn(cx._ctx, 1) == 0
        assert not decode_and_check()  # tiles 2.. took a wrong prefix
        # the count is poisoned whatever tile gave up (the last tile checks every word)
        assert int(o.n_valid.item()) & 0xFFFFFFFF == 0xFFFFFFFF  # int32 storage of the u32
        with pytest.raises(RskError, match="0x1"):
            cx.check_device_errors()
        assert cx.check_device_errors() == 0  # read and cleared
        for _ in range(3):  # state re-zeroed at the next call: right again, epochs run on
            assert decode_and_check()
        assert cx.check_device_errors() == 0
        flags = ctypes.c_uint32(7)
        assert lib().rsk_check_device_errors(cx._ctx, ctypes.byref(flags)) == 0 and flags.value == 0
        assert _abi.DEVERR_LOOKBACK == 1
    finally:
        cx.close()


def test_capture_needs_reserved_stream_and_release(gpu):
    """A compacting decode captured on a stream whose scratch was never set up is refused (RSK_EINVAL,
    rsk_codec.h "Streams"), not recorded with a memset that has not run; after reserve + one eager call
    the capture works; rsk_release_stream frees the stream's scratch and a later call re-creates it."""
    import torch

    from rsock_amd.codec import Codec, DecodeBuffers, RskError

    n = 8192
    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM)
        torch.cuda.synchronize()
        o = DecodeBuffers.alloc(n, gpu)
        s = torch.cuda.Stream(gpu)
        g = torch.cuda.CUDAGraph()
        with pytest.raises(RskError):
            with torch.cuda.graph(g, stream=s):
                cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s)
        torch.cuda.synchronize()
        s2 = torch.cuda.Stream(gpu)
        cx.reserve(n, stream=s2)
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s2)  # eager: initialises the state
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s2):
            cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s2)
        o.n_valid.zero_()
        g2.replay()
        torch.cuda.synchronize()
        assert int(o.n_valid.item()) == n
        del g2
        cx.release_stream(s2)
        o.n_valid.zero_()
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s2)  # scratch re-created
        torch.cuda.synchronize()
        assert int(o.n_valid.item()) == n
        assert cx.check_device_errors() == 0
    finally:
        cx.close()


def _c3_frames(codec, gpu, w, path, stream=None):
    import torch

    codec.set_encode_path(path)
    w.frame.zero_()
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=stream)
    torch.cuda.synchronize()
    return w.frame.clone(), w.status.clone()


def test_two_pass_encode_in_captured_graph(gpu):
    """The two-pass encode (header records in the capture stream's scratch, then one wave per packet)
    captured into a hipGraph and replayed gives the per-set kernel's bytes; a stream whose records were
    not reserved captures the per-set kernel instead (same bytes), never an allocation."""
    import torch

    from rsock_amd.codec import Codec

    n = 1 << 17
    d = workload.describe("c3", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        ref_f, ref_s = _c3_frames(cx, gpu, w, 1)
        for reserved in (True, False):
            s = torch.cuda.Stream(gpu)
            cx.set_encode_path(2)
            if reserved:  # reserves the records because the context is held to the two-pass path
                cx.reserve(n, stream=s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                                w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
            assert cx.last_encode_path == (2 if reserved else 1)
            for _ in range(2):
                w.frame.zero_()
                w.status.fill_(-9)
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                assert torch.equal(w.frame, ref_f) and torch.equal(w.status, ref_s)
            del g
            cx.set_encode_path(0)
            cx.release_stream(s)
    finally:
        cx.close()


def test_two_pass_encode_two_streams(codec, gpu):
    """Two streams of one context encode different batches on the two-pass path at once: each stream
    has its own header records (per-stream scratch), so neither batch sees the other's headers."""
    import torch

    n = 1 << 17
    da = workload.describe("c3", 0, n, n=2 * n)
    db = workload.describe("c3", n, 2 * n, n=2 * n)
    wa, wb = workload.DeviceWorkload(da, gpu), workload.DeviceWorkload(db, gpu)
    ref = [_c3_frames(codec, gpu, w, 1) for w in (wa, wb)]
    sa, sb = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
    codec.set_encode_path(2)
    try:
        for w in (wa, wb):
            w.frame.zero_()
        torch.cuda.synchronize()
        for _ in range(3):
            for w, s in ((wa, sa), (wb, sb)):
                codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame,
                                   w.frame_off, w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
        torch.cuda.synchronize()
    finally:
        codec.set_encode_path(0)
    for w, (f, st) in zip((wa, wb), ref):
        assert torch.equal(w.frame, f) and torch.equal(w.status, st)


def test_two_pass_copy_k_in_captured_graph(gpu):
    """The two-pass encode with 1, 2 and 4 packets per copy wave, in several chunks of heads / copy
    (rsk__set_two_pass_chunk: each chunk's launches start at a packet offset), captured into a hipGraph on
    a reserved stream and replayed: the per-set kernel's bytes."""
    import torch

    from rsock_amd.codec import Codec

    n = (1 << 17) + 77
    d = workload.describe("c4", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        ref_f, ref_s = _c3_frames(cx, gpu, w, 1)
        for k, chunk in ((1, 0), (2, 50_000), (4, 0), (4, 33_333)):
            s = torch.cuda.Stream(gpu)
            cx.set_encode_path(2)
            cx.set_copy_k(k)
            cx.set_two_pass_chunk(chunk)
            cx.reserve(n, stream=s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                                w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
            assert cx.last_encode_path == 2
            for _ in range(2):
                w.frame.zero_()
                w.status.fill_(-9)
                torch.cuda.synchronize()
                g.replay()
                torch.cuda.synchronize()
                assert torch.equal(w.frame, ref_f) and torch.equal(w.status, ref_s), (k, chunk)
            del g
            cx.release_stream(s)
        cx.set_encode_path(0)
        cx.set_copy_k(0)
        cx.set_two_pass_chunk(0)
        assert cx.check_device_errors() == 0  # a captured context waits for the device here
    finally:
        cx.close()


def test_check_errors_after_stream_destroyed_unreleased(gpu):
    """a stream that ran a compacting decode is destroyed without rsk_release_stream.
    rsk_check_device_errors must still work (the stale handle's scratch is dropped, not synced forever
    as an error), and the context keeps decoding on other streams."""
    import ctypes

    import torch

    from rsock_amd.codec import Codec, DecodeBuffers

    hip = ctypes.CDLL("libamdhip64.so")
    n = 50_000
    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM)
        torch.cuda.synchronize()
        o = DecodeBuffers.alloc(n, gpu)
        for _ in range(2):
            raw = ctypes.c_void_p()
            assert hip.hipStreamCreate(ctypes.byref(raw)) == 0
            cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=raw.value)
            assert hip.hipStreamSynchronize(raw) == 0
            assert int(o.n_valid.item()) == n
            assert hip.hipStreamDestroy(raw) == 0  # no rsk_release_stream
            assert cx.check_device_errors() == 0
            assert cx.check_device_errors() == 0
        o.n_valid.zero_()
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o)
        torch.cuda.synchronize()
        assert int(o.n_valid.item()) == n and cx.check_device_errors() == 0
    finally:
        cx.close()


def test_auto_capture_takes_two_pass_after_back_to_back_calls(gpu):
    """bench.py's sequence on an AUTO context: reserve the stream, a few eager calls issued back to back
    (all of them run before the first batch statistic reaches the host, so they take the per-set kernel),
    synchronize, capture.  The capture must take the two-pass form with its reserved records -- in r05's
    first build the records were not reserved for AUTO contexts and the graph silently captured the
    per-set kernel (4 % of the bench line)."""
    import torch

    from rsock_amd.codec import Codec

    n = 1 << 17
    d = workload.describe("c3", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        s = torch.cuda.Stream(gpu)
        cx.reserve(n, stream=s)
        with torch.cuda.stream(s):
            for _ in range(5):
                cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                                w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
        torch.cuda.synchronize()
        ref = w.frame.clone()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                            w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
        assert (cx.last_encode_path, cx.last_copy_k) == (2, 1)
        w.frame.zero_()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(w.frame, ref)
        del g
    finally:
        cx.close()


def test_reserve_records_only_for_encoding_contexts(gpu):
    """rsk_reserve_stream allocates the two-pass records (32 B per packet) only for a context
    that encodes -- a decode-only AUTO context reserves the compaction state alone; after one encode call
    the same reserve on a new stream also takes the records."""
    import torch

    from rsock_amd.codec import Codec

    n = 1 << 22
    cx = Codec(b"hello135", 0)
    try:
        s1, s2 = torch.cuda.Stream(gpu), torch.cuda.Stream(gpu)
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(gpu)[0]
        cx.reserve(n, stream=s1)
        torch.cuda.synchronize()
        used_dec = free0 - torch.cuda.mem_get_info(gpu)[0]
        assert used_dec < 16 * n, used_dec  # the compaction state (a few B per packet), no records
        m = 20_000
        d = workload.describe("c3", 0, m, n=m)
        w = workload.DeviceWorkload(d, gpu)
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM, pad16=True)
        torch.cuda.synchronize()
        free1 = torch.cuda.mem_get_info(gpu)[0]
        cx.reserve(n, stream=s2)
        torch.cuda.synchronize()
        used_enc = free1 - torch.cuda.mem_get_info(gpu)[0]
        assert used_enc >= 32 * n, used_enc
        cx.release_stream(s1)
        cx.release_stream(s2)
    finally:
        cx.close()


def test_forget_captures(gpu):
    """a captured call makes rsk_check_device_errors wait for the whole device; once the
    graph is gone, rsk_forget_captures returns the context to waiting for its own streams."""
    import torch

    from rsock_amd.codec import Codec, DecodeBuffers

    n = 50_000
    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    cx = Codec(b"hello135", 0)
    try:
        s = torch.cuda.Stream(gpu)
        o = DecodeBuffers.alloc(n, gpu)
        cx.reserve(n, stream=s)
        with torch.cuda.stream(s):
            cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                            w.status, id_uniform=workload.ID_UNIFORM, stream=s)
            cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s)
        o.n_valid.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert int(o.n_valid.item()) == n
        assert cx.check_device_errors() == 0
        del g
        cx.forget_captures()
        assert cx.check_device_errors() == 0
        o.n_valid.zero_()
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, o, stream=s)
        torch.cuda.synchronize()
        assert int(o.n_valid.item()) == n and cx.check_device_errors() == 0
    finally:
        cx.close()
