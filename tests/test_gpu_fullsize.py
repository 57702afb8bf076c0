"""Full BASELINE sizes (C2 1M x 64 B, C3 4M x 1400 B, C4 1M mixed, a C5 shard of 8M x 1400 B)
through size-independent properties checked on the device:
  * encode -> decode round trip: every framed packet verifies, compaction is the identity list
  * frame payload region == payload bytes; header bytes == the SoA fields (LE)
  * tag bytes == the oracle's 256-entry tag table at payload[0] (the tag depends only on it)
  * C4: exactly the corrupted frames drop, valid_idx is the order-stable list of the others
"""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import workload
from tests.enc_paths import ENC_PATHS, held, path_id

pytestmark = pytest.mark.gpu
KEY = b"hello135"


def _tag_table(oracle, gpu):
    import torch

    t = np.frombuffer(b"".join(oracle.tag(KEY, b) for b in range(256)), np.uint8).reshape(256, 8)
    return torch.from_numpy(t.copy()).to(gpu)


def _le_bytes(x, nbytes):
    import torch

    x = x.to(torch.int64)
    return torch.stack([(x >> (8 * k)) & 0xFF for k in range(nbytes)], dim=1).to(torch.uint8)


@pytest.fixture(params=ENC_PATHS, ids=path_id)
def pcodec(request, codec):
    """The codec held to one encode path (tests/enc_paths.py): each encode asserts the path it took."""
    with held(codec, *request.param) as c:
        yield c


@pytest.mark.parametrize("cfg", ["c3", "c2", "c4"])
@pytest.mark.parametrize("pad16", [True, False])
def test_fullsize_roundtrip(pcodec, gpu, oracle, cfg, pad16):
    _roundtrip(pcodec, gpu, oracle, workload.describe(cfg), pad16)


# what AUTO (path 0) takes for each BASELINE config once it has sampled one batch of it
# (rsk_kernels.hip, enc_path / copy_k: by the sampled mean payload): (path, packets per copy wave)
AUTO_EXPECT = {"c2": (3, 0), "c3": (2, 1), "c4": (2, 4)}


def test_encode_path_choice(codec, gpu):
    """Path 0 (the default) picks per call from the previous batch's sampled mean payload:
    the frames are the same whichever path runs, and after ONE call of a new traffic mix the next call
    takes that mix's path -- C2 then C3 then C4 then C2 then C3, each switch within one call."""
    import torch

    ref = {}
    for cfg in ("c3", "c4", "c2"):
        d = workload.describe(cfg, 0, 40_000, n=40_000)
        w = workload.DeviceWorkload(d, gpu)
        codec.set_encode_path(1)
        w.frame.zero_()
        codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                           w.status, id_uniform=workload.ID_UNIFORM, pad16=True)
        torch.cuda.synchronize()
        ref[cfg] = (w, w.frame.clone())
    codec.set_encode_path(0)
    for cfg in ("c2", "c3", "c4", "c2", "c3"):
        w, rf = ref[cfg]
        for call in range(2):
            w.frame.zero_()
            codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                               w.status, id_uniform=workload.ID_UNIFORM, pad16=True)
            torch.cuda.synchronize()
            assert torch.equal(w.frame, rf), (cfg, call)
        path, k = AUTO_EXPECT[cfg]
        assert codec.last_encode_path == path, (cfg, codec.last_encode_path)
        if path == 2:
            assert codec.last_copy_k == k, (cfg, codec.last_copy_k)


@pytest.mark.parametrize("cfg", ["c3", "c4", "c2"])
def test_encode_path_first_call(gpu, cfg):
    """A fresh context has no batch statistic: its first AUTO call of >= 16384 packets samples its own
    batch (one 64-thread launch, waited for once) and already takes the table's path, and so do calls
    issued back to back after it without synchronisation (gpurun_out/r05f1/c3 showed 5 eager calls on
    the per-set kernel before this)."""
    import torch
    from rsock_amd.codec import Codec

    d = workload.describe(cfg, 0, 40_000, n=40_000)
    w = workload.DeviceWorkload(d, gpu)
    path, k = AUTO_EXPECT[cfg]
    s = torch.cuda.Stream(gpu)
    torch.cuda.synchronize()
    c = Codec(b"hello135", 0)
    try:
        for call in range(3):
            c.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                           w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=s)
            assert c.last_encode_path == path, (cfg, call, c.last_encode_path)
            if path == 2:
                assert c.last_copy_k == k, (cfg, call, c.last_copy_k)
        torch.cuda.synchronize()
        assert torch.equal(w.status.to(torch.int64), (w.pay_len.to(torch.int64) & 0xFFFF) + 31)
    finally:
        c.close()
    # on the legacy NULL stream the first call does not wait: it takes the per-set kernel
    # (same bytes), and once its sample has landed the table's path follows
    c = Codec(b"hello135", 0)
    try:
        null = 0  # the legacy NULL stream
        c.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=null)
        assert c.last_encode_path == 1, (cfg, c.last_encode_path)
        torch.cuda.synchronize()
        c.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM, pad16=True, stream=null)
        assert c.last_encode_path == path, (cfg, c.last_encode_path)
        torch.cuda.synchronize()
        assert torch.equal(w.status.to(torch.int64), (w.pay_len.to(torch.int64) & 0xFFFF) + 31)
    finally:
        c.close()


@pytest.mark.parametrize("rank", [7, 0])
def test_c5_shard_roundtrip(pcodec, gpu, oracle, rank):
    """BASELINE config 5 (64M x 1400-B packets sharded 8 ways): the shard rank `rank` of 8 runs on
    one device (8M packets, ~23 GB of arenas) — what each GPU of the 8-GPU bench line computes."""
    codec = pcodec
    lo, hi = workload.shard_range(64 << 20, rank, 8)
    d = workload.describe("c5", lo, hi, n=64 << 20)
    assert d.n == 8 << 20 and d.first == lo
    _roundtrip(codec, gpu, oracle, d, True)


def _roundtrip(codec, gpu, oracle, d, pad16):
    import torch

    w = workload.DeviceWorkload(d, gpu)
    n = d.n
    # the device-generated arena is this shard's slice of the config's payload byte stream
    head = workload.splitmix_bytes_np(d.payload_seed, 1 << 16, d.first * d.pay_pitch)
    assert np.array_equal(w.payload[: 1 << 16].cpu().numpy(), head)
    codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                       w.status, id_uniform=workload.ID_UNIFORM, pad16=pad16)
    torch.cuda.synchronize()
    plen = w.pay_len.to(torch.int64) & 0xFFFF
    assert torch.equal(w.status.to(torch.int64), plen + 31)
    frames = w.frame.view(n, d.frame_pitch)
    pays = w.payload.view(n, d.pay_pitch)
    tags = _tag_table(oracle, gpu)
    assert torch.equal(frames[:, :8], tags[pays[:, 0].long()])
    hdr = frames[:, 8:31]
    assert bool((hdr[:, 0] == 23).all()) and torch.equal(hdr[:, 1], w.cmd)
    idu = torch.frombuffer(bytearray(workload.ID_UNIFORM), dtype=torch.uint8).to(gpu)
    assert bool((hdr[:, 2:10] == idu).all())
    assert torch.equal(hdr[:, 10:14], _le_bytes(w.conv.to(torch.int64) & 0xFFFFFFFF, 4))
    assert torch.equal(hdr[:, 14:22], _le_bytes(w.conn_key, 8))
    assert bool((hdr[:, 22] == 0).all())
    # payload region, per distinct payload length (C3/C2 uniform; C4 bucketed)
    for p in torch.unique(plen).tolist():
        sel = (plen == p).nonzero().squeeze(1)
        for lo in range(0, sel.numel(), 1 << 18):
            s = sel[lo: lo + (1 << 18)]
            assert torch.equal(frames[s, 31:31 + p], pays[s, :p]), f"payload mismatch at P={p}"
            if pad16:
                end = 31 + p
                pad_end = (end + 15) // 16 * 16
                if pad_end > end:
                    assert bool((frames[s, end:pad_end] == 0).all())
    # decode: corrupt C4's marked frames first
    w.corrupt_frames()
    codec.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec)
    torch.cuda.synchronize()
    keep = torch.from_numpy(~d.corrupt).to(gpu)
    st = w.dec.status.to(torch.int64)
    assert torch.equal(st == 1, keep)
    nv = int(w.dec.n_valid.item())
    exp_idx = keep.nonzero().squeeze(1).to(torch.int32)
    assert nv == exp_idx.numel()
    assert torch.equal(w.dec.valid_idx[:nv], exp_idx)
    ok = keep
    assert torch.equal((w.dec.pay_len.to(torch.int64) & 0xFFFF)[ok], plen[ok])
    assert bool((w.dec.pay_off[ok] == 31).all()) and bool((w.dec.hlen[ok] == 23).all())
    assert torch.equal(w.dec.conv[ok], w.conv[ok]) and torch.equal(w.dec.conn_key[ok], w.conn_key[ok])
    assert torch.equal(w.dec.cmd[ok], w.cmd[ok])
    assert bool((w.dec.id.view(n, 8)[ok] == idu).all())
    # dropped frames expose zero fields
    bad = ~keep
    if bool(bad.any()):
        assert bool((w.dec.conv[bad] == 0).all()) and bool((w.dec.hlen[bad] == 0).all())


def test_compaction_large_random(codec, gpu, oracle):
    """n > 4096 scan blocks x 256 (many k_compact tiles): random validity pattern, order-stable."""
    import torch

    n = 5_000_003
    g = torch.Generator(device=gpu)
    g.manual_seed(1234)
    # frames of 32 B in 32-B slots: tag of byte 0 or a wrong tag, chosen at random
    valid = torch.rand(n, device=gpu, generator=g) < 0.37
    tags = _tag_table(oracle, gpu)
    body = torch.randint(0, 256, (n,), device=gpu, generator=g, dtype=torch.int64).to(torch.uint8)
    frames = torch.zeros(n, 32, dtype=torch.uint8, device=gpu)
    frames[:, :8] = tags[body.long()]
    frames[~valid, 0] ^= 0x55
    frames[:, 8] = 23
    frames[:, 31] = body
    off = torch.arange(n, device=gpu, dtype=torch.int64) * 32
    flen = torch.full((n,), 32, dtype=torch.int16, device=gpu)
    from rsock_amd.codec import DecodeBuffers

    out = DecodeBuffers.alloc(n, gpu)
    codec.onrecv_batch(frames.view(-1), off, flen, out)
    torch.cuda.synchronize()
    exp = valid.nonzero().squeeze(1).to(torch.int32)
    nv = int(out.n_valid.item())
    assert nv == exp.numel()
    assert torch.equal(out.valid_idx[:nv], exp)
    assert torch.equal(out.status == 1, valid)


def test_encode_paths_beyond_one_grid(codec, gpu, oracle):
    """A batch of 2^26 + 4097 packets: one grid of the two-pass copy (64 work-items per packet, or per K
    packets) would exceed the 2^32 - 1 work-items a grid may hold for K = 1 (r04's C5-on-one-GPU run
    failed exactly there: "invalid configuration argument"), so the copy runs in launches of 2^25
    packets; every path's frames must equal the per-set kernel's, and the tags the oracle's table at
    payload[0] (C2-shaped: ~11 GB of arenas)."""
    import torch

    n = (1 << 26) + 4097
    assert 64 * n > 2**32 - 1  # an unsplit copy grid would be illegal
    d = workload.describe("c2", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    ref = None
    for pk in [(1, 0), (2, 1), (2, 4), (3, 0)]:
        with held(codec, *pk):
            w.frame.zero_()
            codec.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                               w.status, id_uniform=workload.ID_UNIFORM, pad16=True)
            torch.cuda.synchronize()
        if ref is None:
            ref = w.frame.clone()
            frames = ref.view(n, d.frame_pitch)
            pays = w.payload.view(n, d.pay_pitch)
            assert torch.equal(frames[:, :8], _tag_table(oracle, gpu)[pays[:, 0].long()])
        else:
            assert torch.equal(w.frame, ref), f"path {pk} differs from the per-set kernel"
