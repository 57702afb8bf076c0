"""GPU: the output-stationary copy of the two-pass encode (k_encode_heads_os + k_encode_os, round 6):
waves own 1-KB blocks of the frame arena instead of packets, so the chunk two byte-packed frames
share is written once, whole.  Every case compares the bytes of the whole arena (frames, pads and
the bytes outside every frame, pre-filled at random) with the oracle (orc_encode_batch), with the
copy held to the output-stationary form and the path asserted (tests/enc_paths.held):
  - byte-packed C4-sized batches, with and without resets and oversize packets, 16-B packed with
    RSK_ENC_ZERO_PAD16;
  - 300 resets in a row at one offset (one block's window walks past 64 packets);
  - frames out of order and gaps of 4 KB (the header pass flags the layout and the same launch
    copies packet by packet);
  - AUTO: a byte-packed batch takes the output-stationary copy from the second call on (the
    sampled frames lie back to back), slots do not."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import workload
from tests.enc_paths import held
from tests.test_gpu_parity import KEY, _rand_fields, run_encode

pytestmark = pytest.mark.gpu


def _case(rng, n, plen, layout, pad=0):
    plen = np.asarray(plen, np.uint16)
    pay_off = (np.arange(n, dtype=np.int64) * 1472 + rng.integers(0, 16, n)).astype(np.uint64)
    payload = rng.integers(0, 256, int(pay_off[-1]) + 1600, dtype=np.uint8)
    framed = (plen >= 1) & (plen <= 1469)  # RSK_MAX_PAYLOAD
    flen = np.where(framed, plen.astype(np.int64) + 31, 0)
    if pad:
        flen = np.where(framed, (flen + pad - 1) // pad * pad, 0)
    if layout == "packed":  # with a pad: 16-B packed (frames start on 16-B boundaries)
        frame_off = (0 if pad else 5) + np.concatenate([[0], np.cumsum(flen)[:-1]])
    elif layout == "reversed":  # packed, in reverse packet order
        fo = 5 + np.concatenate([[0], np.cumsum(flen[::-1])[:-1]])
        frame_off = fo[::-1].copy()
    elif layout == "gap4k":
        frame_off = np.arange(n, dtype=np.int64) * 4096 + 3
    elif layout == "swapped":  # packed, two frames of equal length trade places
        frame_off = 5 + np.concatenate([[0], np.cumsum(flen)[:-1]])
        i = int(np.nonzero(framed[100:])[0][0]) + 100
        j = i + 1 + int(np.nonzero(flen[i + 1:] == flen[i])[0][0])
        frame_off[[i, j]] = frame_off[[j, i]]
    else:
        raise ValueError(layout)
    return payload, pay_off, plen, frame_off.astype(np.uint64)


def _check(codec, gpu, oracle, rng, payload, pay_off, plen, frame_off, pad=0):
    n = len(plen)
    cmd, conv, ckey = _rand_fields(rng, n)
    frame_bytes = int(frame_off.max()) + 1700
    fill = rng.integers(0, 256, frame_bytes, dtype=np.uint8)
    got, st = run_encode(codec, gpu, payload, pay_off, plen, cmd, conv, ckey, frame_off, frame_bytes,
                         frame_init=fill, pad16=pad == 16)

    class D:
        pass

    d = D()
    d.n, d.pay_off, d.pay_len, d.cmd, d.conv, d.conn_key, d.frame_off = n, pay_off, plen, cmd, conv, ckey, frame_off
    ef, es = oracle.encode_batch(KEY, payload, d, workload.ID_UNIFORM, frame_bytes=frame_bytes)
    assert np.array_equal(st, es)
    exp = fill.copy()
    for i in range(n):  # frames in packet order (a later frame's bytes win where pads overlap)
        if es[i] > 0:
            o = int(frame_off[i])
            exp[o:o + es[i]] = ef[o:o + es[i]]
            if pad:
                e = o + int(es[i])
                exp[e:(e + pad - 1) // pad * pad] = 0
    return got, exp


@pytest.mark.parametrize("n,resets", [(70000, False), (70000, True), (4096, True)])
def test_os_packed(codec, gpu, oracle, n, resets):
    rng = np.random.default_rng(n + resets)
    plen = rng.integers(1, 1401, n)
    if resets:
        plen[rng.integers(0, n, n // 50)] = 0
        plen[rng.integers(0, n, n // 200)] = 1470 + rng.integers(0, 300, n // 200)  # oversize: dropped
    args = _case(rng, n, plen, "packed")
    with held(codec, 2, -1):
        got, exp = _check(codec, gpu, oracle, rng, *args)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


def test_os_packed16_pad16(codec, gpu, oracle):
    rng = np.random.default_rng(16)
    n = 30000
    plen = rng.integers(1, 1401, n)
    plen[rng.integers(0, n, 100)] = 0
    args = _case(rng, n, plen, "packed", pad=16)
    with held(codec, 2, -1):
        got, exp = _check(codec, gpu, oracle, rng, *args, pad=16)
    assert np.array_equal(got, exp)


def test_os_long_reset_run(codec, gpu, oracle):
    """300 consecutive resets share one frame offset: a block's packet window runs past 64 packets."""
    rng = np.random.default_rng(300)
    n = 5000
    plen = rng.integers(1, 200, n)
    plen[1000:1300] = 0
    plen[4000:4100] = 0
    args = _case(rng, n, plen, "packed")
    with held(codec, 2, -1):
        got, exp = _check(codec, gpu, oracle, rng, *args)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("layout", ["reversed", "swapped", "gap4k"])
def test_os_fallback_layouts(codec, gpu, oracle, layout):
    """Layouts the block map cannot take: frames in reverse packet order, two frames trading places,
    gaps of 4 KB per frame.  The same launch copies packet by packet; bytes equal the oracle's."""
    rng = np.random.default_rng(len(layout))
    n = 20000
    plen = rng.integers(1, 1401, n)
    plen[rng.integers(0, n, 40)] = 0
    args = _case(rng, n, plen, layout)
    with held(codec, 2, -1):
        got, exp = _check(codec, gpu, oracle, rng, *args)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"{bad.size} bytes differ, first at {bad[:8]}"


def test_os_auto_choice(codec, gpu, oracle):
    """AUTO: the second call on a byte-packed C4-like batch takes the output-stationary copy (the
    statistic of the first call saw the frames back to back); a slots batch keeps the K-packet waves."""
    rng = np.random.default_rng(4)
    n = 40000
    plen = rng.integers(1, 1401, n)
    args = _case(rng, n, plen, "packed")
    codec.set_encode_path(0)
    codec.set_copy_k(0)
    for _ in range(2):
        got, exp = _check(codec, gpu, oracle, rng, *args)
    assert codec.last_encode_path == 2 and codec.last_copy_k == -1
    assert np.array_equal(got, exp)
    payload, pay_off, pl, _ = args
    slots = (np.arange(n, dtype=np.int64) * 1536).astype(np.uint64)
    for _ in range(2):
        got, exp = _check(codec, gpu, oracle, rng, payload, pay_off, pl, slots)
    assert codec.last_encode_path == 2 and codec.last_copy_k == 4
    assert np.array_equal(got, exp)
