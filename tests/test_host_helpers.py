"""CPU: host batch helpers of the header-only path (no GPU): rsk_stage_decode_headers equals the
per-frame rsk_stage_decode_header and the vectorised staging; rsk_assemble_frames rebuilds the
oracle's RConn::Output frames from their 32-B header slots and the payloads."""
from __future__ import annotations

import ctypes

import numpy as np

from rsock_amd import _abi
from rsock_amd import codec as rc
from rsock_amd import workload

KEY = b"hello135"


def _p(a):
    return a.ctypes.data


def test_stage_batch_matches_single_and_numpy():
    lib = _abi.load()
    rng = np.random.default_rng(11)
    n = 20000
    lens = rng.integers(0, 300, n).astype(np.uint16)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 3)[:-1]]).astype(np.uint64)
    arena = rng.integers(0, 256, int(offs[-1]) + 400, dtype=np.uint8)
    arena[offs.astype(np.int64) + 8] = np.where(rng.random(n) < 0.7, 23, rng.integers(0, 256, n)).astype(np.uint8)
    slots = np.zeros(32 * n, np.uint8)
    assert lib.rsk_stage_decode_headers(n, _p(arena), _p(offs), _p(lens), _p(slots), 8) == 0
    assert np.array_equal(slots.reshape(n, 32), rc.stage_decode_headers(arena, offs, lens))
    for i in range(0, n, 997):
        one = ctypes.create_string_buffer(32)
        lib.rsk_stage_decode_header(arena[int(offs[i]):].tobytes(), int(lens[i]), one)
        assert one.raw == slots[32 * i: 32 * i + 32].tobytes()


def test_assemble_frames_matches_oracle(oracle):
    lib = _abi.load()
    d = workload.describe("c4", 0, 4000, n=4000)
    payload = workload.payload_bytes_np(d)
    frames, status = oracle.encode_batch(KEY, payload, d, workload.ID_UNIFORM)
    hdr = np.zeros(32 * d.n, np.uint8)
    fo = d.frame_off.astype(np.int64)
    for i in range(d.n):
        if status[i] > 0:
            hdr[32 * i: 32 * i + 32] = frames[fo[i]: fo[i] + 32]
    out = np.zeros_like(frames)
    po = d.pay_off.astype(np.uint64)
    fo64 = d.frame_off.astype(np.uint64)
    assert lib.rsk_assemble_frames(d.n, _p(hdr), _p(status), _p(payload), _p(po), _p(out), _p(fo64), 4) == 0
    for i in range(d.n):
        if status[i] > 0:
            assert out[fo[i]: fo[i] + status[i]].tobytes() == frames[fo[i]: fo[i] + status[i]].tobytes(), i


def test_stage_capture_slots_matches_numpy():
    rng = np.random.default_rng(12)
    n = 9000
    cl = rng.integers(0, 400, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(cl.astype(np.uint64) + 5)[:-1]]).astype(np.uint64)
    arena = rng.integers(0, 256, int(offs[-1]) + 400, dtype=np.uint8)
    for slot in (64, 96, 128, 512):
        got = rc.stage_capture_slots(arena, offs, cl, slot)
        k = np.arange(slot)
        idx = offs.astype(np.int64)[:, None] + k[None, :]
        exp = np.where(k[None, :] < cl.astype(np.int64)[:, None], arena[np.minimum(idx, len(arena) - 1)], 0)
        assert np.array_equal(got, exp.astype(np.uint8)), slot


def test_stage_capture_slots_rejects_bad_slot():
    lib = _abi.load()
    a = np.zeros(256, np.uint8)
    o = np.zeros(1, np.uint64)
    c = np.full(1, 100, np.uint32)
    out = np.zeros(256, np.uint8)
    for slot in (0, 48, 72, 100):  # below RSK_CAP_SLOT_MIN or not a multiple of 16
        assert lib.rsk_stage_capture_slots(1, _p(a), _p(o), _p(c), slot, _p(out), 1) == _abi.EINVAL
