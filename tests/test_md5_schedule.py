"""CPU: the device tag path's MD5 schedule, run on the host (rsk__host_tag in librsk.so).

Round 4 specialises the per-lane MD5 on the word that holds payload[0] (rsk_md5.h md5_tag_bw: every
other message word uniform, steps 0 .. bword - 1 precomputed by the host into KeySched::pre) and
dispatches on the key's word index at run time (md5_tag_lane).  The same templates run here on the
CPU: every key length 0..200 (every payload word index 0..15, one- and two-block tails, midstates of
1..3 key-only blocks) x every first byte must give the oracle's tag (util/rhash.cpp:20-41), and the
reference's own golden tags (tests/golden/tags.npz).  The GPU tests check the device build."""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def host_tag():
    from rsock_amd.codec import lib

    fn = lib().rsk__host_tag
    fn.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    fn.restype = ctypes.c_int
    out = (ctypes.c_uint32 * 2)()

    def tag(key: bytes, b: int) -> bytes:
        assert fn(key, len(key), b, out) == 0
        return int(out[0]).to_bytes(4, "little") + int(out[1]).to_bytes(4, "little")

    return tag


def test_every_key_length_and_byte(oracle, host_tag):
    rng = np.random.default_rng(4)
    for kl in range(0, 201):
        key = rng.integers(0, 256, kl, dtype=np.uint8).tobytes()
        bs = range(256) if kl % 16 in (0, 3, 13, 14, 15) else rng.integers(0, 256, 24)
        for b in bs:
            assert host_tag(key, int(b)) == oracle.tag(key, int(b)), (kl, int(b))


def test_golden_tags(host_tag):
    g = np.load(os.path.join(GOLD, "tags.npz"), allow_pickle=False)
    kb, ko, kl = g["key_bytes"], g["key_off"], g["key_len"]
    for k in range(len(kl)):
        key = kb[int(ko[k]): int(ko[k]) + int(kl[k])].tobytes()
        for b in range(256):
            assert host_tag(key, b) == g["tags"][k, b].tobytes(), (len(key), b)


def test_rejects_bad_args(host_tag):
    from rsock_amd.codec import lib

    out = (ctypes.c_uint32 * 2)()
    assert lib().rsk__host_tag(b"k", 1, 256, out) != 0
    assert lib().rsk__host_tag(None, 3, 0, out) != 0
