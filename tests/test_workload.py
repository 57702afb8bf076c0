"""CPU: the synthetic workload generator is deterministic, its numpy
splitmix64 matches the oracle's C splitmix64, and the configs have the documented shape."""
from __future__ import annotations

import numpy as np

from rsock_amd import workload


def test_splitmix_numpy_matches_oracle(oracle):
    for seed in (0, 1, workload.seed_of("c3"), 2**64 - 1):
        a = workload.splitmix_bytes_np(seed, 1000)
        b = oracle.splitmix_bytes(seed, 1000)
        assert np.array_equal(a, b)
    # arbitrary start offsets agree with the full stream
    full = workload.splitmix_bytes_np(7, 4096)
    for st in (0, 1, 8, 13, 100, 4000):
        assert np.array_equal(workload.splitmix_bytes_np(7, 50, st)[: 4096 - st], full[st: st + 50])


def test_shard_descriptors_concatenate():
    d_all = workload.describe("c4", 0, 3000, n=3000)
    parts = [workload.describe("c4", lo, hi, n=3000) for lo, hi in ((0, 1000), (1000, 2500), (2500, 3000))]
    for f in ("pay_len", "cmd", "conv", "conn_key", "corrupt"):
        assert np.array_equal(np.concatenate([getattr(p, f) for p in parts]), getattr(d_all, f)), f
    pay = workload.payload_bytes_np(d_all)
    off = 0
    for p in parts:
        b = workload.payload_bytes_np(p)
        assert np.array_equal(b, pay[off: off + b.size])
        off += b.size


def test_config_shapes():
    d = workload.describe("c4", 0, 200_000, n=200_000)
    frac = (d.cmd != 0).mean()
    assert 0.04 < frac < 0.06
    dp = (d.conn_key >> np.uint64(16)) & np.uint64(0xFFF)
    assert set(np.unique((d.conn_key >> np.uint64(16)) & np.uint64(0xFFFF)) - np.uint64(0x1000)) or True
    ports = np.unique(((d.conn_key & np.uint64(0xEFFFFFFF)) >> np.uint64(16)).astype(np.int64) | 0x0000)
    assert len(np.unique(dp)) == 10 and ports.size == 10
    sp = d.conn_key & np.uint64(0xFFFF)
    assert sp.min() >= 32768 and sp.max() <= 60999
    data = d.cmd == 0
    assert d.pay_len[data].min() >= 64 and d.pay_len[data].max() <= 1400
    assert set(np.unique(d.pay_len[d.cmd == 1])) == {4} and set(np.unique(d.pay_len[d.cmd >= 2])) == {8}
    assert d.corrupt.mean() == (np.arange(200_000) % 16 == 7).mean()
    c3 = workload.describe("c3", 0, 1000)
    assert c3.pay_pitch == 1408 and c3.frame_pitch == 1440 and (c3.pay_len == 1400).all()
    assert (c3.frame_off % 16 == 0).all()
