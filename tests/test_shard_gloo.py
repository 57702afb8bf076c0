"""CPU, 2 ranks over gloo: the sharded multi-GPU path's bookkeeping.  Each rank
decodes its contiguous shard of C4 frames (oracle stands in for the device here), and the gathered
global VALID list equals the single-process result — no data-path collective involved."""
from __future__ import annotations

import os
import socket

import numpy as np
import torch.multiprocessing as mp

KEY = b"hello135"
N = 6000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from rsock_amd import shard, workload
    from tests.oracle_lib import Oracle

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard.shard_range(N, rank, world)
    d = workload.describe("c4", lo, hi, n=N)
    orc = Oracle()
    frames, st = orc.encode_batch(KEY, workload.payload_bytes_np(d), d, workload.ID_UNIFORM, nthreads=1)
    for i in np.nonzero(d.corrupt)[0]:
        frames[int(d.frame_off[i])] ^= 1
    out = orc.decode_batch(KEY, frames, d.frame_off, d.frame_len, nthreads=1)
    local = torch.from_numpy(out["valid_idx"][: out["n_valid"]].astype(np.int64))
    glob, counts = shard.gather_valid(local, lo)
    if rank == 0:
        q.put((glob.numpy(), counts))
    dist.destroy_process_group()


def test_two_rank_gather_matches_single_process(oracle):
    from rsock_amd import workload

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    glob, counts = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    d = workload.describe("c4", 0, N, n=N)
    frames, st = oracle.encode_batch(KEY, workload.payload_bytes_np(d), d, workload.ID_UNIFORM)
    for i in np.nonzero(d.corrupt)[0]:
        frames[int(d.frame_off[i])] ^= 1
    out = oracle.decode_batch(KEY, frames, d.frame_off, d.frame_len)
    assert np.array_equal(glob, out["valid_idx"][: out["n_valid"]].astype(np.int64))
    assert sum(counts) == out["n_valid"] == N - int(d.corrupt.sum())


def test_shard_range_covers():
    from rsock_amd.shard import shard_range

    for n in (0, 1, 7, 1000, 64 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
