"""The multi-GPU path on the one-GPU box (BASELINE configs[4]): ranks share cuda:0
and rendezvous over gloo, so the launch and bookkeeping run exactly as on an 8-GPU node.

  * bench.py --gpus 2 starts its own two rank processes and reports one line for both
  * two ranks each decode their C4 shard through the HIP library; shard.gather_valid's global
    VALID list equals the oracle's single-process list
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY = b"hello135"
N = 20000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_self_launches_two_ranks(gpu):
    # no --dist-backend: the default the driver's multi-GPU run takes (gloo; bench.py never uses RCCL
    # unless asked)
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--same-device",
           "--config", "c5", "--packets", str(1 << 16), "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["scaling"] == "strong"
    assert rec["config"]["packets_total"] == 1 << 16 and rec["config"]["packets_per_gpu"] == 1 << 15
    assert rec["value"] > 0 and "cpu_baseline" not in rec


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from rsock_amd import codec, shard, workload

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda:0")
        lo, hi = shard.shard_range(N, rank, world)
        d = workload.describe("c4", lo, hi, n=N)
        w = workload.DeviceWorkload(d, dev)
        cx = codec.Codec(KEY, 0)
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM)
        w.corrupt_frames()
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec)
        torch.cuda.synchronize()
        nv = int(w.dec.n_valid.item())
        local = w.dec.valid_idx[:nv].cpu().to(torch.int64)
        glob, counts = shard.gather_valid(local, lo)
        cx.close()
        if rank == 0:
            q.put((glob.numpy(), counts))
    finally:
        dist.destroy_process_group()


def test_two_rank_device_decode_gather(oracle, gpu):
    import torch.multiprocessing as mp

    from rsock_amd import workload

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        glob, counts = q.get(timeout=180)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in ps)
    d = workload.describe("c4", 0, N, n=N)
    frames, st = oracle.encode_batch(KEY, workload.payload_bytes_np(d), d, workload.ID_UNIFORM)
    for i in np.nonzero(d.corrupt)[0]:
        frames[int(d.frame_off[i])] ^= 1
    out = oracle.decode_batch(KEY, frames, d.frame_off, d.frame_len)
    assert np.array_equal(glob, out["valid_idx"][: out["n_valid"]].astype(np.int64))
    assert sum(counts) == out["n_valid"] == N - int(d.corrupt.sum())
