#!/usr/bin/env python3
"""Benchmark: device-resident EncHead+MD5 encode then decode+verify+compact (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5] [--tag md5|table]
                  [--no-cpu-baseline] [--eager]

One step = one pass of the hot path over one batch: k_encode (RConn::Output framing of every
packet) followed by k_decode + k_compact (RConn::OnRecv of every frame), inputs resident in HBM.
The headline computes the tag by one MD5 compression per packet and lane in both kernels
(RSK_TAG_MD5, as util/rhash.cpp:20-41 does per packet); at N = 1 the same step with the tag looked
up in the key's 256-entry table (RSK_TAG_TABLE) is timed afterwards and reported under its own
label (`variant_tag_table_lut`), never as `value`.
The timed region replays a HIP graph of the step (one host launch per step; --eager: the three
library calls per step instead); the per-kernel times behind `roofline` come from HIP events on
the step's stream around the same launches issued one by one right after the timed region.

Workload: N = 1 defaults to C3 (4M x 1400-B packets, the metric's target config); N > 1 defaults
to C5 (BASELINE configs[4]: 64M x 1400-B packets in total, contiguous shards, strong scaling), so
`--gpus 8` IS config 5.  The scaling curve's N = 1 point is the `scale_n1_c5` key of the default
N = 1 line: after the C3 headline (and its tag variant) the C3 arenas are freed and C5 is timed whole
on the same GPU with the same step (`--gpus 1 --config c5` makes it the headline instead).  A
1/2/4/8 curve therefore reads scale_n1_c5.value at N = 1 and value at N = 2, 4, 8.

N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) this process is one rank;
without a launcher, `--gpus N` starts the N rank processes itself (from this parent, which never
touches the GPU) and relays rank 0's line.  No data-path collective: the only collectives are the
timing barrier and the max over ranks, and both run over gloo on the CPU by default (RCCL is not
used: --dist-backend nccl is opt-in).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpkt/s + GiB/s device-resident EncHead+MD5 encode/decode at 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# tag modes (rsk_set_tag_mode): the headline computes MD5 per lane, as the reference does per packet
TAG_LABEL = {"md5": "md5_per_lane", "table": "tag_table_lut"}
# rsk__last_encode_path: the library picks the encode path per call (rsk_encode_batch, enc_path)
ENC_PATH_TEXT = {1: "k_encode", 2: "k_encode_heads + k_encode_copy (two-pass, {k} packet(s) per copy wave)",
                 3: "k_encode (short frames: every set on the flat chunk list)"}
TAG_TEXT = {"md5": "one MD5 compression per packet and lane",
            "table": "lookup in the key's 256-entry tag table staged in LDS (MD5 run once per key, 256 tags)"}


def enc_bytes_per_pkt(p):
    """Algorithmic bytes of k_encode per packet: reads payload P, cmd 1,
    conv 4, connKey 8, pay_len 2, pay_off 8, frame_off 8; writes frame 31+P, status 4."""
    return p + 1 + 4 + 8 + 2 + 8 + 8 + (31 + p) + 4


def dec_bytes_per_pkt() -> int:
    """Algorithmic bytes of decode per packet: reads frame[0..32) 32, frame_off 8, frame_len 2;
    writes hlen 1, cmd 1, id 8, conv 4, connKey 8, pay_off 2, pay_len 2, status 1, valid_idx 4
    (+ the ballot mask, 1/8 B per packet, rounded out)."""
    return 32 + 8 + 2 + 1 + 1 + 8 + 4 + 8 + 2 + 2 + 1 + 4


def load_traffic(cfg: str, n: int, frame_pitch: int) -> dict | None:
    """HBM traffic per k_encode launch measured by tools/pmc_traffic.py (separate rocprofv3 --pmc
    passes, gfx950 FETCH_SIZE x2 correction) for this (config, packets, frame slot pitch), if
    profiles/ holds one."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(path):
        return None
    try:
        table = json.load(open(path))
    except Exception:
        return None
    if "config" in table:  # single-record form
        table = {f"{table['config']}:{table['packets']}": table}
    rec = table.get(f"{cfg}:{n}")
    if rec is None or rec.get("frame_pitch") != frame_pitch:
        return None  # measured on another layout (or before the layout was recorded)
    return rec


def _cpu_quota() -> float | None:
    """CPUs the cgroup grants this process (cgroup v2 cpu.max), None when unlimited/unknown."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def cpu_baseline(cfg: str, n_sample: int, min_seconds: float, use_ref: bool = False) -> dict:
    """The clean-room C restatement (oracle/rsk_oracle.c, "port", SURVEY.md §8d: "the build's own
    clean-room restatement ... the reference binary itself never goes to the GPU box") timed on this
    host's cores over a bounded sample: std::thread x every core of the affinity mask, contiguous
    shards, plus a 1-thread number on the same arenas.  use_ref (--cpu-baseline-ref, a cross-check
    in the build container): the reference's own codec compiled into oracle/_ref instead."""
    from rsock_amd import workload
    from tests import oracle_lib

    cores = len(os.sched_getaffinity(0))
    d = workload.describe(cfg, 0, n_sample)
    payload = workload.payload_bytes_np(d)
    frames = np.zeros(d.n * d.frame_pitch, np.uint8)
    key = b"hello135"
    if use_ref:
        if not oracle_lib.ref_available():
            raise SystemExit("bench: --cpu-baseline-ref needs oracle/_ref (make -C oracle ref)")
        ref = oracle_lib.RefOracle()
        kind = "reference"

        def run(threads, m):
            ref.bench_codec(key, payload, _prefix(d, m), workload.ID_UNIFORM, frames, threads)
    else:
        orc = oracle_lib.Oracle()
        kind = "port"

        def run(threads, m):
            orc.bench_codec(key, payload, _prefix(d, m), workload.ID_UNIFORM, frames, threads)

    def timed(threads, m, seconds):
        run(threads, m)  # warm (page faults on the frame arena)
        reps, t0 = 0, time.perf_counter()
        while True:
            run(threads, m)
            reps += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                return reps * m / el / 1e6, reps, el

    # every core of the affinity mask; when a cgroup quota grants fewer CPUs than the
    # mask shows, that many threads too, and the faster of the two is the baseline
    quota = _cpu_quota()
    runs = {cores: timed(cores, d.n, min_seconds)}
    if quota and int(quota) < cores:
        runs[max(1, int(quota))] = timed(max(1, int(quota)), d.n, min_seconds)
    best = max(runs, key=lambda t: runs[t][0])
    v_all, reps_all, el_all = runs[best]
    m1 = min(d.n, 1 << 16)
    v_one, reps_one, el_one = timed(1, m1, min_seconds / 2)
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    p = d.pay_len.astype(np.int64)
    pay = f"{int(p[0])}-B payloads" if p.min() == p.max() else \
        f"mixed {int(p.min())}-{int(p.max())}-B payloads, mean {p.mean():.0f} B"
    return {
        "value": round(v_all, 3),
        "unit": "Mpkt/s",
        "cores": best,
        "kind": kind,
        "value_1thread": round(v_one, 3),
        "by_threads": {str(t): round(r[0], 3) for t, r in sorted(runs.items())},
        "affinity_cpus": cores,
        "cgroup_cpus": quota,
        "sample": f"{d.n} packets of {cfg.upper()} ({pay}) x {reps_all} passes on {best} threads "
                  f"({el_all:.1f} s; threads tried: {sorted(runs)} = affinity mask"
                  + (f", cgroup quota {quota} CPUs" if quota else "") + f"), and {m1} packets x {reps_one} passes "
                  f"on 1 thread ({el_one:.1f} s); per packet: RConn::Output framing (compute_hash + Enc2Buf + memcpy "
                  f"into a zeroed 1500-B buffer) then DecodeBuf + hash_equal; {cpu_model}",
    }


def _prefix(d, m: int):
    """The first m packets of a shard's descriptors (same arenas)."""
    import dataclasses

    if m >= d.n:
        return d
    return dataclasses.replace(d, n=m, pay_off=d.pay_off[:m], pay_len=d.pay_len[:m], cmd=d.cmd[:m],
                               conv=d.conv[:m], conn_key=d.conn_key[:m], frame_off=d.frame_off[:m],
                               frame_len=d.frame_len[:m], corrupt=d.corrupt[:m])


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script (this parent never
    initialises the GPU), rank r on GPU r, rendezvous on 127.0.0.1; rank 0's stdout is ours.
    A failed rank ends the others (their exact PIDs) and its exit code is returned."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in pending:
                    q.kill()
        time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def make_runner(torch, dist, workload, d, w, cx, stream, graph_mode: bool):
    """The timed step on one shard: returns timed(mode, steps, warmup, sync_ranks) -> (elapsed, evs)
    and the holder of the encode path the captured graph replays."""
    cx.reserve(d.n, stream=stream)

    def step(ev=None):
        if ev is not None:
            ev[0].record(stream)
        cx.output_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, w.frame, w.frame_off,
                        w.status, id_uniform=workload.ID_UNIFORM, pad16=d.pad == 16, pad128=d.pad == 128,
                        stream=stream)
        if ev is not None:
            ev[1].record(stream)
        cx.onrecv_batch(w.frame, w.frame_off, w.frame_len, w.dec, stream=stream)
        if ev is not None:
            ev[2].record(stream)

    # correctness gate on the measured data: every packet must verify
    expect_valid = int(((d.pay_len >= 1) & (d.pay_len <= 1469)).sum())

    def gate(when):
        nv = int(w.dec.n_valid.item())
        if nv != expect_valid:
            raise SystemExit(f"bench: decode verified {nv} of {expect_valid} packets ({when}, tag {cx.tag_mode})")

    captured_path = [None]

    def timed(mode: str, steps: int, warmup: int, sync_ranks: bool):
        """Warm up, capture the step as a graph (the tag mode is fixed at capture), time `steps`
        replays between barriers, then per-kernel HIP events on the step's stream."""
        cx.set_tag_mode(mode)
        with torch.cuda.stream(stream):
            for _ in range(warmup):
                step()
        torch.cuda.synchronize()
        gate("warmup")
        graph = None
        if graph_mode:
            # the whole step (k_encode, k_decode, k_compact) as one HIP graph: one launch per step from
            # the host instead of three library calls, so the timed region measures the GPU, not Python
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=stream):
                step()
            captured_path[0] = (cx.last_encode_path, cx.last_copy_k)  # the path the graph replays
            w.dec.n_valid.zero_()
            graph.replay()
            torch.cuda.synchronize()
            gate("graph replay")
            for _ in range(warmup):  # the warmup steps again, as replays of the graph
                graph.replay()
            torch.cuda.synchronize()
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(steps)]
        if sync_ranks:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k in range(steps):
            if graph is not None:
                graph.replay()
            else:
                step(evs[k])
        torch.cuda.synchronize()
        if sync_ranks:
            dist.barrier()
        el = time.perf_counter() - t0
        gate("timed region")
        cx.check_device_errors()  # raises if a compaction look-back gave up (rsk_check_device_errors)
        if graph is not None:
            # per-kernel durations for the roofline: HIP events on the step's stream around the same
            # launches, issued one by one (the graph replays the identical kernels and arguments)
            with torch.cuda.stream(stream):
                for k in range(steps):
                    step(evs[k])
            torch.cuda.synchronize()
            del graph
        return el, evs

    return timed, captured_path


def scale_anchor_c5(torch, dist, rc, workload, dev, gpu, tag: str, steps: int, warmup: int, graph_mode: bool):
    """The 1 -> 8 GPU curve's N = 1 point: BASELINE config 5 whole (64M x 1400-B
    packets, ~185 GB of arenas) on this one GPU, the same step and timing as the N > 1 default
    (`--gpus N` runs C5 split N ways, strong scaling).  Reported under `scale_n1_c5`, never as value."""
    n_total = workload.CONFIGS["c5"][1]
    d = workload.describe("c5", 0, n_total, n=n_total)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", gpu, tag_mode=tag)
    stream = torch.cuda.Stream(dev) if graph_mode else torch.cuda.current_stream()
    try:
        timed, captured = make_runner(torch, dist, workload, d, w, cx, stream, graph_mode)
        el, evs = timed(tag, steps, warmup, False)
        enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
        dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
        enc_bytes = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
        path = captured[0] if graph_mode else (cx.last_encode_path, cx.last_copy_k)
        return {
            "label": "NOT the headline: the scaling curve's N = 1 point -- C5 (64M x 1400-B packets, BASELINE "
                     "configs[4]) whole on one GPU, the workload `--gpus N` (N > 1) splits N ways",
            "config": "c5", "packets": d.n, "steps": steps, "warmup": warmup,
            "value": round(d.n * steps / el / 1e6, 2), "unit": "Mpkt/s",
            "ms_per_step": round(el / steps * 1e3, 4),
            "kernels_ms": {"encode": round(enc_ms, 4), "decode+compact": round(dec_ms, 4)},
            "encode_path": ENC_PATH_TEXT.get(path[0], "?").format(k=path[1]),
            "roofline_frac": round(enc_bytes / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
        }
    finally:
        cx.close()
        del w
        torch.cuda.synchronize()
        torch.cuda.empty_cache()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=None, choices=["c2", "c3", "c4", "c5"],
                    help="c2/c3/c4: that config per GPU (weak scaling); c5: BASELINE config 5, 64M 1400-B "
                         "packets in total split over the ranks (strong scaling; 1 GPU holds all 64M: ~185 GB). "
                         "Default: c3 at N = 1, c5 at N > 1")
    ap.add_argument("--packets", type=int, default=0,
                    help="packets per GPU (c2-c4) or in total (c5); default: the config's")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1 << 20)
    ap.add_argument("--cpu-seconds", type=float, default=6.0)
    ap.add_argument("--dist-backend", default="gloo",
                    help="gloo (default): the ranks exchange only the timing barrier and one float, on the CPU; "
                         "nccl (= RCCL, opt-in): the same two operations over the GPUs. There is no "
                         "data-path collective either way (SURVEY.md §8e)")
    ap.add_argument("--eager", action="store_true",
                    help="launch the step's kernels one by one in the timed region instead of replaying a "
                         "captured HIP graph of the step")
    ap.add_argument("--tag", default="md5", choices=["md5", "table"],
                    help="tag mode of the headline (default md5: MD5 per lane; table: the LUT variant)")
    ap.add_argument("--no-tag-variant", action="store_true",
                    help="skip timing the other tag mode after the headline (N = 1)")
    ap.add_argument("--cpu-baseline-ref", action="store_true",
                    help="time the reference's own codec (oracle/_ref, build container only) as the CPU "
                         "baseline instead of the clean-room restatement")
    ap.add_argument("--no-scale-anchor", action="store_true",
                    help="skip the C5-on-one-GPU point (`scale_n1_c5`) timed after the C3 headline at N = 1")
    ap.add_argument("--same-device", action="store_true",
                    help="rehearsal only: every rank uses GPU 0 (N ranks on a 1-GPU box)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    import torch
    import torch.distributed as dist

    from rsock_amd import codec as rc
    from rsock_amd import workload

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    gpu = 0 if args.same_device else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    cfg = args.config or ("c3" if world == 1 else "c5")
    strong = cfg == "c5"
    if strong:
        # strong scaling: the config's total is split over the ranks (contiguous shards)
        n_total = args.packets or workload.CONFIGS[cfg][1]
        lo, hi = workload.shard_range(n_total, rank, world)
        d = workload.describe(cfg, lo, hi, n=n_total)
    else:
        n = args.packets or workload.CONFIGS[cfg][1]
        # weak scaling: rank r owns packets [r*n, (r+1)*n) of the config's global stream
        d = workload.describe(cfg, rank * n, (rank + 1) * n, n=world * n)
    w = workload.DeviceWorkload(d, dev)
    cx = rc.Codec(b"hello135", gpu, tag_mode=args.tag)
    graph_mode = not args.eager
    # graph capture needs a stream other than the null stream; the codec's per-stream workspaces are
    # sized on it by the warmup, before the capture
    stream = torch.cuda.Stream(dev) if graph_mode else torch.cuda.current_stream()
    timed, captured_path = make_runner(torch, dist, workload, d, w, cx, stream, graph_mode)

    elapsed, evs = timed(args.tag, args.steps, args.warmup, world > 1)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed_max = float(t.item())

    # the path the timed region ran: the graph's (captured) path, else the eager calls'
    run_path = captured_path[0] if graph_mode else (cx.last_encode_path, cx.last_copy_k)
    enc_path = ENC_PATH_TEXT.get(run_path[0], "?").format(k=run_path[1])
    if graph_mode and run_path != (cx.last_encode_path, cx.last_copy_k):
        # the per-kernel events time the eager calls after the timed region: they must be the same path
        raise SystemExit(f"bench: graph captured encode path {run_path}, eager calls took "
                         f"{(cx.last_encode_path, cx.last_copy_k)}")
    enc_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    dec_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in evs]))
    total_pkts = (n_total if strong else world * d.n) * args.steps
    mpkts = total_pkts / elapsed_max / 1e6
    p = int(d.pay_len[0]) if workload.CONFIGS[cfg][2] == workload.CONFIGS[cfg][3] else int(d.pay_len.mean())
    # algorithmic bytes of this rank's launch, summed over its packets' actual payload lengths
    enc_bytes = int(enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum())
    bytes_step = enc_bytes + d.n * dec_bytes_per_pkt()
    achieved = enc_bytes / (enc_ms * 1e-3) / 1e9

    other = None
    if world == 1 and not args.no_tag_variant:
        # the other tag mode, reported beside the headline under its own label
        omode = "table" if args.tag == "md5" else "md5"
        el_o, evs_o = timed(omode, args.steps, max(2, args.warmup // 2), False)
        enc_o = float(np.mean([e[0].elapsed_time(e[1]) for e in evs_o]))
        dec_o = float(np.mean([e[1].elapsed_time(e[2]) for e in evs_o]))
        other = (omode, el_o, enc_o, dec_o)

    anchor = None
    if world == 1 and cfg == "c3" and not args.packets and not args.no_scale_anchor:
        # free the C3 arenas, then the curve's N = 1 point on the same GPU (C5 whole: 185 of 288 GB)
        cx.close()
        cx = None
        del w
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        anchor = scale_anchor_c5(torch, dist, rc, workload, dev, gpu, args.tag, min(args.steps, 10),
                                 min(args.warmup, 3), graph_mode)

    if rank == 0:
        tr = load_traffic(cfg, d.n, d.frame_pitch)
        line = {
            "metric": METRIC,
            "value": round(mpkts, 2),
            "unit": "Mpkt/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 payloads/fields, SURVEY.md §8d)",
            "config": {
                "workload": f"{cfg.upper()}: {d.n} packets/GPU, {p}-B payloads, encode (tag = "
                            f"{TAG_TEXT[args.tag]} + EncHead + payload copy) then decode + tag verify + compact, "
                            f"device-resident",
                "packets_per_gpu": d.n,
                "packets_total": n_total if strong else world * d.n,
                "payload_bytes": p,
                "frame_slot_bytes": d.frame_pitch,
                "zero_pad": d.pad,
                "key": "hello135",
                "tag": TAG_LABEL[args.tag],
                "parallelism": f"shard{world} (no collective)",
            },
            "gib_per_s": round(world * bytes_step * args.steps / elapsed_max / 2**30, 2),
            "kernels_ms": {"encode": round(enc_ms, 4), "decode+compact": round(dec_ms, 4)},
            "encode_path": enc_path,
            "launch": ("hipGraph replay of the step (encode, k_decode, k_compact); kernel times: HIP events "
                       "around the same launches issued one by one after the timed region") if graph_mode else
                      "eager launches; kernel times: HIP events in the timed region",
            "roofline": {
                "kernel": enc_path,
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if tr is None else tr["bytes_per_launch"],
                "algorithmic_bytes_per_launch": enc_bytes,
            },
        }
        if tr is not None:
            line["roofline"]["traffic_source"] = tr.get("source", "profiles/traffic.json")
        if other is not None:
            omode, el_o, enc_o, dec_o = other
            line[f"variant_{TAG_LABEL[omode]}"] = {
                "label": f"NOT the headline: same step with the tag = {TAG_TEXT[omode]}",
                "value": round(d.n * args.steps / el_o / 1e6, 2),
                "unit": "Mpkt/s",
                "ms_per_step": round(el_o / args.steps * 1e3, 4),
                "kernels_ms": {"encode": round(enc_o, 4), "decode+compact": round(dec_o, 4)},
                "roofline_frac": round(enc_bytes / (enc_o * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            }
        if anchor is not None:
            line["scale_n1_c5"] = anchor
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(cfg, min(args.cpu_sample, d.n), args.cpu_seconds,
                                                use_ref=args.cpu_baseline_ref)
        print(json.dumps(line), flush=True)
    if cx is not None:
        cx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
