"""Host-side pieces of bench.py (no GPU): the algorithmic byte counts the roofline divides by, the
PMC traffic lookup, the tag-mode labels of the headline and of the table variant, and the CPU
baseline leg (the clean-room C restatement, `kind: "port"`) on a tiny sample."""
import json
import os

import numpy as np
import pytest

import bench
from rsock_amd import workload
from tests import oracle_lib


def test_enc_bytes_per_packet_matches_design():
    # 2P + 66 per packet (C3: 2866 B, 12.02 GB per 4M-packet launch)
    assert bench.enc_bytes_per_pkt(1400) == 2866
    assert bench.enc_bytes_per_pkt(64) == 194
    d = workload.describe("c3", 0, 4 << 20, n=4 << 20)
    assert int(bench.enc_bytes_per_pkt(d.pay_len.astype(np.int64)).sum()) == 12020875264
    # decode reads a 32-B header window + offsets and writes the SoA fields: 73 B
    assert bench.dec_bytes_per_pkt() == 73


def test_traffic_lookup_is_keyed_by_layout():
    path = os.path.join(bench.ROOT, "profiles", "traffic.json")
    table = json.load(open(path))
    for key, rec in table.items():
        cfg, n = key.split(":")
        got = bench.load_traffic(cfg, int(n), rec["frame_pitch"])
        assert got is not None and got["bytes_per_launch"] == rec["bytes_per_launch"]
        # PMC bytes are read + write (FETCH_SIZE x 2, KiB x 1024), never below the algorithmic bytes
        assert got["bytes_per_launch"] == pytest.approx(got["read_bytes_per_launch"] + got["write_bytes_per_launch"])
        assert got["ratio_to_algorithmic"] >= 1.0
        # another slot pitch is another layout: no traffic figure for it
        assert bench.load_traffic(cfg, int(n), rec["frame_pitch"] + 16) is None
    assert bench.load_traffic("c3", 12345, 1440) is None


def test_headline_tag_is_md5_per_lane():
    # the measured kernel computes MD5 per lane; the table variant is labelled
    assert bench.TAG_LABEL["md5"] == "md5_per_lane"
    assert "MD5 compression per packet" in bench.TAG_TEXT["md5"]
    assert "table" in bench.TAG_TEXT["table"]


def test_cpu_baseline_port_runs_on_a_small_sample():
    if not os.path.exists(oracle_lib.ORACLE_SO):
        pytest.skip("oracle/liboracle.so not built (make -C oracle)")
    r = bench.cpu_baseline("c2", 4096, 0.05)
    assert r["kind"] == "port" and r["unit"] == "Mpkt/s"
    assert r["value"] > 0 and r["value_1thread"] > 0
    assert r["cores"] in (int(t) for t in r["by_threads"])
    assert "C2" in r["sample"] and "1 thread" in r["sample"]
