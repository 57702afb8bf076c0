#!/usr/bin/env python3
"""Generates tests/golden/demux.npz from the REFERENCE's own receive routing
(oracle/_ref/librsk_ref_demux.so: ServerGroup / SubGroup / ClientGroup / IAppGroup / INetGroup
compiled from /root/reference by `make -C oracle ref`; oracle/ref_demux_harness.cpp).  Run in the
build container:

    make -C oracle ref && python tests/golden/make_demux_golden.py

Each case stores its inputs (the decoded fields of a receive batch) and, per packet, what the
reference's routing did with it in arrival order (tests/demux_ref.py:outcomes).  Data only.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from tests import demux_ref as D  # noqa: E402
from tests.oracle_lib import RefDemux  # noqa: E402

# name, stack, n, groups, nets, convs, p_ctrl, p_valid, p_bad_cmd, control packets at
TILE_EDGES = (511, 512, 1023, 1024, 4095, 4096, 4097, 8191, 8192)
CASES = [
    ("server_small", D.SERVER, 2000, 3, 4, 6, 0.01, 0.9, 0.0, ()),
    ("server_many_groups", D.SERVER, 20000, 40, 8, 50, 0.002, 0.85, 0.0, ()),
    ("server_dense_ctrl", D.SERVER, 3000, 2, 3, 4, 0.2, 0.9, 0.05, ()),
    ("server_tile_edges", D.SERVER, 9000, 1, 3, 2, 0.0, 1.0, 0.0, TILE_EDGES),
    ("server_one_conv_many_conns", D.SERVER, 70000, 1, 16, 1, 0.0005, 0.95, 0.0, ()),
    ("server_one_packet", D.SERVER, 1, 1, 1, 1, 0.0, 1.0, 0.0, ()),
    ("server_all_dropped", D.SERVER, 500, 2, 2, 2, 0.0, 0.0, 0.0, ()),
    ("client_small", D.CLIENT, 3000, 1, 6, 10, 0.01, 0.9, 0.0, ()),
    ("client_large", D.CLIENT, 50000, 1, 12, 64, 0.001, 0.95, 0.001, ()),
    ("client_tile_edges", D.CLIENT, 9000, 1, 2, 3, 0.0, 1.0, 0.0, TILE_EDGES),
]


def main():
    ref = RefDemux()
    out = {}
    names = []
    for ci, (name, stack, n, ng, nn, nc, pc, pv, pb, at) in enumerate(CASES):
        rng = np.random.default_rng(0xDE3A + ci)
        status, cmd, ids, conv, ckey, dst = D.rsock_case(rng, n, ng, nn, nc, pc, pv, pb, at)
        known_keys, known_convs = (), ()
        if stack == D.CLIENT:  # the connected fake-TCP conns and the local apps' convs: most, not all
            keys = np.unique(ckey)
            known_keys = keys[rng.random(len(keys)) < 0.8]
            known_convs = np.arange(1, nc + 1)[rng.random(nc) < 0.75].astype(np.uint32)
        log = ref.run(stack, status, cmd, ids, conv, ckey, dst, known_keys=known_keys, known_convs=known_convs)
        o = D.outcomes(RefDemux, log, n)
        fields = D.SERVER_FIELDS if stack == D.SERVER else D.CLIENT_FIELDS
        p = f"c{ci}_"
        out.update({p + "status": status, p + "cmd": cmd, p + "id": ids, p + "conv": conv, p + "conn_key": ckey,
                    p + "dst": dst, p + "known_keys": np.asarray(known_keys, np.uint64),
                    p + "known_convs": np.asarray(known_convs, np.uint32),
                    p + "meta": np.array([stack, fields, n], np.int64)})
        out.update({p + k: v for k, v in o.items()})
        names.append(name)
        nleaf = int(o["leaf"].max()) + 1 if n else 0
        print(f"{name}: n={n} valid={(status == 1).sum()} leaves={nleaf} ctrl={int(o['ctrl'].sum())} "
              f"conv_rst={(o['rst_conv'] >= 0).sum()}")
    out["names"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "demux.npz"), **out)


if __name__ == "__main__":
    main()
