"""GPU: the RConn-shaped batching adapter (include/rsk_rconn.h) — per-packet Output/OnRecv with
RConn's return contract, batched through the GPU, callbacks in input order — against the oracle."""
from __future__ import annotations

import ctypes

import numpy as np
import pytest

from rsock_amd import _abi

pytestmark = pytest.mark.gpu
KEY = b"hello135"


class Adapter:
    def __init__(self, batch):
        self.L = _abi.load()
        self.r = self.L.rsk_rconn_create(KEY, len(KEY), 0, batch)
        assert self.r, self.L.rsk_last_error()
        self.sent, self.resets, self.recvd, self.events = [], [], [], []
        self._send = _abi.SEND_FN(lambda f, n, u, a: (self.sent.append((ctypes.string_at(f, n), u)),
                                                      self.events.append(("send", u)), 0)[2])
        self._reset = _abi.RESET_FN(lambda u, a: (self.resets.append(u), self.events.append(("reset", u)), 7)[2])

        def recv(st, hlen, cmd, idp, conv, key, pay, plen, u, a):
            rec = (st, u)
            if st == 1:
                rec = (st, u, hlen, cmd, ctypes.string_at(idp, 8), conv, key, ctypes.string_at(pay, plen))
            self.recvd.append(rec)
            return 0

        self._recv = _abi.RECV_FN(recv)
        self.L.rsk_rconn_set_callbacks(self.r, ctypes.cast(self._send, ctypes.c_void_p),
                                       ctypes.cast(self._reset, ctypes.c_void_p),
                                       ctypes.cast(self._recv, ctypes.c_void_p), None)

    def close(self):
        self.L.rsk_rconn_destroy(self.r)


@pytest.mark.parametrize("batch", [1, 37, 4096])
def test_adapter_output_onrecv(gpu, oracle, batch):
    rng = np.random.default_rng(batch)
    ad = Adapter(batch)
    try:
        pkts = []
        lens = [0, 1, 1469, 1470, 5000] + list(rng.integers(1, 1470, 300))
        lens[40:40] = [0]  # a reset in the middle of a batch (and at a batch edge for batch 37)
        lens[74:74] = [0, 0]
        for k, ln in enumerate(lens):
            p = rng.integers(0, 256, int(ln), dtype=np.uint8).tobytes()
            fields = (int(rng.integers(0, 5)), rng.integers(0, 256, 8, dtype=np.uint8).tobytes(),
                      int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)))
            r = ad.L.rsk_rconn_output(ad.r, len(p), p, fields[0], fields[1], fields[2], fields[3], k + 1)
            exp = 0 if ln == 0 else (-1 if ln + 31 > 1500 else ln + 31)  # resets are queued: 0
            assert r == exp, (ln, r)
            pkts.append((p, fields, k + 1))
        assert ad.L.rsk_rconn_flush(ad.r) == 0
        assert ad.resets == [u for p, _, u in pkts if len(p) == 0] and len(ad.resets) == 4
        # send and reset callbacks interleave in input order (RConn::Output is synchronous)
        assert ad.events == [("reset" if len(p) == 0 else "send", u) for p, _, u in pkts if len(p) <= 1469]
        framed = [(p, f, u) for p, f, u in pkts if 0 < len(p) <= 1469]
        assert [u for _, u in ad.sent] == [u for _, _, u in framed]  # input order
        for (frame, _), (p, f, u) in zip(ad.sent, framed):
            st, exp = oracle.rconn_output(KEY, p, *f)
            assert frame == exp
        # receive side: the frames back, some corrupted / truncated / oversize, FIN/RST flags
        frames = []
        for k, (frame, u) in enumerate(ad.sent):
            g = bytearray(frame)
            if k % 7 == 1:
                g[3] ^= 0x10
            if k % 11 == 2:
                g = g[: int(rng.integers(0, 32))]
            frames.append((bytes(g), bool(k & 1), 1000 + k))
        big = bytearray(oracle.rconn_output(KEY, b"\x42" + bytes(50), 0, b"abcdefgh", 5, 6)[1])
        big += bytes(3000)  # 3081-B frame (UDP can deliver it): longer than a staging slot
        frames.append((bytes(big), False, 99999))
        for f, c, u in frames:
            assert ad.L.rsk_rconn_onrecv(ad.r, len(f), f, int(c), u) == 0
        assert ad.L.rsk_rconn_flush(ad.r) == 0
        assert len(ad.recvd) == len(frames)
        for got, (f, c, u) in zip(ad.recvd, frames):
            d = oracle.rconn_onrecv(KEY, f, close=c)
            assert got[0] == d.status and got[1] == u
            if d.status == 1:
                assert got[2:7] == (d.hlen, d.cmd, bytes(d.id), d.conv, d.conn_key)
                assert got[7] == f[d.pay_off: d.pay_off + d.pay_len]
        assert ad.recvd[-1][0] == 1 and len(ad.recvd[-1][7]) == len(big) - 31
    finally:
        ad.close()
