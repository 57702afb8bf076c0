"""TEST INFRASTRUCTURE: ctypes wrappers over oracle/liboracle.so (clean-room C restatement) and
oracle/_ref/librsk_ref.so (the reference's own codec sources compiled here).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "librsk_ref.so")
REF_PARSE_SO = os.path.join(ROOT, "oracle", "_ref", "librsk_ref_parse.so")
REF_DEMUX_SO = os.path.join(ROOT, "oracle", "_ref", "librsk_ref_demux.so")

_vp = ctypes.c_void_p


def _p(a: np.ndarray | None):
    return None if a is None else a.ctypes.data


class OrcDec(ctypes.Structure):
    _fields_ = [("hlen", ctypes.c_uint8), ("cmd", ctypes.c_uint8), ("id", ctypes.c_uint8 * 8),
                ("conv", ctypes.c_uint32), ("conn_key", ctypes.c_uint64), ("pay_off", ctypes.c_uint16),
                ("pay_len", ctypes.c_uint16), ("status", ctypes.c_int8)]


class OrcTcpInfo(ctypes.Structure):
    _fields_ = [("src", ctypes.c_uint32), ("dst", ctypes.c_uint32), ("sp", ctypes.c_uint16),
                ("dp", ctypes.c_uint16), ("seq", ctypes.c_uint32), ("ack", ctypes.c_uint32),
                ("flag", ctypes.c_uint8), ("parse_status", ctypes.c_int8),
                ("cap_pay_off", ctypes.c_uint16), ("cap_pay_len", ctypes.c_uint16)]


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = self.L = ctypes.CDLL(path)
        L.orc_md5.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]
        L.orc_compute_hash.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint8]
        L.orc_hash_equal.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                     ctypes.c_int]
        L.orc_enchead_encode.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint8, ctypes.c_char_p,
                                         ctypes.c_uint32, ctypes.c_uint64]
        L.orc_enchead_decode.argtypes = [ctypes.c_char_p, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]
        L.orc_rconn_output.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int,
                                       ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64,
                                       ctypes.c_char_p]
        L.orc_rconn_onrecv.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int,
                                       ctypes.c_int, ctypes.POINTER(OrcDec)]
        L.orc_rawinput.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                   ctypes.c_int, ctypes.POINTER(OrcTcpInfo)]
        L.orc_tcpinfo_encode.argtypes = [ctypes.POINTER(OrcTcpInfo), ctypes.c_char_p]
        L.orc_tcpinfo_decode.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(OrcTcpInfo)]
        L.orc_syncinput.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_int,
                                    ctypes.POINTER(OrcTcpInfo), ctypes.POINTER(OrcDec)]
        L.orc_build_wire.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16,
                                     ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8,
                                     ctypes.c_uint16, ctypes.c_char_p, ctypes.c_char_p]
        L.orc_inet_csum.restype = ctypes.c_uint16
        L.orc_inet_csum.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
        L.orc_key_for_tcp.restype = ctypes.c_uint64
        L.orc_capture_filter.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, _vp]
        L.orc_filter_str.argtypes = [_vp, ctypes.c_char_p, ctypes.c_size_t]
        L.orc_demux_batch.argtypes = [ctypes.c_uint32] + [_vp] * 6 + [ctypes.c_uint32] + [_vp] * 5
        L.orc_demux_batch.restype = ctypes.c_int
        L.orc_key_for_tcp.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        L.orc_key_for_udp.restype = ctypes.c_uint64
        L.orc_key_for_udp.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        L.orc_splitmix64_at.restype = ctypes.c_uint64
        L.orc_splitmix64_at.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_fill_splitmix.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_bench_codec.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32] + [_vp] * 9 + [ctypes.c_int]
        L.orc_bench_codec.restype = ctypes.c_uint64
        L.orc_encode_batch.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32] + [_vp] * 11 + [ctypes.c_int]
        L.orc_decode_batch.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32] + [_vp] * 14 + [ctypes.c_int]
        L.orc_parse_decode_batch.argtypes = ([ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32, _vp, _vp, _vp,
                                              _vp, ctypes.c_int, ctypes.c_int] + [_vp] * 20)
        L.orc_tcp_send_seq_batch.argtypes = [ctypes.c_uint32, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp]
        L.orc_tcp_recv_ack_batch.argtypes = [ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_uint32, _vp]

    # ---- scalar ----
    def md5(self, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(16)
        self.L.orc_md5(msg, len(msg), out)
        return out.raw

    def tag(self, key: bytes, b: int) -> bytes:
        out = ctypes.create_string_buffer(8)
        self.L.orc_compute_hash(out, key, len(key), b)
        return out.raw

    def hash_equal(self, tag: bytes, key: bytes, data: bytes | None, data_len: int) -> bool:
        return bool(self.L.orc_hash_equal(tag, key, len(key), data, data_len))

    def enchead_encode(self, buf_len: int, cmd: int, idb: bytes, conv: int, key: int):
        out = ctypes.create_string_buffer(max(buf_len, 23))
        r = self.L.orc_enchead_encode(out, buf_len, cmd, idb, conv, key)
        return None if r < 0 else out.raw[:23]

    def enchead_decode(self, buf: bytes, buf_len: int):
        ln, cmd = ctypes.c_uint8(), ctypes.c_uint8()
        idb = ctypes.create_string_buffer(8)
        conv, key = ctypes.c_uint32(), ctypes.c_uint64()
        r = self.L.orc_enchead_decode(bytes(buf), buf_len, ctypes.addressof(ln), ctypes.addressof(cmd),
                                      ctypes.addressof(idb), ctypes.addressof(conv), ctypes.addressof(key))
        if r < 0:
            return None
        return ln.value, cmd.value, idb.raw, conv.value, key.value

    def rconn_output(self, key: bytes, payload: bytes, cmd: int, idb: bytes, conv: int, ckey: int):
        frame = ctypes.create_string_buffer(1600)
        st = self.L.orc_rconn_output(key, len(key), payload, len(payload), cmd, idb, conv, ckey, frame)
        return st, (frame.raw[:st] if st > 0 else b"")

    def rconn_onrecv(self, key: bytes, frame: bytes, nread: int | None = None, close: bool = False) -> OrcDec:
        d = OrcDec()
        if nread is None:
            nread = len(frame)
        self.L.orc_rconn_onrecv(key, len(key), bytes(frame), nread, int(close), ctypes.byref(d))
        return d

    def rawinput(self, pkt: bytes, wire_len: int, cap_len: int, datalink: int, flags: int) -> OrcTcpInfo:
        t = OrcTcpInfo()
        self.L.orc_rawinput(bytes(pkt), wire_len, cap_len, datalink, flags, ctypes.byref(t))
        return t

    def syncinput(self, key: bytes, rec: bytes, nread: int) -> tuple[OrcTcpInfo, OrcDec]:
        """RawTcp::syncInput -> RConn::OnRecv on one hand-off record (rec holds >= 21 bytes)."""
        t, d = OrcTcpInfo(), OrcDec()
        self.L.orc_syncinput(key, len(key), bytes(rec), nread, ctypes.byref(t), ctypes.byref(d))
        return t, d

    def tcpinfo_encode(self, t: OrcTcpInfo) -> bytes:
        out = ctypes.create_string_buffer(21)
        self.L.orc_tcpinfo_encode(ctypes.byref(t), out)
        return out.raw

    def key_for_tcp(self, sp: int, dp: int) -> int:
        return self.L.orc_key_for_tcp(sp, dp)

    def key_for_udp(self, sp: int, dp: int) -> int:
        return self.L.orc_key_for_udp(sp, dp)

    def build_wire(self, frame: bytes, src, dst, sp, dp, seq, ack, flag, ip_id, eth: bytes | None = None) -> bytes:
        out = ctypes.create_string_buffer(len(frame) + 64)
        n = self.L.orc_build_wire(frame, len(frame), src, dst, sp, dp, seq, ack, flag, ip_id, eth, out)
        return out.raw[:n]

    def capture_filter(self, pkt: bytes, datalink: int, filt, cap_len: int | None = None) -> int:
        cl = len(pkt) if cap_len is None else cap_len
        return self.L.orc_capture_filter(bytes(pkt) + b"\0" * 64, cl, datalink, ctypes.addressof(filt))

    def filter_str(self, filt) -> str:
        buf = ctypes.create_string_buffer(16384)
        n = self.L.orc_filter_str(ctypes.addressof(filt), buf, len(buf))
        assert n >= 0
        return buf.value.decode()

    def demux_batch(self, status, cmd, fields: int, id=None, conv=None, conn_key=None, dst=None):
        """-> list of (first packet, [packet indices]) in segment order (orc_demux_batch)."""
        n = len(status)
        arrs = [np.ascontiguousarray(status, np.int8), np.ascontiguousarray(cmd, np.uint8)]
        opt = [None if x is None else np.ascontiguousarray(x, dt)
               for x, dt in ((id, np.uint8), (conv, np.uint32), (conn_key, np.uint64), (dst, np.uint32))]
        perm = np.zeros(max(n, 1), np.uint32)
        seg_off = np.zeros(n + 1, np.uint32)
        first = np.zeros(max(n, 1), np.uint32)
        ns, nv = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        r = self.L.orc_demux_batch(n, *[_p(a) for a in arrs], *[_p(a) for a in opt], fields, _p(perm), _p(seg_off),
                                   _p(first), _p(ns), _p(nv))
        assert r == 0
        S = int(ns[0])
        return [(int(first[s]), perm[seg_off[s]:seg_off[s + 1]].tolist()) for s in range(S)], int(nv[0])

    def tcp_send_seq_batch(self, conn, status, conn_seq, ip_id_next: int):
        """-> (seq, ip_id, conn_seq after, ip_id_next after) (orc_tcp_send_seq_batch)."""
        n = len(conn)
        c = np.ascontiguousarray(conn, np.uint32)
        st = np.ascontiguousarray(status, np.int32)
        cs = np.array(conn_seq, np.uint32)
        ipn = np.array([ip_id_next], np.uint16)
        seq = np.zeros(max(n, 1), np.uint32)
        ipid = np.zeros(max(n, 1), np.uint16)
        self.L.orc_tcp_send_seq_batch(n, _p(c), _p(st), len(cs), _p(cs), _p(ipn), _p(seq), _p(ipid))
        return seq[:n], ipid[:n], cs, int(ipn[0])

    def tcp_recv_ack_batch(self, conn, delivered, seq, conn_ack):
        n = len(conn)
        c = np.ascontiguousarray(conn, np.uint32)
        dl = np.ascontiguousarray(delivered, np.uint8)
        sq = np.ascontiguousarray(seq, np.uint32)
        ca = np.array(conn_ack, np.uint32)
        self.L.orc_tcp_recv_ack_batch(n, _p(c), _p(dl), _p(sq), len(ca), _p(ca))
        return ca

    def splitmix_bytes(self, seed: int, n: int) -> np.ndarray:
        out = np.empty(n, np.uint8)
        self.L.orc_fill_splitmix(_p(out), n, seed)
        return out

    # ---- batch (numpy SoA) ----
    def encode_batch(self, key: bytes, payload: np.ndarray, d, id_uniform: bytes, nthreads: int = 8,
                     frame_bytes: int | None = None, idarr: np.ndarray | None = None):
        n = d.n
        if frame_bytes is None:
            frame_bytes = n * d.frame_pitch
        frames = np.zeros(frame_bytes, np.uint8)
        status = np.zeros(n, np.int32)
        idu = np.frombuffer(bytes(id_uniform)[:8].ljust(8, b"\0"), np.uint8).copy()
        arrs = [np.ascontiguousarray(x) for x in (payload, d.pay_off.astype(np.uint64), d.pay_len.astype(np.uint16),
                                                   d.cmd.astype(np.uint8), d.conv.astype(np.uint32),
                                                   d.conn_key.astype(np.uint64))]
        fo = np.ascontiguousarray(d.frame_off.astype(np.uint64))  # keep alive across the call
        self.L.orc_encode_batch(key, len(key), n, *[_p(a) for a in arrs], _p(idarr), _p(idu), _p(frames),
                                _p(fo), _p(status), nthreads)
        return frames, status

    def bench_codec(self, key: bytes, payload: np.ndarray, d, idb: bytes, frames: np.ndarray, nthreads: int) -> int:
        """orc_bench_codec: framing into a zeroed 1500-B buffer + store + OnRecv per packet (the
        clean-room CPU baseline, bench.py); returns the verified count."""
        arrs = [np.ascontiguousarray(x) for x in (payload, d.pay_off.astype(np.uint64), d.pay_len.astype(np.uint16),
                                                   d.cmd.astype(np.uint8), d.conv.astype(np.uint32),
                                                   d.conn_key.astype(np.uint64))]
        idu = np.frombuffer(bytes(idb)[:8].ljust(8, b"\0"), np.uint8).copy()
        fo = np.ascontiguousarray(d.frame_off.astype(np.uint64))
        return int(self.L.orc_bench_codec(key, len(key), d.n, *[_p(a) for a in arrs], _p(idu), _p(frames), _p(fo),
                                          nthreads))

    def decode_batch(self, key: bytes, frames: np.ndarray, frame_off: np.ndarray, frame_len: np.ndarray,
                     is_tcp_close: np.ndarray | None = None, nthreads: int = 8) -> dict:
        n = len(frame_len)
        out = {
            "hlen": np.zeros(n, np.uint8), "cmd": np.zeros(n, np.uint8), "id": np.zeros(8 * n, np.uint8),
            "conv": np.zeros(n, np.uint32), "conn_key": np.zeros(n, np.uint64),
            "pay_off": np.zeros(n, np.uint16), "pay_len": np.zeros(n, np.uint16),
            "status": np.zeros(n, np.int8), "valid_idx": np.zeros(max(n, 1), np.uint32),
        }
        nv = ctypes.c_uint32()
        fo = np.ascontiguousarray(frame_off.astype(np.uint64))
        fl = np.ascontiguousarray(frame_len.astype(np.uint16))
        cl = None if is_tcp_close is None else np.ascontiguousarray(is_tcp_close.astype(np.uint8))
        self.L.orc_decode_batch(key, len(key), n, _p(frames), _p(fo), _p(fl), _p(cl),
                                *[_p(out[k]) for k in ("hlen", "cmd", "id", "conv", "conn_key", "pay_off",
                                                       "pay_len", "status", "valid_idx")],
                                ctypes.addressof(nv), nthreads)
        out["n_valid"] = nv.value
        return out

    def parse_decode_batch(self, key: bytes, cap: np.ndarray, cap_off, wire_len, cap_len, datalink: int,
                           flags: int) -> dict:
        n = len(wire_len)
        spec = [("src", np.uint32), ("dst", np.uint32), ("sp", np.uint16), ("dp", np.uint16),
                ("seq", np.uint32), ("ack", np.uint32), ("flag", np.uint8), ("parse_status", np.int8),
                ("cap_pay_off", np.uint16), ("cap_pay_len", np.uint16), ("hlen", np.uint8), ("cmd", np.uint8)]
        out = {k: np.zeros(n, dt) for k, dt in spec}
        out["id"] = np.zeros(8 * n, np.uint8)
        for k, dt in (("conv", np.uint32), ("conn_key", np.uint64), ("pay_off", np.uint16),
                      ("pay_len", np.uint16), ("status", np.int8)):
            out[k] = np.zeros(n, dt)
        out["valid_idx"] = np.zeros(max(n, 1), np.uint32)
        nv = ctypes.c_uint32()
        co = np.ascontiguousarray(np.asarray(cap_off, np.uint64))
        wl = np.ascontiguousarray(np.asarray(wire_len, np.uint32))
        cl = np.ascontiguousarray(np.asarray(cap_len, np.uint32))
        order = ["src", "dst", "sp", "dp", "seq", "ack", "flag", "parse_status", "cap_pay_off", "cap_pay_len",
                 "hlen", "cmd", "id", "conv", "conn_key", "pay_off", "pay_len", "status", "valid_idx"]
        self.L.orc_parse_decode_batch(key, len(key), n, _p(cap), _p(co), _p(wl), _p(cl), datalink, flags,
                                      *[_p(out[k]) for k in order], ctypes.addressof(nv))
        out["n_valid"] = nv.value
        return out


class RefOracle:
    """The reference's own functions (oracle/_ref/librsk_ref.so), for pinning and the CPU baseline."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.L = ctypes.CDLL(path)
        L.ref_compute_hash.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.ref_hash_equal.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        L.ref_enc2buf.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32,
                                  ctypes.c_uint64]
        L.ref_decodebuf.argtypes = [ctypes.c_char_p, ctypes.c_int, _vp, _vp, _vp, _vp]
        L.ref_rconn_output.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint8,
                                       ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_char_p]
        L.ref_rconn_onrecv.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_int,
                                       _vp, _vp, _vp, _vp, _vp, _vp, _vp]
        L.ref_key_for_tcp.restype = ctypes.c_uint64
        L.ref_key_for_tcp.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        L.ref_key_for_udp.restype = ctypes.c_uint64
        L.ref_key_for_udp.argtypes = [ctypes.c_uint16, ctypes.c_uint16]
        L.ref_tcpinfo_encode.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_uint16,
                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint8, ctypes.c_char_p,
                                         ctypes.c_int]
        L.ref_tcpinfo_decode.argtypes = [ctypes.c_char_p, ctypes.c_int, _vp]
        L.ref_bench_codec.restype = ctypes.c_uint64
        L.ref_bench_codec.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_uint32] + [_vp] * 9 + [ctypes.c_int]

    def tag(self, key: bytes, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(8)
        self.L.ref_compute_hash(out, key, len(key), data, len(data))
        return out.raw

    def hash_equal(self, tag: bytes, key: bytes, data: bytes | None, data_len: int) -> bool:
        return bool(self.L.ref_hash_equal(tag, key, len(key), data, data_len))

    def enc2buf(self, buf_len: int, cmd: int, idb: bytes, conv: int, key: int):
        out = ctypes.create_string_buffer(max(buf_len, 23))
        r = self.L.ref_enc2buf(out, buf_len, cmd, idb, conv, key)
        return None if r < 0 else out.raw[:r]

    def decodebuf(self, buf: bytes, buf_len: int):
        cmd = ctypes.c_uint8()
        idb = ctypes.create_string_buffer(8)
        conv, key = ctypes.c_uint32(), ctypes.c_uint64()
        r = self.L.ref_decodebuf(bytes(buf), buf_len, ctypes.addressof(cmd), ctypes.addressof(idb),
                                 ctypes.addressof(conv), ctypes.addressof(key))
        if r < 0:
            return None
        return bytes(buf)[0], cmd.value, idb.raw, conv.value, key.value

    def rconn_output(self, key: bytes, payload: bytes, cmd: int, idb: bytes, conv: int, ckey: int):
        frame = ctypes.create_string_buffer(1600)
        st = self.L.ref_rconn_output(key, len(key), payload, len(payload), cmd, idb, conv, ckey, frame)
        return st, (frame.raw[:st] if st > 0 else b"")

    def rconn_onrecv(self, key: bytes, frame: bytes, nread: int | None = None, close: bool = False):
        if nread is None:
            nread = len(frame)
        hlen, cmd = ctypes.c_uint8(), ctypes.c_uint8()
        idb = ctypes.create_string_buffer(8)
        conv, ckey = ctypes.c_uint32(), ctypes.c_uint64()
        po, pl = ctypes.c_int(), ctypes.c_int()
        st = self.L.ref_rconn_onrecv(key, len(key), bytes(frame), nread, int(close), ctypes.addressof(hlen),
                                     ctypes.addressof(cmd), ctypes.addressof(idb), ctypes.addressof(conv),
                                     ctypes.addressof(ckey), ctypes.addressof(po), ctypes.addressof(pl))
        if st != 1:
            return st, None
        return st, (hlen.value, cmd.value, idb.raw, conv.value, ckey.value, po.value, pl.value)

    def key_for_tcp(self, sp: int, dp: int) -> int:
        return self.L.ref_key_for_tcp(sp, dp)

    def key_for_udp(self, sp: int, dp: int) -> int:
        return self.L.ref_key_for_udp(sp, dp)

    def tcpinfo_encode(self, src, dst, sp, dp, seq, ack, flag) -> bytes:
        out = ctypes.create_string_buffer(64)
        r = self.L.ref_tcpinfo_encode(src, dst, sp, dp, seq, ack, flag, out, 64)
        return out.raw[:r]

    def bench_codec(self, key: bytes, payload: np.ndarray, d, idb: bytes, frames: np.ndarray, nthreads: int) -> int:
        arrs = [np.ascontiguousarray(x) for x in (d.pay_off.astype(np.uint64), d.pay_len.astype(np.uint16),
                                                   d.cmd.astype(np.uint8), d.conv.astype(np.uint32),
                                                   d.conn_key.astype(np.uint64))]
        fo = np.ascontiguousarray(d.frame_off.astype(np.uint64))
        return self.L.ref_bench_codec(key, len(key), d.n, _p(payload), *[_p(a) for a in arrs], idb, _p(frames),
                                      _p(fo), nthreads)


class RefParse:
    """The reference's own RawTcp::RawInput (oracle/_ref/librsk_ref_parse.so, conn/RawTcp.cpp:138-237
    compiled with the objects it needs; oracle/ref_parse_harness.cpp).  Loaded with RTLD_LAZY: the
    libnet / pcap / service functions RawInput never calls stay unbound (oracle/Makefile)."""

    FIELDS = ("ret", "called", "src", "dst", "sp", "dp", "seq", "ack", "flag", "pay_off", "payload_len",
              "base_ret", "pool_n", "pool_src", "pool_dst", "pool_sp", "pool_dp", "pool_seq", "pool_ack",
              "pool_flag")

    def __init__(self, path: str = REF_PARSE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.L = ctypes.CDLL(path, mode=os.RTLD_LAZY)
        L.ref_rawinput.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, _vp]

    def rawinput(self, pkt: bytes, wire_len: int, cap_len: int, datalink: int, is_server: bool,
                 with_ack_pool: bool) -> dict:
        out = np.zeros(20, np.uint32)
        # the reference reads headers without looking at caplen: give it slack past the packet
        self.L.ref_rawinput(bytes(pkt) + bytes(128), wire_len, cap_len, datalink, int(is_server),
                            int(with_ack_pool), out.ctypes.data)
        r = {k: int(v) for k, v in zip(self.FIELDS, out)}
        for k in ("ret", "payload_len", "base_ret"):
            r[k] = int(np.int32(np.uint32(r[k])))
        return r


class RefDemux:
    """The reference's own receive routing (oracle/_ref/librsk_ref_demux.so: ServerGroup, SubGroup,
    ClientGroup, IAppGroup, INetGroup, IGroup, IConn, INetConn, CConn compiled from /root/reference;
    oracle/ref_demux_harness.cpp records what reaches each conn).  RTLD_LAZY as RefParse."""

    SERVER, CLIENT = 0, 1
    EV_CREATE, EV_DELIVER, EV_RST_IN, EV_KA_IN, EV_CONV_RST, EV_NETCONN_RST, EV_DEFAULT_IN = range(1, 8)
    LV_GROUP, LV_NET, LV_LEAF = 0, 1, 2

    def __init__(self, path: str = REF_DEMUX_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.L = ctypes.CDLL(path, mode=os.RTLD_LAZY)
        L.ref_demux_run.argtypes = [ctypes.c_int, ctypes.c_uint32] + [_vp] * 7 + [ctypes.c_uint32, _vp,
                                    ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint32, _vp,
                                    _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp]

    def run(self, stack: int, status, cmd, ids, conv, conn_key, dst, order=None, known_keys=(),
            known_convs=()) -> dict:
        """Route the VALID packets in `order` (default: arrival order).  Returns the raw log:
        ret [n] int32 (0 for packets not routed), ev [k, 4] int64 (kind, conn, pkt, aux) and the conn
        table (level, parent, key bytes)."""
        n = len(status)
        c = lambda a, t: np.ascontiguousarray(np.asarray(a, t))
        valid = c(np.asarray(status) == 1, np.int8)  # RSK_RECV_VALID: what RConn::OnRecv passes up
        cmd, conv, dst = c(cmd, np.uint8), c(conv, np.uint32), c(dst, np.uint32)
        ids, conn_key = c(ids, np.uint8).reshape(-1), c(conn_key, np.uint64)
        order = c(np.arange(n) if order is None else order, np.uint32)
        kk, kc = c(list(known_keys), np.uint64), c(list(known_convs), np.uint32)
        ret = np.zeros(n, np.int32)
        ev_cap = 4 * n + 16
        conn_cap = 3 * n + len(kk) + len(kc) + 16
        ev = np.zeros((ev_cap, 4), np.int64)
        lvl, par = np.zeros(conn_cap, np.int32), np.zeros(conn_cap, np.int32)
        key, klen = np.zeros((conn_cap, 48), np.uint8), np.zeros(conn_cap, np.uint32)
        n_ev, n_conn = np.zeros(1, np.uint32), np.zeros(1, np.uint32)
        rc = self.L.ref_demux_run(stack, n, _p(valid), _p(cmd), _p(ids), _p(conv), _p(conn_key), _p(dst),
                                  _p(order), len(order), _p(kk), len(kk), _p(kc), len(kc), _p(ret), _p(ev),
                                  ev_cap, _p(n_ev), _p(lvl), _p(par), _p(key), _p(klen), conn_cap, _p(n_conn))
        assert rc == 0, rc
        nc = int(n_conn[0])
        conns = [(int(lvl[i]), int(par[i]), bytes(key[i, :klen[i]])) for i in range(nc)]
        return {"ret": ret, "ev": ev[:int(n_ev[0])].copy(), "conns": conns}

    @classmethod
    def conn_path(cls, conns, c: int) -> tuple:
        """A conn's identity: its (level, key) and those of the groups above it."""
        out = []
        while c >= 0:
            lv, par, k = conns[c]
            out.append((lv, k))
            c = par
        return tuple(reversed(out))

    @classmethod
    def trace(cls, log: dict) -> dict:
        """The observable effect of a routing run: per conn (by identity) the packets it received in
        order, the order each level created its conns, and the control / reset events in order."""
        conns, per_conn, created, events = log["conns"], {}, {}, []
        for kind, c, pkt, aux in log["ev"].tolist():
            if kind == cls.EV_CREATE:
                created.setdefault(conns[c][0], []).append(cls.conn_path(conns, c))
            elif kind == cls.EV_DELIVER:
                per_conn.setdefault(cls.conn_path(conns, c), []).append(pkt)
            else:
                events.append((kind, pkt, aux))
        return {"per_conn": per_conn, "created": created, "events": events, "ret": log["ret"]}


def ref_demux_available() -> bool:
    return os.path.exists(REF_DEMUX_SO)


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref_parse_available() -> bool:
    return os.path.exists(REF_PARSE_SO)
