"""Host-side mirror of rsock's codec surface over the HIP C-ABI.

Names follow the reference:
  * ``Codec.compute_hash`` / ``Codec.hash_equal``   <- util/rhash.h:13-17
  * ``Codec.enc2buf`` / ``Codec.decodebuf``          <- EncHead::Enc2Buf / DecodeBuf (bean/EncHead.h:38-40)
  * ``Codec.output_batch`` (RConn::Output framing)   <- conn/RConn.cpp:87-105
  * ``Codec.onrecv_batch`` (RConn::OnRecv)           <- conn/RConn.cpp:64-85
  * ``Codec.rawinput_batch`` (RawTcp::RawInput + OnRecv) <- conn/RawTcp.cpp:138-244
Batch arguments are torch tensors on the codec's device (torch is used only for memory and
streams).  Every call goes through ``rsock_amd/librsk.so``; there is no CPU path here.
"""
from __future__ import annotations

import ctypes

import numpy as np
from dataclasses import dataclass, fields

import torch

from . import _abi

_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = _abi.load()
    return _lib


def _ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


class RskError(RuntimeError):
    pass


def _check(rc: int, what: str) -> None:
    if rc != 0:
        err = lib().rsk_last_error()
        raise RskError(f"{what} failed: rc={rc} ({err.decode() if err else ''})")


@dataclass
class DecodeBuffers:
    """SoA outputs of RConn::OnRecv for n frames (rsk_decode_out)."""

    hlen: torch.Tensor
    cmd: torch.Tensor
    id: torch.Tensor  # n*8 bytes
    conv: torch.Tensor  # int32 storage of u32
    conn_key: torch.Tensor  # int64 storage of u64
    pay_off: torch.Tensor  # int16 storage of u16
    pay_len: torch.Tensor  # int16 storage of u16
    status: torch.Tensor  # int8
    valid_idx: torch.Tensor  # int32 storage of u32
    n_valid: torch.Tensor  # int32 [1]

    @classmethod
    def alloc(cls, n: int, device) -> "DecodeBuffers":
        e = lambda k, dt: torch.empty(k, dtype=dt, device=device)  # noqa: E731
        return cls(
            hlen=e(n, torch.uint8),
            cmd=e(n, torch.uint8),
            id=e(n * 8, torch.uint8),
            conv=e(n, torch.int32),
            conn_key=e(n, torch.int64),
            pay_off=e(n, torch.int16),
            pay_len=e(n, torch.int16),
            status=e(n, torch.int8),
            valid_idx=e(max(n, 1), torch.int32),
            n_valid=e(1, torch.int32),
        )

    def abi(self, compact: bool = True) -> _abi.DecodeOut:
        return _abi.DecodeOut(
            _ptr(self.hlen), _ptr(self.cmd), _ptr(self.id), _ptr(self.conv), _ptr(self.conn_key),
            _ptr(self.pay_off), _ptr(self.pay_len), _ptr(self.status),
            _ptr(self.valid_idx) if compact else None, _ptr(self.n_valid) if compact else None,
        )

    def to_host(self) -> dict:
        out = {}
        for f in fields(self):
            out[f.name] = getattr(self, f.name).cpu().numpy()
        return out


def stage_capture_slots(arena: np.ndarray, offs: np.ndarray, cap_len: np.ndarray, slot: int,
                        nthreads: int = 8) -> np.ndarray:
    """Host staging for rsk_parse_decode_slots_batch (rsk_stage_capture_slots): an (n, slot) uint8
    array, row i = the first min(cap_len[i], slot) captured bytes of packet i, zero-filled."""
    n = len(offs)
    arena = np.ascontiguousarray(arena, np.uint8)
    offs = np.ascontiguousarray(offs, np.uint64)
    cap_len = np.ascontiguousarray(cap_len, np.uint32)
    slots = np.empty((n, slot), np.uint8)
    _check(lib().rsk_stage_capture_slots(n, arena.ctypes.data, offs.ctypes.data, cap_len.ctypes.data, slot,
                                         slots.ctypes.data, nthreads), "rsk_stage_capture_slots")
    return slots


def stage_decode_headers(arena: np.ndarray, offs: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """Host staging for rsk_decode_headers_batch, vectorised (same bytes as rsk_stage_decode_header):
    slot = frame[0:min(32, len)] zero-filled, byte 31 = frame[8 + frame[8]] when that is inside."""
    n = len(offs)
    offs = offs.astype(np.int64)
    lens = lens.astype(np.int64)
    k = np.arange(32)
    idx = offs[:, None] + k[None, :]
    inside = k[None, :] < lens[:, None]
    slots = np.where(inside, arena[np.minimum(idx, len(arena) - 1)], 0).astype(np.uint8)
    has8 = lens > 8
    ln = np.where(has8, arena[np.minimum(offs + 8, len(arena) - 1)], 0).astype(np.int64)
    at = 8 + ln
    ok = has8 & (at < lens)
    slots[ok, 31] = arena[(offs + at)[ok]]
    return slots.reshape(n, 32)


def ip_u32(ip: str) -> int:
    """Dotted IPv4 -> the u32 the header stores (network-order bytes read little-endian)."""
    b = bytes(int(x) for x in ip.split("."))
    return int.from_bytes(b, "little")


def make_filter(src_ip: str | None = None, dst_ip: str | None = None, src_singles=(), src_ranges=(), dst_singles=(),
                dst_ranges=(), is_server: bool = False) -> _abi.CaptureFilter:
    """rsk_capture_filter from BuildFilterStr's inputs (srcIp, dstIp, srcPorts, dstPorts, isServer)."""
    f = _abi.CaptureFilter()
    if src_ip:
        f.src_ip, f.has_src_ip = ip_u32(src_ip), 1
    if dst_ip:
        f.dst_ip, f.has_dst_ip = ip_u32(dst_ip), 1
    f.is_server = 1 if is_server else 0
    for pl, singles, ranges in ((f.src_ports, src_singles, src_ranges), (f.dst_ports, dst_singles, dst_ranges)):
        assert len(singles) <= _abi.FILTER_MAX_PORTS and len(ranges) <= _abi.FILTER_MAX_PORTS
        pl.n_single, pl.n_range = len(singles), len(ranges)
        for q, v in enumerate(singles):
            pl.single[q] = v
        for q, (a, b) in enumerate(ranges):
            pl.range[q][0], pl.range[q][1] = a, b
    return f


def filter_str(filt: _abi.CaptureFilter) -> str:
    """BuildFilterStr's string for this filter (host function of librsk; no GPU needed)."""
    buf = ctypes.create_string_buffer(16384)
    n = lib().rsk_filter_str(ctypes.byref(filt), buf, len(buf))
    if n < 0:
        raise RskError("rsk_filter_str: buffer too small")
    return buf.value.decode()


@dataclass
class DemuxBuffers:
    """Outputs of rsk_demux_batch for a batch of n packets (rsk_demux_out)."""

    perm: torch.Tensor
    seg_off: torch.Tensor
    seg_first: torch.Tensor
    n_seg: torch.Tensor
    n_valid: torch.Tensor

    @classmethod
    def alloc(cls, n: int, device) -> "DemuxBuffers":
        e = lambda k: torch.empty(k, dtype=torch.int32, device=device)  # noqa: E731
        return cls(perm=e(max(n, 1)), seg_off=e(n + 1), seg_first=e(max(n, 1)), n_seg=e(1), n_valid=e(1))

    def abi(self) -> _abi.DemuxOut:
        return _abi.DemuxOut(*[_ptr(getattr(self, f.name)) for f in fields(self)])

    def segments(self):
        """Host view: list of (first packet, [packet indices]) in segment order."""
        ns, nv = int(self.n_seg.item()), int(self.n_valid.item())
        perm = self.perm[:nv].cpu().numpy().astype("uint32")
        off = self.seg_off[: ns + 1].cpu().numpy().astype("uint32")
        first = self.seg_first[:ns].cpu().numpy().astype("uint32")
        return [(int(first[s]), perm[off[s]:off[s + 1]].tolist()) for s in range(ns)]


@dataclass
class TcpInfoBuffers:
    """SoA TcpInfo outputs of RawTcp::RawInput for n captured packets (rsk_tcpinfo_out)."""

    src: torch.Tensor
    dst: torch.Tensor
    sp: torch.Tensor
    dp: torch.Tensor
    seq: torch.Tensor
    ack: torch.Tensor
    flag: torch.Tensor
    parse_status: torch.Tensor
    cap_pay_off: torch.Tensor
    cap_pay_len: torch.Tensor

    @classmethod
    def alloc(cls, n: int, device) -> "TcpInfoBuffers":
        e = lambda dt: torch.empty(n, dtype=dt, device=device)  # noqa: E731
        return cls(
            src=e(torch.int32), dst=e(torch.int32), sp=e(torch.int16), dp=e(torch.int16),
            seq=e(torch.int32), ack=e(torch.int32), flag=e(torch.uint8),
            parse_status=e(torch.int8), cap_pay_off=e(torch.int16), cap_pay_len=e(torch.int16),
        )

    def abi(self) -> _abi.TcpInfoOut:
        return _abi.TcpInfoOut(*[_ptr(getattr(self, f.name)) for f in fields(self)])

    def to_host(self) -> dict:
        return {f.name: getattr(self, f.name).cpu().numpy() for f in fields(self)}


TAG_MODES = {"md5": _abi.TAG_MD5, "table": _abi.TAG_TABLE}


class Codec:
    """One rsk_ctx: a hash key bound to a HIP device.  ``tag_mode`` "md5" (default: the MD5
    compression per packet, as util/rhash.cpp:20-41 computes it) or "table" (the key's 256 tags
    looked up; identical outputs), see rsk_set_tag_mode."""

    def __init__(self, key: bytes = b"hello135", device: int = 0, tag_mode: str = "md5"):
        self.key = bytes(key)
        self.device = int(device)
        self._ctx = lib().rsk_create(self.key, len(self.key), self.device)
        if not self._ctx:
            raise RskError(f"rsk_create failed: {lib().rsk_last_error().decode()}")
        self.set_tag_mode(tag_mode)

    def set_tag_mode(self, mode) -> None:
        """rsk_set_tag_mode: "md5" / "table" (or the RSK_TAG_* value)."""
        m = TAG_MODES[mode] if isinstance(mode, str) else int(mode)
        _check(lib().rsk_set_tag_mode(self._ctx, m), "rsk_set_tag_mode")

    @property
    def tag_mode(self) -> str:
        m = lib().rsk_get_tag_mode(self._ctx)
        return {v: k for k, v in TAG_MODES.items()}.get(m, str(m))

    def close(self) -> None:
        if self._ctx:
            lib().rsk_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def set_encode_path(self, path: int) -> None:
        """rsk_set_encode_path for output_batch: 0 = chosen per call from the last sampled batch's mean
        payload (default), 1 = the per-set kernel k_encode, 2 = the two-pass form for long frames
        (k_encode_heads, then k_encode_copy: 1 / 2 / 4 packets per wave, set_copy_k), 3 = the short-frame
        kernel (k_encode with every set on the flat chunk list).  Every path gives identical bytes."""
        _check(lib().rsk_set_encode_path(self._ctx, path), "rsk_set_encode_path")

    @property
    def last_encode_path(self) -> int:
        """The path the last output_batch took (1 .. 3 as set_encode_path; 0 before any)."""
        fn = lib().rsk__last_encode_path
        fn.argtypes = [ctypes.c_void_p]
        return int(fn(self._ctx))

    @property
    def last_copy_k(self) -> int:
        """Packets per copy wave of the last two-pass output_batch (1, 2, 4; -1: the output-stationary copy;
        0 before any)."""
        fn = lib().rsk__last_copy_k
        fn.argtypes = [ctypes.c_void_p]
        return int(fn(self._ctx))

    def set_copy_k(self, k: int = 0) -> None:
        """Internal knob of the two-pass encode (rsk__set_copy_k): packets per copy wave (1, 2, 4), or -1 for the
        output-stationary copy (k_encode_os: waves own 1-KB blocks of the frame arena, for frames laid back to
        back); 0 = chosen from the last sampled statistic: output-stationary when the sampled frames lie back
        to back, else 4 below a mean payload of 880 B, 2 below 1160 B, 1 above (rsk_kernels.hip kAutoK*)."""
        fn = lib().rsk__set_copy_k
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _check(fn(self._ctx, k), "rsk__set_copy_k")

    def set_two_pass_chunk(self, packets: int = 0) -> None:
        """Internal knob of the two-pass encode (rsk__set_two_pass_chunk): header pass then copy per chunk
        of `packets` (0 = the whole batch)."""
        fn = lib().rsk__set_two_pass_chunk
        fn.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
        _check(fn(self._ctx, packets), "rsk__set_two_pass_chunk")

    def set_send_seq_groupby(self, v: int) -> None:
        """Internal knob for rsk_tcp_send_seq_batch: 0 the per-tile table path when n_conn < 2048
        (default), 1 the demux group-by path for every n_conn, 2 the table path with the one-kernel
        column scan (parity tests and A/B)."""
        fn = lib().rsk__set_send_seq_groupby
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        _check(fn(self._ctx, v), "rsk__set_send_seq_groupby")

    def check_device_errors(self) -> int:
        """rsk_check_device_errors: waits for the device, returns the sticky RSK_DEVERR_* flags (and
        clears them); raises RskError when any is set (that call's compaction / demux outputs were
        wrong; the look-back state is re-initialised at the next call)."""
        f = ctypes.c_uint32(0)
        rc = lib().rsk_check_device_errors(self._ctx, ctypes.byref(f))
        if rc != 0:
            raise RskError(f"device error flags 0x{f.value:x}: {lib().rsk_last_error().decode()}")
        return f.value

    def forget_captures(self) -> None:
        """rsk_forget_captures: the graphs that captured this context's calls are gone, so
        check_device_errors waits for the context's streams again, not the whole device."""
        _check(lib().rsk_forget_captures(self._ctx), "rsk_forget_captures")

    def release_stream(self, stream=None) -> None:
        """rsk_release_stream: wait for `stream` and free its scratch."""
        _check(lib().rsk_release_stream(self._ctx, _stream(stream)), "rsk_release_stream")

    def reserve(self, n_max: int, stream=None) -> None:
        """Pre-size the compaction scratch of `stream` (default: torch's current stream)."""
        _check(lib().rsk_reserve_stream(self._ctx, n_max, _stream(stream)), "rsk_reserve_stream")

    # ---- batch paths ---------------------------------------------------------------------
    def output_batch(self, payload, pay_off, pay_len, cmd, conv, conn_key, frame, frame_off, status,
                     id=None, id_uniform: bytes = b"\0" * 8, pad16: bool = False, pad128: bool = False,
                     stream=None) -> None:
        """RConn::Output framing for n packets (rsk_encode_batch).  pad16 / pad128 set
        RSK_ENC_ZERO_PAD16 / RSK_ENC_ZERO_PAD128."""
        n = pay_len.numel()
        ein = _abi.EncodeIn(_ptr(payload), _ptr(pay_off), _ptr(pay_len), _ptr(cmd), _ptr(conv),
                            _ptr(conn_key), _ptr(id),
                            (ctypes.c_uint8 * 8)(*bytes(id_uniform)[:8].ljust(8, b"\0")))
        eout = _abi.EncodeOut(_ptr(frame), _ptr(frame_off), _ptr(status),
                              (_abi.ENC_ZERO_PAD16 if pad16 else 0) | (_abi.ENC_ZERO_PAD128 if pad128 else 0))
        _check(lib().rsk_encode_batch(self._ctx, n, ctypes.byref(ein), ctypes.byref(eout),
                                      _stream(stream)), "rsk_encode_batch")

    def output_wire_batch(self, payload, pay_off, pay_len, cmd, conv, conn_key, src, dst, sp, dp, seq, ack, flag,
                          ip_id, wire, wire_off, status, eth: bytes | None = None, id=None,
                          id_uniform: bytes = b"\0" * 8, pad16: bool = False, pad128: bool = False,
                          stream=None) -> None:
        """RConn::Output + RawTcp::SendRawTcp (libnet IPv4/TCP build with checksums) for n packets
        (rsk_encode_wire_batch).  eth=None: LIBNET_RAW4 layout; else a 14-byte link header.  pad16 /
        pad128 set RSK_ENC_ZERO_PAD16 / RSK_ENC_ZERO_PAD128."""
        n = pay_len.numel()
        ein = _abi.EncodeIn(_ptr(payload), _ptr(pay_off), _ptr(pay_len), _ptr(cmd), _ptr(conv),
                            _ptr(conn_key), _ptr(id),
                            (ctypes.c_uint8 * 8)(*bytes(id_uniform)[:8].ljust(8, b"\0")))
        win = _abi.WireIn(_ptr(src), _ptr(dst), _ptr(sp), _ptr(dp), _ptr(seq), _ptr(ack), _ptr(flag), _ptr(ip_id),
                          (ctypes.c_uint8 * 14)(*(bytes(eth or b"")[:14].ljust(14, b"\0"))), 1 if eth else 0)
        eout = _abi.EncodeOut(_ptr(wire), _ptr(wire_off), _ptr(status),
                              (_abi.ENC_ZERO_PAD16 if pad16 else 0) | (_abi.ENC_ZERO_PAD128 if pad128 else 0))
        _check(lib().rsk_encode_wire_batch(self._ctx, n, ctypes.byref(ein), ctypes.byref(win), ctypes.byref(eout),
                                           _stream(stream)), "rsk_encode_wire_batch")

    def onrecv_batch(self, frame, frame_off, frame_len, out: DecodeBuffers, is_tcp_close=None,
                     compact: bool = True, stream=None) -> None:
        """RConn::OnRecv for n frames (rsk_decode_batch)."""
        n = frame_len.numel()
        dout = out.abi(compact)
        _check(lib().rsk_decode_batch(self._ctx, n, _ptr(frame), _ptr(frame_off), _ptr(frame_len),
                                      _ptr(is_tcp_close), ctypes.byref(dout), _stream(stream)),
               "rsk_decode_batch")

    def rawinput_batch(self, cap, cap_off, wire_len, cap_len, datalink: int, flags: int,
                       tcp: TcpInfoBuffers, out: DecodeBuffers, compact: bool = True,
                       stream=None) -> None:
        """RawTcp::RawInput -> cap2uv -> RConn::OnRecv for n captured packets."""
        n = wire_len.numel()
        tout = tcp.abi()
        dout = out.abi(compact)
        _check(lib().rsk_parse_decode_batch(self._ctx, n, _ptr(cap), _ptr(cap_off), _ptr(wire_len),
                                            _ptr(cap_len), datalink, flags, ctypes.byref(tout),
                                            ctypes.byref(dout), _stream(stream)),
               "rsk_parse_decode_batch")

    def syncinput_batch(self, rec, rec_off, nread, tcp: TcpInfoBuffers, out: DecodeBuffers, compact: bool = True,
                        stream=None) -> None:
        """RawTcp::syncInput -> TcpInfo::Decode -> RConn::OnRecv for n hand-off records (21-B TcpInfo
        + frame, nread[i] bytes at rec + rec_off[i])."""
        n = nread.numel()
        tout = tcp.abi()
        dout = out.abi(compact)
        _check(lib().rsk_syncinput_decode_batch(self._ctx, n, _ptr(rec), _ptr(rec_off), _ptr(nread),
                                                ctypes.byref(tout), ctypes.byref(dout), _stream(stream)),
               "rsk_syncinput_decode_batch")

    def rawinput_slots_batch(self, slots, slot: int, wire_len, cap_len, datalink: int, flags: int,
                             tcp: TcpInfoBuffers, out: DecodeBuffers, compact: bool = True, stream=None) -> None:
        """rawinput_batch on host-staged header slots (rsk_parse_decode_slots_batch): packet i's first
        min(cap_len, slot) bytes at slots[slot * i:]; RSK_PARSE_SLOT_SHORT marks packets to resubmit whole."""
        n = wire_len.numel()
        tout = tcp.abi()
        dout = out.abi(compact)
        _check(lib().rsk_parse_decode_slots_batch(self._ctx, n, _ptr(slots), slot, _ptr(wire_len), _ptr(cap_len),
                                                  datalink, flags, ctypes.byref(tout), ctypes.byref(dout),
                                                  _stream(stream)), "rsk_parse_decode_slots_batch")

    def tcp_send_seq_batch(self, conn, status, conn_seq, ip_id_next, seq, ip_id, stream=None) -> None:
        """FakeTcp::Output's seq advance + RawTcp::Output's mIpId++ for a batch sent in order
        (rsk_tcp_send_seq_batch); conn_seq / ip_id_next are device state updated in place."""
        n = conn.numel()
        _check(lib().rsk_tcp_send_seq_batch(self._ctx, n, _ptr(conn), _ptr(status), conn_seq.numel(), _ptr(conn_seq),
                                            _ptr(ip_id_next), _ptr(seq), _ptr(ip_id), _stream(stream)),
               "rsk_tcp_send_seq_batch")

    def tcp_recv_ack_batch(self, conn, delivered, seq, conn_ack, stream=None) -> None:
        """FakeTcp::OnRecv's ack update over a batch (rsk_tcp_recv_ack_batch)."""
        n = conn.numel()
        _check(lib().rsk_tcp_recv_ack_batch(self._ctx, n, _ptr(conn), _ptr(delivered), _ptr(seq), conn_ack.numel(),
                                            _ptr(conn_ack), _stream(stream)), "rsk_tcp_recv_ack_batch")

    def tcpinfo_encode_batch(self, src, dst, sp, dp, seq, ack, flag, rec, stream=None) -> None:
        n = src.numel()
        _check(lib().rsk_tcpinfo_encode_batch(self._ctx, n, _ptr(src), _ptr(dst), _ptr(sp), _ptr(dp),
                                              _ptr(seq), _ptr(ack), _ptr(flag), _ptr(rec),
                                              _stream(stream)), "rsk_tcpinfo_encode_batch")

    def output_headers_batch(self, first_byte, pay_len, cmd, conv, conn_key, hdr, status, id=None,
                             id_uniform: bytes = b"\0" * 8, stream=None) -> None:
        """Header-only RConn::Output (rsk_encode_headers_batch): hdr[32 i:32 i+32] = frame bytes [0, 32)."""
        n = pay_len.numel()
        ein = _abi.EncodeHdrIn(_ptr(first_byte), _ptr(pay_len), _ptr(cmd), _ptr(conv), _ptr(conn_key), _ptr(id),
                               (ctypes.c_uint8 * 8)(*bytes(id_uniform)[:8].ljust(8, b"\0")))
        _check(lib().rsk_encode_headers_batch(self._ctx, n, ctypes.byref(ein), _ptr(hdr), _ptr(status),
                                              _stream(stream)), "rsk_encode_headers_batch")

    def onrecv_headers_batch(self, hdr, frame_len, out: DecodeBuffers, is_tcp_close=None, stream=None) -> None:
        """Header-only RConn::OnRecv (rsk_decode_headers_batch) on 32-B slots (stage_decode_headers)."""
        n = frame_len.numel()
        _check(lib().rsk_decode_headers_batch(self._ctx, n, _ptr(hdr), _ptr(frame_len), _ptr(is_tcp_close),
                                              ctypes.byref(out.abi()), _stream(stream)),
               "rsk_decode_headers_batch")

    def filter_rawinput_batch(self, cap, cap_off, wire_len, cap_len, datalink: int, flags: int,
                              filt: "_abi.CaptureFilter", match, tcp: TcpInfoBuffers, out: DecodeBuffers,
                              compact: bool = True, stream=None) -> None:
        """Capture filter + RawTcp::RawInput + RConn::OnRecv in one pass (rsk_filter_parse_decode_batch)."""
        n = wire_len.numel()
        tout = tcp.abi()
        dout = out.abi(compact)
        _check(lib().rsk_filter_parse_decode_batch(self._ctx, n, _ptr(cap), _ptr(cap_off), _ptr(wire_len),
                                                   _ptr(cap_len), datalink, flags, ctypes.byref(filt), _ptr(match),
                                                   ctypes.byref(tout), ctypes.byref(dout), _stream(stream)),
               "rsk_filter_parse_decode_batch")

    def capture_filter_batch(self, cap, cap_off, cap_len, datalink: int, filt: "_abi.CaptureFilter", match,
                             match_idx=None, n_match=None, stream=None) -> None:
        """The capture filter RCap installs (rsk_capture_filter_batch) over a batch."""
        n = cap_off.numel()
        _check(lib().rsk_capture_filter_batch(self._ctx, n, _ptr(cap), _ptr(cap_off), _ptr(cap_len), datalink,
                                              ctypes.byref(filt), _ptr(match), _ptr(match_idx), _ptr(n_match),
                                              _stream(stream)), "rsk_capture_filter_batch")

    def demux_batch(self, status, cmd, fields: int, out: "DemuxBuffers", id=None, conv=None, conn_key=None,
                    dst=None, stream=None) -> None:
        """Stable group-by of the VALID packets on `fields` (rsk_demux_batch):
        segment s = out.perm[out.seg_off[s]:out.seg_off[s + 1]], keyed by packet out.seg_first[s]."""
        n = status.numel()
        din = _abi.DemuxIn(_ptr(status), _ptr(cmd), _ptr(id), _ptr(conv), _ptr(conn_key), _ptr(dst))
        _check(lib().rsk_demux_batch(self._ctx, n, ctypes.byref(din), fields, ctypes.byref(out.abi()),
                                     _stream(stream)), "rsk_demux_batch")

    # ---- reference single-call signatures (GPU round trip each) -----------------------------
    def compute_hash(self, data: bytes) -> bytes | None:
        tag = ctypes.create_string_buffer(8)
        r = lib().rsk_compute_hash(self._ctx, tag, bytes(data), len(data))
        return tag.raw if r else None

    def hash_equal(self, tag: bytes, data: bytes) -> bool:
        return bool(lib().rsk_hash_equal(self._ctx, bytes(tag), bytes(data), len(data)))

    def enc2buf(self, cmd: int, id: bytes, conv: int, conn_key: int, buf_len: int = 1492) -> bytes | None:
        buf = ctypes.create_string_buffer(max(buf_len, 23))
        r = lib().rsk_enchead_enc2buf(self._ctx, buf, buf_len, cmd, bytes(id)[:8].ljust(8, b"\0"),
                                      conv & 0xFFFFFFFF, conn_key & 0xFFFFFFFFFFFFFFFF)
        return buf.raw[:23] if r else None

    def decodebuf(self, buf: bytes, buf_len: int | None = None):
        """-> (len, cmd, id, conv, conn_key) or None (EncHead::DecodeBuf returned nullptr)."""
        if buf_len is None:
            buf_len = len(buf)
        b = bytes(buf).ljust(23, b"\0")
        ln, cmd = ctypes.c_uint8(), ctypes.c_uint8()
        idb = ctypes.create_string_buffer(8)
        conv, key = ctypes.c_uint32(), ctypes.c_uint64()
        r = lib().rsk_enchead_decodebuf(self._ctx, b, buf_len, ctypes.byref(ln), ctypes.byref(cmd),
                                        idb, ctypes.byref(conv), ctypes.byref(key))
        if not r:
            return None
        return ln.value, cmd.value, idb.raw, conv.value, key.value


def key_for_tcp(sp: int, dp: int) -> int:
    return lib().rsk_key_for_tcp(sp, dp)


def key_for_udp(sp: int, dp: int) -> int:
    return lib().rsk_key_for_udp(sp, dp)


def fill_splitmix(t: torch.Tensor, seed: int, stream=None) -> None:
    _check(lib().rsk_fill_splitmix(_ptr(t), t.numel() * t.element_size(), seed & (2**64 - 1),
                                   _stream(stream)), "rsk_fill_splitmix")
