"""ctypes mirror of include/rsk_codec.h.

Loads the in-tree ``rsock_amd/librsk.so`` (built by ``__graft_entry__.build()`` /
``make -C rsock_amd``).  There is no fallback: if the library is missing or fails to load, importing
this module raises, so nothing can silently run a non-HIP path.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# RSK_LIB selects another in-tree build of the same library (tools: a saved copy of an earlier build,
# for an A/B between builds in separate processes)
LIB_PATH = os.path.join(_HERE, os.environ.get("RSK_LIB", "librsk.so"))

# ---- constants (include/rsk_codec.h) ------------------------------------------------------------
HASH_BUF_SIZE = 8
ID_BUF_SIZE = 8
ENC_HEAD_SIZE = 23
HEAD_SIZE = 31
MAX_PKT_SIZE = 1500
MAX_PAYLOAD = MAX_PKT_SIZE - HEAD_SIZE
TCPINFO_WIRE_SIZE = 21

CMD_DATA, CMD_CONV_RST, CMD_NETCONN_RST, CMD_KEEP_ALIVE_REQ, CMD_KEEP_ALIVE_RESP = 0, 1, 2, 3, 4
TH_FIN, TH_SYN, TH_RST, TH_PUSH, TH_ACK = 0x01, 0x02, 0x04, 0x08, 0x10
DLT_NULL, DLT_EN10MB = 0, 1

OK, EINVAL, ENOMEM, EDEVICE = 0, -22, -12, -5
SEND_OVERSIZE, SEND_RESET = -1, 0
MAX_BATCH = 0xFFFF0000
RECV_VALID, RECV_CLOSE, RECV_DROP = 1, 0, -1
PARSE_DROP, PARSE_DELIVER, PARSE_SYN, PARSE_MALFORMED, PARSE_SLOT_SHORT = 0, 1, 2, 3, 4
CAP_SLOT_MIN = 64
PARSE_HAS_ACK_POOL, PARSE_IS_SERVER = 0x1, 0x2
FILTER_MAX_PORTS = 64
TAG_MD5, TAG_TABLE = 0, 1
DEVERR_LOOKBACK = 0x1
DEVERR_TABLE = 0x2
DEMUX_ID, DEMUX_CONN_KEY, DEMUX_CONV, DEMUX_DST, DEMUX_CMD_BARRIER = 0x01, 0x02, 0x04, 0x08, 0x10
DEMUX_GROUP_BARRIER = 0x20

_vp = ctypes.c_void_p
_u8p = ctypes.c_void_p  # all arrays passed as raw addresses


class EncodeIn(ctypes.Structure):
    _fields_ = [
        ("payload_arena", _vp),
        ("pay_off", _vp),
        ("pay_len", _vp),
        ("cmd", _vp),
        ("conv", _vp),
        ("conn_key", _vp),
        ("id", _vp),
        ("id_uniform", ctypes.c_uint8 * 8),
    ]


class EncodeOut(ctypes.Structure):
    _fields_ = [("frame_arena", _vp), ("frame_off", _vp), ("status", _vp), ("flags", ctypes.c_uint32)]


ENC_ZERO_PAD16 = 0x1
ENC_ZERO_PAD128 = 0x2
ENC_PATH_AUTO, ENC_PATH_PER_SET, ENC_PATH_TWO_PASS, ENC_PATH_SHORT = 0, 1, 2, 3


class WireIn(ctypes.Structure):
    _fields_ = [
        ("src", _vp), ("dst", _vp), ("sp", _vp), ("dp", _vp), ("seq", _vp), ("ack", _vp), ("flag", _vp),
        ("ip_id", _vp), ("eth", ctypes.c_uint8 * 14), ("with_eth", ctypes.c_uint8),
    ]


class DecodeOut(ctypes.Structure):
    _fields_ = [
        ("hlen", _vp),
        ("cmd", _vp),
        ("id", _vp),
        ("conv", _vp),
        ("conn_key", _vp),
        ("pay_off", _vp),
        ("pay_len", _vp),
        ("status", _vp),
        ("valid_idx", _vp),
        ("n_valid", _vp),
    ]


class TcpInfoOut(ctypes.Structure):
    _fields_ = [
        ("src", _vp),
        ("dst", _vp),
        ("sp", _vp),
        ("dp", _vp),
        ("seq", _vp),
        ("ack", _vp),
        ("flag", _vp),
        ("parse_status", _vp),
        ("cap_pay_off", _vp),
        ("cap_pay_len", _vp),
    ]


class EncodeHdrIn(ctypes.Structure):
    _fields_ = [("first_byte", _vp), ("pay_len", _vp), ("cmd", _vp), ("conv", _vp), ("conn_key", _vp), ("id", _vp),
                ("id_uniform", ctypes.c_uint8 * 8)]


class DemuxIn(ctypes.Structure):
    _fields_ = [("status", _vp), ("cmd", _vp), ("id", _vp), ("conv", _vp), ("conn_key", _vp), ("dst", _vp)]


class DemuxOut(ctypes.Structure):
    _fields_ = [("perm", _vp), ("seg_off", _vp), ("seg_first", _vp), ("n_seg", _vp), ("n_valid", _vp)]


class PortList(ctypes.Structure):
    _fields_ = [("n_single", ctypes.c_uint16), ("n_range", ctypes.c_uint16),
                ("single", ctypes.c_uint16 * FILTER_MAX_PORTS), ("range", (ctypes.c_uint16 * 2) * FILTER_MAX_PORTS)]


class CaptureFilter(ctypes.Structure):
    _fields_ = [("src_ip", ctypes.c_uint32), ("dst_ip", ctypes.c_uint32), ("has_src_ip", ctypes.c_uint8),
                ("has_dst_ip", ctypes.c_uint8), ("is_server", ctypes.c_uint8), ("reserved", ctypes.c_uint8),
                ("src_ports", PortList), ("dst_ports", PortList)]


# (name, restype, argtypes) for every symbol the header declares
SIGNATURES = [
    ("rsk_create", _vp, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int]),
    ("rsk_destroy", None, [_vp]),
    ("rsk_set_tag_mode", ctypes.c_int, [_vp, ctypes.c_int]),
    ("rsk_get_tag_mode", ctypes.c_int, [_vp]),
    ("rsk_set_encode_path", ctypes.c_int, [_vp, ctypes.c_int]),
    ("rsk_reserve", ctypes.c_int, [_vp, ctypes.c_uint32]),
    ("rsk_reserve_stream", ctypes.c_int, [_vp, ctypes.c_uint32, _vp]),
    ("rsk_release_stream", ctypes.c_int, [_vp, _vp]),
    ("rsk_check_device_errors", ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint32)]),
    ("rsk_forget_captures", ctypes.c_int, [_vp]),
    ("rsk_last_error", ctypes.c_char_p, []),
    ("rsk_version", ctypes.c_char_p, []),
    ("rsk_encode_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, ctypes.POINTER(EncodeIn), ctypes.POINTER(EncodeOut), _vp]),
    ("rsk_encode_wire_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, ctypes.POINTER(EncodeIn), ctypes.POINTER(WireIn), ctypes.POINTER(EncodeOut), _vp]),
    ("rsk_encode_headers_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, ctypes.POINTER(EncodeHdrIn), _vp, _vp, _vp]),
    ("rsk_decode_headers_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.POINTER(DecodeOut), _vp]),
    ("rsk_stage_decode_header", None, [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p]),
    ("rsk_stage_decode_headers", ctypes.c_int, [ctypes.c_uint32, _vp, _vp, _vp, _vp, ctypes.c_int]),
    ("rsk_assemble_frames", ctypes.c_int, [ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int]),
    ("rsk_decode_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, ctypes.POINTER(DecodeOut), _vp]),
    ("rsk_parse_decode_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int,
      ctypes.POINTER(TcpInfoOut), ctypes.POINTER(DecodeOut), _vp]),
    ("rsk_parse_decode_slots_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp, _vp, ctypes.c_int, ctypes.c_int,
      ctypes.POINTER(TcpInfoOut), ctypes.POINTER(DecodeOut), _vp]),
    ("rsk_stage_capture_slots", ctypes.c_int, [ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_uint32, _vp, ctypes.c_int]),
    ("rsk_tcpinfo_encode_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("rsk_syncinput_decode_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.POINTER(TcpInfoOut), ctypes.POINTER(DecodeOut), _vp]),
    ("rsk_capture_filter_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_int, ctypes.POINTER(CaptureFilter), _vp, _vp, _vp, _vp]),
    ("rsk_filter_str", ctypes.c_int, [ctypes.POINTER(CaptureFilter), ctypes.c_char_p, ctypes.c_size_t]),
    ("rsk_filter_parse_decode_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(CaptureFilter), _vp,
      ctypes.POINTER(TcpInfoOut), ctypes.POINTER(DecodeOut), _vp]),
    ("rsk_tcp_send_seq_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, _vp, _vp, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp]),
    ("rsk_tcp_recv_ack_batch", ctypes.c_int, [_vp, ctypes.c_uint32, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp]),
    ("rsk_demux_batch", ctypes.c_int,
     [_vp, ctypes.c_uint32, ctypes.POINTER(DemuxIn), ctypes.c_uint32, ctypes.POINTER(DemuxOut), _vp]),
    ("rsk_compute_hash", _vp, [_vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]),
    ("rsk_hash_equal", ctypes.c_int, [_vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int]),
    ("rsk_enchead_enc2buf", _vp,
     [_vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32,
      ctypes.c_uint64]),
    ("rsk_enchead_decodebuf", _vp,
     [_vp, ctypes.c_char_p, ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    ("rsk_key_for_tcp", ctypes.c_uint64, [ctypes.c_uint16, ctypes.c_uint16]),
    ("rsk_key_for_udp", ctypes.c_uint64, [ctypes.c_uint16, ctypes.c_uint16]),
    ("rsk_fill_splitmix", ctypes.c_int, [_vp, ctypes.c_uint64, ctypes.c_uint64, _vp]),
    # include/rsk_rconn.h (RConn-shaped batching adapter)
    ("rsk_rconn_create", _vp, [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint32]),
    ("rsk_rconn_destroy", None, [_vp]),
    ("rsk_rconn_set_callbacks", None, [_vp, _vp, _vp, _vp, _vp]),
    ("rsk_rconn_output", ctypes.c_int,
     [_vp, ctypes.c_int64, ctypes.c_char_p, ctypes.c_uint8, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint64, _vp]),
    ("rsk_rconn_onrecv", ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_char_p, ctypes.c_int, _vp]),
    ("rsk_rconn_flush", ctypes.c_int, [_vp]),
    ("rsk_rconn_callback_failures", ctypes.c_uint64, [_vp]),
]

SEND_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
RESET_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)
RECV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_int, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_void_p, ctypes.c_uint32,
                           ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p)


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    if not os.path.exists(path):
        raise ImportError(
            f"rsock_amd: HIP library {path} not built; run `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(path)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)  # AttributeError here = header/library mismatch
        fn.restype = res
        fn.argtypes = args
    return lib


def header_symbols(header_paths: list[str] | None = None) -> list[str]:
    """Names of every function declared in include/rsk_codec.h and include/rsk_rconn.h."""
    import re

    if header_paths is None:
        inc = os.path.join(os.path.dirname(_HERE), "include")
        header_paths = [os.path.join(inc, "rsk_codec.h"), os.path.join(inc, "rsk_rconn.h")]
    names = set()
    for hp in header_paths:
        text = re.sub(r"/\*.*?\*/", "", open(hp).read(), flags=re.S)
        text = re.sub(r"typedef[^;]*;", "", text)  # callback typedefs are not exported symbols
        names |= set(re.findall(r"\b(rsk_[a-z0-9_]+)\s*\(", text))
    return sorted(names)
