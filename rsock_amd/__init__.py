"""rsock_amd — MI355X-native framing codec for rsock (EncHead + MD5 hash-tag, pcap parse).

The codec runs in hand-written HIP kernels (``rsock_amd/csrc``) behind the C ABI declared in
``include/rsk_codec.h``; this package is the Python host mirror used by tests and bench.py.
"""
from ._abi import (  # noqa: F401
    CMD_CONV_RST, CMD_DATA, CMD_KEEP_ALIVE_REQ, CMD_KEEP_ALIVE_RESP, CMD_NETCONN_RST, DLT_EN10MB,
    DLT_NULL, ENC_HEAD_SIZE, HASH_BUF_SIZE, HEAD_SIZE, MAX_PAYLOAD, MAX_PKT_SIZE, PARSE_DELIVER,
    PARSE_DROP, PARSE_HAS_ACK_POOL, PARSE_IS_SERVER, PARSE_MALFORMED, PARSE_SYN, RECV_CLOSE,
    RECV_DROP, RECV_VALID, SEND_OVERSIZE, SEND_RESET, TCPINFO_WIRE_SIZE, TH_ACK, TH_FIN, TH_PUSH,
    TH_RST, TH_SYN,
)

__version__ = "0.1.0"


def __getattr__(name):
    # Lazy: importing the package must not require the GPU library (CPU tests import constants).
    if name in ("Codec", "DecodeBuffers", "TcpInfoBuffers", "RskError", "key_for_tcp", "key_for_udp",
                "fill_splitmix", "lib"):
        from . import codec

        return getattr(codec, name)
    raise AttributeError(name)
