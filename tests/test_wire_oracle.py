"""CPU: the wire-build oracle (RawTcp::SendRawTcp via libnet, conn/RawTcp.cpp:280-341) against an
independent Python restatement of RFC 791 / RFC 793 / RFC 1071.  libnet 1.1.6 exists only as the
reference's prebuilt .a, which is never run, so this row is pinned to the RFCs."""
from __future__ import annotations

import socket
import struct

import numpy as np
import pytest


def py_csum(b: bytes) -> int:
    if len(b) % 2:
        b += b"\0"
    s = sum(struct.unpack("!%dH" % (len(b) // 2), b))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return ~s & 0xFFFF


def py_wire(frame, src, dst, sp, dp, seq, ack, flag, ip_id, eth=None):
    tot = 40 + len(frame)
    sb, db = struct.pack("<I", src), struct.pack("<I", dst)  # stored network-order words
    ip = struct.pack("!BBHHHBBH4s4s", 0x45, 0, tot, ip_id, 0x4000, 64, 6, 0, sb, db)
    ip = ip[:10] + struct.pack("!H", py_csum(ip)) + ip[12:]
    tcp = struct.pack("!HHIIBBHHH", sp, dp, seq, ack, 0x50, flag, 65535, 0, 0)
    pseudo = sb + db + struct.pack("!BBH", 0, 6, 20 + len(frame))
    ck = py_csum(pseudo + tcp + frame)
    tcp = tcp[:16] + struct.pack("!H", ck) + tcp[18:]
    return (eth or b"") + ip + tcp + frame


def test_wire_oracle_matches_rfc_restatement(oracle):
    rng = np.random.default_rng(4)
    for k in range(300):
        frame = rng.integers(0, 256, int(rng.integers(0, 1501)), dtype=np.uint8).tobytes()
        f = (int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)), int(rng.integers(0, 65536)),
             int(rng.integers(0, 65536)), int(rng.integers(0, 2**32)), int(rng.integers(0, 2**32)),
             int(rng.integers(0, 256)), int(rng.integers(0, 65536)))
        eth = rng.integers(0, 256, 14, dtype=np.uint8).tobytes() if k % 2 else None
        assert oracle.build_wire(frame, *f, eth=eth) == py_wire(frame, *f, eth=eth)


def test_wire_known_layout(oracle):
    """The SURVEY's loopback frame shape: 10.0.0.1:10001 -> 10.0.0.2:43932 (stored words), 95-B frame."""
    src = struct.unpack("<I", socket.inet_aton("10.0.0.1"))[0]
    dst = struct.unpack("<I", socket.inet_aton("10.0.0.2"))[0]
    w = oracle.build_wire(bytes(95), src, dst, 10001, 43932, 256, 512, 0x10, 7)
    assert len(w) == 135 and w[:2] == b"\x45\x00" and w[2:4] == struct.pack("!H", 135)
    assert w[6:10] == b"\x40\x00\x40\x06" and w[12:16] == socket.inet_aton("10.0.0.1")
    assert w[32:36] == b"\x50\x10\xff\xff" and py_csum(w[:20]) == 0
