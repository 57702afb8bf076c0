"""Crafting eth/IPv4/TCP capture records for parse tests (RFC 791 / RFC 793 layouts)."""
from __future__ import annotations

import struct

import numpy as np


def ipv4_tcp(src: str, sport: int, dst: str, dport: int, seq: int, ack: int, flags: int, payload: bytes,
             ihl_words: int = 5, thl_words: int = 5, proto: int = 6, ip_len: int | None = None,
             datalink: int = 1, ethertype: int = 0x0800, null_family: int = 2) -> bytes:
    """One captured packet: link header + IPv4 (ihl_words*4 B) + TCP (thl_words*4 B) + payload."""
    ip_opts = b"\x01" * (ihl_words * 4 - 20)
    tcp_opts = b"\x01" * (thl_words * 4 - 20)
    tot = ihl_words * 4 + thl_words * 4 + len(payload) if ip_len is None else ip_len
    sb = bytes(int(x) for x in src.split("."))
    db = bytes(int(x) for x in dst.split("."))
    ip = struct.pack("!BBHHHBBH4s4s", 0x40 | ihl_words, 0, tot & 0xFFFF, 0x1234, 0x4000, 64, proto, 0, sb, db)
    tcp = struct.pack("!HHIIBBHHH", sport, dport, seq & 0xFFFFFFFF, ack & 0xFFFFFFFF, thl_words << 4, flags,
                      65535, 0, 0)
    if datalink == 1:
        link = b"\x02" * 6 + b"\x04" * 6 + struct.pack("!H", ethertype)
    else:
        link = struct.pack("<I", null_family)
    return link + ip + ip_opts + tcp + tcp_opts + payload


def pack_records(pkts: list[bytes], align: int = 1, base_pad: int = 0):
    """Concatenate packets into one arena; returns (arena uint8, offsets uint64, lengths uint32)."""
    offs, cur = [], base_pad
    for p in pkts:
        cur = (cur + align - 1) // align * align
        offs.append(cur)
        cur += len(p)
    arena = np.zeros(cur + 64, np.uint8)
    for o, p in zip(offs, pkts):
        arena[o:o + len(p)] = np.frombuffer(p, np.uint8)
    return arena, np.array(offs, np.uint64), np.array([len(p) for p in pkts], np.uint32)
