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


def rand_capture(rng, datalink: int, ports=(10001, 10002, 10003, 443, 53, 40000, 40001),
                 ips=("10.0.0.1", "10.0.0.2", "192.168.1.7"), sports=None, dports=None, srcs=None,
                 dsts=None) -> tuple[bytes, int]:
    """A random captured packet for capture-filter tests: IPv4 TCP/UDP/SCTP/ICMP with fragment
    offsets and IHL variants (incl. invalid IHL < 5), IPv6 TCP/UDP (direct or behind a fragment
    header), ARP / VLAN frames, DLT_NULL families 2/24/28/30/10; returns (bytes, cap_len) with
    cap_len sometimes cutting the packet short."""
    sp, dp = (int(rng.choice(pool or ports)) if rng.random() < 0.7 else int(rng.integers(1, 65536))
              for pool in (sports, dports))
    src, dst = (str(rng.choice(pool or ips)) for pool in (srcs, dsts))
    flags = int(rng.choice([0x02, 0x12, 0x10, 0x18, 0x11, 0x04]))
    kind = rng.random()
    if kind < 0.6:  # IPv4
        proto = int(rng.choice([6, 6, 6, 17, 132, 1]))
        ihl = int(rng.choice([5, 5, 5, 6, 15, 3]))
        body = ipv4_tcp(src, sp, dst, dp, int(rng.integers(0, 2**32)), 0, flags, bytes(rng.integers(0, 256, 12,
                        dtype=np.uint8)), ihl_words=max(ihl, 5), proto=proto, datalink=datalink)
        L = 14 if datalink == 1 else 4
        b = bytearray(body)
        if ihl < 5:  # malformed IHL: the header says 3 words, ports are read there
            b[L] = 0x40 | ihl
        if rng.random() < 0.15:  # fragment offset / MF
            fo = int(rng.choice([0x2000, 0x0001, 0x00B9]))
            b[L + 6:L + 8] = struct.pack("!H", fo)
        pkt = bytes(b)
    elif kind < 0.85:  # IPv6
        nxt = int(rng.choice([6, 6, 17, 44, 44, 58]))
        inner = int(rng.choice([6, 17])) if nxt == 44 else nxt
        tr = struct.pack("!HHIIBBHHH", sp, dp, 1, 2, 0x50, flags, 65535, 0, 0)
        ext = struct.pack("!BBHI", inner, 0, 0, 7) if nxt == 44 else b""
        ip6 = struct.pack("!IHBB", 0x60000000, len(ext) + len(tr), nxt, 64) + bytes(16) + bytes(16)
        if datalink == 1:
            link = b"\x02" * 6 + b"\x04" * 6 + struct.pack("!H", 0x86DD)
        else:
            link = struct.pack("<I", int(rng.choice([24, 28, 30, 10])))
        pkt = link + ip6 + ext + tr + b"xyz"
    else:  # not IP: ARP / VLAN-tagged IPv4 / other families
        if datalink == 1:
            et = int(rng.choice([0x0806, 0x8100, 0x88CC]))
            pkt = b"\x02" * 6 + b"\x04" * 6 + struct.pack("!H", et) + bytes(rng.integers(0, 256, 60, dtype=np.uint8))
        else:
            pkt = struct.pack("<I", int(rng.choice([0, 7, 17]))) + bytes(rng.integers(0, 256, 60, dtype=np.uint8))
    cl = len(pkt)
    if rng.random() < 0.15:
        cl = int(rng.integers(0, len(pkt) + 1))
    return pkt, cl
