"""Synthetic packet workloads of SURVEY.md §8d (configs C2-C5), SoA-laid-out for the codec.

Every random quantity comes from a splitmix64 stream (seed = config index XOR 0x5EED), so a host
(numpy) build and a device build of the same config are byte-identical:
  * per-packet descriptor words: r[4i .. 4i+3] of stream ``seed``
  * payload bytes: the byte stream of splitmix64 seeded ``seed ^ PAYLOAD_SALT`` over the arena

HBM layout: payload slots at a 16-B pitch >= P_max, frame slots at a 16-B pitch
>= 31 + P_max, so every frame starts 16-B aligned and the encode kernel takes its vector path.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

ID_UNIFORM = b"abcdefgh"  # IdBuf used by the SURVEY's verified frame (§8c)
PAYLOAD_SALT = 0xA5A5_5A5A_0F0F_F0F0
HEAD = 31

CONFIGS = {
    # name: (index, n, pmin, pmax, ports, mixed_cmd, corrupt_every)
    "c2": (2, 1 << 20, 64, 64, 1, False, 0),
    "c3": (3, 4 << 20, 1400, 1400, 1, False, 0),
    "c4": (4, 1 << 20, 64, 1400, 10, True, 16),
    "c5": (5, 64 << 20, 1400, 1400, 1, False, 0),
}


def seed_of(name: str) -> int:
    return CONFIGS[name][0] ^ 0x5EED


_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64_np(seed: int, start: int, count: int) -> np.ndarray:
    """Outputs start..start+count-1 of splitmix64 seeded `seed` (numpy uint64, wraps mod 2^64)."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def splitmix_bytes_np(seed: int, nbytes: int, start_byte: int = 0) -> np.ndarray:
    w0 = start_byte // 8
    w1 = (start_byte + nbytes + 7) // 8
    words = splitmix64_np(seed, w0, w1 - w0)
    b = words.view(np.uint8)
    off = start_byte - 8 * w0
    return b[off:off + nbytes].copy()


def round16(x: int) -> int:
    return (x + 15) & ~15


def round128(x: int) -> int:
    return (x + 127) & ~127


@dataclass
class Descriptors:
    """Host SoA descriptors for packets [lo, hi) of a config."""

    n: int
    pay_off: np.ndarray  # uint64 (offsets relative to the shard's payload arena)
    pay_len: np.ndarray  # uint16
    cmd: np.ndarray  # uint8
    conv: np.ndarray  # uint32
    conn_key: np.ndarray  # uint64
    frame_off: np.ndarray  # uint64
    frame_len: np.ndarray  # uint16 (31 + P, the encoded length)
    corrupt: np.ndarray  # bool: flip a tag bit before decode
    pay_pitch: int
    frame_pitch: int
    pad: int  # zero-pad granularity the slots allow: 128 (line-aligned slots) or 16
    payload_seed: int
    first: int  # global index of packet 0 of this shard


def describe(name: str, lo: int = 0, hi: int | None = None, n: int | None = None,
             frame_pitch: int | None = None) -> Descriptors:
    """Descriptors of packets [lo, hi) of config `name` (n overrides the config's packet count;
    frame_pitch overrides the frame slot pitch, a multiple of 16 >= 31 + P_max)."""
    idx, n_cfg, pmin, pmax, ports, mixed, corrupt_every = CONFIGS[name]
    n_total = n_cfg if n is None else n
    if hi is None:
        hi = n_total
    cnt = hi - lo
    seed = seed_of(name)
    r = splitmix64_np(seed, 4 * lo, 4 * cnt).reshape(cnt, 4)
    gi = np.arange(lo, hi, dtype=np.uint64)
    conv = (r[:, 0] & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    sp = (np.uint64(32768) + r[:, 1] % np.uint64(28232)).astype(np.uint64)
    dp = (np.uint64(10001) + gi % np.uint64(ports)).astype(np.uint64)
    conn_key = np.uint64(0x10000000) | (dp << np.uint64(16)) | sp  # KeyGenerator::KeyForTcp
    if mixed:
        u = r[:, 2] % np.uint64(100)
        alt = (np.uint64(1) + (r[:, 2] >> np.uint64(32)) % np.uint64(4)).astype(np.uint8)
        cmd = np.where(u < 95, np.uint8(0), alt).astype(np.uint8)
    else:
        cmd = np.zeros(cnt, np.uint8)
    if pmin == pmax:
        plen = np.full(cnt, pmin, np.uint16)
    else:
        plen = (np.uint64(pmin) + r[:, 3] % np.uint64(pmax - pmin + 1)).astype(np.uint16)
    # control bodies: conv reset carries a 4-byte conv, the others an 8-byte key
    plen = np.where(cmd == 1, np.uint16(4), np.where(cmd >= 2, np.uint16(8), plen)).astype(np.uint16)
    pay_pitch = round16(pmax)
    # Frame slots: frames of one length tile densely at 16-B granularity (every line is written
    # whole by neighbouring frames); frames of mixed lengths get 128-B-aligned slots, zero-padded to
    # the line (RSK_ENC_ZERO_PAD128), so no frame leaves a partly written line behind.
    if frame_pitch is None:
        frame_pitch = round16(HEAD + pmax) if pmin == pmax else round128(HEAD + pmax)
    frame_pitch = int(frame_pitch)
    assert frame_pitch % 16 == 0 and frame_pitch >= HEAD + pmax
    local = np.arange(cnt, dtype=np.uint64)
    corrupt = (gi % np.uint64(corrupt_every) == np.uint64(7)) if corrupt_every else np.zeros(cnt, bool)
    return Descriptors(
        n=cnt,
        pay_off=local * np.uint64(pay_pitch),
        pay_len=plen,
        cmd=cmd,
        conv=conv,
        conn_key=conn_key.astype(np.uint64),
        frame_off=local * np.uint64(frame_pitch),
        frame_len=(plen.astype(np.uint32) + HEAD).astype(np.uint16),
        corrupt=corrupt,
        pay_pitch=pay_pitch,
        frame_pitch=frame_pitch,
        pad=128 if frame_pitch % 128 == 0 else 16,
        payload_seed=(seed ^ PAYLOAD_SALT) & 0xFFFFFFFFFFFFFFFF,
        first=lo,
    )


def payload_bytes_np(d: Descriptors) -> np.ndarray:
    """Host payload arena of a shard: the payload byte stream at this shard's arena offset."""
    return splitmix_bytes_np(d.payload_seed, d.n * d.pay_pitch, d.first * d.pay_pitch)


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous shard [lo, hi) of n packets for `rank` of `world`."""
    return (n * rank) // world, (n * (rank + 1)) // world


# ---------------------------------------------------------------------------------------------
# Device (torch) materialisation
# ---------------------------------------------------------------------------------------------
class DeviceWorkload:
    """A shard of a config resident in HBM: inputs, frame arena and decode outputs."""

    def __init__(self, d: Descriptors, device, stream=None):
        import torch

        from . import codec

        self.d = d
        self.device = device
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(device)  # noqa: E731
        self.pay_off = t(d.pay_off, np.int64)
        self.pay_len = t(d.pay_len, np.int16)
        self.cmd = t(d.cmd, np.uint8)
        self.conv = t(d.conv, np.int32)
        self.conn_key = t(d.conn_key, np.int64)
        self.frame_off = t(d.frame_off, np.int64)
        self.frame_len = t(d.frame_len, np.int16)
        self.corrupt_idx = torch.from_numpy(np.nonzero(d.corrupt)[0].astype(np.int64)).to(device)
        self.payload = torch.empty(d.n * d.pay_pitch, dtype=torch.uint8, device=device)
        # the stream of this shard starts at byte first*pay_pitch: fill whole words from the
        # word-aligned start (pitch is a multiple of 16, so the start is word-aligned)
        assert (d.first * d.pay_pitch) % 8 == 0
        self._fill_payload(codec, stream)
        self.frame = torch.zeros(d.n * d.frame_pitch, dtype=torch.uint8, device=device)
        self.status = torch.empty(d.n, dtype=torch.int32, device=device)
        self.dec = codec.DecodeBuffers.alloc(d.n, device)

    def _fill_payload(self, codec, stream):
        # word w of the arena is splitmix word (first*pitch/8 + w): generate via seed offset.
        # splitmix output i for seed s equals output 0.. of seed s + i*gamma, so shift the seed.
        d = self.d
        w0 = (d.first * d.pay_pitch) // 8
        seed = (d.payload_seed + w0 * 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        codec.fill_splitmix(self.payload, seed, stream)

    def corrupt_frames(self):
        """Flip bit 0 of the tag of the frames the config marks corrupted (C4: 1 in 16)."""
        if self.corrupt_idx.numel():
            pos = self.frame_off[self.corrupt_idx]
            self.frame[pos] ^= 1
