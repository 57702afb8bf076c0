"""GPU: rsk_capture_filter_batch against the oracle packet by packet: random
captures (IPv4 / IPv6 / non-IP, fragments, IHL variants, truncation) at unaligned offsets for
random client and server filters on both link types, the order-stable match list, the wire packets
of rsk_encode_wire_batch through a client and a server filter, and argument errors."""
from __future__ import annotations

import numpy as np
import pytest

from rsock_amd import codec as rc
from rsock_amd import workload
from tests.pkt import pack_records, rand_capture
from tests.test_filter_oracle import pools_for, rand_filter_args

pytestmark = pytest.mark.gpu


def run_gpu(codec, gpu, arena, offs, lens, dl, f):
    import torch

    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt)).to(gpu)  # noqa: E731
    n = len(offs)
    match = torch.empty(n, dtype=torch.uint8, device=gpu)
    midx = torch.empty(max(n, 1), dtype=torch.int32, device=gpu)
    nm = torch.empty(1, dtype=torch.int32, device=gpu)
    codec.capture_filter_batch(t(arena, np.uint8), t(offs, np.int64), t(lens, np.int32), dl, f, match, midx, nm)
    torch.cuda.synchronize()
    k = int(nm.item())
    return match.cpu().numpy(), midx[:k].cpu().numpy().astype(np.uint32)


@pytest.mark.parametrize("dl", [0, 1])
@pytest.mark.parametrize("seed", range(10))
def test_filter_random(codec, gpu, oracle, dl, seed):
    rng = np.random.default_rng(777 + 31 * seed + dl)
    a = rand_filter_args(rng)
    f = rc.make_filter(**a)
    pools = pools_for(a, rng)
    caps = [rand_capture(rng, dl, **pools) for _ in range(3000)]
    arena, offs, _ = pack_records([p for p, _ in caps], align=1, base_pad=int(rng.integers(0, 8)))
    lens = np.array([cl for _, cl in caps], np.uint32)
    match, midx = run_gpu(codec, gpu, arena, offs, lens, dl, f)
    exp = np.array([oracle.capture_filter(p, dl, f, cap_len=cl) for p, cl in caps], np.uint8)
    assert exp.sum() > 0
    bad = np.nonzero(match != exp)[0]
    assert bad.size == 0, [(int(i), caps[i][0].hex(), caps[i][1]) for i in bad[:3]]
    assert np.array_equal(midx, np.nonzero(exp)[0].astype(np.uint32))


def test_filter_wire_packets(codec, gpu, oracle):
    """Ethernet packets built by rsk_encode_wire_batch (dst 10.0.0.2, dport 10001..10010, ACK|PSH)
    pass the client filter for that address/port set and the server filter's non-SYN branch."""
    import torch

    n = 5000
    d = workload.describe("c4", 0, n, n=n)
    w = workload.DeviceWorkload(d, gpu)
    src = torch.full((n,), rc.ip_u32("10.0.0.1"), dtype=torch.int64, device=gpu).to(torch.int32)
    dst = torch.full((n,), rc.ip_u32("10.0.0.2"), dtype=torch.int64, device=gpu).to(torch.int32)
    sp = torch.full((n,), 43000, dtype=torch.int32, device=gpu).to(torch.int16)
    dp = (10001 + torch.arange(n, device=gpu) % 12).to(torch.int16)
    z32 = torch.zeros(n, dtype=torch.int32, device=gpu)
    flag = torch.full((n,), 0x18, dtype=torch.uint8, device=gpu)
    pitch = 1488
    wire = torch.zeros(n * pitch, dtype=torch.uint8, device=gpu)
    woff = torch.arange(n, device=gpu, dtype=torch.int64) * pitch
    st = torch.empty(n, dtype=torch.int32, device=gpu)
    codec.output_wire_batch(w.payload, w.pay_off, w.pay_len, w.cmd, w.conv, w.conn_key, src, dst, sp, dp, z32, z32,
                            flag, z32.to(torch.int16), wire, woff, st, eth=bytes(12) + b"\x08\x00",
                            id_uniform=workload.ID_UNIFORM)
    fc = rc.make_filter(dst_ip="10.0.0.2", dst_singles=[10001, 10002], dst_ranges=[(10003, 10010)])
    fs = rc.make_filter(dst_ip="10.0.0.2", dst_singles=[10001, 10002], dst_ranges=[(10003, 10010)], is_server=True)
    exp_ok = ((dp.cpu().numpy().astype(np.int32) & 0xFFFF) <= 10010) & (st.cpu().numpy() > 0)
    for f in (fc, fs):
        match = torch.empty(n, dtype=torch.uint8, device=gpu)
        codec.capture_filter_batch(wire, woff, st, 1, f, match)
        torch.cuda.synchronize()
        assert np.array_equal(match.cpu().numpy().astype(bool), exp_ok)
    # spot-check against the oracle on the bytes
    h, sts = wire.cpu().numpy(), st.cpu().numpy()
    for i in range(0, n, 97):
        if sts[i] > 0:
            pkt = h[i * pitch: i * pitch + sts[i]].tobytes()
            assert oracle.capture_filter(pkt, 1, fs) == int(exp_ok[i])


def test_filter_errors(codec, gpu):
    import torch

    from rsock_amd.codec import RskError

    z = torch.zeros(4, dtype=torch.int64, device=gpu)
    m = torch.zeros(4, dtype=torch.uint8, device=gpu)
    arena = torch.zeros(64, dtype=torch.uint8, device=gpu)
    with pytest.raises(RskError):
        codec.capture_filter_batch(arena, z, z.to(torch.int32), 1, rc.make_filter(dst_ranges=[(5, 5)]), m)
    with pytest.raises(RskError):
        codec.capture_filter_batch(arena, z, z.to(torch.int32), 7, rc.make_filter(), m)
    nm = torch.full((1,), 9, dtype=torch.int32, device=gpu)
    e = torch.zeros(0, dtype=torch.int64, device=gpu)
    codec.capture_filter_batch(arena, e, e.to(torch.int32), 1, rc.make_filter(), m, None, nm)
    torch.cuda.synchronize()
    assert int(nm.item()) == 0
