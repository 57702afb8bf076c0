"""GPU vs the REFERENCE's own outputs (tests/golden, produced by oracle/_ref from /root/reference
sources): encode the golden inputs and decode the golden frames through the C-ABI; bytes and
fields must equal the reference's, bit for bit."""
from __future__ import annotations

import os

import numpy as np
import pytest

from tests.enc_paths import ENC_PATHS, held, path_id
from tests.test_gpu_parity import DEC_VIEWS, dev, run_decode, run_encode, vcodec  # noqa: F401

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KEY = b"hello135"


def gold(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def _golden_encode(cx, gpu, g, pad16=False):
    n = len(g["status"])
    frame_off = (np.arange(n) * 1504).astype(np.uint64)
    return run_encode(cx, gpu, g["payload"], g["pay_off"], np.minimum(g["pay_len"], 65535).astype(np.uint16),
                      g["cmd"], g["conv"], g["conn_key"], frame_off, n * 1504, idarr=g["id"], pad16=pad16)


@pytest.mark.parametrize("pad16", [False, True])
def test_encode_matches_reference_frames(vcodec, gpu, pad16):
    """The reference's own RConn::Output frames (frames.npz, oracle/_ref) through EVERY encode path
    (vcodec: held to one path, the path asserted after the encode), both tag modes."""
    codec = vcodec
    g = gold("frames.npz")
    n = len(g["status"])
    pitch = 1504
    fr, st = _golden_encode(codec, gpu, g, pad16)
    assert np.array_equal(st, g["status"])
    for i in range(n):
        if st[i] > 0:
            o = int(g["frame_off"][i])
            assert fr[i * pitch: i * pitch + st[i]].tobytes() == g["frames"][o: o + int(g["frame_len"][i])].tobytes(), i


def test_decode_matches_reference_onrecv(codec, gpu):
    g = gold("onrecv.npz")
    got = run_decode(codec, gpu, g["frames"], g["frame_off"], g["frame_len"].astype(np.uint16), g["close"])
    for k, dt in DEC_VIEWS.items():
        assert np.array_equal(got[k].view(dt), g[k]), k
    nv = int(got["n_valid"][0])
    assert nv == int((g["status"] == 1).sum())
    assert np.array_equal(got["valid_idx"][:nv].view(np.uint32), np.nonzero(g["status"] == 1)[0].astype(np.uint32))


@pytest.mark.parametrize("pk", ENC_PATHS, ids=path_id)
def test_tags_all_keys_match_reference(gpu, tag_mode, pk):
    """tags.npz (the reference's compute_hash for all 256 first bytes x 10 key lengths: 1-block,
    2-block and midstate schedules) through every encode path, both tag modes."""
    from rsock_amd.codec import Codec

    g = gold("tags.npz")
    kb, ko, kl = g["key_bytes"], g["key_off"], g["key_len"]
    for k in range(len(kl)):
        key = kb[int(ko[k]): int(ko[k]) + int(kl[k])].tobytes()
        cx = Codec(key, 0, tag_mode=tag_mode)
        try:
            with held(cx, *pk):
                payload = np.repeat(np.arange(256, dtype=np.uint8), 16)
                z = np.zeros(256, np.uint8)
                fr, st = run_encode(cx, gpu, payload, (np.arange(256) * 16).astype(np.uint64),
                                    np.full(256, 16, np.uint16), z, z.astype(np.uint32), z.astype(np.uint64),
                                    (np.arange(256) * 48).astype(np.uint64), 256 * 48)
            assert np.array_equal(fr.reshape(256, 48)[:, :8], g["tags"][k]), len(key)
        finally:
            cx.close()


def test_golden_roundtrip_every_path(vcodec, gpu, oracle):
    """frames.npz's inputs encoded by the held path, then decoded: the frames equal the reference's, every
    framed packet comes back VALID with the reference's fields, and the decode of the reference's own
    frames (onrecv.npz's rule: the oracle pinned to it) agrees field for field."""
    codec = vcodec
    g = gold("frames.npz")
    n = len(g["status"])
    pitch = 1504
    fr, st = _golden_encode(codec, gpu, g)
    ok = st > 0
    flen = np.where(ok, st, 0).astype(np.uint16)
    off = (np.arange(n) * pitch).astype(np.uint64)
    got = run_decode(codec, gpu, fr, off, flen)
    exp = oracle.decode_batch(KEY, fr, off, flen)
    for k, dt in DEC_VIEWS.items():
        assert np.array_equal(got[k].view(dt), exp[k]), k
    assert np.array_equal(got["status"].view(np.int8) == 1, ok)
    assert np.array_equal(got["conv"].view(np.uint32)[ok], g["conv"][ok].astype(np.uint32))
    assert np.array_equal(got["conn_key"].view(np.uint64)[ok], g["conn_key"][ok].astype(np.uint64))
    assert np.array_equal(got["cmd"][ok], g["cmd"][ok].astype(np.uint8))


def test_tcpinfo_records_match_reference(codec, gpu):
    import torch

    g = gold("tcpinfo_keys.npz")
    n = len(g["src"])
    rec = torch.zeros(21 * n, dtype=torch.uint8, device=gpu)
    codec.tcpinfo_encode_batch(dev(g["src"], gpu, np.int32), dev(g["dst"], gpu, np.int32), dev(g["sp"], gpu, np.int16),
                               dev(g["dp"], gpu, np.int16), dev(g["seq"], gpu, np.int32), dev(g["ack"], gpu, np.int32),
                               dev(g["flag"], gpu), rec)
    assert np.array_equal(rec.cpu().numpy(), g["records"])


def test_enchead_shims_match_reference(codec):
    g = gold("enchead.npz")
    for i in range(len(g["enc_buf_len"])):
        h = codec.enc2buf(int(g["enc_cmd"][i]), g["enc_id"][8 * i: 8 * i + 8].tobytes(), int(g["enc_conv"][i]),
                          int(g["enc_key"][i]), buf_len=int(g["enc_buf_len"][i]))
        assert (h is not None) == bool(g["enc_ok"][i])
        if h is not None:
            assert h == g["enc_out"][23 * i: 23 * i + 23].tobytes()
    for i in range(0, len(g["dec_buf_len"]), 3):
        r = codec.decodebuf(g["dec_in"][23 * i: 23 * i + 23].tobytes(), int(g["dec_buf_len"][i]))
        assert (r is not None) == bool(g["dec_ok"][i]), i
        if r is not None:
            assert r[1:] == (int(g["dec_cmd"][i]), g["dec_id"][8 * i: 8 * i + 8].tobytes(), int(g["dec_conv"][i]),
                             int(g["dec_key"][i]))


@pytest.mark.parametrize("flags", [0, 1, 3])
@pytest.mark.parametrize("align", [1, 16])
def test_parse_matches_reference_rawinput(codec, gpu, oracle, flags, align):
    """k_parse_decode == the reference's own RawTcp::RawInput (tests/golden/parse.npz, made by
    tests/golden/make_parse_golden.py from oracle/_ref/librsk_ref_parse.so) on every case of the
    SURVEY §8c parse list; the decode half == the oracle (itself pinned to the reference's OnRecv)."""
    import torch

    from rsock_amd.codec import DecodeBuffers, TcpInfoBuffers
    from tests import pkt as P
    from tests.test_gpu_parity import assert_dec_equal

    g = gold("parse.npz")
    j = list(g["flags"]).index(flags)
    for dl in (1, 0):
        sel = np.nonzero(g["datalink"] == dl)[0]
        recs = [g["arena"][int(g["off"][i]): int(g["off"][i]) + int(g["cap_len"][i])].tobytes() for i in sel]
        arena, offs, cl = P.pack_records(recs, align=align, base_pad=0 if align == 16 else 3)
        wl = g["wire_len"][sel].astype(np.uint32)
        n = len(sel)
        tcp, out = TcpInfoBuffers.alloc(n, gpu), DecodeBuffers.alloc(n, gpu)
        codec.rawinput_batch(dev(arena, gpu), dev(offs, gpu, np.int64), dev(wl, gpu, np.int32), dev(cl, gpu, np.int32),
                             dl, flags, tcp, out)
        torch.cuda.synchronize()
        th = tcp.to_host()
        st = th["parse_status"].view(np.int8)
        refused = g["syn_refused"][sel, j]
        exp_st = np.where(refused, 2, g["status"][sel, j])
        bad = np.nonzero(st != exp_st)[0]
        assert bad.size == 0, (dl, sel[bad[:5]], st[bad[:5]], exp_st[bad[:5]])
        pin = (exp_st == 1) | ((exp_st == 2) & ~refused)
        for k, dt in (("src", np.uint32), ("dst", np.uint32), ("sp", np.uint16), ("dp", np.uint16), ("seq", np.uint32),
                      ("ack", np.uint32), ("flag", np.uint8)):
            assert np.array_equal(th[k].view(dt)[pin], g[k][sel, j][pin]), (dl, k)
        dl_ = exp_st == 1
        assert np.array_equal(th["cap_pay_off"].view(np.uint16)[dl_], g["pay_off"][sel, j][dl_])
        assert np.array_equal(th["cap_pay_len"].view(np.uint16)[dl_], g["pay_len"][sel, j][dl_])
        assert_dec_equal(out.to_host(), oracle.parse_decode_batch(KEY, arena, offs, wl, cl, dl, flags))


def test_tag_mode_api(gpu):
    """rsk_set_tag_mode / rsk_get_tag_mode: a context starts in RSK_TAG_MD5, takes RSK_TAG_TABLE and
    back, refuses unknown modes, and both modes frame the golden frames identically."""
    from rsock_amd import _abi
    from rsock_amd.codec import Codec, RskError, lib

    cx = Codec(b"hello135", 0)
    try:
        assert lib().rsk_get_tag_mode(cx._ctx) == _abi.TAG_MD5 and cx.tag_mode == "md5"
        assert lib().rsk_set_tag_mode(cx._ctx, 7) == _abi.EINVAL
        assert lib().rsk_set_tag_mode(cx._ctx, -1) == _abi.EINVAL
        assert cx.tag_mode == "md5"  # unchanged by a refused mode
        assert lib().rsk_set_tag_mode(None, 0) == _abi.EINVAL and lib().rsk_get_tag_mode(None) == _abi.EINVAL
        g = gold("frames.npz")
        outs = []
        for mode in ("table", "md5"):
            cx.set_tag_mode(mode)
            assert cx.tag_mode == mode
            fr, st = _golden_encode(cx, gpu, g)
            outs.append((fr, st))
        assert np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
        with pytest.raises(RskError):
            cx.set_tag_mode(5)
    finally:
        cx.close()
