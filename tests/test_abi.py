"""CPU: the C-ABI library loads and exports every symbol include/rsk_codec.h declares; the ctypes
struct mirrors match the C layout (checked by compiling a probe with gcc); host-only helpers match
the reference fixtures.  No GPU compute calls."""
from __future__ import annotations

import os
import subprocess
import tempfile

import numpy as np
import pytest

from rsock_amd import _abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    syms = _abi.header_symbols()
    assert len(syms) >= 15
    out = subprocess.run(["nm", "-D", "--defined-only", _abi.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    assert sorted(n for n, _, _ in _abi.SIGNATURES) == syms
    lib = _abi.load()  # binds every signature
    assert lib.rsk_version().startswith(b"rsk ")


def test_no_gpu_create_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _abi.load()
    assert not lib.rsk_create(b"hello135", 8, 0)
    assert b"device" in lib.rsk_last_error().lower()


PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "rsk_codec.h"
#define F(T, m) printf(#T "." #m " %zu\n", offsetof(T, m));
#define S(T) printf(#T " %zu\n", sizeof(T));
int main(void) {
  S(rsk_encode_in) F(rsk_encode_in, payload_arena) F(rsk_encode_in, id) F(rsk_encode_in, id_uniform)
  S(rsk_encode_out) F(rsk_encode_out, status) F(rsk_encode_out, flags)
  S(rsk_decode_out) F(rsk_decode_out, status) F(rsk_decode_out, valid_idx) F(rsk_decode_out, n_valid)
  S(rsk_tcpinfo_out) F(rsk_tcpinfo_out, flag) F(rsk_tcpinfo_out, cap_pay_len)
  return 0;
}
"""


def test_struct_layouts_match_header():
    import ctypes

    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.c")
        open(src, "w").write(PROBE)
        exe = os.path.join(d, "probe")
        subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    c = {ln.split()[0]: int(ln.split()[1]) for ln in lines if ln.strip()}
    m = {"rsk_encode_in": _abi.EncodeIn, "rsk_encode_out": _abi.EncodeOut, "rsk_decode_out": _abi.DecodeOut,
         "rsk_tcpinfo_out": _abi.TcpInfoOut}
    for k, v in c.items():
        if "." in k:
            t, f = k.split(".")
            assert getattr(m[t], f).offset == v, k
        else:
            assert ctypes.sizeof(m[k]) == v, k


def test_host_key_helpers_match_reference_fixtures():
    g = np.load(os.path.join(ROOT, "tests", "golden", "tcpinfo_keys.npz"), allow_pickle=False)
    lib = _abi.load()
    for a, b, kt, ku in zip(g["key_sp"], g["key_dp"], g["key_tcp"], g["key_udp"]):
        assert lib.rsk_key_for_tcp(int(a), int(b)) == int(kt)
        assert lib.rsk_key_for_udp(int(a), int(b)) == int(ku)


def test_constants_match_header():
    text = open(os.path.join(ROOT, "include", "rsk_codec.h")).read()
    import re

    defs = dict(re.findall(r"#define (RSK_[A-Z0-9_]+) \(?(0x[0-9a-fA-F]+|-?\d+)u?\)?", text))
    for name, val in defs.items():
        py = getattr(_abi, name[4:], None)
        if py is not None:
            assert py == int(val, 0), name
