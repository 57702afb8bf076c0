"""The encode paths of rsk_encode_batch every GPU encode test runs explicitly (rsk_set_encode_path),
and a holder that asserts after EVERY encode that the library really took the path it was held to
(rsk__last_encode_path): a silent fallback to another path must fail the test, not pass it on the
other path's bytes."""
from __future__ import annotations

import contextlib

# (path, packets per copy wave of the two-pass form; 0 = not the two-pass form)
#   1 = the per-set kernel k_encode; 2 = the two-pass form (k_encode_heads, then k_encode_copy with k
#   packets per wave: 1 for long frames, 4 for mid-length ones; k = -1: the output-stationary copy
#   k_encode_os AUTO takes for byte-packed frames, which copies packet by packet when the header pass
#   finds the frames out of order or far apart); 3 = the short-frame kernel (every set on the flat
#   chunk list)
ENC_PATHS = [(1, 0), (2, 1), (2, 2), (2, 4), (2, -1), (3, 0)]


def path_id(pk) -> str:
    p, k = pk
    return f"path{p}" + (("os" if k < 0 else f"k{k}") if p == 2 else "")


@contextlib.contextmanager
def held(codec, path: int, k: int = 0):
    """codec held to encode path `path` (and fused k); every output_batch inside asserts the path."""
    codec.set_encode_path(path)
    if path == 2:
        codec.set_copy_k(k)
    cls_fn = type(codec).output_batch

    def checked(*a, **kw):
        cls_fn(codec, *a, **kw)
        got = codec.last_encode_path
        assert got == path, f"encode held to path {path} ran path {got}"
        if path == 2 and k:
            assert codec.last_copy_k == k, f"two-pass copy held to k = {k} ran k = {codec.last_copy_k}"

    codec.output_batch = checked
    try:
        yield codec
    finally:
        del codec.output_batch
        codec.set_encode_path(0)
        codec.set_copy_k(0)
