#!/bin/bash
# Round 4, GPU call M (runs ON THE GPU BOX from the repo root): why the look-ahead encode (k_encode_la)
# is 2x slower than the two-pass form: flag loaded before the chunk loads (96 / 97), no flag at all
# (98, timing only), and the two-pass copy (76) held to 6 / 8 blocks per CU (676 / 876 in that build's v + 100 cap encoding, now 6076 / 8076; k_encode_la's
# 106 SGPRs admit 6 blocks of 256 threads per CU, k_enc_copy1's 35 admit 8).  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04m
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,93,96,97,98,76,676,876 --pads 16 --rounds 5 --reps 5 > "$OUT/la_c3.json" 2> "$OUT/la_c3.err"
rc=$?
cat "$OUT"/la_*.json 2>/dev/null
exit $rc
