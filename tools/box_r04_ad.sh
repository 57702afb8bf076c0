#!/bin/bash
# Round 4, GPU call AD (runs ON THE GPU BOX from the repo root): the per-set kernel without the TAG form
# (MODE 18, A/B 123: the long-frame copy's registers out) against the shipped MODE 12 (108) on C4.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ad
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c4 --variants 0,108,123 --pads 128,0 --rounds 6 --reps 5 > "$OUT/notag_c4.json" 2> "$OUT/notag_c4.err"
rc=$?
cat "$OUT"/notag_c4.json 2>/dev/null
exit $rc
