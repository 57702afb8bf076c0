#!/bin/bash
# Round 4, GPU call W (runs ON THE GPU BOX from the repo root): the per-set kernel with a per-packet
# set's short frames moved to the flat list (MODE 13 / 14: under 256 / 512 B; A/B variants 117 / 118)
# against the shipped MODE 12 (108) on C4 (slots PAD128, no pad), C2 and C3; frames and status
# byte-checked against variant 0.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04w
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c4 --variants 0,108,117,118 --pads 128,0 --rounds 6 --reps 5 > "$OUT/hy_c4.json" 2> "$OUT/hy_c4.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c2 --variants 0,108,117,118 --pads 16 --rounds 6 --reps 10 > "$OUT/hy_c2.json" 2> "$OUT/hy_c2.err" &&
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,108,117 --pads 16 --rounds 4 --reps 5 > "$OUT/hy_c3.json" 2> "$OUT/hy_c3.err"
rc=$?
cat "$OUT"/hy_*.json 2>/dev/null
exit $rc
