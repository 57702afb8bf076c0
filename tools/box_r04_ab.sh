#!/bin/bash
# Round 4, GPU call AB (runs ON THE GPU BOX from the repo root): the per-set kernel with every set on the
# flat list (MODE 16: the per-packet path's registers out of the kernel; A/B 120 / 121 / 122 = flat
# unroll 4 / 2 / 8) against the shipped MODE 12 on C2 (and C4 for reference).  Byte-checked vs v0.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ab
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c2 --variants 0,108,120,121,122 --pads 16 --rounds 8 --reps 10 > "$OUT/flat_c2.json" 2> "$OUT/flat_c2.err" &&
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c4 --variants 0,108,120 --pads 128 --rounds 4 --reps 5 > "$OUT/flat_c4.json" 2> "$OUT/flat_c4.err"
rc=$?
cat "$OUT"/flat_*.json 2>/dev/null
exit $rc
