#!/bin/bash
# Round 4, GPU call H (runs ON THE GPU BOX from the repo root): does C2's flat path gain from occupancy?
# k_encode forced to 8 / 6 waves per SIMD (A/B variants 83 / 84) against the shipped kernel, MD5 and
# table modes (ab_encode runs the context's default, MD5).  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04h
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export RSK_LIB=librsk_ab.so
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c2 --variants 0,83,84 --pads 16 --rounds 8 --reps 10 > "$OUT/ab_c2.json" 2> "$OUT/ab_c2.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c4 --variants 0,83,84 --pads 128 --rounds 6 --reps 10 > "$OUT/ab_c4.json" 2> "$OUT/ab_c4.err" &&
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,83,84 --pads 16 --rounds 4 --reps 5 > "$OUT/ab_c3.json" 2> "$OUT/ab_c3.err"
rc=$?
cat "$OUT"/ab_*.json
exit $rc
