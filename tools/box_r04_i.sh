#!/bin/bash
# Round 4, GPU call I (runs ON THE GPU BOX from the repo root): C3 copy-structure probes (plain copies,
# wrong bytes): 74 one wave per packet; 85 / 88 persistent waves, one packet per iteration (8192 /
# 16384 waves); 86 the same with the next packet's loads before the current stores; 87 / 89 one-shot
# waves of 8 / 2 consecutive packets, one at a time; 73 the shipped mapping; 0 the shipped kernel.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04i
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,73,74,85,86,87,88,89 --pads 16 --rounds 5 --reps 5 > "$OUT/ab_c3.json" 2> "$OUT/ab_c3.err"
rc=$?
cat "$OUT"/ab_c3.json
exit $rc
