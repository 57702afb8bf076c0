#!/bin/bash
# Round 4, GPU call AH (runs ON THE GPU BOX from the repo root): BASELINE config 5 on ONE GPU (64M x
# 1400-B packets, ~185 GB of arenas: the scaling curve's N = 1 point) with the two-pass encode.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ah
mkdir -p "$OUT"
timeout -k 10 600 python3 "$R/bench.py" --gpus 1 --config c5 --steps 5 --warmup 3 --no-tag-variant > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
rc=$?
grep -o '"value": [0-9.]*\|"encode": [0-9.]*\|"frac": [0-9.]*\|"encode_path": "[^"]*"' "$OUT/bench_c5.json" | head -6
tail -3 "$OUT/bench_c5.err"
exit $rc
