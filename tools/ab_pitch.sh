#!/bin/bash
# Runs ON THE GPU BOX: k_encode at three frame-slot pitches (C3), each in its own process on the same
# box, plus FETCH_SIZE / WRITE_SIZE PMC passes per pitch (separate rocprofv3 runs).
set -uo pipefail
R=$(pwd); OUT=$R/gpurun_out/ab_pitch; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for cfg in "1440 16" "1536 128" "1472 16"; do
  set -- $cfg
  timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0 --pads $2 --frame-pitch $1 \
      > "$OUT/ab_$1.json" 2>> "$OUT/err.log" || exit 1
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/f_$1" -o p --output-format csv -- python3 "$R/tools/ab_encode.py" \
      --config c3 --variants 0 --pads $2 --frame-pitch $1 --rounds 1 --reps 2 > /dev/null 2>> "$OUT/err.log" || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/w_$1" -o p --output-format csv -- python3 "$R/tools/ab_encode.py" \
      --config c3 --variants 0 --pads $2 --frame-pitch $1 --rounds 1 --reps 2 > /dev/null 2>> "$OUT/err.log" || exit 1
done
