#!/bin/bash
# Round 4, GPU call Y (runs ON THE GPU BOX from the repo root): the copy pass with normal stores for
# each frame's first / last 128 B (A/B 119) against the shipped pair (116) on C3, and both passes'
# WRITE_SIZE in separate processes.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04y
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,116,119 --pads 16 --rounds 6 --reps 5 > "$OUT/edge_c3.json" 2> "$OUT/edge_c3.err" &&
(cd /tmp && export TMPDIR=/tmp &&
 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc116" -o pmc --output-format csv -- python3 "$R/tools/ab_encode.py" --config c3 --variants 116 --pads 16 --rounds 1 --reps 2 > "$OUT/pmc116.log" 2>&1 &&
 timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc119" -o pmc --output-format csv -- python3 "$R/tools/ab_encode.py" --config c3 --variants 119 --pads 16 --rounds 1 --reps 2 > "$OUT/pmc119.log" 2>&1)
rc=$?
cat "$OUT"/edge_c3.json 2>/dev/null
exit $rc
