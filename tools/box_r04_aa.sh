#!/bin/bash
# Round 4, GPU call AA (runs ON THE GPU BOX from the repo root): encode time of both paths over payload
# lengths (tools/path_threshold.py), to place the two-pass threshold.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04aa
mkdir -p "$OUT"
timeout -k 10 500 python3 "$R/tools/path_threshold.py" > "$OUT/thr.json" 2> "$OUT/thr.err"
rc=$?
cat "$OUT/thr.json" 2>/dev/null
exit $rc
