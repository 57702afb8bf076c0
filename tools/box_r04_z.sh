#!/bin/bash
# Round 4, GPU call Z (runs ON THE GPU BOX from the repo root): the round's last build -- every GPU
# test and smoke, then the default bench line.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04z
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
(cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1) &&
timeout -k 10 420 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
tail -2 "$OUT/gpu_tests.log"; cat "$OUT/smoke.log" 2>/dev/null; grep -o '"value": [0-9.]*' "$OUT/bench.json" | head -3
exit $rc
