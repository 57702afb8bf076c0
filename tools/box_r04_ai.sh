#!/bin/bash
# Round 4, GPU call AI (runs ON THE GPU BOX from the repo root): the copy pass split into launches of
# 2^25 packets -- the new beyond-one-launch test, the encode tests, then C5 on one GPU (64M packets).
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ai
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_streams.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
timeout -k 10 600 python3 "$R/bench.py" --gpus 1 --config c5 --steps 5 --warmup 3 --no-tag-variant > "$OUT/bench_c5.json" 2> "$OUT/bench_c5.err"
rc=$?
grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -1
grep -o '"value": [0-9.]*\|"encode": [0-9.]*\|"frac": [0-9.]*\|"encode_path": "[^"]*"' "$OUT/bench_c5.json" | head -6
tail -2 "$OUT/bench_c5.err"
exit $rc
