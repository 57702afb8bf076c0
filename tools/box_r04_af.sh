#!/bin/bash
# Round 4, GPU call AF (runs ON THE GPU BOX from the repo root): the lean two-pass records (16-B tags,
# EncHead words built in the copy wave) against the 32-B header records (librsk_big.so): encode tests,
# then C3 encode on path 2 in separate processes alternated three times, then the bench line.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04af
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_streams.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for rep in 1 2 3; do
    RSK_LIB=librsk_big.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c3 --only encode --encode-path 2 --rounds 5 --reps 5 > "$OUT/big_$rep.json" 2> "$OUT/big_$rep.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c3 --only encode --encode-path 2 --rounds 5 --reps 5 > "$OUT/lean_$rep.json" 2> "$OUT/lean_$rep.err" || exit 1
done &&
timeout -k 10 420 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -1
for f in "$OUT"/big_*.json "$OUT"/lean_*.json; do echo "$(basename $f) $(python3 -c "import json; print(json.load(open('$f'))['paths']['encode']['ms'])")"; done
grep -o '"value": [0-9.]*\|"encode": [0-9.]*' "$OUT/bench.json" | head -3
exit $rc
