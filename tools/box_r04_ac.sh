#!/bin/bash
# Round 4, GPU call AC (runs ON THE GPU BOX from the repo root): the short-frame path (every set on the
# flat chunk list, RSK_ENC_PATH_SHORT) -- GPU tests (every encode test on paths 1 / 2 / 3), then C2 encode
# per path (separate processes, alternated) and the C2 bench line.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ac
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for rep in 1 2; do
    for p in 1 3; do
        timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c2 --only encode --encode-path $p --rounds 5 --reps 10 > "$OUT/c2_p${p}_$rep.json" 2> "$OUT/c2_p${p}_$rep.err" || exit 1
    done
done &&
timeout -k 10 420 python3 "$R/bench.py" --config c2 > "$OUT/bench_c2.json" 2> "$OUT/bench_c2.err"
rc=$?
grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -1
for f in "$OUT"/c2_p*.json; do echo "$(basename $f) $(python3 -c "import json; print(json.load(open('$f'))['paths']['encode']['ms'])")"; done
grep -o '"value": [0-9.]*\|"encode_path": "[^"]*"\|"encode": [0-9.]*' "$OUT/bench_c2.json" | head -5
exit $rc
