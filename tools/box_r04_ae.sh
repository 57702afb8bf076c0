#!/bin/bash
# Round 4, GPU call AE (runs ON THE GPU BOX from the repo root): the short-frame path with the generic
# MD5 schedule (MODE 19, 82 VGPRs, 6 waves per SIMD) against the word-specialised one (MODE 16, 97
# VGPRs, 5 waves; librsk_m16.so), C2 encode on path 3, separate processes alternated; then the GPU
# tests of the encode paths.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ae
mkdir -p "$OUT"
for rep in 1 2 3; do
    RSK_LIB=librsk_m16.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c2 --only encode --encode-path 3 --rounds 5 --reps 10 > "$OUT/m16_$rep.json" 2> "$OUT/m16_$rep.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c2 --only encode --encode-path 3 --rounds 5 --reps 10 > "$OUT/m19_$rep.json" 2> "$OUT/m19_$rep.err" || exit 1
done &&
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1)
rc=$?
for f in "$OUT"/m1*.json; do echo "$(basename $f) $(python3 -c "import json; print(json.load(open('$f'))['paths']['encode']['ms'])")"; done
grep -E "passed|failed" "$OUT/gpu_tests.log" | tail -1
exit $rc
