#!/bin/bash
# Round 4, GPU call Q (runs ON THE GPU BOX from the repo root): the per-set kernel with the flat sets'
# MD5 on the payload-word-specialised schedule (MODE 12, every key word position compiled) -- GPU tests,
# then per-set encode times against the build before the two-pass change (librsk_r04base.so, MODE 11),
# separate processes, alternated twice.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04q
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for rep in 1 2; do
  for cfg in c2 c4 c3; do
    RSK_LIB=librsk_r04base.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --rounds 5 --reps 10 > "$OUT/base_${cfg}_$rep.json" 2> "$OUT/base_${cfg}_$rep.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --encode-path 1 --rounds 5 --reps 10 > "$OUT/p1_${cfg}_$rep.json" 2> "$OUT/p1_${cfg}_$rep.err" || exit 1
  done
done
rc=$?
tail -2 "$OUT/gpu_tests.log"
for f in "$OUT"/base_*.json "$OUT"/p1_*.json; do echo "$(basename $f) $(python3 -c "import json,sys; print(json.load(open('$f'))['paths']['encode']['ms'])")"; done
exit $rc
