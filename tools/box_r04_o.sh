#!/bin/bash
# Round 4, GPU call O (runs ON THE GPU BOX from the repo root): the shipped two-pass encode path for
# long-frame batches.  GPU tests (both encode paths), smoke, the bench line (C3), then per-path encode
# times against the build before it (librsk_r04base.so, separate processes): C3 / C4 / C2.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04o
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
(cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1) &&
timeout -k 10 420 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
for cfg in c3 c4 c2; do
    RSK_LIB=librsk_r04base.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --rounds 5 --reps 5 > "$OUT/base_$cfg.json" 2> "$OUT/base_$cfg.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --encode-path 1 --rounds 5 --reps 5 > "$OUT/p1_$cfg.json" 2> "$OUT/p1_$cfg.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --encode-path 2 --rounds 5 --reps 5 > "$OUT/p2_$cfg.json" 2> "$OUT/p2_$cfg.err" || exit 1
done
rc=$?
tail -2 "$OUT/gpu_tests.log"; cat "$OUT/smoke.log" "$OUT/bench.json" "$OUT"/base_*.json "$OUT"/p1_*.json "$OUT"/p2_*.json 2>/dev/null
exit $rc
