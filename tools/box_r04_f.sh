#!/bin/bash
# Round 4, GPU call F (runs ON THE GPU BOX from the repo root): GPU tests, then the wire build (per-packet
# copy: dead slot 1 skipped) against the round-3 build on C4 / C3 / C2 (HIP events, separate processes).
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04f
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for cfg in c4 c3 c2; do
    RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode,encode_wire_raw4,encode_wire_eth --rounds 5 --reps 5 > "$OUT/w_old_$cfg.json" 2> "$OUT/w_old_$cfg.err" &&
    RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode,encode_wire_raw4,encode_wire_eth --rounds 5 --reps 5 > "$OUT/w_new_$cfg.json" 2> "$OUT/w_new_$cfg.err" || exit 1
done
rc=$?
cat "$OUT"/w_*.json
exit $rc
