#!/bin/bash
# Round 4, GPU call T (runs ON THE GPU BOX from the repo root): the two-pass wire build (k_wire_heads +
# k_wire_copy) -- GPU tests (wire tests on both paths), then encode / wire paths per encode path on C3
# and C4, and a kernel trace of the C3 wire paths.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04t
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for cfg in c3 c4; do
    for p in 1 2; do
        timeout -k 10 240 python3 "$R/tools/bench_paths.py" --config $cfg --only encode,encode_wire_raw4,encode_wire_eth --encode-path $p --rounds 5 --reps 5 > "$OUT/p${p}_$cfg.json" 2> "$OUT/p${p}_$cfg.err" || exit 1
    done
done &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/tools/bench_paths.py" --config c3 --only encode_wire_raw4,encode_wire_eth --encode-path 2 --rounds 1 --reps 3 > "$OUT/kt.log" 2>&1)
rc=$?
tail -2 "$OUT/gpu_tests.log"; cat "$OUT"/p*.json 2>/dev/null
exit $rc
