#!/bin/bash
# Round 4, GPU call V (runs ON THE GPU BOX from the repo root): k_encode layouts (slots / packed16 /
# byte-packed / odd offsets) on C3 and C4 for both encode paths (tools/bench_layouts.py).
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04v
mkdir -p "$OUT"
for cfg in c3 c4; do
    for p in 1 2; do
        timeout -k 10 300 python3 "$R/tools/bench_layouts.py" --config $cfg --encode-path $p --rounds 4 --reps 5 > "$OUT/lay_${cfg}_p$p.json" 2> "$OUT/lay_${cfg}_p$p.err" || exit 1
    done
done
rc=$?
cat "$OUT"/lay_*.json 2>/dev/null
exit $rc
