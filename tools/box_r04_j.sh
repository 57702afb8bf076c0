#!/bin/bash
# Round 4, GPU call J (runs ON THE GPU BOX from the repo root): k_encode with the dead-lane zeroing moved
# from pkt_issue to pkt_store (the pipelined copy's loads no longer waited for at issue) -- GPU tests,
# then this build against the round-3 build (ab_tag.py: k_encode + decode, MD5 and table modes, separate
# processes, alternated), then the bench line.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04j
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for cfg in c3 c4 c2; do
    for rep in 1 2; do
        RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config $cfg --rounds 4 --reps 5 > "$OUT/tag_old_${cfg}_$rep.json" 2> "$OUT/tag_old_${cfg}_$rep.err" &&
        RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config $cfg --rounds 4 --reps 5 > "$OUT/tag_new_${cfg}_$rep.json" 2> "$OUT/tag_new_${cfg}_$rep.err" || exit 1
    done
done &&
timeout -k 10 420 python3 "$R/bench.py" --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
cat "$OUT/bench.json"
exit $rc
