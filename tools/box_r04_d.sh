#!/bin/bash
# Round 4, GPU call D (runs ON THE GPU BOX from the repo root): GPU tests, demux of this build against
# the round-3 build (HIP events, separate processes) and its per-kernel trace, the bench line.
# Every GPU step under its own time limit, chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04d
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
for cfg in c3 c4; do
    RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only demux,demux_64conn --rounds 3 --reps 5 > "$OUT/dm_old_$cfg.json" 2> "$OUT/dm_old_$cfg.err" &&
    RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only demux,demux_64conn --rounds 3 --reps 5 > "$OUT/dm_new_$cfg.json" 2> "$OUT/dm_new_$cfg.err" &&
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt_$cfg" -o kt --output-format csv -- \
        python3 "$R/tools/bench_paths.py" --config $cfg --only demux,demux_64conn --rounds 1 --reps 3 > "$OUT/kt_$cfg.log" 2>&1 || exit 1
done &&
timeout -k 10 420 python3 "$R/bench.py" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?
cat "$OUT"/dm_*.json "$OUT/bench.json" 2>/dev/null
exit $rc
