#!/bin/bash
# Round 4, GPU call E (runs ON THE GPU BOX from the repo root): where k_dm_insert's time goes on C3
# (A/B build, RSK_DM_VARIANT: 0 shipped, 1 no global probe, 2 plain first load, 3 no key confirmation;
# 1 and 3 are timing-only, their segments are wrong), per-kernel traces.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04e
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export RSK_LIB=librsk_ab.so
for v in 0 1 2 3; do
    RSK_DM_VARIANT=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt_v$v" -o kt --output-format csv -- \
        python3 "$R/tools/bench_paths.py" --config c3 --only demux,demux_64conn --rounds 1 --reps 3 > "$OUT/kt_v$v.log" 2>&1 || exit 1
done
