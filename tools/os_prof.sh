#!/bin/bash
# Runs ON THE GPU BOX: kernel trace + SQ / traffic counters of the output-stationary encode copy on
# C4's byte-packed layout (tools/bench_layouts.py --layouts packed --copy-k -1).  usage: TAG [copy_k]
set -uo pipefail
TAG=${1:-os_prof}; K=${2:--1}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD=(python3 "$R/tools/bench_layouts.py" --config c4 --layouts packed --encode-path 2 --copy-k "$K" --rounds 2 --reps 5)
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${CMD[@]}" \
    > "$OUT/kt.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU -T -d "$OUT/pmc_sq" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_sq.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_write.log" 2>&1
