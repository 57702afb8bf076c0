#!/bin/bash
# Round 4, GPU call AG (runs ON THE GPU BOX from the repo root): SQ counters of the two-pass encode's
# kernels on C3 (one pass of 8 SQ counters over a short bench run).
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04ag
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -T -d "$OUT/sq" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 2 --no-cpu-baseline --no-tag-variant > "$OUT/sq.log" 2>&1
rc=$?
tail -3 "$OUT/sq.log"
exit $rc
