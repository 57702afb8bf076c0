#!/bin/bash
# Runs ON THE GPU BOX (via gpurun, from the repo root): bench line, rocprofv3 kernel-trace stats,
# and the HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate passes: they do not fit one TCC
# pass on gfx950).  Every GPU step has its own time limit; steps are chained with &&.
#   usage: tools/profile_box.sh TAG [bench args...]
set -uo pipefail
TAG=${1:-r01}; shift || true
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 "$R/bench.py" --steps 50 --warmup 10 "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-tag-variant --no-scale-anchor "$@" > "$OUT/kt.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-tag-variant --no-scale-anchor "$@" > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-tag-variant --no-scale-anchor "$@" > "$OUT/pmc_write.log" 2>&1
rc=$?
find "$OUT" -name "*.csv" | head -50 > "$OUT/files.txt"
exit $rc
