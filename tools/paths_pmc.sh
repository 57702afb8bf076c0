#!/bin/bash
# Runs ON THE GPU BOX: HBM PMC passes (FETCH_SIZE, WRITE_SIZE separately) over one round of every
# per-path op of tools/bench_paths.py, for per-kernel traffic (tools/paths_traffic.py).
#   usage: tools/paths_pmc.sh TAG [config]
set -uo pipefail
TAG=${1:-paths_pmc}; CFG=${2:-c3}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 "$R/tools/bench_paths.py" --config "$CFG" --rounds 1 --reps 1 > "$OUT/fetch.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o pmc --output-format csv -- \
    python3 "$R/tools/bench_paths.py" --config "$CFG" --rounds 1 --reps 1 > "$OUT/write.log" 2>&1
