#!/bin/bash
# Runs ON THE GPU BOX: kernel trace + SQ instruction counters + FETCH/WRITE of the encode and wire
# builds on one config (tools/bench_paths.py), for where the two-pass wire copy's time goes.
#   usage: tools/wire_pmc.sh TAG [config]
set -uo pipefail
TAG=${1:-wire_pmc}; CFG=${2:-c4}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD=(python3 "$R/tools/bench_paths.py" --config "$CFG" --only encode,encode_wire_raw4,encode_wire_raw4_perset --rounds 1 --reps 3)
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${CMD[@]}" \
    > "$OUT/kt.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY -T -d "$OUT/pmc_sq" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_sq.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_write.log" 2>&1
