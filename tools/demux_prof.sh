#!/bin/bash
# Runs ON THE GPU BOX: kernel trace of the receive demux (tools/bench_paths.py --only demux,demux_64conn,demux_server,demux_server_group)
# and two SQ counter passes over the same command, for where each demux kernel's time goes.
#   usage: tools/demux_prof.sh TAG [config]
set -uo pipefail
TAG=${1:-demux_prof}; CFG=${2:-c3}
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
CMD=(python3 "$R/tools/bench_paths.py" --config "$CFG" --only demux,demux_64conn,demux_server,demux_server_group --rounds 3 --reps 5)
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o kt --output-format csv -- "${CMD[@]}" \
    > "$OUT/kt.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -T -d "$OUT/pmc_sq" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_sq.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_fetch.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o pmc --output-format csv -- "${CMD[@]}" \
    > "$OUT/pmc_write.log" 2>&1
