#!/bin/bash
# Round 4, GPU call R (runs ON THE GPU BOX from the repo root): the two-pass encode's passes, A/B build:
# header pass held to 80 SGPRs with 1 / 2 packets per lane and generic / word-specialised MD5
# (109-112), copy pass in blocks of 512 / 1024 / 64 threads (113-115) and with nontemporal loads (116),
# against the shipped pair (76) and the per-set kernel (0); then their kernel trace.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04r
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 400 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,76,109,110,111,112,113,114,115,116 --pads 16 --rounds 6 --reps 5 > "$OUT/tp_c3.json" 2> "$OUT/tp_c3.err" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/tools/ab_encode.py" --config c3 --variants 76,109,110,111,112 --pads 16 --rounds 1 --reps 3 > "$OUT/kt.log" 2>&1)
rc=$?
cat "$OUT"/tp_c3.json 2>/dev/null
exit $rc
