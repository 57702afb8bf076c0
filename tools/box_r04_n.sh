#!/bin/bash
# Round 4, GPU call N (runs ON THE GPU BOX from the repo root): the one-wave-per-packet copy's floor
# with real frames: k_enc_copy1 alone on records already in place (99), the two-pass form serial (76)
# and with its header pass on a second stream beside the copy (100), against the shipped k_encode (0);
# the look-ahead kernel held to 80 SGPRs (104-107); the flat sets' MD5 on the specialised schedule
# (108) on C2 / C4; then a per-kernel trace.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04n
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,76,99,100,93,101,104,105,106,107 --pads 16 --rounds 5 --reps 5 > "$OUT/pc_c3.json" 2> "$OUT/pc_c3.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c2 --variants 0,108 --pads 16 --rounds 8 --reps 10 > "$OUT/md5flat_c2.json" 2> "$OUT/md5flat_c2.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c4 --variants 0,108 --pads 128 --rounds 6 --reps 5 > "$OUT/md5flat_c4.json" 2> "$OUT/md5flat_c4.err" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/tools/ab_encode.py" --config c3 --variants 0,76,99,100,104,105 --pads 16 --rounds 1 --reps 3 > "$OUT/kt.log" 2>&1)
rc=$?
cat "$OUT"/pc_*.json "$OUT"/md5flat_*.json 2>/dev/null
exit $rc
