#!/bin/bash
# Round 4, GPU call L (runs ON THE GPU BOX from the repo root): the look-ahead one-wave-per-packet encode
# (A/B variants 90-95, k_encode_la) against the shipped k_encode (0) and the two-pass form (76), frames
# and status byte-checked against variant 0; its per-kernel trace; then the pipelined wire A/B of call K
# (variants 11 / 12 against 0).  Every GPU step under its own limit, chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04l
mkdir -p "$OUT"
export RSK_LIB=librsk_ab.so
timeout -k 10 300 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,90,91,92,93,94,95,76 --pads 16 --rounds 6 --reps 5 > "$OUT/la_c3.json" 2> "$OUT/la_c3.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c3 --packets 1048576 --variants 0,92,93 --pads 0 --rounds 4 --reps 5 > "$OUT/la_c3_pad0.json" 2> "$OUT/la_c3_pad0.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c4 --variants 0,92,93 --pads 128,0 --rounds 4 --reps 5 > "$OUT/la_c4.json" 2> "$OUT/la_c4.err" &&
timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c2 --variants 0,92 --pads 16 --rounds 4 --reps 5 > "$OUT/la_c2.json" 2> "$OUT/la_c2.err" &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/kt" -o kt --output-format csv -- \
    python3 "$R/tools/ab_encode.py" --config c3 --variants 0,92,93 --pads 16 --rounds 1 --reps 3 > "$OUT/kt.log" 2>&1) &&
for cfg in c4 c3; do
    timeout -k 10 240 python3 "$R/tools/bench_paths.py" --config $cfg --only encode,encode_wire_raw4,encode_wire_eth,encode_wire_raw4_v11,encode_wire_eth_v11,encode_wire_raw4_v12,encode_wire_eth_v12 --wire-variants 11,12 --rounds 5 --reps 5 > "$OUT/w_$cfg.json" 2> "$OUT/w_$cfg.err" || exit 1
done
rc=$?
cat "$OUT"/la_*.json "$OUT"/w_*.json 2>/dev/null
exit $rc
