#!/bin/bash
# Round 4, GPU call K (runs ON THE GPU BOX from the repo root): the software-pipelined wire copy with its
# loads no longer waited for at issue (A/B wire variants 11 / 12: 4 / 3 packets per batch) against the
# shipped unpipelined 8-packet copy (0), RAW4 and Ethernet, C4 / C3 / C2.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04k
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export RSK_LIB=librsk_ab.so
for cfg in c4 c3 c2; do
    timeout -k 10 240 python3 "$R/tools/bench_paths.py" --config $cfg --only encode,encode_wire_raw4,encode_wire_eth,encode_wire_raw4_v11,encode_wire_eth_v11,encode_wire_raw4_v12,encode_wire_eth_v12 --wire-variants 11,12 --rounds 5 --reps 5 > "$OUT/w_$cfg.json" 2> "$OUT/w_$cfg.err" || exit 1
done
cat "$OUT"/w_*.json
