#!/bin/bash
# scratch (GPU box): encode tail-shaping variants on C3 / C4 / C2 (in-process A/B, frames checked equal)
set -o pipefail
O=gpurun_out/${1:-r03g}
mkdir -p $O
for cfg in c3 c4 c2; do
V=0,73,75,81,79,80,83

timeout -k 10 240 python tools/ab_encode.py --config $cfg --variants $V --pads 16 --rounds 8 > $O/enc_$cfg.json 2>> $O/ab.err || { echo ab_encode failed; tail $O/ab.err; exit 1; }
cat $O/enc_$cfg.json
done
