#!/bin/bash
# Runs ON THE GPU BOX (via gpurun, from the repo root): parity tests of the named encode variants,
# then in-process A/B of those variants against the default on C3, C4 and C2.
#   usage: tools/ab_run.sh TAG "13,14,15"
set -uo pipefail
TAG=${1:-ab}; V=${2:-13,14,15}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
K=$(echo "$V" | sed 's/\([0-9]*\)/encv\1/g; s/,/ or /g')
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "$K" > "$OUT/tests.log" 2>&1 &&
timeout -k 10 200 python tools/ab_encode.py --config c3 --variants "0,$V" --pads 16 > "$OUT/c3.json" 2> "$OUT/ab.err" &&
timeout -k 10 200 python tools/ab_encode.py --config c4 --variants "0,$V" --pads 16 > "$OUT/c4.json" 2>> "$OUT/ab.err" &&
timeout -k 10 200 python tools/ab_encode.py --config c2 --variants "0,$V" --pads 16 > "$OUT/c2.json" 2>> "$OUT/ab.err"
