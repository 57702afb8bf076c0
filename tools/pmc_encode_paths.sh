#!/bin/bash
# Runs ON THE GPU BOX (gpurun, repo root): HBM traffic per encode path variant -- one rocprofv3 pass per
# counter (FETCH_SIZE, WRITE_SIZE: MI355X_MICROARCH.md §HBM, never both in one pass) over a short
# tools/enc_paths_ab.py run of each variant; summarise with tools/pmc_encode_paths.py.
#   usage: tools/pmc_encode_paths.sh TAG CONFIG VARIANT [VARIANT ...]     (VARIANT as enc_paths_ab.py)
set -uo pipefail
TAG=$1; CFG=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  case_=$(echo "$V" | tr ':' '_')
  for CTR in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 120 rocprofv3 --pmc $CTR -T -d "$OUT/pmc_${case_}_$CTR" -o pmc --output-format csv -- \
      python3 "$R/tools/enc_paths_ab.py" --config "$CFG" --variants "$V" --rounds 1 --reps 2 \
      > "$OUT/pmc_${case_}_$CTR.log" 2>&1 || exit 1
  done
done
