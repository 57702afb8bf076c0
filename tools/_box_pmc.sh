#!/bin/bash
# scratch (GPU box): HBM traffic (FETCH_SIZE / WRITE_SIZE, separate passes) of encode variants on C4 (pad128)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${1:-r03pmc}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for v in ${2:-0,56}; do :; done
for v in $(echo ${2:-0,56} | tr , ' '); do
for c in FETCH_SIZE WRITE_SIZE; do
timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc_v${v}_$c -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/ab_encode.py --config c4 --variants $v --pads 128 --rounds 1 --reps 3 > $O/pmc_v${v}_$c.log 2>&1 || { echo pmc $v $c failed; tail $O/pmc_v${v}_$c.log; exit 1; }
done
done
cd $GRAFT_REPO_ROOT
python tools/pmc_cases.py $O --kernel k_encode --algorithmic 1528521696 | tee $O/traffic.json
timeout -k 10 240 python tools/ab_encode.py --config c4 --variants ${2:-0,56} --pads 128 --rounds 8 | tee $O/enc_c4.json
