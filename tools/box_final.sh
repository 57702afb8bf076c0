#!/bin/bash
# Runs ON THE GPU BOX: the round's validation (GPU suite, smoke, C3 bench + rocprofv3 stats + PMC
# passes: tools/box_validate.sh), then every path's timing on C3 and C4 (tools/bench_paths.py).
set -o pipefail
TAG=${1:-r03z}
O=gpurun_out/$TAG
bash tools/box_validate.sh $TAG || exit 1
for cfg in c3 c4; do
timeout -k 10 300 python tools/bench_paths.py --config $cfg > $O/paths_$cfg.json 2> $O/paths_$cfg.err || { echo paths $cfg failed; tail $O/paths_$cfg.err; exit 1; }
python -c "import json; d=json.load(open('$O/paths_$cfg.json')); print('$cfg', {k: v['ms'] for k, v in d['paths'].items()})"
done
