#!/bin/bash
# Runs ON THE GPU BOX (gpurun, repo root): the GPU test suite, smoke(), then the C3 bench with the
# rocprofv3 kernel-trace stats and PMC traffic passes (tools/profile_box.sh).  usage: TAG
set -o pipefail
TAG=${1:-r03v}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile_box.sh $TAG/c3 --config c3 || { echo profile failed; exit 1; }
cat $O/c3/bench.json
