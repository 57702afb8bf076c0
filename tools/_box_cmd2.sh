#!/bin/bash
# scratch: parity of the encode paths after a change, then the layout A/B
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python tools/bench_layouts.py --config c4 > $O/layouts_c4.json 2> $O/layouts.err || { echo layouts failed; tail $O/layouts.err; exit 1; }
cat $O/layouts_c4.json
timeout -k 10 300 python tools/bench_layouts.py --config c3 --packets 1048576 > $O/layouts_c3.json 2>> $O/layouts.err || { echo layouts failed; tail $O/layouts.err; exit 1; }
cat $O/layouts_c3.json
