#!/bin/bash
# scratch (GPU box): encode parity, then k_encode layouts (slots / packed16 / byte-packed / odd) for two libraries
set -o pipefail
O=gpurun_out/${1:-r03lay}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in librsk_prev.so librsk.so librsk_prev.so librsk.so; do
RSK_LIB=$lib timeout -k 10 200 python tools/bench_layouts.py --config c4 > $O/l.json 2>> $O/err.log || { echo layouts failed; tail $O/err.log; exit 1; }
python -c "import json; d=json.load(open('$O/l.json')); print('c4', '$lib', json.dumps(d))" | tee -a $O/summary.txt
done
for lib in librsk_prev.so librsk.so; do
RSK_LIB=$lib timeout -k 10 200 python tools/bench_layouts.py --config c3 --packets 1048576 > $O/l.json 2>> $O/err.log || { echo layouts failed; tail $O/err.log; exit 1; }
python -c "import json; d=json.load(open('$O/l.json')); print('c3', '$lib', json.dumps(d))" | tee -a $O/summary.txt
done
