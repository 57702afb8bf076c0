#!/bin/bash
# scratch (GPU box): demux tile size A/B (RSK_DM_ITEMS 16 shipped / 8 / 4): parity, then C3 / C4 timings
set -o pipefail
O=gpurun_out/${1:-r03dm}
mkdir -p $O
for lib in librsk.so librsk_dm8.so; do
RSK_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_demux.py tests/test_gpu_tcpstate.py -x -q --timeout 120 --timeout-method thread > $O/tests_$lib.log 2>&1 || { echo tests $lib failed; tail -30 $O/tests_$lib.log; exit 1; }
tail -1 $O/tests_$lib.log
done
for cfg in c3 c4; do
for lib in librsk_dmseq.so librsk.so librsk_dm8.so librsk_dmseq.so librsk.so librsk_dm8.so; do
RSK_LIB=$lib timeout -k 10 200 python tools/bench_paths.py --config $cfg --only demux,demux_64conn,tcp_send_seq_groupby --rounds 5 > $O/p.json 2>> $O/err.log || { echo paths failed; tail $O/err.log; exit 1; }
python -c "import json,sys; d=json.load(open('$O/p.json')); print('$cfg', '$lib', {k: v['ms'] for k, v in d['paths'].items()})" | tee -a $O/summary.txt
done
done
