#!/bin/bash
# scratch (GPU box): parity of the encode paths, then the tag-mode A/B of two libraries and encode variants
set -o pipefail
O=gpurun_out/${1:-r03f}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests failed; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for cfg in c3 c4; do
  for lib in librsk.so librsk_old.so librsk.so librsk_old.so; do
    RSK_LIB=$lib timeout -k 10 200 python tools/ab_tag.py --config $cfg --rounds 6 >> $O/tag_$cfg.jsonl 2>> $O/ab.err || { echo ab_tag failed; tail $O/ab.err; exit 1; }
  done
done
cat $O/tag_c3.jsonl $O/tag_c4.jsonl
timeout -k 10 240 python tools/ab_encode.py --config c3 --variants 0,57,58,59,65,69,70,71,72,73,74 --pads 16 --rounds 6 > $O/enc_c3.json 2>> $O/ab.err || { echo ab_encode failed; tail $O/ab.err; exit 1; }
cat $O/enc_c3.json
timeout -k 10 240 python tools/ab_encode.py --config c4 --variants 0,57,58,59,65,69,70,71,72,73,74 --pads 16 --rounds 6 > $O/enc_c4.json 2>> $O/ab.err || { echo ab_encode failed; tail $O/ab.err; exit 1; }
cat $O/enc_c4.json
