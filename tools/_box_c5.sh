#!/bin/bash
# scratch (GPU box): C5 (64M packets) on one GPU, MD5 per lane (the per-GPU shard at N = 8 is 8M)
set -o pipefail
O=gpurun_out/${1:-r03c5}
mkdir -p $O
timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { echo c5 failed; tail $O/bench_c5.err; exit 1; }
cat $O/bench_c5.json
