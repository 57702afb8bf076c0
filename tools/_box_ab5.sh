#!/bin/bash
# scratch (GPU box): encode tail variants (tile-decided) on C3 / C4 / C2, then a kernel trace of the C3 demux
set -o pipefail
O=gpurun_out/${1:-r03l}
mkdir -p $O
for cfg in c3 c4 c2; do
timeout -k 10 240 python tools/ab_encode.py --config $cfg --variants 0,300,75,84,85,86 --pads 16 --rounds 8 > $O/enc_$cfg.json 2>> $O/ab.err || { echo ab_encode failed; tail $O/ab.err; exit 1; }
cat $O/enc_$cfg.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/dm -o dm --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/bench_paths.py --config c3 --only demux,demux_64conn --rounds 3 --reps 5 > $GRAFT_REPO_ROOT/$O/dm.log 2>&1 || { echo demux trace failed; tail $GRAFT_REPO_ROOT/$O/dm.log; exit 1; }
tail -2 $GRAFT_REPO_ROOT/$O/dm.log
find $GRAFT_REPO_ROOT/$O/dm -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-150
