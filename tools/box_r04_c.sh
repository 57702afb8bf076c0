#!/bin/bash
# Round 4, GPU call C (runs ON THE GPU BOX from the repo root): the GPU tests on the shipped library,
# k_enc_few (few packets per wave, variants 77-82) against k_encode, the MD5 schedule split (generic in
# the framing kernels, specialised in decode) against the round-3 build, and per-kernel demux traces.
# Every GPU step under its own time limit, chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04c
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
AB="$R/tools/ab_encode.py"
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
RSK_LIB=librsk_ab.so timeout -k 10 300 python3 "$AB" --config c3 --variants 0,74,77,78,79,80,81,82 --pads 16 --rounds 6 --reps 5 > "$OUT/ab_c3.json" 2> "$OUT/ab_c3.err" &&
RSK_LIB=librsk_ab.so timeout -k 10 200 python3 "$AB" --config c4 --variants 0,78,79,80,81 --pads 128 --rounds 6 --reps 10 > "$OUT/ab_c4.json" 2> "$OUT/ab_c4.err" &&
RSK_LIB=librsk_ab.so timeout -k 10 200 python3 "$AB" --config c2 --variants 0,79,81 --pads 16 --rounds 6 --reps 10 > "$OUT/ab_c2.json" 2> "$OUT/ab_c2.err" &&
for cfg in c2 c4; do
    RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config $cfg --rounds 6 --reps 10 > "$OUT/tag_old_$cfg.json" 2> "$OUT/tag_old_$cfg.err" &&
    RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config $cfg --rounds 6 --reps 10 > "$OUT/tag_new_$cfg.json" 2> "$OUT/tag_new_$cfg.err" || exit 1
done &&
for cfg in c3 c4; do
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -T -d "$OUT/dm_$cfg" -o kt --output-format csv -- \
        python3 "$R/tools/bench_paths.py" --config $cfg --only demux,demux_64conn --rounds 1 --reps 3 > "$OUT/dm_$cfg.log" 2>&1 || exit 1
done
rc=$?
cat "$OUT"/ab_c*.json 2>/dev/null
exit $rc
