#!/bin/bash
# Round 4, GPU call B (runs ON THE GPU BOX from the repo root): C3 k_encode against memory-pattern
# probes of the same chunks (73: shipped mapping, 74: one wave per packet) and the two-pass form
# (75 / 76), then the MD5 schedule before / after (ab_tag.py on the round-3 build and this one),
# then k_decode traffic.  Every GPU step under its own time limit, chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04b
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
AB="$R/tools/ab_encode.py"
# the shipped library first: every GPU test (MD5 schedule, compaction taint, bench backend default)
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
RSK_LIB=librsk_ab.so timeout -k 10 300 python3 "$AB" --config c3 --variants 0,73,74,75,76,13 --pads 16 --rounds 6 --reps 5 > "$OUT/ab_c3.json" 2> "$OUT/ab_c3.err" &&
RSK_LIB=librsk_ab.so timeout -k 10 200 python3 "$AB" --config c4 --variants 0,73,74,75,76 --pads 128 --rounds 6 --reps 10 > "$OUT/ab_c4.json" 2> "$OUT/ab_c4.err" &&
RSK_LIB=librsk_ab.so timeout -k 10 200 python3 "$AB" --config c2 --variants 0,75 --pads 16 --rounds 6 --reps 10 > "$OUT/ab_c2.json" 2> "$OUT/ab_c2.err" &&
RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config c2 --rounds 6 --reps 10 > "$OUT/tag_old_c2.json" 2> "$OUT/tag_old_c2.err" &&
RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config c2 --rounds 6 --reps 10 > "$OUT/tag_new_c2.json" 2> "$OUT/tag_new_c2.err" &&
RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config c4 --rounds 6 --reps 10 > "$OUT/tag_old_c4.json" 2> "$OUT/tag_old_c4.err" &&
RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config c4 --rounds 6 --reps 10 > "$OUT/tag_new_c4.json" 2> "$OUT/tag_new_c4.err" &&
RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config c3 --rounds 4 --reps 5 > "$OUT/tag_old_c3.json" 2> "$OUT/tag_old_c3.err" &&
RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/ab_tag.py" --config c3 --rounds 4 --reps 5 > "$OUT/tag_new_c3.json" 2> "$OUT/tag_new_c3.err" &&
RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c3 --only demux,demux_64conn --rounds 3 --reps 3 > "$OUT/dm_old_c3.json" 2> "$OUT/dm_old_c3.err" &&
RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c3 --only demux,demux_64conn --rounds 3 --reps 3 > "$OUT/dm_new_c3.json" 2> "$OUT/dm_new_c3.err" &&
RSK_LIB=librsk_r03md5.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c4 --only demux,demux_64conn --rounds 3 --reps 5 > "$OUT/dm_old_c4.json" 2> "$OUT/dm_old_c4.err" &&
RSK_LIB=librsk.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config c4 --only demux,demux_64conn --rounds 3 --reps 5 > "$OUT/dm_new_c4.json" 2> "$OUT/dm_new_c4.err" &&
RSK_LIB=librsk_ab.so timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/pmc_fetch" -o pmc --output-format csv -- \
    python3 "$AB" --config c3 --variants 0,74,75 --pads 16 --rounds 1 --reps 2 > "$OUT/fetch.log" 2>&1 &&
RSK_LIB=librsk_ab.so timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/pmc_write" -o pmc --output-format csv -- \
    python3 "$AB" --config c3 --variants 0,74,75 --pads 16 --rounds 1 --reps 2 > "$OUT/write.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -T -d "$OUT/dec_fetch" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-tag-variant > "$OUT/dec_fetch.log" 2>&1 &&
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -T -d "$OUT/dec_write" -o pmc --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-tag-variant > "$OUT/dec_write.log" 2>&1
rc=$?
cat "$OUT"/ab_c*.json "$OUT"/tag_*.json 2>/dev/null
exit $rc
