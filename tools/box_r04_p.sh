#!/bin/bash
# Round 4, GPU call P (runs ON THE GPU BOX from the repo root): validation of the two-pass encode path
# with the per-set kernel restored -- GPU tests, smoke, bench + rocprofv3 stats + PMC traffic for C3
# (two-pass) and C4 / C2 (per-set), per-path encode times against the build before (librsk_r04base.so),
# and the flat-MD5 A/B (MODE 12, v108) on C3.  Chained with &&.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04p
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
(cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1) &&
bash "$R/tools/profile_box.sh" r04p/c3 &&
bash "$R/tools/profile_box.sh" r04p/c4 --config c4 &&
bash "$R/tools/profile_box.sh" r04p/c2 --config c2 &&
for cfg in c3 c4 c2; do
    RSK_LIB=librsk_r04base.so timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --rounds 5 --reps 5 > "$OUT/base_$cfg.json" 2> "$OUT/base_$cfg.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --encode-path 1 --rounds 5 --reps 5 > "$OUT/p1_$cfg.json" 2> "$OUT/p1_$cfg.err" &&
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode --encode-path 2 --rounds 5 --reps 5 > "$OUT/p2_$cfg.json" 2> "$OUT/p2_$cfg.err" || exit 1
done &&
RSK_LIB=librsk_ab.so timeout -k 10 200 python3 "$R/tools/ab_encode.py" --config c3 --variants 0,108 --pads 16 --rounds 5 --reps 5 > "$OUT/md5flat_c3.json" 2> "$OUT/md5flat_c3.err"
rc=$?
tail -2 "$OUT/gpu_tests.log"; cat "$OUT/smoke.log" "$OUT"/c*/bench.json "$OUT"/base_*.json "$OUT"/p1_*.json "$OUT"/p2_*.json "$OUT"/md5flat_c3.json 2>/dev/null
exit $rc
