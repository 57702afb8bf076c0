#!/bin/bash
# Round 4, GPU call G (runs ON THE GPU BOX from the repo root): the round's validation -- every GPU
# test, smoke(), then tools/profile_box.sh (bench line + rocprofv3 kernel-trace stats + FETCH_SIZE /
# WRITE_SIZE passes) for C3 (the headline), C2 and C4.  Chained with &&; each step has its own limit.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04g
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
(cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1) &&
bash "$R/tools/profile_box.sh" r04g/c3 &&
bash "$R/tools/profile_box.sh" r04g/c2 --config c2 &&
bash "$R/tools/profile_box.sh" r04g/c4 --config c4 &&
for cfg in c4 c3; do
    timeout -k 10 200 python3 "$R/tools/bench_paths.py" --config $cfg --only encode,encode_wire_raw4,encode_wire_eth,decode,demux,demux_64conn --rounds 5 --reps 5 > "$OUT/paths_$cfg.json" 2> "$OUT/paths_$cfg.err" || exit 1
done
rc=$?
tail -2 "$OUT/gpu_tests.log"; cat "$OUT/smoke.log" "$OUT"/c*/bench.json 2>/dev/null
exit $rc
