#!/bin/bash
# Round 4, GPU call X (runs ON THE GPU BOX from the repo root): final validation of the round's build --
# every GPU test, smoke, then bench + rocprofv3 stats + PMC traffic for C3 (the headline), C4, C2.
set -uo pipefail
R=$(pwd)
OUT=$R/gpurun_out/r04xf
mkdir -p "$OUT"
(cd "$R" && timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1) &&
(cd "$R" && timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$OUT/smoke.log" 2>&1) &&
bash "$R/tools/profile_box.sh" r04xf/c3 &&
bash "$R/tools/profile_box.sh" r04xf/c4 --config c4 &&
bash "$R/tools/profile_box.sh" r04xf/c2 --config c2
rc=$?
tail -2 "$OUT/gpu_tests.log"; cat "$OUT/smoke.log" "$OUT"/c*/bench.json 2>/dev/null
exit $rc
