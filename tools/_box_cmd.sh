mkdir -p gpurun_out/autont3
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/autont3/tests.log 2>&1 &&
timeout -k 10 200 python tools/ab_encode.py --config c3 --variants 0,20,18 --pads 16,0 > gpurun_out/autont3/c3.json 2>/dev/null &&
timeout -k 10 200 python tools/ab_encode.py --config c4 --variants 0,20,18 --pads 16,0 > gpurun_out/autont3/c4.json 2>/dev/null &&
timeout -k 10 200 python tools/ab_encode.py --config c2 --variants 0,20,18 --pads 16,0 > gpurun_out/autont3/c2.json 2>/dev/null &&
bash tools/profile_box.sh r01d
