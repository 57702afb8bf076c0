mkdir -p gpurun_out/dec
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "decv" > gpurun_out/dec/tests.log 2>&1 &&
timeout -k 10 200 python tools/ab_decode.py --config c3 > gpurun_out/dec/c3.json 2>/dev/null &&
timeout -k 10 200 python tools/ab_decode.py --config c4 > gpurun_out/dec/c4.json 2>/dev/null &&
timeout -k 10 200 python tools/ab_decode.py --config c2 > gpurun_out/dec/c2.json 2>/dev/null
