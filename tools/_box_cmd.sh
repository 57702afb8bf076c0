mkdir -p gpurun_out/pack
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "encv22 or encv23" > gpurun_out/pack/tests.log 2>&1 &&
timeout -k 10 200 python tools/ab_encode.py --config c4 --variants 0,22,23 --pads 16,0 > gpurun_out/pack/c4.json 2>/dev/null &&
timeout -k 10 200 python tools/ab_encode.py --config c3 --variants 0,22,23 --pads 16 > gpurun_out/pack/c3.json 2>/dev/null &&
timeout -k 10 200 python tools/ab_encode.py --config c2 --variants 0,22 --pads 16 > gpurun_out/pack/c2.json 2>/dev/null
