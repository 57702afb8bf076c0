mkdir -p gpurun_out/wire
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wire/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_paths.py --config c3 --wire-variants 4,5,6,7,0 > gpurun_out/wire/c3.json 2>/dev/null &&
timeout -k 10 300 python tools/bench_paths.py --config c4 --wire-variants 4,5,6,7,0 > gpurun_out/wire/c4.json 2>/dev/null &&
timeout -k 10 300 python tools/bench_paths.py --config c2 --wire-variants 4,5,6,7,0 > gpurun_out/wire/c2.json 2>/dev/null
