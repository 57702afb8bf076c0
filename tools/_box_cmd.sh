mkdir -p gpurun_out/wirent
timeout -k 10 300 python -u -m pytest tests/test_gpu_wire.py tests/test_gpu_filter.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wirent/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_paths.py --config c3 --wire-variants 4 > gpurun_out/wirent/c3.json 2>/dev/null &&
timeout -k 10 300 python tools/bench_paths.py --config c4 --wire-variants 4 > gpurun_out/wirent/c4.json 2>/dev/null &&
timeout -k 10 300 python tools/bench_paths.py --config c2 > gpurun_out/wirent/c2.json 2>/dev/null
