mkdir -p gpurun_out/c5
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c5/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/c5/bench_c5.json 2> gpurun_out/c5/bench_c5.err
