mkdir -p gpurun_out/slots
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_wire.py -x -q --timeout 120 --timeout-method thread -k "slots or parse_decode or wire" > gpurun_out/slots/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_pcap_host.py > gpurun_out/slots/pcap_host.json 2> gpurun_out/slots/pcap_host.err
