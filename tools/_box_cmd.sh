mkdir -p gpurun_out/pcap2
timeout -k 10 300 python tools/bench_pcap_host.py > gpurun_out/pcap2/c3.json 2> gpurun_out/pcap2/c3.err &&
timeout -k 10 300 python tools/bench_pcap_host.py --chunk 1048576 > gpurun_out/pcap2/c3_1m.json 2>> gpurun_out/pcap2/c3.err
