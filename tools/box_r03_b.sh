#!/bin/bash
# Runs ON THE GPU BOX: C4 and C2 bench + rocprofv3 stats + PMC passes, then the host-resident rates.
set -o pipefail
TAG=${1:-r03x}
O=gpurun_out/$TAG
mkdir -p $O
bash tools/profile_box.sh $TAG/c4 --config c4 || { echo profile c4 failed; exit 1; }
cat $O/c4/bench.json
bash tools/profile_box.sh $TAG/c2 --config c2 || { echo profile c2 failed; exit 1; }
cat $O/c2/bench.json
timeout -k 10 300 python tools/bench_host.py > $O/host.json 2> $O/host.err || { echo bench_host failed; tail $O/host.err; exit 1; }
cat $O/host.json
timeout -k 10 300 python tools/bench_pcap_host.py > $O/pcap_host.json 2> $O/pcap_host.err || { echo bench_pcap_host failed; tail $O/pcap_host.err; exit 1; }
cat $O/pcap_host.json
