timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r01c.log 2>&1 &&
bash tools/profile_box.sh r01c
