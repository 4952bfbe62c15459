set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "pos_conv or step_matches_reference_golden or full_size" > gpurun_out/pc_tests.log 2>&1 || { tail -40 gpurun_out/pc_tests.log; exit 1; }
tail -5 gpurun_out/pc_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
