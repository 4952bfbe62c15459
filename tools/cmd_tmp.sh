set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "seed_epoch or step_graph or deferred or adam" > gpurun_out/graph_tests.log 2>&1 || { tail -40 gpurun_out/graph_tests.log; exit 1; }
tail -5 gpurun_out/graph_tests.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
