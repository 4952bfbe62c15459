set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -30 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json | cut -c1-200
