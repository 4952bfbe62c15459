set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | cut -c1-300
