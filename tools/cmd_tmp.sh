set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bf16_err.py conformer 32 > gpurun_out/bf16err.log 2>&1 || { tail -20 gpurun_out/bf16err.log; exit 1; }
grep rel gpurun_out/bf16err.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t.log 2>&1 || { tail -40 gpurun_out/t.log; exit 1; }
tail -2 gpurun_out/t.log
