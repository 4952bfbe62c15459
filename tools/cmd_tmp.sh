set -e
mkdir -p gpurun_out
export LD_LIBRARY_PATH=$PWD/wav2vec2forbrain_amd:$LD_LIBRARY_PATH
for s in "7968 1536 8192 0" "7968 3072 768 2 1"; do
  timeout -k 10 60 tools/_bin/pp_probe $s 2>&1 | grep "us/launch" >> gpurun_out/pp_var.txt
  B2P_GEMM16_PP=0 timeout -k 10 60 tools/_bin/pp_probe $s 2>&1 | grep "us/launch" | sed 's/^/small /' >> gpurun_out/pp_var.txt
done
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
