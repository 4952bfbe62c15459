set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_kernels_gpu.py -m gpu -k "conf or step_graph" > gpurun_out/t2.log 2>&1 || { tail -40 gpurun_out/t2.log; exit 1; }
tail -2 gpurun_out/t2.log
timeout -k 10 300 python -u bench.py --config conformer --no-cpu-baseline > gpurun_out/bc.log 2>&1 || { tail -30 gpurun_out/bc.log; exit 1; }
tail -1 gpurun_out/bc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['ctc_loss'], d['roofline']['achieved'])"
