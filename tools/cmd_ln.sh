cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ln
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "layernorm or ln or encoder_layer" > gpurun_out/ln/pytest.log 2>&1 || { tail -20 gpurun_out/ln/pytest.log; exit 1; }
tail -2 gpurun_out/ln/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ln/prof -o run -- python bench.py --config conformer --steps 5 --warmup 3 --no-parity --no-cpu-baseline --no-roofline > gpurun_out/ln/bench.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/ln/bench.log
f=$(find gpurun_out/ln/prof -name "*kernel_stats.csv" | head -1)
grep -E "ln_|Name" "$f" | cut -d, -f1-8
