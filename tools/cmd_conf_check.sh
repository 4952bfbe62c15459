set -u
# Conformer numerics + step profile after a Conformer-path change: bash tools/cmd_conf_check.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-conf}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_configs34_gpu.py tests/test_model_gpu.py tests/test_kernels_gpu.py -x -v -s --timeout 200 --timeout-method thread -k "conformer" > $O/pytest.log 2>&1 || { grep -E "FAILED|Error|rel \[" $O/pytest.log | tail -20; tail -5 $O/pytest.log; exit 1; }
grep -E "rel \[|worst relative" $O/pytest.log | tail -8
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python bench.py --config conformer --steps 5 --warmup 3 --no-parity --no-cpu-baseline --no-roofline > $O/bench.log 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
