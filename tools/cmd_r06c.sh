set -u
# asm LDS-DMA + buffer-resource operands in the ping-pong GEMM, attention VGPR form + keep LUT: GEMM and kernel
# tests, the attention bench, then one replayed step of base
# and Conformer kernel by kernel with every GEMM launch listed
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_wgrad_batch_gpu.py tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/pytest.log | tail; exit $rc; }
timeout -k 10 120 python3 tools/attn_bench.py > $O/attn_bench.txt 2>&1 || { tail -5 $O/attn_bench.txt; exit 1; }; grep attn16 $O/attn_bench.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tb -o kt -- python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline \
  --no-parity --no-roofline --no-conformer > $O/base.log 2>&1 || { tail -20 $O/base.log; exit 1; }
python3 tools/step_breakdown.py $O/tb 8 40 --gemm > $O/base_replay_step.txt 2>&1; head -3 $O/base_replay_step.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc -o kt -- python3 bench.py --config conformer --steps 8 --warmup 3 \
  --no-cpu-baseline --no-parity --no-roofline > $O/conf.log 2>&1 || { tail -20 $O/conf.log; exit 1; }
python3 tools/step_breakdown.py $O/tc 8 40 --gemm > $O/conformer_replay_step.txt 2>&1; head -3 $O/conformer_replay_step.txt
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
grep -E '"value"' $O/base.log $O/conf.log | cut -c1-200
