set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/grumc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "gru" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 120 python tools/gru512_bench.py > $O/mc.txt 2>&1 || { tail -20 $O/mc.txt; exit 1; }
echo "multi-CU:"; tail -1 $O/mc.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config conformer --steps 3 --warmup 2 --no-cpu-baseline --no-parity --no-roofline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof adam 1 > $O/timeline.txt 2>&1
head -45 $O/timeline.txt
