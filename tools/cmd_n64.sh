set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/n64; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 0 1; do
  B2P_GEMM16_N64=$v timeout -k 10 120 python tools/bench_gemm.py b16 > $O/g$v.jsonl 2> $O/g$v.err || { tail -5 $O/g$v.err; exit 1; }
  echo "== N64=$v"; head -9 $O/g$v.jsonl
done
for v in 0 1; do
  B2P_GEMM16_N64=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-parity > $O/b$v.json 2> $O/b$v.err || { tail -5 $O/b$v.err; exit 1; }
  echo "== bench N64=$v"; tail -1 $O/b$v.json | cut -c1-200
done
B2P_GEMM16_N64=1 timeout -k 10 300 python bench.py --config conformer --no-cpu-baseline --no-parity --steps 10 --warmup 3 > $O/c1.json 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
echo "== conformer N64=1"; tail -1 $O/c1.json | cut -c1-200
