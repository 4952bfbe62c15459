set -u
# colsum 32-row bands + B-fragment keep (TN): GEMM / model tests, TN A/B (variant 1 = no keep), epilogue A/B, bench
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06j; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gemm_gpu.py \
  tests/test_wgrad_batch_gpu.py tests/test_model_gpu.py tests/test_layerdrop_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
GEMM_AB_ONLY=3072x768x7968,768x768x7968,4096x1024x7968 timeout -k 10 120 python3 tools/gemm_ab.py > $O/ab_keep.log 2>&1 || { tail $O/ab_keep.log; exit 1; }
B2P_GEMM16_VARIANT=1 GEMM_AB_ONLY=3072x768x7968,768x768x7968,4096x1024x7968 timeout -k 10 120 python3 tools/gemm_ab.py > $O/ab_nokeep.log 2>&1 || exit 1
GEMM_AB_ONLY=3072x768x7968,768x768x7968,4096x1024x7968 timeout -k 10 120 python3 tools/gemm_ab.py >> $O/ab_keep.log 2>&1 || exit 1
B2P_GEMM16_VARIANT=1 GEMM_AB_ONLY=3072x768x7968,768x768x7968,4096x1024x7968 timeout -k 10 120 python3 tools/gemm_ab.py >> $O/ab_nokeep.log 2>&1 || exit 1
cat $O/ab_keep.log $O/ab_nokeep.log
timeout -k 10 200 python3 tools/epi_ab.py 7968 3072 768 > $O/epi.log 2>&1 || { tail $O/epi.log; exit 1; }
tail -12 $O/epi.log
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -3 $O/bench.log
