set -u
# 4-wave 256x256 kernel: tile-config test, then gemm_ab default / W4=1 / W4=2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-w4}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread -k "tile_configs" > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab.log 2>&1 && tail -16 $O/gemm_ab.log
B2P_GEMM16_W4=1 timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab_w41.log 2>&1 && tail -16 $O/gemm_ab_w41.log
B2P_GEMM16_W4=2 timeout -k 10 200 python -u tools/gemm_ab.py > $O/gemm_ab_w42.log 2>&1 && tail -16 $O/gemm_ab_w42.log
