set -u
# SiLU through v_rcp_f32 in the 16-bit GEMM register epilogue: epilogue A/B on the Conformer FFN shape
# (IEEE-division library copy vs the new one), model / trajectory tests, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06q; mkdir -p $O
export B2P_EPI_VARIANTS=bH,bsH,bsdH,bsdHB,gh,gdh
B2P_LIB_PATH=probe_bin/libb2p_hip_ieee.so timeout -k 10 200 python3 tools/epi_ab.py 7968 4096 1024 > $O/epi_ieee.log 2>&1 || { tail $O/epi_ieee.log; exit 1; }
timeout -k 10 200 python3 tools/epi_ab.py 7968 4096 1024 > $O/epi_fast.log 2>&1 || { tail $O/epi_fast.log; exit 1; }
unset B2P_EPI_VARIANTS
grep -v amdgpu.ids $O/epi_ieee.log $O/epi_fast.log
timeout -k 10 600 python3 -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_configs34_gpu.py -k "conformer" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "conformer.*rel|passed|failed" $O/tests.log | tail -12
bash tools/cmd_ab_env.sh r06q_step "B2P_LIB_PATH=probe_bin/libb2p_hip_ieee.so" || exit 1
