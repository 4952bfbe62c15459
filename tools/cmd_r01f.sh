set -u
# Round profile r01f: GPU parity tests, then the base round profile (PMC traffic, kernel stats, bench line).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r01f_pytest_gpu.log 2>&1 \
  || { tail -30 gpurun_out/r01f_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r01f_pytest_gpu.log
bash tools/round_profile.sh r01f > gpurun_out/r01f_profile.out 2>&1 || { tail -20 gpurun_out/r01f_profile.out; exit 1; }
tail -3 gpurun_out/r01f_profile.out
