set -u
# configs[4]: the GRU layers in the bf16 mode under the bf16x3 policy (form gru1): timed replayed steps +
# trajectory (tools/ft_policy_ab.py), then the trajectory test with that policy. usage: bash tools/cmd_ft_gru.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ft_gru}; mkdir -p $O
timeout -k 10 500 python3 -u tools/ft_policy_ab.py "wgrad,grurec1;grurec1" > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep single_pass $O/ab.log
B2P_X3_POLICY=wgrad,grurec1 timeout -k 10 600 python3 -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_configs34_gpu.py -k ft_bs8 > $O/tests.log 2>&1; rc=$?
grep -E "ft_bs8.*(rel|sign-lost)|passed|failed" $O/tests.log | tail -6
exit $rc
