set -u
# configs[4] policy: two-term split images per role (timed replayed steps + trajectory vs the reference)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06m; mkdir -p $O
timeout -k 10 600 python3 -u tools/ft_policy_ab.py "wgrad;wgrad,fwd2a;wgrad,fwd2b;wgrad,dgrad2a;wgrad,dgrad2b;wgrad,fwd2a,dgrad2a" > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep single_pass $O/ab.log
# frozen weight gradients flushed per encoder block, unsplit (few long workgroups beside the main stream)
bash tools/cmd_ab_env.sh r06m_flush "B2P_WGRAD_FLUSH=block B2P_DEFER_SPLIT=0" "B2P_WGRAD_FLUSH=block" || exit 1
