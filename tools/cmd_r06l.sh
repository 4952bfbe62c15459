set -u
# configs[4] policy attribution: bf16x3 with single-pass roles (trajectory vs the reference) + timed steps;
# replayed exact-fp32 figure
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06l; mkdir -p $O
timeout -k 10 300 python3 -u tools/traj_err_ft.py conformer_large_ft_bs8 "M:bf16x3,M:bf16x3/x3f16fwd,M:bf16x3/x3tn1,M:bf16x3/x3nn1,M:bf16x3/x3f16fwd+x3nn1" > $O/traj.log 2>&1 || { tail -30 $O/traj.log; exit 1; }
grep -A1 "loss rel" $O/traj.log
timeout -k 10 400 python3 -u tools/ft_policy_ab.py ";fwd;fwd,dgrad;wgrad" > $O/ab.log 2>&1 || { tail -30 $O/ab.log; exit 1; }
grep single_pass $O/ab.log
timeout -k 10 200 python3 -u -c "
import argparse, json, bench
a = argparse.Namespace(bs=32, seq=1024)
print(json.dumps(bench.fp32_mode_record('base', a, 'cuda:0')))
" > $O/fp32.log 2>&1 || { tail -30 $O/fp32.log; exit 1; }
tail -1 $O/fp32.log
