set -u
# one replayed step of base and Conformer, kernel by kernel, every GEMM launch listed
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r06h; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tb -o kt -- python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline \
  --no-parity --no-roofline --no-conformer > $O/base.log 2>&1 || { tail -20 $O/base.log; exit 1; }
python3 tools/step_breakdown.py $O/tb 8 60 --gemm > $O/base_replay_step.txt 2>&1; head -3 $O/base_replay_step.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc -o kt -- python3 bench.py --config conformer --steps 8 --warmup 3 \
  --no-cpu-baseline --no-parity --no-roofline > $O/conf.log 2>&1 || { tail -20 $O/conf.log; exit 1; }
python3 tools/step_breakdown.py $O/tc 8 60 --gemm > $O/conformer_replay_step.txt 2>&1; head -3 $O/conformer_replay_step.txt
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
