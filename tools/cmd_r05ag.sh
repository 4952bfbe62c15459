set -u
# keep masks with an LDS request (no co-residency with the GRU): step-time A/B, base and Conformer timelines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ag; mkdir -p $O
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
run base_ka1 base B2P_ATTN_KEEP_AHEAD=1 && run base_ka0 base B2P_ATTN_KEEP_AHEAD=0 && run base_ka1b base B2P_ATTN_KEEP_AHEAD=1 && \
run conf_ka1 conformer B2P_ATTN_KEEP_AHEAD=1 && run conf_ka0 conformer B2P_ATTN_KEEP_AHEAD=0 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tb -o kt -- python3 bench.py --steps 8 --warmup 3 --no-cpu-baseline \
  --no-parity --no-roofline --no-conformer --no-extra > $O/base.log 2>&1 || { tail -20 $O/base.log; exit 1; }
python3 tools/step_timeline.py $O/tb 8 15 > $O/base_timeline.txt 2>&1; tail -1 $O/base_timeline.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tc -o kt -- python3 bench.py --config conformer --steps 8 --warmup 3 \
  --no-cpu-baseline --no-parity --no-roofline --no-extra > $O/conf.log 2>&1 || { tail -20 $O/conf.log; exit 1; }
python3 tools/step_breakdown.py $O/tc 8 60 > $O/conformer_replay_step.txt 2>&1; head -1 $O/conformer_replay_step.txt
python3 tools/step_timeline.py $O/tc 8 40 > $O/conformer_timeline.txt 2>&1; tail -1 $O/conformer_timeline.txt
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
