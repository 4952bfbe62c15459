set -u
# GRU backward launch order vs the frozen weight-gradient branch (B2P_GRU_BWD_MODE after / first / fork):
# step times (base, Conformer) and base replay timelines
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ak; mkdir -p $O
run() {  # tag config env...
  local tag=$1 C=$2; shift 2
  env B2P_ATTN_KEEP_AHEAD=0 "$@" timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$tag.json 2> $O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag $(python3 -c "import json; d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('ctc_loss'))") ms"
}
tr() {  # tag env...
  local tag=$1; shift
  env B2P_ATTN_KEEP_AHEAD=0 "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_$tag -o kt -- python3 bench.py --steps 8 \
    --warmup 3 --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/$tag.log 2>&1 \
    || { tail -20 $O/$tag.log; return 1; }
  python3 tools/step_timeline.py $O/t_$tag 8 15 > $O/${tag}_timeline.txt 2>&1
  echo "== $tag: $(head -1 $O/${tag}_timeline.txt)"; grep -E "gru16_bwd|513u|adam_gated" $O/${tag}_timeline.txt | cut -c1-110
}
run base_after base && run base_first base B2P_GRU_BWD_MODE=first && run base_fork base B2P_GRU_BWD_MODE=fork && \
tr first B2P_GRU_BWD_MODE=first && tr fork B2P_GRU_BWD_MODE=fork && \
run conf_after conformer && run conf_fork conformer B2P_GRU_BWD_MODE=fork || exit 1
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
