set -u
# when do the frozen weight-gradient launches start relative to the GRU backward? base step traced as a
# replay (default), as an eager step (--graph 0) and as a replay with 8 hardware queues per process
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ah; mkdir -p $O
tr() {  # tag env... -- extra bench args
  local tag=$1; shift
  env B2P_ATTN_KEEP_AHEAD=0 "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_$tag -o kt -- python3 bench.py --steps 8 \
    --warmup 3 --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra $EXTRA > $O/$tag.log 2>&1 \
    || { tail -20 $O/$tag.log; return 1; }
  python3 tools/step_timeline.py $O/t_$tag 8 15 > $O/${tag}_timeline.txt 2>&1
  echo "== $tag: $(head -1 $O/${tag}_timeline.txt)"; grep -E "gru16_bwd|513u|adam_gated" $O/${tag}_timeline.txt | cut -c1-120
}
EXTRA="" tr graph && EXTRA="--graph 0" tr eager && EXTRA="" tr q8 GPU_MAX_HW_QUEUES=8 || exit 1
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
