set -u
# HIP graph executor switches vs when the frozen weight-gradient branch starts (base replay traces) and
# the untraced step time of each
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05ai; mkdir -p $O
tr() {  # tag env...
  local tag=$1; shift
  env B2P_ATTN_KEEP_AHEAD=0 "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_$tag -o kt -- python3 bench.py --steps 8 \
    --warmup 3 --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/$tag.log 2>&1 \
    || { tail -20 $O/$tag.log; return 1; }
  python3 tools/step_timeline.py $O/t_$tag 8 15 > $O/${tag}_timeline.txt 2>&1
  echo "== $tag: $(head -1 $O/${tag}_timeline.txt)"; grep -E "gru16_bwd|513u|adam_gated" $O/${tag}_timeline.txt | cut -c1-110
  env B2P_ATTN_KEEP_AHEAD=0 "$@" timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-roofline --no-conformer --no-extra > $O/b_$tag.json 2>$O/b_$tag.err || { tail -5 $O/b_$tag.err; return 1; }
  echo "$tag untraced $(python3 -c "import json; print(json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
}
tr pc0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 && tr gq8 DEBUG_HIP_FORCE_GRAPH_QUEUES=8 && tr gq2 DEBUG_HIP_FORCE_GRAPH_QUEUES=2 || exit 1
find $O -name "*.db" -delete; find $O -name "*.csv" -delete
