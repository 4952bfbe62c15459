set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05o; mkdir -p $O
for C in conformer base; do for V in 1000000000 256; do
  B2P_PP_SPLIT_MAX_BLOCKS=$V timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_${C}_$V.json 2> $O/b_${C}_$V.err || { tail -5 $O/b_${C}_$V.err; exit 1; }
  echo "$C PP_SPLIT_MAX_BLOCKS=$V $(python3 -c "import json; print(json.loads(open('$O/b_${C}_$V.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done; done
