set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05y; mkdir -p $O
timeout -k 10 200 python3 tools/blaslt_ab.py > $O/ab_ws0.txt 2>&1 || { tail -5 $O/ab_ws0.txt; exit 1; }; cat $O/ab_ws0.txt
B2P_BLASLT_WS=64 timeout -k 10 200 python3 tools/blaslt_ab.py > $O/ab_ws64.txt 2>&1 || { tail -5 $O/ab_ws64.txt; exit 1; }; echo ws64; cat $O/ab_ws64.txt
for V in 0 64; do
  B2P_BLASLT_WS=$V timeout -k 10 300 python3 bench.py --config base --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$V.json 2> $O/b_$V.err || { tail -5 $O/b_$V.err; exit 1; }
  echo "base WS=$V $(python3 -c "import json; print(json.loads(open('$O/b_$V.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
