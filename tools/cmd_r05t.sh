set -u
# LayerDrop skip-gradient fold + LN parameter-reduce / partial layout: tests, step A/B, and a Conformer
# replay trace dumped around the remaining torch kernels and casts
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layerdrop_gpu.py tests/test_kernels_gpu.py tests/test_trainer_gpu.py -x -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
for C in base conformer; do
  for V in 0 1; do
    B2P_LD_SKIP_FOLD=$V timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
      --no-conformer --no-extra --no-roofline > $O/b_${C}_$V.json 2> $O/b_${C}_$V.err || { tail -5 $O/b_${C}_$V.err; exit 1; }
    echo "$C LD_SKIP_FOLD=$V $(python3 -c "import json; print(json.loads(open('$O/b_${C}_$V.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_conf -o kt -- python3 bench.py --config conformer --steps 3 --warmup 2 \
  --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/tconf.json 2> $O/tconf.err || { tail -20 $O/tconf.err; exit 1; }
python3 tools/step_dump.py $O/t_conf "at::native,rocclr,cast16_2d,conv_perm,i64_fill" 3 > $O/conf_step_dump.txt 2>&1; head -5 $O/conf_step_dump.txt
python3 tools/replay_summary.py $O/t_conf 2 60 > $O/conf_summary.txt 2>&1
find $O/t_conf -name "*.db" -delete; find $O/t_conf -name "*trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_base -o kt -- python3 bench.py --steps 3 --warmup 2 \
  --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/tbase.json 2> $O/tbase.err || { tail -20 $O/tbase.err; exit 1; }
python3 tools/step_dump.py $O/t_base "at::native,rocclr,cast16_2d,conv_perm,i64_fill,pad_rows16" 3 > $O/base_step_dump.txt 2>&1
find $O/t_base -name "*.db" -delete; find $O/t_base -name "*trace.csv" -delete
echo DONE
