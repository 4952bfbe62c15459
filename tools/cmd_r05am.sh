set -u
# device lens / CTC targets / cached loss seed: tests and step times; attention times + PMC at HEAD; GEMM
# family HBM traffic at HEAD (FETCH_SIZE / WRITE_SIZE passes, hipBLASLt launches included)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05am; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py::test_unfold_lens_and_ctc_targets_match_reference_expressions \
  tests/test_model_gpu.py tests/test_trainer_gpu.py tests/test_experiment_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for C in base conformer; do
  timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity --no-conformer --no-extra \
    --no-roofline > $O/b_$C.json 2> $O/b_$C.err || { tail -5 $O/b_$C.err; exit 1; }
  echo "$C $(python3 -c "import json; print(json.loads(open('$O/b_$C.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
bash tools/cmd_r05al.sh || exit 1
for C in base conformer; do
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$C -o pmc -- python3 bench.py --config $C --steps 2 --warmup 1 \
    --no-cpu-baseline --no-parity --no-conformer --no-extra > $O/pf_$C.log 2>&1 || { tail -5 $O/pf_$C.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/pw_$C -o pmc -- python3 bench.py --config $C --steps 2 --warmup 1 \
    --no-cpu-baseline --no-parity --no-conformer --no-extra > $O/pw_$C.log 2>&1 || { tail -5 $O/pw_$C.log; exit 1; }
  SUF=$([ $C = base ] && echo "" || echo "_conformer")
  python3 tools/traffic.py $(find $O/pf_$C -name "*.db" | head -1) $(find $O/pw_$C -name "*.db" | head -1) $O/gemm_traffic$SUF.json
  find $O -name "*.db" -delete
  cat $O/gemm_traffic$SUF.json | grep traffic_bytes
done
