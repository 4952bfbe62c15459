set -u
# scaled FFN bias cached, pos-conv fast-path gradients through the deferred accumulation, CTC backward
# scale on the device; hipBLASLt kernel names on the yardstick shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r05w; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_trainer_gpu.py tests/test_layerdrop_gpu.py -x -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" $O/tests.log | head -20; exit $rc; }
for C in base conformer; do
  timeout -k 10 300 python3 bench.py --config $C --steps 20 --warmup 5 --no-cpu-baseline --no-parity \
    --no-conformer --no-extra --no-roofline > $O/b_$C.json 2> $O/b_$C.err || { tail -5 $O/b_$C.err; exit 1; }
  echo "$C $(python3 -c "import json; print(json.loads(open('$O/b_$C.json').read().strip().splitlines()[-1])['ms_per_step'])") ms"
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t_base -o kt -- python3 bench.py --steps 3 --warmup 2 \
  --no-cpu-baseline --no-parity --no-roofline --no-conformer --no-extra > $O/tbase.json 2> $O/tbase.err || { tail -20 $O/tbase.err; exit 1; }
python3 tools/step_dump.py $O/t_base "at::native,rocclr" 2 > $O/base_step_dump.txt 2>&1; grep -c "^>" $O/base_step_dump.txt
find $O/t_base -name "*.db" -delete; find $O/t_base -name "*trace.csv" -delete
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/blas -o blas -- python3 tools/gemm_vs_blas.py > $O/gemm_vs_blas.txt 2>&1 || { tail -5 $O/gemm_vs_blas.txt; exit 1; }
python3 tools/kernel_names.py $O/blas Cijk > $O/blas_kernels.txt 2>&1; head -30 $O/blas_kernels.txt | cut -c1-250
find $O/blas -name "*.db" -delete; find $O/blas -name "*trace.csv" -delete
echo DONE
