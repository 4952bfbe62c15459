set -e
mkdir -p gpurun_out
for e in "B2P_DIAG_SKIP_SMALL_ACC=0" "B2P_DIAG_SKIP_SMALL_ACC=1"; do
env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1 || { tail -30 gpurun_out/b.log; exit 1; }
echo $e $(tail -1 gpurun_out/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
done
