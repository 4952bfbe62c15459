set -u
# Round-end evidence on one fresh box: the driver's commands (pytest -m gpu, smoke, default bench line), one
# replayed step per config kernel by kernel, and the rocprofv3 --kernel-trace --stats summary of a bench run
# (GEMM-family mean launch time beside bench.py's HIP-event figure). usage: bash tools/cmd_final.sh <tag>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-final}
# SKIP_REHEARSAL=1: only the profiles (the rehearsal already ran on this tree)
[ "${SKIP_REHEARSAL:-0}" = 1 ] || bash tools/cmd_rehearsal.sh $T || exit 1
mkdir -p gpurun_out/$T
O=gpurun_out/$T
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline \
  --no-parity --no-conformer --no-extra > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof 6 40 > $O/prof_summary_base.txt 2>&1
python3 - "$O" <<'PY' >> $O/prof_summary_base.txt
import json, sys
sys.path.insert(0, "tools")
from prof_summary import rows_from   # the stats csv, or the rocpd database's top_kernels view
o = sys.argv[1]
g = [r for r in rows_from(f"{o}/prof") if any(k in r[0] for k in ("gemm16_kernel<", "gemm_kernel<", "gemm16_pp_kernel<", "gemm16_pn_kernel<"))]
calls = sum(r[1] for r in g); tot = sum(r[2] for r in g)
line = [l for l in open(f"{o}/prof.log") if l.startswith("{")][-1]
b = json.loads(line)["roofline"]
print(f"GEMM family under rocprofv3: {calls} launches, mean {tot / calls / 1e3:.2f} us; bench.py HIP events in the same run: "
      f"{b['launches']} launches, mean {b['avg_launch_us']} us, frac {b['frac']}")
PY
tail -1 $O/prof_summary_base.txt
find $O/prof -name "*.db" -delete; find $O/prof -name "*kernel_trace.csv" -delete
[ "${SKIP_BREAKDOWN:-0}" = 1 ] || bash tools/cmd_step_breakdown.sh $T || exit 1
