"""One bench workload's Trainer steps, eager (no graph replay), for the rocprofv3 --pmc passes of
tools/traffic.py (round_profile-style GEMM traffic per launch): usage
    B2P_SERIAL_SIDE=1 rocprofv3 --pmc FETCH_SIZE -d <dir> -o pmc -- python3 tools/traffic_run.py <kind>
kind: base | conformer | large | conformer_ft (bench.py's timed_run kinds: configs[1] .. configs[4])."""
import argparse
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "base"
args = argparse.Namespace(gpus=1, steps=2, warmup=1, bs=32, seq=1024, no_cpu_baseline=True, no_parity=True,
                          no_roofline=True, no_conformer=True, no_extra=True, evaluator=False, graph=0, config="base")
r = bench.timed_run(kind, args, 1, 0, "cuda:0", False, steps=2, warmup=1, roofline=False)
print(kind, r["precision"], r["step_mode"], round(r["dt"] / r["steps"] * 1e3, 2), "ms/step")
