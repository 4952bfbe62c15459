"""Per-GEMM-call census of one bench training step: shapes logged by functional.gemm in launch order,
zipped with the rocprofv3 kernel trace of the same step. Two modes:
  python tools/gemm_census.py run <outdir>      (the profiled program: warm-up + 1 logged step)
  python tools/gemm_census.py report <outdir>   (after rocprofv3 --kernel-trace --output-format csv)"""
import csv
import glob
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    import torch
    import bench
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.optim import HipAdam
    Fn.set_precision("bf16")
    cfg = bench.make_config(32, 1024, os.environ.get("CENSUS_CONFIG", "base"))
    model = bench.build(cfg, "cuda")
    model.train()
    opt = HipAdam(model.brain_encoder.parameters(), lr=1e-3)
    batch = bench.batch_on(cfg, "cuda")

    def step():
        opt.zero_grad()
        out = model(batch)
        out.loss.backward()
        opt.step()

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    Fn.GEMM_LOG = []
    step()
    torch.cuda.synchronize()
    os.makedirs(out, exist_ok=True)
    json.dump(Fn.GEMM_LOG, open(os.path.join(out, "gemm_log.json"), "w"))
    print(f"logged {len(Fn.GEMM_LOG)} gemm calls")


def report(out):
    log = json.load(open(os.path.join(out, "gemm_log.json")))
    f = glob.glob(os.path.join(out, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    gem = [r for r in rows if "gemm_kernel<" in r["Kernel_Name"] or "gemm16_kernel<" in r["Kernel_Name"]
           or "gemm16_pp_kernel<" in r["Kernel_Name"]]
    red = [r for r in rows if "splitk_reduce" in r["Kernel_Name"]]
    gem = gem[-len(log):]
    agg = {}
    tot = 0.0
    for rec, r in zip(log, gem):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        key = (f"{rec['M']}x{rec['N']}x{rec['K']}" + (f"*{rec['nz']}" if rec['nz'] > 1 else "")
               + f" {'A' if rec['ak'] else 'a'}{'B' if rec['bk'] else 'b'}" + (" bf16" if rec["a16"] else " f32")
               + (" convA" if rec["aconv"] else "") + (" convB" if rec["bconv"] else "")
               + (f" ks{rec['ksplit']}" if rec["ksplit"] > 1 else "") + f" [{rec['epi']}]")
        fl = 2.0 * rec["M"] * rec["N"] * rec["K"] * rec["nz"]
        a = agg.setdefault(key, [0, 0.0, 0.0, r["Kernel_Name"][:60]])
        a[0] += 1
        a[1] += us
        a[2] += fl
        tot += us
    print(f"{len(log)} gemm calls, {tot / 1e3:.2f} ms GEMM time in the logged step; "
          f"{len(red)} splitk_reduce dispatches in the trace")
    for k, (n, us, fl, kn) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        print(f"{us / 1e3:7.3f} ms {n:3d}x {us / n:8.1f} us {fl / us / 1e6:7.1f} TF/s  {k}  <{kn}>")


if __name__ == "__main__":
    {"run": run, "report": report}[sys.argv[1]](sys.argv[2])
