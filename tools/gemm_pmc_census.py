"""Per-shape GEMM table of one eager bench training step: launch shapes (functional.GEMM_LOG) zipped,
in launch order, with rocprofv3 per-dispatch PMC counters and durations. One counter set per
rocprofv3 pass (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass).

  python tools/gemm_pmc_census.py run <outdir>                 (the profiled program)
  python tools/gemm_pmc_census.py report <outdir> <db> [<db> ...] > table.txt

Columns per shape (mean per launch): time, TF/s, algorithmic operand + output bytes, HBM bytes
(FETCH_SIZE x 2, the gfx950 wide-read correction, + WRITE_SIZE), and the SQ busy / instruction
counters present in the databases."""
import collections
import json
import os
import sqlite3
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(out):
    import torch
    from wav2vec2forbrain_amd import build_lib
    build_lib.ensure_built()
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import bench_config, build_model, device_batch, SyntheticStepExperiment
    Fn.set_precision("bf16")
    cfg = bench_config(os.environ.get("CENSUS_CONFIG", "base"))
    model = build_model(cfg, "cuda", train_dropouts=True)
    model.train()
    model.sync_metrics = False
    trainer = Trainer(SyntheticStepExperiment(model))
    batch = device_batch(cfg)
    for _ in range(2):
        trainer._eager_body(batch)
    torch.cuda.synchronize()
    Fn.GEMM_LOG = []
    trainer._eager_body(batch)
    torch.cuda.synchronize()
    os.makedirs(out, exist_ok=True)
    json.dump(Fn.GEMM_LOG, open(os.path.join(out, "gemm_log.json"), "w"))
    print(f"logged {len(Fn.GEMM_LOG)} gemm calls")


GEMM_KERNELS = ("gemm_kernel<", "gemm16_kernel<", "gemm16_pp_kernel<", "gemm16_pn_kernel<")


def _dispatches(db):
    """[(dispatch_id, kernel_name, duration_ns, {counter: value})] of the GEMM kernels, issue order."""
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, sum(value), max(end - start) "
                     "from counters_collection group by dispatch_id, counter_name order by dispatch_id").fetchall()
    d = collections.OrderedDict()
    for did, name, cn, v, dur in rows:
        if not any(k in name for k in GEMM_KERNELS):
            continue
        e = d.setdefault(did, [did, name, dur, {}])
        e[3][cn] = v
    return list(d.values())


def _key(rec):
    return (f"{rec['M']}x{rec['N']}x{rec['K']}" + (f"*{rec['nz']}" if rec['nz'] > 1 else "")
            + f" {'A' if rec['ak'] else 'a'}{'B' if rec['bk'] else 'b'}" + (" bf16" if rec["a16"] else " f32")
            + (" convA" if rec["aconv"] else "") + (f" ks{rec['ksplit']}" if rec["ksplit"] > 1 else "")
            + f" [{rec['epi']}]")


def _alg_bytes(rec):
    """Operand + output bytes one launch must move at least once: A and B at their element size, C at
    4 B if written in fp32, 2 B per 16-bit output (C16 / pre16), + residual / aux reads."""
    M, N, K, nz = rec["M"], rec["N"], rec["K"], rec["nz"]
    el = 2 if rec["a16"] else 4
    b = (M * K + K * N) * el * nz
    out = rec.get("out_bytes")
    if out is None:
        out = 4 * M * N * nz
    return b + out


def report(out, dbs):
    log = json.load(open(os.path.join(out, "gemm_log.json")))
    per = collections.OrderedDict()
    for db in dbs:
        ds = _dispatches(db)[-len(log):]
        if len(ds) != len(log):
            raise SystemExit(f"{db}: {len(ds)} GEMM dispatches for {len(log)} logged calls")
        for rec, (did, name, dur, cnt) in zip(log, ds):
            a = per.setdefault(_key(rec), {"n": 0, "rec": rec, "dur": [], "cnt": collections.defaultdict(list)})
            if db == dbs[0]:
                a["n"] += 1
            a["dur"].append(dur)
            for cn, v in cnt.items():
                a["cnt"][cn].append(v)
    cols = sorted({cn for a in per.values() for cn in a["cnt"]})
    hdr = ["ms_tot", "n", "us", "TF/s", "alg_MB", "hbm_MB", "hbm/alg"] + [c for c in cols if c not in ("FETCH_SIZE", "WRITE_SIZE")]
    print("shape".ljust(46) + "  " + "  ".join(h.rjust(10) for h in hdr))
    tot_ms = 0.0
    for k, a in sorted(per.items(), key=lambda kv: -sum(kv[1]["dur"]) / len(dbs)):
        rec = a["rec"]
        us = sum(a["dur"]) / len(a["dur"]) / 1e3
        fl = 2.0 * rec["M"] * rec["N"] * rec["K"] * rec["nz"]
        mean = {cn: sum(v) / len(v) for cn, v in a["cnt"].items()}
        hbm = None
        if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
            hbm = (2 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024   # counters are in KB
        alg = _alg_bytes(rec)
        ms_tot = us * a["n"] / 1e3
        tot_ms += ms_tot
        vals = [f"{ms_tot:.3f}", str(a["n"]), f"{us:.1f}", f"{fl / us / 1e6:.0f}", f"{alg / 1e6:.1f}",
                "-" if hbm is None else f"{hbm / 1e6:.1f}", "-" if hbm is None else f"{hbm / alg:.2f}"]
        vals += [f"{mean[c]:.4g}" if c in mean else "-" for c in hdr[7:]]
        print(k[:46].ljust(46) + "  " + "  ".join(v.rjust(10) for v in vals))
    print(f"total GEMM time of the step (profiled): {tot_ms:.2f} ms")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        report(sys.argv[2], sys.argv[3:])
