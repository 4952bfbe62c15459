"""configs[4] per GPU (Conformer-large, whole encoder trained, bs 8): timed replayed Trainer steps and the
3-step trajectory against the reference's (tests/golden/conformer_large_ft_bs8.npz) for each set of
bf16x3 roles run single-pass or on two-term images (functional.X3_POLICY_FORMS: fwd / dgrad / wgrad,
suffix 1 = single pass, 2a / 2b = two-term images, see functional._x3_form).
usage: python tools/ft_policy_ab.py "<roles>;<roles>;..."   e.g. ";wgrad;wgrad,dgrad2b" ('' = three-term everywhere)"""
import argparse
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from wav2vec2forbrain_amd import functional as Fn  # noqa: E402

sels = (sys.argv[1] if len(sys.argv) > 1 else ";wgrad,dgrad2b").split(";")
args = argparse.Namespace(gpus=1, steps=10, warmup=3, bs=32, seq=1024, no_cpu_baseline=True, no_parity=True,
                          no_roofline=True, no_conformer=True, no_extra=True, evaluator=False, graph=1, config="base")
device = "cuda:0"
for sel in sels:
    Fn.X3_POLICY_FORMS = frozenset(filter(None, sel.split(",")))
    r = bench.timed_run("conformer_ft", args, 1, 0, device, True, steps=10, warmup=3, roofline=False)
    par = bench.fixture_parity("conformer_large_ft_bs8", device)
    print(json.dumps({"single_pass_roles": sel or "-", "precision": r["precision"], "step_mode": r["step_mode"],
                      "ms_per_step": round(r["dt"] / r["steps"] * 1e3, 2), "rel_err": par["rel_err"],
                      "pass": par["pass"]}), flush=True)
