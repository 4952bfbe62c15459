"""Why is the Conformer step slower after a base run in the same process? Each variant runs in its own
subprocess: [what runs first] then timed Conformer Trainer steps (bench.timed_run).
usage: python tools/nested_probe.py [variant ...]"""
import os
import subprocess
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(variant):
    import torch
    import bench
    from wav2vec2forbrain_amd import functional as Fn
    torch.manual_seed(1234)
    Fn.SEEDS.reseed(1234 * 65537)
    Fn.set_precision("bf16")
    args = types.SimpleNamespace(bs=32, seq=1024, steps=8, warmup=3, evaluator=False, no_roofline=True)
    dev = "cuda:0"
    if variant.endswith("_nodefer"):   # frozen-weight gradients in-order on the main stream (no side branch)
        orig = Fn.set_deferred_wgrad
        Fn.set_deferred_wgrad = lambda params: orig([])
        variant = variant[:-len("_nodefer")]
    if variant == "base_graph":
        r = bench.timed_run("base", args, 1, 0, dev, True)
        print(f"{variant}: base {r['dt'] / args.steps * 1e3:.2f} ms", flush=True)
    elif variant == "base_eager":
        r = bench.timed_run("base", args, 1, 0, dev, False)
        print(f"{variant}: base {r['dt'] / args.steps * 1e3:.2f} ms", flush=True)
    elif variant == "conf_twice":
        r = bench.timed_run("conformer", args, 1, 0, dev, True)
        print(f"{variant}: first conformer {r['dt'] / args.steps * 1e3:.2f} ms", flush=True)
    elif variant == "base_nosync":
        r = bench.timed_run("base", args, 1, 0, dev, True)
        Fn.set_deferred_wgrad([])
        Fn._W16.clear()
        Fn._CAST_CACHE.clear()
        print(f"{variant}: base {r['dt'] / args.steps * 1e3:.2f} ms (caches cleared)", flush=True)
    r = bench.timed_run("conformer", args, 1, 0, dev, True)
    print(f"{variant}: conformer {r['dt'] / args.steps * 1e3:.2f} ms ({r['step_mode']})", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--one":
        one(sys.argv[2])
        sys.exit(0)
    for v in sys.argv[1:] or ["alone", "conf_twice", "base_eager", "base_graph", "base_nosync"]:
        p = subprocess.run([sys.executable, "-u", __file__, "--one", v], timeout=400)
        print(f"== {v}: rc {p.returncode}", flush=True)
