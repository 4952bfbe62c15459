"""bench.py — b2p2t_gru+w2v training step on MI355X (BASELINE.json metric:
"train steps/sec + CTC loss, b2p2t_gru+w2v bs=32 seq=1024 at 1/2/4/8 MI355X").

Workload (BASELINE.json configs[1]): wav2vec2-base architecture (768/12L/12H/3072, random-init,
hub unreachable), GRU H256x2 bidirectional, fc [] -> 768, bs=32 per GPU, 1024-bin x 256-channel
synthetic windows (x ~ N(0,1)), train mode (dropout 0.1 / LayerDrop 0.1 as the checkpoint config),
unfreeze_strategy=brain_encoder (Adam over the brain encoder; the frozen w2v still computes weight
gradients, as the reference does). One step = forward + backward + DDP gradient all-reduce (N>1)
+ Adam + CTC loss readback (.item(), as the reference's forward does), inputs pre-staged in HBM.

usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip table)
# train-step FLOPs, base bs=32 L=1024 = 3 x 1738.7 GFLOP forward
STEP_TFLOP_BASE_BS32 = 5.216


# train-step FLOPs per config at bs=32, L=1024
STEP_TFLOP = {"base": 5.216, "conformer": 30.06}


def make_config(bs, L, kind="base"):
    if kind == "conformer":
        # BASELINE configs[2]: wav2vec2-conformer-rope-large (1024/24L/16H/4096, k31), README brain
        # encoder H512x3, fc [256]
        return dict(name="bench_conformer", seed=42, B=bs, L=L, in_lens=[L] * bs, tgt_range=(60, 120),
                    hidden_size=1024, layers=24, heads=16, ffn=4096, pos_k=128, pos_groups=16, gru_hidden=512,
                    gru_layers=3, bidirectional=True, fc_hidden=[256], learnable_h0=False, full_grad_max=0,
                    infeasible=False, conformer=True, dw_kernel=31)
    return dict(name="bench_base", seed=42, B=bs, L=L, in_lens=[L] * bs, tgt_range=(60, 120), hidden_size=768,
                layers=12, heads=12, ffn=3072, pos_k=128, pos_groups=16, gru_hidden=256, gru_layers=2,
                bidirectional=True, fc_hidden=[], learnable_h0=False, full_grad_max=0, infeasible=False)


def build(cfg, device, train_dropouts=True):
    from tests.helpers import build_model
    return build_model(cfg, device=device, train_dropouts=train_dropouts)


def batch_on(cfg, device):
    from tests.golden.configs import make_batch
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    x, day, il, tgt, tl = make_batch(cfg)
    b = make_b2t_batch(x, tgt, day, il, tl)
    return b.cuda() if device != "cpu" else b


def host_cpu_info():
    """(threads to use, physical cores on the host, CPU model). Threads = the host's physical cores,
    capped by what this process may actually run on (affinity mask, cgroup CPU quota, and
    OMP_NUM_THREADS, which the GPU box sets to its 16-CPU share)."""
    phys, model = set(), "unknown"
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                model = v
            elif k in ("physical id", "core id"):
                cur[k] = v
            elif not k and cur:
                phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    n_phys = len(phys) or (os.cpu_count() or 1)
    caps = [n_phys, len(os.sched_getaffinity(0))]
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            caps.append(max(1, int(int(q) / int(per))))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        caps.append(int(os.environ["OMP_NUM_THREADS"]))
    return min(caps), n_phys, model


def cpu_baseline(bs=32, L=1024, kind="base", steps=5):
    """The CPU oracle (torch-CPU fp32 restatement, oracle/b2p2t_oracle.py) timed on the host cores:
    SURVEY 8(d5) — same workload (train mode, the same dropouts, fwd + bwd + Adam over the brain
    encoder) at the bench's batch size, 1 warm-up step, median of `steps` timed steps."""
    from oracle.b2p2t_oracle import loss_and_grads, conformer_loss_and_grads, adam_step
    from tests.helpers import oracle_cfg
    threads, n_phys, model_name = host_cpu_info()
    torch.set_num_threads(threads)
    cfg = make_config(bs, L, kind)
    ocfg = oracle_cfg(cfg)
    ocfg.hidden_dropout = ocfg.activation_dropout = ocfg.attention_dropout = ocfg.final_dropout = 0.1
    ocfg.layerdrop = 0.1
    if kind == "conformer":
        ocfg.conformer_conv_dropout = 0.1
    model = build(cfg, "cpu")
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    from tests.golden.configs import make_batch
    x, day, il, tgt, tl = make_batch(cfg)
    b = dict(x=x, day_idxs=day, input_lens=il, target=tgt, target_lens=tl)
    brain = [k for k in sd if k.startswith("brain_encoder.") and sd[k].is_floating_point()
             and "gaussian" not in k]
    state = {k: (torch.zeros_like(sd[k]), torch.zeros_like(sd[k])) for k in brain}

    def step(i):
        if kind == "conformer":
            loss, grads, _bn = conformer_loss_and_grads(sd, b, ocfg, training=True)
        else:
            loss, grads = loss_and_grads(sd, b, ocfg, training=True)
        for k in brain:
            m, v = state[k]
            sd[k], m, v = adam_step(sd[k], grads[k], m, v, i + 1, 1e-3)
            state[k] = (m, v)
        return float(loss)

    step(0)
    times = []
    for i in range(steps):
        t0 = time.perf_counter()
        step(i + 1)
        times.append(time.perf_counter() - t0)
    med = sorted(times)[len(times) // 2]
    return {"value": round(1.0 / med, 5), "unit": "steps/s", "cores": threads, "kind": "port",
            "host_physical_cores": n_phys, "cpu_model": model_name,
            "sample": f"oracle fwd+bwd+Adam (fp32, torch-CPU, {threads} threads), bs={bs} L={L} train mode, "
                      f"median of {steps} steps after 1 warm-up: {med:.2f} s/step "
                      f"(all: {', '.join(f'{t:.2f}' for t in times)})"}


def parity_check(cfg, device, kind="base", steps=2):
    """north_star parity: per-step CTC loss of the HIP bf16 step vs the fp32 CPU oracle on identical
    weights and inputs, deterministic mode (dropout 0, LayerDrop 0; the reference's Philox masks
    cannot be reproduced), `steps` consecutive steps with Adam (lr 1e-3) over the brain encoder, so
    step 2 also checks the optimizer update. Tolerance 1e-3 rel (BASELINE.json north_star)."""
    from oracle.b2p2t_oracle import loss_and_grads, conformer_loss_and_grads, adam_step
    from tests.helpers import oracle_cfg
    from wav2vec2forbrain_amd.optim import HipAdam
    model = build(cfg, device, train_dropouts=False)
    model.train()
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    opt = HipAdam(model.brain_encoder.parameters(), lr=1e-3)
    batch = batch_on(cfg, device)
    hip = []
    for _ in range(steps):
        opt.zero_grad()
        out = model(batch)
        out.loss.backward()
        opt.step()
        hip.append(float(out.metrics["ctc_loss"]))
    torch.cuda.synchronize()
    del model, opt
    threads, _, _ = host_cpu_info()
    torch.set_num_threads(threads)
    ocfg = oracle_cfg(cfg)
    from tests.golden.configs import make_batch
    x, day, il, tgt, tl = make_batch(cfg)
    b = dict(x=x, day_idxs=day, input_lens=il, target=tgt, target_lens=tl)
    brain = [k for k in sd if k.startswith("brain_encoder.") and sd[k].is_floating_point() and "gaussian" not in k]
    state = {k: (torch.zeros_like(sd[k]), torch.zeros_like(sd[k])) for k in brain}
    ref = []
    for i in range(steps):
        if kind == "conformer":
            loss, grads, _bn = conformer_loss_and_grads(sd, b, ocfg, training=True)
        else:
            loss, grads = loss_and_grads(sd, b, ocfg, training=True)
        ref.append(float(loss))
        for k in brain:
            m, v = state[k]
            sd[k], m, v = adam_step(sd[k], grads[k], m, v, i + 1, 1e-3)
            state[k] = (m, v)
    rel = [abs(h - r) / abs(r) for h, r in zip(hip, ref)]
    return {"mode": "deterministic (dropout 0, LayerDrop 0), bf16 HIP step vs fp32 CPU oracle, same weights/inputs",
            "steps": steps, "hip_ctc_loss": [round(v, 6) for v in hip], "oracle_ctc_loss": [round(v, 6) for v in ref],
            "max_rel_err": float(f"{max(rel):.3e}"), "tolerance": 1e-3, "pass": max(rel) <= 1e-3}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--no-roofline", action="store_true",
                    help="skip the eager GEMM-timing pass after the timed region (profiling runs)")
    ap.add_argument("--evaluator", action="store_true",
                    help="include the train evaluator's greedy CTC decode + WER (on the device) in every step")
    ap.add_argument("--graph", type=int, default=None,
                    help="1/0: replay the step as a captured HIP graph (default 1)")
    ap.add_argument("--config", choices=["base", "conformer"], default="base",
                    help="base = BASELINE configs[1] (headline); conformer = configs[2]")
    args = ap.parse_args()
    # the committed tree carries sources only: build the library before the first HIP call
    from wav2vec2forbrain_amd import build_lib
    build_lib.ensure_built()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # B2P_DIST_BACKEND=gloo (with more ranks than GPUs, ranks share devices) rehearses the N>1 path
    # on a one-GPU box; the driver's N>1 runs use RCCL ("nccl"), one rank per GPU
    backend = os.environ.get("B2P_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = f"cuda:{local}"
    torch.cuda.set_device(local)
    torch.manual_seed(1234 + rank)

    from wav2vec2forbrain_amd import functional as Fn, _lib
    from wav2vec2forbrain_amd.optim import HipAdam
    from wav2vec2forbrain_amd.train.ddp import GradBucketReducer, unused_param_names

    Fn.set_precision("bf16")
    cfg = make_config(args.bs, args.seq, args.config)
    model = build(cfg, device)
    model.train()
    if os.environ.get("B2P_DIAG_LAYERDROP"):   # diagnostic only: override the encoder's LayerDrop
        enc = model.w2v_encoder
        enc = enc.wav2vec2_conformer.encoder if hasattr(enc, "wav2vec2_conformer") else enc.wav2vec2.encoder
        enc.config.layerdrop = float(os.environ["B2P_DIAG_LAYERDROP"])
    skip = unused_param_names(model)
    brain_params = [p for n, p in model.named_parameters() if n.startswith("brain_encoder.") and n not in skip]
    opt = HipAdam(model.brain_encoder.parameters(), lr=1e-3)
    use_graph = True if args.graph is None else bool(args.graph)
    # graph mode: backward is captured, so the bucket all-reduce runs after each replay instead of
    # from the backward hooks
    reducer = GradBucketReducer(brain_params, overlap=not use_graph) if world > 1 else None
    if world > 1 and use_graph and hasattr(model, "sync_batchnorm"):
        # no collective is captured into the replayed step: the Conformer's BatchNorm uses per-rank
        # statistics there (DDP's default); eager steps (--graph 0) synchronise them
        model.sync_batchnorm = False
    # the frozen w2v's weight gradients (computed, as the reference does) run beside the GRU backward
    if os.environ.get("B2P_DIAG_NO_FROZEN_GRAD") == "1":   # diagnostic only (not the reference's work)
        for n, p in model.named_parameters():
            if not n.startswith("brain_encoder."):
                p.requires_grad_(False)
    if os.environ.get("B2P_DEFER_WGRAD", "1") != "0":
        Fn.set_deferred_wgrad([p for n, p in model.named_parameters() if not n.startswith("brain_encoder.")])
    batch = batch_on(cfg, device)

    # the reference reads ctc_loss.item() inside forward (w2v_custom_feat_extractor.py:94): a host
    # sync per step that lets the GPU drain and idle while the host enqueues the backward. The bench
    # keeps the loss on the device and reads every step's value after the timed region instead.
    for m in model.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = False

    def metrics(out):
        # the loss, plus (--evaluator) the train evaluator's greedy-decode WER computed on the device
        # (SURVEY 8(d1) "with the evaluator"; the reference does it on the host every step)
        if not args.evaluator:
            return out.metrics["ctc_loss"].reshape(1)
        wer = Fn.ctc_greedy_wer(out.logits.detach(), batch.target)[0]
        return torch.stack([out.metrics["ctc_loss"].reshape(()), wer])

    def zero_grad():
        # N>1: the trainable gradients live in the reducer's bucket buffers (bound as p.grad views)
        reducer.zero_grad() if reducer is not None else opt.zero_grad()

    def step():
        zero_grad()
        out = model(batch)
        out.loss.backward()
        Fn.join_wgrad()
        if reducer is not None:
            reducer.finish()
        opt.step()
        return metrics(out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # The step is captured once as a HIP graph and replayed (train/step_graph.py): one host call per
    # step instead of ~650 Python-issued launches. N=1: forward, CTC, backward, side-stream frozen-
    # weight gradients and Adam are all in the graph. N>1: the graph holds forward + backward; after
    # each replay the gradient buckets are all-reduced over RCCL and Adam runs (no collective is
    # captured). --graph 0: eager steps (RCCL bucket hooks inside backward).
    sg = None
    if use_graph:
        from wav2vec2forbrain_amd.train.step_graph import StepGraph
        if world == 1:
            sg = StepGraph(step, opt)
            run = sg.replay
        else:
            def fwd_bwd():
                zero_grad()
                out = model(batch)
                out.loss.backward()
                Fn.join_wgrad()
                return metrics(out)
            sg = StepGraph(fwd_bwd, None)

            def run():
                loss = sg.replay()
                reducer.finish()
                opt.step()
                return loss
        sg.capture()
    else:
        run = step
    if world > 1:
        dist.barrier()
    # every step reads its loss back to the host: an async copy into pinned memory,
    # stream-ordered after the step, instead of the reference's blocking .item()
    loss_host = torch.zeros(args.steps, 2 if args.evaluator else 1, dtype=torch.float32).pin_memory()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss_host[i].copy_(run(), non_blocking=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    losses = loss_host[:, 0].tolist()
    wers = loss_host[:, 1].tolist() if args.evaluator else None
    # GEMM roofline: HIP events around every GEMM launch of the same number of steps, run eagerly
    # right after the timed region (a captured graph cannot carry the per-launch events); the
    # kernels and their durations are the ones the graph replays.
    ms = (0.0, 0, 0.0)
    if not args.no_roofline:
        _lib.check(_lib.load().b2p_timing_enable(_lib.TIMING_GEMM, 100000), "timing_enable")
        Fn.set_gemm_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        Fn.set_gemm_timing(False)
        ms = ctypes_read_timing()
        _lib.check(_lib.load().b2p_timing_enable(_lib.TIMING_GEMM, 0), "timing_disable")
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    if rank != 0:
        dist.destroy_process_group() if world > 1 else None
        return
    # whole-job throughput: the units all ranks processed / time. A unit is one training step of one
    # rank over its own bs-sample batch (weak scaling: N ranks process N batches per global step).
    steps_per_s = world * args.steps / dt
    gemm_ms, gemm_n, gemm_flops = ms
    achieved = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
    step_tflop = STEP_TFLOP[args.config] * args.bs / 32 * args.seq / 1024
    res = {
        "metric": "train steps/sec + CTC loss, b2p2t_gru+w2v bs=32 seq=1024",
        "value": round(steps_per_s, 4),
        "unit": "steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "steps_per_s_per_rank": round(args.steps / dt, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16",
        "data": "synthetic (x~N(0,1) 256-ch windows, random-init weights of the "
                + ("wav2vec2-base" if args.config == "base" else "wav2vec2-conformer-rope-large") + " architecture)",
        "config": {"workload": ("b2p2t_gru+w2v wav2vec2-base (12L/768), GRU H256x2 bidir, train mode, "
                                "unfreeze=brain_encoder, Adam") if args.config == "base" else
                               ("b2p2t_gru+w2v_conformer rope-large (24L/1024, k31), GRU H512x3 bidir, fc [256], "
                                "train mode, unfreeze=brain_encoder, Adam"), "global_batch": args.bs * world,
                   "per_gpu_batch": args.bs, "seq_len": args.seq, "parallelism": f"dp{world}"},
        "ctc_loss": round(losses[-1], 5),
        "train_evaluator": ({"on_device": True, "word_error_rate": round(wers[-1], 4)} if args.evaluator else None),
        "step_mode": "hip-graph replay" if use_graph else "eager",
        "samples_per_s": round(steps_per_s * args.bs, 2),
        "step_mfma_frac": round(step_tflop * steps_per_s / world / BF16_DENSE_PEAK_TFLOPS, 4),
        "roofline": {"bound": "mfma", "kernel": "b2p_gemm (all GEMM launches of the step)",
                     "achieved": round(achieved, 2), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4), "traffic": gemm_traffic(args.config),
                     "launches": gemm_n, "avg_launch_us": round(gemm_ms * 1e3 / max(gemm_n, 1), 2),
                     "algorithmic_flop_per_launch": round(gemm_flops / max(gemm_n, 1), 1)},
    }
    if args.config != "base":
        res["metric"] = "train steps/sec + CTC loss, b2p2t_gru+w2v_conformer bs=32 seq=1024"
    def log(msg):
        print(f"bench: {msg}", file=sys.stderr, flush=True)

    log(f"timed {args.steps} steps: {dt / args.steps * 1e3:.3f} ms/step")
    if world == 1 and not args.no_parity:
        log("parity: deterministic HIP steps vs CPU oracle")
        res["parity"] = parity_check(cfg, device, args.config, steps=2 if args.config == "base" else 1)
    if world == 1 and not args.no_cpu_baseline:
        log("cpu_baseline: oracle steps on the host cores")
        if args.config == "base":
            res["cpu_baseline"] = cpu_baseline(bs=args.bs, L=args.seq, kind="base", steps=5)
        else:
            # Conformer-large: one fp32 CPU step at bs=32 is ~100 s, so the bounded sample is bs=4
            # (5 timed steps), scaled to the bench batch (the CPU step is linear in batch size)
            cb = cpu_baseline(bs=4, L=args.seq, kind="conformer", steps=5)
            cb["value"] = round(cb["value"] * 4 / args.bs, 6)
            cb["sample"] += f"; scaled x{args.bs / 4:g} to bs={args.bs}"
            res["cpu_baseline"] = cb
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def gemm_traffic(kind="base"):
    """HBM bytes per GEMM launch from the newest committed PMC measurement of this same bench command
    (profiles/*_gemm_traffic.json for the base config, profiles/*_gemm_traffic_conformer.json for
    --config conformer; written by tools/round_profile.sh: FETCH_SIZE x2 + WRITE_SIZE); None when the
    config has no measurement."""
    import glob
    fs = glob.glob(os.path.join(ROOT, "profiles", "*_gemm_traffic*.json"))
    fs = sorted((f for f in fs if f.endswith("_conformer.json") == (kind == "conformer")), key=os.path.basename)
    if not fs:
        return None
    d = json.load(open(fs[-1]))
    return {"bytes_per_launch": round(d["traffic_bytes_per_launch"]), "source": os.path.relpath(fs[-1], ROOT),
            "method": d["method"]}


def ctypes_read_timing():
    import ctypes
    from wav2vec2forbrain_amd import _lib
    ms = ctypes.c_float()
    n = ctypes.c_int32()
    fl = ctypes.c_double()
    _lib.check(_lib.load().b2p_timing_read(_lib.TIMING_GEMM, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)),
               "timing_read")
    return ms.value, n.value, fl.value


if __name__ == "__main__":
    main()
