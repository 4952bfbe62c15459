"""bench.py — b2p2t_gru+w2v training step on MI355X (BASELINE.json metric:
"train steps/sec + CTC loss, b2p2t_gru+w2v bs=32 seq=1024 at 1/2/4/8 MI355X").

Workload (BASELINE.json configs[1]): wav2vec2-base architecture (768/12L/12H/3072, random-init,
hub unreachable), GRU H256x2 bidirectional, fc [] -> 768, bs=32 per GPU, 1024-bin x 256-channel
synthetic windows (x ~ N(0,1)), train mode (dropout 0.1 / LayerDrop 0.1 as the checkpoint config),
unfreeze_strategy=brain_encoder (Adam over the brain encoder; the frozen w2v still computes weight
gradients, as the reference does). One step = Trainer.train_step (train/train_loop.py, the step
run.py executes; reference src/train/train_loop.py:41-84): forward + backward + DDP gradient
all-reduce (N>1) + Adam, replayed as a captured HIP graph, plus the CTC loss readback (into pinned
host memory, stream-ordered), inputs pre-staged in HBM. N=1 base runs add a nested record for the
north-star target (configs[2], Conformer-large bs=32) with its own parity and CPU baseline.

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
# train-step FLOPs per config at bs=32, L=1024
STEP_TFLOP = {"base": 5.216, "conformer": 30.06, "large": 16.14}


def make_config(bs, L, kind="base"):
    from wav2vec2forbrain_amd.workloads import bench_config
    return bench_config(kind, bs, L)


def build(cfg, device, train_dropouts=True):
    from wav2vec2forbrain_amd.workloads import build_model
    return build_model(cfg, device=device, train_dropouts=train_dropouts)


def batch_on(cfg, device):
    from wav2vec2forbrain_amd.workloads import device_batch
    return device_batch(cfg, device)


def oracle_batch(cfg):
    from wav2vec2forbrain_amd.workloads import make_batch
    x, day, il, tgt, tl = make_batch(cfg)
    return dict(x=x, day_idxs=day, input_lens=il, target=tgt, target_lens=tl)


def oracle_cfg(cfg, train_dropouts=False):
    """The oracle's config for a workload (oracle/ is the CPU checker: imported only here, in the
    cpu_baseline / parity legs after the timed region)."""
    from oracle.b2p2t_oracle import OracleConfig, ConformerOracleConfig
    kw = dict(gru_hidden=cfg["gru_hidden"], gru_layers=cfg["gru_layers"], bidirectional=cfg["bidirectional"],
              fc_hidden_sizes=list(cfg["fc_hidden"]), learnable_initial_state=cfg["learnable_h0"],
              hidden_size=cfg["hidden_size"], num_hidden_layers=cfg["layers"], num_attention_heads=cfg["heads"],
              intermediate_size=cfg["ffn"], num_conv_pos_embeddings=cfg["pos_k"],
              num_conv_pos_embedding_groups=cfg["pos_groups"])
    if cfg.get("conformer"):
        c = ConformerOracleConfig(conv_depthwise_kernel_size=cfg["dw_kernel"], **kw)
    else:
        c = OracleConfig(do_stable_layer_norm=cfg.get("stable", False), **kw)
    if train_dropouts:
        c.hidden_dropout = c.activation_dropout = c.attention_dropout = c.final_dropout = 0.1
        c.layerdrop = 0.1
        if cfg.get("conformer"):
            c.conformer_conv_dropout = 0.1
    return c


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
    caps = {"physical_cores": n_phys, "affinity": len(os.sched_getaffinity(0))}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            caps["cgroup_quota"] = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        caps["OMP_NUM_THREADS"] = int(os.environ["OMP_NUM_THREADS"])
    HOST_CAPS.clear()
    HOST_CAPS.update(caps)
    return min(caps.values()), n_phys, model


HOST_CAPS: dict = {}   # the thread caps host_cpu_info() saw (recorded beside the CPU baseline)




def brain_keys(sd):
    return [k for k in sd if k.startswith("brain_encoder.") and sd[k].is_floating_point() and "gaussian" not in k]


def oracle_steps(cfg, sd, steps, train_dropouts, lr=1e-3):
    """`steps` CPU oracle training steps (oracle/b2p2t_oracle.py, torch-CPU fp32: forward, backward,
    Adam over the brain encoder as unfreeze_strategy=brain_encoder does) from state dict `sd`, each
    timed on the host cores. Returns (losses, seconds per step, threads, physical cores, CPU model)."""
    from oracle.b2p2t_oracle import loss_and_grads, conformer_loss_and_grads, adam_step
    threads, n_phys, model_name = host_cpu_info()
    torch.set_num_threads(threads)
    ocfg = oracle_cfg(cfg, train_dropouts)
    b = oracle_batch(cfg)
    sd = dict(sd)
    brain = brain_keys(sd)
    state = {k: (torch.zeros_like(sd[k]), torch.zeros_like(sd[k])) for k in brain}
    losses, times = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        if cfg.get("conformer"):
            loss, grads, _bn = conformer_loss_and_grads(sd, b, ocfg, training=True)
        else:
            loss, grads = loss_and_grads(sd, b, ocfg, training=True)
        for k in brain:
            m, v = state[k]
            sd[k], m, v = adam_step(sd[k], grads[k], m, v, i + 1, lr)
            state[k] = (m, v)
        times.append(time.perf_counter() - t0)
        losses.append(float(loss))
    return losses, times, threads, n_phys, model_name


def cpu_record(times, threads, n_phys, model_name, sample):
    med = sorted(times)[len(times) // 2]
    bound = sorted(k for k, v in HOST_CAPS.items() if v == threads)
    return {"value": round(1.0 / med, 5), "unit": "steps/s", "cores": threads, "kind": "port",
            "host_physical_cores": n_phys, "cpu_model": model_name,
            "thread_caps": dict(HOST_CAPS), "bound_by": bound,
            "sample": f"{sample}: median {med:.2f} s/step (all: {', '.join(f'{t:.2f}' for t in times)})"}


def cpu_baseline(cfg, steps=5):
    """the CPU oracle (the build's torch-CPU fp32 restatement) timed on the host cores on
    the bench workload itself — train mode with the same dropouts / LayerDrop, fwd + bwd + Adam over the
    brain encoder, same batch size — 1 warm-up step, median of `steps` timed steps."""
    model = build(cfg, "cpu")
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    del model
    _, times, threads, n_phys, model_name = oracle_steps(cfg, sd, steps + 1, train_dropouts=True)
    return cpu_record(times[1:], threads, n_phys, model_name,
                      f"oracle fwd+bwd+Adam (fp32, torch-CPU, {threads} threads), bs={cfg['B']} L={cfg['L']} train mode, "
                      f"{steps} steps after 1 warm-up")


def _hip_losses(cfg, device, steps, mode):
    """CTC losses of `steps` consecutive deterministic Trainer steps (HipAdam lr 1e-3 over the brain
    encoder) in precision `mode`, from the workload's deterministic weights; also returns them."""
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    model = build(cfg, device, train_dropouts=False)
    model.train()
    sd = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    with Fn.precision(mode):
        trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
        hip = [float(trainer._eager_body(batch_on(cfg, device)).metrics["ctc_loss"]) for _ in range(steps)]
    torch.cuda.synchronize()
    Fn.set_deferred_wgrad([])
    del trainer, model
    free_device()
    return hip, sd


def parity_check(cfg, device, steps=2):
    """north_star parity: the CTC loss of `steps` consecutive Trainer steps vs the fp32 CPU oracle on
    identical weights and inputs, deterministic mode (dropout 0, LayerDrop 0: the reference's Philox
    masks cannot be reproduced), HipAdam lr 1e-3 over the brain encoder between steps. Two HIP runs:
      bf16  the bench's precision; every step must be within the north-star 1e-3 relative. After the
            first update the losses are those of different weights: Adam's early updates are
            ~lr * sign(g), so every gradient entry whose sign the rounding flips moves its parameter by
            2 lr (tools/traj_err.py measures how much each block's rounding contributes).
      fp32  exact-fp32 MFMA mode: the same trajectory must track the oracle step by step (1e-4), which
            separates rounding drift from a wrong update.
    Returns the record and the oracle's per-step times (the Conformer's CPU baseline reuses them)."""
    b16, sd = _hip_losses(cfg, device, steps, "bf16")
    f32, _ = _hip_losses(cfg, device, steps, "fp32")
    ref, times, threads, n_phys, model_name = oracle_steps(cfg, sd, steps, train_dropouts=False)
    rel = lambda hip: [abs(h - r) / abs(r) for h, r in zip(hip, ref)]
    rb, rf = rel(b16), rel(f32)
    rec = {"mode": "deterministic (dropout 0, LayerDrop 0) HIP Trainer steps vs fp32 CPU oracle, same "
                   "weights/inputs, Adam lr 1e-3 over the brain encoder between steps",
           "steps": steps, "oracle_ctc_loss": [round(v, 6) for v in ref],
           "hip_ctc_loss": [round(v, 6) for v in b16], "rel_err": [float(f"{r:.3e}") for r in rb],
           "max_rel_err": float(f"{max(rb):.3e}"),
           "fp32_mode": {"hip_ctc_loss": [round(v, 6) for v in f32], "rel_err": [float(f"{r:.3e}") for r in rf],
                         "tolerance": 1e-4},
           "tolerance": 1e-3,
           "criterion": "every bf16 step <= 1e-3 (north_star) and every fp32-mode step <= 1e-4",
           "pass": max(rb) <= 1e-3 and max(rf) <= 1e-4}
    return rec, (times, threads, n_phys, model_name)


def free_device():
    import gc
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def log(msg):
    print(f"bench: {msg}", file=sys.stderr, flush=True)


# BASELINE configs[4] per GPU (global batch 64 over 8 GPUs): the Conformer-large with the whole encoder
# trained (unfreeze_strategy=brain_encoder+w2v: two param groups, w2v lr 1e-4, L2 weight decay 1e-5,
# b2t_gru_w2v_conformer_experiment.py:87-123)
FT = dict(bs=8, lr=1e-3, w2v_lr=1e-4, wd=1e-5)


def experiment_for(kind, model):
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    if kind == "conformer_ft":
        return SyntheticStepExperiment(model, unfreeze="brain_encoder+w2v", lr=FT["lr"], w2v_lr=FT["w2v_lr"],
                                       weight_decay=FT["wd"])
    return SyntheticStepExperiment(model, lr=1e-3)


def timed_run(kind, args, world, rank, device, use_graph, steps=None, warmup=None, evaluator=None, roofline=None):
    """W warm-up steps + K timed steps of the Trainer's training step (train/train_loop.py, the step
    run.py executes) on the workload, then the GEMM-timing pass. Graph mode: the first W steps run
    eagerly, the next one captures the step (untimed), the K timed steps are replays."""
    import argparse as _ap
    from wav2vec2forbrain_amd import functional as Fn, _lib
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    args = _ap.Namespace(**vars(args))
    args.steps = steps or args.steps
    args.warmup = args.warmup if warmup is None else warmup
    args.evaluator = args.evaluator if evaluator is None else evaluator
    args.no_roofline = args.no_roofline if roofline is None else not roofline
    if kind == "conformer_ft":
        cfg = make_config(FT["bs"], args.seq, "conformer")
    else:
        cfg = make_config(args.bs, args.seq, kind)
    model = build(cfg, device)
    model.train()
    if world > 1 and hasattr(model, "sync_batchnorm"):
        # the Conformer under DP: BatchNorm statistics over the global batch (SyncBN, the default); the
        # replayed step is captured in segments split at those all-reduces (train/step_graph.py).
        # B2P_BENCH_SYNCBN=0: per-rank statistics (torch DDP's default semantics), one graph
        model.sync_batchnorm = os.environ.get("B2P_BENCH_SYNCBN", "1") != "0"
    # the reference reads ctc_loss.item() inside forward (w2v_custom_feat_extractor.py:94): a host sync
    # per step. The bench keeps the loss on the device and reads every step's value into pinned host
    # memory (stream-ordered) instead, and reads them all after the timed region.
    for m in model.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = False
    trainer = Trainer(experiment_for(kind, model))
    trainer.use_graphs = use_graph and trainer.use_graphs
    trainer.capture_after = args.warmup
    prec = trainer.step_precision() or "bf16"
    batch = batch_on(cfg, device)

    def metrics(out):
        # the loss, plus (--evaluator) the train evaluator's greedy-decode WER computed on the device
        # (SURVEY 8(d1) "with the evaluator"; the reference does it on the host every step)
        loss = out.loss.detach().reshape(1)
        if not args.evaluator:
            return loss
        wer = Fn.ctc_greedy_wer(out.logits.detach(), batch.target)[0]
        return torch.cat([loss, wer.reshape(1).float()])

    for _ in range(args.warmup + (1 if trainer.use_graphs else 0)):
        metrics(trainer.train_step(batch))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    loss_host = torch.zeros(args.steps, 2 if args.evaluator else 1, dtype=torch.float32).pin_memory()
    g0 = trainer.graph_steps
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss_host[i].copy_(metrics(trainer.train_step(batch)), non_blocking=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    replayed = trainer.graph_steps - g0
    Fn.check_gru_status()   # a multi-CU GRU timeout in any timed step raises here
    # GEMM roofline: HIP events around every GEMM launch of the same number of eager Trainer steps,
    # right after the timed region (a captured graph cannot carry per-launch events); the kernels and
    # their shapes are the ones the graph replays.
    gemm = (0.0, 0, 0.0)
    if not args.no_roofline:
        _lib.check(_lib.load().b2p_timing_enable(_lib.TIMING_GEMM, 100000), "timing_enable")
        Fn.set_gemm_timing(True)
        if trainer.reducer is not None:
            trainer.reducer.use_layer_gates(None)
        with trainer.precision_context():
            for _ in range(args.steps):
                trainer._eager_body(batch)
        torch.cuda.synchronize()
        Fn.set_gemm_timing(False)
        gemm = ctypes_read_timing()
        _lib.check(_lib.load().b2p_timing_enable(_lib.TIMING_GEMM, 0), "timing_disable")
    if world > 1:
        t = torch.tensor([dt], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = t.item()
    res = dict(cfg=cfg, dt=dt, losses=loss_host[:, 0].tolist(), precision=prec, steps=args.steps, warmup=args.warmup,
               wers=loss_host[:, 1].tolist() if args.evaluator else None, gemm=gemm,
               step_mode=("hip-graph replay" if replayed == args.steps else
                          "eager" if replayed == 0 else f"mixed ({replayed}/{args.steps} replayed)"))
    trainer.release_graphs()
    del trainer, model, batch
    free_device()
    return res


def roofline_record(gemm, kind):
    gemm_ms, gemm_n, gemm_flops = gemm
    achieved = gemm_flops / (gemm_ms * 1e-3) / 1e12 if gemm_ms > 0 else 0.0
    return {"bound": "mfma", "kernel": "b2p_gemm (all GEMM launches of the step)",
            "achieved": round(achieved, 2), "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": round(achieved / BF16_DENSE_PEAK_TFLOPS, 4), "traffic": gemm_traffic(kind),
            "launches": gemm_n, "avg_launch_us": round(gemm_ms * 1e3 / max(gemm_n, 1), 2),
            "algorithmic_flop_per_launch": round(gemm_flops / max(gemm_n, 1), 1)}


WORKLOAD_TEXT = {
    "base": "b2p2t_gru+w2v wav2vec2-base (12L/768), GRU H256x2 bidir, train mode, unfreeze=brain_encoder, Adam",
    "conformer": "b2p2t_gru+w2v_conformer rope-large (24L/1024, k31), GRU H512x3 bidir, fc [256], train mode, "
                 "unfreeze=brain_encoder, Adam",
    "large": "b2p2t_gru+w2v wav2vec2-large-960h (24L/1024, post-LN), GRU H256x2 bidir, train mode, "
             "unfreeze=brain_encoder, Adam",
}
ARCH_TEXT = {"base": "wav2vec2-base", "conformer": "wav2vec2-conformer-rope-large", "large": "wav2vec2-large-960h"}


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
    ap.add_argument("--no-conformer", action="store_true",
                    help="N=1 base runs: skip the nested Conformer-large (configs[2], the north-star target) record")
    ap.add_argument("--no-extra", action="store_true",
                    help="N=1 base runs: skip the nested configs[3] / configs[4] / evaluator / fp32-mode records")
    ap.add_argument("--evaluator", action="store_true",
                    help="include the train evaluator's greedy CTC decode + WER (on the device) in every step")
    ap.add_argument("--graph", type=int, default=None,
                    help="1/0: Trainer steps replayed as captured HIP graphs (default 1) / eager")
    ap.add_argument("--config", choices=["base", "conformer", "large"], default="base",
                    help="base = BASELINE configs[1] (headline); conformer = configs[2]; large = configs[3] per GPU")
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
    # model weights are deterministic (util/init.py) and equal on every rank; dropout / LayerDrop
    # masks differ per rank
    torch.manual_seed(1234)
    from wav2vec2forbrain_amd import functional as Fn
    Fn.SEEDS.reseed(1234 * 65537 + rank)
    Fn.LD_SEEDS.reseed(1234 * 65537 + 7919)   # device LayerDrop draws: equal on every rank
    Fn.set_precision("bf16")
    use_graph = True if args.graph is None else bool(args.graph)

    r = timed_run(args.config, args, world, rank, device, use_graph)
    if rank != 0:
        dist.destroy_process_group() if world > 1 else None
        return
    dt = r["dt"]
    # whole-job throughput: the units all ranks processed / time. A unit is one training step of one
    # rank over its own bs-sample batch (weak scaling: N ranks process N batches per global step).
    steps_per_s = world * args.steps / dt
    step_tflop = STEP_TFLOP[args.config] * args.bs / 32 * args.seq / 1024
    log(f"timed {args.steps} steps: {dt / args.steps * 1e3:.3f} ms/step ({r['step_mode']})")
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
        "data": f"synthetic (x~N(0,1) 256-ch windows, random-init weights of the {ARCH_TEXT[args.config]} architecture)",
        "config": {"workload": WORKLOAD_TEXT[args.config], "global_batch": args.bs * world,
                   "per_gpu_batch": args.bs, "seq_len": args.seq, "parallelism": f"dp{world}"},
        "ctc_loss": round(r["losses"][-1], 5),
        "train_evaluator": ({"on_device": True, "word_error_rate": round(r["wers"][-1], 4)} if args.evaluator
                            else None),
        "step_mode": r["step_mode"] + " of Trainer.train_step (train/train_loop.py, the step run.py runs)",
        "samples_per_s": round(steps_per_s * args.bs, 2),
        "step_mfma_frac": round(step_tflop * steps_per_s / world / BF16_DENSE_PEAK_TFLOPS, 4),
        "roofline": roofline_record(r["gemm"], args.config),
    }
    if args.config == "conformer":
        res["metric"] = "train steps/sec + CTC loss, b2p2t_gru+w2v_conformer bs=32 seq=1024"
    elif args.config == "large":
        res["metric"] = "train steps/sec + CTC loss, b2p2t_gru+w2v wav2vec2-large-960h bs=32 seq=1024"
    cfg = r["cfg"]
    if world == 1 and not args.no_parity:
        log("parity: deterministic HIP Trainer steps vs CPU oracle")
        res["parity"], _ = parity_check(cfg, device, steps=2)
    if world == 1 and not args.no_cpu_baseline:
        log("cpu_baseline: oracle steps on the host cores")
        res["cpu_baseline"] = cpu_baseline(cfg, steps=5 if args.config == "base" else 3)
        res["vs_cpu"] = round(res["value"] / res["cpu_baseline"]["value"], 1)
    if world == 1 and args.config == "base" and not args.no_conformer:
        res["conformer_large"] = conformer_record(args, device)
    if world == 1 and args.config == "base" and not args.no_extra:
        res["train_evaluator_record"] = evaluator_record(args, device)
        log("base: exact-fp32 mode steps")
        res["fp32_mode"] = fp32_mode_record("base", args, device)
        if "cpu_baseline" in res:
            res["fp32_mode"]["vs_cpu"] = round(res["fp32_mode"]["value"] / res["cpu_baseline"]["value"], 1)
        res["large960"] = large_record(args, device)
        res["conformer_large_ft"] = ft_record(args, device)
    print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def conformer_record(args, device):
    """The north-star target (BASELINE configs[2], b2p2t_gru+w2v_conformer-large bs=32 seq=1024) on the
    same GPU in the same run: timed Trainer steps with their GEMM roofline, CTC-loss parity of 3
    consecutive deterministic steps against the CPU oracle, and the CPU baseline at bs=32 — the
    oracle's own per-step times of those 3 parity steps (deterministic mode: the CPU skips the dropout
    / LayerDrop work the timed GPU steps do, so the GPU/CPU ratio is conservative)."""
    log("conformer_large: timed Trainer steps")
    r = timed_run("conformer", args, 1, 0, device, True if args.graph is None else bool(args.graph))
    sps = args.steps / r["dt"]
    rec = {"metric": "train steps/sec + CTC loss, b2p2t_gru+w2v_conformer bs=32 seq=1024", "value": round(sps, 4),
           "unit": "steps/s", "ms_per_step": round(r["dt"] / args.steps * 1e3, 3), "steps": args.steps,
           "warmup": args.warmup, "config": {"workload": WORKLOAD_TEXT["conformer"], "per_gpu_batch": args.bs,
                                              "seq_len": args.seq, "parallelism": "dp1"},
           "step_mode": r["step_mode"], "ctc_loss": round(r["losses"][-1], 5),
           "step_mfma_frac": round(STEP_TFLOP["conformer"] * args.bs / 32 * args.seq / 1024 * sps
                                   / BF16_DENSE_PEAK_TFLOPS, 4),
           "roofline": roofline_record(r["gemm"], "conformer")}
    if not args.no_parity:
        log("conformer_large: parity (3 deterministic steps) + CPU oracle timing")
        rec["parity"], (times, threads, n_phys, model_name) = parity_check(r["cfg"], device, steps=3)
        if not args.no_cpu_baseline:
            rec["cpu_baseline"] = cpu_record(
                times, threads, n_phys, model_name,
                f"oracle fwd+bwd+Adam (fp32, torch-CPU, {threads} threads), bs={args.bs} L={args.seq}, the 3 "
                "deterministic parity steps (dropout / LayerDrop 0, no extrapolation)")
            rec["vs_cpu"] = round(rec["value"] / rec["cpu_baseline"]["value"], 1)
    log("conformer_large: exact-fp32 mode steps")
    rec["fp32_mode"] = fp32_mode_record("conformer", args, device)
    if "cpu_baseline" in rec:
        rec["fp32_mode"]["vs_cpu"] = round(rec["fp32_mode"]["value"] / rec["cpu_baseline"]["value"], 1)
    return rec


def fixture_parity(name, device):
    """The CTC losses of the Trainer's deterministic steps on a golden fixture's model and batch
    (tests/golden/<name>.npz: the reference's own modules and torch.optim.Adam produced that trajectory,
    tests/golden/make_golden.py) under the Trainer's precision policy, the first step eager and the rest
    replays, against the reference's losses."""
    import numpy as np
    from tests.golden.configs import CONFIGS, make_batch as fixture_batch
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.datasets.batch_types import make_b2t_batch
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment, build_model
    cfg = {c["name"]: c for c in CONFIGS}[name]
    a = cfg["adam"]
    ref = [float(v) for v in np.load(os.path.join(ROOT, "tests", "golden", f"{name}.npz"))["adam_losses"]]
    model = build_model(cfg, device=device)
    model.train()
    exp = SyntheticStepExperiment(model, unfreeze="brain_encoder+w2v" if a["w2v_lr"] is not None else "brain_encoder",
                                  lr=a["lr"], w2v_lr=a["w2v_lr"], weight_decay=a["wd"])
    x, day, il, tgt, tl = fixture_batch(cfg)
    batch = make_b2t_batch(x, tgt, day, il, tl).cuda()
    trainer = Trainer(exp)
    trainer.capture_after = 1
    losses = [float(trainer.train_step(batch).loss) for _ in range(a["steps"])]
    prec = trainer.step_precision() or "bf16"
    trainer.release_graphs()
    Fn.set_deferred_wgrad([])
    del trainer, model, exp, batch
    free_device()
    rel = [abs(g - r) / abs(r) for g, r in zip(losses, ref)]
    return {"mode": f"deterministic Trainer steps ({prec}; step 1 eager, then replays) vs the reference's own "
                    f"trajectory (tests/golden/{name}.npz)", "precision": prec,
            "reference_ctc_loss": [round(v, 6) for v in ref], "hip_ctc_loss": [round(v, 6) for v in losses],
            "rel_err": [float(f"{r:.3e}") for r in rel], "max_rel_err": float(f"{max(rel):.3e}"),
            "tolerance": 1e-3, "pass": max(rel) <= 1e-3}


def nested(r, metric, kind_text, extra=None):
    sps = r["steps"] / r["dt"]
    rec = {"metric": metric, "value": round(sps, 4), "unit": "steps/s",
           "ms_per_step": round(r["dt"] / r["steps"] * 1e3, 3), "steps": r["steps"], "warmup": r["warmup"],
           "dtype": r["precision"], "config": dict(kind_text), "step_mode": r["step_mode"],
           "ctc_loss": round(r["losses"][-1], 5)}
    rec.update(extra or {})
    return rec


def evaluator_record(args, device):
    """the headline workload with the reference-equivalent train evaluator in every step
    (reference src/train/train_loop.py:79 -> src/train/evaluator.py:163-229: greedy CTC decode + WER of
    the step's logits; here on the device, its value read with the loss)."""
    log("base + train evaluator: timed Trainer steps")
    r = timed_run("base", args, 1, 0, device, True if args.graph is None else bool(args.graph), evaluator=True,
                  roofline=False)
    return nested(r, "train steps/sec, b2p2t_gru+w2v bs=32 seq=1024 with the train evaluator (greedy decode + WER)",
                  {"workload": WORKLOAD_TEXT["base"] + ", on-device greedy CTC decode + WER every step",
                   "per_gpu_batch": args.bs, "seq_len": args.seq, "parallelism": "dp1"},
                  {"word_error_rate": round(r["wers"][-1], 4)})


def large_record(args, device):
    """BASELINE configs[3] per GPU (global 256 over 8 GPUs = bs 32 each): wav2vec2-large-960h, timed
    Trainer steps + the 2-step Adam trajectory of the reference on its fixture (large960_bs32)."""
    log("large960 (configs[3] per GPU): timed Trainer steps")
    r = timed_run("large", args, 1, 0, device, True if args.graph is None else bool(args.graph), steps=10, warmup=3)
    rec = nested(r, "train steps/sec + CTC loss, b2p2t_gru+w2v wav2vec2-large-960h bs=32 seq=1024 (configs[3] per GPU)",
                 {"workload": WORKLOAD_TEXT["large"], "per_gpu_batch": args.bs, "seq_len": args.seq,
                  "parallelism": "dp1 (configs[3] is dp8, global 256)"},
                 {"roofline": roofline_record(r["gemm"], "large"),
                  "step_mfma_frac": round(STEP_TFLOP["large"] * r["steps"] / r["dt"] / BF16_DENSE_PEAK_TFLOPS, 4)})
    log("large960: fixture trajectory")
    rec["parity"] = fixture_parity("large960_bs32", device)
    return rec


def ft_record(args, device):
    """BASELINE configs[4] per GPU (global 64 over 8 GPUs = bs 8 each): the Conformer-large with the whole
    encoder trained (two param groups), timed Trainer steps in the Trainer's precision policy (bf16x3:
    split-bf16 GEMMs), its 3-step trajectory against the reference's
    (conformer_large_ft_bs8), and the same step with the policy off (pure bf16 / fp16 operands) for the
    cost / accuracy trade."""
    graph = True if args.graph is None else bool(args.graph)
    log("conformer_large_ft (configs[4] per GPU): timed Trainer steps")
    r = timed_run("conformer_ft", args, 1, 0, device, graph, steps=10, warmup=3)
    x3 = r["precision"] == "bf16x3"
    roof = roofline_record(r["gemm"], "conformer_ft")
    if x3:   # bf16 MFMA products per algorithmic multiply-add under the policy's per-role forms
        from wav2vec2forbrain_amd import functional as Fn
        w = Fn.x3_mfma_work(Fn.X3_POLICY_FORMS)
        roof.update(mfma_work_per_flop=round(w, 3), mfma_frac=round(w * roof["frac"], 4),
                    x3_forms=",".join(sorted(Fn.X3_POLICY_FORMS)) or "three-term everywhere")
    rec = nested(r, "train steps/sec + CTC loss, b2p2t_gru+w2v_conformer-large unfreeze=brain_encoder+w2v bs=8 "
                    "seq=1024 (configs[4] per GPU)",
                 {"workload": WORKLOAD_TEXT["conformer"].replace("unfreeze=brain_encoder", "unfreeze=brain_encoder+w2v "
                                                                 "(w2v lr 1e-4, L2 weight decay 1e-5)"),
                  "per_gpu_batch": FT["bs"], "seq_len": args.seq, "parallelism": "dp1 (configs[4] is dp8, global 64)"},
                 {"roofline": roof})
    log("conformer_large_ft: fixture trajectory")
    rec["parity"] = fixture_parity("conformer_large_ft_bs8", device)
    old = os.environ.get("B2P_TRAIN_PRECISION")
    os.environ["B2P_TRAIN_PRECISION"] = "keep"
    try:
        log("conformer_large_ft: policy off (bf16 / fp16 operands)")
        r2 = timed_run("conformer_ft", args, 1, 0, device, graph, steps=10, warmup=3, roofline=False)
        rec["policy_off"] = {"dtype": r2["precision"], "value": round(r2["steps"] / r2["dt"], 4),
                             "ms_per_step": round(r2["dt"] / r2["steps"] * 1e3, 3),
                             "parity": fixture_parity("conformer_large_ft_bs8", device)}
    finally:
        if old is None:
            os.environ.pop("B2P_TRAIN_PRECISION")
        else:
            os.environ["B2P_TRAIN_PRECISION"] = old
    return rec


def fp32_mode_record(kind, args, device, steps=3):
    """Precision-matched throughput: the same Trainer step in the exact-fp32 MFMA mode
    (v_mfma_f32_*_f32: fp32 operands, fp32 accumulate; the reference computes in fp32), train mode,
    eager steps, 1 warm-up + `steps` timed. Its ratio to the CPU baseline is the precision-matched
    GPU/CPU figure; the headline bf16 record stays the bench value."""
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.train.train_loop import Trainer
    from wav2vec2forbrain_amd.workloads import SyntheticStepExperiment
    cfg = make_config(args.bs, args.seq, kind)
    model = build(cfg, device)
    model.train()
    for m in model.modules():
        if hasattr(m, "sync_metrics"):
            m.sync_metrics = False
    with Fn.precision("fp32"):
        trainer = Trainer(SyntheticStepExperiment(model, lr=1e-3))
        graphs = trainer.use_graphs
        trainer.use_graphs = False
        batch = batch_on(cfg, device)
        trainer.train_step(batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = trainer.train_step(batch)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        loss = float(out.loss)
        # the same step captured once and replayed (the bf16 records' step mode): no Python launch cost
        rep = None
        if graphs:
            trainer.use_graphs, trainer.capture_after = True, 0
            trainer.train_step(batch)    # capture (untimed)
            torch.cuda.synchronize()
            g0 = trainer.graph_steps
            t0 = time.perf_counter()
            for _ in range(steps):
                out = trainer.train_step(batch)
            torch.cuda.synchronize()
            dtr = time.perf_counter() - t0
            if trainer.graph_steps - g0 == steps:
                rep = {"value": round(steps / dtr, 4), "ms_per_step": round(dtr / steps * 1e3, 2),
                       "step_mode": "hip-graph replay of Trainer.train_step", "ctc_loss": round(float(out.loss), 5)}
            trainer.release_graphs()
    Fn.set_deferred_wgrad([])
    del trainer, model, batch
    free_device()
    return {"value": round(steps / dt, 4), "unit": "steps/s", "ms_per_step": round(dt / steps * 1e3, 2),
            "steps": steps, "warmup": 1, "dtype": "fp32 (exact-fp32 MFMA, the reference's arithmetic)",
            "step_mode": "eager Trainer.train_step", "ctc_loss": round(loss, 5), "replayed": rep}


def gemm_traffic(kind="base"):
    """HBM bytes per GEMM launch from the newest committed PMC measurement of this same bench command
    (profiles/*_gemm_traffic.json for the base config, profiles/*_gemm_traffic_conformer.json for
    --config conformer; written by tools/round_profile.sh: FETCH_SIZE x2 + WRITE_SIZE); None when the
    config has no measurement."""
    import glob
    fs = glob.glob(os.path.join(ROOT, "profiles", "*_gemm_traffic*.json"))
    fs = sorted((f for f in fs if os.path.basename(f).endswith(f"_gemm_traffic{'' if kind == 'base' else '_' + kind}.json")),
                key=os.path.basename)
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
