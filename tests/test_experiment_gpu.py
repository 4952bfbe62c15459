"""The Experiment layer end to end on the GPU (reference run.py -> get_experiment_from_args ->
Experiment.run, src/experiments/*.py): command line -> experiment -> Trainer epochs on synthetic
trials of the real format -> history.json, model.pt, brain_encoder.pt; the optimizer param groups
and schedules of both unfreeze strategies; checkpoint reload (from_checkpoint, strict keys)."""
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def _argv(tmp, exp="b2p2t_gru+w2v", extra=()):
    return ["--experiment_type", exp, "--batch_size", "2", "--epochs", "2", "--synthetic_samples", "4",
            "--synthetic_min_len", "256", "--synthetic_max_len", "320", "--log_every_n_batches", "1",
            "--scheduler_step_size", "1", *extra]


def _yaml(tmp):
    p = tmp / "config.yaml"
    p.write_text(f"cache_dir: {tmp / 'cache'}\n")
    return str(p)


def test_w2v_experiment_run_writes_results(tmp_path):
    from wav2vec2forbrain_amd.args.argparsing import get_experiment_from_args
    exp = get_experiment_from_args(_argv(tmp_path), config_path=_yaml(tmp_path))
    assert exp.get_name() == "b2p2t_gru+w2v"
    opt = exp.create_optimizer()
    assert len(opt.param_groups) == 1
    assert {id(p) for p in opt.param_groups[0]["params"]} == {id(p) for p in exp.model.brain_encoder.parameters()}
    exp.run()
    files = set(os.listdir(exp.results_dir))
    assert {"config.json", "history.json", "model.pt", "brain_encoder.pt"} <= files
    hist = json.load(open(os.path.join(exp.results_dir, "history.json")))
    assert len(hist["epochs"]) == 2
    tr = hist["epochs"][0]["train"]["history"]
    assert len(tr) == 2 and all("word_error_rate" in b["metrics"] and "char_error_rate" in b["metrics"] for b in tr)
    assert all(b["loss"] > 0 for b in tr)
    test = hist["test"]["history"]
    assert test and test[0]["batch"]["predictions"] is not None   # test mode keeps the decoded strings
    # the stored checkpoints reload strictly (reference from_checkpoint / brain_encoder_path)
    sd = torch.load(os.path.join(exp.results_dir, "model.pt"), weights_only=True)
    exp.model.load_state_dict(sd, strict=True)
    be = torch.load(os.path.join(exp.results_dir, "brain_encoder.pt"), weights_only=True)
    exp.model.brain_encoder.load_state_dict(be, strict=True)


def test_w2v_experiment_full_finetune_groups_and_warmup(tmp_path):
    from wav2vec2forbrain_amd.args.argparsing import get_experiment_from_args
    argv = _argv(tmp_path, extra=("--unfreeze_strategy", "brain_encoder+w2v", "--w2v_learning_rate", "1e-4",
                                  "--w2v_warmup_start_step", "1", "--w2v_warmup_steps", "2",
                                  "--adjust_global_lr_to_w2v_postwarmup_lr", "true", "--epochs", "1",
                                  "--gradient_clipping", "1.0"))
    exp = get_experiment_from_args(argv, config_path=_yaml(tmp_path))
    opt = exp.create_optimizer()
    assert len(opt.param_groups) == 2 and opt.param_groups[1]["lr"] == 1e-4
    sch = exp.get_scheduler(opt)
    lrs = []
    for _ in range(4):
        lrs.append([g["lr"] for g in opt.param_groups])
        sch.step()
    # module 2 (w2v): 0 before the warmup start, then linear to its target; module 1 follows to 1e-4
    assert lrs[0] == [1e-3, 0.0] and abs(lrs[2][1] - 0.5e-4) < 1e-12 and abs(lrs[3][0] - 1e-4) < 1e-12
    # training with the w2v group at full rate from epoch 0 (no warmup): the w2v weights move
    argv = _argv(tmp_path, extra=("--unfreeze_strategy", "brain_encoder+w2v", "--w2v_learning_rate", "1e-4",
                                  "--epochs", "1", "--gradient_clipping", "1.0", "--return_best_model", "false"))
    exp = get_experiment_from_args(argv, config_path=_yaml(tmp_path))
    w0 = exp.model.w2v_encoder.lm_head.weight.detach().clone()
    exp.run()
    assert not torch.equal(w0, exp.model.w2v_encoder.lm_head.weight.detach())   # w2v trained


def test_conformer_experiment_trains(tmp_path):
    from wav2vec2forbrain_amd.args.argparsing import get_experiment_from_args
    argv = _argv(tmp_path, exp="b2p2t_gru+w2v_conformer",
                 extra=("--encoder_gru_hidden_size", "512", "--encoder_num_gru_layers", "3",
                        "--encoder_fc_hidden_sizes", "[256]", "--epochs", "1"))
    exp = get_experiment_from_args(argv, config_path=_yaml(tmp_path))
    assert exp.get_name() == "b2p2t_gru+w2v_conformer"
    exp.run()
    assert os.path.exists(os.path.join(exp.results_dir, "model.pt"))
