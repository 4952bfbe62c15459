"""Experiment layer host logic (CPU): the command-line registry and argument parsing of the
reference (src/args/argparsing.py), config.yaml loading, the optimizer param groups and LR
schedules of both unfreeze strategies, history.json round trips (src/train/history.py) and the
host evaluator metrics (torcheval WordErrorRate / edit_distance CER restated)."""
import json

import pytest
import torch


def test_registry_and_argument_parsing():
    from wav2vec2forbrain_amd.args import argparsing as ap
    assert set(ap.experiments) == {"b2p2t_gru+w2v", "b2p2t_gru+w2v_conformer"}
    argv = ["--experiment_type", "b2p2t_gru+w2v", "--batch_size", "8", "--encoder_fc_hidden_sizes", "[256, 128]",
            "--unfreeze_strategy", "brain_encoder+w2v", "--w2v_learning_rate", "5e-5", "--return_best_model", "f",
            "--gradient_clipping", "0.5", "--w2v_do_stable_layer_norm", "true"]
    ns = ap._create_arg_parser(argv).parse_args(argv)
    assert ns.batch_size == 8 and ns.encoder_fc_hidden_sizes == [256, 128]
    assert ns.unfreeze_strategy == "brain_encoder+w2v" and ns.w2v_learning_rate == 5e-5
    assert ns.return_best_model is False and ns.gradient_clipping == 0.5 and ns.w2v_do_stable_layer_norm is True
    # defaults are the pydantic model's
    model = ap.experiments["b2p2t_gru+w2v"].get_args_model()
    d = model()
    ns0 = ap._create_arg_parser(["--experiment_type", "b2p2t_gru+w2v"]).parse_args(["--experiment_type", "b2p2t_gru+w2v"])
    for k in ("epochs", "learning_rate", "encoder_gru_hidden_size", "wav2vec_checkpoint", "gaussian_smooth_width",
              "unfolder_kernel_len", "lm_decode_beam_width"):
        assert getattr(ns0, k) == getattr(d, k), k
    with pytest.raises(SystemExit):   # Literal choices are enforced
        ap._create_arg_parser(argv).parse_args(argv + ["--unfreeze_strategy", "everything"])
    # the parsed namespace validates into the experiment's args model (what Experiment.__init__ does)
    cfg = model(**vars(ns))
    assert cfg.encoder_fc_hidden_sizes == [256, 128]


def test_yaml_config(tmp_path):
    from wav2vec2forbrain_amd.args.yaml_config import YamlConfig
    assert YamlConfig(str(tmp_path / "missing.yaml")).config.cache_dir == "cache"
    p = tmp_path / "config.yaml"
    p.write_text("cache_dir: /data/cache\ndataset_splits_dir: /data/splits\n")
    c = YamlConfig(str(p)).config
    assert c.cache_dir == "/data/cache" and c.dataset_splits_dir == "/data/splits"


def test_param_groups_and_schedules():
    from types import SimpleNamespace
    from wav2vec2forbrain_amd.experiments.b2t_gru_w2v_experiment import (B2TGruAndW2VArgsModel,
                                                                         trainable_param_groups, w2v_scheduler)
    model = torch.nn.Module()
    model.brain_encoder = torch.nn.Linear(4, 4)
    model.w2v_encoder = torch.nn.Linear(4, 4)
    c = B2TGruAndW2VArgsModel()
    groups = list(trainable_param_groups(model, c))
    assert len(groups) == 2 and all(isinstance(p, torch.nn.Parameter) for p in groups)
    opt = torch.optim.Adam(groups, lr=c.learning_rate)
    exp = SimpleNamespace(config=c, base_config=c)
    sch = w2v_scheduler(exp, opt)
    assert isinstance(sch, torch.optim.lr_scheduler.StepLR)
    with pytest.raises(AssertionError):
        trainable_param_groups(model, B2TGruAndW2VArgsModel(w2v_learning_rate=1e-4))
    c2 = B2TGruAndW2VArgsModel(unfreeze_strategy="brain_encoder+w2v", w2v_learning_rate=1e-4, w2v_warmup_steps=2)
    g2 = trainable_param_groups(model, c2)
    opt2 = torch.optim.Adam(g2, lr=c2.learning_rate)
    assert opt2.param_groups[1]["lr"] == 1e-4
    sch2 = w2v_scheduler(SimpleNamespace(config=c2, base_config=c2), opt2)
    seen = []
    for _ in range(3):
        seen.append(opt2.param_groups[1]["lr"])
        sch2.step()
    assert seen == [0.0, 0.5e-4, 1e-4]


def test_history_json_round_trip(tmp_path):
    from wav2vec2forbrain_amd.train.history import (DecodedPredictionBatch, EpochLosses, MetricEntry,
                                                    SingleEpochHistory, TrainHistory)

    def h(vals, dec=False):
        s = SingleEpochHistory()
        for i, v in enumerate(vals):
            s.add_batch_metric(MetricEntry({"word_error_rate": v / 10, "ctc_loss": v}, v),
                               DecodedPredictionBatch([f"P{i}"], [f"T{i}"]) if dec else None)
        return s

    th = TrainHistory([EpochLosses(h([1.0, 3.0]), h([2.0])), EpochLosses(h([0.5]), h([1.5]))], h([4.0, 6.0], True))
    assert th.epochs[0].train_losses.get_average().loss == 2.0
    assert abs(th.epochs[0].train_losses.get_average().metrics["word_error_rate"] - 0.2) < 1e-12
    p = tmp_path / "history.json"
    p.write_text(json.dumps(th.to_dict()))
    back = TrainHistory.from_json(str(p))
    assert back.to_dict() == th.to_dict()
    assert back.test_losses.decoded[1] == DecodedPredictionBatch(["P1"], ["T1"])


def test_host_error_rates():
    from wav2vec2forbrain_amd.train.evaluator import char_error_rate, cut_after_eos_token, word_error_rate
    pred = ["THE QUICK BROWN", "A LAZY DOG"]
    tgt = ["THE QUICK BROWN FOX", "A LAZY CAT"]
    assert word_error_rate(pred, tgt) == 2 / 7          # one deletion + one substitution over 7 words
    assert char_error_rate(pred, tgt) == (4 + 3) / (19 + 10)
    assert cut_after_eos_token("AB</s>CD</s>") == "AB</s>"


def test_synthetic_dataset_collate():
    from wav2vec2forbrain_amd.datasets.brain2text import SyntheticBrain2TextDataset
    from wav2vec2forbrain_amd.datasets.tokenizer import WAV2VEC2_CTC_VOCAB, create_ctc_tokenizer
    tok = create_ctc_tokenizer()
    ds = SyntheticBrain2TextDataset(5, 40, 60, seed=3)
    b = ds.get_collate_fn(tok)([ds[i] for i in range(5)])
    assert b.input.shape[0] == 5 and b.input.shape[2] == 256 and b.input.shape[1] == int(b.input_lens.max())
    for i in range(5):
        n = int(b.input_lens[i])
        assert n == ds[i].input.shape[0] and float(b.input[i, n:].abs().sum()) == 0.0
        ids = b.target[i].tolist()
        L = int(b.target_lens[i])
        assert all(x > 0 for x in ids[:L]) and all(x == 0 for x in ids[L:])
        text = "".join(" " if WAV2VEC2_CTC_VOCAB[x] == "|" else WAV2VEC2_CTC_VOCAB[x] for x in ids[:L])
        assert text == ds[i].target
