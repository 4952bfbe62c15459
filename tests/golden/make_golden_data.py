"""Generates tests/golden/data_pipeline.npz by running THE REFERENCE's own data pipeline
(/root/reference/src/datasets/brain2text.py Brain2TextDataset + its collate function, which call
src/datasets/preprocessing.py) on the synthetic session files of tests/golden/mat_sessions.py.
The tokenizer passed to the reference collate is the offline wav2vec2 CTC tokenizer
(wav2vec2forbrain_amd/datasets/tokenizer.py; the hub one is unreachable).

Runs only in the build container (reads /root/reference). usage: python tests/golden/make_golden_data.py
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from tests.golden.mat_sessions import write_splits  # noqa: E402
from wav2vec2forbrain_amd.datasets.tokenizer import create_ctc_tokenizer  # noqa: E402

PREPROC = ["seperate_zscoring", "competition_recommended", "only_tx_unnormalized", "seperate_zscoring_2channels"]


def main():
    sys.path.insert(0, "/root/reference")
    sys.dont_write_bytecode = True
    from src.args.base_args import B2TDatasetArgsModel
    from src.args.yaml_config import YamlConfigModel
    from src.datasets.brain2text import Brain2TextDataset
    tok = create_ctc_tokenizer()
    root = write_splits(tempfile.mkdtemp(prefix="b2p_mat_"))
    yc = YamlConfigModel(cache_dir="/tmp", fig_dir="/tmp", n3gram_lm_model_path="", n5gram_lm_model_path="",
                         dataset_splits_dir=root, wandb_api_key="", timit_dataset_splits_dir="",
                         elevenlabs_api_key=None)
    out = {}
    for pre in PREPROC:
        for split in ("train", "val", "test"):
            cfg = B2TDatasetArgsModel(preprocessing=pre)
            ds = Brain2TextDataset(cfg, yc, split, tok)
            key = f"{pre}/{split}"
            items = [ds[i] for i in range(len(ds))]
            out[key + "/n"] = np.array(len(items))
            out[key + "/x"] = np.concatenate([x.reshape(-1).numpy() for x, _ in items]).astype(np.float32)
            out[key + "/shapes"] = np.array([list(x.shape) + [0] * (3 - x.dim()) for x, _ in items])
            out[key + "/day"] = np.array([s.day_idx for s in items])
            out[key + "/text"] = np.array([t for _, t in items])
            batch = ds.get_collate_fn(tok)(items[:3])
            out[key + "/batch_input"] = batch.input.numpy().astype(np.float32)
            out[key + "/batch_target"] = batch.target.numpy()
            out[key + "/batch_day"] = batch.day_idxs.numpy()
            out[key + "/batch_input_lens"] = batch.input_lens.numpy()
            out[key + "/batch_target_lens"] = batch.target_lens.numpy()
    np.savez_compressed(os.path.join(REPO, "tests", "golden", "data_pipeline.npz"), **out)
    print("wrote", len(out), "arrays")


if __name__ == "__main__":
    torch.manual_seed(0)
    main()
