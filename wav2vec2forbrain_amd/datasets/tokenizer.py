"""The CTC character tokenizer of the reference experiments, built offline.

The reference loads `AutoTokenizer.from_pretrained(tokenizer_checkpoint)` (default
facebook/wav2vec2-base-100h, src/experiments/b2t_experiment.py:37-48), a transformers
Wav2Vec2CTCTokenizer over the wav2vec2 32-token character vocabulary. The hub is unreachable here,
so the same tokenizer class is constructed from a local copy of that vocabulary (ids 0-3 the
special tokens, 4 the word delimiter "|", then the letters by frequency and the apostrophe). The
vocabulary itself cannot be checked against the hub offline: parity unpinned, as SURVEY 8(d2) notes.
"""
from __future__ import annotations

import json
import os
import tempfile

WAV2VEC2_CTC_VOCAB = ["<pad>", "<s>", "</s>", "<unk>", "|", "E", "T", "A", "O", "N", "I", "H", "S", "R", "D",
                      "L", "U", "M", "W", "C", "F", "G", "Y", "P", "B", "V", "K", "'", "X", "J", "Q", "Z"]

_CACHE: dict = {}


def create_ctc_tokenizer(cache_dir: str | None = None):
    """A transformers Wav2Vec2CTCTokenizer over WAV2VEC2_CTC_VOCAB (pad = CTC blank = id 0)."""
    from transformers import Wav2Vec2CTCTokenizer
    key = cache_dir or ""
    if key not in _CACHE:
        d = cache_dir or tempfile.mkdtemp(prefix="b2p_tok_")
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "wav2vec2_ctc_vocab.json")
        with open(path, "w") as f:
            json.dump({t: i for i, t in enumerate(WAV2VEC2_CTC_VOCAB)}, f)
        _CACHE[key] = Wav2Vec2CTCTokenizer(path, unk_token="<unk>", pad_token="<pad>", bos_token="<s>",
                                           eos_token="</s>", word_delimiter_token="|")
    return _CACHE[key]


def vocab_of(tokenizer) -> list[str]:
    """Token strings by id (reference B2TExperiment.get_vocab, src/experiments/b2t_experiment.py:101-104)."""
    return tokenizer.convert_ids_to_tokens(list(range(tokenizer.vocab_size)))
