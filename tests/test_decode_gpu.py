"""On-device greedy CTC decode + word error rate (csrc/decode.hip) against the host
path of the reference's train evaluator (src/train/evaluator.py:69-129): transformers'
Wav2Vec2CTCTokenizer.batch_decode on a local copy of the wav2vec2 32-token CTC vocabulary (the
hub tokenizer is unreachable offline; parity of the vocabulary itself is unpinned), the
cut-after-"</s>" step, and torcheval's WordErrorRate restated (sum of word edit distances over
sum of target words)."""
import json

import pytest
import torch

pytestmark = pytest.mark.gpu

VOCAB = ["<pad>", "<s>", "</s>", "<unk>", "|", "E", "T", "A", "O", "N", "I", "H", "S", "R", "D", "L", "U", "M",
         "W", "C", "F", "G", "Y", "P", "B", "V", "K", "'", "X", "J", "Q", "Z"]


def _edit(a, b):
    prev = list(range(len(b) + 1))
    for i, x in enumerate(a, 1):
        cur = [i] + [0] * len(b)
        for j, y in enumerate(b, 1):
            cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (x != y))
        prev = cur
    return prev[-1]


def _host_reference(logits, target, tok):
    pred = tok.batch_decode(logits.argmax(-1).cpu().numpy(), group_tokens=True)
    pred = [p[:p.find("</s>") + 4] if p.find("</s>") != -1 else p for p in pred]
    lab = tok.batch_decode(target.cpu().numpy(), group_tokens=False)
    errs = [_edit(p.split(), t.split()) for p, t in zip(pred, lab)]
    nw = [len(t.split()) for t in lab]
    return pred, errs, nw


def test_ctc_greedy_wer_matches_host_evaluator(tmp_path):
    from transformers import Wav2Vec2CTCTokenizer
    from wav2vec2forbrain_amd import functional as Fn
    f = tmp_path / "vocab.json"
    f.write_text(json.dumps({t: i for i, t in enumerate(VOCAB)}))
    tok = Wav2Vec2CTCTokenizer(str(f))
    g = torch.Generator().manual_seed(3)
    B, T, C, S = 12, 249, 32, 90
    # frame ids with long runs, blanks, delimiters, occasional specials; logits peaked at them
    ids = torch.randint(4, C, (B, T), generator=g)
    ids[torch.rand(B, T, generator=g) < 0.35] = 0
    ids[torch.rand(B, T, generator=g) < 0.08] = 4
    run = torch.rand(B, T, generator=g) < 0.5
    for t in range(1, T):
        ids[:, t] = torch.where(run[:, t], ids[:, t - 1], ids[:, t])
    ids[0, 100] = 2            # an EOS mid-sequence: the prediction is cut after it
    ids[1, 50:52] = 1          # <s> inside a word
    logits = torch.randn(B, T, C, generator=g)
    logits.scatter_(2, ids.unsqueeze(-1), 8.0)
    target = torch.randint(5, C, (B, S), generator=g)
    target[torch.rand(B, S, generator=g) < 0.18] = 4
    lens = torch.randint(20, S + 1, (B,), generator=g)
    target[torch.arange(S).unsqueeze(0) >= lens.unsqueeze(1)] = 0
    pred_s, errs_ref, nw_ref = _host_reference(logits, target, tok)
    wer, errs, nw, toks, ntok = Fn.ctc_greedy_wer(logits.cuda(), target.cuda())
    assert errs.cpu().tolist() == errs_ref
    assert nw.cpu().tolist() == nw_ref
    assert abs(float(wer) - sum(errs_ref) / sum(nw_ref)) < 1e-6
    for b in range(B):   # the collapsed token ids decode to the host evaluator's prediction string
        s = tok.decode(toks[b, :int(ntok[b])].cpu().tolist(), group_tokens=False)
        assert s == pred_s[b], (b, s, pred_s[b])
    # a perfect prediction: zero errors
    perfect = torch.full((1, T, C), -5.0)
    seq = [x for x in target[3].tolist() if x != 0]
    for t, x in enumerate(seq):
        perfect[0, 2 * t, x] = 5.0
        perfect[0, 2 * t + 1, 0] = 5.0
    w1, e1, n1, _, _ = Fn.ctc_greedy_wer(perfect.cuda(), target[3:4].cuda())
    assert int(e1[0]) == 0 and int(n1[0]) == nw_ref[3] and float(w1) == 0.0


def test_ctc_greedy_cer_matches_host_evaluator(tmp_path):
    """Device character error rate (csrc/decode.hip ctc_greedy_cer) vs the reference evaluator's
    calculate_char_error_rate (src/train/evaluator.py:231-242: character Levenshtein of the
    tokenizer-decoded strings, cut after "</s>", summed over the batch / summed target lengths),
    including special tokens rendered as several characters, leading/trailing delimiters and
    repeated delimiters."""
    from transformers import Wav2Vec2CTCTokenizer
    from wav2vec2forbrain_amd import functional as Fn
    f = tmp_path / "vocab.json"
    f.write_text(json.dumps({t: i for i, t in enumerate(VOCAB)}))
    tok = Wav2Vec2CTCTokenizer(str(f))
    g = torch.Generator().manual_seed(5)
    B, T, C, S = 16, 249, 32, 100
    ids = torch.randint(4, C, (B, T), generator=g)
    ids[torch.rand(B, T, generator=g) < 0.35] = 0
    ids[torch.rand(B, T, generator=g) < 0.12] = 4
    ids[torch.rand(B, T, generator=g) < 0.02] = 3           # <unk>: 5 characters
    run = torch.rand(B, T, generator=g) < 0.5
    for t in range(1, T):
        ids[:, t] = torch.where(run[:, t], ids[:, t - 1], ids[:, t])
    ids[0, 120] = 2                                          # EOS: cut after it
    ids[1, 30:33] = 1                                        # <s>
    ids[2, :6] = torch.tensor([4, 0, 4, 4, 7, 0])            # leading delimiters
    ids[3, -5:] = torch.tensor([9, 4, 0, 4, 4])              # trailing delimiters
    logits = torch.randn(B, T, C, generator=g)
    logits.scatter_(2, ids.unsqueeze(-1), 8.0)
    target = torch.randint(5, C, (B, S), generator=g)
    target[torch.rand(B, S, generator=g) < 0.18] = 4
    lens = torch.randint(20, S + 1, (B,), generator=g)
    target[torch.arange(S).unsqueeze(0) >= lens.unsqueeze(1)] = 0
    pred_s, _, _ = _host_reference(logits, target, tok)
    lab = tok.batch_decode(target.numpy(), group_tokens=False)
    errs_ref = [_edit(list(t), list(p)) for p, t in zip(pred_s, lab)]
    n_ref = [len(t) for t in lab]
    cer, errs, nch = Fn.ctc_greedy_cer(logits.cuda(), target.cuda(), VOCAB)
    assert errs.cpu().tolist() == errs_ref
    assert nch.cpu().tolist() == n_ref
    assert abs(float(cer) - sum(errs_ref) / sum(n_ref)) < 1e-6


@pytest.mark.gpu
def test_cer_overflow_row_scored_on_host(tmp_path):
    """A degenerate decode (early training: 512 alternating <unk> / blank frames over the kernel's
    1024-frame maximum = 2,560 characters, past the 2,048-character device buffer) is reported by the
    kernel as char_errs = -1, kept out of the device CER, and the evaluator scores that batch on the
    host instead of silently lowering it."""
    from transformers import Wav2Vec2CTCTokenizer
    from wav2vec2forbrain_amd import functional as Fn
    from wav2vec2forbrain_amd.model.b2tmodel import ModelOutput
    from wav2vec2forbrain_amd.train.evaluator import EvaluatorWithW2vLMDecoder, char_error_rate, cut_after_eos_token
    from wav2vec2forbrain_amd.datasets.batch_types import B2tSampleBatch
    f = tmp_path / "vocab.json"
    f.write_text(json.dumps({t: i for i, t in enumerate(VOCAB)}))
    tok = Wav2Vec2CTCTokenizer(str(f))
    B, T, C, S = 2, 1024, 32, 40
    ids = torch.zeros(B, T, dtype=torch.int64)
    ids[0, 0::2] = 3                                  # <unk> every other frame: > 2048 characters
    ids[1, :40] = torch.randint(5, C, (40,), generator=torch.Generator().manual_seed(3))
    logits = torch.full((B, T, C), -4.0)
    logits.scatter_(2, ids.unsqueeze(-1), 6.0)
    target = torch.randint(5, C, (B, S), generator=torch.Generator().manual_seed(4))
    cer, errs, nch = Fn.ctc_greedy_cer(logits.cuda(), target.cuda(), VOCAB)
    assert int(errs[0]) == -1 and int(errs[1]) >= 0
    ev = EvaluatorWithW2vLMDecoder(tok, "train")
    out = ModelOutput(logits.cuda(), {"ctc_loss": 1.0}, loss=torch.tensor(1.0, device="cuda"))
    ev.track_batch(out, B2tSampleBatch(torch.zeros(B, 1, 1).cuda(), target.cuda()))
    pred = [cut_after_eos_token(x) for x in tok.batch_decode(ids.numpy(), group_tokens=True)]
    ref = char_error_rate(pred, tok.batch_decode(target.numpy(), group_tokens=False))
    got = out.metrics["char_error_rate"]
    assert abs(got - ref) < 1e-9, (got, ref)


@pytest.mark.gpu
@pytest.mark.parametrize("beam,tmin,prune", [(16, -5.0, -10.0), (48, -1e30, -1e30), (1, -5.0, -10.0)])
def test_ctc_prefix_beam_matches_oracle(beam, tmin, prune):
    """Device prefix beam search (csrc/beam.hip) == its CPU restatement (oracle/ctc_beam_oracle.py):
    same best prefix and log probability, with and without pyctcdecode's pruning, ragged lengths."""
    from wav2vec2forbrain_amd import functional as Fn
    from oracle.ctc_beam_oracle import ctc_prefix_beam
    g = torch.Generator().manual_seed(5)
    B, T, C = 6, 50, 32
    logits = torch.randn(B, T, C, generator=g) * 2.5
    logits[:, :, 0] += 2.0            # blank-heavy, as CTC outputs are
    lens = torch.tensor([50, 47, 31, 50, 1, 0], dtype=torch.int32)
    tok, n, score = Fn.ctc_prefix_beam(logits.cuda(), lens.cuda(), beam=beam, token_min_logp=tmin,
                                       beam_prune_logp=prune)
    tok, n, score = tok.cpu().numpy(), n.cpu().numpy(), score.cpu().numpy()
    for b in range(B):
        ref, ref_score = ctc_prefix_beam(logits[b].numpy(), beam, 0, tmin, prune, int(lens[b]))
        assert tuple(tok[b, :n[b]]) == ref, (b, tok[b, :n[b]], ref)
        assert (tok[b, n[b]:] == -1).all()
        assert abs(float(score[b]) - float(ref_score)) <= 1e-4 * max(1.0, abs(float(ref_score))), (b, score[b], ref_score)


@pytest.mark.gpu
@pytest.mark.parametrize("tmin,prune,nb", [(-5.0, -10.0, 8), (-1e30, -1e30, 2)])
def test_ctc_prefix_beam_production_settings(tmin, prune, nb):
    """The reference's test decoding settings: beam 100 (pyctcdecode's default
    lm_decode_beam_width, /root/reference/src/train/evaluator.py:189-198), T' = 249 frames (a
    1,000-bin window), B = 8, the 32-token character vocabulary, ragged lengths, pyctcdecode's pruning
    constants and none. Device search == oracle (best prefix and its log probability); the device time
    of a B = 8 and a B = 32 batch is printed."""
    from wav2vec2forbrain_amd import functional as Fn
    from oracle.ctc_beam_oracle import ctc_prefix_beam
    g = torch.Generator().manual_seed(11)
    B, T, C = 8, 249, 32
    logits = torch.randn(B, T, C, generator=g) * 2.5
    logits[:, :, 0] += 2.0
    lens = torch.tensor([249, 249, 240, 200, 249, 131, 249, 64], dtype=torch.int32)
    tok, n, score = Fn.ctc_prefix_beam(logits.cuda(), lens.cuda(), beam=100, token_min_logp=tmin,
                                       beam_prune_logp=prune)
    tok, n, score = tok.cpu().numpy(), n.cpu().numpy(), score.cpu().numpy()
    for b in range(nb):
        ref, ref_score = ctc_prefix_beam(logits[b].numpy(), 100, 0, tmin, prune, int(lens[b]))
        assert tuple(tok[b, :n[b]]) == ref, (b, tok[b, :n[b]], ref)
        assert abs(float(score[b]) - float(ref_score)) <= 1e-4 * max(1.0, abs(float(ref_score))), (b, score[b], ref_score)
    for bb in (8, 32):
        lg = (torch.randn(bb, T, C, generator=g) * 2.5).cuda()
        Fn.ctc_prefix_beam(lg, beam=100, token_min_logp=tmin, beam_prune_logp=prune)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            Fn.ctc_prefix_beam(lg, beam=100, token_min_logp=tmin, beam_prune_logp=prune)
        e1.record()
        torch.cuda.synchronize()
        print(f"ctc_prefix_beam beam 100 T 249 C 32 B {bb} prune ({tmin:g}, {prune:g}): "
              f"{e0.elapsed_time(e1) / 5:.3f} ms per batch")


@pytest.mark.gpu
def test_ctc_prefix_beam_peaked_path_equals_greedy():
    """With one dominant class per frame the beam search returns the greedy (collapsed) path."""
    from wav2vec2forbrain_amd import functional as Fn
    g = torch.Generator().manual_seed(6)
    B, T, C = 3, 40, 32
    ids = torch.randint(0, C, (B, T), generator=g)
    logits = torch.full((B, T, C), -8.0)
    logits.scatter_(2, ids.unsqueeze(-1), 8.0)
    tok, n, _ = Fn.ctc_prefix_beam(logits.cuda(), beam=8)
    for b in range(B):
        col = [int(v) for i, v in enumerate(ids[b]) if (i == 0 or v != ids[b, i - 1]) and v != 0]
        assert list(tok[b, :n[b]].cpu().numpy()) == col
