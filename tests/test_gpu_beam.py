"""GPU: beam search through mocr_decode_beam.

The reference has no beam search (``beam_size`` in src/inference.py:7 is unused), so
parity is unpinned by the reference: the specification is the CPU restatement
``oracle/model_ref.py:beam_search`` (full-prefix recompute like the reference loop).
Checks:
* hypotheses (all K, rank order) token-exact vs the oracle; scores within 1e-3 (fp32
  sums of log-probs); every case asserts its own candidate margins are far above that;
* finished hypotheses retained + batch stop (EOS-boosted fc_out bias, as the golden
  EOS fixtures do);
* 256 steps with a 260-row positional table (BASELINE config 4's length): beam = 1
  equals greedy up to EOS, and beam = 4 is deterministic with scores in rank order.
Every check runs on the production beam step (the greedy step's folded kernels over the
hypothesis rows: self-attention through the slot tables, the int16 caches of bf16x3
engines) and on MOCR_VARIANT_BEAM_UNFOLDED (round 2's projection + attention kernels).
"""
import numpy as np
import pytest
import torch

from oracle import model_ref
from oracle.gen_golden import apply_eos_boost

pytestmark = pytest.mark.gpu

SCORE_TOL = 1e-3


def run_case(pkg, precision, eos_boost, steps, stop, B=2, K=4, H=96, W=320, seed=1234, variant=()):
    w = apply_eos_boost(pkg.synth.make_weights(seed, "perturbed"), eos_boost)
    imgs = pkg.synth.make_images(B, H, W, seed0=1000)
    eng = pkg.Engine(img_hw=(H, W), max_batch=B, precision=precision, max_beam=K, variant=variant)
    eng.load_weights(w)
    eng.encode(imgs)
    res = eng.beam_search(beam=K, max_steps=steps, stop=stop)
    mem = torch.from_numpy(eng.memory())
    eng.close()
    model = model_ref.build_model(w)
    # the oracle decodes from the engine's own memory: this isolates the decoder/beam
    # logic (the encoder has its own parity tests)
    seqs, scores, n = model_ref.beam_search(model, memory=mem, beam=K, max_steps=steps, stop=stop)
    return res, seqs.numpy(), scores.numpy(), n


VARIANTS = pytest.mark.parametrize("variant", [(), ("beam_unfolded",)], ids=["folded", "unfolded"])


@VARIANTS
@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_beam_matches_oracle(pkg, precision, variant):
    res, seqs, scores, n = run_case(pkg, precision, eos_boost=0.0, steps=16, stop="none", variant=variant)
    assert res.n_steps == n == 16
    np.testing.assert_array_equal(res.beams, seqs)
    assert np.abs(res.scores - scores).max() <= SCORE_TOL
    # rank order and distinct ranks well separated relative to the tolerance
    assert (np.diff(scores, axis=1) <= 0).all()
    assert np.abs(np.diff(scores, axis=1)).min() > 10 * SCORE_TOL


@VARIANTS
@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_beam_finished_hypotheses_and_stop(pkg, precision, variant):
    # EOS boosted so hypotheses finish at different steps and the batch stops early
    res, seqs, scores, n = run_case(pkg, precision, eos_boost=4.0, steps=40, stop="batch", variant=variant)
    assert res.n_steps == n < 40
    np.testing.assert_array_equal(res.beams, seqs)
    assert np.abs(res.scores - scores).max() <= SCORE_TOL
    eos = pkg.synth.EOS_ID
    for b in range(seqs.shape[0]):
        for k in range(seqs.shape[1]):
            row = res.beams[b, k]
            hits = np.nonzero(row == eos)[0]
            assert hits.size, "every hypothesis finished"
            assert (row[hits[0] + 1:] == pkg.synth.PAD_ID).all(), "finished hypotheses are padded"


@VARIANTS
def test_beam_long_sequences(pkg, variant):
    max_pos, steps, B = 260, 256, 2
    w = pkg.synth.make_weights(1234, "perturbed", max_pos=max_pos)
    imgs = pkg.synth.make_images(B, 96, 320, seed0=1000)
    eng = pkg.Engine(img_hw=(96, 320), max_batch=B, precision="fp32", max_pos=max_pos, max_beam=4, variant=variant)
    eng.load_weights(w)
    eng.encode(imgs)
    g = eng.decode(max_steps=steps, stop="none")
    b1 = eng.beam_search(beam=1, max_steps=steps, stop="none")
    eos = pkg.synth.EOS_ID
    for b in range(B):
        row = g.ids[b]
        hits = np.nonzero(row == eos)[0]
        end = hits[0] + 1 if hits.size else row.size
        np.testing.assert_array_equal(b1.ids[b, :end], row[:end])
    r1 = eng.beam_search(beam=4, max_steps=steps, stop="none")
    r2 = eng.beam_search(beam=4, max_steps=steps, stop="none")
    eng.close()
    assert r1.n_steps == steps
    np.testing.assert_array_equal(r1.beams, r2.beams)
    np.testing.assert_array_equal(r1.scores, r2.scores)
    assert (np.diff(r1.scores, axis=1) <= 0).all()
