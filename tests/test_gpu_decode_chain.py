"""Chained decode (lvk_decode_greedy / lvk_decode_chain) against the per-step device path.

lvk_decode_greedy(token, n_past, n) must return exactly the tokens of n chained
lvk_eval_greedy calls and leave the KV cache in the same state (the next eval's logits
are bit-identical).  lvk_eval_greedy itself is pinned to the reference sampler
(tests/test_gpu_sampling.py) and its forward pass to the oracle.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

PROMPT = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32)


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


def _loop(m, tok, n_past, n):
    out = []
    for i in range(n):
        tok = m.eval_greedy(tok, n_past + i)
        out.append(tok)
    return np.array(out, np.int32)


def _check(lvk, path, steps, n_ctx=256, chunks=None):
    m = lvk.Llama(path, n_ctx=n_ctx)
    m.set_prompt_exact(True)
    a = m.eval(PROMPT, 0)
    tok0 = int(np.argmax(a[-1]))
    ref = _loop(m, tok0, len(PROMPT), steps)
    nxt_ref = m.eval([int(ref[-1])], len(PROMPT) + steps)[-1].copy()

    m.eval(PROMPT, 0)
    got, tok, n_past = [], tok0, len(PROMPT)
    for c in (chunks or [steps]):
        part = m.decode_greedy(tok, n_past, c)
        got.append(part)
        tok, n_past = int(part[-1]), n_past + c
    got = np.concatenate(got)
    assert np.array_equal(got, ref), (got[:16], ref[:16])
    nxt = m.eval([int(got[-1])], len(PROMPT) + steps)[-1]
    assert np.array_equal(nxt.view(np.uint32), nxt_ref.view(np.uint32))
    m.close()


def test_chain_matches_eval_greedy_tiny(lvk, tiny_models, gpu_available):
    _check(lvk, tiny_models["tiny_q4_0"], 40)
    _check(lvk, tiny_models["tiny_q4_1"], 24)


def test_chain_in_parts_7b_shaped(lvk, model_dir, gpu_available):
    """7B layer shapes (the CU matvecs, the decode attention across its n_kv 128 switch to
    the score exchange), the chain split over several calls"""
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    _check(lvk, path, 140, n_ctx=256, chunks=[1, 63, 76])


def _check_forced(lvk, path, steps, n_ctx=256):
    """a teacher-forced chain (lvk_decode_chain with a token sequence) against per-step evals of
    the same tokens: every step's device digest equals the digest of the per-step logits row,
    every argmax equals the row's, and the KV cache ends the same"""
    from oracle_lib import forced_tokens
    m = lvk.Llama(path, n_ctx=n_ctx)
    m.eval(PROMPT, 0)
    seq = forced_tokens(steps, seed=11)
    want_d, want_a = [], []
    for i in range(steps):
        row = m.eval([int(seq[i])], len(PROMPT) + i)[-1]
        want_d.append(lvk.logits_digest(row))
        want_a.append(int(np.argmax(row)))
    nxt_ref = m.eval([7], len(PROMPT) + steps)[-1].copy()
    m.eval(PROMPT, 0)
    got, dg = m.decode_chain(seq, len(PROMPT))
    assert dg.tolist() == want_d
    assert got.tolist() == want_a
    nxt = m.eval([7], len(PROMPT) + steps)[-1]
    assert np.array_equal(nxt.view(np.uint32), nxt_ref.view(np.uint32))
    # a forced prefix, then greedy: the tail equals eval_greedy's stream from the prefix's end
    m.eval(PROMPT, 0)
    got2, _ = m.decode_chain(seq[:5], len(PROMPT), 12)
    m.eval(PROMPT, 0)
    for i in range(5):
        m.eval([int(seq[i])], len(PROMPT) + i)
    tail = _loop(m, int(got2[4]), len(PROMPT) + 5, 7)
    assert got2[5:].tolist() == tail[:7].tolist()
    m.close()


def test_forced_chain_digests_tiny(lvk, tiny_models, gpu_available):
    _check_forced(lvk, tiny_models["tiny_q4_0"], 40)
    _check_forced(lvk, tiny_models["tiny_q4_1"], 24)


def test_forced_chain_digests_7b_shaped(lvk, model_dir, gpu_available):
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    _check_forced(lvk, path, 150, n_ctx=256)


def test_chain_errors(lvk, tiny_models, gpu_available):
    m = lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=64)
    m.eval(PROMPT, 0)
    with pytest.raises(RuntimeError):
        m.decode_greedy(5, 60, 8)          # runs past n_ctx
    with pytest.raises(RuntimeError):
        m.decode_greedy(40000, 8, 4)       # token id out of range
    with pytest.raises(RuntimeError):
        m.decode_greedy(5, 8, 0)           # no steps
    # the context still works
    t = m.decode_greedy(5, 8, 4)
    assert t.shape == (4,)
    m.close()
