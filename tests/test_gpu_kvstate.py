"""Device-side KV state: lvk_kv_copy hands a prompt prefix's K/V from
one context to another in HBM; the receiving context then decodes exactly as the
source would (bit-identical logits), and as a context that evaluated the prefix itself."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("name", ["tiny_q4_0", "tiny_q4_1"])
def test_kv_copy_prefix_then_decode(lvk, tiny_models, name):
    path = tiny_models[name]
    a = lvk.Llama(path, n_ctx=128)
    b = lvk.Llama(path, n_ctx=128)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263, 1243, 29889], np.int32)
    la = a.eval(toks, 0)
    b.eval(np.array([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15], np.int32), 0)   # stale contents
    b.kv_copy_from(a, len(toks))
    assert b.kv_cache_token_count() == len(toks)
    n_past, tok = len(toks), int(np.argmax(la[-1]))
    for _ in range(12):
        la = a.eval([tok], n_past)
        lb = b.eval([tok], n_past)
        assert np.array_equal(bits(la), bits(lb)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(la[-1]))
    a.close()
    b.close()


def test_kv_copy_partial_prefix_matches_fresh_context(lvk, tiny_models):
    """copy only the first 6 of 10 positions, re-evaluate the rest: same as a context that
    re-evaluates them over its own prefix"""
    path = tiny_models["tiny_q4_0"]
    a = lvk.Llama(path, n_ctx=128)
    b = lvk.Llama(path, n_ctx=128)
    c = lvk.Llama(path, n_ctx=128)
    for m in (a, b, c):
        m.set_prompt_exact(True)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263, 1243, 29889], np.int32)
    a.eval(toks, 0)
    b.kv_copy_from(a, 6)
    lb = b.eval(toks[6:], 6)
    c.eval(toks, 0)                   # same chunking as a for the prefix (SURVEY.md finding 7)
    lc = c.eval(toks[6:], 6)
    assert np.array_equal(bits(lb), bits(lc))
    for m in (a, b, c):
        m.close()


def test_kv_copy_errors(lvk, tiny_models):
    a = lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=128)
    b = lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=64)
    with pytest.raises(RuntimeError):
        b.kv_copy_from(a, 4)          # n_ctx differs
    with pytest.raises(RuntimeError):
        a.kv_copy_from(a, 4)          # same context
    c = lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=128)
    with pytest.raises(RuntimeError):
        c.kv_copy_from(a, 129)        # beyond n_ctx
    for m in (a, b, c):
        m.close()
