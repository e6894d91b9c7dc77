"""On-device greedy sampling against the reference's greedy rule.

The reference picks, for temp <= 0, the first index whose logit is strictly
greater than every earlier one (llama.cpp:1382-1394).  `ref_greedy` restates
that loop; the device argmax (lvk_argmax) and the greedy decode step
(lvk_eval_greedy) must choose the same token on the same logits, including
ties, -inf rows and NaN entries.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def ref_greedy(row):
    """llama.cpp:1382-1394, element by element"""
    best, idx = row[0], 0
    for i in range(1, len(row)):
        if row[i] > best:
            best, idx = row[i], i
    return idx


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


def _cases():
    rng = np.random.default_rng(5)
    yield "random_32000", rng.standard_normal(32000).astype(np.float32)
    x = rng.standard_normal(32000).astype(np.float32)
    x[[17, 9000, 31999]] = 9.0
    yield "ties_first_wins", x
    yield "all_equal", np.full(4097, 2.5, np.float32)
    yield "all_neg_inf", np.full(1000, -np.inf, np.float32)
    x = np.full(3000, -np.inf, np.float32)
    x[2999] = -1e30
    yield "max_at_last", x
    x = rng.standard_normal(5000).astype(np.float32)
    x[0] = np.nan
    yield "nan_at_0", x
    x = rng.standard_normal(5000).astype(np.float32)
    x[[3, 70, 4999]] = np.nan
    x[1234] = 50.0
    yield "nan_inside", x
    yield "single", np.array([-3.0], np.float32)
    yield "n_1025", rng.standard_normal(1025).astype(np.float32)
    x = np.zeros(2048, np.float32)
    x[1] = -0.0
    x[5] = np.float32(1e-45)
    yield "signed_zero_denormal", x


@pytest.mark.parametrize("name,x", list(_cases()), ids=[c[0] for c in _cases()])
def test_device_argmax_matches_reference_rule(lvk, name, x):
    assert lvk.argmax(x) == ref_greedy(x.tolist())


@pytest.mark.parametrize("graph", [True, False])
def test_greedy_decode_matches_host_greedy(lvk, tiny_models, graph):
    """eval_greedy's token stream equals llama_eval + the reference's greedy over host logits"""
    path = tiny_models["tiny_q4_0"]
    a = lvk.Llama(path, n_ctx=256)
    b = lvk.Llama(path, n_ctx=256)
    a.set_graph(graph)
    b.set_graph(graph)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
    la = a.eval(toks, 0)
    b.eval(toks, 0)
    n_past, tok = len(toks), ref_greedy(la[-1].tolist())
    for _ in range(40):
        la = a.eval([tok], n_past)
        want = ref_greedy(la[-1].tolist())
        got = b.eval_greedy(tok, n_past)
        assert got == want, "n_past %d" % n_past
        n_past += 1
        tok = want
    # both contexts hold the same KV cache afterwards
    assert np.array_equal(a.kv_cache(), b.kv_cache())
    a.close()
    b.close()


def test_greedy_decode_7b_shaped_vs_oracle(lvk, oracle, model_dir):
    """LLaMA-7B layer shapes (2 layers): the device greedy tokens follow the oracle's logits"""
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    m = lvk.Llama(path, n_ctx=512)
    m.set_prompt_exact(True)
    om = oracle.model(path, 512)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32)
    m.eval(toks, 0)
    b = om.eval(toks, 0)
    n_past, tok = len(toks), ref_greedy(b[-1].tolist())
    for _ in range(10):
        got = m.eval_greedy(tok, n_past)
        b = om.eval([tok], n_past)
        assert got == ref_greedy(b[-1].tolist()), "n_past %d" % n_past
        n_past += 1
        tok = got
    m.close()
    om.close()


def test_greedy_decode_errors(lvk, tiny_models):
    m = lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=64)
    with pytest.raises(RuntimeError):
        m.eval_greedy(10 ** 6, 0)          # token id out of range
    with pytest.raises(RuntimeError):
        m.eval_greedy(1, 64)               # n_past + 1 > n_ctx
    assert m.eval_greedy(1, 0) >= 0        # the context still works
    m.close()


@pytest.mark.parametrize("top_k,top_p,temp,rp", [(40, 0.95, 0.8, 1.1), (0, 1.0, 1.0, 1.0), (5, 0.5, 0.3, 1.3),
                                                 (1, 0.9, 2.0, 1.1), (40, 0.95, 0.0, 1.1)])
def test_host_sampler_matches_reference_build(lvk, ref, tiny_models, top_k, top_p, temp, rp):
    """llama_sample_top_p_top_k against the reference build (oracle/_ref/libref.so) over a
    40-step sampled decode: same seed (1), same last_n window (main.cpp's 64 zeros then the
    tokens), bit-identical logits -> the same token stream"""
    path = tiny_models["tiny_q4_0"]
    m = lvk.Llama(path, n_ctx=256, seed=1)
    m.set_prompt_exact(True)
    r = ref.model(path, 256)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
    last = [0] * (64 - len(toks)) + toks.tolist()
    a = m.eval(toks, 0)
    b = r.eval(toks, 0)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    n_past = len(toks)
    for step in range(40):
        want = r.sample(last, top_k, top_p, temp, rp)
        got = m.sample(last, top_k=top_k, top_p=top_p, temp=temp, repeat_penalty=rp)
        assert got == want, "step %d" % step
        last = last[1:] + [got]
        m.eval([got], n_past)
        r.eval([got], n_past)
        n_past += 1
    m.close()
    r.close()


# ---------------------------------------------------------------------------
# device sampler (sample.hip, lvk_eval_sample): the O(n_vocab) part of
# llama_sample_top_p_top_k on the GPU, the rest on the host over k candidates
# ---------------------------------------------------------------------------
def _ref_values(x, last, temp, rp):
    """the (value) array the reference sorts (llama.cpp:1398-1414), float32 ops in its order"""
    x = np.asarray(x, np.float32)
    scale = np.float32(1.0) / np.float32(temp)
    s = (x * scale).astype(np.float32)
    v = s.copy()
    inl = np.zeros(x.size, bool)
    for t in last:
        if 0 <= t < x.size:
            inl[t] = True
    neg = x < 0
    v[inl & neg] = (s[inl & neg] * np.float32(rp)).astype(np.float32)
    v[inl & ~neg] = (s[inl & ~neg] / np.float32(rp)).astype(np.float32)
    return v


@pytest.mark.parametrize("n,k,temp,rp,nl", [(32000, 40, 0.8, 1.1, 64), (32000, 1, 2.0, 1.3, 0), (1000, 1000, 1.0, 1.0, 8),
                                             (32000, 1024, 0.3, 1.1, 1024), (7, 3, 0.5, 2.0, 3)])
def test_sample_candidates_random(lvk, n, k, temp, rp, nl):
    """device candidates = every value >= the k-th largest of the reference's scaled/penalized
    values, bit-exact values"""
    rng = np.random.default_rng(n + k)
    x = (rng.standard_normal(n) * 3).astype(np.float32)
    last = rng.integers(0, n, nl).astype(np.int32)
    vals, ids, flags, cnt = lvk.sample_candidates(x, last, k, temp, rp)
    want = _ref_values(x, last, temp, rp)
    kth = np.sort(want)[::-1][k - 1]
    sel = np.nonzero(want >= kth)[0]
    assert flags == 0 and cnt == sel.size
    assert sorted(ids.tolist()) == sel.tolist()
    assert np.array_equal(vals.view(np.uint32), want[ids].view(np.uint32))


def test_sample_candidates_ties_signed_zero_nan(lvk):
    """ties at the k-th value all come out (the host then takes the reference path), +0 / -0
    count as equal, NaN raises the flag"""
    x = np.array([1.0, 5.0, 3.0, 3.0, 3.0, -2.0, 0.5], np.float32)
    vals, ids, flags, cnt = lvk.sample_candidates(x, [], 3, 1.0, 1.0)
    assert flags == 0 and cnt == 4 and sorted(ids.tolist()) == [1, 2, 3, 4]
    z = np.array([-1.0, 0.0, -0.0, -3.0], np.float32)
    vals, ids, flags, cnt = lvk.sample_candidates(z, [], 2, 1.0, 1.0)
    assert sorted(ids.tolist()) == [1, 2] and cnt == 2
    vals, ids, flags, cnt = lvk.sample_candidates(z, [], 1, 1.0, 1.0)
    assert sorted(ids.tolist()) == [1, 2]          # +0 is the max, -0 equals it
    nanx = np.array([1.0, np.nan, 2.0], np.float32)
    assert lvk.sample_candidates(nanx, [], 1, 1.0, 1.0)[2] & 1


@pytest.mark.parametrize("top_k,top_p,temp,rp", [(40, 0.95, 0.8, 1.1), (5, 0.5, 0.3, 1.3), (1, 0.9, 2.0, 1.1),
                                                 (1024, 0.99, 1.5, 1.05), (0, 1.0, 1.0, 1.0), (40, 0.95, 0.0, 1.1)])
def test_device_sampler_matches_reference_build(lvk, ref, tiny_models, top_k, top_p, temp, rp):
    """lvk_eval_sample (decode step + device top-k candidates + host tail) against the
    reference build's llama_eval + llama_sample_top_p_top_k over 40 sampled steps: the same
    token stream from the same seed (top_k 0 takes the all-logits path, temp 0 the argmax)"""
    path = tiny_models["tiny_q4_0"]
    m = lvk.Llama(path, n_ctx=256, seed=1)
    m.set_prompt_exact(True)
    r = ref.model(path, 256)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
    last = [0] * (64 - len(toks)) + toks.tolist()
    m.eval(toks, 0)
    r.eval(toks, 0)
    n_past = len(toks)
    want = r.sample(last, top_k, top_p, temp, rp)
    got = m.sample(last, top_k=top_k, top_p=top_p, temp=temp, repeat_penalty=rp)
    assert got == want
    for step in range(40):
        last = last[1:] + [want]
        r.eval([want], n_past)
        want = r.sample(last, top_k, top_p, temp, rp)
        got = m.eval_sample(got, n_past, last, top_k=top_k, top_p=top_p, temp=temp, repeat_penalty=rp)
        assert got == want, "step %d" % step
        n_past += 1
    m.close()
    r.close()


def test_device_sampler_7b_shaped_vs_host_sampler(lvk, model_dir):
    """on a 7B-shaped model (n_vocab 32000, 2 layers) the device sampler and the host sampler
    of two contexts with the same seed give the same 24-token stream"""
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    a = lvk.Llama(path, n_ctx=256, seed=5)
    b = lvk.Llama(path, n_ctx=256, seed=5)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32)
    a.eval(toks, 0)
    b.eval(toks, 0)
    last = [0] * (64 - len(toks)) + toks.tolist()
    ta = a.sample(last)
    tb = b.sample(last)
    assert ta == tb
    n_past = len(toks)
    for _ in range(24):
        last = last[1:] + [ta]
        ta = a.eval_sample(ta, n_past, last)
        b.eval([tb], n_past)
        tb = b.sample(last)
        assert ta == tb
        n_past += 1
    a.close()
    b.close()
