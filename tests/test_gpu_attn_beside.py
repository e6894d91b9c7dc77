"""Decode attention overlapped with QKV, two forms (lvk_attn_mode): beside the QKV launch on a
second stream (LVK_ATTN_BESIDE=1, mode 1; lvk_context.cpp beside_fits) and inside it
(LVK_QKV_ATTN=1, mode 2; matvec_cu.hip k_qkv_attn, 7B shapes).  Either way the attention reads
the rows of positions < n_past from the KV cache and takes the new position's q / k / v as
tagged granules from the QKV epilogue (matvec_common.h qkv_epilogue; attention_decode_dev.h QB).  The logits
must stay bit-identical to the oracle (llama.cpp:1010-1061, ggml.c:1781-1815,7062-7130) on
the short path (n_kv <= 128) and the score exchange (n_kv > 128), per step and chained, and a
shape whose two roles cannot be guaranteed co-resident (the 65B QKV's 12 waves at 134 VGPRs;
Q4_1 for the merged form) must fall back to the sequential order (mode 0)."""
import os

import numpy as np
import pytest

from oracle_lib import gen_model, prompt_tokens

pytestmark = pytest.mark.gpu


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


ENV = {1: "LVK_ATTN_BESIDE", 2: "LVK_QKV_ATTN"}


@pytest.fixture(params=[1, 2])
def mode(request, monkeypatch):
    for v in ENV.values():
        monkeypatch.delenv(v, raising=False)
    monkeypatch.setenv(ENV[request.param], "1")
    return request.param


def _decode_vs_oracle(lvk, oracle, path, prompt, steps, expect_mode, n_ctx=512):
    m = lvk.Llama(path, n_ctx=n_ctx)
    assert m.attn_mode() == expect_mode
    om = oracle.model(path, n_ctx)
    toks = np.array(prompt, np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past, tok = len(toks), int(np.argmax(a[-1]))
    for _ in range(steps):
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(a[-1]))
    m.close()
    om.close()


@pytest.mark.parametrize("n_prompt, steps", [(8, 12), (120, 14)])
def test_beside_7b_shaped_matches_oracle(lvk, oracle, model_dir, mode, n_prompt, steps):
    """7B layer shapes, 2 layers: positions 8..19 (every workgroup scores all positions) and
    120..133 (crossing into the score exchange at n_kv 129)"""
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    prompt = [1, 450, 4996, 17354, 1701, 29916, 338, 263] if n_prompt == 8 else prompt_tokens(n_prompt)
    _decode_vs_oracle(lvk, oracle, path, prompt, steps, mode)


def test_beside_13b_shaped_q4_1_matches_oracle(lvk, oracle, model_dir, mode):
    """13B Q4_1 layer shapes (n_embd 5120, 40 heads): beside, the Q4_1 QKV epilogue publishes
    the granules; the merged form is Q4_0-only and falls back"""
    path = gen_model(os.path.join(model_dir, "w5120_l2_q41.bin"), ftype=3, n_embd=5120, n_head=40, n_layer=2, seed=11)
    _decode_vs_oracle(lvk, oracle, path, [1, 450, 4996, 17354, 1701, 29916], 10, 1 if mode == 1 else 0, n_ctx=256)


def test_beside_65b_shaped_falls_back(lvk, oracle, model_dir, mode):
    """65B layer shapes: the QKV launch (12 waves x 134 VGPRs per CU) and an attention
    workgroup cannot share a CU's registers, so the attention stays after QKV"""
    path = gen_model(os.path.join(model_dir, "w8192_l2.bin"), n_embd=8192, n_head=64, n_layer=2, ftype=2, seed=13)
    _decode_vs_oracle(lvk, oracle, path, [1, 450, 4996, 17354, 1701, 29916, 338, 263], 4, 0)


@pytest.mark.parametrize("on", [1, 2])
def test_beside_chained_greedy_matches_sequential(lvk, model_dir, monkeypatch, on):
    """lvk_decode_greedy (the step graph replayed back to back) and per-step lvk_eval_greedy
    beside QKV produce the token stream of a context without it, across n_kv 128"""
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    streams = {}
    for md in (0, on):
        for v in ENV.values():
            monkeypatch.delenv(v, raising=False)
        if md:
            monkeypatch.setenv(ENV[md], "1")
        m = lvk.Llama(path, n_ctx=256)
        assert m.attn_mode() == md
        lg = m.eval(prompt_tokens(16), 0)
        tok = int(np.argmax(lg[-1]))
        step = []
        t = tok
        for i in range(130):
            t = m.eval_greedy(t, 16 + i)
            step.append(t)
        m.close()
        m = lvk.Llama(path, n_ctx=256)
        lg = m.eval(prompt_tokens(16), 0)
        chained = m.decode_greedy(int(np.argmax(lg[-1])), 16, 130)
        m.close()
        assert list(chained) == step
        streams[md] = step
    assert streams[0] == streams[on]
