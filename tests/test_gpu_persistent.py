"""The persistent single-token decode kernel (decode_persistent.hip, parked: only in the
dev build lib/dev, opt-in through lvk_set_decode_persistent) against the reference goldens and the CPU oracle, bit for
bit: tiny Q4_0 models (the reference build's golden logits), a 70-step decode across
the f16-dot tail boundaries, LLaMA-7B layer shapes (n_embd 4096, 32 heads, n_ff 11008)
and LLaMA-65B layer shapes (n_embd 8192, 64 heads, n_ff 22016)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    if not m.dev_kernels():
        pytest.skip("parked kernel: run with LVK_LIB=llama.vk_amd/lib/dev/libllama_vk_amd.so")
    return m


def persistent(lvk, path, n_ctx):
    m = lvk.Llama(path, n_ctx=n_ctx)
    m.set_decode_persistent(True)
    m.set_prompt_exact(True)
    return m


@pytest.mark.parametrize("name,graph", [("tiny_q4_0", True), ("tiny_q4_0", False), ("tiny_l80_q4_0", True)])
def test_persistent_matches_reference_golden(lvk, tiny_models, name, graph):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    m = persistent(lvk, tiny_models[name], 512)
    m.set_graph(graph)
    n_past, off, decoded = 0, 0, 0
    for step, n in enumerate(g["chunks"]):
        lg = m.eval(g["tokens"][off:off + n], n_past)
        if n == 1:
            assert m.decode_persistent_active()
            decoded += 1
        assert np.array_equal(bits(lg[-1]), bits(g["logits"][step])), "step %d (n=%d, n_past=%d)" % (step, n, n_past)
        n_past += n
        off += n
    assert decoded > 0
    m.close()


def test_persistent_long_decode_vs_oracle(lvk, oracle, tiny_models):
    path = tiny_models["tiny_q4_0"]
    m = persistent(lvk, path, 256)
    om = oracle.model(path, 256)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    n_past, tok = len(toks), int(np.argmax(a[-1]))
    for _ in range(70):
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(a[-1]))
    m.close()
    om.close()


@pytest.mark.parametrize("cfg,n_ctx,steps", [
    (dict(n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=1), 512, 6),
    (dict(n_embd=8192, n_head=64, n_layer=1, ftype=2, seed=3), 512, 4),
], ids=["7b_shaped", "65b_shaped"])
def test_persistent_shapes_vs_oracle(lvk, oracle, model_dir, cfg, n_ctx, steps):
    from oracle_lib import gen_model, prompt_tokens
    path = gen_model(os.path.join(model_dir, "p_w%d_l%d.bin" % (cfg["n_embd"], cfg["n_layer"])), **cfg)
    m = persistent(lvk, path, n_ctx)
    om = oracle.model(path, n_ctx)
    toks = prompt_tokens(8)
    tok = int(np.argmax(m.eval(toks, 0)[-1]))
    om.eval(toks, 0)
    for i in range(steps):
        a = m.eval([tok], 8 + i)
        assert m.decode_persistent_active()
        b = om.eval([tok], 8 + i)
        assert np.array_equal(bits(a), bits(b)), "decode step %d" % i
        tok = int(np.argmax(a[-1]))
    m.close()
    om.close()
