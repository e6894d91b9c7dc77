"""Whole-model parity through the drop-in llama.h API on the GPU.

The tiny seeded models are evaluated with the reference's chunking (prompt
batches then single-token decode, SURVEY.md finding 7) and compared
bit-for-bit with (a) the golden logits produced by the reference build and
(b) the CPU oracle on the same inputs.
"""
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
    return m


# exact: the prompt chunks of >= 16 tokens on the VALU kernels (True) or on the shipped MFMA
# kernels (False, the default); both are bit-identical to the reference
@pytest.mark.parametrize("name,graph,exact", [("tiny_q4_0", True, True), ("tiny_q4_0", True, False),
                                              ("tiny_q4_0", False, False), ("tiny_q4_1", True, True),
                                              ("tiny_q4_1", True, False), ("tiny_l80_q4_0", True, False)])
def test_tiny_matches_reference_golden(lvk, tiny_models, name, graph, exact):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    m = lvk.Llama(tiny_models[name], n_ctx=512)
    m.set_graph(graph)
    m.set_prompt_exact(exact)
    n_past, off = 0, 0
    for step, n in enumerate(g["chunks"]):
        lg = m.eval(g["tokens"][off:off + n], n_past)
        assert np.array_equal(bits(lg[-1]), bits(g["logits"][step])), "step %d (n=%d, n_past=%d)" % (step, n, n_past)
        n_past += n
        off += n
    m.close()


def test_tiny_q4_0_long_decode_vs_oracle(lvk, oracle, tiny_models):
    path = tiny_models["tiny_q4_0"]
    m = lvk.Llama(path, n_ctx=256)
    om = oracle.model(path, 256)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past = len(toks)
    tok = int(np.argmax(a[-1]))
    for _ in range(130):         # crosses the 32/64-position f16-dot tail boundaries and, past
                                 # n_kv 128, the switch to the cross-workgroup score exchange
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(a[-1]))
    m.close()
    om.close()


@pytest.mark.parametrize("exact", [True, False])
def test_logits_all_and_embeddings(lvk, oracle, tiny_models, exact):
    path = tiny_models["tiny_q4_0"]
    m = lvk.Llama(path, n_ctx=128, logits_all=True, embedding=True)
    m.set_prompt_exact(exact)
    om = oracle.model(path, 128)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 40)], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0, logits_all=True)
    assert a.shape == (40, m.n_vocab)
    assert np.array_equal(bits(a), bits(b))
    e = m.embeddings()
    assert e.shape == (m.n_embd,) and np.isfinite(e).all()
    m.close()
    om.close()


def test_kv_cache_roundtrip(lvk, tiny_models):
    path = tiny_models["tiny_q4_0"]
    m = lvk.Llama(path, n_ctx=128)
    toks = np.arange(1, 20, dtype=np.int32)
    m.eval(toks, 0)
    kv = m.kv_cache()
    a = m.eval([42], 19)
    m2 = lvk.Llama(path, n_ctx=128)
    m2.set_kv_cache(kv, 19)
    b = m2.eval([42], 19)
    assert np.array_equal(bits(a), bits(b))
    m.close()
    m2.close()


def test_eval_errors(lvk, tiny_models):
    m = lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=64)
    with pytest.raises(RuntimeError):
        m.eval(np.arange(1, 70, dtype=np.int32), 0)     # exceeds n_ctx -> llama_eval returns 1
    with pytest.raises(RuntimeError):
        m.eval([40000], 0)                              # token id out of range
    m.close()


@pytest.mark.parametrize("n_prompt", [8, 24])
def test_7b_shaped_decode_vs_oracle(lvk, oracle, model_dir, n_prompt):
    """LLaMA-7B layer shapes (n_embd 4096, n_ff 11008, 32 heads) with 2 layers:
    the decode path runs the CU-balanced kernels compiled for K = 4096 / 11008
    (matvec_cu.hip); the 8-token prompt runs the generic kernels, the
    24-token one the MFMA matmuls.  Bit-exact vs oracle."""
    from oracle_lib import gen_model, prompt_tokens
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    m = lvk.Llama(path, n_ctx=512)
    om = oracle.model(path, 512)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32) if n_prompt == 8 else \
        np.array(prompt_tokens(n_prompt), np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past, tok = len(toks), int(np.argmax(a[-1]))
    for _ in range(12):
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(a[-1]))
    m.close()
    om.close()


@pytest.mark.parametrize("cfg,steps", [(dict(n_embd=5120, n_head=40, n_layer=2, seed=11), 12),
                                       (dict(n_embd=4096, n_head=32, n_layer=2, seed=12), 8)])
def test_q4_1_shaped_decode_vs_oracle(lvk, oracle, model_dir, cfg, steps):
    """LLaMA-13B (n_embd 5120, n_ff 13824, 40 heads) and 7B layer shapes in Q4_1, 2 layers:
    Q4_1 quantizer, the CU-balanced Q4_1 decode matvecs (matvec_cu41.hip: QKV + RoPE, Wo,
    W1|W3 -> f32 u, W2 quantizing u, lm_head) and the attention output quantization on
    the GPU, bit-exact against the oracle over a prompt and `steps` decode positions."""
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w%d_l2_q41.bin" % cfg["n_embd"]), ftype=3, **cfg)
    m = lvk.Llama(path, n_ctx=256)
    om = oracle.model(path, 256)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
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
    # every decode matrix ran on the CU-balanced kernels: one launch per matrix and layer
    m.set_profiling(True)
    m.reset_profile()
    m.eval([tok], n_past)
    pr = m.profile()
    assert pr["qkv"]["launches"] == 2 and pr["wo"]["launches"] == 2 and pr["w2"]["launches"] == 2
    m.close()
    om.close()


# ---------------------------------------------------------------------------
# MFMA prompt path (default for N > 1): bit-exact like the VALU path.
# ---------------------------------------------------------------------------
def test_mfma_prompt_tiny_logits_all_vs_oracle(lvk, oracle, tiny_models):
    """every position of a 100-token prompt (logits_all) through the MFMA matmuls"""
    path = tiny_models["tiny_q4_0"]
    m = lvk.Llama(path, n_ctx=256, logits_all=True)
    om = oracle.model(path, 256)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 100)], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0, logits_all=True)
    assert a.shape == b.shape == (100, m.n_vocab)
    assert np.array_equal(bits(a), bits(b))
    m.close()
    om.close()


@pytest.mark.parametrize("name", ["tiny_q4_0", "tiny_q4_1"])
def test_mfma_prompt_chunks_match_reference_golden(lvk, tiny_models, name):
    """the reference's chunking (prompt batches 16, 8, 24, then decode) with MFMA prompt batches,
    against the logits the reference build produced"""
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    m = lvk.Llama(tiny_models[name], n_ctx=512)
    n_past, off = 0, 0
    for step, n in enumerate(g["chunks"]):
        lg = m.eval(g["tokens"][off:off + n], n_past)
        assert np.array_equal(bits(lg[-1]), bits(g["logits"][step])), "step %d (n=%d, n_past=%d)" % (step, n, n_past)
        n_past += n
        off += n
    m.close()


@pytest.mark.parametrize("a16,rope,swq", [("1", "1", "1"), ("0", "1", "1"), ("1", "0", "0")])
def test_mfma_prompt_7b_shaped_vs_oracle(lvk, oracle, model_dir, monkeypatch, a16, rope, swq):
    """LLaMA-7B layer shapes (K = 4096 / 11008, 32 heads), 2 layers, a 200-token prompt (ragged
    last token tile) through the MFMA matmuls -- A operands from the f16 A-fragment images
    (default) or unpacked from the nibble images (LVK_PROMPT_A16=0); RoPE + KV append in the QKV
    matmul's epilogue (default) or by k_rope_kv (LVK_MM_ROPE=0); the W2 input quantized in the
    W1|W3 epilogue (default) or by k_act_q40_f16_tile (LVK_MM_SWIGLU_Q=0) -- then decode on the
    KV cache it wrote"""
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    monkeypatch.setenv("LVK_PROMPT_A16", a16)
    monkeypatch.setenv("LVK_MM_ROPE", rope)
    monkeypatch.setenv("LVK_MM_SWIGLU_Q", swq)
    m = lvk.Llama(path, n_ctx=512)
    om = oracle.model(path, 512)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 200)], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past, tok = len(toks), int(np.argmax(b[-1]))
    for _ in range(4):
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(b[-1]))
    m.close()
    om.close()


@pytest.mark.parametrize("n_ctx,rope", [(256, "1"), (2048, "1"), (256, "0")])
def test_mfma_prompt_13b_q4_1_shaped_vs_oracle(lvk, oracle, model_dir, monkeypatch, n_ctx, rope):
    """LLaMA-13B layer shapes in Q4_1 (K = 5120 / 13824, 40 heads), 2 layers: a 100-token
    prompt (ragged token tile) through the Q4_1 MFMA matmuls (mm_mfma41.hip), then decode on
    the KV cache it wrote, bit-exact against the oracle.  The Wo input comes from the prompt
    attention's fused Q4_1 epilogue (n_ctx 256) or from the generic attention's ActQ via
    launch_actq41_to_f16 (n_ctx 2048, past the prompt attention's LDS window); RoPE + KV append
    in the QKV matmul's epilogue (default) or by k_rope_kv (LVK_MM_ROPE=0)"""
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w5120_l2_q41.bin"), n_embd=5120, n_head=40, n_layer=2, ftype=3, seed=11)
    monkeypatch.setenv("LVK_MM_ROPE", rope)
    m = lvk.Llama(path, n_ctx=n_ctx)
    om = oracle.model(path, n_ctx)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 100)], np.int32)
    m.set_profiling(True)
    m.reset_profile()
    a = m.eval(toks, 0)
    # the MFMA path ran: activation image and matmul (+ the RoPE/KV kernel unless it is the
    # matmul's epilogue) in the QKV class per layer
    assert m.profile()["qkv"]["launches"] == (4 if rope == "1" else 6)
    m.set_profiling(False)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past, tok = len(toks), int(np.argmax(b[-1]))
    for _ in range(4):
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(b[-1]))
    m.close()
    om.close()


# ---------------------------------------------------------------------------
# LLaMA-65B layer shapes (n_embd 8192, 64 heads, n_ff 22016; llama.cpp:771-778):
# the decode kernels compiled for K = 8192 / 22016, the 64-head attention grid
# (256 workgroups exchanging score granules) and the MFMA prompt matmuls.
# ---------------------------------------------------------------------------
def _model_65b_l2(model_dir):
    from oracle_lib import gen_model
    return gen_model(os.path.join(model_dir, "w8192_l2.bin"), n_embd=8192, n_head=64, n_layer=2, ftype=2, seed=13)


def test_65b_shaped_decode_vs_oracle(lvk, oracle, model_dir):
    """65B layer shapes to n_past 300: the 64-head decode attention through its no-exchange path
    (n_kv <= 128) and the score exchange far past it, teacher-forced with non-repeating tokens
    (every KV row differs), every step bit-identical to the oracle"""
    from oracle_lib import forced_tokens
    path = _model_65b_l2(model_dir)
    m = lvk.Llama(path, n_ctx=512)
    m.set_prompt_exact(True)
    om = oracle.model(path, 512)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past = len(toks)
    seq = forced_tokens(301 - n_past, seed=65)
    bad = []
    for tok in seq:               # n_past 8..300
        a = m.eval([int(tok)], n_past)
        b = om.eval([int(tok)], n_past)
        if not np.array_equal(bits(a), bits(b)):
            bad.append(n_past)
        n_past += 1
    assert not bad, "n_past %s" % bad[:20]
    tok = int(np.argmax(a[-1]))
    m.set_profiling(True)
    m.reset_profile()
    m.eval([tok], n_past)
    pr = m.profile()
    assert pr["qkv"]["launches"] == 2 and pr["w2"]["launches"] == 2
    m.close()
    om.close()


def test_mfma_prompt_65b_shaped_vs_oracle(lvk, oracle, model_dir):
    """a 72-token prompt (ragged token tile) through the MFMA matmuls at K = 8192 / 22016, then decode"""
    path = _model_65b_l2(model_dir)
    m = lvk.Llama(path, n_ctx=256)
    om = oracle.model(path, 256)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 72)], np.int32)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a), bits(b))
    n_past, tok = len(toks), int(np.argmax(b[-1]))
    for _ in range(8):
        a = m.eval([tok], n_past)
        b = om.eval([tok], n_past)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(b[-1]))
    m.close()
    om.close()
