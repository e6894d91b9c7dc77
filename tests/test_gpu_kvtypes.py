"""llama_context_params the reference accepts beyond the default f16 cache: the f32 KV cache
(f16_kv = false, llama.cpp:1614; the attention dots become ggml_vec_dot_f32, ggml.c:1713-1748)
and any positive n_ctx, each bit-compared with the reference build (oracle/_ref/libref.so)
over a prompt and decode steps."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def _run_pair(lvk, ref, path, n_ctx, f16_kv, chunks, steps, exact_prompt=False):
    m = lvk.Llama(path, n_ctx=n_ctx, f16_kv=f16_kv)
    if exact_prompt:
        m.set_prompt_exact(True)
    r = ref.model(path, n_ctx, f16_kv=f16_kv)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    toks = [1] + [100 + (i * 7919) % 31000 for i in range(1, sum(chunks))]
    n_past, off = 0, 0
    for n in chunks:
        a = m.eval(np.array(toks[off:off + n], np.int32), n_past)
        b = r.eval(np.array(toks[off:off + n], np.int32), n_past, n_threads=threads)
        assert np.array_equal(bits(a[-1]), bits(b[-1])), "prompt chunk at n_past %d" % n_past
        n_past += n
        off += n
    tok = int(np.argmax(b[-1]))
    for _ in range(steps):
        a = m.eval([tok], n_past)
        b = r.eval([tok], n_past, n_threads=threads)
        assert np.array_equal(bits(a), bits(b)), "n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(b[-1]))
    m.close()
    r.close()


@pytest.mark.parametrize("name", ["tiny_q4_0", "tiny_q4_1"])
def test_f32_kv_cache_matches_reference_build(lvk, ref, tiny_models, name):
    """f16_kv = false: prompt chunks 16, 8, 24 (the reference's chunking) then 40 decode steps
    (crossing the 32-position SIMD boundary of the f32 P.V dot), bit-identical"""
    _run_pair(lvk, ref, tiny_models[name], 256, False, [16, 8, 24], 40)


def test_f32_kv_cache_7b_full(lvk, ref):
    """f32 KV on the full-size synthetic LLaMA-7B (the reference build cannot load 2-layer
    4096-wide files: llama.cpp picks its buffer sizes by layer count): a 40-token MFMA prompt,
    then decode"""
    from test_gpu_7b_full import CFG, MODEL
    from oracle_lib import gen_model
    if not os.path.exists(MODEL):
        os.makedirs(os.path.dirname(MODEL), exist_ok=True)
        tmp = MODEL + ".tmp%d" % os.getpid()
        gen_model(tmp, **CFG)
        os.replace(tmp, MODEL)
    _run_pair(lvk, ref, MODEL, 512, False, [40], 6)


def test_f32_kv_cache_state_round_trip(lvk, tiny_models):
    """llama_get_kv_cache / llama_set_kv_cache carry the f32 cache (twice the f16 bytes)"""
    path = tiny_models["tiny_q4_0"]
    a = lvk.Llama(path, n_ctx=128, f16_kv=False)
    b = lvk.Llama(path, n_ctx=128, f16_kv=True)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916], np.int32)
    a.eval(toks, 0)
    kv = a.kv_cache()
    assert len(kv) == 2 * len(b.kv_cache())
    c = lvk.Llama(path, n_ctx=128, f16_kv=False)
    c.set_kv_cache(kv, len(toks))
    x = a.eval([338], len(toks))
    y = c.eval([338], len(toks))
    assert np.array_equal(bits(x), bits(y))
    for m in (a, b, c):
        m.close()


@pytest.mark.parametrize("n_ctx,f16_kv", [(48, True), (100, True), (200, False), (33, True)])
def test_any_n_ctx_matches_reference_build(lvk, ref, tiny_models, n_ctx, f16_kv):
    """n_ctx not a multiple of 32 / below 64 (the reference accepts any): the window is
    honoured exactly (an eval past it fails) and the logits match the reference build"""
    path = tiny_models["tiny_q4_0"]
    chunks = [min(16, n_ctx - 8)]
    _run_pair(lvk, ref, path, n_ctx, f16_kv, chunks, n_ctx - chunks[0] - 1)
    m = lvk.Llama(path, n_ctx=n_ctx, f16_kv=f16_kv)
    with pytest.raises(RuntimeError):
        m.eval(np.array([1, 2], np.int32), n_ctx - 1)
    m.close()
