"""Full-size LLaMA-13B Q4_1 parity (BASELINE.json configs[3], the second quant format): the
real 40 x 5120 synthetic 13B Q4_1 model -- the same seeded file bench.py measures -- through
the GPU library, compared with the REFERENCE build (oracle/_ref/libref.so, the AVX2 ggml.c
path compiled from the reference sources) on the same tokens and the same batch chunking:

  * a 16-token prompt batch (the Q4_1 MFMA prompt path, mm_mfma41.hip) then 4 greedy decode
    steps (the CU-balanced Q4_1 decode kernels, matvec_cu41.hip);
  * one 512-token prompt batch.

The bar is bit-identical logits, as for the full 7B (tests/test_gpu_7b_full.py).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MODEL = "/tmp/lvk_bench/llama-13b-q4_1.bin"    # bench.py's file (same generator, seed and shape)
CFG = dict(n_embd=5120, n_head=40, n_layer=40, ftype=3, seed=2)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def model13b(gpu_available):
    from oracle_lib import gen_model
    os.makedirs(os.path.dirname(MODEL), exist_ok=True)
    if not os.path.exists(MODEL):
        tmp = MODEL + ".tmp%d" % os.getpid()
        gen_model(tmp, **CFG)
        os.replace(tmp, MODEL)
    return MODEL


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def test_13b_q4_1_full_prompt16_decode_vs_reference(model13b, ref):
    import lvk
    from oracle_lib import prompt_tokens
    m = lvk.Llama(model13b, n_ctx=512)
    rm = ref.model(model13b, 512)
    toks = prompt_tokens(16)
    a = m.eval(toks, 0)
    b = rm.eval(toks, 0, n_threads=_threads())
    assert np.array_equal(bits(a[-1]), bits(b[-1])), "16-token prompt logits differ"
    n_past, tok = 16, int(np.argmax(b[-1]))
    for _ in range(4):
        a = m.eval([tok], n_past)
        b = rm.eval([tok], n_past, n_threads=_threads())
        assert np.array_equal(bits(a[-1]), bits(b[-1])), "decode logits differ at n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(b[-1]))
    m.close()
    rm.close()


def test_13b_q4_1_full_prompt512_vs_reference(model13b, ref):
    import lvk
    from oracle_lib import prompt_tokens
    m = lvk.Llama(model13b, n_ctx=512)
    rm = ref.model(model13b, 512)
    toks = prompt_tokens(512)
    a = m.eval(toks, 0)
    b = rm.eval(toks, 0, n_threads=_threads())
    assert np.array_equal(bits(a[-1]), bits(b[-1])), "512-token prompt logits differ"
    m.close()
    rm.close()


def test_13b_q4_1_full_context_decode_to_511_vs_reference(model13b, ref):
    """BASELINE configs[3] over the whole window: 496 teacher-forced decode steps (n_past 16..511,
    the no-exchange attention path to n_kv 128 and the score exchange beyond, up to n_kv 512),
    every step's logits bit-identical to the reference build, the chained per-step digests equal
    to the reference's"""
    from test_gpu_7b_full import _full_context
    _full_context(model13b, ref, 511)


def test_13b_q4_1_long_context_2048_vs_reference(model13b, ref):
    """n_ctx 2048 with the second quant format: a 1536-token prompt in 512-token batches (the
    Q4_1 MFMA prompt path and the prompt attention at n_past 0 / 512 / 1024), then 256
    teacher-forced decode steps at n_past 1536..1791 (the 40-head decode attention at n_kv up
    to 1792); every batch's last row and every step's logits bit-identical to the reference"""
    import lvk
    from oracle_lib import forced_tokens, prompt_tokens
    m = lvk.Llama(model13b, n_ctx=2048)
    rm = ref.model(model13b, 2048)
    try:
        toks = prompt_tokens(1536)
        for c in range(3):
            part = toks[512 * c:512 * (c + 1)]
            a = m.eval(part, 512 * c)
            b = rm.eval(part, 512 * c, n_threads=_threads())
            assert np.array_equal(bits(a[-1]), bits(b[-1])), "prompt batch %d logits differ" % c
        seq = forced_tokens(256)
        bad = []
        for i, n_past in enumerate(range(1536, 1792)):
            a = m.eval([int(seq[i])], n_past)
            b = rm.eval([int(seq[i])], n_past, n_threads=_threads())
            if not np.array_equal(bits(a[-1]), bits(b[-1])):
                bad.append(n_past)
        assert not bad, "decode logits differ at n_past %s" % bad[:20]
    finally:
        m.close()
        rm.close()


def test_prompt_image_bytes_follow_the_capacity_rule(model13b):
    """lvk_prompt_image_bytes: the Q4_1 f16 + side images (3 B per weight of the layer matrices
    and the lm_head) are built for 13B; LVK_PROMPT_A16=0 builds none"""
    import lvk
    E, F, L, V = 5120, 13824, 40, 32000
    m = lvk.Llama(model13b, n_ctx=64)
    got = m.prompt_image_bytes()
    m.close()
    assert got >= 3 * (L * (4 * E * E + 3 * E * F)), got
    os.environ["LVK_PROMPT_A16"] = "0"
    try:
        m = lvk.Llama(model13b, n_ctx=64)
        assert m.prompt_image_bytes() == 0
        m.close()
    finally:
        del os.environ["LVK_PROMPT_A16"]
