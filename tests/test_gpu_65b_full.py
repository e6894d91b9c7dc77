"""Full-size LLaMA-65B Q4_0 parity (BASELINE.json configs[4] at one stage): the real 80 x 8192
synthetic 65B Q4_0 model (n_ff 22016, 64 heads; 40.6 GB) -- the same seeded file bench.py
measures -- on ONE GPU through the library, compared with the REFERENCE build
(oracle/_ref/libref.so, the AVX2 ggml.c
path compiled from the reference sources) on the same tokens and the same batch chunking:

  * a 16-token prompt batch (the Q4_0 MFMA prompt path at K = 8192 / 22016) then 3 greedy
    decode steps (the decode kernels compiled for the 65B row lengths, the 64-head attention);
  * 136 teacher-forced decode steps (n_past 16..151: the 64-head decode attention through its
    no-exchange path and, past n_kv 128, the score exchange), every step's logits bit-identical
    to the reference build and lvk_decode_chain's per-step digests equal to the reference's.

The bar is bit-identical logits, as for the full 7B (tests/test_gpu_7b_full.py).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
MODEL = "/tmp/lvk_bench/llama-65b-q4_0.bin"     # bench.py's file (same generator, seed and shape)
CFG = dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3)


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def model65b(gpu_available):
    from oracle_lib import gen_model
    os.makedirs(os.path.dirname(MODEL), exist_ok=True)
    if not os.path.exists(MODEL):
        tmp = MODEL + ".tmp%d" % os.getpid()
        gen_model(tmp, **CFG)
        os.replace(tmp, MODEL)
    return MODEL


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def test_65b_full_prompt16_decode_vs_reference(model65b, ref):
    import lvk
    from oracle_lib import prompt_tokens
    m = lvk.Llama(model65b, n_ctx=512)
    rm = ref.model(model65b, 512)
    toks = prompt_tokens(16)
    a = m.eval(toks, 0)
    b = rm.eval(toks, 0, n_threads=_threads())
    assert np.array_equal(bits(a[-1]), bits(b[-1])), "16-token prompt logits differ"
    n_past, tok = 16, int(np.argmax(b[-1]))
    for _ in range(3):
        a = m.eval([tok], n_past)
        b = rm.eval([tok], n_past, n_threads=_threads())
        assert np.array_equal(bits(a[-1]), bits(b[-1])), "decode logits differ at n_past %d" % n_past
        n_past += 1
        tok = int(np.argmax(b[-1]))
    m.close()
    rm.close()



def test_65b_full_context_decode_to_151_vs_reference(model65b, ref):
    from test_gpu_7b_full import _full_context
    _full_context(model65b, ref, 151, greedy_steps=4)
