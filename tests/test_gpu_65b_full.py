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

  * (round 6) the 512-token prompt bench.py's decode_65b_q4_0.prompt_eval times (one batch,
    n_ctx 512: the MFMA prompt path at K 8192 / 22016 on the full model, the prompt attention
    at n_kv 512), and BASELINE configs[4]'s partition rehearsed on one GPU: the full 80-layer
    model as an 8-stage layer split (10 layers per stage, device-copy hand-offs, 64-token
    prompt micro-batches) through the same 512-token prompt and then 288 teacher-forced decode
    steps at n_past 512..799 (n_ctx 1024), every step against the reference build.

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


PROMPT512_DECODE = 288          # teacher-forced steps after the 512-token prompt: n_past 512..799


@pytest.fixture(scope="module")
def ref65_prompt512(model65b, ref):
    """the reference build on the 65B file: the 512-token prompt in one batch (llama.cpp:1010-1061
    at N 512, ggml.c:6625-6683 / 7062-7130), then PROMPT512_DECODE teacher-forced decode steps;
    the prompt's last logits row and every step's logits row.  n_ctx 1024: the logits do not
    depend on n_ctx (every column runs over n_kv = n_past + N)"""
    from oracle_lib import forced_tokens, prompt_tokens
    rm = ref.model(model65b, 1024)
    toks = prompt_tokens(512)
    last = rm.eval(toks, 0, n_threads=_threads())[-1].copy()
    seq = forced_tokens(PROMPT512_DECODE)
    rows = np.stack([rm.eval([int(t)], 512 + i, n_threads=_threads())[-1] for i, t in enumerate(seq)])
    rm.close()
    return toks, last, seq, rows


def test_65b_full_prompt512_vs_reference(model65b, ref65_prompt512):
    """the unsplit full 65B, n_ctx 512 (bench.py's decode_65b_q4_0.prompt_eval): one 512-token
    batch, last logits row bit-identical to the reference build"""
    import lvk
    toks, last, _, _ = ref65_prompt512
    m = lvk.Llama(model65b, n_ctx=512)
    try:
        a = m.eval(toks, 0)
        assert np.array_equal(bits(a[-1]), bits(last)), "512-token prompt logits differ"
    finally:
        m.close()


def test_65b_split8_prompt512_decode_to_799_vs_reference(model65b, ref65_prompt512):
    """BASELINE configs[4]'s partition on one GPU: 8 stages x 10 layers (lvk_split.cpp; stages on
    one device hand x over by stream-ordered device copies, the rest is the multi-GPU path), the
    512-token prompt in 64-token micro-batches flowing through the stages, then 288
    teacher-forced decode steps (n_past 512..799): the prompt's last row and every step's logits
    bit-identical to the reference build"""
    import lvk
    toks, last, seq, rows = ref65_prompt512
    m = lvk.Llama(model65b, n_ctx=1024, split=[0] * 8, micro=64)
    try:
        assert m.split_info() == (8, False, 64)
        a = m.eval(toks, 0)
        assert np.array_equal(bits(a[-1]), bits(last)), "split prompt logits differ"
        bad = []
        for i, t in enumerate(seq):
            a = m.eval([int(t)], 512 + i)
            if not np.array_equal(bits(a[-1]), bits(rows[i])):
                bad.append(512 + i)
        assert not bad, "split decode logits differ at n_past %s" % bad[:20]
    finally:
        m.close()
