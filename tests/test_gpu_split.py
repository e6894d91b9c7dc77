"""The layer split behind llama.h (lvk_split.cpp), rehearsed on one GPU:
S stage contexts on the same device hand the residual stream over with stream-ordered
device copies (the transport a repeated device selects; distinct devices use grouped
RCCL send/recv, which needs one GPU per stage).  Everything else -- the stage layer
ranges, the interleaved enqueue with one host wait per eval, prompt micro-batches
flowing through the stages, logits_all rows across micro-batches, the greedy argmax on
the last stage, the KV-cache bytes -- is the multi-GPU code path, and every result must
equal the unsplit context's bits (which the other GPU tests pin to the oracle)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


PROMPT = [1, 450, 4996, 17354, 1701, 29916, 338, 263, 1243, 310, 278, 11761, 1788, 29889, 306, 626,
          2599, 304, 1207, 263, 1243, 29892, 322, 306]


def run(m, prompt, steps, greedy=False):
    """prompt, then `steps` greedy decode steps; returns the logits rows and tokens"""
    out = [m.eval(prompt, 0)]
    n_past, tok, toks = len(prompt), int(np.argmax(out[-1][-1])), []
    for _ in range(steps):
        toks.append(tok)
        if greedy:
            tok = m.eval_greedy(tok, n_past)
        else:
            out.append(m.eval([tok], n_past))
            tok = int(np.argmax(out[-1][-1]))
        n_past += 1
    toks.append(tok)
    return out, toks


@pytest.mark.parametrize("stages,micro", [(2, 0), (2, 8), (3, 5), (4, 16)])
def test_split_matches_single_context(lvk, tiny_models, stages, micro):
    path = tiny_models["tiny_q4_0"]
    ref = lvk.Llama(path, n_ctx=128)
    want, wt = run(ref, PROMPT, 8)
    ref.close()
    m = lvk.Llama(path, n_ctx=128, split=[0] * stages, micro=micro)
    assert m.split_info() == (stages, False, micro)
    got, gt = run(m, PROMPT, 8)
    assert gt == wt
    for k, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(bits(a), bits(b)), "eval %d" % k
    m.close()


def test_split_logits_all_across_micro_batches(lvk, tiny_models):
    """logits_all: every prompt row comes back, each written by its micro-batch's lm_head"""
    path = tiny_models["tiny_q4_0"]
    ref = lvk.Llama(path, n_ctx=128, logits_all=True)
    want = ref.eval(PROMPT, 0)
    want2 = ref.eval(PROMPT[:7], len(PROMPT))
    ref.close()
    m = lvk.Llama(path, n_ctx=128, logits_all=True, split=[0, 0, 0], micro=6)
    got = m.eval(PROMPT, 0)
    got2 = m.eval(PROMPT[:7], len(PROMPT))
    assert got.shape == (len(PROMPT), m.n_vocab)
    assert np.array_equal(bits(got), bits(want))
    assert np.array_equal(bits(got2), bits(want2))
    m.close()


def test_split_greedy_on_device(lvk, tiny_models):
    path = tiny_models["tiny_q4_0"]
    ref = lvk.Llama(path, n_ctx=128)
    _, wt = run(ref, PROMPT, 12)
    ref.close()
    m = lvk.Llama(path, n_ctx=128, split=[0, 0])
    _, gt = run(m, PROMPT, 12, greedy=True)
    assert gt == wt
    m.close()


def test_split_kv_cache_bytes_match(lvk, tiny_models):
    """llama_get_kv_cache of a split = the unsplit K | V bytes (stage halves concatenated);
    llama_set_kv_cache into a fresh split resumes identically"""
    path = tiny_models["tiny_q4_0"]
    ref = lvk.Llama(path, n_ctx=128)
    ref.eval(PROMPT, 0)
    kv_ref = ref.kv_cache()
    nxt = ref.eval([PROMPT[3]], len(PROMPT))
    ref.close()
    m = lvk.Llama(path, n_ctx=128, split=[0, 0, 0])
    m.eval(PROMPT, 0)
    kv = m.kv_cache()
    assert kv.size == kv_ref.size and np.array_equal(kv, kv_ref)
    m.close()
    m2 = lvk.Llama(path, n_ctx=128, split=[0, 0])
    m2.set_kv_cache(kv, len(PROMPT))
    assert m2.kv_cache_token_count() == len(PROMPT)
    assert np.array_equal(bits(m2.eval([PROMPT[3]], len(PROMPT))), bits(nxt))
    m2.close()


def test_split_from_environment(lvk, tiny_models):
    """llama_init_from_file reads LVK_SPLIT_DEVICES / LVK_SPLIT_MICRO (what an unmodified
    examples/main gets)"""
    path = tiny_models["tiny_q4_0"]
    ref = lvk.Llama(path, n_ctx=128)
    want, _ = run(ref, PROMPT, 4)
    ref.close()
    os.environ["LVK_SPLIT_DEVICES"] = "0,0"
    os.environ["LVK_SPLIT_MICRO"] = "10"
    try:
        m = lvk.Llama(path, n_ctx=128)
    finally:
        del os.environ["LVK_SPLIT_DEVICES"]
        del os.environ["LVK_SPLIT_MICRO"]
    assert m.split_info() == (2, False, 10)
    got, _ = run(m, PROMPT, 4)
    for a, b in zip(got, want):
        assert np.array_equal(bits(a), bits(b))
    m.close()


def test_split_rejects_rccl_on_one_device(lvk, tiny_models):
    with pytest.raises(RuntimeError):
        lvk.Llama(tiny_models["tiny_q4_0"], n_ctx=128, split=[0, 0], transport="rccl")


@pytest.mark.parametrize("cfg,stages,micro", [
    (dict(n_embd=8192, n_head=64, n_layer=2, ftype=2, seed=3), 2, 16),
    (dict(n_embd=4096, n_head=32, n_layer=4, ftype=2, seed=1), 4, 16),
], ids=["65b_shaped_s2", "7b_shaped_s4"])
def test_split_shapes_vs_oracle(lvk, oracle, model_dir, cfg, stages, micro):
    """65B-shaped layers (n_embd 8192, 64 heads, n_ff 22016) through a 2-stage split and
    7B-shaped ones through 4 stages, with 16-token prompt micro-batches (a 16-token slice on
    the MFMA prompt path, then a 4-token one on the VALU kernels), against the oracle"""
    from oracle_lib import gen_model, prompt_tokens
    path = gen_model(os.path.join(model_dir, "s_w%d_l%d.bin" % (cfg["n_embd"], cfg["n_layer"])), **cfg)
    toks = prompt_tokens(20)
    m = lvk.Llama(path, n_ctx=128, split=[0] * stages, micro=micro)
    om = oracle.model(path, 128)
    a = m.eval(toks, 0)
    b = om.eval(toks, 0)
    assert np.array_equal(bits(a[-1]), bits(b[-1]))
    tok = int(np.argmax(a[-1]))
    for i in range(3):
        a = m.eval([tok], 20 + i)
        b = om.eval([tok], 20 + i)
        assert np.array_equal(bits(a), bits(b)), "decode step %d" % i
        tok = int(np.argmax(a[-1]))
    m.close()
    om.close()


STAGE_CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, %(pkg)r)
import lvk
PROMPT = %(prompt)r
path = %(model)r
def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)
ref = lvk.Llama(path, n_ctx=128)
want = ref.eval(PROMPT, 0)
tok, wt = int(np.argmax(want[-1])), []
for i in range(10):
    wt.append(tok)
    tok = int(np.argmax(ref.eval([tok], len(PROMPT) + i)[-1]))
wt.append(tok)
ref.close()
st = lvk.Llama(path, n_ctx=128, layers=(0, lvk.model_hparams(path)["n_layer"]))
st.stage_connect(lvk.rccl_unique_id(), 1, 0)
assert st.stage_step(PROMPT, len(PROMPT), 0, micro=7) == 0
assert np.array_equal(bits(st.logits()[-1]), bits(want[-1]))
tok, got = wt[0], [wt[0]]
for i in range(10):
    tok = st.stage_step([tok], 1, len(PROMPT) + i, greedy=True)
    got.append(tok)
assert got == wt, (got, wt)
st.close()
print("STAGE-LINK-OK", flush=True)
"""


def test_stage_link_single_rank(lvk, tiny_models):
    """the one-stage-per-process link (lvk_rccl_unique_id / lvk_stage_connect /
    lvk_stage_step, what bench.py's layer-split ranks run) with one rank: RCCL loads, the
    communicator forms, and prompt micro-batches + greedy steps equal the plain context.
    Runs in its own process, as each bench rank does: RCCL's state then lives and is torn
    down with that process only, and the child must also exit cleanly (rc 0)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = STAGE_CHILD % {"pkg": os.path.join(root, "llama.vk_amd"), "prompt": PROMPT,
                          "model": tiny_models["tiny_q4_0"]}
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180)
    assert "STAGE-LINK-OK" in r.stdout, r.stdout + r.stderr[-3000:]
    assert r.returncode == 0, "stage-link child exited with %d: %s" % (r.returncode, r.stderr[-3000:])
