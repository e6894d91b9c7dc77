"""The decode attention's granule tags are (seq << 7) + layer + 1 with seq the 25-bit step
counter of the step block (attention_decode.hip); before the counter
would pass 2^25 the context zeroes the granules on its stream and restarts it
(Context::next_seq).  Contexts whose counter starts just below the wrap (test hook
LVK_SEQ_START) must decode exactly like a fresh one -- the wrap falling inside a run of
per-step evals (lvk_eval_greedy) and at the start of a chained lvk_decode_greedy -- with the
exchange path of the attention active (n_kv > 128) when it happens."""
import os

import numpy as np
import pytest

from oracle_lib import gen_model, prompt_tokens

pytestmark = pytest.mark.gpu


def _run(path, seq_start):
    import lvk
    if seq_start is None:
        os.environ.pop("LVK_SEQ_START", None)
    else:
        os.environ["LVK_SEQ_START"] = str(seq_start)
    try:
        m = lvk.Llama(path, n_ctx=256)
    finally:
        os.environ.pop("LVK_SEQ_START", None)
    lg = m.eval(prompt_tokens(16), 0)
    tok, toks = int(np.argmax(lg[-1])), []
    for i in range(140):                       # n_past 16..155
        tok = m.eval_greedy(tok, 16 + i)
        toks.append(tok)
    part = m.decode_greedy(tok, 156, 60)      # n_past 156..215, chained
    toks += [int(t) for t in part]
    last = m.eval([int(part[-1])], 216)[-1].copy()
    m.close()
    return toks, last


def test_step_counter_wrap_is_invisible(model_dir, gpu_available):
    path = gen_model(os.path.join(model_dir, "w4096_l2_seq.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=11)
    want_t, want_l = _run(path, None)
    W = 1 << 25
    for start in (W - 130, W - 1 - 140 - 30):   # wrap at eval step ~129 (n_past ~145); at the chain's start
        got_t, got_l = _run(path, start)
        assert got_t == want_t, "tokens differ after the wrap (start %d) at step %d" % (
            start, next(i for i, (a, b) in enumerate(zip(got_t, want_t)) if a != b))
        assert np.array_equal(got_l.view(np.uint32), want_l.view(np.uint32))
