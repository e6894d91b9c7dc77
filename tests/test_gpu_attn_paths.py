"""Both decode attention schedules on LLaMA-7B head shapes, bit-exact against each other.

k_attn_d (attention_decode.hip) runs 4 workgroups per head.  Up to n_kv = short_max (128
by default) each workgroup scores every position itself; past it the workgroups split the
positions and exchange score granules.  The in-process parity tests see the exchange only
past position 128, so this test pins both schedules over positions 9..200 in child
processes (short_max is read once per process): LVK_ATTN_SHORT=0 (exchange at every step)
and LVK_ATTN_NOEXCH=1 (never), and checks them against the oracle at the end points.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, %(pkg)r)
import lvk
m = lvk.Llama(%(model)r, n_ctx=256)
m.set_prompt_exact(True)
toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32)
a = m.eval(toks, 0)
n_past, tok, out, seq = len(toks), int(np.argmax(a[-1])), [], []
for _ in range(%(steps)d):
    a = m.eval([tok], n_past)
    out.append(a[-1].copy()); seq.append(tok)
    n_past += 1
    tok = int(np.argmax(a[-1]))
np.savez(%(out)r, logits=np.stack(out), seq=np.array(seq, np.int32))
m.close()
"""


def _run(model, out, env_extra, steps):
    code = CHILD % {"pkg": os.path.join(ROOT, "llama.vk_amd"), "model": model, "out": out, "steps": steps}
    env = {k: v for k, v in os.environ.items() if k not in ("LVK_ATTN_SHORT", "LVK_ATTN_NOEXCH")}
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    return np.load(out)


def test_attention_exchange_and_short_paths_agree(oracle, model_dir, gpu_available, tmp_path):
    from oracle_lib import gen_model
    path = gen_model(os.path.join(model_dir, "w4096_l2.bin"), n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
    steps = 192
    ex = _run(path, str(tmp_path / "exch.npz"), {"LVK_ATTN_SHORT": "0"}, steps)
    sh = _run(path, str(tmp_path / "short.npz"), {"LVK_ATTN_NOEXCH": "1"}, steps)
    assert np.array_equal(ex["seq"], sh["seq"])
    assert np.array_equal(ex["logits"].view(np.uint32), sh["logits"].view(np.uint32))
    # the oracle at the first and the last step of the same token sequence
    om = oracle.model(path, 256)
    toks = np.array([1, 450, 4996, 17354, 1701, 29916, 338, 263], np.int32)
    om.eval(toks, 0)
    n_past = len(toks)
    for i, t in enumerate(ex["seq"]):
        b = om.eval([int(t)], n_past)
        n_past += 1
        if i in (0, steps - 1):
            assert np.array_equal(ex["logits"][i].view(np.uint32), b[-1].view(np.uint32)), "step %d" % i
    om.close()
