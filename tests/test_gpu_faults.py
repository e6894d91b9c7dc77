"""Failure paths of the device-side waits (no silent wrong answers).

The decode attention's workgroups wait on each other's score granules with a
bounded spin (with LVK_ATTN_SHORT=0 at every n_kv; by default only past 128).  The probe build (make -C llama.vk_amd probe) never publishes
position 0's score and gives up after 4096 polls: the timeout must reach the
host as a failed llama_eval (rc 1) / lvk_eval_greedy (-1) and invalid logits,
and the context must stay usable.  Runs in a child process, because lvk.py
binds one library per process.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "llama.vk_amd", "lib", "probe", "libllama_vk_amd.so")

CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, %(pkg)r)
import lvk
assert lvk.LIB_PATH.endswith("probe/libllama_vk_amd.so"), lvk.LIB_PATH
m = lvk.Llama(%(model)r, n_ctx=256)
m.set_prompt_exact(True)
m.eval(np.array([1, 450, 4996], np.int32), 0)          # prompt batch: no decode attention involved
try:
    m.eval([500], 3)
    print("RESULT eval-succeeded")
except RuntimeError:
    print("RESULT eval-failed")
print("SAMPLE", m.sample(np.array([1], np.int32)))       # logits invalid after the failure: -1
try:
    m.eval_greedy(500, 3)
    print("RESULT greedy-succeeded")
except RuntimeError:
    print("RESULT greedy-failed")
m.eval(np.array([1, 450, 4996, 17354], np.int32), 0)   # the context is still usable
print("RESULT recovered")
m.close()
"""


def test_attention_wait_timeout_fails_the_eval(tiny_models, gpu_available):
    if not os.path.exists(PROBE):
        pytest.fail("probe library not built (make -C llama.vk_amd probe)")
    env = dict(os.environ, LVK_LIB=PROBE, LVK_ATTN_SHORT="0")   # every decode step exchanges scores
    code = CHILD % {"pkg": os.path.join(ROOT, "llama.vk_amd"), "model": tiny_models["tiny_q4_0"]}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    out = r.stdout
    assert r.returncode == 0, r.stdout + r.stderr
    assert "RESULT eval-failed" in out, out + r.stderr
    assert "SAMPLE -1" in out, out
    assert "RESULT greedy-failed" in out, out
    assert "RESULT recovered" in out, out
    assert "wait timed out" in r.stderr, r.stderr
