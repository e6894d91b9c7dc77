"""Diagnostic: lvk_eval_greedy on a tiny model, graph on or off (argv[1] = 0/1)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "llama.vk_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lvk  # noqa: E402
from oracle_lib import gen_model  # noqa: E402

big = len(sys.argv) > 2 and sys.argv[2] == "big"
if len(sys.argv) > 2 and sys.argv[2] == "7b":
    path = gen_model("/tmp/diag_7b.bin", n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)
elif big:
    path = gen_model("/tmp/diag_w4096.bin", n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=7)
else:
    path = gen_model("/tmp/diag_tiny.bin", n_embd=256, n_head=2, n_layer=4, ftype=2, seed=1)
m = lvk.Llama(path, n_ctx=128)
m.set_graph(int(sys.argv[1]))
lg = m.eval(np.array([1, 450, 4996], np.int32), 0)
tok = int(np.argmax(lg[-1]))
print("eval ok", tok, flush=True)
for i in range(int(os.environ.get("DIAG_STEPS", "4"))):   # the logits graph first, as in bench.py
    tok = int(np.argmax(m.eval([tok], 3 + i % 100)[-1]))
print("decode ok", tok, flush=True)
m.eval(np.array([1, 450, 4996], np.int32), 0)
for i in range(5):
    tok = m.eval_greedy(tok, 3 + i)
    print("greedy", i, tok, flush=True)
m.close()
print("done", flush=True)
