"""Diagnostic (rocprofv3 --kernel-trace only): the bench's order on the 7B file -- 16-token
prompt, logits-graph decode steps, prompt again, then lvk_eval_greedy -- in one variant
named by argv[1] (argv 2-4: model path, n_ctx, logits-graph steps):
  graph   : the greedy decode graph (the crashing form under the profiler)
  eager   : greedy steps without graphs (lvk_set_graph 0)
  nograph0: the logits decode without graphs, then the greedy graph
Prints one line per phase so the log shows how far it got."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

variant = sys.argv[1] if len(sys.argv) > 1 else 'graph'
path = sys.argv[2] if len(sys.argv) > 2 else '/tmp/lvk_bench/llama-7b-q4_0.bin'
n_ctx = int(sys.argv[3]) if len(sys.argv) > 3 else 512
n_steps = int(sys.argv[4]) if len(sys.argv) > 4 else 8
m = lvk.Llama(path, n_ctx=n_ctx)
toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
tok = int(np.argmax(m.eval(toks, 0)[-1]))
if variant == 'nograph0':
    m.set_graph(False)
for i in range(n_steps):
    tok = int(np.argmax(m.eval([tok], 16 + i)[-1]))
print(variant, 'logits decode ok', flush=True)
m.set_graph(variant != 'eager')
m.eval(toks, 0)
tok = int(np.argmax(m.logits()[-1]))
for i in range(4):
    tok = m.eval_greedy(tok, 16 + i)
    print(variant, 'greedy step', i, tok, flush=True)
m.close()
print(variant, 'done', flush=True)
