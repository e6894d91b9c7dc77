"""Workload for PMC passes: the 7B synthetic file, two 512-token prompt evals (MFMA path).
usage: prompt_once.py [n_tokens] [7b|13b]  (13b: the bench's seeded 13B Q4_1 file, Q4_1 MFMA path)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
which = sys.argv[2] if len(sys.argv) > 2 else '7b'
fname, cfg = {'7b': ('llama-7b-q4_0.bin', dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)),
              '13b': ('llama-13b-q4_1.bin', dict(n_embd=5120, n_head=40, n_layer=40, ftype=3, seed=2))}[which]
path = '/tmp/lvk_bench/' + fname
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'), **cfg)
m = lvk.Llama(path, n_ctx=512)
toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, n)], np.int32)
for _ in range(2):
    m.eval(toks, 0)
m.close()
print('prompt_once done', flush=True)
