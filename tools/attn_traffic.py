"""Workload for PMC passes over the decode attention: the 7B synthetic file, a 16-token prompt,
then decode steps all at position P (argv[1], default 255): every k_attn_d launch reads the
K and V rows of n_kv = P + 1 positions, 2 * n_kv * n_embd * 2 bytes per layer."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

P = int(sys.argv[1]) if len(sys.argv) > 1 else 255
path = '/tmp/lvk_bench/llama-7b-q4_0.bin'
m = lvk.Llama(path, n_ctx=512)
m.set_graph(False)
toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
tok = int(np.argmax(m.eval(toks, 0)[-1]))
for _ in range(8):
    tok = int(np.argmax(m.eval([tok], P)[-1]))
m.close()
print('attn_traffic done P=%d' % P, flush=True)
