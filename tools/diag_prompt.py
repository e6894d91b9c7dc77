"""Diagnostic: GPU vs oracle logits for prompt lengths / n_ctx variants."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk
from oracle_lib import Oracle, gen_model
path = gen_model('/tmp/diag_tiny.bin', n_embd=256, n_head=2, n_layer=32, ftype=2, seed=1)
orc = Oracle()
for nctx in (512, 256):
    m = lvk.Llama(path, n_ctx=nctx)
    om = orc.model(path, nctx)
    for n in (1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 16, 17):
        toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, n)], np.int32)
        a = m.eval(toks, 0); b = om.eval(toks, 0)
        d = np.abs(a - b).max()
        print('nctx', nctx, 'n', n, 'equal', np.array_equal(a, b), 'maxdiff', d, flush=True)
    m.close(); om.close()
