"""Diagnostic: MFMA prompt path vs oracle, per layer count."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk
from oracle_lib import Oracle, gen_model
orc = Oracle()
for nl in (1, 2, 4, 32):
    path = gen_model('/tmp/diag_mfma_%d.bin' % nl, n_embd=256, n_head=2, n_layer=nl, ftype=2, seed=1)
    m = lvk.Llama(path, n_ctx=256, logits_all=True)
    om = orc.model(path, 256)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 100)], np.int32)
    a = m.eval(toks, 0); b = om.eval(toks, 0, logits_all=True)
    rel = np.abs(a - b).max(-1) / np.abs(b).max(-1)
    m.set_prompt_exact(True)
    c = m.eval(toks, 0)
    print('layers', nl, 'rel max %.3g median %.3g' % (rel.max(), np.median(rel)), 'argmax agree', (a.argmax(-1) == b.argmax(-1)).mean(),
          'exact path equal', np.array_equal(c, b), 'worst pos', int(rel.argmax()), flush=True)
    m.close(); om.close()
