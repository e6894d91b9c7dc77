"""Experiment: per-kernel decode times when the weights are Infinity-Cache (MALL) hot
(1- and 2-layer 7B-shaped models: 208 / 335 MB per token) against the 32-layer model
(4.1 GB per token, always cold).  Prints one JSON line per model."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

for nl in [int(a) for a in (sys.argv[1:] or ['1', '2', '32'])]:
    path = '/tmp/lvk_exp/l%d.bin' % nl
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'),
                      n_embd=4096, n_head=32, n_layer=nl, ftype=2, seed=1)
    m = lvk.Llama(path, n_ctx=512)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    lg = m.eval(toks, 0)
    tok = int(np.argmax(lg[-1]))
    for i in range(16):
        tok = int(np.argmax(m.eval([tok], 16 + i)[-1]))
    t0 = time.perf_counter()
    n = 128
    for i in range(n):
        tok = int(np.argmax(m.eval([tok], 32 + i)[-1]))
    dt = (time.perf_counter() - t0) / n
    m.set_profiling(True)
    m.reset_profile()
    for i in range(32):
        tok = int(np.argmax(m.eval([tok], 200 + i)[-1]))
    p = m.profile()
    m.set_profiling(False)
    m.close()
    print(json.dumps({'layers': nl, 'ms_per_token': dt * 1e3,
                      'kernels_us': {k: round(v['ms'] / v['launches'] * 1e3, 2) for k, v in p.items() if v['launches']}}),
          flush=True)
