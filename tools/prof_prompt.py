"""Diagnostic: per-kernel-class device time of one 512-token prompt eval (7B Q4_0 synthetic)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk
path = '/tmp/lvk_bench/llama-7b-q4_0.bin'
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    lvk.gen_model(path, n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)
m = lvk.Llama(path, n_ctx=512)
toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 512)], np.int32)
for n in (512, 128, 32):
    m.eval(toks[:n], 0)
    t0 = time.perf_counter(); m.eval(toks[:n], 0); t1 = time.perf_counter()
    m.set_profiling(True); m.reset_profile(); m.eval(toks[:n], 0); p = m.profile(); m.set_profiling(False)
    print('N=%d wall %.2f ms' % (n, (t1 - t0) * 1e3))
    for k, v in p.items():
        if v['launches']:
            print('  %-8s %8.3f ms  %4d launches' % (k, v['ms'], v['launches']))
