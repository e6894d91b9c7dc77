"""Diagnostic: prompt-eval wall time per batch size N for the MFMA and the VALU
(bit-faithful chains on VALU) matmul paths, plus a per-kernel-class profile at N=512
(7B Q4_0 synthetic)."""
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
for n in (2, 4, 8, 16, 32, 64, 128, 512):
    row = []
    for exact in (False, True):
        m.set_prompt_exact(exact)
        m.eval(toks[:n], 0)
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter(); m.eval(toks[:n], 0); best = min(best, time.perf_counter() - t0)
        row.append(best * 1e3)
    print('N=%4d  mfma %8.2f ms (%7.0f tok/s)   valu %8.2f ms (%7.0f tok/s)' % (n, row[0], n / row[0] * 1e3, row[1], n / row[1] * 1e3), flush=True)
m.set_prompt_exact(False)
m.set_profiling(True); m.reset_profile(); m.eval(toks, 0); p = m.profile(); m.set_profiling(False)
print('N=512 profile (MFMA path):')
for k, v in p.items():
    if v['launches']:
        print('  %-8s %8.3f ms  %4d launches' % (k, v['ms'], v['launches']))
