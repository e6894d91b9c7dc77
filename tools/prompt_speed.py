"""Dev tool: 7B 512-token prompt eval time (best of 3) and per-kernel-class milliseconds, plus
a hash of the last logits row (equal hashes across LVK_PROMPT_A16=0/1 = identical bits).
usage: prompt_speed.py [n_tokens] [7b|13b|65b]  (the bench's seeded files)"""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
which = sys.argv[2] if len(sys.argv) > 2 else '7b'
fname, cfg = {'7b': ('llama-7b-q4_0.bin', dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)),
              '13b': ('llama-13b-q4_1.bin', dict(n_embd=5120, n_head=40, n_layer=40, ftype=3, seed=2)),
              '65b': ('llama-65b-q4_0.bin', dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3))}[which]
path = '/tmp/lvk_bench/' + fname
if not os.path.exists(path):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'), **cfg)
t0 = time.perf_counter()
m = lvk.Llama(path, n_ctx=512)
load_s = time.perf_counter() - t0
image = m.prompt_image_bytes()
toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, n)], np.int32)
best = 1e30
for _ in range(3):
    t0 = time.perf_counter()
    lg = m.eval(toks, 0)
    best = min(best, time.perf_counter() - t0)
h = hashlib.sha1(np.ascontiguousarray(lg[-1]).tobytes()).hexdigest()[:16]
m.set_profiling(True)
m.reset_profile()
m.eval(toks, 0)
p = m.profile()
m.set_profiling(False)
m.close()
print(json.dumps({'model': which, 'a16': os.environ.get('LVK_PROMPT_A16', '1'), 'n': n, 'ms': round(best * 1e3, 2),
                  'tok_s': round(n / best, 1), 'logits_sha1': h, 'a16_image_bytes': image, 'load_s': round(load_s, 2),
                  'kernels_ms': {k: round(v['ms'], 3) for k, v in p.items() if v['launches']}}), flush=True)
