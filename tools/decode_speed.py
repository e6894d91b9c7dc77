"""Dev tool: single-stream greedy decode speed and per-kernel microseconds of one
synthetic model (the bench's seeded files).  usage: decode_speed.py 7b|13b|65b [steps]
Prints one JSON line; LVK_LIB selects a library build (e.g. lib/sweep with LVK_CFG41)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

CFG = {'7b': ('llama-7b-q4_0.bin', dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)),
       '13b': ('llama-13b-q4_1.bin', dict(n_embd=5120, n_head=40, n_layer=40, ftype=3, seed=2)),
       '65b': ('llama-65b-q4_0.bin', dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3))}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else '13b'
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    fn, cfg = CFG[name]
    path = os.path.join('/tmp/lvk_bench', fn)
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'), **cfg)
    m = lvk.Llama(path, n_ctx=512)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    tok = int(np.argmax(m.eval(toks, 0)[-1]))
    for i in range(8):
        tok = int(np.argmax(m.eval([tok], 16 + i)[-1]))
    t0 = time.perf_counter()
    for i in range(steps):
        tok = int(np.argmax(m.eval([tok], 24 + i)[-1]))
    dt = (time.perf_counter() - t0) / steps
    m.set_profiling(True)
    m.reset_profile()
    for i in range(16):
        tok = int(np.argmax(m.eval([tok], 24 + steps + i)[-1]))
    p = m.profile()
    m.set_profiling(False)
    m.close()
    ks = {k: round(v['ms'] / v['launches'] * 1e3, 2) for k, v in p.items() if v['launches']}
    gbs = {k: round(v['bytes'] / (v['ms'] * 1e-3) / 1e9, 0) for k, v in p.items() if v['launches'] and v.get('bytes')}
    print(json.dumps({'model': name, 'lib': os.environ.get('LVK_LIB', 'default'), 'cfg41': os.environ.get('LVK_CFG41'),
                      'tok_s': round(1 / dt, 1), 'ms_per_token': round(dt * 1e3, 3), 'kernels_us': ks, 'gbs': gbs}),
          flush=True)


if __name__ == '__main__':
    main()
