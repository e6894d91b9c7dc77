"""Dev tool (round 6): decode tok/s with and without the overlapped Wo launch (LVK_OVERLAP),
same process, alternating contexts; positions spread over 16..511 after the window is filled.
Every timed step's logits digest must be equal across the modes.
usage: overlap_ab.py [steps] [rounds] [model 7b|65b]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

CFG = {'7b': ('llama-7b-q4_0.bin', dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)),
       '65b': ('llama-65b-q4_0.bin', dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3))}


MODES = os.environ.get('OV_MODES', '0,1').split(',')


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 124
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    name = sys.argv[3] if len(sys.argv) > 3 else '7b'
    fn, cfg = CFG[name]
    path = os.path.join('/tmp/lvk_bench', fn)
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'), **cfg)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    res, dig = {}, {}
    for r in range(rounds):
        for mode in MODES:
            os.environ['LVK_OVERLAP'] = mode
            m = lvk.Llama(path, n_ctx=512)
            tok = int(np.argmax(m.eval(toks, 0)[-1]))
            for p in range(16, 512):
                tok = int(np.argmax(m.eval([tok], p, copy=False)[-1]))
            tok = int(np.argmax(m.eval(toks, 0)[-1]))
            t0 = time.perf_counter()
            for i in range(steps):
                tok = int(np.argmax(m.eval([tok], 16 + i * 496 // steps, copy=False)[-1]))
            dt = (time.perf_counter() - t0) / steps
            res.setdefault(mode, []).append(round(1 / dt, 1))
            # digests of a teacher-forced pass (every step, both modes)
            m.eval(toks, 0)
            d = [lvk.logits_digest(m.eval([int(t)], 16 + i)[-1]) for i, t in enumerate(range(1000, 1000 + 48))]
            dig.setdefault(mode, d)
            if d != dig[mode]:
                dig[mode + '_unstable'] = True
            m.close()
    print(json.dumps({'model': name, 'tok_s': res, 'digests_equal': all(dig[k] == dig[MODES[0]] for k in MODES),
                      'stable': not any(k.endswith('_unstable') for k in dig)}), flush=True)


if __name__ == '__main__':
    main()
