"""Dev tool (round 6): single-token decode through the captured step graph vs eager launches
of the same kernels (lvk_set_graph).  Positions spread over 16..511 after the window is filled.
usage: eager_vs_graph.py [steps] [rounds]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 124
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    path = '/tmp/lvk_bench/llama-7b-q4_0.bin'
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1,
                      vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'))
    m = lvk.Llama(path, n_ctx=512)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    tok = int(np.argmax(m.eval(toks, 0)[-1]))
    for p in range(16, 512):
        tok = int(np.argmax(m.eval([tok], p, copy=False)[-1]))
    res = {}
    for r in range(rounds):
        for mode in (True, False):
            m.set_graph(mode)
            tok = int(np.argmax(m.eval(toks, 0)[-1]))
            t0 = time.perf_counter()
            for i in range(steps):
                tok = int(np.argmax(m.eval([tok], 16 + i * 496 // steps, copy=False)[-1]))
            dt = (time.perf_counter() - t0) / steps
            res.setdefault('graph' if mode else 'eager', []).append(round(1 / dt, 1))
    m.set_graph(True)
    m.close()
    print(json.dumps({'tok_s': res}), flush=True)


if __name__ == '__main__':
    main()
