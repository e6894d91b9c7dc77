"""Dev tool (round 6): a short 7B decode for a rocprofv3 kernel trace, overlap mode from the
environment (LVK_OVERLAP).  usage: ov_trace.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    path = '/tmp/lvk_bench/llama-7b-q4_0.bin'
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        lvk.gen_model(path, n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1,
                      vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'))
    m = lvk.Llama(path, n_ctx=512)
    toks = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 16)], np.int32)
    tok = int(np.argmax(m.eval(toks, 0)[-1]))
    for i in range(steps):
        tok = int(np.argmax(m.eval([tok], 16 + i * 15, copy=False)[-1]))
    m.close()


if __name__ == '__main__':
    main()
