"""Dev tool (round 6): how often the fused RMSNorm prologues leave the fast path of
rms_mean_wave (lvk_device.h) on the bench's workloads.  Runs the `make rmscount` build
(LVK_LIB=lib/rmscount/...), whose kernels count, per calling wave: calls, rows that needed the
exactness certificate (the tree mean within 4n double-ulps of a float midpoint), and rows that
fell back to the serial index-order re-sum.  usage: rms_fallback_count.py [7b|13b|65b ...]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("LVK_LIB", os.path.join(ROOT, "llama.vk_amd", "lib", "rmscount", "libllama_vk_amd.so"))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk

CFG = {'7b': ('llama-7b-q4_0.bin', dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1)),
       '13b': ('llama-13b-q4_1.bin', dict(n_embd=5120, n_head=40, n_layer=40, ftype=3, seed=2)),
       '65b': ('llama-65b-q4_0.bin', dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3))}
TUS = ("lvk_probe_rms_mv", "lvk_probe_rms_mv41", "lvk_probe_rms_mm", "lvk_probe_rms_misc")


def counters():
    out = {}
    for name in TUS:
        buf = (C.c_ulonglong * 3)()
        getattr(lvk.lib, name)(buf)
        out[name[len("lvk_probe_rms_"):]] = list(buf)
    return out


def diff(a, b):
    return {k: [y - x for x, y in zip(a[k], b[k])] for k in a}


def main():
    for name in sys.argv[1:] or ["7b"]:
        fn, cfg = CFG[name]
        path = os.path.join('/tmp/lvk_bench', fn)
        if not os.path.exists(path):
            os.makedirs(os.path.dirname(path), exist_ok=True)
            lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'), **cfg)
        m = lvk.Llama(path, n_ctx=512)
        c0 = counters()
        p512 = np.array([1] + [100 + (i * 7919) % 31000 for i in range(1, 512)], np.int32)
        m.eval(p512, 0)
        c1 = counters()
        toks = p512[:16]
        tok = int(np.argmax(m.eval(toks, 0)[-1]))
        c2 = counters()
        steps = 124
        for i in range(steps):
            tok = int(np.argmax(m.eval([tok], 16 + i * 496 // steps)[-1]))
        c3 = counters()
        m.close()
        print(json.dumps({"model": name, "prompt512": diff(c0, c1), "decode_%d_steps" % steps: diff(c2, c3),
                          "fields": ["calls (per calling wave)", "certificate tried", "index-order re-sum"]}),
              flush=True)


if __name__ == '__main__':
    main()
