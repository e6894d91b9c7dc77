"""Dev check: the persistent decode kernel against the launch-per-phase path (and the
CPU oracle on the small models), then decode tok/s on the 7B file.  Prints one line per
check; exits non-zero on the first mismatch."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
import numpy as np
import lvk
from oracle_lib import Oracle, gen_model, prompt_tokens


def run(path, n_ctx, steps, persistent, ptoks=8):
    m = lvk.Llama(path, n_ctx=n_ctx)
    m.set_decode_persistent(persistent)
    toks = prompt_tokens(ptoks)
    out = [m.eval(toks, 0)[-1].copy()]
    tok = int(np.argmax(out[-1]))
    act = None
    for i in range(steps):
        lg = m.eval([tok], ptoks + i)[-1].copy()
        if act is None:
            act = m.decode_persistent_active()
        out.append(lg)
        tok = int(np.argmax(lg))
    m.close()
    return np.array(out), act


def main():
    d = '/tmp/lvk_chk'
    os.makedirs(d, exist_ok=True)
    orc = Oracle()
    PT = int(os.environ.get('CHK_PROMPT', '8'))
    TL = int(os.environ.get('CHK_TINY_LAYERS', '4'))
    TC = int(os.environ.get('CHK_TINY_NCTX', '128'))
    cases = [('tiny%d' % TL, dict(n_embd=256, n_head=2, n_layer=TL, ftype=2, seed=1), TC, 12),
             ('w4096_l2', dict(n_embd=4096, n_head=32, n_layer=2, ftype=2, seed=1), 512, 6)]
    if len(sys.argv) > 1 and sys.argv[1] == 'nospeed':
        pass
    if len(sys.argv) > 1 and sys.argv[1] == 'big':
        cases.append(('w8192_l1', dict(n_embd=8192, n_head=64, n_layer=1, ftype=2, seed=3), 512, 4))
    for name, cfg, n_ctx, steps in cases:
        path = gen_model(os.path.join(d, name + '.bin'), **cfg)
        a, act = run(path, n_ctx, steps, True, PT)
        b, _ = run(path, n_ctx, steps, False, PT)
        om = orc.model(path, n_ctx)
        toks = prompt_tokens(PT)
        ref = [om.eval(toks, 0)[-1]]
        tok = int(np.argmax(ref[-1]))
        for i in range(steps):
            ref.append(om.eval([tok], PT + i)[-1])
            tok = int(np.argmax(ref[-1]))
        om.close()
        ref = np.array(ref)
        same_l = np.array_equal(a.view(np.uint32), b.view(np.uint32))
        same_o = np.array_equal(a.view(np.uint32), ref.view(np.uint32))
        print('%-10s persistent_active=%s  equal_to_launches=%s  equal_to_oracle=%s  max|d|=%.3g' %
              (name, act, same_l, same_o, float(np.max(np.abs(a - ref)))), flush=True)
        if not (same_l and same_o):
            for k in range(len(a)):
                print('   step %d: max|p-o| %.3g  max|l-o| %.3g' % (k, np.max(np.abs(a[k] - ref[k])), np.max(np.abs(b[k] - ref[k]))))
            sys.exit(1)
    if len(sys.argv) > 1 and sys.argv[1] == 'nospeed':
        return
    if len(sys.argv) > 1 and sys.argv[1] == 'deep':
        # persistent vs launch path on deeper files (the launch path is oracle-exact)
        for name, cfg in [('w4096_l12', dict(n_embd=4096, n_head=32, n_layer=12, ftype=2, seed=1)),
                          ('w512_l12', dict(n_embd=512, n_head=4, n_layer=12, ftype=2, seed=1))]:
            path = gen_model(os.path.join(d, name + '.bin'), **cfg)
            a, _ = run(path, 512, 3, True, PT)
            b, _ = run(path, 512, 3, False, PT)
            print('%-10s equal_to_launches=%s max|d|=%.3g' % (name, np.array_equal(a.view(np.uint32), b.view(np.uint32)),
                                                             float(np.max(np.abs(a - b)))), flush=True)
        return
    # speed on the 7B file (and the 65B one with 'big')
    runs = [('7B', '/tmp/lvk_bench/llama-7b-q4_0.bin', dict(n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1))]
    if len(sys.argv) > 1 and sys.argv[1] == 'big':
        runs.append(('65B', '/tmp/lvk_bench/llama-65b-q4_0.bin', dict(n_embd=8192, n_head=64, n_layer=80, ftype=2, seed=3)))
    for name, path, cfg in runs:
        if not os.path.exists(path):
            os.makedirs(os.path.dirname(path), exist_ok=True)
            lvk.gen_model(path, vocab=os.path.join(ROOT, 'tests', 'golden', 'vocab32000.bin'), **cfg)
        timing(name, path)


def timing(name, path):
    for persistent in (True, False):
        m = lvk.Llama(path, n_ctx=512)
        m.set_decode_persistent(persistent)
        toks = prompt_tokens(16)
        tok = int(np.argmax(m.eval(toks, 0)[-1]))
        for i in range(8):
            tok = int(np.argmax(m.eval([tok], 16 + i)[-1]))
        n = 128 if name == '7B' else 24
        t0 = time.perf_counter()
        for i in range(n):
            tok = int(np.argmax(m.eval([tok], 16 + i)[-1]))
        dt = (time.perf_counter() - t0) / n
        m.set_profiling(True)
        m.reset_profile()
        for i in range(16):
            tok = int(np.argmax(m.eval([tok], 200 + i)[-1]))
        p = m.profile()
        m.set_profiling(False)
        m.close()
        ks = {k: round(v['ms'] / v['launches'] * 1e3, 2) for k, v in p.items() if v['launches']}
        print('%s persistent=%s: %.1f tok/s (%.3f ms/token)  kernels_us=%s' % (name, persistent, 1 / dt, dt * 1e3, ks), flush=True)


if __name__ == '__main__':
    main()
