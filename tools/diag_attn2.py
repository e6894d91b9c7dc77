import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk
from oracle_lib import Oracle
orc = Oracle()
E, H, C = 512, 4, 256
def run(n_past, N, fix):
    rng = np.random.default_rng(n_past * 131 + N)
    k = rng.standard_normal(C * E).astype(np.float16); v = rng.standard_normal(C * E).astype(np.float16)
    nden = int((np.abs(k[:(n_past+N)*E].astype(np.float32)) < 6.1035e-05).sum() - (k[:(n_past+N)*E] == 0).sum())
    if fix:
        for a in (k, v):
            a[(np.abs(a.astype(np.float32)) < 6.1035e-05)] = 0
    kc = k.view(np.uint16).copy(); vc = v.view(np.uint16).copy()
    q = rng.standard_normal(N * E).astype(np.float32)
    got = lvk.attention(kc, vc, q, E, H, C, n_past, N).reshape(N, H, 128)
    want = np.zeros(N * E, np.float32)
    orc.lib.orc_attention(kc, vc, q, E, H, C, n_past, N, want)
    want = want.reshape(N, H, 128)
    bad = np.argwhere(got != want)
    print((n_past, N), 'fix', fix, 'denormK', nden, 'mismatch', len(bad), sorted(set(map(tuple, bad[:, :2].tolist())))[:5], flush=True)
for case in [(60, 37), (10, 100)]:
    for fix in (False, True):
        run(*case, fix)
# f16 denormal conversion probe via the quantize path is not available; probe via attention with tiny values
