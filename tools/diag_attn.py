import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk
from oracle_lib import Oracle
orc = Oracle()
E, H, C = 512, 4, 256
for (n_past, N) in [(0, 33), (0, 40), (0, 64), (0, 65), (1, 32), (1, 31), (60, 37), (10, 100), (32, 2), (31, 2), (62, 2), (63, 2), (64, 2)]:
    rng = np.random.default_rng(n_past * 131 + N)
    kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    q = rng.standard_normal(N * E).astype(np.float32)
    got = lvk.attention(kc, vc, q, E, H, C, n_past, N).reshape(N, H, 128)
    want = np.zeros(N * E, np.float32)
    orc.lib.orc_attention(kc, vc, q, E, H, C, n_past, N, want)
    want = want.reshape(N, H, 128)
    bad = np.argwhere(got != want)
    toks = sorted(set(bad[:, 0].tolist()))
    print((n_past, N), 'n_kv', n_past + N, 'mismatch elems', len(bad), 'tokens', toks[:20], 'maxrel', (np.abs(got - want) / (np.abs(want) + 1e-6)).max(), flush=True)
