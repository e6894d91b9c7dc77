import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests')); sys.path.insert(0, os.path.join(ROOT, 'llama.vk_amd'))
import numpy as np
import lvk
from oracle_lib import Oracle
orc = Oracle()
E, H, C = 512, 4, 256
hd = 128
for (n_past, N, t, h) in [(60, 37, 3, 2), (10, 100, 23, 3)]:
    rng = np.random.default_rng(n_past * 131 + N)
    kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    q = rng.standard_normal(N * E).astype(np.float32)
    out, sc, gp16 = lvk.attention_scores(kc, vc, q, E, H, C, n_past, N)
    q16 = q.reshape(N, E)[t, h*hd:(h+1)*hd].astype(np.float16).view(np.uint16).copy()
    n_kv = n_past + N
    scale = np.float32(1.0) / np.sqrt(np.float32(128.0), dtype=np.float32)
    for p in range(n_kv):
        kr = kc.reshape(C, E)[p, h*hd:(h+1)*hd].copy()
        ref = np.float32(orc.lib.orc_vec_dot_f16(hd, kr, q16)) * scale
        if p > n_past + t: ref = -np.inf
        g = sc[t, h, p]
        if not (g == ref or (np.isinf(g) and np.isinf(ref))):
            print('score mismatch', (n_past, N, t, h), 'p', p, g, ref)
    print('checked scores', (n_past, N, t, h), flush=True)
    # softmax in numpy emulating the oracle
    s = sc[t, h, :n_kv].astype(np.float32).copy()
    mx = s.max()
    print('max', mx, 'argmax', s.argmax(), 'n finite', np.isfinite(s).sum())
    tab = orc.table_exp()
    e = np.zeros(n_kv, np.float32)
    for p in range(n_kv):
        if np.isfinite(s[p]):
            e[p] = np.float16(np.float32(s[p] - mx)).view(np.uint16)
            e[p] = np.uint16(tab[int(np.float16(np.float32(s[p] - mx)).view(np.uint16))]).view(np.float16).astype(np.float32)
    tot = float(np.sum(e.astype(np.float64)))
    scf = np.float32(1.0 / tot)
    P = (e * scf).astype(np.float32)
    P16 = P.astype(np.float16)
    den = np.where((np.abs(P16.astype(np.float32)) < 6.1035e-05) & (P16 != 0))[0]
    print('denormal P16 positions', den.tolist(), P16[den].astype(np.float32).tolist(), flush=True)
    dm = s - mx
    den2 = np.where(np.isfinite(dm) & (np.abs(dm) < 6.1035e-05) & (dm != 0))[0]
    print('denormal (s-max) positions', den2.tolist())
    g16 = gp16[t, h, :n_kv]
    r16 = P.astype(np.float16).view(np.uint16)
    diff = np.nonzero(g16 != r16)[0]
    print('P16 diffs at', diff.tolist()[:10], [(hex(g16[i]), hex(r16[i]), float(P[i]), float(e[i])) for i in diff[:5]], 'scf', scf, 'tot', tot, flush=True)
