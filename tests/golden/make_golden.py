"""Generate the committed golden fixtures from the REFERENCE build.

Run in the build container (needs oracle/_ref/libref.so, built from
/root/reference by `make -C oracle ref`).  Fixtures are data only: seeded
inputs and the reference's outputs.  Regenerate with:

    python tests/golden/make_golden.py

Outputs (tests/golden/):
  ops_q4.npz         quantize_row_q4_{0,1} (AVX2), file quantizers, vec_dot_q4_{0,1},
                     rms_norm, rope, silu, attention block -- reference outputs
  tiny_q4_0.npz      logits of the seeded tiny Q4_0 model (lvk-gen-model
                     --n-embd 256 --n-head 2 --n-layer 32 --seed 1) for a chunked
                     16+8+24-token prompt then 6 greedy decode steps (main-style)
  tiny_q4_1.npz      same for the tiny 40-layer Q4_1 model (--ftype 3 --seed 7)
  tiny_l80_q4_0.npz  same for an 80-layer Q4_0 model (the reference's 65B layer count, --seed 3)
  test_quantize.json known answers of the reference's tests/test-quantize.c
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_lib import Ref, gen_model, prompt_tokens  # noqa: E402

TINY = {
    "tiny_q4_0": dict(n_embd=256, n_head=2, n_layer=32, ftype=2, seed=1),
    "tiny_q4_1": dict(n_embd=256, n_head=2, n_layer=40, ftype=3, seed=7),
    # 80 layers: the reference's MODEL_65B branch (llama.cpp:778) on a model small enough for a fixture
    "tiny_l80_q4_0": dict(n_embd=256, n_head=2, n_layer=80, ftype=2, seed=3),
}
CHUNKS = (16, 8, 24)
N_DECODE = 6


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


def ops(ref):
    rng = np.random.default_rng(1234)
    out = {}
    x = np.concatenate([rng.standard_normal((6, 4096)) * s for s in (1e-3, 1.0, 37.0)]).astype(np.float32)
    x[0, :64] = 0.0
    w = (rng.standard_normal((6, 4096)) * 0.02).astype(np.float32)
    out["x"] = x
    out["w"] = w
    for qt in (2, 3):
        out["q%d" % qt] = np.stack([ref.quantize(r, qt) for r in x])
        out["wq%d" % qt] = np.stack([ref.quantize(r, qt, reference=True) for r in w])
        out["dot%d" % qt] = np.array([[ref.vec_dot(qt, 4096, out["wq%d" % qt][i], out["q%d" % qt][j])
                                       for j in range(len(x))] for i in range(len(w))], np.float32)
        out["deq%d" % qt] = np.stack([ref.dequantize(r, qt, 4096) for r in out["wq%d" % qt]])
    xs = (rng.standard_normal((5, 4096)) * 3).astype(np.float32)
    y = np.zeros_like(xs)
    ref.lib.ref_rms_norm(xs, 4096, 5, y)
    out["rms_x"], out["rms_y"] = xs, y
    xr = rng.standard_normal((7, 32, 128)).astype(np.float32)
    yr = np.zeros_like(xr)
    ref.lib.ref_rope(xr, 128, 32, 7, 300, yr)
    out["rope_x"], out["rope_y"] = xr, yr
    xsl = (rng.standard_normal(20000) * 4).astype(np.float32)
    ysl = np.zeros_like(xsl)
    ref.lib.ref_silu(xsl, xsl.size, ysl)
    out["silu_x"], out["silu_y"] = xsl, ysl
    E, H, C = 512, 4, 128
    for (n_past, N) in [(5, 1), (40, 3), (60, 37)]:
        kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
        vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
        q = rng.standard_normal(N * E).astype(np.float32)
        o = np.zeros(N * E, np.float32)
        ref.lib.ref_attention(kc, vc, q, E, H, C, n_past, N, o)
        key = "attn_%d_%d" % (n_past, N)
        out[key + "_kc"], out[key + "_vc"], out[key + "_q"], out[key + "_o"] = kc, vc, q, o
    np.savez_compressed(os.path.join(HERE, "ops_q4.npz"), **out)


def tiny(ref, name, cfg, tmp):
    path = gen_model(os.path.join(tmp, name + ".bin"), **cfg)
    m = ref.model(path, 512)
    toks = prompt_tokens(sum(CHUNKS))
    steps, tokens_fed = [], []
    n_past = 0
    for ch in CHUNKS:
        lg = m.eval(toks[n_past:n_past + ch], n_past)
        steps.append(lg[-1])
        tokens_fed.append(toks[n_past:n_past + ch])
        n_past += ch
    tok = int(np.argmax(steps[-1]))
    for _ in range(N_DECODE):
        lg = m.eval([tok], n_past)
        steps.append(lg[-1])
        tokens_fed.append(np.array([tok], np.int32))
        n_past += 1
        tok = int(np.argmax(lg[-1]))
    m.close()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), logits=np.stack(steps),
                        tokens=np.concatenate(tokens_fed), chunks=np.array([len(t) for t in tokens_fed], np.int32),
                        model_sha256=np.array(sha256(path)), cfg=np.array(json.dumps(cfg)))


def main():
    ref = Ref()
    only = sys.argv[1:]          # optional: regenerate only these fixtures (names without .npz)
    if not only:
        ops(ref)
    tmp = "/tmp/lvk_golden"
    os.makedirs(tmp, exist_ok=True)
    for name, cfg in TINY.items():
        if not only or name in only:
            tiny(ref, name, cfg, tmp)
    if only:
        return
    # reference tests/test-quantize.c known answers (src[i] = i+1)
    src = np.arange(1, 33, dtype=np.float32)
    q0 = ref.quantize(src, 2, reference=True)
    q1 = ref.quantize(src, 3, reference=True)
    json.dump({"src": src.tolist(), "q4_0": q0.tolist(), "q4_1": q1.tolist()},
              open(os.path.join(HERE, "test_quantize.json"), "w"))
    print("golden fixtures written")


if __name__ == "__main__":
    main()
