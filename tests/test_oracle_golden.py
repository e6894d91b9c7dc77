"""The CPU oracle against the reference's own golden vectors (no GPU).

Fixtures in tests/golden/ were produced by the reference build itself
(tests/golden/make_golden.py); the reference's tests/test-quantize.c known
answers are reproduced in test_quantize.json.  Everything must be bit-exact.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle_lib import prompt_tokens

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def ops():
    return np.load(os.path.join(GOLD, "ops_q4.npz"), allow_pickle=False)


@pytest.mark.parametrize("qt", [2, 3])
def test_activation_quantizer(oracle, ops, qt):
    for i, row in enumerate(ops["x"]):
        assert np.array_equal(oracle.quantize(row, qt), ops["q%d" % qt][i]), "row %d" % i


@pytest.mark.parametrize("qt", [2, 3])
def test_file_quantizer_and_dequant(oracle, ops, qt):
    for i, row in enumerate(ops["w"]):
        wq = oracle.quantize(row, qt, reference=True)
        assert np.array_equal(wq, ops["wq%d" % qt][i])
        assert np.array_equal(bits(oracle.dequantize(wq, qt, 4096)), bits(ops["deq%d" % qt][i]))


@pytest.mark.parametrize("qt", [2, 3])
def test_vec_dot(oracle, ops, qt):
    got = np.array([[oracle.vec_dot(qt, 4096, ops["wq%d" % qt][i], ops["q%d" % qt][j])
                     for j in range(len(ops["x"]))] for i in range(len(ops["w"]))], np.float32)
    assert np.array_equal(bits(got), bits(ops["dot%d" % qt]))


def test_rms_norm_rope_silu(oracle, ops):
    x = ops["rms_x"]
    y = np.zeros_like(x)
    oracle.lib.orc_rms_norm(x, x.shape[1], x.shape[0], y)
    assert np.array_equal(bits(y), bits(ops["rms_y"]))
    xr = ops["rope_x"]
    yr = np.zeros_like(xr)
    oracle.lib.orc_rope(np.ascontiguousarray(xr), 128, 32, 7, 300, yr)
    assert np.array_equal(bits(yr), bits(ops["rope_y"]))
    xs = ops["silu_x"]
    ys = np.zeros_like(xs)
    oracle.lib.orc_silu(xs, xs.size, ys)
    assert np.array_equal(bits(ys), bits(ops["silu_y"]))


@pytest.mark.parametrize("n_past,N", [(5, 1), (40, 3), (60, 37)])
def test_attention(oracle, ops, n_past, N):
    key = "attn_%d_%d" % (n_past, N)
    o = np.zeros(N * 512, np.float32)
    oracle.lib.orc_attention(ops[key + "_kc"], ops[key + "_vc"], ops[key + "_q"], 512, 4, 128, n_past, N, o)
    assert np.array_equal(bits(o), bits(ops[key + "_o"]))


def test_reference_test_quantize_known_answers(oracle):
    # reference tests/test-quantize.c: src[i] = i+1 -> d = 32/7, q = roundf(x/d)+8; q4_1 d = 31/15, m = 1
    g = json.load(open(os.path.join(GOLD, "test_quantize.json")))
    src = np.array(g["src"], np.float32)
    q0 = oracle.quantize(src, 2, reference=True)
    q1 = oracle.quantize(src, 3, reference=True)
    assert q0.tolist() == g["q4_0"] and q1.tolist() == g["q4_1"]
    d = q0[:4].view(np.float32)[0]
    assert d == np.float32(32.0) / np.float32(7.0)
    for i in range(32):
        nib = (q0[4 + i // 2] >> 4) if i % 2 else (q0[4 + i // 2] & 15)
        assert nib == int(np.round(src[i] / d)) + 8 or nib == np.floor(src[i] / d + np.float32(0.5)) + 8


def sha256(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for b in iter(lambda: f.read(1 << 20), b""):
            h.update(b)
    return h.hexdigest()


@pytest.mark.parametrize("name", ["tiny_q4_0", "tiny_q4_1", "tiny_l80_q4_0"])
def test_tiny_model_logits(oracle, tiny_models, name):
    g = np.load(os.path.join(GOLD, name + ".npz"), allow_pickle=False)
    path = tiny_models[name]
    assert sha256(path) == str(g["model_sha256"]), "synthetic generator is not reproducing the golden model"
    m = oracle.model(path, 512)
    n_past, off = 0, 0
    for step, n in enumerate(g["chunks"]):
        lg = m.eval(g["tokens"][off:off + n], n_past)
        assert np.array_equal(bits(lg[-1]), bits(g["logits"][step])), "step %d" % step
        n_past += n
        off += n
    m.close()
