"""Operator-level parity of the HIP kernels against the CPU oracle (bit-exact).

Each op runs the production kernel through include/lvk_ops.h on seeded
inputs; the oracle restates the reference AVX2 arithmetic (pinned by
test_oracle_golden.py against the reference's own outputs).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def lvk(gpu_available):
    import lvk as m
    return m


@pytest.mark.parametrize("k", [256, 4096, 11008])
@pytest.mark.parametrize("qt", [2, 3])
def test_quantize_rows(lvk, oracle, k, qt):
    rng = np.random.default_rng(k)
    x = np.concatenate([rng.standard_normal((4, k)) * s for s in (1e-3, 1.0, 50.0)]).astype(np.float32)
    x[0, :32] = 0.0          # an all-zero block (id = 0 branch)
    x[1, 5] = 1e-30          # tiny values
    x[2, 64:96] = -0.0       # a block of negative zeros (max/min tree order)
    x[3, 96:128] = 7.25      # a constant block (d = 0 for Q4_1)
    got = lvk.quantize_rows(x, qt)
    for i, row in enumerate(x):
        assert np.array_equal(got[i], oracle.quantize(row, qt)), "row %d" % i


def _weights(oracle, rng, m, k, qt, scale=0.02):
    w = (rng.standard_normal((m, k)) * scale).astype(np.float32)
    return np.stack([oracle.quantize(r, qt, reference=True) for r in w])


def _oracle_mm(oracle, wq, xq_rows, k, qt):
    return np.array([[oracle.vec_dot(qt, k, wr, xr) for wr in wq] for xr in xq_rows], np.float32)


@pytest.mark.parametrize("m,k,n", [(64, 256, 1), (48, 4096, 1), (32, 11008, 1), (64, 4096, 5), (16, 4096, 9),
                                   (40, 8192, 1), (24, 22016, 1)])
def test_mul_mat_q4_0(lvk, oracle, m, k, n):
    rng = np.random.default_rng(m * 7 + k + n)
    wq = _weights(oracle, rng, m, k, 2)
    x = (rng.standard_normal((n, k)) * 1.3).astype(np.float32)
    got = lvk.mul_mat_q(2, wq, m, k, x)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, 2) for r in x], k, 2)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("m,k,n", [(64, 256, 1), (32, 5120, 1), (16, 13824, 1), (48, 5120, 3), (16, 1024, 8),
                                   (4104, 5120, 1), (264, 4096, 1), (40, 11008, 1)])
def test_mul_mat_q4_1(lvk, oracle, m, k, n):
    rng = np.random.default_rng(m * 5 + k + n)
    wq = _weights(oracle, rng, m, k, 3)
    x = (rng.standard_normal((n, k)) * 0.9).astype(np.float32)
    x[0, :32] = 0.25                                        # constant block: d = 0
    got = lvk.mul_mat_q(3, wq, m, k, x)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, 3) for r in x], k, 3)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("m,k,n", [(64, 256, 1), (32, 5120, 1), (32, 5120, 5), (2056, 5120, 1), (136, 4096, 1)])
def test_mul_mat_q4_1_rmsnorm_prologue(lvk, oracle, m, k, n):
    rng = np.random.default_rng(m + k * 7 + n)
    wq = _weights(oracle, rng, m, k, 3)
    x = (rng.standard_normal((n, k)) * 2.0).astype(np.float32)
    g = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float32)
    got = lvk.mul_mat_q_norm(3, wq, m, k, g, x)
    xn = np.zeros_like(x)
    oracle.lib.orc_rms_norm(x, k, n, xn)
    xn = (g[None, :] * xn).astype(np.float32)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, 3) for r in xn], k, 3)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("m,k,n", [(64, 256, 1), (64, 4096, 1), (64, 4096, 6), (128, 8192, 1)])
def test_mul_mat_q4_0_rmsnorm_prologue(lvk, oracle, m, k, n):
    rng = np.random.default_rng(m + k * 3 + n)
    wq = _weights(oracle, rng, m, k, 2)
    x = (rng.standard_normal((n, k)) * 2.0).astype(np.float32)
    g = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float32)
    got = lvk.mul_mat_q_norm(2, wq, m, k, g, x)
    xn = np.zeros_like(x)
    oracle.lib.orc_rms_norm(x, k, n, xn)
    xn = (g[None, :] * xn).astype(np.float32)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, 2) for r in xn], k, 2)
    assert np.array_equal(bits(got), bits(want))


def test_exp_self_check(lvk):
    # the softmax computes fp16(expf(h)) in registers only when it equals this
    # host's table_exp_f16 on every argument h <= 0; on this image it must
    assert lvk.exp_table_mismatches() == 0


@pytest.mark.parametrize("exp_path", ["computed", "table"])
@pytest.mark.parametrize("n_past,N,C,qs", [(0, 1, 256, 1), (5, 1, 256, 1), (31, 1, 256, 1), (32, 1, 256, 1),
                                           (200, 1, 256, 1), (40, 3, 256, 1), (60, 37, 256, 1), (0, 64, 256, 1),
                                           (10, 100, 256, 1), (200, 1, 256, 8), (700, 1, 1024, 1),
                                           (511, 2, 1024, 4), (1000, 3, 1024, 1)])
def test_attention(lvk, oracle, monkeypatch, exp_path, n_past, N, C, qs):
    # C = 1024 runs V steps past the 16 staged in LDS; qs scales q so the
    # softmax reaches deep-negative exp arguments (fp16 underflow to 0)
    if exp_path == "table":
        monkeypatch.setenv("LVK_EXP_TABLE", "1")
    E, H = 512, 4
    rng = np.random.default_rng(n_past * 131 + N + C)
    kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    q = (qs * rng.standard_normal(N * E)).astype(np.float32)
    got = lvk.attention(kc, vc, q, E, H, C, n_past, N)
    want = np.zeros(N * E, np.float32)
    oracle.lib.orc_attention(kc, vc, q, E, H, C, n_past, N, want)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("exp_path", ["computed", "table"])
@pytest.mark.parametrize("n_past,N,C,qs", [(0, 2, 256, 1), (40, 3, 256, 1), (60, 37, 256, 1), (0, 64, 256, 1),
                                           (10, 100, 256, 8), (0, 512, 512, 1), (100, 300, 512, 4),
                                           (511, 2, 1024, 4), (1000, 3, 1024, 1), (64, 900, 1024, 1)])
def test_attention_prompt_kernels(lvk, oracle, monkeypatch, exp_path, n_past, N, C, qs):
    """the prompt-batch attention (attention_prompt.hip) is bit-identical to the reference graph"""
    if exp_path == "table":
        monkeypatch.setenv("LVK_EXP_TABLE", "1")
    E, H = 512, 4
    rng = np.random.default_rng(n_past * 17 + N + C)
    kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    q = (qs * rng.standard_normal(N * E)).astype(np.float32)
    got = lvk.attention_prompt(kc, vc, q, E, H, C, n_past, N)
    want = np.zeros(N * E, np.float32)
    oracle.lib.orc_attention(kc, vc, q, E, H, C, n_past, N, want)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("exp_path", ["computed", "table"])
@pytest.mark.parametrize("n_past,C,qs", [(0, 256, 1), (5, 256, 1), (31, 256, 1), (32, 256, 1), (63, 256, 8),
                                         (64, 256, 1), (200, 256, 1), (255, 256, 4), (511, 512, 1), (700, 1024, 1),
                                         (1000, 1024, 8), (2047, 2048, 1)])
def test_attention_decode_kernels(lvk, oracle, monkeypatch, exp_path, n_past, C, qs):
    """the split single-token attention (attention_decode.hip) is bit-identical to the reference graph"""
    if exp_path == "table":
        monkeypatch.setenv("LVK_EXP_TABLE", "1")
    E, H = 512, 4
    rng = np.random.default_rng(n_past * 7 + C)
    kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    q = (qs * rng.standard_normal(E)).astype(np.float32)
    got = lvk.attention_decode(kc, vc, q, E, H, C, n_past)
    want = np.zeros(E, np.float32)
    oracle.lib.orc_attention(kc, vc, q, E, H, C, n_past, 1, want)
    assert np.array_equal(bits(got), bits(want))


@pytest.mark.parametrize("n_past", [0, 37, 300, 511])
def test_attention_decode_65b_heads(lvk, oracle, n_past):
    """LLaMA-65B attention shape: 64 heads x 128 (grid 64 x 4 = 256 workgroups exchanging
    score granules), bit-identical to the reference graph"""
    E, H, C = 8192, 64, 512
    rng = np.random.default_rng(n_past + 65)
    kc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    vc = rng.standard_normal(C * E).astype(np.float16).view(np.uint16).copy()
    q = (2 * rng.standard_normal(E)).astype(np.float32)
    got = lvk.attention_decode(kc, vc, q, E, H, C, n_past)
    want = np.zeros(E, np.float32)
    oracle.lib.orc_attention(kc, vc, q, E, H, C, n_past, 1, want)
    assert np.array_equal(bits(got), bits(want))


def test_rms_norm_mul(lvk, oracle):
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((4, 4096)) * 3).astype(np.float32)
    g = (1 + 0.1 * rng.standard_normal(4096)).astype(np.float32)
    got = lvk.rms_norm_mul(x, g)
    want = np.zeros_like(x)
    oracle.lib.orc_rms_norm(x, 4096, 4, want)
    want = (g[None, :] * want).astype(np.float32)
    assert np.array_equal(bits(got), bits(want))


# ---------------------------------------------------------------------------
# MFMA prompt matmul (mm_mfma.hip): the matrix cores produce the per-chain
# integer partials, the VALU runs the reference's fp32 chains -> bit-exact
# against ggml_vec_dot_q4_0's AVX2 order, incl. the fused RMSNorm+quantize.  Both A
# operand sources: the f16 A-fragment image (default) and the nibble unpack
# (LVK_PROMPT_A16=0).
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("a16", ["1", "0"])
@pytest.mark.parametrize("m,k,n,norm", [(128, 256, 2, False), (256, 4096, 64, True), (128, 4096, 70, False),
                                        (128, 11008, 17, False), (384, 1024, 130, True), (128, 5120, 3, True)])
def test_mul_mat_mfma_bit_exact(lvk, oracle, monkeypatch, m, k, n, norm, a16):
    monkeypatch.setenv("LVK_PROMPT_A16", a16)
    rng = np.random.default_rng(m + 3 * k + 11 * n)
    wq = _weights(oracle, rng, m, k, 2)
    x = (rng.standard_normal((n, k)) * 1.7).astype(np.float32)
    x[0, :32] = 0.0                                   # an all-zero activation block (d = 0)
    g = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float32) if norm else None
    got = lvk.mul_mat_q_mfma(2, wq, m, k, x, g=g)
    xin = x
    if norm:
        xn = np.zeros_like(x)
        oracle.lib.orc_rms_norm(x, k, n, xn)
        xin = (g[None, :] * xn).astype(np.float32)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, 2) for r in xin], k, 2)
    assert np.array_equal(bits(got), bits(want))


# the Q4_1 MFMA matmul (mm_mfma41.hip): chain partials, cross-term sums and scale
# products on the matrix cores, ggml_vec_dot_q4_1's chains on the VALU -> bit-exact.
# Shapes: LLaMA-13B rows (K 5120 / 13824), ragged token tiles, a 130-token batch; blocks
# with d = 0 (all-zero and constant activations, constant weight blocks).
@pytest.mark.parametrize("dma", ["1", "0"])
@pytest.mark.parametrize("m,k,n,norm", [(128, 256, 2, False), (256, 5120, 40, True), (128, 13824, 17, False),
                                        (384, 1024, 130, True), (128, 4096, 16, False), (128, 5120, 3, True)])
def test_mul_mat_mfma_q4_1_bit_exact(lvk, oracle, monkeypatch, m, k, n, norm, dma):
    """both operand streams: the LDS-DMA ring (default) and the register ring (LVK_MM41_DMA=0)"""
    monkeypatch.setenv("LVK_MM41_DMA", dma)
    rng = np.random.default_rng(7 * m + k + 13 * n)
    w = (rng.standard_normal((m, k)) * 0.02).astype(np.float32)
    w[1, 32:64] = 0.01                                # a constant weight block (d = 0, m = 0.01)
    w[2, :32] = 0.0                                   # an all-zero weight block
    wq = np.stack([oracle.quantize(r, 3, reference=True) for r in w])
    x = (rng.standard_normal((n, k)) * 1.7).astype(np.float32)
    x[0, :32] = 0.0                                   # an all-zero activation block
    x[-1, 64:96] = -0.5                               # a constant activation block
    g = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float32) if norm else None
    got = lvk.mul_mat_q_mfma(3, wq, m, k, x, g=g)
    xin = x
    if norm:
        xn = np.zeros_like(x)
        oracle.lib.orc_rms_norm(x, k, n, xn)
        xin = (g[None, :] * xn).astype(np.float32)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, 3) for r in xin], k, 3)
    assert np.array_equal(bits(got), bits(want))


# ---------------------------------------------------------------------------
# the reference's op-level codec table (ggml.h:803-814) exported by this library
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("qt,k", [(2, 256), (2, 4096), (2, 96), (3, 5120), (3, 4096), (3, 160)])
def test_ggml_internal_get_quantize_fn_vs_oracle(lvk, oracle, qt, k):
    """ggml_internal_get_quantize_fn(GGML_TYPE_Q4_0 / _Q4_1): quantize_row_q (AVX2 rules),
    quantize_row_q_reference (roundf), dequantize_row_q and vec_dot_q, each on the GPU, bit-exact
    against the oracle's restatement of the same reference functions (k not a multiple of 256
    exercises the zero-block padding of vec_dot_q)"""
    f = lvk.QuantizeFns(0 if qt == 2 else 1)
    assert f.valid
    rng = np.random.default_rng(qt * 1000 + k)
    x = (rng.standard_normal(k) * 1.7).astype(np.float32)
    x[:32] = 0.0                                   # an all-zero block
    if k >= 96:
        x[64:96] = np.float32(2.5) * (np.arange(32) % 2 * 2 - 1)   # ties at the rounding boundary
    for ref in (False, True):
        got = f.quantize_row(x, reference=ref)
        assert np.array_equal(got, oracle.quantize(x, qt, reference=ref)), "reference=%s" % ref
    q = oracle.quantize(x, qt)
    assert np.array_equal(f.dequantize_row(q, k).view(np.uint32), oracle.dequantize(q, qt, k).view(np.uint32))
    w = oracle.quantize((rng.standard_normal(k) * 0.6).astype(np.float32), qt)
    got = np.float32(f.vec_dot(k, w, q))
    want = np.float32(oracle.vec_dot(qt, k, w, q))
    assert got.view(np.uint32) == want.view(np.uint32)


def test_ggml_internal_get_quantize_fn_vs_reference_build(lvk, ref):
    """the same four functions against the reference build's own table (oracle/_ref/libref.so)"""
    for qt in (2, 3):
        f = lvk.QuantizeFns(0 if qt == 2 else 1)
        rng = np.random.default_rng(qt)
        x = (rng.standard_normal(4096) * 2.2).astype(np.float32)
        for reff in (False, True):
            assert np.array_equal(f.quantize_row(x, reference=reff), ref.quantize(x, qt, reference=reff))
        q = ref.quantize(x, qt)
        assert np.array_equal(f.dequantize_row(q, 4096).view(np.uint32), ref.dequantize(q, qt, 4096).view(np.uint32))
        w = ref.quantize((rng.standard_normal(4096) * 0.4).astype(np.float32), qt)
        assert np.float32(f.vec_dot(4096, w, q)).view(np.uint32) == np.float32(ref.vec_dot(qt, 4096, w, q)).view(np.uint32)
    assert not lvk.QuantizeFns(6).valid          # GGML_TYPE_F32: no codec entry


# ---------------------------------------------------------------------------
# RMSNorm rows whose float mean depends on the summation order (RMSNorm
# order; lvk_device.h rms_mean).  x[0]^2 + x[1]^2 puts sum / K exactly on a float rounding
# midpoint, and each of the K - 2 equal tiny squares is below half an ulp of that sum: the
# reference's index-order double sum (ggml.c:6060-6065) drops them all and the tie rounds to
# even, while a tree that adds the tiny terms first keeps them and rounds up.  Found by a
# seeded search over 12-bit x[0], x[1] (tests/golden/make_rms_order_rows.py).
# ---------------------------------------------------------------------------
_RMS_ORDER_ROWS = {
    256: (1.1416015625, 0.574951171875, 7.450580596923828e-09),
    4096: (0.95947265625, 0.394775390625, 7.450580596923828e-09),
    5120: (17.3515625, 4.544921875, 1.1920928955078125e-07),
}


def _rms_order_rows(rng, k, n, scale=1.0):
    """n rows: even rows are the order-sensitive row (times a power of two), odd rows random"""
    a, b, t = _RMS_ORDER_ROWS[k]
    x = (rng.standard_normal((n, k)) * 1.3).astype(np.float32)
    for i in range(0, n, 2):
        x[i] = np.float32(t)
        x[i, 0], x[i, 1] = a, b
        x[i] *= np.float32(scale * 2.0 ** (i % 3))
    return x


def _rms_exact_sum(x, g):
    """g * rms_norm(x) with the exactly rounded sum of squares (what a tree that keeps every
    tiny term gives here) instead of the index-order one"""
    import math
    out = np.empty_like(x)
    k = x.shape[1]
    for i, row in enumerate(x):
        sq = (row * row).astype(np.float32)
        mean = np.float32(math.fsum(float(v) for v in sq) / k)
        sc = np.float32(1.0) / np.sqrt(np.float32(mean + np.float32(1e-6)), dtype=np.float32)
        out[i] = g * (row * sc).astype(np.float32)
    return out.astype(np.float32)


def _rms_oracle(oracle, x, g):
    n, k = x.shape
    xn = np.zeros_like(x)
    oracle.lib.orc_rms_norm(np.ascontiguousarray(x), k, n, xn)
    return (g[None, :] * xn).astype(np.float32)


def test_rms_norm_order_sensitive_rows_vs_oracle(lvk, oracle):
    """the row helper of the embeddings path (k_rmsnorm_rows): the index-order mean"""
    rng = np.random.default_rng(61)
    x = _rms_order_rows(rng, 4096, 4)
    g = (1 + 0.1 * rng.standard_normal(4096)).astype(np.float32)
    want = _rms_oracle(oracle, x, g)
    assert not np.array_equal(bits(want[0]), bits(_rms_exact_sum(x[:1], g)[0])), "row not order-sensitive"
    assert np.array_equal(bits(lvk.rms_norm_mul(x, g)), bits(want))


@pytest.mark.parametrize("qt,k,n,mfma", [(2, 4096, 1, False), (2, 4096, 5, False), (2, 256, 1, False),
                                         (2, 4096, 17, True), (3, 5120, 1, False), (3, 5120, 3, False),
                                         (3, 5120, 17, True), (3, 256, 1, False)])
def test_rmsnorm_prologues_order_sensitive_rows(lvk, oracle, qt, k, n, mfma):
    """every fused RMSNorm prologue -- decode matvecs (k_mv_cu / k_mv_cu41), batched matvecs
    (k_matvec_q40 / q41) and the prompt activation kernels (k_act_q40_f16 / q41) -- on rows
    whose mean the summation order changes: the products equal the oracle's, which follows
    the reference's index order, and differ from what the exactly rounded sum would give"""
    rng = np.random.default_rng(qt * 100 + k + n)
    m = 128
    wq = _weights(oracle, rng, m, k, qt)
    x = _rms_order_rows(rng, k, n)
    g = (1.0 + 0.1 * rng.standard_normal(k)).astype(np.float32)
    want = _oracle_mm(oracle, wq, [oracle.quantize(r, qt) for r in _rms_oracle(oracle, x, g)], k, qt)
    other = _oracle_mm(oracle, wq, [oracle.quantize(r, qt) for r in _rms_exact_sum(x, g)], k, qt)
    assert not np.array_equal(bits(want[0]), bits(other[0])), "row 0 not order-sensitive through the matvec"
    got = lvk.mul_mat_q_mfma(qt, wq, m, k, x, g=g) if mfma else lvk.mul_mat_q_norm(qt, wq, m, k, g, x)
    assert np.array_equal(bits(got), bits(want))
