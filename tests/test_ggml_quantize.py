"""The file-creation quantizers of the ggml surface without a GPU: ggml_quantize_q4_0 /
ggml_quantize_q4_1 (reference ggml.h:772-773, ggml.c:10520-10564) and the system-info calls
(ggml.h:779-790).

* the reference's own unit test (tests/test-quantize.c), compiled unmodified against
  include/ggml.h and linked to this library (tools/dropin/Makefile), exits 0;
* bytes, return value and histogram equal the reference build's ggml_quantize_q4_x
  (oracle/_ref/libref.so, compiled from the reference sources) on seeded rows with ties at
  .5, zero blocks and several rows per call, and the CPU oracle's quantize_row_q4_x_reference
  (pinned to the golden vectors in test_oracle_golden.py);
* every ggml_cpu_has_* returns what the reference build (compiled with the survey's AVX2
  flags, oracle/Makefile) returns on this host; avx512, which that build leaves out at
  compile time, reports the host CPU (/proc/cpuinfo) as a native -march build would.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("LVK_LIB") or os.path.join(ROOT, "llama.vk_amd", "lib", "libllama_vk_amd.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
TEST_QUANTIZE = os.path.join(ROOT, "tools", "dropin", "bin", "test-quantize")
HAS = ["avx", "avx2", "avx512", "fma", "neon", "arm_fma", "f16c", "fp16_va", "wasm_simd", "blas", "sse3", "vsx"]


def _q(lib, name):
    f = getattr(lib, name)
    f.restype = C.c_size_t
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_void_p]
    return f


def _rows(rng, n_rows, k):
    x = (rng.standard_normal((n_rows, k)) * rng.uniform(0.01, 10.0, (n_rows, 1))).astype(np.float32)
    x[0, :32] = 0.0                                   # an all-zero block: d = 0, id = 0
    x[1, :32] = np.arange(32, dtype=np.float32) - 14  # amax 17: x * (7/17) hits .5 ties
    x[1, 32:64] = np.float32(3.5)                     # q4_1: max == min -> d = 0
    return x


def _run(lib, name, x, k):
    bs = 20 if name.endswith("q4_0") else 24
    y = np.zeros(x.size // 32 * bs, np.uint8)
    hist = np.zeros(16, np.int64)
    n = _q(lib, name)(x.ctypes.data, y.ctypes.data, x.size, k, hist.ctypes.data)
    return n, y, hist


def test_reference_test_quantize_relinked():
    if not os.path.exists(TEST_QUANTIZE):
        pytest.skip("tools/dropin/bin/test-quantize not built (needs /root/reference)")
    p = subprocess.run([TEST_QUANTIZE], capture_output=True, timeout=60)
    assert p.returncode == 0, p.stderr.decode(errors="replace")


@pytest.mark.parametrize("name,qtype", [("ggml_quantize_q4_0", 2), ("ggml_quantize_q4_1", 3)])
@pytest.mark.parametrize("k", [32, 256, 4096])
def test_quantize_matches_reference_build(name, qtype, k):
    lib = C.CDLL(LIB)
    x = _rows(np.random.default_rng(k + qtype), 6, k)
    n, y, hist = _run(lib, name, x, k)
    assert n == y.size
    # histogram = the nibbles of the bytes written
    nib = y.reshape(-1, 20 if qtype == 2 else 24)[:, 4 if qtype == 2 else 8:]
    want = np.bincount(np.concatenate([nib & 0xF, nib >> 4]).ravel(), minlength=16)
    assert np.array_equal(hist, want)
    # the oracle's quantize_row_q4_x_reference, row by row
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle_lib import Oracle
    o = np.concatenate([Oracle().quantize(r, qtype, reference=True) for r in x])
    assert np.array_equal(o, y)
    if os.path.exists(REF_SO):
        rn, ry, rh = _run(C.CDLL(REF_SO), name, x, k)
        assert rn == n and np.array_equal(ry, y) and np.array_equal(rh, hist)


def test_cpu_has_matches_reference_build():
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref/libref.so not built")
    lib, ref = C.CDLL(LIB), C.CDLL(REF_SO)
    flags = open("/proc/cpuinfo").read().split()
    for h in HAS:
        want = int("avx512f" in flags) if h == "avx512" else getattr(ref, "ggml_cpu_has_" + h)()
        assert getattr(lib, "ggml_cpu_has_" + h)() == want, h
