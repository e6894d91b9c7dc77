"""The ggml operator surface (include/ggml.h, runtime/ggml_graph.cpp) without a GPU: the same
ggml caller (tools/ggml_graph/graph_test.c: the llama_eval_internal graph, reference
llama.cpp:927-1197) builds identical graphs -- node count, leaf count, op / type / shape /
stride sequence -- and identical memory-pool accounting (ggml_used_mem) against this library
and against the reference ggml.c (oracle/_ref/graph_test_ref); host-side helpers (fp16
conversion, sizes) agree with the reference's definitions (ggml.h:192-193, 341-351)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LVK_BIN = os.path.join(ROOT, "tools", "ggml_graph", "bin", "graph_test_lvk")
REF_BIN = os.path.join(ROOT, "oracle", "_ref", "graph_test_ref")
LIB = os.path.join(ROOT, "llama.vk_amd", "lib", "libllama_vk_amd.so")


def _build():
    if not os.path.exists(LVK_BIN):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "tools", "ggml_graph")], stdout=subprocess.DEVNULL)


@pytest.mark.parametrize("wtype,kv", [(0, 1), (1, 1), (0, 0)])
def test_graph_topology_and_pool_match_reference(wtype, kv, tmp_path):
    _build()
    if not os.path.exists(REF_BIN):
        pytest.skip("reference build oracle/_ref/graph_test_ref not present")
    env = dict(os.environ, GRAPH_TEST_BUILD_ONLY="1")
    if os.environ.get("LVK_LIB"):       # another build of the library (the sanitizer run)
        env["LD_LIBRARY_PATH"] = os.path.dirname(os.environ["LVK_LIB"])
    outs = []
    for b in (REF_BIN, LVK_BIN):
        r = subprocess.run([b, str(tmp_path / "x.bin"), str(wtype), str(kv)], capture_output=True, text=True,
                           env=env, timeout=120)
        assert r.returncode == 0, r.stderr
        outs.append(r.stderr)
    assert outs[0] == outs[1]
    assert outs[0].count("topology") == 4


def test_fp16_and_sizes():
    lib = C.CDLL(LIB)
    lib.ggml_fp32_to_fp16.restype = C.c_uint16
    lib.ggml_fp32_to_fp16.argtypes = [C.c_float]
    lib.ggml_fp16_to_fp32.restype = C.c_float
    lib.ggml_fp16_to_fp32.argtypes = [C.c_uint16]
    rng = np.random.default_rng(1)
    for x in list(rng.standard_normal(200).astype(np.float32) * 100) + [65520.0, 1e-8, -0.0, 6.1e-5]:
        assert lib.ggml_fp32_to_fp16(float(x)) == int(np.float16(x).view(np.uint16)), x
    for h in (0, 1, 0x3C00, 0x7BFF, 0x8001, 0xFC00):
        assert lib.ggml_fp16_to_fp32(h) == float(np.uint16(h).view(np.float16))
    lib.ggml_type_size.restype = C.c_size_t
    lib.ggml_blck_size.restype = C.c_int
    assert [lib.ggml_type_size(t) for t in range(7)] == [20, 24, 1, 2, 4, 2, 4]
    assert [lib.ggml_blck_size(t) for t in range(7)] == [32, 32, 1, 1, 1, 1, 1]
