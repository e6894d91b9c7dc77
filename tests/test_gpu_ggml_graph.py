"""ggml_graph_compute on the GPU against the reference ggml.c: one ggml caller
(tools/ggml_graph/graph_test.c) builds the LLaMA graph of llama_eval_internal
(reference llama.cpp:927-1197: get_rows, rms_norm, mul/repeat, Q4 mul_mat, reshape, rope,
cpy into the KV views, permute, f16/f32 mul_mat, scale, diag_mask_inf, soft_max, add, silu)
for a 7-token prompt, a 33-token batch and two decode steps, computes it with this library
(every node on the GPU) and with the reference's CPU AVX2 ggml.c, and both dumps -- logits of
every step and both KV caches -- must be bit-identical.  Weights Q4_0 or Q4_1, KV f16 or f32."""
import os
import subprocess

import numpy as np
import pytest

from test_ggml_graph import LVK_BIN, REF_BIN, _build


@pytest.mark.gpu
@pytest.mark.parametrize("wtype,kv", [(0, 1), (1, 1), (0, 0)])
def test_graph_compute_matches_reference_ggml(gpu_available, wtype, kv, tmp_path):
    _build()
    if not os.path.exists(REF_BIN):
        pytest.skip("reference build oracle/_ref/graph_test_ref not present")
    dumps = []
    for b, name in ((REF_BIN, "ref"), (LVK_BIN, "lvk")):
        out = tmp_path / ("%s.bin" % name)
        r = subprocess.run([b, str(out), str(wtype), str(kv)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        dumps.append(np.fromfile(out, np.uint8))
    assert dumps[0].size == dumps[1].size and dumps[0].size > 0
    V = 512
    n_logits = V * (7 + 33 + 1 + 1)
    a = dumps[0][:n_logits * 4].view(np.float32)
    b = dumps[1][:n_logits * 4].view(np.float32)
    bad = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32))
    assert bad.size == 0, "logits differ at %d places, first %s: %r vs %r" % (bad.size, bad[:5], a[bad[:5]], b[bad[:5]])
    assert np.array_equal(dumps[0], dumps[1]), "KV caches differ"


@pytest.mark.gpu
@pytest.mark.parametrize("cache", ["1", "2"])
@pytest.mark.parametrize("wtype", [0, 1])
def test_graph_compute_uploads_weights_once(gpu_available, wtype, cache, tmp_path):
    """ggml_graph_compute keeps its device state across calls: the weights (a read-only
    buffer of the caller, like llama.cpp's PROT_READ model mapping) go host -> device and
    are repacked in the first call only; each later decode step uploads just what the host
    may have changed (its token ids, the KV positions it reads -- well under the weight
    bytes) and copies back just the bytes its nodes wrote.  The logits of the compared
    steps stay those of the plain run (test above)."""
    _build()
    env = dict(os.environ, GRAPH_TEST_REPEAT="6", LVK_GGML_CACHE=cache)
    r = subprocess.run([LVK_BIN, str(tmp_path / "x.bin"), str(wtype), "1"], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    calls = []
    for ln in r.stderr.splitlines():
        if ln.startswith("compute "):
            f = ln.split()
            calls.append({f[i]: float(f[i + 1]) for i in range(2, len(f) - 1, 2)})
    assert len(calls) == 10, r.stderr[-2000:]
    E, F, V, L = 256, 768, 512, 2
    blk = 20 if wtype == 0 else 24
    wbytes = (L * (4 * E * E + 3 * E * F) + 2 * E * V) // 32 * blk
    assert calls[0]["h2d"] >= wbytes and calls[0]["repack"] >= wbytes - E * V // 32 * blk
    for c in calls[4:]:
        assert c["repack"] == 0, calls
        assert c["h2d"] < wbytes / 4, calls
        assert c["d2h"] < wbytes / 4, calls
        assert c["mode"] == int(cache), calls
    print("per-call ms:", [round(c["ms"], 3) for c in calls], "h2d:", [int(c["h2d"]) for c in calls])


@pytest.mark.gpu
@pytest.mark.parametrize("cache", ["1", "2"])
@pytest.mark.parametrize("mode", ["private", "pinned", "shared", "remap", "mprotect"])
def test_graph_compute_sees_untracked_host_writes(gpu_available, mode, cache):
    """the mirrors must not keep a stale device copy of host bytes that change where the CPU
    page tables cannot see it between two calls: a hipMemcpy D2H (DMA) into a pinned context
    buffer, a write through a second MAP_SHARED view of the buffer's pages, and a plain CPU
    write, a read-only file mapping replaced by another file's at the same address, and pages
    written and then made read-only (tools/ggml_graph/volatile_test.cpp: z = x + y checked
    after each); under the
    default caching (1) and under the opt-in soft-dirty tracking of writable pages (2)"""
    b = os.path.join(os.path.dirname(LVK_BIN), "volatile_test")
    if not os.path.exists(b):
        subprocess.check_call(["make", "-C", os.path.dirname(os.path.dirname(b))], stdout=subprocess.DEVNULL)
    r = subprocess.run([b, mode], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, LVK_GGML_CACHE=cache))
    assert r.returncode == 0 and ("ok %s" % mode) in r.stdout, r.stderr[-2000:]
