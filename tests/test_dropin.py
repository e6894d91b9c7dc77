"""The reference's own example programs, unmodified, linked to this library.

tools/dropin/Makefile compiles /root/reference/examples/{main,perplexity,
embedding,quantize,quantize-stats} against include/llama.h (+ include/ggml.h,
include/llama_internal.h) and links them
to libllama_vk_amd.so instead of the reference's llama.o/ggml.o -- the drop-in
boundary of INTEGRATION.md.  The reference CPU build of the same main
(oracle/_ref/main) is the checker: with greedy sampling, bit-exact logits give
the identical generated text.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DROPIN = os.path.join(ROOT, "tools", "dropin", "bin")
REF_MAIN = os.path.join(ROOT, "oracle", "_ref", "main")


def _need(path):
    if not os.path.exists(path):
        pytest.skip("%s not built (make -C tools/dropin / oracle needs /root/reference)" % path)


def _run(args, timeout=300):
    p = subprocess.run(args, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-2000:]
    return p.stdout, p.stderr


def test_dropin_quantize_matches_library_tool(tmp_path):
    """examples/quantize (reference source) on this library: f32 -> q4_0/q4_1 bytes
    equal llama_model_quantize called directly (pinned against the reference in
    test_abi.py)."""
    exe = os.path.join(DROPIN, "quantize")
    _need(exe)
    import numpy as np
    import lvk
    from test_abi import _f32_model
    src = str(tmp_path / "f32.bin")
    _f32_model(src, np.random.default_rng(5))
    for itype in (2, 3):
        a = str(tmp_path / ("a%d.bin" % itype))
        b = str(tmp_path / ("b%d.bin" % itype))
        _run([exe, src, a, str(itype)])
        assert lvk.lib.llama_model_quantize(src.encode(), b.encode(), itype) == 0
        assert open(a, "rb").read() == open(b, "rb").read()


@pytest.mark.gpu
def test_dropin_main_greedy_text_matches_reference_cpu(tiny_models):
    """examples/main on the GPU library vs the reference AVX2 build on the CPU:
    same model, prompt, seed and greedy sampling -> the same text."""
    exe = os.path.join(DROPIN, "main")
    _need(exe)
    _need(REF_MAIN)
    args = ["-m", tiny_models["tiny_q4_0"], "-p", "Building a website can be done in 10 simple steps:",
            "-n", "48", "--temp", "0", "-s", "1", "-c", "256", "--ignore-eos"]
    # both prompt paths are bit-exact: the default MFMA matmuls and the VALU kernels
    gpu_out, gpu_err = _run([exe] + args + ["-t", "1"])
    os.environ["LVK_PROMPT_EXACT"] = "1"
    try:
        exact_out, _ = _run([exe] + args + ["-t", "1"])
    finally:
        del os.environ["LVK_PROMPT_EXACT"]
    assert exact_out == gpu_out
    cpu_out, _ = _run([REF_MAIN] + args + ["-t", "8"])
    assert gpu_out == cpu_out
    assert len(gpu_out) > 60
    assert b"llama_print_timings" in gpu_err


@pytest.mark.gpu
def test_dropin_main_context_swap_matches_reference_cpu(tiny_models):
    """main's infinite generation (main.cpp:246-266): at n_ctx 64 with --keep 4 it keeps
    the first 4 prompt tokens and re-evaluates half of the last 60 as one batch, over and
    over; the GPU library and the reference CPU build print the same text"""
    exe = os.path.join(DROPIN, "main")
    _need(exe)
    _need(REF_MAIN)
    args = ["-m", tiny_models["tiny_q4_0"], "-p", "Building a website can be done in 10 simple steps:",
            "-n", "160", "--temp", "0", "-s", "1", "-c", "64", "--keep", "4", "--ignore-eos"]
    gpu_out, _ = _run([exe] + args + ["-t", "1"])
    cpu_out, _ = _run([REF_MAIN] + args + ["-t", "8"])
    assert gpu_out == cpu_out
    assert len(gpu_out) > 200


@pytest.mark.gpu
def test_dropin_main_layer_split_matches_reference_cpu(tiny_models):
    """the unmodified main on a 3-stage layer split (LVK_SPLIT_DEVICES; one GPU here, so the
    stages hand off by device copy) with 8-token prompt micro-batches: the same text"""
    exe = os.path.join(DROPIN, "main")
    _need(exe)
    _need(REF_MAIN)
    args = ["-m", tiny_models["tiny_q4_0"], "-p", "Building a website can be done in 10 simple steps:",
            "-n", "48", "--temp", "0", "-s", "1", "-c", "256", "--ignore-eos"]
    env = dict(os.environ, LVK_SPLIT_DEVICES="0,0,0", LVK_SPLIT_MICRO="8")
    p = subprocess.run([exe] + args + ["-t", "1"], stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=300,
                       env=env)
    assert p.returncode == 0, p.stderr.decode(errors="replace")[-2000:]
    assert b"layer split over 3 stages" in p.stderr
    cpu_out, _ = _run([REF_MAIN] + args + ["-t", "8"])
    assert p.stdout == cpu_out


def _ppl_values(out):
    """the `[i]ppl,` fields examples/perplexity prints (perplexity.cpp:76)"""
    import re
    return [(int(a), float(b)) for a, b in re.findall(rb"\[(\d+)\]([0-9.]+),", out)]


@pytest.mark.gpu
def test_dropin_perplexity_matches_reference_cpu(tiny_models, tmp_path):
    """examples/perplexity (logits_all, n_ctx-token batches) on the GPU library vs the
    reference build: the same running perplexity after every chunk."""
    exe = os.path.join(DROPIN, "perplexity")
    ref_exe = os.path.join(ROOT, "oracle", "_ref", "perplexity")
    _need(exe)
    _need(ref_exe)
    words = ["the", "model", "reads", "every", "token", "of", "this", "text", "and", "predicts", "next",
             "one", "from", "its", "context", "window", "while", "perplexity", "measures", "surprise"]
    text = " ".join(words[(i * 7) % len(words)] + ("." if i % 11 == 10 else "") for i in range(600))
    f = tmp_path / "ppl.txt"
    f.write_text(text)
    args = ["-m", tiny_models["tiny_q4_0"], "-f", str(f), "-c", "128", "-s", "1"]
    cpu_out, _ = _run([ref_exe] + args + ["-t", "8"])
    want = _ppl_values(cpu_out)
    assert len(want) >= 3
    os.environ["LVK_PROMPT_EXACT"] = "1"
    try:
        exact_out, _ = _run([exe] + args + ["-t", "1"])
    finally:
        del os.environ["LVK_PROMPT_EXACT"]
    assert _ppl_values(exact_out) == want        # bit-exact logits -> the same printed digits
    mfma_out, _ = _run([exe] + args + ["-t", "1"])
    assert _ppl_values(mfma_out) == want         # the MFMA prompt path is bit-exact too


@pytest.mark.gpu
def test_dropin_embedding_matches_reference_cpu(tiny_models):
    """examples/embedding (embedding.cpp:81-90: the last token's normed embedding printed
    with %f) on the GPU library vs the reference build: the same printed vector"""
    exe = os.path.join(DROPIN, "embedding")
    ref_exe = os.path.join(ROOT, "oracle", "_ref", "embedding")
    _need(exe)
    _need(ref_exe)
    args = ["-m", tiny_models["tiny_q4_0"], "-p", "Building a website can be done in 10 simple steps:",
            "-c", "128", "-s", "1"]
    gpu_out, _ = _run([exe] + args + ["-t", "1"])
    cpu_out, _ = _run([ref_exe] + args + ["-t", "8"])
    vals = gpu_out.split()
    assert len(vals) == 256
    assert gpu_out == cpu_out


def _qstats_lines(out):
    # everything but the wall-clock line (quantize-stats.cpp:346-351)
    return [l for l in out.decode().splitlines() if "time" not in l]


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [["-l", "norm", "-p"], ["-l", "norm", "-r", "--histogram", "-t", "q4_1"]])
def test_dropin_quantize_stats_matches_reference_cpu(tiny_models, flags):
    """examples/quantize-stats, unmodified, on this library: llama_internal_get_tensor_map
    (the file's tensors by name) + ggml_internal_get_quantize_fn (quantize / dequantize on the
    GPU) print the same per-layer and total error statistics as the reference build (the
    float tensors of a Q4 file: the norms)"""
    exe = os.path.join(DROPIN, "quantize-stats")
    ref_exe = os.path.join(ROOT, "oracle", "_ref", "quantize-stats")
    _need(exe)
    _need(ref_exe)
    args = ["-m", tiny_models["tiny_q4_0"]] + flags
    gpu_out, _ = _run([exe] + args)
    cpu_out, _ = _run([ref_exe] + args)
    got, want = _qstats_lines(gpu_out), _qstats_lines(cpu_out)
    assert len(want) >= 4
    assert got == want
