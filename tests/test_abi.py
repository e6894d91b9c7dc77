"""Boundary tests that need no GPU: the C-ABI library loads, exports every
symbol include/*.h declares, mirrors the reference's defaults/struct layout,
and its host-side pieces (tokenizer, quantize tool) match the reference.
"""
import ctypes as C
import json
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "llama.vk_amd", "lib", "libllama_vk_amd.so")
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def lvk():
    if not os.path.exists(LIB):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "llama.vk_amd"), "-j8"], stdout=subprocess.DEVNULL)
    import lvk as m
    return m


def declared_symbols():
    syms = []
    for h in ("llama.h", "lvk_ops.h", "ggml.h"):
        txt = open(os.path.join(ROOT, "include", h)).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = "\n".join(ln for ln in txt.splitlines() if not ln.lstrip().startswith("#"))
        for m in re.finditer(r"(?:LLAMA_API|LVK_API|LVK_GGML_API)\s+[^;(]*?\b(\w+)\s*\(", txt):
            syms.append(m.group(1))
    return syms


def test_exports_every_declared_symbol(lvk):
    syms = declared_symbols()
    assert len(syms) >= 35
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = [s for s in syms if s not in exported]
    assert not missing, missing
    # include/llama_internal.h: the one C++ entry point (reference llama_internal.h:104)
    out = subprocess.check_output(["nm", "-DC", "--defined-only", LIB]).decode()
    assert "llama_internal_get_tensor_map[abi:cxx11](llama_context*)" in out


def test_reference_llama_api_symbols_present(lvk):
    # every llama_* function of the reference llama.h:68-163
    ref_api = ["llama_context_default_params", "llama_mmap_supported", "llama_mlock_supported", "llama_init_from_file",
               "llama_free", "llama_model_quantize", "llama_get_kv_cache", "llama_get_kv_cache_size",
               "llama_get_kv_cache_token_count", "llama_set_kv_cache", "llama_eval", "llama_tokenize", "llama_n_vocab",
               "llama_n_ctx", "llama_n_embd", "llama_get_logits", "llama_get_embeddings", "llama_token_to_str",
               "llama_token_bos", "llama_token_eos", "llama_sample_top_p_top_k", "llama_print_timings",
               "llama_reset_timings", "llama_print_system_info"]
    for s in ref_api:
        assert hasattr(lvk.lib, s), s


def test_default_params_match_reference(lvk):
    p = lvk.lib.llama_context_default_params()   # llama.cpp:702-718
    assert (p.n_ctx, p.n_parts, p.seed) == (512, -1, 0)
    assert (p.f16_kv, p.logits_all, p.vocab_only, p.use_mmap, p.use_mlock, p.embedding) == \
           (False, False, False, True, False, False)
    assert C.sizeof(lvk.llama_context_params) == 40
    assert lvk.lib.llama_token_bos() == 1 and lvk.lib.llama_token_eos() == 2


def test_tokenizer_matches_reference(lvk, tiny_models):
    m = lvk.Llama(tiny_models["tiny_q4_0"], vocab_only=True)
    assert m.n_vocab == 32000
    for case in json.load(open(os.path.join(GOLD, "tokenizer_cases.json"))):
        got = m.tokenize(case["text"], add_bos=case["bos"]).tolist()
        assert got == case["ids"], case["text"]
    assert m.token_to_str(10994) == b"Hello"
    assert m.token_to_str(40000) is None
    m.close()


def test_init_failure_returns_null(lvk, tmp_path):
    bad = tmp_path / "bad.bin"
    bad.write_bytes(b"not a model at all")
    p = lvk.lib.llama_context_default_params()
    p.progress_callback = lvk.PROGRESS_CB(lambda a, b: None)
    assert not lvk.lib.llama_init_from_file(str(bad).encode(), p)
    assert not lvk.lib.llama_init_from_file(str(tmp_path / "missing.bin").encode(), p)


def _f32_model(path, rng):
    """tiny f32 ggjt model for the quantize tool (n_embd 256, 32 layers)"""
    import struct
    vocab = open(os.path.join(GOLD, "vocab32000.bin"), "rb").read()
    E, F, V, L = 256, 768, 32000, 32
    out = bytearray(struct.pack("<II7I", 0x67676a74, 1, V, E, 256, 2, L, 128, 0)) + vocab

    def tensor(name, shape, data):
        nonlocal out
        out += struct.pack("<III", len(shape), len(name), 0) + struct.pack("<%dI" % len(shape), *shape) + name.encode()
        out += b"\0" * ((32 - len(out) % 32) % 32)
        out += data.astype(np.float32).tobytes()
    tensor("tok_embeddings.weight", (E, V), rng.standard_normal((V, E)) * 0.02)
    tensor("norm.weight", (E,), 1 + 0.1 * rng.standard_normal(E))
    tensor("output.weight", (E, V), rng.standard_normal((V, E)) * 0.05)
    for i in range(L):
        p = "layers.%d." % i
        tensor(p + "attention_norm.weight", (E,), 1 + 0.1 * rng.standard_normal(E))
        for w in ("wq", "wk", "wv", "wo"):
            tensor(p + "attention.%s.weight" % w, (E, E), rng.standard_normal((E, E)) * 0.05)
        tensor(p + "ffn_norm.weight", (E,), 1 + 0.1 * rng.standard_normal(E))
        tensor(p + "feed_forward.w1.weight", (E, F), rng.standard_normal((F, E)) * 0.05)
        tensor(p + "feed_forward.w2.weight", (F, E), rng.standard_normal((E, F)) * 0.03)
        tensor(p + "feed_forward.w3.weight", (E, F), rng.standard_normal((F, E)) * 0.05)
    open(path, "wb").write(bytes(out))


@pytest.mark.parametrize("itype", [2, 3])
def test_quantize_tool_matches_reference(lvk, ref, tmp_path, itype):
    src = str(tmp_path / "f32.bin")
    _f32_model(src, np.random.default_rng(itype))
    a, b = str(tmp_path / "ours.bin"), str(tmp_path / "ref.bin")
    assert lvk.lib.llama_model_quantize(src.encode(), a.encode(), itype) == 0
    ref.lib.llama_model_quantize.restype = C.c_int
    ref.lib.llama_model_quantize.argtypes = [C.c_char_p, C.c_char_p, C.c_int]
    assert ref.lib.llama_model_quantize(src.encode(), b.encode(), itype) == 0
    assert open(a, "rb").read() == open(b, "rb").read()


def test_logits_digest_c_abi_matches_numpy_twin(lvk):
    """lvk_logits_digest (the host twin of the chained decode's device digest, include/lvk_ops.h)
    equals lvk.logits_digest bit for bit, on rows with the special values a logits row can hold
    (+-0, +-inf, NaN, denormals), and is order- and bit-sensitive"""
    rng = np.random.RandomState(11)
    rows = [rng.standard_normal(32000).astype(np.float32) * 8,
            np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 3.4e38], np.float32),
            np.zeros(5, np.float32), np.ones(1, np.float32)]
    for row in rows:
        got = lvk.lib.lvk_logits_digest(np.ascontiguousarray(row), len(row))
        assert got == lvk.logits_digest(row)
    r = rows[0].copy()
    base = lvk.logits_digest(r)
    r[[5, 9]] = r[[9, 5]]
    assert lvk.logits_digest(r) != base                      # a swapped pair changes it
    r = rows[0].copy()
    r.view(np.uint32)[123] ^= 1                               # one ulp anywhere changes it
    assert lvk.lib.lvk_logits_digest(r, len(r)) != base
    assert lvk.lib.lvk_logits_digest(rows[0], 0) == 0         # empty row


def test_forced_tokens_are_seeded_non_repeating_ids():
    """the teacher-forced streams of the chained checks (tests/oracle_lib.forced_tokens)"""
    import oracle_lib
    a = oracle_lib.forced_tokens(496)
    assert len(set(a.tolist())) == 496 and a.min() >= 3 and a.max() < 32000
    assert np.array_equal(a, oracle_lib.forced_tokens(496))
    assert not np.array_equal(a, oracle_lib.forced_tokens(496, seed=6))
