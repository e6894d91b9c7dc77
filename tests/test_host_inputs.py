"""Host code on caller-controlled bytes, without a GPU (also the body of the sanitizer run,
tests/test_host_sanitize.py): the ggjt loader (lvk_model.cpp; reference llama.cpp:360-560)
on truncated and corrupted model files, the tokenizer (llama_api.cpp; llama.cpp:1203-1350)
on arbitrary bytes, and the quantize tool (quantize.cpp; llama.cpp:1461-1577) on a truncated
input.  Every bad file must make llama_init_from_file return NULL / llama_model_quantize
return 1 -- never crash, hang or read outside the file."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def lvk():
    import lvk as m
    return m


def _params(lvk, vocab_only):
    p = lvk.lib.llama_context_default_params()
    p.vocab_only = vocab_only
    p.progress_callback = lvk.PROGRESS_CB(lambda a, b: None)
    return p


def _init(lvk, path, vocab_only=False):
    ctx = lvk.lib.llama_init_from_file(str(path).encode(), _params(lvk, vocab_only))
    if ctx:
        lvk.lib.llama_free(ctx)
    return bool(ctx)


def _layout(data):
    """offsets in a ggjt file: end of the 9 header words, end of the vocab, tensor records"""
    n_vocab = struct.unpack_from("<I", data, 8)[0]
    off = 36
    for _ in range(n_vocab):
        off += 4 + struct.unpack_from("<I", data, off)[0] + 4
    vocab_end = off
    tensors = []
    while off < len(data):
        nd, nl, ft = struct.unpack_from("<III", data, off)
        ne = struct.unpack_from("<%dI" % nd, data, off + 12)
        name_off = off + 12 + 4 * nd
        d = name_off + nl
        d += (32 - d % 32) % 32
        rows = ne[1] if nd > 1 else 1
        size = {0: 4 * ne[0], 1: 2 * ne[0], 2: ne[0] // 32 * 20, 3: ne[0] // 32 * 24}[ft] * rows
        tensors.append((off, name_off, d, size))
        off = d + size
    return vocab_end, tensors


@pytest.fixture(scope="module")
def small_file(tiny_models):
    return open(tiny_models["tiny_q4_0"], "rb").read()


def test_truncated_files_fail_cleanly(lvk, small_file, tmp_path):
    data = small_file
    vocab_end, tensors = _layout(data)
    cuts = [0, 3, 4, 7, 8, 20, 35, 36, 41, vocab_end // 2, vocab_end - 1, vocab_end, vocab_end + 5]
    for off, name_off, d, size in (tensors[0], tensors[1], tensors[len(tensors) // 2], tensors[-1]):
        cuts += [off + 2, name_off + 1, d, d + size // 2, d + size - 1]
    path = tmp_path / "cut.bin"
    for c in sorted(set(cuts)):
        path.write_bytes(data[:c])
        assert not _init(lvk, path), "a file cut at %d bytes loaded" % c
        # vocab_only reads the header and the vocab only
        assert _init(lvk, path, vocab_only=True) == (c >= vocab_end), c


def _patched(data, off, fmt, value):
    b = bytearray(data)
    struct.pack_into(fmt, b, off, value)
    return bytes(b)


def test_corrupt_headers_fail_cleanly(lvk, small_file, tmp_path):
    data = small_file
    vocab_end, tensors = _layout(data)
    t0, t1 = tensors[0], tensors[3]
    bad = {
        "magic": _patched(data, 0, "<I", 0x12345678),
        "version": _patched(data, 4, "<I", 7),
        "n_vocab_huge": _patched(data, 8, "<I", 0x7FFFFFFF),
        "n_embd_zero": _patched(data, 12, "<I", 0),
        "n_mult_zero": _patched(data, 16, "<I", 0),
        "n_head_zero": _patched(data, 20, "<I", 0),
        "n_layer_huge": _patched(data, 24, "<I", 100000),
        "ftype": _patched(data, 32, "<I", 99),
        "token_len_huge": _patched(data, 36, "<I", 0xFFFFFFF0),
        "tensor_ndims": _patched(data, t0[0], "<I", 7),
        "tensor_name_len": _patched(data, t0[0] + 4, "<I", 0xFFFFFF00),
        "tensor_type": _patched(data, t0[0] + 8, "<I", 42),
        "tensor_ne0_huge": _patched(data, t1[0] + 12, "<I", 0xFFFFFFE0),
        "tensor_ne1_huge": _patched(data, t1[0] + 16, "<I", 0xFFFFFFFF),
        "tensor_ne0_zero": _patched(data, t0[0] + 12, "<I", 0),
    }
    for name, b in bad.items():
        p = tmp_path / (name + ".bin")
        p.write_bytes(b)
        assert not _init(lvk, p), name


def test_random_header_corruption_never_crashes(lvk, small_file, tmp_path):
    """bytes flipped at random in the header, the vocab and the tensor records: the loader
    returns NULL or a context, and never reads outside the file (the sanitizer run's check)"""
    data = small_file
    vocab_end, tensors = _layout(data)
    recs = [range(o, d) for o, _, d, _ in tensors]
    rng = np.random.default_rng(7)
    p = tmp_path / "fz.bin"
    for i in range(60):
        b = bytearray(data)
        for _ in range(int(rng.integers(1, 6))):
            if i % 3 == 0:
                pos = int(rng.integers(0, 36))
            elif i % 3 == 1:
                pos = int(rng.integers(36, vocab_end))
            else:
                r = recs[int(rng.integers(0, len(recs)))]
                pos = int(rng.integers(r.start, r.stop))
            b[pos] = int(rng.integers(0, 256))
        p.write_bytes(bytes(b))
        _init(lvk, p)
        _init(lvk, p, vocab_only=True)


def test_tokenizer_on_arbitrary_bytes(lvk, tiny_models):
    m = lvk.Llama(tiny_models["tiny_q4_0"], vocab_only=True)
    rng = np.random.default_rng(3)
    texts = [b"", b"\xff\xfe\xfd", b"\xe2\x82", "héllo wörld ✓ 日本語".encode(), b"\x00abc" * 3,
             bytes(rng.integers(1, 256, 4096, dtype=np.uint8))]
    for t in texts:
        out = np.zeros(8192, np.int32)
        n = lvk.lib.llama_tokenize(m.ctx, t.split(b"\x00")[0], out, 8192, True)
        assert 0 <= n <= 8192
        # too small an output array: the reference returns -(needed)
        if n > 2:
            k = lvk.lib.llama_tokenize(m.ctx, t.split(b"\x00")[0], out, 1, True)
            assert k == -n
    for i in (-1, 32000, 1 << 30):
        assert lvk.lib.llama_token_to_str(m.ctx, i) is None
    m.close()


def test_quantize_truncated_input_fails(lvk, tmp_path):
    from test_abi import _f32_model
    src = tmp_path / "f32.bin"
    _f32_model(str(src), np.random.default_rng(1))
    data = src.read_bytes()
    for cut in (0, 10, 36, 200000, len(data) - 7):
        p = tmp_path / "t.bin"
        p.write_bytes(data[:cut])
        assert lvk.lib.llama_model_quantize(str(p).encode(), str(tmp_path / "o.bin").encode(), 2) == 1, cut
