"""ctypes bindings for the test-only CPU oracle and the reference build.

TEST INFRASTRUCTURE ONLY.  `Oracle` wraps oracle/liboracle.so (our scalar
restatement of the reference AVX2 arithmetic, oracle/lvk_oracle.c); `Ref`
wraps oracle/_ref/libref.so (the reference llama.cpp/ggml.c compiled from
/root/reference by oracle/Makefile).  Neither is ever used by the product.
"""
import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref.so")
GEN_BIN = os.path.join(ROOT, "llama.vk_amd", "bin", "lvk-gen-model")
VOCAB = os.path.join(ROOT, "tests", "golden", "vocab32000.bin")

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")

BLOCK_BYTES = {2: 20, 3: 24}


def _sig(lib, name, res, args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args
    return fn


class Oracle:
    def __init__(self, path=ORACLE_SO):
        L = self.lib = C.CDLL(path)
        _sig(L, "orc_init_tables", None, [])
        _sig(L, "orc_fp32_to_fp16", C.c_uint16, [C.c_float])
        _sig(L, "orc_table_exp_f16", C.POINTER(C.c_uint16), [])
        _sig(L, "orc_table_silu_f16", C.POINTER(C.c_uint16), [])
        for n in ("orc_quantize_row_q4_0", "orc_quantize_row_q4_1",
                  "orc_quantize_row_q4_0_reference", "orc_quantize_row_q4_1_reference"):
            _sig(L, n, None, [f32p, u8p, C.c_int])
        for n in ("orc_dequantize_row_q4_0", "orc_dequantize_row_q4_1"):
            _sig(L, n, None, [u8p, f32p, C.c_int])
        for n in ("orc_vec_dot_q4_0", "orc_vec_dot_q4_1", "orc_vec_dot_q4_0_blockorder"):
            _sig(L, n, C.c_float, [C.c_int, u8p, u8p])
        _sig(L, "orc_vec_dot_f16", C.c_float, [C.c_int, u16p, u16p])
        _sig(L, "orc_rms_norm", None, [f32p, C.c_int, C.c_int, f32p])
        _sig(L, "orc_rope", None, [f32p, C.c_int, C.c_int, C.c_int, C.c_int, f32p])
        _sig(L, "orc_silu", None, [f32p, C.c_int, f32p])
        _sig(L, "orc_softmax_row", None, [f32p, C.c_int])
        _sig(L, "orc_attention", None, [u16p, u16p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p])
        _sig(L, "orc_model_load", C.c_void_p, [C.c_char_p, C.c_int])
        _sig(L, "orc_model_free", None, [C.c_void_p])
        _sig(L, "orc_n_vocab", C.c_int, [C.c_void_p])
        _sig(L, "orc_n_embd", C.c_int, [C.c_void_p])
        _sig(L, "orc_eval", C.c_int, [C.c_void_p, i32p, C.c_int, C.c_int, C.c_int, f32p])
        _sig(L, "orc_kv_k", C.POINTER(C.c_uint16), [C.c_void_p, C.c_int])
        _sig(L, "orc_kv_v", C.POINTER(C.c_uint16), [C.c_void_p, C.c_int])
        _sig(L, "orc_set_threads", None, [C.c_int])
        L.orc_init_tables()

    def table_exp(self):
        return np.ctypeslib.as_array(self.lib.orc_table_exp_f16(), shape=(65536,)).copy()

    def table_silu(self):
        return np.ctypeslib.as_array(self.lib.orc_table_silu_f16(), shape=(65536,)).copy()

    def quantize(self, x, qtype, reference=False):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 32 * BLOCK_BYTES[qtype], np.uint8)
        n = "orc_quantize_row_q4_%d%s" % (qtype - 2, "_reference" if reference else "")
        getattr(self.lib, n)(x, y, x.size)
        return y

    def dequantize(self, q, qtype, k):
        y = np.zeros(k, np.float32)
        getattr(self.lib, "orc_dequantize_row_q4_%d" % (qtype - 2))(np.ascontiguousarray(q, np.uint8), y, k)
        return y

    def vec_dot(self, qtype, k, x, y):
        return getattr(self.lib, "orc_vec_dot_q4_%d" % (qtype - 2))(k, x, y)

    def model(self, path, n_ctx=512):
        return OracleModel(self, path, n_ctx)


class OracleModel:
    def __init__(self, orc, path, n_ctx):
        self.orc = orc
        self.h = orc.lib.orc_model_load(path.encode(), n_ctx)
        if not self.h:
            raise RuntimeError("oracle failed to load %s" % path)
        self.n_vocab = orc.lib.orc_n_vocab(self.h)
        self.n_embd = orc.lib.orc_n_embd(self.h)
        self.n_ctx = n_ctx

    def eval(self, tokens, n_past, logits_all=False):
        t = np.ascontiguousarray(tokens, np.int32)
        out = np.zeros((len(t) if logits_all else 1) * self.n_vocab, np.float32)
        rc = self.orc.lib.orc_eval(self.h, t, len(t), n_past, int(logits_all), out)
        if rc != 0:
            raise RuntimeError("oracle eval failed")
        return out.reshape(-1, self.n_vocab)

    def kv(self, il):
        n = self.n_ctx * self.n_embd
        k = np.ctypeslib.as_array(self.orc.lib.orc_kv_k(self.h, il), shape=(n,)).copy()
        v = np.ctypeslib.as_array(self.orc.lib.orc_kv_v(self.h, il), shape=(n,)).copy()
        return k, v

    def close(self):
        if self.h:
            self.orc.lib.orc_model_free(self.h)
            self.h = None

    __del__ = close


class Ref:
    def __init__(self, path=REF_SO):
        L = self.lib = C.CDLL(path)
        _sig(L, "ref_open", C.c_void_p, [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int])
        _sig(L, "ref_close", None, [C.c_void_p])
        _sig(L, "ref_eval", C.c_int, [C.c_void_p, i32p, C.c_int, C.c_int, C.c_int])
        _sig(L, "ref_get_logits", None, [C.c_void_p, f32p, C.c_int])
        _sig(L, "ref_n_vocab", C.c_int, [C.c_void_p])
        _sig(L, "ref_sample", C.c_int, [C.c_void_p, i32p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float])
        _sig(L, "ref_tokenize", C.c_int, [C.c_void_p, C.c_char_p, i32p, C.c_int, C.c_int])
        _sig(L, "ref_quantize_row", None, [C.c_int, f32p, u8p, C.c_int])
        _sig(L, "ref_quantize_row_reference", None, [C.c_int, f32p, u8p, C.c_int])
        _sig(L, "ref_dequantize_row", None, [C.c_int, u8p, f32p, C.c_int])
        _sig(L, "ref_vec_dot", C.c_float, [C.c_int, C.c_int, u8p, u8p])
        _sig(L, "ref_rms_norm", None, [f32p, C.c_int, C.c_int, f32p])
        _sig(L, "ref_rope", None, [f32p, C.c_int, C.c_int, C.c_int, C.c_int, f32p])
        _sig(L, "ref_silu", None, [f32p, C.c_int, f32p])
        _sig(L, "ref_attention", None, [u16p, u16p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p])

    def quantize(self, x, qtype, reference=False):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 32 * BLOCK_BYTES[qtype], np.uint8)
        (self.lib.ref_quantize_row_reference if reference else self.lib.ref_quantize_row)(qtype, x, y, x.size)
        return y

    def dequantize(self, q, qtype, k):
        y = np.zeros(k, np.float32)
        self.lib.ref_dequantize_row(qtype, np.ascontiguousarray(q, np.uint8), y, k)
        return y

    def vec_dot(self, qtype, k, x, y):
        return self.lib.ref_vec_dot(qtype, k, x, y)

    def model(self, path, n_ctx=512, logits_all=False, f16_kv=True):
        return RefModel(self, path, n_ctx, logits_all, f16_kv)


class RefModel:
    def __init__(self, ref, path, n_ctx, logits_all, f16_kv=True):
        self.ref = ref
        self.logits_all = logits_all
        self.h = ref.lib.ref_open(path.encode(), n_ctx, int(f16_kv), int(logits_all), 1)
        if not self.h:
            raise RuntimeError("reference failed to load %s" % path)
        self.n_vocab = ref.lib.ref_n_vocab(self.h)

    def eval(self, tokens, n_past, n_threads=8):
        t = np.ascontiguousarray(tokens, np.int32)
        rc = self.ref.lib.ref_eval(self.h, t, len(t), n_past, n_threads)
        if rc != 0:
            raise RuntimeError("reference eval failed")
        rows = len(t) if self.logits_all else 1
        out = np.zeros(rows * self.n_vocab, np.float32)
        self.ref.lib.ref_get_logits(self.h, out, out.size)
        return out.reshape(rows, self.n_vocab)

    def sample(self, last_tokens, top_k, top_p, temp, repeat_penalty):
        """llama_sample_top_p_top_k of the reference build (llama.cpp:1777-1805)"""
        t = np.ascontiguousarray(last_tokens, np.int32)
        return self.ref.lib.ref_sample(self.h, t, len(t), top_k, top_p, temp, repeat_penalty)

    def close(self):
        if self.h:
            self.ref.lib.ref_close(self.h)
            self.h = None

    __del__ = close


def gen_model(path, n_embd=256, n_head=2, n_layer=32, ftype=2, seed=1, n_vocab=32000, n_mult=256):
    import subprocess
    if os.path.exists(path):
        return path
    subprocess.check_call([GEN_BIN, path, "--n-embd", str(n_embd), "--n-head", str(n_head),
                           "--n-layer", str(n_layer), "--ftype", str(ftype), "--seed", str(seed),
                           "--n-vocab", str(n_vocab), "--n-mult", str(n_mult), "--vocab", VOCAB],
                          stderr=subprocess.DEVNULL)
    return path


def prompt_tokens(n, start=1):
    """SURVEY.md C3 prompt: [1] + [100 + (i*7919) % 31000 ...]"""
    return np.array([start] + [100 + (i * 7919) % 31000 for i in range(1, n)], np.int32)


def forced_tokens(n, seed=5):
    """a seeded, non-repeating teacher-forced token sequence (ids 3..31999): decode steps fed these
    read a KV cache whose rows all differ, unlike the greedy stream of a synthetic model, which
    settles on one token"""
    return np.random.RandomState(seed).permutation(np.arange(3, 32000, dtype=np.int32))[:n].astype(np.int32)
