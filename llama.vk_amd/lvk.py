"""Python host mirror of the llama.vk_amd C ABI (include/llama.h, include/lvk_ops.h).

A thin ctypes layer over lib/libllama_vk_amd.so, mirroring the reference
llama.h surface (same function names and argument meaning) for tests and
bench.py.  There is no fallback: if the shared library is missing or fails to
load, importing this module raises.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# LVK_LIB selects another build of the same library (the fault-injection probe build, tests only)
LIB_PATH = os.environ.get("LVK_LIB") or os.path.join(HERE, "lib", "libllama_vk_amd.so")
GEN_BIN = os.path.join(HERE, "bin", "lvk-gen-model")

# One HIP runtime per process: torch bundles its own libamdhip64 / libhsa-runtime64 /
# librccl (ROCm 7.0, NEEDED as "libamdhip64.so"), this library links /opt/rocm's
# (SONAME libamdhip64.so.7).  In one process the two either bind this library to torch's
# runtime (torch imported first) or load both runtimes side by side (this library first),
# which ended a round-2 test process in a glibc double free (profiles/r03_runtime_mix.md).
# Keep torch in other processes (bench.py and the tests do); LVK_ALLOW_TORCH=1 overrides.
if "torch" in __import__("sys").modules and os.environ.get("LVK_ALLOW_TORCH") != "1":
    raise ImportError("llama.vk_amd: torch is already imported in this process; its bundled HIP runtime "
                      "conflicts with this library's (run lvk in a process without torch, or set LVK_ALLOW_TORCH=1)")
if not os.path.exists(LIB_PATH):
    raise ImportError("llama.vk_amd: %s not built (run __graft_entry__.build() or make -C llama.vk_amd)" % LIB_PATH)
lib = C.CDLL(LIB_PATH)

f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
u16p = np.ctypeslib.ndpointer(np.uint16, flags="C_CONTIGUOUS")
u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")

PROGRESS_CB = C.CFUNCTYPE(None, C.c_float, C.c_void_p)


class llama_context_params(C.Structure):
    """reference llama.h:49-66, field for field"""
    _fields_ = [
        ("n_ctx", C.c_int),
        ("n_parts", C.c_int),
        ("seed", C.c_int),
        ("f16_kv", C.c_bool),
        ("logits_all", C.c_bool),
        ("vocab_only", C.c_bool),
        ("use_mmap", C.c_bool),
        ("use_mlock", C.c_bool),
        ("embedding", C.c_bool),
        ("progress_callback", PROGRESS_CB),
        ("progress_callback_user_data", C.c_void_p),
    ]


def _sig(name, res, args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = args
    return fn


# llama.h
_sig("llama_context_default_params", llama_context_params, [])
_sig("llama_mmap_supported", C.c_bool, [])
_sig("llama_mlock_supported", C.c_bool, [])
_sig("llama_init_from_file", C.c_void_p, [C.c_char_p, llama_context_params])
_sig("llama_free", None, [C.c_void_p])
_sig("llama_model_quantize", C.c_int, [C.c_char_p, C.c_char_p, C.c_int])
_sig("llama_get_kv_cache", C.POINTER(C.c_uint8), [C.c_void_p])
_sig("llama_get_kv_cache_size", C.c_size_t, [C.c_void_p])
_sig("llama_get_kv_cache_token_count", C.c_int, [C.c_void_p])
_sig("llama_set_kv_cache", None, [C.c_void_p, u8p, C.c_size_t, C.c_int])
_sig("llama_eval", C.c_int, [C.c_void_p, i32p, C.c_int, C.c_int, C.c_int])
_sig("llama_tokenize", C.c_int, [C.c_void_p, C.c_char_p, i32p, C.c_int, C.c_bool])
_sig("llama_n_vocab", C.c_int, [C.c_void_p])
_sig("llama_n_ctx", C.c_int, [C.c_void_p])
_sig("llama_n_embd", C.c_int, [C.c_void_p])
_sig("llama_get_logits", C.POINTER(C.c_float), [C.c_void_p])
_sig("llama_get_embeddings", C.POINTER(C.c_float), [C.c_void_p])
_sig("llama_token_to_str", C.c_char_p, [C.c_void_p, C.c_int])
_sig("llama_token_bos", C.c_int, [])
_sig("llama_token_eos", C.c_int, [])
_sig("lvk_eval_sample", C.c_int, [C.c_void_p, C.c_int, C.c_int, i32p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float])
_sig("llama_sample_top_p_top_k", C.c_int, [C.c_void_p, i32p, C.c_int, C.c_int, C.c_float, C.c_float, C.c_float])
_sig("llama_print_timings", None, [C.c_void_p])
_sig("llama_reset_timings", None, [C.c_void_p])
_sig("llama_print_system_info", C.c_char_p, [])
# lvk_ops.h
_sig("lvk_device_count", C.c_int, [])
_sig("lvk_version", C.c_char_p, [])
_sig("lvk_set_device", C.c_int, [C.c_int])
_sig("lvk_quantize_rows", C.c_int, [C.c_int, f32p, C.c_int, C.c_int, u8p])
_sig("lvk_mul_mat_q", C.c_int, [C.c_int, u8p, C.c_int, C.c_int, f32p, C.c_int, f32p])
_sig("lvk_mul_mat_q_norm", C.c_int, [C.c_int, u8p, C.c_int, C.c_int, f32p, f32p, C.c_int, f32p])
_sig("lvk_mul_mat_q_mfma", C.c_int, [C.c_int, u8p, C.c_int, C.c_int, C.c_void_p, f32p, C.c_int, f32p])
_sig("lvk_attention", C.c_int, [u16p, u16p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p])
_sig("lvk_attention_prompt", C.c_int, [u16p, u16p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p])
_sig("lvk_attention_decode", C.c_int, [u16p, u16p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, f32p])
_sig("lvk_attention_scores", C.c_int, [u16p, u16p, f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, f32p, f32p])
_sig("lvk_rms_norm_mul", C.c_int, [f32p, f32p, C.c_int, C.c_int, f32p])
_sig("lvk_exp_table_mismatches", C.c_int, [])
_sig("lvk_host_tables", None, [u16p, u16p])
_sig("lvk_set_profiling", None, [C.c_void_p, C.c_int])
_sig("lvk_get_profile", C.c_int, [C.c_void_p, f64p, i64p, f64p, C.c_int])
_sig("lvk_reset_profile", None, [C.c_void_p])
_sig("lvk_weight_bytes", C.c_size_t, [C.c_void_p])
_sig("lvk_prompt_image_bytes", C.c_size_t, [C.c_void_p])
_sig("lvk_set_graph", None, [C.c_void_p, C.c_int])
_sig("lvk_set_prompt_exact", None, [C.c_void_p, C.c_int])
_sig("lvk_eval_greedy", C.c_int, [C.c_void_p, C.c_int, C.c_int])
_sig("lvk_decode_greedy", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p])
_sig("lvk_decode_chain", C.c_int, [C.c_void_p, i32p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p])
_sig("lvk_logits_digest", C.c_uint64, [f32p, C.c_int])
_sig("lvk_argmax", C.c_int, [f32p, C.c_int])
_sig("lvk_sample_candidates", C.c_int, [f32p, C.c_int, i32p, C.c_int, C.c_int, C.c_float, C.c_float, f32p, i32p, C.POINTER(C.c_int)])
_sig("lvk_kv_copy", C.c_int, [C.c_void_p, C.c_void_p, C.c_int])
_sig("lvk_init_stage", C.c_void_p, [C.c_char_p, llama_context_params, C.c_int, C.c_int])
_sig("lvk_stage_eval", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int])
_sig("lvk_stage_get_x", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int])
_sig("lvk_stage_set_x", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int])
_sig("lvk_stage_layers", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int)])
_sig("lvk_rccl_unique_id", C.c_int, [C.c_void_p, C.c_size_t])
_sig("lvk_stage_connect", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int])
_sig("lvk_stage_connect_shm", C.c_int, [C.c_void_p, C.c_char_p, C.c_int, C.c_int])
_sig("lvk_stage_step", C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int])
_sig("lvk_stage_link_probe", C.c_int, [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double)])
_sig("lvk_init_split", C.c_void_p, [C.c_char_p, llama_context_params, C.c_int, i32p, C.c_char_p, C.c_int])
_sig("lvk_split_info", C.c_int, [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)])

BLOCK_BYTES = {2: 20, 3: 24}


def logits_digest(row):
    """lvk_logits_digest in numpy: sum (mod 2^64) over k of splitmix64((k << 32) | bits(row[k]))"""
    bits = np.ascontiguousarray(row, np.float32).view(np.uint32).astype(np.uint64)
    z = (np.arange(bits.size, dtype=np.uint64) << np.uint64(32)) | bits
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
        return int(np.sum(z, dtype=np.uint64))
KCLASS = ["embed", "qkv", "attention", "wo", "w13", "w2", "lm_head"]


def _check(rc, what):
    if rc != 0:
        raise RuntimeError("%s failed (rc=%d)" % (what, rc))


class Llama:
    """One llama_context (reference llama.h API, GPU forward pass)."""

    def __init__(self, path, n_ctx=512, seed=1, logits_all=False, embedding=False, vocab_only=False, f16_kv=True,
                 layers=None, split=None, transport=None, micro=64):
        """layers=(begin, end): a pipeline stage holding only those layers (lvk_init_stage);
        split=[dev0, dev1, ...]: the whole model layer-split over those HIP devices in this
        process (lvk_init_split; transport "rccl" / "copy" / None = rccl when distinct)"""
        p = lib.llama_context_default_params()
        p.n_ctx = n_ctx
        p.seed = seed
        p.f16_kv = f16_kv
        p.logits_all = logits_all
        p.embedding = embedding
        p.vocab_only = vocab_only
        self._cb = PROGRESS_CB(lambda prog, ud: None)
        p.progress_callback = self._cb
        if split is not None:
            d = np.ascontiguousarray(split, np.int32)
            self.ctx = lib.lvk_init_split(path.encode(), p, len(d), d, transport.encode() if transport else None,
                                          int(micro))
        elif layers is None:
            self.ctx = lib.llama_init_from_file(path.encode(), p)
        else:
            self.ctx = lib.lvk_init_stage(path.encode(), p, int(layers[0]), int(layers[1]))
        if not self.ctx:
            raise RuntimeError("llama_init_from_file failed for %s" % path)
        self.logits_all = logits_all
        self.n_vocab = lib.llama_n_vocab(self.ctx)
        self.n_embd = lib.llama_n_embd(self.ctx)
        self.n_ctx = lib.llama_n_ctx(self.ctx)
        self._last_n = 1

    def eval(self, tokens, n_past, n_threads=1, copy=True):
        """llama_eval; returns the logits rows (copy=False: a read-only view of the context's
        host buffer, valid until the next eval -- what a C caller of llama_get_logits holds)"""
        t = np.ascontiguousarray(tokens, np.int32)
        _check(lib.llama_eval(self.ctx, t, len(t), n_past, n_threads), "llama_eval")
        self._last_n = len(t)
        return self.logits(copy)

    def kv_cache_token_count(self):
        return lib.llama_get_kv_cache_token_count(self.ctx)

    def kv_copy_from(self, src, n_tokens):
        """take positions [0, n_tokens) of src's KV cache, device to device (lvk_kv_copy)"""
        _check(lib.lvk_kv_copy(self.ctx, src.ctx, int(n_tokens)), "lvk_kv_copy")

    def eval_greedy(self, token, n_past):
        """decode one token and pick the next greedily on the device (lvk_eval_greedy);
        host logits are not refreshed"""
        r = lib.lvk_eval_greedy(self.ctx, int(token), int(n_past))
        if r < 0:
            raise RuntimeError("lvk_eval_greedy failed")
        return r

    def decode_greedy(self, token, n_past, n_steps):
        """n_steps greedy decode steps on the device in one call (lvk_decode_greedy): the tokens
        n_steps chained eval_greedy calls would return, as an int32 array"""
        out = np.zeros(int(n_steps), np.int32)
        r = lib.lvk_decode_greedy(self.ctx, int(token), int(n_past), int(n_steps), out.ctypes.data)
        if r != 0:
            raise RuntimeError("lvk_decode_greedy failed")
        return out

    def decode_chain(self, tokens, n_past, n_steps=None, digests=True):
        """n_steps chained decode steps in one call (lvk_decode_chain): step i evaluates tokens[i]
        (teacher forcing) while i < len(tokens), then the previous step's argmax.  Returns the
        per-step argmax tokens (int32) and, with digests=True, the per-step logits digests
        (uint64, logits_digest of each step's logits row, computed on the device)."""
        t = np.ascontiguousarray(tokens, np.int32).reshape(-1)
        n_steps = len(t) if n_steps is None else int(n_steps)
        out = np.zeros(n_steps, np.int32)
        dg = np.zeros(n_steps, np.uint64) if digests else None
        r = lib.lvk_decode_chain(self.ctx, t, len(t), int(n_past), n_steps, out.ctypes.data,
                                 dg.ctypes.data if digests else None)
        if r != 0:
            raise RuntimeError("lvk_decode_chain failed")
        return (out, dg) if digests else out

    # ---- pipeline stage (lvk_init_stage contexts)
    def stage_eval(self, tokens, n_tokens, n_past):
        """first stage: tokens (int32 array); later stages: tokens=None, input set by set_x"""
        if tokens is None:
            _check(lib.lvk_stage_eval(self.ctx, None, n_tokens, n_past), "lvk_stage_eval")
        else:
            t = np.ascontiguousarray(tokens, np.int32)
            _check(lib.lvk_stage_eval(self.ctx, t.ctypes.data, len(t), n_past), "lvk_stage_eval")
        self._last_n = n_tokens

    def get_x(self, ptr, n_tokens, on_device):
        """residual stream [n_tokens][n_embd] f32 -> ptr (device pointer if on_device)"""
        _check(lib.lvk_stage_get_x(self.ctx, C.c_void_p(ptr), n_tokens, int(on_device)), "lvk_stage_get_x")

    def set_x(self, ptr, n_tokens, on_device):
        _check(lib.lvk_stage_set_x(self.ctx, C.c_void_p(ptr), n_tokens, int(on_device)), "lvk_stage_set_x")

    def split_info(self):
        """(stages, rccl, micro) of a layer-split context; (1, False, 0) otherwise"""
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        lib.lvk_split_info(self.ctx, C.byref(a), C.byref(b), C.byref(c))
        return a.value, bool(b.value), c.value

    def stage_connect(self, uid, n_stages, stage):
        """join the RCCL communicator of a one-stage-per-process pipeline (lvk_stage_connect)"""
        buf = C.create_string_buffer(bytes(uid), 128)
        _check(lib.lvk_stage_connect(self.ctx, buf, int(n_stages), int(stage)), "lvk_stage_connect")

    def stage_connect_shm(self, name, n_stages, stage):
        """join a one-stage-per-process pipeline over a host shared-memory ring
        (lvk_stage_connect_shm): returns once every stage has opened `name`"""
        _check(lib.lvk_stage_connect_shm(self.ctx, name.encode(), int(n_stages), int(stage)), "lvk_stage_connect_shm")

    def stage_link_probe(self, nbytes, iters=64):
        """microseconds per hop of the connected stage link (lvk_stage_link_probe; every stage
        calls it)"""
        us = C.c_double(0.0)
        _check(lib.lvk_stage_link_probe(self.ctx, int(nbytes), int(iters), C.byref(us)), "lvk_stage_link_probe")
        return us.value

    def stage_step(self, tokens, n_tokens, n_past, greedy=False, micro=64):
        """recv inpL -> this stage's layers -> send (lvk_stage_step); the greedy token on the
        first/last stage when greedy"""
        t = None if tokens is None else np.ascontiguousarray(tokens, np.int32)
        r = lib.lvk_stage_step(self.ctx, None if t is None else t.ctypes.data, int(n_tokens), int(n_past),
                               int(greedy), int(micro))
        if r < 0:
            raise RuntimeError("lvk_stage_step failed")
        self._last_n = n_tokens
        return r

    def stage_layers(self):
        b, e = C.c_int(), C.c_int()
        n = lib.lvk_stage_layers(self.ctx, C.byref(b), C.byref(e))
        return b.value, e.value, n

    def logits(self, copy=True):
        rows = self._last_n if self.logits_all else 1
        ptr = lib.llama_get_logits(self.ctx)
        v = np.ctypeslib.as_array(ptr, shape=(rows * self.n_vocab,)).reshape(rows, self.n_vocab)
        if copy:
            return v.copy()
        v.flags.writeable = False
        return v

    def embeddings(self):
        return np.ctypeslib.as_array(lib.llama_get_embeddings(self.ctx), shape=(self.n_embd,)).copy()

    def tokenize(self, text, add_bos=True):
        buf = np.zeros(len(text.encode()) + 8, np.int32)
        n = lib.llama_tokenize(self.ctx, text.encode(), buf, len(buf), add_bos)
        if n < 0:
            raise RuntimeError("llama_tokenize: too many tokens")
        return buf[:n].copy()

    def token_to_str(self, tok):
        return lib.llama_token_to_str(self.ctx, tok)

    def eval_sample(self, token, n_past, last_tokens, top_k=40, top_p=0.95, temp=0.8, repeat_penalty=1.1):
        """lvk_eval_sample: one decode step + the sampler with its O(n_vocab) part on the GPU"""
        lt = np.ascontiguousarray(last_tokens, dtype=np.int32)
        r = lib.lvk_eval_sample(self.ctx, int(token), int(n_past), lt, len(lt), top_k, top_p, temp, repeat_penalty)
        if r < 0:
            raise RuntimeError("lvk_eval_sample failed")
        return r

    def sample(self, last_tokens, top_k=40, top_p=0.95, temp=0.8, repeat_penalty=1.1):
        lt = np.ascontiguousarray(last_tokens, np.int32)
        return lib.llama_sample_top_p_top_k(self.ctx, lt, len(lt), top_k, top_p, temp, repeat_penalty)

    def kv_cache(self):
        n = lib.llama_get_kv_cache_size(self.ctx)
        return np.ctypeslib.as_array(lib.llama_get_kv_cache(self.ctx), shape=(n,)).copy()

    def set_kv_cache(self, buf, n_tokens):
        buf = np.ascontiguousarray(buf, np.uint8)
        lib.llama_set_kv_cache(self.ctx, buf, buf.size, n_tokens)

    def set_profiling(self, on):
        lib.lvk_set_profiling(self.ctx, int(on))

    def set_graph(self, on):
        lib.lvk_set_graph(self.ctx, int(on))

    def set_prompt_exact(self, on):
        """prompt batches on the bit-faithful VALU path (True) or the MFMA path (False, default)"""
        lib.lvk_set_prompt_exact(self.ctx, int(on))

    def reset_profile(self):
        lib.lvk_reset_profile(self.ctx)

    def profile(self):
        k = len(KCLASS)
        ms = np.zeros(k, np.float64)
        la = np.zeros(k, np.int64)
        by = np.zeros(k, np.float64)
        n = min(k, lib.lvk_get_profile(self.ctx, ms, la, by, k))
        return {KCLASS[i]: {"ms": float(ms[i]), "launches": int(la[i]), "bytes": float(by[i])} for i in range(n)}

    def weight_bytes(self):
        return int(lib.lvk_weight_bytes(self.ctx))

    def prompt_image_bytes(self):
        return int(lib.lvk_prompt_image_bytes(self.ctx))

    def print_timings(self):
        lib.llama_print_timings(self.ctx)

    def close(self):
        if getattr(self, "ctx", None):
            lib.llama_free(self.ctx)
            self.ctx = None

    __del__ = close


# ---------------------------------------------------------------- operator level
def model_hparams(path):
    """ggjt/ggmf/ggml header hparams (n_vocab, n_embd, n_mult, n_head, n_layer, n_rot, ftype); llama.cpp:328-350"""
    import struct
    with open(path, "rb") as f:
        head = f.read(40)
    magic = struct.unpack("<I", head[:4])[0]
    off = 4 if magic == 0x67676d6c else 8      # 'ggml' has no version field
    return dict(zip(("n_vocab", "n_embd", "n_mult", "n_head", "n_layer", "n_rot", "ftype"),
                    struct.unpack("<7I", head[off:off + 28])))


def quantize_rows(x, qtype):
    x = np.ascontiguousarray(x, np.float32)
    n, k = x.shape
    y = np.zeros(n * (k // 32) * BLOCK_BYTES[qtype], np.uint8)
    _check(lib.lvk_quantize_rows(qtype, x, n, k, y), "lvk_quantize_rows")
    return y.reshape(n, -1)


def mul_mat_q(qtype, w_rows, m, k, x):
    x = np.ascontiguousarray(x, np.float32)
    n = x.shape[0]
    y = np.zeros(n * m, np.float32)
    _check(lib.lvk_mul_mat_q(qtype, np.ascontiguousarray(w_rows, np.uint8).ravel(), m, k, x, n, y), "lvk_mul_mat_q")
    return y.reshape(n, m)


def mul_mat_q_norm(qtype, w_rows, m, k, g, x):
    x = np.ascontiguousarray(x, np.float32)
    n = x.shape[0]
    y = np.zeros(n * m, np.float32)
    _check(lib.lvk_mul_mat_q_norm(qtype, np.ascontiguousarray(w_rows, np.uint8).ravel(), m, k,
                                  np.ascontiguousarray(g, np.float32), x, n, y), "lvk_mul_mat_q_norm")
    return y.reshape(n, m)


def mul_mat_q_mfma(qtype, w_rows, m, k, x, g=None):
    """the MFMA prompt matmul (lvk_mul_mat_q_mfma); g: optional RMSNorm weight"""
    x = np.ascontiguousarray(x, np.float32)
    n = x.shape[0]
    y = np.zeros(n * m, np.float32)
    gp = None
    if g is not None:
        g = np.ascontiguousarray(g, np.float32)
        gp = g.ctypes.data_as(C.c_void_p)
    _check(lib.lvk_mul_mat_q_mfma(qtype, np.ascontiguousarray(w_rows, np.uint8).ravel(), m, k, gp, x, n, y),
           "lvk_mul_mat_q_mfma")
    return y.reshape(n, m)


def attention_prompt(kc, vc, q, n_embd, n_head, n_ctx, n_past, n):
    """the prompt-batch attention kernels (lvk_attention_prompt)"""
    out = np.zeros(n * n_embd, np.float32)
    _check(lib.lvk_attention_prompt(kc, vc, np.ascontiguousarray(q, np.float32), n_embd, n_head, n_ctx, n_past, n, out),
           "lvk_attention_prompt")
    return out


def attention_decode(kc, vc, q, n_embd, n_head, n_ctx, n_past):
    """the single-token attention kernels (lvk_attention_decode)"""
    out = np.zeros(n_embd, np.float32)
    _check(lib.lvk_attention_decode(kc, vc, np.ascontiguousarray(q, np.float32), n_embd, n_head, n_ctx, n_past, out),
           "lvk_attention_decode")
    return out


def attention(kc, vc, q, n_embd, n_head, n_ctx, n_past, n):
    out = np.zeros(n * n_embd, np.float32)
    _check(lib.lvk_attention(np.ascontiguousarray(kc, np.uint16), np.ascontiguousarray(vc, np.uint16),
                             np.ascontiguousarray(q, np.float32).ravel(), n_embd, n_head, n_ctx, n_past, n, out),
           "lvk_attention")
    return out


def attention_scores(kc, vc, q, n_embd, n_head, n_ctx, n_past, n):
    out = np.zeros(n * n_embd, np.float32)
    m = n * n_head * n_ctx
    sc = np.zeros(m + (m + 1) // 2, np.float32)
    _check(lib.lvk_attention_scores(np.ascontiguousarray(kc, np.uint16), np.ascontiguousarray(vc, np.uint16),
                                    np.ascontiguousarray(q, np.float32).ravel(), n_embd, n_head, n_ctx, n_past, n,
                                    out, sc), "lvk_attention_scores")
    p16 = sc[m:].view(np.uint16)[:m].reshape(n, n_head, n_ctx)
    return out, sc[:m].reshape(n, n_head, n_ctx), p16


def exp_table_mismatches():
    """Arguments h <= 0 where the device's computed exp differs from table_exp_f16."""
    return int(lib.lvk_exp_table_mismatches())


def argmax(x):
    """device greedy argmax (first strict maximum; 0 when x[0] is NaN)"""
    x = np.ascontiguousarray(x, np.float32).ravel()
    r = lib.lvk_argmax(x, x.size)
    if r < 0:
        raise RuntimeError("lvk_argmax failed")
    return r


class _QuantizeFns(C.Structure):      # quantize_fns_t (include/ggml.h, reference ggml.h:808-813)
    _fields_ = [("dequantize_row_q", C.c_void_p), ("quantize_row_q", C.c_void_p),
                ("quantize_row_q_reference", C.c_void_p), ("vec_dot_q", C.c_void_p)]


_DEQ_T = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int)
_Q_T = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p, C.c_int)
_DOT_T = C.CFUNCTYPE(None, C.c_int, C.POINTER(C.c_float), C.c_void_p, C.c_void_p)
_sig("ggml_internal_get_quantize_fn", _QuantizeFns, [C.c_size_t])


class QuantizeFns:
    """ggml_internal_get_quantize_fn(ggml_type) as Python callables (numpy in and out)"""

    def __init__(self, ggml_type):
        t = lib.ggml_internal_get_quantize_fn(ggml_type)
        self.valid = bool(t.vec_dot_q)
        self.bb = 20 if ggml_type == 0 else 24
        if self.valid:
            self._deq = _DEQ_T(t.dequantize_row_q)
            self._q = _Q_T(t.quantize_row_q)
            self._qr = _Q_T(t.quantize_row_q_reference)
            self._dot = _DOT_T(t.vec_dot_q)

    def quantize_row(self, x, reference=False):
        x = np.ascontiguousarray(x, np.float32)
        y = np.zeros(x.size // 32 * self.bb, np.uint8)
        (self._qr if reference else self._q)(x.ctypes.data, y.ctypes.data, x.size)
        return y

    def dequantize_row(self, q, k):
        q = np.ascontiguousarray(q, np.uint8)
        y = np.zeros(k, np.float32)
        self._deq(q.ctypes.data, y.ctypes.data, k)
        return y

    def vec_dot(self, n, x, y):
        x = np.ascontiguousarray(x, np.uint8)
        y = np.ascontiguousarray(y, np.uint8)
        s = C.c_float(0.0)
        self._dot(n, C.byref(s), x.ctypes.data, y.ctypes.data)
        return s.value


def sample_candidates(x, last, k, temp, rp):
    """lvk_sample_candidates: (values, ids, flags) of the device top-k candidate selection"""
    x = np.ascontiguousarray(x, np.float32)
    last = np.ascontiguousarray(last, np.int32)
    vals = np.zeros(1024, np.float32)
    ids = np.zeros(1024, np.int32)
    fl = C.c_int(0)
    n = lib.lvk_sample_candidates(x, x.size, last, last.size, k, temp, rp, vals, ids, C.byref(fl))
    if n < 0:
        raise RuntimeError("lvk_sample_candidates failed")
    m = min(n, 1024)
    return vals[:m], ids[:m], fl.value, n


def rms_norm_mul(x, g):
    x = np.ascontiguousarray(x, np.float32)
    n, k = x.shape
    y = np.zeros_like(x)
    _check(lib.lvk_rms_norm_mul(x, np.ascontiguousarray(g, np.float32), k, n, y), "lvk_rms_norm_mul")
    return y


def host_tables():
    e = np.zeros(65536, np.uint16)
    s = np.zeros(65536, np.uint16)
    lib.lvk_host_tables(e, s)
    return e, s


def set_device(dev):
    _check(lib.lvk_set_device(dev), "lvk_set_device")


def device_count():
    return lib.lvk_device_count()


def gen_model(path, n_embd=4096, n_head=32, n_layer=32, ftype=2, seed=1, n_vocab=32000, n_mult=256, vocab=None):
    """Write a seeded synthetic ggjt model with the bundled generator."""
    import subprocess
    cmd = [GEN_BIN, path, "--n-embd", str(n_embd), "--n-head", str(n_head), "--n-layer", str(n_layer),
           "--ftype", str(ftype), "--seed", str(seed), "--n-vocab", str(n_vocab), "--n-mult", str(n_mult)]
    if vocab:
        cmd += ["--vocab", vocab]
    subprocess.check_call(cmd, stderr=subprocess.DEVNULL)
    return path


def rccl_unique_id():
    """a fresh RCCL communicator id (128 bytes) for lvk_stage_connect; rank 0 makes it"""
    buf = C.create_string_buffer(128)
    _check(lib.lvk_rccl_unique_id(buf, 128), "lvk_rccl_unique_id")
    return buf.raw
