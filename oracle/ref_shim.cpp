// oracle/ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A thin, plain-argument C shim over the *reference* llama.cpp/ggml.c build
// (compiled from /root/reference by oracle/Makefile into oracle/_ref/).  It
// exists so the Python tests and bench.py's cpu_baseline leg can drive the
// reference through ctypes without mirroring llama_context_params by value.
//
// Nothing in the product (llama.vk_amd/) links or loads this file.
//
// Reference interfaces used (all unmodified):
//   llama.h:74-76   llama_init_from_file
//   llama.h:108-113 llama_eval
//   llama.h:133     llama_get_logits
//   ggml.h:803-814  ggml_internal_get_quantize_fn (op-level codec access)
#include "llama.h"
#include "ggml.h"

#include <cstdint>
#include <cstring>
#include <cmath>

extern "C" {

// Open a model with the context parameters the survey's dumplogits harness
// uses: n_ctx, f16 KV, optional logits_all.
void * ref_open(const char * path, int n_ctx, int f16_kv, int logits_all, int seed) {
    llama_context_params p = llama_context_default_params();
    p.n_ctx = n_ctx;
    p.f16_kv = f16_kv != 0;
    p.logits_all = logits_all != 0;
    p.seed = seed;
    p.use_mmap = true;
    p.progress_callback = [](float, void *) {};
    return llama_init_from_file(path, p);
}

void ref_close(void * ctx) { llama_free((llama_context *) ctx); }

int ref_eval(void * ctx, const int * toks, int n, int n_past, int n_threads) {
    return llama_eval((llama_context *) ctx, toks, n, n_past, n_threads);
}

// copy n floats of the logits buffer (last row, or all rows with logits_all)
void ref_get_logits(void * ctx, float * out, int n) {
    std::memcpy(out, llama_get_logits((llama_context *) ctx), sizeof(float) * (size_t) n);
}

int ref_n_vocab(void * ctx) { return llama_n_vocab((llama_context *) ctx); }

int ref_tokenize(void * ctx, const char * text, int * out, int n_max, int add_bos) {
    return llama_tokenize((llama_context *) ctx, text, out, n_max, add_bos != 0);
}

int ref_sample(void * ctx, const int * last, int n_last, int top_k, float top_p, float temp, float rp) {
    return llama_sample_top_p_top_k((llama_context *) ctx, last, n_last, top_k, top_p, temp, rp);
}

// Op-level access to the reference codecs.  `type` is the ggjt file ftype
// (2 = Q4_0, 3 = Q4_1, llama.cpp:387-395), mapped to enum ggml_type (ggml.h:199-208).
static size_t ggml_type_of(int ftype) { return ftype == 2 ? GGML_TYPE_Q4_0 : GGML_TYPE_Q4_1; }
void ref_quantize_row(int type, const float * x, void * y, int k) {
    ggml_internal_get_quantize_fn(ggml_type_of(type)).quantize_row_q(x, y, k);
}
void ref_quantize_row_reference(int type, const float * x, void * y, int k) {
    ggml_internal_get_quantize_fn(ggml_type_of(type)).quantize_row_q_reference(x, y, k);
}
void ref_dequantize_row(int type, const void * x, float * y, int k) {
    ggml_internal_get_quantize_fn(ggml_type_of(type)).dequantize_row_q(x, y, k);
}
float ref_vec_dot(int type, int n, const void * x, const void * y) {
    float s = 0.0f;
    ggml_internal_get_quantize_fn(ggml_type_of(type)).vec_dot_q(n, &s, x, y);
    return s;
}
size_t ref_quantize_file_q4_0(const float * src, void * dst, int n, int k, int64_t * hist) {
    return ggml_quantize_q4_0(src, dst, n, k, hist);
}
size_t ref_quantize_file_q4_1(const float * src, void * dst, int n, int k, int64_t * hist) {
    return ggml_quantize_q4_1(src, dst, n, k, hist);
}

} // extern "C"

// ---------------------------------------------------------------------------
// Graph-level op shims: each builds the same ggml sub-graph llama_eval_internal
// builds (llama.cpp:981-1061) on caller data and runs it single-threaded, so
// tests can pin individual restated ops against the reference arithmetic.
// ---------------------------------------------------------------------------
#include <vector>

namespace {
struct RefCtx {
    std::vector<uint8_t> buf;
    ggml_context * ctx;
    explicit RefCtx(size_t bytes) : buf(bytes) {
        ggml_init_params ip = { bytes, buf.data(), false };
        ctx = ggml_init(ip);
    }
    ~RefCtx() { ggml_free(ctx); }
    void run(ggml_tensor * out) {
        ggml_cgraph gf = ggml_build_forward(out);
        gf.n_threads = 1;
        ggml_graph_compute(ctx, &gf);
    }
};
}

extern "C" {

// y[N][K] = rms_norm(x[N][K])  (llama.cpp:981, ggml.c:6024-6080)
void ref_rms_norm(const float * x, int K, int N, float * y) {
    RefCtx r(64u << 20);
    ggml_tensor * t = ggml_new_tensor_2d(r.ctx, GGML_TYPE_F32, K, N);
    std::memcpy(t->data, x, sizeof(float) * (size_t) K * N);
    ggml_tensor * o = ggml_rms_norm(r.ctx, t);
    r.run(o);
    std::memcpy(y, o->data, sizeof(float) * (size_t) K * N);
}

// y = rope(x) with x viewed as [head_dim, n_head, N] (llama.cpp:992, mode 0)
void ref_rope(const float * x, int head_dim, int n_head, int N, int n_past, float * y) {
    RefCtx r(64u << 20);
    ggml_tensor * t = ggml_new_tensor_3d(r.ctx, GGML_TYPE_F32, head_dim, n_head, N);
    std::memcpy(t->data, x, sizeof(float) * (size_t) head_dim * n_head * N);
    ggml_tensor * o = ggml_rope(r.ctx, t, n_past, head_dim, 0);
    r.run(o);
    std::memcpy(y, o->data, sizeof(float) * (size_t) head_dim * n_head * N);
}

// y = silu(x) (GGML_SILU_FP16 table path, ggml.c:2495-2503)
void ref_silu(const float * x, int n, float * y) {
    RefCtx r(16u << 20);
    ggml_tensor * t = ggml_new_tensor_1d(r.ctx, GGML_TYPE_F32, n);
    std::memcpy(t->data, x, sizeof(float) * (size_t) n);
    ggml_tensor * o = ggml_silu(r.ctx, t);
    r.run(o);
    std::memcpy(y, o->data, sizeof(float) * (size_t) n);
}

// Self-attention block of one layer exactly as llama.cpp:1010-1061 builds it,
// on a f16 KV cache of one layer: kc [n_ctx][n_embd], vc [n_embd][n_ctx].
// q: rope'd query rows [N][n_embd] f32.  out: [N][n_embd] f32 (KQV merged).
void ref_attention(const uint16_t * kc, const uint16_t * vc, const float * q,
                   int n_embd, int n_head, int n_ctx, int n_past, int N, float * out) {
    const int hd = n_embd / n_head;
    const int n_kv = n_past + N;
    RefCtx r((size_t) 256u << 20);
    ggml_tensor * kbuf = ggml_new_tensor_1d(r.ctx, GGML_TYPE_F16, (int64_t) n_ctx * n_embd);
    ggml_tensor * vbuf = ggml_new_tensor_1d(r.ctx, GGML_TYPE_F16, (int64_t) n_ctx * n_embd);
    std::memcpy(kbuf->data, kc, 2u * (size_t) n_ctx * n_embd);
    std::memcpy(vbuf->data, vc, 2u * (size_t) n_ctx * n_embd);
    ggml_tensor * Qcur = ggml_new_tensor_3d(r.ctx, GGML_TYPE_F32, hd, n_head, N);
    std::memcpy(Qcur->data, q, sizeof(float) * (size_t) n_embd * N);
    ggml_tensor * Q = ggml_permute(r.ctx, Qcur, 0, 2, 1, 3);
    ggml_tensor * K = ggml_permute(r.ctx,
        ggml_reshape_3d(r.ctx, ggml_view_1d(r.ctx, kbuf, (int64_t) n_kv * n_embd, 0), hd, n_head, n_kv),
        0, 2, 1, 3);
    ggml_tensor * KQ = ggml_mul_mat(r.ctx, K, Q);
    ggml_tensor * KQs = ggml_scale(r.ctx, KQ, ggml_new_f32(r.ctx, 1.0f / sqrtf(float(n_embd) / n_head)));
    ggml_tensor * KQm = ggml_diag_mask_inf(r.ctx, KQs, n_past);
    ggml_tensor * KQsm = ggml_soft_max(r.ctx, KQm);
    ggml_tensor * V = ggml_view_3d(r.ctx, vbuf, n_kv, hd, n_head,
                                   (size_t) n_ctx * 2, (size_t) n_ctx * 2 * hd, 0);
    ggml_tensor * KQV = ggml_mul_mat(r.ctx, V, KQsm);
    ggml_tensor * merged = ggml_permute(r.ctx, KQV, 0, 2, 1, 3);
    ggml_tensor * o = ggml_cpy(r.ctx, merged, ggml_new_tensor_2d(r.ctx, GGML_TYPE_F32, n_embd, N));
    r.run(o);
    std::memcpy(out, o->data, sizeof(float) * (size_t) n_embd * N);
}

} // extern "C"
