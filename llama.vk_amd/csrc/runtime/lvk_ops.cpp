// lvk_ops.cpp -- operator-level C ABI (include/lvk_ops.h): each op runs the
// production kernel on host buffers so tests can pin it against the oracle.
#include <algorithm>
#include <immintrin.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../../../include/llama.h"
#include "../../../include/lvk_ops.h"
#include "lvk_split.h"

namespace {

struct Dev {
    std::vector<void *> ptrs;
    void * get(size_t n) {
        void * p = nullptr;
        LVK_HIP(hipMalloc(&p, n ? n : 16));
        ptrs.push_back(p);
        return p;
    }
    template <class T> T * up(const T * h, size_t n) {
        T * d = (T *) get(n * sizeof(T));
        LVK_HIP(hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
        return d;
    }
    ~Dev() { for (void * p : ptrs) (void) hipFree(p); }
};

int fail(const char * fn, const std::string & m) {
    fprintf(stderr, "%s: %s\n", fn, m.c_str());
    return -1;
}

size_t block_bytes(int type) { return type == lvk::Q4_0 ? 20 : 24; }

__attribute__((target("f16c"))) uint16_t h_f32_to_f16(float f) { return _cvtss_sh(f, 0); }

}  // namespace

extern "C" {

int lvk_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int lvk_set_device(int dev) { return hipSetDevice(dev) == hipSuccess ? 0 : -1; }

const char * lvk_version(void) { return "llama.vk_amd 0.1 (gfx950)"; }

int lvk_quantize_rows(int type, const float * x, int n, int k, void * y) {
    try {
        if (k % 32) return fail(__func__, "k must be a multiple of 32");
        Dev dv;
        const size_t nb = (size_t) k / 32;
        float * xd = dv.up(x, (size_t) n * k);
        lvk::ActQ q;
        q.nb = (int) nb;
        q.d = (float *) dv.get((size_t) n * nb * 4);
        q.m = (float *) dv.get((size_t) n * nb * 4);
        q.qs = (uint4 *) dv.get((size_t) n * nb * 16);
        LVK_HIP(lvk::launch_quantize_act(xd, n, k, type, q, nullptr));
        std::vector<float> d((size_t) n * nb), m((size_t) n * nb);
        std::vector<uint8_t> qs((size_t) n * nb * 16);
        LVK_HIP(hipMemcpy(d.data(), q.d, d.size() * 4, hipMemcpyDeviceToHost));
        LVK_HIP(hipMemcpy(m.data(), q.m, m.size() * 4, hipMemcpyDeviceToHost));
        LVK_HIP(hipMemcpy(qs.data(), q.qs, qs.size(), hipMemcpyDeviceToHost));
        uint8_t * out = (uint8_t *) y;
        const size_t bb = block_bytes(type);
        for (size_t i = 0; i < (size_t) n * nb; ++i) {
            std::memcpy(out + i * bb, &d[i], 4);
            if (type == lvk::Q4_1) std::memcpy(out + i * bb + 4, &m[i], 4);
            std::memcpy(out + i * bb + bb - 16, &qs[i * 16], 16);
        }
        return 0;
    } catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

static int mul_mat_impl(int type, const void * w, int m, int k, const float * g, const float * x, int n, float * y,
                        bool norm) {
    if (m % 8 || k % 256) return fail("lvk_mul_mat_q", "need m % 8 == 0 and k % 256 == 0");
    Dev dv;
    const size_t nb = (size_t) k / 32, bb = block_bytes(type);
    void * wd = dv.up((const uint8_t *) w, (size_t) m * nb * bb);
    lvk::QMatrix q;
    q.qtype = type; q.M = m; q.K = k;
    q.nib = (const uint4 *) dv.get(lvk::qimage_nib_bytes(m, k));
    q.scl = dv.get(lvk::qimage_scl_bytes(m, k, type));
    LVK_HIP(lvk::launch_repack(wd, type, m, k, (uint4 *) q.nib, (void *) q.scl, nullptr));
    lvk::StepParams sp{0, n, 0, 0};
    lvk::StepParams * spd = dv.up(&sp, 1);
    float * yd = (float *) dv.get((size_t) n * m * 4);
    lvk::MvLaunch L;
    L.w = q; L.sp = spd; L.n_tokens = n; L.y = yd;
    float * xd = dv.up(x, (size_t) n * k);
    if (type == lvk::Q4_1) {
        // Q4_1 kernels quantize the f32 input in their prologue
        L.x = xd;
        if (norm) L.g = dv.up(g, (size_t) k);
        const int pro = norm ? lvk::PRO_NORM : lvk::PRO_ACTF;
        // single column: the CU-balanced decode kernel (matvec_cu41.hip) where compiled in
        hipError_t e = hipErrorNotSupported;
        if (n == 1 && lvk::matvec_cu_supported(k, lvk::Q4_1)) e = lvk::launch_matvec_cu(L, pro, lvk::EPI_STORE, nullptr);
        if (e == hipErrorNotSupported) e = lvk::launch_matvec(L, pro, lvk::EPI_STORE, nullptr);
        LVK_HIP(e);
    } else if (n == 1 && lvk::matvec_cu_supported(k)) {
        // single column: the decode kernel (matvec_cu.hip), quantizing in its prologue
        L.x = xd;
        if (norm) L.g = dv.up(g, (size_t) k);
        LVK_HIP(lvk::launch_matvec_cu(L, norm ? lvk::PRO_NORM : lvk::PRO_ACTF, lvk::EPI_STORE, nullptr));
    } else if (norm) {
        L.x = xd;
        L.g = dv.up(g, (size_t) k);
        LVK_HIP(lvk::launch_matvec(L, lvk::PRO_NORM, lvk::EPI_STORE, nullptr));
    } else {
        lvk::ActQ a;
        a.nb = (int) nb;
        a.d = (float *) dv.get((size_t) n * nb * 4);
        a.m = (float *) dv.get((size_t) n * nb * 4);
        a.qs = (uint4 *) dv.get((size_t) n * nb * 16);
        LVK_HIP(lvk::launch_quantize_act(xd, n, k, type, a, nullptr));
        L.xq = a;
        LVK_HIP(lvk::launch_matvec(L, lvk::PRO_ACTQ, lvk::EPI_STORE, nullptr));
    }
    LVK_HIP(hipMemcpy(y, yd, (size_t) n * m * 4, hipMemcpyDeviceToHost));
    return 0;
}

int lvk_mul_mat_q(int type, const void * w, int m, int k, const float * x, int n, float * y) {
    try { return mul_mat_impl(type, w, m, k, nullptr, x, n, y, false); }
    catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

int lvk_mul_mat_q_norm(int type, const void * w, int m, int k, const float * g, const float * x, int n, float * y) {
    try { return mul_mat_impl(type, w, m, k, g, x, n, y, true); }
    catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

int lvk_mul_mat_q_mfma(int type, const void * w, int m, int k, const float * g, const float * x, int n, float * y) {
    try {
        if (type != lvk::Q4_0 && type != lvk::Q4_1) return fail(__func__, "Q4_0 / Q4_1 only");
        if (m % 128 || k % 256 || n < 1) return fail(__func__, "need m % 128 == 0, k % 256 == 0, n >= 1");
        Dev dv;
        const size_t nb = (size_t) k / 32;
        void * wd = dv.up((const uint8_t *) w, (size_t) m * nb * (type == lvk::Q4_0 ? 20 : 24));
        lvk::QMatrix q;
        q.qtype = type; q.M = m; q.K = k;
        q.nib = (const uint4 *) dv.get(lvk::qimage_nib_bytes(m, k));
        q.scl = dv.get(lvk::qimage_scl_bytes(m, k, type));
        LVK_HIP(lvk::launch_repack(wd, type, m, k, (uint4 *) q.nib, (void *) q.scl, nullptr));
        if (type == lvk::Q4_1) {            // the Q4_1 path always runs on its f16 + side images
            q.a16 = dv.get(lvk::mm_a16_bytes(m, k));
            q.side = dv.get(lvk::mm41_side_bytes(m, k));
            LVK_HIP(lvk::launch_build_mm41(q, (void *) q.a16, (void *) q.side, nullptr));
        } else if (lvk::prompt_a16_env()) {  // the f16 A-fragment variant, as the model loader builds it
            q.a16 = dv.get(lvk::mm_a16_bytes(m, k));
            LVK_HIP(lvk::launch_build_a16(q, (void *) q.a16, nullptr));
        }
        float * xd = dv.up(x, (size_t) n * k);
        const float * gd = g ? dv.up(g, (size_t) k) : nullptr;
        void * xh = dv.get(lvk::mm_act_bytes(n, k));
        LVK_HIP(hipMemset(xh, 0, lvk::mm_act_bytes(n, k)));
        float * yd = (float *) dv.get((size_t) n * m * 4);
        if (type == lvk::Q4_1) {
            void * xs = dv.get(lvk::mm41_act_side_bytes(n, k));
            LVK_HIP(lvk::launch_act41_f16(xd, gd, n, k, xh, xs, nullptr));
            LVK_HIP(lvk::launch_mm_mfma41(q, xh, xs, n, yd, m, lvk::EPI_STORE, nullptr, nullptr));
        } else {
            float * da = (float *) dv.get((size_t) n * nb * 4);
            LVK_HIP(lvk::launch_act_f16(xd, gd, n, k, xh, da, nullptr));
            LVK_HIP(lvk::launch_mm_mfma(q, xh, da, n, yd, m, 0, lvk::EPI_STORE, nullptr, nullptr));
        }
        LVK_HIP(hipMemcpy(y, yd, (size_t) n * m * 4, hipMemcpyDeviceToHost));
        return 0;
    } catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

int lvk_attention_scores(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                         int n_ctx, int n_past, int n, float * out, float * scores_out);
int lvk_attention(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head, int n_ctx,
                  int n_past, int n, float * out) {
    return lvk_attention_scores(kc, vc, q, n_embd, n_head, n_ctx, n_past, n, out, nullptr);
}

static int attention_impl(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                          int n_ctx, int n_past, int n, float * out, float * scores_out, int kind);

int lvk_attention_scores(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                         int n_ctx, int n_past, int n, float * out, float * scores_out) {
    return attention_impl(kc, vc, q, n_embd, n_head, n_ctx, n_past, n, out, scores_out, 0);
}

int lvk_attention_prompt(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                         int n_ctx, int n_past, int n, float * out) {
    if (!lvk::attention_prompt_supported(n_embd, n_head, n_ctx))
        return fail(__func__, "needs head_dim 128, n_ctx % 32 == 0, n_ctx <= 1024");
    return attention_impl(kc, vc, q, n_embd, n_head, n_ctx, n_past, n, out, nullptr, 1);
}

int lvk_attention_decode(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                         int n_ctx, int n_past, float * out) {
    if (!lvk::attention_decode_supported(n_embd, n_head, n_ctx))
        return fail(__func__, "needs head_dim 128, n_ctx % 64 == 0, n_ctx <= 2048");
    return attention_impl(kc, vc, q, n_embd, n_head, n_ctx, n_past, 1, out, nullptr, 2);
}

static int attention_impl(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                          int n_ctx, int n_past, int n, float * out, float * scores_out, int kind) {
    const char * fn = kind == 1 ? "lvk_attention_prompt" : kind == 2 ? "lvk_attention_decode" : "lvk_attention";
    try {
        Dev dv;
        const size_t CE = (size_t) n_ctx * n_embd;
        std::vector<uint16_t> q16((size_t) n * n_embd);
        for (size_t i = 0; i < q16.size(); ++i) q16[i] = h_f32_to_f16(q[i]);   // ggml.c:6420-6433
        lvk::StepParams sp{n_past, n, 0, 0};
        lvk::AttnLaunch A{};
        A.q16 = dv.up(q16.data(), q16.size());
        A.kc = dv.up(kc, CE);
        A.vc = dv.up(vc, CE);
        A.scores = (float *) dv.get((size_t) n * n_head * n_ctx * 4);
        A.out.nb = n_embd / 32;
        A.out.d = (float *) dv.get((size_t) n * n_embd / 32 * 4);
        A.out.m = (float *) dv.get((size_t) n * n_embd / 32 * 4);
        A.out.qs = (uint4 *) dv.get((size_t) n * n_embd / 32 * 16);
        A.out_qtype = lvk::Q4_0;
        std::vector<uint16_t> te, ts;
        lvk::host_fp16_tables(te, ts);
        A.exp_tab = dv.up(te.data(), te.size());
        A.exp_computed = lvk::pick_exp_mode(A.exp_tab);
        A.sp = dv.up(&sp, 1);
        A.n_tokens = n; A.n_embd = n_embd; A.n_head = n_head; A.n_ctx = n_ctx;
        float * od = (float *) dv.get((size_t) n * n_embd * 4);
        A.out_f32 = od;
        uint16_t * pd = nullptr;
        if (scores_out) pd = (uint16_t *) dv.get((size_t) n * n_head * n_ctx * 2);
        A.p16_out = pd;
        if (kind == 1) LVK_HIP(lvk::launch_attention_prompt(A, (uint16_t *) A.scores, nullptr, nullptr, nullptr));
        else if (kind == 2) {
            void * gran = dv.get(lvk::attention_decode_scratch_bytes(n_head, n_ctx));
            LVK_HIP(hipMemset(gran, 0, lvk::attention_decode_scratch_bytes(n_head, n_ctx)));
            LVK_HIP(lvk::launch_attention_decode(A, gran, 1, nullptr));
        }
        else LVK_HIP(lvk::launch_attention(A, nullptr));
        LVK_HIP(hipMemcpy(out, od, (size_t) n * n_embd * 4, hipMemcpyDeviceToHost));
        if (scores_out) {
            LVK_HIP(hipMemcpy(scores_out, A.scores, (size_t) n * n_head * n_ctx * 4, hipMemcpyDeviceToHost));
            // debug: the f16 probabilities overwrite the second half of scores_out's bytes? no -- appended
            LVK_HIP(hipMemcpy(scores_out + (size_t) n * n_head * n_ctx, pd, (size_t) n * n_head * n_ctx * 2,
                              hipMemcpyDeviceToHost));
        }
        return 0;
    } catch (const lvk::Error & e) { return fail(fn, e.msg); }
}

int lvk_exp_table_mismatches(void) {
    try {
        Dev dv;
        std::vector<uint16_t> te, ts;
        lvk::host_fp16_tables(te, ts);
        const uint16_t * tab = dv.up(te.data(), te.size());
        int * bad_d = (int *) dv.get(2 * sizeof(int));
        int bad[2] = {-1, -1};
        LVK_HIP(lvk::exp_check(tab, bad_d, nullptr));
        LVK_HIP(hipMemcpy(bad, bad_d, sizeof(bad), hipMemcpyDeviceToHost));
        return bad[1] == 0 ? 0 : bad[0];     // the computed exp a context would use (f32, else double)
    } catch (const std::exception & e) {
        return fail("lvk_exp_table_mismatches", e.what());
    }
}

int lvk_rms_norm_mul(const float * x, const float * g, int k, int n, float * y) {
    try {
        Dev dv;
        float * xd = dv.up(x, (size_t) n * k);
        float * gd = dv.up(g, (size_t) k);
        float * yd = (float *) dv.get((size_t) n * k * 4);
        LVK_HIP(lvk::launch_rmsnorm_rows(xd, gd, k, n, yd, nullptr));
        LVK_HIP(hipMemcpy(y, yd, (size_t) n * k * 4, hipMemcpyDeviceToHost));
        return 0;
    } catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

void lvk_host_tables(uint16_t * exp_tab, uint16_t * silu_tab) {
    std::vector<uint16_t> te, ts;
    lvk::host_fp16_tables(te, ts);
    std::memcpy(exp_tab, te.data(), 65536 * 2);
    std::memcpy(silu_tab, ts.data(), 65536 * 2);
}

// settings and profiles of a layer-split context cover every stage
void lvk_set_profiling(struct llama_context * ctx, int on) {
    for (lvk::Context * c : ctx->stages()) c->profiling = on != 0;
}
void lvk_reset_profile(struct llama_context * ctx) {
    for (lvk::Context * c : ctx->stages()) c->prof = lvk::Profile{};
}
int lvk_get_profile(struct llama_context * ctx, double * ms, long * launches, double * bytes, int n) {
    for (int i = 0; i < n && i < lvk::K_NCLASS; ++i) {
        ms[i] = 0;
        launches[i] = 0;
        bytes[i] = 0;
        for (lvk::Context * c : ctx->stages()) {
            ms[i] += c->prof.ms[i];
            launches[i] += c->prof.launches[i];
            bytes[i] += c->prof.bytes[i];
        }
    }
    return lvk::K_NCLASS;
}
size_t lvk_weight_bytes(struct llama_context * ctx) {
    size_t b = 0;
    for (lvk::Context * c : ctx->stages()) b += c->model.weight_bytes;
    return b;
}
size_t lvk_prompt_image_bytes(struct llama_context * ctx) {
    size_t b = 0;
    for (lvk::Context * c : ctx->stages()) b += c->model.prompt_image_bytes;
    return b;
}
void lvk_set_graph(struct llama_context * ctx, int on) {
    for (lvk::Context * c : ctx->stages()) c->use_graph = on != 0;
}
void lvk_set_prompt_exact(struct llama_context * ctx, int on) {
    for (lvk::Context * c : ctx->stages()) c->prompt_exact = on != 0;
}

int lvk_kv_copy(struct llama_context * dst, struct llama_context * src, int n_tokens) {
    try {
        if (!dst || !src || dst == src) throw lvk::Error("need two distinct contexts");
        if (dst->split || src->split) throw lvk::Error("layer-split contexts copy KV state through llama_get_kv_cache");
        dst->c.kv_copy_from(src->c, n_tokens);
        return 0;
    } catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

int lvk_argmax(const float * x, int n) {
    try {
        if (n <= 0) throw lvk::Error("n must be positive");
        Dev dv;
        float * xd = dv.up(x, (size_t) n);
        int * od = (int *) dv.get(4);
        int r = -1;
        LVK_HIP(lvk::launch_argmax(xd, n, od, nullptr));
        LVK_HIP(hipMemcpy(&r, od, 4, hipMemcpyDeviceToHost));
        return r;
    } catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

int lvk_sample_candidates(const float * x, int n, const int * last, int n_last, int k, float temp, float rp,
                          float * vals, int * ids, int * flags) {
    try {
        if (n <= 0 || n > lvk::SAMPLE_MAX_VOCAB || k < 1 || k > std::min(n, lvk::SAMPLE_CAP) || temp <= 0 ||
            n_last < 0 || n_last > lvk::SAMPLE_MAX_LAST || (n_last > 0 && !last))
            throw lvk::Error("arguments out of range");
        Dev dv;
        float * xd = dv.up(x, (size_t) n);
        lvk::SampleParams p{};
        p.k = k;
        p.n_last = n_last;
        p.scale = 1.0f / temp;
        p.rp = rp;
        if (n_last > 0) std::memcpy(p.last, last, sizeof(int) * (size_t) n_last);
        auto * pd = (lvk::SampleParams *) dv.get(sizeof(p));
        LVK_HIP(hipMemcpy(pd, &p, sizeof(p), hipMemcpyHostToDevice));
        auto * od = (lvk::SampleOut *) dv.get(sizeof(lvk::SampleOut));
        LVK_HIP(lvk::launch_sample_cand(xd, n, pd, od, nullptr));
        lvk::SampleOut o;
        LVK_HIP(hipMemcpy(&o, od, sizeof(o), hipMemcpyDeviceToHost));
        const int m = std::min(o.count, lvk::SAMPLE_CAP);
        std::memcpy(vals, o.val, sizeof(float) * (size_t) m);
        std::memcpy(ids, o.id, sizeof(int) * (size_t) m);
        *flags = o.flags;
        return o.count;
    } catch (const lvk::Error & e) { return fail(__func__, e.msg); }
}

int lvk_eval_greedy(struct llama_context * ctx, int token, int n_past) {
    lvk::Context & c = ctx->c;
    const int64_t t0 = lvk::now_us();
    int r;
    try {
        if (ctx->split) {
            ctx->split->eval(&token, 1, n_past, true);
            r = *c.greedy_h;
        } else {
            r = c.eval_greedy(token, n_past);
        }
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: failed to eval: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    c.t_eval_us += lvk::now_us() - t0;   // counted as a decode eval (llama.cpp:1186-1195)
    c.n_eval++;
    return r;
}

int lvk_decode_chain(struct llama_context * ctx, const int * tokens, int n_tokens, int n_past, int n_steps,
                     int * out_tokens, uint64_t * out_digests) {
    if (!ctx || !tokens || !out_tokens) {
        fprintf(stderr, "%s: null argument\n", __func__);
        return -1;
    }
    if (ctx->split) {
        fprintf(stderr, "%s: not available on a layer split (use lvk_eval_greedy per step)\n", __func__);
        return -1;
    }
    lvk::Context & c = ctx->c;
    const int64_t t0 = lvk::now_us();
    try {
        c.decode_chain(tokens, n_tokens, n_past, n_steps, out_tokens, (unsigned long long *) out_digests);
    } catch (const lvk::Error & e) {
        fprintf(stderr, "%s: failed to eval: %s\n", __func__, e.msg.c_str());
        return -1;
    }
    c.t_eval_us += lvk::now_us() - t0;   // n_steps decode evals (llama.cpp:1186-1195)
    c.n_eval += n_steps;
    return 0;
}

int lvk_decode_greedy(struct llama_context * ctx, int token, int n_past, int n_steps, int * out_tokens) {
    return lvk_decode_chain(ctx, &token, 1, n_past, n_steps, out_tokens, nullptr);
}

uint64_t lvk_logits_digest(const float * x, int n) {
    uint64_t d = 0;
    for (int k = 0; k < n; ++k) {
        uint32_t bits;
        std::memcpy(&bits, x + k, 4);
        uint64_t z = ((uint64_t) k << 32 | bits) + 0x9E3779B97F4A7C15ull;   // splitmix64 finalizer
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        d += z ^ (z >> 31);
    }
    return d;
}

}  // extern "C"
