// lvk_context.cpp -- llama_eval on one HIP stream.
//
// The reference builds a ~1253-node ggml graph per token and runs it on a CPU
// thread pool (llama.cpp:927-1137, ggml.c:9230-9651).  Here the same forward
// pass is 5 fused kernels per layer (+ embedding and lm_head) on one stream:
//   QKV matvec  (rms_norm*g -> Q4 quantize -> Wq|Wk|Wv -> RoPE -> KV append)
//   attention   (scores; softmax -> P.V -> Q4 quantize of the merged heads)
//   Wo matvec   (+ residual)
//   W1|W3 matvec(rms_norm*g -> quantize -> silu(w1x)*w3x -> Q4 quantize)
//   W2 matvec   (+ residual)
// Single-token decode is captured once into a hipGraph; the position and the
// token come from a 16-byte step block copied to HBM before each replay, so
// the same graph serves every n_past.
#include "lvk_context.h"

#include <immintrin.h>

#include <cmath>
#include <cstring>

#include "../../../include/llama.h"

namespace lvk {

int64_t now_us() {
    return std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

namespace {
// host F16C conversion, identical to the reference's GGML_FP32_TO_FP16 (ggml.c:183)
__attribute__((target("f16c"))) uint16_t h_f32_to_f16(float f) { return _cvtss_sh(f, 0); }
__attribute__((target("f16c"))) float h_f16_to_f32(uint16_t h) { return _cvtsh_ss(h); }
}  // namespace

void host_fp16_tables(std::vector<uint16_t> & te, std::vector<uint16_t> & ts) {
    te.resize(65536);
    ts.resize(65536);
    for (int i = 0; i < 65536; ++i) {
        const float f = h_f16_to_f32((uint16_t) i);
        ts[i] = h_f32_to_f16(f / (1.0f + expf(-f)));
        te[i] = h_f32_to_f16(expf(f));
    }
}

// the softmax may compute exp instead of reading the table, but only in a mode
// that reproduces this host's table on every argument it can see: 2 (device
// expf) if exact, else 1 (double exp) if exact, else 0 (table).  LVK_EXP_TABLE
// forces the table.
int pick_exp_mode(const uint16_t * exp_tab_d) {
    if (getenv("LVK_EXP_TABLE")) return 0;
    int * bad_d = nullptr;
    LVK_HIP(hipMalloc((void **) &bad_d, 2 * sizeof(int)));
    int bad[2] = {-1, -1};
    const hipError_t e1 = exp_check(exp_tab_d, bad_d, nullptr);
    const hipError_t e2 = e1 == hipSuccess ? hipMemcpy(bad, bad_d, sizeof(bad), hipMemcpyDeviceToHost) : e1;
    (void) hipFree(bad_d);
    LVK_HIP(e2);
    return bad[1] == 0 ? 2 : bad[0] == 0 ? 1 : 0;
}

Context::~Context() {
    if (graph_exec) (void) hipGraphExecDestroy(graph_exec);
    if (graph) (void) hipGraphDestroy(graph);
    if (graph_greedy_exec) (void) hipGraphExecDestroy(graph_greedy_exec);
    if (graph_greedy) (void) hipGraphDestroy(graph_greedy);
    if (graph_sample_exec) (void) hipGraphExecDestroy(graph_sample_exec);
    if (graph_sample) (void) hipGraphDestroy(graph_sample);
    if (graph_chain_exec) (void) hipGraphExecDestroy(graph_chain_exec);
    if (graph_chain) (void) hipGraphDestroy(graph_chain);
    if (chain_h) (void) hipHostFree(chain_h);
    if (chain_ctl_h) (void) hipHostFree(chain_ctl_h);
    if (forced_h) (void) hipHostFree(forced_h);
    if (digest_h) (void) hipHostFree(digest_h);
    if (samp_h) (void) hipHostFree(samp_h);
    if (sout_h) (void) hipHostFree(sout_h);
    if (greedy_h) (void) hipHostFree(greedy_h);
    for (auto & e : ev_pool) { (void) hipEventDestroy(e.first); (void) hipEventDestroy(e.second); }
    if (sp_h) (void) hipHostFree(sp_h);
    if (tok_h) (void) hipHostFree(tok_h);
    if (err_h) (void) hipHostFree(err_h);
    if (stream) (void) hipStreamDestroy(stream);
}

void Context::init(const llama_context_params & p) {
    // the caller's window (llama.h accepts any positive n_ctx); buffers and kernels use it
    // rounded up to the 32-position attention tile, at least 128 (positions past the
    // caller's window are never written or read)
    if (p.n_ctx <= 0) throw Error("llama.vk_amd: n_ctx must be positive");
    n_ctx_user = p.n_ctx;
    n_ctx = std::max(128, (p.n_ctx + 31) / 32 * 32);
    logits_all = p.logits_all;
    want_embedding = p.embedding;
    const HParams & hp = model.hp;
    const size_t E = hp.n_embd, L = model.layers.size(), V = hp.n_vocab, H = hp.n_head, F = hp.n_ff();
    const size_t hd = E / H, C = (size_t) n_ctx;
    // KV cache element type (llama.cpp:1614): f16, or f32 when the caller asks for it
    kv32 = !p.f16_kv;
    const size_t es = kv_elem_bytes();
    kc = (uint16_t *) model.alloc(L * C * E * es);
    vc = (uint16_t *) model.alloc(L * C * E * es);
    LVK_HIP(hipMemset(kc, 0, L * C * E * es));
    LVK_HIP(hipMemset(vc, 0, L * C * E * es));
    x = (float *) model.alloc(C * E * 4);
    q16 = (uint16_t *) model.alloc(C * E * es);      // queries in the KV element type
    scores = (float *) model.alloc(C * H * C * 4);
    aq_attn.nb = (int) (E / 32);
    aq_attn.d = (float *) model.alloc(C * (E / 32) * 4);
    aq_attn.m = (float *) model.alloc(C * (E / 32) * 4);
    aq_attn.qs = (uint4 *) model.alloc(C * (E / 32) * 16);
    aq_ffn.nb = (int) (F / 32);
    aq_ffn.d = (float *) model.alloc(C * (F / 32) * 4);
    aq_ffn.m = (float *) model.alloc(C * (F / 32) * 4);
    aq_ffn.qs = (uint4 *) model.alloc(C * (F / 32) * 16);
    u_ffn = (float *) model.alloc(F * 4);
    {
        const size_t Cp = (C + 63) / 64 * 64, KX = std::max(E, F);
        xh = (uint16_t *) model.alloc(mm_act_bytes((int) Cp, (int) KX));
        LVK_HIP(hipMemset(xh, 0, mm_act_bytes((int) Cp, (int) KX)));   // masked slots stay zero
        xda = (float *) model.alloc(Cp * (KX / 32) * 4);
        if (model.qtype == Q4_1) xside = model.alloc(mm41_act_side_bytes((int) Cp, (int) KX));
        const char * sq = getenv("LVK_MM_SWIGLU_Q");
        if (model.qtype == Q4_0 && (!sq || atoi(sq) != 0)) {
            xh2 = (uint16_t *) model.alloc(mm_act_bytes((int) Cp, (int) F));
            LVK_HIP(hipMemset(xh2, 0, mm_act_bytes((int) Cp, (int) F)));   // masked slots stay zero
            xda2 = (float *) model.alloc(Cp * (F / 32) * 4);
        }
        qkv32 = (float *) model.alloc(C * 3 * E * 4);
        uf = (float *) model.alloc(C * F * 4);
        prompt_exact = getenv("LVK_PROMPT_EXACT") && atoi(getenv("LVK_PROMPT_EXACT")) != 0;
        old_attention = getenv("LVK_ATTN_V1") && atoi(getenv("LVK_ATTN_V1")) != 0;
        attn_gran = model.alloc(attention_decode_scratch_bytes((int) H, (int) C));
        LVK_HIP(hipMemset(attn_gran, 0, attention_decode_scratch_bytes((int) H, (int) C)));
        // granule tags (seq << 7) + layer + 1 stay unique per token with up to 126 layers
        seq_epochs = L <= 126;
        // test hook (tests/test_gpu_seq_wrap.py): start the step counter near its 25-bit wrap
        if (const char * e = getenv("LVK_SEQ_START")) seq = (unsigned) strtoul(e, nullptr, 0) & ((1u << 25) - 1);
    }
    logits_d = (float *) model.alloc(C * V * 4);
    emb_d = (float *) model.alloc(E * 4);
    sp_d = (StepParams *) model.alloc(sizeof(StepParams));
    tok_d = (int *) model.alloc(C * 4);
    LVK_HIP(hipHostMalloc((void **) &sp_h, (1 + C) * sizeof(StepParams), hipHostMallocDefault));
    LVK_HIP(hipHostMalloc((void **) &tok_h, C * 4, hipHostMallocDefault));
    LVK_HIP(hipGetDevice(&device));
    LVK_HIP(hipHostMalloc((void **) &err_h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    *err_h = 0;
    LVK_HIP(hipHostGetDevicePointer((void **) &err_d, err_h, 0));
    greedy_d = (int *) model.alloc(4);
    chain_d = (int *) model.alloc((CHAIN_HDR + C) * 4);
    forced_d = (int *) model.alloc(C * 4);
    digest_d = (unsigned long long *) model.alloc(C * 8);
    LVK_HIP(hipHostMalloc((void **) &chain_h, C * 4, hipHostMallocDefault));
    LVK_HIP(hipHostMalloc((void **) &chain_ctl_h, CHAIN_HDR * 4, hipHostMallocDefault));
    LVK_HIP(hipHostMalloc((void **) &forced_h, C * 4, hipHostMallocDefault));
    LVK_HIP(hipHostMalloc((void **) &digest_h, C * 8, hipHostMallocDefault));
    // the device argmax also stores the token straight into host-mapped memory
    LVK_HIP(hipHostMalloc((void **) &greedy_h, 64, hipHostMallocMapped | hipHostMallocCoherent));
    LVK_HIP(hipHostGetDevicePointer((void **) &greedy_hd, greedy_h, 0));
    samp_d = (SampleParams *) model.alloc(sizeof(SampleParams));
    LVK_HIP(hipHostMalloc((void **) &samp_h, sizeof(SampleParams), hipHostMallocDefault));
    std::memset(samp_h, 0, sizeof(SampleParams));
    LVK_HIP(hipHostMalloc((void **) &sout_h, sizeof(SampleOut), hipHostMallocMapped | hipHostMallocCoherent));
    LVK_HIP(hipHostGetDevicePointer((void **) &sout_d, sout_h, 0));

    // fp16 exp / silu tables (ggml.c:2915-2927), built with this host's glibc
    std::vector<uint16_t> te, ts;
    host_fp16_tables(te, ts);
    exp_tab = (uint16_t *) model.alloc(65536 * 2);
    silu_tab = (uint16_t *) model.alloc(65536 * 2);
    LVK_HIP(hipMemcpy(exp_tab, te.data(), 65536 * 2, hipMemcpyHostToDevice));
    LVK_HIP(hipMemcpy(silu_tab, ts.data(), 65536 * 2, hipMemcpyHostToDevice));
    exp_computed = pick_exp_mode(exp_tab);
    // RoPE cos/sin table (ggml.c:7209-7213): theta = powf(10000, -i0/n_dims), angle = p*theta
    std::vector<float2> rt(C * (hd / 2));
    for (size_t pos = 0; pos < C; ++pos)
        for (size_t i0 = 0; i0 < hd; i0 += 2) {
            const float theta = powf(10000.0f, ((float) -(int) i0) / (float) hd);
            const float ang = (float) (int) pos * theta;
            rt[pos * (hd / 2) + i0 / 2] = make_float2(cosf(ang), sinf(ang));
        }
    rope = (float2 *) model.alloc(rt.size() * sizeof(float2));
    LVK_HIP(hipMemcpy(rope, rt.data(), rt.size() * sizeof(float2), hipMemcpyHostToDevice));

    LVK_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    logits.reserve(logits_all ? C * V : V);
    if (want_embedding) embedding.resize(E);
}

void Context::check_device_error() {
    const unsigned e = __atomic_load_n(err_h, __ATOMIC_ACQUIRE);
    if (e == LVK_ERR_NONE) return;
    __atomic_store_n(err_h, 0u, __ATOMIC_RELEASE);
    logits_valid = false;
    throw Error(e == LVK_ERR_ATTN_SPIN ? "llama.vk_amd: decode attention: a workgroup wait timed out (results discarded)"
                                       : "llama.vk_amd: a kernel wait timed out (results discarded)");
}

void Context::timed_launch(int cls, double bytes, const std::function<hipError_t()> & fn) {
    if (!profiling) {
        LVK_HIP(fn());
        return;
    }
    if (ev_used == ev_pool.size()) {
        hipEvent_t a, b;
        LVK_HIP(hipEventCreate(&a));
        LVK_HIP(hipEventCreate(&b));
        ev_pool.push_back({a, b});
        ev_class.push_back(0);
    }
    auto & e = ev_pool[ev_used];
    ev_class[ev_used] = cls;
    ++ev_used;
    g_launch_events = {e.first, e.second};
    const hipError_t err = fn();
    g_launch_events = {};
    LVK_HIP(err);
    prof.launches[cls] += 1;
    prof.bytes[cls] += bytes;
}

void Context::collect_profile() {
    for (size_t i = 0; i < ev_used; ++i) {
        float ms = 0.0f;
        LVK_HIP(hipEventElapsedTime(&ms, ev_pool[i].first, ev_pool[i].second));
        prof.ms[ev_class[i]] += ms;
    }
    ev_used = 0;
}

static double qbytes(const QMatrix & w) { return (double) w.M * (w.K / 32) * (w.qtype == Q4_0 ? 20 : 24); }

// decode kernels: the CU-balanced path (matvec_cu.hip) where its row length is
// compiled in, else the generic kernel
static hipError_t mv_launch(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.n_tokens == 1 && matvec_cu_supported(L.w.K, L.w.qtype)) {
        const hipError_t e = launch_matvec_cu(L, pro, epi, s);
        if (e != hipErrorNotSupported) return e;
    }
    return launch_matvec(L, pro, epi, s);
}

// prompt batches go through the MFMA matmuls when every matrix of the model fits them
bool Context::use_mfma(int n) const {
    // below 16 tokens the per-row VALU kernels win (the MFMA tile is 16 tokens wide)
    if (n < 16 || prompt_exact) return false;
    for (const Layer & ly : model.layers)
        if (!mm_mfma_supported(ly.wqkv) || !mm_mfma_supported(ly.wo) || !mm_mfma_supported(ly.w13) ||
            !mm_mfma_supported(ly.w2))
            return false;
    return true;
}

void Context::enqueue_forward(int n, bool last_only, const int * tok_src, int logit_row, bool head, bool embed) {
    const HParams & hp = model.hp;
    if (!tok_src) tok_src = tok_d;
    float * const logits_out = logits_d + (size_t) logit_row * hp.n_vocab;
    const int E = (int) hp.n_embd, H = (int) hp.n_head, hd = E / H, F = (int) hp.n_ff();
    if (use_mfma(n)) {
        // prompt batch on the matrix cores: per layer
        //   act(norm) -> QKV (store) -> RoPE + KV append -> attention -> act -> Wo (+x)
        //   act(norm) -> W1|W3 (silu * mul) -> act -> W2 (+x)
        // Q4_0: mm_mfma.hip (activation scales da); Q4_1: mm_mfma41.hip (side image xs)
        const bool q41 = model.qtype == Q4_1;
        auto act = [&](const float * xin, const float * g, int K) {
            return q41 ? launch_act41_f16(xin, g, n, K, xh, xside, stream) : launch_act_f16(xin, g, n, K, xh, xda, stream);
        };
        auto mm = [&](const QMatrix & w, float * y, int ldy, int epi, const uint16_t * st) {
            return q41 ? launch_mm_mfma41(w, xh, xside, n, y, ldy, epi, st, stream)
                       : launch_mm_mfma(w, xh, xda, n, y, ldy, 0, epi, st, stream);
        };
        if (model.has_embed)
            timed_launch(K_EMBED, 0, [&] { return launch_embed(model.tok_emb, model.emb_type, E, tok_src, n, x, stream); });
        for (size_t il = 0; il < model.layers.size(); ++il) {
            const Layer & ly = model.layers[il];
            uint16_t * kcl = kc_layer(il);
            uint16_t * vcl = vc_layer(il);
            timed_launch(K_QKV, 0, [&] { return act(x, ly.attn_norm, E); });
            if (!kv32 && mm_rope_fused) {
                // RoPE + KV append in the matmul's epilogue (the f32 rows never reach memory)
                const RopeKV rk{rope, sp_d, n_ctx, E, hd, q16, kcl, vcl};
                timed_launch(K_QKV, qbytes(ly.wqkv), [&] {
                    return q41 ? launch_mm_mfma41(ly.wqkv, xh, xside, n, nullptr, 0, EPI_ROPE_KV, nullptr, stream, &rk)
                               : launch_mm_qkv_rope(ly.wqkv, xh, xda, n, rk, stream);
                });
            } else {
                timed_launch(K_QKV, qbytes(ly.wqkv), [&] { return mm(ly.wqkv, qkv32, 3 * E, EPI_STORE, nullptr); });
                timed_launch(K_QKV, 0, [&] {
                    return launch_rope_kv(qkv32, n, E, hd, rope, sp_d, n_ctx, q16, kcl, vcl, stream, kv32);
                });
            }
            AttnLaunch at{q16, kcl, vcl, scores, aq_attn, model.qtype, exp_tab, sp_d, n, E, H, n_ctx};
            at.exp_computed = exp_computed;
            at.err = err_d;
            at.kv32 = kv32;
            if (!kv32 && attention_prompt_supported(E, H, n_ctx)) {
                // writes the Wo input in both forms (ActQ and the MFMA operand images)
                timed_launch(K_ATTN, 0, [&] {
                    return q41 ? launch_attention_prompt(at, (uint16_t *) scores, xh, nullptr, stream, xside)
                               : launch_attention_prompt(at, (uint16_t *) scores, xh, xda, stream);
                });
            } else {
                timed_launch(K_ATTN, 0, [&] { return launch_attention(at, stream); });
                timed_launch(K_WO, 0, [&] {
                    return q41 ? launch_actq41_to_f16(aq_attn, n, E, xh, xside, stream)
                               : launch_actq_to_f16(aq_attn, n, E, xh, xda, stream);
                });
            }
            timed_launch(K_WO, qbytes(ly.wo), [&] { return mm(ly.wo, x, E, EPI_RESID, nullptr); });
            timed_launch(K_W13, 0, [&] { return act(x, ly.ffn_norm, E); });
            if (!q41 && xh2) {
                // SwiGLU + the W2 input's quantization in the W1|W3 epilogue
                timed_launch(K_W13, qbytes(ly.w13), [&] {
                    return launch_mm_w13_q(ly.w13, xh, xda, n, silu_tab, xh2, xda2, stream);
                });
                timed_launch(K_W2, qbytes(ly.w2), [&] {
                    return launch_mm_mfma(ly.w2, xh2, xda2, n, x, E, 0, EPI_RESID, nullptr, stream);
                });
            } else {
                timed_launch(K_W13, qbytes(ly.w13), [&] { return mm(ly.w13, uf, F, EPI_SWIGLU_F32, silu_tab); });
                timed_launch(K_W2, 0, [&] { return act(uf, nullptr, F); });
                timed_launch(K_W2, qbytes(ly.w2), [&] { return mm(ly.w2, x, E, EPI_RESID, nullptr); });
            }
        }
        if (!model.has_head || !head) return;
        if (last_only || !mm_mfma_supported(model.output)) {
            MvLaunch o;
            o.w = model.output; o.x = x; o.g = model.norm; o.sp = sp_d; o.y = logits_out;
            o.tok0 = last_only ? n - 1 : 0;
            o.n_tokens = last_only ? 1 : n;
            timed_launch(K_LMHEAD, qbytes(model.output), [&] { return mv_launch(o, PRO_NORM, EPI_STORE, stream); });
        } else {
            timed_launch(K_LMHEAD, 0, [&] { return act(x, model.norm, E); });
            timed_launch(K_LMHEAD, qbytes(model.output), [&] {
                return mm(model.output, logits_out, (int) hp.n_vocab, EPI_STORE, nullptr);
            });
        }
        if (want_embedding)
            LVK_HIP(launch_rmsnorm_rows(x + (size_t) (n - 1) * E, model.norm, E, 1, emb_d, stream));
        return;
    }
    // single-token FFN: W1|W3 hands silu(w1 x)*(w3 x) to W2 in f32, W2 quantizes it
    const bool ffn_f32 = n == 1 && matvec_cu_supported(E, model.qtype) && matvec_cu_supported(F, model.qtype);
    const bool seq_ep = seq_epochs;
    if (n == 1 && !old_attention && attention_decode_supported(E, H, n_ctx) && !seq_ep)
        // the decode attention's score granules carry epoch = layer + 1: zero them once per token
        LVK_HIP(hipMemsetAsync(attn_gran, 0, attention_decode_scratch_bytes(H, n_ctx), stream));
    if (model.has_embed && embed)
        // a single-token eval takes its token from the step block (one H2D copy per token)
        timed_launch(K_EMBED, 0, [&] {
            return launch_embed(model.tok_emb, model.emb_type, E, n == 1 ? &sp_d->pad0 : tok_src, n, x, stream);
        });
    for (size_t il = 0; il < model.layers.size(); ++il) {
        const Layer & ly = model.layers[il];
        MvLaunch a;
        a.w = ly.wqkv; a.x = x; a.g = ly.attn_norm; a.sp = sp_d; a.n_tokens = n;
        a.q16 = q16; a.kc = kc_layer(il); a.vc = vc_layer(il); a.rope.cs = rope;
        a.n_embd = E; a.head_dim = hd; a.n_ctx = n_ctx; a.kv32 = kv32;
        AttnLaunch at{q16, kc_layer(il), vc_layer(il), scores, aq_attn, model.qtype, exp_tab, sp_d, n, E, H, n_ctx};
        at.exp_computed = exp_computed;
        at.err = err_d;
        at.kv32 = kv32;
        at.seq_epochs = seq_ep ? 1 : 0;
        timed_launch(K_QKV, qbytes(ly.wqkv), [&] { return mv_launch(a, PRO_NORM, EPI_QKV, stream); });
        if (n > 1 && !kv32 && attention_prompt_supported(E, H, n_ctx))
            timed_launch(K_ATTN, 0, [&] { return launch_attention_prompt(at, (uint16_t *) scores, nullptr, nullptr, stream); });
        else if (n == 1 && !old_attention && !kv32 && attention_decode_supported(E, H, n_ctx))
            timed_launch(K_ATTN, 0, [&] { return launch_attention_decode(at, attn_gran, (unsigned) il + 1, stream); });
        else
            timed_launch(K_ATTN, 0, [&] { return launch_attention(at, stream); });
        MvLaunch b;
        b.w = ly.wo; b.xq = aq_attn; b.y = x; b.sp = sp_d; b.n_tokens = n;
        timed_launch(K_WO, qbytes(ly.wo), [&] { return mv_launch(b, PRO_ACTQ, EPI_RESID, stream); });
        MvLaunch c;
        c.w = ly.w13; c.x = x; c.g = ly.ffn_norm; c.sp = sp_d; c.n_tokens = n; c.silu_tab = silu_tab;
        c.out_q = aq_ffn; c.u = u_ffn;
        MvLaunch d;
        d.w = ly.w2; d.xq = aq_ffn; d.x = u_ffn; d.y = x; d.sp = sp_d; d.n_tokens = n;
        if (ffn_f32) {
            timed_launch(K_W13, qbytes(ly.w13), [&] { return launch_matvec_cu(c, PRO_NORM, EPI_SWIGLU_F32, stream); });
            timed_launch(K_W2, qbytes(ly.w2), [&] { return launch_matvec_cu(d, PRO_ACTF, EPI_RESID, stream); });
        } else {
            timed_launch(K_W13, qbytes(ly.w13), [&] { return launch_matvec(c, PRO_NORM, EPI_SWIGLU, stream); });
            timed_launch(K_W2, qbytes(ly.w2), [&] { return launch_matvec(d, PRO_ACTQ, EPI_RESID, stream); });
        }
    }
    if (!model.has_head || !head) return;   // not the last pipeline stage: x is the output
    MvLaunch o;
    o.w = model.output; o.x = x; o.g = model.norm; o.sp = sp_d; o.y = logits_out;
    o.tok0 = last_only ? n - 1 : 0;
    o.n_tokens = last_only ? 1 : n;
    timed_launch(K_LMHEAD, qbytes(model.output), [&] { return mv_launch(o, PRO_NORM, EPI_STORE, stream); });
    if (want_embedding && model.has_head)
        LVK_HIP(launch_rmsnorm_rows(x + (size_t) (n - 1) * E, model.norm, E, 1, emb_d, stream));
}

void Context::build_graph(int kind) {
    // one replay per token: the step block H2D, the forward pass and the logits D2H
    // (both host buffers page-locked, the logits one sized before the capture); the
    // greedy variant ends in the device argmax (token into host-mapped memory), the sample
    // variant copies the sampler block in and ends in the device top-k candidates
    LVK_HIP(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    try {
        if (kind == 3) {
            // a chained step: the step block and x were left by the previous step (or the
            // call's setup); the argmax advances both for the next replay
            enqueue_forward(1, true, nullptr, 0, true, false);
            LVK_HIP(launch_argmax_step(logits_d, (int) model.hp.n_vocab, sp_d, chain_d, forced_d, digest_d, model.tok_emb, model.emb_type,
                                       (int) model.hp.n_embd, x, stream));
        } else {
            LVK_HIP(hipMemcpyAsync(sp_d, sp_h, sizeof(StepParams), hipMemcpyHostToDevice, stream));
            if (kind == 2) LVK_HIP(hipMemcpyAsync(samp_d, samp_h, sizeof(SampleParams), hipMemcpyHostToDevice, stream));
            enqueue_forward(1, true);
            if (kind == 1) {
                enqueue_argmax();
            } else if (kind == 2) {
                LVK_HIP(launch_sample_cand(logits_d, (int) model.hp.n_vocab, samp_d, sout_d, stream));
            } else if (model.has_head) {
                LVK_HIP(hipMemcpyAsync(logits.data(), logits_d, sizeof(float) * logits.size(), hipMemcpyDeviceToHost,
                                       stream));
            }
        }
    } catch (...) {
        hipGraph_t g;
        (void) hipStreamEndCapture(stream, &g);
        throw;
    }
    hipGraph_t & g = kind == 1 ? graph_greedy : kind == 2 ? graph_sample : kind == 3 ? graph_chain : graph;
    hipGraphExec_t & ge = kind == 1 ? graph_greedy_exec : kind == 2 ? graph_sample_exec : kind == 3 ? graph_chain_exec : graph_exec;
    LVK_HIP(hipStreamEndCapture(stream, &g));
    LVK_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
}

// greedy token of the last logits row: the device word feeds the stage link (lvk_split.cpp),
// the host-mapped one the caller (read after the stream sync; no D2H copy node)
void Context::enqueue_argmax() {
    LVK_HIP(launch_argmax(logits_d, (int) model.hp.n_vocab, greedy_d, stream, greedy_hd));
}

// One decode step whose sampler is greedy, chosen on the device:
// the same forward pass and KV append as eval(&token, 1, n_past), then the argmax
// of llama_sample_top_p_top_k(temp <= 0) (llama.cpp:1382-1394) over the logits in
// HBM.  Host logits are not refreshed (llama_get_logits keeps the previous eval's).
int Context::eval_greedy(int token, int n_past) {
    if (!model.has_head || !model.has_embed) throw Error("llama.vk_amd: greedy eval needs the whole model");
    EvalPart part;
    part.greedy = true;
    begin_eval_safe(&token, 1, n_past, part);
    end_eval(true);
    return *greedy_h;
}

// the step counter of the next device step (StepParams::seq); before it would run past the
// 25 bits that keep (seq << 7) + layer + 1 unique, the granules are zeroed (stream-ordered
// ahead of the steps that use the restarted counter) and the count restarts
unsigned Context::next_seq(unsigned k) {
    if (seq + k >= (1u << 25)) {
        if (attn_gran)
            LVK_HIP(hipMemsetAsync(attn_gran, 0, attention_decode_scratch_bytes((int) model.hp.n_head, n_ctx), stream));
        seq = 0;
    }
    const unsigned first = seq + 1;
    seq += k;
    return first;
}

// n_steps decode steps in one call (lvk_decode_chain): step i evaluates token t_i at n_past + i,
// t_0 = tokens[0], t_{i+1} = tokens[i + 1] while i + 1 < n_tokens (teacher forcing), else the
// argmax of step i's logits (greedy: n_tokens = 1).  The same logits as n_steps single-token
// evals, but the host only sets the step block up once and replays the chained graph back to back
// (no host round trip, step-block copy or embedding launch between the steps).  out[i]: the
// argmax of step i; digests (optional): lvk_logits_digest of step i's logits row.
int Context::decode_chain(const int * tokens, int n_tokens, int n_past, int n_steps, int * out,
                          unsigned long long * digests) {
    if (!model.has_head || !model.has_embed) throw Error("llama.vk_amd: chained decode needs the whole model");
    if (logits_all) throw Error("llama.vk_amd: chained decode needs last-token logits");
    if (n_steps <= 0 || n_past < 0 || n_past + n_steps > n_ctx_user)
        throw Error("llama.vk_amd: n_past + n_steps exceeds n_ctx");
    if (!tokens || n_tokens < 1 || n_tokens > n_steps) throw Error("llama.vk_amd: chained decode needs 1..n_steps tokens");
    for (int i = 0; i < n_tokens; ++i)
        if (tokens[i] < 0 || tokens[i] >= (int) model.hp.n_vocab) throw Error("llama.vk_amd: token id out of range");
    if (!use_graph || profiling)
        throw Error("llama.vk_amd: chained decode needs the launch-per-phase decode graph");
    try {
        StepParams * sh = sp_h;
        sh->n_past = n_past;
        sh->n_tokens = 1;
        sh->pad0 = tokens[0];
        sh->seq = next_seq((unsigned) n_steps);     // the steps take seq, seq + 1, ...
        LVK_HIP(hipMemcpyAsync(sp_d, sh, sizeof(StepParams), hipMemcpyHostToDevice, stream));
        chain_ctl_h[0] = 0;
        chain_ctl_h[1] = n_tokens > 1 ? n_tokens : 0;
        chain_ctl_h[2] = digests ? 1 : 0;
        chain_ctl_h[3] = 0;
        LVK_HIP(hipMemcpyAsync(chain_d, chain_ctl_h, CHAIN_HDR * 4, hipMemcpyHostToDevice, stream));
        if (n_tokens > 1) {
            std::memcpy(forced_h, tokens, sizeof(int) * (size_t) n_tokens);
            LVK_HIP(hipMemcpyAsync(forced_d, forced_h, sizeof(int) * (size_t) n_tokens, hipMemcpyHostToDevice, stream));
        }
        LVK_HIP(launch_embed(model.tok_emb, model.emb_type, (int) model.hp.n_embd, &sp_d->pad0, 1, x, stream));
        if (!graph_chain_exec) build_graph(3);
        for (int i = 0; i < n_steps; ++i) LVK_HIP(hipGraphLaunch(graph_chain_exec, stream));
        LVK_HIP(hipMemcpyAsync(chain_h, chain_d + CHAIN_HDR, sizeof(int) * (size_t) n_steps, hipMemcpyDeviceToHost, stream));
        if (digests)
            LVK_HIP(hipMemcpyAsync(digest_h, digest_d, 8 * (size_t) n_steps, hipMemcpyDeviceToHost, stream));
    } catch (...) {
        (void) hipStreamSynchronize(stream);
        logits_valid = false;
        throw;
    }
    end_eval(true);
    std::memcpy(out, chain_h, sizeof(int) * (size_t) n_steps);
    if (digests) std::memcpy(digests, digest_h, 8 * (size_t) n_steps);
    return out[n_steps - 1];
}

// One decode step whose sampler runs its O(n_vocab) part on the device:
// the forward pass of eval(&token, 1, n_past), then sample.hip's repeat penalty, temperature
// and top-k candidates over the logits in HBM (parameters in *samp_h).  Host logits are not
// refreshed (llama_get_logits keeps the previous eval's).
void Context::eval_sample(int token, int n_past) {
    if (!model.has_head || !model.has_embed) throw Error("llama.vk_amd: sampling eval needs the whole model");
    if ((int) model.hp.n_vocab > SAMPLE_MAX_VOCAB) throw Error("llama.vk_amd: vocabulary too large for the device sampler");
    EvalPart part;
    part.sample = true;
    begin_eval_safe(&token, 1, n_past, part);
    end_eval(true);
}

void Context::fetch_logits() {
    const size_t V = model.hp.n_vocab;
    logits.resize(V);
    LVK_HIP(hipMemcpy(logits.data(), logits_d, V * sizeof(float), hipMemcpyDeviceToHost));
    logits_valid = true;
}

void Context::eval(const int * tokens, int n, int n_past) {
    begin_eval_safe(tokens, n, n_past, EvalPart{});
    end_eval(false);
}

// begin_eval for a caller that ends the eval itself: if the enqueue fails part-way, the
// work already queued drains, the step blocks are released and the host logits are marked
// stale before the error propagates (llama_get_logits then refuses them)
void Context::begin_eval_safe(const int * tokens, int n, int n_past, const EvalPart & part) {
    try {
        begin_eval(tokens, n, n_past, part);
    } catch (...) {
        (void) hipStreamSynchronize(stream);
        sp_next = 1;
        logits_valid = false;
        throw;
    }
}

void Context::begin_eval(const int * tokens, int n, int n_past, const EvalPart & part) {
    const HParams & hp = model.hp;
    const int V = (int) hp.n_vocab;
    const int n_total = part.n_total < 0 ? n : part.n_total;
    if (n <= 0 || n_past < 0 || n_past + n > n_ctx_user || part.tok_off < 0 || part.tok_off + n > n_total)
        throw Error("llama.vk_amd: n_past + n_tokens exceeds n_ctx");
    if ((part.greedy || part.sample) && (!model.has_head || n != 1 || logits_all))
        throw Error("llama.vk_amd: greedy / sampling eval needs the lm_head stage, one token and last-token logits");
    if (model.has_embed) {
        if (!tokens) throw Error("llama.vk_amd: the first stage needs tokens");
        for (int i = 0; i < n; ++i)
            if (tokens[i] < 0 || tokens[i] >= V) throw Error("llama.vk_amd: token id out of range");
        std::memcpy(tok_h + part.tok_off, tokens, sizeof(int) * (size_t) n);
    }
    const bool last_only = !logits_all;
    const bool single = part.n_total < 0 || part.n_total == n;
    const bool graph_ok = n == 1 && last_only && single && use_graph && !profiling;
    // the graphs read step block 0; eager slices each take their own (the H2D copy reads
    // the pinned block when it executes, after the host may have queued further slices)
    if (!graph_ok && sp_next > n_ctx) throw Error("llama.vk_amd: too many slices before a sync");
    StepParams * sh = graph_ok ? sp_h : sp_h + sp_next++;
    sh->n_past = n_past;
    sh->n_tokens = n;
    sh->pad0 = (n == 1 && model.has_embed) ? tokens[0] : 0;
    sh->seq = next_seq();
    if (model.has_head && part.tok_off == 0)   // within the reserve: the pointer never moves
        logits.resize((size_t) (last_only ? 1 : n_total) * V);
    if (graph_ok) {
        const int kind = part.greedy ? 1 : part.sample ? 2 : 0;
        hipGraphExec_t & ge = kind == 1 ? graph_greedy_exec : kind == 2 ? graph_sample_exec : graph_exec;
        if (!ge) build_graph(kind);
        LVK_HIP(hipGraphLaunch(ge, stream));
    } else {
        LVK_HIP(hipMemcpyAsync(sp_d, sh, sizeof(StepParams), hipMemcpyHostToDevice, stream));
        if (part.sample) LVK_HIP(hipMemcpyAsync(samp_d, samp_h, sizeof(SampleParams), hipMemcpyHostToDevice, stream));
        if (n > 1)
            LVK_HIP(hipMemcpyAsync(tok_d + part.tok_off, tok_h + part.tok_off, sizeof(int) * (size_t) n,
                                   hipMemcpyHostToDevice, stream));
        enqueue_forward(n, last_only, tok_d + part.tok_off, last_only ? 0 : part.tok_off, part.head);
        if (part.greedy) {
            enqueue_argmax();
        } else if (part.sample) {
            LVK_HIP(launch_sample_cand(logits_d, V, samp_d, sout_d, stream));
        } else if (model.has_head && part.copy_out) {
            LVK_HIP(hipMemcpyAsync(logits.data(), logits_d, sizeof(float) * logits.size(), hipMemcpyDeviceToHost,
                                   stream));
        }
    }
    if (want_embedding && model.has_head && part.copy_out && !part.greedy && !part.sample) {
        embedding.resize(hp.n_embd);
        LVK_HIP(hipMemcpyAsync(embedding.data(), emb_d, sizeof(float) * hp.n_embd, hipMemcpyDeviceToHost, stream));
    }
}

void Context::end_eval(bool no_host_logits) {
    sp_next = 1;
    LVK_HIP(hipStreamSynchronize(stream));
    if (profiling) collect_profile();
    check_device_error();
    // after lvk_eval_greedy llama_get_logits still holds an earlier eval's row
    logits_valid = model.has_head && !no_host_logits;
}

size_t Context::kv_bytes() const {
    return 2u * (size_t) model.layers.size() * n_ctx * model.hp.n_embd * kv_elem_bytes();
}

void Context::kv_get() {
    const size_t half = kv_bytes() / 2;
    kv_host.resize(kv_bytes());
    LVK_HIP(hipMemcpy(kv_host.data(), kc, half, hipMemcpyDeviceToHost));
    LVK_HIP(hipMemcpy(kv_host.data() + half, vc, half, hipMemcpyDeviceToHost));
}

void Context::kv_set(const uint8_t * src, size_t n) {
    if (n != kv_bytes()) throw Error("llama_set_kv_cache: size mismatch");
    const size_t half = n / 2;
    LVK_HIP(hipMemcpy(kc, src, half, hipMemcpyHostToDevice));
    LVK_HIP(hipMemcpy(vc, src + half, half, hipMemcpyHostToDevice));
}

// device-to-device copy of positions [0, n_tokens) of every layer's K and V from
// another context of the same shape (a shared prompt prefix): K rows
// [L][n_ctx][E] are one pitched block per layer, V [L][E][n_ctx] one short row per
// (layer, dim).  Only the n_tokens positions move, not the whole cache.
void Context::kv_copy_from(const Context & src, int n_tokens) {
    const size_t E = model.hp.n_embd, L = model.layers.size(), C = (size_t) n_ctx;
    if (src.model.hp.n_embd != model.hp.n_embd || src.model.layers.size() != L || src.n_ctx != n_ctx || src.n_ctx_user != n_ctx_user ||
        src.model.hp.n_head != model.hp.n_head || src.model.layer_begin != model.layer_begin)
        throw Error("lvk_kv_copy: contexts differ in n_embd, n_head, n_layer, layer range or n_ctx");
    if (src.device != device) throw Error("lvk_kv_copy: contexts live on different HIP devices");
    // the K/V bytes are only meaningful under the weights that wrote them: same model
    // file contents (size and quantization type are checked; the caller owns identity)
    if (src.model.qtype != model.qtype || src.model.file_bytes != model.file_bytes)
        throw Error("lvk_kv_copy: contexts hold different models");
    if (src.kv32 != kv32) throw Error("lvk_kv_copy: contexts differ in the KV cache type (f16_kv)");
    if (n_tokens < 0 || n_tokens > n_ctx_user) throw Error("lvk_kv_copy: n_tokens out of range");
    if (n_tokens > 0) {
        const size_t n = (size_t) n_tokens;
        LVK_HIP(hipStreamSynchronize(src.stream));
        const size_t es = kv_elem_bytes();
        LVK_HIP(hipMemcpy2DAsync(kc, C * E * es, src.kc, C * E * es, n * E * es, L, hipMemcpyDeviceToDevice, stream));
        LVK_HIP(hipMemcpy2DAsync(vc, C * es, src.vc, C * es, n * es, L * E, hipMemcpyDeviceToDevice, stream));
        LVK_HIP(hipStreamSynchronize(stream));
    }
    kv_n = n_tokens;
}

}  // namespace lvk

namespace lvk {
// pipeline stages: the residual stream crosses stage boundaries
void Context::x_copy(void * buf, int n, bool to_ctx, bool on_device) {
    if (n <= 0 || n > n_ctx) throw Error("llama.vk_amd: bad token count for the stage residual stream");
    const size_t bytes = sizeof(float) * (size_t) n * model.hp.n_embd;
    const hipMemcpyKind k = to_ctx ? (on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice)
                                   : (on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost);
    if (to_ctx) LVK_HIP(hipMemcpyAsync(x, buf, bytes, k, stream));
    else LVK_HIP(hipMemcpyAsync(buf, x, bytes, k, stream));
    LVK_HIP(hipStreamSynchronize(stream));
}
}  // namespace lvk
