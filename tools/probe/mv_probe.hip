// mv_probe: times the decode kernels of llama.vk_amd on one synthetic 7B Q4_0 token
// (32 layers of distinct weight images, so nothing is served from the 256 MiB MALL)
// and compares with the pure weight-stream floor measured by bw_probe.
// Build: make -C tools/probe ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>
#include "lvk_kernels.h"
#include <cmath>
#include <vector>
// this host's fp16 exp table (as lvk_context.cpp host_fp16_tables: glibc expf, RNE to fp16)
static void probe_exp_table(std::vector<uint16_t> & te) {
    te.resize(65536);
    for (int i = 0; i < 65536; ++i) {
        uint16_t hi = (uint16_t) i; _Float16 hf; memcpy(&hf, &hi, 2);
        const _Float16 e = (_Float16) expf((float) hf);
        memcpy(&te[i], &e, 2);
    }
}
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)
using namespace lvk;
#ifdef LVK_PROBE_TIMING
namespace lvk { void * lvk_probe_trace(); void * lvk_probe_atrace(); void * lvk_probe_dtrace(); }
#endif

__global__ void k_fill_u32(uint32_t * p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) i * 2654435761u ^ seed; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = h;
    }
}
__global__ void k_fill_f32(float * p, size_t n, float lo, float hi, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) i * 2654435761u ^ seed; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = lo + (hi - lo) * (h & 0xFFFFFF) / 16777216.0f;
    }
}
__global__ void k_fill_f16(uint16_t * p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) i * 2654435761u ^ seed; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = (uint16_t) (0x2C00 + (h & 0x3FF)) | (uint16_t) ((h >> 16) & 0x8000);
    }
}
// side-stream prefetch: pulls a byte range through the memory hierarchy (MALL allocation)
template <int U>
__global__ void k_prefetch(const uint4 * __restrict__ p, size_t n, unsigned * out) {
    unsigned acc = 0;
    const size_t stride = (size_t) gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n; i += stride * U) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) { size_t j = i + u * stride; j = j < n ? j : n - 1; v[u] = p[j]; }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
static void fill_u32(void * p, size_t bytes, uint32_t seed) { hipLaunchKernelGGL(k_fill_u32, dim3(1024), dim3(256), 0, 0, (uint32_t *) p, bytes / 4, seed); }
static void fill_f32(void * p, size_t n, float lo, float hi, uint32_t seed) { hipLaunchKernelGGL(k_fill_f32, dim3(1024), dim3(256), 0, 0, (float *) p, n, lo, hi, seed); }
static void * dalloc(size_t b) { void * p; CK(hipMalloc(&p, b + 4096)); return p; }

static QMatrix mkmat(int M, int K, uint32_t seed) {
    QMatrix q; q.qtype = Q4_0; q.M = M; q.K = K;
    size_t nb = qimage_nib_bytes(M, K), sb = qimage_scl_bytes(M, K);
    void * n = dalloc(nb); void * s = dalloc(sb);
    fill_u32(n, nb, seed); fill_f32(s, sb / 4, 0.001f, 0.01f, seed + 1);
    q.nib = (const uint4 *) n; q.scl = s;
    return q;
}

int main(int argc, char ** argv) {
    const int E = 4096, F = 11008, H = 32, L = 32, V = 32000, C = 512, hd = 128;
    const int n_past = argc > 1 ? atoi(argv[1]) : 256;
    struct Lay { QMatrix qkv, wo, w13, w2; };
    std::vector<Lay> ly(L);
    const bool hot = getenv("LVK_PROBE_HOT") != nullptr;   // every layer aliases layer 0 (MALL-resident)
    for (int l = 0; l < L; l++) {
        if (hot && l > 0) { ly[l] = ly[0]; continue; }
        ly[l].qkv = mkmat(3 * E, E, 100 * l + 1); ly[l].wo = mkmat(E, E, 100 * l + 2);
        ly[l].w13 = mkmat(2 * F, E, 100 * l + 3); ly[l].w2 = mkmat(E, F, 100 * l + 4);
    }
    QMatrix lm = mkmat(V, E, 7);
    float * x = (float *) dalloc(E * 4); fill_f32(x, E, -1.f, 1.f, 11);
    float * g = (float *) dalloc(E * 4); fill_f32(g, E, 0.9f, 1.1f, 12);
    uint16_t * q16 = (uint16_t *) dalloc(E * 2);
    uint16_t * kc = (uint16_t *) dalloc((size_t) L * C * E * 2); uint16_t * vc = (uint16_t *) dalloc((size_t) L * C * E * 2);
    hipLaunchKernelGGL(k_fill_f16, dim3(1024), dim3(256), 0, 0, kc, (size_t) L * C * E, 5u);
    hipLaunchKernelGGL(k_fill_f16, dim3(1024), dim3(256), 0, 0, vc, (size_t) L * C * E, 6u);
    float * scores = (float *) dalloc((size_t) H * C * 4);
    ActQ aqa; aqa.nb = E / 32; aqa.d = (float *) dalloc(E / 32 * 4); aqa.m = (float *) dalloc(E / 32 * 4); aqa.qs = (uint4 *) dalloc(E / 32 * 16);
    ActQ aqf; aqf.nb = F / 32; aqf.d = (float *) dalloc(F / 32 * 4); aqf.m = (float *) dalloc(F / 32 * 4); aqf.qs = (uint4 *) dalloc(F / 32 * 16);
    fill_f32(aqa.d, E / 32, 0.01f, 0.1f, 13); fill_u32(aqa.qs, E / 32 * 16, 14);
    fill_f32(aqf.d, F / 32, 0.01f, 0.1f, 15); fill_u32(aqf.qs, F / 32 * 16, 16);
    float * logits = (float *) dalloc((size_t) V * 4);
    float2 * rope = (float2 *) dalloc((size_t) C * hd / 2 * 8); fill_f32(rope, (size_t) C * hd, -1.f, 1.f, 17);
    uint16_t * etab = (uint16_t *) dalloc(65536 * 2); uint16_t * stab = (uint16_t *) dalloc(65536 * 2);
    hipLaunchKernelGGL(k_fill_f16, dim3(256), dim3(256), 0, 0, etab, 65536, 8u);
    hipLaunchKernelGGL(k_fill_f16, dim3(256), dim3(256), 0, 0, stab, 65536, 9u);
    StepParams sph{n_past, 1, 0, 0};
    StepParams * sp = (StepParams *) dalloc(16); CK(hipMemcpy(sp, &sph, 16, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
    hipStream_t s; CK(hipStreamCreate(&s));
    int exp_mode = 1;
    {
        // the exp mode a context would pick (checked against this host's table)
        std::vector<uint16_t> te;
        probe_exp_table(te);
        uint16_t * tb = (uint16_t *) dalloc(65536 * 2);
        CK(hipMemcpy(tb, te.data(), 65536 * 2, hipMemcpyHostToDevice));
        int * bad_d = (int *) dalloc(8); int bad[2];
        CK(exp_check(tb, bad_d, 0)); CK(hipMemcpy(bad, bad_d, 8, hipMemcpyDeviceToHost));
        exp_mode = getenv("LVK_EXP_TABLE") ? 0 : bad[1] == 0 ? 2 : bad[0] == 0 ? 1 : 0;
        printf("exp check: double %d f32 %d mismatches -> mode %d\n", bad[0], bad[1], exp_mode);
    }

    float * u = (float *) dalloc(F * 4); fill_f32(u, F, -1.f, 1.f, 18);
    void * gran = dalloc(attention_decode_scratch_bytes(H, C));
    CK(hipMemset(gran, 0, attention_decode_scratch_bytes(H, C)));
    const bool cu = getenv("LVK_PROBE_GENERIC") == nullptr;
    auto mv = [&](const MvLaunch & L, int pro, int epi) {
        if (cu) { hipError_t e = launch_matvec_cu(L, pro, epi, s); if (e != hipErrorNotSupported) return e; }
        return launch_matvec(L, pro, epi, s);
    };
    auto op = [&](int k, int l) {
        const Lay & y = ly[l];
        if (k == 0) {
            MvLaunch a; a.w = y.qkv; a.x = x; a.g = g; a.sp = sp; a.n_tokens = 1; a.q16 = q16;
            a.kc = kc + (size_t) l * C * E; a.vc = vc + (size_t) l * C * E; a.rope.cs = rope; a.n_embd = E; a.head_dim = hd; a.n_ctx = C;
            CK(mv(a, PRO_NORM, EPI_QKV));
        } else if (k == 1) {
            AttnLaunch at{q16, kc + (size_t) l * C * E, vc + (size_t) l * C * E, scores, aqa, Q4_0, etab, sp, 1, E, H, C};
            at.exp_computed = exp_mode;   // timing only: random table, mode of the real table check
            if (getenv("LVK_ATTN_V1")) CK(launch_attention(at, s));
            else CK(launch_attention_decode(at, gran, (unsigned) l + 1, s));
        } else if (k == 2) {
            MvLaunch b; b.w = y.wo; b.xq = aqa; b.y = x; b.sp = sp; b.n_tokens = 1;
            CK(mv(b, PRO_ACTQ, EPI_RESID));
        } else if (k == 3) {
            MvLaunch c; c.w = y.w13; c.x = x; c.g = g; c.sp = sp; c.n_tokens = 1; c.silu_tab = stab; c.out_q = aqf; c.u = u;
            if (cu) CK(launch_matvec_cu(c, PRO_NORM, EPI_SWIGLU_F32, s)); else CK(launch_matvec(c, PRO_NORM, EPI_SWIGLU, s));
        } else if (k == 4) {
            MvLaunch d; d.w = y.w2; d.xq = aqf; d.x = u; d.y = x; d.sp = sp; d.n_tokens = 1;
            if (cu) CK(launch_matvec_cu(d, PRO_ACTF, EPI_RESID, s)); else CK(launch_matvec(d, PRO_ACTQ, EPI_RESID, s));
        } else {
            MvLaunch o; o.w = lm; o.x = x; o.g = g; o.sp = sp; o.y = logits; o.n_tokens = 1;
            CK(mv(o, PRO_NORM, EPI_STORE));
        }
    };
    const char * names[6] = {"qkv", "attn", "wo", "w13", "w2", "lm_head"};
    const double bytes[6] = {3.0 * E * E / 32 * 20, 0, 1.0 * E * E / 32 * 20, 2.0 * F * E / 32 * 20, 1.0 * F * E / 32 * 20, 1.0 * V * E / 32 * 20};
    // x is re-normalised by every RESID add; keep it bounded by re-filling before each graph (not timed)
    hipGraph_t gr; hipGraphExec_t ge;
    const int pf = getenv("LVK_PROBE_PF") ? atoi(getenv("LVK_PROBE_PF")) : 0;   // prefetch WG count
    const int pft = getenv("LVK_PROBE_PFT") ? atoi(getenv("LVK_PROBE_PFT")) : 128;
    const int pfk = getenv("LVK_PROBE_PFK") ? atoi(getenv("LVK_PROBE_PFK")) : 0;  // fork after op k of layer l
    hipStream_t s2; CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    unsigned * pfo = (unsigned *) dalloc(64);
    std::vector<hipEvent_t> evs(L + 1);
    for (auto & ev : evs) CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    auto prefetch = [&](const QMatrix & q) {
        size_t nb = qimage_nib_bytes(q.M, q.K) / 16, sb = qimage_scl_bytes(q.M, q.K) / 16;
        hipLaunchKernelGGL(k_prefetch<8>, dim3(pf), dim3(pft), 0, s2, q.nib, nb, pfo);
        hipLaunchKernelGGL(k_prefetch<8>, dim3(pf), dim3(pft), 0, s2, (const uint4 *) q.scl, sb, pfo);
    };
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(hipMemsetAsync(gran, 0, attention_decode_scratch_bytes(H, C), s));   // per token (as the context)
    for (int l = 0; l < L; l++) {
        for (int k = 0; k < 5; k++) {
            op(k, l);
            if (pf && k == pfk && l + 1 < L) {
                CK(hipEventRecord(evs[l], s));
                CK(hipStreamWaitEvent(s2, evs[l], 0));
                prefetch(ly[l + 1].qkv); prefetch(ly[l + 1].wo); prefetch(ly[l + 1].w13); prefetch(ly[l + 1].w2);
            }
        }
    }
    if (pf) { CK(hipEventRecord(evs[L], s2)); CK(hipStreamWaitEvent(s, evs[L], 0)); }
    op(5, 0);
    CK(hipStreamEndCapture(s, &gr));
    CK(hipGraphInstantiate(&ge, gr, nullptr, nullptr, 0));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    const int R = 20;
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < R; i++) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    printf("n_past %d  token %.3f ms  (%.0f tok/s)\n", n_past, ms / R, 1e3 * R / ms);
    // per kind: one graph per kind with its 32 (or 8) launches back to back
    for (int k = 0; k < 6; k++) {
        hipGraph_t g2; hipGraphExec_t ge2;
        int n = k < 5 ? L : 8;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        if (k == 1) CK(hipMemsetAsync(gran, 0, attention_decode_scratch_bytes(H, C), s));
        for (int l = 0; l < n; l++) op(k, l);
        CK(hipStreamEndCapture(s, &g2));
        CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge2, s)); CK(hipStreamSynchronize(s));
        CK(hipEventRecord(e0, s));
        for (int i = 0; i < 5; i++) CK(hipGraphLaunch(ge2, s));
        CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        double us = ms * 1e3 / (5 * n);
        printf("  %-8s %7.2f us/launch  %6.2f TB/s\n", names[k], us, bytes[k] ? bytes[k] / (us * 1e-6) / 1e12 : 0.0);
        CK(hipGraphExecDestroy(ge2)); CK(hipGraphDestroy(g2));
    }
#ifdef LVK_PROBE_TIMING
    {
        const int kind = getenv("LVK_TRACE_KIND") ? atoi(getenv("LVK_TRACE_KIND")) : 5;
        if (kind == 1 && !getenv("LVK_ATTN_V1")) {
            void * at = lvk_probe_dtrace();
            std::vector<unsigned long long> h(32 * 4 * 4 * 16);
            for (int l = 0; l < 4; l++) op(1, l);
            CK(hipStreamSynchronize(s));
            CK(hipMemset(gran, 0, attention_decode_scratch_bytes(H, C)));
            CK(hipMemset(at, 0, h.size() * 8));
            op(1, 4);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), at, h.size() * 8, hipMemcpyDeviceToHost));
            // per wave: cycles from its entry; per workgroup: entry spread and last end
            double acc[16] = {0}, mxv[16] = {0}; int n = 0;
            unsigned long long t0min = ~0ull, t0max = 0, tend = 0;
            for (int w = 0; w < 32 * 4 * 4; w++) {
                unsigned long long * e = &h[(size_t) w * 16];
                if (!e[0] || !e[11]) continue;
                n++;
                t0min = std::min(t0min, e[0]); t0max = std::max(t0max, e[0]); tend = std::max(tend, e[11]);
                for (int k = 1; k < 14; k++) { acc[k] += (double) (e[k] - e[0]); mxv[k] = std::max(mxv[k], (double) (e[k] - e[0])); }
            }
            const char * nm[14] = {"", "dma-issued", "scores", "exchange", "softmax", "dma-wait", "qk-issued", "v-dma", "max-sync", "sum-sync", "pv", "end", "npast-known", "q-issued"};
            const int ord[13] = {12, 13, 6, 7, 1, 2, 3, 8, 9, 4, 5, 10, 11};
            printf("decode attention trace (%d waves, entry spread %llu, first entry -> last end %llu cycles), avg (max) from wave entry:\n ",
                   n, t0max - t0min, tend - t0min);
            for (int i = 0; i < 13; i++) printf(" %s %.0f (%.0f)", nm[ord[i]], acc[ord[i]] / n, mxv[ord[i]]);
            printf("\n");
            return 0;
        }
        if (kind == 1) {
            void * at = lvk_probe_atrace();
            std::vector<unsigned long long> h(64 * 64);
            for (int l = 0; l < 4; l++) op(1, l);
            CK(hipStreamSynchronize(s));
            CK(hipMemset(at, 0, h.size() * 8));
            op(1, 4);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), at, h.size() * 8, hipMemcpyDeviceToHost));
            double acc[6] = {0}; int n = 0;
            for (int w = 0; w < 64 * 4; w++) {
                unsigned long long * e = &h[(size_t) w * 16];
                if (!e[0] || !e[5]) continue;
                n++;
                for (int k = 1; k < 6; k++) acc[k] += (double) (e[k] - e[0]);
            }
            printf("attention trace (%d waves): loads-issued %.0f  scores %.0f  softmax %.0f  pv %.0f  end %.0f cycles\n",
                   n, acc[1] / n, acc[2] / n, acc[3] / n, acc[4] / n, acc[5] / n);
            return 0;
        }
        void * tr = lvk_probe_trace();
        const size_t n = 256 * 16 * 64;
        if (getenv("LVK_TRACE_RAW")) {
            // per wave index: the average cycles of events 1..7 after the wave's entry (event 0)
            std::vector<unsigned long long> h(n);
            for (int l = 0; l < 4; l++) op(kind, l);
            CK(hipStreamSynchronize(s));
            CK(hipMemset(tr, 0, n * 8));
            op(kind, 4);
            CK(hipStreamSynchronize(s));
            CK(hipMemcpy(h.data(), tr, n * 8, hipMemcpyDeviceToHost));
            unsigned long long t0 = ~0ull, tend = 0;
            for (int w = 0; w < 256 * 16; w++) if (h[(size_t) w * 64]) { t0 = std::min(t0, h[(size_t) w * 64]); }
            printf("raw trace kind %s (cycles after the wave's entry; entry after the first wave's entry):\n", names[kind]);
            for (int wi = 0; wi < 16; wi++) {
                double a[40] = {0}; int c[40] = {0}; int nw = 0; double ent = 0;
                for (int b = 0; b < 256; b++) {
                    unsigned long long * e = &h[((size_t) b * 16 + wi) * 64];
                    if (!e[0]) continue;
                    nw++; ent += (double) (e[0] - t0);
                    for (int k = 1; k < 40; k++) if (e[k]) { a[k] += (double) (e[k] - e[0]); c[k]++; tend = std::max(tend, e[k]); }
                }
                if (!nw) continue;
                printf("  wave %2d (%3d wgs) entry %6.0f:", wi, nw, ent / nw);
                for (int k = 1; k < 40; k++) if (c[k]) printf(" e%d %.0f", k, a[k] / c[k]);
                printf("\n");
            }
            printf("  first entry -> last stamp %llu cycles\n", tend - t0);
            return 0;
        }
        std::vector<unsigned long long> h(n);
        // warm the same launch, then trace the 5th layer's instance
        for (int l = 0; l < 4; l++) op(kind, l);
        CK(hipStreamSynchronize(s));
        CK(hipMemset(tr, 0, n * 8));
        op(kind, 4);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(h.data(), tr, n * 8, hipMemcpyDeviceToHost));
        double sum_pro = 0, sum_end = 0, sum_issue = 0; int nw = 0;
        double pe[4] = {0, 0, 0, 0}; int npw = 0;
        std::vector<double> cs(60, 0), cw(60, 0); std::vector<int> cn(60, 0);
        double maxend = 0;
        for (int w = 0; w < 256 * 16; w++) {
            unsigned long long * e = &h[(size_t) w * 64];
            if (e[60] && e[63]) { npw++; pe[0] += e[61] - e[0]; pe[1] += e[62] - e[0]; pe[2] += e[63] - e[0]; }
            if (!e[0] || !e[3]) continue;
            nw++;
            sum_issue += e[1] - e[0]; sum_pro += e[2] - e[0]; sum_end += e[3] - e[0];
            maxend = std::max(maxend, (double) (e[3] - e[0]));
            unsigned long long prev = e[2];
            for (int q = 4; q + 1 < 56 && e[q] && e[q + 1]; q += 2) {
                int ci = (q - 4) / 2;
                cs[ci] += e[q + 1] - e[q]; cw[ci] += e[q] - prev; cn[ci]++;
                prev = e[q + 1];
            }
        }
        printf("trace kind %s: %d compute waves; avg cycles from entry: staged-seen %.0f act-ready %.0f end %.0f (max end %.0f)\n",
               names[kind], nw, sum_issue / nw, sum_pro / nw, sum_end / nw, maxend);
        {
            double a[3] = {0, 0, 0}; int c[3] = {0, 0, 0};
            double first_entry = 1e30, last_entry = 0;
            for (int w = 0; w < 256 * 16; w++) {
                unsigned long long * e = &h[(size_t) w * 64];
                if (!e[0] || !e[3]) continue;
                first_entry = std::min(first_entry, (double) e[0]); last_entry = std::max(last_entry, (double) e[0]);
                for (int q = 0; q < 3; q++) if (e[58 + q]) { a[q] += e[58 + q] - e[0]; c[q]++; }
            }
            printf("  inputs-landed %.0f  weights-issued %.0f  norm-synced %.0f\n",
                   c[0] ? a[0] / c[0] : -1.0, c[1] ? a[1] / c[1] : -1.0, c[2] ? a[2] / c[2] : -1.0);
            // per workgroup: the last wave's end; grouped by blockIdx % 8 (the XCD under
            // round-robin placement) and the spread over workgroups
            double xe[8] = {0}; int xn[8] = {0};
            std::vector<double> wg_end;
            for (int b = 0; b < 256; b++) {
                double mx = 0; bool any = false;
                for (int w = 0; w < 16; w++) {
                    unsigned long long * e = &h[(size_t) (b * 16 + w) * 64];
                    if (!e[0] || !e[3]) continue;
                    any = true; mx = std::max(mx, (double) (e[3] - e[0]));
                }
                if (!any) continue;
                wg_end.push_back(mx); xe[b % 8] += mx; xn[b % 8]++;
            }
            std::sort(wg_end.begin(), wg_end.end());
            if (!wg_end.empty())
                printf("  workgroup end: min %.0f p10 %.0f median %.0f p90 %.0f max %.0f | by b%%8:", wg_end.front(),
                       wg_end[wg_end.size() / 10], wg_end[wg_end.size() / 2], wg_end[wg_end.size() * 9 / 10], wg_end.back());
            for (int x = 0; x < 8; x++) printf(" %.0f", xn[x] ? xe[x] / xn[x] : 0.0);
            printf("\n");
        }
        printf("  (loader waves %d) staged-issued %.0f  first-publish %.0f  end %.0f\n", npw, pe[0] / std::max(1, npw), pe[1] / std::max(1, npw), pe[2] / std::max(1, npw));
        for (int c = 0; c < 26 && cn[c]; c++)
            printf("  chunk %2d: n %5d  gap-before %6.0f  body %6.0f\n", c, cn[c], cw[c] / cn[c], cs[c] / cn[c]);
    }
#endif
    return 0;
}
