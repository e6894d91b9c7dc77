/* graph_test.c -- a caller of the ggml operator surface (ggml.h) that builds the LLaMA
 * graph of the reference's llama_eval_internal (llama.cpp:927-1197) over seeded synthetic
 * weights and runs it with ggml_graph_compute, then writes the logits and both KV caches.
 *
 * The same source is compiled twice (tools/ggml_graph/Makefile): against include/ggml.h +
 * libllama_vk_amd.so (every node on the GPU) and against the reference ggml.c
 * (oracle/_ref, its CPU AVX2 build).  tests/test_gpu_ggml_graph.py compares the two dumps
 * bit for bit.
 *
 * usage: graph_test <out.bin> <wtype 0=Q4_0 1=Q4_1> <kv type 1=F16 0=F32>
 * Steps: a 7-token prompt at n_past 0, a 33-token batch at n_past 7 (n_kv 40 crosses the
 * 32-element f16-dot tail), two single-token decode steps.
 *
 * The weights live in a buffer the caller maps itself and makes read-only once filled (as a
 * PROT_READ model-file mapping is), the KV cache in a second, writable context.  With
 * GRAPH_TEST_REPEAT=n, n more decode steps follow the dump, each timed, and -- when the
 * library exports lvk_ggml_stats (llama.vk_amd; a weak reference, so the same source links
 * against the reference ggml.c) -- the bytes each call moved are printed to stderr.
 */
#define _GNU_SOURCE   /* mmap MAP_ANONYMOUS, clock_gettime under -std=c11 */
#include <execinfo.h>
#include <math.h>
#include <signal.h>
#include <unistd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "ggml.h"

enum { E = 256, H = 2, HD = 128, F = 768, V = 512, L = 2, C = 64 };

static uint32_t rng = 12345u;
static uint32_t next_u32(void) {
    rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5;
    return rng;
}
static float next_f(float lo, float hi) { return lo + (hi - lo) * (float) (next_u32() >> 8) / 16777216.0f; }

/* random but valid quantized rows: block scales in [lo, hi), random nibbles */
static void fill_q(struct ggml_tensor * t, float lo, float hi) {
    const int64_t nb = ggml_nelements(t) / 32;
    uint8_t * p = (uint8_t *) t->data;
    const size_t bs = ggml_type_size(t->type);
    for (int64_t b = 0; b < nb; ++b) {
        uint8_t * blk = p + b * bs;
        float d = next_f(lo, hi);
        memcpy(blk, &d, 4);
        int off = 4;
        if (t->type == GGML_TYPE_Q4_1) {
            float m = -8.0f * d + next_f(-0.1f * d, 0.1f * d);
            memcpy(blk + 4, &m, 4);
            off = 8;
        }
        for (int k = 0; k < 16; ++k) blk[off + k] = (uint8_t) next_u32();
    }
}
static void fill_f32(struct ggml_tensor * t, float lo, float hi) {
    float * p = (float *) t->data;
    for (int64_t i = 0; i < ggml_nelements(t); ++i) p[i] = next_f(lo, hi);
}

extern int lvk_ggml_stats(uint64_t * out, int n) __attribute__((weak));

struct layer {
    struct ggml_tensor *an, *fn, *wq, *wk, *wv, *wo, *w1, *w2, *w3;
};

/* a crash prints its raw backtrace (addresses map to the library with addr2line) */
static void on_fault(int sig) {
    void * bt[64];
    const int n = backtrace(bt, 64);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

int main(int argc, char ** argv) {
    signal(SIGSEGV, on_fault);
    signal(SIGBUS, on_fault);
    if (argc < 4) {
        fprintf(stderr, "usage: %s out.bin wtype(0 q4_0, 1 q4_1) kv(1 f16, 0 f32)\n", argv[0]);
        return 2;
    }
    const enum ggml_type wt = atoi(argv[2]) ? GGML_TYPE_Q4_1 : GGML_TYPE_Q4_0;
    const enum ggml_type kt = atoi(argv[3]) ? GGML_TYPE_F16 : GGML_TYPE_F32;
    const int build_only = getenv("GRAPH_TEST_BUILD_ONLY") != NULL;
    ggml_time_init();

    const size_t wbytes = 64u << 20;
    void * wbuf = mmap(NULL, wbytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (wbuf == MAP_FAILED) return 1;
    struct ggml_init_params wp = {wbytes, wbuf, false};
    struct ggml_context * wctx = ggml_init(wp);
    struct ggml_tensor * tok = ggml_new_tensor_2d(wctx, wt, E, V);
    struct ggml_tensor * norm = ggml_new_tensor_1d(wctx, GGML_TYPE_F32, E);
    struct ggml_tensor * out = ggml_new_tensor_2d(wctx, wt, E, V);
    struct layer ly[L];
    const float ws = 1.0f / (sqrtf((float) E) * 4.6f);
    fill_q(tok, 0.05f, 0.15f);
    fill_f32(norm, 0.9f, 1.1f);
    fill_q(out, 0.5f * ws, 1.5f * ws);
    for (int l = 0; l < L; ++l) {
        ly[l].an = ggml_new_tensor_1d(wctx, GGML_TYPE_F32, E);
        ly[l].fn = ggml_new_tensor_1d(wctx, GGML_TYPE_F32, E);
        ly[l].wq = ggml_new_tensor_2d(wctx, wt, E, E);
        ly[l].wk = ggml_new_tensor_2d(wctx, wt, E, E);
        ly[l].wv = ggml_new_tensor_2d(wctx, wt, E, E);
        ly[l].wo = ggml_new_tensor_2d(wctx, wt, E, E);
        ly[l].w1 = ggml_new_tensor_2d(wctx, wt, E, F);
        ly[l].w2 = ggml_new_tensor_2d(wctx, wt, F, E);
        ly[l].w3 = ggml_new_tensor_2d(wctx, wt, E, F);
        fill_f32(ly[l].an, 0.9f, 1.1f);
        fill_f32(ly[l].fn, 0.9f, 1.1f);
        fill_q(ly[l].wq, 0.5f * ws, 1.5f * ws);
        fill_q(ly[l].wk, 0.5f * ws, 1.5f * ws);
        fill_q(ly[l].wv, 0.5f * ws, 1.5f * ws);
        fill_q(ly[l].wo, 0.5f * ws, 1.5f * ws);
        fill_q(ly[l].w1, 0.5f * ws, 1.5f * ws);
        fill_q(ly[l].w2, 0.5f / (sqrtf((float) F) * 4.6f), 1.5f / (sqrtf((float) F) * 4.6f));
        fill_q(ly[l].w3, 0.5f * ws, 1.5f * ws);
    }
    /* every weight written: the buffer becomes read-only (ggml_init wrote its object list
     * into it; no tensor is created in wctx after this) */
    if (mprotect(wbuf, wbytes, PROT_READ) != 0) return 1;
    struct ggml_init_params kp = {16u << 20, NULL, false};
    struct ggml_context * kctx = ggml_init(kp);
    struct ggml_tensor * kv_k = ggml_new_tensor_1d(kctx, kt, (int64_t) L * C * E);
    struct ggml_tensor * kv_v = ggml_new_tensor_1d(kctx, kt, (int64_t) L * C * E);
    memset(kv_k->data, 0, ggml_nbytes(kv_k));
    memset(kv_v->data, 0, ggml_nbytes(kv_v));

    FILE * fo = fopen(argv[1], "wb");
    if (!fo) return 1;
    const int steps[4][2] = {{7, 0}, {33, 7}, {1, 40}, {1, 41}};
    const int repeat = getenv("GRAPH_TEST_REPEAT") ? atoi(getenv("GRAPH_TEST_REPEAT")) : 0;
    int last = 1;
    for (int st = 0; st < 4 + (repeat < C - 42 ? repeat : C - 42); ++st) {
        const int N = st < 4 ? steps[st][0] : 1, n_past = st < 4 ? steps[st][1] : 42 + (st - 4);
        if (st == 4) {
            /* the dump covers the four compared steps only */
            fwrite(kv_k->data, 1, ggml_nbytes(kv_k), fo);
            fwrite(kv_v->data, 1, ggml_nbytes(kv_v), fo);
            fclose(fo);
            fo = NULL;
        }
        struct ggml_init_params cp = {256u << 20, NULL, false};
        struct ggml_context * ctx0 = ggml_init(cp);
        struct ggml_cgraph gf;
        memset(&gf, 0, sizeof(gf));
        gf.n_threads = 4;
        struct ggml_tensor * embd = ggml_new_tensor_1d(ctx0, GGML_TYPE_I32, N);
        for (int i = 0; i < N; ++i) ((int32_t *) embd->data)[i] = (i == 0 && st == 0) ? 1 : (last + 37 * i) % V;
        struct ggml_tensor * inpL = ggml_get_rows(ctx0, tok, embd);
        for (int il = 0; il < L; ++il) {
            struct ggml_tensor * inpSA = inpL;
            struct ggml_tensor * cur = ggml_rms_norm(ctx0, inpL);
            cur = ggml_mul(ctx0, ggml_repeat(ctx0, ly[il].an, cur), cur);
            struct ggml_tensor * Qcur =
                ggml_rope(ctx0, ggml_reshape_3d(ctx0, ggml_mul_mat(ctx0, ly[il].wq, cur), HD, H, N), n_past, HD, 0);
            struct ggml_tensor * Kcur =
                ggml_rope(ctx0, ggml_reshape_3d(ctx0, ggml_mul_mat(ctx0, ly[il].wk, cur), HD, H, N), n_past, HD, 0);
            struct ggml_tensor * Vcur = ggml_transpose(ctx0, ggml_reshape_2d(ctx0, ggml_mul_mat(ctx0, ly[il].wv, cur), E, N));
            const size_t es = ggml_element_size(kv_k);
            struct ggml_tensor * k = ggml_view_1d(ctx0, kv_k, (int64_t) N * E, (es * E) * (size_t) (il * C + n_past));
            struct ggml_tensor * v = ggml_view_2d(ctx0, kv_v, N, E, C * es, (size_t) il * C * es * E + (size_t) n_past * es);
            ggml_build_forward_expand(&gf, ggml_cpy(ctx0, Kcur, k));
            ggml_build_forward_expand(&gf, ggml_cpy(ctx0, Vcur, v));
            struct ggml_tensor * Q = ggml_permute(ctx0, Qcur, 0, 2, 1, 3);
            struct ggml_tensor * K = ggml_permute(
                ctx0, ggml_reshape_3d(ctx0, ggml_view_1d(ctx0, kv_k, (int64_t) (n_past + N) * E, (size_t) il * C * es * E), HD, H, n_past + N),
                0, 2, 1, 3);
            struct ggml_tensor * KQ = ggml_mul_mat(ctx0, K, Q);
            struct ggml_tensor * KQs = ggml_scale(ctx0, KQ, ggml_new_f32(ctx0, 1.0f / sqrtf((float) E / H)));
            struct ggml_tensor * KQm = ggml_diag_mask_inf(ctx0, KQs, n_past);
            struct ggml_tensor * KQsm = ggml_soft_max(ctx0, KQm);
            struct ggml_tensor * Vv = ggml_view_3d(ctx0, kv_v, n_past + N, HD, H, C * es, C * es * HD, (size_t) il * C * es * E);
            struct ggml_tensor * KQV = ggml_mul_mat(ctx0, Vv, KQsm);
            struct ggml_tensor * KQVm = ggml_permute(ctx0, KQV, 0, 2, 1, 3);
            cur = ggml_cpy(ctx0, KQVm, ggml_new_tensor_2d(ctx0, GGML_TYPE_F32, E, N));
            cur = ggml_mul_mat(ctx0, ly[il].wo, cur);
            struct ggml_tensor * inpFF = ggml_add(ctx0, cur, inpSA);
            cur = ggml_rms_norm(ctx0, inpFF);
            cur = ggml_mul(ctx0, ggml_repeat(ctx0, ly[il].fn, cur), cur);
            struct ggml_tensor * tmp = ggml_mul_mat(ctx0, ly[il].w3, cur);
            cur = ggml_mul_mat(ctx0, ly[il].w1, cur);
            cur = ggml_silu(ctx0, cur);
            cur = ggml_mul(ctx0, cur, tmp);
            cur = ggml_mul_mat(ctx0, ly[il].w2, cur);
            inpL = ggml_add(ctx0, cur, inpFF);
        }
        inpL = ggml_rms_norm(ctx0, inpL);
        inpL = ggml_mul(ctx0, ggml_repeat(ctx0, norm, inpL), inpL);
        struct ggml_tensor * logits = ggml_mul_mat(ctx0, out, inpL);
        ggml_build_forward_expand(&gf, logits);
        if (build_only) {
            /* graph topology and pool accounting only (no compute): op sequence and shapes */
            uint64_t h = 1469598103934665603ull;
            for (int i = 0; i < gf.n_nodes; ++i) {
                const struct ggml_tensor * t = gf.nodes[i];
                const int64_t v[6] = {t->op, t->type, t->ne[0], t->ne[1], t->ne[2], (int64_t) t->nb[1]};
                for (int q = 0; q < 6; ++q) { h ^= (uint64_t) v[q]; h *= 1099511628211ull; }
            }
            fprintf(stderr, "topology %d: %016llx\n", st, (unsigned long long) h);
            memset(logits->data, 0, sizeof(float) * (size_t) V * N);
        } else {
            struct timespec t0, t1;
            clock_gettime(CLOCK_MONOTONIC, &t0);
            ggml_graph_compute(ctx0, &gf);
            clock_gettime(CLOCK_MONOTONIC, &t1);
            uint64_t sv[6] = {0};
            if (lvk_ggml_stats) lvk_ggml_stats(sv, 6);
            fprintf(stderr, "compute %d: ms %.3f h2d %llu d2h %llu repack %llu mirrored %llu mode %llu\n", st,
                    (t1.tv_sec - t0.tv_sec) * 1e3 + (t1.tv_nsec - t0.tv_nsec) * 1e-6, (unsigned long long) sv[0],
                    (unsigned long long) sv[1], (unsigned long long) sv[2], (unsigned long long) sv[3],
                    (unsigned long long) sv[4]);
        }
        if (fo) fwrite(logits->data, sizeof(float), (size_t) V * N, fo);
        /* next tokens: argmax of the last row */
        const float * lr = (const float *) logits->data + (size_t) V * (N - 1);
        int best = 0;
        for (int i = 1; i < V; ++i)
            if (lr[i] > lr[best]) best = i;
        last = best;
        fprintf(stderr, "step %d: N %d n_past %d nodes %d leafs %d used %zu argmax %d\n", st, N, n_past, gf.n_nodes,
                gf.n_leafs, ggml_used_mem(ctx0), best);
        ggml_free(ctx0);
    }
    if (fo) {
        fwrite(kv_k->data, 1, ggml_nbytes(kv_k), fo);
        fwrite(kv_v->data, 1, ggml_nbytes(kv_v), fo);
        fclose(fo);
    }
    ggml_free(kctx);
    ggml_free(wctx);
    munmap(wbuf, wbytes);
    return 0;
}
