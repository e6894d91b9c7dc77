/* track_cost.c -- the host-side cost of ggml_graph_compute's device mirrors at model size.
 *
 * A Q4_0 matrix of `gib` GiB (4096-wide rows, as the 7B / 65B weights) lives in a buffer the
 * caller maps itself.  `mode` ro makes it read-only after filling (a PROT_READ model-file
 * mapping); rw leaves it writable, so only the soft-dirty pagemap bits can vouch for its pages.
 * Every call computes one mul_mat of the matrix with a 4096-vector.  The first call uploads the
 * matrix; the later calls time what the mirror bookkeeping costs on top of the matvec.
 * lvk_ggml_stats reports the bytes each call moved and its host time in the tracking.
 *
 * usage: track_cost <gib> <calls> <ro|rw>
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <time.h>

#include "ggml.h"

extern int lvk_ggml_stats(uint64_t * out, int n) __attribute__((weak));

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

int main(int argc, char ** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 4.0;
    const int calls = argc > 2 ? atoi(argv[2]) : 5;
    const int ro = argc > 3 ? strcmp(argv[3], "rw") != 0 : 1;
    const int K = 4096;
    const size_t row_bytes = (size_t) K / 32 * 20;
    const int64_t rows = (int64_t) (gib * (1u << 30) / row_bytes) / 32 * 32;
    const size_t wbytes = (size_t) rows * row_bytes + (64u << 20);
    void * wbuf = mmap(NULL, wbytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (wbuf == MAP_FAILED) return 1;
    struct ggml_init_params wp = {wbytes, wbuf, false};
    struct ggml_context * wctx = ggml_init(wp);
    struct ggml_tensor * W = ggml_new_tensor_2d(wctx, GGML_TYPE_Q4_0, K, rows);
    /* valid blocks: scale 0.5, nibbles 0x5 / 0xA */
    uint8_t blk[20];
    const float d = 0.5f;
    memcpy(blk, &d, 4);
    memset(blk + 4, 0xA5, 16);
    for (size_t i = 0; i < (size_t) rows * (K / 32); ++i) memcpy((uint8_t *) W->data + i * 20, blk, 20);
    if (ro && mprotect(wbuf, wbytes, PROT_READ) != 0) return 2;

    struct ggml_init_params cp = {64u << 20, NULL, false};
    struct ggml_context * ctx = ggml_init(cp);
    struct ggml_tensor * x = ggml_new_tensor_1d(ctx, GGML_TYPE_F32, K);
    for (int i = 0; i < K; ++i) ((float *) x->data)[i] = (float) ((i * 7919) % 101) / 101.0f - 0.5f;
    struct ggml_tensor * y = ggml_mul_mat(ctx, W, x);
    struct ggml_cgraph gf = ggml_build_forward(y);
    gf.n_threads = 1;
    printf("{\"gib\": %.2f, \"rows\": %lld, \"mode\": \"%s\", \"calls\": [", (double) rows * row_bytes / (1u << 30),
           (long long) rows, ro ? "ro" : "rw");
    for (int c = 0; c < calls; ++c) {
        const double t0 = now_ms();
        ggml_graph_compute(ctx, &gf);
        const double t1 = now_ms();
        uint64_t sv[8] = {0};
        if (lvk_ggml_stats) lvk_ggml_stats(sv, 8);
        printf("%s{\"ms\": %.3f, \"h2d\": %llu, \"d2h\": %llu, \"repack\": %llu, \"mirrored\": %llu, \"tracking\": %llu, "
               "\"track_us\": %llu, \"clear_us\": %llu}",
               c ? ", " : "", t1 - t0, (unsigned long long) sv[0], (unsigned long long) sv[1], (unsigned long long) sv[2],
               (unsigned long long) sv[3], (unsigned long long) sv[4], (unsigned long long) sv[6],
               (unsigned long long) sv[7]);
    }
    printf("], \"y0\": %.6f}\n", ((float *) y->data)[0]);
    ggml_free(ctx);
    ggml_free(wctx);
    return 0;
}
