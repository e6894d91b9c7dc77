/* oracle/lvk_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * Scalar CPU restatement of the reference AVX2 ggml.c arithmetic on the
 * quantized LLaMA forward pass.  Every function cites the reference
 * file:line it restates.  Rules that make it bit-exact:
 *   - compile with -std=c11 -ffp-contract=off; fmaf exactly where the
 *     reference uses _mm256_fmadd_ps, separate mul/add elsewhere;
 *   - nearbyintf (RNE) where the reference uses _mm256_round_ps(NEAREST);
 *   - F16C _cvtss_sh(x,0) for every f32->f16 conversion;
 *   - fp16 exp/silu tables built with this host's glibc expf;
 *   - AVX2 lane structure of the q4 dots and the 4x8 accumulators + hadd
 *     tree of ggml_vec_dot_f16, double sums in rms_norm/softmax/f16 tails.
 * Parallelism is over rows/heads only (never inside a reduction), so the
 * result is thread-count invariant like the reference (ggml.c:6648-6683).
 */
#define _GNU_SOURCE
#include "lvk_oracle.h"

#include <fcntl.h>
#include <immintrin.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define QK 32

typedef struct { float d; uint8_t qs[16]; } blk_q4_0;          /* ggml.c:492-497 */
typedef struct { float d; float m; uint8_t qs[16]; } blk_q4_1; /* ggml.c:501-506 */

/* ------------------------------------------------------------------ fp16 */
uint16_t orc_fp32_to_fp16(float x) { return _cvtss_sh(x, 0); }   /* ggml.c:183 */
float orc_fp16_to_fp32(uint16_t h) { return _cvtsh_ss(h); }       /* ggml.c:182 */

static uint16_t g_exp_f16[1 << 16];
static uint16_t g_silu_f16[1 << 16];
static int g_tables_ready = 0;

/* ggml.c:2915-2927 */
void orc_init_tables(void) {
    if (g_tables_ready) return;
    for (int i = 0; i < (1 << 16); ++i) {
        const float f = orc_fp16_to_fp32((uint16_t) i);
        g_silu_f16[i] = orc_fp32_to_fp16(f / (1.0f + expf(-f)));   /* ggml.c:2486-2488 */
        g_exp_f16[i] = orc_fp32_to_fp16(expf(f));
    }
    g_tables_ready = 1;
}
const uint16_t* orc_table_exp_f16(void) { orc_init_tables(); return g_exp_f16; }
const uint16_t* orc_table_silu_f16(void) { orc_init_tables(); return g_silu_f16; }

static int g_threads = 0;
void orc_set_threads(int n) { g_threads = n; }
static int nthreads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}

/* ---------------------------------------------------- AVX2 pack emulation */
/* _mm256_cvtps_epi32 of an already-rounded value: NaN/out-of-range -> INT_MIN */
static int32_t cvt_ps_epi32(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int32_t) 0x80000000u;
    return (int32_t) v;
}
static int8_t sat8(int32_t v) {   /* packs_epi32 then packs_epi16 */
    if (v > 32767) v = 32767;
    if (v < -32768) v = -32768;
    if (v > 127) v = 127;
    if (v < -128) v = -128;
    return (int8_t) v;
}
/* packNibbles (ggml.c:438-452): 16-bit lane (b0 | b1<<8) -> b0 | (b1<<4), packus */
static uint8_t pack_nib(uint8_t b0, uint8_t b1) {
    int v = (int) b0 | ((int) b1 << 4);
    return (uint8_t) (v > 255 ? 255 : v);
}

/* ----------------------------------------------------------- quantizers */
/* quantize_row_q4_0, AVX2 branch (ggml.c:621-685) */
void orc_quantize_row_q4_0(const float* x, void* vy, int k) {
    blk_q4_0* y = (blk_q4_0*) vy;
    const int nb = k / QK;
    for (int i = 0; i < nb; ++i) {
        const float* xb = x + i * QK;
        float amax = 0.0f;
        for (int l = 0; l < QK; ++l) {
            const float a = fabsf(xb[l]);
            amax = a > amax ? a : amax;
        }
        const float d = amax / 7.0f;
        const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
        y[i].d = d;
        uint8_t b[QK];
        for (int l = 0; l < QK; ++l) {
            const float v = xb[l] * id;
            b[l] = (uint8_t) (sat8(cvt_ps_epi32(nearbyintf(v))) + 8);
        }
        for (int l = 0; l < QK / 2; ++l) y[i].qs[l] = pack_nib(b[2 * l], b[2 * l + 1]);
    }
}

/* quantize_row_q4_1, AVX2 branch (ggml.c:847-920) */
void orc_quantize_row_q4_1(const float* x, void* vy, int k) {
    blk_q4_1* y = (blk_q4_1*) vy;
    const int nb = k / QK;
    for (int i = 0; i < nb; ++i) {
        const float* xb = x + i * QK;
        /* exact AVX2 max/min tree (ggml.c:859-880): max_ps(a,b) = a > b ? a : b,
         * so the sign of a zero extremum follows the reference's lane order */
        float vx[8], vn[8];
        for (int l = 0; l < 8; ++l) {
            float a = xb[l], b = xb[8 + l];
            vx[l] = a > b ? a : b;       vn[l] = a < b ? a : b;
            b = xb[16 + l]; vx[l] = vx[l] > b ? vx[l] : b; vn[l] = vn[l] < b ? vn[l] : b;
            b = xb[24 + l]; vx[l] = vx[l] > b ? vx[l] : b; vn[l] = vn[l] < b ? vn[l] : b;
        }
        float x4[4], n4[4];
        for (int l = 0; l < 4; ++l) {
            x4[l] = vx[4 + l] > vx[l] ? vx[4 + l] : vx[l];
            n4[l] = vn[4 + l] < vn[l] ? vn[4 + l] : vn[l];
        }
        for (int l = 0; l < 2; ++l) {
            x4[l] = x4[l] > x4[l + 2] ? x4[l] : x4[l + 2];
            n4[l] = n4[l] < n4[l + 2] ? n4[l] : n4[l + 2];
        }
        const float mx = x4[0] > x4[1] ? x4[0] : x4[1];
        const float mn = n4[0] < n4[1] ? n4[0] : n4[1];
        const float d = (mx - mn) / 15.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].m = mn;
        y[i].d = d;
        uint8_t b[QK];
        for (int l = 0; l < QK; ++l) {
            const float t = xb[l] - mn;   /* separate sub and mul (ggml.c:874-877) */
            const float v = t * id;
            b[l] = (uint8_t) sat8(cvt_ps_epi32(nearbyintf(v)));
        }
        for (int l = 0; l < QK / 2; ++l) y[i].qs[l] = pack_nib(b[2 * l], b[2 * l + 1]);
    }
}

/* quantize_row_q4_0_reference (ggml.c:509-543): roundf, half away from zero */
void orc_quantize_row_q4_0_reference(const float* x, void* vy, int k) {
    blk_q4_0* y = (blk_q4_0*) vy;
    const int nb = k / QK;
    for (int i = 0; i < nb; ++i) {
        float amax = 0.0f;
        for (int l = 0; l < QK; ++l) {
            const float v = fabsf(x[i * QK + l]);
            amax = amax > v ? amax : v;
        }
        const float d = amax / 7.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].d = d;
        for (int l = 0; l < QK; l += 2) {
            const float v0 = x[i * QK + l] * id, v1 = x[i * QK + l + 1] * id;
            const uint8_t q0 = (uint8_t) ((int8_t) roundf(v0) + 8);
            const uint8_t q1 = (uint8_t) ((int8_t) roundf(v1) + 8);
            y[i].qs[l / 2] = (uint8_t) (q0 | (q1 << 4));
        }
    }
}

/* quantize_row_q4_1_reference (ggml.c:799-838) */
void orc_quantize_row_q4_1_reference(const float* x, void* vy, int k) {
    blk_q4_1* y = (blk_q4_1*) vy;
    const int nb = k / QK;
    for (int i = 0; i < nb; ++i) {
        float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
        for (int l = 0; l < QK; ++l) {
            const float v = x[i * QK + l];
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
        const float d = (mx - mn) / 15.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        y[i].d = d;
        y[i].m = mn;
        for (int l = 0; l < QK; l += 2) {
            const float v0 = (x[i * QK + l] - mn) * id, v1 = (x[i * QK + l + 1] - mn) * id;
            const uint8_t q0 = (uint8_t) roundf(v0), q1 = (uint8_t) roundf(v1);
            y[i].qs[l / 2] = (uint8_t) (q0 | (q1 << 4));
        }
    }
}

/* dequantize_row_q4_0 AVX2 (ggml.c:968-1000): (float)(q-8) * d */
void orc_dequantize_row_q4_0(const void* vx, float* y, int k) {
    const blk_q4_0* x = (const blk_q4_0*) vx;
    for (int i = 0; i < k / QK; ++i)
        for (int l = 0; l < QK / 2; ++l) {
            const uint8_t v = x[i].qs[l];
            y[i * QK + 2 * l] = (float) ((int) (v & 15) - 8) * x[i].d;
            y[i * QK + 2 * l + 1] = (float) ((int) (v >> 4) - 8) * x[i].d;
        }
}

/* dequantize_row_q4_1 AVX2 (ggml.c:1086-1115): q*d then + m (no FMA) */
void orc_dequantize_row_q4_1(const void* vx, float* y, int k) {
    const blk_q4_1* x = (const blk_q4_1*) vx;
    for (int i = 0; i < k / QK; ++i)
        for (int l = 0; l < QK / 2; ++l) {
            const uint8_t v = x[i].qs[l];
            const float a = (float) (v & 15) * x[i].d;
            const float b = (float) (v >> 4) * x[i].d;
            y[i * QK + 2 * l] = a + x[i].m;
            y[i * QK + 2 * l + 1] = b + x[i].m;
        }
}

/* -------------------------------------------------------------- dots */
/* horizontal sum of an 8-lane AVX accumulator (ggml.c:2019-2024) */
static float hsum8(const float a[8]) {
    const float r0 = a[0] + a[4], r1 = a[1] + a[5], r2 = a[2] + a[6], r3 = a[3] + a[7];
    return (r0 + r2) + (r1 + r3);
}

/* Test-only model of the MFMA prompt matmul's order (see lvk_oracle.h): the
 * block dot of ggml_vec_dot_q4_0 (ggml.c:1950-2026) as one exact integer per
 * block, one fp32 chain over the blocks. */
float orc_vec_dot_q4_0_blockorder(int n, const void* vx, const void* vy) {
    const blk_q4_0* x = (const blk_q4_0*) vx;
    const blk_q4_0* y = (const blk_q4_0*) vy;
    float acc = 0.0f;
    for (int i = 0; i < n / QK; ++i) {
        int p = 0;
        for (int b = 0; b < QK / 2; ++b) {
            const int xl = (x[i].qs[b] & 15) - 8, xh = (x[i].qs[b] >> 4) - 8;
            const int yl = (y[i].qs[b] & 15) - 8, yh = (y[i].qs[b] >> 4) - 8;
            p += xl * yl + xh * yh;
        }
        const float s = x[i].d * y[i].d;
        acc = fmaf(s, (float) p, acc);
    }
    return acc;
}

/* ggml_vec_dot_q4_0 AVX2 (ggml.c:1950-2026).  Lane j of the 8-float acc
 * receives the block's elements 4j..4j+3 (madd of low-nibble and high-nibble
 * int16 vectors, ggml.c:2006-2010). */
float orc_vec_dot_q4_0(int n, const void* vx, const void* vy) {
    const blk_q4_0* x = (const blk_q4_0*) vx;
    const blk_q4_0* y = (const blk_q4_0*) vy;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < n / QK; ++i) {
        const float s = x[i].d * y[i].d;
        for (int j = 0; j < 8; ++j) {
            int p = 0;
            for (int b = 2 * j; b < 2 * j + 2; ++b) {
                const int xl = (x[i].qs[b] & 15) - 8, xh = (x[i].qs[b] >> 4) - 8;
                const int yl = (y[i].qs[b] & 15) - 8, yh = (y[i].qs[b] >> 4) - 8;
                p += xl * yl + xh * yh;
            }
            acc[j] = fmaf(s, (float) p, acc[j]);
        }
    }
    return hsum8(acc);
}

/* ggml_vec_dot_q4_1 AVX2 (ggml.c:2188-2258).  bytesFromNibbles keeps the
 * natural element order; lane j int = elems {2j,2j+1,16+2j,17+2j}; cross term
 * lanes: even j -> d0*m1 * sum(x[8q..8q+7]), odd j -> m0*d1 * sum(y[8q..]),
 * q = j/2 (sad_epu8 + blend 0xAA). */
float orc_vec_dot_q4_1(int n, const void* vx, const void* vy) {
    const blk_q4_1* x = (const blk_q4_1*) vx;
    const blk_q4_1* y = (const blk_q4_1*) vy;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float acc_off = 0.0f;
    for (int i = 0; i < n / QK; ++i) {
        uint8_t ex[QK], ey[QK];
        for (int l = 0; l < QK / 2; ++l) {
            ex[2 * l] = x[i].qs[l] & 15; ex[2 * l + 1] = x[i].qs[l] >> 4;
            ey[2 * l] = y[i].qs[l] & 15; ey[2 * l + 1] = y[i].qs[l] >> 4;
        }
        const float s01 = x[i].d * y[i].d;
        const float s0 = x[i].d * y[i].m;   /* scale_0 = d0*m1 */
        const float s1 = x[i].m * y[i].d;   /* scale_1 = m0*d1 */
        for (int j = 0; j < 8; ++j) {
            const int p = ex[2 * j] * ey[2 * j] + ex[2 * j + 1] * ey[2 * j + 1]
                        + ex[16 + 2 * j] * ey[16 + 2 * j] + ex[17 + 2 * j] * ey[17 + 2 * j];
            const int q = j / 2;
            int sum = 0;
            for (int e = 8 * q; e < 8 * q + 8; ++e) sum += (j & 1) ? ey[e] : ex[e];
            acc[j] = fmaf(s01, (float) p, acc[j]);
            acc[j] = fmaf((j & 1) ? s1 : s0, (float) sum, acc[j]);
        }
        const float mm = x[i].m * y[i].m;
        acc_off = acc_off + mm;
    }
    const float off = acc_off * (float) QK;
    return hsum8(acc) + off;
}

/* ggml_vec_dot_f16 (ggml.c:1781-1815) with the AVX F32Cx8 macros: 4 regs x 8
 * lanes of fmaf, REDUCE (ggml.c:1318-1337), leftovers in double. */
float orc_vec_dot_f16(int n, const uint16_t* x, const uint16_t* y) {
    const int np = n & ~31;
    float sum[4][8];
    memset(sum, 0, sizeof(sum));
    for (int i = 0; i < np; i += 32)
        for (int r = 0; r < 4; ++r)
            for (int l = 0; l < 8; ++l) {
                const int e = i + 8 * r + l;
                sum[r][l] = fmaf(orc_fp16_to_fp32(x[e]), orc_fp16_to_fp32(y[e]), sum[r][l]);
            }
    for (int l = 0; l < 8; ++l) {
        sum[0][l] = sum[0][l] + sum[1][l];
        sum[2][l] = sum[2][l] + sum[3][l];
        sum[0][l] = sum[0][l] + sum[2][l];
    }
    const float t0 = sum[0][0] + sum[0][4], t1 = sum[0][1] + sum[0][5];
    const float t2 = sum[0][2] + sum[0][6], t3 = sum[0][3] + sum[0][7];
    double sumf = (double) ((t0 + t1) + (t2 + t3));
    for (int i = np; i < n; ++i) {
        const float p = orc_fp16_to_fp32(x[i]) * orc_fp16_to_fp32(y[i]);
        sumf += (double) p;
    }
    return (float) sumf;
}

/* ------------------------------------------------------------ row ops */
/* ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076) */
void orc_rms_norm(const float* x, int K, int N, float* y) {
    for (int t = 0; t < N; ++t) {
        const float* xr = x + (size_t) t * K;
        double sum = 0.0;
        for (int i = 0; i < K; ++i) {
            const float sq = xr[i] * xr[i];
            sum += (double) sq;
        }
        const float mean = (float) (sum / (double) K);
        const float scale = 1.0f / sqrtf(mean + 1e-6f);
        for (int i = 0; i < K; ++i) y[(size_t) t * K + i] = xr[i] * scale;
    }
}

/* ggml_compute_forward_rope_f32 mode 0 (ggml.c:7200-7224) */
void orc_rope(const float* x, int hd, int nh, int N, int n_past, float* y) {
    for (int t = 0; t < N; ++t) {
        const int p = n_past + t;
        for (int h = 0; h < nh; ++h)
            for (int i0 = 0; i0 < hd; i0 += 2) {
                const float theta = powf(10000.0f, ((float) -i0) / hd);
                const float ang = (float) p * theta;
                const float c = cosf(ang), s = sinf(ang);
                const size_t o = ((size_t) t * nh + h) * hd + i0;
                const float x0 = x[o], x1 = x[o + 1];
                const float a = x0 * c, b = x1 * s, e = x0 * s, f = x1 * c;
                y[o] = a - b;
                y[o + 1] = e + f;
            }
    }
}

/* ggml_vec_silu_f32 with GGML_SILU_FP16 (ggml.c:2495-2503) */
void orc_silu(const float* x, int n, float* y) {
    orc_init_tables();
    for (int i = 0; i < n; ++i) y[i] = orc_fp16_to_fp32(g_silu_f16[orc_fp32_to_fp16(x[i])]);
}

/* ggml_compute_forward_soft_max_f32 (ggml.c:7099-7121) */
void orc_softmax_row(float* p, int n) {
    orc_init_tables();
    float mx = -INFINITY;
    for (int i = 0; i < n; ++i) mx = mx > p[i] ? mx : p[i];   /* MAX(max, x[i]) */
    double sum = 0.0;
    for (int i = 0; i < n; ++i) {
        if (p[i] == -INFINITY) {
            p[i] = 0.0f;
        } else {
            const float v = orc_fp16_to_fp32(g_exp_f16[orc_fp32_to_fp16(p[i] - mx)]);
            sum += (double) v;
            p[i] = v;
        }
    }
    sum = 1.0 / sum;
    const float sc = (float) sum;
    for (int i = 0; i < n; ++i) p[i] *= sc;
}

/* one layer's attention (llama.cpp:1010-1061): KQ (f16 dot, Q rounded to f16
 * in the mul_mat INIT, ggml.c:6420-6433), scale, causal mask, softmax, P->f16,
 * KQV (f16 dot over n_kv = n_past + N for every column), merge heads. */
void orc_attention(const uint16_t* kc, const uint16_t* vc, const float* q,
                   int n_embd, int n_head, int n_ctx, int n_past, int N, float* out) {
    const int hd = n_embd / n_head;
    const int n_kv = n_past + N;
    const float scale = 1.0f / sqrtf((float) n_embd / (float) n_head);
    #pragma omp parallel for collapse(2) num_threads(nthreads()) schedule(static)
    for (int t = 0; t < N; ++t)
        for (int h = 0; h < n_head; ++h) {
            uint16_t* q16 = (uint16_t*) malloc(sizeof(uint16_t) * hd);
            float* s = (float*) malloc(sizeof(float) * n_kv);
            uint16_t* p16 = (uint16_t*) malloc(sizeof(uint16_t) * n_kv);
            for (int d = 0; d < hd; ++d) q16[d] = orc_fp32_to_fp16(q[(size_t) t * n_embd + h * hd + d]);
            for (int p = 0; p < n_kv; ++p) {
                const float kq = orc_vec_dot_f16(hd, kc + (size_t) p * n_embd + h * hd, q16);
                s[p] = kq * scale;
                if (p > n_past + t) s[p] = -INFINITY;           /* ggml.c:7028-7031 */
            }
            orc_softmax_row(s, n_kv);
            for (int p = 0; p < n_kv; ++p) p16[p] = orc_fp32_to_fp16(s[p]);
            for (int d = 0; d < hd; ++d)
                out[(size_t) t * n_embd + h * hd + d] =
                    orc_vec_dot_f16(n_kv, vc + (size_t) (h * hd + d) * n_ctx, p16);
            free(q16); free(s); free(p16);
        }
}

/* --------------------------------------------------------------- model */
enum { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q4_1 = 3 };

typedef struct { int type; int ne0, ne1; const uint8_t* data; } otensor;

typedef struct {
    otensor an, wq, wk, wv, wo, fn, w1, w2, w3;
} olayer;

struct orc_model {
    int n_vocab, n_embd, n_mult, n_head, n_layer, n_rot, ftype, n_ff, n_ctx;
    void* map; size_t map_size;
    otensor tok, norm, out;
    olayer* L;
    uint16_t* kc;   /* [L][n_ctx][n_embd] */
    uint16_t* vc;   /* [L][n_embd][n_ctx] */
};

static size_t row_bytes(int type, int k) {
    switch (type) {
        case T_F32: return 4u * (size_t) k;
        case T_F16: return 2u * (size_t) k;
        case T_Q4_0: return (size_t) k / QK * 20u;
        default: return (size_t) k / QK * 24u;
    }
}

static int find_tensor(const uint8_t* base, size_t size, size_t off0, const char* name, otensor* t) {
    size_t off = off0;
    const size_t nl = strlen(name);
    while (off + 12 <= size) {
        uint32_t nd, nlen, ft;
        memcpy(&nd, base + off, 4); memcpy(&nlen, base + off + 4, 4); memcpy(&ft, base + off + 8, 4);
        off += 12;
        uint32_t ne[2] = {1, 1};
        for (uint32_t i = 0; i < nd && i < 2; ++i) memcpy(&ne[i], base + off + 4 * i, 4);
        off += 4u * nd;
        const char* nm = (const char*) base + off;
        off += nlen;
        off += (32 - (off & 31)) & 31;                    /* llama.cpp:397-400 */
        const size_t bytes = row_bytes((int) ft, (int) ne[0]) * ne[1];
        if (nlen == nl && memcmp(nm, name, nl) == 0) {
            t->type = (int) ft; t->ne0 = (int) ne[0]; t->ne1 = (int) ne[1]; t->data = base + off;
            return 0;
        }
        off += bytes;
    }
    return -1;
}

orc_model* orc_model_load(const char* path, int n_ctx) {
    orc_init_tables();
    int fd = open(path, O_RDONLY);
    if (fd < 0) return NULL;
    struct stat st;
    fstat(fd, &st);
    void* map = mmap(NULL, (size_t) st.st_size, PROT_READ, MAP_SHARED, fd, 0);
    close(fd);
    if (map == MAP_FAILED) return NULL;
    const uint8_t* b = (const uint8_t*) map;
    uint32_t magic, ver, hp[7];
    memcpy(&magic, b, 4); memcpy(&ver, b + 4, 4);
    if (magic != 0x67676a74u || ver != 1) { munmap(map, (size_t) st.st_size); return NULL; }
    memcpy(hp, b + 8, 28);
    orc_model* m = (orc_model*) calloc(1, sizeof(orc_model));
    m->map = map; m->map_size = (size_t) st.st_size;
    m->n_vocab = (int) hp[0]; m->n_embd = (int) hp[1]; m->n_mult = (int) hp[2];
    m->n_head = (int) hp[3]; m->n_layer = (int) hp[4]; m->n_rot = (int) hp[5]; m->ftype = (int) hp[6];
    m->n_ff = ((2 * (4 * m->n_embd) / 3 + m->n_mult - 1) / m->n_mult) * m->n_mult;   /* llama.cpp:771 */
    m->n_ctx = n_ctx;
    size_t off = 36;
    for (int i = 0; i < m->n_vocab; ++i) { uint32_t len; memcpy(&len, b + off, 4); off += 4 + len + 4; }
    int bad = 0;
    bad |= find_tensor(b, m->map_size, off, "tok_embeddings.weight", &m->tok);
    bad |= find_tensor(b, m->map_size, off, "norm.weight", &m->norm);
    bad |= find_tensor(b, m->map_size, off, "output.weight", &m->out);
    m->L = (olayer*) calloc((size_t) m->n_layer, sizeof(olayer));
    char nm[128];
#define GET(field, suffix) \
    snprintf(nm, sizeof(nm), "layers.%d.%s", il, suffix); bad |= find_tensor(b, m->map_size, off, nm, &m->L[il].field)
    for (int il = 0; il < m->n_layer; ++il) {
        GET(an, "attention_norm.weight"); GET(wq, "attention.wq.weight"); GET(wk, "attention.wk.weight");
        GET(wv, "attention.wv.weight"); GET(wo, "attention.wo.weight"); GET(fn, "ffn_norm.weight");
        GET(w1, "feed_forward.w1.weight"); GET(w2, "feed_forward.w2.weight"); GET(w3, "feed_forward.w3.weight");
    }
#undef GET
    if (bad) { orc_model_free(m); return NULL; }
    const size_t kv = (size_t) m->n_layer * n_ctx * m->n_embd;
    m->kc = (uint16_t*) calloc(kv, 2);
    m->vc = (uint16_t*) calloc(kv, 2);
    return m;
}

void orc_model_free(orc_model* m) {
    if (!m) return;
    if (m->map) munmap(m->map, m->map_size);
    free(m->L); free(m->kc); free(m->vc); free(m);
}
int orc_n_vocab(const orc_model* m) { return m->n_vocab; }
int orc_n_embd(const orc_model* m) { return m->n_embd; }
const uint16_t* orc_kv_k(const orc_model* m, int il) { return m->kc + (size_t) il * m->n_ctx * m->n_embd; }
const uint16_t* orc_kv_v(const orc_model* m, int il) { return m->vc + (size_t) il * m->n_ctx * m->n_embd; }

/* ggml_compute_forward_mul_mat_q_f32 (ggml.c:6625-6683): quantize every
 * column of x, then one vec_dot_q per (row, column).  y[t][row]. */
static void mul_mat_q(const otensor* w, const float* x, int N, float* y) {
    const int K = w->ne0, M = w->ne1;
    const size_t rb = row_bytes(w->type, K);
    uint8_t* xq = (uint8_t*) malloc(rb * (size_t) N);
    for (int t = 0; t < N; ++t) {
        if (w->type == T_Q4_0) orc_quantize_row_q4_0(x + (size_t) t * K, xq + rb * t, K);
        else orc_quantize_row_q4_1(x + (size_t) t * K, xq + rb * t, K);
    }
    #pragma omp parallel for num_threads(nthreads()) schedule(static)
    for (int r = 0; r < M; ++r) {
        const uint8_t* wr = w->data + rb * (size_t) r;
        for (int t = 0; t < N; ++t)
            y[(size_t) t * M + r] = (w->type == T_Q4_0) ? orc_vec_dot_q4_0(K, wr, xq + rb * t)
                                                         : orc_vec_dot_q4_1(K, wr, xq + rb * t);
    }
    free(xq);
}

static void get_row(const otensor* t, int r, float* y) {
    const uint8_t* p = t->data + row_bytes(t->type, t->ne0) * (size_t) r;
    switch (t->type) {
        case T_F32: memcpy(y, p, 4u * (size_t) t->ne0); break;
        case T_F16: for (int i = 0; i < t->ne0; ++i) { uint16_t h; memcpy(&h, p + 2 * i, 2); y[i] = orc_fp16_to_fp32(h); } break;
        case T_Q4_0: orc_dequantize_row_q4_0(p, y, t->ne0); break;
        default: orc_dequantize_row_q4_1(p, y, t->ne0); break;
    }
}

/* y = g * rms_norm(x) for N rows (llama.cpp:981-986: mul(repeat(g), norm)) */
static void norm_mul(const float* x, const otensor* g, int K, int N, float* y) {
    orc_rms_norm(x, K, N, y);
    const float* gv = (const float*) g->data;
    for (int t = 0; t < N; ++t)
        for (int i = 0; i < K; ++i) y[(size_t) t * K + i] = gv[i] * y[(size_t) t * K + i];
}

/* llama_eval_internal (llama.cpp:927-1197) */
int orc_eval(orc_model* m, const int* tokens, int N, int n_past, int logits_all, float* logits_out) {
    const int E = m->n_embd, F = m->n_ff, H = m->n_head, V = m->n_vocab, C = m->n_ctx;
    const int hd = E / H;
    if (n_past + N > C || N <= 0) return 1;
    float* x = (float*) malloc(sizeof(float) * (size_t) N * E);
    float* cur = (float*) malloc(sizeof(float) * (size_t) N * E);
    float* qv = (float*) malloc(sizeof(float) * (size_t) N * E);
    float* kv = (float*) malloc(sizeof(float) * (size_t) N * E);
    float* vv = (float*) malloc(sizeof(float) * (size_t) N * E);
    float* tmp = (float*) malloc(sizeof(float) * (size_t) N * E);
    float* a = (float*) malloc(sizeof(float) * (size_t) N * F);
    float* bb = (float*) malloc(sizeof(float) * (size_t) N * F);
    for (int t = 0; t < N; ++t) get_row(&m->tok, tokens[t], x + (size_t) t * E);
    for (int il = 0; il < m->n_layer; ++il) {
        const olayer* l = &m->L[il];
        norm_mul(x, &l->an, E, N, cur);
        mul_mat_q(&l->wq, cur, N, tmp); orc_rope(tmp, hd, H, N, n_past, qv);
        mul_mat_q(&l->wk, cur, N, tmp); orc_rope(tmp, hd, H, N, n_past, kv);
        mul_mat_q(&l->wv, cur, N, vv);
        uint16_t* K16 = m->kc + (size_t) il * C * E;
        uint16_t* V16 = m->vc + (size_t) il * C * E;
        for (int t = 0; t < N; ++t)
            for (int i = 0; i < E; ++i) {
                K16[(size_t) (n_past + t) * E + i] = orc_fp32_to_fp16(kv[(size_t) t * E + i]);
                V16[(size_t) i * C + n_past + t] = orc_fp32_to_fp16(vv[(size_t) t * E + i]);
            }
        orc_attention(K16, V16, qv, E, H, C, n_past, N, cur);
        mul_mat_q(&l->wo, cur, N, tmp);
        for (size_t i = 0; i < (size_t) N * E; ++i) x[i] = tmp[i] + x[i];        /* llama.cpp:1071 */
        norm_mul(x, &l->fn, E, N, cur);
        mul_mat_q(&l->w3, cur, N, a);                                            /* llama.cpp:1085 */
        mul_mat_q(&l->w1, cur, N, bb);                                           /* llama.cpp:1089 */
        orc_silu(bb, N * F, bb);
        for (size_t i = 0; i < (size_t) N * F; ++i) bb[i] = bb[i] * a[i];      /* llama.cpp:1096 */
        mul_mat_q(&l->w2, bb, N, tmp);
        for (size_t i = 0; i < (size_t) N * E; ++i) x[i] = tmp[i] + x[i];        /* llama.cpp:1103 */
    }
    norm_mul(x, &m->norm, E, N, cur);
    float* lg = (float*) malloc(sizeof(float) * (size_t) N * V);
    mul_mat_q(&m->out, cur, N, lg);
    if (logits_all) memcpy(logits_out, lg, sizeof(float) * (size_t) N * V);
    else memcpy(logits_out, lg + (size_t) (N - 1) * V, sizeof(float) * (size_t) V);
    free(lg); free(x); free(cur); free(qv); free(kv); free(vv); free(tmp); free(a); free(bb);
    return 0;
}
