// matvec_q41.hip -- bit-faithful Q4_1 matrix x quantized-activation product
// (the 13B Q4_1 configuration), prompt and decode, any K % 256 == 0.
//
// Reference arithmetic (ggml_vec_dot_q4_1 AVX2, ggml.c:2188-2258), x = weight
// row, y = activation, per block i in order and chain j = 0..7:
//   p_j   = sum over e in {2j, 2j+1, 16+2j, 17+2j} of qx_e * qy_e     (exact int)
//   acc_j = fmaf(dx*dy, (float) p_j, acc_j)
//   acc_j = fmaf(j even ? dx*my : mx*dy, (float) S_j, acc_j)
//           S_j = sum of qx (j even) or qy (j odd) over elements 8(j/2)..8(j/2)+7
//   off   = off + mx*my
// result = ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7)) + off*32.
// The activation is quantized by quantize_row_q4_1 (AVX2, ggml.c:847-920).
//
// Layout: the octet image of matvec_q4.hip with chain j's 16-bit group
// a(i,j) = qs[j] | qs[8+j] << 8 (the 4 nibbles of chain j, unsigned), and two
// float4 per lane and chunk (d, then m).  The weight sums S_j of even chains
// are formed on the fly: per-byte nibble sums, a quad DPP sum, and a half-row
// mirror between the two quads of a row.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {
using namespace mv;

struct P41 {
    const uint4 * nib;
    const float4 * scl;       // [g][NC][2][64]: d, then m
    int M, K, nb, NC;
    const float * x;
    const float * g;
    ActQ xq;
    const StepParams * sp;
    int n_tokens, tok0, out_tok0;
    float * y;
    uint16_t * q16;
    uint16_t * kc;
    uint16_t * vc;
    const float2 * rope;
    int n_embd, head_dim, n_ctx;
    int kv32;                   // f32 KV cache and queries (f16_kv = false)
    const uint16_t * silu_tab;
    ActQ out_q;
};

// ---------------------------------------------------------------------------
// NT threads = NT/64 row groups of 8 rows; T tokens; D chunks in flight.
// ---------------------------------------------------------------------------
template <int NT, int T, int PRO, int EPI, int D>
__global__ __launch_bounds__(NT) void k_matvec_q41(P41 P) {
    constexpr int NW = NT / 64;
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int j = lane & 7;
    const int r = lane >> 3;
    const int g = blockIdx.x * NW + wave;
    const int t0 = blockIdx.y * T;
    const int nt = min(T, P.n_tokens - t0);
    if (nt <= 0) return;
    const int nb = P.nb, NC = P.NC, K = P.K;

    // LDS carve
    uint32_t * act_base = (uint32_t *) smem;                                   // T * nb * 32 B
    float * dyv_base = (float *) (smem + (size_t) T * nb * 32);               // T * NC * 32
    float * myv_base = dyv_base + (size_t) T * NC * 32;                       // T * NC * 32
    float * ys_base = myv_base + (size_t) T * NC * 32;                        // T * nb * 4
    float * sbuf = ys_base + (size_t) T * nb * 4;                             // NW * T * 1024
    double * red = (double *) (sbuf + (size_t) NW * T * 1024);              // T * NW
    float * s_scale = (float *) (red + T * NW);                              // T

    // 1. weight stream (clamped unconditional loads: exact vmcnt bookkeeping)
    const uint4 * nib = P.nib + (size_t) g * NC * 4 * 64 + lane;
    const float4 * scl = P.scl + (size_t) g * NC * 128 + lane;
    const int nsub = nb / 8;
    uint4 W[D][4];
    float4 SD[D], SM[D];
#define LVK_ISSUE41(slot, cc)                                                                      \
    do {                                                                                           \
        const int cl_ = min((cc), NC - 1);                                                         \
        _Pragma("unroll") for (int sb = 0; sb < 4; ++sb)                                           \
            W[slot][sb] = ld_nt(nib + (size_t) min(cl_ * 4 + sb, nsub - 1) * 64);                  \
        SD[slot] = scl[(size_t) cl_ * 128];                                                        \
        SM[slot] = scl[(size_t) cl_ * 128 + 64];                                                   \
    } while (0)
#pragma unroll
    for (int d = 0; d < D; ++d) LVK_ISSUE41(d, d);

    // 2. activation table (RMSNorm + quantize, plain quantize, or pre-quantized)
    if constexpr (PRO == PRO_NORM || PRO == PRO_ACTF) {
        const int nunits = K / 8;
        if constexpr (PRO == PRO_NORM) {
            // ggml.c:6058-6076: float squares summed in double (RMSNorm order)
            for (int tt = 0; tt < T; ++tt) {
                double acc = 0.0;
                if (tt < nt) {
                    const float * xr = P.x + (size_t) (P.tok0 + t0 + tt) * K;
                    for (int u = tid; u < nunits; u += NT) {
                        const float4 a = ((const float4 *) xr)[2 * u], b = ((const float4 *) xr)[2 * u + 1];
                        const float e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                        for (int q = 0; q < 8; ++q) { const float sq = e[q] * e[q]; acc += (double) sq; }
                    }
                }
                acc = wave_sum_d(acc);
                if (lane == 0) red[tt * NW + wave] = acc;
            }
            __syncthreads();
            if (tid < T) {
                double s = 0.0;
                for (int w = 0; w < NW; ++w) s += red[tid * NW + w];
                // rows tid >= nt summed nothing: s == 0 never re-reads x
                const float mean = rms_mean(s, P.x + (size_t) (P.tok0 + t0 + tid) * K, K);
                s_scale[tid] = 1.0f / sqrtf(mean + 1e-6f);
            }
            __syncthreads();
        }
        for (int tt = 0; tt < nt; ++tt) {
            const float * xr = P.x + (size_t) (P.tok0 + t0 + tt) * K;
            const float scale = PRO == PRO_NORM ? s_scale[tt] : 1.0f;
            uint32_t * act = act_base + (size_t) tt * nb * 8;
            float * dyv = dyv_base + (size_t) tt * NC * 32;
            float * myv = myv_base + (size_t) tt * NC * 32;
            float * ys = ys_base + (size_t) tt * nb * 4;
            // whole quads stay together: nunits % 4 == 0 and NT % 4 == 0
            for (int u0 = 0; u0 < nunits; u0 += NT) {
                const int u = min(u0 + tid, nunits - 1);
                const float4 a = ((const float4 *) xr)[2 * u], b = ((const float4 *) xr)[2 * u + 1];
                float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
                if constexpr (PRO == PRO_NORM) {
                    const float4 ga = ((const float4 *) P.g)[2 * u], gb = ((const float4 *) P.g)[2 * u + 1];
                    const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float yn = v[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                        v[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                    }
                }
                float d, m;
                uint32_t qw;
                q41_quad(v, d, m, qw);
                // gather the block's 4 qs words into every lane of the quad
                uint32_t qs[4];
                qs[0] = __builtin_bit_cast(uint32_t, quad_bcast<0>(__builtin_bit_cast(float, qw)));
                qs[1] = __builtin_bit_cast(uint32_t, quad_bcast<1>(__builtin_bit_cast(float, qw)));
                qs[2] = __builtin_bit_cast(uint32_t, quad_bcast<2>(__builtin_bit_cast(float, qw)));
                qs[3] = __builtin_bit_cast(uint32_t, quad_bcast<3>(__builtin_bit_cast(float, qw)));
                if (u0 + tid < nunits && (u & 3) == 0) act41_store(act, dyv, myv, ys, u >> 2, qs, d, m);
            }
        }
    } else {
        for (int tt = 0; tt < nt; ++tt) {
            const int t = t0 + tt + P.tok0;
            uint32_t * act = act_base + (size_t) tt * nb * 8;
            float * dyv = dyv_base + (size_t) tt * NC * 32;
            float * myv = myv_base + (size_t) tt * NC * 32;
            float * ys = ys_base + (size_t) tt * nb * 4;
            for (int b = tid; b < nb; b += NT) {
                const uint4 q4 = P.xq.qs[(size_t) t * P.xq.nb + b];
                const uint32_t qs[4] = {q4.x, q4.y, q4.z, q4.w};
                act41_store(act, dyv, myv, ys, b, qs, P.xq.d[(size_t) t * P.xq.nb + b],
                            P.xq.m[(size_t) t * P.xq.nb + b]);
            }
        }
    }
    __syncthreads();

    // 3. the faithful chains
    float acc[T], off[T];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) { acc[tt] = 0.0f; off[tt] = 0.0f; }
    const bool even = (j & 1) == 0;
    const bool other = (j == 2 || j == 4);
    const uint32_t wsh = j >= 4 ? 8u : 0u;
    float * sw = sbuf + (size_t) wave * T * 1024;
    const int ngrp = (NC + D - 1) / D;
    for (int gi = 0; gi < ngrp; ++gi) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int c = gi * D + d;
            if (c < NC) {
                // products of blocks 32c + 8m + j of this lane's row (ggml.c:2205-2212):
                // s = dx*dy, ce = dx*my, co = mx*dy, mm = mx*my
#pragma unroll
                for (int tt = 0; tt < T; ++tt) {
                    const float4 dy = *(const float4 *) (dyv_base + (size_t) tt * NC * 32 + (size_t) c * 32 + j * 4);
                    const float4 my = *(const float4 *) (myv_base + (size_t) tt * NC * 32 + (size_t) c * 32 + j * 4);
                    // slot 8m + j = block 32c + 8m + j (block order within the chunk)
                    float * sl = sw + tt * 1024 + r * 32 + j;
                    const float dxa[4] = {SD[d].x, SD[d].y, SD[d].z, SD[d].w};
                    const float mxa[4] = {SM[d].x, SM[d].y, SM[d].z, SM[d].w};
                    const float dya[4] = {dy.x, dy.y, dy.z, dy.w};
                    const float mya[4] = {my.x, my.y, my.z, my.w};
#pragma unroll
                    for (int mq = 0; mq < 4; ++mq) {
                        sl[mq * 8] = dxa[mq] * dya[mq];
                        sl[256 + mq * 8] = dxa[mq] * mya[mq];
                        sl[512 + mq * 8] = mxa[mq] * dya[mq];
                        sl[768 + mq * 8] = mxa[mq] * mya[mq];
                    }
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int tt = 0; tt < T; ++tt) {
                    const float * srow = sw + tt * 1024 + r * 32;
                    const float * xrow = srow + (even ? 256 : 512);
                    const float * mrow = srow + 768;
                    const uint32_t * act = act_base + (size_t) tt * nb * 8;
                    const float * ys = ys_base + (size_t) tt * nb * 4;
#pragma unroll
                    for (int sb = 0; sb < 4; ++sb) {
                        if (c * 4 + sb < nsub) {
                            const uint32_t wd[4] = {W[d][sb].x, W[d][sb].y, W[d][sb].z, W[d][sb].w};
#pragma unroll
                            for (int pp = 0; pp < 2; ++pp) {
                                const int u = c * 8 + sb * 2 + pp;            // group of 4 blocks
                                const int bi = sb * 8 + pp * 4;               // first block within chunk
                                const uint4 a = *(const uint4 *) (act + ((size_t) u * 8 + j) * 4);
                                const float4 s4 = *(const float4 *) (srow + bi);
                                const float4 x4 = *(const float4 *) (xrow + bi);
                                const float4 m4 = *(const float4 *) (mrow + bi);
                                const float4 y4 = *(const float4 *) (ys + (size_t) u * 16 + (j >> 1) * 4);
                                const uint32_t w01 = wsum_word(wd[2 * pp], other, wsh);
                                const uint32_t w23 = wsum_word(wd[2 * pp + 1], other, wsh);
                                const float S[4] = {even ? (float) (w01 & 0xFFFFu) : y4.x, even ? (float) (w01 >> 16) : y4.y,
                                                    even ? (float) (w23 & 0xFFFFu) : y4.z, even ? (float) (w23 >> 16) : y4.w};
                                const int p[4] = {udot8(wd[2 * pp], a.x), udot8(wd[2 * pp], a.y),
                                                  udot8(wd[2 * pp + 1], a.z), udot8(wd[2 * pp + 1], a.w)};
                                const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
                                const float xv[4] = {x4.x, x4.y, x4.z, x4.w};
                                const float mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
                                for (int k = 0; k < 4; ++k) {
                                    acc[tt] = __builtin_fmaf(sv[k], (float) p[k], acc[tt]);
                                    acc[tt] = __builtin_fmaf(xv[k], S[k], acc[tt]);
                                    off[tt] = off[tt] + mv[k];
                                }
                            }
                        }
                    }
                }
            }
            LVK_ISSUE41(d, c + D);
#pragma unroll
            for (int tt = 0; tt < T; ++tt) { asm volatile("" : "+v"(acc[tt]), "+v"(off[tt])); }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#undef LVK_ISSUE41

    // 4. epilogue
    const int row = g * 8 + r;
    float res[T];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) {
        const float h = octet_reduce(acc[tt]);
        const float o = off[tt] * 32.0f;        // acc_offset * QK (ggml.c:2249)
        res[tt] = h + o;
    }
    if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (tt < nt && j == 0) P.y[(size_t) (P.out_tok0 + t0 + tt) * P.M + row] = res[tt];
    } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (tt < nt && j == 0) {
                float * yp = P.y + (size_t) (P.out_tok0 + t0 + tt) * P.M + row;
                *yp = res[tt] + *yp;                 // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
            }
    } else if constexpr (EPI == EPI_QKV) {
        const int E = P.n_embd, hd = P.head_dim;
        const int which = row / E;
        const int e = row - which * E;
        const int n_past = P.sp->n_past;
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
            const float other_r = __shfl_xor(res[tt], 8);
            if (tt < nt && j == 0) {
                const int pos = n_past + t0 + tt;
                if (which < 2) {
                    // ggml_compute_forward_rope_f32 mode 0 (ggml.c:7209-7223)
                    const int i0 = e % hd;
                    const float2 cs = P.rope[(size_t) pos * (hd / 2) + (i0 >> 1)];
                    float out;
                    if ((i0 & 1) == 0) { const float a = res[tt] * cs.x, b = other_r * cs.y; out = a - b; }
                    else               { const float a = other_r * cs.y, b = res[tt] * cs.x; out = a + b; }
                    if (which == 0) kv_store(P.q16, (size_t) (t0 + tt) * E + e, out, P.kv32);
                    else            kv_store(P.kc, (size_t) pos * E + e, out, P.kv32);
                } else {
                    kv_store(P.vc, (size_t) e * P.n_ctx + pos, res[tt], P.kv32);
                }
            }
        }
    } else if constexpr (EPI == EPI_SWIGLU) {
        // WG = 8 waves = rows [64b, 64b+64) of the fused W1|W3 image (interleaved
        // per 4 rows): wave k rows 0-3 are w1 rows 32b+4k..+3, rows 4-7 the w3 rows
        __syncthreads();
        float * ures = (float *) smem;                               // T x 64 floats
        float * ub = ures + T * 64;                                  // T x 32 u values
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (j == 0) ures[tt * 64 + wave * 8 + r] = res[tt];
        __syncthreads();
        if (tid < T * 32) {
            const int tt = tid >> 5, e = tid & 31;
            if (tt < nt) {
                const float a1 = ures[tt * 64 + (e >> 2) * 8 + (e & 3)];        // w1 x
                const float a3 = ures[tt * 64 + (e >> 2) * 8 + 4 + (e & 3)];    // w3 x
                const float sl = f16_to_f32(P.silu_tab[f32_to_f16(a1)]);   // ggml_vec_silu_f32 (ggml.c:2495)
                ub[tt * 32 + e] = sl * a3;                                  // ggml_mul (llama.cpp:1096)
            }
        }
        __syncthreads();
        if (tid < T * 32) {
            const int tt = tid >> 5, k = tid & 31;
            if (tt < nt && k < 4) {
                float d, m;
                uint32_t qw;
                q41_block_lds(ub + tt * 32, k, d, m, qw);
                const int t = P.out_tok0 + t0 + tt;
                const int blk = blockIdx.x;
                ((uint32_t *) (P.out_q.qs + (size_t) t * P.out_q.nb + blk))[k] = qw;
                if (k == 0) {
                    P.out_q.d[(size_t) t * P.out_q.nb + blk] = d;
                    P.out_q.m[(size_t) t * P.out_q.nb + blk] = m;
                }
            }
        }
    }
}

template <int NT, int T, int PRO, int EPI, int D>
hipError_t go41(const P41 & P, int ngroups, int ntok, hipStream_t s) {
    constexpr int NW = NT / 64;
    size_t lds = (size_t) T * P.nb * 32 + (size_t) 2 * T * P.NC * 128 + (size_t) T * P.nb * 16 +
                 (size_t) NW * T * 4096 + T * NW * 8 + 64;
    if (EPI == EPI_SWIGLU) lds = std::max(lds, (size_t) T * 384);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid(ngroups / NW, (ntok + T - 1) / T);
    LVK_LAUNCH((k_matvec_q41<NT, T, PRO, EPI, D>), grid, dim3(NT), lds, s, P);
    return hipGetLastError();
}

template <int NT, int T, int D>
hipError_t dispatch41(const P41 & P, int pro, int epi, int ng, int N, hipStream_t s) {
    switch (epi) {
        case EPI_QKV: if (pro == PRO_NORM) return go41<NT, T, PRO_NORM, EPI_QKV, D>(P, ng, N, s); break;
        case EPI_STORE:
            if (pro == PRO_NORM) return go41<NT, T, PRO_NORM, EPI_STORE, D>(P, ng, N, s);
            if (pro == PRO_ACTQ) return go41<NT, T, PRO_ACTQ, EPI_STORE, D>(P, ng, N, s);
            if (pro == PRO_ACTF) return go41<NT, T, PRO_ACTF, EPI_STORE, D>(P, ng, N, s);
            break;
        case EPI_RESID:
            if (pro == PRO_ACTQ) return go41<NT, T, PRO_ACTQ, EPI_RESID, D>(P, ng, N, s);
            break;
    }
    return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_matvec_q41(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.M % 8 || L.w.K % 256) return hipErrorInvalidValue;
    P41 P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.M = L.w.M; P.K = L.w.K; P.nb = L.w.K / 32; P.NC = (P.nb + 31) / 32;
    P.x = L.x; P.g = L.g; P.xq = L.xq; P.sp = L.sp;
    P.n_tokens = L.n_tokens; P.tok0 = L.tok0; P.out_tok0 = L.out_tok0;
    P.y = L.y; P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx; P.kv32 = L.kv32;
    P.silu_tab = L.silu_tab; P.out_q = L.out_q;
    const int ng = L.w.M / 8;
    const int N = L.n_tokens;
    if (epi == EPI_SWIGLU) {
        if (pro != PRO_NORM || ng % 8) return hipErrorInvalidValue;
        return N > 1 ? go41<512, 2, PRO_NORM, EPI_SWIGLU, 2>(P, ng, N, s)
                     : go41<512, 1, PRO_NORM, EPI_SWIGLU, 2>(P, ng, N, s);
    }
    if (ng % 2) return hipErrorInvalidValue;
    return N > 1 ? dispatch41<128, 2, 2>(P, pro, epi, ng, N, s) : dispatch41<128, 1, 4>(P, pro, epi, ng, N, s);
}

}  // namespace lvk
