// matvec_q4.hip -- bit-faithful Q4_0 matrix x quantized-activation product for
// gfx950, with fused prologues (RMSNorm + activation quantizer, or a
// pre-quantized input) and epilogues (residual add, RoPE + KV append,
// SwiGLU + requantize, plain store).
//
// Reference arithmetic reproduced bit-for-bit:
//   ggml_compute_forward_mul_mat_q_f32 (ggml.c:6510-6696) quantizes every
//   activation column with quantize_row_q4_0 (AVX2, ggml.c:621-685) and runs
//   one ggml_vec_dot_q4_0 (AVX2, ggml.c:1950-2026) per (row, column):
//   8 fp32 accumulators acc_j = fma(dw_i*dx_i, P_ij, acc_j) over blocks i in
//   order, P_ij = exact int sum over block elements 4j..4j+3, then
//   ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7)).
//
// MI355X mapping ("octet" layout):
//   * one wavefront = 8 weight rows; lane 8r+j owns row r's accumulator chain
//     j -- the reference's 8 sequential fp32 chains per row are the only
//     parallelism inside a row, so each becomes one lane;
//   * the weight image is pre-swizzled so a wave streams 1 KiB per
//     global_load_dwordx4 (nibble slices of 8 blocks) plus 1 KiB of block
//     scales per 32 blocks; nibbles are pre-XORed to signed 4-bit so one
//     v_dot8_i32_i4 against a zero-padded activation word gives P_ij exactly;
//   * the 32 block-scale products dw*dx of a chunk are formed once per row
//     (4 per lane) and exchanged through a per-wave LDS slot, so the inner
//     loop is dot8 + cvt + fma per block per lane;
//   * weight loads are issued unconditionally D chunks ahead (clamped
//     addresses), keeping hipcc's vmcnt bookkeeping exact.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {
using namespace mv;

constexpr int CB = 32;    // blocks per chunk (one float4 of scales per lane)

struct Params {
    const uint4 * nib;
    const float4 * scl;
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
// Prologue A (PRO_NORM): x[t] -> rms_norm -> * g -> quantize_row_q4_0, into
// the LDS table.  ggml.c:6058-6076 then llama.cpp:984.  The double sum of
// squares is reduced as a tree; rms_mean (lvk_device.h) returns the index-order
// mean (a re-sum when the tree's lies near a float rounding boundary).
// Work unit = 8 consecutive elements; a block's 4 units are a thread quad.
// ---------------------------------------------------------------------------
template <int NT, int T, int UMAX, bool PRE>
__device__ void prologue_norm(const Params & P, int t0, int nt, uint32_t * act_base, float * dxp_base,
                              double * red, float * s_scale, const float4 (&xv)[UMAX][2],
                              const float4 (&gv)[UMAX][2]) {
    const int tid = threadIdx.x;
    const int K = P.K;
    const int nunits = K / 8;
    auto ldx = [&](int tt, int k, float v[8]) {
        float4 a, b;
        if constexpr (PRE) { a = xv[k][0]; b = xv[k][1]; }
        else {
            const float4 * xp = (const float4 *) (P.x + (size_t) (P.tok0 + t0 + tt) * K + (size_t) (k * NT + tid) * 8);
            a = xp[0]; b = xp[1];
        }
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    };
    auto ldg = [&](int k, float v[8]) {
        float4 a, b;
        if constexpr (PRE) { a = gv[k][0]; b = gv[k][1]; }
        else { const float4 * gp = (const float4 *) (P.g + (size_t) (k * NT + tid) * 8); a = gp[0]; b = gp[1]; }
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    };
    for (int tt = 0; tt < T; ++tt) {
        double acc = 0.0;
#pragma unroll
        for (int k = 0; k < UMAX; ++k) {
            if (k * NT + tid < nunits && tt < nt) {
                float e[8];
                ldx(tt, k, e);
#pragma unroll
                for (int q = 0; q < 8; ++q) { const float sq = e[q] * e[q]; acc += (double) sq; }
            }
        }
        acc = warp_sum_d(acc);
        if ((tid & 63) == 0) red[tt * (NT / 64) + (tid >> 6)] = acc;
    }
    __syncthreads();
    if (tid < T) {
        double s = 0.0;
        for (int w = 0; w < NT / 64; ++w) s += red[tid * (NT / 64) + w];
        // rows tid >= nt summed nothing: s == 0 never re-reads x
        const float mean = rms_mean(s, P.x + (size_t) (P.tok0 + t0 + tid) * K, K);
        s_scale[tid] = 1.0f / sqrtf(mean + 1e-6f);
    }
    __syncthreads();
    for (int tt = 0; tt < nt; ++tt) {
        const float scale = s_scale[tt];
        uint32_t * act = act_base + (size_t) tt * P.nb * 8;
        float * dxp = dxp_base + (size_t) tt * P.NC * 32;
#pragma unroll
        for (int k = 0; k < UMAX; ++k) {
            if (k * NT >= nunits) break;
            const int u = k * NT + tid;
            const bool live = u < nunits;
            float v[8], gg[8];
            if (live) { ldx(tt, k, v); ldg(k, gg); }
            else {
#pragma unroll
                for (int e = 0; e < 8; ++e) { v[e] = 0.0f; gg[e] = 0.0f; }
            }
            float amax = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float yn = v[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                v[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                const float a = fabsf(v[e]);
                amax = a > amax ? a : amax;
            }
            const float o0 = quad_bcast<0>(amax), o1 = quad_bcast<1>(amax);
            const float o2 = quad_bcast<2>(amax), o3 = quad_bcast<3>(amax);
            const float m01 = o1 > o0 ? o1 : o0, m23 = o3 > o2 ? o3 : o2;
            amax = m23 > m01 ? m23 : m01;
            const float d = amax / 7.0f;                              // ggml.c:651
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
            const uint32_t w = q40_pack8(v, id);
            if (live) act_store(act, dxp, u >> 2, u & 3, w, d, (u & 3) == 0);
        }
    }
}

// Prologue B (PRO_ACTQ): pre-quantized Q4_0 blocks (d + qs) -> LDS table
template <int NT, int T, int BMAX, bool PRE>
__device__ void prologue_actq(const Params & P, int t0, int nt, uint32_t * act_base, float * dxp_base,
                              const uint4 (&qv)[BMAX], const float (&dv)[BMAX]) {
    const int tid = threadIdx.x;
    if constexpr (PRE) {
#pragma unroll
        for (int k = 0; k < BMAX; ++k) {
            const int b = k * NT + tid;
            if (b < P.nb) {
                act_store(act_base, dxp_base, b, 0, qv[k].x, dv[k], true);
                act_store(act_base, dxp_base, b, 1, qv[k].y, 0.0f, false);
                act_store(act_base, dxp_base, b, 2, qv[k].z, 0.0f, false);
                act_store(act_base, dxp_base, b, 3, qv[k].w, 0.0f, false);
            }
        }
    } else {
        for (int tt = 0; tt < nt; ++tt) {
            const int t = t0 + tt + P.tok0;
            uint32_t * act = act_base + (size_t) tt * P.nb * 8;
            float * dxp = dxp_base + (size_t) tt * P.NC * 32;
            for (int b = tid; b < P.nb; b += NT) {
                const uint4 qs = P.xq.qs[(size_t) t * P.nb + b];
                const float d = P.xq.d[(size_t) t * P.nb + b];
                act_store(act, dxp, b, 0, qs.x, d, true);
                act_store(act, dxp, b, 1, qs.y, 0.0f, false);
                act_store(act, dxp, b, 2, qs.z, 0.0f, false);
                act_store(act, dxp, b, 3, qs.w, 0.0f, false);
            }
        }
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// NT threads = NT/64 row groups of 8 rows; T tokens per lane; D chunks of 32
// blocks in flight; UMAX = units (PRO_NORM) or blocks (PRO_ACTQ) per thread.
// KT > 0 compiles the row length in: every load count is then exact and
// static (no clamped duplicate requests); KT == 0 is the generic path.
// ---------------------------------------------------------------------------
template <int NT, int T, int UMAX, int PRO, int EPI, int D, int KT>
__global__ __launch_bounds__(NT) void k_matvec_q40(Params P) {
    constexpr bool PRE = (T == 1);
    constexpr int NW = NT / 64;
    constexpr int UM = KT == 0 ? UMAX : (PRO == PRO_NORM ? (KT / 8 + NT - 1) / NT : (KT / 32 + NT - 1) / NT);
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int j = lane & 7;
    const int r = lane >> 3;
    const int g = blockIdx.x * NW + wave;      // row group
    const int t0 = blockIdx.y * T;
    const int nt = min(T, P.n_tokens - t0);
    if (nt <= 0) return;
    const int nb = KT ? KT / 32 : P.nb;
    const int NC = KT ? (KT / 32 + CB - 1) / CB : P.NC;
    const int K = KT ? KT : P.K;

    // LDS carve (16-byte aligned pieces)
    uint32_t * act_base = (uint32_t *) smem;                                   // T * nb * 32 B
    float * dxp_base = (float *) (smem + (size_t) T * nb * 32);               // T * NC * 128 B
    float * sbuf = dxp_base + (size_t) T * NC * 32;                           // NW * 2 * T * 256 floats
    double * red = (double *) (sbuf + (size_t) NW * 2 * T * 256);            // T * NW doubles
    float * s_scale = (float *) (red + T * NW);                              // T floats

    // 1. prologue inputs into registers (issued first: in-order vmcnt)
    float4 xv[UM][2];
    float4 gv[UM][2];
    uint4 qv[UM];
    float dv[UM];
    if constexpr (PRE && PRO == PRO_NORM) {
        const int nunits = K / 8;
#pragma unroll
        for (int k = 0; k < UM; ++k) {
            const int u = min(k * NT + tid, nunits - 1);
            const float4 * gp = (const float4 *) (P.g + (size_t) u * 8);
            const float4 * xp = (const float4 *) (P.x + (size_t) (P.tok0 + t0) * K + (size_t) u * 8);
            gv[k][0] = gp[0]; gv[k][1] = gp[1];
            xv[k][0] = xp[0]; xv[k][1] = xp[1];
        }
    }
    if constexpr (PRE && PRO == PRO_ACTQ) {
#pragma unroll
        for (int k = 0; k < UM; ++k) {
            const int b = min(k * NT + tid, nb - 1);
            qv[k] = P.xq.qs[(size_t) (P.tok0 + t0) * nb + b];
            dv[k] = P.xq.d[(size_t) (P.tok0 + t0) * nb + b];
        }
    }

    // 2. weight stream: D chunks ahead.  Generic path: unconditional clamped
    //    loads (keeps hipcc's vmcnt bookkeeping exact); KT path: exact loads.
    const uint4 * nib = P.nib + (size_t) g * NC * 4 * 64 + lane;
    const float4 * scl = P.scl + (size_t) g * NC * 64 + lane;
    const int nsub = nb / 8;                   // valid 8-block sub-chunks
    uint4 W[D][4];
    float4 S[D];
#define LVK_ISSUE(slot, cc)                                                                         \
    do {                                                                                            \
        const int c_ = (cc);                                                                        \
        if (KT == 0 || c_ < NC) {                                                                   \
            const int cl_ = KT ? c_ : min(c_, NC - 1);                                              \
            _Pragma("unroll") for (int sb = 0; sb < 4; ++sb) {                                      \
                if (KT == 0) W[slot][sb] = ld_nt(nib + (size_t) min(cl_ * 4 + sb, nsub - 1) * 64);  \
                else if (cl_ * 4 + sb < nsub) W[slot][sb] = ld_nt(nib + (size_t) (cl_ * 4 + sb) * 64); \
            }                                                                                       \
            S[slot] = scl[(size_t) cl_ * 64];                                                       \
        }                                                                                           \
    } while (0)
#pragma unroll
    for (int d = 0; d < D; ++d) LVK_ISSUE(d, d);

    // 3. activation table
#ifdef LVK_PROBE_NOPRO   // dev probe builds only (tools/probe): time the stream without the prologue
    if (false)
#else
    if constexpr (PRO == PRO_NORM)
#endif
        prologue_norm<NT, T, UM, PRE>(P, t0, nt, act_base, dxp_base, red, s_scale, xv, gv);
    else
        prologue_actq<NT, T, UM, PRE>(P, t0, nt, act_base, dxp_base, qv, dv);
    __syncthreads();

    // 4. the faithful chains: lane j of row r
    float acc[T];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) acc[tt] = 0.0f;
    float * sw = sbuf + (size_t) wave * 2 * T * 256;
    const int ngrp = (NC + D - 1) / D;
#pragma unroll
    for (int gi = 0; gi < ngrp; ++gi) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int c = gi * D + d;
#ifdef LVK_PROBE_NOCOMPUTE   // dev probe builds only: consume the weights trivially
            if (c < NC) acc[0] += __uint_as_float(W[d][0].x ^ W[d][1].y ^ W[d][2].z ^ W[d][3].w) * S[d].x;
            if (false) {
#else
            if (c < NC) {
#endif
                float * sl = sw + (size_t) (c & 1) * T * 256;
                // s = dw * dx for blocks 32c + 8m + j of this lane's row (ggml.c:1968)
#pragma unroll
                for (int tt = 0; tt < T; ++tt) {
                    const float4 dx = *(const float4 *) (dxp_base + (size_t) tt * NC * 32 + (size_t) c * 32 + j * 4);
                    float4 sv;
                    sv.x = S[d].x * dx.x; sv.y = S[d].y * dx.y; sv.z = S[d].z * dx.z; sv.w = S[d].w * dx.w;
                    *(float4 *) (sl + tt * 256 + r * 32 + j * 4) = sv;
                }
                __builtin_amdgcn_wave_barrier();
#pragma unroll
                for (int tt = 0; tt < T; ++tt) {
                    float sa[8][4];
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) {
                        const float4 v = *(const float4 *) (sl + tt * 256 + r * 32 + jj * 4);
                        sa[jj][0] = v.x; sa[jj][1] = v.y; sa[jj][2] = v.z; sa[jj][3] = v.w;
                    }
                    const uint32_t * act = act_base + (size_t) tt * nb * 8;
#pragma unroll
                    for (int sb = 0; sb < 4; ++sb) {
                        if (c * 4 + sb < nsub) {
                            const uint32_t wd[4] = {W[d][sb].x, W[d][sb].y, W[d][sb].z, W[d][sb].w};
#pragma unroll
                            for (int pp = 0; pp < 2; ++pp) {
                                const int bi = sb * 8 + pp * 4;                 // block within chunk
                                const uint4 a = *(const uint4 *) (act + ((size_t) (c * 8 + sb * 2 + pp) * 8 + j) * 4);
                                const int p0 = dot8(wd[2 * pp], a.x);
                                const int p1 = dot8(wd[2 * pp], a.y);
                                const int p2 = dot8(wd[2 * pp + 1], a.z);
                                const int p3 = dot8(wd[2 * pp + 1], a.w);
                                acc[tt] = __builtin_fmaf(sa[(bi + 0) & 7][(bi + 0) >> 3], (float) p0, acc[tt]);
                                acc[tt] = __builtin_fmaf(sa[(bi + 1) & 7][(bi + 1) >> 3], (float) p1, acc[tt]);
                                acc[tt] = __builtin_fmaf(sa[(bi + 2) & 7][(bi + 2) >> 3], (float) p2, acc[tt]);
                                acc[tt] = __builtin_fmaf(sa[(bi + 3) & 7][(bi + 3) >> 3], (float) p3, acc[tt]);
                            }
                        }
                    }
                }
            }
            LVK_ISSUE(d, c + D);
            // keep chunks in program order (pinned chain values): otherwise the
            // fully unrolled KT path sinks all arithmetic below all LDS reads
#pragma unroll
            for (int tt = 0; tt < T; ++tt) asm volatile("" : "+v"(acc[tt]));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#undef LVK_ISSUE

    // 5. epilogue
    const int row = g * 8 + r;
    float res[T];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) res[tt] = octet_reduce(acc[tt]);

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
        const int which = row / E;          // 0 q, 1 k, 2 v (uniform per wave: E % 8 == 0)
        const int e = row - which * E;
        const int n_past = P.sp->n_past;
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
            const float other = __shfl_xor(res[tt], 8);   // row e^1 lives in lanes of row r^1
            if (tt < nt && j == 0) {
                const int pos = n_past + t0 + tt;
                if (which < 2) {
                    // ggml_compute_forward_rope_f32 mode 0 (ggml.c:7209-7223)
                    const int i0 = e % hd;
                    const float2 cs = P.rope[(size_t) pos * (hd / 2) + (i0 >> 1)];
                    float out;
                    if ((i0 & 1) == 0) { const float a = res[tt] * cs.x, b = other * cs.y; out = a - b; }
                    else               { const float a = other * cs.y, b = res[tt] * cs.x; out = a + b; }
                    if (which == 0) kv_store(P.q16, (size_t) (t0 + tt) * E + e, out, P.kv32);
                    else            kv_store(P.kc, (size_t) pos * E + e, out, P.kv32);
                } else {
                    kv_store(P.vc, (size_t) e * P.n_ctx + pos, res[tt], P.kv32);
                }
            }
        }
    } else if constexpr (EPI == EPI_SWIGLU) {
        // WG = 8 waves = rows [64b, 64b+64) of the fused W1|W3 image, which is
        // interleaved per 4 rows: wave k rows 0-3 are w1 rows 32b+4k..+3, rows
        // 4-7 the matching w3 rows (llama.cpp:1085-1096)
        __syncthreads();
        float * ures = (float *) smem;                               // T x 64 floats
        uint32_t * scratch = (uint32_t *) (smem + (size_t) T * 64 * 4);
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (j == 0) ures[tt * 64 + wave * 8 + r] = res[tt];
        __syncthreads();
        const int blk = blockIdx.x;
        for (int tt = wave * 2 + (lane >> 5); tt < nt; tt += NW * 2) {
            const int e = lane & 31;
            const float a1 = ures[tt * 64 + (e >> 2) * 8 + (e & 3)];        // w1 x
            const float a3 = ures[tt * 64 + (e >> 2) * 8 + 4 + (e & 3)];    // w3 x
            const float sl = f16_to_f32(P.silu_tab[f32_to_f16(a1)]);   // ggml_vec_silu_f32 (ggml.c:2495)
            const float u = sl * a3;                                    // ggml_mul (llama.cpp:1096)
            const int t = P.out_tok0 + t0 + tt;
            quantize32_q40(u, lane, P.out_q.d + (size_t) t * P.out_q.nb + blk,
                           P.out_q.qs + (size_t) t * P.out_q.nb + blk, scratch + (tid >> 5) * 4);
        }
    }
}

// ---------------------------------------------------------------------------
// host launch
// ---------------------------------------------------------------------------
namespace {
template <int NT, int T, int UMAX, int PRO, int EPI, int D, int KT>
hipError_t go1(const Params & P, int ngroups, int ntok, hipStream_t s) {
    constexpr int NW = NT / 64;
    size_t lds = (size_t) T * P.nb * 32 + (size_t) T * P.NC * 128 + (size_t) NW * 2 * T * 1024 + T * NW * 8 + 64;
    if (EPI == EPI_SWIGLU) lds = std::max(lds, (size_t) T * 256 + NT / 2 * 16);
    if (lds > 160 * 1024) return hipErrorInvalidValue;
    dim3 grid(ngroups / NW, (ntok + T - 1) / T);
    LVK_LAUNCH((k_matvec_q40<NT, T, UMAX, PRO, EPI, D, KT>), grid, dim3(NT), lds, s, P);
    return hipGetLastError();
}
// row lengths of the LLaMA family compiled in (n_embd and n_ff of 7B); others take the generic path
template <int NT, int T, int UMAX, int PRO, int EPI, int D>
hipError_t go(const Params & P, int ngroups, int ntok, hipStream_t s) {
    // single-token launches with these K go to matvec_cu.hip; here only the
    // multi-token (prompt) kernels get the compiled-in row lengths
    if (T == 1) return go1<NT, T, UMAX, PRO, EPI, D, 0>(P, ngroups, ntok, s);
    switch (P.K) {
        case 4096: return go1<NT, T, UMAX, PRO, EPI, D, 4096>(P, ngroups, ntok, s);
        case 11008: return go1<NT, T, UMAX, PRO, EPI, D, 11008>(P, ngroups, ntok, s);
        default: return go1<NT, T, UMAX, PRO, EPI, D, 0>(P, ngroups, ntok, s);
    }
}
}  // namespace

hipError_t launch_matvec(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype == Q4_1) return launch_matvec_q41(L, pro, epi, s);
    if (L.w.qtype != Q4_0) return hipErrorNotSupported;
    if (L.w.M % 8 || L.w.K % 256) return hipErrorInvalidValue;
    Params P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.M = L.w.M; P.K = L.w.K; P.nb = L.w.K / 32; P.NC = (P.nb + CB - 1) / CB;
    P.x = L.x; P.g = L.g; P.xq = L.xq; P.sp = L.sp;
    P.n_tokens = L.n_tokens; P.tok0 = L.tok0; P.out_tok0 = L.out_tok0;
    P.y = L.y; P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx; P.kv32 = L.kv32;
    P.silu_tab = L.silu_tab; P.out_q = L.out_q;
    const int ng = L.w.M / 8;
    const int N = L.n_tokens;
    const bool prefill = N > 1;
    switch (epi) {
        case EPI_QKV:
            if (pro != PRO_NORM || ng % 4 || P.K > 8192) return hipErrorInvalidValue;
            return prefill ? go<256, 4, 4, PRO_NORM, EPI_QKV, 2>(P, ng, N, s)
                           : go<256, 1, 4, PRO_NORM, EPI_QKV, 4>(P, ng, N, s);
        case EPI_SWIGLU:
            if (pro != PRO_NORM || ng % 8 || P.K > 16384) return hipErrorInvalidValue;
            return prefill ? go<512, 4, 4, PRO_NORM, EPI_SWIGLU, 2>(P, ng, N, s)
                           : go<512, 1, 4, PRO_NORM, EPI_SWIGLU, 4>(P, ng, N, s);
        case EPI_STORE:
            if (pro == PRO_NORM) {
                if (ng % 4 || P.K > 8192) return hipErrorInvalidValue;
                return prefill ? go<256, 4, 4, PRO_NORM, EPI_STORE, 2>(P, ng, N, s)
                               : go<256, 1, 4, PRO_NORM, EPI_STORE, 4>(P, ng, N, s);
            }
            if (P.nb > 12 * 64) return hipErrorInvalidValue;
            return prefill ? go<64, 4, 12, PRO_ACTQ, EPI_STORE, 2>(P, ng, N, s)
                           : go<64, 1, 12, PRO_ACTQ, EPI_STORE, 8>(P, ng, N, s);
        case EPI_RESID:
            if (pro != PRO_ACTQ || P.nb > 12 * 64) return hipErrorInvalidValue;
            return prefill ? go<64, 4, 12, PRO_ACTQ, EPI_RESID, 2>(P, ng, N, s)
                           : go<64, 1, 12, PRO_ACTQ, EPI_RESID, 8>(P, ng, N, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace lvk
