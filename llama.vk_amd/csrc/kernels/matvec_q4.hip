// matvec_q4.hip -- bit-faithful Q4_0 / Q4_1 matrix x quantized-activation
// product for gfx950, with fused prologues (RMSNorm + activation quantizer,
// or pre-quantized input) and epilogues (residual add, RoPE + KV append,
// SwiGLU + requantize, plain store).
//
// Reference arithmetic being reproduced bit-for-bit:
//   ggml_compute_forward_mul_mat_q_f32 (ggml.c:6510-6696): quantize every
//   activation column to the weight's block format (quantize_row_q4_0 AVX2,
//   ggml.c:621-685), then one ggml_vec_dot_q4_0 (ggml.c:1950-2026) per
//   (row, column): 8 fp32 accumulators acc_j += (dw*dx) * P_j, P_j = exact
//   int sum over block elements 4j..4j+3, final ((a0+a4)+(a2+a6))+((a1+a5)+(a3+a7)).
//
// MI355X mapping:
//   * one wavefront = 16 weight rows; lane 4r+q owns row r and the two
//     sequential accumulator chains j = 2q, 2q+1 (the only parallelism the
//     sequential fp32 chains allow besides rows/tokens);
//   * weights stream once from HBM in a pre-swizzled image: every wave
//     instruction is a 1 KiB coalesced dwordx4 load; nibbles are pre-XORed so
//     one v_dot8_i32_i4 yields an exact P_j for one block;
//   * the per-block weight scale is owned by lane q = block%4 of the quad and
//     broadcast with a quad_perm DPP move (no LDS round trip);
//   * the quantized activation lives in LDS as zero-padded nibble words, read
//     with broadcast ds_read_b128 (all 16 rows of a wave share one address).
#include "lvk_device.h"
#include "lvk_kernels.h"

namespace lvk {

namespace {

constexpr int CH = 8;   // blocks per chunk (one dwordx4 pair + one float2 per lane)

// LDS activation table of one token (Q4_0):
//   tbl[nb/2][4] uint4 {AX_i, AX_i+1, AY_i, AY_i+1} of block pair (i, i+1) and quad lane q
//   dxs[nb] float
struct ActTableQ40 {
    uint4 * tbl;
    float * dxs;
};

// RNE quantization of one 8-element unit (ggml.c:655-684): returns the dword
// of nibbles (q+8) in the reference's packing (element 2k low nibble of byte k).
__device__ __forceinline__ uint32_t q40_pack8(const float v[8], float id) {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int q = (int) __builtin_rintf(v[k] * id) + 8;
        w |= (uint32_t) (q & 15) << (4 * k);
    }
    return w;
}

// Store one block's quad-lane word into the LDS table.  `dw` holds elements
// 8q..8q+7 of block i (reference nibble convention, unsigned q+8).
__device__ __forceinline__ void tbl_store_q40(uint4 * tbl, int i, int q, uint32_t dw) {
    const uint32_t s = dw ^ 0x88888888u;        // signed 4-bit (q) for v_dot8_i32_i4
    const uint32_t gx = s & 0xFFFFu;             // group 2q   (elements 8q..8q+3)
    const uint32_t gy = s >> 16;                 // group 2q+1 (elements 8q+4..8q+7)
    uint32_t * t = (uint32_t *) (tbl + (size_t) (i >> 1) * 4 + q);
    if (i & 1) { t[1] = gx << 16; t[3] = gy << 16; }
    else       { t[0] = gx;       t[2] = gy; }
}

struct Params {
    const uint4 * nib;
    const float2 * scl;
    int M, K, nb, C;
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
    const uint16_t * silu_tab;
    ActQ out_q;
};

// ---------------------------------------------------------------------------
// Prologue A (PRO_NORM): rows x[t] (f32) -> rms_norm -> * g -> Q4_0 quantize,
// straight into the LDS table.  ggml.c:6058-6076 (sum of (double)(x*x) ->
// mean as float -> 1/sqrtf(mean+1e-6f) -> scale) then llama.cpp:984 (g * y).
// The double sum is reduced in tree order: every partial is a float square
// carried exactly in double, so any order reaches the same float mean except
// when the sum sits within ~1e-13 relative of a float rounding boundary.
// Work unit = 8 consecutive elements; the 4 units of a block sit in 4
// consecutive threads (a quad), which reduce amax with DPP.
// ---------------------------------------------------------------------------
template <int NT, int T, int UMAX, bool PRE>
__device__ void prologue_norm(const Params & P, int t0, int nt, uint4 * tbl_base, float * dx_base,
                              double * red, float * s_scale,
                              const float4 (&xv)[UMAX][2], const float4 (&gv)[UMAX][2]) {
    const int tid = threadIdx.x;
    const int K = P.K;
    const int nunits = K / 8;
    // unit k of token tt: preloaded registers (decode) or straight from L2 (prefill)
    auto ldx = [&](int tt, int k, float v[8]) {
        float4 a, b;
        if constexpr (PRE) { a = xv[k][0]; b = xv[k][1]; }
        else {
            const int u = k * NT + tid;
            const float4 * xp = (const float4 *) (P.x + (size_t) (P.tok0 + t0 + tt) * K + (size_t) u * 8);
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
            const int u = k * NT + tid;
            if (u < nunits && tt < nt) {
                float e[8];
                ldx(tt, k, e);
#pragma unroll
                for (int j = 0; j < 8; ++j) { const float sq = e[j] * e[j]; acc += (double) sq; }
            }
        }
        acc = warp_sum_d(acc);
        if ((tid & 63) == 0) red[tt * (NT / 64) + (tid >> 6)] = acc;
    }
    __syncthreads();
    if (tid < T) {
        double s = 0.0;
        for (int w = 0; w < NT / 64; ++w) s += red[tid * (NT / 64) + w];
        const float mean = (float) (s / (double) K);
        s_scale[tid] = 1.0f / sqrtf(mean + 1e-6f);
    }
    __syncthreads();
    for (int tt = 0; tt < T; ++tt) {
        if (tt >= nt) break;
        const float scale = s_scale[tt];
        uint4 * tbl = tbl_base + (size_t) tt * (P.nb / 2) * 4;
        float * dxs = dx_base + (size_t) tt * P.nb;
#pragma unroll
        for (int k = 0; k < UMAX; ++k) {
            const int u = k * NT + tid;
            // a block's 4 units are 4 consecutive threads of one quad: same k, same liveness
            if (k * NT >= nunits) break;
            const bool live = u < nunits;
            float v[8], gg[8];
            if (live) { ldx(tt, k, v); ldg(k, gg); }
            else {
#pragma unroll
                for (int j = 0; j < 8; ++j) { v[j] = 0.0f; gg[j] = 0.0f; }
            }
            float amax = 0.0f;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float yn = v[j] * scale;       // ggml_vec_scale_f32 (ggml.c:6076)
                v[j] = gg[j] * yn;                   // ggml_mul(repeat(g), cur) (llama.cpp:984)
                const float a = fabsf(v[j]);
                amax = a > amax ? a : amax;
            }
            // quad max (exact in any order for non-negative values)
            const float o0 = quad_bcast<0>(amax), o1 = quad_bcast<1>(amax);
            const float o2 = quad_bcast<2>(amax), o3 = quad_bcast<3>(amax);
            float m01 = o1 > o0 ? o1 : o0, m23 = o3 > o2 ? o3 : o2;
            amax = m23 > m01 ? m23 : m01;
            const float d = amax / 7.0f;                              // ggml.c:651
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
            const uint32_t w = q40_pack8(v, id);
            if (live) {
                const int blk = u >> 2, q = u & 3;
                tbl_store_q40(tbl, blk, q, w);
                if (q == 0) dxs[blk] = d;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Prologue B (PRO_ACTQ): expand pre-quantized Q4_0 blocks (d + qs) into the
// LDS table.  One thread per block.
// ---------------------------------------------------------------------------
template <int NT, int T, int BMAX, bool PRE>
__device__ void prologue_actq(const Params & P, int t0, int nt, uint4 * tbl_base, float * dx_base,
                              const uint4 (&qv)[BMAX], const float (&dv)[BMAX]) {
    const int tid = threadIdx.x;
    if constexpr (PRE) {
        uint4 * tbl = tbl_base;
#pragma unroll
        for (int k = 0; k < BMAX; ++k) {
            const int b = k * NT + tid;
            if (b < P.nb) {
                tbl_store_q40(tbl, b, 0, qv[k].x);
                tbl_store_q40(tbl, b, 1, qv[k].y);
                tbl_store_q40(tbl, b, 2, qv[k].z);
                tbl_store_q40(tbl, b, 3, qv[k].w);
                dx_base[b] = dv[k];
            }
        }
    } else {
        for (int tt = 0; tt < nt; ++tt) {
            const int t = t0 + tt + P.tok0;
            uint4 * tbl = tbl_base + (size_t) tt * (P.nb / 2) * 4;
            float * dxs = dx_base + (size_t) tt * P.nb;
            for (int b = tid; b < P.nb; b += NT) {
                const uint4 qs = P.xq.qs[(size_t) t * P.nb + b];
                const float d = P.xq.d[(size_t) t * P.nb + b];
                tbl_store_q40(tbl, b, 0, qs.x);
                tbl_store_q40(tbl, b, 1, qs.y);
                tbl_store_q40(tbl, b, 2, qs.z);
                tbl_store_q40(tbl, b, 3, qs.w);
                dxs[b] = d;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// The faithful chain over one chunk of 8 blocks for T tokens.
// ---------------------------------------------------------------------------
template <int T>
__device__ __forceinline__ void chunk_q40(float (&acc)[T][2], const uint4 w0, const uint4 w1, const float2 sc,
                                          const uint4 * tbl_base, const float * dx_base, int c, int q,
                                          int nb) {
    // weight scale of each of the 8 blocks, broadcast from its owner lane
    float dw[8];
    dw[0] = quad_bcast<0>(sc.x); dw[1] = quad_bcast<1>(sc.x); dw[2] = quad_bcast<2>(sc.x); dw[3] = quad_bcast<3>(sc.x);
    dw[4] = quad_bcast<0>(sc.y); dw[5] = quad_bcast<1>(sc.y); dw[6] = quad_bcast<2>(sc.y); dw[7] = quad_bcast<3>(sc.y);
    const uint32_t wx[4] = {w0.x, w0.z, w1.x, w1.z};   // X words of pairs 0..3
    const uint32_t wy[4] = {w0.y, w0.w, w1.y, w1.w};   // Y words of pairs 0..3
#pragma unroll
    for (int tt = 0; tt < T; ++tt) {
        const uint4 * tbl = tbl_base + (size_t) tt * (nb / 2) * 4;
        const float4 * dx4 = (const float4 *) (dx_base + (size_t) tt * nb + c * CH);
        const float4 da = dx4[0], db = dx4[1];
        const float dx[8] = {da.x, da.y, da.z, da.w, db.x, db.y, db.z, db.w};
#pragma unroll
        for (int pp = 0; pp < 4; ++pp) {
            const uint4 a = tbl[(size_t) (c * 4 + pp) * 4 + q];
            const int p0 = dot8(wx[pp], a.x);   // block 2pp,   chain 2q
            const int p1 = dot8(wx[pp], a.y);   // block 2pp+1, chain 2q
            const int p2 = dot8(wy[pp], a.z);   // block 2pp,   chain 2q+1
            const int p3 = dot8(wy[pp], a.w);   // block 2pp+1, chain 2q+1
            const float s0 = dw[2 * pp] * dx[2 * pp];          // x.d * y.d (ggml.c:1968)
            const float s1 = dw[2 * pp + 1] * dx[2 * pp + 1];
            acc[tt][0] = __builtin_fmaf(s0, (float) p0, acc[tt][0]);
            acc[tt][1] = __builtin_fmaf(s0, (float) p2, acc[tt][1]);
            acc[tt][0] = __builtin_fmaf(s1, (float) p1, acc[tt][0]);
            acc[tt][1] = __builtin_fmaf(s1, (float) p3, acc[tt][1]);
        }
    }
}

// ---------------------------------------------------------------------------
// Epilogue helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ float quad_reduce8(float c0, float c1) {
    // a_{2q} = c0 of lane q, a_{2q+1} = c1 of lane q (ggml.c:2019-2024)
    const float a0 = quad_bcast<0>(c0), a1 = quad_bcast<0>(c1);
    const float a2 = quad_bcast<1>(c0), a3 = quad_bcast<1>(c1);
    const float a4 = quad_bcast<2>(c0), a5 = quad_bcast<2>(c1);
    const float a6 = quad_bcast<3>(c0), a7 = quad_bcast<3>(c1);
    const float r0 = a0 + a4, r1 = a1 + a5, r2 = a2 + a6, r3 = a3 + a7;
    return (r0 + r2) + (r1 + r3);
}

// quantize 32 consecutive values held one per lane in lanes [32h, 32h+32) of a
// wave into a reference Q4_0 block (quantize_row_q4_0 AVX2, ggml.c:621-685)
__device__ __forceinline__ void quantize32_q40(float v, int lane, float * d_out, uint4 * qs_out, uint32_t * scratch) {
    float amax = fabsf(v);
    for (int o = 16; o > 0; o >>= 1) { const float w = __shfl_xor(amax, o); amax = w > amax ? w : amax; }
    const float d = amax / 7.0f;
    const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
    const uint32_t q = (uint32_t) ((int) __builtin_rintf(v * id) + 8) & 15u;
    // gather 8 nibbles per dword: element e -> dword e/8, nibble e%8
    const int e = lane & 31;
    uint32_t part = q << (4 * (e & 7));
    part |= __shfl_xor(part, 1);
    part |= __shfl_xor(part, 2);
    part |= __shfl_xor(part, 4);
    if ((e & 7) == 0) scratch[e >> 3] = part;
    __builtin_amdgcn_wave_barrier();
    if (e == 0) {
        *d_out = d;
        *qs_out = make_uint4(scratch[0], scratch[1], scratch[2], scratch[3]);
    }
}

}  // namespace

// ---------------------------------------------------------------------------
// The kernel.  NT threads (NT/64 waves = NT/64 row groups of 16 rows), T tokens
// per lane, UMAX = max 8-element units per thread in the norm prologue.
// ---------------------------------------------------------------------------
template <int NT, int T, int UMAX, int PRO, int EPI, int D>
__global__ __launch_bounds__(NT) void k_matvec_q40(Params P) {
    constexpr bool PRE = (T == 1);            // decode: stage prologue inputs in registers
    constexpr int BMAX = UMAX;                // PRO_ACTQ: blocks per thread
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int q = lane & 3;
    const int r = lane >> 2;
    const int g = blockIdx.x * (NT / 64) + wave;      // row group
    const int t0 = blockIdx.y * T;
    const int nt = min(T, P.n_tokens - t0);
    if (nt <= 0) return;
    const int nb = P.nb, C = P.C;

    uint4 * tbl_base = (uint4 *) smem;                                        // T * nb/2 * 4 uint4
    float * dx_base = (float *) (smem + (size_t) T * (nb / 2) * 64);         // T * nb floats
    double * red = (double *) (smem + (size_t) T * (nb / 2) * 64 + (size_t) T * nb * 4);   // T*(NT/64) doubles
    float * s_scale = (float *) (red + T * (NT / 64));                                          // T floats

    // 1. prologue inputs into registers (issued before the weight stream so
    //    the compiler's in-order vmcnt lets the prologue run under it)
    float4 xv[UMAX][2];
    float4 gv[UMAX][2];
    uint4 qv[BMAX];
    float dv[BMAX];
    if constexpr (PRE && PRO == PRO_NORM) {
        const int nunits = P.K / 8;
#pragma unroll
        for (int k = 0; k < UMAX; ++k) {
            // unconditional (clamped) loads keep the vmcnt bookkeeping static
            const int u = min(k * NT + tid, nunits - 1);
            const float4 * gp = (const float4 *) (P.g + (size_t) u * 8);
            const float4 * xp = (const float4 *) (P.x + (size_t) (P.tok0 + t0) * P.K + (size_t) u * 8);
            gv[k][0] = gp[0]; gv[k][1] = gp[1];
            xv[k][0] = xp[0]; xv[k][1] = xp[1];
        }
    }
    if constexpr (PRE && PRO == PRO_ACTQ) {
#pragma unroll
        for (int k = 0; k < BMAX; ++k) {
            const int b = min(k * NT + tid, nb - 1);
            qv[k] = P.xq.qs[(size_t) (P.tok0 + t0) * nb + b];
            dv[k] = P.xq.d[(size_t) (P.tok0 + t0) * nb + b];
        }
    }

    // 2. weight stream: D chunks in flight.  Every iteration issues its loads
    //    unconditionally (past-the-end chunks re-read the last one, an L1/L2
    //    hit), so the compiler's in-order vmcnt bookkeeping stays exact and
    //    waits only for the chunk being consumed (3*(D-1) loads left in flight).
    const uint4 * nib = P.nib + (size_t) g * C * 2 * 64 + lane;
    const float2 * scl = P.scl + (size_t) g * C * 64 + lane;
    uint4 W0[D], W1[D];
    float2 S[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const int cl = min(d, C - 1);
        W0[d] = ld_nt(nib + (size_t) cl * 128);
        W1[d] = ld_nt(nib + (size_t) cl * 128 + 64);
        S[d] = scl[(size_t) cl * 64];
    }

    // 3. activation table
    if constexpr (PRO == PRO_NORM) {
        prologue_norm<NT, T, UMAX, PRE>(P, t0, nt, tbl_base, dx_base, red, s_scale, xv, gv);
    } else {
        prologue_actq<NT, T, BMAX, PRE>(P, t0, nt, tbl_base, dx_base, qv, dv);
    }
    __syncthreads();

    // 4. faithful chains
    float acc[T][2];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) acc[tt][0] = acc[tt][1] = 0.0f;

    const int ngrp = (C + D - 1) / D;
    for (int gi = 0; gi < ngrp; ++gi) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const int c = gi * D + d;
            if (c < C) chunk_q40<T>(acc, W0[d], W1[d], S[d], tbl_base, dx_base, c, q, nb);
            const int cn = min(c + D, C - 1);
            W0[d] = ld_nt(nib + (size_t) cn * 128);
            W1[d] = ld_nt(nib + (size_t) cn * 128 + 64);
            S[d] = scl[(size_t) cn * 64];
        }
    }

    // 5. epilogue
    const int row = g * 16 + r;
    float res[T];
#pragma unroll
    for (int tt = 0; tt < T; ++tt) res[tt] = quad_reduce8(acc[tt][0], acc[tt][1]);

    if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (tt < nt && q == 0) P.y[(size_t) (P.out_tok0 + t0 + tt) * P.M + row] = res[tt];
    } else if constexpr (EPI == EPI_RESID) {
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (tt < nt && q == 0) {
                float * yp = P.y + (size_t) (P.out_tok0 + t0 + tt) * P.M + row;
                *yp = res[tt] + *yp;                 // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
            }
    } else if constexpr (EPI == EPI_QKV) {
        const int E = P.n_embd, hd = P.head_dim;
        const int which = row / E;          // 0 = q, 1 = k, 2 = v  (uniform per wave: E % 16 == 0)
        const int e = row - which * E;
        const int n_past = P.sp->n_past;
#pragma unroll
        for (int tt = 0; tt < T; ++tt) {
            const float other = __shfl_xor(res[tt], 4);   // row e^1 lives in quad r^1
            if (tt < nt && q == 0) {
                const int pos = n_past + t0 + tt;
                if (which < 2) {
                    // ggml_compute_forward_rope_f32 mode 0 (ggml.c:7209-7223)
                    const int i0 = e % hd;
                    const float2 cs = P.rope[(size_t) pos * (hd / 2) + (i0 >> 1)];
                    float out;
                    if ((i0 & 1) == 0) { const float x0 = res[tt], x1 = other; const float a = x0 * cs.x, b = x1 * cs.y; out = a - b; }
                    else               { const float x0 = other, x1 = res[tt]; const float a = x0 * cs.y, b = x1 * cs.x; out = a + b; }
                    if (which == 0) P.q16[(size_t) (t0 + tt) * E + e] = f32_to_f16(out);
                    else            P.kc[(size_t) pos * E + e] = f32_to_f16(out);
                } else {
                    P.vc[(size_t) e * P.n_ctx + pos] = f32_to_f16(res[tt]);
                }
            }
        }
    } else if constexpr (EPI == EPI_SWIGLU) {
        // WG = 4 waves = rows [64b, 64b+64) of the fused W1|W3 image: waves 0,1
        // hold w1 rows 32b..32b+31, waves 2,3 the w3 rows (llama.cpp:1085-1096)
        float * ures = (float *) smem;     // reuse: T x 64 floats (table no longer needed)
        uint32_t * scratch = (uint32_t *) (smem + (size_t) T * 64 * 4);
        __syncthreads();
#pragma unroll
        for (int tt = 0; tt < T; ++tt)
            if (q == 0) ures[tt * 64 + wave * 16 + r] = res[tt];
        __syncthreads();
        const int blk = blockIdx.x;        // output block index in [0, n_ff/32)
        // wave w handles tokens w, w+4, ...; lanes 0..31 one token, 32..63 the next
        for (int tt = wave * 2 + (lane >> 5); tt < nt; tt += (NT / 64) * 2) {
            const int e = lane & 31;
            const float a1 = ures[tt * 64 + e];          // w1 x
            const float a3 = ures[tt * 64 + 32 + e];     // w3 x
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
template <int NT, int T, int UMAX, int PRO, int EPI, int D>
hipError_t go(const Params & P, int ngroups, int ntok, hipStream_t s) {
    const size_t lds = (size_t) T * (P.nb / 2) * 64 + (size_t) T * P.nb * 4 + 8 * 64 + 64;
    dim3 grid(ngroups / (NT / 64), (ntok + T - 1) / T);
    hipLaunchKernelGGL((k_matvec_q40<NT, T, UMAX, PRO, EPI, D>), grid, dim3(NT), lds, s, P);
    return hipGetLastError();
}
}  // namespace

hipError_t launch_matvec(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype != Q4_0) return hipErrorNotSupported;
    if (L.w.M % 16 || L.w.K % 256) return hipErrorInvalidValue;
    Params P{};
    P.nib = L.w.nib;
    P.scl = (const float2 *) L.w.scl;
    P.M = L.w.M; P.K = L.w.K; P.nb = L.w.K / 32; P.C = L.w.K / 256;
    P.x = L.x; P.g = L.g; P.xq = L.xq; P.sp = L.sp;
    P.n_tokens = L.n_tokens; P.tok0 = L.tok0; P.out_tok0 = L.out_tok0;
    P.y = L.y; P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx;
    P.silu_tab = L.silu_tab; P.out_q = L.out_q;
    const int ng = L.w.M / 16;
    const int N = L.n_tokens;
    const bool prefill = N > 1;
    // norm prologue: 8-element units per thread = K/8/NT <= UMAX
    switch (epi) {
        case EPI_QKV:
            if (pro != PRO_NORM || ng % 2) return hipErrorInvalidValue;
            if (P.K > 8192) return hipErrorInvalidValue;
            return prefill ? go<128, 4, 8, PRO_NORM, EPI_QKV, 4>(P, ng, N, s)
                           : go<128, 1, 8, PRO_NORM, EPI_QKV, 12>(P, ng, N, s);
        case EPI_SWIGLU:
            if (pro != PRO_NORM || ng % 4 || P.K > 8192) return hipErrorInvalidValue;
            return prefill ? go<256, 4, 4, PRO_NORM, EPI_SWIGLU, 4>(P, ng, N, s)
                           : go<256, 1, 4, PRO_NORM, EPI_SWIGLU, 8>(P, ng, N, s);
        case EPI_STORE:
            if (pro == PRO_NORM) {
                if (ng % 4 || P.K > 8192) return hipErrorInvalidValue;
                return prefill ? go<256, 4, 4, PRO_NORM, EPI_STORE, 4>(P, ng, N, s)
                               : go<256, 1, 4, PRO_NORM, EPI_STORE, 8>(P, ng, N, s);
            }
            if (P.nb > 12 * 64) return hipErrorInvalidValue;
            return prefill ? go<64, 4, 12, PRO_ACTQ, EPI_STORE, 4>(P, ng, N, s)
                           : go<64, 1, 12, PRO_ACTQ, EPI_STORE, 16>(P, ng, N, s);
        case EPI_RESID:
            if (pro != PRO_ACTQ) return hipErrorInvalidValue;
            if (P.nb > 12 * 64) return hipErrorInvalidValue;
            return prefill ? go<64, 4, 12, PRO_ACTQ, EPI_RESID, 4>(P, ng, N, s)
                           : go<64, 1, 12, PRO_ACTQ, EPI_RESID, 16>(P, ng, N, s);
    }
    return hipErrorInvalidValue;
}

}  // namespace lvk
