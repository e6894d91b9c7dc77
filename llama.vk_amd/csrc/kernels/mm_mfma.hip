// mm_mfma.hip -- prompt-eval (N > 1) Q4_0 matmul on the CDNA4 matrix cores,
// bit-faithful to the reference AVX2 arithmetic.
//
// ggml_compute_forward_mul_mat_q_f32 (ggml.c:6510-6696) evaluates every
// (row m, token n) as ggml_vec_dot_q4_0 (ggml.c:1950-2026): 8 fp32 chains
//   acc_j = fmaf(dw_b * da_b, (float) P_bj, acc_j)   over blocks b in order,
//   P_bj  = sum_{e=4j}^{4j+3} (qw_e - 8) * (qa_e - 8)  (exact integer),
// then ((a0+a4)+(a2+a6)) + ((a1+a5)+(a3+a7)).  Those 8.5e11 sequential FMAs
// (7B, 512-token prompt) are the floor of any bit-exact implementation; the
// integer partials are what the matrix cores can take over.
//
// Here v_mfma_f32_32x32x8_f16 produces the partials: in its operand layout
// lane half h holds k = 4h..4h+3, i.e. exactly one chain (2c+h) of a block's
// elements 8c..8c+7.  The B columns are (16 tokens) x (2 chain parities jj);
// lanes with h != jj hold zeros, so output column (n, jj) of the MFMA for
// chain pair c is P_{b,2c+jj}[m, n] for 32 rows m: exact (|products| <= 64,
// sums of 4 in f32).  The VALU then runs exactly the reference's chains:
//   s = dw*da (ggml.c:1968), acc_j = fmaf(s, P_bj, acc_j) (ggml.c:2013),
// and the final AVX2 horizontal order (ggml.c:2019-2024).  Every output is
// bit-identical to ggml_vec_dot_q4_0 (pinned by tests/test_gpu_ops.py).
//
// Operands:
//   A (weights): the decode "octet" image (lvk_kernels.h) read straight into
//     registers: MFMA lane (row, h) loads octet lanes 8r + 2c + h (chains
//     2c+h, c = 0..3) of its row group, 4 x 16 B per 8 blocks; nibbles -> f16
//     with the magic-exponent trick (0x6400|q = 1024+q, 0x4C00|q<<4 = 16+q/4)
//     in the chain order e0 e2 e1 e3.
//   B (activations): Q4_0-quantized tokens as f16 values q-8, written by the
//     activation quantizer straight into the masked fragment image
//       xm[token tile][block][c/2][64 lanes][c%2] x 8 B   (lvk_device.h xm_slot)
//     (lane (h, jj, n): chain 2c+h of token n when h == jj, else zero), so a
//     wave loads each fragment with one coalesced global_load_dwordx2 -- no
//     LDS staging and no barrier per K step; 2 blocks are kept in flight (a
//     ring of 4 pushes the kernel past 256 VGPRs into scratch).
//   Scales: dw (octet image) and da staged per 32-block chunk in LDS (one
//     barrier per chunk); s = dw*da of 32 rows x 16 tokens x 2 blocks comes
//     from one v_mfma_f32_32x32x1f32 outer product (exact f32 products).
// Workgroup = 4 waves, tile 128 rows x 16 tokens (wave w: rows 32w..32w+31,
// all 8 chains: 64 accumulator registers); workgroups are mapped so the 8
// XCDs each sweep contiguous row tiles with the token tiles innermost (the
// weight tile is fetched into that XCD's L2 once for all its token tiles).
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

#include <cstdlib>

namespace lvk {

namespace {

typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x32_t __attribute__((ext_vector_type(32)));

constexpr int TM = 128;     // rows per workgroup
constexpr int TN = 16;      // tokens per workgroup (one token tile)
constexpr int NT = 256;     // threads (4 waves)
// LVK_MM_EXP (dev probe builds only, tools/probe), bit flags: 1 no fp32 chains, 2 no MFMA, 4 no B loads,
// 64 no B stage global loads (LDS B path), 128 no scale outer-product MFMA, 256 no loop barriers,
// 8 no A loads, 16 / 32 L2-hot A / B (below)
#ifndef LVK_MM_EXP
#define LVK_MM_EXP 0
#endif
#ifndef LVK_MM_PD
#define LVK_MM_PD 2
#endif
constexpr int PD = LVK_MM_PD;   // B blocks in flight per wave (ring size divides 8; 4 spills at 256 VGPRs)
#ifndef LVK_MM_PDA
#define LVK_MM_PDA 4
#endif
// A16 variant: A and B blocks in flight per wave.  4 + 4 measured fastest (7B 512-token
// prompt 45.4 ms; 4 + 2: 47.7, 2 + 4: 50.7, nibble unpack path 47.3) although it leaves
// 4-6 VGPRs in scratch at the 256-VGPR budget of two waves per SIMD
constexpr int PDA = LVK_MM_PDA;
#ifndef LVK_MM_PDB16
#define LVK_MM_PDB16 4
#endif

constexpr int DWS = TM + 8;                         // padded row stride of the dw image (conflict-free stores)
constexpr int DAS = TN + 1;                         // padded stride of the da image
constexpr int LDS_DW = 32 * DWS * 4;                // [block of chunk][row]
constexpr int LDS_DA = (32 * DAS * 4 + 15) / 16 * 16;   // [block of chunk][token]
constexpr int OFF_DW0 = 0, OFF_DW1 = LDS_DW;
constexpr int OFF_DA0 = 2 * LDS_DW, OFF_DA1 = OFF_DA0 + LDS_DA;
constexpr int LDS_TOTAL = OFF_DA1 + LDS_DA;         // ~37 KiB
// A16 + LVK_MM_BLDS: the token tile's B fragments of one sub-chunk (8 blocks x 2 x 64 lanes x
// 16 B) staged once per workgroup in LDS, double-buffered, instead of each wave loading them
#ifndef LVK_MM_BLDS
#define LVK_MM_BLDS 1
#endif
constexpr int LDS_BSUB = 8 * 128 * 16;               // 16 KiB per sub-chunk
constexpr int OFF_B0 = LDS_TOTAL, OFF_B1 = OFF_B0 + LDS_BSUB;
constexpr int LDS_TOTAL_BL = OFF_B1 + LDS_BSUB;     // ~69 KiB: two workgroups per CU

struct MmParams {
    const uint4 * nib;
    const float4 * scl;
    const uint2 * a16;       // A16 variant: f16 A-fragment image [M/32][nb][4][64] (QMatrix::a16)
    int M, K, nb, NC;
    const uint2 * xm;        // masked B fragment image [ntt][nb][4][64]
    const float * da;        // [N][nb]
    int N;                   // tokens
    int ntt;                 // token tiles
    float * y;               // output
    int ldy;
    int out_tok0;
    const uint16_t * silu_tab;
    int supertile;           // 1: super tiles of 4 row tiles (default; LVK_MM_SUPERTILE=0: row tiles)
    RopeKV rk;               // EPI_ROPE_KV only
    uint2 * xq;              // EPI_SWIGLU_Q: the W2 input's fragment image, scales, blocks per token
    float * xqda;
    int nbq;
};

__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t o) {
    uint32_t r;
    asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(m), "v"(o));
    return r;
}

// 16-bit chain field (4 unsigned nibbles e0..e3) selected by sel from X -> f16 e0 e2 e1 e3
__device__ __forceinline__ half4_t unpack_chain(uint32_t X, uint32_t sel) {
    const uint32_t t = __builtin_amdgcn_perm(X, X, sel);            // byte0 | byte1 << 16
    const uint32_t lo = and_or(t, 0x000F000Fu, 0x64006400u);        // (e0, e2) = 1024 + q
    const uint32_t hi = and_or(t, 0x00F000F0u, 0x4C004C00u);        // (e1, e3) = 16 + q/4
    const half2_t c1032 = {(_Float16) -1032.0f, (_Float16) -1032.0f};
    const half2_t c4 = {(_Float16) 4.0f, (_Float16) 4.0f};
    const half2_t c72 = {(_Float16) -72.0f, (_Float16) -72.0f};
    const half2_t h0 = __builtin_bit_cast(half2_t, lo) + c1032;                           // q - 8
    const half2_t h1 = __builtin_elementwise_fma(__builtin_bit_cast(half2_t, hi), c4, c72); // q - 8
    half4_t r;
    r[0] = h0[0]; r[1] = h0[1]; r[2] = h1[0]; r[3] = h1[1];
    return r;
}

__device__ __forceinline__ f32x16_t fake_mfma(half4_t a, half4_t b) {   // LVK_MM_EXP & 2 only
    f32x16_t r;
    const float v = (float) a[0] + (float) b[1];
#pragma unroll
    for (int i = 0; i < 16; ++i) r[i] = v;
    return r;
}

// AVX2 horizontal order (ggml.c:2019-2024) and the epilogue of a wave's 32 rows x 16 tokens:
// lane (h, n, jj) register set c holds chain 2c+jj; r_j = a_j + a_{j+4} (same lane, sets c and
// c+2), (r0+r2) | (r1+r3) in lanes jj = 0 | 1, then across the lane pair (xor 16)
template <int EPI>
__device__ __forceinline__ void mm_store(const MmParams & P, const f32x16_t (&acc)[4], int lane, int w, int m0, int n0) {
    const int h = lane >> 5;
    const int jj = (lane >> 4) & 1;
    float2 cs[4][2];                                  // EPI_ROPE_KV: cos / sin (rope_kv_cs)
    if constexpr (EPI == EPI_ROPE_KV) rope_kv_cs(P.rk, P.N, n0 + (lane & 15), h, w, m0, cs);
    float res[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float r0 = acc[0][i] + acc[2][i];       // r_jj     = a_jj + a_{jj+4}
        const float r2 = acc[1][i] + acc[3][i];       // r_{2+jj} = a_{2+jj} + a_{6+jj}
        const float v = r0 + r2;
        res[i] = v + __shfl_xor(v, 16);               // (r0 + r2) + (r1 + r3) in the jj = 0 lanes
    }

    // ---- epilogue: jj = 0 lanes hold rows 32w + 8q + 4h + p (i = 4q + p) of token n ----
    const int n = n0 + (lane & 15);
    if constexpr (EPI == EPI_SWIGLU_F32) {
        // W1|W3 image interleaved per 4 rows: h = 0 lanes hold the w1 rows, h = 1 the w3 rows of the
        // same outputs (llama.cpp:1085-1096)
        float o[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) o[i] = __shfl_xor(res[i], 32);
        if (jj == 0 && h == 0 && n < P.N) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float uu[4];
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const float sl = f16_to_f32(P.silu_tab[f32_to_f16(res[4 * q + p])]);  // ggml.c:2495
                    uu[p] = sl * o[4 * q + p];                                            // llama.cpp:1096
                }
                const int row = m0 + 32 * w + 8 * q;
                *(float4 *) (P.y + (size_t) (P.out_tok0 + n) * P.ldy + row / 2) = make_float4(uu[0], uu[1], uu[2], uu[3]);
            }
        }
    } else if constexpr (EPI == EPI_SWIGLU_Q) {
        // SwiGLU as EPI_SWIGLU_F32, then quantize_row_q4_0 of the W2 input (ggml.c:621-685, the
        // arithmetic of k_act_q40_f16_tile) straight into its fragment image: the wave's 16
        // outputs (features m0/2 + 16w ..) are half of Q4_0 block b, the other half in wave
        // w ^ 1, the amax exchanged through LDS (free after the main loop's last barrier)
        extern __shared__ __attribute__((aligned(16))) uint8_t smem_e[];
        float uu[16];
        float am = 0.0f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float o = __shfl_xor(res[i], 32);
            const float sl = f16_to_f32(P.silu_tab[f32_to_f16(res[i])]);    // ggml.c:2495
            uu[i] = sl * o;                                                  // llama.cpp:1096
            const float a = fabsf(uu[i]);
            am = a > am ? a : am;
        }
        __syncthreads();
        float * red = (float *) smem_e;
        if (jj == 0 && h == 0) red[w * 16 + (lane & 15)] = am;
        __syncthreads();
        if (jj == 0 && h == 0 && n < P.N) {
            const float ao = red[(w ^ 1) * 16 + (lane & 15)];
            const float amax = (w & 1) ? (am > ao ? am : ao) : (ao > am ? ao : am);
            const float d = amax / 7.0f;                              // ggml.c:651
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
            const int b = ((m0 >> 1) + 16 * w) >> 5;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                uint32_t hh[4];
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    const int qv = ((int) __builtin_rintf(uu[4 * q + p] * id) + 8) & 15;   // ggml.c:655-684
                    hh[p] = __builtin_bit_cast(uint16_t, (_Float16) (float) (qv - 8));
                }
                // elements 16 (w & 1) + 4q + p of the block: group c = 2 (w & 1) + q / 2, its
                // first half (q even) in lane n, its second in lane 48 + n (k_act_q40_f16 order)
                const int c = 2 * (w & 1) + (q >> 1);
                P.xq[xm_slot(n, P.nbq, b, c, (q & 1) ? 48 + (n & 15) : (n & 15))] =
                    make_uint2(hh[0] | hh[2] << 16, hh[1] | hh[3] << 16);
            }
            if ((w & 1) == 0) P.xqda[(size_t) n * P.nbq + b] = d;
        }
    } else if constexpr (EPI == EPI_ROPE_KV) {
        // RoPE + the f16 q / K / V stores (rope_kv_store); a wave's 32 rows lie in one of Q, K, V
        if (jj == 0 && n < P.N) rope_kv_store(P.rk, res, cs, n, h, w, m0);
    } else {
        if (jj == 0 && n < P.N) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float4 * yp = (float4 *) (P.y + (size_t) (P.out_tok0 + n) * P.ldy + m0 + 32 * w + 8 * q + 4 * h);
                if constexpr (EPI == EPI_RESID) {
                    const float4 r = *yp;                 // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
                    *yp = make_float4(res[4 * q] + r.x, res[4 * q + 1] + r.y, res[4 * q + 2] + r.z, res[4 * q + 3] + r.w);
                } else {
                    *yp = make_float4(res[4 * q], res[4 * q + 1], res[4 * q + 2], res[4 * q + 3]);
                }
            }
        }
    }
}

// A16: the A fragments come ready-made from the f16 image (one global_load_dwordx2 per
// MFMA, ring of PD blocks like B) instead of the nibble octet image + unpack (5 VALU per
// MFMA, a third of the loop's VALU work)
template <int EPI, bool A16>
__global__ __launch_bounds__(NT, 2) void k_mm_q40_mfma(MmParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    // XCD-aware tile order: workgroup b runs on XCD b % 8; give each XCD a
    // contiguous range of (row tile, token tile) with token tiles innermost
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int full = nwg & ~7;
    const int L = bid < full ? (bid & 7) * (full >> 3) + (bid >> 3) : bid;
    int tt, rt;
    mm_tile(L, P.ntt, P.M / TM, P.supertile, rt, tt);
    const int m0 = rt * TM;
    const int n0 = tt * TN;
    const int nb = P.nb, NC = P.NC;
    const int G0 = m0 / 8;
    const int U = nb / 8;                      // sub-chunks of 8 blocks

    // ---- scales: chunk c (32 blocks) staged into LDS buffer c & 1 ----
    float rda[2];
    float4 rdw[4];
    auto load_scales = [&](int c) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int Li = i * NT + tid;
            rdw[i] = P.scl[(size_t) (G0 + (Li >> 6)) * NC * 64 + (size_t) c * 64 + (Li & 63)];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int Li = i * NT + tid;
            const int n = Li >> 5, jb = Li & 31;
            const int tok = min(n0 + n, P.N - 1);
            rda[i] = P.da[(size_t) tok * nb + min(c * 32 + jb, nb - 1)];
        }
    };
    auto store_scales = [&](int c) {
        float * wl = (float *) (smem + ((c & 1) ? OFF_DW1 : OFF_DW0));
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int Li = i * NT + tid;
            const int G = Li >> 6, l = Li & 63;
            const int r = l >> 3, j = l & 7;
            const float v[4] = {rdw[i].x, rdw[i].y, rdw[i].z, rdw[i].w};
#pragma unroll
            for (int m = 0; m < 4; ++m) wl[(8 * m + j) * DWS + 8 * G + r] = v[m];
        }
        float * dl = (float *) (smem + ((c & 1) ? OFF_DA1 : OFF_DA0));
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int Li = i * NT + tid;
            dl[(Li & 31) * DAS + (Li >> 5)] = rda[i];
        }
    };

    // ---- A operand: MFMA lane (row rho, half h) <- octet lanes 8r + 2c + h ----
    const int rho = lane & 31, h = lane >> 5;
    const int arow = m0 + 32 * w + rho;
    const uint4 * ap = P.nib + (size_t) (arow >> 3) * NC * 256 + 8 * (arow & 7) + h;
    auto load_a = [&](int u, uint4 (&A)[4]) {              // sub-chunk u = 8 blocks
        const uint4 * p = ap + (size_t) u * 64;            // (c*4 + sb) * 64 == u * 64
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            if (LVK_MM_EXP & 8) A[c] = make_uint4(u, c, u ^ c, 7);
            else A[c] = p[2 * c];
        }
    };
    // A16: lane (rho, h) of wave w reads the fragment of rows m0 + 32w + rho, chain 2c + h
    // LVK_MM_EXP & 16 / 32 (probe builds only): every workgroup reads the weights of row tiles 0..3 /
    // the activations of token tiles 0..1 (always L2-hot; timing only)
    const int a_rt = (LVK_MM_EXP & 16) ? (rt & 3) : rt;
    const uint4 * a16p = A16 ? (const uint4 *) P.a16 + (size_t) (a_rt * TM / 32 + w) * nb * 128 + lane : nullptr;
    uint2 aq[A16 ? PDA : 1][4];
    auto load_aq = [&](int blk, uint2 (&q)[4]) {
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
            const uint4 v = (LVK_MM_EXP & 8) ? make_uint4(blk, c2, 7, 1) : a16p[(size_t) blk * 128 + c2 * 64];
            q[2 * c2] = make_uint2(v.x, v.y);
            q[2 * c2 + 1] = make_uint2(v.z, v.w);
        }
    };
    // ---- B operand: masked fragments of this token tile, 4 per block ----
    const uint4 * bp = (const uint4 *) P.xm + (size_t) tt * nb * 128 + lane;   // xm_slot pairs
    constexpr bool BL = LVK_MM_BLDS;
    constexpr int PB = BL ? 1 : A16 ? LVK_MM_PDB16 : PD;       // B blocks in flight
    uint2 bq[PB][4];
    // BL: sub-chunk u of the token tile is 1024 contiguous uint4; thread tid stages 4 of them
    const uint4 * bsp = (const uint4 *) P.xm + (size_t) ((LVK_MM_EXP & 32) ? (tt & 1) : tt) * nb * 128 + tid;
    uint4 bs0, bs1, bs2, bs3;                  // (named: an array of them stays in scratch)
    auto stage_load = [&](int u) {
        const uint4 * g = bsp + (size_t) u * 1024;
        if (LVK_MM_EXP & 64) {
            bs0 = make_uint4(u, 1, 2, 3); bs1 = make_uint4(u, 5, 6, 7); bs2 = make_uint4(u, 9, 1, 2); bs3 = make_uint4(u, 3, 4, 5);
        } else {
            bs0 = g[0]; bs1 = g[NT]; bs2 = g[2 * NT]; bs3 = g[3 * NT];
        }
    };
    auto stage_store = [&](int u) {
        uint4 * bl = (uint4 *) (smem + ((u & 1) ? OFF_B1 : OFF_B0)) + tid;
        bl[0] = bs0; bl[NT] = bs1; bl[2 * NT] = bs2; bl[3 * NT] = bs3;
    };
    auto lds_bq = [&](int u, int jb, uint2 (&q)[4]) {
        const uint4 * bl = (const uint4 *) (smem + ((u & 1) ? OFF_B1 : OFF_B0)) + jb * 128 + lane;
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
            const uint4 v = bl[c2 * 64];
            q[2 * c2] = make_uint2(v.x, v.y);
            q[2 * c2 + 1] = make_uint2(v.z, v.w);
        }
    };
    auto load_bq = [&](int blk, uint2 (&q)[4]) {
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
            const uint4 v = (LVK_MM_EXP & 4) ? make_uint4(blk, c2, 0, 1) : bp[(size_t) blk * 128 + c2 * 64];
            q[2 * c2] = make_uint2(v.x, v.y);
            q[2 * c2 + 1] = make_uint2(v.z, v.w);
        }
    };

    f32x16_t acc[4];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[c][i] = 0.0f;

    uint32_t X[4][4];                                     // signed octet nibbles -> unsigned q
    auto make_x = [&](const uint4 (&A)[4]) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            X[c][0] = A[c].x ^ 0x88888888u; X[c][1] = A[c].y ^ 0x88888888u;
            X[c][2] = A[c].z ^ 0x88888888u; X[c][3] = A[c].w ^ 0x88888888u;
        }
    };

    uint4 Anext[4];
    load_scales(0);
    if constexpr (A16) {
#pragma unroll
        for (int d = 0; d < PDA; ++d) load_aq(min(d, nb - 1), aq[d]);
    } else {
        load_a(0, Anext);
    }
    if constexpr (BL) {
        stage_load(0);
        stage_store(0);
    } else {
#pragma unroll
        for (int d = 0; d < PB; ++d) load_bq(min(d, nb - 1), bq[d]);
    }
    store_scales(0);
    if constexpr (!A16) make_x(Anext);
    __syncthreads();

    for (int u = 0; u < U; ++u) {
        const int ch = u >> 2;
        const bool chunk_last = (u & 3) == 3 || u == U - 1;
        const bool scales_next = chunk_last && u + 1 < U;
        if (!A16 && u + 1 < U) load_a(u + 1, Anext);
        if (scales_next) load_scales(ch + 1);
        if (BL && u + 1 < U) stage_load(u + 1);
        const float * wl = (const float *) (smem + ((ch & 1) ? OFF_DW1 : OFF_DW0));
        const float * dl = (const float *) (smem + ((ch & 1) ? OFF_DA1 : OFF_DA0));
        // the block scales s = dw * da (ggml.c:1968) of every (row, token) output come from
        // the matrix core as an outer product, K = 1: each element is one rounded f32
        // multiply, bit-identical to the VALU product.  v_mfma_f32_32x32x1f32 (2 blocks):
        // lane half h feeds block jb + h (dw of row l&31, da of token (l&31)&15); block b
        // lands in registers 16b..16b+15 in the standard 32x32 C/D layout, i.e. exactly the
        // (rows, column) of the chain partials below.
        f32x32_t SC;
#pragma unroll
        for (int jb = 0; jb < 8; ++jb) {
            const int blk = 8 * u + jb;
            const uint32_t sel = (jb & 1) ? 0x0C030C02u : 0x0C010C00u;
            uint2 (&bf)[4] = bq[jb % PB];
            if constexpr (BL) lds_bq(u, jb, bf);
            if ((jb & 1) == 0) {
                const int jc = (u & 3) * 8 + jb + h;        // block of the chunk this lane half feeds
                const float dwa = wl[jc * DWS + 32 * w + rho];
                const float dab = dl[jc * DAS + (lane & 15)];
                if (LVK_MM_EXP & 128) {
#pragma unroll
                    for (int i = 0; i < 32; ++i) SC[i] = dwa + dab;
                } else {
                    SC = __builtin_amdgcn_mfma_f32_32x32x1f32(dwa, dab, (f32x32_t){}, 0, 0, 0);
                }
            }
            float sc[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) sc[i] = SC[16 * (jb & 1) + i];
            // software pipeline: the MFMA of chain pair c+1 is in flight while the VALU runs the
            // chains of pair c (ggml.c:2013: acc_j = fmaf(d, P_j, acc_j))
            f32x16_t Pc[2];
#define LVK_MFMA(a, b) ((LVK_MM_EXP & 2) ? fake_mfma(a, b) : __builtin_amdgcn_mfma_f32_32x32x8f16(a, b, (f32x16_t){}, 0, 0, 0))
            uint2 (&af)[4] = aq[A16 ? jb % PDA : 0];
            auto afrag = [&](int c) __attribute__((always_inline)) -> half4_t {
                if constexpr (A16) return __builtin_bit_cast(half4_t, af[c]);
                else return unpack_chain(X[c][jb >> 1], sel);
            };
            Pc[0] = LVK_MFMA(afrag(0), __builtin_bit_cast(half4_t, bf[0]));
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                if (c + 1 < 4)
                    Pc[(c + 1) & 1] = LVK_MFMA(afrag(c + 1), __builtin_bit_cast(half4_t, bf[c + 1]));
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    if (LVK_MM_EXP & 1) acc[c][i] += (i == 0 ? Pc[c & 1][0] + sc[0] : 0.0f);
                    else acc[c][i] = __builtin_fmaf(sc[i], Pc[c & 1][i], acc[c][i]);
                }
            }
            // refill this slot with block blk + PD (its MFMAs have read the old fragments)
            if constexpr (!BL) load_bq(min(blk + PB, nb - 1), bf);
            if constexpr (A16) load_aq(min(blk + PDA, nb - 1), af);
            // block order pinned: unconstrained, hipcc hoists later blocks' MFMAs and spills
#pragma unroll
            for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(acc[c]));
        }
        if (!A16 && u + 1 < U) make_x(Anext);
        if (BL && u + 1 < U) stage_store(u + 1);
        if (scales_next) store_scales(ch + 1);
        if ((scales_next || (BL && u + 1 < U)) && !(LVK_MM_EXP & 256))
            __syncthreads();            // chunk ch+1's scales / sub-chunk u+1's B visible; the buffers of
                                        // chunk ch-1 / sub-chunk u-1 free again
    }

    mm_store<EPI>(P, acc, lane, w, m0, n0);
}

// ---------------------------------------------------------------------------
// Activation quantizer for the MFMA path: x[t] (optionally rms_norm * g) ->
// quantize_row_q4_0 (AVX2 branch, ggml.c:621-685) -> f16 values q-8 in the
// A-unpack k order + da.  One workgroup per token; the RMSNorm double sum is
// the same per-thread strided / wave tree / in-order-waves reduction as the
// matvec prologue (matvec_q4.hip prologue_norm).
// ---------------------------------------------------------------------------
template <bool NORM>
__global__ __launch_bounds__(256) void k_act_q40_f16(const float * __restrict__ x, const float * __restrict__ g,
                                                     int N, int K, uint2 * __restrict__ xm, float * __restrict__ da) {
    __shared__ double red[4];
    __shared__ float s_scale;
    const int t = xcd_grouped_token(blockIdx.x);
    if (t >= N) return;
    const int tid = threadIdx.x;
    const int nunits = K / 8;
    const float * xr = x + (size_t) t * K;
    float scale = 1.0f;
    if constexpr (NORM) {
        double acc = 0.0;
        for (int u = tid; u < nunits; u += 256) {
            const float4 a = *(const float4 *) (xr + u * 8), b = *(const float4 *) (xr + u * 8 + 4);
            const float e[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
            for (int q = 0; q < 8; ++q) { const float sq = e[q] * e[q]; acc += (double) sq; }
        }
        acc = warp_sum_d(acc);
        if ((tid & 63) == 0) red[tid >> 6] = acc;
        __syncthreads();
        if (tid < 64) {             // wave 0: rms_mean_wave splits a re-check over its lanes
            double s = 0.0;
            for (int wv = 0; wv < 4; ++wv) s += red[wv];
            const float mean = rms_mean_wave(s, xr, K);           // ggml.c:6058-6071
            if (tid == 0) s_scale = 1.0f / sqrtf(mean + 1e-6f);
        }
        __syncthreads();
        scale = s_scale;
    }
    for (int u0 = 0; u0 < nunits; u0 += 256) {
        const int u = u0 + tid;
        const bool live = u < nunits;          // nunits % 4 == 0: quads are all live or all dead
        float v[8];
        if (live) {
            const float4 a = *(const float4 *) (xr + u * 8), b = *(const float4 *) (xr + u * 8 + 4);
            v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
            if constexpr (NORM) {
                const float4 ga = *(const float4 *) (g + u * 8), gb = *(const float4 *) (g + u * 8 + 4);
                const float gg[8] = {ga.x, ga.y, ga.z, ga.w, gb.x, gb.y, gb.z, gb.w};
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float yn = v[e] * scale;     // ggml_vec_scale_f32 (ggml.c:6076)
                    v[e] = gg[e] * yn;                 // ggml_mul(repeat(g), cur) (llama.cpp:984)
                }
            }
        } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 0.0f;
        }
        float amax = 0.0f;
#pragma unroll
        for (int e = 0; e < 8; ++e) { const float a = fabsf(v[e]); amax = a > amax ? a : amax; }
        const float o0 = quad_bcast<0>(amax), o1 = quad_bcast<1>(amax);
        const float o2 = quad_bcast<2>(amax), o3 = quad_bcast<3>(amax);
        const float m01 = o1 > o0 ? o1 : o0, m23 = o3 > o2 ? o3 : o2;
        amax = m23 > m01 ? m23 : m01;
        const float d = amax / 7.0f;                              // ggml.c:651
        const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
        if (live) {
            uint16_t h[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int q = ((int) __builtin_rintf(v[e] * id) + 8) & 15;   // ggml.c:655-684
                h[e] = __builtin_bit_cast(uint16_t, (_Float16) (float) (q - 8));
            }
            // masked fragment image: chain 2c -> lane n (h = jj = 0), chain 2c+1 -> lane 48 + n (h = jj = 1),
            // each in the order e0 e2 e1 e3
            const int nb = K / 32, c = u & 3;
            xm[xm_slot(t, nb, u >> 2, c, t & 15)] = make_uint2(h[0] | (uint32_t) h[2] << 16, h[1] | (uint32_t) h[3] << 16);
            xm[xm_slot(t, nb, u >> 2, c, 48 + (t & 15))] =
                make_uint2(h[4] | (uint32_t) h[6] << 16, h[5] | (uint32_t) h[7] << 16);
            if ((u & 3) == 0) da[(size_t) t * (K / 32) + (u >> 2)] = d;
        }
    }
}

// The quantizer without RMSNorm (the W2 input) by token tiles: a wave takes one 32-block b of
// the tile's 16 tokens (lane quad = token, lane = 8 values), so each of its two stores fills
// whole 256-byte runs of the fragment image (lanes 0-15 | 48-63 of chain pair c/2) instead of
// 16-byte pieces of lines the other 15 tokens' workgroups -- on other XCDs -- also write
// (14 us per 512 x 11008 activation that way).  Same arithmetic per block as k_act_q40_f16.
__global__ __launch_bounds__(256) void k_act_q40_f16_tile(const float * __restrict__ x, int N, int K,
                                                          uint2 * __restrict__ xm, float * __restrict__ da) {
    const int nb = K / 32;
    const int lane = threadIdx.x & 63;
    const int b = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (b >= nb) return;                                     // wave-uniform; no barriers below
    const int tl = lane >> 2, c = lane & 3;
    const int t = blockIdx.x * 16 + tl;
    const bool live = t < N;
    float v[8];
    if (live) {
        const float * xp = x + (size_t) t * K + b * 32 + c * 8;
        const float4 a = *(const float4 *) xp, bb = *(const float4 *) (xp + 4);
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = bb.x; v[5] = bb.y; v[6] = bb.z; v[7] = bb.w;
    } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = 0.0f;
    }
    float amax = 0.0f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float a = fabsf(v[e]); amax = a > amax ? a : amax; }
    const float o0 = quad_bcast<0>(amax), o1 = quad_bcast<1>(amax);
    const float o2 = quad_bcast<2>(amax), o3 = quad_bcast<3>(amax);
    const float m01 = o1 > o0 ? o1 : o0, m23 = o3 > o2 ? o3 : o2;
    amax = m23 > m01 ? m23 : m01;
    const float d = amax / 7.0f;                              // ggml.c:651
    const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
    if (live) {
        uint16_t h[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const int q = ((int) __builtin_rintf(v[e] * id) + 8) & 15;   // ggml.c:655-684
            h[e] = __builtin_bit_cast(uint16_t, (_Float16) (float) (q - 8));
        }
        xm[xm_slot(t, nb, b, c, tl)] = make_uint2(h[0] | (uint32_t) h[2] << 16, h[1] | (uint32_t) h[3] << 16);
        xm[xm_slot(t, nb, b, c, 48 + tl)] = make_uint2(h[4] | (uint32_t) h[6] << 16, h[5] | (uint32_t) h[7] << 16);
        if (c == 0) da[(size_t) t * nb + b] = d;
    }
}

// pre-quantized Q4_0 blocks (ActQ: d + reference nibble qs) -> masked fragment image + da
__global__ void k_actq_to_f16(ActQ q, int N, int K, uint2 * __restrict__ xm, float * __restrict__ da) {
    const int nb = K / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;   // (token, block, group of 8)
    if (idx >= (long) N * nb * 4) return;
    const int c = (int) (idx & 3);
    const long tb = idx >> 2;
    const uint4 qs = q.qs[tb];
    const uint32_t wd[4] = {qs.x, qs.y, qs.z, qs.w};
    const uint32_t word = wd[c];               // elements 8c..8c+7: element 2k = byte k low nibble
    uint16_t h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int qv = (int) ((word >> (4 * e)) & 15u);
        h[e] = __builtin_bit_cast(uint16_t, (_Float16) (float) (qv - 8));
    }
    const int t = (int) (tb / nb), b = (int) (tb % nb);
    xm[xm_slot(t, nb, b, c, t & 15)] = make_uint2(h[0] | (uint32_t) h[2] << 16, h[1] | (uint32_t) h[3] << 16);
    xm[xm_slot(t, nb, b, c, 48 + (t & 15))] = make_uint2(h[4] | (uint32_t) h[6] << 16, h[5] | (uint32_t) h[7] << 16);
    if (c == 0) da[tb] = q.d[tb];
}

// RoPE mode 0 (ggml.c:7156-7227) + KV append (llama.cpp:996-1008) of the
// stored Q|K|V rows [N][3E] -> q16 [N][E], K cache [pos][E], V cache [E][pos]
__global__ void k_rope_kv(const float * __restrict__ qkv, int N, int E, int hd, const float2 * __restrict__ rope,
                          const StepParams * __restrict__ sp, int n_ctx, uint16_t * __restrict__ q16,
                          uint16_t * __restrict__ kc, uint16_t * __restrict__ vc, int kv32) {
    const int t = blockIdx.y;
    const int e2 = blockIdx.x * blockDim.x + threadIdx.x;     // pair index over Q|K (E/2 each) then V
    const int pos = sp->n_past + t;
    const float * row = qkv + (size_t) t * 3 * E;
    if (e2 < E) {                // Q and K pairs: e2 in [0, E): which = e2 / (E/2)
        const int which = e2 / (E / 2);
        const int e = 2 * (e2 - which * (E / 2));
        const float x0 = row[which * E + e], x1 = row[which * E + e + 1];
        const int i0 = e % hd;
        const float2 cs = rope[(size_t) pos * (hd / 2) + (i0 >> 1)];
        const float a0 = x0 * cs.x, b0 = x1 * cs.y;
        const float o0 = a0 - b0;
        const float a1 = x0 * cs.y, b1 = x1 * cs.x;
        const float o1 = a1 + b1;
        if (which == 0) {
            kv_store(q16, (size_t) t * E + e, o0, kv32);
            kv_store(q16, (size_t) t * E + e + 1, o1, kv32);
        } else {
            kv_store(kc, (size_t) pos * E + e, o0, kv32);
            kv_store(kc, (size_t) pos * E + e + 1, o1, kv32);
        }
    } else if (e2 < E + E / 2) {
        const int e = 2 * (e2 - E);
        kv_store(vc, (size_t) e * n_ctx + pos, row[2 * E + e], kv32);
        kv_store(vc, (size_t) (e + 1) * n_ctx + pos, row[2 * E + e + 1], kv32);
    }
}

// f16 A-fragment image of a Q4_0 octet image (QMatrix::a16): a16[M/32][nb][c/2][lane][c%2] x 8 B,
// lane (rho, h) = row 32 rt + rho, chain 2c + h: its 4 elements as f16 (q - 8) in the
// fragment order e0 e2 e1 e3 (the order the activation image uses).  One thread per
// 8-byte fragment, read from the octet word that holds the chain (k_repack_q40 layout).
__global__ void k_a16_from_octet(const uint4 * __restrict__ nib, int M, int K, uint2 * __restrict__ a16) {
    const int nb = K / 32, NC = (nb + 31) / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;     // ((rt * nb + b) * 4 + c) * 64 + lane
    if (idx >= (long) (M / 32) * nb * 256) return;
    const int lane = (int) (idx & 63), c = (int) ((idx >> 6) & 3);
    const long rb = idx >> 8;
    const int b = (int) (rb % nb), rt = (int) (rb / nb);
    const int row = rt * 32 + (lane & 31), jc = 2 * c + (lane >> 5);
    const uint4 v = nib[(((size_t) (row >> 3) * NC + (b >> 5)) * 4 + ((b & 31) >> 3)) * 64 + 8 * (row & 7) + jc];
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
    const uint32_t t = ((wd[(b & 7) >> 1] >> (16 * (b & 1))) & 0xFFFFu) ^ 0x8888u;   // byte0: e0 e1, byte1: e2 e3
    uint16_t hq[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) hq[e] = __builtin_bit_cast(uint16_t, (_Float16) (float) ((int) ((t >> (4 * e)) & 15u) - 8));
    // chain pairs 2q, 2q+1 side by side per lane (as xm_slot): one 16-byte load per 2 MFMAs
    a16[((((size_t) rt * nb + b) * 2 + (c >> 1)) * 64 + lane) * 2 + (c & 1)] =
        make_uint2(hq[0] | (uint32_t) hq[2] << 16, hq[1] | (uint32_t) hq[3] << 16);
}

}  // namespace

int mm_supertile() {
    static const int v = [] { const char * e = getenv("LVK_MM_SUPERTILE"); return e ? atoi(e) : 1; }();
    return v;
}

size_t mm_a16_bytes(int M, int K) { return (size_t) (M / 32) * (K / 32) * 256 * 8; }

hipError_t launch_build_a16(const QMatrix & w, void * a16, hipStream_t s) {
    if (w.qtype != Q4_0 || w.M % 32 || w.K % 256) return hipErrorInvalidValue;
    const long n = (long) (w.M / 32) * (w.K / 32) * 256;
    LVK_LAUNCH(k_a16_from_octet, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, w.nib, w.M, w.K, (uint2 *) a16);
    return hipGetLastError();
}

bool mm_mfma_supported(const QMatrix & w) {
    if (w.qtype == Q4_1) return mm_mfma41_supported(w);
    return w.qtype == Q4_0 && w.M % TM == 0 && w.K % 256 == 0;
}

size_t mm_act_bytes(int N, int K) { return (size_t) ((N + TN - 1) / TN) * (K / 32) * 4 * 64 * 8; }

hipError_t launch_mm_mfma(const QMatrix & w, const void * xm, const float * da, int N, float * y, int ldy,
                          int out_tok0, int epi, const uint16_t * silu_tab, hipStream_t s) {
    if (w.qtype != Q4_0 || !mm_mfma_supported(w) || N <= 0) return hipErrorInvalidValue;
    MmParams P{};
    P.nib = w.nib; P.scl = (const float4 *) w.scl;
    P.M = w.M; P.K = w.K; P.nb = w.K / 32; P.NC = (P.nb + 31) / 32;
    P.xm = (const uint2 *) xm; P.da = da; P.N = N; P.ntt = (N + TN - 1) / TN;
    P.y = y; P.ldy = ldy; P.out_tok0 = out_tok0; P.silu_tab = silu_tab;
    P.a16 = (const uint2 *) w.a16;
    P.supertile = mm_supertile();
    const dim3 grid((w.M / TM) * P.ntt);
#define LVK_MM_GO(E)                                                                      \
    do {                                                                                  \
        if (P.a16) LVK_LAUNCH((k_mm_q40_mfma<E, true>), grid, dim3(NT), LVK_MM_BLDS ? LDS_TOTAL_BL : LDS_TOTAL, s, P); \
        else LVK_LAUNCH((k_mm_q40_mfma<E, false>), grid, dim3(NT), LVK_MM_BLDS ? LDS_TOTAL_BL : LDS_TOTAL, s, P); \
    } while (0)
    switch (epi) {
        case EPI_STORE: LVK_MM_GO(EPI_STORE); break;
        case EPI_RESID: LVK_MM_GO(EPI_RESID); break;
        case EPI_SWIGLU_F32: LVK_MM_GO(EPI_SWIGLU_F32); break;
        default: return hipErrorInvalidValue;
    }
#undef LVK_MM_GO
    return hipGetLastError();
}

hipError_t launch_mm_qkv_rope(const QMatrix & w, const void * xm, const float * da, int N, const RopeKV & r,
                              hipStream_t s) {
    if (w.qtype != Q4_0 || !mm_mfma_supported(w) || N <= 0 || w.M != 3 * r.E || r.E % 32 || r.hd % 4 || !r.sp)
        return hipErrorInvalidValue;
    MmParams P{};
    P.nib = w.nib; P.scl = (const float4 *) w.scl;
    P.M = w.M; P.K = w.K; P.nb = w.K / 32; P.NC = (P.nb + 31) / 32;
    P.xm = (const uint2 *) xm; P.da = da; P.N = N; P.ntt = (N + TN - 1) / TN;
    P.a16 = (const uint2 *) w.a16;
    P.supertile = mm_supertile();
    P.rk = r;
    const dim3 grid((w.M / TM) * P.ntt);
    if (P.a16) LVK_LAUNCH((k_mm_q40_mfma<EPI_ROPE_KV, true>), grid, dim3(NT), LVK_MM_BLDS ? LDS_TOTAL_BL : LDS_TOTAL, s, P);
    else LVK_LAUNCH((k_mm_q40_mfma<EPI_ROPE_KV, false>), grid, dim3(NT), LVK_MM_BLDS ? LDS_TOTAL_BL : LDS_TOTAL, s, P);
    return hipGetLastError();
}

hipError_t launch_mm_w13_q(const QMatrix & w, const void * xm, const float * da, int N, const uint16_t * silu_tab,
                           void * xq, float * xqda, hipStream_t s) {
    if (w.qtype != Q4_0 || !mm_mfma_supported(w) || N <= 0 || w.M % 64 || !silu_tab || !xq || !xqda)
        return hipErrorInvalidValue;
    MmParams P{};
    P.nib = w.nib; P.scl = (const float4 *) w.scl;
    P.M = w.M; P.K = w.K; P.nb = w.K / 32; P.NC = (P.nb + 31) / 32;
    P.xm = (const uint2 *) xm; P.da = da; P.N = N; P.ntt = (N + TN - 1) / TN;
    P.a16 = (const uint2 *) w.a16;
    P.supertile = mm_supertile();
    P.silu_tab = silu_tab;
    P.xq = (uint2 *) xq; P.xqda = xqda; P.nbq = w.M / 64;
    const dim3 grid((w.M / TM) * P.ntt);
    if (P.a16) LVK_LAUNCH((k_mm_q40_mfma<EPI_SWIGLU_Q, true>), grid, dim3(NT), LVK_MM_BLDS ? LDS_TOTAL_BL : LDS_TOTAL, s, P);
    else LVK_LAUNCH((k_mm_q40_mfma<EPI_SWIGLU_Q, false>), grid, dim3(NT), LVK_MM_BLDS ? LDS_TOTAL_BL : LDS_TOTAL, s, P);
    return hipGetLastError();
}

hipError_t launch_act_f16(const float * x, const float * g, int N, int K, void * xm, float * da, hipStream_t s) {
    if (K % 256 || N <= 0) return hipErrorInvalidValue;
    static const bool tile = [] { const char * e = getenv("LVK_ACT_TILE"); return !e || atoi(e) != 0; }();
    const dim3 gt((unsigned) ((N + 127) / 128 * 128));   // k_act_q40_f16: XCD-grouped token order
    if (g) LVK_LAUNCH(k_act_q40_f16<true>, gt, dim3(256), 0, s, x, g, N, K, (uint2 *) xm, da);
    else if (tile)
        LVK_LAUNCH(k_act_q40_f16_tile, dim3((N + 15) / 16, (K / 32 + 3) / 4), dim3(256), 0, s, x, N, K, (uint2 *) xm, da);
    else LVK_LAUNCH(k_act_q40_f16<false>, gt, dim3(256), 0, s, x, g, N, K, (uint2 *) xm, da);
    return hipGetLastError();
}

hipError_t launch_actq_to_f16(const ActQ & q, int N, int K, void * xm, float * da, hipStream_t s) {
    const long n = (long) N * (K / 32) * 4;
    LVK_LAUNCH(k_actq_to_f16, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, q, N, K, (uint2 *) xm, da);
    return hipGetLastError();
}

hipError_t launch_rope_kv(const float * qkv, int N, int E, int hd, const float2 * rope, const StepParams * sp,
                          int n_ctx, uint16_t * q16, uint16_t * kc, uint16_t * vc, hipStream_t s, int kv32) {
    const int pairs = E + E / 2;
    LVK_LAUNCH(k_rope_kv, dim3((pairs + 255) / 256, N), dim3(256), 0, s, qkv, N, E, hd, rope, sp, n_ctx, q16, kc, vc,
               kv32);
    return hipGetLastError();
}

}  // namespace lvk

LVK_RMS_ACCESSOR(lvk_probe_rms_mm)
