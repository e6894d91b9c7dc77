// mm_mfma41.hip -- prompt-eval (N > 1) Q4_1 matmul on the CDNA4 matrix cores,
// bit-faithful to the reference AVX2 arithmetic (the 13B Q4_1 prompt path).
//
// ggml_vec_dot_q4_1 (ggml.c:2188-2258) evaluates every (row m, token n) as 8 fp32
// chains j = 0..7 over the blocks b in order, plus one offset chain:
//   P_bj   = sum of qx_e * qy_e over e in {2j, 2j+1, 16+2j, 17+2j}   (unsigned nibbles)
//   acc_j  = fmaf(dx*dy, P_bj, acc_j)                                 (ggml.c:2244)
//   acc_j  = fmaf(j even ? dx*my : mx*dy, S_bj, acc_j)                (ggml.c:2236-2247)
//            S_bj = j even ? sum(qx_{8q..8q+7}) : sum(qy_{8q..8q+7}),  q = j/2
//   off    = off + mx*my                                              (ggml.c:2226)
// result = hsum8(acc) + off * 32 (ggml.c:2250-2257).  Every integer above is exact in
// f16 operands and f32 MFMA sums, so the matrix cores produce them and the VALU runs
// exactly the reference's chains:
//   * P (4 x v_mfma_f32_32x32x8_f16 per block): as mm_mfma.hip's Q4_0 kernel -- A the
//     weight chain fragments (f16 image, QMatrix::a16), B the masked activation
//     fragments (lane (n, jj, h) holds chain 2c+h of token n when h == jj), output
//     column (n, jj) = chain 2c+jj.
//   * S (4 more v_mfma_f32_32x32x8_f16 per block): the cross term's integer operand in
//     the same output layout -- A lane (row, h): h = 0 the row's 4 weight sums of the
//     block, h = 1 ones; B lane (n, jj, h): (0, 0) the unit vector e_c, (1, 1) the
//     token's activation sum of group c at slot c, else zero.  Output column (n, 0) =
//     S of the even chain 2c (weight sum), (n, 1) = S of the odd chain 2c+1.
//   * the scale products: v_mfma_f32_32x32x1f32 (2 blocks) of A = (d | m of the row by
//     lane half) and B = (d | m of the token) gives dx*dy and mx*my; v_mfma_f32_32x32x2f32
//     of the same A and B = (h == jj ? (m | d) : 0) gives dx*my in the even and mx*dy in
//     the odd columns (one product plus an exact zero: the rounded VALU product, and the
//     chains can never hold -0, so a +-0 product term never changes a sum).
// Operand images (all built so a lane's operand is one 16-byte load):
//   weights a16  [M/32][nb][2][64] x 16 B  chain fragments (as the Q4_0 image, values q)
//           side [M/32][nb][64] x 16 B     {S operand (4 x f16), d | m (f32), 0}
//   tokens  xm   [N/16][nb][2][64] x 16 B  masked chain fragments (lvk_device.h xm_slot)
//           xs   [N/16][nb][64] x 16 B     {S operand, d | m, (m | d) masked}
// No LDS and no barrier: every operand streams straight into registers, 3 blocks deep
// (13B 512-token prompt: 1 block 188.7 ms, 2: 172.4, 3: 170.0, 4: 235.8 -- spills).
// Workgroup = 4 waves, tile 128 rows x 16 tokens, XCD-aware tile order (mm_mfma.hip).
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"
#include "mm41_common.h"

namespace lvk {

namespace {

typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
typedef float f32x32_t __attribute__((ext_vector_type(32)));

constexpr int TM = 128;     // rows per workgroup
constexpr int TN = 16;      // tokens per workgroup
constexpr int NT = 256;     // 4 waves
#ifndef LVK_MM41_PD
#define LVK_MM41_PD 3
#endif
constexpr int PD = LVK_MM41_PD;   // blocks of every operand in flight per wave

struct Mm41Params {
    const uint4 * a16;       // [M/32][nb][2][64]
    const uint4 * side;      // [M/32][nb][64]
    const uint4 * xm;        // [ntt][nb][2][64]
    const uint4 * xs;        // [ntt][nb][64]
    int M, nb, N, ntt;
    float * y;
    int ldy;
    const uint16_t * silu_tab;
    int supertile;           // mm_tile order (mm_mfma.hip)
    RopeKV rk;               // EPI_ROPE_KV only
};

struct Blk {                 // one block's operands of one lane
    uint4 a[2], b[2], sa, sb;
};

// AVX2 horizontal order + offset, then the role's store (shared by both kernels)
template <int EPI>
__device__ __forceinline__ void epilogue41(const Mm41Params & P, const f32x16_t (&acc)[4], const f32x16_t & off,
                                           int lane, int w, int m0, int n0) {
    // AVX2 horizontal order (ggml.c:2250-2256) as in mm_mfma.hip, then + off * 32 (QK)
    const int jj = (lane >> 4) & 1, h = lane >> 5;
    float2 cs[4][2];                                  // EPI_ROPE_KV: cos / sin (rope_kv_cs)
    if constexpr (EPI == EPI_ROPE_KV) rope_kv_cs(P.rk, P.N, n0 + (lane & 15), h, w, m0, cs);
    float res[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const float r0 = acc[0][i] + acc[2][i];
        const float r2 = acc[1][i] + acc[3][i];
        const float v = r0 + r2;
        const float hs = v + __shfl_xor(v, 16);
        res[i] = hs + off[i] * 32.0f;
    }
    const int n = n0 + (lane & 15);
    if constexpr (EPI == EPI_SWIGLU_F32) {
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
                *(float4 *) (P.y + (size_t) n * P.ldy + row / 2) = make_float4(uu[0], uu[1], uu[2], uu[3]);
            }
        }
    } else if constexpr (EPI == EPI_ROPE_KV) {
        if (jj == 0 && n < P.N) rope_kv_store(P.rk, res, cs, n, h, w, m0);
    } else {
        if (jj == 0 && n < P.N) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                float4 * yp = (float4 *) (P.y + (size_t) n * P.ldy + m0 + 32 * w + 8 * q + 4 * h);
                if constexpr (EPI == EPI_RESID) {
                    const float4 r = *yp;
                    *yp = make_float4(res[4 * q] + r.x, res[4 * q + 1] + r.y, res[4 * q + 2] + r.z, res[4 * q + 3] + r.w);
                } else {
                    *yp = make_float4(res[4 * q], res[4 * q + 1], res[4 * q + 2], res[4 * q + 3]);
                }
            }
        }
    }
}

template <int EPI>
__global__ __launch_bounds__(NT, 2) void k_mm_q41_mfma(Mm41Params P) {
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int full = nwg & ~7;
    const int L = bid < full ? (bid & 7) * (full >> 3) + (bid >> 3) : bid;
    int tt, rtile;
    mm_tile(L, P.ntt, P.M / TM, P.supertile, rtile, tt);
    const int m0 = rtile * TM;
    const int n0 = tt * TN;
    const int nb = P.nb;
    const int rt = m0 / 32 + w;                              // this wave's 32-row tile

    const uint4 * ap = P.a16 + (size_t) rt * nb * 128 + lane;
    const uint4 * sap = P.side + (size_t) rt * nb * 64 + lane;
    const uint4 * bp = P.xm + (size_t) tt * nb * 128 + lane;
    const uint4 * sbp = P.xs + (size_t) tt * nb * 64 + lane;
    auto load = [&](int blk, Blk & o) {
        o.a[0] = ap[(size_t) blk * 128];
        o.a[1] = ap[(size_t) blk * 128 + 64];
        o.b[0] = bp[(size_t) blk * 128];
        o.b[1] = bp[(size_t) blk * 128 + 64];
        o.sa = sap[(size_t) blk * 64];
        o.sb = sbp[(size_t) blk * 64];
    };

    f32x16_t acc[4], off;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[c][i] = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) off[i] = 0.0f;

    Blk ring[PD];
#pragma unroll
    for (int d = 0; d < PD; ++d) load(min(d, nb - 1), ring[d]);

    for (int b0 = 0; b0 < nb; b0 += PD) {
#pragma unroll
        for (int d = 0; d < PD; ++d) {
            const int blk = b0 + d;
            if (blk >= nb) break;
            Blk & o = ring[d];
            const float sw = __builtin_bit_cast(float, o.sa.z);      // d | m of the row
            const float sb1 = __builtin_bit_cast(float, o.sb.z);     // d | m of the token
            const float sb2 = __builtin_bit_cast(float, o.sb.w);     // (m | d) where h == jj, else 0
            // dx*dy (registers 0..15) and mx*my (16..31); dx*my | mx*dy by column parity
            const f32x32_t SM = __builtin_amdgcn_mfma_f32_32x32x1f32(sw, sb1, (f32x32_t){}, 0, 0, 0);
            const f32x16_t SX = __builtin_amdgcn_mfma_f32_32x32x2f32(sw, sb2, (f32x16_t){}, 0, 0, 0);
            const half4_t ax = __builtin_bit_cast(half4_t, make_uint2(o.sa.x, o.sa.y));
            const uint32_t bfr[8] = {o.b[0].x, o.b[0].y, o.b[0].z, o.b[0].w, o.b[1].x, o.b[1].y, o.b[1].z, o.b[1].w};
            const uint32_t afr[8] = {o.a[0].x, o.a[0].y, o.a[0].z, o.a[0].w, o.a[1].x, o.a[1].y, o.a[1].z, o.a[1].w};
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const half4_t a = __builtin_bit_cast(half4_t, make_uint2(afr[2 * c], afr[2 * c + 1]));
                const half4_t b = __builtin_bit_cast(half4_t, make_uint2(bfr[2 * c], bfr[2 * c + 1]));
                // the S operand's B fragment: slot c of the token's sums (or of e_c)
                const uint32_t yw = (c < 2) ? o.sb.x : o.sb.y;
                const uint32_t ym = yw & ((c & 1) ? 0xFFFF0000u : 0x0000FFFFu);
                const half4_t bs = __builtin_bit_cast(half4_t, (c < 2) ? make_uint2(ym, 0u) : make_uint2(0u, ym));
                const f32x16_t Pc = __builtin_amdgcn_mfma_f32_32x32x8f16(a, b, (f32x16_t){}, 0, 0, 0);
                const f32x16_t Sc = __builtin_amdgcn_mfma_f32_32x32x8f16(ax, bs, (f32x16_t){}, 0, 0, 0);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    acc[c][i] = __builtin_fmaf(SM[i], Pc[i], acc[c][i]);      // ggml.c:2244
                    acc[c][i] = __builtin_fmaf(SX[i], Sc[i], acc[c][i]);      // ggml.c:2247
                }
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) off[i] = off[i] + SM[16 + i];      // ggml.c:2226
            // refill this slot PD blocks ahead (its MFMAs have consumed it)
            load(min(blk + PD, nb - 1), o);
#pragma unroll
            for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(acc[c]));
        }
    }

    epilogue41<EPI>(P, acc, off, lane, w, m0, n0);
}

// ---------------------------------------------------------------------------
// The same matmul with the operands streamed through a per-wave LDS ring by LDS-DMA
// (global_load_lds_dwordx4).  hipcc's waitcnt pass
// puts a vmcnt(0) at the register-ring loop's header (the refill issued last in a trip
// is waited for at once); the DMAs are invisible to it, so the wave keeps RS blocks in
// flight and waits with its own count.  Per wave RS slots of 6 x 1 KiB (a16 pair halves,
// side, xm pair halves, xs: one 16-byte lane row each, read back with one ds_read_b128
// per lane and operand); 72 KiB per workgroup, two workgroups per CU.
// ---------------------------------------------------------------------------
#ifndef LVK_MM41_RS
#define LVK_MM41_RS 3
#endif
#ifndef LVK_MM41_OCC
#define LVK_MM41_OCC 2
#endif
constexpr int RS = LVK_MM41_RS;             // ring slots (blocks in flight) per wave
constexpr int OCC41 = LVK_MM41_OCC;         // workgroups per CU (LDS: OCC41 * LDS41 <= 160 KiB)
#ifndef LVK_MM41_PIPE
#define LVK_MM41_PIPE 0
#endif
constexpr int SLOT = 6 * 1024;
constexpr int LDS41 = 4 * RS * SLOT;

__device__ __forceinline__ unsigned lds_addr41(const void * p) {
    return (unsigned) (uintptr_t) (const __attribute__((address_space(3))) uint8_t *) p;
}
// one 1 KiB LDS-DMA: lane l's 16 bytes at gsrc land at LDS byte lds_dst + 16 l
__device__ __forceinline__ void dma1k(const void * gsrc, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

template <int EPI>
__global__ __launch_bounds__(NT, OCC41) void k_mm_q41_dma(Mm41Params P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int w = tid >> 6;
    const int nwg = gridDim.x;
    const int bid = blockIdx.x;
    const int full = nwg & ~7;
    const int L = bid < full ? (bid & 7) * (full >> 3) + (bid >> 3) : bid;
    int tt, rtile;
    mm_tile(L, P.ntt, P.M / TM, P.supertile, rtile, tt);
    const int m0 = rtile * TM;
    const int n0 = tt * TN;
    const int nb = P.nb;
    const int rt = m0 / 32 + w;

    const uint4 * ap = P.a16 + (size_t) rt * nb * 128 + lane;
    const uint4 * sap = P.side + (size_t) rt * nb * 64 + lane;
    const uint4 * bp = P.xm + (size_t) tt * nb * 128 + lane;
    const uint4 * sbp = P.xs + (size_t) tt * nb * 64 + lane;
    uint8_t * ring = smem + w * RS * SLOT;
    const unsigned ring_l = __builtin_amdgcn_readfirstlane(lds_addr41(ring));
    auto issue = [&](int blk, int slot) {
        const unsigned d = ring_l + slot * SLOT;
        dma1k(ap + (size_t) blk * 128, d);
        dma1k(ap + (size_t) blk * 128 + 64, d + 1024);
        dma1k(sap + (size_t) blk * 64, d + 2048);
        dma1k(bp + (size_t) blk * 128, d + 3072);
        dma1k(bp + (size_t) blk * 128 + 64, d + 4096);
        dma1k(sbp + (size_t) blk * 64, d + 5120);
    };

    f32x16_t acc[4], off;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[c][i] = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; ++i) off[i] = 0.0f;

#pragma unroll
    for (int sl = 0; sl < RS; ++sl) issue(min(sl, nb - 1), sl);

    int slot = 0;
    for (int blk = 0; blk < nb; ++blk) {
        // this block's 6 DMAs landed: at most the later RS - 1 blocks' are still in flight
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(6 * (RS - 1)) : "memory");
        const uint4 * sp = (const uint4 *) (ring + slot * SLOT) + lane;   // ds_read (LDS pointer inferred)
        Blk o;
        o.a[0] = sp[0]; o.a[1] = sp[64]; o.sa = sp[128];
        o.b[0] = sp[192]; o.b[1] = sp[256]; o.sb = sp[320];
        // the slot is free once its reads returned: refill it RS blocks ahead
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(min(blk + RS, nb - 1), slot);
        slot = slot + 1 == RS ? 0 : slot + 1;

        const float sw = __builtin_bit_cast(float, o.sa.z);
        const float sb1 = __builtin_bit_cast(float, o.sb.z);
        const float sb2 = __builtin_bit_cast(float, o.sb.w);
        const f32x32_t SM = __builtin_amdgcn_mfma_f32_32x32x1f32(sw, sb1, (f32x32_t){}, 0, 0, 0);
        const f32x16_t SX = __builtin_amdgcn_mfma_f32_32x32x2f32(sw, sb2, (f32x16_t){}, 0, 0, 0);
        const half4_t ax = __builtin_bit_cast(half4_t, make_uint2(o.sa.x, o.sa.y));
        const uint32_t bfr[8] = {o.b[0].x, o.b[0].y, o.b[0].z, o.b[0].w, o.b[1].x, o.b[1].y, o.b[1].z, o.b[1].w};
        const uint32_t afr[8] = {o.a[0].x, o.a[0].y, o.a[0].z, o.a[0].w, o.a[1].x, o.a[1].y, o.a[1].z, o.a[1].w};
        auto mfma_p = [&](int c) __attribute__((always_inline)) {
            const half4_t a = __builtin_bit_cast(half4_t, make_uint2(afr[2 * c], afr[2 * c + 1]));
            const half4_t b = __builtin_bit_cast(half4_t, make_uint2(bfr[2 * c], bfr[2 * c + 1]));
            return __builtin_amdgcn_mfma_f32_32x32x8f16(a, b, (f32x16_t){}, 0, 0, 0);
        };
        auto mfma_s = [&](int c) __attribute__((always_inline)) {
            const uint32_t yw = (c < 2) ? o.sb.x : o.sb.y;
            const uint32_t ym = yw & ((c & 1) ? 0xFFFF0000u : 0x0000FFFFu);
            const half4_t bs = __builtin_bit_cast(half4_t, (c < 2) ? make_uint2(ym, 0u) : make_uint2(0u, ym));
            return __builtin_amdgcn_mfma_f32_32x32x8f16(ax, bs, (f32x16_t){}, 0, 0, 0);
        };
#if LVK_MM41_PIPE
        // software pipeline: chain pair c+1's MFMAs are issued before chain pair c's FMAs
        f32x16_t Pn = mfma_p(0), Sn = mfma_s(0);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const f32x16_t Pc = Pn, Sc = Sn;
            if (c < 3) { Pn = mfma_p(c + 1); Sn = mfma_s(c + 1); }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc[c][i] = __builtin_fmaf(SM[i], Pc[i], acc[c][i]);      // ggml.c:2244
                acc[c][i] = __builtin_fmaf(SX[i], Sc[i], acc[c][i]);      // ggml.c:2247
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#else
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const f32x16_t Pc = mfma_p(c);
            const f32x16_t Sc = mfma_s(c);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc[c][i] = __builtin_fmaf(SM[i], Pc[i], acc[c][i]);      // ggml.c:2244
                acc[c][i] = __builtin_fmaf(SX[i], Sc[i], acc[c][i]);      // ggml.c:2247
            }
        }
#endif
#pragma unroll
        for (int i = 0; i < 16; ++i) off[i] = off[i] + SM[16 + i];      // ggml.c:2226
#pragma unroll
        for (int c = 0; c < 4; ++c) asm volatile("" : "+v"(acc[c]));
    }
    // the trailing refills must land before the workgroup's LDS is released
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    epilogue41<EPI>(P, acc, off, lane, w, m0, n0);
}

// activation quantizer for the Q4_1 MFMA path: x[t] (optionally rms_norm * g) ->
// quantize_row_q4_1 (AVX2 branch, ggml.c:847-920; matvec_common.h q41_quad) -> the
// fragment and side images.  One workgroup per token, one lane quad per block.
template <bool NORM>
__global__ __launch_bounds__(256) void k_act_q41_f16(const float * __restrict__ x, const float * __restrict__ g, int N,
                                                     int K, uint4 * __restrict__ xm, uint4 * __restrict__ xs) {
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
        float d, m;
        uint32_t qword;
        mv::q41_quad(v, d, m, qword);
        if (live) act41_emit(t, K / 32, u >> 2, u & 3, qword, d, m, xm, xs);
    }
}

// pre-quantized Q4_1 blocks (ActQ: d, m + reference nibble qs) -> fragment and side images;
// one lane quad per block
__global__ void k_actq41_to_f16(ActQ q, int N, int K, uint4 * __restrict__ xm, uint4 * __restrict__ xs) {
    const int nb = K / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;   // (token, block, quad lane)
    const long tb = idx >> 2;
    const bool live = tb < (long) N * nb;
    const int k = (int) (idx & 3);
    const long tbc = live ? tb : 0;
    const uint4 qs = q.qs[tbc];
    const uint32_t wd[4] = {qs.x, qs.y, qs.z, qs.w};
    if (live) act41_emit((int) (tbc / nb), nb, (int) (tbc % nb), k, wd[k], q.d[tbc], q.m[tbc], xm, xs);
}

// weight images of a Q4_1 octet image (k_repack_q41 layout): one thread per (32-row tile,
// block, lane (rho, h)).  a16: the chain fragments 2c+h (c = 0..3) of row 32 rt + rho as
// f16 q in the order e0 e2 e1 e3, pairs side by side; side: h = 0 {the row's four group
// sums of the block as f16, d}, h = 1 {ones, m}
__global__ void k_mm41_images(const uint4 * __restrict__ nibi, const float * __restrict__ scl, int M, int K,
                              uint2 * __restrict__ a16, uint4 * __restrict__ side) {
    const int nb = K / 32, NC = (nb + 31) / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;     // (rt * nb + b) * 64 + lane
    if (idx >= (long) (M / 32) * nb * 64) return;
    const int lane = (int) (idx & 63), h = lane >> 5;
    const long rb = idx >> 6;
    const int b = (int) (rb % nb), rt = (int) (rb / nb);
    const int row = rt * 32 + (lane & 31);
    const size_t gbase = (((size_t) (row >> 3) * NC + (b >> 5)) * 4 + ((b & 31) >> 3)) * 64 + 8 * (row & 7);
    uint32_t field[8];                          // chain j: nibbles {2j, 2j+1, 16+2j, 17+2j}
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint4 v = nibi[gbase + j];
        const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
        field[j] = (wd[(b & 7) >> 1] >> (16 * (b & 1))) & 0xFFFFu;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const uint32_t tf = field[2 * c + h];
        a16[((((size_t) rt * nb + b) * 2 + (c >> 1)) * 64 + lane) * 2 + (c & 1)] =
            make_uint2(h16(nib(tf, 0)) | h16(nib(tf, 2)) << 16, h16(nib(tf, 1)) | h16(nib(tf, 3)) << 16);
    }
    // group q = elements 8q..8q+7: the low (q < 2) or high (q >= 2) nibble pairs of chains 4(q&1)..+3
    uint32_t gs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        uint32_t s = 0;
#pragma unroll
        for (int j = 4 * (q & 1); j < 4 * (q & 1) + 4; ++j) s += nib(field[j], 2 * (q >> 1)) + nib(field[j], 2 * (q >> 1) + 1);
        gs[q] = s;
    }
    // d / m of block b: scl[g][c][dm][8r + j] component mq, b = 32c + 8mq + j
    const size_t sidx = ((((size_t) (row >> 3) * NC + (b >> 5)) * 2 + h) * 64 + 8 * (row & 7) + (b & 7)) * 4 + ((b & 31) >> 3);
    const uint32_t sv = __builtin_bit_cast(uint32_t, scl[sidx]);
    side[idx] = h == 0 ? make_uint4(h16(gs[0]) | h16(gs[1]) << 16, h16(gs[2]) | h16(gs[3]) << 16, sv, 0u)
                       : make_uint4(F16_ONE | F16_ONE << 16, F16_ONE | F16_ONE << 16, sv, 0u);
}

}  // namespace

size_t mm41_side_bytes(int M, int K) { return (size_t) (M / 32) * (K / 32) * 64 * 16; }
size_t mm41_act_side_bytes(int N, int K) { return (size_t) ((N + TN - 1) / TN) * (K / 32) * 64 * 16; }

hipError_t launch_build_mm41(const QMatrix & w, void * a16, void * side, hipStream_t s) {
    if (w.qtype != Q4_1 || w.M % 32 || w.K % 256) return hipErrorInvalidValue;
    const long n = (long) (w.M / 32) * (w.K / 32) * 64;
    LVK_LAUNCH(k_mm41_images, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, w.nib, (const float *) w.scl, w.M,
               w.K, (uint2 *) a16, (uint4 *) side);
    return hipGetLastError();
}

bool mm_mfma41_supported(const QMatrix & w) {
    return w.qtype == Q4_1 && w.a16 && w.side && w.M % TM == 0 && w.K % 256 == 0;
}

hipError_t launch_mm_mfma41(const QMatrix & w, const void * xm, const void * xs, int N, float * y, int ldy, int epi,
                            const uint16_t * silu_tab, hipStream_t s, const RopeKV * rk) {
    if (!mm_mfma41_supported(w) || N <= 0 || (epi == EPI_ROPE_KV) != (rk != nullptr)) return hipErrorInvalidValue;
    Mm41Params P{};
    if (rk) {
        if (w.M != 3 * rk->E || rk->E % 32 || rk->hd % 4 || !rk->sp) return hipErrorInvalidValue;
        P.rk = *rk;
    }
    P.a16 = (const uint4 *) w.a16; P.side = (const uint4 *) w.side;
    P.xm = (const uint4 *) xm; P.xs = (const uint4 *) xs;
    P.M = w.M; P.nb = w.K / 32; P.N = N; P.ntt = (N + TN - 1) / TN;
    P.y = y; P.ldy = ldy; P.silu_tab = silu_tab;
    P.supertile = mm_supertile();
    const dim3 grid((w.M / TM) * P.ntt);
    // LVK_MM41_DMA=0: the register-ring kernel instead of the LDS-DMA ring
    const char * dma_env = getenv("LVK_MM41_DMA");
    const bool dma = !dma_env || atoi(dma_env) != 0;
#define LVK_MM41_GO(E)                                                                   \
    do {                                                                                 \
        if (dma) LVK_LAUNCH(k_mm_q41_dma<E>, grid, dim3(NT), LDS41, s, P);               \
        else LVK_LAUNCH(k_mm_q41_mfma<E>, grid, dim3(NT), 0, s, P);                      \
    } while (0)
    switch (epi) {
        case EPI_STORE: LVK_MM41_GO(EPI_STORE); break;
        case EPI_RESID: LVK_MM41_GO(EPI_RESID); break;
        case EPI_SWIGLU_F32: LVK_MM41_GO(EPI_SWIGLU_F32); break;
        case EPI_ROPE_KV: LVK_MM41_GO(EPI_ROPE_KV); break;
        default: return hipErrorInvalidValue;
    }
#undef LVK_MM41_GO
    return hipGetLastError();
}

hipError_t launch_act41_f16(const float * x, const float * g, int N, int K, void * xm, void * xs, hipStream_t s) {
    if (K % 256 || N <= 0) return hipErrorInvalidValue;
    const dim3 gt((unsigned) ((N + 127) / 128 * 128));   // XCD-grouped token order
    if (g) LVK_LAUNCH(k_act_q41_f16<true>, gt, dim3(256), 0, s, x, g, N, K, (uint4 *) xm, (uint4 *) xs);
    else LVK_LAUNCH(k_act_q41_f16<false>, gt, dim3(256), 0, s, x, g, N, K, (uint4 *) xm, (uint4 *) xs);
    return hipGetLastError();
}

hipError_t launch_actq41_to_f16(const ActQ & q, int N, int K, void * xm, void * xs, hipStream_t s) {
    if (K % 32 || N <= 0) return hipErrorInvalidValue;
    const long n = (long) N * (K / 32) * 4;
    LVK_LAUNCH(k_actq41_to_f16, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s, q, N, K, (uint4 *) xm,
               (uint4 *) xs);
    return hipGetLastError();
}

}  // namespace lvk
