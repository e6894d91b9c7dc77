// matvec_common.h -- device helpers shared by the Q4_0 matvec kernels
// (activation table in LDS, reference Q4_0 quantizer pieces, octet reduce).
#pragma once
#include "lvk_device.h"
#include "lvk_kernels.h"

namespace lvk {
namespace mv {

// Marks loaded values as produced here for hipcc's wait-count pass.  A load whose result is
// first used after a branch join (e.g. the optional weight issue of a matvec prologue) is
// otherwise waited for with the most conservative count of the two paths -- vmcnt(1) behind
// a weight burst, i.e. the whole burst.  Passing the values through an empty asm statement
// where the exact count is known (right after the burst, in each branch) puts the precise
// wait there and none later.
__device__ __forceinline__ void launder(float4 & v) {
    float a = v.x, b = v.y, c = v.z, d = v.w;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    v = make_float4(a, b, c, d);
}
__device__ __forceinline__ void launder(uint4 & v) {
    uint32_t a = v.x, b = v.y, c = v.z, d = v.w;
    asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
    v = make_uint4(a, b, c, d);
}
__device__ __forceinline__ void launder(float & v) { asm volatile("" : "+v"(v)); }

// LDS activation table of one token:
//   act[nb/4][8] uint4 : for 4 blocks 4u..4u+3 and chain j:
//       {a(4u,j), a(4u+1,j) << 16, a(4u+2,j), a(4u+3,j) << 16}
//     a(i,j) = signed nibbles of elements 4j..4j+3 of block i (16 bits)
//   dxp[NC][8][4] float : dx of block 32c + 8m + j at [c][j][m]
__device__ __forceinline__ void act_store(uint32_t * act, float * dxp, int i, int q, uint32_t dw_ref, float d,
                                          bool write_d) {
    // dw_ref = elements 8q..8q+7 of block i in the reference nibble convention (q+8)
    const uint32_t s = dw_ref ^ 0x88888888u;
    const uint32_t lo = s & 0xFFFFu, hi = s >> 16;       // chains 2q, 2q+1
    const int slot = i & 3;
    const uint32_t sh = (slot & 1) ? 16u : 0u;
    uint32_t * base = act + (size_t) (i >> 2) * 32;      // 8 chains x 4 dwords
    base[(2 * q) * 4 + slot] = lo << sh;
    base[(2 * q + 1) * 4 + slot] = hi << sh;
    if (write_d) dxp[(size_t) (i >> 5) * 32 + (i & 7) * 4 + ((i >> 3) & 3)] = d;
}

// RNE quantization of 8 values (ggml.c:655-684) -> reference nibble dword
__device__ __forceinline__ uint32_t q40_pack8(const float v[8], float id) {
    uint32_t w = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int q = (int) __builtin_rintf(v[k] * id) + 8;
        w |= (uint32_t) (q & 15) << (4 * k);
    }
    return w;
}

// quantize 32 values held one per lane in a 32-lane half into a reference
// Q4_0 block (quantize_row_q4_0 AVX2, ggml.c:621-685)
__device__ __forceinline__ void quantize32_q40(float v, int lane, float * d_out, uint4 * qs_out, uint32_t * scratch) {
    float amax = fabsf(v);
    for (int o = 16; o > 0; o >>= 1) { const float w = __shfl_xor(amax, o); amax = w > amax ? w : amax; }
    const float d = amax / 7.0f;
    const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
    const uint32_t q = (uint32_t) ((int) __builtin_rintf(v * id) + 8) & 15u;
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

// fixed AVX2 horizontal order of the 8 chains of a row (ggml.c:2019-2024):
// lanes 8r..8r+7 hold a_0..a_7; every lane returns the row's dot product
__device__ __forceinline__ float octet_reduce(float a) {
    const float b = a + __shfl_xor(a, 4);       // r_j = a_j + a_{j+4}
    const float c = b + __shfl_xor(b, 2);       // r0+r2, r1+r3
    return c + __shfl_xor(c, 1);                // (r0+r2) + (r1+r3)
}

// AVX2 emulation helpers (ggml.c:890-915): cvtps_epi32 of an out-of-range value
// gives INT_MIN; packs_epi32 + packs_epi16 saturate to int8; packNibbles packs
// (b0 | b1 << 4) with unsigned saturation (ggml.c:440-452)
__device__ __forceinline__ int32_t cvt_ps_epi32(float v) {
    if (!(v >= -2147483648.0f && v < 2147483648.0f)) return (int32_t) 0x80000000u;
    return (int32_t) v;
}
__device__ __forceinline__ uint32_t sat8u(int32_t v) {
    v = v > 127 ? 127 : (v < -128 ? -128 : v);
    return (uint32_t) (uint8_t) (int8_t) v;
}
__device__ __forceinline__ uint32_t pack_nib(uint32_t b0, uint32_t b1) {
    const uint32_t v = b0 | (b1 << 4);
    return v > 255u ? 255u : v;
}

// the AVX2 max/min tree of quantize_row_q4_1 (ggml.c:857-871) on a block whose
// element e is e8[l] of "lane" k = e/8, l = e%8: max(a,b) = a > b ? a : b, so
// the sign of a zero extremum follows the reference's lane order
struct MinMax { float mx, mn; };
__device__ __forceinline__ MinMax q41_tree(const float (&cm)[8], const float (&cn)[8]) {
    float x4[4], n4[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        x4[l] = cm[4 + l] > cm[l] ? cm[4 + l] : cm[l];
        n4[l] = cn[4 + l] < cn[l] ? cn[4 + l] : cn[l];
    }
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        x4[l] = x4[l] > x4[l + 2] ? x4[l] : x4[l + 2];
        n4[l] = n4[l] < n4[l + 2] ? n4[l] : n4[l + 2];
    }
    return {x4[0] > x4[1] ? x4[0] : x4[1], n4[0] < n4[1] ? n4[0] : n4[1]};
}

// quantize 8 elements of a block given its min and 1/d: 4 qs bytes
__device__ __forceinline__ uint32_t q41_pack8(const float v[8], float vmin, float id) {
    uint32_t qword = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const float t0 = v[2 * p] - vmin, t1 = v[2 * p + 1] - vmin;     // sub, then mul (ggml.c:883-886)
        const float w0 = t0 * id, w1 = t1 * id;
        const uint32_t b0 = sat8u(cvt_ps_epi32(__builtin_rintf(w0)));
        const uint32_t b1 = sat8u(cvt_ps_epi32(__builtin_rintf(w1)));
        qword |= pack_nib(b0, b1) << (8 * p);
    }
    return qword;
}


// quantize_row_q4_1 of 32 values staged in LDS (xb[0..31]); lanes k < 4 of the
// calling group return qs word k; every lane returns d and m
__device__ __forceinline__ void q41_block_lds(const float * xb, int k, float & d, float & m, uint32_t & qword) {
    float cm[8], cn[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float a0 = xb[l], a1 = xb[8 + l], a2 = xb[16 + l], a3 = xb[24 + l];
        float x = a0 > a1 ? a0 : a1;  x = x > a2 ? x : a2;  x = x > a3 ? x : a3;
        float n = a0 < a1 ? a0 : a1;  n = n < a2 ? n : a2;  n = n < a3 ? n : a3;
        cm[l] = x; cn[l] = n;
    }
    const MinMax mm = q41_tree(cm, cn);
    d = (mm.mx - mm.mn) / 15.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    m = mm.mn;
    float v[8];
    const int kk = k & 3;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = xb[8 * kk + e];
    qword = q41_pack8(v, mm.mn, id);
}

// ---- Q4_1 pieces shared by matvec_q41.hip and matvec_cu41.hip

// quantize_row_q4_1 of one block held by a lane quad (lane k: elements 8k..8k+7)
__device__ __forceinline__ void q41_quad(const float v[8], float & d, float & m, uint32_t & qword) {
    float cm[8], cn[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float a0 = quad_bcast<0>(v[l]), a1 = quad_bcast<1>(v[l]);
        const float a2 = quad_bcast<2>(v[l]), a3 = quad_bcast<3>(v[l]);
        float x = a0 > a1 ? a0 : a1;  x = x > a2 ? x : a2;  x = x > a3 ? x : a3;
        float n = a0 < a1 ? a0 : a1;  n = n < a2 ? n : a2;  n = n < a3 ? n : a3;
        cm[l] = x; cn[l] = n;
    }
    const MinMax mm = q41_tree(cm, cn);
    d = (mm.mx - mm.mn) / 15.0f;                          // ggml.c:874
    const float id = d != 0.0f ? 1.0f / d : 0.0f;         // ggml.c:875
    m = mm.mn;
    qword = q41_pack8(v, mm.mn, id);
}

// Q4_1 activation table of one token:
//   act[nb/4][8] uint4 : {a(4u,j), a(4u+1,j) << 16, a(4u+2,j), a(4u+3,j) << 16}
//   dyv, myv [NC][8][4] : d / m of block 32c + 8m + j at [c][j][m]
//   ysum[nb/4][4 q][4]  : sum of the 8 nibbles 8q..8q+7 of block 4u+t at [u][q][t]
// ysum: float per (block, chain pair) for matvec_q41.hip; one byte each for
// matvec_cu41.hip (the sums are integers <= 120), same index
template <typename YS>
__device__ __forceinline__ void act41_store(uint32_t * act, float * dyv, float * myv, YS * ysum, int i,
                                            const uint32_t qs[4], float d, float m) {
    const int slot = i & 3;
    const uint32_t sh = (slot & 1) ? 16u : 0u;
    uint32_t * base = act + (size_t) (i >> 2) * 32;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const uint32_t lo = (qs[j >> 2] >> (8 * (j & 3))) & 0xFFu;
        const uint32_t hi = (qs[2 + (j >> 2)] >> (8 * (j & 3))) & 0xFFu;
        base[j * 4 + slot] = (lo | (hi << 8)) << sh;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) ysum[(size_t) (i >> 2) * 16 + q * 4 + slot] = (YS) udot8(qs[q], 0x11111111u);
    const int o = (i >> 5) * 32 + (i & 7) * 4 + ((i >> 3) & 3);
    dyv[o] = d;
    myv[o] = m;
}

// even-chain weight sums of two blocks packed in one weight word (low 16 bits
// block A, high 16 bits block B; each 16-bit group = [qs byte j, qs byte 8+j]).
// Quad 0 of a row holds chains 0-3 (first bytes: elements 0-7, second bytes:
// 16-23), quad 1 chains 4-7 (8-15, 24-31); chain 2q needs elements 8q..8q+7:
// j=0 own quad first, j=2 other quad first, j=4 other quad second, j=6 own
// quad second.  Returns {S_A, S_B} in the low/high 16 bits (odd lanes: junk).
__device__ __forceinline__ uint32_t wsum_word(uint32_t w, bool other, uint32_t shift) {
    uint32_t t = (w & 0x0F0F0F0Fu) + ((w >> 4) & 0x0F0F0F0Fu);                  // per byte: its 2 nibbles
    t += (uint32_t) __builtin_amdgcn_mov_dpp((int) t, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    t += (uint32_t) __builtin_amdgcn_mov_dpp((int) t, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
    const uint32_t mir = (uint32_t) __builtin_amdgcn_mov_dpp((int) t, 0x141, 0xF, 0xF, false);   // row_half_mirror
    return ((other ? mir : t) >> shift) & 0x00FF00FFu;
}

// QKV epilogue of both decode matvecs, per output row (lane row r of an 8-row group, chain
// lane j): RoPE mode 0 on q and k (ggml.c:7209-7223; rows e and e^1 are lanes l and l^8),
// the q row / K-cache row / V-cache column stores (llama.cpp:996-1008).
__device__ __forceinline__ void qkv_epilogue(float res, int row, int j, int E, int hd, int pos,
                                             const float2 * rope, uint16_t * q16, uint16_t * kc, uint16_t * vc,
                                             int n_ctx, int kv32) {
    const int which = row / E;              // 0 q, 1 k, 2 v (uniform per wave: E % 8 == 0)
    const int e = row - which * E;
    const float other = __shfl_xor(res, 8);   // row e^1 lives in lanes of row r^1
    float out = res;
    if (which < 2) {
        const int i0 = e % hd;
        const float2 cs = rope[(size_t) pos * (hd / 2) + (i0 >> 1)];
        if ((i0 & 1) == 0) { const float a = res * cs.x, b = other * cs.y; out = a - b; }
        else               { const float a = other * cs.y, b = res * cs.x; out = a + b; }
    }
    if (j == 0) {
        if (which == 0)      kv_store(q16, e, out, kv32);
        else if (which == 1) kv_store(kc, (size_t) pos * E + e, out, kv32);
        else                 kv_store(vc, (size_t) e * n_ctx + pos, out, kv32);
    }
}

// qkv_epilogue with the lane's RoPE pair already loaded (cs: rope[pos * hd / 2 + (e % hd) / 2])
__device__ __forceinline__ void qkv_epilogue_cs(float res, int row, int j, int E, int hd, int pos, float2 cs,
                                                uint16_t * q16, uint16_t * kc, uint16_t * vc, int n_ctx, int kv32) {
    const int which = row / E;
    const int e = row - which * E;
    const float other = __shfl_xor(res, 8);
    float out = res;
    if (which < 2) {
        const int i0 = e % hd;
        if ((i0 & 1) == 0) { const float a = res * cs.x, b = other * cs.y; out = a - b; }
        else               { const float a = other * cs.y, b = res * cs.x; out = a + b; }
    }
    if (j == 0) {
        if (which == 0)      kv_store(q16, e, out, kv32);
        else if (which == 1) kv_store(kc, (size_t) pos * E + e, out, kv32);
        else                 kv_store(vc, (size_t) e * n_ctx + pos, out, kv32);
    }
}

}  // namespace mv
// the RoPE + KV epilogue of a prompt-matmul lane (mm_mfma.hip, mm_mfma41.hip): the lane holds
// rows m0 + 32w + 8q + 4h + p (p = 0..3) of token n; rows [0, E) Q, [E, 2E) K, [2E, 3E) V.
// rope_kv_cs loads the 8 cos / sin pairs (before the reduction and any store: issued between
// stores they each wait a full latency), rope_kv_store does RoPE (ggml.c:7209-7232, as
// k_rope_kv) and the f16 stores of the cache views (llama.cpp:1010-1024)
__device__ __forceinline__ void rope_kv_cs(const RopeKV & r, int N, int n, int h, int w, int m0, float2 (&cs)[4][2]) {
    const int pos = r.sp->n_past + (n < N ? n : N - 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = (m0 + 32 * w + 8 * q + 4 * h) % r.hd;
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) cs[q][pp] = r.rope[(size_t) pos * (r.hd / 2) + (e >> 1) + pp];
    }
}
__device__ __forceinline__ void rope_kv_store(const RopeKV & r, const float (&res)[16], const float2 (&cs)[4][2], int n,
                                              int h, int w, int m0) {
    const int pos = r.sp->n_past + n;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = m0 + 32 * w + 8 * q + 4 * h;
        const int which = row / r.E, e = row - which * r.E;
        if (which < 2) {
            uint32_t hw[2];
#pragma unroll
            for (int pp = 0; pp < 4; pp += 2) {
                const float x0 = res[4 * q + pp], x1 = res[4 * q + pp + 1];
                const float2 c = cs[q][pp >> 1];
                const float a0 = x0 * c.x, b0 = x1 * c.y;
                const float o0 = a0 - b0;
                const float a1 = x0 * c.y, b1 = x1 * c.x;
                const float o1 = a1 + b1;
                hw[pp >> 1] = (uint32_t) f32_to_f16(o0) | (uint32_t) f32_to_f16(o1) << 16;
            }
            uint16_t * dst = which == 0 ? r.q16 + (size_t) n * r.E + e : r.kc + (size_t) pos * r.E + e;
            *(uint2 *) dst = make_uint2(hw[0], hw[1]);
        } else {
#pragma unroll
            for (int pp = 0; pp < 4; ++pp) r.vc[(size_t) (e + pp) * r.n_ctx + pos] = f32_to_f16(res[4 * q + pp]);
        }
    }
}

}  // namespace lvk
