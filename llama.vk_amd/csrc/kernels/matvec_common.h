// matvec_common.h -- device helpers shared by the Q4_0 matvec kernels
// (activation table in LDS, reference Q4_0 quantizer pieces, octet reduce).
#pragma once
#include "lvk_device.h"

namespace lvk {
namespace mv {

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

}  // namespace mv
}  // namespace lvk
