// mm41_common.h -- the Q4_1 MFMA prompt path's activation operand writer (mm_mfma41.hip),
// shared by its activation quantizers and the prompt attention's Wo-input epilogue.
#pragma once
#include "lvk_device.h"

namespace lvk {

constexpr uint32_t F16_ONE = 0x3C00u;

__device__ __forceinline__ uint32_t h16(uint32_t q) { return __builtin_bit_cast(uint16_t, (_Float16) (float) q); }
__device__ __forceinline__ uint32_t nib(uint32_t w, int i) { return (w >> (4 * i)) & 15u; }

// the operand writes of one quantized block of token t held by a lane quad: quad lane k
// has the block's elements 8k..8k+7 as qword (nibble i = element 8k+i), d and m
// Fragment image xm (chain pairs, as xm_slot) and side image xs [N/16][nb][64] x 16 B:
//   lane (n, jj 0, h 0) {ones, d, m}, (n, 1, 0) {0, d, 0}, (n, 0, 1) {0, m, 0},
//   (n, 1, 1) {the four group sums, m, d}
__device__ __forceinline__ void act41_emit(int t, int nb, int b, int k, uint32_t qword, float d, float m,
                                           uint4 * __restrict__ xm, uint4 * __restrict__ xs) {
    const int lane = threadIdx.x & 63;
    const int base = lane & ~3;
    // chain pair (2k, 2k+1) = elements 4k..4k+3 (quad lane k/2) and 16+4k.. (quad lane 2+k/2)
    const uint32_t lo = (uint32_t) __shfl((int) qword, base | (k >> 1));
    const uint32_t hi = (uint32_t) __shfl((int) qword, base | (2 + (k >> 1)));
    const int o = 4 * (k & 1);
    // fragment order e0 e2 e1 e3 with e = {2j, 2j+1, 16+2j, 17+2j} (as the a16 image)
    const uint2 f0 = make_uint2(h16(nib(lo, o)) | h16(nib(hi, o)) << 16, h16(nib(lo, o + 1)) | h16(nib(hi, o + 1)) << 16);
    const uint2 f1 = make_uint2(h16(nib(lo, o + 2)) | h16(nib(hi, o + 2)) << 16,
                                h16(nib(lo, o + 3)) | h16(nib(hi, o + 3)) << 16);
    uint2 * xm2 = (uint2 *) xm;
    const int n = t & 15;
    xm2[xm_slot(t, nb, b, k, n)] = f0;          // chain 2k   -> lane (n, jj 0, h 0)
    xm2[xm_slot(t, nb, b, k, 48 + n)] = f1;     // chain 2k+1 -> lane (n, jj 1, h 1)
    // the activation sums of groups 0..3 (quad lane q sums group q)
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += nib(qword, i);
    const float sf = (float) s;
    const uint32_t y0 = h16((uint32_t) quad_bcast<0>(sf)), y1 = h16((uint32_t) quad_bcast<1>(sf));
    const uint32_t y2 = h16((uint32_t) quad_bcast<2>(sf)), y3 = h16((uint32_t) quad_bcast<3>(sf));
    const uint32_t db = __builtin_bit_cast(uint32_t, d), mb = __builtin_bit_cast(uint32_t, m);
    uint4 v;
    switch (k) {
        case 0: v = make_uint4(F16_ONE | F16_ONE << 16, F16_ONE | F16_ONE << 16, db, mb); break;  // (jj 0, h 0)
        case 1: v = make_uint4(0u, 0u, db, 0u); break;                                           // (jj 1, h 0)
        case 2: v = make_uint4(0u, 0u, mb, 0u); break;                                           // (jj 0, h 1)
        default: v = make_uint4(y0 | y1 << 16, y2 | y3 << 16, mb, db); break;                    // (jj 1, h 1)
    }
    xs[((size_t) (t >> 4) * nb + b) * 64 + 16 * k + n] = v;
}

}  // namespace lvk
