// lvk_device.h -- gfx950 device helpers shared by the llama.vk_amd kernels.
//
// Numerics contract: every kernel is compiled with
// -ffp-contract=off; fmaf appears exactly where the reference AVX2 code uses
// _mm256_fmadd_ps; float div/sqrt are the correctly rounded sequences hipcc
// emits by default on gfx950; f32->f16 is IEEE RNE (v_cvt_f16_f32), matching
// F16C _cvtss_sh(x, 0) (ggml.c:182-183).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lvk {

constexpr int QK = 32;    // elements per quant block (ggml.c:416)
constexpr int WAVE = 64;  // CDNA wavefront

// f32 -> f16 RNE as an opaque instruction: a plain (_Float16) cast lets the
// backend fold a preceding f32 mul/add into v_fma_mixlo_f16, which rounds the
// exact product straight to f16 (one rounding instead of the reference's two:
// f32 result, then _cvtss_sh) -- observed on ROCm 7.2 in the softmax P->f16.
__device__ __forceinline__ uint16_t f32_to_f16(float x) {
    uint32_t r;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r) : "v"(x));
    return (uint16_t) r;
}
__device__ __forceinline__ float f16_to_f32(uint16_t h) {
    return (float) __builtin_bit_cast(_Float16, h);   // exact
}

// KV-cache / query element store: f16 (the reference's f32 -> f16 cpy, RNE) or, with the
// f32 KV cache (llama_context_params.f16_kv = false, llama.cpp:1614), the f32 value itself;
// `base` then addresses floats (the buffer is sized for 4-byte elements)
__device__ __forceinline__ void kv_store(uint16_t * base, size_t i, float v, int f32) {
    if (f32) ((float *) base)[i] = v;
    else base[i] = f32_to_f16(v);
}

// table_exp_f16[h] (ggml.c:2915-2927: fp16(expf(fp16->f32(h))), built with the
// host's glibc) for the arguments softmax produces (h <= 0, not NaN).
// mode 0 reads the uploaded table; mode 1 computes exp in double, mode 2 with
// the device expf, both rounded to f32 then f16 like the table.  A context
// uses mode 2 or 1 only after exp_check() found it equal to the table on every
// such h (lvk_exp_table_mismatches).
__device__ __forceinline__ uint16_t exp_f16(uint16_t hx, const uint16_t * __restrict__ tab, int mode) {
    if (mode != 0 && ((hx & 0x8000u) || hx == 0) && (hx & 0x7fffu) <= 0x7c00u) {
        const float x = f16_to_f32(hx);
        return f32_to_f16(mode == 2 ? expf(x) : (float) exp((double) x));
    }
    return tab[hx];
}

// softmax exp (exp_f16 semantics) for EM != 0 without a vector load on the common path:
// only NaN arguments (the table covers them; softmax arguments are <= 0 otherwise) take the
// uploaded table, behind a wave-uniform branch, so no vmcnt wait -- which would also wait
// for loads in flight (the decode attention's V DMA) -- sits in the loop
template <int EM>
__device__ __forceinline__ uint16_t exp_softmax(uint16_t hx, const uint16_t * __restrict__ tab, int mode) {
    if constexpr (EM < 0) {
        return exp_f16(hx, tab, mode);
    } else if constexpr (EM == 0) {
        return tab[hx];
    } else {
        const float x = f16_to_f32(hx);
        uint16_t e = f32_to_f16(EM == 2 ? expf(x) : (float) exp((double) x));
        const bool table = !(((hx & 0x8000u) || hx == 0) && (hx & 0x7fffu) <= 0x7c00u);
        if (__builtin_amdgcn_ballot_w64(table) != 0) {
            const uint16_t t = tab[hx];
            e = table ? t : e;
            asm volatile("" : "+v"(e));
        }
        return e;
    }
}

// quad_perm DPP broadcast of lane k (0..3) of each 4-lane quad
template <int K>
__device__ __forceinline__ float quad_bcast(float v) {
    constexpr int ctrl = K | (K << 2) | (K << 4) | (K << 6);
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), ctrl, 0xF, 0xF, false));
}
__device__ __forceinline__ float quad_get(float v, int k) {
    switch (k) {
        case 0: return quad_bcast<0>(v);
        case 1: return quad_bcast<1>(v);
        case 2: return quad_bcast<2>(v);
        default: return quad_bcast<3>(v);
    }
}

// signed int4 x int4 8-way dot (v_dot8_i32_i4, VOP3P with an inline 0
// accumulator: the builtin lowers to v_dot8c + a v_mov of the 0 per call)
__device__ __forceinline__ int dot8(uint32_t a, uint32_t b) {
    int r;
    asm("v_dot8_i32_i4 %0, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// unsigned u4 x u4 8-way dot (v_dot8_u32_u4)
__device__ __forceinline__ int udot8(uint32_t a, uint32_t b) {
    return (int) __builtin_amdgcn_udot8(a, b, 0u, false);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// streamed-once weight loads: non-temporal (nt) global_load_dwordx4
__device__ __forceinline__ uint4 ld_nt(const uint4 * p) {
    const u32x4 v = __builtin_nontemporal_load((const u32x4 *) p);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ double warp_sum_d(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// ggml_compute_forward_rms_norm_f32 (ggml.c:6060-6065) adds the float squares x[i] * x[i] to a
// double in index order; the kernels add the same terms as a tree.  For n nonnegative terms
// either order lies within (n - 1)u of the exact sum (u = 2^-53), so the two means sum / n (one
// more rounding each) differ by at most 2n ulps of the double r = sum / n.  (float) r rounds on
// the 29 double significand bits below the float's; its only rounding boundary is the midpoint
// pattern 2^28.  rms_mean keeps the tree's mean when those bits are more than 4n from the
// midpoint (r a normal float, or 0), else (about one row in 1e5) it returns the mean of an
// index-order re-sum of x[0 .. n): the reference's float mean either way.
// The cold path is out of line, so that its loop adds no registers to the kernels.
__device__ __noinline__ float rms_mean_in_order(const float * x, int n) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) { const float v = x[i]; const float sq = v * v; s += (double) sq; }
    return (float) (s / (double) n);
}
__device__ __forceinline__ float rms_mean(double tree, const float * x, int n) {
    const double r = tree / (double) n;
    const uint64_t rb = (uint64_t) __double_as_longlong(r);
    const uint32_t ex = (uint32_t) (rb >> 52);                  // r >= 0: no sign bit
    const int32_t mid = (int32_t) (uint32_t) (rb & 0x1fffffffu) - (1 << 28);
    const bool safe = rb == 0 || (ex >= 1023 - 126 && ex < 1023 + 128 && (mid > 4 * n || mid < -4 * n));
    if (__builtin_expect(safe, 1)) return (float) r;
    return rms_mean_in_order(x, n);
}
// rms_mean for a call made by all 64 lanes of a wave with the same arguments.  Before the
// index-order re-sum it tries an exactness certificate, split over the lanes: when every square
// is a multiple of 2^m and the sum is below 2^(m+53), every partial sum in any order is exact,
// so the tree's sum is the index-order one.  The synthetic models' activations carry few
// significant bits and often sit exactly on a midpoint, and this certificate covers them.
#ifdef LVK_PROBE_RMSCOUNT
// dev probe build only (make rmscount, tools/rms_fallback_count.py): per-translation-unit
// counters of rms_mean_wave's paths {calls, certificate tried, index-order re-sum}, one count
// per calling wave
static __device__ unsigned long long lvk_rms_ctr[3];
#define LVK_RMS_COUNT(k) do { if ((threadIdx.x & 63) == 0) atomicAdd(&lvk_rms_ctr[k], 1ull); } while (0)
#define LVK_RMS_ACCESSOR(name)                                                                    \
    extern "C" __attribute__((visibility("default"))) int name(unsigned long long * out) {        \
        return (int) hipMemcpyFromSymbol(out, HIP_SYMBOL(::lvk::lvk_rms_ctr), sizeof(::lvk::lvk_rms_ctr));     \
    }
#else
#define LVK_RMS_COUNT(k) do { } while (0)
#define LVK_RMS_ACCESSOR(name)
#endif
__device__ __forceinline__ float rms_mean_wave(double tree, const float * x, int n) {
    const double r = tree / (double) n;
    const uint64_t rb = (uint64_t) __double_as_longlong(r);
    const uint32_t ex = (uint32_t) (rb >> 52);
    const int32_t mid = (int32_t) (uint32_t) (rb & 0x1fffffffu) - (1 << 28);
    const bool safe = rb == 0 || (ex >= 1023 - 126 && ex < 1023 + 128 && (mid > 4 * n || mid < -4 * n));
    LVK_RMS_COUNT(0);
    if (__builtin_expect(safe, 1)) return (float) r;
    LVK_RMS_COUNT(1);
    int mlow = 1 << 20;            // lowest set-bit exponent over the nonzero squares
    for (int i = (int) (threadIdx.x & 63); i < n; i += 64) {
        const float v = x[i];
        const float sq = v * v;
        const uint32_t b = __float_as_uint(sq);
        if (b != 0u) {
            const uint32_t e = b >> 23, man = (b & 0x7fffffu) | (e ? 0x800000u : 0u);
            const int low = (e ? (int) e - 150 : -149) + __builtin_ctz(man);
            mlow = low < mlow ? low : mlow;
        }
    }
    for (int o = 32; o > 0; o >>= 1) { const int t = __shfl_xor(mlow, o); mlow = t < mlow ? t : mlow; }
    if (mlow == (1 << 20) || tree <= ldexp(1.0, mlow + 52)) return (float) r;
    LVK_RMS_COUNT(2);
    return rms_mean_in_order(x, n);
}
// whole-wave double sum through DPP (quad xor 1, xor 2, half-row and row
// mirrors) and four readlanes; every lane returns the same value, and the
// association order is fixed: ((row0 + row1) + (row2 + row3)) of 16-lane trees
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const int2 i = __builtin_bit_cast(int2, v);
    int2 o;
    o.x = __builtin_amdgcn_mov_dpp(i.x, CTRL, 0xF, 0xF, false);
    o.y = __builtin_amdgcn_mov_dpp(i.y, CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, o);
}
__device__ __forceinline__ double wave_sum_d(double v) {
    v += dpp_d<0xB1>(v);     // quad_perm [1,0,3,2]
    v += dpp_d<0x4E>(v);     // quad_perm [2,3,0,1]
    v += dpp_d<0x141>(v);    // row_half_mirror
    v += dpp_d<0x140>(v);    // row_mirror
    const int2 i = __builtin_bit_cast(int2, v);
    double r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        int2 o;
        o.x = __builtin_amdgcn_readlane(i.x, 16 * k);
        o.y = __builtin_amdgcn_readlane(i.y, 16 * k);
        r[k] = __builtin_bit_cast(double, o);
    }
    return (r[0] + r[1]) + (r[2] + r[3]);
}
// whole-wave float max through DPP + readlanes (max is exact in any order)
__device__ __forceinline__ float wave_max_f(float v) {
    auto mx = [](float a, float b) { return b > a ? b : a; };
    v = mx(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false)));
    v = mx(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false)));
    v = mx(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)));
    v = mx(v, __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)));
    const int i = __builtin_bit_cast(int, v);
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 0));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 16));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 32));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(i, 48));
    return mx(mx(r0, r1), mx(r2, r3));
}
__device__ __forceinline__ float warp_max(float v) {
    for (int o = 32; o > 0; o >>= 1) { const float w = __shfl_xor(v, o); v = w > v ? w : v; }
    return v;
}

// Masked B fragment image of the MFMA prompt matmul (mm_mfma.hip): token t, block b of nb,
// chain pair c (chains 2c, 2c+1), fragment lane l.  The fragments of chain pairs 2q and 2q+1
// sit side by side per lane, so a wave fetches two MFMA B operands with one 16-byte-per-lane
// load (the texture unit's cost is per load instruction: 8-byte loads moved half the bytes
// per cycle).  Returns the index in 8-byte units.
__device__ __forceinline__ size_t xm_slot(int t, int nb, int b, int c, int l) {
    return ((((size_t) (t >> 4) * nb + b) * 2 + (c >> 1)) * 64 + l) * 2 + (c & 1);
}

// token of workgroup i in a one-workgroup-per-token launch of ceil(N/128)*128 workgroups:
// workgroup i runs on XCD i % 8, and the 16 tokens of token tile tau all go to XCD tau % 8,
// so the 16-byte pieces they write into the same fragment-image lines (xm_slot) meet in one
// L2 instead of being merged from 8 XCDs (>= N: no token)
__device__ __forceinline__ int xcd_grouped_token(int i) {
    const int tau = ((i >> 7) << 3) | (i & 7);
    return tau * 16 + ((i >> 3) & 15);
}

// prompt-matmul tile of workgroup slot L (its XCD-contiguous index, mm_mfma.hip): row tile
// rt, token tile tt.  Row tiles outer, token tiles inner; supertile: groups of 4 row tiles x
// every token tile with the token tiles outer, so the 64 workgroups an XCD runs at once share
// 4 weight tiles and 16 activation tiles in its L2 instead of 2 weight tiles and the whole
// activation image (7B 512-token prompt 45.3 -> 43.7 ms, profiles/r04_prompt_variants.jsonl);
// LVK_MM_SUPERTILE = R > 1 sets the group width (A/B)
__device__ __forceinline__ void mm_tile(int L, int ntt, int nrt, int supertile, int & rt, int & tt) {
    tt = L % ntt;
    rt = L / ntt;
    const int R = supertile == 1 ? 4 : supertile;     // row tiles per super tile (1: the default 4)
    if (R > 1) {
        const int per = R * ntt, sidx = L / per, wi = L % per;
        if (R * sidx + R - 1 < nrt) { tt = wi / R; rt = R * sidx + wi % R; }
    }
}

// fmaf(f16 half HA of a, f16 half HB of b, c): v_fma_mix converts both f16 operands
// exactly and rounds once, the same result as fmaf on the converted values
template <int HA, int HB>
__device__ __forceinline__ float fma_mix_hh(uint32_t a, uint32_t b, float c) {
    float d;
    if constexpr (HA == 0 && HB == 0)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[0,0,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    else if constexpr (HA == 1 && HB == 1)
        asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    else
        static_assert(HA == HB, "same halves only");
    return d;
}

}  // namespace lvk
