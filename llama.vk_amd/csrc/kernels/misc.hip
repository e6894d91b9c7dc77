// misc.hip -- token embedding rows, one-time weight repack into the
// quad-sliced HBM image, and a standalone activation quantizer.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"
#include <climits>

namespace lvk {
thread_local LaunchEvents g_launch_events;

namespace {

// get_rows + dequantize_row_q4_0/q4_1 AVX2 (ggml.c:6868-6895, 968-1000, 1086-1115)
__global__ void k_embed(const uint8_t * __restrict__ emb, int type, int E, const int * __restrict__ tokens,
                        float * __restrict__ x) {
    const int t = blockIdx.y;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E) return;
    const size_t tok = (size_t) tokens[t];
    float v;
    if (type == Q4_0) {
        const uint8_t * b = emb + tok * (size_t) (E / 32) * 20 + (size_t) (e / 32) * 20;
        const float d = *(const float *) b;
        const uint8_t byte = b[4 + (e % 32) / 2];
        const int qv = (e & 1) ? (byte >> 4) : (byte & 15);
        v = (float) (qv - 8) * d;
    } else if (type == Q4_1) {
        const uint8_t * b = emb + tok * (size_t) (E / 32) * 24 + (size_t) (e / 32) * 24;
        const float d = *(const float *) b, m = *(const float *) (b + 4);
        const uint8_t byte = b[8 + (e % 32) / 2];
        const int qv = (e & 1) ? (byte >> 4) : (byte & 15);
        const float a = (float) qv * d;
        v = a + m;
    } else if (type == 1) {   // f16
        v = f16_to_f32(((const uint16_t *) emb)[tok * E + e]);
    } else {                  // f32
        v = ((const float *) emb)[tok * E + e];
    }
    x[(size_t) t * E + e] = v;
}

// Q4_0 file rows -> octet image (matvec_q4.hip).  One thread per
// (row, 32-block chunk c, chain j):
//   a(i,j)  = (qs_i[2j] | qs_i[2j+1] << 8) ^ 0x8888   (elements 4j..4j+3, signed)
//   W(p,j)  = a(2p,j) | a(2p+1,j) << 16              (block pair p)
//   nib[g][c][sb][8r+j] = {W(16c+4sb+k, j), k = 0..3}  (blocks 32c+8sb .. +7)
//   scl[g][c][8r+j]     = {d(32c+8m+j), m = 0..3}
// Sub-chunks / blocks past the row end are zero (never consumed).
__global__ void k_repack_q40(const uint8_t * __restrict__ src, int M, int K, uint4 * __restrict__ nib,
                             float4 * __restrict__ scl, int il4) {
    const int nb = K / 32, NC = (nb + 31) / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long) M * NC * 8) return;
    const int j = (int) (idx & 7);
    const long rc = idx >> 3;
    const int row = (int) (rc / NC), c = (int) (rc % NC);
    const int g = row / 8, r = row % 8;
    const int lane = 8 * r + j;
    // il4: src holds two M/2-row matrices [A; B], fused per 4 rows (A0-3 B0-3 A4-7 ...)
    const int srow = il4 ? ((row & 7) < 4 ? (row >> 3) * 4 + (row & 7) : M / 2 + (row >> 3) * 4 + (row & 7) - 4) : row;
    const uint8_t * rb = src + (size_t) srow * nb * 20;
    auto grp = [&](int i) -> uint32_t {
        if (i >= nb) return 0u;
        const uint8_t * b = rb + (size_t) i * 20;
        return ((uint32_t) b[4 + 2 * j] | ((uint32_t) b[5 + 2 * j] << 8)) ^ 0x8888u;
    };
    for (int sb = 0; sb < 4; ++sb) {
        uint32_t w[4];
        for (int k = 0; k < 4; ++k) {
            const int i = 32 * c + 8 * sb + 2 * k;
            w[k] = (i < nb) ? (grp(i) | (grp(i + 1) << 16)) : 0u;
        }
        nib[(((size_t) g * NC + c) * 4 + sb) * 64 + lane] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    float d[4];
    for (int m = 0; m < 4; ++m) {
        const int i = 32 * c + 8 * m + j;
        d[m] = (i < nb) ? *(const float *) (rb + (size_t) i * 20) : 0.0f;
    }
    scl[((size_t) g * NC + c) * 64 + lane] = make_float4(d[0], d[1], d[2], d[3]);
}

// Q4_1 file rows (d, m, qs[16]) -> octet image (matvec_q41.hip):
//   a(i,j) = qs_i[j] | qs_i[8+j] << 8    (elements 2j, 2j+1, 16+2j, 17+2j, unsigned)
//   W(p,j) = a(2p,j) | a(2p+1,j) << 16
//   scl[g][c][0][8r+j] = {d(32c+8m+j)}, scl[g][c][1][8r+j] = {m(32c+8m+j)}, m = 0..3
__global__ void k_repack_q41(const uint8_t * __restrict__ src, int M, int K, uint4 * __restrict__ nib,
                             float4 * __restrict__ scl, int il4) {
    const int nb = K / 32, NC = (nb + 31) / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long) M * NC * 8) return;
    const int j = (int) (idx & 7);
    const long rc = idx >> 3;
    const int row = (int) (rc / NC), c = (int) (rc % NC);
    const int g = row / 8, r = row % 8;
    const int lane = 8 * r + j;
    const int srow = il4 ? ((row & 7) < 4 ? (row >> 3) * 4 + (row & 7) : M / 2 + (row >> 3) * 4 + (row & 7) - 4) : row;
    const uint8_t * rb = src + (size_t) srow * nb * 24;
    auto grp = [&](int i) -> uint32_t {
        if (i >= nb) return 0u;
        const uint8_t * b = rb + (size_t) i * 24 + 8;
        return (uint32_t) b[j] | ((uint32_t) b[8 + j] << 8);
    };
    for (int sb = 0; sb < 4; ++sb) {
        uint32_t w[4];
        for (int k = 0; k < 4; ++k) {
            const int i = 32 * c + 8 * sb + 2 * k;
            w[k] = (i < nb) ? (grp(i) | (grp(i + 1) << 16)) : 0u;
        }
        nib[(((size_t) g * NC + c) * 4 + sb) * 64 + lane] = make_uint4(w[0], w[1], w[2], w[3]);
    }
    float d[4], m[4];
    for (int q = 0; q < 4; ++q) {
        const int i = 32 * c + 8 * q + j;
        d[q] = (i < nb) ? *(const float *) (rb + (size_t) i * 24) : 0.0f;
        m[q] = (i < nb) ? *(const float *) (rb + (size_t) i * 24 + 4) : 0.0f;
    }
    scl[(((size_t) g * NC + c) * 2) * 64 + lane] = make_float4(d[0], d[1], d[2], d[3]);
    scl[(((size_t) g * NC + c) * 2 + 1) * 64 + lane] = make_float4(m[0], m[1], m[2], m[3]);
    // weight-sum image after the d/m images (lvk_kernels.h q41_wsum): lane (r, j) holds
    // chain 2k = 2(j/2)'s sums of blocks 32c + 16(j%2) + t, t = 0..15, one byte each
    const int k = j >> 1;
    uint32_t ws[4] = {0u, 0u, 0u, 0u};
    for (int t = 0; t < 16; ++t) {
        const int i = 32 * c + 16 * (j & 1) + t;
        if (i >= nb) break;
        const uint8_t * q = rb + (size_t) i * 24 + 8 + 4 * k;
        uint32_t sum = 0;
        for (int e = 0; e < 4; ++e) sum += (q[e] & 15u) + (q[e] >> 4);
        ws[t >> 2] |= sum << (8 * (t & 3));
    }
    uint4 * wsum = (uint4 *) (scl + (size_t) M * NC * 16);     // d + m: M * NC * 256 bytes
    wsum[((size_t) g * NC + c) * 64 + lane] = make_uint4(ws[0], ws[1], ws[2], ws[3]);
}

// standalone Q4_1 activation quantizer (quantize_row_q4_1 AVX2, ggml.c:847-920),
// one thread per block; output split d / m / qs in the reference nibble layout
__global__ void k_quantize_q41(const float * __restrict__ x, int N, int K, ActQ out) {
    const int nb = K / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long) N * nb) return;
    const int t = (int) (idx / nb), b = (int) (idx % nb);
    const float * xb = x + (size_t) t * K + (size_t) b * 32;
    float cm[8], cn[8];
    for (int l = 0; l < 8; ++l) {
        const float a0 = xb[l], a1 = xb[8 + l], a2 = xb[16 + l], a3 = xb[24 + l];
        float mx = a0 > a1 ? a0 : a1;  mx = mx > a2 ? mx : a2;  mx = mx > a3 ? mx : a3;
        float mn = a0 < a1 ? a0 : a1;  mn = mn < a2 ? mn : a2;  mn = mn < a3 ? mn : a3;
        cm[l] = mx; cn[l] = mn;
    }
    const mv::MinMax mm = mv::q41_tree(cm, cn);
    const float d = (mm.mx - mm.mn) / 15.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    uint32_t w[4];
    for (int k = 0; k < 4; ++k) {
        float v[8];
        for (int e = 0; e < 8; ++e) v[e] = xb[8 * k + e];
        w[k] = mv::q41_pack8(v, mm.mn, id);
    }
    out.d[idx] = d;
    out.m[idx] = mm.mn;
    out.qs[idx] = make_uint4(w[0], w[1], w[2], w[3]);
}

// standalone activation quantizer (quantize_row_q4_0 AVX2, ggml.c:621-685)
// one thread per block; output split d / qs in the reference nibble layout
__global__ void k_quantize_q40(const float * __restrict__ x, int N, int K, ActQ out) {
    const int nb = K / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long) N * nb) return;
    const int t = (int) (idx / nb), b = (int) (idx % nb);
    const float * xb = x + (size_t) t * K + (size_t) b * 32;
    float v[32];
    float amax = 0.0f;
#pragma unroll
    for (int l = 0; l < 32; ++l) { v[l] = xb[l]; const float a = fabsf(v[l]); amax = a > amax ? a : amax; }
    const float d = amax / 7.0f;
    const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
    uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
    for (int l = 0; l < 32; ++l) {
        const uint32_t q = (uint32_t) ((int) __builtin_rintf(v[l] * id) + 8) & 15u;
        w[l / 8] |= q << (4 * (l % 8));
    }
    out.d[(size_t) t * out.nb + b] = d;
    out.qs[(size_t) t * out.nb + b] = make_uint4(w[0], w[1], w[2], w[3]);
}

// the reference's scalar quantizers (quantize_row_q4_0_reference / _q4_1_reference,
// ggml.c:509-545 / 799-840): roundf (half away from zero) and id = 1/d, unlike the AVX2
// quantizers above (RNE, id = 7/amax); one thread per block, output split like ActQ
__global__ void k_quantize_ref(const float * __restrict__ x, int N, int K, int qtype, ActQ out) {
    const int nb = K / 32;
    const long idx = (long) blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= (long) N * nb) return;
    const int t = (int) (idx / nb), b = (int) (idx % nb);
    const float * xb = x + (size_t) t * K + (size_t) b * 32;
    uint32_t w[4] = {0, 0, 0, 0};
    float d, mn = 0.0f;
    if (qtype == Q4_0) {
        float amax = 0.0f;
        for (int l = 0; l < 32; ++l) { const float a = fabsf(xb[l]); amax = amax > a ? amax : a; }   // MAX(amax, |v|)
        d = amax / 7.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        for (int l = 0; l < 32; ++l) {
            const uint32_t q = (uint32_t) (uint8_t) ((int8_t) roundf(xb[l] * id) + 8);
            w[l / 8] |= (q & 0xFFu) << (4 * (l % 8));
        }
    } else {
        float mx = -3.402823466e+38f;
        mn = 3.402823466e+38f;
        for (int l = 0; l < 32; ++l) {
            const float v = xb[l];
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
        d = (mx - mn) / 15.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        for (int l = 0; l < 32; ++l) {
            const uint32_t q = (uint32_t) (uint8_t) roundf((xb[l] - mn) * id);
            w[l / 8] |= (q & 0xFFu) << (4 * (l % 8));
        }
    }
    out.d[(size_t) t * out.nb + b] = d;
    if (qtype == Q4_1) out.m[(size_t) t * out.nb + b] = mn;
    out.qs[(size_t) t * out.nb + b] = make_uint4(w[0], w[1], w[2], w[3]);
}

}  // namespace

hipError_t launch_quantize_ref(const float * x, int N, int K, int qtype, ActQ out, hipStream_t s) {
    if (K % 32 || (qtype != Q4_0 && qtype != Q4_1)) return hipErrorInvalidValue;
    const long n = (long) N * (K / 32);
    hipLaunchKernelGGL(k_quantize_ref, dim3((unsigned) ((n + 127) / 128)), dim3(128), 0, s, x, N, K, qtype, out);
    return hipGetLastError();
}

hipError_t launch_embed(const void * emb, int emb_type, int n_embd, const int * tokens, int n, float * x,
                        hipStream_t s) {
    dim3 grid((n_embd + 255) / 256, n);
    LVK_LAUNCH(k_embed, grid, dim3(256), 0, s, (const uint8_t *) emb, emb_type, n_embd, tokens, x);
    return hipGetLastError();
}

hipError_t launch_repack(const void * src_rows, int qtype, int M, int K, uint4 * nib, void * scl, hipStream_t s,
                         int interleave4) {
    if (M % 8 || K % 256) return hipErrorInvalidValue;
    const long n = (long) M * ((K / 32 + 31) / 32) * 8;
    if (qtype == Q4_0) {
        hipLaunchKernelGGL(k_repack_q40, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s,
                           (const uint8_t *) src_rows, M, K, nib, (float4 *) scl, interleave4);
        return hipGetLastError();
    }
    if (qtype == Q4_1) {
        hipLaunchKernelGGL(k_repack_q41, dim3((unsigned) ((n + 255) / 256)), dim3(256), 0, s,
                           (const uint8_t *) src_rows, M, K, nib, (float4 *) scl, interleave4);
        return hipGetLastError();
    }
    return hipErrorNotSupported;
}

hipError_t launch_quantize_act(const float * x, int N, int K, int qtype, ActQ out, hipStream_t s) {
    if (K % 32) return hipErrorInvalidValue;
    const long n = (long) N * (K / 32);
    if (qtype == Q4_0) {
        hipLaunchKernelGGL(k_quantize_q40, dim3((unsigned) ((n + 127) / 128)), dim3(128), 0, s, x, N, K, out);
        return hipGetLastError();
    }
    if (qtype == Q4_1) {
        hipLaunchKernelGGL(k_quantize_q41, dim3((unsigned) ((n + 127) / 128)), dim3(128), 0, s, x, N, K, out);
        return hipGetLastError();
    }
    return hipErrorNotSupported;
}

}  // namespace lvk

namespace lvk {
namespace {
// ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076) + mul by g, one WG per row
__global__ __launch_bounds__(256) void k_rmsnorm_rows(const float * __restrict__ x, const float * __restrict__ g,
                                                      int K, float * __restrict__ y) {
    __shared__ double red[4];
    const int t = blockIdx.x;
    const float * xr = x + (size_t) t * K;
    double acc = 0.0;
    for (int i = threadIdx.x; i < K; i += 256) { const float sq = xr[i] * xr[i]; acc += (double) sq; }
    acc = warp_sum_d(acc);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
    __syncthreads();
    const double s = (red[0] + red[1]) + (red[2] + red[3]);
    const float mean = rms_mean_wave(s, xr, K);
    const float scale = 1.0f / sqrtf(mean + 1e-6f);
    for (int i = threadIdx.x; i < K; i += 256) { const float yn = xr[i] * scale; y[(size_t) t * K + i] = g[i] * yn; }
}
}  // namespace

hipError_t launch_rmsnorm_rows(const float * x, const float * g, int K, int n, float * y, hipStream_t s) {
    hipLaunchKernelGGL(k_rmsnorm_rows, dim3(n), dim3(256), 0, s, x, g, K, y);
    return hipGetLastError();
}
}  // namespace lvk

namespace lvk {
namespace {
// Greedy token choice on the device (llama.cpp:1382-1394): the first index whose
// logit is strictly greater than every earlier one.  Sequentially that is
// "index 0 if x[0] is NaN, else the first maximum over the non-NaN entries"
// (NaN never compares greater, and nothing beats a NaN start).  One workgroup:
// each thread scans a strided slice in increasing index order, then the
// (value, index) pairs reduce with ties going to the lower index.
struct ArgBest {
    float v;
    int i;   // INT_MAX: no non-NaN entry seen
};
__device__ inline ArgBest arg_pick(ArgBest a, ArgBest b) {
    if (b.i == INT_MAX) return a;
    if (a.i == INT_MAX) return b;
    return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}
__device__ inline void arg_take(ArgBest & b, float v, int i) {
    if (v == v && (b.i == INT_MAX || v > b.v)) b = {v, i};
}
// this thread's best over x[0..n): float4 slices t, t + 1024, ... with up to 8 of them in
// flight per trip (a 32000-entry vocabulary is one trip), entries in increasing index order
// per thread; unaligned or ragged inputs take the scalar stride
__device__ inline ArgBest arg_scan(const float * __restrict__ x, int n) {
    ArgBest b{-INFINITY, INT_MAX};
    const int t = threadIdx.x;
    if ((((uintptr_t) x) & 15) == 0 && (n & 3) == 0) {
        const float4 * x4 = (const float4 *) x;
        const int n4 = n >> 2;
        constexpr int U = 8;
        for (int base = 0; base < n4; base += U * 1024) {
            float4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int k = base + u * 1024 + t;
                v[u] = k < n4 ? x4[k] : make_float4(NAN, NAN, NAN, NAN);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = (base + u * 1024 + t) * 4;
                arg_take(b, v[u].x, i); arg_take(b, v[u].y, i + 1);
                arg_take(b, v[u].z, i + 2); arg_take(b, v[u].w, i + 3);
            }
        }
    } else {
        for (int i = t; i < n; i += 1024) arg_take(b, x[i], i);
    }
    return b;
}
__global__ __launch_bounds__(1024) void k_argmax_first(const float * __restrict__ x, int n, int * __restrict__ out,
                                                       int * __restrict__ out2) {
    __shared__ ArgBest red[16];
    ArgBest b = arg_scan(x, n);
    for (int off = 32; off > 0; off >>= 1) {
        ArgBest o;
        o.v = __shfl_xor(b.v, off, 64);
        o.i = __shfl_xor(b.i, off, 64);
        b = arg_pick(b, o);
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    __syncthreads();
    if (threadIdx.x == 0) {
        ArgBest r = red[0];
        for (int w = 1; w < 16; ++w) r = arg_pick(r, red[w]);
        const bool nan0 = n > 0 && !(x[0] == x[0]);
        const int tok = (nan0 || r.i == INT_MAX) ? 0 : r.i;
        out[0] = tok;
        if (out2) out2[0] = tok;     // e.g. host-mapped memory: visible after the stream completes
    }
}

// the last kernel of a chained decode step (lvk_decode_chain): the argmax of k_argmax_first
// goes to chain[CHAIN_HDR + i] (chain[0] counts the steps), the digest of the logits row
// (lvk_logits_digest) to digest[i] when chain[2] != 0, and the next token -- forced[i + 1] while
// i + 1 < chain[1] (a teacher-forced sequence), else the argmax -- into the step block (n_past + 1,
// the token, seq + 1) and, as its embedding row (k_embed's dequantization), into x: everything
// the next replay of the step graph reads
__device__ __forceinline__ unsigned long long digest_mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;                      // splitmix64 finalizer
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ __launch_bounds__(1024) void k_argmax_step(const float * __restrict__ logits, int n, StepParams * sp,
                                                      int * chain, const int * __restrict__ forced,
                                                      unsigned long long * __restrict__ digest,
                                                      const uint8_t * __restrict__ emb, int type, int E,
                                                      float * __restrict__ x) {
    __shared__ ArgBest red[16];
    __shared__ unsigned long long dred[16];
    __shared__ int s_tok;
    const int i = chain[0], n_forced = chain[1];
    const bool want_digest = chain[2] != 0;
    ArgBest b = arg_scan(logits, n);
    for (int off = 32; off > 0; off >>= 1) {
        ArgBest o;
        o.v = __shfl_xor(b.v, off, 64);
        o.i = __shfl_xor(b.i, off, 64);
        b = arg_pick(b, o);
    }
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = b;
    if (want_digest) {
        // sum over the row of mix(index << 32 | bits): wrap-around adds, any order gives the same
        unsigned long long dg = 0;
        for (int k = threadIdx.x; k < n; k += 1024)
            dg += digest_mix(((unsigned long long) k << 32) | __float_as_uint(logits[k]));
        for (int off = 32; off > 0; off >>= 1) dg += __shfl_xor(dg, off, 64);
        if ((threadIdx.x & 63) == 0) dred[threadIdx.x >> 6] = dg;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        ArgBest r = red[0];
        for (int w = 1; w < 16; ++w) r = arg_pick(r, red[w]);
        const bool nan0 = n > 0 && !(logits[0] == logits[0]);
        const int amax = (nan0 || r.i == INT_MAX) ? 0 : r.i;
        const int tok = i + 1 < n_forced ? forced[i + 1] : amax;
        s_tok = tok;
        chain[CHAIN_HDR + i] = amax;
        chain[0] = i + 1;
        if (want_digest) {
            unsigned long long dg = 0;
            for (int w = 0; w < 16; ++w) dg += dred[w];
            digest[i] = dg;
        }
        StepParams st = *sp;
        st.n_past += 1;
        st.pad0 = tok;
        st.seq += 1;
        *sp = st;
    }
    __syncthreads();
    const size_t tok = (size_t) s_tok;
    for (int e = threadIdx.x; e < E; e += 1024) {
        float v;
        if (type == Q4_0) {
            const uint8_t * blk = emb + tok * (size_t) (E / 32) * 20 + (size_t) (e / 32) * 20;
            const float d = *(const float *) blk;
            const uint8_t byte = blk[4 + (e % 32) / 2];
            const int qv = (e & 1) ? (byte >> 4) : (byte & 15);
            v = (float) (qv - 8) * d;
        } else if (type == Q4_1) {
            const uint8_t * blk = emb + tok * (size_t) (E / 32) * 24 + (size_t) (e / 32) * 24;
            const float d = *(const float *) blk, m = *(const float *) (blk + 4);
            const uint8_t byte = blk[8 + (e % 32) / 2];
            const int qv = (e & 1) ? (byte >> 4) : (byte & 15);
            const float a = (float) qv * d;
            v = a + m;
        } else if (type == 1) {
            v = f16_to_f32(((const uint16_t *) emb)[tok * E + e]);
        } else {
            v = ((const float *) emb)[tok * E + e];
        }
        x[e] = v;
    }
}
}  // namespace

hipError_t launch_argmax_step(const float * logits, int n, StepParams * sp, int * chain, const int * forced,
                              unsigned long long * digest, const void * emb, int emb_type, int n_embd, float * x,
                              hipStream_t s) {
    if (n <= 0 || n_embd <= 0 || n_embd % 32) return hipErrorInvalidValue;
    LVK_LAUNCH(k_argmax_step, dim3(1), dim3(1024), 0, s, logits, n, sp, chain, forced, digest, (const uint8_t *) emb,
               emb_type, n_embd, x);
    return hipGetLastError();
}

hipError_t launch_argmax(const float * x, int n, int * out, hipStream_t s, int * out2) {
    if (n <= 0) return hipErrorInvalidValue;
    LVK_LAUNCH(k_argmax_first, dim3(1), dim3(1024), 0, s, x, n, out, out2);
    return hipGetLastError();
}
}  // namespace lvk

LVK_RMS_ACCESSOR(lvk_probe_rms_misc)
