// graph_ops.hip -- device kernels behind include/ggml.h's graph operators
// (csrc/runtime/ggml_graph.cpp): every node of a ggml graph runs here, on strided 4-D
// views of the graph's buffers mirrored in HBM, with the arithmetic of the reference's
// AVX2 build (each kernel cites the ggml.c function it follows).
// These are operator-level kernels (one node per launch, generic strides): the fused
// single-token and prompt paths of llama_eval are the matvec / MFMA / attention kernels.
#include "lvk_device.h"
#include "lvk_kernels.h"

namespace lvk {

namespace {

__device__ __forceinline__ void unflatten(int64_t i, const int64_t ne[4], int64_t & i0, int64_t & i1, int64_t & i2,
                                          int64_t & i3) {
    i0 = i % ne[0]; i /= ne[0];
    i1 = i % ne[1]; i /= ne[1];
    i2 = i % ne[2];
    i3 = i / ne[2];
}

__device__ __forceinline__ char * at(const GView & v, int64_t i0, int64_t i1, int64_t i2, int64_t i3) {
    return v.p + i0 * v.nb[0] + i1 * v.nb[1] + i2 * v.nb[2] + i3 * v.nb[3];
}

__device__ __forceinline__ float load_f(const GView & v, int64_t i0, int64_t i1, int64_t i2, int64_t i3) {
    const char * p = at(v, i0, i1, i2, i3);
    return v.type == GT_F16 ? f16_to_f32(*(const uint16_t *) p) : *(const float *) p;
}

__device__ __forceinline__ void store_f(const GView & v, int64_t i0, int64_t i1, int64_t i2, int64_t i3, float x) {
    char * p = at(v, i0, i1, i2, i3);
    if (v.type == GT_F16) *(uint16_t *) p = f32_to_f16(x);
    else *(float *) p = x;
}

__device__ __forceinline__ int64_t nel(const GView & v) { return v.ne[0] * v.ne[1] * v.ne[2] * v.ne[3]; }

// dup / cpy (ggml.c ggml_compute_forward_dup_*): the k-th element of src in logical
// (row-major, i0 fastest) order goes to the k-th element of dst; f32 <-> f16 RNE
__global__ void k_g_cpy(GView s, GView d) {
    const int64_t n = nel(d);
    for (int64_t k = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; k < n; k += (int64_t) gridDim.x * blockDim.x) {
        int64_t a0, a1, a2, a3, b0, b1, b2, b3;
        unflatten(k, s.ne, a0, a1, a2, a3);
        unflatten(k, d.ne, b0, b1, b2, b3);
        if (s.type == d.type && s.type == GT_F16)
            *(uint16_t *) at(d, b0, b1, b2, b3) = *(const uint16_t *) at(s, a0, a1, a2, a3);
        else if (s.type == d.type && s.type == GT_I32)
            *(int32_t *) at(d, b0, b1, b2, b3) = *(const int32_t *) at(s, a0, a1, a2, a3);
        else
            store_f(d, b0, b1, b2, b3, load_f(s, a0, a1, a2, a3));
    }
}

// add / sub / mul / div of same-shape f32 tensors (ggml.c:5039-5194), repeat (5504)
__global__ void k_g_binary(GView a, GView b, GView d, int op) {
    const int64_t n = nel(d);
    for (int64_t k = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; k < n; k += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unflatten(k, d.ne, i0, i1, i2, i3);
        float r;
        if (op == GOP_REPEAT) {
            // a is smaller than d: index it modulo its own shape only
            r = *(const float *) at(a, i0 % a.ne[0], i1 % a.ne[1], i2 % a.ne[2], i3 % a.ne[3]);
        } else {
            const float x = *(const float *) at(a, i0, i1, i2, i3);
            const float y = *(const float *) at(b, i0, i1, i2, i3);
            switch (op) {
                case GOP_ADD: r = x + y; break;
                case GOP_SUB: r = x - y; break;
                case GOP_MUL: r = x * y; break;
                default: r = x / y; break;
            }
        }
        *(float *) at(d, i0, i1, i2, i3) = r;
    }
}

// scale (ggml.c:6757-6790: v * x per element), silu through the fp16 table
// (ggml.c:2495-2503, 5875-5914), diag_mask_inf (7001-7035): element-wise, strided
__global__ void k_g_unary(GView s, GView d, int op, float v, int n_past, const uint16_t * tab) {
    const int64_t n = nel(d);
    for (int64_t k = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; k < n; k += (int64_t) gridDim.x * blockDim.x) {
        int64_t i0, i1, i2, i3;
        unflatten(k, d.ne, i0, i1, i2, i3);
        const float x = *(const float *) at(s, i0, i1, i2, i3);
        float r = x;
        if (op == GOP_SCALE) r = x * v;
        else if (op == GOP_SILU) r = f16_to_f32(tab[f32_to_f16(x)]);
        else if (op == GOP_DIAG_MASK) r = (i0 > n_past + i1) ? -INFINITY : x;
        *(float *) at(d, i0, i1, i2, i3) = r;
    }
}

// rms_norm (ggml.c:6024-6080): per row, float squares summed in double IN INDEX ORDER by
// one lane (bit-exact by construction), mean = (float)(sum / ne0), scale = 1/sqrtf(mean +
// 1e-6f), y = x * scale.  One 64-lane wave per row; the other lanes scale.
__global__ void k_g_rms_norm(GView s, GView d) {
    const int64_t row = blockIdx.x;
    const int64_t i1 = row % s.ne[1], i2 = (row / s.ne[1]) % s.ne[2], i3 = row / (s.ne[1] * s.ne[2]);
    __shared__ float scale_s;
    if (threadIdx.x == 0) {
        double sum = 0.0;
        for (int64_t i0 = 0; i0 < s.ne[0]; ++i0) {
            const float x = *(const float *) at(s, i0, i1, i2, i3);
            const float sq = x * x;
            sum += (double) sq;
        }
        const float mean = (float) (sum / (double) s.ne[0]);
        scale_s = 1.0f / sqrtf(mean + 1e-6f);
    }
    __syncthreads();
    const float sc = scale_s;
    for (int64_t i0 = threadIdx.x; i0 < s.ne[0]; i0 += blockDim.x)
        *(float *) at(d, i0, i1, i2, i3) = *(const float *) at(s, i0, i1, i2, i3) * sc;
}

// soft_max (ggml.c:7062-7130), in place per row: max, e = exp_f16(fp16(p - max)) for
// p != -inf (-inf -> 0), sum in double (exact in any order: fp16 terms in [0,1]),
// p *= (float)(1.0 / sum)
__global__ void k_g_soft_max(GView d, const uint16_t * exp_tab, int exp_mode) {
    const int64_t row = blockIdx.x;
    const int64_t i1 = row % d.ne[1], i2 = (row / d.ne[1]) % d.ne[2], i3 = row / (d.ne[1] * d.ne[2]);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ float redf[4];
    __shared__ double redd[4];
    float mx = -INFINITY;
    for (int64_t i0 = tid; i0 < d.ne[0]; i0 += blockDim.x) {
        const float v = *(const float *) at(d, i0, i1, i2, i3);
        mx = v > mx ? v : mx;              // ggml_vec_max_f32: max = MAX(max, x)
    }
    mx = wave_max_f(mx);
    if (lane == 0) redf[wave] = mx;
    __syncthreads();
    {
        const float a = redf[0] > redf[1] ? redf[0] : redf[1], b = redf[2] > redf[3] ? redf[2] : redf[3];
        mx = a > b ? a : b;
    }
    double sum = 0.0;
    for (int64_t i0 = tid; i0 < d.ne[0]; i0 += blockDim.x) {
        float * p = (float *) at(d, i0, i1, i2, i3);
        const float v = *p;
        float e = 0.0f;
        if (v != -INFINITY) e = f16_to_f32(exp_f16(f32_to_f16(v - mx), exp_tab, exp_mode));
        sum += (double) e;
        *p = e;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) redd[wave] = sum;
    __syncthreads();
    sum = (redd[0] + redd[1]) + (redd[2] + redd[3]);
    const float scl = (float) (1.0 / sum);
    for (int64_t i0 = tid; i0 < d.ne[0]; i0 += blockDim.x) {
        float * p = (float *) at(d, i0, i1, i2, i3);
        *p = *p * scl;
    }
}

// rope f32 (ggml.c:7156-7227) with the host-built glibc {cos, sin} of (p, i0): pairs
// (i0, i0+1) of every row i1 of slice i2 (position slot i2 - i2_0 of the table)
__global__ void k_g_rope(GView s, GView d, const float2 * cs, int n_dims, int i2_0) {
    const int np = n_dims / 2;
    const int64_t n = (int64_t) np * s.ne[1] * (s.ne[2] - i2_0) * s.ne[3];
    for (int64_t k = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; k < n; k += (int64_t) gridDim.x * blockDim.x) {
        int64_t t = k;
        const int pr = (int) (t % np); t /= np;
        const int64_t i1 = t % s.ne[1]; t /= s.ne[1];
        const int64_t i2 = i2_0 + t % (s.ne[2] - i2_0);
        const int64_t i3 = t / (s.ne[2] - i2_0);
        const float2 c = cs[(i2 - i2_0) * np + pr];
        const float x0 = *(const float *) at(s, 2 * pr, i1, i2, i3);
        const float x1 = *(const float *) at(s, 2 * pr + 1, i1, i2, i3);
        const float a = x0 * c.x, b = x1 * c.y, e = x0 * c.y, f = x1 * c.x;
        *(float *) at(d, 2 * pr, i1, i2, i3) = a - b;
        *(float *) at(d, 2 * pr + 1, i1, i2, i3) = e + f;
    }
}

// get_rows (ggml.c:6868-6895): dst row r = dequantize(src0 row idx[r]); Q4_0 (q - 8) * d,
// Q4_1 q * d then + m (ggml.c:968-1000, 1086-1115), f16 exact, f32 copy
__global__ void k_g_get_rows(GView s, const int32_t * idx, GView d) {
    const int64_t r = blockIdx.y;
    const int64_t row = idx[r];
    if (row < 0 || row >= s.ne[1]) return;     // (the host rejects such ids of a leaf index tensor)
    const char * src = s.p + row * s.nb[1];
    for (int64_t i0 = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; i0 < d.ne[0]; i0 += (int64_t) gridDim.x * blockDim.x) {
        float v;
        if (s.type == GT_Q4_0) {
            const char * b = src + (i0 / 32) * 20;
            const float dd = *(const float *) b;
            const uint8_t q = ((const uint8_t *) (b + 4))[(i0 % 32) / 2];
            const int qi = (int) ((i0 & 1) ? (q >> 4) : (q & 15)) - 8;
            v = (float) qi * dd;
        } else if (s.type == GT_Q4_1) {
            const char * b = src + (i0 / 32) * 24;
            const float dd = *(const float *) b, mm = *(const float *) (b + 4);
            const uint8_t q = ((const uint8_t *) (b + 8))[(i0 % 32) / 2];
            const float t = (float) ((i0 & 1) ? (q >> 4) : (q & 15)) * dd;
            v = t + mm;
        } else if (s.type == GT_F16) {
            v = f16_to_f32(((const uint16_t *) src)[i0]);
        } else {
            v = ((const float *) src)[i0];
        }
        *(float *) at(d, i0, r, 0, 0) = v;
    }
}

// mul_mat f16 x f32 (ggml.c:6299-6487): src1 already converted to contiguous f16 rows
// (the INIT phase, RNE), then dst[ic][i01] = ggml_vec_dot_f16 (ggml.c:1781-1815): 4 x 8
// fp32 FMA accumulators over n & ~31, the F32Cx8 reduce, the tail in double.  Also
// f32 x f32 (ggml_vec_dot_f32, ggml.c:1713-1748: same accumulators and reduce, the tail
// summed in float) when s0.type == GT_F32 (y then f32 contiguous rows).
__global__ void k_g_mm_dot(GView s0, const void * y, int64_t ne11, GView d) {
    const int64_t n = s0.ne[0];
    const int64_t total = s0.ne[1] * ne11 * s0.ne[2] * s0.ne[3];
    for (int64_t k = blockIdx.x * (int64_t) blockDim.x + threadIdx.x; k < total; k += (int64_t) gridDim.x * blockDim.x) {
        int64_t t = k;
        const int64_t i01 = t % s0.ne[1]; t /= s0.ne[1];
        const int64_t ic = t % ne11; t /= ne11;
        const int64_t i02 = t % s0.ne[2];
        const int64_t i03 = t / s0.ne[2];
        const char * xr = at(s0, 0, i01, i02, i03);
        const int64_t col = (i03 * s0.ne[2] + i02) * ne11 + ic;
        const bool h = s0.type == GT_F16;
        float sum[4][8];
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int l = 0; l < 8; ++l) sum[r][l] = 0.0f;
        const int64_t np = n & ~(int64_t) 31;
        auto xv = [&](int64_t i) { return h ? f16_to_f32(((const uint16_t *) xr)[i]) : ((const float *) xr)[i]; };
        auto yv = [&](int64_t i) {
            return h ? f16_to_f32(((const uint16_t *) y)[col * n + i]) : ((const float *) y)[col * n + i];
        };
        for (int64_t i = 0; i < np; i += 32)
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int l = 0; l < 8; ++l) sum[r][l] = __builtin_fmaf(xv(i + 8 * r + l), yv(i + 8 * r + l), sum[r][l]);
        float S[8];
#pragma unroll
        for (int l = 0; l < 8; ++l) {
            const float a = sum[0][l] + sum[1][l], b = sum[2][l] + sum[3][l];
            S[l] = a + b;
        }
        const float t0 = S[0] + S[4], t1 = S[1] + S[5], t2 = S[2] + S[6], t3 = S[3] + S[7];
        const float res = (t0 + t1) + (t2 + t3);
        float out;
        if (h) {
            double sumf = (double) res;
            for (int64_t i = np; i < n; ++i) {
                const float p = xv(i) * yv(i);
                sumf += (double) p;
            }
            out = (float) sumf;
        } else {
            // the reference is built as ISO C (-std=c11: no contraction): product, then sum
            float sumf = res;
            for (int64_t i = np; i < n; ++i) {
                const float p = xv(i) * yv(i);
                sumf = sumf + p;
            }
            out = sumf;
        }
        *(float *) at(d, i01, ic, i02, i03) = out;
    }
}

unsigned grid_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (unsigned) (b < 1 ? 1 : (b > 65535 ? 65535 : b));
}

}  // namespace

hipError_t launch_g_cpy(const GView & s, const GView & d, hipStream_t st) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    hipLaunchKernelGGL(k_g_cpy, dim3(grid_for(n)), dim3(256), 0, st, s, d);
    return hipGetLastError();
}

hipError_t launch_g_binary(const GView & a, const GView & b, const GView & d, int op, hipStream_t st) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    hipLaunchKernelGGL(k_g_binary, dim3(grid_for(n)), dim3(256), 0, st, a, b, d, op);
    return hipGetLastError();
}

hipError_t launch_g_unary(const GView & s, const GView & d, int op, float v, int n_past, const uint16_t * tab,
                          hipStream_t st) {
    const int64_t n = d.ne[0] * d.ne[1] * d.ne[2] * d.ne[3];
    hipLaunchKernelGGL(k_g_unary, dim3(grid_for(n)), dim3(256), 0, st, s, d, op, v, n_past, tab);
    return hipGetLastError();
}

hipError_t launch_g_rms_norm(const GView & s, const GView & d, hipStream_t st) {
    const int64_t rows = s.ne[1] * s.ne[2] * s.ne[3];
    if (rows > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_g_rms_norm, dim3((unsigned) rows), dim3(256), 0, st, s, d);
    return hipGetLastError();
}

hipError_t launch_g_soft_max(const GView & d, const uint16_t * exp_tab, int exp_mode, hipStream_t st) {
    const int64_t rows = d.ne[1] * d.ne[2] * d.ne[3];
    if (rows > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_g_soft_max, dim3((unsigned) rows), dim3(256), 0, st, d, exp_tab, exp_mode);
    return hipGetLastError();
}

hipError_t launch_g_rope(const GView & s, const GView & d, const float2 * cs, int n_dims, int i2_0, hipStream_t st) {
    const int64_t n = (int64_t) (n_dims / 2) * s.ne[1] * (s.ne[2] - i2_0) * s.ne[3];
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_g_rope, dim3(grid_for(n)), dim3(256), 0, st, s, d, cs, n_dims, i2_0);
    return hipGetLastError();
}

hipError_t launch_g_get_rows(const GView & s, const int32_t * idx, int64_t n_rows, const GView & d, hipStream_t st) {
    if (n_rows <= 0) return hipSuccess;
    if (n_rows > 65535) return hipErrorInvalidValue;
    const unsigned gx = (unsigned) ((d.ne[0] + 255) / 256);
    hipLaunchKernelGGL(k_g_get_rows, dim3(gx, (unsigned) n_rows), dim3(256), 0, st, s, idx, d);
    return hipGetLastError();
}

hipError_t launch_g_mm_dot(const GView & s0, const void * y, int64_t ne11, const GView & d, hipStream_t st) {
    const int64_t n = s0.ne[1] * ne11 * s0.ne[2] * s0.ne[3];
    hipLaunchKernelGGL(k_g_mm_dot, dim3(grid_for(n)), dim3(256), 0, st, s0, y, ne11, d);
    return hipGetLastError();
}

}  // namespace lvk
