// attention.hip -- one layer of causal self-attention over the f16 KV cache,
// bit-faithful to the reference graph (llama.cpp:1010-1061):
//   KQ   = mul_mat(K_view f16, Q)  -> Q rounded to f16 (ggml.c:6420-6433),
//          each score one ggml_vec_dot_f16 over head_dim (ggml.c:1781-1815)
//   KQ  *= 1/sqrtf(n_embd/n_head)   (separate multiply, llama.cpp:1026-1029)
//   mask  p > n_past + t -> -inf    (ggml.c:7028-7031)
//   softmax: max, fp16 exp table, double sum, * (float)(1.0/sum) (ggml.c:7099-7121)
//   KQV  = mul_mat(V_view f16, P)   -> P rounded to f16; every column's dot
//          runs over n_kv = n_past + N (SIMD part n_kv & ~31, double tail)
//   then the merged heads are quantized to the Wo weight format here, so the
//   Wo matvec reads 20 B/block instead of 128 B of f32.
//
// With the f32 KV cache (f16_kv = false, llama.cpp:1614) the same kernel runs F32 = true:
// KQ = mul_mat(K_view f32, Q f32) and KQV = mul_mat(V_view f32, P f32) are
// ggml_compute_forward_mul_mat_f32 (ggml.c:6134-6297), i.e. ggml_vec_dot_f32
// (ggml.c:1713-1748): the same 4 x 8 accumulators and reduce, no f16 rounding of Q or P,
// leftovers summed in float.
//
// ggml_vec_dot_f16 structure reproduced: element i of a 32-wide step feeds
// accumulator (r, l) = (i/8, i%8) of 4 AVX registers x 8 lanes via fmaf; the
// reduce is (s0+s1)+(s2+s3) per lane l, then t_l = S[l]+S[l+4] (l<4), then
// (t0+t1)+(t2+t3); leftovers are added in double.  Here the 4 registers r of a
// dot are the 4 lanes of a quad (16-byte loads), so loads are contiguous and
// the reduce is a fixed DPP pattern.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {

#ifdef LVK_PROBE_TIMING   // dev probe builds only: per-wave s_memtime trace of the attention kernel
__device__ unsigned long long g_atrace[64 * 4 * 16];
#define LVK_AT(ev)                                                                                    \
    do {                                                                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                   \
        if ((threadIdx.x & 63) == 0 && blockIdx.y == 0)                                               \
            g_atrace[((blockIdx.x * 2 + blockIdx.z) & 63) * 64 + (threadIdx.x >> 6) * 16 + (ev)] = t_; \
    } while (0)
#else
#define LVK_AT(ev) do { } while (0)
#endif

__device__ __forceinline__ void unpack8h(const uint4 v, float f[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = f16_to_f32((uint16_t) (w[k] & 0xFFFFu));
        f[2 * k + 1] = f16_to_f32((uint16_t) (w[k] >> 16));
    }
}

// one 1 KiB LDS-DMA piece per wave: lane l moves 16 bytes from src to
// lds + 16*l (global_load_lds_dwordx4, no VGPR destination)
__device__ __forceinline__ void dma16(const void * src, uint8_t * lds) {
    __builtin_amdgcn_global_load_lds((const void *) src, (__attribute__((address_space(3))) void *) lds, 16, 0, 0);
}

// reduce the quad's 4x8 accumulators in the AVX2 F32Cx8_REDUCE order
__device__ __forceinline__ float quad_f16dot_reduce(const float s[8]) {
    float S[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float v0 = quad_bcast<0>(s[l]), v1 = quad_bcast<1>(s[l]);
        const float v2 = quad_bcast<2>(s[l]), v3 = quad_bcast<3>(s[l]);
        const float a = v0 + v1, b = v2 + v3;     // x[0]+=x[1]; x[2]+=x[3]
        S[l] = a + b;                              // x[0]+=x[2]
    }
    const float t0 = S[0] + S[4], t1 = S[1] + S[5], t2 = S[2] + S[6], t3 = S[3] + S[7];
    return (t0 + t1) + (t2 + t3);                  // hadd, hadd
}

// table_exp_f16[h] (ggml.c:2915-2927: fp16(expf(fp16->f32(h)))) for the
// arguments softmax produces (h <= 0, not NaN), computed in double and rounded
// to f32 then f16 -- the two roundings the table went through.  Used only when
// exp_check() has shown it equal to the uploaded host table on every such h.

// bad[m-1]: arguments where mode m (1 double, 2 device expf) differs from the table
__global__ void k_exp_check(const uint16_t * __restrict__ tab, int * __restrict__ bad) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h < 65536u && ((h & 0x8000u) || h == 0) && (h & 0x7fffu) <= 0x7c00u) {
        if (exp_f16((uint16_t) h, tab, 1) != tab[h]) atomicAdd(bad, 1);
        if (exp_f16((uint16_t) h, tab, 2) != tab[h]) atomicAdd(bad + 1, 1);
    }
}

// ---------------------------------------------------------------------------
// Fused attention for one (token t, head h, half of the head dims):
//   phase 1  scores of every position p < n_kv into LDS (quad = one position,
//            4 passes of 64 positions in flight per unrolled step)
//   phase 2  softmax in LDS, P rounded to f16
//   phase 3  P.V for HD/2 output dims (quad = one dim), V loads unrolled x8
//   phase 4  quantize the HD/2 outputs (HD/64 weight blocks) for Wo
// grid (H, N, 2), 256 threads.
// ---------------------------------------------------------------------------
// 8 elements of a step from one 16-byte (f16) or two 16-byte (f32) loads
template <bool F32> struct Vec8 { uint4 w[F32 ? 2 : 1]; };
template <bool F32>
__device__ __forceinline__ Vec8<F32> ld8(const uint16_t * base, size_t elem) {
    Vec8<F32> v;
    if constexpr (F32) {
        const uint4 * p = (const uint4 *) ((const float *) base + elem);
        v.w[0] = p[0]; v.w[1] = p[1];
    } else {
        v.w[0] = *(const uint4 *) (base + elem);
    }
    return v;
}
template <bool F32>
__device__ __forceinline__ void unpack8(const Vec8<F32> & v, float f[8]) {
    if constexpr (F32) {
        const uint32_t w[8] = {v.w[0].x, v.w[0].y, v.w[0].z, v.w[0].w, v.w[1].x, v.w[1].y, v.w[1].z, v.w[1].w};
#pragma unroll
        for (int k = 0; k < 8; ++k) f[k] = __uint_as_float(w[k]);
    } else {
        unpack8h(v.w[0], f);
    }
}

template <int HD, int QT, bool F32>
__global__ __launch_bounds__(256) void k_attn(const uint16_t * __restrict__ q16, const uint16_t * __restrict__ kc,
                                              const uint16_t * __restrict__ vc, const uint16_t * __restrict__ exp_tab,
                                              ActQ out, const StepParams * sp, int E, int n_ctx, float scale,
                                              float * __restrict__ scores_dbg, float * __restrict__ out_f32,
                                              uint16_t * __restrict__ p16_out, int exp_computed) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    constexpr int NSTEP = HD / 32;
    const int n_past = sp->n_past, N = sp->n_tokens;
    const int n_kv = n_past + N;
    const int h = blockIdx.x, t = blockIdx.y, half = blockIdx.z;
    if (t >= N) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = tid & 3;
    float * sc = (float *) smem;                                   // n_ctx scores / exp values
    uint16_t * p16 = (uint16_t *) (smem + (size_t) n_ctx * 4);     // n_ctx f16 probabilities
    float * red = (float *) (smem + (size_t) n_ctx * 6);           // 8 floats
    double * redd = (double *) (smem + (size_t) n_ctx * 6 + 32);   // 4 doubles
    const int lim = n_past + t;                                    // last unmasked position

    // ---- all global loads first: Q, the first 512 positions of K (8 passes of
    // 64 positions, a lane quad per position) and of V (16 steps of 32
    // positions for this thread's output dim).  Nothing here depends on the
    // softmax, so one memory round trip covers the whole kernel at n_kv <= 512.
    constexpr int KP = F32 ? 4 : 8, VS = F32 ? 8 : 16, PB = KP * 64;
    constexpr int VSB = F32 ? 8192 : 4096;            // LDS bytes per V step of 64 dims x 32 positions
    Vec8<F32> qv[NSTEP];
#pragma unroll
    for (int st = 0; st < NSTEP; ++st) qv[st] = ld8<F32>(q16, (size_t) t * E + h * HD + st * 32 + r * 8);
    const int npos = min(n_kv, lim + 1);     // masked positions get -inf without a dot
    Vec8<F32> kv[KP][NSTEP];
    auto load_k = [&](int pb) {
#pragma unroll
        for (int ps = 0; ps < KP; ++ps) {
            if (pb + ps * 64 < npos) {          // wave-uniform: no duplicate requests past n_kv
                const int pp = min(pb + ps * 64 + (tid >> 2), npos - 1);
#pragma unroll
                for (int st = 0; st < NSTEP; ++st) kv[ps][st] = ld8<F32>(kc, (size_t) pp * E + h * HD + st * 32 + r * 8);
            }
        }
    };
    const int d = half * (HD / 2) + (tid >> 2);
    const size_t vrow = (size_t) (h * HD + d) * n_ctx;   // element offset of this thread's V row
    const int np = n_kv & ~31;
    const int nvs = (n_kv + 31) / 32;                  // V steps including a partial one
    // V steps 0..VS-1 go to LDS by DMA: step s of the workgroup's 64 dims is VSB bytes at
    // vlds + s*VSB, thread tid's first 16 bytes at + tid*16 (f32: the second at + 4096 + tid*16)
    uint8_t * vlds = smem + (size_t) n_ctx * 6 + 64;
    LVK_AT(0);
    load_k(0);
    {
        uint8_t * vl = vlds + (tid & ~63) * 16;       // wave-uniform base
        const int nd = min(nvs, VS);
        for (int st = 0; st < nd; ++st) {
            if constexpr (F32) {
                const float * vf = (const float *) vc + vrow + (size_t) st * 32 + r * 8;
                dma16(vf, vl + st * VSB);
                dma16(vf + 4, vl + st * VSB + 4096);
            } else {
                dma16(vc + vrow + (size_t) st * 32 + r * 8, vl + st * VSB);
            }
        }
    }
    LVK_AT(1);

    // ---- phase 1: KQ (ggml_vec_dot_f16 over HD, Q in f16) ----
    for (int pb = 0; pb < npos; pb += PB) {
        if (pb > 0) load_k(pb);
#pragma unroll
        for (int ps = 0; ps < KP; ++ps) {
            if (pb + ps * 64 < npos) {
                float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int st = 0; st < NSTEP; ++st) {
                    float kf[8], qf[8];
                    unpack8<F32>(kv[ps][st], kf);
                    unpack8<F32>(qv[st], qf);
#pragma unroll
                    for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(kf[l], qf[l], s[l]);
                }
                const float kq = quad_f16dot_reduce(s);
                const int pp = pb + ps * 64 + (tid >> 2);
                if (r == 0 && pp < npos) sc[pp] = kq * scale;      // ggml_vec_scale_f32 (llama.cpp:1026)
            }
        }
    }
    LVK_AT(2);
    for (int p = npos + tid; p < n_kv; p += 256) sc[p] = -INFINITY;   // ggml.c:7028-7031
    __syncthreads();
    if (scores_dbg && half == 0)
        for (int p = tid; p < n_kv; p += 256) scores_dbg[((size_t) t * gridDim.x + h) * n_ctx + p] = sc[p];

    // ---- phase 2: softmax (ggml.c:7099-7121) ----
    float mx = -INFINITY;
    for (int p = tid; p < n_kv; p += 256) { const float v = sc[p]; mx = v > mx ? v : mx; }
    mx = wave_max_f(mx);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    {
        const float a = red[0] > red[1] ? red[0] : red[1], b = red[2] > red[3] ? red[2] : red[3];
        mx = a > b ? a : b;
    }
    double sum = 0.0;   // exact in any order: every term is an fp16 value in [0,1]
    for (int p = tid; p < n_kv; p += 256) {
        const float v = sc[p];
        float e = 0.0f;
        if (v != -INFINITY) {
            e = f16_to_f32(exp_f16(f32_to_f16(v - mx), exp_tab, exp_computed));
            sum += (double) e;
        }
        sc[p] = e;
    }
    sum = wave_sum_d(sum);     // any order: the sum is exact
    if (lane == 0) redd[wave] = sum;
    __syncthreads();
    sum = (redd[0] + redd[1]) + (redd[2] + redd[3]);
    const float scl = (float) (1.0 / sum);
    const int n_pad = (n_kv + 31) & ~31;
    if constexpr (F32) {
        for (int p = tid; p < n_pad; p += 256) sc[p] = p < n_kv ? sc[p] * scl : 0.0f;   // P stays f32
    } else {
        for (int p = tid; p < n_pad; p += 256) p16[p] = p < n_kv ? f32_to_f16(sc[p] * scl) : (uint16_t) 0;
    }
    __syncthreads();
    if (!F32 && p16_out && half == 0)
        for (int p = tid; p < n_kv; p += 256) p16_out[((size_t) t * gridDim.x + h) * n_ctx + p] = p16[p];

    LVK_AT(3);
    // ---- phase 3: KQV = ggml_vec_dot_f16(n_kv, V row, P) ----
    __syncthreads();     // vmcnt(0) + barrier: every wave's V DMA has landed
    const int nsteps = min(np, lim + 1 + 31) / 32;     // steps holding at least one unmasked position
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    auto pv_step = [&](const Vec8<F32> & v8, int st) {
        float vf[8], pf[8];
        unpack8<F32>(v8, vf);
        if constexpr (F32) {
#pragma unroll
            for (int l = 0; l < 8; ++l) pf[l] = sc[st * 32 + r * 8 + l];
        } else {
            unpack8h(*((const uint4 *) (p16 + st * 32) + r), pf);
        }
#pragma unroll
        for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(vf[l], pf[l], s[l]);
    };
    const int nl = min(nsteps, VS);
    for (int st = 0; st < nl; ++st) {
        Vec8<F32> v8;
        v8.w[0] = *((const uint4 *) (vlds + (size_t) st * VSB) + tid);
        if constexpr (F32) v8.w[1] = *((const uint4 *) (vlds + (size_t) st * VSB + 4096) + tid);
        pv_step(v8, st);
    }
    for (int st = VS; st < nsteps; ++st) pv_step(ld8<F32>(vc, vrow + (size_t) st * 32 + r * 8), st);
    const float res = quad_f16dot_reduce(s);
    float o = res;
    if (F32 && np < n_kv && np <= lim) {
        // leftovers in float, in position order (ggml.c:1736-1739: sumf += x[i]*y[i])
        if (r == 0) {
            const int ne = min(n_kv, lim + 1);
            const float * vrf = (const float *) vc + vrow;
            float sumf = res;
            for (int i = np; i < ne; ++i) { const float pr = vrf[i] * sc[i]; sumf = sumf + pr; }
            o = sumf;
        }
    } else if (!F32 && np < n_kv && np <= lim) {
        // leftovers in double, in position order (ggml.c:1806-1808), from registers
        const int ts = np / 32;
        uint4 vt[4], pt[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            pt[k] = *((const uint4 *) (p16 + np) + k);
            if (ts < VS) vt[k] = *((const uint4 *) (vlds + (size_t) ts * VSB) + (tid & ~3) + k);
        }
        if (ts >= VS)
#pragma unroll
            for (int k = 0; k < 4; ++k) vt[k] = *((const uint4 *) (vc + vrow + np) + k);
        if (r == 0) {
            const int nt_ = min(n_kv, lim + 1) - np;
            double sumf = (double) res;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float vf[8], pf[8];
                unpack8h(vt[k], vf);
                unpack8h(pt[k], pf);
#pragma unroll
                for (int l = 0; l < 8; ++l)
                    if (8 * k + l < nt_) { const float pr = vf[l] * pf[l]; sumf += (double) pr; }
            }
            o = (float) sumf;
        }
    }
    if (r == 0 && out_f32) out_f32[(size_t) t * E + h * HD + d] = o;

    LVK_AT(4);
    // ---- phase 4: quantize HD/2 outputs = HD/64 weight blocks ----
    __syncthreads();
    float * ob = sc;
    if (r == 0) ob[tid >> 2] = o;
    __syncthreads();
    if (tid < HD / 2) {
        const float v = ob[tid];
        const int blk = (h * HD + half * (HD / 2)) / 32 + (tid >> 5);
        uint32_t * scratch = (uint32_t *) (sc + 128) + (tid >> 5) * 4;
        if constexpr (QT == Q4_0) {
            float amax = fabsf(v);
            for (int o2 = 16; o2 > 0; o2 >>= 1) { const float w = __shfl_xor(amax, o2); amax = w > amax ? w : amax; }
            const float dd = amax / 7.0f;
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
            const uint32_t qq = (uint32_t) ((int) __builtin_rintf(v * id) + 8) & 15u;
            uint32_t part = qq << (4 * (lane & 7));
            part |= __shfl_xor(part, 1);
            part |= __shfl_xor(part, 2);
            part |= __shfl_xor(part, 4);
            if ((lane & 7) == 0) scratch[(lane & 31) >> 3] = part;
            __builtin_amdgcn_wave_barrier();
            if ((lane & 31) == 0) {
                out.d[(size_t) t * out.nb + blk] = dd;
                out.qs[(size_t) t * out.nb + blk] = make_uint4(scratch[0], scratch[1], scratch[2], scratch[3]);
            }
        }
    }
    if constexpr (QT == Q4_1) {
        // quantize_row_q4_1 (ggml.c:847-920) of the HD/64 blocks staged in ob
        if (tid < HD / 16) {
            const int bb = tid >> 2, k = tid & 3;
            const int blk = (h * HD + half * (HD / 2)) / 32 + bb;
            float dd, mm;
            uint32_t qw;
            mv::q41_block_lds(ob + bb * 32, k, dd, mm, qw);
            ((uint32_t *) (out.qs + (size_t) t * out.nb + blk))[k] = qw;
            if (k == 0) {
                out.d[(size_t) t * out.nb + blk] = dd;
                out.m[(size_t) t * out.nb + blk] = mm;
            }
        }
    }
    LVK_AT(5);
}

}  // namespace

#ifdef LVK_PROBE_TIMING
void * lvk_probe_atrace() { void * p = nullptr; (void) hipGetSymbolAddress(&p, HIP_SYMBOL(g_atrace)); return p; }
#endif

hipError_t exp_check(const uint16_t * exp_tab, int * bad_d, hipStream_t s) {
    hipError_t e = hipMemsetAsync(bad_d, 0, 2 * sizeof(int), s);
    if (e != hipSuccess) return e;
    k_exp_check<<<256, 256, 0, s>>>(exp_tab, bad_d);
    return hipGetLastError();
}

hipError_t launch_attention(const AttnLaunch & A, hipStream_t s) {
    const int hd = A.n_embd / A.n_head;
    if (hd != 128 || A.n_ctx % 32 || A.n_ctx < 128) return hipErrorInvalidValue;
    if (A.kv32 && A.p16_out) return hipErrorInvalidValue;
    if (A.out_qtype != Q4_0 && A.out_qtype != Q4_1) return hipErrorNotSupported;
    const float scale = 1.0f / sqrtf((float) A.n_embd / (float) A.n_head);   // llama.cpp:1028
    dim3 grid(A.n_head, A.n_tokens, 2);
    // scores, P16, reductions, then V steps 0..15 by DMA (4 KiB each)
    const size_t lds = (size_t) A.n_ctx * 6 + 64 + 16 * 4096;
#define LVK_ATTN_GO(QT_, F32_)                                                                                  \
    LVK_LAUNCH((k_attn<128, QT_, F32_>), grid, dim3(256), lds, s, A.q16, A.kc, A.vc, A.exp_tab, A.out, A.sp,  \
               A.n_embd, A.n_ctx, scale, A.scores, A.out_f32, A.p16_out, A.exp_computed)
    if (A.out_qtype == Q4_1) {
        if (A.kv32) LVK_ATTN_GO(Q4_1, true); else LVK_ATTN_GO(Q4_1, false);
    } else {
        if (A.kv32) LVK_ATTN_GO(Q4_0, true); else LVK_ATTN_GO(Q4_0, false);
    }
#undef LVK_ATTN_GO
    return hipGetLastError();
}

}  // namespace lvk
