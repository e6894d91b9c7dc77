// attention_decode.hip -- single-token (decode) attention over the f16 KV
// cache, bit-faithful to the reference graph (llama.cpp:1010-1061) like
// attention.hip, split so that the KV bytes of a layer are read by 4x as many
// CUs in ONE launch.
//
// A decode step reads 2 * n_kv * 256 B of K and V per head; one workgroup per
// head pulls ~100 KB through one CU at ~17 B/cycle.  Here 4 workgroups share a
// head, grid (H, 4):
//   1. workgroup (h, s) DMAs the V rows of its 32-dim slice (one weight block
//      of the merged heads) into LDS, and scores the positions of 64-position
//      chunks s, s+4, ... (a lane quad per position): KQ = ggml_vec_dot_f16
//      (ggml.c:1781-1815, Q in f16) * 1/sqrt(head_dim) (llama.cpp:1026);
//   2. the scores are exchanged through global memory as 8-byte {tag, value}
//      granules, each one agent-scope 8-B store (the data is the flag:
//      cdna_hip_programming.md Guideline 16, R2); every thread polls the
//      granules it needs until their tag equals this layer's epoch (layer + 1;
//      the granule array is zeroed once per token), bounded;
//   3. softmax (max, fp16 exp, exact double sum, ggml.c:7099-7121), P in f16,
//      P.V with the AVX accumulator layout (a quad per dim) and the double
//      tail past n_kv & ~31 (ggml.c:1806-1808); the slice is quantized to the
//      Wo weight format (quantize_row_q4_0 / _q4_1, ggml.c:621-685 / 847-920).
// All 4*H workgroups are co-resident (grid <= CUs), which the exchange needs;
// the spin is bounded so a violated assumption cannot hang the GPU.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {

constexpr int HD = 128;

__device__ __forceinline__ void unpack8(const uint4 v, float f[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = f16_to_f32((uint16_t) (w[k] & 0xFFFFu));
        f[2 * k + 1] = f16_to_f32((uint16_t) (w[k] >> 16));
    }
}

// the quad's 4 x 8 accumulators in the AVX2 F32Cx8_REDUCE order (as attention.hip)
__device__ __forceinline__ float quad_reduce(const float s[8]) {
    float S[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float v0 = quad_bcast<0>(s[l]), v1 = quad_bcast<1>(s[l]);
        const float v2 = quad_bcast<2>(s[l]), v3 = quad_bcast<3>(s[l]);
        const float a = v0 + v1, b = v2 + v3;
        S[l] = a + b;
    }
    const float t0 = S[0] + S[4], t1 = S[1] + S[5], t2 = S[2] + S[6], t3 = S[3] + S[7];
    return (t0 + t1) + (t2 + t3);
}

typedef unsigned long long u64g __attribute__((address_space(1)));

#ifdef LVK_PROBE_TIMING   // dev probe builds only: per-wave s_memtime phase stamps
__device__ unsigned long long g_dtrace[32 * 4 * 4 * 8];
#define LVK_DT(ev)                                                                                       \
    do {                                                                                                 \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                      \
        if ((threadIdx.x & 63) == 0) g_dtrace[((blockIdx.x * 4 + blockIdx.y) * 4 + (threadIdx.x >> 6)) * 8 + (ev)] = t_; \
    } while (0)
#else
#define LVK_DT(ev) do { } while (0)
#endif

template <int QT>
__global__ __launch_bounds__(256) void k_attn_d(const uint16_t * __restrict__ q16, const uint16_t * __restrict__ kc,
                                                const uint16_t * __restrict__ vc, unsigned long long * gran,
                                                const uint16_t * __restrict__ exp_tab, const StepParams * sp, int E,
                                                int n_ctx, float scale, unsigned epoch, ActQ out,
                                                float * __restrict__ out_f32, int exp_mode) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int h = blockIdx.x, sl = blockIdx.y, d0 = h * HD + sl * 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = tid & 3;
    uint16_t * vl = (uint16_t *) smem;                           // [32 dims][n_ctx]
    float * sc = (float *) (smem + (size_t) 32 * n_ctx * 2);     // [n_ctx]
    uint16_t * pl = (uint16_t *) (sc + n_ctx);                   // [n_ctx]
    float * red = (float *) (pl + n_ctx);                        // 8 floats
    double * redd = (double *) (red + 8);                        // 4 doubles
    u64g * g = (u64g *) (gran + (size_t) h * n_ctx);
    LVK_DT(0);

    // 1a. loads that do not depend on n_past go out before the step block is read (its
    // load is a full memory round trip): Q, the K rows of this workgroup's first two
    // 64-position chunks and the first 512 positions of its 32 V rows (addresses inside
    // the caches; positions past n_kv are never used)
    const uint4 * qp = (const uint4 *) (q16 + h * HD) + r;
    uint4 qv[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) qv[st] = qp[st * 4];
    uint4 kv[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const int p = min(sl * 64 + c * 256 + (tid >> 2), n_ctx - 1);
        const uint4 * kp = (const uint4 *) (kc + (size_t) p * E + h * HD) + r;
#pragma unroll
        for (int st = 0; st < 4; ++st) kv[c][st] = kp[st * 4];
    }
    auto v_dma = [&](int p0, int lim) {             // positions [p0, p0 + 512) of the 32 rows, below lim
        for (int row = wave; row < 32; row += 4)
            if (p0 + lane * 8 < lim)
                __builtin_amdgcn_global_load_lds((const void *) (vc + (size_t) (d0 + row) * n_ctx + p0 + lane * 8),
                                                 (__attribute__((address_space(3))) void *) (vl + (size_t) row * n_ctx + p0),
                                                 16, 0, 0);
    };
    LVK_DT(6);
    v_dma(0, min(n_ctx, 512));
    LVK_DT(7);
    const int n_kv = sp->n_past + 1;
    const int n_pad = (n_kv + 31) & ~31;
    const int np = n_kv & ~31;
    for (int p0 = 512; p0 < n_pad; p0 += 512) v_dma(p0, n_pad);
    LVK_DT(1);

    // 1b. scores of chunks sl, sl+4, ... (one position per lane quad)
    {
        float qf[4][8];
#pragma unroll
        for (int st = 0; st < 4; ++st) unpack8(qv[st], qf[st]);
        auto score = [&](const uint4 (&k4)[4], int p) {
            float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                float kf[8];
                unpack8(k4[st], kf);
#pragma unroll
                for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(kf[l], qf[st][l], s[l]);
            }
            const float kq = quad_reduce(s);
            if (r == 0 && p < n_kv) {
                const float v = kq * scale;                      // ggml_vec_scale_f32 (llama.cpp:1026)
                __hip_atomic_store(g + p, ((unsigned long long) epoch << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        };
#pragma unroll
        for (int c = 0; c < 2; ++c)
            if (sl * 64 + c * 256 < n_kv) score(kv[c], sl * 64 + c * 256 + (tid >> 2));
        for (int c0 = sl * 64 + 512; c0 < n_kv; c0 += 256) {
            const int p = c0 + (tid >> 2);
            const uint4 * kp = (const uint4 *) (kc + (size_t) min(p, n_kv - 1) * E + h * HD) + r;
            uint4 k4[4];
#pragma unroll
            for (int st = 0; st < 4; ++st) k4[st] = kp[st * 4];
            score(k4, p);
        }
    }
    LVK_DT(2);
    // 2. every score of the head: poll each granule until it carries this layer's epoch
    float mx = -INFINITY;
    for (int p = tid; p < n_kv; p += 256) {
        unsigned long long x;
        for (int spins = 0;; ++spins) {
            x = __hip_atomic_load(g + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((unsigned) (x >> 32) == epoch || spins > (1 << 22)) break;      // bounded: never hang
            __builtin_amdgcn_s_sleep(1);
        }
        const float v = __uint_as_float((unsigned) x);
        sc[p] = v;
        mx = v > mx ? v : mx;
    }
    LVK_DT(3);
    mx = wave_max_f(mx);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    {
        const float a = red[0] > red[1] ? red[0] : red[1], b = red[2] > red[3] ? red[2] : red[3];
        mx = a > b ? a : b;
    }
    // softmax (ggml.c:7099-7121): no position is masked in a decode step
    double sum = 0.0;    // exact in any order: every term is an fp16 value in [0,1]
    for (int p = tid; p < n_kv; p += 256) {
        const float e = f16_to_f32(exp_f16(f32_to_f16(sc[p] - mx), exp_tab, exp_mode));
        sum += (double) e;
        sc[p] = e;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) redd[wave] = sum;
    __syncthreads();
    sum = (redd[0] + redd[1]) + (redd[2] + redd[3]);
    const float scl = (float) (1.0 / sum);
    for (int p = tid; p < n_pad; p += 256) pl[p] = p < n_kv ? f32_to_f16(sc[p] * scl) : (uint16_t) 0;
    LVK_DT(4);
    __syncthreads();          // vmcnt(0) + barrier: the V DMA has landed too
    LVK_DT(5);

    // P.V: quad q = dim d0 + q (waves 0-1)
    float o = 0.0f;
    if (tid < 128) {
        const int q = tid >> 2;
        const uint16_t * vr = vl + (size_t) q * n_ctx;
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int ns = np / 32;
        int st = 0;
        for (; st + 2 <= ns; st += 2) {          // two steps' LDS reads in flight
            const uint4 v0 = *((const uint4 *) (vr + st * 32) + r), p0 = *((const uint4 *) (pl + st * 32) + r);
            const uint4 v1 = *((const uint4 *) (vr + st * 32 + 32) + r), p1 = *((const uint4 *) (pl + st * 32 + 32) + r);
            float vf[8], pf[8];
            unpack8(v0, vf);
            unpack8(p0, pf);
#pragma unroll
            for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(vf[l], pf[l], s[l]);
            unpack8(v1, vf);
            unpack8(p1, pf);
#pragma unroll
            for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(vf[l], pf[l], s[l]);
        }
        if (st < ns) {
            float vf[8], pf[8];
            unpack8(*((const uint4 *) (vr + st * 32) + r), vf);
            unpack8(*((const uint4 *) (pl + st * 32) + r), pf);
#pragma unroll
            for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(vf[l], pf[l], s[l]);
        }
        const float res = quad_reduce(s);
        o = res;
        if (np < n_kv) {      // leftovers in double, in position order (ggml.c:1806-1808)
            double sumf = (double) res;
            for (int p = np; p < n_kv; ++p) {
                const float prod = f16_to_f32(vr[p]) * f16_to_f32(pl[p]);
                sumf += (double) prod;
            }
            o = (float) sumf;
        }
    }
    __syncthreads();
    float * ob = sc;          // reuse: 32 outputs
    if (tid < 128 && r == 0) ob[tid >> 2] = o;
    __syncthreads();
    if (tid < 32) {
        const float v = ob[tid];
        if (out_f32) out_f32[d0 + tid] = v;
        const int blk = d0 / 32;
        if constexpr (QT == Q4_0) {
            float amax = fabsf(v);
            for (int o2 = 16; o2 > 0; o2 >>= 1) { const float w = __shfl_xor(amax, o2); amax = w > amax ? w : amax; }
            const float dd = amax / 7.0f;
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
            const uint32_t qq = (uint32_t) ((int) __builtin_rintf(v * id) + 8) & 15u;
            uint32_t part = qq << (4 * (tid & 7));
            part |= __shfl_xor(part, 1);
            part |= __shfl_xor(part, 2);
            part |= __shfl_xor(part, 4);
            const uint32_t w0 = __shfl(part, 0), w1 = __shfl(part, 8), w2 = __shfl(part, 16), w3 = __shfl(part, 24);
            if (tid == 0) {
                out.d[blk] = dd;
                out.qs[blk] = make_uint4(w0, w1, w2, w3);
            }
        }
    }
    if constexpr (QT == Q4_1) {
        // quantize_row_q4_1 (ggml.c:847-920) of the 32 outputs staged in ob
        if (tid < 4) {
            const int blk = d0 / 32;
            float dd, mm;
            uint32_t qw;
            mv::q41_block_lds(ob, tid, dd, mm, qw);
            ((uint32_t *) (out.qs + blk))[tid] = qw;
            if (tid == 0) {
                out.d[blk] = dd;
                out.m[blk] = mm;
            }
        }
    }
}

}  // namespace

#ifdef LVK_PROBE_TIMING
void * lvk_probe_dtrace() { void * p = nullptr; (void) hipGetSymbolAddress(&p, HIP_SYMBOL(g_dtrace)); return p; }
#endif

bool attention_decode_supported(int n_embd, int n_head, int n_ctx) {
    return n_embd / n_head == HD && n_ctx % 64 == 0 && n_ctx <= 2048 && n_head * 4 <= 1024;
}

size_t attention_decode_scratch_bytes(int n_head, int n_ctx) { return (size_t) n_head * n_ctx * 8; }

hipError_t launch_attention_decode(const AttnLaunch & A, void * gran, unsigned epoch, hipStream_t s) {
    if (!attention_decode_supported(A.n_embd, A.n_head, A.n_ctx) || A.n_tokens != 1 || epoch == 0)
        return hipErrorNotSupported;
    if (A.out_qtype != Q4_0 && A.out_qtype != Q4_1) return hipErrorNotSupported;
    const float scale = 1.0f / sqrtf((float) A.n_embd / (float) A.n_head);   // llama.cpp:1028
    const size_t lds = (size_t) 32 * A.n_ctx * 2 + (size_t) A.n_ctx * 6 + 64;
    if (A.out_qtype == Q4_1)
        LVK_LAUNCH(k_attn_d<Q4_1>, dim3(A.n_head, HD / 32), dim3(256), lds, s, A.q16, A.kc, A.vc,
                   (unsigned long long *) gran, A.exp_tab, A.sp, A.n_embd, A.n_ctx, scale, epoch, A.out, A.out_f32,
                   A.exp_computed);
    else
        LVK_LAUNCH(k_attn_d<Q4_0>, dim3(A.n_head, HD / 32), dim3(256), lds, s, A.q16, A.kc, A.vc,
                   (unsigned long long *) gran, A.exp_tab, A.sp, A.n_embd, A.n_ctx, scale, epoch, A.out, A.out_f32,
                   A.exp_computed);
    return hipGetLastError();
}

}  // namespace lvk
