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
// ggml_vec_dot_f16 structure reproduced: element i of a 32-wide step feeds
// accumulator (r, l) = (i/8, i%8) of 4 AVX registers x 8 lanes via fmaf; the
// reduce is (s0+s1)+(s2+s3) per lane l, then t_l = S[l]+S[l+4] (l<4), then
// (t0+t1)+(t2+t3); leftovers are added in double.  Here the 4 registers r of a
// dot are the 4 lanes of a quad (16-byte loads), so loads are contiguous and
// the reduce is a fixed DPP pattern.
#include "lvk_device.h"
#include "lvk_kernels.h"

namespace lvk {

namespace {

__device__ __forceinline__ void unpack8h(const uint4 v, float f[8]) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[2 * k] = f16_to_f32((uint16_t) (w[k] & 0xFFFFu));
        f[2 * k + 1] = f16_to_f32((uint16_t) (w[k] >> 16));
    }
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

// ---------------------------------------------------------------------------
// scores[t][h][p] = (K[p,h,:] . f16(q[t,h,:])) * scale, or -inf when masked.
// grid (ceil(n_ctx/64), H, N), 256 threads: quad = one position.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_attn_scores(const uint16_t * __restrict__ q16, const uint16_t * __restrict__ kc,
                                                     float * __restrict__ scores, const StepParams * sp,
                                                     int E, int hd, int n_ctx, float scale) {
    const int n_past = sp->n_past, N = sp->n_tokens;
    const int n_kv = n_past + N;
    const int t = blockIdx.z, h = blockIdx.y;
    const int p = blockIdx.x * 64 + (threadIdx.x >> 2);
    const int r = threadIdx.x & 3;
    if (blockIdx.x * 64 >= n_kv || t >= N) return;
    const bool valid = p < n_kv;
    const bool masked = p > n_past + t;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (valid && !masked) {
        const uint4 * kp = (const uint4 *) (kc + (size_t) p * E + h * hd) + r;
        const uint4 * qp = (const uint4 *) (q16 + (size_t) t * E + h * hd) + r;
        for (int step = 0; step < hd / 32; ++step) {
            float kf[8], qf[8];
            unpack8h(kp[step * 4], kf);
            unpack8h(qp[step * 4], qf);
#pragma unroll
            for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(kf[l], qf[l], s[l]);
        }
    }
    const float kq = quad_f16dot_reduce(s);
    if (valid && r == 0) {
        const float v = kq * scale;                   // ggml_vec_scale_f32
        scores[((size_t) t * gridDim.y + h) * n_ctx + p] = masked ? -INFINITY : v;
    }
}

// ---------------------------------------------------------------------------
// softmax + P.V for 32 output dims of one head and one token, then quantize
// those 32 values (one weight block) for the Wo matvec.
// grid (hd/32, H, N), 128 threads: quad = one output dim.
// ---------------------------------------------------------------------------
template <int QT>
__global__ __launch_bounds__(128) void k_attn_pv(const float * __restrict__ scores, const uint16_t * __restrict__ vc,
                                                 const uint16_t * __restrict__ exp_tab, ActQ out,
                                                 const StepParams * sp, int E, int hd, int n_ctx,
                                                 float * __restrict__ out_f32, uint16_t * __restrict__ p16_out) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int n_past = sp->n_past, N = sp->n_tokens;
    const int n_kv = n_past + N;
    const int t = blockIdx.z, h = blockIdx.y, dc = blockIdx.x;
    if (t >= N) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    float * ev = (float *) smem;                                        // n_ctx floats
    uint16_t * p16 = (uint16_t *) (smem + (size_t) n_ctx * 4);          // n_ctx halves (+32 pad)
    float * red = (float *) (smem + (size_t) n_ctx * 6 + 64);           // small scratch
    double * redd = (double *) (red + 16);
    const float * srow = scores + ((size_t) t * gridDim.y + h) * n_ctx;

    // softmax (ggml.c:7099-7121)
    float mx = -INFINITY;
    for (int p = tid; p < n_kv; p += 128) { const float v = srow[p]; mx = v > mx ? v : mx; }
    mx = warp_max(mx);
    if (lane == 0) red[wave] = mx;
    __syncthreads();
    mx = red[0] > red[1] ? red[0] : red[1];
    double sum = 0.0;   // exact in any order: every term is an fp16 value in [0,1]
    for (int p = tid; p < n_kv; p += 128) {
        const float v = srow[p];
        float e = 0.0f;
        if (v != -INFINITY) {
            e = f16_to_f32(exp_tab[f32_to_f16(v - mx)]);
            sum += (double) e;
        }
        ev[p] = e;
    }
    sum = warp_sum_d(sum);
    if (lane == 0) redd[wave] = sum;
    __syncthreads();
    sum = redd[0] + redd[1];
    const float sc = (float) (1.0 / sum);
    const int n_pad = (n_kv + 31) & ~31;
    for (int p = tid; p < n_pad; p += 128) p16[p] = p < n_kv ? f32_to_f16(ev[p] * sc) : (uint16_t) 0;
    __syncthreads();
    if (p16_out && dc == 0)
        for (int p = tid; p < n_kv; p += 128) p16_out[((size_t) t * gridDim.y + h) * n_ctx + p] = p16[p];

    // KQV: ggml_vec_dot_f16(n_kv, V row, P)
    const int d = dc * 32 + (tid >> 2);
    const int r = tid & 3;
    const uint16_t * vrow = vc + (size_t) (h * hd + d) * n_ctx;
    const int np = n_kv & ~31;
    const int lim = n_past + t;       // last unmasked position of this column
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < np && i <= lim; i += 32) {      // fully masked steps add exact zeros: skipped
        float vf[8], pf[8];
        unpack8h(*((const uint4 *) (vrow + i) + r), vf);
        unpack8h(*((const uint4 *) (p16 + i) + r), pf);
#pragma unroll
        for (int l = 0; l < 8; ++l) s[l] = __builtin_fmaf(vf[l], pf[l], s[l]);
    }
    const float res = quad_f16dot_reduce(s);
    float o = res;
    if (r == 0) {
        double sumf = (double) res;
        for (int i = np; i < n_kv && i <= lim; ++i) {
            const float pr = f16_to_f32(vrow[i]) * f16_to_f32(p16[i]);
            sumf += (double) pr;
        }
        o = (float) sumf;
    }
    // gather the 32 outputs in LDS, quantize as one block (quantize_row_q4_x)
    __syncthreads();
    float * ob = ev;
    if (r == 0) ob[tid >> 2] = o;
    if (r == 0 && out_f32) out_f32[(size_t) t * E + h * hd + d] = o;
    __syncthreads();
    if (wave == 0 && lane < 32) {
        const float v = ob[lane];
        const int blk = (h * hd + dc * 32) / 32;
        uint32_t * scratch = (uint32_t *) (ev + 64);
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
            if ((lane & 7) == 0) scratch[lane >> 3] = part;
            __builtin_amdgcn_wave_barrier();
            if (lane == 0) {
                out.d[(size_t) t * out.nb + blk] = dd;
                out.qs[(size_t) t * out.nb + blk] = make_uint4(scratch[0], scratch[1], scratch[2], scratch[3]);
            }
        }
    }
}

}  // namespace

hipError_t launch_attention(const AttnLaunch & A, hipStream_t s) {
    const int hd = A.n_embd / A.n_head;
    if (hd % 32 || A.n_ctx % 32) return hipErrorInvalidValue;
    if (A.out_qtype != Q4_0) return hipErrorNotSupported;
    const float scale = 1.0f / sqrtf((float) A.n_embd / (float) A.n_head);   // llama.cpp:1028
    dim3 g1((A.n_ctx + 63) / 64, A.n_head, A.n_tokens);
    hipLaunchKernelGGL(k_attn_scores, g1, dim3(256), 0, s, A.q16, A.kc, A.scores, A.sp, A.n_embd, hd, A.n_ctx, scale);
    dim3 g2(hd / 32, A.n_head, A.n_tokens);
    const size_t lds = (size_t) A.n_ctx * 6 + 64 + 256;
    hipLaunchKernelGGL(k_attn_pv<Q4_0>, g2, dim3(128), lds, s, A.scores, A.vc, A.exp_tab, A.out, A.sp,
                       A.n_embd, hd, A.n_ctx, A.out_f32, A.p16_out);
    return hipGetLastError();
}

}  // namespace lvk
