// attention_prompt.hip -- causal self-attention of a prompt batch (N > 1
// tokens) over the f16 KV cache, bit-faithful to the reference graph
// (llama.cpp:1010-1061) exactly like attention.hip, but organised for many
// query tokens: the decode kernel's one-workgroup-per-(token, head) layout
// re-streams K and V for every token (22 ms of a 512-token 7B prompt).
//
//   k_attn_p_scores  grid (H, ceil(N/16)/2): a pair of mirrored 16-token
//                    blocks per workgroup (equal causal work everywhere); Q
//                    in LDS; K streamed in 64-position tiles (a lane per
//                    position, its K row in registers, Q broadcast from LDS);
//                    scores KQ*scale (ggml_vec_dot_f16 order, ggml.c:1781-1815)
//                    in LDS; -inf past n_past+t; softmax with the fp16 exp
//                    and the exact double sum (ggml.c:7099-7121); P rounded
//                    to f16 -> global scratch P[h][t][n_ctx].
//   k_attn_p_pv      grid (H, ceil(N/32), HD/32), longest blocks first: V rows of one 32-dim slice
//                    and P of 32 tokens in LDS; each lane quad owns 4 dims x 4
//                    tokens (16 dots, 8 AVX accumulators each); leftovers past
//                    n_kv & ~31 in double (ggml.c:1806-1808); the slice is one
//                    Q4_0 block of the merged heads: quantize_row_q4_0
//                    (ggml.c:621-685) fused, written as the Wo input (ActQ and,
//                    for the MFMA Wo, the masked fragment image).
#include "lvk_device.h"
#include "mm41_common.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

#include <cstdlib>

// knockout build (dev only, `make apko KO=n`, timing attribution -- wrong results): &1 the
// score dots, &2 the softmax exp, &4 the whole softmax but the P store, &8 the P.V dots
#ifndef LVK_ATTN_P_KO
#define LVK_ATTN_P_KO 0
#endif

namespace lvk {

namespace {

constexpr int HD = 128;

// the quad's 4 x 8 accumulators in the AVX2 F32Cx8_REDUCE order (lane j = AVX register j):
// two DPP butterflies give (v0 + v1) + (v2 + v3) in every lane of the quad (fp
// addition is commutative, so lane 1's v1 + v0 and lane 2's (v2 + v3) + (v0 + v1) are the same
// bits) -- 4 instructions per accumulator instead of 7
__device__ __forceinline__ float quad_reduce_bf(const float s[8]) {
    float S[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) {
        const float x = s[l];
        const float y = x + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), 0xB1, 0xF, 0xF, false));
        S[l] = y + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, y), 0x4E, 0xF, 0xF, false));
    }
    const float t0 = S[0] + S[4], t1 = S[1] + S[5], t2 = S[2] + S[6], t3 = S[3] + S[7];
    return (t0 + t1) + (t2 + t3);
}

// ---------------------------------------------------------------------------
// scores + softmax.  A workgroup (4 waves) owns one head and two T-token blocks, the block
// nblk-1-y and its mirror y, one after the other: the causal 64-position tiles of the pair sum
// to about the same count in every workgroup, so each SIMD keeps 2 busy waves to the end (a
// VALU-bound wave alone issues at about half the rate, profiles/r04_valu_cycles.log).  Wave w
// takes tokens w, w+4, ..; a lane owns position p = pb + lane of each tile, its K row packed in
// 64 VGPRs with the next tile's row in flight, and runs all 32 AVX accumulators of
// ggml_vec_dot_f16 itself with v_fma_mix (f16 operands converted exactly, one rounding), then
// the F32Cx8 reduce in registers.  EM: the softmax exp mode (lvk_device.h exp_softmax).
// ---------------------------------------------------------------------------
template <int T, int EM>
__global__ __launch_bounds__(256) void k_attn_p_scores(const uint16_t * __restrict__ q16, const uint16_t * __restrict__ kc,
                                                       const uint16_t * __restrict__ exp_tab, const StepParams * sp,
                                                       int E, int n_ctx, float scale, uint16_t * __restrict__ P,
                                                       int exp_mode) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int n_past = sp->n_past, N = sp->n_tokens;
    const int n_kv = n_past + N;
    const int nblk = (N + T - 1) / T;
    const int h = blockIdx.x;
    // wave made visibly uniform: the token loops branch on scalars, not exec masks
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    uint4 * qs = (uint4 *) smem;                             // [T][16] uint4: Q rows (f16)
    float * sc = (float *) (smem + T * 256);                  // [T][n_ctx] scores, then exp values
    const int n_pad = (n_kv + 31) & ~31;

    for (int ph = 0; ph < 2; ++ph) {
        const int b = ph == 0 ? nblk - 1 - (int) blockIdx.y : (int) blockIdx.y;
        if (ph == 1) {
            if (b >= nblk - 1 - b) break;                   // odd block count: the middle block alone
            __syncthreads();                                 // the first block's rows are read out
        }
        const int t0 = b * T;
        const int nt = min(T, N - t0);
        const int lim_hi = n_past + t0 + nt - 1;             // last unmasked position of the block
        for (int i = tid; i < T * 16; i += 256) {
            const int t = i >> 4;
            qs[i] = t < nt ? *((const uint4 *) (q16 + (size_t) (t0 + t) * E + h * HD) + (i & 15)) : make_uint4(0, 0, 0, 0);
        }
        __syncthreads();

        auto load = [&](uint4 (&kr)[16], int pb) {
            const uint4 * kp = (const uint4 *) (kc + (size_t) min(pb + lane, lim_hi) * E + h * HD);
#pragma unroll
            for (int i = 0; i < 16; ++i) kr[i] = kp[i];
        };
        auto tile = [&](const uint4 (&kr)[16], int pb) {
            const int p = pb + lane;
            const bool live = p <= lim_hi;
            // wave < nt: at least one token, so the first pass consumes the tile's loads and the
            // compiler knows them done when the registers are reloaded
            int t = wave;
            do {
                // accumulator (j, l) of ggml_vec_dot_f16 (ggml.c:1781-1815): elements 32 st + 8 j + l,
                // st = 0..3 in order; uint4 4 st + j holds the 8 of (st, j), word w elements 2w, 2w + 1
                float acc[4][8];
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int l = 0; l < 8; ++l) acc[j][l] = 0.0f;
#pragma unroll
                for (int st = 0; st < ((LVK_ATTN_P_KO & 1) ? 0 : 4); ++st) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const uint4 q = qs[t * 16 + 4 * st + j];          // wave-uniform: an LDS broadcast
                        const uint4 k = kr[4 * st + j];
                        const uint32_t qw[4] = {q.x, q.y, q.z, q.w}, kw[4] = {k.x, k.y, k.z, k.w};
#pragma unroll
                        for (int w = 0; w < 4; ++w) {
                            acc[j][2 * w] = fma_mix_hh<0, 0>(kw[w], qw[w], acc[j][2 * w]);
                            acc[j][2 * w + 1] = fma_mix_hh<1, 1>(kw[w], qw[w], acc[j][2 * w + 1]);
                        }
                    }
                }
                // F32Cx8 reduce: accumulator j plays the AVX register j (quad_reduce order)
                float S[8];
#pragma unroll
                for (int l = 0; l < 8; ++l) {
                    const float a = acc[0][l] + acc[1][l], c = acc[2][l] + acc[3][l];
                    S[l] = a + c;
                }
                const float t0v = S[0] + S[4], t1v = S[1] + S[5], t2v = S[2] + S[6], t3v = S[3] + S[7];
                float kq = (t0v + t1v) + (t2v + t3v);
                if (LVK_ATTN_P_KO & 1) kq = __builtin_bit_cast(float, (kr[0].x ^ (uint32_t) t) & 0xBFFFFFFFu) * 1e-30f;
                if (live) sc[(size_t) t * n_ctx + p] = p <= n_past + t0 + t ? kq * scale : -INFINITY;
                t += 4;
            } while (t < nt);
        };
        if (wave < nt) {
            // tiles in pairs, the next tile's K loads always in flight (clamped to lim_hi): one
            // loop exit, and a skipped second tile drains its loads itself, so the compiler's
            // wait before each tile's first use counts only that tile's loads
            uint4 ka[16], kb[16];
            load(ka, 0);
            for (int pb = 0; pb <= lim_hi; pb += 128) {
                load(kb, pb + 64);
                tile(ka, pb);
                load(ka, pb + 128);
                if (pb + 64 <= lim_hi) tile(kb, pb + 64);
                else __builtin_amdgcn_s_waitcnt(0x0F70);     // vmcnt(0)
            }
        }
        __syncthreads();

        // ---- softmax per token row (ggml.c:7099-7121); wave w owns rows w, w+4, ... ----
        for (int t = wave; t < nt; t += 4) {
            float * row = sc + (size_t) t * n_ctx;
            const int lim = n_past + t0 + t;
            // positions lim+1 .. n_kv-1 are -inf (ggml.c:7028-7031): max over the live ones
            float mx = -INFINITY;
            if (!(LVK_ATTN_P_KO & 4))
                for (int p = lane; p <= lim; p += 64) { const float v = row[p]; mx = v > mx ? v : mx; }
            mx = wave_max_f(mx);
            double sum = 0.0;      // exact in any order: every term is an fp16 value in [0,1]
            if (!(LVK_ATTN_P_KO & 4))
                for (int p = lane; p <= lim; p += 64) {
                    const float e = (LVK_ATTN_P_KO & 2) ? row[p] - mx
                                                        : f16_to_f32(exp_softmax<EM>(f32_to_f16(row[p] - mx), exp_tab, exp_mode));
                    sum += (double) e;
                    row[p] = e;
                }
            sum = wave_sum_d(sum);
            const float scl = (float) (1.0 / sum);
            // P rounded to f16 (the mul_mat's src1 conversion), two positions per lane
            uint32_t * prow = (uint32_t *) (P + ((size_t) h * N + t0 + t) * n_ctx);
            for (int p = 2 * lane; p < n_pad; p += 128) {
                const uint32_t lo = p <= lim ? f32_to_f16(row[p] * scl) : 0u;
                const uint32_t hi = p + 1 <= lim ? f32_to_f16(row[p + 1] * scl) : 0u;
                prow[p >> 1] = lo | hi << 16;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// P.V for one 32-dim slice (one Q4_0 block of the merged heads) and 32 tokens.
// Quad (qd, qt): dims 4qd..4qd+3, tokens 4qt..4qt+3 of the slice / block.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_attn_p_pv(const uint16_t * __restrict__ vc, const uint16_t * __restrict__ P,
                                                   const StepParams * sp, int E, int n_ctx, ActQ out, uint2 * xm,
                                                   float * xda, float * __restrict__ out_f32, int q41,
                                                   uint4 * xs41) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int n_past = sp->n_past, N = sp->n_tokens;
    const int n_kv = n_past + N;
    // the longest blocks (most causal steps) first, so the tail of the launch is short ones
    const int h = blockIdx.x, t0 = (gridDim.y - 1 - blockIdx.y) * 32, ds = blockIdx.z;
    const int nt = min(32, N - t0);
    const int tid = threadIdx.x, r = tid & 3, quad = tid >> 2;
    const int qd = quad & 7, qt = quad >> 3;
    const int n_pad = (n_kv + 31) & ~31;
    const int np = n_kv & ~31;
    const int lim_hi = n_past + t0 + nt - 1;
    const int nsteps = min(np, lim_hi + 1 + 31) / 32;        // steps holding at least one unmasked position
    const int nfill = min(n_pad, (lim_hi + 32) & ~31);        // positions any dot of the block reads
    uint16_t * vl = (uint16_t *) smem;                         // [32 dims][n_pad]
    uint16_t * pl = vl + (size_t) 32 * n_pad;                  // [32 tokens][n_pad]
    const int d0 = h * HD + ds * 32;

    // stage V rows d0..d0+31 and the P rows of the block (16-byte pieces), 8 + 8 loads in
    // flight per thread before the LDS writes
    const int per = nfill / 8, tot = 32 * per;
    for (int i0 = 0; i0 < tot; i0 += 256 * 8) {
        uint4 va[8], pa[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + 256 * u + tid;
            const int row = i / per, c = i - row * per;
            va[u] = pa[u] = make_uint4(0, 0, 0, 0);
            if (i < tot) {
                va[u] = ((const uint4 *) (vc + (size_t) (d0 + row) * n_ctx))[c];
                if (row < nt) pa[u] = ((const uint4 *) (P + ((size_t) h * N + t0 + row) * n_ctx))[c];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + 256 * u + tid;
            const int row = i / per, c = i - row * per;
            if (i < tot) {
                ((uint4 *) (vl + (size_t) row * n_pad))[c] = va[u];
                ((uint4 *) (pl + (size_t) row * n_pad))[c] = pa[u];
            }
        }
    }
    __syncthreads();

    float s[4][4][8];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int l = 0; l < 8; ++l) s[a][b][l] = 0.0f;
    for (int st = 0; st < ((LVK_ATTN_P_KO & 8) ? 0 : nsteps); ++st) {
        // the f16 operands straight into v_fma_mix (converted exactly, one rounding = fmaf of the
        // converted values): no separate conversions
        uint32_t vw[4][4], pw[4][4];
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const uint4 v = *((const uint4 *) (vl + (size_t) (4 * qd + a) * n_pad + st * 32) + r);
            vw[a][0] = v.x; vw[a][1] = v.y; vw[a][2] = v.z; vw[a][3] = v.w;
        }
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint4 v = *((const uint4 *) (pl + (size_t) (4 * qt + b) * n_pad + st * 32) + r);
            pw[b][0] = v.x; pw[b][1] = v.y; pw[b][2] = v.z; pw[b][3] = v.w;
        }
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    s[a][b][2 * w] = fma_mix_hh<0, 0>(vw[a][w], pw[b][w], s[a][b][2 * w]);
                    s[a][b][2 * w + 1] = fma_mix_hh<1, 1>(vw[a][w], pw[b][w], s[a][b][2 * w + 1]);
                }
    }
    // reduce + double leftovers (ggml.c:1806-1808), in position order
    float o[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const float res = quad_reduce_bf(s[a][b]);
            const int t = 4 * qt + b;
            const int lim = n_past + t0 + t;
            float v = res;
            if (np < n_kv && np <= lim) {
                double sumf = (double) res;
                const uint16_t * vr = vl + (size_t) (4 * qd + a) * n_pad;
                const uint16_t * pr = pl + (size_t) t * n_pad;
                for (int p = np; p < n_kv; ++p) {
                    const float prod = f16_to_f32(vr[p]) * f16_to_f32(pr[p]);
                    sumf += (double) prod;
                }
                v = (float) sumf;
            }
            o[a][b] = v;
        }
    // ---- merged heads: this slice is one Q4_0 block per token; quantize (ggml.c:621-685) ----
    __syncthreads();
    float * ob = (float *) smem;                               // [32 tokens][33]
    if (r == 0) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b) ob[(4 * qt + b) * 33 + 4 * qd + a] = o[a][b];
    }
    __syncthreads();
    // one 32-lane half-wave per token: 8 tokens per pass
    const int e = tid & 31;
    const int nb = E / 32, blk = d0 / 32;
    for (int t = tid >> 5; t < nt; t += 8) {
        const float v = ob[t * 33 + e];
        const int tok = t0 + t;
        if (out_f32) out_f32[(size_t) tok * E + d0 + e] = v;
        if (q41) {
            // Q4_1 model: quantize_row_q4_1 (AVX2, ggml.c:847-920) of the block by the lane
            // quad e < 4, written as the ActQ and (xs41 given) the Q4_1 MFMA operands (mm_mfma41.hip)
            if (e < 4) {
                float dd, mm;
                uint32_t qword;
                mv::q41_block_lds(ob + t * 33, e, dd, mm, qword);
                const int base = (tid & 63) & ~3;
                const uint32_t q0 = __shfl(qword, base), q1 = __shfl(qword, base + 1);
                const uint32_t q2 = __shfl(qword, base + 2), q3 = __shfl(qword, base + 3);
                if (e == 0) {
                    out.d[(size_t) tok * out.nb + blk] = dd;
                    out.m[(size_t) tok * out.nb + blk] = mm;
                    out.qs[(size_t) tok * out.nb + blk] = make_uint4(q0, q1, q2, q3);
                }
                if (xs41) act41_emit(tok, nb, blk, e, qword, dd, mm, (uint4 *) xm, xs41);
            }
            continue;
        }
        float amax = fabsf(v);
        for (int o2 = 16; o2 > 0; o2 >>= 1) { const float w = __shfl_xor(amax, o2); amax = w > amax ? w : amax; }
        const float dd = amax / 7.0f;
        const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
        const uint32_t qq = (uint32_t) ((int) __builtin_rintf(v * id) + 8) & 15u;
        uint32_t part = qq << (4 * (e & 7));
        part |= __shfl_xor(part, 1);
        part |= __shfl_xor(part, 2);
        part |= __shfl_xor(part, 4);
        // the reference block (d + 16 nibble bytes): lanes e = 0, 8, 16, 24 hold its 4 words
        const uint32_t w0 = __shfl(part, (tid & 32) + 0), w1 = __shfl(part, (tid & 32) + 8);
        const uint32_t w2 = __shfl(part, (tid & 32) + 16), w3 = __shfl(part, (tid & 32) + 24);
        if (e == 0) {
            out.d[(size_t) tok * out.nb + blk] = dd;
            out.qs[(size_t) tok * out.nb + blk] = make_uint4(w0, w1, w2, w3);
        }
        if (xm && e < 4) {
            // the masked MFMA fragment image of the Wo input (mm_mfma.hip): group c = e holds
            // elements 8c..8c+7 = word c; chain 2c -> lane n, chain 2c+1 -> lane 48 + n
            const uint32_t word = e == 0 ? w0 : e == 1 ? w1 : e == 2 ? w2 : w3;
            uint16_t hh[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                hh[k] = __builtin_bit_cast(uint16_t, (_Float16) (float) ((int) ((word >> (4 * k)) & 15u) - 8));
            xm[xm_slot(tok, nb, blk, e, tok & 15)] = make_uint2(hh[0] | (uint32_t) hh[2] << 16, hh[1] | (uint32_t) hh[3] << 16);
            xm[xm_slot(tok, nb, blk, e, 48 + (tok & 15))] =
                make_uint2(hh[4] | (uint32_t) hh[6] << 16, hh[5] | (uint32_t) hh[7] << 16);
            if (e == 0) xda[(size_t) tok * nb + blk] = dd;
        }
    }
}

}  // namespace

bool attention_prompt_supported(int n_embd, int n_head, int n_ctx) {
    return n_embd / n_head == HD && n_ctx % 32 == 0 && n_ctx <= 1024;
}

hipError_t launch_attention_prompt(const AttnLaunch & A, uint16_t * p_scratch, void * xm, float * xda,
                                   hipStream_t s, void * xs41) {
    if (!attention_prompt_supported(A.n_embd, A.n_head, A.n_ctx)) return hipErrorNotSupported;
    // Q4_1 writes its MFMA operands (xm + xs41) or nothing but the ActQ; Q4_0 xm + xda
    if (A.out_qtype == Q4_1 ? (xm != nullptr) != (xs41 != nullptr) : A.out_qtype != Q4_0 || xs41)
        return hipErrorNotSupported;
    const float scale = 1.0f / sqrtf((float) A.n_embd / (float) A.n_head);   // llama.cpp:1028
    constexpr int T = 16;
    EventSplit ev;
    ev.first();
    const size_t lds1 = (size_t) T * 256 + (size_t) T * A.n_ctx * 4;
    const int nblk = (A.n_tokens + T - 1) / T;
    const dim3 g1(A.n_head, (nblk + 1) / 2);
    if (A.exp_computed == 2)
        LVK_LAUNCH((k_attn_p_scores<T, 2>), g1, dim3(256), lds1, s, A.q16, A.kc, A.exp_tab, A.sp, A.n_embd, A.n_ctx,
                   scale, p_scratch, A.exp_computed);
    else if (A.exp_computed == 1)
        LVK_LAUNCH((k_attn_p_scores<T, 1>), g1, dim3(256), lds1, s, A.q16, A.kc, A.exp_tab, A.sp, A.n_embd, A.n_ctx,
                   scale, p_scratch, A.exp_computed);
    else
        LVK_LAUNCH((k_attn_p_scores<T, 0>), g1, dim3(256), lds1, s, A.q16, A.kc, A.exp_tab, A.sp, A.n_embd, A.n_ctx,
                   scale, p_scratch, A.exp_computed);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds2 = (size_t) 64 * A.n_ctx * 2;
    ev.last();
    LVK_LAUNCH(k_attn_p_pv, dim3(A.n_head, (A.n_tokens + 31) / 32, HD / 32), dim3(256), lds2, s, A.vc, p_scratch,
               A.sp, A.n_embd, A.n_ctx, A.out, (uint2 *) xm, xda, A.out_f32, A.out_qtype == Q4_1 ? 1 : 0,
               (uint4 *) xs41);
    return hipGetLastError();
}

}  // namespace lvk
