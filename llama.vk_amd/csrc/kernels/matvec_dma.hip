// matvec_dma.hip -- single-token Q4_0 matvec whose weight stream lands in LDS by LDS-DMA,
// for the decode shapes with few row groups per CU (Wo, W2: 2 per CU on the 7B shapes).
//
// Same arithmetic as matvec_cu.hip (ggml_vec_dot_q4_0 AVX2 chains, ggml.c:1950-2026, on an
// activation quantized by quantize_row_q4_0, ggml.c:621-685; lane 8r+j = chain j of row r)
// and the same octet image, row-group split (one workgroup per CU, contiguous row groups)
// and epilogues.  What differs is where a wave's weights wait for their chain:
//
//   * matvec_cu keeps D chunks (5 KiB each) per wave in VGPRs.  With two compute waves per
//     CU that is 20-40 KiB in flight per CU, and at the loaded HBM latency a CU then pulls
//     10-20 GB/s: Wo (41 KiB per CU) and W2 (110 KiB per CU) are bound by the bytes a CU
//     keeps in flight (Little's law), not by HBM.
//   * here each compute wave DMAs its chunks (global_load_lds_dwordx4, 1 KiB per wave
//     instruction, no VGPRs) into a ring of R slots of its own in LDS: R = 4 (Wo) or 11 (W2)
//     is the whole row group, i.e. every weight byte of the launch is requested in the
//     first microsecond while prologue waves load the input and build the activation
//     table.  The chains then read their operands with ds_read_b128.
//
// The DMAs are inline asm, invisible to hipcc's wait-count pass: the wave waits for its own
// chunk i with s_waitcnt vmcnt(5 x the chunks issued after it) (every chunk is exactly 5
// DMAs -- a row's partial last chunk loads filler into its unused sub-chunk space), and the
// workgroup barrier between the table and the chains is an LDS-only barrier (a
// __syncthreads would wait for every DMA in flight).
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

#include <cstdlib>
#include <type_traits>
#include <utility>

namespace lvk {

namespace {
using namespace mv;

struct DmaParams {
    const uint4 * nib;
    const float4 * scl;
    int G;                      // row groups (M / 8)
    const float * x;            // PRO_ACTF / PRO_NORM: f32 input [K]
    const float * g;            // PRO_NORM: norm weight [K]
    ActQ xq;                    // PRO_ACTQ: quantized input
    float * y;                  // EPI_RESID / EPI_STORE
    // EPI_QKV (matvec_cu.hip): RoPE + KV append of the stacked Wq|Wk|Wv rows
    const StepParams * sp;
    uint16_t * q16;
    uint16_t * kc;
    uint16_t * vc;
    const float2 * rope;
    int n_embd, head_dim, n_ctx;
    int kv32;
};

constexpr int SRS = 40, SPL = 8 * SRS;      // per-wave scale table (matvec_cu.hip)
constexpr int SLOT = 5 * 1024;              // one chunk: 4 x 1 KiB nibbles + 1 KiB scales

__device__ __forceinline__ unsigned lds_u32(const void * p) {
    return (unsigned) (uintptr_t) (const __attribute__((address_space(3))) uint8_t *) p;
}
// one 1 KiB LDS-DMA: lane l's 16 bytes at gsrc land at LDS byte lds_dst + 16 l
__device__ __forceinline__ void dma1k(const void * gsrc, unsigned lds_dst) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
// s_waitcnt vmcnt(N): the DMAs are invisible to hipcc's wait-count pass
template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
// f(std::integral_constant<int, 0>), ..., f(std::integral_constant<int, N - 1>): a chunk loop
// whose index is a constant expression (wait counts are instruction immediates)
template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F && f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F && f) { static_for_impl(f, std::make_integer_sequence<int, N>{}); }

template <int NW, int NP, int R, int PRO, int EPI, int KT>
__global__ __launch_bounds__((NW + NP) * 64) void k_mv_dma(DmaParams P) {
    constexpr int nb = KT / 32;                 // blocks per row
    constexpr int nsub = nb / 8;                // 8-block sub-chunks
    constexpr int NC = (nb + 31) / 32;          // chunks of 32 blocks
    constexpr int PT = NP * 64;                 // prologue threads
    static_assert(nb % 8 == 0, "K must be a multiple of 256");
    static_assert(NP > 0, "prologue waves build the table");

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t * act = (uint32_t *) smem;                                 // nb * 32 B
    float * dxp = (float *) (smem + nb * 32);                           // NC * 128 B
    float * sbuf = dxp + NC * 32;                                       // NW * 2 * SPL floats
    uint8_t * ring0 = (uint8_t *) (sbuf + NW * 2 * SPL);                // NW * NC * SLOT

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    if (wave >= NW) {
        // ---- prologue waves: the activation table (the compute waves' DMAs are in flight)
        const int pt = tid - NW * 64;
        if constexpr (PRO == PRO_ACTF || PRO == PRO_NORM) {
            constexpr int nunits = KT / 8;
            constexpr int UMP = (nunits + PT - 1) / PT;
            float4 xv[UMP][2];
            float4 gv[PRO == PRO_NORM ? UMP : 1][2];
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int un = min(k * PT + pt, nunits - 1);
                const float4 * xp = (const float4 *) (P.x + (size_t) un * 8);
                xv[k][0] = xp[0]; xv[k][1] = xp[1];
                if constexpr (PRO == PRO_NORM) {
                    const float4 * gp = (const float4 *) (P.g + (size_t) un * 8);
                    gv[k][0] = gp[0]; gv[k][1] = gp[1];
                }
            }
            constexpr int XPL = PRO == PRO_NORM ? KT / 4 / 64 : 1;
            float4 xs[XPL];
            if constexpr (PRO == PRO_NORM) {
#pragma unroll
                for (int q = 0; q < XPL; ++q) xs[q] = ((const float4 *) P.x)[q * 64 + lane];
            }
            // barrier A: the inputs enter the CU's texture queue ahead of the DMA burst
            __builtin_amdgcn_s_barrier();
            float scale = 1.0f;
            if constexpr (PRO == PRO_NORM) {
                // ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076): every prologue wave
                // sums all K squares itself (lane-strided, then a butterfly that leaves the
                // same double in every lane); float squares carried in double
                double acc = 0.0;
#pragma unroll
                for (int q = 0; q < XPL; ++q) {
                    const float e[4] = {xs[q].x, xs[q].y, xs[q].z, xs[q].w};
#pragma unroll
                    for (int t = 0; t < 4; ++t) { const float sq = e[t] * e[t]; acc += (double) sq; }
                }
                acc = warp_sum_d(acc);
                const float mean = (float) (acc / (double) KT);
                scale = 1.0f / sqrtf(mean + 1e-6f);
            }
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                if (k * PT >= nunits) break;
                const int un = k * PT + pt;
                float v[8] = {xv[k][0].x, xv[k][0].y, xv[k][0].z, xv[k][0].w,
                              xv[k][1].x, xv[k][1].y, xv[k][1].z, xv[k][1].w};
                if constexpr (PRO == PRO_NORM) {
                    const float gg[8] = {gv[k][0].x, gv[k][0].y, gv[k][0].z, gv[k][0].w,
                                         gv[k][1].x, gv[k][1].y, gv[k][1].z, gv[k][1].w};
#pragma unroll
                    for (int e = 0; e < 8; ++e) {
                        const float yn = v[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                        v[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                    }
                }
                float amax = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) { const float a = fabsf(v[e]); amax = a > amax ? a : amax; }
                // the 4 units of a block are a lane quad: block amax (ggml.c:636-649)
                const float o0 = quad_bcast<0>(amax), o1 = quad_bcast<1>(amax);
                const float o2 = quad_bcast<2>(amax), o3 = quad_bcast<3>(amax);
                const float m01 = o1 > o0 ? o1 : o0, m23 = o3 > o2 ? o3 : o2;
                amax = m23 > m01 ? m23 : m01;
                const float d = amax / 7.0f;                              // ggml.c:651
                const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
                const uint32_t w = q40_pack8(v, id);
                if (un < nunits) act_store(act, dxp, un >> 2, un & 3, w, d, (un & 3) == 0);
            }
        } else {
            constexpr int UMP = (nb + PT - 1) / PT;
            uint4 qv[UMP];
            float dv[UMP];
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int b = min(k * PT + pt, nb - 1);
                qv[k] = P.xq.qs[b];
                dv[k] = P.xq.d[b];
            }
            __builtin_amdgcn_s_barrier();       // barrier A (see above)
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int b = k * PT + pt;
                if (b < nb) {
                    const uint4 qs = qv[k];
                    const float d = dv[k];
                    act_store(act, dxp, b, 0, qs.x, d, true);
                    act_store(act, dxp, b, 1, qs.y, 0.0f, false);
                    act_store(act, dxp, b, 2, qs.z, 0.0f, false);
                    act_store(act, dxp, b, 3, qs.w, 0.0f, false);
                }
            }
        }
        lds_barrier();          // table ready (the compute waves join this barrier)
        return;
    }

    // ---- compute waves: row group g0 + wave of this workgroup (one per wave: the host
    // launches NW >= the row groups of any CU), its NC chunks all in flight at once
    const int j = lane & 7;
    const int r = lane >> 3;
    const int nwg = gridDim.x;
    const int g0 = (int) (blockIdx.x * (unsigned) P.G / (unsigned) nwg);     // G * n_cu < 2^32
    const int g1 = (int) ((blockIdx.x + 1) * (unsigned) P.G / (unsigned) nwg);
    __builtin_amdgcn_s_barrier();               // barrier A: the prologue's input loads went out first
    if (g0 + wave >= g1) { lds_barrier(); return; }
    const int grp = g0 + wave;
    uint8_t * ring = ring0 + (size_t) wave * NC * SLOT;
    const unsigned ring_l = __builtin_amdgcn_readfirstlane(lds_u32(ring));
    // chunk cc into slot cc: 4 nibble sub-chunks + the scales; a partial last chunk of a row
    // loads its scales again into the unused sub-chunk space, so every chunk is 5 DMAs
    static_for<NC>([&](auto cv) __attribute__((always_inline)) {
        constexpr int cc = decltype(cv)::value;
        const uint4 * src = P.nib + ((size_t) grp * NC * 4 + cc * 4) * 64 + lane;
        const float4 * ssrc = P.scl + ((size_t) grp * NC + cc) * 64 + lane;
        const unsigned d = ring_l + (unsigned) cc * SLOT;
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            if (cc * 4 + sb < nsub) dma1k(src + sb * 64, d + sb * 1024);
            else dma1k(ssrc, d + sb * 1024);
        }
        dma1k(ssrc, d + 4096);
    });

    float * sw = sbuf + wave * 2 * SPL;
    auto make_table = [&](int buf, int cc) __attribute__((always_inline)) {
        const float4 Sv = *((const float4 *) (ring + (size_t) cc * SLOT + 4096) + lane);
        const float4 dx = *(const float4 *) (dxp + cc * 32 + j * 4);
        float4 sv;
        sv.x = Sv.x * dx.x; sv.y = Sv.y * dx.y; sv.z = Sv.z * dx.z; sv.w = Sv.w * dx.w;   // ggml.c:1968
        *(float4 *) (sw + buf * SPL + r * SRS + j * 4) = sv;
    };

    lds_barrier();              // the activation table (dxp) is ready
    wait_vm<5 * (NC - 1)>();    // chunk 0 landed (the later chunks may still be in flight)
    make_table(0, 0);
    __builtin_amdgcn_wave_barrier();

    float acc = 0.0f;
    static_for<NC>([&](auto cv) __attribute__((always_inline)) {
        constexpr int c = decltype(cv)::value;
        constexpr int tb = c & 1;
        const uint4 * wl = (const uint4 *) (ring + (size_t) c * SLOT) + lane;
        uint4 W[4];
#pragma unroll
        for (int sb = 0; sb < 4; ++sb)
            if (c * 4 + sb < nsub) W[sb] = wl[sb * 64];
        uint4 A[8];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (c * 4 + q / 2 < nsub) A[q] = *(const uint4 *) (act + ((c * 8 + q) * 8 + j) * 4);
        const float * sl = sw + tb * SPL;
        float sa[8][4];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const float4 v = *(const float4 *) (sl + r * SRS + jj * 4);
            sa[jj][0] = v.x; sa[jj][1] = v.y; sa[jj][2] = v.z; sa[jj][3] = v.w;
        }
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            if (c * 4 + sb < nsub) {
                const uint32_t wd[4] = {W[sb].x, W[sb].y, W[sb].z, W[sb].w};
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    const int bi = sb * 8 + pp * 4;
                    const uint4 a = A[sb * 2 + pp];
                    const int p0 = dot8(wd[2 * pp], a.x);
                    const int p1 = dot8(wd[2 * pp], a.y);
                    const int p2 = dot8(wd[2 * pp + 1], a.z);
                    const int p3 = dot8(wd[2 * pp + 1], a.w);
                    acc = __builtin_fmaf(sa[(bi + 0) & 7][(bi + 0) >> 3], (float) p0, acc);
                    acc = __builtin_fmaf(sa[(bi + 1) & 7][(bi + 1) >> 3], (float) p1, acc);
                    acc = __builtin_fmaf(sa[(bi + 2) & 7][(bi + 2) >> 3], (float) p2, acc);
                    acc = __builtin_fmaf(sa[(bi + 3) & 7][(bi + 3) >> 3], (float) p3, acc);
                }
            }
        }
        // the next chunk's scale table; its DMAs landed once the NC - 2 - c after it may
        // still be in flight
        if constexpr (c + 1 < NC) {
            wait_vm<5 * (NC - 2 - c)>();
            make_table(tb ^ 1, c + 1);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("" : "+v"(acc));     // chunks in program order (matvec_cu.hip rule 4)
        __builtin_amdgcn_sched_barrier(0);
    });
    const float res = octet_reduce(acc);
    const int row = grp * 8 + r;
    if constexpr (EPI == EPI_STORE) {
        if (j == 0) P.y[row] = res;
    } else if constexpr (EPI == EPI_RESID) {
        if (j == 0) P.y[row] = res + P.y[row];      // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
    } else if constexpr (EPI == EPI_QKV) {
        const int E = P.n_embd, hd = P.head_dim;
        const int which = row / E;          // 0 q, 1 k, 2 v (uniform per wave: E % 8 == 0)
        const int e = row - which * E;
        const int pos = P.sp->n_past;
        const float other = __shfl_xor(res, 8);   // row e^1 lives in lanes of row r^1
        if (j == 0) {
            if (which < 2) {
                // ggml_compute_forward_rope_f32 mode 0 (ggml.c:7209-7223)
                const int i0 = e % hd;
                const float2 cs = P.rope[(size_t) pos * (hd / 2) + (i0 >> 1)];
                float out;
                if ((i0 & 1) == 0) { const float a = res * cs.x, b = other * cs.y; out = a - b; }
                else               { const float a = other * cs.y, b = res * cs.x; out = a + b; }
                if (which == 0) kv_store(P.q16, e, out, P.kv32);
                else            kv_store(P.kc, (size_t) pos * E + e, out, P.kv32);
            } else {
                kv_store(P.vc, (size_t) e * P.n_ctx + pos, res, P.kv32);     // llama.cpp:996-1008
            }
        }
    }
}

// ---- Q4_1 (13B): the k_mv_cu41 chains (ggml_vec_dot_q4_1 AVX2, ggml.c:2188-2258) with
// the chunk's nibbles, d, m and even-chain weight sums (7 KiB, 7 DMAs) from the LDS ring
constexpr int SWF41 = 4 * SPL;                 // per-wave product tables: s, dx*my, mx*dy, mx*my
constexpr int SLOT41 = 7 * 1024;

struct Dma41Params {
    const uint4 * nib;
    const float4 * scl;         // [G][NC][2][64]: d, then m
    const uint4 * wsum;         // [G][NC][64]
    int G;
    const float * x;            // PRO_ACTF
    ActQ xq;                    // PRO_ACTQ (d, m, qs)
    float * y;
};

template <int NW, int NP, int R, int PRO, int EPI, int KT>
__global__ __launch_bounds__((NW + NP) * 64) void k_mv_dma41(Dma41Params P) {
    constexpr int nb = KT / 32;
    constexpr int nsub = nb / 8;
    constexpr int NC = (nb + 31) / 32;
    constexpr int PT = NP * 64;
    static_assert(nb % 8 == 0 && NP > 0, "shape");

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t * act = (uint32_t *) smem;                          // nb * 32 B
    float * dyv = (float *) (smem + nb * 32);                    // NC * 32
    float * myv = dyv + NC * 32;                                 // NC * 32
    uint8_t * ys = (uint8_t *) (myv + NC * 32);                  // nb * 4 bytes (room: nb * 16)
    float * sbuf = (float *) (ys + nb * 16);                     // NW * SWF41
    uint8_t * ring0 = (uint8_t *) (sbuf + NW * SWF41);           // NW * R * SLOT41

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    if (wave >= NW) {
        const int pt = tid - NW * 64;
        if constexpr (PRO == PRO_ACTF) {
            constexpr int nunits = KT / 8;
            constexpr int UMP = (nunits + PT - 1) / PT;
            float4 xv[UMP][2];
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int un = min(k * PT + pt, nunits - 1);
                const float4 * xp = (const float4 *) (P.x + (size_t) un * 8);
                xv[k][0] = xp[0]; xv[k][1] = xp[1];
            }
            __builtin_amdgcn_s_barrier();       // barrier A: inputs ahead of the DMA burst
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                if (k * PT >= nunits) break;
                const int un = k * PT + pt;
                float v[8] = {xv[k][0].x, xv[k][0].y, xv[k][0].z, xv[k][0].w,
                              xv[k][1].x, xv[k][1].y, xv[k][1].z, xv[k][1].w};
                // quantize_row_q4_1 of the block held by this lane quad (ggml.c:847-920)
                float d, m;
                uint32_t qw;
                q41_quad(v, d, m, qw);
                uint32_t qs[4];
                qs[0] = __builtin_bit_cast(uint32_t, quad_bcast<0>(__builtin_bit_cast(float, qw)));
                qs[1] = __builtin_bit_cast(uint32_t, quad_bcast<1>(__builtin_bit_cast(float, qw)));
                qs[2] = __builtin_bit_cast(uint32_t, quad_bcast<2>(__builtin_bit_cast(float, qw)));
                qs[3] = __builtin_bit_cast(uint32_t, quad_bcast<3>(__builtin_bit_cast(float, qw)));
                if (un < nunits && (un & 3) == 0) act41_store(act, dyv, myv, ys, un >> 2, qs, d, m);
            }
        } else {
            constexpr int UMP = (nb + PT - 1) / PT;
            uint4 qv[UMP];
            float dv[UMP], mv_[UMP];
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int b = min(k * PT + pt, nb - 1);
                qv[k] = P.xq.qs[b];
                dv[k] = P.xq.d[b];
                mv_[k] = P.xq.m[b];
            }
            __builtin_amdgcn_s_barrier();       // barrier A
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int b = k * PT + pt;
                if (b < nb) {
                    const uint32_t qs[4] = {qv[k].x, qv[k].y, qv[k].z, qv[k].w};
                    act41_store(act, dyv, myv, ys, b, qs, dv[k], mv_[k]);
                }
            }
        }
        lds_barrier();          // table ready
        return;
    }

    // one row group per compute wave (the host launches NW >= the row groups of any CU);
    // its chunks stream through a ring of R slots, chunk c in slot c % R
    const int j = lane & 7;
    const int r = lane >> 3;
    const int nwg = gridDim.x;
    const int g0 = (int) (blockIdx.x * (unsigned) P.G / (unsigned) nwg);
    const int g1 = (int) ((blockIdx.x + 1) * (unsigned) P.G / (unsigned) nwg);
    __builtin_amdgcn_s_barrier();               // barrier A
    if (g0 + wave >= g1) { lds_barrier(); return; }
    const int grp = g0 + wave;
    uint8_t * ring = ring0 + (size_t) wave * R * SLOT41;
    const unsigned ring_l = __builtin_amdgcn_readfirstlane(lds_u32(ring));
    // chunk cc into its slot: 4 nibble sub-chunks (filler past a row's end), d, m, wsum
    auto issue = [&](auto cv) __attribute__((always_inline)) {
        constexpr int cc = decltype(cv)::value;
        const uint4 * src = P.nib + ((size_t) grp * NC * 4 + cc * 4) * 64 + lane;
        const float4 * ssrc = P.scl + ((size_t) grp * NC + cc) * 128 + lane;
        const uint4 * wsrc = P.wsum + ((size_t) grp * NC + cc) * 64 + lane;
        const unsigned d = ring_l + (unsigned) (cc % R) * SLOT41;
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            if (cc * 4 + sb < nsub) dma1k(src + sb * 64, d + sb * 1024);
            else dma1k(wsrc, d + sb * 1024);
        }
        dma1k(ssrc, d + 4096);
        dma1k(ssrc + 64, d + 5120);
        dma1k(wsrc, d + 6144);
    };
    static_for<(R < NC ? R : NC)>(issue);

    lds_barrier();              // the activation table is ready
    const bool even = (j & 1) == 0;
    const uint32_t * ys32 = (const uint32_t *) ys;
    float * sw = sbuf + wave * SWF41;
    float acc = 0.0f, off = 0.0f;
    static_for<NC>([&](auto cv) __attribute__((always_inline)) {
        constexpr int c = decltype(cv)::value;
        // chunk c landed once at most the chunks issued after it are in flight
        wait_vm<7 * ((c + R - 1 < NC - 1 ? c + R - 1 : NC - 1) - c)>();
        const uint4 * wl = (const uint4 *) (ring + (size_t) (c % R) * SLOT41) + lane;
        uint4 W[4];
#pragma unroll
        for (int sb = 0; sb < 4; ++sb)
            if (c * 4 + sb < nsub) W[sb] = wl[sb * 64];
        const float4 SD = *(const float4 *) (wl + 256);
        const float4 SM = *(const float4 *) (wl + 320);
        const uint4 WS = wl[384];
        // products of blocks 32c + 8m + j of this lane's row (ggml.c:2205-2212)
        const float4 dy = *(const float4 *) (dyv + c * 32 + j * 4);
        const float4 my = *(const float4 *) (myv + c * 32 + j * 4);
        float * sl = sw + r * SRS + j;
        const float dxa[4] = {SD.x, SD.y, SD.z, SD.w};
        const float mxa[4] = {SM.x, SM.y, SM.z, SM.w};
        const float dya[4] = {dy.x, dy.y, dy.z, dy.w};
        const float mya[4] = {my.x, my.y, my.z, my.w};
#pragma unroll
        for (int mq = 0; mq < 4; ++mq) {
            sl[mq * 8] = dxa[mq] * dya[mq];
            sl[SPL + mq * 8] = dxa[mq] * mya[mq];
            sl[2 * SPL + mq * 8] = mxa[mq] * dya[mq];
            sl[3 * SPL + mq * 8] = mxa[mq] * mya[mq];
        }
        // the slot's operands are in registers: refill it with chunk c + R
        if constexpr (c + R < NC) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue(std::integral_constant<int, c + R>{});
        }
        __builtin_amdgcn_wave_barrier();
        const float * srow = sw + r * SRS;
        const float * xrow = srow + (even ? SPL : 2 * SPL);
        const float * mrow = srow + 3 * SPL;
        // even chains: the precomputed weight sums (blocks 0-15 of the chunk in their own
        // word, 16-31 in the odd neighbour's: DPP quad_perm [1,1,3,3]); odd chains: the
        // activation sums from LDS (ggml.c:2236-2240), one byte per block
        const uint32_t wown[4] = {WS.x, WS.y, WS.z, WS.w};
        uint32_t wnb[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) wnb[q] = (uint32_t) __builtin_amdgcn_mov_dpp((int) wown[q], 0xF5, 0xF, 0xF, false);
#pragma unroll
        for (int sb = 0; sb < 4; ++sb) {
            if (c * 4 + sb < nsub) {
                const uint32_t wd[4] = {W[sb].x, W[sb].y, W[sb].z, W[sb].w};
#pragma unroll
                for (int pp = 0; pp < 2; ++pp) {
                    const int uu = c * 8 + sb * 2 + pp;
                    const int bi = sb * 8 + pp * 4;
                    const uint4 a = *(const uint4 *) (act + ((size_t) uu * 8 + j) * 4);
                    const float4 s4 = *(const float4 *) (srow + bi);
                    const float4 x4 = *(const float4 *) (xrow + bi);
                    const float4 m4 = *(const float4 *) (mrow + bi);
                    const uint32_t ydw = ys32[(size_t) uu * 4 + (j >> 1)];
                    const uint32_t wdw = sb < 2 ? wown[(sb & 1) * 2 + pp] : wnb[(sb & 1) * 2 + pp];
                    const uint32_t sdw = even ? wdw : ydw;
                    const float S[4] = {(float) (sdw & 0xFFu), (float) ((sdw >> 8) & 0xFFu),
                                        (float) ((sdw >> 16) & 0xFFu), (float) (sdw >> 24)};
                    const int p[4] = {udot8(wd[2 * pp], a.x), udot8(wd[2 * pp], a.y),
                                      udot8(wd[2 * pp + 1], a.z), udot8(wd[2 * pp + 1], a.w)};
                    const float sv[4] = {s4.x, s4.y, s4.z, s4.w};
                    const float xs[4] = {x4.x, x4.y, x4.z, x4.w};
                    const float ms[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        acc = __builtin_fmaf(sv[q], (float) p[q], acc);    // ggml.c:2244
                        acc = __builtin_fmaf(xs[q], S[q], acc);            // ggml.c:2247
                        off = off + ms[q];                                 // ggml.c:2226
                    }
                }
            }
        }
        // the product tables are rewritten by the next chunk
        asm volatile("" : "+v"(acc), "+v"(off));
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_sched_barrier(0);
    });
    const float res = octet_reduce(acc) + off * 32.0f;      // acc_offset * QK (ggml.c:2249)
    const int row = grp * 8 + r;
    if constexpr (EPI == EPI_STORE) {
        if (j == 0) P.y[row] = res;
    } else {
        if (j == 0) P.y[row] = res + P.y[row];      // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
    }
}

template <int NW, int NP, int R, int PRO, int EPI, int KT>
hipError_t go41(const Dma41Params & P, hipStream_t s) {
    constexpr int nb = KT / 32, NC = (nb + 31) / 32;
    const int nwg = std::min(cu_count(), P.G);
    if ((P.G + nwg - 1) / nwg > NW) return hipErrorNotSupported;      // one row group per wave
    const size_t lds = (size_t) nb * 32 + 2 * NC * 128 + (size_t) nb * 16 + (size_t) NW * SWF41 * 4 +
                       (size_t) NW * R * SLOT41;
    if (lds > 160 * 1024) return hipErrorNotSupported;
    LVK_LAUNCH((k_mv_dma41<NW, NP, R, PRO, EPI, KT>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P);
    return hipGetLastError();
}

template <int NW, int NP, int R, int PRO, int EPI, int KT>
hipError_t go(const DmaParams & P, hipStream_t s) {
    constexpr int nb = KT / 32, NC = (nb + 31) / 32;
    static_assert(R == NC, "the Q4_0 form keeps a whole row group in flight");
    const int nwg = std::min(cu_count(), P.G);
    if ((P.G + nwg - 1) / nwg > NW) return hipErrorNotSupported;      // one row group per wave
    const size_t lds = (size_t) nb * 32 + NC * 128 + (size_t) NW * 2 * SPL * 4 + (size_t) NW * NC * SLOT;
    if (lds > 160 * 1024) return hipErrorNotSupported;
    LVK_LAUNCH((k_mv_dma<NW, NP, R, PRO, EPI, KT>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P);
    return hipGetLastError();
}

}  // namespace

// LVK_MV_DMA=0 keeps Wo / W2 on matvec_cu.hip (A/B runs)
bool matvec_dma_enabled() {
    static const bool on = [] { const char * e = getenv("LVK_MV_DMA"); return !e || atoi(e) != 0; }();
    return on;
}

hipError_t launch_matvec_dma41(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype != Q4_1 || L.n_tokens != 1 || L.w.M % 8 || epi != EPI_RESID) return hipErrorNotSupported;
    Dma41Params P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.wsum = q41_wsum(L.w);
    P.G = L.w.M / 8;
    P.x = L.x ? L.x + (size_t) L.tok0 * L.w.K : nullptr;
    P.xq = L.xq;
    if (P.xq.qs) {
        P.xq.qs += (size_t) L.tok0 * L.xq.nb;
        P.xq.d += (size_t) L.tok0 * L.xq.nb;
        P.xq.m += (size_t) L.tok0 * L.xq.nb;
    }
    P.y = L.y ? L.y + (size_t) L.out_tok0 * L.w.M : nullptr;
    const int nwg = std::min(cu_count(), P.G);
    const int per_cu = (P.G + nwg - 1) / nwg;
    // 13B: 2-3 row groups per CU, one per compute wave
    if (L.w.K == 5120 && pro == PRO_ACTQ && per_cu <= 3) return go41<3, 2, 5, PRO_ACTQ, EPI_RESID, 5120>(P, s);
    if (L.w.K == 13824 && pro == PRO_ACTF && per_cu <= 3) return go41<3, 5, 4, PRO_ACTF, EPI_RESID, 13824>(P, s);
    return hipErrorNotSupported;
}

hipError_t launch_matvec_dma(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype == Q4_1) return launch_matvec_dma41(L, pro, epi, s);
    if (L.w.qtype != Q4_0 || L.n_tokens != 1 || L.w.M % 8 || (epi != EPI_RESID && epi != EPI_QKV))
        return hipErrorNotSupported;
    DmaParams P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.G = L.w.M / 8;
    P.x = L.x ? L.x + (size_t) L.tok0 * L.w.K : nullptr;
    P.g = L.g;
    P.xq = L.xq;
    if (P.xq.qs) { P.xq.qs += (size_t) L.tok0 * L.xq.nb; P.xq.d += (size_t) L.tok0 * L.xq.nb; }
    P.y = L.y ? L.y + (size_t) L.out_tok0 * L.w.M : nullptr;
    P.sp = L.sp;
    P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx; P.kv32 = L.kv32;
    const int per_cu = (P.G + std::min(cu_count(), P.G) - 1) / std::min(cu_count(), P.G);
    // QKV (LVK_MV_DMA_QKV=1, A/B): six row groups per CU, one per compute wave, all in flight
    if (epi == EPI_QKV) {
        static const bool qkv = [] { const char * e = getenv("LVK_MV_DMA_QKV"); return e && atoi(e) != 0; }();
        if (qkv && L.w.K == 4096 && pro == PRO_NORM && per_cu <= 6) return go<6, 2, 4, PRO_NORM, EPI_QKV, 4096>(P, s);
        return hipErrorNotSupported;
    }
    // two compute waves (one row group each on the 7B shapes), the whole row group in flight
    if (L.w.K == 4096 && pro == PRO_ACTQ && per_cu <= 2) return go<2, 2, 4, PRO_ACTQ, EPI_RESID, 4096>(P, s);
    if (L.w.K == 11008 && pro == PRO_ACTF && per_cu <= 2) return go<2, 6, 11, PRO_ACTF, EPI_RESID, 11008>(P, s);
    return hipErrorNotSupported;
}

}  // namespace lvk
