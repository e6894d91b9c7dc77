// matvec_cu.hip -- CU-balanced single-token Q4_0 matvec (the decode hot path).
//
// Same arithmetic as matvec_q4.hip (bit-faithful ggml_vec_dot_q4_0 AVX2
// chains, ggml.c:1950-2026, on an activation quantized by quantize_row_q4_0,
// ggml.c:621-685), organised for the batch-1 weight stream:
//
//   * A decode matvec reads every weight byte once, so it is bound by how fast
//     each CU can pull bytes (~25-30 GB/s per CU; MI355X_MICROARCH.md, HBM) and
//     by how evenly the bytes are spread over the 256 CUs.  The grid is one
//     workgroup per CU and workgroup w owns row groups [w*G/n, (w+1)*G/n)
//     (a row group = 8 rows = one wavefront's work), so every CU streams the
//     same number of bytes (+-1 row group).
//   * The activation table (RMSNorm + quantize, or a plain quantize) is built
//     once per workgroup in LDS while the first D chunks of weights are
//     already in flight.
//   * Each wave walks its row groups with a D-chunk register prefetch that
//     runs across group boundaries, so a CU's weight stream never drains
//     between groups.  Row length K is a template constant: all loads are
//     exact and static (hipcc's vmcnt accounting stays precise).
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {
using namespace mv;

#ifdef LVK_PROBE_TIMING   // dev probe builds only: per-wave s_memtime trace
__device__ unsigned long long g_trace[256 * 16 * 64];
#define LVK_T(ev)                                                                                  \
    do {                                                                                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                \
        if (lane == 0 && (ev) < 64) g_trace[((blockIdx.x & 255) * 16 + (wave & 15)) * 64 + (ev)] = t_; \
    } while (0)
#else
#define LVK_T(ev) do { } while (0)
#endif

struct CuParams {
    const uint4 * nib;
    const float4 * scl;
    int G;                      // row groups (M / 8)
    const float * x;            // PRO_NORM / PRO_ACTF: f32 input [K]
    const float * g;            // PRO_NORM: norm weight [K]
    ActQ xq;                    // PRO_ACTQ: quantized input
    const StepParams * sp;
    float * y;                  // EPI_STORE / EPI_RESID
    float * u;                  // EPI_SWIGLU_F32: silu(w1 x) * (w3 x) [M/2]
    uint16_t * q16;
    uint16_t * kc;
    uint16_t * vc;
    const float2 * rope;
    int n_embd, head_dim, n_ctx;
    int kv32;                   // f32 KV cache and queries (f16_kv = false)
    const uint16_t * silu_tab;
};

// per-wave block-scale table s = dw * dx in LDS (two buffers, 8 rows x 32 blocks): the row
// stride is padded to 40 floats so the rows start on banks 0, 40, 16, 56, 32, 8, 48, 24 of
// the 64 and the per-row broadcast float4 reads are bank-conflict free
constexpr int SRS = 40, SPL = 8 * SRS;

// the workgroup body (bid of nwg workgroups)
template <int NW, int NP, int D, int PRO, int EPI, int KT, int PF>
__device__ __forceinline__ void mv_cu_run(const CuParams & P, const int bid, const int nwg, uint8_t * smem) {
    constexpr int PT = NP * 64;                 // prologue threads
    constexpr int nb = KT / 32;                 // blocks per row
    constexpr int nsub = nb / 8;                // 8-block sub-chunks (one uint4 per lane each)
    constexpr int NC = (nb + 31) / 32;          // chunks of 32 blocks
    constexpr bool XG = (NC % D) == 0;          // prefetch may cross into the next group
    constexpr int nunits = KT / 8;              // f32 prologue work units (8 elements)
    static_assert(D <= NC, "prefetch deeper than a row");
    static_assert(nb % 8 == 0, "K must be a multiple of 256");

    uint32_t * act = (uint32_t *) smem;                          // nb * 32 B
    float * dxp = (float *) (smem + nb * 32);                    // NC * 128 B
    float * sbuf = dxp + NC * 32;                                // NW * 2 * SPL floats

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
    [[maybe_unused]] int tq = 4;   // trace event index (probe builds)
    LVK_T(0);

    if (NP > 0 && wave >= NW) {
        // ---- prologue waves: build the activation table while the compute
        // waves put the CU's weight stream in flight (they never wait on x)
        const int pt = tid - NW * 64;
        constexpr int PT_ = PT > 0 ? PT : 64;   // (NP == 0: branch never taken)
        if constexpr (PRO == PRO_NORM || PRO == PRO_ACTF) {
            constexpr int UMP = (nunits + PT_ - 1) / PT_;
            float4 xv[UMP][2];
            float4 gv[PRO == PRO_NORM ? UMP : 1][2];
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int un = min(k * PT_ + pt, nunits - 1);
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
                for (int i = 0; i < XPL; ++i) xs[i] = ((const float4 *) P.x)[i * 64 + lane];
            }
            // barrier A: the inputs enter the CU's texture queue ahead of the weight burst
            __builtin_amdgcn_s_barrier();
            float scale = 1.0f;
            if constexpr (PRO == PRO_NORM) {
                // ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076): every
                // prologue wave sums all K squares itself (lane-strided, then a
                // butterfly that leaves the same double in every lane), so no
                // cross-wave reduction is needed.  Terms are float squares
                // carried in double (RMSNorm order).
                double acc = 0.0;
#pragma unroll
                for (int i = 0; i < XPL; ++i) {
                    const float e[4] = {xs[i].x, xs[i].y, xs[i].z, xs[i].w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) { const float sq = e[q] * e[q]; acc += (double) sq; }
                }
                LVK_T(56);
                acc = warp_sum_d(acc);
                const float mean = rms_mean_wave(acc, P.x, KT);
                scale = 1.0f / sqrtf(mean + 1e-6f);
                LVK_T(57);
            }
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                if (k * PT_ >= nunits) break;
                const int un = k * PT_ + pt;
                float v[8] = {xv[k][0].x, xv[k][0].y, xv[k][0].z, xv[k][0].w,
                              xv[k][1].x, xv[k][1].y, xv[k][1].z, xv[k][1].w};
                float amax = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if constexpr (PRO == PRO_NORM) {
                        const float gg[8] = {gv[k][0].x, gv[k][0].y, gv[k][0].z, gv[k][0].w,
                                             gv[k][1].x, gv[k][1].y, gv[k][1].z, gv[k][1].w};
                        const float yn = v[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                        v[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                    }
                    const float a = fabsf(v[e]);
                    amax = a > amax ? a : amax;
                }
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
            __builtin_amdgcn_s_barrier();       // barrier A (see above)
            constexpr int UMP = (nb + PT_ - 1) / PT_;
#pragma unroll
            for (int k = 0; k < UMP; ++k) {
                const int b = k * PT_ + pt;
                if (b < nb) {
                    const uint4 qs = P.xq.qs[b];
                    const float d = P.xq.d[b];
                    act_store(act, dxp, b, 0, qs.x, d, true);
                    act_store(act, dxp, b, 1, qs.y, 0.0f, false);
                    act_store(act, dxp, b, 2, qs.z, 0.0f, false);
                    act_store(act, dxp, b, 3, qs.w, 0.0f, false);
                }
            }
        }
        LVK_T(2);
        __syncthreads();
        return;
    }

    // ---- compute waves
    const int j = lane & 7;
    const int r = lane >> 3;
    const int g0 = (int) ((unsigned) bid * (unsigned) P.G / (unsigned) nwg);     // G * n_cu < 2^32
    const int g1 = (int) ((unsigned) (bid + 1) * (unsigned) P.G / (unsigned) nwg);
    const int ng = max(0, (g1 - g0 - wave + NW - 1) / NW);      // row groups of this wave
    if (NP > 0 && ng == 0) { __builtin_amdgcn_s_barrier(); __syncthreads(); return; }
    int gc = min(g0 + wave, P.G - 1);
    // the QKV epilogue's position, loaded here ahead of the prologue inputs (vmcnt retires in
    // order: the inputs' wait covers it), so that the RoPE pair can be loaded at a row group's
    // start (pre_epi below).  An atomic load: a plain one is sunk to its use; a scalar one sinks
    // too and then holds up the prologue's first barrier, whose lgkmcnt wait covers it.
    [[maybe_unused]] int pos0 = 0;
    if constexpr (EPI == EPI_QKV)
        pos0 = __hip_atomic_load((const __attribute__((address_space(1))) int *) &P.sp->n_past, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);

    // NP == 0: the compute waves build the activation table themselves; its
    // inputs are issued first (vmcnt retires in order)
    constexpr int NT = NW * 64;
    constexpr bool FPRO = (PRO == PRO_NORM || PRO == PRO_ACTF);
    constexpr int UM = NP > 0 ? 1 : (FPRO ? (nunits + NT - 1) / NT : (nb + NT - 1) / NT);
    float4 xv[UM][2];
    float4 gv[UM][2];
    uint4 qv[UM];
    float dv[UM];
    if constexpr (NP == 0) {
        if constexpr (FPRO) {
#pragma unroll
            for (int k = 0; k < UM; ++k) {
                const int un = min(k * NT + tid, nunits - 1);
                const float4 * xp = (const float4 *) (P.x + (size_t) un * 8);
                xv[k][0] = xp[0]; xv[k][1] = xp[1];
                if constexpr (PRO == PRO_NORM) {
                    const float4 * gp = (const float4 *) (P.g + (size_t) un * 8);
                    gv[k][0] = gp[0]; gv[k][1] = gp[1];
                }
            }
        } else {
#pragma unroll
            for (int k = 0; k < UM; ++k) {
                const int b = min(k * NT + tid, nb - 1);
                qv[k] = P.xq.qs[b];
                dv[k] = P.xq.d[b];
            }
        }
    }

    // the prologue inputs, marked landed where the wait count is exact (matvec_common.h):
    // hipcc then waits for exactly them, never for weight loads issued behind them
    auto launder_inputs = [&]() __attribute__((always_inline)) {
        if constexpr (NP == 0) {
#pragma unroll
            for (int k = 0; k < UM; ++k) {
                if constexpr (FPRO) {
                    launder(xv[k][0]); launder(xv[k][1]);
                    if constexpr (PRO == PRO_NORM) { launder(gv[k][0]); launder(gv[k][1]); }
                } else {
                    launder(qv[k]); launder(dv[k]);
                }
            }
        }
    };

    // first D chunks of this wave's first row group (wave-uniform base +
    // 32-bit lane offset: the scalar-base load form).  A wave without row groups (it only
    // helps build the table) issues the same loads with every lane on one 16-byte word:
    // no branch around the issue, so hipcc's wait counts stay exact on every path.
    const bool issue = NP > 0 || ng > 0;
    const uint32_t loff = issue ? (uint32_t) lane * 16u : 0u;
    uint4 W[D][4];
    float4 S[D];
    // the scales of a chunk go out before its nibbles: the scale table of chunk c+1 is
    // built while chunk c's nibbles may still be in flight (vmcnt retires in order)
#define LVK_ISSUE(slot, grp, cc)                                                                        \
    do {                                                                                                \
        const uint4 * nb_ = P.nib + ((size_t) (grp) * NC * 4 + (cc) * 4) * 64;                          \
        S[slot] = *(const float4 *) ((const char *) (P.scl + ((size_t) (grp) * NC + (cc)) * 64) + loff); \
        _Pragma("unroll") for (int sb = 0; sb < 4; ++sb) if ((cc) * 4 + sb < nsub)                      \
            W[slot][sb] = ld_nt((const uint4 *) ((const char *) (nb_ + sb * 64) + loff));               \
        __builtin_amdgcn_sched_barrier(0);                                                              \
    } while (0)
    // Order of the prologue and the first weight loads (PF):
    //   0: the inputs, then the weights are issued, then the activation table is built as
    //      soon as the inputs land (the weights stay in flight);
    //   1: the inputs land, then the weights are issued, then the table is built;
    //   2: the inputs land and the table is built, then the weights are issued;
    //   3: as 2, but the weights are issued after the workgroup barrier;
    //   4: as 0, but only chunk 0 goes out before the table, chunks 1..D-1 after the barrier
    //      (the barriers wait for the slowest wave's issue, which the memory system throttles
    //      to the return rate once the CU's queue is full);
    //   5: as 4, but the inputs land before chunk 0 is issued.
    // A CU's texture unit takes a 1 KiB wave load in ~16 cycles: issuing 80-160 KiB of
    // weights keeps every wave of the CU in its issue for 1.3-4k cycles, so with 0 or 1 the
    // table (and the first chain) waits for the wave's own share of the burst to be issued.
    constexpr bool SPLIT = PF == 4 || PF == 5;
    if constexpr (PF != 0 && PF != 4) launder_inputs();
    // prologue waves (NP > 0): the weight burst goes out behind their inputs (barrier A)
    if constexpr (NP > 0) __builtin_amdgcn_s_barrier();
    LVK_T(58);
    if constexpr (PF <= 1) {
#pragma unroll
        for (int d = 0; d < D; ++d) LVK_ISSUE(d, gc, d);
    } else if constexpr (SPLIT) {
        LVK_ISSUE(0, gc, 0);
    }
    if constexpr (PF == 0 || PF == 4) launder_inputs();
    LVK_T(59);

    if constexpr (NP == 0) {
        double * red = (double *) (sbuf + NW * 2 * SPL); // NW doubles (after the s buffers)
        if constexpr (FPRO) {
            float scale = 1.0f;
            if constexpr (PRO == PRO_NORM) {
                // ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076): float
                // squares summed in double; per-thread units, a DPP wave tree,
                // then the NW wave sums in order (RMSNorm order)
                double acc = 0.0;
#pragma unroll
                for (int k = 0; k < UM; ++k) {
                    if (k * NT + tid < nunits) {
                        const float e[8] = {xv[k][0].x, xv[k][0].y, xv[k][0].z, xv[k][0].w,
                                            xv[k][1].x, xv[k][1].y, xv[k][1].z, xv[k][1].w};
#pragma unroll
                        for (int q = 0; q < 8; ++q) { const float sq = e[q] * e[q]; acc += (double) sq; }
                    }
                }
                acc = wave_sum_d(acc);
                if (lane == 0) red[wave] = acc;
                __syncthreads();
                LVK_T(60);
                double sum = red[0];
                for (int w = 1; w < NW; ++w) sum += red[w];
                const float mean = rms_mean_wave(sum, P.x, KT);
                scale = 1.0f / sqrtf(mean + 1e-6f);
            }
#pragma unroll
            for (int k = 0; k < UM; ++k) {
                if (k * NT >= nunits) break;
                const int un = k * NT + tid;
                float v[8] = {xv[k][0].x, xv[k][0].y, xv[k][0].z, xv[k][0].w,
                              xv[k][1].x, xv[k][1].y, xv[k][1].z, xv[k][1].w};
                float amax = 0.0f;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if constexpr (PRO == PRO_NORM) {
                        const float gg[8] = {gv[k][0].x, gv[k][0].y, gv[k][0].z, gv[k][0].w,
                                             gv[k][1].x, gv[k][1].y, gv[k][1].z, gv[k][1].w};
                        const float yn = v[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                        v[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                    }
                    const float a = fabsf(v[e]);
                    amax = a > amax ? a : amax;
                }
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
#pragma unroll
            for (int k = 0; k < UM; ++k) {
                const int b = k * NT + tid;
                if (b < nb) {
                    act_store(act, dxp, b, 0, qv[k].x, dv[k], true);
                    act_store(act, dxp, b, 1, qv[k].y, 0.0f, false);
                    act_store(act, dxp, b, 2, qv[k].z, 0.0f, false);
                    act_store(act, dxp, b, 3, qv[k].w, 0.0f, false);
                }
            }
        }
    }
    if constexpr (PF == 2) {
#pragma unroll
        for (int d = 0; d < D; ++d) LVK_ISSUE(d, gc, d);
    }
    LVK_T(1);
    __syncthreads();            // activation table ready
    LVK_T(2);
    if (NP == 0 && ng == 0) return;
    if constexpr (PF == 3) {
        // 3: the table first, then every wave issues its own weights and starts its chain
        // as soon as they land (no workgroup barrier behind the issue)
#pragma unroll
        for (int d = 0; d < D; ++d) LVK_ISSUE(d, gc, d);
    } else if constexpr (SPLIT) {
#pragma unroll
        for (int d = 1; d < D; ++d) LVK_ISSUE(d, gc, d);
    }

    // 4. row groups: chunk loop with cross-group prefetch.  Per chunk: the chunk's
    // activation words and scale products are read from LDS together up front (one exposed
    // LDS latency per chunk instead of one per 4 blocks), the chains run, the slot is
    // refilled, and the scale products of the NEXT chunk are written to the other table
    // buffer (s = dw * dx, ggml.c:1968), so no write -> read round trip precedes a chain.
    float * sw = sbuf + wave * 2 * SPL;
    int tbuf = 0;
    auto make_table = [&](int buf, const float4 & Sv, int cc) __attribute__((always_inline)) {
        const float4 dx = *(const float4 *) (dxp + cc * 32 + j * 4);
        float4 sv;
        sv.x = Sv.x * dx.x; sv.y = Sv.y * dx.y; sv.z = Sv.z * dx.z; sv.w = Sv.w * dx.w;
        *(float4 *) (sw + buf * SPL + r * SRS + j * 4) = sv;
    };
#ifndef LVK_PROBE_EXP
#define LVK_PROBE_EXP 0
#endif
    // dev probe builds only (tools/probe mv_probe_xN): cost of the chain's parts.  1: four
    // independent accumulators per lane instead of one serial chain; 2: no int -> float
    // conversion (bit cast); 4: the scale products taken from registers, not the LDS table.
    // None of these is bit-exact; the product build has LVK_PROBE_EXP = 0.
    constexpr bool X_IND = (LVK_PROBE_EXP & 1) != 0, X_NOCVT = (LVK_PROBE_EXP & 2) != 0;
    constexpr bool X_NOSA = (LVK_PROBE_EXP & 4) != 0;
    auto body = [&](auto has_next, int grp, int gnext) __attribute__((always_inline)) {
        float acc = 0.0f, acc1 = 0.0f, acc2 = 0.0f, acc3 = 0.0f;
        auto cv = [](int p) __attribute__((always_inline)) { return X_NOCVT ? __int_as_float(p) : (float) p; };
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int slot = c % D;
            LVK_T(tq); ++tq;
            constexpr int NQ = 8;                   // 4-block activation groups per chunk
#ifdef LVK_PROBE_NOCOMPUTE   // dev probe builds only: consume the weights trivially
            acc += __uint_as_float(W[slot][0].x ^ W[slot][nsub > 1 ? 1 : 0].y) * S[slot].x;
            if (false) {
#else
            {
#endif
            const float * sl = sw + tbuf * SPL;
            uint4 A[NQ];
#pragma unroll
            for (int q = 0; q < NQ; ++q)
                if (c * 4 + q / 2 < nsub) A[q] = *(const uint4 *) (act + ((c * 8 + q) * 8 + j) * 4);
            float sa[8][4];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float4 v = X_NOSA ? S[slot] : *(const float4 *) (sl + r * SRS + jj * 4);
                sa[jj][0] = v.x; sa[jj][1] = v.y; sa[jj][2] = v.z; sa[jj][3] = v.w;
            }
#pragma unroll
            for (int sb = 0; sb < 4; ++sb) {
                if (c * 4 + sb < nsub) {
                    const uint32_t wd[4] = {W[slot][sb].x, W[slot][sb].y, W[slot][sb].z, W[slot][sb].w};
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        const int bi = sb * 8 + pp * 4;
                        const uint4 a = A[sb * 2 + pp];
                        const int p0 = dot8(wd[2 * pp], a.x);
                        const int p1 = dot8(wd[2 * pp], a.y);
                        const int p2 = dot8(wd[2 * pp + 1], a.z);
                        const int p3 = dot8(wd[2 * pp + 1], a.w);
                        acc = __builtin_fmaf(sa[(bi + 0) & 7][(bi + 0) >> 3], cv(p0), acc);
                        float & a1 = X_IND ? acc1 : acc;
                        a1 = __builtin_fmaf(sa[(bi + 1) & 7][(bi + 1) >> 3], cv(p1), a1);
                        float & a2 = X_IND ? acc2 : acc;
                        a2 = __builtin_fmaf(sa[(bi + 2) & 7][(bi + 2) >> 3], cv(p2), a2);
                        float & a3 = X_IND ? acc3 : acc;
                        a3 = __builtin_fmaf(sa[(bi + 3) & 7][(bi + 3) >> 3], cv(p3), a3);
                    }
                }
            }
            }
            if (c + D < NC) LVK_ISSUE(slot, grp, c + D);
            else if constexpr (decltype(has_next)::value && XG) LVK_ISSUE(slot, gnext, c + D - NC);
            // the next chunk's scale table: chunk c+1 of this group, or chunk 0 of the next
            // (its scales sit in slot (c+1) % D either way)
            if (c + 1 < NC) make_table(tbuf ^ 1, S[(c + 1) % D], c + 1);
            else if constexpr (decltype(has_next)::value) make_table(tbuf ^ 1, S[(c + 1) % D], 0);
            __builtin_amdgcn_wave_barrier();
            tbuf ^= 1;
            // keep chunks in program order: the chain value is pinned here, so
            // chunk c's arithmetic cannot sink below chunk c+1's reads
            asm volatile("" : "+v"(acc));
            if constexpr (X_IND) asm volatile("" : "+v"(acc1), "+v"(acc2), "+v"(acc3));
            LVK_T(tq); ++tq;
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (X_IND) acc = (acc + acc1) + (acc2 + acc3);
        return octet_reduce(acc);
    };

    // the epilogue's memory operand of a row group -- the lane's RoPE pair, or the residual term --
    // issued before the group's chunk loop: loaded in the epilogue it was a full memory round
    // trip in every wave's tail (QKV 7.60 -> 7.45, Wo 4.41 -> 4.25, W2 7.33 -> 7.26 us;
    // profiles/r06/decode_ab/epilogue_summary.txt)
    struct EpiPre { float2 cs; float rv; };
    auto pre_epi = [&](int grp) __attribute__((always_inline)) {
        EpiPre e{make_float2(0.0f, 0.0f), 0.0f};
        if constexpr (EPI == EPI_QKV) {
            const int row = grp * 8 + r;
            const int i0 = (row - (row / P.n_embd) * P.n_embd) % P.head_dim;   // V rows: an unused pair
            e.cs = P.rope[(size_t) pos0 * (P.head_dim / 2) + (i0 >> 1)];
        } else if constexpr (EPI == EPI_RESID) {
            e.rv = P.y[grp * 8 + r];
        }
        return e;
    };
    auto epilogue = [&](int grp, float res, const EpiPre & pe) __attribute__((always_inline)) {
        const int row = grp * 8 + r;
        if constexpr (EPI == EPI_STORE) {
            if (j == 0) P.y[row] = res;
        } else if constexpr (EPI == EPI_RESID) {
            // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
            if (j == 0) P.y[row] = res + pe.rv;
        } else if constexpr (EPI == EPI_QKV) {
            qkv_epilogue_cs(res, row, j, P.n_embd, P.head_dim, pos0, pe.cs, P.q16, P.kc, P.vc, P.n_ctx, P.kv32);
        } else if constexpr (EPI == EPI_SWIGLU_F32) {
            // fused W1|W3 image interleaved per 4 rows: rows 0-3 of the group are
            // w1 rows 4grp..4grp+3, rows 4-7 the w3 rows (llama.cpp:1085-1096)
            const float a3 = __shfl_xor(res, 32);
            if (r < 4 && j == 0) {
                const float sl = f16_to_f32(P.silu_tab[f32_to_f16(res)]);   // ggml_vec_silu_f32 (ggml.c:2495)
                P.u[grp * 4 + r] = sl * a3;                                  // ggml_mul (llama.cpp:1096)
            }
        }
    };

    make_table(0, S[0], 0);                 // chunk 0 of the first group
    __builtin_amdgcn_wave_barrier();
    if constexpr (XG) {
        for (int k = 0; k + 1 < ng; ++k) {
            const EpiPre pe = pre_epi(gc);
            const float res = body(std::true_type{}, gc, gc + NW);
            epilogue(gc, res, pe);
            gc += NW;
        }
    }
    const EpiPre pe = pre_epi(gc);
    const float res = body(std::false_type{}, gc, gc);
    epilogue(gc, res, pe);
    LVK_T(3);
#undef LVK_ISSUE
}

template <int NW, int NP, int D, int PRO, int EPI, int KT, int PF>
__global__ __launch_bounds__((NW + NP) * 64) void k_mv_cu(CuParams P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    mv_cu_run<NW, NP, D, PRO, EPI, KT, PF>(P, blockIdx.x, gridDim.x, smem);
}

// -- host -------------------------------------------------------------------

// prologue order (k_mv_cu PF): PFD per launch shape (measured, tools/probe sweeps); the sweep
// probe build (LVK_PROBE_SWEEP) reads LVK_MV_PF=0..5 to override it for A/B runs, the product
// library carries only the shipped order
#ifdef LVK_PROBE_SWEEP
static int mv_pf_env() {
    static const int v = [] { const char * e = getenv("LVK_MV_PF"); return e ? atoi(e) : -1; }();
    return v;
}
#endif

template <int NW, int NP, int D, int PRO, int EPI, int KT, int PFD = 2>
hipError_t go(const CuParams & P, hipStream_t s) {
    constexpr int nb = KT / 32, NC = (nb + 31) / 32;
    constexpr bool XG = (NC % D) == 0;
    const int nwg = std::min(cu_count(), P.G);
    // without cross-group prefetch every wave must own at most one group
    if (!XG && (P.G + nwg - 1) / nwg > NW) return hipErrorNotSupported;
    const size_t lds = (size_t) nb * 32 + NC * 128 + NW * 2 * SPL * 4 + NW * 8;
#ifdef LVK_PROBE_SWEEP
    const int pf = mv_pf_env() >= 0 ? mv_pf_env() : PFD;
    switch (pf) {
        case 0: LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, 0>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P); break;
        case 1: LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, 1>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P); break;
        case 2: LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, 2>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P); break;
        case 3: LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, 3>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P); break;
        case 4: LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, 4>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P); break;
        default: LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, 5>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P); break;
    }
#else
    LVK_LAUNCH((k_mv_cu<NW, NP, D, PRO, EPI, KT, PFD>), dim3(nwg), dim3((NW + NP) * 64), lds, s, P);
#endif
    return hipGetLastError();
}

}  // namespace

// CUs of the current device, cached per device id (a one-process layer split may drive
// devices of different sizes or CU-masked partitions)
int cu_count() {
    constexpr int MAXDEV = 64;
    static int n[MAXDEV] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (dev < 0 || dev >= MAXDEV) dev = 0;
    if (n[dev] == 0) {
        int v = 0;
        n[dev] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
    }
    return n[dev];
}

#ifdef LVK_PROBE_TIMING
void * lvk_probe_trace() { void * p = nullptr; (void) hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace)); return p; }
#endif
// row lengths compiled in: the LLaMA 7B/13B-free Q4_0 shapes (n_embd 4096 / 8192,
// n_ff 11008 / 22016; llama.cpp:771-779)
bool matvec_cu_supported(int K, int qtype) {
    if (qtype == Q4_1) return matvec_cu41_supported(K);
    return K == 4096 || K == 11008 || K == 8192 || K == 22016;
}

namespace {
CuParams cu_params(const MvLaunch & L) {
    CuParams P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.G = L.w.M / 8;
    P.x = L.x + (size_t) L.tok0 * L.w.K;
    P.g = L.g;
    P.xq = L.xq;
    if (P.xq.qs) { P.xq.qs += (size_t) L.tok0 * L.xq.nb; P.xq.d += (size_t) L.tok0 * L.xq.nb; }
    P.sp = L.sp;
    P.y = L.y ? L.y + (size_t) L.out_tok0 * L.w.M : nullptr;
    P.u = L.u;
    P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx; P.kv32 = L.kv32;
    P.silu_tab = L.silu_tab;
    return P;
}
}  // namespace

hipError_t launch_matvec_cu(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype == Q4_1) return launch_matvec_cu41(L, pro, epi, s);
    if (L.w.qtype != Q4_0 || L.n_tokens != 1 || L.w.M % 8) return hipErrorNotSupported;
    const CuParams P = cu_params(L);
    const int K = L.w.K;
#ifdef LVK_PROBE_SWEEP   // dev probe builds only: LVK_CFG selects a launch shape
    {
        static int cfg = getenv("LVK_CFG") ? atoi(getenv("LVK_CFG")) : 0;
#define SW4(E, PR, K_, a0, a1, a2, a3)                                                          \
        switch (cfg) { case 0: return go<a0, PR, E, K_>(P, s); case 1: return go<a1, PR, E, K_>(P, s); \
                       case 2: return go<a2, PR, E, K_>(P, s); default: return go<a3, PR, E, K_>(P, s); }
#define C3(a, b, c) a, b, c
        if (K == 4096 && epi == EPI_QKV) SW4(EPI_QKV, PRO_NORM, 4096, C3(8, 0, 2), C3(8, 0, 4), C3(12, 0, 2), C3(6, 0, 4))
        if (K == 4096 && epi == EPI_SWIGLU_F32) SW4(EPI_SWIGLU_F32, PRO_NORM, 4096, C3(12, 0, 2), C3(12, 0, 4), C3(16, 0, 2), C3(8, 0, 4))
        if (K == 4096 && epi == EPI_STORE) SW4(EPI_STORE, PRO_NORM, 4096, C3(16, 0, 2), C3(16, 0, 4), C3(12, 0, 4), C3(8, 0, 4))
        if (K == 4096 && epi == EPI_RESID) SW4(EPI_RESID, PRO_ACTQ, 4096, C3(2, 0, 2), C3(2, 0, 4), C3(4, 0, 2), C3(4, 0, 4))
        if (K == 11008) SW4(EPI_RESID, PRO_ACTF, 11008, C3(2, 6, 4), C3(2, 6, 2), C3(2, 10, 4), C3(2, 4, 4))
        if (K == 22016 && epi == EPI_RESID) SW4(EPI_RESID, PRO_ACTF, 22016, C3(4, 0, 2), C3(4, 12, 2), C3(4, 4, 2), C3(4, 8, 2))
    }
#endif
    // launch shapes (waves NW, prefetch depth D) per row length and role, measured on
    // the 7B shapes (tools/probe, LVK_PROBE_SWEEP) and scaled for 65B: enough waves that
    // every CU keeps ~60-120 KB of weights in flight
    if (K == 4096) {
        switch (epi) {
            // prologue order 5 (inputs, chunk 0, table, the rest after the barrier): QKV 7.6 vs
            // 7.7-8.4 us, Wo 4.4 vs 4.5-4.9 over orders 0-2 (profiles/r03_pf_sweep.txt)
            case EPI_QKV: if (pro == PRO_NORM) return go<8, 0, 2, PRO_NORM, EPI_QKV, 4096, 5>(P, s); break;
            case EPI_SWIGLU_F32: if (pro == PRO_NORM) return go<12, 0, 2, PRO_NORM, EPI_SWIGLU_F32, 4096, 5>(P, s); break;
            case EPI_STORE: if (pro == PRO_NORM) return go<16, 0, 2, PRO_NORM, EPI_STORE, 4096, 1>(P, s); break;
            case EPI_RESID:
                if (pro == PRO_ACTQ) return go<2, 0, 2, PRO_ACTQ, EPI_RESID, 4096, 5>(P, s);
                break;
        }
        // operator API (lvk_mul_mat_q: plain quantize of an f32 input)
        if (epi == EPI_STORE && pro == PRO_ACTF) return go<8, 0, 2, PRO_ACTF, EPI_STORE, 4096>(P, s);
    } else if (K == 8192) {
        switch (epi) {
            // prologue orders on the 65B shapes (round-3 sweep, profiles/r03_pf65.txt): 0 for
            // QKV / W1|W3 (22.4 / 38.6 vs 23.1 / 40.1 us at order 2), 5 for Wo (8.2 vs 8.4)
            case EPI_QKV: if (pro == PRO_NORM) return go<12, 0, 2, PRO_NORM, EPI_QKV, 8192, 0>(P, s); break;
            case EPI_SWIGLU_F32: if (pro == PRO_NORM) return go<12, 0, 2, PRO_NORM, EPI_SWIGLU_F32, 8192, 0>(P, s); break;
            case EPI_STORE: if (pro == PRO_NORM) return go<12, 0, 2, PRO_NORM, EPI_STORE, 8192>(P, s); break;
            case EPI_RESID: if (pro == PRO_ACTQ) return go<4, 0, 2, PRO_ACTQ, EPI_RESID, 8192, 5>(P, s); break;
        }
        if (epi == EPI_STORE && pro == PRO_ACTF) return go<8, 0, 2, PRO_ACTF, EPI_STORE, 8192>(P, s);
    } else if (K == 11008) {
        // 2 compute waves (one row group each) put the weight burst in flight at once, behind
        // the u loads of 6 prologue waves that quantize u meanwhile (tools/gpu_sweep_np.sh,
        // profiles/r03_np_sweep.txt: 7.0 us against 8.6-9.3 for 8 waves that all quantize u
        // and then issue the weights)
        if (epi == EPI_RESID && pro == PRO_ACTF) {
            // (needs at most 2 row groups per CU: a device with fewer CUs takes 8 waves that
            // all quantize u, then issue the weights)
            const hipError_t e = go<2, 6, 4, PRO_ACTF, EPI_RESID, 11008, 0>(P, s);
            if (e != hipErrorNotSupported) return e;
            return go<8, 0, 4, PRO_ACTF, EPI_RESID, 11008, 2>(P, s);
        }
        if (epi == EPI_STORE && pro == PRO_ACTF) return go<4, 0, 4, PRO_ACTF, EPI_STORE, 11008>(P, s);
        if (epi == EPI_STORE && pro == PRO_NORM) return go<4, 0, 4, PRO_NORM, EPI_STORE, 11008>(P, s);
    } else if (K == 22016) {
        // 4 compute + 8 prologue waves (the 11008 rule): 20.0 vs 22.1 us (profiles/r03_sweep65.txt)
        if (epi == EPI_RESID && pro == PRO_ACTF) return go<4, 8, 2, PRO_ACTF, EPI_RESID, 22016, 0>(P, s);
        if (epi == EPI_STORE && pro == PRO_ACTF) return go<4, 0, 2, PRO_ACTF, EPI_STORE, 22016>(P, s);
        if (epi == EPI_STORE && pro == PRO_NORM) return go<4, 0, 2, PRO_NORM, EPI_STORE, 22016>(P, s);
    }
    return hipErrorNotSupported;
}

}  // namespace lvk

LVK_RMS_ACCESSOR(lvk_probe_rms_mv)
