// matvec_cu41.hip -- CU-balanced single-token Q4_1 matvec (the 13B Q4_1 decode path).
//
// The streaming skeleton of matvec_cu.hip (one workgroup per CU, each CU owns an equal
// share of the 8-row groups, every wave keeps D chunks of its weight stream in flight
// across group boundaries, the activation table built in LDS while the first chunks
// are already in flight) with the Q4_1 arithmetic of matvec_q41.hip:
//
//   ggml_vec_dot_q4_1 AVX2 (ggml.c:2188-2258), x = weight row, y = activation,
//   per block i in order and chain j = 0..7:
//     acc_j = fmaf(dx*dy, (float) p_j, acc_j)
//     acc_j = fmaf(j even ? dx*my : mx*dy, (float) S_j, acc_j)
//     off   = off + mx*my
//   result = hsum(acc) + off * 32
//
// on an activation quantized by quantize_row_q4_1 (ggml.c:847-920).  One chunk of
// the image is 8 rows x 32 blocks: 4 KiB of nibbles + 1 KiB of d + 1 KiB of m (24 B
// per 32 weights, the file's bytes).  Row lengths are template constants (the 13B
// shapes 5120 / 13824 and the 7B shapes 4096 / 11008), so every load is exact and
// static.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {
using namespace mv;

struct Cu41Params {
    const uint4 * nib;
    const float4 * scl;         // [G][NC][2][64]: d, then m
    const uint4 * wsum;         // [G][NC][64]: even-chain weight sums (lvk_kernels.h q41_wsum)
    int G;                      // row groups (M / 8)
    const float * x;            // PRO_NORM / PRO_ACTF: f32 input [K]
    const float * g;            // PRO_NORM: norm weight [K]
    ActQ xq;                    // PRO_ACTQ: quantized input (d, m, qs)
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

// per-wave block-product tables in LDS: 4 tables (s, dx*my, mx*dy, mx*my) of 8 rows x 32
// blocks; the row stride is padded to 40 floats so the 8 rows start on banks 0, 40, 16, 56,
// 32, 8, 48, 24 (64 banks): the per-row broadcast float4 reads and the lane stores are
// bank-conflict free (a 32-float stride put rows 0/2/4/6 on the same banks)
constexpr int SRS = 40, SPL = 8 * SRS, SWF = 4 * SPL;

// SPLIT: only chunk 0 goes out before the activation table, chunks 1..D-1 after the workgroup
// barrier (the barriers wait for the slowest wave's issue, which the memory system throttles
// to the return rate once the CU's queue is full; matvec_cu.hip prologue order 5)
// HALF: the unit of work is a 4-row half group, not an 8-row group: each CU owns an equal share
// of the 2 G halves and a wave runs two at once (lanes 0-31 and 32-63 read the two 512-byte
// halves of different groups' 1 KiB slices).  With M = 5120 (13B Wo, W2) every CU then streams
// exactly 20 rows instead of 16 or 24 (640 groups on 256 CUs).  Not for the W1|W3 epilogue,
// which pairs the w1 half of a group with its w3 half inside the wave.
template <int NW, int D, int PRO, int EPI, int KT, int SPLIT = 0, int HALF = 0>
__global__ __launch_bounds__(NW * 64) void k_mv_cu41(Cu41Params P) {
    static_assert(!(HALF && EPI == EPI_SWIGLU_F32), "W1|W3 pairs the halves of one group");
    constexpr int nb = KT / 32;                 // blocks per row
    constexpr int nsub = nb / 8;                // 8-block sub-chunks (one uint4 per lane each)
    constexpr int NC = (nb + 31) / 32;          // chunks of 32 blocks
    constexpr bool XG = (NC % D) == 0;          // prefetch may cross into the next group
    constexpr int nunits = KT / 8;              // f32 prologue work units (8 elements)
    constexpr int NT = NW * 64;
    static_assert(D <= NC, "prefetch deeper than a row");
    static_assert(nb % 8 == 0, "K must be a multiple of 256");

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t * act = (uint32_t *) smem;                          // nb * 32 B
    float * dyv = (float *) (smem + nb * 32);                    // NC * 32
    float * myv = dyv + NC * 32;                                 // NC * 32
    uint8_t * ys = (uint8_t *) (myv + NC * 32);                  // nb * 4 bytes: activation sums
    float * sbuf = (float *) (ys + nb * 16);                     // NW * SWF (after nb * 4 floats of room)
    double * red = (double *) (sbuf + NW * SWF);                 // NW

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 7;
    const int r = lane >> 3;
    const int nwg = gridDim.x;
    // this CU's work items: row groups [i0, i1) (HALF = 0) or half groups [i0, i1) run in pairs
    const unsigned NI = HALF ? 2u * (unsigned) P.G : (unsigned) P.G;
    const int i0 = (int) (blockIdx.x * NI / (unsigned) nwg);
    const int i1 = (int) ((blockIdx.x + 1) * NI / (unsigned) nwg);
    const int nitems = HALF ? (i1 - i0 + 1) / 2 : i1 - i0;
    const int ng = max(0, (nitems - wave + NW - 1) / NW);      // work items of this wave
    // the lane's half group of item k of this CU: unit (g << 1 | hh), g its group, hh the half;
    // byte offsets of its slices inside a chunk of each image: lp + hh 512 (lanes 32-63 of a
    // whole group read the second half); a wave without items reads one word (every lane)
    auto unit_of = [&](int k, bool & valid) __attribute__((always_inline)) {
        if constexpr (HALF) {
            const int raw = i0 + 2 * k + (lane >> 5);
            valid = raw < i1;
            return min(raw, i1 - 1);
        } else {
            valid = true;
            return 2 * min(i0 + k, P.G - 1) + (lane >> 5);
        }
    };
    const uint32_t lp = (uint32_t) (lane & 31) * 16u;
    int gc = wave;           // item index of the wave's current row group / half-group pair
    // the QKV epilogue's position, loaded ahead of the inputs so that the RoPE pair can be loaded at
    // an item's start (pre_epi; matvec_cu.hip has the measurements)
    [[maybe_unused]] int pos0 = 0;
    if constexpr (EPI == EPI_QKV)
        pos0 = __hip_atomic_load((const __attribute__((address_space(1))) int *) &P.sp->n_past, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);

    // activation inputs first (vmcnt retires in order)
    constexpr bool FPRO = (PRO == PRO_NORM || PRO == PRO_ACTF);
    constexpr int UM = FPRO ? (nunits + NT - 1) / NT : (nb + NT - 1) / NT;
    float4 xv[UM][2];
    float4 gv[PRO == PRO_NORM ? UM : 1][2];
    uint4 qv[FPRO ? 1 : UM];
    float dv[FPRO ? 1 : UM], mv_[FPRO ? 1 : UM];
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
            mv_[k] = P.xq.m[b];
        }
    }

    // first D chunks of this wave's first item.  Per chunk c of group g the images hold
    // nib [g][c][4 sub][1 KiB], d | m [g][c][2][1 KiB], wsum [g][c][1 KiB]; a lane's slice of
    // each 1 KiB is 16 bytes at (hh 512 + lp).  Lane bases per item: lb_n / lb_s / lb_w.
    uint4 W[D][4];
    uint4 WS[D];
    float4 SD[D], SM[D];
    size_t lb_n, lb_s, lb_w;          // the current item's lane bases
    auto lane_bases = [&](int k, size_t & bn, size_t & bs, size_t & bw) __attribute__((always_inline)) {
        bool v;
        const int u = unit_of(k, v);
        const size_t gq = (size_t) (u >> 1) * NC;
        const uint32_t o = ng > 0 ? (uint32_t) (u & 1) * 512u + lp : 0u;
        bn = gq * 4096 + o;
        bs = gq * 2048 + o;
        bw = gq * 1024 + o;
    };
    lane_bases(gc, lb_n, lb_s, lb_w);
#define LVK_ISSUE41(slot, BN, BS, BW, cc)                                                               \
    do {                                                                                                \
        _Pragma("unroll") for (int sb = 0; sb < 4; ++sb) if ((cc) * 4 + sb < nsub)                      \
            W[slot][sb] = ld_nt((const uint4 *) ((const char *) P.nib + (BN) + ((cc) * 4 + sb) * 1024)); \
        const char * sc_ = (const char *) P.scl + (BS) + (cc) * 2048;                                   \
        SD[slot] = *(const float4 *) sc_;                                                               \
        SM[slot] = *(const float4 *) (sc_ + 1024);                                                      \
        WS[slot] = ld_nt((const uint4 *) ((const char *) P.wsum + (BW) + (cc) * 1024));                 \
        __builtin_amdgcn_sched_barrier(0);                                                              \
    } while (0)
#pragma unroll
    for (int d = 0; d < (SPLIT ? 1 : D); ++d) LVK_ISSUE41(d, lb_n, lb_s, lb_w, d);

    // activation table
    if constexpr (FPRO) {
        float scale = 1.0f;
        if constexpr (PRO == PRO_NORM) {
            // ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076): float squares summed
            // in double; per-thread units, a DPP wave tree, the NW wave sums in order
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
            if constexpr (PRO == PRO_NORM) {
                const float gg[8] = {gv[k][0].x, gv[k][0].y, gv[k][0].z, gv[k][0].w,
                                     gv[k][1].x, gv[k][1].y, gv[k][1].z, gv[k][1].w};
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const float yn = v[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                    v[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                }
            }
            // the 4 units of a block are a lane quad (nunits % 4 == 0, NT % 4 == 0)
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
#pragma unroll
        for (int k = 0; k < UM; ++k) {
            const int b = k * NT + tid;
            if (b < nb) {
                const uint32_t qs[4] = {qv[k].x, qv[k].y, qv[k].z, qv[k].w};
                act41_store(act, dyv, myv, ys, b, qs, dv[k], mv_[k]);
            }
        }
    }
    __syncthreads();            // activation table ready
    if (ng == 0) return;
    if constexpr (SPLIT) {
#pragma unroll
        for (int d = 1; d < D; ++d) LVK_ISSUE41(d, lb_n, lb_s, lb_w, d);
    }

    // row groups: chunk loop with cross-group prefetch
    const bool even = (j & 1) == 0;
    const uint32_t * ys32 = (const uint32_t *) ys;
    float * sw = sbuf + wave * SWF;
    auto body = [&](auto has_next, float & off) __attribute__((always_inline)) {
        float acc = 0.0f;
        off = 0.0f;
        size_t nb_n = 0, nb_s = 0, nb_w = 0;        // the next item's lane bases (cross-item prefetch)
        if constexpr (decltype(has_next)::value) lane_bases(gc + NW, nb_n, nb_s, nb_w);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int slot = c % D;
            {
                // products of blocks 32c + 8m + j of this lane's row (ggml.c:2205-2212):
                // s = dx*dy, ce = dx*my, co = mx*dy, mm = mx*my; slot 8m + j = block 32c + 8m + j
                const float4 dy = *(const float4 *) (dyv + c * 32 + j * 4);
                const float4 my = *(const float4 *) (myv + c * 32 + j * 4);
                float * sl = sw + r * SRS + j;
                const float dxa[4] = {SD[slot].x, SD[slot].y, SD[slot].z, SD[slot].w};
                const float mxa[4] = {SM[slot].x, SM[slot].y, SM[slot].z, SM[slot].w};
                const float dya[4] = {dy.x, dy.y, dy.z, dy.w};
                const float mya[4] = {my.x, my.y, my.z, my.w};
#pragma unroll
                for (int mq = 0; mq < 4; ++mq) {
                    sl[mq * 8] = dxa[mq] * dya[mq];
                    sl[SPL + mq * 8] = dxa[mq] * mya[mq];
                    sl[2 * SPL + mq * 8] = mxa[mq] * dya[mq];
                    sl[3 * SPL + mq * 8] = mxa[mq] * mya[mq];
                }
                __builtin_amdgcn_wave_barrier();
                const float * srow = sw + r * SRS;
                const float * xrow = srow + (even ? SPL : 2 * SPL);
                const float * mrow = srow + 3 * SPL;
                // the block sums multiplying the cross scales (ggml.c:2236-2240): even chains
                // take the precomputed weight sums (blocks 0-15 of the chunk in their own word,
                // 16-31 in the odd neighbour's: DPP quad_perm [1,1,3,3]), odd chains the
                // activation sums from LDS; one byte per block, exact as floats
                const uint32_t wown[4] = {WS[slot].x, WS[slot].y, WS[slot].z, WS[slot].w};
                uint32_t wnb[4];
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    wnb[q] = (uint32_t) __builtin_amdgcn_mov_dpp((int) wown[q], 0xF5, 0xF, 0xF, false);
#ifdef LVK_PROBE_NOCOMPUTE41   // dev probe build only (make nocomp41): the weights consumed trivially
                acc += __uint_as_float((W[slot][0].x ^ W[slot][nsub > 1 ? 1 : 0].y ^ WS[slot].z) & 0x3f7fffffu) * SD[slot].x;
                off += SM[slot].y;
                if (false)
#endif
#pragma unroll
                for (int sb = 0; sb < 4; ++sb) {
                    if (c * 4 + sb < nsub) {
                        const uint32_t wd[4] = {W[slot][sb].x, W[slot][sb].y, W[slot][sb].z, W[slot][sb].w};
#pragma unroll
                        for (int pp = 0; pp < 2; ++pp) {
                            const int uu = c * 8 + sb * 2 + pp;           // group of 4 blocks
                            const int bi = sb * 8 + pp * 4;               // first block within chunk
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
                            for (int k = 0; k < 4; ++k) {
                                acc = __builtin_fmaf(sv[k], (float) p[k], acc);
                                acc = __builtin_fmaf(xs[k], S[k], acc);
                                off = off + ms[k];
                            }
                        }
                    }
                }
            }
            if (c + D < NC) LVK_ISSUE41(slot, lb_n, lb_s, lb_w, c + D);
            else if constexpr (decltype(has_next)::value && XG) LVK_ISSUE41(slot, nb_n, nb_s, nb_w, c + D - NC);
            // chunks stay in program order; the product buffer is rewritten by the next chunk
            asm volatile("" : "+v"(acc), "+v"(off));
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_sched_barrier(0);
        }
        return octet_reduce(acc);
    };

    // the epilogue's memory operand of an item (the lane's RoPE pair, or the residual term), loaded
    // before the item's chunk loop instead of in the wave's tail (as matvec_cu.hip)
    struct EpiPre { float2 cs; float rv; };
    auto pre_epi = [&](int item) __attribute__((always_inline)) {
        EpiPre e{make_float2(0.0f, 0.0f), 0.0f};
        if constexpr (EPI == EPI_QKV || EPI == EPI_RESID) {
            bool valid;
            const int u = unit_of(item, valid);
            const int row = (u >> 1) * 8 + (u & 1) * 4 + (r & 3);
            if constexpr (EPI == EPI_QKV) {
                const int i0 = (row - (row / P.n_embd) * P.n_embd) % P.head_dim;   // V rows: an unused pair
                e.cs = P.rope[(size_t) pos0 * (P.head_dim / 2) + (i0 >> 1)];
            } else {
                e.rv = P.y[row];
            }
        }
        return e;
    };
    auto epilogue = [&](int item, float h, float off, const EpiPre & pe) __attribute__((always_inline)) {
        const float res = h + off * 32.0f;        // acc_offset * QK (ggml.c:2249)
        bool valid;
        const int u = unit_of(item, valid);
        const int grp = u >> 1;
        const int row = grp * 8 + (u & 1) * 4 + (r & 3);
        if constexpr (EPI == EPI_STORE) {
            if (j == 0 && valid) P.y[row] = res;
        } else if constexpr (EPI == EPI_RESID) {
            if (j == 0 && valid) P.y[row] = res + pe.rv;         // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
        } else if constexpr (EPI == EPI_QKV) {
            // (a duplicated half, !valid, recomputed its original's rows bit for bit: its stores
            // write the same values, and the RoPE partner exchange stays convergent)
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

    if constexpr (XG) {
        for (int k = 0; k + 1 < ng; ++k) {
            float off;
            const EpiPre pe = pre_epi(gc);
            const float h = body(std::true_type{}, off);
            epilogue(gc, h, off, pe);
            gc += NW;
            lane_bases(gc, lb_n, lb_s, lb_w);
        }
    }
    float off;
    const EpiPre pe = pre_epi(gc);
    const float h = body(std::false_type{}, off);
    epilogue(gc, h, off, pe);
#undef LVK_ISSUE41
}

template <int NW, int D, int PRO, int EPI, int KT, int SPLIT = 0, int HALF = 0>
hipError_t go(const Cu41Params & P, hipStream_t s) {
    constexpr int nb = KT / 32, NC = (nb + 31) / 32;
    constexpr bool XG = (NC % D) == 0;
    const int nwg = std::min(cu_count(), P.G);
    // work items per CU (row groups, or pairs of half groups): without cross-group prefetch
    // every wave must own at most one
    const int items = HALF ? ((2 * P.G + nwg - 1) / nwg + 1) / 2 : (P.G + nwg - 1) / nwg;
    if (!XG && items > NW) return hipErrorNotSupported;
    const size_t lds = (size_t) nb * 32 + 2 * NC * 128 + (size_t) nb * 16 + NW * SWF * 4 + NW * 8;
    LVK_LAUNCH((k_mv_cu41<NW, D, PRO, EPI, KT, SPLIT, HALF>), dim3(nwg), dim3(NW * 64), lds, s, P);
    return hipGetLastError();
}

}  // namespace

bool matvec_cu41_supported(int K) { return K == 4096 || K == 5120 || K == 11008 || K == 13824; }

hipError_t launch_matvec_cu41(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype != Q4_1 || L.n_tokens != 1 || L.w.M % 8) return hipErrorNotSupported;
    Cu41Params P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.wsum = q41_wsum(L.w);
    P.G = L.w.M / 8;
    P.x = L.x ? L.x + (size_t) L.tok0 * L.w.K : nullptr;
    P.g = L.g;
    P.xq = L.xq;
    if (P.xq.qs) {
        P.xq.qs += (size_t) L.tok0 * L.xq.nb;
        P.xq.d += (size_t) L.tok0 * L.xq.nb;
        P.xq.m += (size_t) L.tok0 * L.xq.nb;
    }
    P.sp = L.sp;
    P.y = L.y ? L.y + (size_t) L.out_tok0 * L.w.M : nullptr;
    P.u = L.u;
    P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx; P.kv32 = L.kv32;
    P.silu_tab = L.silu_tab;
    const int K = L.w.K;
    // half-group work units (HALF) where they even out the rows per CU: opt-in (LVK_MV41_HALF=1).
    // Measured on 13B (profiles/r05_ab13.jsonl): 312.1 / 312.4 tok/s against 319.3 / 312.0 with
    // whole groups, Wo 7.4 vs 6.9-7.3 us, W2 19.3 vs 18.9-19.5 us -- the 20 % byte imbalance of
    // M = 5120 is not what sets these kernels' time (each wave's serial chain is)
    static const bool half_env = [] { const char * e = getenv("LVK_MV41_HALF"); return e && atoi(e) != 0; }();
    const int nwg = std::min(cu_count(), P.G);
    const bool half = half_env && P.G % nwg != 0 && (2 * P.G) % nwg == 0;
#ifdef LVK_PROBE_SWEEP   // dev probe builds only: LVK_CFG41 selects a launch shape (waves, prefetch depth)
    {
        static int cfg = getenv("LVK_CFG41") ? atoi(getenv("LVK_CFG41")) : 0;
        if (K == 5120 && epi == EPI_QKV) {
            if (cfg == 1) return go<8, 2, PRO_NORM, EPI_QKV, 5120, 1>(P, s);
            if (cfg == 2) return go<8, 1, PRO_NORM, EPI_QKV, 5120>(P, s);
            if (cfg == 3) return go<6, 5, PRO_NORM, EPI_QKV, 5120, 1>(P, s);
        }
        if (K == 5120 && epi == EPI_SWIGLU_F32) {
            if (cfg == 3) return go<6, 5, PRO_NORM, EPI_SWIGLU_F32, 5120, 1>(P, s);
        }
        if (K == 5120 && epi == EPI_RESID) {
            if (cfg == 1) return go<3, 2, PRO_ACTQ, EPI_RESID, 5120, 1>(P, s);
            if (cfg == 3) return go<3, 5, PRO_ACTQ, EPI_RESID, 5120, 1>(P, s);
        }
        if (K == 13824 && epi == EPI_RESID) {
            if (cfg == 1) return go<8, 2, PRO_ACTF, EPI_RESID, 13824, 1>(P, s);
            // deeper prefetch with 8 waves (each owns at most one row group: no cross-group prefetch)
            if (cfg == 4) return go<8, 4, PRO_ACTF, EPI_RESID, 13824, 1>(P, s);
            if (cfg == 5) return go<8, 5, PRO_ACTF, EPI_RESID, 13824, 1>(P, s);
            if (cfg == 8) return go<8, 4, PRO_ACTF, EPI_RESID, 13824, 0>(P, s);
        }
        if (K == 5120 && epi == EPI_RESID) {
            if (cfg == 9) return go<3, 4, PRO_ACTQ, EPI_RESID, 5120, 1>(P, s);
            if (cfg == 10) return go<3, 5, PRO_ACTQ, EPI_RESID, 5120, 0>(P, s);
            if (cfg == 11) return go<4, 5, PRO_ACTQ, EPI_RESID, 5120, 1>(P, s);
        }
        if (K == 5120 && epi == EPI_STORE && pro == PRO_NORM) {
            if (cfg == 3) return go<6, 5, PRO_NORM, EPI_STORE, 5120, 1>(P, s);
        }
    }
#endif
    // launch shapes per row length and role (waves NW, chunks in flight per wave D): every
    // CU keeps ~60-280 KB of weights in flight.  K = 5120 has NC = 5 chunks per row: D = 2
    // does not divide the row (every wave owns at most one 8-row group, so W1|W3 and the
    // lm_head would need 14-16 waves = 128 VGPRs, which spills); with 8 waves they prefetch
    // across groups (D = 1: 190 VGPRs, no scratch; measured on 13B: W1|W3 25.2 us vs 27.9
    // at D = 5 and 29.3 for 14 waves, lm_head 27.4 vs 30.1)
    if (K == 5120) {
        switch (epi) {
            // SPLIT (chunk 1 after the table barrier): 16.9 vs 17.5 us, W2 19.5 vs 19.8
            // (profiles/r03_sweep13_split.txt)
            case EPI_QKV:
                if (pro == PRO_NORM) {
                    if (half) return go<8, 2, PRO_NORM, EPI_QKV, 5120, 1, 1>(P, s);
                    return go<8, 2, PRO_NORM, EPI_QKV, 5120, 1>(P, s);
                }
                break;
            case EPI_SWIGLU_F32: if (pro == PRO_NORM) return go<8, 1, PRO_NORM, EPI_SWIGLU_F32, 5120>(P, s); break;
            case EPI_STORE:
                if (pro == PRO_NORM) return go<8, 1, PRO_NORM, EPI_STORE, 5120>(P, s);
                if (pro == PRO_ACTF) return go<8, 1, PRO_ACTF, EPI_STORE, 5120>(P, s);
                break;
            case EPI_RESID:
                if (pro == PRO_ACTQ) {
                    if (half) return go<3, 2, PRO_ACTQ, EPI_RESID, 5120, 0, 1>(P, s);
                    return go<3, 2, PRO_ACTQ, EPI_RESID, 5120>(P, s);
                }
                break;
        }
    } else if (K == 13824) {
        // 8 waves: the 5-6 without a row group help quantize u (r03 sweep: 19.9 vs 20.9 us;
        // D = 7 / 14 with 4 waves: 23.5 / 28.3)
        if (epi == EPI_RESID && pro == PRO_ACTF) {
            if (half) return go<8, 2, PRO_ACTF, EPI_RESID, 13824, 1, 1>(P, s);
            return go<8, 2, PRO_ACTF, EPI_RESID, 13824, 1>(P, s);
        }
        if (epi == EPI_STORE && pro == PRO_ACTF) return go<4, 2, PRO_ACTF, EPI_STORE, 13824>(P, s);
    } else if (K == 4096) {
        switch (epi) {
            case EPI_QKV: if (pro == PRO_NORM) return go<8, 2, PRO_NORM, EPI_QKV, 4096>(P, s); break;
            case EPI_SWIGLU_F32: if (pro == PRO_NORM) return go<8, 2, PRO_NORM, EPI_SWIGLU_F32, 4096>(P, s); break;
            case EPI_STORE:
                if (pro == PRO_NORM) return go<8, 2, PRO_NORM, EPI_STORE, 4096>(P, s);
                if (pro == PRO_ACTF) return go<8, 2, PRO_ACTF, EPI_STORE, 4096>(P, s);
                break;
            case EPI_RESID: if (pro == PRO_ACTQ) return go<2, 2, PRO_ACTQ, EPI_RESID, 4096>(P, s); break;
        }
    } else if (K == 11008) {
        if (epi == EPI_RESID && pro == PRO_ACTF) return go<4, 4, PRO_ACTF, EPI_RESID, 11008>(P, s);
        if (epi == EPI_STORE && pro == PRO_ACTF) return go<4, 4, PRO_ACTF, EPI_STORE, 11008>(P, s);
    }
    return hipErrorNotSupported;
}

}  // namespace lvk

LVK_RMS_ACCESSOR(lvk_probe_rms_mv41)
