// matvec_cu.hip -- single-token Q4_0 matvec for decode: one workgroup per CU,
// weights streamed into an LDS ring by loader waves (LDS-DMA), consumed by
// compute waves.
//
// Same arithmetic as matvec_q4.hip (bit-faithful ggml_vec_dot_q4_0 AVX2
// chains, ggml.c:1950-2026, on an activation quantized by quantize_row_q4_0,
// ggml.c:621-685).  Organisation:
//
//   * Decode reads every weight byte once: the kernel is bound by how fast each
//     CU pulls bytes and by how evenly bytes are spread over the CUs.  The grid
//     is one workgroup per CU; workgroup w owns row groups [w*G/n, (w+1)*G/n)
//     (a row group = 8 rows = one wavefront's work), so every CU streams the
//     same number of bytes (+-1 row group).
//   * NL loader waves issue nothing but global_load_lds_dwordx4 (1 KiB per
//     instruction): first the prologue input (x, norm weight / quantized
//     activation) into a staging area, then the CU's weight chunks (32 blocks
//     x 8 rows = 4 KiB of nibbles + 1 KiB of scales) into a ring of R slots.
//     They count their own vmcnt and publish a chunk with an LDS flag once it
//     has landed.  The stream starts at t=0 and never waits on the activation.
//   * C compute waves build the activation table from the staged input (each
//     wave sums all K squares itself: no cross-wave reduction), then walk their
//     row groups chunk by chunk out of the ring and release every slot.
//   * The ring is filled in consumption order: the C compute waves' chunk
//     streams are interleaved chunk by chunk.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

namespace lvk {

namespace {
using namespace mv;

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
    const uint16_t * silu_tab;
};

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

constexpr int SLOT = 5120;        // ring slot: 4 KiB nibbles + 1 KiB scales
constexpr int LDS_MAX = 163840;   // 160 KiB per workgroup

// one 1 KiB LDS-DMA piece: every lane moves 16 bytes from src to lds + 16*lane
// (cdna_hip_programming.md 5.7 recipe; nt: weights are streamed once)
__device__ __forceinline__ void dma16(const void * src, uint32_t lds) {
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(src), "s"(lds) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "i"(N) : "memory"); }

__device__ __forceinline__ uint32_t lds_ld(const uint32_t * p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(uint32_t * p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int PRO, int KT>
struct Stage {   // bytes of staged prologue input
    static constexpr int nb = KT / 32;
    static constexpr int bytes = PRO == PRO_NORM ? 2 * KT * 4
                               : PRO == PRO_ACTF ? KT * 4
                               : nb * 16 + ((nb * 4 + 1023) / 1024) * 1024;
    static constexpr int pieces = (bytes + 1023) / 1024;
};

template <int C, int PRO, int KT>
struct Ring {
    static constexpr int nb = KT / 32, NC = (nb + 31) / 32;
    static constexpr int fixed = Stage<PRO, KT>::pieces * 1024 + nb * 32 + NC * 128 + C * 2048 + 1024;
    static constexpr int R0 = (LDS_MAX - fixed) / SLOT;
    static constexpr int R = R0 > 64 ? 64 : R0;
    static constexpr int bytes = fixed + R * SLOT;
};

// ---------------------------------------------------------------------------
// C compute waves (0..C-1) + NL loader waves (C..C+NL-1); each loader keeps up
// to L chunks (5L DMA pieces, vmcnt <= 63) in flight.
// ---------------------------------------------------------------------------
template <int C, int NL, int L, int PRO, int EPI, int KT>
__global__ __launch_bounds__((C + NL) * 64) void k_mv_ring(CuParams P) {
    using RG = Ring<C, PRO, KT>;
    using ST = Stage<PRO, KT>;
    constexpr int nb = KT / 32;                 // blocks per row
    constexpr int nsub = nb / 8;                // 8-block sub-chunks (one uint4 per lane each)
    constexpr int NC = (nb + 31) / 32;          // chunks of 32 blocks per row group
    constexpr int R = RG::R;
    constexpr int nunits = KT / 8;              // f32 prologue work units (8 elements)
    static_assert(nb % 8 == 0, "K must be a multiple of 256");
    static_assert(5 * L <= 63, "vmcnt holds at most 63 pieces");
    static_assert(R >= NL * L + C, "ring too small");

    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t * ring = smem;                                          // R * SLOT
    uint8_t * stage = smem + R * SLOT;                              // staged input
    uint32_t * act = (uint32_t *) (stage + ST::pieces * 1024);      // nb * 32 B
    float * dxp = (float *) ((uint8_t *) act + nb * 32);            // NC * 128 B
    float * sbuf = dxp + NC * 32;                                   // C * 2 * 256 floats
    uint32_t * full = (uint32_t *) (sbuf + C * 512);                // [R] sequence of the chunk in the slot
    uint32_t * freed = full + 64;                                   // [R] sequence of the last chunk released
    uint32_t * flags = freed + 64;     // [0] staged pieces landed (waves), [1] act table (waves), [2] staging issued, [3] norm partials
    double * red = (double *) (flags + 8);                          // [C] RMSNorm partial sums

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (SGPR)
    const int nwg = gridDim.x;
    const int g0 = (int) (blockIdx.x * (unsigned) P.G / (unsigned) nwg);     // G * n_cu < 2^32
    const int g1 = (int) ((blockIdx.x + 1) * (unsigned) P.G / (unsigned) nwg);
    const int ngc = g1 - g0;                    // row groups of this CU (>= 1)
    // compute wave c owns local groups c, c+C, ...: ga groups for c < gr, ga-1 after
    const int ga = (ngc + C - 1) / C, gr = ngc - (ga - 1) * C;
    const int ra = (ga - 1) * NC;               // chunk rounds in which all C waves take part
    LVK_T(0);

    if (wave == C) {
        full[lane] = 0xFFFFFFFFu;
        freed[lane] = 0xFFFFFFFFu;
        if (lane < 8) flags[lane] = 0;
    }
    __syncthreads();

    if (wave >= C) {
        // ================= loader =================
        const int lw = wave - C;
        const uint32_t ring_lds = (uint32_t) (uintptr_t) ring;
        LVK_T(60);
        // the compute waves stage the prologue input first; hold the weight
        // stream until it has landed, so the activation's latency is that of an
        // idle fabric rather than of a full one (the ring absorbs the delay)
#ifdef LVK_PROBE_EARLY
        while (lds_ld(&flags[2]) < (uint32_t) C) __builtin_amdgcn_s_sleep(1);
#else
        while (lds_ld(&flags[0]) < (uint32_t) C) __builtin_amdgcn_s_sleep(1);
#endif
        LVK_T(61);
        // 2. weight chunks in consumption order.  Sequence q <-> (compute wave
        //    c, its chunk i): rounds i < ra have all C waves, later rounds the
        //    first gr only.
        const int Q = ra * C + NC * gr;                     // chunks of this CU
        const int my_n = (Q - lw + NL - 1) / NL;            // this loader's chunks: q = lw + NL*k
        int pub = 0;                                        // next own chunk to publish
        for (int k = 0; k < my_n; ++k) {
            const int q = lw + NL * k;
            const int slot = q % R;
            if (q >= R) {
                const uint32_t want = (uint32_t) (q - R);
                while (lds_ld(&freed[slot]) != want) __builtin_amdgcn_s_sleep(1);
            }
            int c, i;
            if (q < ra * C) { c = q % C; i = q / C; }
            else { const int t = q - ra * C; c = t % gr; i = ra + t / gr; }
            const int grp = g0 + c + C * (i / NC);
            const int ci = i % NC;
            const char * nsrc = (const char *) (P.nib + ((size_t) grp * NC + ci) * 4 * 64) + lane * 16;
            const char * ssrc = (const char *) (P.scl + ((size_t) grp * NC + ci) * 64) + lane * 16;
            const uint32_t dst = ring_lds + slot * SLOT;
            dma16(nsrc, dst);
            dma16(nsrc + 1024, dst + 1024);
            dma16(nsrc + 2048, dst + 2048);
            dma16(nsrc + 3072, dst + 3072);
            dma16(ssrc, dst + 4096);
            // publish the chunk issued L-1 chunks ago once it has landed
            if (k >= L - 1) {
                wait_vm<5 * (L - 1)>();
                if (lane == 0) lds_st(&full[(lw + NL * pub) % R], (uint32_t) (lw + NL * pub));
                if (pub == 0) LVK_T(62);
                ++pub;
            }
        }
        wait_vm<0>();
        if (lane == 0)
            for (; pub < my_n; ++pub) lds_st(&full[(lw + NL * pub) % R], (uint32_t) (lw + NL * pub));
        LVK_T(63);
        return;
    }

    // ================= compute waves =================
    const int cw = wave;
    const int j = lane & 7;
    const int r = lane >> 3;
    int tq = 4;   // trace event index (probe builds)

    // 1. stage the prologue input (x and norm weight, or the quantized
    //    activation) by LDS-DMA: these are the first requests of the CU
    {
        const uint32_t st_lds = (uint32_t) (uintptr_t) stage;
        for (int i = cw; i < ST::pieces; i += C) {
            if constexpr (PRO == PRO_NORM) {
                constexpr int half = KT * 4 / 1024;   // x pieces, then g pieces
                const char * src = i < half ? (const char *) P.x + (size_t) i * 1024
                                            : (const char *) P.g + (size_t) (i - half) * 1024;
                dma16(src + lane * 16, st_lds + i * 1024);
            } else if constexpr (PRO == PRO_ACTF) {
                // the last piece may run past x: clamp lanes to its final 16 bytes
                const int off = min(i * 1024 + lane * 16, KT * 4 - 16);
                dma16((const char *) P.x + off, st_lds + i * 1024);
            } else {
                constexpr int qsp = nb * 16 / 1024;   // qs pieces, then d pieces
                if (i < qsp) dma16((const char *) P.xq.qs + i * 1024 + lane * 16, st_lds + i * 1024);
                else {
                    const int off = min((i - qsp) * 1024 + lane * 16, nb * 4 - 16);
                    dma16((const char *) P.xq.d + off, st_lds + i * 1024);
                }
            }
        }
        if (lane == 0) __hip_atomic_fetch_add(&flags[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        wait_vm<0>();
        if (lane == 0) __hip_atomic_fetch_add(&flags[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (lds_ld(&flags[0]) < (uint32_t) C) __builtin_amdgcn_s_sleep(0);
    }
    LVK_T(1);
    {
        constexpr int CT = C * 64;
        const int ct = tid;
        if constexpr (PRO == PRO_NORM || PRO == PRO_ACTF) {
            const float * xs = (const float *) stage;
            const float * gs = xs + KT;
            float scale = 1.0f;
            if constexpr (PRO == PRO_NORM) {
                // ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076): float
                // squares summed in double; wave cw sums slice cw (lane-strided,
                // DPP tree), the C partials are added in wave order
                // (RMSNorm order)
                static_assert(KT % (256 * C) == 0, "norm slices");
                double acc = 0.0;
#pragma unroll
                for (int i = 0; i < KT / 256 / C; ++i) {
                    const float4 v = ((const float4 *) xs)[(cw * (KT / 256 / C) + i) * 64 + lane];
                    const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int q = 0; q < 4; ++q) { const float sq = e[q] * e[q]; acc += (double) sq; }
                }
                acc = wave_sum_d(acc);
                if (lane == 0) {
                    red[cw] = acc;
                    __hip_atomic_fetch_add(&flags[3], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                }
                while (lds_ld(&flags[3]) < (uint32_t) C) __builtin_amdgcn_s_sleep(0);
                double sum = red[0];
#pragma unroll
                for (int w = 1; w < C; ++w) sum += red[w];
                const float mean = (float) (sum / (double) KT);
                scale = 1.0f / sqrtf(mean + 1e-6f);
            }
            constexpr int UMC = (nunits + CT - 1) / CT;
#pragma unroll
            for (int k = 0; k < UMC; ++k) {
                if (k * CT >= nunits) break;
                const int un = min(k * CT + ct, nunits - 1);
                const float4 xa = ((const float4 *) xs)[un * 2], xb = ((const float4 *) xs)[un * 2 + 1];
                float v[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
                if constexpr (PRO == PRO_NORM) {
                    const float4 ga4 = ((const float4 *) gs)[un * 2], gb4 = ((const float4 *) gs)[un * 2 + 1];
                    const float gg[8] = {ga4.x, ga4.y, ga4.z, ga4.w, gb4.x, gb4.y, gb4.z, gb4.w};
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
                if (k * CT + ct < nunits) act_store(act, dxp, un >> 2, un & 3, w, d, (un & 3) == 0);
            }
        } else {
            const uint4 * qs = (const uint4 *) stage;
            const float * ds = (const float *) (stage + nb * 16);
            for (int b = ct; b < nb; b += CT) {
                const uint4 q4 = qs[b];
                const float d = ds[b];
                act_store(act, dxp, b, 0, q4.x, d, true);
                act_store(act, dxp, b, 1, q4.y, 0.0f, false);
                act_store(act, dxp, b, 2, q4.z, 0.0f, false);
                act_store(act, dxp, b, 3, q4.w, 0.0f, false);
            }
        }
        // count this wave in, then wait for all C (a wave's LDS ops retire in order)
        if (lane == 0) __hip_atomic_fetch_add(&flags[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        while (lds_ld(&flags[1]) < (uint32_t) C) __builtin_amdgcn_s_sleep(1);
    }
    LVK_T(2);

    // 2. this wave's row groups, chunk by chunk out of the ring
    const int myg = cw < gr ? ga : ga - 1;
    float * sl0 = sbuf + cw * 512;
    for (int gk = 0; gk < myg; ++gk) {
        const int grp = g0 + cw + C * gk;
        float acc = 0.0f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            const int i = gk * NC + c;
            const int q = i < ra ? i * C + cw : ra * C + (i - ra) * gr + cw;
            const int slot = q % R;
            while (lds_ld(&full[slot]) != (uint32_t) q) __builtin_amdgcn_s_sleep(0);
            const uint8_t * sp = ring + slot * SLOT + lane * 16;
            uint4 Wv[4];
#pragma unroll
            for (int sb = 0; sb < 4; ++sb) if (c * 4 + sb < nsub) Wv[sb] = *(const uint4 *) (sp + sb * 1024);
            const float4 Sv = *(const float4 *) (sp + 4096);
            LVK_T(tq); ++tq;
#ifdef LVK_PROBE_NOCOMPUTE   // dev probe builds only: consume the weights trivially
            acc += __uint_as_float(Wv[0].x ^ Wv[nsub > 1 ? 1 : 0].y) * Sv.x;
#else
            float * sl = sl0 + (c & 1) * 256;
            // s = dw * dx of blocks 32c + 8m + j of row r (ggml.c:1968)
            const float4 dx = *(const float4 *) (dxp + c * 32 + j * 4);
            float4 sv;
            sv.x = Sv.x * dx.x; sv.y = Sv.y * dx.y; sv.z = Sv.z * dx.z; sv.w = Sv.w * dx.w;
            *(float4 *) (sl + r * 32 + j * 4) = sv;
            __builtin_amdgcn_wave_barrier();
            float sa[8][4];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) {
                const float4 v = *(const float4 *) (sl + r * 32 + jj * 4);
                sa[jj][0] = v.x; sa[jj][1] = v.y; sa[jj][2] = v.z; sa[jj][3] = v.w;
            }
#pragma unroll
            for (int sb = 0; sb < 4; ++sb) {
                if (c * 4 + sb < nsub) {
                    const uint32_t wd[4] = {Wv[sb].x, Wv[sb].y, Wv[sb].z, Wv[sb].w};
#pragma unroll
                    for (int pp = 0; pp < 2; ++pp) {
                        const int bi = sb * 8 + pp * 4;
                        const uint4 a = *(const uint4 *) (act + ((c * 8 + sb * 2 + pp) * 8 + j) * 4);
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
#endif
            // release the slot: its bytes were consumed by the instructions above
            asm volatile("" : "+v"(acc));
            if (lane == 0) lds_st(&freed[slot], (uint32_t) q);
            LVK_T(tq); ++tq;
            __builtin_amdgcn_sched_barrier(0);
        }
        const float res = octet_reduce(acc);

        // epilogue
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
                    if (which == 0) P.q16[e] = f32_to_f16(out);
                    else            P.kc[(size_t) pos * E + e] = f32_to_f16(out);
                } else {
                    P.vc[(size_t) e * P.n_ctx + pos] = f32_to_f16(res);
                }
            }
        } else if constexpr (EPI == EPI_SWIGLU_F32) {
            // fused W1|W3 image interleaved per 4 rows: rows 0-3 of the group are
            // w1 rows 4grp..4grp+3, rows 4-7 the w3 rows (llama.cpp:1085-1096)
            const float a3 = __shfl_xor(res, 32);
            if (r < 4 && j == 0) {
                const float sl = f16_to_f32(P.silu_tab[f32_to_f16(res)]);   // ggml_vec_silu_f32 (ggml.c:2495)
                P.u[grp * 4 + r] = sl * a3;                                  // ggml_mul (llama.cpp:1096)
            }
        }
    }
    LVK_T(3);
}

// -- host -------------------------------------------------------------------

int cu_count() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return 256;
        hipDeviceProp_t p;
        if (hipGetDeviceProperties(&p, dev) != hipSuccess) return 256;
        n = p.multiProcessorCount;
    }
    return n;
}

template <int C, int NL, int L, int PRO, int EPI, int KT>
hipError_t go(const CuParams & P, hipStream_t s) {
    using RG = Ring<C, PRO, KT>;
    const int nwg = std::min(cu_count(), P.G);
    hipLaunchKernelGGL((k_mv_ring<C, NL, L, PRO, EPI, KT>), dim3(nwg), dim3((C + NL) * 64), (size_t) RG::bytes, s, P);
    return hipGetLastError();
}

}  // namespace

#ifdef LVK_PROBE_TIMING
void * lvk_probe_trace() { void * p = nullptr; (void) hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace)); return p; }
#endif

bool matvec_cu_supported(int K) { return K == 4096 || K == 11008; }

hipError_t launch_matvec_cu(const MvLaunch & L, int pro, int epi, hipStream_t s) {
    if (L.w.qtype != Q4_0 || L.n_tokens != 1 || L.w.M % 8) return hipErrorNotSupported;
    CuParams P{};
    P.nib = L.w.nib;
    P.scl = (const float4 *) L.w.scl;
    P.G = L.w.M / 8;
    P.x = L.x ? L.x + (size_t) L.tok0 * L.w.K : nullptr;
    P.g = L.g;
    P.xq = L.xq;
    if (P.xq.qs) { P.xq.qs += (size_t) L.tok0 * L.xq.nb; P.xq.d += (size_t) L.tok0 * L.xq.nb; }
    P.sp = L.sp;
    P.y = L.y ? L.y + (size_t) L.out_tok0 * L.w.M : nullptr;
    P.u = L.u;
    P.q16 = L.q16; P.kc = L.kc; P.vc = L.vc; P.rope = L.rope.cs;
    P.n_embd = L.n_embd; P.head_dim = L.head_dim; P.n_ctx = L.n_ctx;
    P.silu_tab = L.silu_tab;
    const int K = L.w.K;
#ifdef LVK_PROBE_SWEEP   // dev probe builds only: LVK_CFG selects a launch shape
    {
        static int cfg = getenv("LVK_CFG") ? atoi(getenv("LVK_CFG")) : 0;
#define SW4(E, PR, K_, a0, a1, a2, a3)                                                          \
        switch (cfg) { case 0: return go<a0, PR, E, K_>(P, s); case 1: return go<a1, PR, E, K_>(P, s); \
                       case 2: return go<a2, PR, E, K_>(P, s); default: return go<a3, PR, E, K_>(P, s); }
#define C3(a, b, c) a, b, c
        if (K == 4096 && epi == EPI_QKV) SW4(EPI_QKV, PRO_NORM, 4096, C3(8, 2, 5), C3(4, 2, 5), C3(8, 1, 10), C3(8, 2, 4))
        if (K == 4096 && epi == EPI_SWIGLU_F32) SW4(EPI_SWIGLU_F32, PRO_NORM, 4096, C3(8, 2, 5), C3(4, 2, 5), C3(8, 1, 10), C3(8, 2, 4))
        if (K == 4096 && epi == EPI_STORE) SW4(EPI_STORE, PRO_NORM, 4096, C3(8, 2, 5), C3(4, 2, 5), C3(8, 1, 10), C3(8, 2, 4))
        if (K == 4096 && epi == EPI_RESID) SW4(EPI_RESID, PRO_ACTQ, 4096, C3(2, 1, 8), C3(2, 2, 4), C3(2, 1, 4), C3(2, 2, 2))
        if (K == 11008) SW4(EPI_RESID, PRO_ACTF, 11008, C3(2, 1, 10), C3(2, 2, 6), C3(2, 2, 4), C3(2, 1, 6))
    }
#endif
    if (K == 4096) {
        switch (epi) {
            case EPI_QKV: if (pro == PRO_NORM) return go<8, 2, 5, PRO_NORM, EPI_QKV, 4096>(P, s); break;
            case EPI_SWIGLU_F32: if (pro == PRO_NORM) return go<8, 2, 5, PRO_NORM, EPI_SWIGLU_F32, 4096>(P, s); break;
            case EPI_STORE: if (pro == PRO_NORM) return go<8, 2, 5, PRO_NORM, EPI_STORE, 4096>(P, s); break;
            case EPI_RESID: if (pro == PRO_ACTQ) return go<2, 1, 8, PRO_ACTQ, EPI_RESID, 4096>(P, s); break;
        }
    } else if (K == 11008) {
        if (epi == EPI_RESID && pro == PRO_ACTF) return go<2, 2, 6, PRO_ACTF, EPI_RESID, 11008>(P, s);
    }
    return hipErrorNotSupported;
}

}  // namespace lvk
