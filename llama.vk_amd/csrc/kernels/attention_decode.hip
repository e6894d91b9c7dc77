// attention_decode.hip -- single-token (decode) attention over the f16 KV
// cache, bit-faithful to the reference graph (llama.cpp:1010-1061) like
// attention.hip, split so that the KV bytes of a layer are read by 4x as many
// CUs in ONE launch.
//
// A decode step reads 2 * n_kv * 256 B of K and V per head; one workgroup per
// head pulls ~100 KB through one CU at ~17 B/cycle.  Here 4 workgroups share a
// head:
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
//
// k_attn_wo runs the same attention and the Wo matvec + residual add
// (llama.cpp:1064-1071) in ONE launch.  The first workgroups of its grid are
// Wo workgroups laid out like matvec_cu.hip (one per CU, contiguous row
// groups, a wave per row group): each wave puts its whole first row group in
// flight at launch, then takes the attention output -- the Q4_0 blocks of the
// merged heads -- from 5 granules per block that the attention workgroups
// publish (same R2 form), builds its activation table and finishes its rows.
// That removes the launch boundary between attention and Wo and hides Wo's
// weight stream behind the attention.
//
// Every workgroup of a launch is resident at once (the host checks it), which
// the exchanges need; every spin is bounded so a violated assumption cannot
// hang the GPU.
#include "attention_decode_dev.h"

#include <algorithm>
#include <cstdlib>

namespace lvk {

namespace {

template <int QT, int EM, bool QB>
__global__ __launch_bounds__(256) void k_attn_d(AttnDArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    attn_d_run<QT, EM, true, QB>(A, blockIdx.x, blockIdx.y, smem, threadIdx.x, threadIdx.x == 0);
}

#ifdef LVK_DEV_KERNELS   // parked (measured slower than two launches): lib/dev only
// ---- k_attn_wo: the Wo workgroups (row length n_embd = 4096 compiled in) ----
namespace wo {
constexpr int KT = 4096;
constexpr int NB = KT / 32;        // blocks per row
constexpr int NC = NB / 32;        // chunks of 32 blocks (4 x uint4 + 1 float4 per lane each)
constexpr int NW = 4;              // waves per Wo workgroup
constexpr int D = NC;              // a whole row group in flight
constexpr int LDS_WAVE = NB * 32 + NC * 128 + 2 * 256 * 4;   // activation table | dx | s staging
}  // namespace wo

struct WoArgs {
    const uint4 * nib;
    const float4 * scl;
    int G;          // row groups (M / 8)
    float * y;      // residual stream: y[row] += (Wo x)[row] (llama.cpp:1071)
    int nwg;        // Wo workgroups = the first nwg of the grid
};

__device__ __forceinline__ void wo_run(const WoArgs & P, unsigned long long * ogran, unsigned * ocount,
                                       const unsigned target, const unsigned epoch, const int b, uint8_t * smem,
                                       unsigned * err) {
    using namespace wo;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int j = lane & 7, r = lane >> 3;
    const int g0 = (int) ((unsigned) b * (unsigned) P.G / (unsigned) P.nwg);
    const int g1 = (int) ((unsigned) (b + 1) * (unsigned) P.G / (unsigned) P.nwg);
    const int ng = (g1 - g0 - wave + NW - 1) / NW;       // row groups of this wave
    if (ng <= 0 || LVK_PROBE_WO_MODE == 1) return;
    int gc = g0 + wave;

    // 1. the wave's first row group in flight before anything waits (matvec_cu.hip image
    // and load form: wave-uniform base + 32-bit lane offset, nt policy)
    const uint32_t loff = (uint32_t) lane * 16u;
    uint4 W[D][4];
    float4 S[D];
#define LVK_WO_ISSUE(slot, grp, cc)                                                                      \
    do {                                                                                                 \
        const uint4 * nb_ = P.nib + ((size_t) (grp) * NC * 4 + (cc) * 4) * 64;                           \
        _Pragma("unroll") for (int sb = 0; sb < 4; ++sb)                                                 \
            W[slot][sb] = ld_nt((const uint4 *) ((const char *) (nb_ + sb * 64) + loff));                \
        S[slot] = *(const float4 *) ((const char *) (P.scl + ((size_t) (grp) * NC + (cc)) * 64) + loff); \
        __builtin_amdgcn_sched_barrier(0);                                                               \
    } while (0)
    if constexpr (LVK_PROBE_WO_MODE == 3) {
        // let the attention's own loads go first: its start is bandwidth-bound, its
        // score exchange and softmax are not
        __builtin_amdgcn_s_sleep(127);
        __builtin_amdgcn_s_sleep(127);
    }
    if constexpr (LVK_PROBE_WO_MODE != 2) {
#pragma unroll
        for (int d = 0; d < D; ++d) LVK_WO_ISSUE(d, gc, d);
    }

    // 2. the Wo input: 5 granules per block from the attention workgroups, into this
    // wave's own activation table (matvec_common.h layout)
    uint32_t * act = (uint32_t *) (smem + (size_t) wave * LDS_WAVE);
    float * dxp = (float *) (smem + (size_t) wave * LDS_WAVE + NB * 32);
    float * sw = dxp + NC * 32;
    // one lane waits for every attention workgroup's count (a single word, slow poll),
    // then the wave reads the 640 granules once; a tag that is not yet this layer's is
    // polled again (not expected after the count)
    if (lane == 0) {
        // the attention takes several microseconds: sleep through most of it before the
        // first poll, then poll sparsely (hundreds of pollers on one word cost the chip)
        if constexpr (LVK_PROBE_WO_MODE != 3) {
            __builtin_amdgcn_s_sleep(127);
            __builtin_amdgcn_s_sleep(127);
        }
        for (int spins = 0; __hip_atomic_load((u32g *) ocount, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target;
             ++spins) {
            if (spins > (LVK_SPIN_LIMIT >> 2)) { raise_error(err, LVK_ERR_ATTN_SPIN); break; }
            __builtin_amdgcn_s_sleep(LVK_PROBE_WO_MODE == 3 ? 4 : 16);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");     // no granule load above the wait
    if constexpr (LVK_PROBE_WO_MODE == 2) {
#pragma unroll
        for (int d = 0; d < D; ++d) LVK_WO_ISSUE(d, gc, d);
    }
    u64g * og = (u64g *) ogran;
    static_assert(NB * 5 == 10 * 64, "granules per lane");
    unsigned long long gv[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) gv[k] = __hip_atomic_load(og + lane + 64 * k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const int i = lane + 64 * k;
        const unsigned word = (unsigned) ((unsigned) (gv[k] >> 32) == epoch ? gv[k] : poll_granule(og + i, epoch, err));
        const int blk = i / 5, k5 = i - blk * 5;
        if (k5 == 0) dxp[(blk >> 5) * 32 + (blk & 7) * 4 + ((blk >> 3) & 3)] = __uint_as_float(word);
        else mv::act_store(act, dxp, blk, k5 - 1, word, 0.0f, false);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // other lanes of this wave read the table

    // 3. the rows: ggml_vec_dot_q4_0 AVX2 chains (ggml.c:1950-2026) as in matvec_cu.hip
    auto body = [&](auto has_next, int gnext) __attribute__((always_inline)) {
        float acc = 0.0f;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
            float * sl = sw + (c & 1) * 256;
            // s = dw * dx of blocks 32c + 8m + j of row r (ggml.c:1968)
            const float4 dx = *(const float4 *) (dxp + c * 32 + j * 4);
            float4 sv;
            sv.x = S[c].x * dx.x; sv.y = S[c].y * dx.y; sv.z = S[c].z * dx.z; sv.w = S[c].w * dx.w;
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
                const uint32_t wd[4] = {W[c][sb].x, W[c][sb].y, W[c][sb].z, W[c][sb].w};
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
            // this slot is free: the same chunk of the wave's next row group
            if constexpr (decltype(has_next)::value) LVK_WO_ISSUE(c, gnext, c);
            asm volatile("" : "+v"(acc));     // chunks in program order (matvec_cu.hip rule 4)
            __builtin_amdgcn_sched_barrier(0);
        }
        return mv::octet_reduce(acc);
    };
    for (int k = 0; k + 1 < ng; ++k) {
        const float res = body(std::true_type{}, gc + NW);
        if (j == 0) P.y[gc * 8 + r] = res + P.y[gc * 8 + r];       // ggml_add(cur, inpSA) (llama.cpp:1071)
        gc += NW;
    }
    const float res = body(std::false_type{}, gc);
    if (j == 0) P.y[gc * 8 + r] = res + P.y[gc * 8 + r];
#undef LVK_WO_ISSUE
}

__global__ __launch_bounds__(256) void k_attn_wo(AttnDArgs A, WoArgs P) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const int b = blockIdx.x;
    // attention workgroups first (dispatched first, one per CU on half the chip; the 4
    // slices of a head on one XCD as in k_attn_d's (H, 4) grid), then the Wo workgroups
    const int nattn = (int) gridDim.x - P.nwg;
    if (b < nattn) attn_d_run<Q4_0, -1, false>(A, (b & 7) + 8 * (b >> 5), (b >> 3) & 3, smem, threadIdx.x, threadIdx.x == 0);
    else wo_run(P, A.ogran, A.ocount, (unsigned) nattn * A.epoch, A.epoch, b - nattn, smem, A.err);
}
#endif

#ifdef LVK_DEV_KERNELS
int n_cus() { return cu_count(); }
#endif



}  // namespace

#ifdef LVK_PROBE_TIMING
void * lvk_probe_dtrace() { void * p = nullptr; (void) hipGetSymbolAddress(&p, HIP_SYMBOL(g_dtrace)); return p; }
#endif

bool attention_decode_supported(int n_embd, int n_head, int n_ctx) {
    return n_embd / n_head == HD && n_ctx % 64 == 0 && n_ctx <= 2048 && n_head * 4 <= 1024;
}

size_t attention_decode_scratch_bytes(int n_head, int n_ctx) {
    // score granules [H][n_ctx], then k_attn_wo's output granules [E/32][5] (room for 6)
    return (size_t) n_head * n_ctx * 8 + (size_t) n_head * (HD / 32) * 6 * 8;
}

hipError_t launch_attention_decode(const AttnLaunch & A, void * gran, unsigned epoch, hipStream_t s) {
    if (!attention_decode_supported(A.n_embd, A.n_head, A.n_ctx) || A.n_tokens != 1 || epoch == 0)
        return hipErrorNotSupported;
    if (A.out_qtype != Q4_0 && A.out_qtype != Q4_1) return hipErrorNotSupported;
    const AttnDArgs a = attn_args(A, gran, epoch);
    const size_t lds = std::max(attn_lds(A.n_ctx), A.lds_min);
    const dim3 grid(A.n_head, HD / 32);
#define LVK_ATTN_EM(QT_, QB_)                                                                 \
    switch (a.exp_mode) {                                                                     \
        case 2: LVK_LAUNCH((k_attn_d<QT_, 2, QB_>), grid, dim3(256), lds, s, a); break;       \
        case 1: LVK_LAUNCH((k_attn_d<QT_, 1, QB_>), grid, dim3(256), lds, s, a); break;       \
        default: LVK_LAUNCH((k_attn_d<QT_, 0, QB_>), grid, dim3(256), lds, s, a); break;      \
    }
    const bool qb = a.qkv_gran != nullptr;
    if (A.out_qtype == Q4_1) {
        if (qb) { LVK_ATTN_EM(Q4_1, true) } else { LVK_ATTN_EM(Q4_1, false) }
    } else {
        if (qb) { LVK_ATTN_EM(Q4_0, true) } else { LVK_ATTN_EM(Q4_0, false) }
    }
#undef LVK_ATTN_EM
    return hipGetLastError();
}

#ifdef LVK_DEV_KERNELS
bool attention_wo_supported(int n_embd, int n_head, int n_ctx, const QMatrix & w) {
    if (!attention_decode_supported(n_embd, n_head, n_ctx)) return false;
    if (n_embd != wo::KT || w.qtype != Q4_0 || w.K != wo::KT || w.M <= 0 || w.M % 8) return false;
    // every workgroup resident at once: the Wo workgroups plus 4 per head at two per CU
    const int nwg = std::min(n_cus(), w.M / 8);
    const size_t lds = std::max(attn_lds(n_ctx), (size_t) wo::NW * wo::LDS_WAVE);
    return n_head % 8 == 0 && nwg + 4 * n_head <= 2 * n_cus() && 2 * lds <= 160 * 1024;
}

hipError_t launch_attention_wo(const AttnLaunch & A, const QMatrix & w, float * y, void * gran, unsigned epoch,
                               hipStream_t s) {
    if (!attention_wo_supported(A.n_embd, A.n_head, A.n_ctx, w) || A.n_tokens != 1 || epoch == 0 ||
        A.out_qtype != Q4_0 || !y)
        return hipErrorNotSupported;
    AttnDArgs a = attn_args(A, gran, epoch);
    a.seq_epochs = 0;     // its output counter needs the per-token zeroing anyway
    a.ogran = a.gran + (size_t) A.n_head * A.n_ctx;
    a.ocount = (unsigned *) (a.ogran + (size_t) A.n_head * (HD / 32) * 5);   // inside the 6-per-block room
    const WoArgs P{w.nib, (const float4 *) w.scl, w.M / 8, y, std::min(n_cus(), w.M / 8)};
    const size_t lds = std::max(attn_lds(A.n_ctx), (size_t) wo::NW * wo::LDS_WAVE);
    LVK_LAUNCH(k_attn_wo, dim3(P.nwg + 4 * A.n_head), dim3(256), lds, s, a, P);
    return hipGetLastError();
}
#else
bool attention_wo_supported(int, int, int, const QMatrix &) { return false; }
hipError_t launch_attention_wo(const AttnLaunch &, const QMatrix &, float *, void *, unsigned, hipStream_t) {
    return hipErrorNotSupported;
}
#endif

}  // namespace lvk
