// decode_persistent.hip -- one launch per decode token: the whole single-token
// forward pass (llama.cpp:927-1163 at N = 1) as a persistent kernel whose weight
// stream never stops at a layer or phase boundary.
//
// Why: a decode token streams 4.13 GB of Q4_0 weights (7B) through ~160 small
// dependent matvecs.  As separate launches every one of them pays a kernel
// boundary, a cold start of its weight stream and a drain (round-1 measurement:
// Wo 4.4 us for 1.3 us of bytes), and the attention runs with the HBM idle.  Here
// the weights do not wait for the activations: they do not depend on them.
//
// Structure (one workgroup per CU, every workgroup resident):
//   * LOADER waves (NLW) walk this CU's whole weight sequence for the token --
//     layer by layer, phase by phase (QKV, Wo, W1|W3, W2, then lm_head), chunk by
//     chunk -- and DMA each 5 KiB chunk (8 rows x 32 blocks of the octet image,
//     matvec_cu.hip layout: 4 KiB nibbles + 1 KiB block scales) into an LDS ring
//     with global_load_lds (nt).  A slot is published with a FULL word once the
//     wave's own vmcnt shows it landed; it is reused after its consumer wrote
//     FREE.  The loaders never wait on an activation: across every dependency the
//     ring keeps filling, so the next phase's weights are already on chip when
//     its input arrives.
//   * CONSUMER waves (CW) run the phases: build the phase's activation table in
//     LDS (RMSNorm + quantize_row_q4_0, ggml.c:621-685 / 6024-6080), take their
//     row groups' chunks from the ring and run the reference's AVX2 chains
//     (ggml_vec_dot_q4_0, ggml.c:1950-2026: exact int4 dot, fp32 FMA chains in
//     block order, fixed horizontal order), then the fused epilogues (RoPE + KV
//     append, residual add, silu * w3).  The consumers of 4 workgroups per head
//     also run the head's attention (the k_attn_d algorithm of
//     attention_decode.hip: scores exchanged as tagged granules, fp16 softmax,
//     P.V with the AVX accumulator layout, Q4_0 quantize of the 32-dim slice).
//
// Hand-offs between workgroups inside the launch (MI355X_MICROARCH.md, valid
// hand-off forms, row 1): producers store every handed-off byte write-through
// (sc1), drain (s_waitcnt vmcnt(0)) and, behind an LDS barrier of the consumer
// waves, ONE lane adds to a counter (sharded 8 ways where every workgroup
// arrives); a consumer polls the counter(s) with sc1 loads, and every load of the
// handed-off bytes is an sc1 load.  Score granules are the R2 form.  Every wait
// is bounded: a timeout raises the context's error word and the eval fails.
// All counters and granules are zeroed by a memset node before every launch.  Every
// handed-off vector has its own buffer per layer and phase (X: 2 per layer, U, the
// attention output and this token's q|k|v: 1 per layer): no address is stored twice in
// a launch, so no XCD can hold a stale copy of a line from an earlier phase (measured:
// reusing one buffer per vector gave wrong logits from the 12th layer on).
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

#ifdef LVK_DEV_KERNELS   // parked: built only into lib/dev (make -C llama.vk_amd dev)
namespace lvk {

namespace {
using namespace mv;

typedef unsigned u32g __attribute__((address_space(1)));
typedef unsigned long long u64g __attribute__((address_space(1)));
typedef unsigned short u16g __attribute__((address_space(1)));

#ifndef LVK_SPIN_LIMIT
#define LVK_SPIN_LIMIT (1 << 22)
#endif

constexpr int HD = 128;          // head dim (llama.cpp:1026; every LLaMA size)
constexpr int CW = 8;            // consumer waves
constexpr int NLW = 2;           // loader waves
constexpr int NT = CW * 64;      // consumer threads
constexpr int SLOT = 5120;       // ring slot: one chunk = 4 x 1 KiB nibble sub-chunks + 1 KiB scales
constexpr int RLOAD = 8;         // chunks in flight per loader wave (5 DMAs each: 40 <= vmcnt 63)
constexpr int VB = 512;          // V positions staged in LDS per attention batch
constexpr int SMAX = 40;         // ring slots at most (flag arrays)
constexpr int GW = 4;            // row groups per consumer wave per phase at most (host-checked)
constexpr int LDS_BYTES = 160 * 1024;

// counter block (u32 words; zeroed before every launch): 8-way sharded counters on
// their own 128-byte lines, then one word per head on 64-byte lines
constexpr int C_X = 0, C_U = 256, C_ATT = 512, C_ABORT = 768, C_HEAD = 800;   // shard k at +32 k
constexpr int CTR_WORDS = C_HEAD + 64 * 16;

// LDS layout (bytes)
constexpr int L_FLAGS = 0;                      // [0] consumer barrier, [1] error-seen
constexpr int L_FULL = 64;                      // [SMAX]
constexpr int L_FREE = L_FULL + SMAX * 4;       // [SMAX]
constexpr int L_RED = L_FREE + SMAX * 4;        // CW doubles + CW floats
constexpr int L_XRES = L_RED + CW * 12 + 16;    // this CU's residual rows (runtime count)

__device__ __forceinline__ void raise_error(unsigned * err, unsigned code) {
    if (err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// LDS words shared by the waves of the workgroup, addressed as LDS (address space 3):
// through a generic pointer hipcc emits FLAT instructions, which count in vmcnt and
// complete out of order with the loader's LDS-DMAs -- the loaders' counted vmcnt waits
// would then publish chunks that have not landed
typedef unsigned lu32 __attribute__((address_space(3)));
__device__ __forceinline__ unsigned lds_ld(const lu32 * p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_st(lu32 * p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ unsigned lds_addr(const void * p) {
    return (unsigned) (uintptr_t) (const __attribute__((address_space(3))) uint8_t *) p;
}

// agent-scope (sc1) global accesses: the hand-off forms
__device__ __forceinline__ unsigned g_ld32(const void * p) {
    return __hip_atomic_load((const u32g *) p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long g_ld64(const void * p) {
    return __hip_atomic_load((const u64g *) p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st32(void * p, unsigned v) {
    __hip_atomic_store((u32g *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_st16(void * p, uint16_t v) {
    __hip_atomic_store((u16g *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_add(unsigned * p, unsigned v) {
    __hip_atomic_fetch_add((u32g *) p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// every wait of the launch is bounded: past the limit it raises the error word (the
// host fails the eval) and the launch-wide abort word, which makes every other wait
// of every workgroup give up at its next check -- a broken launch ends in
// milliseconds instead of waiting out each bound in turn
__device__ __forceinline__ bool give_up(int & spins, unsigned * err, unsigned * ctr, unsigned code) {
    ++spins;
    if ((spins & 255) == 0 && g_ld32(ctr + C_ABORT)) return true;
    if (spins > LVK_SPIN_LIMIT) {
        raise_error(err, code);
        g_st32(ctr + C_ABORT, 1u);
        return true;
    }
    return false;
}
__device__ __forceinline__ bool give_up(int & spins, const DecodeArgs & A, unsigned code) {
    return give_up(spins, A.err, A.ctr, code);
}

// one 1 KiB LDS-DMA: lane l's 16 bytes at gsrc land at LDS byte lds_dst + 16 l
// (cdna_hip_programming.md 5.7 recipe; invisible to hipcc's vmcnt bookkeeping, so
// the issuing wave counts completions itself)
template <bool NT_POLICY>
__device__ __forceinline__ void dma16(const void * gsrc, unsigned lds_dst) {
    unsigned keep;
    if constexpr (NT_POLICY)
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
    else
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep) : "v"(gsrc), "s"(lds_dst) : "memory");
}

#ifdef LVK_DP_TRACE   // dev trace builds only (lib/trace): per-workgroup phase stamps and stall cycles
constexpr int TR_EV = 16, TR_L = 96;
__device__ unsigned long long g_dpt[256 * (TR_L * TR_EV + 16)];
__device__ unsigned long long g_dps[256 * 16];
#define DP_EV(k)                                                                                      \
    do {                                                                                              \
        if (wave == 0 && lane == 0 && b < 256 && l < TR_L)                                            \
            g_dpt[(size_t) b * (TR_L * TR_EV + 16) + l * TR_EV + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#ifdef LVK_DP_STALL
#define DP_STALL_BEGIN const unsigned long long st0_ = __builtin_amdgcn_s_memtime()
#define DP_STALL_END stall_ += __builtin_amdgcn_s_memtime() - st0_
#define DP_STALL_STORE(w) do { if (lane == 0 && b < 256) g_dps[b * 16 + (w)] = stall_; } while (0)
#else
#define DP_STALL_BEGIN do { } while (0)
#define DP_STALL_END do { } while (0)
#define DP_STALL_STORE(w) do { } while (0)
#endif
#else
#define DP_EV(k) do { } while (0)
#define DP_STALL_BEGIN do { } while (0)
#define DP_STALL_END do { } while (0)
#define DP_STALL_STORE(w) do { } while (0)
#endif

// activation table of a phase: the nibble words in matvec_common.h's layout, the block
// scales dx of block 32 c + 8 m + jj at [c][m][jj] (8 contiguous floats per sub-chunk)
__device__ __forceinline__ void act_put(uint32_t * act, float * dxp, int i, int q, uint32_t dw_ref, float d,
                                        bool write_d) {
    act_store(act, dxp, i, q, dw_ref, 0.0f, false);
    if (write_d) dxp[i] = d;
}

#ifdef LVK_DP_VERIFY
__device__ unsigned g_dpv[16 + 64 * 16 + 32 * 8];
extern "C" __attribute__((visibility("default"))) int lvk_dp_verify(void * out) {
    void * p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_dpv)) != hipSuccess) return -1;
    return hipMemcpy(out, p, sizeof(g_dpv), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

// ---------------------------------------------------------------------------
// the CU's share of a matrix: row groups [g0, g1) of G (contiguous, +-1 group)
struct Share {
    int g0, ng;
};
__device__ __forceinline__ Share share(int G, int b, int NB) {
    const int g0 = (int) ((unsigned) b * (unsigned) G / (unsigned) NB);
    const int g1 = (int) ((unsigned) (b + 1) * (unsigned) G / (unsigned) NB);
    return {g0, g1 - g0};
}

// ---------------------------------------------------------------------------
// LOADER
struct LoaderState {
    unsigned q;          // position in the CU's chunk sequence
    unsigned pend0;      // oldest issued-but-unpublished chunk of this wave
    int npend;
};

template <int KE, int KF>
struct Loader {
    const DecodeArgs & A;
    lu32 * FULL;
    lu32 * FREE;
    unsigned ring;       // LDS byte address of slot 0
    int S, lw, lane, b, NB;
    LoaderState st;
#ifdef LVK_DP_TRACE
    unsigned long long stall_ = 0;
#endif

    __device__ __forceinline__ void publish(unsigned qq) { lds_st(&FULL[qq % (unsigned) S], qq / (unsigned) S + 1u); }

    __device__ __forceinline__ void publish_all() {
        drain();
        for (int k = 0; k < st.npend; ++k) publish(st.pend0 + (unsigned) (k * NLW));
        st.npend = 0;
    }

    __device__ __forceinline__ void chunk(const uint4 * nib, const float4 * scl, int ncimg, int nsubc, int grp, int c) {
        if ((int) (st.q % NLW) == lw) {
            const unsigned slot = st.q % (unsigned) S, gen = st.q / (unsigned) S;
            if (lds_ld(&FREE[slot]) != gen) {
                // the ring is full at this slot: everything in flight is published first
                // (its consumers may be the ones holding the slot), then wait
                DP_STALL_BEGIN;
                publish_all();
                for (int spins = 0; lds_ld(&FREE[slot]) != gen;) {
                    if (give_up(spins, A, LVK_ERR_DECODE_SPIN)) break;
                    __builtin_amdgcn_s_sleep(1);
                }
                DP_STALL_END;
            }
#ifdef LVK_DP_VERIFY
            {
                const unsigned fv = lds_ld(&FREE[slot]);
                if (fv != gen && lane == 0) {
                    const unsigned k = atomicAdd(&g_dpv[1], 1u);
                    if (k < 32) {
                        unsigned * e = g_dpv + 16 + 64 * 16 + k * 8;
                        e[0] = b; e[1] = lw; e[2] = st.q; e[3] = slot; e[4] = gen; e[5] = fv; e[6] = S; e[7] = 0xABCD;
                    }
                }
            }
#endif
            const size_t base = (size_t) grp * ncimg + c;
            const uint4 * nb = nib + base * 256 + lane;
            const unsigned dst = __builtin_amdgcn_readfirstlane(ring + slot * SLOT);
#pragma unroll
            for (int sb = 0; sb < 4; ++sb)   // a sub-chunk past the row end re-reads sub-chunk 0 (an L2 hit)
                dma16<true>(nb + (sb < nsubc ? sb : 0) * 64, dst + sb * 1024);
            dma16<true>(scl + base * 64 + lane, dst + 4096);
            if (st.npend == 0) st.pend0 = st.q;
            ++st.npend;
            if (st.npend == RLOAD) {
                asm volatile("s_waitcnt vmcnt(%0)" :: "n"(5 * (RLOAD - 1)) : "memory");   // the oldest of RLOAD chunks landed
                publish(st.pend0);
                st.pend0 += NLW;
                --st.npend;
            }
        }
        ++st.q;
    }

    __device__ __forceinline__ void phase(const uint4 * nib, const float4 * scl, int G, int K) {
        const Share sh = share(G, b, NB);
        const int nb = K / 32, nc = (nb + 31) / 32, nsub = nb / 8;
        for (int c = 0; c < nc; ++c) {
            const int nsubc = min(4, nsub - 4 * c);
            for (int g = 0; g < sh.ng; ++g) chunk(nib, scl, nc, nsubc, sh.g0 + g, c);
        }
    }

    __device__ __forceinline__ void run() {
        st = {0u, 0u, 0};
        for (int l = 0; l < A.n_layer; ++l) {
            const DecodeLayer & ly = A.layers[l];
            phase(ly.nib[0], ly.scl[0], 3 * KE / 8, KE);
            phase(ly.nib[1], ly.scl[1], KE / 8, KE);
            phase(ly.nib[2], ly.scl[2], 2 * KF / 8, KE);
            phase(ly.nib[3], ly.scl[3], KE / 8, KF);
        }
        if (A.out_nib) phase(A.out_nib, A.out_scl, A.n_vocab / 8, KE);
        publish_all();
        DP_STALL_STORE(CW + lw);
    }
};

// ---------------------------------------------------------------------------
// CONSUMERS
enum PhaseEpi : int { P_QKV = 0, P_WO = 1, P_W13 = 2, P_W2 = 3, P_LM = 4 };

// per-layer slices of the exchange buffers start on their own 256-byte lines
constexpr int aqd_stride(int E) { return ((E / 32) * 4 + 255) / 256 * 64; }

template <int KE, int KF>
struct Consumer {
    static constexpr int AQD_STRIDE = aqd_stride(KE);
    const DecodeArgs & A;
    uint8_t * smem;
    lu32 * FULL;
    lu32 * FREE;
    const uint8_t * ring;
    int S, b, NB, tid, lane, wave;
    unsigned cgen;       // consumer barrier generation
    unsigned q;          // chunk sequence position at the current phase's start
    int pos;             // n_past
    int l;               // current layer
    bool att;            // this workgroup runs attention for (h, s)
    int h, s;
    int row0;            // first residual row owned by this CU (Wo / W2 share)
    bool failed;
#ifdef LVK_DP_TRACE
    unsigned long long stall_ = 0;
#endif

    __device__ __forceinline__ uint32_t * act() const { return (uint32_t *) (smem + A.l_act); }
    __device__ __forceinline__ float * dxp() const { return (float *) (smem + A.l_act + A.act_bytes); }
    __device__ __forceinline__ float * xres() const { return (float *) (smem + L_XRES); }
    __device__ __forceinline__ double * redd() const { return (double *) (smem + L_RED); }
    __device__ __forceinline__ float * redf() const { return (float *) (smem + L_RED + CW * 8); }

    // opaque per layer: keeps hipcc from hoisting the thread-index arithmetic of every
    // phase out of the layer loop (hundreds of VGPRs live across the whole token)
    __device__ __forceinline__ void refresh() {
        asm volatile("" : "+v"(tid), "+v"(lane));
        wave = __builtin_amdgcn_readfirstlane(wave);
    }

    // barrier of the consumer waves only (the loaders never stop): an LDS counter
    __device__ __forceinline__ void cbar() {
        ++cgen;
        lu32 * ctr = (lu32 *) (smem + L_FLAGS);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const unsigned target = cgen * (unsigned) CW;
        for (int spins = 0; lds_ld(ctr) < target;) {
            if (give_up(spins, A, LVK_ERR_DECODE_SPIN)) break;
            __builtin_amdgcn_s_sleep(0);
        }
        asm volatile("" ::: "memory");
    }

    // wave 0 polls n counter words (stride 32 words: the 8-way sharded counters, or one
    // word) until word k >= target(k); the other consumer waves wait at the barrier after
    // (shard k of n_shards expects per x the workgroups b % n_shards == k of [0, n_arr))
    __device__ __forceinline__ void wait_ge(const unsigned * p, int n, int stride, unsigned per, int n_arr) {
        if (wave == 0) {
            const bool mine = lane < n;
            const unsigned tgt = per * (unsigned) (n == 1 ? 1 : shard_count(n_arr, lane));
            for (int spins = 0;;) {
                const bool ok = !mine || g_ld32(p + lane * stride) >= tgt;
                if (__all(ok)) break;
                if (give_up(spins, A, LVK_ERR_DECODE_SPIN)) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        cbar();
    }

    // arrivals of the 8-way sharded counters: shard k counts the workgroups b % 8 == k of [0, n)
    __device__ __forceinline__ static int shard_count(int n, int k) { return n > k ? (n - k + 7) / 8 : 0; }

    // signal: every consumer wave drained its stores; then lane 0 of wave 0 adds
    __device__ __forceinline__ void arrive(unsigned * ctr_word, unsigned v) {
        drain();
        cbar();
        if (wave == 0 && lane == 0) g_add(ctr_word, v);
    }

    // ---- activation tables ------------------------------------------------
    // x (norm * g, or plain) -> quantize_row_q4_0 into act/dxp.  MODE: 0 f32 source in
    // global written by another workgroup in this launch (sc1 loads), 1 plain source
    // (written before the launch), 2 the token's embedding row (dequantized here)
    template <int K, bool NORM>
    __device__ __forceinline__ void build(const float * src, int mode, const float * g, bool keep_rows) {
        constexpr int nunits = K / 8;
        constexpr int UM = (nunits + NT - 1) / NT;
        float v[UM][8];
#pragma unroll
        for (int k = 0; k < UM; ++k) {
            const int un = min(k * NT + tid, nunits - 1);
            if (mode == 0) {
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const unsigned long long w = g_ld64(src + (size_t) un * 8 + 2 * e);
                    v[k][2 * e] = __uint_as_float((unsigned) w);
                    v[k][2 * e + 1] = __uint_as_float((unsigned) (w >> 32));
                }
            } else if (mode == 1) {
                const float4 a = ((const float4 *) src)[2 * un], c = ((const float4 *) src)[2 * un + 1];
                v[k][0] = a.x; v[k][1] = a.y; v[k][2] = a.z; v[k][3] = a.w;
                v[k][4] = c.x; v[k][5] = c.y; v[k][6] = c.z; v[k][7] = c.w;
            } else {
                // get_rows + dequantize_row_q4_0 / _q4_1 (ggml.c:6868-6895, 968-1000, 1086-1115)
                const size_t tok = (size_t) A.sp->pad0;
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const int el = un * 8 + e;
                    float x;
                    if (A.emb_type == Q4_0) {
                        const uint8_t * bk = (const uint8_t *) A.tok_emb + tok * (size_t) (K / 32) * 20 + (size_t) (el / 32) * 20;
                        const float d = *(const float *) bk;
                        const uint8_t by = bk[4 + (el % 32) / 2];
                        x = (float) (((el & 1) ? (by >> 4) : (by & 15)) - 8) * d;
                    } else if (A.emb_type == Q4_1) {
                        const uint8_t * bk = (const uint8_t *) A.tok_emb + tok * (size_t) (K / 32) * 24 + (size_t) (el / 32) * 24;
                        const float d = *(const float *) bk, m = *(const float *) (bk + 4);
                        const uint8_t by = bk[8 + (el % 32) / 2];
                        const float a = (float) ((el & 1) ? (by >> 4) : (by & 15)) * d;
                        x = a + m;
                    } else if (A.emb_type == 1) {
                        x = f16_to_f32(((const uint16_t *) A.tok_emb)[tok * K + el]);
                    } else {
                        x = ((const float *) A.tok_emb)[tok * K + el];
                    }
                    v[k][e] = x;
                }
            }
        }
        if (keep_rows) {   // layer 0 / stage input: this CU's residual rows
#pragma unroll
            for (int k = 0; k < UM; ++k) {
                const int un = k * NT + tid;
                if (un < nunits && un * 8 >= row0 && un * 8 < row0 + A.xres_rows)
#pragma unroll
                    for (int e = 0; e < 8; ++e) xres()[un * 8 + e - row0] = v[k][e];
            }
        }
        float scale = 1.0f;
        if constexpr (NORM) {
            // ggml_compute_forward_rms_norm_f32 (ggml.c:6058-6076): float squares summed in
            // double; per-thread units, DPP wave tree, the waves in order
            double acc = 0.0;
#pragma unroll
            for (int k = 0; k < UM; ++k)
                if (k * NT + tid < nunits)
#pragma unroll
                    for (int e = 0; e < 8; ++e) { const float sq = v[k][e] * v[k][e]; acc += (double) sq; }
            acc = wave_sum_d(acc);
            if (lane == 0) redd()[wave] = acc;
            cbar();
            double sum = redd()[0];
            for (int w = 1; w < CW; ++w) sum += redd()[w];
            const float mean = (float) (sum / (double) K);
            scale = 1.0f / sqrtf(mean + 1e-6f);
        }
#pragma unroll
        for (int k = 0; k < UM; ++k) {
            if (k * NT >= nunits) break;
            const int un = k * NT + tid;
            const int ug = min(un, nunits - 1);
            float gg[8];
            if constexpr (NORM) {
                const float4 a = ((const float4 *) g)[2 * ug], c = ((const float4 *) g)[2 * ug + 1];
                gg[0] = a.x; gg[1] = a.y; gg[2] = a.z; gg[3] = a.w; gg[4] = c.x; gg[5] = c.y; gg[6] = c.z; gg[7] = c.w;
            }
            float x[8];
            float amax = 0.0f;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                x[e] = v[k][e];
                if constexpr (NORM) {
                    const float yn = x[e] * scale;      // ggml_vec_scale_f32 (ggml.c:6076)
                    x[e] = gg[e] * yn;                  // ggml_mul(repeat(g), cur) (llama.cpp:984)
                }
                const float a = fabsf(x[e]);
                amax = a > amax ? a : amax;
            }
            // the 4 units of a block are a lane quad: block amax (ggml.c:636-649)
            const float o0 = quad_bcast<0>(amax), o1 = quad_bcast<1>(amax);
            const float o2 = quad_bcast<2>(amax), o3 = quad_bcast<3>(amax);
            const float m01 = o1 > o0 ? o1 : o0, m23 = o3 > o2 ? o3 : o2;
            amax = m23 > m01 ? m23 : m01;
            const float d = amax / 7.0f;                              // ggml.c:651
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;     // ggml.c:653
            const uint32_t w = q40_pack8(x, id);
            if (un < nunits) act_put(act(), dxp(), un >> 2, un & 3, w, d, (un & 3) == 0);
        }
        cbar();
    }

    // the attention output (Q4_0 blocks published by the attention workgroups)
    __device__ __forceinline__ void build_from_blocks() {
        constexpr int nb = KE / 32;
        for (int bk = tid; bk < nb; bk += NT) {
            const float d = __uint_as_float(g_ld32(A.aq_d + (size_t) l * AQD_STRIDE + bk));
            const unsigned long long q0 = g_ld64((const uint32_t *) (A.aq_qs + (size_t) l * nb + bk));
            const unsigned long long q1 = g_ld64((const uint32_t *) (A.aq_qs + (size_t) l * nb + bk) + 2);
            act_put(act(), dxp(), bk, 0, (uint32_t) q0, d, true);
            act_put(act(), dxp(), bk, 1, (uint32_t) (q0 >> 32), 0.0f, false);
            act_put(act(), dxp(), bk, 2, (uint32_t) q1, 0.0f, false);
            act_put(act(), dxp(), bk, 3, (uint32_t) (q1 >> 32), 0.0f, false);
        }
        cbar();
    }

    // ---- one matvec phase over this CU's row groups ------------------------
    template <int K, int EPI>
    __device__ __forceinline__ void rows(int G, int rot, const uint4 * P_nib = nullptr, const float4 * P_scl = nullptr) {
        constexpr int nb = K / 32, NC = (nb + 31) / 32, nsub = nb / 8;
        const Share sh = share(G, b, NB);
        // local groups of this wave: g = (wave - rot) mod CW, + CW, ... (at most GW: host-checked)
        const int gfirst = ((wave - rot) % CW + CW) % CW;
        const int ngw = min(GW, gfirst < sh.ng ? (sh.ng - gfirst + CW - 1) / CW : 0);
        const int j = lane & 7, r = lane >> 3;
        float acc[GW];
#pragma unroll
        for (int gi = 0; gi < GW; ++gi) acc[gi] = 0.0f;
        // everything the loop reads from the argument block, as register values: a scalar
        // load inside the loop shares lgkmcnt with the LDS reads and returns out of order,
        // so hipcc would wait for every LDS read at each use
        const uint32_t * const actp = act();
        const float * const dxpp = dxp();
        const uint8_t * const ringp = ring;
        unsigned * const errp = A.err;
        unsigned * const ctrp = A.ctr;
        if (ngw > 0) {
#pragma unroll 1
            for (int c = 0; c < NC; ++c) {
                const int nsubc = min(4, nsub - 4 * c);
#pragma unroll
                for (int gi = 0; gi < GW; ++gi) {
                    if (gi >= ngw) break;
                    const unsigned qq = q + (unsigned) (c * sh.ng + gfirst + gi * CW);
                    const unsigned slot = qq % (unsigned) S, gen = qq / (unsigned) S + 1u;
                    if (lds_ld(&FULL[slot]) != gen) {
                        DP_STALL_BEGIN;
                        for (int spins = 0; lds_ld(&FULL[slot]) != gen;) {
                            if (give_up(spins, errp, ctrp, LVK_ERR_DECODE_SPIN)) break;
                            __builtin_amdgcn_s_sleep(1);
                        }
                        DP_STALL_END;
                    }
                    asm volatile("" ::: "memory");
                    // every LDS read of the chunk in one round trip: the ring slot's nibble words
                    // and the row's 32 block scales, the activation's nibble words and scales
                    const uint8_t * sp = ringp + (size_t) slot * SLOT;
                    uint4 W[4], av[8];
                    float4 sv[8], dx[8];
#pragma unroll
                    for (int sb = 0; sb < 4; ++sb) W[sb] = *(const uint4 *) (sp + sb * 1024 + lane * 16);
#pragma unroll
                    for (int jj = 0; jj < 8; ++jj) sv[jj] = *(const float4 *) (sp + 4096 + (r * 8 + jj) * 16);
#pragma unroll
                    for (int k = 0; k < 8; ++k) {
                        av[k] = *(const uint4 *) (actp + ((c * 8 + k) * 8 + j) * 4);
                        dx[k] = *(const float4 *) (dxpp + c * 32 + k * 4);
                    }
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#ifdef LVK_DP_VERIFY   // debug builds: the ring slot must hold exactly the chunk's image bytes
                    {
                        const size_t base = (size_t) (sh.g0 + gfirst + gi * CW) * NC + c;
                        const uint4 * gn = P_nib + base * 256 + lane;
                        bool bad = false;
                        for (int sb = 0; sb < nsubc; ++sb) {
                            const uint4 g = gn[sb * 64];
                            bad |= g.x != W[sb].x || g.y != W[sb].y || g.z != W[sb].z || g.w != W[sb].w;
                        }
                        const float4 gs = P_scl[base * 64 + lane];
                        const float4 ls = *(const float4 *) (sp + 4096 + lane * 16);
                        bad |= gs.x != ls.x || gs.y != ls.y || gs.z != ls.z || gs.w != ls.w;
                        if (__any(bad) && lane == 0) {
                            raise_error(A.err, 3u);
                            const unsigned k = atomicAdd(&g_dpv[0], 1u);
                            if (k < 64) {
                                unsigned * e = g_dpv + 16 + k * 16;
                                e[0] = b; e[1] = l; e[2] = EPI; e[3] = c; e[4] = gi; e[5] = slot; e[6] = gen;
                                e[7] = qq; e[8] = S; e[9] = wave; e[10] = (unsigned) (sh.g0 + gfirst + gi * CW);
                                e[11] = nsubc; e[12] = lds_ld(&FULL[slot]); e[13] = lds_ld(&FREE[slot]);
                                // which sub-chunks / scales differ
                                unsigned m = 0;
                                for (int sb = 0; sb < nsubc; ++sb) {
                                    const uint4 g = gn[sb * 64];
                                    if (g.x != W[sb].x || g.y != W[sb].y || g.z != W[sb].z || g.w != W[sb].w) m |= 1u << sb;
                                }
                                if (gs.x != ls.x || gs.y != ls.y || gs.z != ls.z || gs.w != ls.w) m |= 16u;
                                e[14] = m;
                                e[15] = (unsigned) (size_t) ringp;
                            }
                        }
                    }
#endif
                    if (lane == 0) lds_st(&FREE[slot], gen);     // the slot's bytes are in registers
                    float a_ = acc[gi];
#pragma unroll
                    for (int sb = 0; sb < 4; ++sb) {
                        if (sb < nsubc) {
                            // d0 * d1 of block 8 sb + jj (ggml.c:1968): sv[jj] holds d of blocks
                            // 8 m + jj (m = 0..3) of row r, dx[2 sb + jj / 4] the activation's
                            const float dxa[8] = {dx[2 * sb].x, dx[2 * sb].y, dx[2 * sb].z, dx[2 * sb].w,
                                                  dx[2 * sb + 1].x, dx[2 * sb + 1].y, dx[2 * sb + 1].z, dx[2 * sb + 1].w};
                            float svm[8];
#pragma unroll
                            for (int jj = 0; jj < 8; ++jj)
                                svm[jj] = sb == 0 ? sv[jj].x : sb == 1 ? sv[jj].y : sb == 2 ? sv[jj].z : sv[jj].w;
                            const uint32_t wd[4] = {W[sb].x, W[sb].y, W[sb].z, W[sb].w};
#pragma unroll
                            for (int pp = 0; pp < 2; ++pp) {
                                const uint4 a = av[sb * 2 + pp];
                                const int p0 = dot8(wd[2 * pp], a.x);
                                const int p1 = dot8(wd[2 * pp], a.y);
                                const int p2 = dot8(wd[2 * pp + 1], a.z);
                                const int p3 = dot8(wd[2 * pp + 1], a.w);
                                const int t = pp * 4;
                                a_ = __builtin_fmaf(svm[t] * dxa[t], (float) p0, a_);
                                a_ = __builtin_fmaf(svm[t + 1] * dxa[t + 1], (float) p1, a_);
                                a_ = __builtin_fmaf(svm[t + 2] * dxa[t + 2], (float) p2, a_);
                                a_ = __builtin_fmaf(svm[t + 3] * dxa[t + 3], (float) p3, a_);
                            }
                        }
                        asm volatile("" : "+v"(a_));
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    acc[gi] = a_;
                }
            }
#pragma unroll
            for (int gi = 0; gi < GW; ++gi) {
                if (gi >= ngw) break;
                const float res = octet_reduce(acc[gi]);
                epilogue<EPI>(sh.g0 + gfirst + gi * CW, res, r, j);
            }
        }
        q += (unsigned) (NC * sh.ng);
    }

    template <int EPI>
    __device__ __forceinline__ void epilogue(int grp, float res, int r, int j) {
        const int row = grp * 8 + r;
        if constexpr (EPI == P_QKV) {
            const int E = KE;
            const int which = row / E;              // 0 q, 1 k, 2 v (uniform per wave: E % 8 == 0)
            const int e = row - which * E;
            const float other = __shfl_xor(res, 8); // row e ^ 1 lives in the lanes of row r ^ 1
            if (j == 0) {
                const DecodeLayer & ly = A.layers[l];
                uint16_t hv;
                if (which < 2) {
                    // ggml_compute_forward_rope_f32 mode 0 (ggml.c:7209-7223)
                    const int i0 = e % HD;
                    const float2 cs = A.rope[(size_t) pos * (HD / 2) + (i0 >> 1)];
                    float out;
                    if ((i0 & 1) == 0) { const float a = res * cs.x, bb = other * cs.y; out = a - bb; }
                    else               { const float a = other * cs.y, bb = res * cs.x; out = a + bb; }
                    hv = f32_to_f16(out);
                    if (which == 1) ly.kc[(size_t) pos * E + e] = hv;     // KV append (llama.cpp:996-1008)
                } else {
                    hv = f32_to_f16(res);
                    ly.vc[(size_t) e * A.n_ctx + pos] = hv;
                }
                g_st16(A.cur + (size_t) l * 3 * E + which * E + e, hv);   // this token's q | k | v for the attention
            }
        } else if constexpr (EPI == P_WO || EPI == P_W2) {
            if (j == 0) {
                float * xr = xres() + (row - row0);
                const float xn = res + *xr;          // ggml_add(cur, inpSA) (llama.cpp:1071,1103)
                *xr = xn;
                g_st32(A.X + (size_t) (2 * l + (EPI == P_W2 ? 1 : 0)) * KE + row, __float_as_uint(xn));
                if (EPI == P_W2 && A.xout && l == A.n_layer - 1) A.xout[row] = xn;
            }
        } else if constexpr (EPI == P_W13) {
            // fused W1|W3 image interleaved per 4 rows: rows 0-3 w1, rows 4-7 w3 (llama.cpp:1085-1096)
            const float a3 = __shfl_xor(res, 32);
            if (r < 4 && j == 0) {
                const float sl = f16_to_f32(A.silu_tab[f32_to_f16(res)]);   // ggml_vec_silu_f32 (ggml.c:2495)
                g_st32(A.U + (size_t) l * KF + grp * 4 + r, __float_as_uint(sl * a3));          // ggml_mul (llama.cpp:1096)
            }
        } else {
            if (j == 0) A.logits[row] = res;
        }
    }

    // ---- attention of head h, dims 32 s .. 32 s + 31 (attention_decode.hip k_attn_d) ----
    __device__ __forceinline__ void v_dma(uint16_t * vl, const uint16_t * vc, int d0, int p0, int lim) {
        for (int row = wave; row < 32; row += CW)
            if (p0 + lane * 8 < lim)
                dma16<false>(vc + (size_t) (d0 + row) * A.n_ctx + p0 + lane * 8,
                             __builtin_amdgcn_readfirstlane(lds_addr(vl + (size_t) row * VB)));
    }

    __device__ __forceinline__ void attention() {
        const int E = KE, n_ctx = A.n_ctx;
        const int n_kv = pos + 1, n_pad = (n_kv + 31) & ~31, np = n_kv & ~31;
        const int d0 = h * HD + s * 32;
        const int r = tid & 3;
        const DecodeLayer & ly = A.layers[l];
        uint8_t * at = smem + A.l_att;
        uint16_t * vl = (uint16_t *) at;                          // [32][VB]
        float * sc = (float *) (at + 32 * VB * 2);                // [n_ctx]
        uint16_t * pl = (uint16_t *) (sc + n_ctx);                // [n_ctx]
        uint16_t * kq = pl + n_ctx;                               // q [128] | k_pos [128] | v_pos [32]
        float * ob = (float *) (kq + 288);                        // [32]
        u64g * gr = (u64g *) (A.gran + (size_t) h * n_ctx);
        const unsigned epoch = (unsigned) l + 1u;

        // 1. the V rows of the slice, positions < n_pad of the first batch (written by
        //    earlier launches; position pos is patched from this token's hand-off)
        v_dma(vl, ly.vc, d0, 0, min(n_pad, VB));
        // 2. this token's q / k / v rows of head h: 3 * 128 rows from the QKV workgroups
        wait_ge(A.ctr + C_HEAD + h * 16, 1, 0, 3u * HD * (unsigned) (l + 1), 1);
        DP_EV(4);
        if (tid < 64) {
            const uint16_t * cur = A.cur + (size_t) l * 3 * E;
            ((uint32_t *) kq)[tid] = g_ld32(cur + h * HD + 2 * tid);                 // q
            ((uint32_t *) kq)[64 + tid] = g_ld32(cur + E + h * HD + 2 * tid);        // k at pos
            if (tid < 16) ((uint32_t *) kq)[128 + tid] = g_ld32(cur + 2 * E + d0 + 2 * tid);   // v at pos (slice)
        }
        cbar();
        // 3. scores of the 64-position chunks s, s + 4, ... (a lane quad per position;
        //    two chunks per pass): KQ = ggml_vec_dot_f16 (ggml.c:1781-1815) * 1/sqrt(hd)
        {
            float qf[4][8];
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const uint4 qv = *((const uint4 *) kq + st * 4 + r);
                const uint32_t w4[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    qf[st][2 * k] = f16_to_f32((uint16_t) (w4[k] & 0xFFFFu));
                    qf[st][2 * k + 1] = f16_to_f32((uint16_t) (w4[k] >> 16));
                }
            }
            const int half = tid >> 8, qd = (tid & 255) >> 2;
            for (int c0 = (s + 4 * half) * 64; c0 < n_kv; c0 += 512) {
                const int p = c0 + qd;
                const uint4 * kp = p == pos ? (const uint4 *) (kq + 128) + r
                                            : (const uint4 *) (ly.kc + (size_t) min(p, n_kv - 1) * E + h * HD) + r;
                float sacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
                for (int st = 0; st < 4; ++st) {
                    const uint4 kv = kp[st * 4];
                    const uint32_t w4[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        sacc[2 * k] = __builtin_fmaf(f16_to_f32((uint16_t) (w4[k] & 0xFFFFu)), qf[st][2 * k], sacc[2 * k]);
                        sacc[2 * k + 1] = __builtin_fmaf(f16_to_f32((uint16_t) (w4[k] >> 16)), qf[st][2 * k + 1], sacc[2 * k + 1]);
                    }
                }
                // the quad's 4 x 8 accumulators in the AVX2 F32Cx8_REDUCE order
                float S8[8];
#pragma unroll
                for (int ll = 0; ll < 8; ++ll) {
                    const float v0 = quad_bcast<0>(sacc[ll]), v1 = quad_bcast<1>(sacc[ll]);
                    const float v2 = quad_bcast<2>(sacc[ll]), v3 = quad_bcast<3>(sacc[ll]);
                    const float a = v0 + v1, bb = v2 + v3;
                    S8[ll] = a + bb;
                }
                const float t0 = S8[0] + S8[4], t1 = S8[1] + S8[5], t2 = S8[2] + S8[6], t3 = S8[3] + S8[7];
                const float kqv = (t0 + t1) + (t2 + t3);
                if (r == 0 && p < n_kv) {
                    const float v = kqv * A.scale;                    // ggml_vec_scale_f32 (llama.cpp:1026)
                    __hip_atomic_store(gr + p, ((unsigned long long) epoch << 32) | __float_as_uint(v),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        // 4. every score of the head (granules tagged with this layer's epoch)
        float mx = -INFINITY;
        for (int p = tid; p < n_kv; p += NT) {
            unsigned long long x;
            for (int spins = 0;;) {
                x = __hip_atomic_load(gr + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if ((unsigned) (x >> 32) == epoch) break;
                if (give_up(spins, A, LVK_ERR_ATTN_SPIN)) break;
                __builtin_amdgcn_s_sleep(1);
            }
            const float v = __uint_as_float((unsigned) x);
            sc[p] = v;
            mx = v > mx ? v : mx;
        }
        mx = wave_max_f(mx);
        if (lane == 0) redf()[wave] = mx;
        cbar();
        mx = redf()[0];
        for (int w = 1; w < CW; ++w) mx = redf()[w] > mx ? redf()[w] : mx;
        // softmax (ggml.c:7099-7121): the double sum of fp16 values is exact in any order
        double sum = 0.0;
        for (int p = tid; p < n_kv; p += NT) {
            const float e = f16_to_f32(exp_f16(f32_to_f16(sc[p] - mx), A.exp_tab, A.exp_mode));
            sum += (double) e;
            sc[p] = e;
        }
        sum = wave_sum_d(sum);
        if (lane == 0) redd()[wave] = sum;
        cbar();
        sum = redd()[0];
        for (int w = 1; w < CW; ++w) sum += redd()[w];
        const float scl = (float) (1.0 / sum);
        for (int p = tid; p < n_pad; p += NT) pl[p] = p < n_kv ? f32_to_f16(sc[p] * scl) : (uint16_t) 0;
        // 5. P.V, batch by batch of VB positions (quad q = dim d0 + q, waves 0-1)
        float sv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int qd = tid >> 2;
        for (int b0 = 0; b0 < n_pad; b0 += VB) {
            if (b0 > 0) v_dma(vl, ly.vc, d0, b0, min(n_pad, b0 + VB));
            drain();                // this wave's V DMA has landed
            cbar();                 // ... and every wave's; the probabilities are in LDS
            if (tid < 32 && pos >= b0 && pos < b0 + VB) vl[tid * VB + (pos - b0)] = kq[256 + tid];
            cbar();
            if (tid < 128) {
                const uint16_t * vr = vl + (size_t) qd * VB;
                const int e1 = min(np, b0 + VB);
                for (int p = b0; p < e1; p += 32) {
                    const uint4 v0 = *((const uint4 *) (vr + (p - b0)) + r), p0 = *((const uint4 *) (pl + p) + r);
                    const uint32_t a4[4] = {v0.x, v0.y, v0.z, v0.w}, b4[4] = {p0.x, p0.y, p0.z, p0.w};
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        sv[2 * k] = __builtin_fmaf(f16_to_f32((uint16_t) (a4[k] & 0xFFFFu)),
                                                   f16_to_f32((uint16_t) (b4[k] & 0xFFFFu)), sv[2 * k]);
                        sv[2 * k + 1] = __builtin_fmaf(f16_to_f32((uint16_t) (a4[k] >> 16)),
                                                       f16_to_f32((uint16_t) (b4[k] >> 16)), sv[2 * k + 1]);
                    }
                }
            }
            if (b0 + VB < n_pad) cbar();   // the next batch overwrites vl
        }
        if (tid < 128) {
            float S8[8];
#pragma unroll
            for (int ll = 0; ll < 8; ++ll) {
                const float v0 = quad_bcast<0>(sv[ll]), v1 = quad_bcast<1>(sv[ll]);
                const float v2 = quad_bcast<2>(sv[ll]), v3 = quad_bcast<3>(sv[ll]);
                const float a = v0 + v1, bb = v2 + v3;
                S8[ll] = a + bb;
            }
            const float t0 = S8[0] + S8[4], t1 = S8[1] + S8[5], t2 = S8[2] + S8[6], t3 = S8[3] + S8[7];
            float o = (t0 + t1) + (t2 + t3);
            if (np < n_kv) {      // leftovers in double, in position order (ggml.c:1806-1808)
                const int bl = ((n_pad - 1) / VB) * VB;     // the last batch (it holds [np, n_kv))
                const uint16_t * vr = vl + (size_t) qd * VB;
                double sumf = (double) o;
                for (int p = np; p < n_kv; ++p) {
                    const float prod = f16_to_f32(vr[p - bl]) * f16_to_f32(pl[p]);
                    sumf += (double) prod;
                }
                o = (float) sumf;
            }
            if (r == 0) ob[qd] = o;
        }
        cbar();
        // 6. quantize_row_q4_0 of the 32 outputs (ggml.c:621-685) -> the Wo input block
        if (tid < 32) {
            const float v = ob[tid];
            float amax = fabsf(v);
            for (int o2 = 16; o2 > 0; o2 >>= 1) { const float w = __shfl_xor(amax, o2); amax = w > amax ? w : amax; }
            const float dd = amax / 7.0f;
            const float id = (amax != 0.0f) ? 7.0f / amax : 0.0f;
            const uint32_t qq = (uint32_t) ((int) __builtin_rintf(v * id) + 8) & 15u;
            uint32_t part = qq << (4 * (tid & 7));
            part |= __shfl_xor(part, 1);
            part |= __shfl_xor(part, 2);
            part |= __shfl_xor(part, 4);
            const int blk = d0 / 32;
            if ((tid & 7) == 0) g_st32((uint32_t *) (A.aq_qs + (size_t) l * (E / 32) + blk) + (tid >> 3), part);
            if (tid == 0) g_st32(A.aq_d + (size_t) l * AQD_STRIDE + blk, __float_as_uint(dd));
        }
        arrive(A.ctr + C_ATT + (b & 7) * 32, 1u);
    }

    __device__ __forceinline__ void run() {
        cgen = 0;
        q = 0;
        pos = A.sp->n_past;
        failed = false;
        const int NA = A.n_attn_wg;
        att = b < NA;
        if (A.n_head % 8 == 0) { h = (b & 7) + 8 * (b >> 5); s = (b >> 3) & 3; }
        else { h = b >> 2; s = b & 3; }
        row0 = share(KE / 8, b, NB).g0 * 8;

        // layer 0 input: the token's embedding row, or the stage input written before the launch
        for (int ll = 0; ll < A.n_layer; ++ll) {
            l = ll;
            refresh();
            DP_EV(0);
            const DecodeLayer & ly = A.layers[l];
            // ---- QKV (rms_norm * attention_norm -> quantize -> Wq|Wk|Wv -> RoPE -> KV)
            if (l == 0) build<KE, true>(A.xin, A.xin ? 1 : 2, ly.attn_norm, true);
            else {
                wait_ge(A.ctr + C_X, 8, 32, (unsigned) (2 * l), NB);
                DP_EV(1);
                build<KE, true>(A.X + (size_t) (2 * l - 1) * KE, 0, ly.attn_norm, false);
            }
            DP_EV(2);
            rows<KE, P_QKV>(3 * KE / 8, 0, ly.nib[0], ly.scl[0]);
            DP_EV(3);
            {
                // per-head row counts of this CU's share of the fused QKV rows
                drain();
                cbar();
                if (wave == 0 && lane < A.n_head) {
                    const Share sh = share(3 * KE / 8, b, NB);
                    const int r0 = sh.g0 * 8, r1 = (sh.g0 + sh.ng) * 8;
                    int n = 0;
                    for (int w = 0; w < 3; ++w) {
                        const int a0 = w * KE + lane * HD, a1 = a0 + HD;
                        const int lo = max(a0, r0), hi = min(a1, r1);
                        n += hi > lo ? hi - lo : 0;
                    }
                    if (n > 0) g_add(A.ctr + C_HEAD + lane * 16, (unsigned) n);
                }
            }
            // ---- attention (4 workgroups per head)
            if (att) attention();
            DP_EV(5);
            // ---- Wo (+ residual)
            wait_ge(A.ctr + C_ATT, 8, 32, (unsigned) (l + 1), NA);
            DP_EV(6);
            build_from_blocks();
            DP_EV(7);
            rows<KE, P_WO>(KE / 8, 3, ly.nib[1], ly.scl[1]);
            arrive(A.ctr + C_X + (b & 7) * 32, 1u);
            DP_EV(8);
            // ---- W1|W3 (rms_norm * ffn_norm -> quantize -> silu(w1 x) * w3 x)
            wait_ge(A.ctr + C_X, 8, 32, (unsigned) (2 * l + 1), NB);
            DP_EV(9);
            build<KE, true>(A.X + (size_t) (2 * l) * KE, 0, ly.ffn_norm, false);
            DP_EV(10);
            rows<KE, P_W13>(2 * KF / 8, 5, ly.nib[2], ly.scl[2]);
            arrive(A.ctr + C_U + (b & 7) * 32, 1u);
            DP_EV(11);
            // ---- W2 (quantize u -> W2 -> + residual)
            wait_ge(A.ctr + C_U, 8, 32, (unsigned) (l + 1), NB);
            DP_EV(12);
            build<KF, false>(A.U + (size_t) l * KF, 0, nullptr, false);
            DP_EV(13);
            rows<KF, P_W2>(KE / 8, 1, ly.nib[3], ly.scl[3]);
            arrive(A.ctr + C_X + (b & 7) * 32, 1u);
            DP_EV(14);
        }
        if (A.out_nib) {
            // ---- final rms_norm * norm -> lm_head (llama.cpp:1112-1135)
            wait_ge(A.ctr + C_X, 8, 32, (unsigned) (2 * A.n_layer), NB);
            build<KE, true>(A.X + (size_t) (2 * A.n_layer - 1) * KE, 0, A.out_norm, false);
            rows<KE, P_LM>(A.n_vocab / 8, 7, A.out_nib, A.out_scl);
        }
        l = A.n_layer;
        DP_EV(15);
        DP_STALL_STORE(wave);
    }

};

// the launch arguments live in device memory (written once per context): a by-value
// kernel argument that the roles hold by reference is copied to scratch by hipcc
template <int KE, int KF>
__global__ __launch_bounds__((CW + NLW) * 64) void k_decode(const DecodeArgs * __restrict__ Ap) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const DecodeArgs & A = *Ap;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int b = blockIdx.x, NB = gridDim.x;
    const bool att = b < A.n_attn_wg;
    const int ring_off = att ? A.l_ring_att : A.l_att;
    const int S = min(SMAX, (LDS_BYTES - ring_off) / SLOT);
    lu32 * FULL = (lu32 *) (smem + L_FULL);
    lu32 * FREE = (lu32 *) (smem + L_FREE);
    // LDS words start at zero (the one full barrier of the launch)
    for (int i = tid; i < L_RED / 4; i += blockDim.x) ((unsigned *) smem)[i] = 0u;
    __syncthreads();
    if (wave >= CW) {
        Loader<KE, KF> ld{A, FULL, FREE, (unsigned) __builtin_amdgcn_readfirstlane(lds_addr(smem + ring_off)), S, wave - CW,
                          lane, b, NB, {}};
        ld.run();
        return;
    }
    Consumer<KE, KF> cs{A, smem, FULL, FREE, smem + ring_off, S, b, NB, tid, lane, wave};
    cs.run();
}

template <int KE, int KF>
hipError_t go(const DecodeArgs * A_dev, int nb_cu, hipStream_t s) {
    LVK_LAUNCH((k_decode<KE, KF>), dim3(nb_cu), dim3((CW + NLW) * 64), LDS_BYTES, s, A_dev);
    return hipGetLastError();
}

}  // namespace

#ifdef LVK_DP_TRACE
extern "C" __attribute__((visibility("default"))) int lvk_dp_trace(void * stamps, void * stalls) {
    void * p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_dpt)) != hipSuccess) return -1;
    if (hipMemcpy(stamps, p, sizeof(g_dpt), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_dps)) != hipSuccess) return -1;
    if (hipMemcpy(stalls, p, sizeof(g_dps), hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return TR_L * TR_EV + 16;
}
#endif

// host-side layout (mirrors the device constants above)
bool decode_persistent_layout(DecodeArgs & A, int n_cu) {
    const int E = A.n_embd, F = A.n_ff, H = A.n_head;
    const int nb = std::max(E, F) / 32;
    const int nc = (nb + 31) / 32;
    A.xres_rows = 8 * ((E / 8 + n_cu - 1) / n_cu);
    A.act_bytes = nb * 32;
    A.l_act = (L_XRES + A.xres_rows * 4 + 15) & ~15;
    A.l_att = (A.l_act + A.act_bytes + nc * 128 + 15) & ~15;
    const int att_bytes = 32 * VB * 2 + A.n_ctx * 6 + 288 * 2 + 32 * 4;
    A.l_ring_att = (A.l_att + att_bytes + 127) & ~127;
    A.n_attn_wg = 4 * H;
    const int s_att = (LDS_BYTES - A.l_ring_att) / SLOT;
    // a loader publishes everything it has in flight before it waits for a slot, so any
    // ring is deadlock-free; a useful one holds more than the loaders keep in flight
    return s_att >= NLW * RLOAD && A.n_attn_wg <= n_cu;
}

size_t decode_persistent_scratch_bytes(int n_head, int n_ctx) {
    return (size_t) CTR_WORDS * 4 + (size_t) n_head * n_ctx * 8;
}

size_t decode_persistent_aq_d_floats(int n_embd, int n_layer) { return (size_t) aqd_stride(n_embd) * n_layer; }

bool decode_persistent_supported(int E, int F, int n_head, int n_ctx, int n_vocab, int qtype) {
    if (qtype != Q4_0 || E / n_head != HD || E % n_head || n_vocab % 8 || n_ctx % 32 || n_head > 64) return false;
    return (E == 4096 && F == 11008) || (E == 8192 && F == 22016) || (E == 256 && F == 768) || (E == 512 && F == 1536);
}

bool decode_persistent_prepare(DecodeArgs & A, void * scratch, int n_cu) {
    if (!decode_persistent_supported(A.n_embd, A.n_ff, A.n_head, A.n_ctx, A.out_nib ? A.n_vocab : 8, Q4_0)) return false;
    if (!decode_persistent_layout(A, n_cu)) return false;
    // every phase's row groups fit GW per consumer wave (each wave runs its groups side by side)
    auto gpw = [&](int G) { return ((G + n_cu - 1) / n_cu + CW - 1) / CW; };
    if (gpw(3 * A.n_embd / 8) > GW || gpw(2 * A.n_ff / 8) > GW || (A.out_nib && gpw(A.n_vocab / 8) > GW)) return false;
    A.ctr = (unsigned *) scratch;
    A.gran = (unsigned long long *) ((uint8_t *) scratch + CTR_WORDS * 4);
    A.scale = 1.0f / sqrtf((float) HD);     // llama.cpp:1028 (n_embd / n_head = 128)
    return true;
}

hipError_t launch_decode_persistent(const DecodeArgs & A, const DecodeArgs * A_dev, int n_cu, hipStream_t s) {
    hipError_t e = hipMemsetAsync(A.ctr, 0, decode_persistent_scratch_bytes(A.n_head, A.n_ctx), s);
    if (e != hipSuccess) return e;
    if (A.n_embd == 4096) return go<4096, 11008>(A_dev, n_cu, s);
    if (A.n_embd == 8192) return go<8192, 22016>(A_dev, n_cu, s);
    if (A.n_embd == 512) return go<512, 1536>(A_dev, n_cu, s);
    return go<256, 768>(A_dev, n_cu, s);
}

}  // namespace lvk
extern "C" __attribute__((visibility("default"))) int lvk_dev_kernels(void) { return 1; }
#else
extern "C" __attribute__((visibility("default"))) int lvk_dev_kernels(void) { return 0; }
namespace lvk {
// the product library does not carry the parked persistent kernel: a context never
// selects it (lvk_set_decode_persistent keeps the launch-per-phase graph)
bool decode_persistent_supported(int, int, int, int, int, int) { return false; }
size_t decode_persistent_scratch_bytes(int, int) { return 16; }
size_t decode_persistent_aq_d_floats(int, int) { return 0; }
bool decode_persistent_prepare(DecodeArgs &, void *, int) { return false; }
hipError_t launch_decode_persistent(const DecodeArgs &, const DecodeArgs *, int, hipStream_t) {
    return hipErrorNotSupported;
}
}  // namespace lvk
#endif
