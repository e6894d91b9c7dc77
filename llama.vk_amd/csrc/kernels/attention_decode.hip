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
//      granules it needs until their tag equals this layer's epoch, bounded;
//   3. softmax (max, fp16 exp, exact double sum, ggml.c:7099-7121), P in f16,
//      P.V with the AVX accumulator layout and the double tail past
//      n_kv & ~31 (ggml.c:1806-1808); the slice is quantized to the Wo weight
//      format (quantize_row_q4_0 / _q4_1, ggml.c:621-685 / 847-920).
//
// Every workgroup of a launch is resident at once (4 H <= 1024 workgroups of
// <= 42 KB LDS), which the exchange needs; every spin is bounded so a violated
// assumption cannot hang the GPU.
#include "lvk_device.h"
#include "lvk_kernels.h"
#include "matvec_common.h"

#include <algorithm>
#include <cstdlib>

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


// a workgroup barrier for LDS hand-offs only: __syncthreads() also drains vmcnt, which
// would make every wave with V rows in flight wait for them
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

typedef unsigned long long u64g __attribute__((address_space(1)));

#ifndef LVK_SPIN_LIMIT   // probe builds may lower it to exercise the timeout path
#define LVK_SPIN_LIMIT (1 << 22)
#endif

// a spin that gave up: the error word (host-mapped, lvk_kernels.h LVK_ERR_*) tells
// the host, which fails the eval instead of returning wrong numbers
__device__ __forceinline__ void raise_error(unsigned * err, unsigned code) {
    if (err) __hip_atomic_store(err, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// relaxed agent-scope poll of one granule until it carries `epoch`; bounded so a
// violated residency assumption can never hang the GPU -- it raises the error word
__device__ __forceinline__ unsigned long long poll_granule(u64g * p, unsigned epoch, unsigned * err) {
    unsigned long long x;
    for (int spins = 0;; ++spins) {
        x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if ((unsigned) (x >> 32) == epoch) break;
        if (spins > LVK_SPIN_LIMIT) { raise_error(err, LVK_ERR_ATTN_SPIN); break; }
        __builtin_amdgcn_s_sleep(1);
    }
    return x;
}

#ifdef LVK_PROBE_TIMING   // dev probe builds only: per-wave s_memtime phase stamps
__device__ unsigned long long g_dtrace[32 * 4 * 4 * 16];
#define LVK_DT(ev)                                                                                        \
    do {                                                                                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                       \
        if ((tid & 63) == 0 && h < 32) g_dtrace[((h * 4 + sl) * 4 + (tid >> 6)) * 16 + (ev)] = t_; \
    } while (0)
#else
#define LVK_DT(ev) do { } while (0)
#endif

struct AttnDArgs {
    const uint16_t * q16;
    const uint16_t * kc;
    const uint16_t * vc;
    unsigned long long * gran;    // [H][n_ctx] score granules
    const uint16_t * exp_tab;
    const StepParams * sp;
    int E, n_ctx;
    float scale;
    unsigned epoch;
    ActQ out;
    float * out_f32;
    int exp_mode;
    unsigned * err;               // host-mapped error word (nullptr: none)
    int short_max;                // n_kv <= short_max: no score exchange (every workgroup scores all)
    int seq_epochs;               // epoch += sp->seq << 7 (granules never zeroed between tokens)
};

// The 4 workgroups of a head either split the scores and exchange them as granules, or
// (n_kv <= A.short_max, DYN) every workgroup scores all positions itself (4x the K reads,
// from the XCD's L2).  !DYN: always the exchange.  EM: the exp mode compiled in (exp_f16;
// -1 reads A.exp_mode) -- a runtime mode puts the table path's load, and its vmcnt wait,
// into the softmax loop.
template <int QT, int EM, bool DYN = true>
__device__ __forceinline__ void attn_d_run(const AttnDArgs & A, const int h, const int sl, uint8_t * smem,
                                           const int tid) {
    const int E = A.E, n_ctx = A.n_ctx, d0 = h * HD + sl * 32;
    const int lane = tid & 63, wave = tid >> 6, r = tid & 3;
    const int VS = n_ctx + 32;                                   // V row stride (halves): rows 16 banks apart
    uint16_t * vl = (uint16_t *) smem;                           // [32 dims][VS]
    float * sc = (float *) (smem + (size_t) 32 * VS * 2);        // [n_ctx]
    uint16_t * pl = (uint16_t *) (sc + n_ctx);                   // [n_ctx]
    float * red = (float *) (pl + n_ctx);                        // 8 floats
    double * redd = (double *) (red + 8);                        // 4 doubles
    auto bar = [&]() __attribute__((always_inline)) { lds_barrier(); };   // LDS hand-off barrier
    u64g * g = (u64g * ) (A.gran + (size_t) h * n_ctx);
    LVK_DT(0);
    // the step block through the scalar cache (constant address space: s_load, counted by
    // lgkmcnt): a vector load here would retire behind every Q / K / V load issued below
    // (vmcnt is in order) and hold the n_kv-dependent loads back by a full HBM latency.  Both
    // words are read here, ahead of the Q loads (the sched barriers keep the scalar loads in
    // front and their first use -- and wait -- behind the Q issue): with the granule tag
    // computed up front, hipcc waited for the step block before issuing anything
    const __attribute__((address_space(4))) StepParams * spc = (const __attribute__((address_space(4))) StepParams *) A.sp;
    const int n_past = spc->n_past;
    const unsigned seqv = spc->seq;
    __builtin_amdgcn_sched_barrier(0);

    // 1a. Q goes out before the step block is known; V follows behind the first scores (1b)
    uint4 qv[4];
    {
        const uint4 * qp = (const uint4 *) (A.q16 + h * HD) + r;
#pragma unroll
        for (int st = 0; st < 4; ++st) qv[st] = qp[st * 4];
    }
    LVK_DT(13);
    __builtin_amdgcn_sched_barrier(0);
#ifdef LVK_PROBE_TIMING
    asm volatile("" ::"s"(n_past));
    LVK_DT(12);
#endif
    auto v_dma = [&](int p0, int lo, int lim) {     // positions [max(p0, lo), min(p0 + 512, lim)) of rows 8 wave ..
#pragma unroll
        for (int i = 0; i < 8; ++i) {               // a static count: the score waits can count past it
            const int row = wave * 8 + i;
            if (p0 + lane * 8 >= lo && p0 + lane * 8 < lim)
                __builtin_amdgcn_global_load_lds((const void *) (A.vc + (size_t) (d0 + row) * n_ctx + p0 + lane * 8),
                                                 (__attribute__((address_space(3))) void *) (vl + (size_t) row * VS + p0),
                                                 16, 0, 0);
        }
    };
    // this layer's granule tag: unique per (step, layer) when the step counter is used
    const unsigned ep = A.epoch + (A.seq_epochs ? seqv << 7 : 0u);
    const int n_kv = n_past + 1;
    const int n_pad = (n_kv + 31) & ~31;
    const int np = n_kv & ~31;
    const bool exch = DYN ? n_kv > A.short_max : true;
    const int cs = exch ? 256 : 64;                     // position stride of this workgroup's chunks
    const int cb = exch ? sl * 64 : 0;                  // its first chunk
    // this workgroup's first two K chunks, issued once n_past is known.  (A speculative load
    // of positions 0..63 before the step block, which only the short schedule and workgroup 0
    // use, measured 0.1-0.25 us slower per launch: it queued ahead of the chunks an exchange
    // workgroup needs; profiles/r06/decode_ab/)
    uint4 kv[2][4];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        const int p = min(cb + k * cs + (tid >> 2), n_kv - 1);
        const uint4 * kp = (const uint4 *) (A.kc + (size_t) p * E + h * HD) + r;
#pragma unroll
        for (int st = 0; st < 4; ++st) kv[k][st] = kp[st * 4];
    }
    LVK_DT(6);

    // 1b. scores of chunks sl, sl+4, ... (exchange) or of every chunk (one position per lane quad)
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
                const float v = kq * A.scale;                    // ggml_vec_scale_f32 (llama.cpp:1026)
                if (!exch) sc[p] = v;
#ifdef LVK_PROBE_DROP_GRANULE   // fault-injection probe build only: position 0's score is never published
                else if (p == 0) {}
#endif
                else __hip_atomic_store(g + p, ((unsigned long long) ep << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
        };
        score(kv[0], cb + (tid >> 2));               // positions past n_kv publish nothing
        if (cb + cs < n_kv) score(kv[1], cb + cs + (tid >> 2));
        // the V slice goes out behind the first two chunks' scores: those wait only for their
        // own K rows, the V rows are needed after the softmax.  (Chunk 0 of V issued with Q
        // and K chunk 0, or right after the n_past-dependent K loads: 5.66-5.73 / 5.71-5.77 us
        // against 5.42-5.47 us per launch here, 7B decode_speed, profiles/r04_attn_vorder.jsonl)
        for (int p0 = 0; p0 < n_pad; p0 += 512) v_dma(p0, 0, n_pad);
        LVK_DT(7);
        LVK_DT(1);
        for (int c0 = cb + 2 * cs; c0 < n_kv; c0 += cs) {
            const int p = c0 + (tid >> 2);
            const uint4 * kp = (const uint4 *) (A.kc + (size_t) min(p, n_kv - 1) * E + h * HD) + r;
            uint4 k4[4];
#pragma unroll
            for (int st = 0; st < 4; ++st) k4[st] = kp[st * 4];
            score(k4, p);
        }
    }
    LVK_DT(2);
    // 2. softmax (ggml.c:7099-7121; no position is masked in a decode step).  Exchange: the
    // granules are read four at a time; the ones without this layer's epoch are polled.
    float mx = -INFINITY;
    if (!exch) {
        bar();
        for (int p = tid; p < n_kv; p += 256) mx = sc[p] > mx ? sc[p] : mx;
    } else {
        for (int p0 = tid; p0 < n_kv; p0 += 1024) {
            unsigned long long x[4];
#pragma unroll
            for (int k = 0; k < 4; ++k)
                x[k] = __hip_atomic_load(g + min(p0 + 256 * k, n_kv - 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int p = p0 + 256 * k;
                if (p < n_kv) {
                    const unsigned long long y =
                        (unsigned) (x[k] >> 32) == ep ? x[k] : poll_granule(g + p, ep, A.err);
                    const float v = __uint_as_float((unsigned) y);
                    sc[p] = v;
                    mx = v > mx ? v : mx;
                }
            }
        }
    }
    LVK_DT(3);
    mx = wave_max_f(mx);
    if (lane == 0) red[wave] = mx;
    bar();
    LVK_DT(8);
    {
        const float a = red[0] > red[1] ? red[0] : red[1], b = red[2] > red[3] ? red[2] : red[3];
        mx = a > b ? a : b;
    }
    double sum = 0.0;    // exact in any order: every term is an fp16 value in [0,1]
    for (int p = tid; p < n_kv; p += 256) {
        const float e = f16_to_f32(exp_softmax<EM>(f32_to_f16(sc[p] - mx), A.exp_tab, A.exp_mode));
        sum += (double) e;
        sc[p] = e;
    }
    sum = wave_sum_d(sum);
    if (lane == 0) redd[wave] = sum;
    bar();
    LVK_DT(9);
    sum = (redd[0] + redd[1]) + (redd[2] + redd[3]);
    const float scl = (float) (1.0 / sum);
    for (int p = tid; p < n_pad; p += 256) pl[p] = p < n_kv ? f32_to_f16(sc[p] * scl) : (uint16_t) 0;
    LVK_DT(4);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    bar();                    // the V DMA has landed too
    LVK_DT(5);

#ifdef LVK_ATTN_PV_QUAD   // probe A/B only: the round-2 P.V (a lane quad per dim on waves 0-1)
    float o = 0.0f;
    const int q = tid >> 2;
    const uint16_t * vr = vl + (size_t) q * VS;
    if (tid < 128) {
        float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        const int ns = np / 32;
        int st = 0;
        for (; st + 2 <= ns; st += 2) {
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
        if (np < n_kv) {
            double sumf = (double) res;
            for (int p = np; p < n_kv; ++p) {
                const float prod = f16_to_f32(vr[p]) * f16_to_f32(pl[p]);
                sumf += (double) prod;
            }
            o = (float) sumf;
        }
    }
#define LVK_OB_LANE (tid < 128 && r == 0)
#else
    // P.V (ggml_vec_dot_f16, ggml.c:1781-1815): 8 threads per dim (wave w: dims 8w..8w+7),
    // thread (r, hf) runs the AVX accumulators 4hf..4hf+3 of lane quad member r -- positions
    // 32 st + 8 r + 4 hf + i -- with v_fma_mix (the f16 operands converted exactly, one
    // rounding: fmaf of the converted values), then the F32Cx8 reduce order of quad_reduce.
    float o = 0.0f;
    const int q = tid >> 3, hf = (tid >> 2) & 1;
    const uint16_t * vr = vl + (size_t) q * VS;
    {
        float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f, s3 = 0.0f;
        const int ns = np / 32;
        const int off = r * 8 + hf * 4;
        auto step = [&](int st) __attribute__((always_inline)) {
            const uint2 v = *(const uint2 *) (vr + st * 32 + off);
            const uint2 pp = *(const uint2 *) (pl + st * 32 + off);
            s0 = fma_mix_hh<0, 0>(v.x, pp.x, s0);
            s1 = fma_mix_hh<1, 1>(v.x, pp.x, s1);
            s2 = fma_mix_hh<0, 0>(v.y, pp.y, s2);
            s3 = fma_mix_hh<1, 1>(v.y, pp.y, s3);
        };
        int st = 0;
        for (; st + 4 <= ns; st += 4) { step(st); step(st + 1); step(st + 2); step(st + 3); }
        for (; st < ns; ++st) step(st);
        // S[l] = (r0 + r1) + (r2 + r3) over the quad, then t_i = S[i] + S[i + 4] (halves 0, 1)
        auto qsum = [](float v) {
            const float v0 = quad_bcast<0>(v), v1 = quad_bcast<1>(v), v2 = quad_bcast<2>(v), v3 = quad_bcast<3>(v);
            return (v0 + v1) + (v2 + v3);
        };
        // the other half's S (lane ^ 4 inside the 8-lane group): row_ror:n hands lane l the
        // value of lane (l - n) mod 16, so half 0 takes ror 12 (l + 4), half 1 ror 4 (l - 4)
        auto other = [&](float v) {
            const int i = __builtin_bit_cast(int, v);
            const int a = __builtin_amdgcn_update_dpp(0, i, 0x124, 0xF, 0xF, false);   // row_ror:4
            const int b = __builtin_amdgcn_update_dpp(0, i, 0x12C, 0xF, 0xF, false);   // row_ror:12
            return __builtin_bit_cast(float, hf ? a : b);
        };
        const float S0 = qsum(s0), S1 = qsum(s1), S2 = qsum(s2), S3 = qsum(s3);
        const float t0 = S0 + other(S0), t1 = S1 + other(S1);
        const float t2 = S2 + other(S2), t3 = S3 + other(S3);
        o = (t0 + t1) + (t2 + t3);
    }
    if (np < n_kv) {
        // leftovers in double, in position order (ggml.c:1806-1808): the 8 lanes of a dim form
        // the products of positions np + 8k + lane (-0.0 past n_kv: an exact no-op in the sum),
        // row_shl moves them to the dim's first lane, which adds them in order
        const int sub = tid & 7;
        float pr[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int p = np + 8 * k + sub;
            pr[k] = p < n_kv ? f16_to_f32(vr[p]) * f16_to_f32(pl[p]) : -0.0f;
        }
        double sumf = (double) o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (8 * k >= n_kv - np) break;
            const int i = __builtin_bit_cast(int, pr[k]);
            float v[8];
            v[0] = pr[k];
            v[1] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x101, 0xF, 0xF, false));
            v[2] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x102, 0xF, 0xF, false));
            v[3] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x103, 0xF, 0xF, false));
            v[4] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x104, 0xF, 0xF, false));
            v[5] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x105, 0xF, 0xF, false));
            v[6] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x106, 0xF, 0xF, false));
            v[7] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, i, 0x107, 0xF, 0xF, false));
#pragma unroll
            for (int j = 0; j < 8; ++j) sumf += (double) v[j];
        }
        o = (float) sumf;     // meaningful in the dim's first lane
    }
#define LVK_OB_LANE ((tid & 7) == 0)
#endif
    LVK_DT(10);
    float * ob = sc;          // reuse: 32 outputs (sc was last read before the barrier above)
    if (LVK_OB_LANE) ob[q] = o;
#undef LVK_OB_LANE
    bar();
    if (tid < 32) {
        const float v = ob[tid];
        if (A.out_f32) A.out_f32[d0 + tid] = v;
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
                A.out.d[blk] = dd;
                A.out.qs[blk] = make_uint4(w0, w1, w2, w3);
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
            ((uint32_t *) (A.out.qs + blk))[tid] = qw;
            if (tid == 0) {
                A.out.d[blk] = dd;
                A.out.m[blk] = mm;
            }
        }
    }
    LVK_DT(11);
}

// LDS of one decode-attention workgroup (V slice, scores, probabilities, reductions)
__host__ __device__ inline size_t attn_lds(int n_ctx) { return (size_t) 32 * (n_ctx + 32) * 2 + (size_t) n_ctx * 6 + 80; }

// kernel arguments of a decode-attention launch (host side)
inline AttnDArgs attn_args(const AttnLaunch & A, void * gran, unsigned epoch) {
    AttnDArgs a{};
    a.q16 = A.q16;
    a.kc = A.kc;
    a.vc = A.vc;
    a.gran = (unsigned long long *) gran;
    a.exp_tab = A.exp_tab;
    a.sp = A.sp;
    a.E = A.n_embd;
    a.n_ctx = A.n_ctx;
    a.scale = 1.0f / sqrtf((float) A.n_embd / (float) A.n_head);   // llama.cpp:1028
    a.epoch = epoch;
    a.out = A.out;
    a.out_f32 = A.out_f32;
    a.exp_mode = A.exp_computed;
    a.err = A.err;
    // short contexts skip the score exchange: every workgroup of a head scores all n_kv
    // positions itself (tools/probe r03: 4.8 vs 5.4 us at n_kv 33, 5.9 vs 6.3 at 101)
    static const int short_max = [] {
        const char * e = getenv("LVK_ATTN_SHORT");
        if (getenv("LVK_ATTN_NOEXCH") && atoi(getenv("LVK_ATTN_NOEXCH")) != 0) return 1 << 30;
        return e ? atoi(e) : 128;
    }();
    a.short_max = short_max;
    a.seq_epochs = A.seq_epochs;
    return a;
}

template <int QT, int EM>
__global__ __launch_bounds__(256) void k_attn_d(AttnDArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    attn_d_run<QT, EM, true>(A, blockIdx.x, blockIdx.y, smem, threadIdx.x);
}

}  // namespace

#ifdef LVK_PROBE_TIMING
void * lvk_probe_dtrace() { void * p = nullptr; (void) hipGetSymbolAddress(&p, HIP_SYMBOL(g_dtrace)); return p; }
#endif

bool attention_decode_supported(int n_embd, int n_head, int n_ctx) {
    return n_embd / n_head == HD && n_ctx % 64 == 0 && n_ctx <= 2048 && n_head * 4 <= 1024;
}

size_t attention_decode_scratch_bytes(int n_head, int n_ctx) {
    // score granules [H][n_ctx]
    return (size_t) n_head * n_ctx * 8;
}

hipError_t launch_attention_decode(const AttnLaunch & A, void * gran, unsigned epoch, hipStream_t s) {
    if (!attention_decode_supported(A.n_embd, A.n_head, A.n_ctx) || A.n_tokens != 1 || epoch == 0)
        return hipErrorNotSupported;
    if (A.out_qtype != Q4_0 && A.out_qtype != Q4_1) return hipErrorNotSupported;
    const AttnDArgs a = attn_args(A, gran, epoch);
    const size_t lds = attn_lds(A.n_ctx);
    const dim3 grid(A.n_head, HD / 32);
#define LVK_ATTN_EM(QT_)                                                                  \
    switch (a.exp_mode) {                                                                 \
        case 2: LVK_LAUNCH((k_attn_d<QT_, 2>), grid, dim3(256), lds, s, a); break;        \
        case 1: LVK_LAUNCH((k_attn_d<QT_, 1>), grid, dim3(256), lds, s, a); break;        \
        default: LVK_LAUNCH((k_attn_d<QT_, 0>), grid, dim3(256), lds, s, a); break;       \
    }
    if (A.out_qtype == Q4_1) { LVK_ATTN_EM(Q4_1) } else { LVK_ATTN_EM(Q4_0) }
#undef LVK_ATTN_EM
    return hipGetLastError();
}

}  // namespace lvk
