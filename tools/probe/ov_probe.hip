// ov_probe: can the 7B decode layer's weight stream keep running under its dependency edges?
// (dev probe, not product code; round-6 verdict item 2, the probe gate before any product change)
//
// One token = 32 x {QKV 31.5 MB, attention (128 workgroups, latency only), Wo 10.5 MB,
// W1|W3 56.4 MB, W2 28.2 MB} + lm_head 81.9 MB of distinct weight buffers, streamed with
// trivial compute by 256-workgroup launches (the decode matvecs' byte volumes and grid).
//
// Modes (argv[1]):
//   graph   -- plain launches captured once into a hipGraph, replayed per token (the product
//              structure: each launch starts its weight stream after the previous one ended)
//   eager   -- the same plain launches, enqueued per token
//   seq     -- flag-chained kernels (prefetch, counter wait, publish) on one stream, plain
//              launches (barrier bit set): the cost of the flag mechanism with no overlap
//   any     -- flag-chained kernels launched with hipExtAnyOrderLaunch on one stream
//   two     -- flag-chained kernels alternating over two streams
// Flag-chained kernel: every wave issues its first R weight loads (1 KiB each), then lane 0
// polls the predecessor's arrival counter (sc1 loads, s_sleep, bounded), a workgroup barrier,
// the activation vector is read with sc1 loads, the rest of the slice streams; the outputs
// are sc1 stores, every wave waits vmcnt(0), a barrier, one agent atomic add arrives.
// argv[2] = attention spin (us, default 5), argv[3] = tokens (default 50).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1);} } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

struct Ph {
    const char * w;          // weights of this launch
    unsigned nload;          // 1 KiB wave loads per workgroup slice
    unsigned * wait;         // arrival counter of the predecessor (nullptr: none)
    unsigned target;         // per shard
    unsigned * done;         // own arrival counter (nullptr: none)
    int shards;              // 1: one counter; 8: one per blockIdx % 8 (the XCD under round-robin), 64 B apart
    const u32x4 * act;       // activation vector, act_loads 16-B loads per thread
    unsigned act_loads;
    u32x4 * out;             // one 16-B word per wave
    unsigned spin;           // realtime ticks (100 MHz) of latency-only work after the wait
    unsigned * err;
    unsigned long long * tstamp;   // [2]: min start, max end (realtime), or nullptr
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void * p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short) 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ u32x4 ld_nt(const u32x4 * p) { return __builtin_nontemporal_load(p); }

template <int NW, int R, bool FLAG>
__global__ __launch_bounds__(NW * 64) void k_ph(Ph p) {
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    if (p.tstamp && tid == 0) atomicMin(&p.tstamp[0], (unsigned long long) __builtin_amdgcn_s_memrealtime());
    const char * base = p.w + (size_t) blockIdx.x * p.nload * 1024;
    const unsigned nw = p.nload > (unsigned) wave ? (p.nload - wave + NW - 1) / NW : 0;
    const unsigned last = nw ? nw - 1 : 0;
    auto addr = [&](unsigned i) {
        const unsigned li = wave + (i < last ? i : last) * NW;
        return (const u32x4 *) (base + (size_t) li * 1024 + lane * 16);
    };
    u32x4 v[R];
    if constexpr (FLAG) {
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = ld_nt(addr(r));
        if (p.wait) {
            if (wave == 0) {
                // lanes 0..shards-1 poll one shard each (one sc1 load instruction per poll)
                const int sh = lane < p.shards ? lane : 0;
                unsigned n = 0;
                while (true) {
                    const unsigned v = __hip_atomic_load(p.wait + sh * 16, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (__builtin_amdgcn_read_exec() == 0 || __all(v >= p.target)) break;
                    __builtin_amdgcn_s_sleep(1);
                    if (++n > (1u << 24)) { if (lane == 0) atomicOr(p.err, 1u); break; }
                }
            }
            __builtin_amdgcn_s_barrier();
        }
    }
    unsigned acc = 0;
    for (unsigned k = 0; k < p.act_loads; ++k) {
        const u32x4 a = FLAG ? __builtin_amdgcn_raw_buffer_load_b128(rsrc(p.act), (k * blockDim.x + tid) * 16, 0, 16)
                             : p.act[k * blockDim.x + tid];
        acc += a.x ^ a.w;
    }
    if (p.spin) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        while (__builtin_amdgcn_s_memrealtime() - t0 < p.spin) __builtin_amdgcn_s_sleep(2);
    }
    if constexpr (!FLAG) {
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = ld_nt(addr(r));
    }
    for (unsigned i = 0; i < nw; i += R) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (i + r < nw) acc ^= v[r].x + v[r].y * 3u + v[r].z * 5u + v[r].w * 7u;
            v[r] = ld_nt(addr(i + r + R));
        }
    }
    if (lane == 0) {
        const u32x4 o = {acc, acc ^ 1u, acc ^ 2u, acc ^ 3u};
        if constexpr (FLAG) __builtin_amdgcn_raw_buffer_store_b128(o, rsrc(p.out), (blockIdx.x * NW + wave) * 16, 0, 16);
        else p.out[blockIdx.x * NW + wave] = o;
    }
    if constexpr (FLAG) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0 && p.done)
            __hip_atomic_fetch_add(p.done + (blockIdx.x % p.shards) * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (p.tstamp && tid == 0) atomicMax(&p.tstamp[1], (unsigned long long) __builtin_amdgcn_s_memrealtime());
}

constexpr int NW = 8;

int main(int argc, char ** argv) {
    const char * mode = argc > 1 ? argv[1] : "graph";
    const double spin_us = argc > 2 ? atof(argv[2]) : 5.0;
    const int T = argc > 3 ? atoi(argv[3]) : 50;
    const int R = argc > 4 ? atoi(argv[4]) : 16;
    const int shards = argc > 5 ? atoi(argv[5]) : 8;
    const bool flag = strcmp(mode, "graph") && strcmp(mode, "eager");
    const int L = 32;
    const size_t mats[4] = {3ull * 4096 * 4096 / 32 * 20, 4096ull * 4096 / 32 * 20,
                            2ull * 11008 * 4096 / 32 * 20, 11008ull * 4096 / 32 * 20};
    const size_t lm = 32000ull * 4096 / 32 * 20;
    // kernel list of one token: per layer QKV, ATT, Wo, W13, W2; then lm_head
    struct K { size_t bytes; int nwg; unsigned act_loads; unsigned spin; };
    std::vector<K> ks;
    const unsigned spin = (unsigned) (spin_us * 100.0);
    for (int l = 0; l < L; ++l) {
        ks.push_back({mats[0], 256, 2, 0});        // x (16 KiB) over 512 threads: 2 loads
        ks.push_back({0, 128, 2, spin});           // attention: q / K / V reads, latency
        ks.push_back({mats[1], 256, 2, 0});
        ks.push_back({mats[2], 256, 2, 0});
        ks.push_back({mats[3], 256, 6, 0});        // u (44 KiB)
    }
    ks.push_back({lm, 256, 2, 0});
    const int NK = (int) ks.size();
    std::vector<char *> w(NK, nullptr);
    size_t total = 0;
    for (int k = 0; k < NK; ++k) {
        if (!ks[k].bytes) continue;
        CK(hipMalloc(&w[k], ks[k].bytes + (1 << 20)));
        CK(hipMemset(w[k], k & 0xff, ks[k].bytes + (1 << 20)));
        total += ks[k].bytes;
    }
    u32x4 * act; CK(hipMalloc(&act, 1 << 20)); CK(hipMemset(act, 0, 1 << 20));
    u32x4 * out; CK(hipMalloc(&out, 1 << 20));
    unsigned * cnt; CK(hipMalloc(&cnt, NK * 1024)); CK(hipMemset(cnt, 0, NK * 1024));
    unsigned * err; CK(hipMalloc(&err, 64)); CK(hipMemset(err, 0, 64));
    unsigned long long * ts; CK(hipMalloc(&ts, NK * 16));
    hipStream_t s[2];
    if (getenv("OV_NONBLOCKING")) { CK(hipStreamCreateWithFlags(&s[0], hipStreamNonBlocking)); CK(hipStreamCreateWithFlags(&s[1], hipStreamNonBlocking)); }
    else { CK(hipStreamCreate(&s[0])); CK(hipStreamCreate(&s[1])); }
    printf("mode %s, token bytes %.1f MB, %d launches, attention spin %.1f us\n", mode, total / 1e6, NK, spin_us);

    auto params = [&](int k, int tok, bool stamp) {
        Ph p{};
        p.w = w[k] ? w[k] : (char *) act;
        p.nload = ks[k].bytes ? (unsigned) ((ks[k].bytes / ks[k].nwg + 1023) / 1024) : 0;
        if (flag) {
            // counter of kernel k lives at cnt[k * 64]; kernel k waits on k - 1 (previous token's
            // lm_head for k = 0)
            const int pk = k ? k - 1 : NK - 1;
            const int ptok = k ? tok : tok - 1;
            if (ptok >= 0) { p.wait = cnt + pk * 256; p.target = (unsigned) (ptok + 1) * ks[pk].nwg / shards; }
            p.done = cnt + k * 256;
            p.shards = shards;
        }
        p.act = act; p.act_loads = ks[k].act_loads; p.out = out; p.spin = ks[k].spin; p.err = err;
        p.tstamp = stamp ? ts + 2 * k : nullptr;
        return p;
    };
    auto launch = [&](int k, int tok, bool stamp, hipStream_t st, int flags) {
        Ph p = params(k, tok, stamp);
        void * args[] = {&p};
        const void * fn = R == 4 ? (flag ? (const void *) k_ph<NW, 4, true> : (const void *) k_ph<NW, 4, false>)
                        : R == 8 ? (flag ? (const void *) k_ph<NW, 8, true> : (const void *) k_ph<NW, 8, false>)
                                 : (flag ? (const void *) k_ph<NW, 16, true> : (const void *) k_ph<NW, 16, false>);
        CK(hipExtLaunchKernel(fn, dim3(ks[k].nwg), dim3(NW * 64), args, 0, st, nullptr, nullptr, flags));
    };
    int tok = 0;
    auto token = [&](bool stamp) {
        for (int k = 0; k < NK; ++k) {
            if (!strcmp(mode, "two")) launch(k, tok, stamp, s[k & 1], 0);
            // "mixed": only the launch after each attention (Wo) is any-order, as in the library
            else if (!strcmp(mode, "mixed")) launch(k, tok, stamp, s[0], (k % 5 == 2) ? hipExtAnyOrderLaunch : 0);
            else launch(k, tok, stamp, s[0], !strncmp(mode, "any", 3) ? hipExtAnyOrderLaunch : 0);
        }
        ++tok;
    };
    hipGraphExec_t ge = nullptr;
    std::vector<hipGraphExec_t> gtok;
    if (!strcmp(mode, "anyg")) {
        // one captured graph per token (the counter targets are baked into the arguments)
        for (int t = 0; t < 5 + T + 1; ++t) {
            hipGraph_t g; hipGraphExec_t x;
            CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeGlobal));
            token(t == 5 + T);
            CK(hipStreamEndCapture(s[0], &g));
            CK(hipGraphInstantiate(&x, g, nullptr, nullptr, 0));
            gtok.push_back(x);
        }
        tok = 0;
    }
    if (!strcmp(mode, "graph")) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s[0], hipStreamCaptureModeGlobal));
        token(false);
        CK(hipStreamEndCapture(s[0], &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    auto run = [&](bool stamp) {
        if (ge) CK(hipGraphLaunch(ge, s[0]));
        else if (!gtok.empty()) CK(hipGraphLaunch(gtok[tok++], s[0]));
        else token(stamp);
        CK(hipStreamSynchronize(s[0]));
        CK(hipStreamSynchronize(s[1]));
    };
    for (int i = 0; i < 5; ++i) run(false);
    std::vector<double> ms;
    for (int i = 0; i < T; ++i) {
        auto t0 = std::chrono::steady_clock::now();
        run(false);
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    unsigned herr = 0; CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    std::sort(ms.begin(), ms.end());
    const double med = ms[ms.size() / 2];
    printf("%s: median %.3f ms/token (%.0f tok/s, %.3f of 8 TB/s), min %.3f, per layer %.2f us%s\n", mode, med,
           1e3 / med, total / (med * 1e-3) / 8e12, ms[0], med * 1e3 / L, herr ? "  SPIN TIMEOUT" : "");
    if (!ge && gtok.empty()) {
        // one stamped token: first-start / last-end per launch, overlap with the predecessor
        std::vector<unsigned long long> h(NK * 2);
        for (int k = 0; k < NK; ++k) { h[2 * k] = ~0ull; h[2 * k + 1] = 0; }
        CK(hipMemcpy(ts, h.data(), NK * 16, hipMemcpyHostToDevice));
        run(true);
        CK(hipMemcpy(h.data(), ts, NK * 16, hipMemcpyDeviceToHost));
        int ov = 0;
        double kind_dur[5] = {}, kind_gap[5] = {};
        for (int k = 1; k < NK - 1; ++k) {
            const long long gap = (long long) h[2 * k] - (long long) h[2 * (k - 1) + 1];
            if (gap < 0) ++ov;
            kind_dur[k % 5] += (double) (h[2 * k + 1] - h[2 * k]) * 0.01 / L;
            kind_gap[k % 5] += (double) gap * 0.01 / L;
        }
        printf("  launches starting before their predecessor ended: %d of %d\n", ov, NK - 2);
        const char * nm[5] = {"qkv", "att", "wo", "w13", "w2"};
        for (int c = 0; c < 5; ++c)
            printf("  %-4s span %.2f us, start - predecessor end %.2f us\n", nm[c], kind_dur[c], kind_gap[c]);
        printf("  token span %.1f us\n", (double) (h[2 * (NK - 1) + 1] - h[0]) * 0.01);
    }
    return herr ? 2 : 0;
}
