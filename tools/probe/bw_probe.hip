// bw_probe: how fast can the 7B decode weight stream go on this chip?
// Streams one token's worth of Q4_0 weight bytes (32 layers x {qkv, wo, w13, w2} + lm_head,
// 4.13 GB in distinct buffers) with trivial compute, as one graph of 129 launches, and
// reports per-matrix kernel time and per-token time for several launch shapes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void k_stream(const u32x4 * __restrict__ p, size_t n_per_wg, unsigned * out) {
    const u32x4 * q = p + (size_t)blockIdx.x * n_per_wg;
    unsigned acc = 0;
    for (size_t i = threadIdx.x; i < n_per_wg; i += (size_t)blockDim.x * U) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            size_t j = i + (size_t)u * blockDim.x;
            j = j < n_per_wg ? j : n_per_wg - 1;
            v[u] = NT ? __builtin_nontemporal_load(q + j) : q[j];
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc ^= v[u].x + v[u].y * 3 + v[u].z * 5 + v[u].w * 7;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

struct Shape { const char * name; int nt; int u; int wg_bytes; bool ntl; };

int main() {
    const size_t mats[4] = {3ull * 4096 * 4096 / 32 * 20, 4096ull * 4096 / 32 * 20, 2ull * 11008 * 4096 / 32 * 20,
                            11008ull * 4096 / 32 * 20};
    const size_t lm = 32000ull * 4096 / 32 * 20;
    const int L = 32;
    std::vector<u32x4 *> buf(L * 4 + 1);
    size_t total = 0;
    for (int l = 0; l < L; l++)
        for (int m = 0; m < 4; m++) { CK(hipMalloc(&buf[l * 4 + m], mats[m] + 65536)); total += mats[m]; }
    CK(hipMalloc(&buf[L * 4], lm + 65536)); total += lm;
    for (auto b : buf) CK(hipMemset(b, 1, 1 << 20));
    unsigned * out; CK(hipMalloc(&out, 1 << 20));
    printf("token bytes %.1f MB\n", total / 1e6);
    hipStream_t s; CK(hipStreamCreate(&s));
    Shape shapes[] = {
        {"256thr u4 20KB/wg", 256, 4, 20480, false}, {"256thr u8 40KB/wg", 256, 8, 40960, false},
        {"256thr u8 80KB/wg", 256, 8, 81920, false}, {"256thr u8 160KB/wg", 256, 8, 163840, false},
        {"512thr u8 80KB/wg", 512, 8, 81920, false}, {"256thr u8 40KB/wg nt", 256, 8, 40960, true},
        {"256thr u8 80KB/wg nt", 256, 8, 81920, true}, {"256thr u16 80KB/wg nt", 256, 16, 81920, true},
        {"1024thr u8 160KB/wg nt", 1024, 8, 163840, true}, {"256thr u4 10KB/wg nt", 256, 4, 10240, true},
    };
    for (auto & sh : shapes) {
        auto launch = [&](const u32x4 * p, size_t bytes) {
            size_t n = (bytes + sh.wg_bytes - 1) / sh.wg_bytes;
            size_t per = sh.wg_bytes / 16;
#define L_(U, NT) hipLaunchKernelGGL((k_stream<U, NT>), dim3(n), dim3(sh.nt), 0, s, p, per, out)
            if (sh.u == 4) { if (sh.ntl) L_(4, true); else L_(4, false); }
            else if (sh.u == 8) { if (sh.ntl) L_(8, true); else L_(8, false); }
            else { if (sh.ntl) L_(16, true); else L_(16, false); }
        };
        hipGraph_t g; hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int l = 0; l < L; l++) for (int m = 0; m < 4; m++) launch(buf[l * 4 + m], mats[m]);
        launch(buf[L * 4], lm);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 3; i++) CK(hipGraphLaunch(ge, s));
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0, s));
        const int R = 20;
        for (int i = 0; i < R; i++) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        double tok = ms / R;
        // per-matrix: time 32 launches of one matrix kind back to back
        double per[5];
        for (int m = 0; m < 5; m++) {
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < 4; r++)
                for (int l = 0; l < (m < 4 ? L : 8); l++) launch(m < 4 ? buf[l * 4 + m] : buf[L * 4], m < 4 ? mats[m] : lm);
            CK(hipEventRecord(e1, s)); CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&ms, e0, e1));
            per[m] = ms * 1e3 / (4 * (m < 4 ? L : 8));
        }
        printf("%-24s token %.3f ms (%.0f tok/s, %.2f TB/s) | qkv %.1f wo %.1f w13 %.1f w2 %.1f lm %.1f us\n", sh.name, tok,
               1e3 / tok, total / (tok * 1e-3) / 1e12, per[0], per[1], per[2], per[3], per[4]);
        CK(hipGraphExecDestroy(ge)); CK(hipGraphDestroy(g));
    }
    return 0;
}
