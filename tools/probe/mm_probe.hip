// mm_probe: times the MFMA prompt matmul (mm_mfma.hip) on 7B shapes, N = 512,
// with random weights/activations.  Build: make -C tools/probe mm_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "lvk_kernels.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1);} } while (0)
using namespace lvk;
__global__ void k_fill_u32(uint32_t * p, size_t n, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) i * 2654435761u ^ seed; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; p[i] = h;
    }
}
__global__ void k_fill_f32(float * p, size_t n, float lo, float hi, uint32_t seed) {
    for (size_t i = blockIdx.x * (size_t) blockDim.x + threadIdx.x; i < n; i += (size_t) gridDim.x * blockDim.x) {
        uint32_t h = (uint32_t) i * 2654435761u ^ seed; h ^= h >> 15; h *= 2246822519u; h ^= h >> 13;
        p[i] = lo + (hi - lo) * (h & 0xFFFFFF) / 16777216.0f;
    }
}
static void * dalloc(size_t b) { void * p; CK(hipMalloc(&p, b + 4096)); return p; }
int main(int argc, char ** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 512;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    struct Sh { const char * name; int M, K; int epi; } sh[] = {
        {"qkv", 12288, 4096, EPI_STORE}, {"wo", 4096, 4096, EPI_RESID}, {"w13", 22016, 4096, EPI_SWIGLU_F32},
        {"w2", 4096, 11008, EPI_RESID}};
    const int KX = 11008;
    float * x = (float *) dalloc((size_t) N * KX * 4);
    hipLaunchKernelGGL(k_fill_f32, dim3(1024), dim3(256), 0, 0, x, (size_t) N * KX, -2.f, 2.f, 3u);
    void * xh = dalloc(mm_act_bytes(N, KX));
    CK(hipMemset(xh, 0, mm_act_bytes(N, KX)));
    float * da = (float *) dalloc((size_t) N * KX / 32 * 4);
    float * y = (float *) dalloc((size_t) N * 22016 * 4);
    uint16_t * stab = (uint16_t *) dalloc(65536 * 2);
    CK(hipMemset(stab, 0, 65536 * 2));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    double total = 0;
    for (auto & s : sh) {
        QMatrix q; q.qtype = Q4_0; q.M = s.M; q.K = s.K;
        void * nib = dalloc(qimage_nib_bytes(s.M, s.K)); void * scl = dalloc(qimage_scl_bytes(s.M, s.K));
        hipLaunchKernelGGL(k_fill_u32, dim3(1024), dim3(256), 0, 0, (uint32_t *) nib, qimage_nib_bytes(s.M, s.K) / 4, 7u);
        hipLaunchKernelGGL(k_fill_f32, dim3(1024), dim3(256), 0, 0, (float *) scl, qimage_scl_bytes(s.M, s.K) / 4, 0.001f, 0.01f, 9u);
        q.nib = (const uint4 *) nib; q.scl = scl;
        void * a16 = nullptr;
        if (getenv("MM_A16") && atoi(getenv("MM_A16"))) {       // the product's f16 A image
            a16 = dalloc(mm_a16_bytes(s.M, s.K));
            CK(launch_build_a16(q, a16, 0));
            q.a16 = a16;
        }
        CK(launch_act_f16(x, nullptr, N, s.K, xh, da, 0));
        const int ldy = s.epi == EPI_SWIGLU_F32 ? s.M / 2 : s.M;
        // one launch on a zeroed y: FNV hash of the output bits (variants must agree)
        CK(hipMemset(y, 0, (size_t) N * ldy * 4));
        CK(launch_mm_mfma(q, xh, da, N, y, ldy, 0, s.epi, stab, 0));
        CK(hipDeviceSynchronize());
        {
            std::vector<uint32_t> h((size_t) N * ldy);
            CK(hipMemcpy(h.data(), y, h.size() * 4, hipMemcpyDeviceToHost));
            uint64_t f = 1469598103934665603ull;
            for (uint32_t v : h) { f ^= v; f *= 1099511628211ull; }
            printf("%-4s hash %016llx\n", s.name, (unsigned long long) f);
        }
        for (int i = 0; i < 2; ++i) CK(launch_mm_mfma(q, xh, da, N, y, ldy, 0, s.epi, stab, 0));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, 0));
        for (int i = 0; i < reps; ++i) CK(launch_mm_mfma(q, xh, da, N, y, s.epi == EPI_SWIGLU_F32 ? s.M / 2 : s.M, 0, s.epi, stab, 0));
        CK(hipEventRecord(e1, 0)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / reps;
        const double partials = (double) s.M * N * s.K / 4;     // 4-element chain partials
        printf("%-4s M %5d K %5d N %d: %8.1f us  %.2f Tpartial/s  %.1f TMAC/s (dense)\n", s.name, s.M, s.K, N, us,
               partials / us * 1e-6, (double) s.M * N * s.K / us * 1e-6);
        total += us;
        CK(hipFree(nib)); CK(hipFree(scl));
        if (a16) CK(hipFree(a16));
    }
    printf("layer total %.1f us -> 32 layers %.2f ms\n", total, total * 32 / 1e3);
    return 0;
}
