// mfma_cycles: issue cost of the MFMA forms the prompt matmul could use, measured on this
// chip (one wave, 4 independent accumulators, back-to-back).  Build: make -C tools/probe
// mfma_cycles.  Prints cycles per instruction (s_memtime ticks).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f32v __attribute__((ext_vector_type(32)));

#define N_IT 512

template <int KIND>
__global__ void k_mfma(float * out, unsigned long long * cyc) {
    const int l = threadIdx.x;
    h4 a4 = {(_Float16) (l & 3), (_Float16) 1, (_Float16) 2, (_Float16) 3};
    h8 a8 = {(_Float16) (l & 3), (_Float16) 1, (_Float16) 2, (_Float16) 3, (_Float16) 1, (_Float16) 1, (_Float16) 1, (_Float16) 1};
    float fa = (float) l;
    f16v c16[4] = {};
    f32v c32[4] = {};
    f4 c4[4] = {};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; ++it) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if constexpr (KIND == 0) c16[q] = __builtin_amdgcn_mfma_f32_32x32x8f16(a4, a4, c16[q], 0, 0, 0);
            if constexpr (KIND == 1) c16[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a8, a8, c16[q], 0, 0, 0);
            if constexpr (KIND == 2) c4[q] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, c4[q], 0, 0, 0);
            if constexpr (KIND == 3) c4[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, c4[q], 0, 0, 0);
            if constexpr (KIND == 4) c32[q] = __builtin_amdgcn_mfma_f32_32x32x4f16(a4, a4, c32[q], 0, 0, 0);
            if constexpr (KIND == 5) c16[q] = __builtin_amdgcn_mfma_f32_16x16x4f16(a4, a4, c16[q], 0, 0, 0);
            if constexpr (KIND == 6) c4[q] = __builtin_amdgcn_mfma_f32_4x4x4f16(a4, a4, c4[q], 0, 0, 0);
            if constexpr (KIND == 7) c32[q] = __builtin_amdgcn_mfma_f32_32x32x1f32(fa, fa, c32[q], 0, 0, 0);
            if constexpr (KIND == 8) c16[q] = __builtin_amdgcn_mfma_f32_16x16x1f32(fa, fa, c16[q], 0, 0, 0);
            if constexpr (KIND == 9) c16[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa, fa, c16[q], 0, 0, 0);
            if constexpr (KIND == 10) c4[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(fa, fa, c4[q], 0, 0, 0);
            if constexpr (KIND == 11) c4[q] = __builtin_amdgcn_mfma_f32_4x4x1f32(fa, fa, c4[q], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        for (int i = 0; i < 16; ++i) s += c16[q][i];
        for (int i = 0; i < 32; ++i) s += c32[q][i];
        for (int i = 0; i < 4; ++i) s += c4[q][i];
    }
    out[blockIdx.x * blockDim.x + l] = s;
    if (l == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND>
static void run(const char * name, float * out, unsigned long long * cyc, int waves) {
    hipLaunchKernelGGL(k_mfma<KIND>, dim3(1), dim3(64 * waves), 0, 0, out, cyc);
    hipLaunchKernelGGL(k_mfma<KIND>, dim3(1), dim3(64 * waves), 0, 0, out, cyc);
    unsigned long long h = 0;
    hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-28s waves %d: %6.1f ticks per instruction\n", name, waves, (double) h / (N_IT * 4));
}

int main() {
    float * out; unsigned long long * cyc;
    hipMalloc(&out, 64 * 64 * 4); hipMalloc(&cyc, 64 * 8);
    for (int w : {1, 4}) {
        run<0>("32x32x8 f16", out, cyc, w);
        run<1>("32x32x16 f16", out, cyc, w);
        run<2>("16x16x16 f16", out, cyc, w);
        run<3>("16x16x32 f16", out, cyc, w);
        run<4>("32x32x4 2b f16", out, cyc, w);
        run<5>("16x16x4 4b f16", out, cyc, w);
        run<6>("4x4x4 16b f16", out, cyc, w);
        run<7>("32x32x1 2b f32", out, cyc, w);
        run<8>("16x16x1 4b f32", out, cyc, w);
        run<9>("32x32x2 f32", out, cyc, w);
        run<10>("16x16x4 f32", out, cyc, w);
        run<11>("4x4x1 16b f32", out, cyc, w);
    }
    return 0;
}
