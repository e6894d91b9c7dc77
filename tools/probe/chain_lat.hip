// chain_lat: cycles per step of a dependent f32 FMA chain on one wave (the decode matvec's
// per-lane accumulator chain), for v_fma_f32 and v_fma_mix_f32 (f32 x f16 -> f32), with 1, 2 and
// 4 independent chains interleaved in the wave, and with 1 or 2 waves per SIMD.
// Build: make -C tools/probe chain_lat.  Prints cycles (s_memtime) per chain step.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define N_IT 64
#define STEPS 32   // dependent steps per chain per iteration

template <int KIND, int CH>
__global__ __launch_bounds__(512) void k_chain(unsigned long long * cyc, float * out, int nwaves) {
    const int wave = threadIdx.x >> 6;
    if (wave >= nwaves) return;
    float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1.0f, a2 = a0 + 2.0f, a3 = a0 + 3.0f;
    const float s = 1.0000001f, c = 1e-7f;
    const unsigned p = 0x3c003c00u;    // f16 1.0 | 1.0
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < N_IT; ++it) {
#pragma unroll
        for (int k = 0; k < STEPS; ++k) {
            if constexpr (KIND == 0) {
                asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a0) : "v"(s), "v"(c));
                if constexpr (CH > 1) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a1) : "v"(s), "v"(c));
                if constexpr (CH > 2) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a2) : "v"(s), "v"(c));
                if constexpr (CH > 3) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a3) : "v"(s), "v"(c));
            } else {
                asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,0]" : "+v"(a0) : "v"(s), "v"(p));
                if constexpr (CH > 1) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(a1) : "v"(s), "v"(p));
                if constexpr (CH > 2) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,0]" : "+v"(a2) : "v"(s), "v"(p));
                if constexpr (CH > 3) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(a3) : "v"(s), "v"(p));
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 8 + wave] = t1 - t0;
    out[blockIdx.x * 512 + threadIdx.x] = a0 + a1 + a2 + a3;
}

template <int KIND, int CH>
void run(const char * name, unsigned long long * cyc, float * out, int nwaves) {
    // 256 workgroups of 8 waves: one workgroup per CU, `nwaves` of them run (1: one SIMD; 4: one
    // wave per SIMD; 8: two per SIMD)
    hipLaunchKernelGGL((k_chain<KIND, CH>), dim3(256), dim3(512), 0, 0, cyc, out, nwaves);
    hipLaunchKernelGGL((k_chain<KIND, CH>), dim3(256), dim3(512), 0, 0, cyc, out, nwaves);
    hipDeviceSynchronize();
    unsigned long long h[2048];
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double s = 0; int n = 0;
    for (int b = 0; b < 256; ++b) for (int w = 0; w < nwaves; ++w) { s += (double) h[b * 8 + w]; ++n; }
    printf("%-14s chains %d  waves/CU %d: %.2f cycles per chain step (%.2f per instruction)\n", name, CH, nwaves,
           s / n / (N_IT * STEPS), s / n / (N_IT * STEPS * CH));
}

int main() {
    unsigned long long * cyc; float * out;
    hipMalloc(&cyc, 2048 * 8); hipMalloc(&out, 256 * 512 * 4);
    for (int nw : {1, 4, 8}) {
        run<0, 1>("v_fma_f32", cyc, out, nw);
        run<0, 2>("v_fma_f32", cyc, out, nw);
        run<0, 4>("v_fma_f32", cyc, out, nw);
        run<1, 1>("v_fma_mix_f32", cyc, out, nw);
        run<1, 2>("v_fma_mix_f32", cyc, out, nw);
        run<1, 4>("v_fma_mix_f32", cyc, out, nw);
    }
    return 0;
}
