// kp_probe.hip -- dev probe: does kernel-argument preloading shorten a dependent launch chain?
//
// Every decode launch starts with an s_load of its kernel arguments (the CuParams struct) before
// its first weight or input load can be addressed.  gfx950 can preload leading scalar arguments
// into SGPRs (LLVM -amdgpu-kernarg-preload-count; the code object carries a 256-byte preamble
// that loads them the old way, which preload-capable firmware skips).  A by-value struct is not
// preloaded.  This probe times hipGraphs of 160 dependent launches (a 7B token's matvec launch
// count) of the same small body in three forms:
//   struct : k_body_struct(Args a)                      -- the library's form
//   scalar : k_body_scalar(x, w, y, n, ...)             -- leading scalars
// built twice (make kp_probe: without / with -amdgpu-kernarg-preload-count=16).  Each launch:
// 256 workgroups x 256 threads, every wave loads 1 KiB of a 64 MiB buffer (one HBM round trip)
// and one input word written by the previous launch, then writes one word per thread.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

struct Args {
    const float * x;
    const uint4 * w;
    float * y;
    int n;
    int wstride;
    const void * pad[14];       // the library's params are ~150 bytes
};

__device__ __forceinline__ void body(const float * x, const uint4 * w, float * y, int n, int wstride) {
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint4 v = w[(size_t) blockIdx.x * wstride + threadIdx.x];
    const float a = x[tid % n];
    y[tid % n] = a * 0.5f + (float) (v.x & 1u);
}

__global__ __launch_bounds__(256) void k_body_struct(Args a) { body(a.x, a.w, a.y, a.n, a.wstride); }

__global__ __launch_bounds__(256) void k_body_scalar(const float * x, const uint4 * w, float * y, int n, int wstride) {
    body(x, w, y, n, wstride);
}

int main(int argc, char ** argv) {
    const int launches = 160, reps = argc > 1 ? atoi(argv[1]) : 50;
    const int nwg = 256, nt = 256, n = nwg * nt;
    const int wstride = 64 * 1024 / 16;                      // 64 KiB apart per workgroup: 16 MiB touched
    float *x, *y;
    uint4 * w;
    CK(hipMalloc(&x, n * 4)); CK(hipMalloc(&y, n * 4));
    CK(hipMalloc(&w, (size_t) nwg * wstride * 16 * 4));
    CK(hipMemset(x, 0, n * 4)); CK(hipMemset(y, 0, n * 4)); CK(hipMemset(w, 0, (size_t) nwg * wstride * 16 * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int form = 0; form < 2; ++form) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < launches; ++i) {
            // ping-pong x / y so each launch depends on the previous one; w rotates over 4 MiB slices
            const float * in = (i & 1) ? y : x;
            float * out = (i & 1) ? x : y;
            const uint4 * wi = w + (size_t) (i % 4) * wstride / 4;
            if (form == 0) {
                Args a{};
                a.x = in; a.w = wi; a.y = out; a.n = n; a.wstride = wstride;
                hipLaunchKernelGGL(k_body_struct, dim3(nwg), dim3(nt), 0, s, a);
            } else {
                hipLaunchKernelGGL(k_body_scalar, dim3(nwg), dim3(nt), 0, s, in, wi, out, n, wstride);
            }
        }
        CK(hipStreamEndCapture(s, &g));
        hipGraphExec_t ge;
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int i = 0; i < 5; ++i) CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        std::vector<float> per;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0, s));
            CK(hipGraphLaunch(ge, s));
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            per.push_back(ms * 1e3f / launches);
        }
        std::sort(per.begin(), per.end());
        printf("{\"form\": \"%s\", \"us_per_launch_median\": %.3f, \"min\": %.3f, \"max\": %.3f}\n",
               form == 0 ? "struct" : "scalar", per[per.size() / 2], per.front(), per.back());
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    CK(hipStreamDestroy(s));
    return 0;
}
