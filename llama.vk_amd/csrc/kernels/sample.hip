// sample.hip -- the device half of llama_sample_top_p_top_k (llama.cpp:1356-1459).
//
// The reference builds (logit * scale [* or / repeat_penalty], id) for every vocabulary
// entry, std::partial_sort's the top k by value, then runs a softmax, the top-p cut and
// std::discrete_distribution over those k on the host.  Here one workgroup does the
// O(n_vocab) part on the logits in HBM -- the repeat-penalty flags (an LDS bitmap of the
// last-n ids, instead of a std::find per logit), the scaled values with the reference's
// float operation order, and a 4-pass 8-bit radix select of the k-th largest value -- and
// writes every candidate whose value is >= that k-th value (ties and +-0 included) to
// host-mapped memory.  The host sorts the <= cap candidates; when all their values are
// distinct the descending order is exactly partial_sort's, so the rest of the reference
// (expf, double sums, top-p, the RNG draw) runs unchanged on the host over k values.
// Ties, NaNs or more candidates than the cap are flagged and the caller falls back to the
// reference path over all logits (so the result is the reference's in every case).
#include "lvk_device.h"
#include "lvk_kernels.h"

namespace lvk {

namespace {

constexpr int ST = 1024;                          // threads (one workgroup)
constexpr int PER = (SAMPLE_MAX_VOCAB + ST - 1) / ST;

// float -> unsigned key with the same order (-0 sorts below +0; NaN never reaches here)
__device__ __forceinline__ unsigned fkey(float v) {
    const unsigned u = __float_as_uint(v);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float keyf(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

__global__ __launch_bounds__(ST) void k_sample_cand(const float * __restrict__ x, int n,
                                                    const SampleParams * __restrict__ P, SampleOut * out) {
    __shared__ unsigned bits[SAMPLE_MAX_VOCAB / 32];
    __shared__ unsigned hist[256];
    __shared__ unsigned s_prefix, s_rem, s_count, s_flags;
    const int tid = threadIdx.x;
    for (int i = tid; i < (n + 31) / 32; i += ST) bits[i] = 0u;
    if (tid == 0) { s_prefix = 0u; s_count = 0u; s_flags = 0u; s_rem = (unsigned) P->k; }
    __syncthreads();
    const int nl = P->n_last;
    for (int i = tid; i < nl; i += ST) {
        const int t = P->last[i];
        if (t >= 0 && t < n) atomicOr(&bits[t >> 5], 1u << (t & 31));
    }
    __syncthreads();
    // the reference's values (llama.cpp:1400-1414): plogits[i]*scale, then *rp or /rp
    const float scale = P->scale, rp = P->rp;
    float v[PER];
    unsigned key[PER];
    bool nan = false;
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int i = j * ST + tid;
        float y = 0.0f;
        if (i < n) {
            const float l = x[i];
            const float s = l * scale;
            if ((bits[i >> 5] >> (i & 31)) & 1u) y = l < 0.0f ? s * rp : s / rp;
            else y = s;
            nan |= !(y == y);
        }
        v[j] = y;
        key[j] = i < n ? fkey(y) : 0u;     // key 0 sorts below every real value
    }
    if (nan) atomicOr(&s_flags, SAMPLE_FLAG_NAN);
    // radix select of the k-th largest key, 8 bits per pass from the top
    unsigned mask = 0u;
#pragma unroll 1
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int b = tid; b < 256; b += ST) hist[b] = 0u;
        __syncthreads();
        const unsigned pre = s_prefix;
#pragma unroll
        for (int j = 0; j < PER; ++j)
            if (j * ST + tid < n && (key[j] & mask) == pre) atomicAdd(&hist[(key[j] >> shift) & 255u], 1u);
        __syncthreads();
        if (tid == 0) {
            unsigned rem = s_rem, b = 255u;
            for (;; --b) {
                if (hist[b] >= rem || b == 0u) break;
                rem -= hist[b];
            }
            s_rem = rem;
            s_prefix = pre | (b << shift);
        }
        mask |= 255u << shift;
        __syncthreads();
    }
    // candidates: every value >= the k-th largest, compared as floats (so a +0 / -0 pair at
    // the boundary both come out and read as a tie on the host)
    const float T = keyf(s_prefix);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
        const int i = j * ST + tid;
        if (i < n && v[j] >= T) {
            const unsigned slot = atomicAdd(&s_count, 1u);
            if (slot < (unsigned) SAMPLE_CAP) { out->val[slot] = v[j]; out->id[slot] = i; }
        }
    }
    __syncthreads();
    if (tid == 0) {
        unsigned f = s_flags;
        if (s_count > (unsigned) SAMPLE_CAP) f |= SAMPLE_FLAG_OVERFLOW;
        out->count = (int) s_count;
        out->flags = (int) f;
    }
}

}  // namespace

hipError_t launch_sample_cand(const float * logits, int n, const SampleParams * P, SampleOut * out, hipStream_t s) {
    if (n <= 0 || n > SAMPLE_MAX_VOCAB) return hipErrorInvalidValue;
    LVK_LAUNCH(k_sample_cand, dim3(1), dim3(ST), 0, s, logits, n, P, out);
    return hipGetLastError();
}

}  // namespace lvk
