// lvk_kernels.h -- host-visible launch interface of the llama.vk_amd HIP kernels.
//
// Every launcher is stream-ordered and capture-safe (no allocation, no sync),
// so the decode step can be recorded into one hipGraph.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lvk {

enum QType : int { Q4_0 = 2, Q4_1 = 3 };

// ---------------------------------------------------------------------------
// Device weight image of one quantized matrix W[M][K] (ggml row-major, K = row
// length) in the "quad-sliced" layout:
//   rows are grouped 16 per wavefront; lane l = 4*r + q of the wave owns row r
//   of the group and the two AVX2 accumulator chains j = 2q, 2q+1 of the
//   reference dot product (ggml.c:1950-2026).
//   nib : [M/16][K/256][2][64] uint4   -- nibble slices, 8 blocks per chunk
//   scl : [M/16][K/256][64]   float2  -- Q4_0: d of blocks 8c+q, 8c+4+q
//                                        (Q4_1: float4 {d0,d1,m0,m1})
// Bytes per row equal the file's (20 B / 24 B per 32 weights).
struct QMatrix {
    int qtype = Q4_0;
    int M = 0, K = 0;
    const uint4 * nib = nullptr;
    const void * scl = nullptr;
};

// Activation quantized to the weight format, stored split: d[N][nb] floats,
// m[N][nb] (Q4_1 only), qs[N][nb] uint4 (reference nibble convention).
struct ActQ {
    float * d = nullptr;
    float * m = nullptr;
    uint4 * qs = nullptr;
    int nb = 0;
};

// the runtime scalar block the decode graph reads (so one captured graph
// serves every position): written by a 16-byte H2D copy before each step.
struct StepParams {
    int n_past;
    int n_tokens;
    int pad0, pad1;
};

struct RopeTable {            // host-built with glibc powf/cosf/sinf (ggml.c:7209-7213)
    const float2 * cs;        // [n_ctx][hd/2] {cos, sin}
};

// prologue (how the matvec obtains its quantized input)
enum Pro : int { PRO_NORM = 0, PRO_ACTQ = 1 };
// epilogue (what it does with row results)
enum Epi : int { EPI_STORE = 0, EPI_RESID = 1, EPI_QKV = 2, EPI_SWIGLU = 3 };

struct MvLaunch {
    QMatrix w;
    // input
    const float * x = nullptr;       // PRO_NORM: f32 [N][K]
    const float * g = nullptr;       // PRO_NORM: norm weight [K]
    ActQ xq;                         // PRO_ACTQ: quantized input
    const StepParams * sp = nullptr; // device step params (n_past, n_tokens)
    int n_tokens = 1;                // host-known token count of this launch
    int tok0 = 0;                    // first token row of x / xq to use
    int out_tok0 = 0;                // first output row to write
    // outputs
    float * y = nullptr;             // EPI_STORE: [N][M];  EPI_RESID: residual [N][M] (in place)
    // EPI_QKV
    uint16_t * q16 = nullptr;        // [N][E] f16 (post-rope queries)
    uint16_t * kc = nullptr;         // layer K cache [n_ctx][E]
    uint16_t * vc = nullptr;         // layer V cache [E][n_ctx]
    RopeTable rope{};
    int n_embd = 0, head_dim = 0, n_ctx = 0;
    // EPI_SWIGLU
    const uint16_t * silu_tab = nullptr;   // 64Ki fp16 table
    ActQ out_q;                            // quantized u = silu(w1 x) * (w3 x)
};

hipError_t launch_matvec(const MvLaunch & L, int pro, int epi, hipStream_t s);

// token embedding rows: x[t] = dequant(tok_emb[tokens[t]]) (ggml.c:6868-6895)
hipError_t launch_embed(const void * emb, int emb_type, int n_embd, const int * tokens, int n,
                        float * x, hipStream_t s);

// attention, one layer (llama.cpp:1010-1061)
struct AttnLaunch {
    const uint16_t * q16;     // [N][E]
    const uint16_t * kc;      // [n_ctx][E]
    const uint16_t * vc;      // [E][n_ctx]
    float * scores;           // scratch [N][H][n_ctx]
    ActQ out;                 // quantized attention output (Wo input), Q4_0 or Q4_1
    int out_qtype;
    const uint16_t * exp_tab; // 64Ki fp16 exp table
    const StepParams * sp;
    int n_tokens, n_embd, n_head, n_ctx;
    float * out_f32 = nullptr; // optional: also store the unquantized merged heads [N][E]
    uint16_t * p16_out = nullptr; // optional (debug): f16 probabilities [N][H][n_ctx]
};
hipError_t launch_attention(const AttnLaunch & A, hipStream_t s);

// one-time weight repack: file-layout rows (ggml blocks) -> quad-sliced image
hipError_t launch_repack(const void * src_rows, int qtype, int M, int K, uint4 * nib, void * scl,
                         hipStream_t s);

// operator-level helpers used by the C ABI tests
hipError_t launch_quantize_act(const float * x, int N, int K, int qtype, ActQ out, hipStream_t s);

}  // namespace lvk

namespace lvk {
// y[t] = g * rms_norm(x[t]) as f32 (the embeddings output, llama.cpp:1117-1124)
hipError_t launch_rmsnorm_rows(const float * x, const float * g, int K, int n, float * y, hipStream_t s);
}  // namespace lvk
