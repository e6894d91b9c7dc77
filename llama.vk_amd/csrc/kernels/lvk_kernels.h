// lvk_kernels.h -- host-visible launch interface of the llama.vk_amd HIP kernels.
//
// Every launcher is stream-ordered and capture-safe (no allocation, no sync),
// so the decode step can be recorded into one hipGraph.
#pragma once
#include <cstdlib>
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>

namespace lvk {

// Profiling hook: when a launcher runs with these set (one kernel per timed
// launch), the kernel is dispatched with hipExtLaunchKernelGGL and the two
// events are stamped by the command processor at its start and end -- the
// same interval rocprofv3's kernel trace reports.
struct LaunchEvents {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};
extern thread_local LaunchEvents g_launch_events;
// a launcher of several kernels times them as one: the start event goes to the
// first kernel, the stop event to the last
struct EventSplit {
    LaunchEvents saved = g_launch_events;
    void first() { g_launch_events = {saved.start, nullptr}; }
    void last() { g_launch_events = {nullptr, saved.stop}; }
    ~EventSplit() { g_launch_events = saved; }
};

#define LVK_LAUNCH(kern, grid, block, lds, stream, ...)                                                        \
    do {                                                                                                       \
        if (::lvk::g_launch_events.start || ::lvk::g_launch_events.stop)                                  \
            hipExtLaunchKernelGGL(kern, grid, block, lds, stream, ::lvk::g_launch_events.start,                \
                                  ::lvk::g_launch_events.stop, 0, __VA_ARGS__);                                \
        else                                                                                                   \
            hipLaunchKernelGGL(kern, grid, block, lds, stream, __VA_ARGS__);                                   \
    } while (0)

enum QType : int { Q4_0 = 2, Q4_1 = 3 };

// error word: kernels whose workgroups wait on each other spin with a bound; a
// spin that gives up stores one of these into the context's host-mapped error
// word (system scope) instead of hanging, and the host fails the eval
enum DevError : unsigned { LVK_ERR_NONE = 0, LVK_ERR_ATTN_SPIN = 1, LVK_ERR_DECODE_SPIN = 2 };

// ---------------------------------------------------------------------------
// Device weight image of one quantized matrix W[M][K] (ggml row-major, K = row
// length) in the "octet" layout: rows are grouped 8 per
// wavefront; lane l = 8*r + j owns row r of the group and the AVX2 accumulator
// chain j of the reference dot product (ggml.c:1950-2026).  NC = ceil(K/1024).
//   nib : [M/8][NC][4][64] uint4   -- nibble slices of 8 blocks per uint4
//   scl : [M/8][NC][64]   float4  -- d of blocks 32c+8m+j, m = 0..3
// Bytes per row equal the file's (20 B per 32 weights; the last chunk of a
// row is zero-padded to 32 blocks when K % 1024 != 0 and never streamed).
struct QMatrix {
    int qtype = Q4_0;
    int M = 0, K = 0;
    const uint4 * nib = nullptr;
    const void * scl = nullptr;
    // optional f16 A-fragment image for the prompt matmul (launch_build_a16): 4x the
    // weight bytes, saves the nibble unpack in k_mm_q40_mfma; nullptr = unpack path
    const void * a16 = nullptr;
    // Q4_1 only: the prompt matmul's per-block side image (launch_build_mm41: weight
    // sums + d / m per lane); with a16 it enables the Q4_1 MFMA path (mm_mfma41.hip)
    const void * side = nullptr;
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
// serves every position): written by a 16-byte H2D copy before each step, or advanced
// on the device by k_argmax_step in a chained greedy decode.
struct StepParams {
    int n_past;
    int n_tokens;
    int pad0;       // the token of a single-token eval (read by the embedding kernel)
    unsigned seq;   // decode step counter: the decode attention's granule epochs are
                    // (seq << 7) + layer + 1, so the granules need no zeroing per token
};

struct RopeTable {            // host-built with glibc powf/cosf/sinf (ggml.c:7209-7213)
    const float2 * cs;        // [n_ctx][hd/2] {cos, sin}
};

// prologue (how the matvec obtains its quantized input)
enum Pro : int { PRO_NORM = 0, PRO_ACTQ = 1, PRO_ACTF = 2 /* f32 input, quantize only */ };
// epilogue (what it does with row results)
enum Epi : int { EPI_STORE = 0, EPI_RESID = 1, EPI_QKV = 2, EPI_SWIGLU = 3, EPI_SWIGLU_F32 = 4, EPI_ROPE_KV = 5, EPI_SWIGLU_Q = 6 };

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
    int kv32 = 0;                    // f32 KV cache and f32 queries (f16_kv = false)
    // EPI_SWIGLU
    const uint16_t * silu_tab = nullptr;   // 64Ki fp16 table
    ActQ out_q;                            // quantized u = silu(w1 x) * (w3 x)
    float * u = nullptr;                   // EPI_SWIGLU_F32: u in f32 [N][M/2]
};

hipError_t launch_matvec(const MvLaunch & L, int pro, int epi, hipStream_t s);
// the same for Q4_1 weights (matvec_q41.hip); launch_matvec forwards here
hipError_t launch_matvec_q41(const MvLaunch & L, int pro, int epi, hipStream_t s);

// single-token decode matvec, one workgroup per CU (matvec_cu.hip for Q4_0,
// matvec_cu41.hip for Q4_1).  Row lengths compiled in: matvec_cu_supported(K, qtype).
// Returns hipErrorNotSupported for anything else (the caller then uses launch_matvec).
bool matvec_cu_supported(int K, int qtype = Q4_0);
hipError_t launch_matvec_cu(const MvLaunch & L, int pro, int epi, hipStream_t s);
bool matvec_cu41_supported(int K);
hipError_t launch_matvec_cu41(const MvLaunch & L, int pro, int epi, hipStream_t s);
// compute units of the current device (one decode workgroup per CU)
int cu_count();

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
    int exp_computed = 0;     // exp mode (lvk_device.h exp_f16): 0 table, 1 double, 2 f32 -- nonzero only after exp_check
    unsigned * err = nullptr; // host-mapped error word (DevError); kernels that spin report a timeout here
    int kv32 = 0;             // f32 K, V and queries (f16_kv = false): launch_attention only
    int seq_epochs = 0;       // decode attention: granule epoch = (sp->seq << 7) + epoch (no per-token zeroing)
};
hipError_t launch_attention(const AttnLaunch & A, hipStream_t s);
// prompt batches (N > 1, Q4_0 / Q4_1 output): scores+softmax per (head, 32 tokens) then
// P.V per (head, 32 tokens, 32 dims) with the Wo quantization fused
// (attention_prompt.hip).  p_scratch: H*N*n_ctx f16; optional: also write the Wo
// input as the MFMA operands -- Q4_0 xm/xda (mm_mfma.hip), Q4_1 xm/xs41 (mm_mfma41.hip).
bool attention_prompt_supported(int n_embd, int n_head, int n_ctx);
hipError_t launch_attention_prompt(const AttnLaunch & A, uint16_t * p_scratch, void * xm, float * xda,
                                   hipStream_t s, void * xs41 = nullptr);
// count into bad_d[0] / bad_d[1] the softmax arguments h <= 0 whose exp computed in
// double / with the device expf differs from exp_tab[h]; 0 means that mode
// reproduces the host table exactly
hipError_t exp_check(const uint16_t * exp_tab, int * bad_d, hipStream_t s);
// single-token attention, 4 workgroups per head in one launch (attention_decode.hip):
// the head's scores are exchanged through `gran` (attention_decode_scratch_bytes, zeroed
// at allocation) tagged with `epoch` (layer + 1, never 0) + (sp->seq << 7) when
// A.seq_epochs is set (else the scratch must be zeroed before every token).  Needs
// A.n_tokens == 1.
bool attention_decode_supported(int n_embd, int n_head, int n_ctx);
size_t attention_decode_scratch_bytes(int n_head, int n_ctx);
hipError_t launch_attention_decode(const AttnLaunch & A, void * gran, unsigned epoch, hipStream_t s);

// one-time weight repack: file-layout rows (ggml blocks) -> quad-sliced image
// interleave4: src_rows holds two (M/2)-row matrices A then B; the image
// interleaves them per 4 rows (A0-3, B0-3, A4-7, ...: the fused W1|W3)
hipError_t launch_repack(const void * src_rows, int qtype, int M, int K, uint4 * nib, void * scl,
                         hipStream_t s, int interleave4 = 0);
// bytes of the two image arrays for an M x K matrix
inline size_t qimage_nib_bytes(int M, int K) { return (size_t) M * ((K / 32 + 31) / 32) * 512; }
// Q4_1: d and m images, then the even-chain weight-sum image (q41_wsum)
inline size_t qimage_scl_bytes(int M, int K, int qtype = Q4_0) {
    return (size_t) M * ((K / 32 + 31) / 32) * 128 * (qtype == Q4_1 ? 3 : 1);
}
// Q4_1 weight sums, precomputed at repack: the AVX2 dot's `sums` term for the even
// chains (ggml.c:2236-2240, _mm256_sad_epu8 of the weight bytes 8k..8k+7 = the nibbles
// of qs[4k..4k+3], chain 2k) as one byte per block.  wsum[g][c][8r+j] (uint4): chain
// 2(j/2) of row 8g+r, blocks 32c + 16(j%2) .. +15 of the chunk, byte t = block +t.
inline const uint4 * q41_wsum(const QMatrix & w) {
    return (const uint4 *) ((const char *) w.scl + (size_t) w.M * ((w.K / 32 + 31) / 32) * 256);
}

// prompt-eval (N > 1) Q4_0 matmul on the MFMA cores (mm_mfma.hip), bit-exact
// like launch_matvec: the matrix cores produce the per-chain integer partials,
// the VALU runs the reference fp32 chains.  Input: the masked B fragment image
// xm (mm_act_bytes(N, K) bytes, ZEROED once at allocation: only the active
// slots are ever written) + da [N][K/32], from launch_act_f16 /
// launch_actq_to_f16.  epi: EPI_STORE, EPI_RESID (y += W x), EPI_SWIGLU_F32
// (fused W1|W3 image -> u = silu(w1 x) * (w3 x)).
bool mm_mfma_supported(const QMatrix & w);
// prompt-matmul tile order: 1 = super tiles of 4 row tiles (default), 0 = row tiles
// (LVK_MM_SUPERTILE; device/lvk_device.h mm_tile)
int mm_supertile();
size_t mm_act_bytes(int N, int K);
// the f16 A-fragment image of a Q4_0 matrix (QMatrix::a16): bytes, and its build from the
// matrix's octet image (M % 32 == 0)
size_t mm_a16_bytes(int M, int K);
hipError_t launch_build_a16(const QMatrix & w, void * a16, hipStream_t s);
// LVK_PROMPT_A16=0 keeps the prompt matmul on the nibble image (no f16 A image)
inline bool prompt_a16_env() {
    const char * e = getenv("LVK_PROMPT_A16");
    return !e || atoi(e) != 0;
}
// LVK_PROMPT_A16=1: build the Q4_0 images whenever they fit; unset: by capacity (lvk_model.cpp)
inline bool prompt_a16_forced() {
    const char * e = getenv("LVK_PROMPT_A16");
    return e && atoi(e) == 1;
}
hipError_t launch_mm_mfma(const QMatrix & w, const void * xm, const float * da, int N, float * y, int ldy,
                          int out_tok0, int epi, const uint16_t * silu_tab, hipStream_t s);
// x[N][K] (rms_norm * g when g != nullptr) -> quantize_row_q4_0 -> xm, da
hipError_t launch_act_f16(const float * x, const float * g, int N, int K, void * xm, float * da, hipStream_t s);
hipError_t launch_actq_to_f16(const ActQ & q, int N, int K, void * xm, float * da, hipStream_t s);
// the Q4_1 prompt matmul (mm_mfma41.hip), bit-exact like launch_matvec: the matrix
// cores produce the chain partials, the cross-term sums and the scale products, the
// VALU runs ggml_vec_dot_q4_1's fp32 chains.  Weights: QMatrix::a16 (mm_a16_bytes, f16
// q values) + QMatrix::side (mm41_side_bytes), both from launch_build_mm41.  Tokens: the
// masked fragment image xm (mm_act_bytes, ZEROED once at allocation) + the side image
// xs (mm41_act_side_bytes), from launch_act41_f16 / launch_actq41_to_f16.
size_t mm41_side_bytes(int M, int K);
size_t mm41_act_side_bytes(int N, int K);
hipError_t launch_build_mm41(const QMatrix & w, void * a16, void * side, hipStream_t s);
bool mm_mfma41_supported(const QMatrix & w);
struct RopeKV;
hipError_t launch_mm_mfma41(const QMatrix & w, const void * xm, const void * xs, int N, float * y, int ldy, int epi,
                            const uint16_t * silu_tab, hipStream_t s, const RopeKV * rk = nullptr);   // rk: EPI_ROPE_KV
hipError_t launch_act41_f16(const float * x, const float * g, int N, int K, void * xm, void * xs, hipStream_t s);
hipError_t launch_actq41_to_f16(const ActQ & q, int N, int K, void * xm, void * xs, hipStream_t s);
// the prompt QKV matmul with RoPE + KV append in its epilogue (Q4_0, f16 KV cache): the
// f32 Q|K|V rows never reach memory; q16 / kc / vc get exactly what launch_rope_kv writes
struct RopeKV {
    const float2 * rope;       // [n_ctx][hd/2] cos, sin
    const StepParams * sp;     // n_past
    int n_ctx, E, hd;
    uint16_t * q16, * kc, * vc;
};
hipError_t launch_mm_qkv_rope(const QMatrix & w, const void * xm, const float * da, int N, const RopeKV & r, hipStream_t s);
// the prompt W1|W3 matmul (Q4_0) with SwiGLU and the W2 input's quantize_row_q4_0 in its
// epilogue: writes the masked fragment image xq (mm_act_bytes(N, M/2), zeroed once) + xqda
// directly, as launch_act_f16(silu(w1 x) * w3 x, nullptr, ...) would
hipError_t launch_mm_w13_q(const QMatrix & w, const void * xm, const float * da, int N, const uint16_t * silu_tab,
                           void * xq, float * xqda, hipStream_t s);
// RoPE + KV append of stored Q|K|V rows qkv [N][3E]
hipError_t launch_rope_kv(const float * qkv, int N, int E, int hd, const float2 * rope, const StepParams * sp,
                          int n_ctx, uint16_t * q16, uint16_t * kc, uint16_t * vc, hipStream_t s, int kv32 = 0);

// operator-level helpers used by the C ABI tests
hipError_t launch_quantize_act(const float * x, int N, int K, int qtype, ActQ out, hipStream_t s);
// the reference's scalar quantize_row_q4_0/1_reference (roundf, id = 1/d)
hipError_t launch_quantize_ref(const float * x, int N, int K, int qtype, ActQ out, hipStream_t s);

}  // namespace lvk

namespace lvk {
// device half of llama_sample_top_p_top_k (sample.hip): repeat penalty + temperature on the
// logits in HBM, radix select of the k-th largest value, every value >= it written to out
// (host-mapped).  SampleParams lives in device memory (one H2D copy per step).
constexpr int SAMPLE_MAX_VOCAB = 32768;   // values per thread kept in registers
constexpr int SAMPLE_CAP = 1024;          // candidates the host can receive (k <= this)
constexpr int SAMPLE_MAX_LAST = 1024;     // last-n window entries
enum SampleFlags : int { SAMPLE_FLAG_NAN = 1, SAMPLE_FLAG_OVERFLOW = 2 };
struct SampleParams {
    int k;                    // top_k (1..SAMPLE_CAP)
    int n_last;               // entries of last[]
    float scale;              // 1.0f / temp
    float rp;                 // repeat_penalty
    int last[SAMPLE_MAX_LAST];
};
struct SampleOut {
    int count;                // candidates (values >= the k-th largest)
    int flags;                // SampleFlags
    int pad[2];
    float val[SAMPLE_CAP];
    int id[SAMPLE_CAP];
};
hipError_t launch_sample_cand(const float * logits, int n, const SampleParams * P, SampleOut * out, hipStream_t s);

// y[t] = g * rms_norm(x[t]) as f32 (the embeddings output, llama.cpp:1117-1124)
hipError_t launch_rmsnorm_rows(const float * x, const float * g, int K, int n, float * y, hipStream_t s);
// greedy argmax over x[0..n) with the reference's first-maximum rule (llama.cpp:1382-1394); *out on the device
// (out2, optional: a second copy of the token, e.g. host-mapped memory)
hipError_t launch_argmax(const float * x, int n, int * out, hipStream_t s, int * out2 = nullptr);
// one chained decode step's tail (lvk_decode_chain): the same argmax into chain[CHAIN_HDR + i]
// (chain[0] = i counts the steps), the logits digest into digest[i] when chain[2] != 0, the next
// token (forced[i + 1] while i + 1 < chain[1], else the argmax) into the step block (n_past + 1,
// token, seq + 1) and its embedding row (launch_embed's) into x[0..n_embd)
constexpr int CHAIN_HDR = 4;
hipError_t launch_argmax_step(const float * logits, int n, StepParams * sp, int * chain, const int * forced,
                              unsigned long long * digest, const void * emb, int emb_type, int n_embd, float * x,
                              hipStream_t s);

// ---------------------------------------------------------------------------
// ggml graph operators (graph_ops.hip; include/ggml.h via runtime/ggml_graph.cpp): one
// node per launch on a strided 4-D view of a device buffer
enum GType : int { GT_Q4_0 = 0, GT_Q4_1 = 1, GT_I32 = 4, GT_F16 = 5, GT_F32 = 6 };   // = enum ggml_type
enum GOp : int { GOP_ADD = 0, GOP_SUB, GOP_MUL, GOP_DIV, GOP_REPEAT, GOP_SCALE, GOP_SILU, GOP_DIAG_MASK };
struct GView {
    char * p = nullptr;
    int64_t ne[4] = {1, 1, 1, 1};
    int64_t nb[4] = {0, 0, 0, 0};
    int type = GT_F32;
};
hipError_t launch_g_cpy(const GView & s, const GView & d, hipStream_t st);
hipError_t launch_g_binary(const GView & a, const GView & b, const GView & d, int op, hipStream_t st);
hipError_t launch_g_unary(const GView & s, const GView & d, int op, float v, int n_past, const uint16_t * tab,
                          hipStream_t st);
hipError_t launch_g_rms_norm(const GView & s, const GView & d, hipStream_t st);
hipError_t launch_g_soft_max(const GView & d, const uint16_t * exp_tab, int exp_mode, hipStream_t st);
hipError_t launch_g_rope(const GView & s, const GView & d, const float2 * cs, int n_dims, int i2_0, hipStream_t st);
hipError_t launch_g_get_rows(const GView & s, const int32_t * idx, int64_t n_rows, const GView & d, hipStream_t st);
// y: contiguous rows (f16 when s0 is f16, else f32) [ne13][ne12][ne11][ne00]
hipError_t launch_g_mm_dot(const GView & s0, const void * y, int64_t ne11, const GView & d, hipStream_t st);

}  // namespace lvk
