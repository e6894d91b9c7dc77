// lvk_context.h -- one inference context: device KV cache, scratch, the
// launch sequence of llama_eval on a HIP stream and the captured decode graph.
#pragma once
#include "lvk_model.h"

#include <array>
#include <chrono>
#include <functional>
#include <memory>
#include <new>

struct llama_context_params;

namespace lvk {

struct Split;       // lvk_split.h
struct StageLink;
struct SplitDel { void operator()(Split * p) const; };
struct StageLinkDel { void operator()(StageLink * p) const; };

// kernel classes timed by the profiler (events around every launch of a class)
enum KClass : int { K_EMBED = 0, K_QKV, K_ATTN, K_WO, K_W13, K_W2, K_LMHEAD, K_NCLASS };

// page-locked host storage: the per-token logits D2H copy runs as one DMA instead of
// being staged through a driver bounce buffer
template <class T>
struct PinnedAlloc {
    using value_type = T;
    PinnedAlloc() = default;
    template <class U>
    PinnedAlloc(const PinnedAlloc<U> &) {}
    T * allocate(size_t n) {
        void * p = nullptr;
        if (hipHostMalloc(&p, n * sizeof(T), hipHostMallocDefault) != hipSuccess) throw std::bad_alloc();
        return (T *) p;
    }
    void deallocate(T * p, size_t) { (void) hipHostFree(p); }
    template <class U>
    bool operator==(const PinnedAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const PinnedAlloc<U> &) const { return false; }
};

struct Profile {
    std::array<double, K_NCLASS> ms{};       // accumulated device time
    std::array<long, K_NCLASS> launches{};   // launches accumulated
    std::array<double, K_NCLASS> bytes{};    // algorithmic HBM bytes accumulated
};

// one slice of an eval call: a whole llama_eval, or one micro-batch of a prompt that a
// layer split pipelines through its stages (lvk_split.cpp)
struct EvalPart {
    int tok_off = 0;      // first token of this slice within the call
    int n_total = -1;     // tokens of the whole call (-1: this slice is the call)
    bool head = true;     // run norm + lm_head (last stage: the call's last slice, or logits_all)
    bool copy_out = true; // copy logits / embedding / the greedy token to the host after this slice
    bool greedy = false;  // end in the device argmax (lvk_eval_greedy) instead of the logits D2H
    bool sample = false;  // end in the device top-k candidates (lvk_eval_sample) instead of the logits D2H
};

struct Context {
    Model model;
    int n_ctx = 512;             // allocated positions (the caller's n_ctx rounded up to 32, >= 128)
    int n_ctx_user = 512;        // llama_context_params.n_ctx: the positions an eval may use
    bool logits_all = false;
    bool want_embedding = false;
    hipStream_t stream = nullptr;

    // device state
    uint16_t * kc = nullptr;     // [L][n_ctx][E] f16, or f32 when kv32
    uint16_t * vc = nullptr;     // [L][E][n_ctx] f16, or f32 when kv32
    bool kv32 = false;           // f32 KV cache and queries (llama_context_params.f16_kv = false)
    size_t kv_elem_bytes() const { return kv32 ? 4 : 2; }
    uint16_t * kc_layer(size_t il) const { return kc + il * (size_t) n_ctx * model.hp.n_embd * (kv_elem_bytes() / 2); }
    uint16_t * vc_layer(size_t il) const { return vc + il * (size_t) n_ctx * model.hp.n_embd * (kv_elem_bytes() / 2); }
    float * x = nullptr;         // residual stream [n_ctx][E]
    uint16_t * q16 = nullptr;    // [n_ctx][E]
    float * scores = nullptr;    // [n_ctx][H][n_ctx]
    ActQ aq_attn;                // [n_ctx][E/32]
    ActQ aq_ffn;                 // [n_ctx][F/32]
    float * u_ffn = nullptr;     // [F] decode: silu(w1 x) * (w3 x) in f32
    float * logits_d = nullptr;  // [n_ctx][V]
    float * emb_d = nullptr;     // [E]
    uint16_t * exp_tab = nullptr;
    int exp_computed = 0;     // softmax exp mode (exp_f16: 0 table, 1 double, 2 f32; verified equal to exp_tab)
    uint16_t * silu_tab = nullptr;
    float2 * rope = nullptr;     // [n_ctx][hd/2]
    StepParams * sp_d = nullptr;
    int * tok_d = nullptr;       // [n_ctx]
    StepParams * sp_h = nullptr; // pinned, [1 + n_ctx] step blocks: [0] for the graphs, the
    int sp_next = 1;             //   rest one per eager slice enqueued before the next sync
    int * tok_h = nullptr;       // pinned [n_ctx]
    unsigned * err_h = nullptr;  // pinned, mapped: the kernels' error word (lvk_kernels.h DevError)
    unsigned * err_d = nullptr;  // its device address
    int device = 0;              // the HIP device of this context
    std::unique_ptr<StageLink, StageLinkDel> link;   // one-stage-per-process link (lvk_stage_connect[_shm])

    // prompt (N > 1) path: MFMA matmuls with exact block dots (default) or the
    // bit-faithful VALU kernels (prompt_exact; env LVK_PROMPT_EXACT=1)
    bool prompt_exact = false;
    bool old_attention = false;  // env LVK_ATTN_V1=1: single-token evals on the one-kernel attention.hip
    void * attn_gran = nullptr;  // [H][n_ctx] {tag, score} granules of the decode attention
    uint16_t * xh = nullptr;     // masked MFMA B-fragment image of the quantized activations (mm_act_bytes)
    float * xda = nullptr;       // [Cpad][max(E,F)/32] their block scales
    // Q4_0 prompt: the W2 input image written by the W1|W3 epilogue (EPI_SWIGLU_Q; the W1|W3
    // launch still reads xh); LVK_MM_SWIGLU_Q=0: f32 uf + k_act_q40_f16_tile instead
    uint16_t * xh2 = nullptr;
    float * xda2 = nullptr;
    void * xside = nullptr;      // Q4_1: the activations' side image (mm41_act_side_bytes)
    float * qkv32 = nullptr;     // [C][3E] Q|K|V rows before RoPE (f32-KV prompts, LVK_MM_ROPE=0)
    // prompt: RoPE + KV append fused into the QKV matmul (LVK_MM_ROPE=0: separate kernel)
    bool mm_rope_fused = [] { const char * e = getenv("LVK_MM_ROPE"); return !e || atoi(e) != 0; }();
    float * uf = nullptr;        // [C][F] silu(w1 x) * (w3 x)

    // decode graph (N = 1, last-token logits)
    hipGraph_t graph = nullptr;
    hipGraphExec_t graph_exec = nullptr;
    bool use_graph = true;
    // greedy decode graph (lvk_eval_greedy): argmax on the device, 4-byte D2H instead of the logits row
    hipGraph_t graph_greedy = nullptr;
    hipGraphExec_t graph_greedy_exec = nullptr;
    // sampling decode graph (lvk_eval_sample): the sampler block H2D, the forward pass and the
    // device top-k candidates (sample.hip) into host-mapped memory instead of the logits row
    hipGraph_t graph_sample = nullptr;
    hipGraphExec_t graph_sample_exec = nullptr;
    SampleParams * samp_h = nullptr;   // pinned host block, filled per call
    SampleParams * samp_d = nullptr;
    SampleOut * sout_h = nullptr;      // host-mapped candidates
    SampleOut * sout_d = nullptr;      // its device address
    // one single-token eval + the device half of the sampler (samp_h filled by the caller);
    // the candidates are in *sout_h afterwards
    void eval_sample(int token, int n_past);
    // the last eval's last-token logits row -> host logits (llama_get_logits valid again)
    void fetch_logits();
    int n_sample_fallback = 0;         // lvk_eval_sample calls that took the all-logits host path
    int * greedy_d = nullptr;
    int * greedy_h = nullptr;    // host-mapped (coherent): the device argmax writes it
    int * greedy_hd = nullptr;   // its device address
    void enqueue_argmax();
    // chained greedy decode (lvk_decode_greedy): one graph per step that reads nothing from
    // the host -- its last kernel (k_argmax_step) picks the token, advances the step block
    // on the device and writes the next step's embedding row -- replayed n times per call
    hipGraph_t graph_chain = nullptr;
    hipGraphExec_t graph_chain_exec = nullptr;
    int * chain_d = nullptr;     // [CHAIN_HDR + n_ctx]: step counter, forced count, digest flag, pad; the argmax tokens
    int * chain_h = nullptr;     // pinned copy of the tokens
    int * chain_ctl_h = nullptr; // pinned header block (CHAIN_HDR ints)
    int * forced_d = nullptr;    // [n_ctx] teacher-forced tokens of a chained decode
    int * forced_h = nullptr;    // pinned staging of them
    unsigned long long * digest_d = nullptr;   // [n_ctx] per-step logits digests
    unsigned long long * digest_h = nullptr;   // pinned copy
    int decode_chain(const int * tokens, int n_tokens, int n_past, int n_steps, int * out, unsigned long long * digests);
    // decode attention granule epochs from the step counter (StepParams::seq): no zeroing per
    // token (off for models with more than 126 layers)
    bool seq_epochs = false;
    unsigned seq = 0;            // the last step counter handed to the device
    unsigned next_seq(unsigned k = 1);

    // host-visible results
    std::vector<float, PinnedAlloc<float>> logits;
    bool logits_valid = false;   // false after lvk_eval_greedy (host logits not refreshed) or a failed eval
    std::vector<float> embedding;
    std::vector<uint8_t> kv_host;
    int kv_n = 0;
    std::mt19937 rng;

    // timings (llama.cpp:1186-1195)
    int64_t t_start_us = 0, t_load_us = 0, t_sample_us = 0, t_eval_us = 0, t_p_eval_us = 0;
    int n_sample = 0, n_eval = 0, n_p_eval = 0;
    bool has_evaluated_once = false;

    // profiling
    bool profiling = false;
    Profile prof;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
    std::vector<int> ev_class;
    size_t ev_used = 0;

    ~Context();
    void init(const llama_context_params & p);
    void eval(const int * tokens, int n, int n_past);
    // eval = begin_eval (everything enqueued on `stream`, no host wait) + end_eval (sync,
    // profile, device error word); a layer split interleaves the stages' begin_evals
    // with the residual-stream hand-offs and ends them together
    void begin_eval(const int * tokens, int n, int n_past, const EvalPart & part);
    void begin_eval_safe(const int * tokens, int n, int n_past, const EvalPart & part);
    void end_eval(bool no_host_logits);
    // stage boundary: copy the residual stream x [n][E] to (to_ctx) or from the context
    void x_copy(void * buf, int n, bool to_ctx, bool on_device);
    void enqueue_forward(int n, bool last_only, const int * tok_src = nullptr, int logit_row = 0, bool head = true,
                         bool embed = true);
    bool use_mfma(int n) const;
    void build_graph(int kind = 0);      // 0 logits, 1 greedy, 2 sample, 3 chained greedy step
    int eval_greedy(int token, int n_past);
    void kv_get();
    void kv_set(const uint8_t * src, size_t n);
    void kv_copy_from(const Context & src, int n_tokens);
    size_t kv_bytes() const;
    void timed_launch(int cls, double bytes, const std::function<hipError_t()> & fn);
    void collect_profile();
    // after a stream sync: throw if a kernel raised the error word (and clear it)
    void check_device_error();
};

int64_t now_us();
// exp mode of the softmax kernels (lvk_device.h exp_f16): 2, 1 or 0 after a device self-check
int pick_exp_mode(const uint16_t * exp_tab_d);
// fp16 exp / silu tables (ggml.c:2915-2927) built with this host's glibc expf
void host_fp16_tables(std::vector<uint16_t> & exp_tab, std::vector<uint16_t> & silu_tab);

}  // namespace lvk

// the opaque handle of the C API (include/llama.h)
struct llama_context {
    lvk::Context c;                                  // the whole model, or the last stage of a split
    std::unique_ptr<lvk::Split, lvk::SplitDel> split;   // layer split over devices (lvk_split.h)
    std::shared_ptr<void> tensor_map;                // llama_internal_get_tensor_map's state (on first use)
    // every stage context in layer order (just &c without a split)
    std::vector<lvk::Context *> stages();
};
