/* include/lvk_ops.h -- operator-level C ABI of llama.vk_amd (secondary boundary).
 *
 * The reference exposes its quantization codecs through quantize_fns_t /
 * ggml_internal_get_quantize_fn (reference ggml.h:803-814, ggml.c:6489-6508)
 * and its ops through the ggml graph API (ggml.h:500-611).  These entry points
 * run the corresponding MI355X kernels on host buffers (H2D, kernel, D2H) so
 * each op can be pinned against the CPU oracle in isolation.  `type` is the
 * ggjt ftype id: 2 = Q4_0, 3 = Q4_1.  All functions return 0 on success and a
 * negative value on failure (message on stderr).
 */
#ifndef LVK_OPS_H
#define LVK_OPS_H

#include <stddef.h>
#include <stdint.h>

#define LVK_API __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

/* number of visible GPUs (0 when none); never fails */
LVK_API int lvk_device_count(void);
/* select the HIP device for subsequent contexts/ops of this host thread (hipSetDevice) */
LVK_API int lvk_set_device(int dev);
/* version string of the library */
LVK_API const char * lvk_version(void);

/* quantize_row_q (ggml.c:621-685 / 847-920): x[n][k] -> n rows of blocks in
 * the reference block layout (20 / 24 bytes per 32 values) */
LVK_API int lvk_quantize_rows(int type, const float * x, int n, int k, void * y);

/* y[t][r] = vec_dot_q(k, w_row r, quantize_row_q(x[t]))  for r < m, t < n
 * (ggml_compute_forward_mul_mat_q_f32, ggml.c:6510-6696).  w: m rows in the
 * file block layout. */
LVK_API int lvk_mul_mat_q(int type, const void * w, int m, int k, const float * x, int n, float * y);

/* same with the fused RMSNorm prologue: y[t][r] = dot(w_r, quant(g * rms_norm(x[t]))) */
LVK_API int lvk_mul_mat_q_norm(int type, const void * w, int m, int k, const float * g, const float * x, int n,
                               float * y);

/* The prompt-batch (N > 1) matmul on the MFMA cores (mm_mfma.hip for Q4_0,
 * mm_mfma41.hip for Q4_1): same inputs and meaning as lvk_mul_mat_q /
 * lvk_mul_mat_q_norm (g != NULL: fused RMSNorm * g), and the same result bits:
 * the matrix cores produce each AVX2 chain's exact 4-element integer partial
 * (Q4_1 also the exact cross-term sums) and the f32 scale products (one rounding
 * each), and the VALU runs the reference's 8 fp32 chains and horizontal order
 * (ggml.c:1950-2026 / 2188-2258).  Needs m % 128 == 0, k % 256 == 0, n >= 1. */
LVK_API int lvk_mul_mat_q_mfma(int type, const void * w, int m, int k, const float * g, const float * x, int n,
                               float * y);

/* one layer's attention block on an f16 KV cache (llama.cpp:1010-1061):
 * kc [n_ctx][n_embd] f16, vc [n_embd][n_ctx] f16, q [n][n_embd] f32 (post-RoPE)
 * -> out [n][n_embd] f32 (merged heads, before the Wo quantization) */
LVK_API int lvk_attention(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                          int n_ctx, int n_past, int n, float * out);

/* lvk_attention plus the pre-softmax scores [n][n_head][n_ctx] (scaled, -inf where masked), followed in
 * scores_out by the f16 probabilities [n][n_head][n_ctx] (so scores_out holds 1.5x that many floats) */
LVK_API int lvk_attention_scores(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                                 int n_ctx, int n_past, int n, float * out, float * scores_out);

/* lvk_attention through the prompt-batch kernels (attention_prompt.hip: scores +
 * softmax per 32 query tokens, P.V per 32-dim slice); same result bits.  Needs
 * head_dim 128, n_ctx % 32 == 0, n_ctx <= 1024. */
LVK_API int lvk_attention_prompt(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                                 int n_ctx, int n_past, int n, float * out);

/* lvk_attention for one token (n = 1) through the decode kernels
 * (attention_decode.hip: scores per 64 positions, softmax + P.V per 32-dim
 * slice); same result bits.  Needs head_dim 128, n_ctx % 64 == 0, n_ctx <= 2048. */
LVK_API int lvk_attention_decode(const uint16_t * kc, const uint16_t * vc, const float * q, int n_embd, int n_head,
                                 int n_ctx, int n_past, float * out);

/* Self-check of the softmax exp: the number of arguments h <= 0 (fp16 bits)
 * where the device's computed fp16(exp(h)) differs from this host's
 * table_exp_f16[h] (ggml.c:2915-2927) -- 0 when the device expf reproduces it,
 * else the count of the double-precision exp.  Contexts compute exp only in a
 * mode with 0 mismatches (env LVK_EXP_TABLE forces the table).  -1 on error. */
LVK_API int lvk_exp_table_mismatches(void);

/* y[t] = g * rms_norm(x[t]) (ggml.c:6024-6080 + llama.cpp:984) */
LVK_API int lvk_rms_norm_mul(const float * x, const float * g, int k, int n, float * y);

/* the 64Ki-entry fp16 exp / silu tables the library uploads (ggml.c:2915-2927) */
LVK_API void lvk_host_tables(uint16_t * exp_tab, uint16_t * silu_tab);

/* decode-step profiling of a llama_context: when enabled, every eval records
 * HIP events around each kernel class (0 embed, 1 qkv, 2 attention, 3 wo,
 * 4 w1|w3, 5 w2, 6 lm_head) and accumulates device ms, launches and algorithmic
 * weight bytes. */
struct llama_context;
LVK_API void lvk_set_profiling(struct llama_context * ctx, int on);
LVK_API int lvk_get_profile(struct llama_context * ctx, double * ms, long * launches, double * bytes, int n);
LVK_API void lvk_reset_profile(struct llama_context * ctx);
/* bytes of quantized weights resident in HBM for this context's model */
LVK_API size_t lvk_weight_bytes(struct llama_context * ctx);
/* bytes of the prompt matmul's f16 A-fragment images (+ the Q4_1 side images) resident in
 * HBM; 0 when they were not built (LVK_PROMPT_A16=0, or too little free memory at load) */
LVK_API size_t lvk_prompt_image_bytes(struct llama_context * ctx);
/* 1 = prompt batches (N > 1) use the bit-faithful VALU matmuls (the reference's
 * exact fp32 chain order), 0 = the MFMA matmuls (default; env LVK_PROMPT_EXACT=1
 * makes 1 the default) */
LVK_API void lvk_set_prompt_exact(struct llama_context * ctx, int on);
/* 1 = replay the captured decode graph for single-token evals (default), 0 = eager */
LVK_API void lvk_set_graph(struct llama_context * ctx, int on);
/* On-device greedy sampling.  lvk_eval_greedy(ctx, token, n_past)
 * is llama_eval(ctx, &token, 1, n_past, .) followed by
 * llama_sample_top_p_top_k(ctx, ., ., ., ., temp <= 0) (llama.cpp:1703-1719,
 * 1382-1394): the argmax runs over the logits in HBM and only the 4-byte token
 * crosses PCIe.  Returns the next token id, or -1 on error (message on stderr).
 * The host logits of llama_get_logits are NOT refreshed by this call.
 * lvk_argmax(x, n) is the op-level kernel on a host array: the first index whose
 * value is strictly greater than all earlier ones (0 when x[0] is NaN). */
LVK_API int lvk_eval_greedy(struct llama_context * ctx, int token, int n_past);
/* n_steps decode steps in one call: step i evaluates token t_i at position n_past + i, with
 * t_0 = tokens[0], t_{i+1} = tokens[i + 1] while i + 1 < n_tokens (a teacher-forced sequence,
 * 1 <= n_tokens <= n_steps) and the argmax of step i's logits after that (n_tokens = 1: greedy).
 * out_tokens[i] is the argmax of step i's logits (what lvk_eval_greedy(ctx, t_i, n_past + i)
 * returns); out_digests (optional, may be NULL) receives lvk_logits_digest of step i's logits
 * row, computed on the device, so a caller can check every step's logits without copying them.
 * The KV cache ends as after the n_steps single-token evals.  The steps run as back-to-back
 * replays of one decode graph whose last kernel picks the next token, advances the step block and
 * writes the next embedding row on the device, so nothing crosses PCIe between steps.
 * n_past + n_steps <= n_ctx.  Returns 0, or -1 on error (layer splits and logits_all contexts
 * refuse it).  The host logits of llama_get_logits are NOT refreshed. */
LVK_API int lvk_decode_chain(struct llama_context * ctx, const int * tokens, int n_tokens, int n_past, int n_steps,
                             int * out_tokens, uint64_t * out_digests);
/* lvk_decode_chain(ctx, &token, 1, n_past, n_steps, out_tokens, NULL) */
LVK_API int lvk_decode_greedy(struct llama_context * ctx, int token, int n_past, int n_steps, int * out_tokens);
/* digest of a logits row: sum over k (mod 2^64) of splitmix64((k << 32) | bits(x[k])) -- position
 * sensitive, order independent, equal for two rows only if (almost surely) bit-identical */
LVK_API uint64_t lvk_logits_digest(const float * x, int n);
/* On-device sampling: lvk_eval_sample(ctx, token, n_past, last_n, n_last,
 * top_k, top_p, temp, repeat_penalty) returns what llama_eval(ctx, &token, 1, n_past, .)
 * followed by llama_sample_top_p_top_k(ctx, last_n, n_last, top_k, top_p, temp,
 * repeat_penalty) returns (llama.cpp:1356-1459, 1703-1719, 1777-1805), drawing from the same
 * mt19937 stream.  The repeat penalty, the temperature and the top-k selection run over the
 * logits in HBM (sample.hip); only the candidates >= the k-th value cross PCIe and the host
 * finishes the reference's softmax / top-p / discrete_distribution over k values.  Ties among
 * the candidates, NaN logits, top_k <= 0 or > 1024, a last-n window > 1024, split or
 * logits_all contexts take the reference path over all logits (same result, slower).
 * temp <= 0 is lvk_eval_greedy.  The host logits of llama_get_logits are NOT refreshed
 * (except on the all-logits path).  Returns the token, or -1 on error. */
/* op-level device candidate selection on a host array (sample.hip): the values the reference
 * sorts (x[i] / temp, with the repeat penalty for ids in last[]), every one >= the k-th largest
 * written to vals/ids (arbitrary order, up to 1024), *flags bit 1 = NaN seen, bit 2 = more than
 * 1024 candidates.  Returns the candidate count, -1 on bad arguments. */
LVK_API int lvk_sample_candidates(const float * x, int n, const int * last, int n_last, int k, float temp, float rp,
                                  float * vals, int * ids, int * flags);
LVK_API int lvk_eval_sample(struct llama_context * ctx, int token, int n_past, const int * last_n, int n_last,
                            int top_k, float top_p, float temp, float repeat_penalty);
LVK_API int lvk_argmax(const float * x, int n);

/* Device-side KV state (the host-bytes form is llama_get_kv_cache /
 * llama_set_kv_cache, llama.cpp:1678-1701): copy positions [0, n_tokens) of every
 * layer's K and V from src to dst in HBM (same model shape and n_ctx, same device) and
 * set dst's KV token count to n_tokens.  dst can then continue with
 * llama_eval(dst, ., ., n_past = n_tokens, .) exactly as src would.  0 / -1. */
LVK_API int lvk_kv_copy(struct llama_context * dst, struct llama_context * src, int n_tokens);

/* Pipeline stages (the 65B layer split).  A stage context holds
 * layers [layer_begin, layer_end) of the model file (weights and KV cache); the
 * first stage (layer_begin == 0) also holds the token embeddings, the last one
 * (layer_end == n_layer) the final norm and lm_head.  This replaces running
 * llama_eval_internal (llama.cpp:927-1197) as one process: the residual stream
 * `inpL` is handed from stage s to s+1 (RCCL send/recv in
 * llama.vk_amd/pipeline.py).  NULL on error. */
LVK_API struct llama_context * lvk_init_stage(const char * path_model, struct llama_context_params params,
                                              int layer_begin, int layer_end);
/* run the stage on n_tokens at positions n_past..: the first stage embeds tokens,
 * the others start from the residual stream set by lvk_stage_set_x; the last
 * stage leaves logits for llama_get_logits.  0 on success, 1 on error. */
LVK_API int lvk_stage_eval(struct llama_context * ctx, const int * tokens, int n_tokens, int n_past);
/* copy the residual stream x [n_tokens][n_embd] f32 out of / into the stage;
 * buf is memory of the context's HIP device when on_device != 0, else host */
LVK_API int lvk_stage_get_x(struct llama_context * ctx, void * buf, int n_tokens, int on_device);
LVK_API int lvk_stage_set_x(struct llama_context * ctx, const void * buf, int n_tokens, int on_device);
/* the stage's layer range; returns the model's n_layer */
LVK_API int lvk_stage_layers(struct llama_context * ctx, int * layer_begin, int * layer_end);

/* One stage per process over RCCL (torchrun, one rank per GPU).  Rank 0 makes the
 * communicator id (lvk_rccl_unique_id: NCCL_UNIQUE_ID_BYTES = 128 bytes into id, n >= 128)
 * and shares it with the other ranks; every rank then joins with its stage context
 * (lvk_init_stage with the layers of stage `stage`, on its own GPU).  lvk_stage_step runs
 * one llama_eval slice of the pipeline on this rank: ncclRecv of inpL from stage-1, the
 * stage's layers, ncclSend to stage+1, all on the context's stream, prompts cut into
 * micro-batches of `micro` tokens (0: none).  greedy != 0 (one token): the last stage's
 * device argmax is sent to stage 0; both return it.  Otherwise 0 (the last stage leaves
 * logits for llama_get_logits).  -1 on error.  Every argument is checked before the first
 * transfer; a step that fails on any rank aborts the link (ncclCommAbort / the shm ring's
 * abort word), so the neighbours' steps fail too instead of waiting, and every wait is
 * bounded by LVK_STAGE_TIMEOUT_S seconds (default 300).  An aborted link must be
 * reconnected.  The replaced code is the single-process llama_eval_internal
 * (reference llama.cpp:927-1197). */
LVK_API int lvk_rccl_unique_id(void * id, size_t n);
LVK_API int lvk_stage_connect(struct llama_context * ctx, const void * id, int n_stages, int stage);
/* The same link through a host shared-memory ring (POSIX shm object `name`, a single path
 * component such as "/lvk_run42"): any stage placement, several stages on one GPU included,
 * no RCCL.  Stage 0 creates a fresh object under the name (removing one a crashed run left),
 * the others wait for it; the call returns once all n_stages stages have joined, and stage 0
 * then unlinks the name, so a reconnect (the only way on after an abort) under the same name
 * starts clean.  Messages travel in 1 MiB pieces: the object takes
 * n_stages * 4 MiB + 4 KiB of /dev/shm (32 MiB at 8 stages), reserved at connect -- a
 * /dev/shm too small fails the connect with an error. */
LVK_API int lvk_stage_connect_shm(struct llama_context * ctx, const char * name, int n_stages, int stage);
LVK_API int lvk_stage_step(struct llama_context * ctx, const int * tokens, int n_tokens, int n_past, int greedy,
                           int micro);
/* The stage link alone (per-hop time of the 65B split): `iters` laps of a `bytes`
 * message (one token's residual stream is n_embd * 4) around the stage ring -- stage 0 sends
 * to 1, ..., the last stage back to 0 -- on the same transport and stream as lvk_stage_step;
 * every stage calls it.  *us_per_hop: the wall time of a lap over the number of stages.  0 on
 * success, -1 on error (the link is aborted as in lvk_stage_step).  No reference counterpart:
 * the reference has no inter-device hop (llama.cpp:927-1197 runs every layer in one process). */
LVK_API int lvk_stage_link_probe(struct llama_context * ctx, int bytes, int iters, double * us_per_hop);

/* ggml_graph_compute keeps the host ranges of its tensors mirrored in HBM across calls and
 * uploads only bytes a node reads before the call writes them, and of those only pages the
 * host may have changed: pages of read-only mappings (a PROT_READ model file, an mprotect'ed
 * buffer) while the mapping is unchanged; writable pages go again on every call unless
 * LVK_GGML_CACHE=2 tracks them with the kernel's soft-dirty bits (process-wide clear_refs,
 * opt-in: measured slower in a HIP process).  Q4 weights are repacked once per upload.
 * lvk_ggml_stats: the last call's out[0] host->device bytes, out[1] device->host bytes (the
 * byte ranges the nodes wrote), out[2] bytes of Q4 weights repacked, out[3] host bytes
 * mirrored in HBM after the call; out[4] the tracking mode (0 off: LVK_GGML_CACHE=0, 1
 * read-only mappings only: the default, 2 soft-dirty pages: LVK_GGML_CACHE=2),
 * out[5] 1 once any graph has run, out[6] the call's host microseconds of tracking
 * bookkeeping, out[7] of them the microseconds in clear_refs.  Fills min(n, 8) values,
 * returns 8 (-1 on bad arguments).
 * lvk_ggml_invalidate: the caller changed [p, p + n) in a way that tracking cannot see
 * (write-enabled a read-only buffer, wrote, protected it again between two calls; or
 * hipHostRegister'ed the range after a call had used it, so that DMA may now write it);
 * its pages are uploaded again by the next call, and whether the range is HIP host memory
 * is decided again.  0 / -1. */
LVK_API int lvk_ggml_stats(uint64_t * out, int n);
LVK_API int lvk_ggml_invalidate(const void * p, size_t n);

/* The layer split behind llama.h, one process driving n_stages HIP
 * devices: stage s holds layers [s*L/S, (s+1)*L/S) on devices[s].  llama_eval /
 * lvk_eval_greedy / llama_get_logits / the KV-cache calls work on the returned context as
 * on a single-device one.  The residual stream moves between stages with grouped
 * ncclSend/ncclRecv (transport "rccl", the default when the devices are distinct) or a
 * stream-ordered device copy ("copy"; also used when a device repeats, e.g. a one-GPU
 * rehearsal); the host waits once per eval.  Prompts are cut into micro-batches of
 * `micro` tokens (0: none) that flow through the stages back to back.
 * llama_init_from_file does the same when the environment holds LVK_SPLIT_DEVICES=0,1,..
 * or LVK_SPLIT=S (devices 0..S-1), with LVK_SPLIT_TRANSPORT and LVK_SPLIT_MICRO (64). */
LVK_API struct llama_context * lvk_init_split(const char * path_model, struct llama_context_params params,
                                              int n_stages, const int * devices, const char * transport, int micro);
/* stages of ctx (1 without a split), whether they hand off over RCCL, the micro-batch */
LVK_API int lvk_split_info(struct llama_context * ctx, int * n_stages, int * rccl, int * micro);

#ifdef __cplusplus
}
#endif
#endif
