/* include/llama.h -- drop-in C ABI of llama.vk_amd (libllama_vk_amd.so).
 *
 * Declares exactly the model-level entry points of the reference's C API
 * (reference llama.h:26-172) with the same names, argument meaning, return
 * conventions and struct layout, so examples/main, examples/perplexity and
 * examples/embedding link against this library unchanged.  The forward pass
 * behind llama_eval runs on an MI355X (gfx950) through hand-written HIP
 * kernels; tokenizer, sampler and timings stay on the host.
 *
 * Each declaration cites the reference declaration it replaces.
 */
#ifndef LLAMA_H
#define LLAMA_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#define LLAMA_API __attribute__((visibility("default")))

#define LLAMA_FILE_VERSION 1                 /* reference llama.h:22 */
#define LLAMA_FILE_MAGIC 0x67676a74          /* 'ggjt', reference llama.h:23 */
#define LLAMA_FILE_MAGIC_UNVERSIONED 0x67676d6c

#ifdef __cplusplus
extern "C" {
#endif

struct llama_context;

typedef int llama_token;

/* reference llama.h:39-45 */
typedef struct llama_token_data {
    llama_token id;
    float p;
    float plog;
} llama_token_data;

typedef void (*llama_progress_callback)(float progress, void * ctx);

/* reference llama.h:49-66 -- identical field order and types */
struct llama_context_params {
    int n_ctx;       /* text context */
    int n_parts;     /* -1 for default */
    int seed;        /* RNG seed, 0 for random */
    bool f16_kv;     /* fp16 KV cache (the GPU path always stores f16) */
    bool logits_all; /* llama_eval computes all logits, not just the last one */
    bool vocab_only; /* only load the vocabulary, no weights */
    bool use_mmap;   /* mmap the model file while uploading */
    bool use_mlock;  /* accepted for compatibility */
    bool embedding;  /* embedding mode */
    llama_progress_callback progress_callback;
    void * progress_callback_user_data;
};

LLAMA_API struct llama_context_params llama_context_default_params(void);   /* llama.h:68 */
LLAMA_API bool llama_mmap_supported(void);                                    /* llama.h:70 */
LLAMA_API bool llama_mlock_supported(void);                                   /* llama.h:71 */

/* llama.h:74-76: load a ggjt model into HBM; NULL on failure (error printed) */
LLAMA_API struct llama_context * llama_init_from_file(const char * path_model, struct llama_context_params params);
/* llama.h:79 */
LLAMA_API void llama_free(struct llama_context * ctx);
/* llama.h:83-86: f16/f32 -> Q4_0 (itype 2) / Q4_1 (itype 3) file quantizer; 0 on success */
LLAMA_API int llama_model_quantize(const char * fname_inp, const char * fname_out, int itype);

/* llama.h:88-106: KV cache state as host bytes (layout: K then V, f16,
 * [n_layer][n_ctx][n_embd] and [n_layer][n_embd][n_ctx]) */
LLAMA_API const uint8_t * llama_get_kv_cache(struct llama_context * ctx);
LLAMA_API size_t llama_get_kv_cache_size(struct llama_context * ctx);
LLAMA_API int llama_get_kv_cache_token_count(struct llama_context * ctx);
LLAMA_API void llama_set_kv_cache(struct llama_context * ctx, const uint8_t * kv_cache, size_t n_size,
                                  int n_token_count);

/* llama.h:108-113: evaluate tokens[0..n_tokens) at positions n_past..; 0 on success */
LLAMA_API int llama_eval(struct llama_context * ctx, const llama_token * tokens, int n_tokens, int n_past,
                         int n_threads);

/* llama.h:119-124 */
LLAMA_API int llama_tokenize(struct llama_context * ctx, const char * text, llama_token * tokens,
                             int n_max_tokens, bool add_bos);

LLAMA_API int llama_n_vocab(struct llama_context * ctx);   /* llama.h:126 */
LLAMA_API int llama_n_ctx(struct llama_context * ctx);     /* llama.h:127 */
LLAMA_API int llama_n_embd(struct llama_context * ctx);    /* llama.h:128 */

/* llama.h:135: logits of the last eval ([n_vocab], or [n_tokens][n_vocab] with logits_all) */
LLAMA_API float * llama_get_logits(struct llama_context * ctx);
/* llama.h:139 */
LLAMA_API float * llama_get_embeddings(struct llama_context * ctx);
/* llama.h:142 */
LLAMA_API const char * llama_token_to_str(struct llama_context * ctx, llama_token token);

LLAMA_API llama_token llama_token_bos(void);   /* llama.h:145 */
LLAMA_API llama_token llama_token_eos(void);   /* llama.h:146 */

/* llama.h:149-156 */
LLAMA_API llama_token llama_sample_top_p_top_k(struct llama_context * ctx, const llama_token * last_n_tokens_data,
                                               int last_n_tokens_size, int top_k, float top_p, float temp,
                                               float repeat_penalty);

LLAMA_API void llama_print_timings(struct llama_context * ctx);   /* llama.h:159 */
LLAMA_API void llama_reset_timings(struct llama_context * ctx);   /* llama.h:160 */
LLAMA_API const char * llama_print_system_info(void);             /* llama.h:163 */

#ifdef __cplusplus
}
#endif

#endif /* LLAMA_H */
