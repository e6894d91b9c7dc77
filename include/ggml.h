/* include/ggml.h -- the part of the reference's ggml.h that the llama.h
 * example programs call directly (examples/quantize/quantize.cpp:11-50):
 * process timing and the context init/free used there only to build ggml's
 * fp16 tables, plus the op-level codec table (ggml_internal_get_quantize_fn).  Same names and signatures as reference ggml.h:328-354; the
 * tensor/graph API itself is not part of this library's surface (the forward
 * pass runs on the GPU behind llama.h; operator access is include/lvk_ops.h).
 */
#ifndef LVK_GGML_H
#define LVK_GGML_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#define LVK_GGML_API __attribute__((visibility("default")))

#ifdef __cplusplus
extern "C" {
#endif

struct ggml_context;

/* ggml.h:328-333 */
struct ggml_init_params {
    size_t mem_size;
    void * mem_buffer;
    bool   no_alloc;
};

/* ggml.h:335-337: monotonic wall clock */
LVK_GGML_API void    ggml_time_init(void);
LVK_GGML_API int64_t ggml_time_ms(void);
LVK_GGML_API int64_t ggml_time_us(void);

/* ggml.h:353-354: the library's tables live on the device and on its own
 * host side, so init only hands back a context token that free releases */
LVK_GGML_API struct ggml_context * ggml_init(struct ggml_init_params params);
LVK_GGML_API void ggml_free(struct ggml_context * ctx);

/* ggml.h:200-209 */
enum ggml_type {
    GGML_TYPE_Q4_0,
    GGML_TYPE_Q4_1,
    GGML_TYPE_I8,
    GGML_TYPE_I16,
    GGML_TYPE_I32,
    GGML_TYPE_F16,
    GGML_TYPE_F32,
    GGML_TYPE_COUNT,
};

/* ggml.h:796-814: the op-level codec table, same names, signatures and block layouts
 * (block_q4_0 {float d; uint8 qs[16]}, block_q4_1 {float d, m; uint8 qs[16]}).  Every
 * function runs on the GPU (llama.vk_amd/csrc/runtime/ggml_quantize_fns.cpp):
 * quantize_row_q is the AVX2 quantizer (RNE), quantize_row_q_reference the scalar one
 * (roundf), vec_dot_q the AVX2 chain order; n / k multiples of 32.  Types other than
 * Q4_0 / Q4_1 get a zeroed table; i >= GGML_TYPE_COUNT aborts (GGML_ASSERT). */
#ifdef __cplusplus
#define LVK_GGML_RESTRICT
#else
#define LVK_GGML_RESTRICT restrict
#endif
typedef void (*dequantize_row_q_t)(const void * LVK_GGML_RESTRICT x, float * LVK_GGML_RESTRICT y, int k);
typedef void (*quantize_row_q_t)(const float * LVK_GGML_RESTRICT x, void * LVK_GGML_RESTRICT y, int k);
typedef void (*vec_dot_q_t)(const int n, float * LVK_GGML_RESTRICT s, const void * LVK_GGML_RESTRICT x,
                            const void * LVK_GGML_RESTRICT y);

typedef struct {
    dequantize_row_q_t dequantize_row_q;
    quantize_row_q_t   quantize_row_q;
    quantize_row_q_t   quantize_row_q_reference;
    vec_dot_q_t        vec_dot_q;
} quantize_fns_t;

LVK_GGML_API quantize_fns_t ggml_internal_get_quantize_fn(size_t i);

#ifdef __cplusplus
}
#endif
#endif
