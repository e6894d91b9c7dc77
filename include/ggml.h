/* include/ggml.h -- the part of the reference's ggml.h that the llama.h
 * example programs call directly (examples/quantize/quantize.cpp:11-50):
 * process timing and the context init/free used there only to build ggml's
 * fp16 tables.  Same names and signatures as reference ggml.h:328-354; the
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

#ifdef __cplusplus
}
#endif
#endif
