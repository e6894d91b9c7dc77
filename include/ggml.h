/* include/ggml.h -- the ggml operator surface of the reference (ggml.h) as far as the
 * LLaMA graph and its callers use it, backed by llama.vk_amd:
 *
 *   - process timing and fp16 conversion (ggml.h:192-193, 335-339);
 *   - contexts with a real memory pool: ggml_init / ggml_free / ggml_used_mem /
 *     ggml_set_scratch (ggml.h:341-346, 353-358), tensors laid out exactly as the
 *     reference's struct ggml_tensor (ggml.h:270-300) so callers that read ne / nb / data
 *     directly keep working;
 *   - tensor constructors, views and accessors (ggml.h:360-420) on host memory;
 *   - the graph operators of llama_eval_internal (llama.cpp:927-1197): get_rows, rms_norm,
 *     mul / add / repeat, mul_mat (Q4_0 / Q4_1 / F16 / F32 x F32), reshape / view / permute /
 *     transpose, rope, cpy, scale, diag_mask_inf, soft_max, silu (ggml.h:430-640);
 *   - ggml_build_forward[_expand] and ggml_graph_compute (ggml.h:656-660): every node runs
 *     on the GPU (llama.vk_amd/csrc/runtime/ggml_graph.cpp, kernels in graph_ops.hip) with
 *     the arithmetic of the AVX2 ggml.c build; the host buffers the
 *     graph touches are mirrored to HBM for the compute call and the node results copied
 *     back.  An operator outside this list aborts (GGML_ASSERT semantics): there is no CPU
 *     fallback.
 *   - the op-level codec table ggml_internal_get_quantize_fn (ggml.h:796-814).
 * Same names, signatures, enum values and struct layouts as the reference header.
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

#define GGML_FILE_MAGIC   0x67676d6c /* "ggml" */
#define GGML_FILE_VERSION 1

#define GGML_MAX_DIMS     4
#define GGML_MAX_NODES    4096
#define GGML_MAX_PARAMS   16
#define GGML_MAX_CONTEXTS 64
#define GGML_MAX_OPT      4

typedef uint16_t ggml_fp16_t;

/* IEEE binary16 <-> binary32, round to nearest even (ggml.c:182-183) */
LVK_GGML_API float       ggml_fp16_to_fp32(ggml_fp16_t x);
LVK_GGML_API ggml_fp16_t ggml_fp32_to_fp16(float x);

struct ggml_object;
struct ggml_context;

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

/* ggml.h:212-256: the full op enumeration (values fixed by the reference) */
enum ggml_op {
    GGML_OP_NONE = 0,

    GGML_OP_DUP,
    GGML_OP_ADD,
    GGML_OP_SUB,
    GGML_OP_MUL,
    GGML_OP_DIV,
    GGML_OP_SQR,
    GGML_OP_SQRT,
    GGML_OP_SUM,
    GGML_OP_MEAN,
    GGML_OP_REPEAT,
    GGML_OP_ABS,
    GGML_OP_SGN,
    GGML_OP_NEG,
    GGML_OP_STEP,
    GGML_OP_RELU,
    GGML_OP_GELU,
    GGML_OP_SILU,
    GGML_OP_NORM,
    GGML_OP_RMS_NORM,

    GGML_OP_MUL_MAT,

    GGML_OP_SCALE,
    GGML_OP_CPY,
    GGML_OP_RESHAPE,
    GGML_OP_VIEW,
    GGML_OP_PERMUTE,
    GGML_OP_TRANSPOSE,
    GGML_OP_GET_ROWS,
    GGML_OP_DIAG_MASK_INF,
    GGML_OP_SOFT_MAX,
    GGML_OP_ROPE,
    GGML_OP_CONV_1D_1S,
    GGML_OP_CONV_1D_2S,

    GGML_OP_FLASH_ATTN,
    GGML_OP_FLASH_FF,

    GGML_OP_COUNT,
};

/* ggml.h:260-266 */
struct ggml_object {
    size_t offs;
    size_t size;

    struct ggml_object * next;

    char padding[8];
};

static const size_t GGML_OBJECT_SIZE = sizeof(struct ggml_object);

/* ggml.h:270-300: n-dimensional tensor (field for field) */
struct ggml_tensor {
    enum ggml_type type;

    int     n_dims;
    int64_t ne[GGML_MAX_DIMS]; /* number of elements */
    size_t  nb[GGML_MAX_DIMS]; /* stride in bytes: nb[0] = type size, nb[i] = nb[i-1] * ne[i-1] (+ padding) */

    enum ggml_op op;

    bool is_param;

    struct ggml_tensor * grad;
    struct ggml_tensor * src0;
    struct ggml_tensor * src1;
    struct ggml_tensor * opt[GGML_MAX_OPT];

    int n_tasks;

    int     perf_runs;
    int64_t perf_cycles;
    int64_t perf_time_us;

    void * data;
    char padding[8];
};

/* ggml.h:303-318 */
struct ggml_cgraph {
    int n_nodes;
    int n_leafs;
    int n_threads;

    size_t work_size;
    struct ggml_tensor * work;

    struct ggml_tensor * nodes[GGML_MAX_NODES];
    struct ggml_tensor * grads[GGML_MAX_NODES];
    struct ggml_tensor * leafs[GGML_MAX_NODES];

    int     perf_runs;
    int64_t perf_cycles;
    int64_t perf_time_us;
};

/* ggml.h:321-325 */
struct ggml_scratch {
    size_t offs;
    size_t size;
    void * data;
};

/* ggml.h:328-333 */
struct ggml_init_params {
    size_t mem_size;   /* bytes */
    void * mem_buffer; /* NULL: allocated by the context */
    bool   no_alloc;   /* tensors get no data (the caller sets tensor->data) */
};

/* ggml.h:335-339: monotonic wall clock */
LVK_GGML_API void    ggml_time_init(void);
LVK_GGML_API int64_t ggml_time_ms(void);
LVK_GGML_API int64_t ggml_time_us(void);
LVK_GGML_API int64_t ggml_cycles(void);
LVK_GGML_API int64_t ggml_cycles_per_ms(void);

LVK_GGML_API void ggml_print_object (const struct ggml_object * obj);
LVK_GGML_API void ggml_print_objects(const struct ggml_context * ctx);

LVK_GGML_API int64_t ggml_nelements(const struct ggml_tensor * tensor);
LVK_GGML_API size_t  ggml_nbytes   (const struct ggml_tensor * tensor);

LVK_GGML_API int    ggml_blck_size (enum ggml_type type);
LVK_GGML_API size_t ggml_type_size (enum ggml_type type);
LVK_GGML_API float  ggml_type_sizef(enum ggml_type type);

LVK_GGML_API size_t ggml_element_size(const struct ggml_tensor * tensor);

LVK_GGML_API struct ggml_context * ggml_init(struct ggml_init_params params);
LVK_GGML_API void ggml_free(struct ggml_context * ctx);

LVK_GGML_API size_t ggml_used_mem(const struct ggml_context * ctx);

LVK_GGML_API size_t ggml_set_scratch(struct ggml_context * ctx, struct ggml_scratch scratch);

LVK_GGML_API struct ggml_tensor * ggml_new_tensor(struct ggml_context * ctx, enum ggml_type type, int n_dims,
                                                  const int64_t * ne);
LVK_GGML_API struct ggml_tensor * ggml_new_tensor_1d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0);
LVK_GGML_API struct ggml_tensor * ggml_new_tensor_2d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0,
                                                     int64_t ne1);
LVK_GGML_API struct ggml_tensor * ggml_new_tensor_3d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0,
                                                     int64_t ne1, int64_t ne2);
LVK_GGML_API struct ggml_tensor * ggml_new_tensor_4d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0,
                                                     int64_t ne1, int64_t ne2, int64_t ne3);

LVK_GGML_API struct ggml_tensor * ggml_new_i32(struct ggml_context * ctx, int32_t value);
LVK_GGML_API struct ggml_tensor * ggml_new_f32(struct ggml_context * ctx, float value);

LVK_GGML_API struct ggml_tensor * ggml_dup_tensor (struct ggml_context * ctx, const struct ggml_tensor * src);
LVK_GGML_API struct ggml_tensor * ggml_view_tensor(struct ggml_context * ctx, const struct ggml_tensor * src);

LVK_GGML_API struct ggml_tensor * ggml_set_zero(struct ggml_tensor * tensor);
LVK_GGML_API struct ggml_tensor * ggml_set_i32 (struct ggml_tensor * tensor, int32_t value);
LVK_GGML_API struct ggml_tensor * ggml_set_f32 (struct ggml_tensor * tensor, float value);

LVK_GGML_API int32_t ggml_get_i32_1d(const struct ggml_tensor * tensor, int i);
LVK_GGML_API void    ggml_set_i32_1d(const struct ggml_tensor * tensor, int i, int32_t value);

LVK_GGML_API float ggml_get_f32_1d(const struct ggml_tensor * tensor, int i);
LVK_GGML_API void  ggml_set_f32_1d(const struct ggml_tensor * tensor, int i, float value);

LVK_GGML_API void *  ggml_get_data    (const struct ggml_tensor * tensor);
LVK_GGML_API float * ggml_get_data_f32(const struct ggml_tensor * tensor);

/* operators (graph nodes; evaluated by ggml_graph_compute) */
LVK_GGML_API struct ggml_tensor * ggml_dup(struct ggml_context * ctx, struct ggml_tensor * a);
LVK_GGML_API struct ggml_tensor * ggml_add(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
LVK_GGML_API struct ggml_tensor * ggml_sub(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
LVK_GGML_API struct ggml_tensor * ggml_mul(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
LVK_GGML_API struct ggml_tensor * ggml_div(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
/* if a has b's shape return a, else repeat(a) to b's shape */
LVK_GGML_API struct ggml_tensor * ggml_repeat(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
LVK_GGML_API struct ggml_tensor * ggml_silu(struct ggml_context * ctx, struct ggml_tensor * a);
LVK_GGML_API struct ggml_tensor * ggml_rms_norm(struct ggml_context * ctx, struct ggml_tensor * a);
/* a: m rows of n, b: p rows of n; result p rows of m */
LVK_GGML_API struct ggml_tensor * ggml_mul_mat(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
/* in place, returns view(a) */
LVK_GGML_API struct ggml_tensor * ggml_scale(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
/* a -> b, returns view(b) */
LVK_GGML_API struct ggml_tensor * ggml_cpy(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
LVK_GGML_API struct ggml_tensor * ggml_reshape(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b);
LVK_GGML_API struct ggml_tensor * ggml_reshape_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0,
                                                  int64_t ne1);
LVK_GGML_API struct ggml_tensor * ggml_reshape_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0,
                                                  int64_t ne1, int64_t ne2);
/* offsets and strides in bytes */
LVK_GGML_API struct ggml_tensor * ggml_view_1d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0,
                                               size_t offset);
LVK_GGML_API struct ggml_tensor * ggml_view_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0,
                                               int64_t ne1, size_t nb1, size_t offset);
LVK_GGML_API struct ggml_tensor * ggml_view_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0,
                                               int64_t ne1, int64_t ne2, size_t nb1, size_t nb2, size_t offset);
LVK_GGML_API struct ggml_tensor * ggml_permute(struct ggml_context * ctx, struct ggml_tensor * a, int axis0,
                                               int axis1, int axis2, int axis3);
LVK_GGML_API struct ggml_tensor * ggml_transpose(struct ggml_context * ctx, struct ggml_tensor * a);
LVK_GGML_API struct ggml_tensor * ggml_get_rows(struct ggml_context * ctx, struct ggml_tensor * a,
                                                struct ggml_tensor * b);
/* in place, returns view(a): elements above the diagonal shifted by n_past -> -INF */
LVK_GGML_API struct ggml_tensor * ggml_diag_mask_inf(struct ggml_context * ctx, struct ggml_tensor * a, int n_past);
/* in place, returns view(a) */
LVK_GGML_API struct ggml_tensor * ggml_soft_max(struct ggml_context * ctx, struct ggml_tensor * a);
/* rotary position embedding, in place, returns view(a); mode 1: skip the first n_past rows */
LVK_GGML_API struct ggml_tensor * ggml_rope(struct ggml_context * ctx, struct ggml_tensor * a, int n_past, int n_dims,
                                            int mode);

LVK_GGML_API void ggml_set_param(struct ggml_context * ctx, struct ggml_tensor * tensor);

LVK_GGML_API void ggml_build_forward_expand(struct ggml_cgraph * cgraph, struct ggml_tensor * tensor);
LVK_GGML_API struct ggml_cgraph ggml_build_forward(struct ggml_tensor * tensor);

LVK_GGML_API void ggml_graph_compute(struct ggml_context * ctx, struct ggml_cgraph * cgraph);
LVK_GGML_API void ggml_graph_reset(struct ggml_cgraph * cgraph);
LVK_GGML_API void ggml_graph_print(const struct ggml_cgraph * cgraph);

/* ggml.h:779-790: system info (the host CPU's SIMD, as the reference reports it) */
LVK_GGML_API int ggml_cpu_has_avx(void);
LVK_GGML_API int ggml_cpu_has_avx2(void);
LVK_GGML_API int ggml_cpu_has_avx512(void);
LVK_GGML_API int ggml_cpu_has_fma(void);
LVK_GGML_API int ggml_cpu_has_neon(void);
LVK_GGML_API int ggml_cpu_has_arm_fma(void);
LVK_GGML_API int ggml_cpu_has_f16c(void);
LVK_GGML_API int ggml_cpu_has_fp16_va(void);
LVK_GGML_API int ggml_cpu_has_wasm_simd(void);
LVK_GGML_API int ggml_cpu_has_blas(void);
LVK_GGML_API int ggml_cpu_has_sse3(void);
LVK_GGML_API int ggml_cpu_has_vsx(void);

/* ggml.h:772-773 (ggml.c:10520-10564): the file-creation quantizers (quantize_row_q4_0/1
 * _reference: roundf, half away from zero) over n values in rows of k, the 16-bin nibble
 * histogram accumulated into hist; returns the bytes written (n/32 blocks).  Host code:
 * llama_model_quantize and the reference's tests/test-quantize.c call them without a GPU. */
LVK_GGML_API size_t ggml_quantize_q4_0(const float * src, void * dst, int n, int k, int64_t * hist);
LVK_GGML_API size_t ggml_quantize_q4_1(const float * src, void * dst, int n, int k, int64_t * hist);

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
