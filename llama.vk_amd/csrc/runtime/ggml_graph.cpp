// ggml_graph.cpp -- the ggml operator surface of include/ggml.h on llama.vk_amd.
//
// The reference builds llama_eval_internal (llama.cpp:927-1197) as a ggml graph over host
// tensors and runs it with ggml_graph_compute (ggml.h:660; dispatch ggml.c:8562-8716).
// This file keeps that API for callers that drive ggml themselves:
//   * contexts are real memory pools with the reference's accounting (an object header,
//     the tensor, its data, 16-byte aligned; scratch buffers), so callers that size their
//     pools like llama.cpp does fit;
//   * struct ggml_tensor is the reference's layout, views / permutes / reshapes are
//     metadata only, as in ggml;
//   * ggml_graph_compute mirrors every host buffer the graph touches into HBM, runs each
//     node on the GPU in graph order (graph_ops.hip, the Q4 matvec kernels), and copies the
//     node results back.  An operator without a GPU implementation aborts -- there is no
//     CPU fallback.
#include <immintrin.h>

#include <algorithm>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "../../../include/ggml.h"
#include "lvk_context.h"

namespace {

constexpr size_t MEM_ALIGN = 16;
static_assert(sizeof(ggml_object) % MEM_ALIGN == 0, "ggml_object size");
static_assert(sizeof(ggml_tensor) % MEM_ALIGN == 0, "ggml_tensor size");

// bytes per block and elements per block (ggml.c GGML_TYPE_SIZE / GGML_BLCK_SIZE)
constexpr size_t TYPE_SIZE[GGML_TYPE_COUNT] = {20, 24, 1, 2, 4, 2, 4};
constexpr int BLCK_SIZE[GGML_TYPE_COUNT] = {32, 32, 1, 1, 1, 1, 1};

[[noreturn]] void gabort(const char * what) {
    fprintf(stderr, "llama.vk_amd ggml: %s\n", what);
    abort();
}
#define G_ASSERT(x)                                                                             \
    do {                                                                                        \
        if (!(x)) gabort("GGML_ASSERT: " #x);                                                   \
    } while (0)

__attribute__((target("f16c"))) uint16_t h_f32_to_f16(float f) { return _cvtss_sh(f, 0); }
__attribute__((target("f16c"))) float h_f16_to_f32(uint16_t h) { return _cvtsh_ss(h); }

}  // namespace

struct ggml_context {
    size_t mem_size = 0;
    char * mem_buffer = nullptr;
    bool mem_owned = false;
    bool no_alloc = false;
    ggml_object * objects_begin = nullptr;
    ggml_object * objects_end = nullptr;
    ggml_scratch scratch{0, 0, nullptr};
    ggml_scratch scratch_save{0, 0, nullptr};
};

namespace {

bool is_contiguous(const ggml_tensor * t) {
    return t->nb[0] == TYPE_SIZE[t->type] && t->nb[1] == (t->nb[0] * t->ne[0]) / BLCK_SIZE[t->type] &&
           t->nb[2] == t->nb[1] * t->ne[1] && t->nb[3] == t->nb[2] * t->ne[2];
}
bool same_shape(const ggml_tensor * a, const ggml_tensor * b) {
    return a->ne[0] == b->ne[0] && a->ne[1] == b->ne[1] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3];
}

ggml_tensor * new_tensor_impl(ggml_context * ctx, ggml_type type, int n_dims, const int64_t * ne, void * data) {
    G_ASSERT(type < GGML_TYPE_COUNT && n_dims >= 1 && n_dims <= GGML_MAX_DIMS);
    ggml_object * cur = ctx->objects_end;
    const size_t cur_end = cur ? cur->offs + cur->size : 0;
    size_t need = 0;
    if (!data && !ctx->no_alloc) {
        need = TYPE_SIZE[type] * (ne[0] / BLCK_SIZE[type]);
        for (int i = 1; i < n_dims; ++i) need *= ne[i];
        need = (need + MEM_ALIGN - 1) / MEM_ALIGN * MEM_ALIGN;
    }
    ggml_object * obj = (ggml_object *) (ctx->mem_buffer + cur_end);
    if (!ctx->scratch.data || data) {
        need += sizeof(ggml_tensor);
        if (cur_end + need + GGML_OBJECT_SIZE > ctx->mem_size) {
            fprintf(stderr, "%s: not enough space in the context's memory pool (needed %zu, available %zu)\n", __func__,
                    cur_end + need + GGML_OBJECT_SIZE, ctx->mem_size);
            gabort("out of context memory");
        }
        *obj = ggml_object{cur_end + GGML_OBJECT_SIZE, need, nullptr, {0}};
    } else {
        if (ctx->scratch.offs + need > ctx->scratch.size) gabort("not enough space in the scratch memory");
        if (cur_end + sizeof(ggml_tensor) + GGML_OBJECT_SIZE > ctx->mem_size) gabort("out of context memory");
        data = (char *) ctx->scratch.data + ctx->scratch.offs;
        *obj = ggml_object{cur_end + GGML_OBJECT_SIZE, sizeof(ggml_tensor), nullptr, {0}};
        ctx->scratch.offs += need;
    }
    if (cur) cur->next = obj;
    else ctx->objects_begin = obj;
    ctx->objects_end = obj;
    ggml_tensor * t = (ggml_tensor *) (ctx->mem_buffer + obj->offs);
    std::memset(t, 0, sizeof(*t));
    t->type = type;
    t->n_dims = n_dims;
    for (int i = 0; i < GGML_MAX_DIMS; ++i) t->ne[i] = 1;
    for (int i = 0; i < n_dims; ++i) t->ne[i] = ne[i];
    t->op = GGML_OP_NONE;
    t->data = (!data && !ctx->no_alloc) ? (void *) (t + 1) : data;
    t->nb[0] = TYPE_SIZE[type];
    t->nb[1] = t->nb[0] * (t->ne[0] / BLCK_SIZE[type]);
    for (int i = 2; i < GGML_MAX_DIMS; ++i) t->nb[i] = t->nb[i - 1] * t->ne[i - 1];
    return t;
}

// a 1-element tensor outside any scratch buffer (ggml_new_i32 / ggml_new_f32 and the
// parameter tensors of rope / diag_mask_inf)
ggml_tensor * new_param_tensor(ggml_context * ctx, ggml_type type, int64_t n) {
    ctx->scratch_save = ctx->scratch;
    ctx->scratch.data = nullptr;
    ggml_tensor * t = new_tensor_impl(ctx, type, 1, &n, nullptr);
    ctx->scratch = ctx->scratch_save;
    return t;
}

ggml_tensor * unary_node(ggml_context * ctx, ggml_tensor * a, ggml_op op) {
    ggml_tensor * r = ggml_dup_tensor(ctx, a);
    r->op = op;
    r->src0 = a;
    return r;
}

ggml_tensor * binary_node(ggml_context * ctx, ggml_tensor * a, ggml_tensor * b, ggml_op op) {
    G_ASSERT(same_shape(a, b));
    ggml_tensor * r = ggml_dup_tensor(ctx, a);
    r->op = op;
    r->src0 = a;
    r->src1 = b;
    return r;
}

}  // namespace

extern "C" {

// ---------------------------------------------------------------------------
// timing, fp16, sizes
// ---------------------------------------------------------------------------
static int64_t g_t0_us = 0;
void ggml_time_init(void) { g_t0_us = lvk::now_us(); }
int64_t ggml_time_ms(void) { return (lvk::now_us() - g_t0_us) / 1000; }
int64_t ggml_time_us(void) { return lvk::now_us() - g_t0_us; }
int64_t ggml_cycles(void) { return (int64_t) __rdtsc(); }
int64_t ggml_cycles_per_ms(void) {
    static int64_t c = 0;
    if (!c) {
        const int64_t t0 = lvk::now_us(), c0 = ggml_cycles();
        while (lvk::now_us() - t0 < 2000) {}
        c = (ggml_cycles() - c0) / 2;
    }
    return c;
}

float ggml_fp16_to_fp32(ggml_fp16_t x) { return h_f16_to_f32(x); }
ggml_fp16_t ggml_fp32_to_fp16(float x) { return h_f32_to_f16(x); }

int64_t ggml_nelements(const struct ggml_tensor * t) { return t->ne[0] * t->ne[1] * t->ne[2] * t->ne[3]; }
size_t ggml_nbytes(const struct ggml_tensor * t) {
    return (size_t) ggml_nelements(t) * TYPE_SIZE[t->type] / BLCK_SIZE[t->type];
}
int ggml_blck_size(enum ggml_type type) { return BLCK_SIZE[type]; }
size_t ggml_type_size(enum ggml_type type) { return TYPE_SIZE[type]; }
float ggml_type_sizef(enum ggml_type type) { return (float) TYPE_SIZE[type] / BLCK_SIZE[type]; }
size_t ggml_element_size(const struct ggml_tensor * t) { return TYPE_SIZE[t->type]; }

void ggml_print_object(const struct ggml_object * obj) {
    fprintf(stderr, " - ggml_object: offset = %zu, size = %zu, next = %p\n", obj->offs, obj->size, (void *) obj->next);
}
void ggml_print_objects(const struct ggml_context * ctx) {
    fprintf(stderr, "%s: objects in context %p:\n", __func__, (const void *) ctx);
    for (const ggml_object * o = ctx->objects_begin; o; o = o->next) ggml_print_object(o);
}

// ---------------------------------------------------------------------------
// contexts
// ---------------------------------------------------------------------------
struct ggml_context * ggml_init(struct ggml_init_params params) {
    ggml_context * c = new ggml_context;
    c->mem_size = params.mem_size;
    c->no_alloc = params.no_alloc;
    if (params.mem_buffer) {
        c->mem_buffer = (char *) params.mem_buffer;
    } else if (params.mem_size) {
        void * p = nullptr;
        if (posix_memalign(&p, MEM_ALIGN, params.mem_size) != 0) {
            delete c;
            return nullptr;
        }
        c->mem_buffer = (char *) p;
        c->mem_owned = true;
    }
    return c;
}

void ggml_free(struct ggml_context * ctx) {
    if (!ctx) return;
    if (ctx->mem_owned) free(ctx->mem_buffer);
    delete ctx;
}

size_t ggml_used_mem(const struct ggml_context * ctx) {
    return ctx->objects_end ? ctx->objects_end->offs + ctx->objects_end->size : 0;
}

size_t ggml_set_scratch(struct ggml_context * ctx, struct ggml_scratch scratch) {
    const size_t used = ctx->scratch.offs;
    ctx->scratch = scratch;
    return used;
}

// ---------------------------------------------------------------------------
// tensors
// ---------------------------------------------------------------------------
struct ggml_tensor * ggml_new_tensor(struct ggml_context * ctx, enum ggml_type type, int n_dims, const int64_t * ne) {
    return new_tensor_impl(ctx, type, n_dims, ne, nullptr);
}
struct ggml_tensor * ggml_new_tensor_1d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0) {
    return new_tensor_impl(ctx, type, 1, &ne0, nullptr);
}
struct ggml_tensor * ggml_new_tensor_2d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1) {
    const int64_t ne[2] = {ne0, ne1};
    return new_tensor_impl(ctx, type, 2, ne, nullptr);
}
struct ggml_tensor * ggml_new_tensor_3d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1,
                                        int64_t ne2) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    return new_tensor_impl(ctx, type, 3, ne, nullptr);
}
struct ggml_tensor * ggml_new_tensor_4d(struct ggml_context * ctx, enum ggml_type type, int64_t ne0, int64_t ne1,
                                        int64_t ne2, int64_t ne3) {
    const int64_t ne[4] = {ne0, ne1, ne2, ne3};
    return new_tensor_impl(ctx, type, 4, ne, nullptr);
}
struct ggml_tensor * ggml_new_i32(struct ggml_context * ctx, int32_t value) {
    ggml_tensor * t = new_param_tensor(ctx, GGML_TYPE_I32, 1);
    ggml_set_i32(t, value);
    return t;
}
struct ggml_tensor * ggml_new_f32(struct ggml_context * ctx, float value) {
    ggml_tensor * t = new_param_tensor(ctx, GGML_TYPE_F32, 1);
    ggml_set_f32(t, value);
    return t;
}
struct ggml_tensor * ggml_dup_tensor(struct ggml_context * ctx, const struct ggml_tensor * src) {
    return new_tensor_impl(ctx, src->type, src->n_dims, src->ne, nullptr);
}
struct ggml_tensor * ggml_view_tensor(struct ggml_context * ctx, const struct ggml_tensor * src) {
    ggml_tensor * t = new_tensor_impl(ctx, src->type, src->n_dims, src->ne, src->data);
    for (int i = 0; i < GGML_MAX_DIMS; ++i) t->nb[i] = src->nb[i];
    return t;
}

struct ggml_tensor * ggml_set_zero(struct ggml_tensor * t) {
    std::memset(t->data, 0, ggml_nbytes(t));
    return t;
}

int32_t ggml_get_i32_1d(const struct ggml_tensor * t, int i) {
    switch (t->type) {
        case GGML_TYPE_I8: return ((int8_t *) t->data)[i];
        case GGML_TYPE_I16: return ((int16_t *) t->data)[i];
        case GGML_TYPE_I32: return ((int32_t *) t->data)[i];
        case GGML_TYPE_F16: return (int32_t) h_f16_to_f32(((uint16_t *) t->data)[i]);
        case GGML_TYPE_F32: return (int32_t) ((float *) t->data)[i];
        default: gabort("ggml_get_i32_1d: quantized tensor");
    }
}
void ggml_set_i32_1d(const struct ggml_tensor * t, int i, int32_t v) {
    switch (t->type) {
        case GGML_TYPE_I8: ((int8_t *) t->data)[i] = (int8_t) v; break;
        case GGML_TYPE_I16: ((int16_t *) t->data)[i] = (int16_t) v; break;
        case GGML_TYPE_I32: ((int32_t *) t->data)[i] = v; break;
        case GGML_TYPE_F16: ((uint16_t *) t->data)[i] = h_f32_to_f16((float) v); break;
        case GGML_TYPE_F32: ((float *) t->data)[i] = (float) v; break;
        default: gabort("ggml_set_i32_1d: quantized tensor");
    }
}
float ggml_get_f32_1d(const struct ggml_tensor * t, int i) {
    switch (t->type) {
        case GGML_TYPE_I8: return ((int8_t *) t->data)[i];
        case GGML_TYPE_I16: return ((int16_t *) t->data)[i];
        case GGML_TYPE_I32: return (float) ((int32_t *) t->data)[i];
        case GGML_TYPE_F16: return h_f16_to_f32(((uint16_t *) t->data)[i]);
        case GGML_TYPE_F32: return ((float *) t->data)[i];
        default: gabort("ggml_get_f32_1d: quantized tensor");
    }
}
void ggml_set_f32_1d(const struct ggml_tensor * t, int i, float v) {
    switch (t->type) {
        case GGML_TYPE_I8: ((int8_t *) t->data)[i] = (int8_t) v; break;
        case GGML_TYPE_I16: ((int16_t *) t->data)[i] = (int16_t) v; break;
        case GGML_TYPE_I32: ((int32_t *) t->data)[i] = (int32_t) v; break;
        case GGML_TYPE_F16: ((uint16_t *) t->data)[i] = h_f32_to_f16(v); break;
        case GGML_TYPE_F32: ((float *) t->data)[i] = v; break;
        default: gabort("ggml_set_f32_1d: quantized tensor");
    }
}
struct ggml_tensor * ggml_set_i32(struct ggml_tensor * t, int32_t v) {
    const int64_t n = ggml_nelements(t);
    for (int64_t i = 0; i < n; ++i) ggml_set_i32_1d(t, (int) i, v);
    return t;
}
struct ggml_tensor * ggml_set_f32(struct ggml_tensor * t, float v) {
    const int64_t n = ggml_nelements(t);
    for (int64_t i = 0; i < n; ++i) ggml_set_f32_1d(t, (int) i, v);
    return t;
}
void * ggml_get_data(const struct ggml_tensor * t) { return t->data; }
float * ggml_get_data_f32(const struct ggml_tensor * t) {
    G_ASSERT(t->type == GGML_TYPE_F32);
    return (float *) t->data;
}

// ---------------------------------------------------------------------------
// operators (graph nodes)
// ---------------------------------------------------------------------------
struct ggml_tensor * ggml_dup(struct ggml_context * ctx, struct ggml_tensor * a) { return unary_node(ctx, a, GGML_OP_DUP); }
struct ggml_tensor * ggml_add(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    return binary_node(ctx, a, b, GGML_OP_ADD);
}
struct ggml_tensor * ggml_sub(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    return binary_node(ctx, a, b, GGML_OP_SUB);
}
struct ggml_tensor * ggml_mul(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    return binary_node(ctx, a, b, GGML_OP_MUL);
}
struct ggml_tensor * ggml_div(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    return binary_node(ctx, a, b, GGML_OP_DIV);
}
struct ggml_tensor * ggml_repeat(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    G_ASSERT(b->ne[0] % a->ne[0] == 0 && b->ne[1] % a->ne[1] == 0 && b->ne[2] % a->ne[2] == 0 &&
             b->ne[3] % a->ne[3] == 0);
    if (same_shape(a, b) && !a->is_param) return a;
    ggml_tensor * r = new_tensor_impl(ctx, a->type, b->n_dims, b->ne, nullptr);
    r->op = GGML_OP_REPEAT;
    r->src0 = a;
    r->src1 = b;
    return r;
}
struct ggml_tensor * ggml_silu(struct ggml_context * ctx, struct ggml_tensor * a) { return unary_node(ctx, a, GGML_OP_SILU); }
struct ggml_tensor * ggml_rms_norm(struct ggml_context * ctx, struct ggml_tensor * a) {
    return unary_node(ctx, a, GGML_OP_RMS_NORM);
}
struct ggml_tensor * ggml_mul_mat(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    G_ASSERT(a->ne[0] == b->ne[0] && a->ne[2] == b->ne[2] && a->ne[3] == b->ne[3]);
    const int64_t ne[4] = {a->ne[1], b->ne[1], a->ne[2], b->ne[3]};
    ggml_tensor * r = new_tensor_impl(ctx, GGML_TYPE_F32, std::min(a->n_dims, b->n_dims), ne, nullptr);
    r->op = GGML_OP_MUL_MAT;
    r->src0 = a;
    r->src1 = b;
    return r;
}
struct ggml_tensor * ggml_scale(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    G_ASSERT(ggml_nelements(b) == 1);
    G_ASSERT(a->nb[0] == TYPE_SIZE[a->type] && a->nb[1] == a->nb[0] * a->ne[0]);   // padded 1d rows
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    r->op = GGML_OP_SCALE;
    r->src0 = a;
    r->src1 = b;
    return r;
}
struct ggml_tensor * ggml_cpy(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    G_ASSERT(ggml_nelements(a) == ggml_nelements(b));
    ggml_tensor * r = ggml_view_tensor(ctx, b);
    r->op = GGML_OP_CPY;
    r->src0 = a;
    r->src1 = b;
    return r;
}
struct ggml_tensor * ggml_reshape(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    G_ASSERT(is_contiguous(a) && is_contiguous(b) && ggml_nelements(a) == ggml_nelements(b));
    ggml_tensor * r = new_tensor_impl(ctx, a->type, b->n_dims, b->ne, a->data);
    r->op = GGML_OP_RESHAPE;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_reshape_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1) {
    G_ASSERT(is_contiguous(a) && ggml_nelements(a) == ne0 * ne1);
    const int64_t ne[2] = {ne0, ne1};
    ggml_tensor * r = new_tensor_impl(ctx, a->type, 2, ne, a->data);
    r->op = GGML_OP_RESHAPE;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_reshape_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1,
                                     int64_t ne2) {
    G_ASSERT(is_contiguous(a) && ggml_nelements(a) == ne0 * ne1 * ne2);
    const int64_t ne[3] = {ne0, ne1, ne2};
    ggml_tensor * r = new_tensor_impl(ctx, a->type, 3, ne, a->data);
    r->op = GGML_OP_RESHAPE;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_view_1d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, size_t offset) {
    ggml_tensor * r = new_tensor_impl(ctx, a->type, 1, &ne0, (char *) a->data + offset);
    r->op = GGML_OP_VIEW;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_view_2d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1,
                                  size_t nb1, size_t offset) {
    const int64_t ne[2] = {ne0, ne1};
    ggml_tensor * r = new_tensor_impl(ctx, a->type, 2, ne, (char *) a->data + offset);
    r->nb[1] = nb1;
    r->nb[2] = r->nb[1] * ne1;
    r->nb[3] = r->nb[2];
    r->op = GGML_OP_VIEW;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_view_3d(struct ggml_context * ctx, struct ggml_tensor * a, int64_t ne0, int64_t ne1,
                                  int64_t ne2, size_t nb1, size_t nb2, size_t offset) {
    const int64_t ne[3] = {ne0, ne1, ne2};
    ggml_tensor * r = new_tensor_impl(ctx, a->type, 3, ne, (char *) a->data + offset);
    r->nb[1] = nb1;
    r->nb[2] = nb2;
    r->nb[3] = r->nb[2] * ne2;
    r->op = GGML_OP_VIEW;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_permute(struct ggml_context * ctx, struct ggml_tensor * a, int axis0, int axis1, int axis2,
                                  int axis3) {
    const int ax[4] = {axis0, axis1, axis2, axis3};
    for (int i = 0; i < 4; ++i) {
        G_ASSERT(ax[i] >= 0 && ax[i] < GGML_MAX_DIMS);
        for (int k = 0; k < i; ++k) G_ASSERT(ax[i] != ax[k]);
    }
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    for (int i = 0; i < 4; ++i) {
        r->ne[ax[i]] = a->ne[i];
        r->nb[ax[i]] = a->nb[i];
    }
    r->op = GGML_OP_PERMUTE;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_transpose(struct ggml_context * ctx, struct ggml_tensor * a) {
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    std::swap(r->ne[0], r->ne[1]);
    std::swap(r->nb[0], r->nb[1]);
    r->op = GGML_OP_TRANSPOSE;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_get_rows(struct ggml_context * ctx, struct ggml_tensor * a, struct ggml_tensor * b) {
    G_ASSERT(a->ne[2] == 1 && a->ne[3] == 1 && b->ne[1] == 1 && b->ne[2] == 1 && b->ne[3] == 1 &&
             b->type == GGML_TYPE_I32);
    ggml_tensor * r = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, a->ne[0], b->ne[0]);
    r->op = GGML_OP_GET_ROWS;
    r->src0 = a;
    r->src1 = b;
    return r;
}
struct ggml_tensor * ggml_diag_mask_inf(struct ggml_context * ctx, struct ggml_tensor * a, int n_past) {
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    ggml_tensor * b = new_param_tensor(ctx, GGML_TYPE_I32, 1);
    ((int32_t *) b->data)[0] = n_past;
    r->op = GGML_OP_DIAG_MASK_INF;
    r->src0 = a;
    r->src1 = b;
    return r;
}
struct ggml_tensor * ggml_soft_max(struct ggml_context * ctx, struct ggml_tensor * a) {
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    r->op = GGML_OP_SOFT_MAX;
    r->src0 = a;
    return r;
}
struct ggml_tensor * ggml_rope(struct ggml_context * ctx, struct ggml_tensor * a, int n_past, int n_dims, int mode) {
    G_ASSERT(n_past >= 0);
    ggml_tensor * r = ggml_view_tensor(ctx, a);
    ggml_tensor * b = new_param_tensor(ctx, GGML_TYPE_I32, 3);
    ((int32_t *) b->data)[0] = n_past;
    ((int32_t *) b->data)[1] = n_dims;
    ((int32_t *) b->data)[2] = mode;
    r->op = GGML_OP_ROPE;
    r->src0 = a;
    r->src1 = b;
    return r;
}

void ggml_set_param(struct ggml_context * ctx, struct ggml_tensor * tensor) {
    tensor->is_param = true;
    G_ASSERT(tensor->grad == nullptr);
    tensor->grad = ggml_dup_tensor(ctx, tensor);
}

// ---------------------------------------------------------------------------
// graphs: depth-first over src0, src1, opt[], leaves before their users (ggml.c
// ggml_visit_parents / ggml_build_forward_impl)
// ---------------------------------------------------------------------------
static void visit_parents(ggml_cgraph * g, ggml_tensor * node) {
    for (int i = 0; i < g->n_nodes; ++i)
        if (g->nodes[i] == node) return;
    for (int i = 0; i < g->n_leafs; ++i)
        if (g->leafs[i] == node) return;
    if (node->src0) visit_parents(g, node->src0);
    if (node->src1) visit_parents(g, node->src1);
    for (int i = 0; i < GGML_MAX_OPT; ++i)
        if (node->opt[i]) visit_parents(g, node->opt[i]);
    if (node->op == GGML_OP_NONE && node->grad == nullptr) {
        G_ASSERT(g->n_leafs < GGML_MAX_NODES);
        g->leafs[g->n_leafs++] = node;
    } else {
        G_ASSERT(g->n_nodes < GGML_MAX_NODES);
        g->nodes[g->n_nodes] = node;
        g->grads[g->n_nodes] = node->grad;
        g->n_nodes++;
    }
}

void ggml_build_forward_expand(struct ggml_cgraph * cgraph, struct ggml_tensor * tensor) {
    const int n0 = cgraph->n_nodes;
    visit_parents(cgraph, tensor);
    if (cgraph->n_nodes > n0) G_ASSERT(cgraph->nodes[cgraph->n_nodes - 1] == tensor);
}

struct ggml_cgraph ggml_build_forward(struct ggml_tensor * tensor) {
    ggml_cgraph g;
    std::memset(&g, 0, sizeof(g));
    ggml_build_forward_expand(&g, tensor);
    return g;
}

void ggml_graph_reset(struct ggml_cgraph * cgraph) {
    for (int i = 0; i < cgraph->n_nodes; ++i)
        if (cgraph->grads[i]) ggml_set_zero(cgraph->grads[i]);
}

void ggml_graph_print(const struct ggml_cgraph * cgraph) {
    fprintf(stderr, "=== GRAPH ===\nn_nodes = %d\n", cgraph->n_nodes);
    for (int i = 0; i < cgraph->n_nodes; ++i) {
        const ggml_tensor * n = cgraph->nodes[i];
        fprintf(stderr, " - %3d: [ %" PRId64 ", %" PRId64 ", %" PRId64 "] op %d\n", i, n->ne[0], n->ne[1], n->ne[2], (int) n->op);
    }
    fprintf(stderr, "n_leafs = %d\n", cgraph->n_leafs);
    for (int i = 0; i < cgraph->n_leafs; ++i) {
        const ggml_tensor * n = cgraph->leafs[i];
        fprintf(stderr, " - %3d: [ %" PRId64 ", %" PRId64 "]\n", i, n->ne[0], n->ne[1]);
    }
    fprintf(stderr, "========================================\n");
}

int ggml_cpu_has_avx(void) { return __builtin_cpu_supports("avx") ? 1 : 0; }
int ggml_cpu_has_avx2(void) { return __builtin_cpu_supports("avx2") ? 1 : 0; }
int ggml_cpu_has_avx512(void) { return __builtin_cpu_supports("avx512f") ? 1 : 0; }
int ggml_cpu_has_fma(void) { return __builtin_cpu_supports("fma") ? 1 : 0; }
int ggml_cpu_has_f16c(void) { return 1; }
int ggml_cpu_has_blas(void) { return 0; }

}  // extern "C"

// ---------------------------------------------------------------------------
// ggml_graph_compute on the GPU
// ---------------------------------------------------------------------------
namespace {

// bytes a strided tensor spans from its data pointer
size_t span_bytes(const ggml_tensor * t) {
    // quantized rows are contiguous blocks; other types may have any stride in any
    // dimension (a transpose swaps nb[0] and nb[1])
    const bool quant = BLCK_SIZE[t->type] > 1;
    size_t s = quant ? (size_t) (t->ne[0] / BLCK_SIZE[t->type]) * TYPE_SIZE[t->type] : TYPE_SIZE[t->type];
    for (int d = quant ? 1 : 0; d < GGML_MAX_DIMS; ++d)
        if (t->ne[d] > 1) s += (size_t) (t->ne[d] - 1) * t->nb[d];
    return s;
}

struct Region {
    char * lo;
    char * hi;
    char * dev = nullptr;
    bool written = false;
};

// the device state of one ggml_graph_compute call
struct GraphRun {
    std::vector<Region> regions;
    std::vector<void *> temps;
    hipStream_t stream = nullptr;

    ~GraphRun() {
        if (stream) (void) hipStreamSynchronize(stream);
        for (Region & r : regions)
            if (r.dev) (void) hipFree(r.dev);
        for (void * p : temps) (void) hipFree(p);
        if (stream) (void) hipStreamDestroy(stream);
    }
    void * temp(size_t n) {
        void * p = nullptr;
        LVK_HIP(hipMalloc(&p, n ? n : 16));
        temps.push_back(p);
        return p;
    }
    Region & region_of(const void * p) {
        const char * c = (const char *) p;
        auto it = std::upper_bound(regions.begin(), regions.end(), c, [](const char * v, const Region & r) { return v < r.lo; });
        if (it == regions.begin()) gabort("ggml_graph_compute: tensor outside the mapped buffers");
        --it;
        if (c >= it->hi) gabort("ggml_graph_compute: tensor outside the mapped buffers");
        return *it;
    }
    char * dev(const void * p) {
        Region & r = region_of(p);
        return r.dev + ((const char *) p - r.lo);
    }
    lvk::GView view(const ggml_tensor * t) {
        lvk::GView v;
        v.p = dev(t->data);
        for (int i = 0; i < 4; ++i) {
            v.ne[i] = t->ne[i];
            v.nb[i] = (int64_t) t->nb[i];
        }
        v.type = (int) t->type;
        return v;
    }
    // contiguous device copy of a f32 tensor's rows, optionally converted to f16 (RNE)
    void * gather(const ggml_tensor * t, lvk::GType to) {
        const size_t es = to == lvk::GT_F16 ? 2 : 4;
        void * p = temp((size_t) ggml_nelements(t) * es);
        lvk::GView d;
        d.p = (char *) p;
        for (int i = 0; i < 4; ++i) d.ne[i] = t->ne[i];
        d.nb[0] = (int64_t) es;
        for (int i = 1; i < 4; ++i) d.nb[i] = d.nb[i - 1] * d.ne[i - 1];
        d.type = to;
        LVK_HIP(lvk::launch_g_cpy(view(t), d, stream));
        return p;
    }
    template <class T> T read_scalar(const ggml_tensor * t, int i) {
        T v;
        LVK_HIP(hipMemcpyAsync(&v, dev((const char *) t->data + (size_t) i * sizeof(T)), sizeof(T), hipMemcpyDeviceToHost, stream));
        LVK_HIP(hipStreamSynchronize(stream));
        return v;
    }
};

// fp16 exp / silu tables of this host's glibc (ggml.c:2915-2927) and the softmax exp mode,
// once per device
struct Tables {
    uint16_t * exp_tab = nullptr;
    uint16_t * silu_tab = nullptr;
    int exp_mode = 0;
};
const Tables & tables() {
    static std::map<int, Tables> per_dev;
    int dev = 0;
    LVK_HIP(hipGetDevice(&dev));
    auto it = per_dev.find(dev);
    if (it != per_dev.end()) return it->second;
    Tables t;
    std::vector<uint16_t> te, ts;
    lvk::host_fp16_tables(te, ts);
    LVK_HIP(hipMalloc(&t.exp_tab, 65536 * 2));
    LVK_HIP(hipMalloc(&t.silu_tab, 65536 * 2));
    LVK_HIP(hipMemcpy(t.exp_tab, te.data(), 65536 * 2, hipMemcpyHostToDevice));
    LVK_HIP(hipMemcpy(t.silu_tab, ts.data(), 65536 * 2, hipMemcpyHostToDevice));
    t.exp_mode = lvk::pick_exp_mode(t.exp_tab);
    return per_dev.emplace(dev, t).first->second;
}

void run_mul_mat_q(GraphRun & R, const ggml_tensor * a, const ggml_tensor * b, ggml_tensor * node) {
    // ggml_compute_forward_mul_mat_q_f32 (ggml.c:6510-6696): every src1 row quantized with
    // the AVX2 quantizer, one vec_dot_q per (row, column) -- the matvec kernels' arithmetic
    const int M = (int) a->ne[1], K = (int) a->ne[0], N = (int) b->ne[1];
    const int qt = a->type == GGML_TYPE_Q4_0 ? lvk::Q4_0 : lvk::Q4_1;
    if (M % 8 || K % 256) gabort("ggml_graph_compute: Q4 mul_mat needs ne01 % 8 == 0 and ne00 % 256 == 0");
    G_ASSERT(a->nb[1] == (size_t) (K / 32) * TYPE_SIZE[a->type]);
    for (int64_t i3 = 0; i3 < a->ne[3]; ++i3)
        for (int64_t i2 = 0; i2 < a->ne[2]; ++i2) {
            lvk::QMatrix q;
            q.qtype = qt; q.M = M; q.K = K;
            q.nib = (const uint4 *) R.temp(lvk::qimage_nib_bytes(M, K));
            q.scl = R.temp(lvk::qimage_scl_bytes(M, K, qt));
            const char * w = R.dev((const char *) a->data + i2 * a->nb[2] + i3 * a->nb[3]);
            LVK_HIP(lvk::launch_repack(w, qt, M, K, (uint4 *) q.nib, (void *) q.scl, R.stream));
            // this batch's src1 rows, contiguous
            ggml_tensor bs = *b;
            bs.data = (char *) b->data + i2 * b->nb[2] + i3 * b->nb[3];
            bs.ne[2] = bs.ne[3] = 1;
            float * x = (float *) R.gather(&bs, lvk::GT_F32);
            float * y = (float *) R.temp((size_t) N * M * 4);
            lvk::StepParams sp{0, N, 0, 0};
            lvk::StepParams * spd = (lvk::StepParams *) R.temp(sizeof sp);
            LVK_HIP(hipMemcpyAsync(spd, &sp, sizeof sp, hipMemcpyHostToDevice, R.stream));
            LVK_HIP(hipStreamSynchronize(R.stream));      // sp is this scope's host memory
            lvk::MvLaunch L;
            L.w = q; L.sp = spd; L.n_tokens = N; L.y = y;
            if (qt == lvk::Q4_1) {
                L.x = x;
                LVK_HIP(lvk::launch_matvec(L, lvk::PRO_ACTF, lvk::EPI_STORE, R.stream));
            } else {
                lvk::ActQ aq;
                aq.nb = K / 32;
                aq.d = (float *) R.temp((size_t) N * aq.nb * 4);
                aq.m = (float *) R.temp((size_t) N * aq.nb * 4);
                aq.qs = (uint4 *) R.temp((size_t) N * aq.nb * 16);
                LVK_HIP(lvk::launch_quantize_act(x, N, K, qt, aq, R.stream));
                L.xq = aq;
                LVK_HIP(lvk::launch_matvec(L, lvk::PRO_ACTQ, lvk::EPI_STORE, R.stream));
            }
            // [N][M] -> the node's (i2, i3) slice
            lvk::GView s;
            s.p = (char *) y;
            s.ne[0] = M; s.ne[1] = N;
            s.nb[0] = 4; s.nb[1] = (int64_t) M * 4; s.nb[2] = s.nb[3] = s.nb[1] * N;
            lvk::GView d = R.view(node);
            d.p += i2 * node->nb[2] + i3 * node->nb[3];
            d.ne[2] = d.ne[3] = 1;
            LVK_HIP(lvk::launch_g_cpy(s, d, R.stream));
        }
}

void run_node(GraphRun & R, ggml_tensor * n) {
    ggml_tensor * a = n->src0;
    ggml_tensor * b = n->src1;
    switch (n->op) {
        case GGML_OP_NONE:
        case GGML_OP_RESHAPE:
        case GGML_OP_VIEW:
        case GGML_OP_PERMUTE:
        case GGML_OP_TRANSPOSE:
            return;
        case GGML_OP_DUP:
        case GGML_OP_CPY:
            G_ASSERT(a->type == GGML_TYPE_F32 || a->type == GGML_TYPE_F16);
            G_ASSERT(n->type == GGML_TYPE_F32 || n->type == GGML_TYPE_F16);
            LVK_HIP(lvk::launch_g_cpy(R.view(a), R.view(n), R.stream));
            return;
        case GGML_OP_ADD:
        case GGML_OP_SUB:
        case GGML_OP_MUL:
        case GGML_OP_DIV: {
            G_ASSERT(a->type == GGML_TYPE_F32 && b->type == GGML_TYPE_F32 && n->type == GGML_TYPE_F32);
            const int op = n->op == GGML_OP_ADD ? lvk::GOP_ADD : n->op == GGML_OP_SUB ? lvk::GOP_SUB
                         : n->op == GGML_OP_MUL ? lvk::GOP_MUL : lvk::GOP_DIV;
            LVK_HIP(lvk::launch_g_binary(R.view(a), R.view(b), R.view(n), op, R.stream));
            return;
        }
        case GGML_OP_REPEAT:
            G_ASSERT(a->type == GGML_TYPE_F32);
            LVK_HIP(lvk::launch_g_binary(R.view(a), R.view(a), R.view(n), lvk::GOP_REPEAT, R.stream));
            return;
        case GGML_OP_SILU:
            G_ASSERT(a->type == GGML_TYPE_F32);
            LVK_HIP(lvk::launch_g_unary(R.view(a), R.view(n), lvk::GOP_SILU, 0.0f, 0, tables().silu_tab, R.stream));
            return;
        case GGML_OP_SCALE:
            G_ASSERT(a->type == GGML_TYPE_F32 && b->type == GGML_TYPE_F32);
            LVK_HIP(lvk::launch_g_unary(R.view(a), R.view(n), lvk::GOP_SCALE, R.read_scalar<float>(b, 0), 0, nullptr,
                                        R.stream));
            return;
        case GGML_OP_DIAG_MASK_INF:
            G_ASSERT(a->type == GGML_TYPE_F32);
            LVK_HIP(lvk::launch_g_unary(R.view(a), R.view(n), lvk::GOP_DIAG_MASK, 0.0f, R.read_scalar<int32_t>(b, 0),
                                        nullptr, R.stream));
            return;
        case GGML_OP_RMS_NORM:
            G_ASSERT(a->type == GGML_TYPE_F32);
            LVK_HIP(lvk::launch_g_rms_norm(R.view(a), R.view(n), R.stream));
            return;
        case GGML_OP_SOFT_MAX: {
            G_ASSERT(a->type == GGML_TYPE_F32);
            const Tables & T = tables();
            if (n->data != a->data) LVK_HIP(lvk::launch_g_cpy(R.view(a), R.view(n), R.stream));
            LVK_HIP(lvk::launch_g_soft_max(R.view(n), T.exp_tab, T.exp_mode, R.stream));
            return;
        }
        case GGML_OP_ROPE: {
            G_ASSERT(a->type == GGML_TYPE_F32 && a->nb[0] == sizeof(float));
            const int n_past = R.read_scalar<int32_t>(b, 0), n_dims = R.read_scalar<int32_t>(b, 1);
            const int mode = R.read_scalar<int32_t>(b, 2);
            G_ASSERT(n_dims % 2 == 0 && n_dims <= a->ne[0]);
            if (n->data != a->data) LVK_HIP(lvk::launch_g_cpy(R.view(a), R.view(n), R.stream));
            // {cos, sin} of p * theta_i0, theta = powf(10000, -i0 / n_dims) (ggml.c:7209-7213)
            const int i2_0 = mode == 0 ? 0 : n_past;
            const int64_t rows = a->ne[2] - i2_0;
            if (rows <= 0) return;
            std::vector<float2> cs((size_t) rows * (n_dims / 2));
            for (int64_t t = 0; t < rows; ++t) {
                const int p = mode == 0 ? n_past + (int) t : i2_0 + (int) t;
                for (int i0 = 0; i0 < n_dims; i0 += 2) {
                    const float theta = powf(10000.0f, ((float) -i0) / (float) n_dims);
                    const float ang = (float) p * theta;
                    cs[(size_t) t * (n_dims / 2) + i0 / 2] = make_float2(cosf(ang), sinf(ang));
                }
            }
            float2 * csd = (float2 *) R.temp(cs.size() * sizeof(float2));
            LVK_HIP(hipMemcpyAsync(csd, cs.data(), cs.size() * sizeof(float2), hipMemcpyHostToDevice, R.stream));
            LVK_HIP(lvk::launch_g_rope(R.view(n), R.view(n), csd, n_dims, i2_0, R.stream));
            LVK_HIP(hipStreamSynchronize(R.stream));     // cs is host memory of this scope
            return;
        }
        case GGML_OP_GET_ROWS:
            G_ASSERT(b->type == GGML_TYPE_I32 && n->type == GGML_TYPE_F32);
            G_ASSERT(a->type == GGML_TYPE_Q4_0 || a->type == GGML_TYPE_Q4_1 || a->type == GGML_TYPE_F16 ||
                     a->type == GGML_TYPE_F32);
            if (b->op == GGML_OP_NONE)
                for (int64_t i = 0; i < b->ne[0]; ++i) {
                    const int32_t id = ((const int32_t *) b->data)[i];
                    if (id < 0 || id >= a->ne[1]) gabort("ggml_get_rows: row index out of range");
                }
            LVK_HIP(lvk::launch_g_get_rows(R.view(a), (const int32_t *) R.dev(b->data), b->ne[0], R.view(n), R.stream));
            return;
        case GGML_OP_MUL_MAT:
            G_ASSERT(b->type == GGML_TYPE_F32 && b->nb[0] == sizeof(float) && n->nb[0] == sizeof(float));
            if (a->type == GGML_TYPE_Q4_0 || a->type == GGML_TYPE_Q4_1) {
                run_mul_mat_q(R, a, b, n);
            } else if (a->type == GGML_TYPE_F16 || a->type == GGML_TYPE_F32) {
                // ggml.c:6134-6487: src1 to contiguous rows (f16 for an f16 src0: the INIT phase)
                G_ASSERT(a->nb[0] == TYPE_SIZE[a->type]);
                void * y = R.gather(b, a->type == GGML_TYPE_F16 ? lvk::GT_F16 : lvk::GT_F32);
                LVK_HIP(lvk::launch_g_mm_dot(R.view(a), y, b->ne[1], R.view(n), R.stream));
            } else {
                gabort("ggml_graph_compute: mul_mat source type not supported");
            }
            return;
        default: {
            char msg[96];
            snprintf(msg, sizeof msg, "ggml_graph_compute: op %d has no GPU implementation in llama.vk_amd", (int) n->op);
            gabort(msg);
        }
    }
}

}  // namespace

extern "C" void ggml_graph_compute(struct ggml_context * ctx, struct ggml_cgraph * cgraph) {
    (void) ctx;
    try {
        GraphRun R;
        // every buffer range the graph reads or writes, merged into regions
        std::vector<const ggml_tensor *> ts;
        auto add = [&](const ggml_tensor * t) {
            if (!t) return;
            if (!t->data) gabort("ggml_graph_compute: a tensor has no data (no_alloc context)");
            ts.push_back(t);
        };
        for (int i = 0; i < cgraph->n_leafs; ++i) add(cgraph->leafs[i]);
        for (int i = 0; i < cgraph->n_nodes; ++i) {
            const ggml_tensor * n = cgraph->nodes[i];
            add(n);
            add(n->src0);
            add(n->src1);
            for (int k = 0; k < GGML_MAX_OPT; ++k) add(n->opt[k]);
        }
        std::vector<Region> sp;
        for (const ggml_tensor * t : ts) sp.push_back({(char *) t->data, (char *) t->data + span_bytes(t)});
        std::sort(sp.begin(), sp.end(), [](const Region & x, const Region & y) { return x.lo < y.lo; });
        for (const Region & r : sp) {
            if (!R.regions.empty() && r.lo <= R.regions.back().hi) R.regions.back().hi = std::max(R.regions.back().hi, r.hi);
            else R.regions.push_back(r);
        }
        LVK_HIP(hipStreamCreateWithFlags(&R.stream, hipStreamNonBlocking));
        for (Region & r : R.regions) {
            LVK_HIP(hipMalloc(&r.dev, (size_t) (r.hi - r.lo) + 16));
            LVK_HIP(hipMemcpyAsync(r.dev, r.lo, (size_t) (r.hi - r.lo), hipMemcpyHostToDevice, R.stream));
        }
        // LVK_GGML_SYNC=1: wait for every node and name the one that fails (debugging)
        static const bool sync_each = getenv("LVK_GGML_SYNC") && atoi(getenv("LVK_GGML_SYNC")) != 0;
        for (int i = 0; i < cgraph->n_nodes; ++i) {
            ggml_tensor * n = cgraph->nodes[i];
            run_node(R, n);
            if (n->op != GGML_OP_NONE) R.region_of(n->data).written = true;
            if (sync_each) {
                const hipError_t e = hipStreamSynchronize(R.stream);
                if (e != hipSuccess) {
                    fprintf(stderr, "ggml_graph_compute: node %d (op %d, type %d, ne %lld %lld %lld %lld) failed: %s\n", i,
                            (int) n->op, (int) n->type, (long long) n->ne[0], (long long) n->ne[1], (long long) n->ne[2],
                            (long long) n->ne[3], hipGetErrorString(e));
                    abort();
                }
            }
        }
        for (Region & r : R.regions)
            if (r.written) LVK_HIP(hipMemcpyAsync(r.lo, r.dev, (size_t) (r.hi - r.lo), hipMemcpyDeviceToHost, R.stream));
        LVK_HIP(hipStreamSynchronize(R.stream));
        cgraph->perf_runs++;
    } catch (const lvk::Error & e) {
        gabort(e.msg.c_str());
    }
}
