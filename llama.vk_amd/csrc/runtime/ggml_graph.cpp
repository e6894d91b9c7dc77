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
//     bytes the nodes wrote back.  The mirrors, the repacked Q4 images and the temporaries'
//     arena persist across calls: only host pages written since the previous call travel
//     again (soft-dirty page tracking, below), so a caller's weights upload once.  An operator without a GPU implementation aborts -- there is no
//     CPU fallback.
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include "../../../include/ggml.h"
#include "../../../include/lvk_ops.h"
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
int ggml_cpu_has_neon(void) { return 0; }
int ggml_cpu_has_arm_fma(void) { return 0; }
int ggml_cpu_has_f16c(void) { return 1; }
int ggml_cpu_has_fp16_va(void) { return 0; }
int ggml_cpu_has_wasm_simd(void) { return 0; }
int ggml_cpu_has_blas(void) { return 0; }
int ggml_cpu_has_sse3(void) { return __builtin_cpu_supports("sse3") ? 1 : 0; }
int ggml_cpu_has_vsx(void) { return 0; }

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

// ---- host change tracking -------------------------------------------------------------
// A graph's tensors live in caller memory that the caller may rewrite between calls (the next
// token ids, a KV cache it restored ...), while most of it -- the weights -- never changes.
// The mirrors below keep host ranges in HBM across calls and upload a page again only when
// the host may have written it since it was uploaded:
//   * pages inside a mapping this process cannot write (llama.cpp's PROT_READ model-file
//     mapping, or a buffer the caller made read-only with mprotect) stay valid while that
//     mapping (address range, offset, device, inode, permissions in /proc/self/maps) is
//     unchanged -- a caller that re-enables writes, writes and protects again between two
//     calls must say so with lvk_ggml_invalidate;
//   * writable pages are uploaded again on every call.  LVK_GGML_CACHE=2 tracks them with
//     the kernel's soft-dirty bits instead (/proc/self/pagemap bit 55, cleared by "4" into
//     /proc/self/clear_refs; a new mapping reads dirty, a page that is neither present nor
//     swapped counts as written).  That is opt-in: the clear is process-wide, and in a HIP
//     process the call after it stalls for ~0.2 s (tools/ggml_graph/track_cost.c, DESIGN.md
//     section 5), more than re-uploading gigabytes of writable pages costs;
//   * pages the CPU-side tracking cannot see written are never kept: pages of shared mappings
//     (another mapping or process may write them; HIP's pinned host allocations are shared
//     mappings of the driver's device file) and host memory registered with HIP (a DMA into
//     it, e.g. hipMemcpy D2H, bypasses this process's page tables) are uploaded on every call;
//   * only bytes a node reads before any node of the call writes them are uploaded at all
//     (a node's output buffer never travels host -> device), and only the bytes the nodes
//     wrote travel back.
// The soft-dirty bits are per process: before a call clears them, every engine (one per
// device) folds the bits into the validity of all its mirrors.
// LVK_GGML_CACHE=0 turns the caching off (every needed page uploaded on every call); 1 (the
// default) keeps pages of read-only mappings; 2 adds the soft-dirty tracking of writable pages.
constexpr size_t PAGE = 4096;

uint64_t ns_since(std::chrono::steady_clock::time_point t0) {
    return (uint64_t) std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
}

struct MapEnt {
    uintptr_t lo = 0, hi = 0;
    uint64_t off = 0, inode = 0;
    char perms[5] = {0};
    char dev[16] = {0};
    bool same(const MapEnt & o) const {
        return lo == o.lo && hi == o.hi && off == o.off && inode == o.inode && !strcmp(perms, o.perms) &&
               !strcmp(dev, o.dev);
    }
};

std::vector<MapEnt> read_maps() {
    std::vector<MapEnt> v;
    FILE * f = fopen("/proc/self/maps", "r");
    if (!f) return v;
    char line[4096];
    while (fgets(line, sizeof line, f)) {
        MapEnt e;
        unsigned long lo = 0, hi = 0, off = 0, ino = 0;
        if (sscanf(line, "%lx-%lx %4s %lx %15s %lu", &lo, &hi, e.perms, &off, e.dev, &ino) < 6) continue;
        e.lo = lo; e.hi = hi; e.off = off; e.inode = ino;
        v.push_back(e);
    }
    fclose(f);
    return v;       // the kernel lists mappings in address order
}

const MapEnt * map_of(const std::vector<MapEnt> & v, uintptr_t a) {
    auto it = std::upper_bound(v.begin(), v.end(), a, [](uintptr_t x, const MapEnt & e) { return x < e.lo; });
    if (it == v.begin()) return nullptr;
    --it;
    return a < it->hi ? &*it : nullptr;
}

struct DirtyTracker {
    int pagemap = -1, clear_refs = -1;
    bool enabled = true;       // LVK_GGML_CACHE != 0
    bool ok = false;           // LVK_GGML_CACHE=2 and the soft-dirty bits work

    bool read(uintptr_t page0, size_t n, std::vector<uint64_t> & e) const {
        e.resize(n);
        const size_t want = n * 8;
        size_t got = 0;
        while (got < want) {
            const ssize_t r = pread(pagemap, (char *) e.data() + got, want - got, (off_t) (page0 * 8 + got));
            if (r <= 0) return false;
            got += (size_t) r;
        }
        return true;
    }
    static bool written(uint64_t e) {
        const bool present = (e >> 63) & 1, swapped = (e >> 62) & 1, soft_dirty = (e >> 55) & 1;
        return soft_dirty || (!present && !swapped);
    }
    bool clear() const { return pwrite(clear_refs, "4", 1, 0) == 1; }

    DirtyTracker() {
        const char * e = getenv("LVK_GGML_CACHE");
        const int mode = e ? atoi(e) : 1;
        if (mode == 0) { enabled = false; return; }
        if (mode != 2) return;
        pagemap = open("/proc/self/pagemap", O_RDONLY | O_CLOEXEC);
        clear_refs = open("/proc/self/clear_refs", O_WRONLY | O_CLOEXEC);
        if (pagemap < 0 || clear_refs < 0) return;
        // self-test on a page of our own: written -> cleared -> written again
        void * p = mmap(nullptr, PAGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) return;
        volatile char * c = (volatile char *) p;
        std::vector<uint64_t> v;
        const uintptr_t pg = (uintptr_t) p / PAGE;
        c[0] = 1;
        bool good = clear() && read(pg, 1, v) && !written(v[0]);
        c[1] = 2;
        good = good && read(pg, 1, v) && written(v[0]);
        munmap(p, PAGE);
        ok = good;
    }
};

DirtyTracker & tracker() {
    static DirtyTracker t;
    return t;
}

// a host range [lo, hi) mirrored in HBM; valid[i]: the bytes of host page (lo / PAGE + i)
// inside the range equal the device copy
struct Mirror {
    char * lo = nullptr;
    char * hi = nullptr;
    char * dev = nullptr;
    std::vector<uint8_t> valid;
    std::vector<int32_t> ro;       // per page: the read-only mapping it was uploaded from, or -1
    uint64_t last_call = 0;
    int hip_host = -1;             // 1: HIP-registered / pinned host memory (never cached); -1 unknown
    uint64_t maps_sig = 0;         // the mappings over [lo, hi) when hip_host was decided
    uintptr_t page0() const { return (uintptr_t) lo / PAGE; }
    size_t pages() const { return (uintptr_t) (hi - 1) / PAGE - page0() + 1; }
};

// a Q4 weight repacked into the decode kernels' octet image, keyed by its host address
struct Repacked {
    const char * lo;
    const char * hi;
    int qt, M, K;
    uint4 * nib = nullptr;
    void * scl = nullptr;
};

// grow-only device (or pinned host) arena, reset per call: no allocation per op
struct Arena {
    bool pinned = false;
    std::vector<std::pair<char *, size_t>> chunks;
    size_t cur = 0, off = 0;
    void * get(size_t n) {
        n = (n + 255) & ~(size_t) 255;
        if (n == 0) n = 256;
        while (cur < chunks.size()) {
            if (off + n <= chunks[cur].second) {
                void * p = chunks[cur].first + off;
                off += n;
                return p;
            }
            ++cur;
            off = 0;
        }
        const size_t sz = std::max(n, chunks.empty() ? (size_t) 1 << 20 : chunks.back().second * 2);
        void * p = nullptr;
        if (pinned) LVK_HIP(hipHostMalloc(&p, sz, hipHostMallocDefault));
        else LVK_HIP(hipMalloc(&p, sz));
        chunks.push_back({(char *) p, sz});
        cur = chunks.size() - 1;
        off = n;
        return p;
    }
    void reset() { cur = 0; off = 0; }
};

struct Span {
    const char * lo;
    const char * hi;
};
bool overlaps(const char * a0, const char * a1, const char * b0, const char * b1) { return a0 < b1 && b0 < a1; }

struct GraphStats {
    uint64_t h2d = 0, d2h = 0, repack = 0, mirrored = 0;
    uint64_t track_ns = 0, clear_ns = 0;   // host time of the validity bookkeeping / of clear_refs
};

// the persistent device state of ggml_graph_compute on one device
struct GraphEngine {
    hipStream_t stream = nullptr;
    std::vector<Mirror *> mirrors;          // sorted by lo, disjoint
    std::vector<Repacked> repacked;
    Arena dev_arena, host_arena;
    uint64_t calls = 0;
    GraphStats last;
    // this call
    std::vector<Mirror *> used;
    std::vector<Span> written;              // node outputs of this call, in order

    GraphEngine() {
        host_arena.pinned = true;
        LVK_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    }

    Mirror & mirror_of(const void * p) {
        const char * c = (const char *) p;
        auto it = std::upper_bound(mirrors.begin(), mirrors.end(), c, [](const char * v, const Mirror * m) { return v < m->lo; });
        if (it == mirrors.begin() || c >= (*(it - 1))->hi) gabort("ggml_graph_compute: tensor outside the mapped buffers");
        return **(it - 1);
    }
    char * dev(const void * p) {
        Mirror & m = mirror_of(p);
        return m.dev + ((const char *) p - m.lo);
    }
    void * temp(size_t n) { return dev_arena.get(n); }
    // host bytes that must reach the device in stream order: copied into pinned staging first,
    // so the caller's memory may go away before the copy runs
    void * upload_small(const void * src, size_t n) {
        void * h = host_arena.get(n);
        std::memcpy(h, src, n);
        void * d = temp(n);
        LVK_HIP(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, stream));
        return d;
    }
    void drop_repacked(const char * lo, const char * hi) {
        for (size_t i = 0; i < repacked.size();) {
            if (overlaps(lo, hi, repacked[i].lo, repacked[i].hi)) {
                (void) hipFree(repacked[i].nib);
                (void) hipFree(repacked[i].scl);
                repacked[i] = repacked.back();
                repacked.pop_back();
            } else {
                ++i;
            }
        }
    }

    // one mirror covering [lo, hi): existing overlapping mirrors are merged into it (their
    // device bytes copied over, their fully covered valid pages kept)
    Mirror & ensure(char * lo, char * hi) {
        std::vector<Mirror *> old;
        for (Mirror * m : mirrors)
            if (m->lo < hi && lo < m->hi) old.push_back(m);
        if (old.size() == 1 && old[0]->lo <= lo && hi <= old[0]->hi) return *old[0];
        Mirror * n = new Mirror;
        n->lo = lo;
        n->hi = hi;
        for (Mirror * m : old) {
            n->lo = std::min(n->lo, m->lo);
            n->hi = std::max(n->hi, m->hi);
        }
        LVK_HIP(hipMalloc(&n->dev, (size_t) (n->hi - n->lo) + 16));
        n->valid.assign(n->pages(), 0);
        n->ro.assign(n->pages(), -1);
        for (Mirror * m : old) {
            LVK_HIP(hipMemcpyAsync(n->dev + (m->lo - n->lo), m->dev, (size_t) (m->hi - m->lo), hipMemcpyDeviceToDevice, stream));
            const size_t np = m->pages(), d = m->page0() - n->page0();
            for (size_t i = 0; i < np; ++i) {
                // a page only partly inside the old range holds bytes the old mirror never had
                const char * p0 = (const char *) ((m->page0() + i) * PAGE);
                const bool whole = p0 >= m->lo && p0 + PAGE <= m->hi;
                const bool edge_ok = (p0 < m->lo ? n->lo >= m->lo : true) && (p0 + PAGE > m->hi ? n->hi <= m->hi : true);
                n->valid[d + i] = m->valid[i] && (whole || edge_ok);
                n->ro[d + i] = m->ro[i];
            }
        }
        LVK_HIP(hipStreamSynchronize(stream));
        for (Mirror * m : old) {
            (void) hipFree(m->dev);
            mirrors.erase(std::find(mirrors.begin(), mirrors.end(), m));
            delete m;
        }
        mirrors.insert(std::upper_bound(mirrors.begin(), mirrors.end(), n, [](const Mirror * a, const Mirror * b) { return a->lo < b->lo; }), n);
        return *n;
    }

    // pages the host may have written since they were uploaded lose their validity
    std::vector<MapEnt> ro_maps;           // identities of the read-only mappings pages came from
    std::vector<uint8_t> ro_alive;         // this call: is ro_maps[i] still mapped, unchanged
    std::vector<MapEnt> maps_now;          // /proc/self/maps of this call (no soft-dirty)
    void snapshot_maps() {
        maps_now = read_maps();
        ro_alive.assign(ro_maps.size(), 0);
        for (size_t i = 0; i < ro_maps.size(); ++i) {
            const MapEnt * e = map_of(maps_now, ro_maps[i].lo);
            ro_alive[i] = e && e->same(ro_maps[i]);
        }
    }
    void refresh_validity(Mirror & m) {
        DirtyTracker & T = tracker();
        if (!T.enabled) { std::fill(m.valid.begin(), m.valid.end(), 0); return; }
        // host memory HIP can DMA into (registered or pinned): no CPU-side tracking sees those
        // writes.  Decided per mirror from its first and last byte (a mirror that spans several
        // allocations with a pinned one in the middle is not detected: probing the mappings in
        // between can reach driver mappings), and decided again whenever the set of mappings
        // over the range changed.  A range passed to hipHostRegister after its first use keeps
        // its mappings: the caller says so with lvk_ggml_invalidate (lvk_ops.h), which also
        // drops this decision.
        {
            uint64_t sig = 1469598103934665603ull;
            for (const MapEnt & e : maps_now) {
                if (e.hi <= (uintptr_t) m.lo || e.lo >= (uintptr_t) m.hi) continue;
                for (uint64_t v : {(uint64_t) e.lo, (uint64_t) e.hi, e.inode, e.off}) sig = (sig ^ v) * 1099511628211ull;
            }
            if (sig != m.maps_sig) { m.hip_host = -1; m.maps_sig = sig; }
            if (m.hip_host < 0) {
                m.hip_host = 0;
                for (const char * q : {(const char *) m.lo, (const char *) m.hi - 1}) {
                    // only addresses mapped now: part of a mirror's range may have been unmapped
                    // since it was mirrored (a freed scratch buffer), and HIP's pointer query
                    // faults on some unmapped host addresses
                    if (!map_of(maps_now, (uintptr_t) q)) continue;
                    hipPointerAttribute_t a{};
                    if (hipPointerGetAttributes(&a, q) == hipSuccess && a.type == hipMemoryTypeHost) m.hip_host = 1;
                    (void) hipGetLastError();
                }
            }
        }
        if (m.hip_host == 1) { std::fill(m.valid.begin(), m.valid.end(), 0); return; }
        if (T.ok) {
            // soft-dirty bits, read per run of pages.  A page uploaded from a read-only private
            // mapping that is still the same mapping (ro_alive: same range, offset, inode, device
            // and permissions) is kept without a read -- the process cannot have written it, and
            // a 7B / 65B weight mirror is almost all such pages.  A page whose mapping is gone or
            // was replaced (munmap + mmap of another file at the same range) is dropped; a page
            // uploaded while writable that now sits in a read-only mapping (written, then
            // mprotect'ed) has its soft-dirty bit read like any writable page.
            std::vector<uint64_t> e;
            const size_t np = m.pages();
            auto it = maps_now.begin();
            for (size_t i = 0; i < np;) {
                const uintptr_t a = (m.page0() + i) * PAGE;
                while (it != maps_now.end() && it->hi <= a) ++it;
                const bool inside = it != maps_now.end() && a >= it->lo;
                const uintptr_t lim = it == maps_now.end() ? UINTPTR_MAX : inside ? it->hi : it->lo;
                size_t j = i + 1;
                while (j < np && (m.page0() + j) * PAGE < lim) ++j;
                const bool ro = inside && !strchr(it->perms, 'w') && it->perms[3] == 'p';
                bool need_read = !ro;
                if (ro) {
                    for (size_t k = i; k < j; ++k) {
                        if (!m.valid[k]) continue;
                        if (m.ro[k] < 0) need_read = true;                        // uploaded writable
                        else if (!ro_alive[(size_t) m.ro[k]]) m.valid[k] = 0;     // another mapping
                    }
                }
                if (need_read) {
                    if (!T.read(m.page0() + i, j - i, e)) {
                        std::fill(m.valid.begin() + i, m.valid.begin() + j, 0);
                    } else {
                        for (size_t k = 0; k < e.size(); ++k)
                            if ((!ro || m.ro[i + k] < 0) && DirtyTracker::written(e[k])) m.valid[i + k] = 0;
                    }
                }
                i = j;
            }
        } else {
            for (size_t i = 0; i < m.valid.size(); ++i)
                if (m.ro[i] < 0 || !ro_alive[(size_t) m.ro[i]]) m.valid[i] = 0;
        }
        // pages of shared mappings (or of no mapping this call saw) are written behind our back
        auto it = maps_now.begin();
        for (size_t i = 0; i < m.valid.size(); ++i) {
            if (!m.valid[i]) continue;
            const uintptr_t a = (m.page0() + i) * PAGE;
            while (it != maps_now.end() && it->hi <= a) ++it;
            if (it == maps_now.end() || a < it->lo || it->perms[3] == 's') m.valid[i] = 0;
        }
    }
    int32_t ro_id(uintptr_t page) {
        const MapEnt * e = map_of(maps_now, page * PAGE);
        if (!e || strchr(e->perms, 'w')) return -1;
        for (size_t i = 0; i < ro_maps.size(); ++i)
            if (ro_maps[i].same(*e)) return (int32_t) i;
        ro_maps.push_back(*e);
        ro_alive.push_back(1);
        return (int32_t) ro_maps.size() - 1;
    }

    // the invalid pages of m that overlap [a, b) travel host -> device
    void upload(Mirror & m, const char * a, const char * b) {
        const size_t np = m.pages();
        const size_t i0 = (uintptr_t) a / PAGE - m.page0(), i1 = std::min(np, (uintptr_t) (b - 1) / PAGE - m.page0() + 1);
        // the mapping identity of every page uploaded from a read-only mapping, in both caching
        // modes (refresh_validity drops the page when that mapping is no longer the same one)
        const bool track_ro = tracker().enabled;
        for (size_t i = i0; i < i1;) {
            if (m.valid[i]) { ++i; continue; }
            size_t j = i;
            while (j < i1 && !m.valid[j]) ++j;
            const char * x = std::max((const char *) ((m.page0() + i) * PAGE), (const char *) m.lo);
            const char * y = std::min((const char *) ((m.page0() + j) * PAGE), (const char *) m.hi);
            LVK_HIP(hipMemcpyAsync(m.dev + (x - m.lo), x, (size_t) (y - x), hipMemcpyHostToDevice, stream));
            last.h2d += (uint64_t) (y - x);
            drop_repacked(x, y);
            for (size_t k = i; k < j; ++k) {
                m.valid[k] = 1;
                m.ro[k] = track_ro ? ro_id(m.page0() + k) : -1;
            }
            i = j;
        }
    }

    // true when no node of this call has written [p, p + n) so far: the host bytes are current
    bool host_current(const void * p, size_t n) const {
        const char * a = (const char *) p;
        for (const Span & w : written)
            if (overlaps(a, a + n, w.lo, w.hi)) return false;
        return true;
    }
    template <class T> T read_scalar(const ggml_tensor * t, int i) {
        const char * p = (const char *) t->data + (size_t) i * sizeof(T);
        T v;
        if (host_current(p, sizeof(T))) {
            std::memcpy(&v, p, sizeof(T));
            return v;
        }
        LVK_HIP(hipMemcpyAsync(&v, dev(p), sizeof(T), hipMemcpyDeviceToHost, stream));
        LVK_HIP(hipStreamSynchronize(stream));
        return v;
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
    // the octet image of the Q4 matrix at host address w (M x K), repacked once and kept
    // until the host bytes change
    lvk::QMatrix qmatrix(const char * w, int qt, int M, int K) {
        const char * hi = w + (size_t) M * (K / 32) * (qt == lvk::Q4_1 ? 24 : 20);
        for (const Repacked & r : repacked)
            if (r.lo == w && r.qt == qt && r.M == M && r.K == K) {
                lvk::QMatrix q;
                q.qtype = qt; q.M = M; q.K = K; q.nib = r.nib; q.scl = r.scl;
                return q;
            }
        Repacked r{w, hi, qt, M, K};
        LVK_HIP(hipMalloc(&r.nib, lvk::qimage_nib_bytes(M, K)));
        LVK_HIP(hipMalloc(&r.scl, lvk::qimage_scl_bytes(M, K, qt)));
        LVK_HIP(lvk::launch_repack(dev(w), qt, M, K, r.nib, r.scl, stream));
        last.repack += (uint64_t) (hi - w);
        repacked.push_back(r);
        lvk::QMatrix q;
        q.qtype = qt; q.M = M; q.K = K; q.nib = r.nib; q.scl = r.scl;
        return q;
    }
};

// one engine per device, behind one lock (ggml contexts may be used from several threads)
std::mutex & engine_mutex() {
    static std::mutex m;
    return m;
}
std::map<int, GraphEngine *> & all_engines() {
    static std::map<int, GraphEngine *> per_dev;
    return per_dev;
}
GraphEngine & engine() {
    std::map<int, GraphEngine *> & per_dev = all_engines();
    int d = 0;
    LVK_HIP(hipGetDevice(&d));
    auto it = per_dev.find(d);
    if (it != per_dev.end()) return *it->second;
    return *per_dev.emplace(d, new GraphEngine).first->second;
}
GraphStats g_last_stats;
bool g_have_engine = false;

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

void run_mul_mat_q(GraphEngine & R, const ggml_tensor * a, const ggml_tensor * b, ggml_tensor * node) {
    // ggml_compute_forward_mul_mat_q_f32 (ggml.c:6510-6696): every src1 row quantized with
    // the AVX2 quantizer, one vec_dot_q per (row, column) -- the matvec kernels' arithmetic
    const int M = (int) a->ne[1], K = (int) a->ne[0], N = (int) b->ne[1];
    const int qt = a->type == GGML_TYPE_Q4_0 ? lvk::Q4_0 : lvk::Q4_1;
    if (M % 8 || K % 256) gabort("ggml_graph_compute: Q4 mul_mat needs ne01 % 8 == 0 and ne00 % 256 == 0");
    G_ASSERT(a->nb[1] == (size_t) (K / 32) * TYPE_SIZE[a->type]);
    for (int64_t i3 = 0; i3 < a->ne[3]; ++i3)
        for (int64_t i2 = 0; i2 < a->ne[2]; ++i2) {
            const lvk::QMatrix q = R.qmatrix((const char *) a->data + i2 * a->nb[2] + i3 * a->nb[3], qt, M, K);
            // this batch's src1 rows, contiguous
            ggml_tensor bs = *b;
            bs.data = (char *) b->data + i2 * b->nb[2] + i3 * b->nb[3];
            bs.ne[2] = bs.ne[3] = 1;
            float * x = (float *) R.gather(&bs, lvk::GT_F32);
            float * y = (float *) R.temp((size_t) N * M * 4);
            const lvk::StepParams sp{0, N, 0, 0};
            lvk::StepParams * spd = (lvk::StepParams *) R.upload_small(&sp, sizeof sp);
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

void run_node(GraphEngine & R, ggml_tensor * n) {
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
            const float2 * csd = (const float2 *) R.upload_small(cs.data(), cs.size() * sizeof(float2));
            LVK_HIP(lvk::launch_g_rope(R.view(n), R.view(n), csd, n_dims, i2_0, R.stream));
            return;
        }
        case GGML_OP_GET_ROWS:
            G_ASSERT(b->type == GGML_TYPE_I32 && n->type == GGML_TYPE_F32);
            G_ASSERT(a->type == GGML_TYPE_Q4_0 || a->type == GGML_TYPE_Q4_1 || a->type == GGML_TYPE_F16 ||
                     a->type == GGML_TYPE_F32);
            if (b->op == GGML_OP_NONE && R.host_current(b->data, (size_t) b->ne[0] * sizeof(int32_t)))
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

// the ops that only reinterpret their source: they write nothing
bool writes_data(int op) {
    return op != GGML_OP_NONE && op != GGML_OP_RESHAPE && op != GGML_OP_VIEW && op != GGML_OP_PERMUTE &&
           op != GGML_OP_TRANSPOSE;
}

}  // namespace

extern "C" void ggml_graph_compute(struct ggml_context * ctx, struct ggml_cgraph * cgraph) {
    (void) ctx;
    std::lock_guard<std::mutex> lock(engine_mutex());
    try {
        GraphEngine & R = engine();
        R.last = GraphStats{};
        R.used.clear();
        R.written.clear();
        R.dev_arena.reset();
        R.host_arena.reset();
        ++R.calls;
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
        std::vector<Span> sp;
        for (const ggml_tensor * t : ts) sp.push_back({(const char *) t->data, (const char *) t->data + span_bytes(t)});
        std::sort(sp.begin(), sp.end(), [](const Span & x, const Span & y) { return x.lo < y.lo; });
        std::vector<Span> regions;
        for (const Span & r : sp) {
            if (!regions.empty() && r.lo <= regions.back().hi) regions.back().hi = std::max(regions.back().hi, r.hi);
            else regions.push_back(r);
        }
        // mirrors: created or merged.  A later region's ensure() may merge (and delete) the mirror
        // an earlier region got, so the mirrors this call uses are looked up after all merges
        for (const Span & r : regions) R.ensure((char *) r.lo, (char *) r.hi);
        for (const Span & r : regions) {
            Mirror & m = R.mirror_of(r.lo);
            if (m.last_call != R.calls) {
                m.last_call = R.calls;
                R.used.push_back(&m);
            }
        }
        DirtyTracker & T = tracker();
        const auto t_track0 = std::chrono::steady_clock::now();
        if (T.enabled) R.snapshot_maps();
        for (Mirror * m : R.used) R.refresh_validity(*m);
        R.last.track_ns += ns_since(t_track0);
        // the bytes a node reads before any earlier node of this call wrote them (leaves, the
        // caller's inputs, a KV cache) are the only ones that must come from the host
        {
            std::vector<Span> wr;          // written so far (unsorted; graphs are small)
            std::vector<Span> need;
            auto read_of = [&](const ggml_tensor * t) {
                if (!t) return;
                Span s{(const char *) t->data, (const char *) t->data + span_bytes(t)};
                // subtract the written spans from s
                std::vector<Span> parts{s};
                for (const Span & w : wr) {
                    std::vector<Span> next;
                    for (const Span & p : parts) {
                        if (!overlaps(p.lo, p.hi, w.lo, w.hi)) { next.push_back(p); continue; }
                        if (p.lo < w.lo) next.push_back({p.lo, w.lo});
                        if (w.hi < p.hi) next.push_back({w.hi, p.hi});
                    }
                    parts.swap(next);
                    if (parts.empty()) break;
                }
                need.insert(need.end(), parts.begin(), parts.end());
            };
            for (int i = 0; i < cgraph->n_nodes; ++i) {
                const ggml_tensor * n = cgraph->nodes[i];
                read_of(n->src0);
                read_of(n->src1);
                for (int k = 0; k < GGML_MAX_OPT; ++k) read_of(n->opt[k]);
                if (writes_data(n->op)) wr.push_back({(const char *) n->data, (const char *) n->data + span_bytes(n)});
            }
            for (const Span & p : need) R.upload(R.mirror_of(p.lo), p.lo, p.hi);
        }
        // LVK_GGML_SYNC=1: wait for every node and name the one that fails (debugging)
        static const bool sync_each = getenv("LVK_GGML_SYNC") && atoi(getenv("LVK_GGML_SYNC")) != 0;
        for (int i = 0; i < cgraph->n_nodes; ++i) {
            ggml_tensor * n = cgraph->nodes[i];
            run_node(R, n);
            if (writes_data(n->op)) {
                const Span w{(const char *) n->data, (const char *) n->data + span_bytes(n)};
                R.written.push_back(w);
                R.drop_repacked(w.lo, w.hi);
            }
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
        // node results back to the host: the written byte ranges only (merged)
        std::vector<Span> wb = R.written;
        std::sort(wb.begin(), wb.end(), [](const Span & x, const Span & y) { return x.lo < y.lo; });
        std::vector<Span> wm;
        for (const Span & w : wb) {
            if (!wm.empty() && w.lo <= wm.back().hi) wm.back().hi = std::max(wm.back().hi, w.hi);
            else wm.push_back(w);
        }
        for (const Span & w : wm) {
            LVK_HIP(hipMemcpyAsync((void *) w.lo, R.dev(w.lo), (size_t) (w.hi - w.lo), hipMemcpyDeviceToHost, R.stream));
            R.last.d2h += (uint64_t) (w.hi - w.lo);
        }
        LVK_HIP(hipStreamSynchronize(R.stream));
        // mirrors unused for 8 calls are freed (a caller's per-call scratch contexts)
        for (size_t i = 0; i < R.mirrors.size();) {
            Mirror * m = R.mirrors[i];
            if (m->last_call + 8 < R.calls) {
                R.drop_repacked(m->lo, m->hi);
                (void) hipFree(m->dev);
                R.mirrors.erase(R.mirrors.begin() + (long) i);
                delete m;
                continue;
            }
            ++i;
        }
        // the soft-dirty bits are process-wide: every engine's mirrors this call did not use
        // (all those of the other devices' engines) note their host writes before the clear
        if (T.ok) {
            const auto t_fold0 = std::chrono::steady_clock::now();
            for (auto & kv : all_engines()) {
                GraphEngine & E = *kv.second;
                if (&E != &R) E.maps_now = R.maps_now;
                for (Mirror * m : E.mirrors)
                    if (&E != &R || m->last_call != R.calls) E.refresh_validity(*m);
            }
            const auto t_clear0 = std::chrono::steady_clock::now();
            if (!T.clear()) {
                T.ok = false;
                for (auto & kv : all_engines())
                    for (Mirror * m : kv.second->mirrors) std::fill(m->valid.begin(), m->valid.end(), 0);
            }
            R.last.clear_ns = ns_since(t_clear0);
            R.last.track_ns += ns_since(t_fold0);
        }
        uint64_t resident = 0;
        for (Mirror * m : R.mirrors) resident += (uint64_t) (m->hi - m->lo);
        R.last.mirrored = resident;
        g_last_stats = R.last;
        g_have_engine = true;
        cgraph->perf_runs++;
    } catch (const lvk::Error & e) {
        gabort(e.msg.c_str());
    }
}

extern "C" int lvk_ggml_stats(uint64_t * out, int n) {
    std::lock_guard<std::mutex> lock(engine_mutex());
    const DirtyTracker & T = tracker();
    const uint64_t v[8] = {g_last_stats.h2d, g_last_stats.d2h, g_last_stats.repack, g_last_stats.mirrored,
                           (uint64_t) (!T.enabled ? 0 : T.ok ? 2 : 1), (uint64_t) (g_have_engine ? 1 : 0),
                           g_last_stats.track_ns / 1000, g_last_stats.clear_ns / 1000};
    if (!out || n < 0) return -1;
    for (int i = 0; i < n && i < 8; ++i) out[i] = v[i];
    return 8;
}

// the caller rewrote [p, p + n) in a way the tracking cannot see (see above): upload it again
extern "C" int lvk_ggml_invalidate(const void * p, size_t n) {
    std::lock_guard<std::mutex> lock(engine_mutex());
    if (!p) return -1;
    try {
        // every device's engine may mirror the range
        const char * a = (const char *) p;
        const char * b = a + n;
        for (auto & kv : all_engines()) {
            GraphEngine & R = *kv.second;
            for (Mirror * m : R.mirrors) {
                if (!overlaps(a, b, m->lo, m->hi)) continue;
                const size_t i0 = (uintptr_t) std::max(a, (const char *) m->lo) / PAGE - m->page0();
                const size_t i1 = (uintptr_t) (std::min(b, (const char *) m->hi) - 1) / PAGE - m->page0() + 1;
                for (size_t i = i0; i < i1; ++i) m->valid[i] = 0;
                m->hip_host = -1;      // e.g. the range was hipHostRegister'ed since its first use
            }
            R.drop_repacked(a, b);
        }
    } catch (const lvk::Error & e) {
        fprintf(stderr, "lvk_ggml_invalidate: %s\n", e.msg.c_str());
        return -1;
    }
    return 0;
}
