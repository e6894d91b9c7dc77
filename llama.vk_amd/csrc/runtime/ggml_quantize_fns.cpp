// ggml_quantize_fns.cpp -- the reference's op-level codec table, ggml_internal_get_quantize_fn
// (ggml.h:803-814, ggml.c:6489-6508), with every function running on the GPU kernels of
// this library:
//   dequantize_row_q         -> k_embed's row dequantizer (AVX2 dequantize_row_q4_0/1 values)
//   quantize_row_q           -> the AVX2-exact activation quantizers (k_quantize_q40/q41)
//   quantize_row_q_reference -> k_quantize_ref (the scalar reference quantizers: roundf, 1/d)
//   vec_dot_q                -> the decode matvec on a one-row weight image (ggml_vec_dot_q4_0/1
//                               AVX2 chains) over the pre-quantized y blocks
// The host side only moves bytes between the reference's block layout and the device
// layouts.  Like the reference (asserts), a failure prints the reason and aborts: the
// function-pointer signatures have no error channel.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../../include/ggml.h"
#include "lvk_model.h"

namespace {

struct DevBufs {
    std::vector<void *> ptrs;
    void * get(size_t n) {
        void * p = nullptr;
        LVK_HIP(hipMalloc(&p, n ? n : 16));
        ptrs.push_back(p);
        return p;
    }
    template <class T> T * up(const T * h, size_t n) {
        T * d = (T *) get(n * sizeof(T));
        LVK_HIP(hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice));
        return d;
    }
    ~DevBufs() { for (void * p : ptrs) (void) hipFree(p); }
};

[[noreturn]] void die(const char * fn, const std::string & m) {
    fprintf(stderr, "%s: %s\n", fn, m.c_str());
    abort();
}

constexpr size_t block_bytes(int qt) { return qt == lvk::Q4_0 ? 20 : 24; }

// reference blocks (block_q4_0 {d, qs[16]} / block_q4_1 {d, m, qs[16]}, ggml.c:492-506) <-> ActQ
void blocks_to_act(int qt, const uint8_t * b, int nb, int nb_pad, std::vector<float> & d, std::vector<float> & m,
                   std::vector<uint8_t> & qs) {
    d.assign((size_t) nb_pad, 0.0f);
    m.assign((size_t) nb_pad, 0.0f);
    qs.assign((size_t) nb_pad * 16, qt == lvk::Q4_0 ? 0x88 : 0x00);   // padding blocks: value 0, d = 0
    const size_t bb = block_bytes(qt);
    for (int i = 0; i < nb; ++i) {
        std::memcpy(&d[(size_t) i], b + i * bb, 4);
        if (qt == lvk::Q4_1) std::memcpy(&m[(size_t) i], b + i * bb + 4, 4);
        std::memcpy(&qs[(size_t) i * 16], b + i * bb + bb - 16, 16);
    }
}

lvk::ActQ act_up(DevBufs & dv, const std::vector<float> & d, const std::vector<float> & m, const std::vector<uint8_t> & qs) {
    lvk::ActQ a;
    a.nb = (int) d.size();
    a.d = dv.up(d.data(), d.size());
    a.m = dv.up(m.data(), m.size());
    a.qs = (uint4 *) dv.up(qs.data(), qs.size());
    return a;
}

void act_down(int qt, const lvk::ActQ & a, int nb, void * y) {
    std::vector<float> d((size_t) nb), m((size_t) nb);
    std::vector<uint8_t> qs((size_t) nb * 16);
    LVK_HIP(hipMemcpy(d.data(), a.d, d.size() * 4, hipMemcpyDeviceToHost));
    if (qt == lvk::Q4_1) LVK_HIP(hipMemcpy(m.data(), a.m, m.size() * 4, hipMemcpyDeviceToHost));
    LVK_HIP(hipMemcpy(qs.data(), a.qs, qs.size(), hipMemcpyDeviceToHost));
    uint8_t * out = (uint8_t *) y;
    const size_t bb = block_bytes(qt);
    for (int i = 0; i < nb; ++i) {
        std::memcpy(out + i * bb, &d[(size_t) i], 4);
        if (qt == lvk::Q4_1) std::memcpy(out + i * bb + 4, &m[(size_t) i], 4);
        std::memcpy(out + i * bb + bb - 16, &qs[(size_t) i * 16], 16);
    }
}

template <int QT>
void dequantize_row(const void * x, float * y, int k) {
    try {
        if (k % 32) throw lvk::Error("k must be a multiple of 32");
        if (k == 0) return;
        DevBufs dv;
        const uint8_t * xd = dv.up((const uint8_t *) x, (size_t) k / 32 * block_bytes(QT));
        const int tok = 0;
        const int * td = dv.up(&tok, 1);
        float * yd = (float *) dv.get((size_t) k * 4);
        LVK_HIP(lvk::launch_embed(xd, QT, k, td, 1, yd, nullptr));   // k_embed: one "table" row
        LVK_HIP(hipMemcpy(y, yd, (size_t) k * 4, hipMemcpyDeviceToHost));
    } catch (const lvk::Error & e) { die("dequantize_row_q", e.msg); }
}

template <int QT, bool REF>
void quantize_row(const float * x, void * y, int k) {
    try {
        if (k % 32) throw lvk::Error("k must be a multiple of 32");
        if (k == 0) return;
        DevBufs dv;
        const int nb = k / 32;
        const float * xd = dv.up(x, (size_t) k);
        lvk::ActQ a;
        a.nb = nb;
        a.d = (float *) dv.get((size_t) nb * 4);
        a.m = (float *) dv.get((size_t) nb * 4);
        a.qs = (uint4 *) dv.get((size_t) nb * 16);
        LVK_HIP(REF ? lvk::launch_quantize_ref(xd, 1, k, QT, a, nullptr) : lvk::launch_quantize_act(xd, 1, k, QT, a, nullptr));
        act_down(QT, a, nb, y);
    } catch (const lvk::Error & e) { die(REF ? "quantize_row_q_reference" : "quantize_row_q", e.msg); }
}

// s = x . y over n elements: x is the weight row, y the activation, both in blocks.  The row
// becomes row 0 of a 16-row octet image (rows 1-15 and the blocks past n up to the next
// multiple of 256 elements are zero blocks with d = 0, which leave every chain unchanged)
template <int QT>
void vec_dot(const int n, float * s, const void * x, const void * y) {
    try {
        if (n % 32) throw lvk::Error("n must be a multiple of 32");
        const int nb = n / 32;
        const int K = (n + 255) / 256 * 256, NB = K / 32, M = 16;
        if (K == 0) { *s = 0.0f; return; }
        DevBufs dv;
        const size_t bb = block_bytes(QT);
        std::vector<uint8_t> rows((size_t) M * NB * bb, 0);
        std::memcpy(rows.data(), x, (size_t) nb * bb);
        if (QT == lvk::Q4_0)   // padding blocks of row 0 and the other rows: q = 8 (value 0), d = 0
            for (size_t i = 0; i < (size_t) M * NB; ++i)
                if (i >= (size_t) nb) std::memset(rows.data() + i * bb + 4, 0x88, 16);
        const uint8_t * rd = dv.up(rows.data(), rows.size());
        lvk::QMatrix w;
        w.qtype = QT; w.M = M; w.K = K;
        w.nib = (const uint4 *) dv.get(lvk::qimage_nib_bytes(M, K));
        w.scl = dv.get(lvk::qimage_scl_bytes(M, K, QT));
        LVK_HIP(lvk::launch_repack(rd, QT, M, K, (uint4 *) w.nib, (void *) w.scl, nullptr));
        std::vector<float> d, m;
        std::vector<uint8_t> qs;
        blocks_to_act(QT, (const uint8_t *) y, nb, NB, d, m, qs);
        const lvk::StepParams sp{0, 1, 0, 0};
        lvk::MvLaunch L;
        L.w = w;
        L.xq = act_up(dv, d, m, qs);
        L.sp = dv.up(&sp, 1);
        L.n_tokens = 1;
        float * yd = (float *) dv.get(M * 4);
        L.y = yd;
        LVK_HIP(lvk::launch_matvec(L, lvk::PRO_ACTQ, lvk::EPI_STORE, nullptr));
        LVK_HIP(hipMemcpy(s, yd, 4, hipMemcpyDeviceToHost));
    } catch (const lvk::Error & e) { die("vec_dot_q", e.msg); }
}

}  // namespace

extern "C" quantize_fns_t ggml_internal_get_quantize_fn(size_t i) {
    if (i >= (size_t) GGML_TYPE_COUNT) {   // GGML_ASSERT(i < GGML_TYPE_COUNT) (ggml.c:6506)
        fprintf(stderr, "ggml_internal_get_quantize_fn: type %zu out of range\n", i);
        abort();
    }
    quantize_fns_t f{};
    if (i == GGML_TYPE_Q4_0) {
        f.dequantize_row_q = dequantize_row<lvk::Q4_0>;
        f.quantize_row_q = quantize_row<lvk::Q4_0, false>;
        f.quantize_row_q_reference = quantize_row<lvk::Q4_0, true>;
        f.vec_dot_q = vec_dot<lvk::Q4_0>;
    } else if (i == GGML_TYPE_Q4_1) {
        f.dequantize_row_q = dequantize_row<lvk::Q4_1>;
        f.quantize_row_q = quantize_row<lvk::Q4_1, false>;
        f.quantize_row_q_reference = quantize_row<lvk::Q4_1, true>;
        f.vec_dot_q = vec_dot<lvk::Q4_1>;
    }
    return f;   // the non-quantized types have no entry (zero-initialised, as in ggml.c:6489)
}
