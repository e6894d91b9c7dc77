// quantize.cpp -- llama_model_quantize: f32/f16 ggml model -> Q4_0/Q4_1 ggjt.
//
// Offline host tool kept for API completeness (reference llama.cpp:1461-1577).
// Every tensor whose name ends in "weight" and is 2-D is quantized with the
// file-creation quantizers (ggml.c:509-543 / 799-838: roundf, half away from
// zero; d = amax/7 resp. (max-min)/15); other tensors are copied.  Output is
// ggjt v1 with 32-byte aligned data, hparams ftype = itype.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include <immintrin.h>

#include "../../../include/ggml.h"
#include "../../../include/llama.h"

namespace {

__attribute__((target("f16c"))) float f16_to_f32(uint16_t h) { return _cvtsh_ss(h); }

struct In {
    std::vector<uint8_t> b;
    size_t off = 0;
    uint32_t u32() {
        if (off + 4 > b.size()) throw std::string("unexpected end of file");
        uint32_t v;
        std::memcpy(&v, &b[off], 4);
        off += 4;
        return v;
    }
    // n bytes at the cursor, bounds-checked, then skipped
    const uint8_t * take(size_t n) {
        if (off > b.size() || n > b.size() - off) throw std::string("unexpected end of file");
        const uint8_t * p = b.data() + off;
        off += n;
        return p;
    }
};

void put(std::vector<uint8_t> & o, const void * p, size_t n) {
    const uint8_t * c = (const uint8_t *) p;
    o.insert(o.end(), c, c + n);
}
void put_u32(std::vector<uint8_t> & o, uint32_t v) { put(o, &v, 4); }

// quantize_row_q4_0_reference (ggml.c:509-543).  MAX(a, b) is ((a) > (b) ? (a) : (b)): a NaN
// input makes amax NaN, exactly as in the reference
void quant_q4_0(const float * x, uint8_t * y, int k) {
    for (int i = 0; i < k / 32; ++i) {
        float amax = 0.0f;
        for (int l = 0; l < 32; ++l) {
            const float a = std::fabs(x[i * 32 + l]);
            amax = amax > a ? amax : a;
        }
        const float d = amax / 7.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        uint8_t * blk = y + (size_t) i * 20;
        std::memcpy(blk, &d, 4);
        for (int l = 0; l < 32; l += 2) {
            const float v0 = x[i * 32 + l] * id, v1 = x[i * 32 + l + 1] * id;
            const uint8_t a = (uint8_t) ((int8_t) roundf(v0) + 8), b = (uint8_t) ((int8_t) roundf(v1) + 8);
            blk[4 + l / 2] = (uint8_t) (a | (b << 4));
        }
    }
}

// quantize_row_q4_1_reference (ggml.c:799-838)
void quant_q4_1(const float * x, uint8_t * y, int k) {
    for (int i = 0; i < k / 32; ++i) {
        float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
        for (int l = 0; l < 32; ++l) {
            const float v = x[i * 32 + l];
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
        const float d = (mx - mn) / 15.0f;
        const float id = d != 0.0f ? 1.0f / d : 0.0f;
        uint8_t * blk = y + (size_t) i * 24;
        std::memcpy(blk, &d, 4);
        std::memcpy(blk + 4, &mn, 4);
        for (int l = 0; l < 32; l += 2) {
            const float v0 = (x[i * 32 + l] - mn) * id, v1 = (x[i * 32 + l + 1] - mn) * id;
            const uint8_t a = (uint8_t) roundf(v0), b = (uint8_t) roundf(v1);
            blk[8 + l / 2] = (uint8_t) (a | (b << 4));
        }
    }
}

// ggml_quantize_q4_0/_q4_1 (ggml.c:10520-10564): rows of k, then the nibble histogram
size_t quantize_hist(const float * src, void * dst, int n, int k, int64_t * hist, bool q41) {
    if (k <= 0 || k % 32 != 0 || n < 0) {
        fprintf(stderr, "ggml_quantize_q4_%d: k must be a positive multiple of 32\n", q41 ? 1 : 0);
        abort();
    }
    const size_t bs = q41 ? 24 : 20, off = q41 ? 8 : 4;
    const int nb = k / 32;
    for (int j = 0; j < n; j += k) {
        uint8_t * y = (uint8_t *) dst + (size_t) (j / 32) * bs;
        if (q41) quant_q4_1(src + j, y, k);
        else quant_q4_0(src + j, y, k);
        for (int i = 0; i < nb; ++i)
            for (int l = 0; l < 16; ++l) {
                const uint8_t q = y[(size_t) i * bs + off + l];
                hist[q & 0xF]++;
                hist[q >> 4]++;
            }
    }
    return (size_t) (n / 32) * bs;
}

size_t row_bytes(uint32_t t, size_t k) {
    switch (t) {
        case 0: return 4 * k;
        case 1: return 2 * k;
        case 2: return k / 32 * 20;
        case 3: return k / 32 * 24;
    }
    throw std::string("unrecognized ftype");
}

void quantize_file(const char * fin, const char * fout, int itype) {
    if (itype != 2 && itype != 3) throw std::string("invalid quantization type ") + std::to_string(itype);
    In in;
    {
        FILE * f = fopen(fin, "rb");
        if (!f) throw std::string("failed to open ") + fin;
        fseek(f, 0, SEEK_END);
        in.b.resize((size_t) ftell(f));
        fseek(f, 0, SEEK_SET);
        if (fread(in.b.data(), 1, in.b.size(), f) != in.b.size()) { fclose(f); throw std::string("read error"); }
        fclose(f);
    }
    const uint32_t magic = in.u32();
    uint32_t version = 0;
    if (magic != LLAMA_FILE_MAGIC_UNVERSIONED) version = in.u32();
    const bool has_scores = magic != LLAMA_FILE_MAGIC_UNVERSIONED;
    const bool aligned = magic == LLAMA_FILE_MAGIC && version == 1;
    if (!(magic == LLAMA_FILE_MAGIC_UNVERSIONED || (magic == 0x67676d66u && version == 1) || aligned))
        throw std::string("unknown (magic, version) combination");
    uint32_t hp[7];
    for (auto & v : hp) v = in.u32();
    std::vector<uint8_t> out;
    put_u32(out, LLAMA_FILE_MAGIC);
    put_u32(out, 1);
    hp[6] = (uint32_t) itype;
    for (uint32_t v : hp) put_u32(out, v);
    for (uint32_t i = 0; i < hp[0]; ++i) {
        const uint32_t len = in.u32();
        put_u32(out, len);
        put(out, in.take(len), len);
        float score = 0.0f;
        if (has_scores) std::memcpy(&score, in.take(4), 4);
        put(out, &score, 4);
    }
    std::vector<float> f32;
    std::vector<uint8_t> q;
    while (in.off < in.b.size()) {
        const uint32_t nd = in.u32(), nl = in.u32(), ft = in.u32();
        if (nd < 1 || nd > 2) throw std::string("bad tensor dims");
        uint32_t ne[2] = {1, 1};
        for (uint32_t i = 0; i < nd; ++i) ne[i] = in.u32();
        const std::string name((const char *) in.take(nl), nl);
        if (aligned) in.take((32 - (in.off & 31)) & 31);
        const unsigned __int128 sz128 = (unsigned __int128) row_bytes(ft, ne[0]) * ne[1];
        if (sz128 > (unsigned __int128) in.b.size()) throw std::string("tensor '" + name + "' data is not within the file");
        const size_t sz = (size_t) sz128;
        const uint8_t * data = in.take(sz);
        const bool quant = name.size() >= 6 && name.compare(name.size() - 6, 6, "weight") == 0 && nd == 2;
        uint32_t new_t = ft;
        const uint8_t * nd_ptr = data;
        size_t new_sz = sz;
        if (quant) {
            const size_t n = (size_t) ne[0] * ne[1];
            f32.resize(n);
            if (ft == 0) std::memcpy(f32.data(), data, n * 4);
            else if (ft == 1) for (size_t i = 0; i < n; ++i) { uint16_t h; std::memcpy(&h, data + 2 * i, 2); f32[i] = f16_to_f32(h); }
            else throw std::string("type unsupported for integer quantization");
            new_t = (uint32_t) itype;
            new_sz = row_bytes(new_t, ne[0]) * ne[1];
            q.assign(new_sz, 0);
            for (uint32_t r = 0; r < ne[1]; ++r) {
                if (itype == 2) quant_q4_0(&f32[(size_t) r * ne[0]], &q[r * row_bytes(2, ne[0])], (int) ne[0]);
                else quant_q4_1(&f32[(size_t) r * ne[0]], &q[r * row_bytes(3, ne[0])], (int) ne[0]);
            }
            nd_ptr = q.data();
        }
        put_u32(out, nd);
        put_u32(out, nl);
        put_u32(out, new_t);
        for (uint32_t i = 0; i < nd; ++i) put_u32(out, ne[i]);
        put(out, name.data(), nl);
        out.resize(out.size() + ((32 - (out.size() & 31)) & 31), 0);
        put(out, nd_ptr, new_sz);
    }
    FILE * f = fopen(fout, "wb");
    if (!f) throw std::string("failed to open ") + fout;
    fwrite(out.data(), 1, out.size(), f);
    fclose(f);
}

}  // namespace

extern "C" size_t ggml_quantize_q4_0(const float * src, void * dst, int n, int k, int64_t * hist) {
    return quantize_hist(src, dst, n, k, hist, false);
}

extern "C" size_t ggml_quantize_q4_1(const float * src, void * dst, int n, int k, int64_t * hist) {
    return quantize_hist(src, dst, n, k, hist, true);
}

extern "C" int llama_model_quantize(const char * fname_inp, const char * fname_out, int itype) {
    try {
        quantize_file(fname_inp, fname_out, itype);
        return 0;
    } catch (const std::string & e) {
        fprintf(stderr, "%s: failed to quantize: %s\n", __func__, e.c_str());
        return 1;
    }
}
