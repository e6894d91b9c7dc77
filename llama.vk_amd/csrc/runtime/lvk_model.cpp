// lvk_model.cpp -- ggjt loader and one-time upload of the weights into their
// HBM images.
//
// File format (llama.cpp:319-418): magic/version,
// 7 u32 hparams, vocab (len, bytes, f32 score), then tensors until EOF:
// n_dims, name_len, ftype, ne[], name, pad to 32 B (ggjt), data.
// Multi-part files (name, name.1, ...) are re-joined exactly like
// llama_model_loader::load_data_for (llama.cpp:607-648): SPLIT_BY_COLUMNS for
// tok_embeddings / wo / w2, SPLIT_BY_ROWS for the other 2-D tensors.
//
// Upload: each layer matrix is copied into a device staging buffer (fused
// matrices assembled there: wq|wk|wv rows, and w1/w3 interleaved per 32-row
// block) and repacked on the GPU into the octet image the matvec
// streams (lvk_kernels.h QMatrix).  The image has exactly the file's bytes.
#include "lvk_model.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <memory>

namespace lvk {

namespace {

enum FileVer { V_GGML, V_GGMF, V_GGJT };

struct Shard {
    uint32_t type = 0;
    std::vector<uint32_t> ne;
    size_t file = 0;
    size_t off = 0;
    size_t size = 0;
};

size_t type_row_bytes(uint32_t type, size_t k) {
    switch (type) {
        case 0: return 4 * k;
        case 1: return 2 * k;
        case 2: return k / 32 * 20;
        case 3: return k / 32 * 24;
    }
    throw Error("unrecognized ftype " + std::to_string(type));
}

struct MappedFile {
    void * addr = nullptr;
    size_t size = 0;
    explicit MappedFile(const std::string & path) {
        int fd = open(path.c_str(), O_RDONLY);
        if (fd < 0) throw Error("failed to open " + path);
        struct stat st;
        fstat(fd, &st);
        size = (size_t) st.st_size;
        addr = size ? mmap(nullptr, size, PROT_READ, MAP_SHARED, fd, 0) : nullptr;
        close(fd);
        if (size && addr == MAP_FAILED) throw Error("mmap failed for " + path);
        if (size) madvise(addr, size, MADV_SEQUENTIAL);
    }
    ~MappedFile() { if (addr && size) munmap(addr, size); }
    const uint8_t * p() const { return (const uint8_t *) addr; }
};

struct Reader {
    const uint8_t * b;
    size_t n, off = 0;
    uint32_t u32() {
        if (off + 4 > n) throw Error("unexpectedly reached end of file");
        uint32_t v;
        std::memcpy(&v, b + off, 4);
        off += 4;
        return v;
    }
    std::string str(size_t len) {
        if (off + len > n) throw Error("unexpectedly reached end of file");
        std::string s((const char *) b + off, len);
        off += len;
        return s;
    }
    float f32() { uint32_t v = u32(); float f; std::memcpy(&f, &v, 4); return f; }
};

struct FileInfo {
    FileVer ver;
    HParams hp;
    size_t data_begin = 0;
};

FileInfo read_header(Reader & rd, Vocab * vocab) {
    FileInfo fi;
    const uint32_t magic = rd.u32();
    uint32_t version = 0;
    if (magic != 0x67676d6cu) version = rd.u32();   // 'ggml' has no version
    if (magic == 0x67676d6cu) fi.ver = V_GGML;
    else if (magic == 0x67676d66u && version == 1) fi.ver = V_GGMF;
    else if (magic == 0x67676a74u && version == 1) fi.ver = V_GGJT;
    else {
        char buf[128];
        snprintf(buf, sizeof buf, "unknown (magic, version) combination: %08x, %08x; is this really a GGML file?",
                 magic, version);
        throw Error(buf);
    }
    fi.hp.n_vocab = rd.u32(); fi.hp.n_embd = rd.u32(); fi.hp.n_mult = rd.u32(); fi.hp.n_head = rd.u32();
    fi.hp.n_layer = rd.u32(); fi.hp.n_rot = rd.u32(); fi.hp.ftype = rd.u32();
    for (uint32_t i = 0; i < fi.hp.n_vocab; ++i) {
        const uint32_t len = rd.u32();
        std::string w = rd.str(len);
        float score = 0.0f;
        if (fi.ver >= V_GGMF) score = rd.f32();
        if (vocab) {
            vocab->token_to_id[w] = (int) i;
            vocab->id_to_token.push_back({std::move(w), score});
        }
    }
    fi.data_begin = rd.off;
    return fi;
}

void read_tensor_index(Reader & rd, FileVer ver, size_t file_idx, std::map<std::string, std::vector<Shard>> & idx,
                       std::vector<FileTensor> * order = nullptr) {
    while (rd.off < rd.n) {
        Shard sh;
        const uint32_t nd = rd.u32();
        const uint32_t name_len = rd.u32();
        sh.type = rd.u32();
        if (nd < 1 || nd > 2) throw Error("tensor should not be " + std::to_string(nd) + "-dimensional");
        for (uint32_t i = 0; i < nd; ++i) sh.ne.push_back(rd.u32());
        std::string name = rd.str(name_len);
        if (ver >= V_GGJT) rd.off += (32 - (rd.off & 31)) & 31;     // llama.cpp:397-400
        sh.file = file_idx;
        sh.off = rd.off;
        const size_t rows = sh.ne.size() > 1 ? sh.ne[1] : 1;
        // in 128 bits: a corrupt shape must fail the bounds check, not wrap around it
        const unsigned __int128 bytes = (unsigned __int128) type_row_bytes(sh.type, sh.ne[0]) * rows;
        if (rd.off > rd.n || bytes > (unsigned __int128) (rd.n - rd.off))
            throw Error("tensor '" + name + "' data is not within the file bounds");
        sh.size = (size_t) bytes;
        rd.off += sh.size;
        if (order) order->push_back({name, sh.type, sh.ne, sh.off, sh.size});
        idx[name].push_back(sh);
    }
}

struct Tensor {
    uint32_t type = 0;
    uint32_t ne0 = 0, ne1 = 1;
    const uint8_t * host = nullptr;     // contiguous host bytes (mmap or re-joined copy)
    size_t size = 0;
};

}  // namespace

void * Model::alloc(size_t n) {
    void * p = nullptr;
    LVK_HIP(hipMalloc(&p, n ? n : 16));
    bufs.push_back({p, n});
    return p;
}

Model::~Model() {
    for (auto & b : bufs) (void) hipFree(b.p);
}

void load_model(Model & m, const std::string & path, bool vocab_only, hipStream_t s,
                void (*progress)(float, void *), void * progress_ud, int layer_begin, int layer_end) {
    const auto t_start = std::chrono::steady_clock::now();
    std::vector<std::unique_ptr<MappedFile>> files;
    files.emplace_back(new MappedFile(path));
    Reader rd{files[0]->p(), files[0]->size};
    FileInfo fi = read_header(rd, &m.vocab);
    m.hp = fi.hp;
    m.path = path;
    if (vocab_only) return;

    std::map<std::string, std::vector<Shard>> idx;
    read_tensor_index(rd, fi.ver, 0, idx);
    // multi-part: n_parts = n_embd / tok_embeddings.ne[0] (llama.cpp:533-540)
    auto te = idx.find("tok_embeddings.weight");
    if (te == idx.end()) throw Error("missing tok_embeddings.weight");
    if (te->second.at(0).ne.at(0) == 0 || m.hp.n_embd == 0 || m.hp.n_head == 0 || m.hp.n_layer == 0 || m.hp.n_mult == 0)
        throw Error("invalid hyperparameters or tok_embeddings.weight shape");
    const uint32_t n_parts = m.hp.n_embd / te->second.at(0).ne.at(0);
    for (uint32_t i = 1; i < n_parts; ++i) {
        const std::string fname = path + "." + std::to_string(i);
        files.emplace_back(new MappedFile(fname));
        Reader r2{files.back()->p(), files.back()->size};
        FileInfo f2 = read_header(r2, nullptr);
        if (f2.hp.n_vocab != m.hp.n_vocab || f2.hp.n_embd != m.hp.n_embd || f2.hp.n_layer != m.hp.n_layer)
            throw Error("hparams inconsistent between files");
        read_tensor_index(r2, f2.ver, i, idx);
    }
    for (auto & f : files) m.file_bytes += f->size;

    std::vector<std::vector<uint8_t>> joined;   // storage for re-joined multi-part tensors
    auto get = [&](const std::string & name, std::vector<uint32_t> ne) -> Tensor {
        auto it = idx.find(name);
        if (it == idx.end()) throw Error("tensor '" + name + "' is missing from model");
        const auto & sh = it->second;
        for (const auto & x : sh)
            if (x.type != sh[0].type) throw Error("inconsistent tensor shard type in '" + name + "'");
        Tensor t;
        t.type = sh[0].type;
        std::vector<uint32_t> full = sh[0].ne;
        const bool by_cols = sh.size() > 1 && full.size() == 2 &&
                             (name.find("tok_embeddings.") == 0 || name.find(".attention.wo.weight") != std::string::npos ||
                              name.find(".feed_forward.w2.weight") != std::string::npos);
        if (sh.size() > 1 && full.size() == 2) {
            if (by_cols) full[0] *= (uint32_t) sh.size();
            else full[1] *= (uint32_t) sh.size();
        }
        if (full != ne) throw Error("tensor '" + name + "' has wrong shape");
        t.ne0 = ne[0];
        t.ne1 = ne.size() > 1 ? ne[1] : 1;
        t.size = type_row_bytes(t.type, t.ne0) * t.ne1;
        if (sh.size() == 1 || full.size() == 1) {
            t.host = files[sh[0].file]->p() + sh[0].off;
        } else {
            joined.emplace_back(t.size);
            uint8_t * dst = joined.back().data();
            if (!by_cols) {
                size_t o = 0;
                for (const auto & x : sh) { std::memcpy(dst + o, files[x.file]->p() + x.off, x.size); o += x.size; }
            } else {
                const size_t per = sh[0].size / t.ne1;
                size_t o = 0;
                for (size_t row = 0; row < t.ne1; ++row)
                    for (const auto & x : sh) { std::memcpy(dst + o, files[x.file]->p() + x.off + row * per, per); o += per; }
            }
            t.host = dst;
        }
        return t;
    };

    const uint32_t E = m.hp.n_embd, V = m.hp.n_vocab, L = m.hp.n_layer, F = m.hp.n_ff();
    if (E % 256 || F % 256 || E % m.hp.n_head || (E / m.hp.n_head) % 32)
        throw Error("llama.vk_amd: unsupported dimensions (need n_embd, n_ff multiples of 256, head_dim multiple of 32)");

    // size the staging buffer for the largest (fused) matrix
    Tensor t_tok = get("tok_embeddings.weight", {E, V});
    Tensor t_norm = get("norm.weight", {E});
    Tensor t_out = get("output.weight", {E, V});
    if (t_out.type != 2 && t_out.type != 3) throw Error("llama.vk_amd: output.weight must be Q4_0/Q4_1");
    m.qtype = (int) t_out.type;
    const size_t rb_E = type_row_bytes(m.qtype, E), rb_F = type_row_bytes(m.qtype, F);
    size_t stage_n = std::max({t_out.size, 3 * E * rb_E, 2 * (size_t) F * rb_E, (size_t) E * rb_F});
    void * stage = nullptr;
    LVK_HIP(hipMalloc(&stage, stage_n));
    struct StageFree { void * p; ~StageFree() { (void) hipFree(p); } } stage_guard{stage};

    if (layer_end < 0) layer_end = (int) L;
    if (layer_begin < 0 || layer_begin >= layer_end || layer_end > (int) L)
        throw Error("llama.vk_amd: bad layer range [" + std::to_string(layer_begin) + ", " + std::to_string(layer_end) + ")");
    m.layer_begin = layer_begin;
    m.layer_end = layer_end;
    m.has_embed = layer_begin == 0;
    m.has_head = layer_end == (int) L;
    const uint32_t LB = (uint32_t) layer_begin, LN = (uint32_t) (layer_end - layer_begin);
    size_t total = (m.has_embed ? t_tok.size : 0) + (m.has_head ? t_out.size : 0), done = 0;
    total += (size_t) LN * (3 * E * rb_E + E * rb_E + 2 * (size_t) F * rb_E + E * rb_F);
    auto tick = [&](size_t n) {
        done += n;
        if (progress) progress((float) ((double) done / (double) total), progress_ud);
    };

    auto make_matrix = [&](int M, int K) -> QMatrix {
        QMatrix q;
        q.qtype = m.qtype; q.M = M; q.K = K;
        const size_t nib = qimage_nib_bytes(M, K);
        const size_t scl = qimage_scl_bytes(M, K, m.qtype);
        q.nib = (const uint4 *) m.alloc(nib);
        q.scl = m.alloc(scl);
        m.weight_bytes += (size_t) M * (K / 32) * (m.qtype == Q4_0 ? 20 : 24);
        return q;
    };
    // the prompt matmul's f16 A-fragment images (mm_mfma.hip, 2 B per weight: 13.2 GB for
    // 7B, 130 GB for 65B), decided by capacity (the A-image table):
    //   * Q4_1: the f16 image plus the per-block side image (mm_mfma41.hip, 3 B per weight in
    //     all) are what the Q4_1 MFMA prompt path runs on -- 13B 512-token prompt 158 ms with
    //     them, 1234 ms on the VALU kernels without -- built whenever they fit next to the Q4
    //     images with 8 GiB to spare;
    //   * Q4_0: the nibble image runs the same MFMA path only 8-12 % slower (7B 44.3 vs 39.6 ms,
    //     65B 403 vs 372 ms), so the image (3.2x the Q4 bytes) is built only when it takes at
    //     most a quarter of the device's memory: 7B / 13B-shaped models and every stage of a
    //     65B split over 8 GPUs, not the whole 65B on one GPU (130 GB of 288 GB);
    //     LVK_PROMPT_A16=1 builds it whenever it fits, =0 never
    bool a16 = prompt_a16_env();
    if (a16) {
        const size_t EE = (size_t) E * E, EF = (size_t) E * F;
        const size_t per_w = m.qtype == Q4_0 ? 2 : 3;
        const size_t need = per_w * ((4 * EE + 3 * EF) * (size_t) LN + (m.has_head ? (size_t) V * E : 0));
        size_t free_b = 0, total_b = 0;
        LVK_HIP(hipMemGetInfo(&free_b, &total_b));
        const size_t q4 = (size_t) ((double) need / per_w * (m.qtype == Q4_0 ? 20.0 : 24.0) / 32.0);
        a16 = free_b > need + q4 + ((size_t) 8 << 30);
        if (a16 && m.qtype == Q4_0 && !prompt_a16_forced()) a16 = need <= total_b / 4;
    }
    auto repack = [&](QMatrix & q, int interleave4 = 0) {
        LVK_HIP(launch_repack(stage, q.qtype, q.M, q.K, (uint4 *) q.nib, (void *) q.scl, s, interleave4));
        if (a16 && q.qtype == Q4_0 && mm_mfma_supported(q)) {
            q.a16 = m.alloc(mm_a16_bytes(q.M, q.K));
            m.prompt_image_bytes += mm_a16_bytes(q.M, q.K);
            LVK_HIP(launch_build_a16(q, (void *) q.a16, s));
        } else if (a16 && q.qtype == Q4_1 && q.M % 128 == 0 && q.K % 256 == 0) {
            q.a16 = m.alloc(mm_a16_bytes(q.M, q.K));
            q.side = m.alloc(mm41_side_bytes(q.M, q.K));
            m.prompt_image_bytes += mm_a16_bytes(q.M, q.K) + mm41_side_bytes(q.M, q.K);
            LVK_HIP(launch_build_mm41(q, (void *) q.a16, (void *) q.side, s));
        }
        LVK_HIP(hipStreamSynchronize(s));
    };
    auto check_q = [&](const Tensor & t, const std::string & name) {
        if ((int) t.type != m.qtype) throw Error("llama.vk_amd: tensor '" + name + "' is not in the model's Q4 format");
    };

    // embeddings stay in file layout (gathered by row, ggml.c:6868-6895)
    m.emb_type = (int) t_tok.type;
    if (m.has_embed) {
        m.tok_emb = m.alloc(t_tok.size);
        LVK_HIP(hipMemcpy(m.tok_emb, t_tok.host, t_tok.size, hipMemcpyHostToDevice));
        tick(t_tok.size);
    }
    if (t_norm.type != 0) throw Error("norm.weight must be f32");
    if (m.has_head) {
        m.norm = (float *) m.alloc(4u * E);
        LVK_HIP(hipMemcpy(m.norm, t_norm.host, 4u * E, hipMemcpyHostToDevice));
        // lm_head
        LVK_HIP(hipMemcpy(stage, t_out.host, t_out.size, hipMemcpyHostToDevice));
        m.output = make_matrix((int) V, (int) E);
        repack(m.output);
        tick(t_out.size);
    }

    m.layers.resize(LN);
    for (uint32_t il = LB; il < LB + LN; ++il) {
        Layer & ly = m.layers[il - LB];
        const std::string p = "layers." + std::to_string(il) + ".";
        Tensor an = get(p + "attention_norm.weight", {E});
        Tensor fn = get(p + "ffn_norm.weight", {E});
        Tensor wq = get(p + "attention.wq.weight", {E, E});
        Tensor wk = get(p + "attention.wk.weight", {E, E});
        Tensor wv = get(p + "attention.wv.weight", {E, E});
        Tensor wo = get(p + "attention.wo.weight", {E, E});
        Tensor w1 = get(p + "feed_forward.w1.weight", {E, F});
        Tensor w2 = get(p + "feed_forward.w2.weight", {F, E});
        Tensor w3 = get(p + "feed_forward.w3.weight", {E, F});
        for (auto * t : {&wq, &wk, &wv, &wo, &w1, &w2, &w3}) check_q(*t, p + "*");
        if (an.type != 0 || fn.type != 0) throw Error("norm weights must be f32");
        ly.attn_norm = (float *) m.alloc(4u * E);
        ly.ffn_norm = (float *) m.alloc(4u * E);
        LVK_HIP(hipMemcpy(ly.attn_norm, an.host, 4u * E, hipMemcpyHostToDevice));
        LVK_HIP(hipMemcpy(ly.ffn_norm, fn.host, 4u * E, hipMemcpyHostToDevice));
        // fused QKV: rows wq | wk | wv
        uint8_t * st = (uint8_t *) stage;
        LVK_HIP(hipMemcpy(st, wq.host, wq.size, hipMemcpyHostToDevice));
        LVK_HIP(hipMemcpy(st + wq.size, wk.host, wk.size, hipMemcpyHostToDevice));
        LVK_HIP(hipMemcpy(st + 2 * wq.size, wv.host, wv.size, hipMemcpyHostToDevice));
        ly.wqkv = make_matrix(3 * (int) E, (int) E);
        repack(ly.wqkv);
        tick(3 * wq.size);
        LVK_HIP(hipMemcpy(stage, wo.host, wo.size, hipMemcpyHostToDevice));
        ly.wo = make_matrix((int) E, (int) E);
        repack(ly.wo);
        tick(wo.size);
        // fused W1|W3, interleaved per 4 output rows by the repack (a row group
        // of 8 holds w1 and w3 rows of the same 4 outputs: SwiGLU stays in a wave)
        LVK_HIP(hipMemcpy(st, w1.host, w1.size, hipMemcpyHostToDevice));
        LVK_HIP(hipMemcpy(st + w1.size, w3.host, w3.size, hipMemcpyHostToDevice));
        ly.w13 = make_matrix(2 * (int) F, (int) E);
        repack(ly.w13, 1);
        tick(2 * w1.size);
        LVK_HIP(hipMemcpy(stage, w2.host, w2.size, hipMemcpyHostToDevice));
        ly.w2 = make_matrix((int) E, (int) F);
        repack(ly.w2);
        tick(w2.size);
    }
    m.load_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_start).count();
}

// the tensor directory of a single-part model file in file order (llama_internal_get_tensor_map)
std::vector<FileTensor> file_tensor_list(const std::string & path, size_t & file_size) {
    MappedFile f(path);
    Reader rd{f.p(), f.size};
    FileInfo fi = read_header(rd, nullptr);
    std::map<std::string, std::vector<Shard>> idx;
    std::vector<FileTensor> order;
    read_tensor_index(rd, fi.ver, 0, idx, &order);
    auto te = idx.find("tok_embeddings.weight");
    if (te != idx.end() && fi.hp.n_embd != te->second.at(0).ne.at(0))
        throw Error("the tensor map of a multi-part model file is not supported");
    file_size = f.size;
    return order;
}

}  // namespace lvk
