// lvk-gen-model: seeded synthetic LLaMA model writer (ggjt v1, Q4_0 / Q4_1).
//
// There are no real checkpoints anywhere in this environment, so every parity
// and performance input is a synthetic ggjt v1 file with the tensor names,
// shapes, order and 32-byte data alignment the reference loader expects
// (llama.cpp:319-418, 859-881).
//
// Content is a pure function of (seed, tensor index, element index) through
// splitmix64, so any row can be regenerated independently and generation is
// embarrassingly parallel (a 7B file is ~4.2 GB).
//   weights : block scale d = (0.5 + U) * s, s = 1/sqrt(K)/4.6
//             (tok_embeddings use s = 0.02/4.6), qs = uniform random bytes,
//             Q4_1 blocks add m = -8*d
//   norms   : 1 + 0.1 * N(0,1)   (Irwin-Hall approximation of N(0,1))
//   vocab   : copied from a ggjt vocab section file, or synthetic tokens.
//
// usage: lvk-gen-model OUT --n-embd 4096 --n-head 32 --n-layer 32
//                      [--n-mult 256] [--n-vocab 32000] [--ftype 2|3]
//                      [--seed 1] [--vocab tests/golden/vocab32000.bin]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// uniform [0,1) from the top 24 bits
float unit(uint64_t h) { return (float) (h >> 40) * (1.0f / 16777216.0f); }

struct Gen {
    uint64_t seed;
    uint64_t key(uint32_t tensor, uint64_t idx) const {
        return splitmix64(seed * 0x100000001B3ull ^ ((uint64_t) tensor << 44) ^ idx);
    }
};

void put_u32(std::vector<uint8_t> & b, uint32_t v) {
    uint8_t t[4]; std::memcpy(t, &v, 4); b.insert(b.end(), t, t + 4);
}

// fill `out` with `nblocks` quantized blocks of a tensor; parallel over blocks
void fill_q4(uint8_t * out, uint64_t nblocks, int ftype, float s, const Gen & g, uint32_t ti) {
    const size_t bs = ftype == 2 ? 20 : 24;
    unsigned nt = std::max(1u, std::thread::hardware_concurrency());
    if (nt > 64) nt = 64;
    std::vector<std::thread> th;
    for (unsigned w = 0; w < nt; ++w) {
        th.emplace_back([=, &g] {
            const uint64_t b0 = nblocks * w / nt, b1 = nblocks * (w + 1) / nt;
            for (uint64_t b = b0; b < b1; ++b) {
                uint8_t * p = out + b * bs;
                const uint64_t h0 = g.key(ti, b * 4);
                const float d = (0.5f + unit(h0)) * s;
                std::memcpy(p, &d, 4);
                size_t o = 4;
                if (ftype == 3) { const float m = -8.0f * d; std::memcpy(p + 4, &m, 4); o = 8; }
                const uint64_t h1 = g.key(ti, b * 4 + 1), h2 = g.key(ti, b * 4 + 2);
                std::memcpy(p + o, &h1, 8);
                std::memcpy(p + o + 8, &h2, 8);
            }
        });
    }
    for (auto & t : th) t.join();
}

}  // namespace

int main(int argc, char ** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s OUT [--n-embd N] [--n-head N] [--n-layer N] [--n-mult N] "
                             "[--n-vocab N] [--ftype 2|3] [--seed S] [--vocab FILE]\n", argv[0]);
        return 2;
    }
    std::string out = argv[1], vocab_path;
    uint32_t n_embd = 4096, n_head = 32, n_layer = 32, n_mult = 256, n_vocab = 32000, ftype = 2;
    uint64_t seed = 1;
    for (int i = 2; i + 1 < argc; i += 2) {
        std::string k = argv[i];
        const char * v = argv[i + 1];
        if (k == "--n-embd") n_embd = (uint32_t) atoi(v);
        else if (k == "--n-head") n_head = (uint32_t) atoi(v);
        else if (k == "--n-layer") n_layer = (uint32_t) atoi(v);
        else if (k == "--n-mult") n_mult = (uint32_t) atoi(v);
        else if (k == "--n-vocab") n_vocab = (uint32_t) atoi(v);
        else if (k == "--ftype") ftype = (uint32_t) atoi(v);
        else if (k == "--seed") seed = (uint64_t) strtoull(v, nullptr, 10);
        else if (k == "--vocab") vocab_path = v;
        else { std::fprintf(stderr, "unknown option %s\n", k.c_str()); return 2; }
    }
    if ((ftype != 2 && ftype != 3) || n_embd % 32 || n_head == 0 || n_embd % n_head) {
        std::fprintf(stderr, "bad hparams\n");
        return 2;
    }
    const uint32_t n_ff = ((2 * (4 * n_embd) / 3 + n_mult - 1) / n_mult) * n_mult;   // llama.cpp:771
    const uint32_t n_rot = n_embd / n_head;
    Gen g{seed};

    std::FILE * f = std::fopen(out.c_str(), "wb");
    if (!f) { std::perror("open"); return 1; }
    std::vector<uint8_t> hdr;
    put_u32(hdr, 0x67676a74u);   // 'ggjt'
    put_u32(hdr, 1);
    for (uint32_t v : {n_vocab, n_embd, n_mult, n_head, n_layer, n_rot, ftype}) put_u32(hdr, v);
    // vocab section
    if (!vocab_path.empty()) {
        std::FILE * vf = std::fopen(vocab_path.c_str(), "rb");
        if (!vf) { std::perror("vocab"); return 1; }
        std::vector<uint8_t> vb;
        uint8_t buf[65536];
        size_t r;
        while ((r = std::fread(buf, 1, sizeof buf, vf)) > 0) vb.insert(vb.end(), buf, buf + r);
        std::fclose(vf);
        // accept either a raw vocab section or a whole ggjt vocab-only file
        size_t off = 0;
        uint32_t m0 = 0;
        std::memcpy(&m0, vb.data(), 4);
        if (m0 == 0x67676a74u) off = 36;
        // copy exactly n_vocab entries
        size_t p = off;
        for (uint32_t i = 0; i < n_vocab; ++i) {
            if (p + 4 > vb.size()) { std::fprintf(stderr, "vocab file too short\n"); return 1; }
            uint32_t len; std::memcpy(&len, vb.data() + p, 4);
            p += 4 + len + 4;
        }
        hdr.insert(hdr.end(), vb.begin() + (long) off, vb.begin() + (long) p);
    } else {
        for (uint32_t i = 0; i < n_vocab; ++i) {
            char tok[32];
            const int n = std::snprintf(tok, sizeof tok, "<t%u>", i);
            put_u32(hdr, (uint32_t) n);
            hdr.insert(hdr.end(), tok, tok + n);
            const float score = -(float) i;
            uint8_t sb[4]; std::memcpy(sb, &score, 4); hdr.insert(hdr.end(), sb, sb + 4);
        }
    }
    std::fwrite(hdr.data(), 1, hdr.size(), f);
    size_t pos = hdr.size();

    uint32_t ti = 0;
    std::vector<uint8_t> data;
    auto tensor = [&](const std::string & name, uint32_t ne0, uint32_t ne1, bool is2d, float s) {
        std::vector<uint8_t> th;
        const uint32_t ft = is2d ? ftype : 0;
        put_u32(th, is2d ? 2 : 1);
        put_u32(th, (uint32_t) name.size());
        put_u32(th, ft);
        put_u32(th, ne0);
        if (is2d) put_u32(th, ne1);
        th.insert(th.end(), name.begin(), name.end());
        const size_t p2 = pos + th.size();
        th.resize(th.size() + ((32 - (p2 & 31)) & 31), 0);   // llama.cpp:397-400
        std::fwrite(th.data(), 1, th.size(), f);
        pos += th.size();
        if (is2d) {
            const uint64_t nb = (uint64_t) ne0 / 32 * ne1;
            data.resize(nb * (ftype == 2 ? 20 : 24));
            fill_q4(data.data(), nb, (int) ftype, s, g, ti);
        } else {
            data.resize(4u * (size_t) ne0);
            float * w = (float *) data.data();
            for (uint32_t i = 0; i < ne0; ++i) {
                float z = 0.0f;
                for (int k = 0; k < 4; ++k) z += unit(g.key(ti, 4ull * i + k));
                w[i] = 1.0f + 0.1f * (z - 2.0f) * 1.7320508f;
            }
        }
        std::fwrite(data.data(), 1, data.size(), f);
        pos += data.size();
        ++ti;
    };
    const float sK = 1.0f / std::sqrt((float) n_embd) / 4.6f;
    const float sF = 1.0f / std::sqrt((float) n_ff) / 4.6f;
    tensor("tok_embeddings.weight", n_embd, n_vocab, true, 0.02f / 4.6f);
    tensor("norm.weight", n_embd, 1, false, 0);
    tensor("output.weight", n_embd, n_vocab, true, sK);
    for (uint32_t il = 0; il < n_layer; ++il) {
        const std::string p = "layers." + std::to_string(il) + ".";
        tensor(p + "attention_norm.weight", n_embd, 1, false, 0);
        tensor(p + "attention.wq.weight", n_embd, n_embd, true, sK);
        tensor(p + "attention.wk.weight", n_embd, n_embd, true, sK);
        tensor(p + "attention.wv.weight", n_embd, n_embd, true, sK);
        tensor(p + "attention.wo.weight", n_embd, n_embd, true, sK);
        tensor(p + "ffn_norm.weight", n_embd, 1, false, 0);
        tensor(p + "feed_forward.w1.weight", n_embd, n_ff, true, sK);
        tensor(p + "feed_forward.w2.weight", n_ff, n_embd, true, sF);
        tensor(p + "feed_forward.w3.weight", n_embd, n_ff, true, sK);
    }
    std::fclose(f);
    std::fprintf(stderr, "lvk-gen-model: wrote %s (%zu bytes, n_embd %u n_head %u n_layer %u n_ff %u ftype %u)\n",
                 out.c_str(), pos, n_embd, n_head, n_layer, n_ff, ftype);
    return 0;
}
