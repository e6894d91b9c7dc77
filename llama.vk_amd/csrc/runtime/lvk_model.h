// lvk_model.h -- host-side model/context structures of the llama.vk_amd runtime.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <random>
#include <string>
#include <vector>

#include "../kernels/lvk_kernels.h"

#define LVK_HIP(call)                                                                              \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) throw lvk::Error(std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

namespace lvk {

struct Error {
    std::string msg;
    explicit Error(std::string m) : msg(std::move(m)) {}
};

// llama_hparams (llama_internal.h / llama.cpp:751-780)
struct HParams {
    uint32_t n_vocab = 32000, n_ctx = 512, n_embd = 4096, n_mult = 256, n_head = 32, n_layer = 32,
             n_rot = 64, ftype = 2;
    uint32_t n_ff() const { return ((2 * (4 * n_embd) / 3 + n_mult - 1) / n_mult) * n_mult; }  // llama.cpp:771
};

struct Vocab {
    struct Tok { std::string text; float score; };
    std::vector<Tok> id_to_token;
    std::map<std::string, int> token_to_id;
};

// one device allocation owned by the model
struct DevBuf {
    void * p = nullptr;
    size_t n = 0;
};

struct Layer {
    float * attn_norm = nullptr;   // [E] f32
    float * ffn_norm = nullptr;    // [E] f32
    QMatrix wqkv;                  // fused [3E][E]: wq | wk | wv rows
    QMatrix wo;                    // [E][E]
    QMatrix w13;                   // fused [2F][E]: per 32-row block b: w1 rows, then w3 rows
    QMatrix w2;                    // [E][F]
};

struct Model {
    HParams hp;
    Vocab vocab;
    int qtype = Q4_0;              // weight format of the layer matrices
    int emb_type = Q4_0;           // tok_embeddings storage type (ggjt ftype id)
    void * tok_emb = nullptr;      // device, file layout
    float * norm = nullptr;        // [E]
    QMatrix output;                // [V][E]
    std::vector<Layer> layers;     // layers [layer_begin, layer_end) of the file
    int layer_begin = 0, layer_end = 0;
    bool has_embed = true;         // first pipeline stage: token embeddings resident
    bool has_head = true;          // last stage: final norm + lm_head resident
    std::vector<DevBuf> bufs;      // owned device memory
    size_t weight_bytes = 0;       // bytes of weights resident in HBM (quad-sliced images)
    size_t prompt_image_bytes = 0; // the prompt matmul's f16 A-fragment (+ Q4_1 side) images
    size_t file_bytes = 0;
    std::string path;              // the model file (llama_internal_get_tensor_map re-maps it)
    double load_ms = 0;

    void * alloc(size_t n);
    ~Model();
};

// one tensor of a model file: ggjt type id, ne (ne[0] = row length), data offset and bytes
struct FileTensor {
    std::string name;
    uint32_t type = 0;
    std::vector<uint32_t> ne;
    size_t off = 0, size = 0;
};
std::vector<FileTensor> file_tensor_list(const std::string & path, size_t & file_size);

// Load a ggjt v1 (or ggmf/ggml vocab-only) file.  vocab_only stops after the
// vocabulary.  layer_end < 0 means all layers; a partial range [layer_begin,
// layer_end) is one pipeline stage: the embeddings are loaded
// only when layer_begin == 0, the final norm + lm_head only when layer_end ==
// n_layer.  Throws lvk::Error.
void load_model(Model & m, const std::string & path, bool vocab_only, hipStream_t s,
                void (*progress)(float, void *), void * progress_ud, int layer_begin = 0, int layer_end = -1);

}  // namespace lvk
