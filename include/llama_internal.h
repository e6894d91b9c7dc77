/* include/llama_internal.h -- the part of the reference's internal header (llama_internal.h)
 * that its tools call across the library boundary: the model's tensors by name, for
 * examples/quantize-stats (quantize-stats.cpp:270).  The tensors are the model FILE's tensors
 * (ggjt type, ne, data mapped read-only from the file, file order as llama_model_load_internal
 * keeps them, reference llama.cpp:886-889), described by the reference's struct ggml_tensor
 * (include/ggml.h); the GPU weight images are separate.  The vector lives as long as the context.
 * Single-part model files only. */
#ifndef LVK_LLAMA_INTERNAL_H
#define LVK_LLAMA_INTERNAL_H

#include "ggml.h"
#include "llama.h"

#include <string>
#include <utility>
#include <vector>

__attribute__((visibility("default"))) std::vector<std::pair<std::string, struct ggml_tensor *>> &
llama_internal_get_tensor_map(struct llama_context * ctx);

#endif
