/* oracle/lvk_oracle.h -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * A scalar CPU restatement of the reference AVX2 ggml.c arithmetic for the
 * quantized LLaMA forward pass.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (llama.vk_amd/) never does.
 *
 * Pinning: tests/test_oracle_golden.py checks the functions below bit-for-bit
 * against the reference build (oracle/_ref/libref.so) and the committed golden
 * vectors in tests/golden/.
 */
#ifndef LVK_ORACLE_H
#define LVK_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ggml.c:182-183 (F16C _cvtss_sh(x,0) = IEEE RNE) and exact widening */
uint16_t orc_fp32_to_fp16(float x);
float    orc_fp16_to_fp32(uint16_t h);

/* ggml.c:2905-2927: 64 Ki-entry fp16 tables built with glibc expf */
void            orc_init_tables(void);
const uint16_t* orc_table_exp_f16(void);
const uint16_t* orc_table_silu_f16(void);

/* activation quantizers, AVX2 semantics (ggml.c:621-685, 847-920) */
void orc_quantize_row_q4_0(const float* x, void* y, int k);
void orc_quantize_row_q4_1(const float* x, void* y, int k);
/* file-creation quantizers (ggml.c:509-543, 799-838) */
void orc_quantize_row_q4_0_reference(const float* x, void* y, int k);
void orc_quantize_row_q4_1_reference(const float* x, void* y, int k);
/* dequantizers (ggml.c:962-1000, 1080-1115) */
void orc_dequantize_row_q4_0(const void* x, float* y, int k);
void orc_dequantize_row_q4_1(const void* x, float* y, int k);

/* block dots, AVX2 accumulation order (ggml.c:1950-2026, 2188-2258) */
float orc_vec_dot_q4_0(int n, const void* x, const void* y);
float orc_vec_dot_q4_1(int n, const void* x, const void* y);
/* NOT a reference function: the accumulation order of llama.vk_amd's MFMA
 * prompt matmul (mm_mfma.hip) -- exact per-block integer dot I_b, then
 * acc = fmaf(dx*dy, (float) I_b, acc) in block order -- so tests can pin that
 * kernel bit-for-bit (its integer dots included) */
float orc_vec_dot_q4_0_blockorder(int n, const void* x, const void* y);
/* f16 dot (ggml.c:1781-1815, AVX F16 macros 1318-1416) */
float orc_vec_dot_f16(int n, const uint16_t* x, const uint16_t* y);

/* row ops */
void orc_rms_norm(const float* x, int K, int N, float* y);             /* ggml.c:6024-6080 */
void orc_rope(const float* x, int head_dim, int n_head, int N, int n_past, float* y); /* 7156-7227 */
void orc_silu(const float* x, int n, float* y);                         /* 2495-2503 */
void orc_softmax_row(float* p, int n);                                  /* 7062-7130 */
/* one layer's attention block on an f16 KV cache (llama.cpp:1010-1061) */
void orc_attention(const uint16_t* kc, const uint16_t* vc, const float* q,
                   int n_embd, int n_head, int n_ctx, int n_past, int N, float* out);

/* whole model (llama.cpp:927-1197).  ggjt v1 files, Q4_0/Q4_1 weights. */
typedef struct orc_model orc_model;
orc_model* orc_model_load(const char* path, int n_ctx);
void       orc_model_free(orc_model* m);
int        orc_n_vocab(const orc_model* m);
int        orc_n_embd(const orc_model* m);
/* evaluates tokens[0..n) at n_past; logits_out gets n_vocab floats for the
 * last token, or n*n_vocab when logits_all != 0.  Returns 0 on success. */
int        orc_eval(orc_model* m, const int* tokens, int n, int n_past, int logits_all, float* logits_out);
/* raw f16 KV cache of layer il: K [n_ctx][n_embd], V [n_embd][n_ctx] */
const uint16_t* orc_kv_k(const orc_model* m, int il);
const uint16_t* orc_kv_v(const orc_model* m, int il);
void       orc_set_threads(int n);

#ifdef __cplusplus
}
#endif
#endif
