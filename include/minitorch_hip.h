/*
 * minitorch_hip.h -- C ABI of libminitorch_hip.so (MI355X / gfx950).
 *
 * Drop-in boundary for the reference's ctypes-loaded CUDA libraries
 * (reference minitorch/cuda_kernel_ops.py:25-29 loads combine.so, softmax_kernel.so,
 * layernorm_kernel.so, flashattention_kernel.so). Two layers:
 *
 *  1. Reference-compatible host-pointer entry points: same names, argument order
 *     and meaning as the reference's extern "C" launchers. Each copies the host
 *     arrays to the device, runs, synchronises and copies the outputs back, like
 *     the reference. Unlike the reference they never exit() the process: errors are
 *     printed to stderr and kept in mt_last_error().
 *
 *  2. Device-pointer entry points (prefix mt_): stream-ordered on a caller-supplied
 *     hipStream_t (passed as void*), int64 sizes and element strides, dtype
 *     selectable (MT_F32 / MT_BF16), return 0 on success or a nonzero status with
 *     the message in mt_last_error(). No allocation, no synchronisation inside
 *     (graph-capturable); scratch is caller-provided.
 *
 * Strides are in ELEMENTS for the (batch, head, seq) axes of a [B, H, N, d] tensor;
 * the head dimension d must be unit-stride. A NULL stride pointer means contiguous
 * [B, H, N, d].
 */
#ifndef MINITORCH_HIP_H
#define MINITORCH_HIP_H

#include <stdint.h>
#include <stdbool.h>

#ifdef __cplusplus
extern "C" {
#endif

/* MT_BF16_F32OUT (forward only): bf16 Q/K/V with an fp32 O (16-B aligned rows, strides
 * multiples of 4), the bf16 path without the final rounding of O to bf16. */
enum { MT_F32 = 0, MT_BF16 = 1, MT_BF16_F32OUT = 2 };

/* ---- status ------------------------------------------------------------- */
const char* mt_last_error(void);
int mt_abi_version(void);
/* Kernel selection for A/B timing. 0 (default): the bf16 MFMA kernels specialised for
 * d in {64, 128} where the layout allows, else the generic kernels; 1: the generic tiled
 * kernels only; other ids: alternative bf16 schedules, each computing the same attention
 * (the list and what each id selects: csrc/capi_flash.hip, enum kPol*). Returns 0, or 1
 * for an id the library does not know (the policy is then unchanged). Process-wide,
 * read atomically at each launch. */
int mt_flash_set_kernel_policy(int policy);
int mt_flash_get_kernel_policy(void);
/* Device scratch the library holds between calls (stream-ordered buffers of the zero-padded
 * head-dim copies and the column-reduction partials, one per (pool, device, stream)): its
 * bytes, and a release that frees every buffer no captured hipGraph was handed (after a
 * synchronize of the buffer's stream). Buffers are re-allocated on the next call that needs
 * them. (The reference allocates and frees inside each launcher,
 * src/flashattention_kernel.cu:319-324; here the padded copies are chunked to at most
 * 512 MiB per call.) */
int64_t mt_scratch_bytes(void);
int mt_scratch_release(void);

/* ---- FlashAttention, device pointers ------------------------------------- */
/* O = softmax(Q Kᵀ/√d [causal]) V;  m[b,h,n] = row max of the scaled logits,
 * l[b,h,n] = Σ exp(s − m)  (P = exp(s − m)/l, the reference contract,
 * src/flashattention_kernel.cu:194). m, l are fp32 [B*H*N] and may be NULL. */
int mt_flash_attn_fwd(int dtype, int causal, const void* q, const void* k, const void* v,
                      void* o, float* m, float* l, int64_t B, int64_t H, int64_t N, int64_t d,
                      const int64_t* q_strides, const int64_t* k_strides,
                      const int64_t* v_strides, const int64_t* o_strides, void* stream);

/* The forward with key padding: kv_len is a device int32 [B] (NULL = none); keys
 * j >= kv_len[b] (clamped to [0, N]) of batch row b are masked for every head and query, as
 * the reference's [B, to_len] additive padding mask does in the fused softmax
 * (src/softmax_kernel.cu:26-33). Queries are not masked (a padded query attends the valid
 * keys). A row with kv_len = 0 gets O = 0, m = -inf, l = 0. bf16 runs the generic / ring
 * kernels here (the d = 64 / 128 MFMA schedules have no per-row key bound). */
int mt_flash_attn_fwd_varlen(int dtype, int causal, const void* q, const void* k, const void* v,
                             void* o, float* m, float* l, int64_t B, int64_t H, int64_t N,
                             int64_t d, const int64_t* q_strides, const int64_t* k_strides,
                             const int64_t* v_strides, const int64_t* o_strides,
                             const int* kv_len, void* stream);

/* Scratch bytes the backward needs: fp32 δ and log2-LSE per row (256-B aligned) and, at
 * d = 64 (N <= 46336), the fused bf16 backward's arrival counters and the dQ partial sums of
 * one group of heads (at most 1 GiB). The layout changed in ABI version 3: size the workspace
 * with this function, never by a formula (mt_flash_attn_bwd_v3 checks the size). */
int64_t mt_flash_attn_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t d);

/* dQ, dK, dV of the forward above, from Q, K, V, O, dO and the forward's (m, l).
 * strides: NULL or 8 consecutive triples for q, k, v, o, dout, dq, dk, dv. */
int mt_flash_attn_bwd(int dtype, int causal, const void* q, const void* k, const void* v,
                      const void* o, const void* dout, const float* m, const float* l,
                      void* dq, void* dk, void* dv, int64_t B, int64_t H, int64_t N,
                      int64_t d, const int64_t* strides, void* workspace, void* stream);
/* The backward of mt_flash_attn_fwd_varlen (same kv_len): padding keys get dK = dV = 0 and
 * add nothing to dQ. */
int mt_flash_attn_bwd_varlen(int dtype, int causal, const void* q, const void* k, const void* v,
                             const void* o, const void* dout, const float* m, const float* l,
                             void* dq, void* dk, void* dv, int64_t B, int64_t H, int64_t N,
                             int64_t d, const int64_t* strides, const int* kv_len,
                             void* workspace, void* stream);
/* ABI 3: mt_flash_attn_bwd_varlen (kv_len may be NULL) with the workspace's size in bytes;
 * returns an error, launching nothing, when it is below mt_flash_attn_bwd_workspace_bytes. */
int mt_flash_attn_bwd_v3(int dtype, int causal, const void* q, const void* k, const void* v,
                         const void* o, const void* dout, const float* m, const float* l,
                         void* dq, void* dk, void* dv, int64_t B, int64_t H, int64_t N,
                         int64_t d, const int64_t* strides, const int* kv_len,
                         void* workspace, int64_t workspace_bytes, void* stream);

/* ---- FlashAttention, reference-compatible host pointers (fp32) ------------ */
/* reference src/flashattention_kernel.cu:259 */
void launch_flashattention_forward(float* Q, float* K, float* V, float* O, float* l, float* m,
                                   int B, int nh, int N, int d);
/* reference src/flashattention_kernel.cu:352 */
void launch_flashattention_backward(float* Q, float* K, float* V, float* O, float* dQ,
                                    float* dK, float* dV, float* dO, float* l, float* m, int B,
                                    int nh, int N, int d);
/* reference src/flashattention_kernel.cu:694 */
void launch_flashattention_forward_causal(float* Q, float* K, float* V, float* O, float* l,
                                          float* m, int B, int nh, int N, int d);
/* reference src/flashattention_kernel.cu:761 */
void launch_flashattention_backward_causal(float* Q, float* K, float* V, float* O, float* dQ,
                                           float* dK, float* dV, float* dO, float* l,
                                           float* m, int B, int nh, int N, int d);


/* ---- companion kernels, device pointers (fp32) ---------------------------- */
/* Row softmax over [B, nh, from, to]: out = exp(x + mask - max) / (sum + 1e-8); out may
 * alias inp. mask: NULL or any tensor broadcastable to [B, nh, from, to] given by 4
 * element strides (b, h, row, col; 0 = broadcast). mask_future masks col > row.
 * (reference src/softmax_kernel.cu:35-224) */
int mt_attn_softmax_fw(float* out, const float* inp, const float* mask, int64_t B, int64_t nh,
                       int64_t from_len, int64_t to_len, const int64_t* mask_strides,
                       int mask_future, void* stream);
/* dinp = soft * (dout - rowsum(dout * soft)); dinp may alias dout. (:308-341) */
int mt_attn_softmax_bw(float* dinp, const float* dout, const float* soft, int64_t rows,
                       int64_t softmax_len, void* stream);
/* LayerNorm over the last dim of [rows, hidden]; var is stored with +1e-8.
 * (reference src/layernorm_kernel.cu:36-98) */
/* Softmax cross-entropy over rows of [rows, classes] fp32 logits (contiguous rows), the
 * reference's softmax_loss (minitorch/nn.py: logsumexp(logits) - logits[target]) in one pass:
 * loss[r] = lse[r] - logits[r, target[r]], lse[r] = log Σ_j exp(logits[r, j]); target holds
 * class ids as floats (minitorch's storage type). Backward:
 * dlogits[r, j] = dloss[r] (exp(logits[r, j] - lse[r]) - [j == target[r]]). */
int mt_softmax_xent_fw(float* loss, float* lse, const float* logits, const float* target, int64_t rows,
                       int64_t classes, void* stream);
int mt_softmax_xent_bw(float* dlogits, const float* dloss, const float* logits, const float* target,
                       const float* lse, int64_t rows, int64_t classes, void* stream);
int mt_layernorm_fw(float* ln_res, float* var, float* mean, const float* inp, const float* gamma,
                    const float* beta, int64_t rows, int64_t hidden, void* stream);
int64_t mt_layernorm_bw_workspace_bytes(int64_t rows, int64_t hidden);
/* (reference src/layernorm_kernel.cu:192-368) */
int mt_layernorm_bw(float* gamma_grad, float* beta_grad, float* inp_grad, const float* out_grad,
                    const float* inp, const float* gamma, const float* beta, const float* var,
                    const float* mean, int64_t rows, int64_t hidden, void* workspace,
                    void* stream);

/* ---- generic strided tensor ops, device pointers (fp32) ------------------- */
/* fn ids as the reference's combine.cu:12-29 (1 add, 2 mul, 3 id, 4 neg, 5 lt, 6 eq,
 * 7 sigmoid, 8 relu, 9 relu_back, 10 log, 11 log_back, 12 exp, 13 inv, 14 inv_back,
 * 15 is_close, 16 max, 17 pow, 18 tanh). Shapes broadcast right-aligned; rank <= 8. */
int mt_tensor_map(int fn, float* out, const int64_t* out_shape, const int64_t* out_strides,
                  int out_dims, const float* in, const int64_t* in_shape,
                  const int64_t* in_strides, int in_dims, void* stream);
int mt_tensor_zip(int fn, float* out, const int64_t* out_shape, const int64_t* out_strides,
                  int out_dims, const float* a, const int64_t* a_shape, const int64_t* a_strides,
                  int a_dims, const float* b, const int64_t* b_shape, const int64_t* b_strides,
                  int b_dims, void* stream);
/* out has a's shape with shape[reduce_dim] = 1; out = fn(start, fn-fold of the axis). */
int mt_tensor_reduce(int fn, float* out, const int64_t* out_shape, const int64_t* out_strides,
                     const float* a, const int64_t* a_shape, const int64_t* a_strides, int dims,
                     int reduce_dim, float start, void* stream);
/* c[b] = a[b] @ b[b]; strides are (batch, row, col) triples, batch stride 0 broadcasts.
 * (reference combine.cu:148-210 MatrixMultiply; cuda_kernel_ops.py:340-437). Plain layouts
 * (a unit stride in one dim of each operand) run on rocBLAS sgemm_strided_batched, others
 * on the library's own fp32 MFMA kernel. */
int mt_matmul_f32(float* c, const float* a, const float* b, int64_t batch, int64_t M, int64_t N,
                  int64_t K, const int64_t* a_strides, const int64_t* b_strides,
                  const int64_t* c_strides, void* stream);
/* 0 (default): rocBLAS for plain layouts; 1: the library's own fp32-MFMA GEMM kernel only;
 * 2: the library's own fp32-accurate GEMM on the bf16 MFMA (three bf16 pieces per operand:
 * 128x128 tiles where they fill the chip, else 64x64 with split-K); 3: that GEMM on 64x64
 * tiles only (A/B). The environment variable MT_GEMM_BACKEND sets the initial value. */
void mt_set_gemm_backend(int backend);

/* out[0..n) <- U[0,1) from a stateless counter-based hash of (seed, index). Replaces the
 * host draws of the reference's dropout paths (minitorch/nn.py dropout via
 * tensor_functions.rand, modules_basic.py Dropout via np.random.binomial), which build and
 * copy a host mask per call. */
int mt_rand_uniform(float* out, int64_t n, uint64_t seed, void* stream);

/* Fused feed-forward pieces (reference minitorch/modules_transfomer.py FeedForward:
 * dropout(linear_out(GELU(linear_in(x))))), fp32, x/dy/out rows of `cols` contiguous floats:
 *   mt_bias_gelu_fw: out = GELU_tanh(x + bias[col])             (linear_in's bias + GELU)
 *   mt_bias_gelu_bw: dx  = dy * GELU_tanh'(x + bias[col])         (dbias = column sums of dx)
 *   mt_dropout:      out = u_i > p ? x * scale : 0, u_i the mt_rand_uniform draw of
 *                    (seed, i), so a backward with the same seed applies the same mask. */
int mt_bias_gelu_fw(float* out, const float* x, const float* bias, int64_t rows, int64_t cols, void* stream);
int mt_bias_gelu_bw(float* dx, const float* dy, const float* x, const float* bias, int64_t rows, int64_t cols,
                    void* stream);
int mt_dropout(float* out, const float* x, int64_t n, float p, float scale, uint64_t seed, void* stream);
/* mt_dropout with the seed read from device memory when the kernel runs (a hipGraph-captured
 * training step writes a fresh seed there before each replay: minitorch/graphs.py) */
int mt_dropout_dseed(float* out, const float* x, int64_t n, float p, float scale, const uint64_t* seed,
                     void* stream);

/* Embedding rows (reference minitorch/modules_basic.py Embedding.forward: one_hot(ids, V) @ W),
 * fp32, ids[ntok] the float token ids, W [V x E] and out / dout [ntok x E] contiguous:
 *   mt_embedding_fw: out[t] = W[ids[t]]            (a zero row for an id outside [0, V))
 *   mt_embedding_bw: dW[v]  = sum over t with ids[t] == v of dout[t] in a fixed order
 *                    (deterministic); every row of dW is written (zero for ids that do not occur) */
int mt_embedding_fw(float* out, const float* ids, const float* weight, int64_t ntok, int64_t V, int64_t E,
                    void* stream);
int mt_embedding_bw(float* dweight, const float* dout, const float* ids, int64_t ntok, int64_t V, int64_t E,
                    void* stream);

/* Multi-tensor Adam step over n_tensors dense fp32 device tensors (parameters, their
 * gradients, first and second moments, numels[t] elements each), in place:
 *   m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2;  p -= step_size m / (sqrt(v) + eps)
 * step_size = lr sqrt(1 - b2^t) / (1 - b1^t) (host-computed bias correction); b1, b2,
 * 1 - b1, 1 - b2, eps and step_size are each rounded to fp32 once; the update divides by
 * (powf(v, 0.5) + eps) through its reciprocal, as the tensor ops do (bit-identical). Replaces the
 * reference's per-parameter tensor-op Adam (minitorch/optim.py:52-75), one launch per 24
 * tensors. */
int mt_adam_step(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                 float* const* exp_avg_sq, const int64_t* numels, double beta1, double beta2, double eps,
                 double step_size, void* stream);
/* mt_adam_step with step_size read (as one fp32) from device memory when the kernel runs: the
 * hipGraph-captured step's per-replay bias correction (minitorch/graphs.py) */
int mt_adam_step_dstep(int n_tensors, float* const* params, const float* const* grads, float* const* exp_avg,
                       float* const* exp_avg_sq, const int64_t* numels, double beta1, double beta2, double eps,
                       const float* step_size, void* stream);

/* ---- reference-compatible host-pointer wrappers (companion + combine) ----- */
/* reference src/softmax_kernel.cu:233 (stream: hipStream_t) */
void launch_attn_softmax(float* inp, const float* attn_mask, int batch_size, int nhead,
                         int from_len, int to_len, bool mask_future, void* stream);
/* reference src/softmax_kernel.cu:345 */
void launch_attn_softmax_bw(float* out_grad, const float* soft_inp, int rows, int softmax_len,
                            void* stream);
/* reference src/layernorm_kernel.cu:101 */
void launch_layernorm(float* ln_res, float* vars, float* means, const float* inp,
                      const float* scale, const float* bias, int batch_size, int hidden_dim,
                      void* stream);
/* reference src/layernorm_kernel.cu:370 */
void launch_layernorm_bw(float* gamma_grad, float* betta_grad, float* inp_grad,
                         const float* out_grad, const float* inp, const float* gamma,
                         const float* betta, const float* vars, const float* means,
                         int batch_size, int hidden_dim, void* stream_1, void* stream_2);
/* reference src/combine.cu:385 */
void tensorMap(float* out, int* out_shape, int* out_strides, int out_size, float* in_storage,
               int* in_shape, int* in_strides, int in_size, int shape_size, int fn_id);
/* reference src/combine.cu:443 */
void tensorZip(float* out, int* out_shape, int* out_strides, int out_size, int out_shape_size,
               float* a_storage, int* a_shape, int* a_strides, int a_size, int a_shape_size,
               float* b_storage, int* b_shape, int* b_strides, int b_size, int b_shape_size,
               int fn_id);
/* reference src/combine.cu:523 */
void tensorReduce(float* out, int* out_shape, int* out_strides, int out_size, float* a_storage,
                  int* a_shape, int* a_strides, int reduce_dim, float reduce_value,
                  int shape_size, int fn_id);
/* reference src/combine.cu:315 */
void MatrixMultiply(float* out, int* out_shape, int* out_strides, float* a_storage, int* a_shape,
                    int* a_strides, float* b_storage, int* b_shape, int* b_strides, int batch,
                    int m, int p);

#ifdef __cplusplus
}
#endif
#endif /* MINITORCH_HIP_H */
