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

enum { MT_F32 = 0, MT_BF16 = 1 };

/* ---- status ------------------------------------------------------------- */
const char* mt_last_error(void);
int mt_abi_version(void);
/* Forward kernel selection (A/B testing). 0 (default): the bf16 MFMA kernel specialised
 * for d in {64, 128} when the layout allows it, else the generic kernel; 1: always the
 * generic tiled kernels; 2, 4, 5, 6: alternative bf16 schedules (see fa_fwd_fast.hip). */
void mt_flash_set_kernel_policy(int policy);

/* ---- FlashAttention, device pointers ------------------------------------- */
/* O = softmax(Q Kᵀ/√d [causal]) V;  m[b,h,n] = row max of the scaled logits,
 * l[b,h,n] = Σ exp(s − m)  (P = exp(s − m)/l, the reference contract,
 * src/flashattention_kernel.cu:194). m, l are fp32 [B*H*N] and may be NULL. */
int mt_flash_attn_fwd(int dtype, int causal, const void* q, const void* k, const void* v,
                      void* o, float* m, float* l, int64_t B, int64_t H, int64_t N, int64_t d,
                      const int64_t* q_strides, const int64_t* k_strides,
                      const int64_t* v_strides, const int64_t* o_strides, void* stream);

/* Scratch bytes mt_flash_attn_bwd needs (fp32 δ and log2-LSE per row). */
int64_t mt_flash_attn_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t d);

/* dQ, dK, dV of the forward above, from Q, K, V, O, dO and the forward's (m, l).
 * strides: NULL or 8 consecutive triples for q, k, v, o, dout, dq, dk, dv. */
int mt_flash_attn_bwd(int dtype, int causal, const void* q, const void* k, const void* v,
                      const void* o, const void* dout, const float* m, const float* l,
                      void* dq, void* dk, void* dv, int64_t B, int64_t H, int64_t N,
                      int64_t d, const int64_t* strides, void* workspace, void* stream);

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

#ifdef __cplusplus
}
#endif
#endif /* MINITORCH_HIP_H */
