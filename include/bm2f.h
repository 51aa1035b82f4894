/*
 * bm2f.h — C ABI of the MI355X (gfx950) Mask2Former hot-path library `libbm2f.so`.
 *
 * Every entry point takes plain device pointers, sizes and a `hipStream_t` passed as `void*`
 * (torch's current stream on the Python side), launches asynchronously on that stream and
 * returns 0 on success or a nonzero M2F_E* code; `m2f_last_error()` then holds a message for the
 * calling thread.  Outputs are allocated by the caller; each function fully initialises them
 * (the reference zero-fills with at::zeros, ms_deform_attn_cuda.cu:59 / :126-128).
 *
 * Reference interfaces replaced (paths relative to the reference root,
 * ops = mask2former/modeling/pixel_decoder/ops):
 *   m2f_msda_fwd_{f32,f64}  <- ms_deform_attn_forward   (ops/src/vision.cpp:19, ops/src/ms_deform_attn.h:25-44,
 *                                                        ops/src/cuda/ms_deform_attn_cuda.cu:25-85)
 *   m2f_msda_bwd_{f32,f64}  <- ms_deform_attn_backward  (ops/src/vision.cpp:20, ops/src/ms_deform_attn.h:46-67,
 *                                                        ops/src/cuda/ms_deform_attn_cuda.cu:88-157)
 *   m2f_attn_mask_*         <- MultiScaleMaskedTransformerDecoder.forward_prediction_heads resize+threshold
 *                              (transformer_decoder/mask2former_transformer_decoder.py:446-450) and the
 *                              fully-masked-row fix (:400)
 *   m2f_masked_attn_*       <- the attention core of nn.MultiheadAttention(attn_mask=bool) used by
 *                              CrossAttentionLayer.forward_post (mask2former_transformer_decoder.py:98-110)
 *   m2f_gemm_f32_*          <- the nn.Linear layers of MSDeformAttnTransformerEncoderLayer (value_proj /
 *                              sampling_offsets+attention_weights / output_proj, ms_deform_attn.py:59-62;
 *                              linear1 / linear2 + ReLU, msdeformattn.py:101-106) in fp32 (:314,320)
 *   m2f_add_layernorm_*     <- norm1(src + dropout1(src2)) / norm2(src + dropout3(src2)) of
 *                              MSDeformAttnTransformerEncoderLayer (pixel_decoder/msdeformattn.py:92-131)
 *
 * Preconditions mirrored from the reference (ms_deform_attn_cuda.cu:33-43, :55-57, :98-124):
 *   batch % min(batch, im2col_step) == 0, else M2F_EINVAL.  All tensors contiguous (checked by the
 *   Python wrapper, which owns the strides).  spatial_shapes / level_start_index are int64 device
 *   arrays of (L,2) and (L,).
 */
#ifndef BM2F_H_
#define BM2F_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  M2F_OK = 0,
  M2F_EINVAL = 1,      /* bad sizes / null pointers / precondition violated */
  M2F_ELAUNCH = 2,     /* HIP launch or runtime error */
  M2F_EUNSUPPORTED = 3 /* configuration this build does not implement */
};

/* Element types of the decoder entry points (`dtype` arguments). */
enum { M2F_F32 = 0, M2F_F16 = 1, M2F_BF16 = 2 };

/* Message for the last nonzero return on this thread ("" if none). */
const char* m2f_last_error(void);
/* ABI version, bumped whenever a signature below changes. */
int m2f_abi_version(void);

/* ---------------------------------------------------------------------------------------------
 * Multi-scale deformable attention.
 *   value            (N, S, M, D)          S = sum_l H_l*W_l
 *   spatial_shapes   (L, 2) int64 [H, W]   device
 *   level_start_index(L,)   int64          device
 *   sampling_loc     (N, Lq, M, L, P, 2)   [x, y] normalised to [0,1]
 *   attn_weight      (N, Lq, M, L, P)
 *   output           (N, Lq, M*D)
 * host_spatial_shapes: optional host copy of spatial_shapes (L*2 int64, may be NULL).  When given
 * and Lq == S (encoder self-attention over the flattened pyramid) the forward reads each level's
 * touched box from LDS windows (bit-identical to the untiled forward) and the backward groups queries
 * by spatial tile and accumulates grad_value in LDS windows (results agree with the untiled path up to
 * the order of fp32 additions).  Both tiled paths take each level's start as the prefix sum of the host
 * shapes and do NOT read spatial_shapes / level_start_index: the caller guarantees spatial_shapes ==
 * host_spatial_shapes and level_start_index == their prefix sums (the Python layer checks both once per
 * tensor, bm2f_amd/msda.py attach_host_shapes / _check_level_starts).  Pass NULL to have the kernels
 * read the device arrays as they are.
 * ------------------------------------------------------------------------------------------- */
int m2f_msda_fwd_f32(const float* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                     const float* sampling_loc, const float* attn_weight,
                     int batch, int spatial_size, int num_heads, int channels,
                     int num_levels, int num_query, int num_point, int im2col_step,
                     const int64_t* host_spatial_shapes, float* output, void* stream);

int m2f_msda_fwd_f64(const double* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                     const double* sampling_loc, const double* attn_weight,
                     int batch, int spatial_size, int num_heads, int channels,
                     int num_levels, int num_query, int num_point, int im2col_step,
                     const int64_t* host_spatial_shapes, double* output, void* stream);

/* grad_value (N,S,M,D) is zeroed and accumulated; grad_sampling_loc / grad_attn_weight are
 * written for every element (zero where the sample fell outside its level). */
int m2f_msda_bwd_f32(const float* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                     const float* sampling_loc, const float* attn_weight, const float* grad_output,
                     int batch, int spatial_size, int num_heads, int channels,
                     int num_levels, int num_query, int num_point, int im2col_step,
                     const int64_t* host_spatial_shapes,
                     float* grad_value, float* grad_sampling_loc, float* grad_attn_weight, void* stream);

int m2f_msda_bwd_f64(const double* value, const int64_t* spatial_shapes, const int64_t* level_start_index,
                     const double* sampling_loc, const double* attn_weight, const double* grad_output,
                     int batch, int spatial_size, int num_heads, int channels,
                     int num_levels, int num_query, int num_point, int im2col_step,
                     const int64_t* host_spatial_shapes,
                     double* grad_value, double* grad_sampling_loc, double* grad_attn_weight, void* stream);

/* MSDA with the sampling front end fused in (encoder layout: num_query == spatial_size, the queries
 * being the flattened pyramid; channels 32, points 4, 1..4 levels).  Replaces the chain
 * sampling_offsets / attention_weights Linear -> softmax -> ref + offset / (W, H) -> ms_deform_attn
 * (ops/modules/ms_deform_attn.py:102-117) after the two projections, so sampling_loc / attn_weight are
 * never materialised:
 *   proj  (N, Lq, proj_ld) fp32: columns [0, M*L*P*2) are the offsets (M, L, P, 2), the next M*L*P the
 *         attention logits (M, L*P) -- the concatenated output of the two Linear layers;
 *   ref   reference points (N, Lq, L, 2) [x, y], batch stride ref_batch_stride elements (0 = broadcast);
 *   host_spatial_shapes (L*2 int64, host, required).
 * The backward writes grad_value (zeroed + accumulated) and grad_proj (N, Lq, M*L*P*3) contiguous:
 * d offsets and d logits (the softmax backward applied in-kernel).  Reference points get no gradient. */
int m2f_msda_fused_fwd_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                           int64_t ref_batch_stride, const int64_t* host_spatial_shapes, int batch,
                           int spatial_size, int num_heads, int channels, int num_levels, int num_query,
                           int num_point, float* output, void* stream);

/* grad_value rows are added with fp32 atomics from the tiled workgroups' LDS windows (each window row is
 * flushed once; values repeat to within fp32 rounding, not bit for bit), and no workspace is needed
 * (m2f_msda_fused_bwd_workspace() reports 0 bytes).  Deterministic mode (m2f_set_option("msda_bwd_det", 1)):
 * grad_value is bitwise repeatable -- each workgroup sums its window rows in a fixed order and adds them, and
 * the out-of-window samples, as 64-bit fixed point (scale 2^k from the launch's max |grad_output|, resolution
 * max|g| * 2^-(61 - ceil(log2 Lq))) with integer atomics, then a pass converts to fp32; it needs the workspace
 * m2f_msda_fused_bwd_workspace() then reports (8 bytes per grad_value element + 16, 16-byte aligned) and
 * returns M2F_EINVAL without it.  A non-finite grad_output sends it down the fp32 atomics (as the reference). */
int m2f_msda_fused_bwd_workspace(const int64_t* host_spatial_shapes, int batch, int spatial_size, int num_heads,
                                 int channels, int num_levels, int num_point, int64_t* workspace_bytes);
int m2f_msda_fused_bwd_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                           int64_t ref_batch_stride, const int64_t* host_spatial_shapes,
                           const float* grad_output, int batch, int spatial_size, int num_heads, int channels,
                           int num_levels, int num_query, int num_point, float* grad_value, float* grad_proj,
                           void* workspace, int64_t workspace_bytes, void* stream);

/* The same two calls with the projection rows head-major: per head m one record
 * [offsets (L, P, 2) | logits (L*P)] of 3*L*P floats, the heads in order (a row permutation of the projection
 * weight, which the module applies: bm2f_amd.msda.MSDeformAttn); grad_proj comes back in the same layout.  Each
 * head's slice is then one 12*L*P-byte piece of the row instead of two, so the 8 heads' workgroups -- dealt to
 * different XCDs -- share fewer 128-byte lines (config 2: backward FETCH -16 %, -2.8 % time; forward -1.5 %).
 * Results are those of the reference layout, bit for bit. */
int m2f_msda_fused_fwd_hm_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                              int64_t ref_batch_stride, const int64_t* host_spatial_shapes, int batch,
                              int spatial_size, int num_heads, int channels, int num_levels, int num_query,
                              int num_point, float* output, void* stream);
int m2f_msda_fused_bwd_hm_f32(const float* value, const float* proj, int proj_ld, const float* ref,
                              int64_t ref_batch_stride, const int64_t* host_spatial_shapes,
                              const float* grad_output, int batch, int spatial_size, int num_heads, int channels,
                              int num_levels, int num_query, int num_point, float* grad_value, float* grad_proj,
                              void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Masked-attention decoder (mask2former_transformer_decoder.py).
 *
 * m2f_attn_mask_bits: logits (B, Q, frames, in_h, in_w) of `dtype` -> bits (B, Q, nwords) uint32, bit k
 * of word w = 1 when key 32*w + k (frame-major, then row-major in out_h x out_w) is BLOCKED, i.e.
 *   dtype( sigmoid( dtype( bilinear_resize(logits, (out_h, out_w), align_corners=False) ) ) ) < 0.5
 * exactly as F.interpolate(...).sigmoid() < 0.5 in that dtype (reference :446-449).  With row_fix != 0
 * a row whose every pixel is blocked is cleared, the fix the reference applies before each
 * cross-attention (:400).  One bit per (b, q, pixel) serves all heads (the reference repeats the
 * bool mask per head).  nwords >= ceil(frames*out_h*out_w / 32); unused tail bits are 0.  frames > 1 is
 * the video decoder's per-frame resize of (B, Q, T, H, W) logits (video_..._decoder.py:453-458).
 * ------------------------------------------------------------------------------------------- */
int m2f_attn_mask_bits(const void* logits, int dtype, int batch, int num_queries, int frames, int in_h,
                       int in_w, int out_h, int out_w, int row_fix, uint32_t* bits, int nwords, void* stream);

/* Mask head with the bitmask epilogue (reference :437-452; video_..._decoder.py:444-461):
 *   masks[b, q, t, n] = dtype( sum_c embed[b, q, c] * feats[b, c, t, n] )      (n = y * width + x)
 * embed (B, Q, C), feats (B, C, frames, height, width), masks (B, Q, frames, height, width), all of `dtype`
 * (bf16 or f16; fp32 accumulation).  With target_h > 0 it also writes into `bits` (zeroed, (B, Q, nwords))
 * the blocked bits m2f_attn_mask_bits would compute from `masks` for (target_h, target_w) before its row
 * fix; height / target_h = width / target_w must be an even integer dividing 128.  Constraints: C % 32 == 0,
 * width % 8 == 0, Q <= 256, 16-byte aligned operands. */
int m2f_mask_heads_fwd(int dtype, const void* embed, const void* feats, int batch, int num_queries, int channels,
                       int frames, int height, int width, int target_h, int target_w, void* masks, uint32_t* bits,
                       int nwords, void* stream);

/* Fully-masked-row fix (:400) after m2f_mask_heads_fwd: each of `rows` bit rows whose `keys` bits are all set
 * is cleared. */
int m2f_mask_row_fix(uint32_t* bits, int rows, int nwords, int keys, void* stream);

/* Mask-head einsum backward (autograd of :442 / video :449), dtype bf16 or f16, fp32 accumulation.
 * m2f_mask_heads_bwd_embed: grad_embed (B, Q, 256) = dtype( grad_masks (B, Q, n) . feats (B, 256, n)^T ), split
 *   over n with fp32 partials summed in a fixed order; workspace from m2f_mask_heads_bwd_workspace.
 *   Needs n % 16 == 0, Q <= 256.
 * m2f_mask_heads_bwd_feats: grad_feats (B, 256, n) = out_dtype( sum_h embed_h^T . grad_masks_h ) over `heads`
 *   heads' gradients (an array of device pointers, each (B, Q, n), no concatenation); embed_t is the
 *   heads' embeds transposed, Et[b][c][k] = embed_{k / padded_queries}[b][k % padded_queries][c] for k < heads *
 *   padded_queries (zero past Q in each head's padded_queries slots, a multiple of 16), stored in MFMA
 *   fragment order: element (b, c, k) at ((((b * 8 + c / 32) * (K / 16) + k / 16) * 2 + (k / 8) % 2) * 32 +
 *   c % 32) * 8 + k % 8, K = heads * padded_queries.  out_dtype = dtype, or M2F_F32 when the features are fp32
 *   (autocast's copy): one rounding either way.  heads <= 16, n % 8 == 0. */
int m2f_mask_heads_bwd_workspace(int batch, int num_queries, int64_t n, int64_t* workspace_bytes);
int m2f_mask_heads_bwd_embed(int dtype, const void* grad_masks, const void* feats, int batch, int num_queries,
                             int channels, int64_t n, void* grad_embed, void* workspace, int64_t workspace_bytes,
                             void* stream);
int m2f_mask_heads_bwd_feats(int dtype, const void* const* grad_masks, int heads, const void* embed_t, int batch,
                             int num_queries, int padded_queries, int channels, int64_t n, int out_dtype,
                             void* grad_feats, void* stream);

/* Work split of the masked attention for these sizes: keys are processed in `num_chunks` ranges of
 * `chunk_len`; the forward / backward need the returned fp32 workspace sizes (0 when one chunk). */
int m2f_masked_attn_plan(int batch, int num_queries, int num_keys, int num_heads, int* chunk_len,
                         int* num_chunks, int64_t* fwd_workspace_bytes, int64_t* bwd_workspace_bytes);

/* out = softmax(scale * q k^T, masked by bits) v, per (batch, head); head_dim must be 32.
 *   q   (B, Lq, H*32) with row stride q_row_stride elements;  k, v (B, Lk, H*32), row stride kv_row_stride
 *   out (B, Lq, H*32) contiguous;  lse (B, H, Lq) fp32 log-sum-exp (base-2, internal) for the backward.
 * A query row with every key blocked yields zeros (the reference never passes one: row_fix). */
int m2f_masked_attn_fwd(int dtype, const void* q, const void* k, const void* v, const uint32_t* bits,
                        int batch, int num_queries, int num_keys, int num_heads, int head_dim,
                        int q_row_stride, int kv_row_stride, int mask_words, float scale, void* out,
                        float* lse, void* workspace, int64_t workspace_bytes, void* stream);

/* Gradients of m2f_masked_attn_fwd: grad_q (B, Lq, H*32), grad_k / grad_v (B, Lk, H*32), all
 * contiguous and fully written.  grad_q is summed over key chunks in a fixed order. */
int m2f_masked_attn_bwd(int dtype, const void* q, const void* k, const void* v, const uint32_t* bits,
                        const void* out, const void* grad_out, const float* lse, int batch,
                        int num_queries, int num_keys, int num_heads, int head_dim, int q_row_stride,
                        int kv_row_stride, int mask_words, float scale, void* grad_q, void* grad_k,
                        void* grad_v, void* workspace, int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Residual add + LayerNorm over the last dimension (fp32), the encoder layer's post-norm:
 *   y = (x - mean) * rstd * gamma + beta,  x = a + b (b may be NULL: plain LayerNorm),
 *   mean / rstd per row (rows,), rstd = 1 / sqrt(var + eps) with the biased variance.
 * a, b, y, grad_* are (rows, C) row-major, 16-byte aligned; C % 4 == 0 and C <= 1024.
 * The backward recomputes x from a and b and returns grad_x (the gradient of both a and b);
 * grad_gamma / grad_beta (may be NULL) are reduced in a fixed order (deterministic) through a
 * caller-provided workspace of m2f_add_layernorm_workspace() bytes. */
int m2f_add_layernorm_workspace(int64_t rows, int C, int64_t* workspace_bytes);
int m2f_add_layernorm_fwd_f32(const float* a, const float* b, const float* gamma, const float* beta,
                              int64_t rows, int C, float eps, float* y, float* mean, float* rstd,
                              void* stream);
int m2f_add_layernorm_bwd_f32(const float* grad_y, const float* a, const float* b, const float* gamma,
                              const float* mean, const float* rstd, int64_t rows, int C, float* grad_x,
                              float* grad_gamma, float* grad_beta, void* workspace,
                              int64_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Exact-fp32 GEMMs on the f32 MFMA (row-major; lda/ldb/ldc/ldm are row pitches in elements).
 *
 * m2f_gemm_f32_nt:  C[M,N] = A[M,K] . B[N,K]^T  (+ bias[N] if bias) then ReLU if relu, or
 *                   C *= (mask[M,N] > 0) if mask (ReLU backward through the saved activation).
 *   K, lda, ldb multiples of 4; A, B 16-byte aligned.  Forward of nn.Linear is B = weight;
 *   its input gradient is B = weight^T (the caller transposes the weight).
 * m2f_gemm_f32_tn:  C[N1,N2] = A[M,N1]^T . B[M,N2] and, if colsum, colsum[N1] = sum_m A[m,:]
 *   (weight and bias gradients of nn.Linear: A = grad_out, B = input).  Rows are split over
 *   workgroups; the fp32 partial slabs are summed in a fixed order (deterministic) through a
 *   workspace of m2f_gemm_f32_tn_workspace() bytes.  N1, N2, lda, ldb multiples of 4. */
int m2f_gemm_f32_nt(const float* A, int64_t lda, const float* B, int64_t ldb, const float* bias, int relu,
                    const float* mask, int64_t ldm, float* C, int64_t ldc, int M, int N, int K, void* stream);
int m2f_gemm_f32_tn_workspace(int M, int N1, int N2, int64_t* workspace_bytes);
int m2f_gemm_f32_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                    float* colsum, int M, int N1, int N2, void* workspace, int64_t workspace_bytes,
                    void* stream);

/* ---------------------------------------------------------------------------------------------
 * fp32 GEMMs on the bf16 MFMA by exact three-way operand splitting (x = h + m + l, three bf16
 * planes; the six products of order <= 2^-16 kept: error at the level of one fp32 rounding), at
 * 2.7x the f32-MFMA peak.  Same math as m2f_gemm_f32_nt / _tn above (fp32 in, fp32 out).
 * m2f_gemm_f32x3_nt:  B is [N][K] (ldb >= K), or [K][N] when b_kn (ldb >= N; e.g. the weight
 *   itself for an input gradient, no transpose copy).  Needs m2f_gemm_f32x3_nt_workspace() bytes
 *   (16-byte aligned) for the split B.  K, lda multiples of 4; A 16-byte aligned.
 * m2f_gemm_f32x3_tn:  as m2f_gemm_f32_tn, with m2f_gemm_f32x3_tn_workspace() bytes; no alignment
 *   requirement. */
int m2f_gemm_f32x3_nt_workspace(int N, int K, int64_t* workspace_bytes);
int m2f_gemm_f32x3_nt(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn, const float* bias,
                      int relu, const float* mask, int64_t ldm, float* C, int64_t ldc, int M, int N, int K,
                      void* workspace, int64_t workspace_bytes, void* stream);
/* m2f_gemm_f32x3_nt_add: as m2f_gemm_f32x3_nt with C = A.B^T (+ bias) + D1 (+ D2), the addends
 *   [M][N] with row stride ldd (C may alias D1 or D2).  Replaces the autograd gradient sums
 *   (AccumulateGrad / AddBackward) over a tensor with several consumers in the encoder layer
 *   (msdeformattn.py:115-131: src feeds value_proj, the query and the residual; its FFN input feeds
 *   linear1 and the residual).  Addends exclude relu and mask; N, ldd, ldc multiples of 4; D1, D2, C
 *   16-byte aligned. */
int m2f_gemm_f32x3_nt_add(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn, const float* bias,
                          int relu, const float* mask, int64_t ldm, const float* D1, const float* D2, int64_t ldd,
                          float* C, int64_t ldc, int M, int N, int K, void* workspace, int64_t workspace_bytes,
                          void* stream);
/* m2f_gemm_f32x3_nt_rowadd: C = A.B^T + R[m % period] -- a row-periodic addend (R [period][N], row stride ldr).  The
 *   encoder's query projection (src + pos) Wq^T + bq (ms_deform_attn.py:97-103 with msdeformattn.py:115) for a
 *   position embedding shared by the batch: R = pos Wq^T + bq is formed once per layer on the S rows of one image,
 *   so the (N*S, C) sum src + pos is never materialised.  Same constraints as the addends of _nt_add. */
int m2f_gemm_f32x3_nt_rowadd(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn, const float* R,
                             int64_t ldr, int period, float* C, int64_t ldc, int M, int N, int K, void* workspace,
                             int64_t workspace_bytes, void* stream);
/* m2f_gemm_f32x3_nt_bits: the FFN's ReLU as a 1-bit mask (msdeformattn.py:101-106).  With bits_out (relu != 0):
 *   C = relu(A.B^T + bias) and bits_out[m][n / 32] bit n % 32 = (C[m][n] > 0).  With bits_in (relu == 0):
 *   C = (A.B^T + bias) where the bit is set, else 0 -- the ReLU backward of grad_h = grad_y . W2 read from
 *   M*N/8 bytes instead of the (M, N) fp32 activation.  Exactly one of bits_out / bits_in; N % 32 == 0,
 *   ldbits (in 32-bit words) >= N / 32, ldc % 4 == 0, C 16-byte aligned. */
int m2f_gemm_f32x3_nt_bits(const float* A, int64_t lda, const float* B, int64_t ldb, int b_kn, const float* bias,
                           int relu, uint32_t* bits_out, const uint32_t* bits_in, int64_t ldbits, float* C,
                           int64_t ldc, int M, int N, int K, void* workspace, int64_t workspace_bytes, void* stream);
int m2f_gemm_f32x3_tn_workspace(int M, int N1, int N2, int64_t* workspace_bytes);
int m2f_gemm_f32x3_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                      float* colsum, int M, int N1, int N2, void* workspace, int64_t workspace_bytes,
                      void* stream);

/* ---------------------------------------------------------------------------------------------
 * fp32 convolutions on the x3 engine (NCHW, stride 1, 1x1 or 3x3 with "same" padding, no groups):
 * the pixel decoder's input_proj / adapter / layer / mask_features convs (msdeformattn.py:213-292),
 * replacing cuDNN/MIOpen calls of F.conv2d.  Needs channels % 16 == 0, H*W % 128 == 0, W % 8 == 0.
 * m2f_conv_f32x3: mode 0 O[N][Co][H][W] = conv(I[N][Ci][H][W], W[Co][Ci][k][k]) (+ bias[Co]);
 *                 mode 1 O[N][Ci][H][W] = input gradient of I = grad_out[N][Co][H][W] (no bias).
 * m2f_conv_f32x3_wgrad: dW_tck[k*k][Ci][Co] (tap-major: the caller permutes to [Co][Ci][k][k]) and,
 *                 if dbias, dbias[Co]; split over pixels, slabs summed in a fixed order.
 * All three take m2f_conv_f32x3_workspace() bytes (16-byte aligned). */
int m2f_conv_f32x3_workspace(int N, int Ci, int Co, int H, int W, int ksize, int64_t* workspace_bytes);
int m2f_conv_f32x3(const float* I, const float* W, const float* bias, float* O, int N, int Ci, int Co, int H, int Wd,
                   int ksize, int mode, void* workspace, int64_t workspace_bytes, void* stream);
int m2f_conv_f32x3_wgrad(const float* grad_out, const float* I, float* dW_tck, float* dbias, int N, int Ci, int Co,
                         int H, int Wd, int ksize, void* workspace, int64_t workspace_bytes, void* stream);
/* The same convolutions on the backbone's 16-bit features without the reference's .float() copy
 * (msdeformattn.py:320, 336; the conversion is exact, so the results are those of the fp32 calls on
 * the upcast tensor): 1x1 only.  m2f_conv_x3_io mode 0 reads I as i_dtype (M2F_F32 / M2F_F16 /
 * M2F_BF16), NCHW or (i_nhwc, 16-bit only) NHWC, and writes fp32 NCHW (o_dtype M2F_F32, o_nhwc 0);
 * mode 1 reads fp32 NCHW grad_out and writes the input gradient as o_dtype, NCHW or (o_nhwc) NHWC,
 * rounded to nearest even (the cast's backward).  m2f_conv_x3_wgrad_io: as m2f_conv_f32x3_wgrad with
 * I of i_dtype / i_nhwc.  Workspace as above. */
int m2f_conv_x3_io(const void* I, int i_dtype, int i_nhwc, const float* W, const float* bias, void* O, int o_dtype,
                   int o_nhwc, int N, int Ci, int Co, int H, int Wd, int ksize, int mode, void* workspace,
                   int64_t workspace_bytes, void* stream);
int m2f_conv_x3_wgrad_io(const float* grad_out, const void* I, int i_dtype, int i_nhwc, float* dW_tck, float* dbias,
                         int N, int Ci, int Co, int H, int Wd, int ksize, void* workspace, int64_t workspace_bytes,
                         void* stream);

/* out[n] (fp32) = ((s_0 + s_1) + ...) + s_{k-1}, every term converted to fp32 (dtype M2F_F16 / M2F_BF16 /
 * M2F_F32) and added in fp32 in order -- the values of out = s_0.float() and k - 1 in-place mixed-dtype adds, in
 * one pass.  srcs: a host array of k <= 8 device pointers; n % 8 == 0, 16-byte aligned.  Replaces the autograd
 * sums of the decoder's memory-token input gradients (mask2former_transformer_decoder.py:103-108). */
int m2f_sum_to_f32(const void* const* srcs, int k, int64_t n, int dtype, float* out, void* stream);

/* Fused per-channel bias (+ residual) + ReLU in place over an NCHW activation (dtype M2F_BF16, M2F_F16
 * or M2F_F32), memory NCHW or (channels_last != 0) NHWC: x = max(x + residual + bias[c], 0).  The
 * benchmark backbone's FrozenBN shift + shortcut + ReLU in one pass (not on the reference's hot path).
 * H*W (NCHW) or C (NHWC) % 8 (bf16 / fp16) / % 4 (fp32), 16-byte aligned. */
int m2f_bias_act_nchw(void* x, const void* residual, const float* bias, int64_t N, int C, int64_t HW, int dtype,
                      int channels_last, void* stream);

/* ReLU backward over the summed gradients of up to 4 consumers of one activation y (the benchmark
 * backbone's block outputs): out = (grads[0] + ... + grads[ngrads-1]) where !(y <= 0), else 0 (torch's
 * threshold_backward rule: a NaN y passes the gradient), summed in fp32 in the given order and rounded once;
 * bf16, fp16 or fp32, contiguous, n % 8 (16-bit) / % 4 (fp32), 16-byte aligned (else M2F_EUNSUPPORTED).
 * Replaces the autograd engine's accumulating adds plus torch's threshold_backward (one pass, k + 1 reads). */
int m2f_relu_bwd_sum(const void* const* grads, int ngrads, const void* y, void* out, int64_t n, int dtype,
                     void* stream);

/* The benchmark backbone's stem max pool (kernel 3, stride 2, padding 1; detectron2 BasicStem; not on the
 * reference's hot path), NCHW, dtype M2F_BF16, M2F_F16 or M2F_F32, planes = N*C, output (H-1)/2+1 x (W-1)/2+1.
 * m2f_maxpool3s2_fwd: torch's max_pool2d_with_indices rule (first maximum in window order, NaN wins); the
 *   winner's window position (0..8) goes to window[planes][OH][OW] (1 byte instead of an int64 index).
 * m2f_maxpool3s2_bwd: grad_x = each input pixel's sum over the windows it won (torch's order, fp32). */
int m2f_maxpool3s2_fwd(const void* x, void* y, uint8_t* window, int64_t planes, int H, int W, int dtype, void* stream);
int m2f_maxpool3s2_bwd(const void* grad_y, const uint8_t* window, void* grad_x, int64_t planes, int H, int W, int dtype,
                       void* stream);
/* The same max pool on a channels-last (NHWC) 16-bit tensor (N, H, W, C), C % 8 == 0: backward = 0 reads src = x
 * and writes dst = y (N, OH, OW, C) and window (N, OH, OW, C) bytes; backward = 1 reads src = grad_y and window and
 * writes dst = grad_x (N, H, W, C). */
int m2f_maxpool3s2_nhwc(int backward, const void* src, void* dst, uint8_t* window, int N, int H, int W, int C,
                        int dtype, void* stream);

/* Explicit tuning options: geometry / engine overrides for tests and tools (the library never reads the
 * environment).  value < 0 restores the built-in default.  Names: msda_threads, msda_tile, msda_tile_w,
 * msda_halo, msda_win_rows, msda_bwd_tiled, msda_fwd_tiled, msda_fwd_quad, msda_fwd_pb, msda_bwd_overlap,
 * msda_bwd_ratio, msda_bwd_det, msda_fwd_lds, msda_fwd_tile, msda_fwd_tile_w, msda_fwd_cap, msda_fwd_halo (MSDA
 * partitions, variants, LDS windows, deterministic mode), msda_bwd_rowsort, msda_bwd_walk4 (tiled backward phase 3:
 * rows by record count, four records per step; both 1 by default), msda_fwd_pair (LDS-window forward with two lanes
 * per query: 1, or a lane quad: 0, the default), msda_fwd_xcd (forward blocks: all heads of a tile on one XCD: 1, or
 * the head fastest: 0, the default), mattn_dq_atomic, mattn_fwd_minblk, mattn_bwd_minblk,
 * mattn_bwd_keys, mattn_xcd (masked-attention dQ variant, key blocks per workgroup at least, keys per wave in the
 * backward: 32 or 16, the heads of one image and key chunk on one XCD: 1 or 0), mattn_combine (forward chunk
 * combine: a thread per row part 0, a wave per row 1), mask_df_stage (mask-einsum feature
 * gradient: k-steps per LDS stage, 4 or 1), gemm_nt_cfg, x3_tn_nw, x3_tn_blocks,
 * x3_nt_cfg (GEMM tilings).  Every option changes
 * the partition or kernel variant only; results agree to fp32 rounding (summation order may differ between
 * variants).  Process-wide; not synchronised with launches in flight on other threads.  Unknown names return
 * M2F_EINVAL. */
int m2f_set_option(const char* name, int64_t value);
int m2f_get_option(const char* name, int64_t* value);

/* Achievable-HBM probe (BASELINE.md §4 asks for measured peaks beside the spec sheet's): out = in over
 * nbytes (16-byte aligned, nbytes % 16 == 0); moves 2 * nbytes.  mode 0: one pass of plain 16-byte loads and
 * stores (4 per thread); mode 1: a fixed grid striding with nontemporal loads and stores. */
int m2f_stream_copy(const void* in, void* out, int64_t nbytes, int mode, void* stream);

/* Achievable L2-gather probe (the MSDA kernels' binding path): n pseudo-random 128-byte rows of `table`
 * (rows x 32 floats, 16-byte aligned) gathered by 8-lane groups, a float4 per lane, four rows in flight;
 * out receives 2048 * 256 floats (out_len >= that).  Gathered bytes = 128 * n. */
int m2f_gather_probe(const float* table, int rows, int64_t n, float* out, int out_len, void* stream);

/* Batched fp32 transpose out[b][q][r] = in[b][r][q] (row strides in_ld / out_ld, batch strides in_bs /
 * out_bs, in elements; B <= 65535): the pixel decoder's level flatten, cat([x_l.flatten(2).transpose(1, 2)],
 * 1) (msdeformattn.py:64-74), and its backward. */
int m2f_transpose_f32(const float* in, int64_t in_bs, int64_t in_ld, float* out, int64_t out_bs, int64_t out_ld,
                      int B, int R, int Q, void* stream);

/* Column sums out[c] = sum_r src[r][c] in fp32 over a row-major (rows, cols) matrix (dtype f32, f16 or bf16):
 * fp32 partials per 1024-row chunk (workspace from m2f_colsum_workspace), added in chunk order, no memset.
 * The gradients of the decoder's memory-token projection biases (nn.MultiheadAttention in_proj,
 * mask2former_transformer_decoder.py:103-108) and of the level embeddings (:376, msdeformattn.py:75). */
int m2f_colsum_workspace(int64_t rows, int cols, int64_t* workspace_floats);
int m2f_colsum(int dtype, const void* src, int64_t rows, int cols, float* workspace, int64_t workspace_floats,
               float* out, void* stream);

/* GroupNorm (+ ReLU when relu != 0) over fp32 NCHW x (N, C, H*W = HW), G groups, affine gamma/beta (may
 * be null): the pixel decoder's GN layers (msdeformattn.py:216-219, :269-281; nn.GroupNorm(32, C)
 * semantics, biased variance, eps).  fwd writes y and the per-(n, g) mean / rstd (N*G floats each) the
 * backward takes; bwd recomputes the ReLU mask from x and writes dx, and dgamma / dbeta if non-null.
 * Statistics and reductions in fp64 with fixed-order combines (deterministic).  HW % 4 == 0; x, y, dy,
 * dx and the workspace (m2f_group_norm_workspace bytes) 16-byte aligned. */
int m2f_group_norm_workspace(int N, int C, int G, int64_t HW, int64_t* workspace_bytes);
int m2f_group_norm_fwd_f32(const float* x, const float* gamma, const float* beta, int N, int C, int G, int64_t HW,
                           float eps, int relu, float* y, float* mean, float* rstd, void* workspace,
                           int64_t workspace_bytes, void* stream);
int m2f_group_norm_bwd_f32(const float* dy, const float* x, const float* mean, const float* rstd, const float* gamma,
                           const float* beta, int N, int C, int G, int64_t HW, int relu, float* dx, float* dgamma,
                           float* dbeta, void* workspace, int64_t workspace_bytes, void* stream);

/* FPN merge of the pixel decoder, msdeformattn.py:343-349 (the lateral plus the bilinear upsample of the
 * coarser map, F.interpolate(..., mode="bilinear", align_corners=False)) for the exact 2x case, fp32:
 * m2f_upsample2x_add_fwd_f32:  out[N][C][2h][2w] = lateral + up2x(src); src (N, C, h, w) read through
 *   element strides (sN, sC, sY, sX), so a transposed (N, HW, C) view needs no copy.  2w % 4 == 0;
 *   lateral and out contiguous, 16-byte aligned.
 * m2f_upsample2x_bwd_f32:  grad_src[N][C][h][w] (contiguous) = the adjoint of up2x applied to
 *   grad_out[N][C][2h][2w] (a gather with the forward's weights: deterministic, no atomics).  The
 *   lateral's gradient is grad_out itself. */
int m2f_upsample2x_add_fwd_f32(const float* src, int64_t sN, int64_t sC, int64_t sY, int64_t sX, const float* lateral,
                               float* out, int N, int C, int h, int w, void* stream);
int m2f_upsample2x_bwd_f32(const float* grad_out, float* grad_src, int N, int C, int h, int w, void* stream);
/* Channels-last coarse map (the encoder's (N, HW, C) output seen as (N, C, h, w); msdeformattn.py:335-349): src is
 * (N, h, w, C) with batch stride sN elements (sN >= h*w*C, a multiple of 4: the level's slice of the (N, S, C) encoder
 * output), grad_src (N, h, w, C) contiguous, lateral / out / grad_out NCHW; C % 64 == 0, even w <= 256; same
 * taps, products and summation order as the NCHW pair above.  Replace the transposing copy before the forward and the
 * mixed-layout gradient sum after the backward. */
int m2f_upsample2x_add_fwd_nhwc_f32(const float* src, int64_t sN, const float* lateral, float* out, int N, int C, int h,
                                    int w, void* stream);
int m2f_upsample2x_bwd_nhwc_f32(const float* grad_out, float* grad_src, int N, int C, int h, int w, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Weak-supervision criterion (SUP_TYPE "mask_projection_and_pairwise"), SURVEY 8(f) ranks 1 and 3.
 * ------------------------------------------------------------------------------------------- */

/* Batched linear sum assignment, replacing scipy.optimize.linear_sum_assignment on C.cpu()
 * (mask2former/modeling/matcher.py:309-311; same shortest-augmenting-path algorithm and tie rule,
 * in fp64).  Problem b is cost[b*batch_stride + r*max_cols + c] for r < rows[b], c < cols[b]
 * (cols == NULL: max_cols).  match[b*max_rows + r] = matched column or -1.  status[b] = 0 ok,
 * 1 infeasible, 2 too large, 3 NaN / -inf entry (scipy raises ValueError for 1 and 3).
 * Limits per problem: min(rows, cols) <= 256, max(rows, cols) <= 1024.  One wavefront per problem. */
int m2f_lsap_batched(const float* cost, int batch, int max_rows, int max_cols, int64_t batch_stride,
                     const int* rows, const int* cols, int* match, int* status, void* stream);

/* Pairwise affinity term s(p,q) = -log(sig(x_p)sig(x_q) + sig(-x_p)sig(-x_q)) over the 8 dilated
 * neighbours of each pixel (criterion.py:156-181, matcher.py:48-83, weaksup_utils.py:7-31; zero
 * padding outside the image as F.unfold).  Row r reads mask x[x_row[r]] (H, W) fp32, neighbour
 * bits[t_row[r]] (H*W bytes, bit k = similarity_k >= thresh) and weight box[box_row[r]] (or 1).
 * NULL index arrays mean identity.  mode 0: out[r, p] = sum_k bit_k s_k;  mode 1: per-tile
 * partials out[r, t] = sum_p w sum_k bit_k s_k and out_den[r, t] = sum_p w popcount(bits), with
 * t < m2f_pairwise_tiles(H, W);  mode 2: out[r, k, p] = s_k (bits unused).  1 <= dilation <= 4,
 * R <= 65535. */
int m2f_pairwise_tiles(int H, int W);
int m2f_pairwise_rows(const float* x, const int* x_row, int R, int H, int W, int dilation, const uint8_t* bits,
                      const int* t_row, const float* box, const int* box_row, int mode, float* out, float* out_den,
                      void* stream);
/* The matcher's fused pass over the (B*Q, H, W) mask logits x (query q of image b is row b*Q+q):
 * part_cost[r, t, g] = sum_{p in tile t} box[b, g, p] sum_k bit_k s_k (bits[b]: the image's neighbour
 * bits; box (B, Gm, H, W); 0 for g >= gcount[b]), rowmax[r, y, tx] / colmax[r, ty, x] = per-tile maxima
 * of x along W / H (tiles: 16 rows x 64 columns, t = ty * ceil(W/64) + tx).  gbox (B, Gm, 4) int32
 * [y0, y1, x0, x1) must contain every nonzero pixel of box[b, g] (tiles outside it are skipped).
 * Gm <= 256. */
int m2f_pairwise_match_cost(const float* x, int B, int Q, int H, int W, int dilation, const uint8_t* bits,
                            const float* box, const int* gcount, const int* gbox, int Gm, float* part_cost,
                            float* rowmax, float* colmax, void* stream);
/* Gradient of sum_r grad_scale[r] * (mode-1 numerator of row r) w.r.t. x[x_row[r]], written to
 * grad[r] (R, H, W) (not accumulated). */
int m2f_pairwise_rows_bwd(const float* x, const int* x_row, int R, int H, int W, int dilation, const uint8_t* bits,
                          const int* t_row, const float* box, const int* box_row, const float* grad_scale,
                          float* grad, void* stream);
/* bits[n, p] = sum_k (sim[n, k, p] >= thr) << k for an (N, 8, HW) similarity. */
int m2f_threshold_bits(const float* sim, int N, int64_t HW, float thr, uint8_t* bits, void* stream);

/* Target preparation (maskformer_model.py:417-440): images (B, 3, Hp, Wp) fp32 in 0..255 (zero
 * padded) -> lab (B, 3, Hp/stride, Wp/stride): stride x stride average pool, Tensor.byte(),
 * skimage.color.rgb2lab (D65/2deg, double precision) -> fp32. */
int m2f_weaksup_lab(const float* images, int B, int Hp, int Wp, int stride, float* lab, void* stream);
/* sim (B, 8, h, w) = exp(-0.5 * ||lab_p - lab_q||) * mask_q, q = p + dilation * tap_k (0 outside),
 * get_images_color_similarity (weaksup_utils.py:34-57) batched over images. */
int m2f_color_similarity(const float* lab, const float* mask, int B, int h, int w, int dilation, float* sim,
                         void* stream);

#ifdef __cplusplus
}
#endif

#endif /* BM2F_H_ */
