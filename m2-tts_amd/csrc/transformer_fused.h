// Fused transformer-layer kernels (transformer_fused.hip).
#pragma once
#include <vector>

#include "m2_common.h"

namespace m2 {

// Hidden sizes with fused-layer instantiations (N_out: output width of ln_gemm).
bool tf_fused_supported(int H, int N_out);
// W [N][K] row-major (nn.Linear.weight) -> B-fragment order for v_mfma_f32_16x16x4_f32.
std::vector<float> pack_bfrag(const float* W, int N, int K);
// W [N][K] -> the fused layers' split-f16 fragment order (same byte count as
// W in fp32); false if a weight is outside the f16 range.
bool pack_bfrag_split(const float* W, int N, int K, std::vector<float>* out);
// y[R][N] = LN(x)[R][K] . W^T (+ bias); Wp from pack_bfrag_split.
int32_t launch_ln_gemm(const float* x, const float* g, const float* b, const float* Wp, const float* bias, int act,
                       int R, int K, int N, float* y, hipStream_t st);
// y = o + FFN(LN2(o)), o = x + att . Wo^T + bo (Wo, W1, W2 from pack_bfrag_split); y may alias x.
int32_t launch_post_attn(const float* att, const float* x, const float* Wo, const float* bo, const float* g2,
                         const float* b2n, const float* W1, const float* b1, const float* W2, const float* b2, int R,
                         int H, float* y, hipStream_t st);
// post_attn followed, on the same row tile, by z = LN(y; gn, bn) . Wn^T (+ bn2)
// with NN output columns (the next layer's LN1 -> QKV, or the final LN -> mel).
bool tf_post_next_supported(int H, int NN);
int32_t launch_post_attn_next(const float* att, const float* x, const float* Wo, const float* bo, const float* g2,
                              const float* b2n, const float* W1, const float* b1, const float* W2, const float* b2,
                              int R, int H, float* y, const float* gn, const float* bn, const float* Wn,
                              const float* bn2, int NN, float* z, hipStream_t st);

// The first layer's LN1 -> QKV with its input rows built in the same launch
// (and stored to x, the residual input): the embedding + positional encoding +
// padding mask of the encoder (embed_pe_kernel), or the length regulator's
// frame expansion of the decoder (lr_expand_kernel).  (H, N) = (32, 96),
// (64, 192), (96, 288).
bool tf_src_fused_supported(int H, int N);
int32_t launch_embed_ln_gemm(const int64_t* ids, const float* emb, const float* pe, int B, int S, int H, int vocab,
                             const int64_t* lengths, uint8_t* mask, float* x, const float* g, const float* b,
                             const float* Wp, int N, float* y, hipStream_t st);
int32_t launch_expand_ln_gemm(const float* enc, const int32_t* cum, int B, int S, int T, int H, float* x,
                              const float* g, const float* b, const float* Wp, int N, float* y, hipStream_t st);

}  // namespace m2
