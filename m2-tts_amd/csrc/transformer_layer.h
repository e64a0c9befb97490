// One-launch-per-layer transformer kernels (transformer_layer.hip).
#pragma once
#include "m2_common.h"

namespace m2 {

// Attention inputs of one layer in the layouts the fused layer kernel reads
// (written by the producing launch's epilogue, split into f16 hi/lo once):
//   q, k  [B*heads][npad][hi DP | lo DP] f16   (DP = head_dim padded to 32;
//          Q pre-scaled by scale*log2(e) when the attention is unmasked)
//   v     [B*heads][npad/32][head_dim][hi 32 | lo 32] f16 (V^T per 32-key chunk,
//          keys in the order the P^T MFMA fragment holds them)
// Rows npad > N are written as zeros.
struct TflBufs {
    unsigned char *q, *k, *v;
};

// Work queue of the tfl launches: each workgroup claims its (utterance, tile)
// from the counter of the XCD it runs on (HW_REG_XCC_ID; utterance b's tiles
// sit in queue b % 8, so a layer's producer and consumer tiles of one
// utterance share an XCD and its L2), stealing from the other queues when its
// own is empty - correct for any placement.  cnt: kTflQueueWords zeroed
// words owned by the caller, two sets used by alternate launches (`seq`
// parity); a launch's workgroup 0 zeroes the other set for the next one.
// One stream per counter buffer.
constexpr int kTflQueueWords = 2 * 8 * 32;
struct TflQueue {
    unsigned* cnt = nullptr;
    unsigned seq = 0;
};

// True when the fused layer path covers (H, heads): heads == 2, H in {32, 64, 96}.
bool tfl_supported(int H, int heads);
// npad and the bytes of one TflBufs set for B utterances of N rows.
int tfl_npad(int N);
size_t tfl_bytes(int B, int N, int H, int heads);
void tfl_carve(unsigned char* base, int B, int N, int H, int heads, TflBufs* out);
// Final-projection widths the last decoder layer can fuse (mel channels).
bool tfl_proj_supported(int H, int NN);

// The first layer's LN1 -> QKV on 16-row tiles of each utterance, rows built
// by the launch itself (and stored to x_out, the residual input):
//   src 0: x_in rows;  1: embedding*scale + pe (+ padding mask);  2: the
//   length regulator's frame expansion of enc (cum = exclusive prefix sums).
struct TflFirst {
    int src = 0;
    const float* x_in = nullptr;
    const int64_t* ids = nullptr;
    const float *emb = nullptr, *pe = nullptr;
    int vocab = 0;
    float escale = 1.f;
    const int64_t* lengths = nullptr;  // embed: mask[b, s] = s < lengths[b] (mask may be null)
    uint8_t* mask = nullptr;
    const float* enc = nullptr;
    const int32_t* cum = nullptr;
    int S = 0;
    const int32_t* dN = nullptr;  // device frame count (dev_frames): N is then the capacity
    // with dN: [seq, T] posted to this host-mapped pair (T = max(1, *dN), also
    // past the capacity) so the host learns T without a copy or a stream sync
    int32_t* post = nullptr;
    int32_t post_seq = 0;
};
int32_t launch_tfl_first(const TflFirst& f, int B, int N, int H, int heads, bool masked, float* x_out,
                         const float* g, const float* bln, const float* Wqkv, const TflBufs& out, TflQueue q,
                         hipStream_t st);

// One pre-LN layer x_out = layer(x_in) (x_out may alias x_in), attention from
// `in`; then, on the same row tile: next == 1: the next layer's LN1 -> QKV
// into `out`; next == 2: LN(y; gn, bn) . Wn^T + bn2 into z [B*N][NN].
// masked: key padding mask from lengths (-1e9 fill, components.py:79-81).
struct TflLayer {
    const float *Wo, *bo, *g2, *b2n, *W1, *b1, *W2, *b2;  // packed (pack_bfrag_split) / fp32
    const float *gn = nullptr, *bn = nullptr, *Wn = nullptr, *bn2 = nullptr;
    // the layer's scores (log2 units) may leave the f16 range: the unmasked
    // head_dim-48 default form (f16 softmax base) gives way to the f32-base one
    bool wide_scores = false;
};
int32_t launch_tfl_layer(const TflLayer& w, int B, int N, int H, int heads, bool masked, const int64_t* lengths,
                         const float* x_in, float* x_out, const TflBufs& in, int next, const TflBufs& out,
                         int NN, float* z, TflQueue q, hipStream_t st, const int32_t* dN = nullptr);

}  // namespace m2
