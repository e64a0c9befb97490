// Fused transformer-layer kernels (gfx950, split-f16 MFMA v_mfma_f32_16x16x32_f16).
//
// One pre-LN layer (components.py:131-140) is three launches:
//   ln_gemm_kernel   qkv = LN1(x) . Wqkv^T                          (components.py:55-56,135)
//   attention_split_kernel (transformer.hip)
//   post_attn_kernel y = o + FFN(LN2(o)),  o = x + att . Wo^T + bo   (components.py:86-90,98-103,136-140)
// instead of five generic linears: the out-projection, LayerNorm, both FFN
// GEMMs and both residuals of a 32-row tile run out of LDS, so the only HBM
// traffic is att + x in and y out (12 B/row/channel instead of ~40).
//
// Arithmetic: the vocoder's split-f16 form: every fp32 operand
// as hi = f16(x), lo = f16(x - hi), every product as hi*hi + hi*lo + lo*hi
// in one fp32 accumulator (~2^-22 relative per product); LayerNorms,
// residuals and biases stay fp32.  Weights are packed once at model creation
// (pack_bfrag_split), activations are split when they are written to LDS.
//
// GEMM tiles: a workgroup (NW = 4 or 8 waves, tf_waves) owns 32 rows; wave w
// computes the 16-column blocks nb = w, w+NW, ... for both 16-row halves, as the transposed
// product D^T = W . X^T: A = the weights (lane: 8 k of one output column,
// packed [n-block][k-step][hi|lo][lane][8 f16], one global_load_dwordx4 per
// lane and k-step, L2-resident), B = the activations from LDS hi / lo planes
// (lane: 8 k of one row, one ds_read_b128; row stride 4K + 32 B, RS/16 = 2
// mod 4: conflict-free).  A lane of D^T then holds 4 consecutive output
// columns of one row, so the epilogues write 16-B fp32 or 8-B f16 pieces.
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "m2_common.h"
#include "transformer_fused.h"
#include "vocoder_fused.h"  // split2u

namespace m2 {
namespace tfx {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef vx_u32x4 u32x4;

__device__ __forceinline__ f32x4 mfma_h(u32x4 a, u32x4 b, f32x4 c) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

constexpr int TR = 32;  // rows per workgroup tile

// Split activation rows in LDS: hi[K] f16, lo[K] f16, pad.
constexpr int srs(int K) { return 4 * K + 32; }
// fp32 rows in LDS (16-B aligned rows).
constexpr int frs(int K) { return K + 4; }

// An n-block's weight strip: hi and lo fragments of its K/32 k-steps.
template <int K>
struct Strip {
    u32x4 w[K / 32][2];
    __device__ __forceinline__ void load(const u32x4* __restrict__ Wp, int nb) {
        const u32x4* p = Wp + (size_t)nb * (K / 32) * 128 + (threadIdx.x & 63);
#pragma unroll
        for (int ks = 0; ks < K / 32; ++ks) {
            w[ks][0] = p[ks * 128];
            w[ks][1] = p[ks * 128 + 64];
        }
    }
};

// acc[rb] (transposed: lane = row rb*16 + (lane&15), columns nb*16 + 4g + r)
// += W[nb cols][0:K] . X[rows][0:K]^T, X = split LDS rows (stride srs(K)).
template <int K>
__device__ __forceinline__ void gemm_strip(const unsigned char* X, const Strip<K>& st, f32x4 (&acc)[2]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
        u32x4 xh[2], xl[2];
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const unsigned char* p = X + (rb * 16 + i) * srs(K) + 2 * (32 * ks + 8 * g);
            xh[rb] = *reinterpret_cast<const u32x4*>(p);
            xl[rb] = *reinterpret_cast<const u32x4*>(p + 2 * K);
        }
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) acc[rb] = mfma_h(st.w[ks][0], xh[rb], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) acc[rb] = mfma_h(st.w[ks][0], xl[rb], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) acc[rb] = mfma_h(st.w[ks][1], xh[rb], acc[rb]);
    }
}

// Columns [nb*16, nb*16+16) of X . W^T for nb = wave, wave+NW, ...: the next
// strip is requested before the current one is consumed (and the first one
// by the caller, before its LDS staging), so weight latency overlaps work.
// epi(nb, acc) consumes each finished block (lane: row rb*16 + (lane&15),
// columns nb*16 + 4*(lane>>4) + r).
template <int K, int NB, int NW, typename Epi>
__device__ __forceinline__ void gemm_cols(const unsigned char* X, const u32x4* __restrict__ Wp, Strip<K>& cur,
                                          const float* __restrict__ bias, Epi epi) {
    const int wave = threadIdx.x >> 6, g = (threadIdx.x & 63) >> 4;
#pragma unroll 1
    for (int nb = wave; nb < NB; nb += NW) {
        Strip<K> nxt;
        if (nb + NW < NB) nxt.load(Wp, nb + NW);
        f32x4 acc[2];
        f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
        if (bias) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[r] = bias[nb * 16 + 4 * g + r];
        }
        acc[0] = acc[1] = bv;
        gemm_strip<K>(X, cur, acc);
        epi(nb, acc);
        if (nb + NW < NB) cur = nxt;
    }
}

// Four consecutive fp32 values -> their hi and lo f16 at p, p + 2K.
template <int K>
__device__ __forceinline__ void put_split4(unsigned char* p, float a, float b, float c, float d) {
    unsigned h0, h1, l0, l1;
    split2u(a, b, h0, l0);
    split2u(c, d, h1, l1);
    *reinterpret_cast<uint2*>(p) = uint2{h0, h1};
    *reinterpret_cast<uint2*>(p + 2 * K) = uint2{l0, l1};
}

// LayerNorm of TR rows of H floats in LDS (src, stride frs(H)) -> split rows
// (dst, stride srs(H)): 8 lanes per row, each H/8 consecutive channels;
// two-pass mean / biased variance as nn.LayerNorm.  Threads 0-255 only (an
// 8-wave workgroup's upper half skips it).
template <int H>
__device__ __forceinline__ void ln_rows(const float* src, unsigned char* dst, const float* __restrict__ g,
                                        const float* __restrict__ b) {
    constexpr int PER = H / 8;
    static_assert(PER % 4 == 0, "H multiple of 32");
    if (threadIdx.x >= 8 * TR) return;
    const int row = threadIdx.x >> 3, part = threadIdx.x & 7;
    const float* xr = src + row * frs(H) + part * PER;
    float v[PER];
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const float4 t = *reinterpret_cast<const float4*>(xr + 4 * q);
        v[4 * q] = t.x;
        v[4 * q + 1] = t.y;
        v[4 * q + 2] = t.z;
        v[4 * q + 3] = t.w;
    }
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) s += v[k];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    const float mean = s / (float)H;
    float var = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const float d = v[k] - mean;
        var += d * d;
    }
    var += __shfl_xor(var, 1);
    var += __shfl_xor(var, 2);
    var += __shfl_xor(var, 4);
    const float rstd = 1.0f / sqrtf(var / (float)H + kLnEps);
    unsigned char* yr = dst + row * srs(H) + 2 * part * PER;
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        float y[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = part * PER + 4 * q + e;
            y[e] = (v[4 * q + e] - mean) * rstd * g[k] + b[k];
        }
        put_split4<H>(yr + 8 * q, y[0], y[1], y[2], y[3]);
    }
}

// Global rows [r0, r0+TR) of width H (zero past R) -> LDS fp32 rows (stride frs(H)).
template <int H>
__device__ __forceinline__ void load_rows(const float* __restrict__ x, int r0, int R, float* dst) {
    constexpr int H4 = H / 4;
    for (int i = threadIdx.x; i < TR * H4; i += blockDim.x) {
        const int r = i / H4, c = (i - r * H4) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + r < R) v = *reinterpret_cast<const float4*>(x + (size_t)(r0 + r) * H + c);
        *reinterpret_cast<float4*>(dst + r * frs(H) + c) = v;
    }
}
// ... -> LDS split rows (stride srs(H)).
template <int H>
__device__ __forceinline__ void load_rows_split(const float* __restrict__ x, int r0, int R, unsigned char* dst) {
    constexpr int H4 = H / 4;
    for (int i = threadIdx.x; i < TR * H4; i += blockDim.x) {
        const int r = i / H4, c = (i - r * H4) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + r < R) v = *reinterpret_cast<const float4*>(x + (size_t)(r0 + r) * H + c);
        put_split4<H>(dst + r * srs(H) + 2 * c, v.x, v.y, v.z, v.w);
    }
}

// Where ln_gemm_kernel's rows come from.  SRC_X: x.  The first layer of a
// stack can build its input rows itself, one launch fewer per stack (the rows
// are also stored to xo, the layer's residual input, so the values are the
// ones the separate launch would have written):
//   SRC_EMBED   x = E[ids] * sqrt(H) + pe[s] and the padding mask (embed_pe_kernel)
//   SRC_EXPAND  x = enc row of the phoneme frame t falls in, zero past the
//               utterance's total (lr_expand_kernel's search)
enum { SRC_X = 0, SRC_EMBED = 1, SRC_EXPAND = 2 };
struct RowSrc {
    const int64_t* ids = nullptr;  // embed: [R] token ids, S positions per utterance
    const float* emb = nullptr;
    const float* pe = nullptr;
    int vocab = 0;
    float scale = 1.f;
    const int64_t* lengths = nullptr;  // optional: mask[r] = s < lengths[b]
    uint8_t* mask = nullptr;
    const float* enc = nullptr;  // expand: [B][S][H] encoder output, cum [B][S + 1]
    const int32_t* cum = nullptr;
    int S = 1, T = 1;
    float* xo = nullptr;
};

template <int H, int SRC>
__device__ __forceinline__ void load_src_rows(const float* __restrict__ x, const RowSrc& src, int r0, int R,
                                              float* dst, int* sp) {
    constexpr int H4 = H / 4;
    if constexpr (SRC == SRC_X) {
        load_rows<H>(x, r0, R, dst);
    } else {
        if constexpr (SRC == SRC_EXPAND) {
            // source phoneme of each of the tile's frames: smallest s with cum[s+1] > t
            if (threadIdx.x < TR) {
                const int row = r0 + threadIdx.x;
                int v = -1;
                if (row < R) {
                    const int b = row / src.T, t = row - b * src.T;
                    const int32_t* c = src.cum + (size_t)b * (src.S + 1);
                    if (t < c[src.S]) {
                        int lo = 0, hi = src.S - 1;
                        while (lo < hi) {
                            const int mid = (lo + hi) >> 1;
                            if (c[mid + 1] > t) hi = mid;
                            else lo = mid + 1;
                        }
                        v = b * src.S + lo;
                    }
                }
                sp[threadIdx.x] = v;
            }
            __syncthreads();
        }
        for (int i = threadIdx.x; i < TR * H4; i += blockDim.x) {
            const int r = i / H4, c = (i - r * H4) * 4, row = r0 + r;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (row < R) {
                if constexpr (SRC == SRC_EMBED) {
                    const int64_t id = src.ids[row];
                    const int s = row % src.S;
                    float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (id >= 0 && id < src.vocab) e = *reinterpret_cast<const float4*>(src.emb + id * H + c);
                    const float4 p = *reinterpret_cast<const float4*>(src.pe + (size_t)s * H + c);
                    v = make_float4(__builtin_fmaf(e.x, src.scale, p.x), __builtin_fmaf(e.y, src.scale, p.y),
                                    __builtin_fmaf(e.z, src.scale, p.z), __builtin_fmaf(e.w, src.scale, p.w));
                    if (src.lengths && c == 0) src.mask[row] = (int64_t)s < src.lengths[row / src.S] ? 1 : 0;
                } else {
                    const int q = sp[r];
                    if (q >= 0) v = *reinterpret_cast<const float4*>(src.enc + (size_t)q * H + c);
                }
                *reinterpret_cast<float4*>(src.xo + (size_t)row * H + c) = v;
            }
            *reinterpret_cast<float4*>(dst + r * frs(H) + c) = v;
        }
    }
}

// y[R][N] = act(LN?(x)[R][K] . W^T + b) for N % 16 == 0; x from SRC (above).
template <int K, int N, bool LN, int ACT, int NW = 4, int SRC = SRC_X>
__global__ __launch_bounds__(64 * NW) void ln_gemm_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                      const float* __restrict__ bln, const u32x4* __restrict__ Wp,
                                                      const float* __restrict__ bias, int R, float* __restrict__ y,
                                                      RowSrc src = RowSrc{}) {
    static_assert(LN, "ln_gemm: LN form only");
    __shared__ __attribute__((aligned(16))) float X[TR * frs(K)];
    __shared__ __attribute__((aligned(16))) unsigned char Xn[TR * srs(K)];
    __shared__ int sp[SRC == SRC_EXPAND ? TR : 1];
    const int r0 = blockIdx.x * TR;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    Strip<K> st;
    if (wave < N / 16) st.load(Wp, wave);
    load_src_rows<K, SRC>(x, src, r0, R, X, sp);
    __syncthreads();
    ln_rows<K>(X, Xn, g, bln);
    __syncthreads();
    gemm_cols<K, N / 16, NW>(Xn, Wp, st, bias, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int row = r0 + rb * 16 + i;
            if (row < R) {
                f32x4 v;
#pragma unroll
                for (int r = 0; r < 4; ++r) v[r] = act_t<ACT>(acc[rb][r]);
                *reinterpret_cast<f32x4*>(y + (size_t)row * N + nb * 16 + 4 * gq) = v;
            }
        }
    });
}

// y = o + (relu(LN2(o) . W1^T + b1) . W2^T + b2),  o = x + att . Wo^T + bo.
// y may alias x (each tile reads its rows before writing them).
// NN > 0: the next launch's row-local LN + GEMM runs on the tile too,
// z = LN(y; gn, bn) . Wn^T (+ bn2) with NN output columns - the next layer's
// LN1 -> QKV, or the decoder's final LN -> mel projection - so y is read back
// from LDS instead of HBM and one launch per layer goes away.
template <int H, int NN = 0, int NW = 4>
__global__ __launch_bounds__(64 * NW) void post_attn_kernel(const float* __restrict__ att, const float* x,
                                                        const u32x4* __restrict__ Wo, const float* __restrict__ bo,
                                                        const float* __restrict__ g2, const float* __restrict__ b2n,
                                                        const u32x4* __restrict__ W1, const float* __restrict__ b1,
                                                        const u32x4* __restrict__ W2, const float* __restrict__ b2,
                                                        int R, float* y, const float* __restrict__ gn = nullptr,
                                                        const float* __restrict__ bn = nullptr,
                                                        const u32x4* __restrict__ Wn = nullptr,
                                                        const float* __restrict__ bn2 = nullptr,
                                                        float* __restrict__ z = nullptr) {
    constexpr int F = 2 * H;
    __shared__ __attribute__((aligned(16))) unsigned char A[TR * srs(H)];   // att tile, then LN2(o) (split)
    __shared__ __attribute__((aligned(16))) float O[TR * frs(H)];           // o (fp32)
    __shared__ __attribute__((aligned(16))) unsigned char Hd[TR * srs(F)];  // relu(FFN1) (split)
    const int r0 = blockIdx.x * TR;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    Strip<H> so;
    if (wave < H / 16) so.load(Wo, wave);
    load_rows_split<H>(att, r0, R, A);
    __syncthreads();
    // o = x + att . Wo^T + bo   (components.py:86, 137: x + dropout(attn(...)))
    gemm_cols<H, H / 16, NW>(A, Wo, so, bo, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int rr = rb * 16 + i, row = r0 + rr, col = nb * 16 + 4 * gq;
            f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
            if (row < R) o = *reinterpret_cast<const f32x4*>(x + (size_t)row * H + col) + acc[rb];
            *reinterpret_cast<f32x4*>(O + rr * frs(H) + col) = o;
        }
    });
    Strip<H> s1;
    if (wave < F / 16) s1.load(W1, wave);
    __syncthreads();
    ln_rows<H>(O, A, g2, b2n);
    __syncthreads();
    gemm_cols<H, F / 16, NW>(A, W1, s1, b1, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const f32x4 v = acc[rb];
            put_split4<F>(Hd + (rb * 16 + i) * srs(F) + 2 * (nb * 16 + 4 * gq), v[0] > 0.f ? v[0] : 0.f,
                          v[1] > 0.f ? v[1] : 0.f, v[2] > 0.f ? v[2] : 0.f, v[3] > 0.f ? v[3] : 0.f);
        }
    });
    Strip<F> s2;
    if (wave < H / 16) s2.load(W2, wave);
    __syncthreads();
    gemm_cols<F, H / 16, NW>(Hd, W2, s2, b2, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb) {
            const int rr = rb * 16 + i, row = r0 + rr, col = nb * 16 + 4 * gq;
            const f32x4 v = *reinterpret_cast<const f32x4*>(O + rr * frs(H) + col) + acc[rb];
            if (row < R) *reinterpret_cast<f32x4*>(y + (size_t)row * H + col) = v;
            if constexpr (NN > 0) *reinterpret_cast<f32x4*>(O + rr * frs(H) + col) = v;  // y kept for the next LN
        }
    });
    if constexpr (NN > 0) {
        Strip<H> sn;
        if (wave < NN / 16) sn.load(Wn, wave);
        __syncthreads();
        ln_rows<H>(O, A, gn, bn);  // same rounding as ln_gemm_kernel's
        __syncthreads();
        gemm_cols<H, NN / 16, NW>(A, Wn, sn, bn2, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
            for (int rb = 0; rb < 2; ++rb) {
                const int row = r0 + rb * 16 + i;
                if (row < R) *reinterpret_cast<f32x4*>(z + (size_t)row * NN + nb * 16 + 4 * gq) = acc[rb];
            }
        });
    }
}

}  // namespace tfx

bool tf_fused_supported(int H, int N_out) {
    return (H == 32 || H == 64 || H == 96) && N_out % 16 == 0;
}

// B-fragment packing for v_mfma_f32_16x16x4_f32: element (n-block nb, k-step
// s, lane) = W[nb*16 + (lane&15)][4*s + (lane>>4)], layout [nb][s/4][lane][s%4].
std::vector<float> pack_bfrag(const float* W, int N, int K) {
    std::vector<float> out((size_t)N * K, 0.f);
    const int KS = K / 4;
    for (int nb = 0; nb < N / 16; ++nb)
        for (int s = 0; s < KS; ++s)
            for (int lane = 0; lane < 64; ++lane) {
                const int n = nb * 16 + (lane & 15), k = 4 * s + (lane >> 4);
                out[(((size_t)nb * (KS / 4) + s / 4) * 64 + lane) * 4 + (s % 4)] = W[(size_t)n * K + k];
            }
    return out;
}

// Split-f16 A-fragment packing for the fused layers' v_mfma_f32_16x16x32_f16
// (D^T = W . X^T): element (n-block nb, k-step ks, half, lane, e) =
// half(W[nb*16 + (lane&15)][32*ks + 8*(lane>>4) + e]), layout
// [nb][ks][hi|lo][lane][8 f16] - as many bytes as W in fp32.  False if a
// weight is outside the f16 range (the caller then keeps the fp32 layers).
bool pack_bfrag_split(const float* W, int N, int K, std::vector<float>* out) {
    out->assign((size_t)N * K, 0.f);
    uint16_t* o = reinterpret_cast<uint16_t*>(out->data());
    const int KS = K / 32;
    for (int nb = 0; nb < N / 16; ++nb)
        for (int ks = 0; ks < KS; ++ks)
            for (int lane = 0; lane < 64; ++lane)
                for (int e = 0; e < 8; ++e) {
                    const float v = W[(size_t)(nb * 16 + (lane & 15)) * K + 32 * ks + 8 * (lane >> 4) + e];
                    if (!(std::fabs(v) < 65504.f)) return false;
                    const _Float16 h = (_Float16)v, l = (_Float16)(v - (float)h);
                    const size_t base = (((size_t)nb * KS + ks) * 2 * 64 + lane) * 8 + e;
                    std::memcpy(&o[base], &h, 2);
                    std::memcpy(&o[base + 64 * 8], &l, 2);
                }
    return true;
}

// Waves per workgroup: 8 when the grid is short of two workgroups per CU
// (small batches: every 32-row tile is then a serial chain of GEMM rounds, and
// 8 waves halve the rounds: post_attn at stage2 B=8 S=100 13.8 -> 10.5 us,
// tools/probe/tf_waves_ab.sh), else 4.  M2_TF_WAVES=4|8 forces one.  (An L2
// warm-up of the layer's weights at kernel start measured 1 us slower: across
// steps they stay L2-resident.)
static int tf_waves(int R) {
    const int forced = sw().tf_waves;
    if (forced) return forced;
    return cdiv(R, tfx::TR) < 2 * 256 ? 8 : 4;
}

int32_t launch_ln_gemm(const float* x, const float* g, const float* b, const float* Wp, const float* bias, int act,
                       int R, int K, int N, float* y, hipStream_t st) {
    if (R == 0) return M2_OK;
    const int nw = tf_waves(R);
    const dim3 grid(cdiv(R, tfx::TR)), blk(64 * nw);
    const vx_u32x4* W = reinterpret_cast<const vx_u32x4*>(Wp);
#define M2_LNG(KK, NN)                                                                                             \
    if (K == KK && N == NN) {                                                                                      \
        if (!g || act != ACT_NONE) return fail(M2_E_SHAPE, "ln_gemm: unsupported mode");                          \
        if (nw == 8)                                                                                               \
            hipLaunchKernelGGL((tfx::ln_gemm_kernel<KK, NN, true, ACT_NONE, 8>), grid, blk, 0, st, x, g, b, W, bias, \
                               R, y);                                                                              \
        else                                                                                                       \
            hipLaunchKernelGGL((tfx::ln_gemm_kernel<KK, NN, true, ACT_NONE, 4>), grid, blk, 0, st, x, g, b, W, bias, \
                               R, y);                                                                              \
        M2_LAUNCHED("ln_gemm_kernel");                                                                             \
        return M2_OK;                                                                                              \
    }
    M2_LNG(32, 96)
    M2_LNG(32, 32)
    M2_LNG(64, 192)
    M2_LNG(64, 64)
    M2_LNG(96, 288)
    M2_LNG(96, 80)
    M2_LNG(32, 64)
    M2_LNG(96, 96)
    M2_LNG(64, 80)
#undef M2_LNG
    return fail(M2_E_SHAPE, "ln_gemm: unsupported (K, N)");
}

// The first layer's LN1 -> QKV on rows it builds itself (SRC_EMBED / SRC_EXPAND).
static int32_t launch_src_ln_gemm(int srcmode, const tfx::RowSrc& src, const float* g, const float* b,
                                  const float* Wp, int R, int K, int N, float* y, hipStream_t st) {
    if (R == 0) return M2_OK;
    const int nw = tf_waves(R);
    const dim3 grid(cdiv(R, tfx::TR)), blk(64 * nw);
    const vx_u32x4* W = reinterpret_cast<const vx_u32x4*>(Wp);
#define M2_SLG(KK, NN, SS)                                                                                        \
    if (K == KK && N == NN && srcmode == SS) {                                                                    \
        if (nw == 8)                                                                                              \
            hipLaunchKernelGGL((tfx::ln_gemm_kernel<KK, NN, true, ACT_NONE, 8, SS>), grid, blk, 0, st, nullptr, g, \
                               b, W, nullptr, R, y, src);                                                         \
        else                                                                                                      \
            hipLaunchKernelGGL((tfx::ln_gemm_kernel<KK, NN, true, ACT_NONE, 4, SS>), grid, blk, 0, st, nullptr, g, \
                               b, W, nullptr, R, y, src);                                                         \
        M2_LAUNCHED("ln_gemm_kernel");                                                                            \
        return M2_OK;                                                                                             \
    }
    M2_SLG(32, 96, tfx::SRC_EMBED)
    M2_SLG(64, 192, tfx::SRC_EMBED)
    M2_SLG(96, 288, tfx::SRC_EMBED)
    M2_SLG(32, 96, tfx::SRC_EXPAND)
    M2_SLG(64, 192, tfx::SRC_EXPAND)
    M2_SLG(96, 288, tfx::SRC_EXPAND)
#undef M2_SLG
    return fail(M2_E_SHAPE, "ln_gemm: unsupported (K, N) for a fused row source");
}

bool tf_src_fused_supported(int H, int N) { return (H == 32 && N == 96) || (H == 64 && N == 192) || (H == 96 && N == 288); }

int32_t launch_embed_ln_gemm(const int64_t* ids, const float* emb, const float* pe, int B, int S, int H, int vocab,
                             const int64_t* lengths, uint8_t* mask, float* x, const float* g, const float* b,
                             const float* Wp, int N, float* y, hipStream_t st) {
    tfx::RowSrc src;
    src.ids = ids;
    src.emb = emb;
    src.pe = pe;
    src.vocab = vocab;
    src.scale = (float)std::sqrt((double)H);  // as launch_embed_pe
    src.lengths = lengths;
    src.mask = mask;
    src.S = S;
    src.xo = x;
    return launch_src_ln_gemm(tfx::SRC_EMBED, src, g, b, Wp, B * S, H, N, y, st);
}

int32_t launch_expand_ln_gemm(const float* enc, const int32_t* cum, int B, int S, int T, int H, float* x,
                              const float* g, const float* b, const float* Wp, int N, float* y, hipStream_t st) {
    tfx::RowSrc src;
    src.enc = enc;
    src.cum = cum;
    src.S = S;
    src.T = T;
    src.xo = x;
    return launch_src_ln_gemm(tfx::SRC_EXPAND, src, g, b, Wp, B * T, H, N, y, st);
}

int32_t launch_post_attn(const float* att, const float* x, const float* Wo, const float* bo, const float* g2,
                         const float* b2n, const float* W1, const float* b1, const float* W2, const float* b2, int R,
                         int H, float* y, hipStream_t st) {
    if (R == 0) return M2_OK;
    const int nw = tf_waves(R);
    const dim3 grid(cdiv(R, tfx::TR)), blk(64 * nw);
    auto f4 = [](const float* p) { return reinterpret_cast<const vx_u32x4*>(p); };
#define M2_PA(HH)                                                                                                   \
    case HH:                                                                                                        \
        if (nw == 8)                                                                                                \
            hipLaunchKernelGGL((tfx::post_attn_kernel<HH, 0, 8>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n,    \
                               f4(W1), b1, f4(W2), b2, R, y);                                                       \
        else                                                                                                        \
            hipLaunchKernelGGL((tfx::post_attn_kernel<HH, 0, 4>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n,    \
                               f4(W1), b1, f4(W2), b2, R, y);                                                       \
        break;
    switch (H) {
        M2_PA(32)
        M2_PA(64)
        M2_PA(96)
        default: return fail(M2_E_SHAPE, "post_attn: unsupported hidden_dim");
    }
#undef M2_PA
    M2_LAUNCHED("post_attn_kernel");
    return M2_OK;
}

bool tf_post_next_supported(int H, int NN) {
    return (H == 32 && (NN == 96 || NN == 32 || NN == 64)) || (H == 64 && (NN == 192 || NN == 64 || NN == 80)) ||
           (H == 96 && (NN == 288 || NN == 80 || NN == 96));
}

int32_t launch_post_attn_next(const float* att, const float* x, const float* Wo, const float* bo, const float* g2,
                              const float* b2n, const float* W1, const float* b1, const float* W2, const float* b2,
                              int R, int H, float* y, const float* gn, const float* bn, const float* Wn,
                              const float* bn2, int NN, float* z, hipStream_t st) {
    if (R == 0) return M2_OK;
    const int nw = tf_waves(R);
    const dim3 grid(cdiv(R, tfx::TR)), blk(64 * nw);
    auto f4 = [](const float* p) { return reinterpret_cast<const vx_u32x4*>(p); };
#define M2_PAN(HH, NNN)                                                                                              \
    if (H == HH && NN == NNN) {                                                                                      \
        if (nw == 8)                                                                                                 \
            hipLaunchKernelGGL((tfx::post_attn_kernel<HH, NNN, 8>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n,   \
                               f4(W1), b1, f4(W2), b2, R, y, gn, bn, f4(Wn), bn2, z);                                \
        else                                                                                                         \
            hipLaunchKernelGGL((tfx::post_attn_kernel<HH, NNN, 4>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n,   \
                               f4(W1), b1, f4(W2), b2, R, y, gn, bn, f4(Wn), bn2, z);                                \
        M2_LAUNCHED("post_attn_kernel");                                                                             \
        return M2_OK;                                                                                                \
    }
    M2_PAN(32, 96)
    M2_PAN(32, 32)
    M2_PAN(32, 64)
    M2_PAN(64, 192)
    M2_PAN(64, 64)
    M2_PAN(64, 80)
    M2_PAN(96, 288)
    M2_PAN(96, 80)
    M2_PAN(96, 96)
#undef M2_PAN
    return fail(M2_E_SHAPE, "post_attn: unsupported (hidden_dim, next width)");
}

}  // namespace m2
