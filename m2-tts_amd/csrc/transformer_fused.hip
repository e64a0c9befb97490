// Fused transformer-layer kernels (gfx950, exact-f32 MFMA v_mfma_f32_16x16x4_f32).
//
// One pre-LN layer (components.py:131-140) is three launches:
//   ln_qkv_kernel    qkv = LN1(x) . Wqkv^T                          (components.py:55-56,135)
//   attention_kernel (transformer.hip)
//   post_attn_kernel y = o + FFN(LN2(o)),  o = x + att . Wo^T + bo   (components.py:86-90,98-103,136-140)
// instead of five generic linears: the out-projection, LayerNorm, both FFN
// GEMMs and both residuals of a 32-row tile run out of LDS, so the only HBM
// traffic is att + x in and y out (12 B/row/channel instead of ~40).
//
// GEMM tiles: a workgroup (4 waves) owns 32 rows; wave w computes the
// 16-column blocks nb = w, w+4, ... for both 16-row halves.  A = activations
// from LDS (row stride K+2 floats: the 16 rows x 2 k-lanes of a ds_read_b32
// half-wave hit 32 distinct banks), B = weights packed in B-fragment order
// [n-block][k-step/4][lane][4] (one global_load_dwordx4 per lane per 4
// k-steps, L2-resident: every workgroup reads the same few tens of KB).
#include "m2_common.h"
#include "transformer_fused.h"

namespace m2 {
namespace tfx {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int TR = 32;  // rows per workgroup tile

// acc[rb] (rows rb*16.., cols nb*16..) += X[rows][0:K] . W[nb*16 + j][0:K]^T
// X: LDS rows of stride XS floats.  Wp: packed, this n-block, lane offset applied.
// An n-block's weight strip: K/4 floats per lane (float4 per 4 k-steps).
template <int K>
struct Strip {
    float4 w[K / 16];
    __device__ __forceinline__ void load(const float4* __restrict__ Wp, int nb) {
        const float4* p = Wp + (size_t)nb * (K / 16) * 64 + (threadIdx.x & 63);
#pragma unroll
        for (int s4 = 0; s4 < K / 16; ++s4) w[s4] = p[s4 * 64];
    }
};

template <int K, int XS>
__device__ __forceinline__ void gemm_strip(const float* X, const Strip<K>& st, f32x4 (&acc)[2]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const float* x0 = X + i * XS + g;
    const float* x1 = x0 + 16 * XS;
#pragma unroll
    for (int s4 = 0; s4 < K / 16; ++s4) {
        const float wv[4] = {st.w[s4].x, st.w[s4].y, st.w[s4].z, st.w[s4].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = (4 * s4 + q) * 4;
            acc[0] = mfma(x0[k], wv[q], acc[0]);
            acc[1] = mfma(x1[k], wv[q], acc[1]);
        }
    }
}

// Columns [nb*16, nb*16+16) of X . W^T for nb = wave, wave+4, ...: the next
// strip is requested before the current one is consumed (and the first one
// by the caller, before its LDS staging), so weight latency overlaps work.
// epi(nb, acc) consumes each finished block.
template <int K, int XS, int NB, typename Epi>
__device__ __forceinline__ void gemm_cols(const float* X, const float4* __restrict__ Wp, Strip<K>& cur,
                                          const float* __restrict__ bias, Epi epi) {
    const int wave = threadIdx.x >> 6, j = threadIdx.x & 15;
#pragma unroll 1
    for (int nb = wave; nb < NB; nb += 4) {
        Strip<K> nxt;
        if (nb + 4 < NB) nxt.load(Wp, nb + 4);
        f32x4 acc[2];
        const float bv = bias ? bias[nb * 16 + j] : 0.f;
        acc[0] = acc[1] = f32x4{bv, bv, bv, bv};
        gemm_strip<K, XS>(X, cur, acc);
        epi(nb, acc);
        if (nb + 4 < NB) cur = nxt;
    }
}

// LayerNorm of TR rows of H floats in LDS (src, stride SS) -> dst (stride DS):
// 8 lanes per row, two-pass mean / biased variance as nn.LayerNorm.
template <int H, int SS, int DS>
__device__ __forceinline__ void ln_rows(const float* src, float* dst, const float* __restrict__ g,
                                        const float* __restrict__ b) {
    const int row = threadIdx.x >> 3, part = threadIdx.x & 7;
    const float* xr = src + row * SS;
    float s = 0.f;
#pragma unroll
    for (int kk = 0; kk < H / 8; ++kk) s += xr[part + 8 * kk];
    s += __shfl_xor(s, 1);
    s += __shfl_xor(s, 2);
    s += __shfl_xor(s, 4);
    const float mean = s / (float)H;
    float v = 0.f;
#pragma unroll
    for (int kk = 0; kk < H / 8; ++kk) {
        const float d = xr[part + 8 * kk] - mean;
        v += d * d;
    }
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    const float rstd = 1.0f / sqrtf(v / (float)H + kLnEps);
    float* yr = dst + row * DS;
#pragma unroll
    for (int kk = 0; kk < H / 8; ++kk) {
        const int k = part + 8 * kk;
        yr[k] = (xr[k] - mean) * rstd * g[k] + b[k];
    }
}

// Global rows [r0, r0+TR) of width H (zero past R) -> LDS (stride S).
template <int H, int S>
__device__ __forceinline__ void load_rows(const float* __restrict__ x, int r0, int R, float* dst) {
    constexpr int H4 = H / 4;
    for (int i = threadIdx.x; i < TR * H4; i += 256) {
        const int r = i / H4, c = (i - r * H4) * 4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + r < R) v = *reinterpret_cast<const float4*>(x + (size_t)(r0 + r) * H + c);
        float* d = dst + r * S + c;
        d[0] = v.x;
        d[1] = v.y;
        d[2] = v.z;
        d[3] = v.w;
    }
}

// y[R][N] = act(LN?(x)[R][K] . W^T + b) for N % 16 == 0.
template <int K, int N, bool LN, int ACT>
__global__ __launch_bounds__(256) void ln_gemm_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                      const float* __restrict__ bln, const float4* __restrict__ Wp,
                                                      const float* __restrict__ bias, int R, float* __restrict__ y) {
    constexpr int XS = K + 2;
    __shared__ float X[TR * XS];
    __shared__ float Xn[LN ? TR * XS : 1];
    const int r0 = blockIdx.x * TR;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, gq = lane >> 4;
    Strip<K> st;
    if (wave < N / 16) st.load(Wp, wave);
    load_rows<K, XS>(x, r0, R, X);
    __syncthreads();
    const float* A = X;
    if (LN) {
        ln_rows<K, XS, XS>(X, Xn, g, bln);
        __syncthreads();
        A = Xn;
    }
    gemm_cols<K, XS, N / 16>(A, Wp, st, bias, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = r0 + rb * 16 + 4 * gq + r;
                if (row < R) y[(size_t)row * N + nb * 16 + j] = act_t<ACT>(acc[rb][r]);
            }
    });
}

// y = o + (relu(LN2(o) . W1^T + b1) . W2^T + b2),  o = x + att . Wo^T + bo.
// y may alias x (each tile reads its rows before writing them).
template <int H>
__global__ __launch_bounds__(256) void post_attn_kernel(const float* __restrict__ att, const float* x,
                                                        const float4* __restrict__ Wo, const float* __restrict__ bo,
                                                        const float* __restrict__ g2, const float* __restrict__ b2n,
                                                        const float4* __restrict__ W1, const float* __restrict__ b1,
                                                        const float4* __restrict__ W2, const float* __restrict__ b2,
                                                        int R, float* y) {
    constexpr int F = 2 * H, HS = H + 2, FS = F + 2;
    __shared__ float A[TR * HS];  // att tile, then LN2(o)
    __shared__ float O[TR * HS];  // o
    __shared__ float Hd[TR * FS]; // relu(FFN1)
    const int r0 = blockIdx.x * TR;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, j = lane & 15, gq = lane >> 4;
    Strip<H> so;
    if (wave < H / 16) so.load(Wo, wave);
    load_rows<H, HS>(att, r0, R, A);
    __syncthreads();
    // o = x + att . Wo^T + bo   (components.py:86, 137: x + dropout(attn(...)))
    gemm_cols<H, HS, H / 16>(A, Wo, so, bo, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rr = rb * 16 + 4 * gq + r, row = r0 + rr, col = nb * 16 + j;
                O[rr * HS + col] = row < R ? x[(size_t)row * H + col] + acc[rb][r] : 0.f;
            }
    });
    Strip<H> s1;
    s1.load(W1, wave);  // F/16 >= 4 blocks: every wave has one
    __syncthreads();
    ln_rows<H, HS, HS>(O, A, g2, b2n);
    __syncthreads();
    gemm_cols<H, HS, F / 16>(A, W1, s1, b1, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float v = acc[rb][r];
                Hd[(rb * 16 + 4 * gq + r) * FS + nb * 16 + j] = v > 0.f ? v : 0.f;
            }
    });
    Strip<F> s2;
    if (wave < H / 16) s2.load(W2, wave);
    __syncthreads();
    gemm_cols<F, FS, H / 16>(Hd, W2, s2, b2, [&](int nb, const f32x4 (&acc)[2]) {
#pragma unroll
        for (int rb = 0; rb < 2; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rr = rb * 16 + 4 * gq + r, row = r0 + rr, col = nb * 16 + j;
                if (row < R) y[(size_t)row * H + col] = O[rr * HS + col] + acc[rb][r];
            }
    });
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

int32_t launch_ln_gemm(const float* x, const float* g, const float* b, const float* Wp, const float* bias, int act,
                       int R, int K, int N, float* y, hipStream_t st) {
    if (R == 0) return M2_OK;
    const dim3 grid(cdiv(R, tfx::TR)), blk(256);
    const float4* W = reinterpret_cast<const float4*>(Wp);
#define M2_LNG(KK, NN)                                                                                           \
    if (K == KK && N == NN) {                                                                                    \
        if (g && act == ACT_NONE)                                                                                \
            hipLaunchKernelGGL((tfx::ln_gemm_kernel<KK, NN, true, ACT_NONE>), grid, blk, 0, st, x, g, b, W, bias, R, \
                               y);                                                                               \
        else                                                                                                     \
            return fail(M2_E_SHAPE, "ln_gemm: unsupported mode");                                               \
        M2_LAUNCHED("ln_gemm_kernel");                                                                           \
        return M2_OK;                                                                                            \
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

int32_t launch_post_attn(const float* att, const float* x, const float* Wo, const float* bo, const float* g2,
                         const float* b2n, const float* W1, const float* b1, const float* W2, const float* b2, int R,
                         int H, float* y, hipStream_t st) {
    if (R == 0) return M2_OK;
    const dim3 grid(cdiv(R, tfx::TR)), blk(256);
    auto f4 = [](const float* p) { return reinterpret_cast<const float4*>(p); };
    switch (H) {
        case 32: hipLaunchKernelGGL((tfx::post_attn_kernel<32>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n, f4(W1), b1, f4(W2), b2, R, y); break;
        case 64: hipLaunchKernelGGL((tfx::post_attn_kernel<64>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n, f4(W1), b1, f4(W2), b2, R, y); break;
        case 96: hipLaunchKernelGGL((tfx::post_attn_kernel<96>), grid, blk, 0, st, att, x, f4(Wo), bo, g2, b2n, f4(W1), b1, f4(W2), b2, R, y); break;
        default: return fail(M2_E_SHAPE, "post_attn: unsupported hidden_dim");
    }
    M2_LAUNCHED("post_attn_kernel");
    return M2_OK;
}

}  // namespace m2
