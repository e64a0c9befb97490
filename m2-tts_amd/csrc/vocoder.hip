// SimpleVocoder kernels (gfx950), per-layer form.
//
//   conv_kernel    Conv1d(k=3 or 1, pad=k/2) + bias [* alpha + beta] [+ act] [+ residual]
//                  input_conv / resblock conv1,conv2 / output_conv
//                  tts_model.py:246,272,287,295; components.py:196-200
//   convT_kernel   ConvTranspose1d(c, c/2, k=2r, s=r, p=r/2) + bias + leaky(0.1)
//                  tts_model.py:255-263,291
//
// Layout [B][C][L], time contiguous: lanes own consecutive time steps so every
// activation load/store is coalesced along T; the weights for the workgroup's
// output channels are wave-uniform (scalar loads, SGPR operands of v_fma).
//
// ConvT as a 2-tap polyphase: with p = r/2, output t = q*r + ph reads exactly
// two input frames,
//     ph + p <  r :  x[q]  * W[ph+p]    + x[q-1] * W[ph+p+r]
//     ph + p >= r :  x[q+1]* W[ph+p-r]  + x[q]   * W[ph+p]
// which is y[co,t] = b[co] + sum_ci sum_{i: k=t+p-i*r in [0,2r)} x[ci,i] W[ci,co,k].
#include <climits>

#include "m2_common.h"

namespace m2 {

template <int KS, int CO_T, int TT, bool RES, bool XT>
__global__ __launch_bounds__(256) void conv_kernel(const float* __restrict__ x,
                                                   const float* __restrict__ w,
                                                   const float* __restrict__ bias,
                                                   const float* __restrict__ alpha,
                                                   const float* __restrict__ beta,
                                                   const float* __restrict__ res, int Cin,
                                                   int Cout, int L, int act,
                                                   float* __restrict__ y) {
    constexpr int PAD = KS / 2;
    const int b = blockIdx.z, co0 = blockIdx.y * CO_T;
    const int t0 = (blockIdx.x * 256 + threadIdx.x) * TT;
    if (t0 >= L) return;
    const float* xb = x + (size_t)b * Cin * L;
    float acc[CO_T][TT];
#pragma unroll
    for (int c = 0; c < CO_T; ++c)
#pragma unroll
        for (int i = 0; i < TT; ++i) acc[c][i] = 0.f;

    for (int ci = 0; ci < Cin; ++ci) {
        float xv[TT + KS - 1];
#pragma unroll
        for (int i = 0; i < TT + KS - 1; ++i) {
            const int t = t0 - PAD + i;
            const bool in = t >= 0 && t < L;
            const size_t off = XT ? (size_t)t * Cin + ci : (size_t)ci * L + t;
            xv[i] = in ? xb[off] : 0.f;
        }
#pragma unroll
        for (int c = 0; c < CO_T; ++c) {
            const float* wr = w + ((size_t)(co0 + c) * Cin + ci) * KS;
            float wk[KS];
#pragma unroll
            for (int k = 0; k < KS; ++k) wk[k] = wr[k];
#pragma unroll
            for (int i = 0; i < TT; ++i) {
                float a = acc[c][i];
#pragma unroll
                for (int k = 0; k < KS; ++k) a = fmaf(wk[k], xv[i + k], a);
                acc[c][i] = a;
            }
        }
    }
#pragma unroll
    for (int c = 0; c < CO_T; ++c) {
        const int co = co0 + c;
        const float bv = bias[co];
        const float al = alpha ? alpha[co] : 1.f, be = alpha ? beta[co] : 0.f;
        const size_t rowo = ((size_t)b * Cout + co) * L;
#pragma unroll
        for (int i = 0; i < TT; ++i) {
            const int t = t0 + i;
            if (t < L) {
                float v = acc[c][i] + bv;
                if (alpha) v = v * al + be;
                v = apply_act(v, act);
                if (RES) v = v + res[rowo + t];
                y[rowo + t] = v;
            }
        }
    }
}

template <int R, int CO_T, int TQ>
__global__ __launch_bounds__(256) void convT_kernel(const float* __restrict__ x,
                                                    const float* __restrict__ w,
                                                    const float* __restrict__ bias, int Cin,
                                                    int Cout, int L, int act,
                                                    float* __restrict__ y) {
    constexpr int P = R / 2;
    const int b = blockIdx.z, co0 = blockIdx.y * CO_T;
    const int q0 = (blockIdx.x * 256 + threadIdx.x) * TQ;
    if (q0 >= L) return;
    const float* xb = x + (size_t)b * Cin * L;
    float acc[CO_T][TQ * R];
#pragma unroll
    for (int c = 0; c < CO_T; ++c)
#pragma unroll
        for (int i = 0; i < TQ * R; ++i) acc[c][i] = 0.f;

    for (int ci = 0; ci < Cin; ++ci) {
        float xv[TQ + 2];  // x[q0-1 .. q0+TQ]
#pragma unroll
        for (int i = 0; i < TQ + 2; ++i) {
            const int q = q0 - 1 + i;
            xv[i] = (q >= 0 && q < L) ? xb[(size_t)ci * L + q] : 0.f;
        }
#pragma unroll
        for (int c = 0; c < CO_T; ++c) {
            const float* wr = w + ((size_t)ci * Cout + co0 + c) * (2 * R);
            float wk[2 * R];
#pragma unroll
            for (int k = 0; k < 2 * R; ++k) wk[k] = wr[k];
#pragma unroll
            for (int qq = 0; qq < TQ; ++qq) {
#pragma unroll
                for (int ph = 0; ph < R; ++ph) {
                    float a = acc[c][qq * R + ph];
                    if (ph + P < R) {
                        a = fmaf(xv[qq + 1], wk[ph + P], a);
                        a = fmaf(xv[qq], wk[ph + P + R], a);
                    } else {
                        a = fmaf(xv[qq + 2], wk[ph + P - R], a);
                        a = fmaf(xv[qq + 1], wk[ph + P], a);
                    }
                    acc[c][qq * R + ph] = a;
                }
            }
        }
    }
    const int Lo = L * R;
#pragma unroll
    for (int c = 0; c < CO_T; ++c) {
        const int co = co0 + c;
        const float bv = bias[co];
        float* yr = y + ((size_t)b * Cout + co) * Lo;
#pragma unroll
        for (int qq = 0; qq < TQ; ++qq) {
            if (q0 + qq < L) {
#pragma unroll
                for (int ph = 0; ph < R; ++ph) yr[(q0 + qq) * R + ph] = apply_act(acc[c][qq * R + ph] + bv, act);
            }
        }
    }
}

// Conv1d with any kernel size, dilation and zero padding (the standalone
// components' general forms: LightweightResBlock(kernel_size, dilation),
// ConvBlock(kernel_size), SimpleVocoder(kernel_size), components.py:143-200,
// tts_model.py:246,272): y[co, t] = b[co] + sum_ci sum_j w[co, ci, j] *
// x[ci, t - pad + j * dil], t < Lo = L + 2 pad - dil (K - 1), then the same
// optional affine / activation / residual as conv_kernel.  Lanes own
// consecutive output steps (coalesced along T), weights are wave-uniform.
template <int CO_T>
__global__ __launch_bounds__(256) void conv_general_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ bias,
                                                           const float* __restrict__ alpha,
                                                           const float* __restrict__ beta,
                                                           const float* __restrict__ res, int Cin, int Cout, int L,
                                                           int Lo, int K, int dil, int pad, int act,
                                                           float* __restrict__ y) {
    const int b = blockIdx.z, co0 = blockIdx.y * CO_T;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= Lo) return;
    const float* xb = x + (size_t)b * Cin * L;
    float acc[CO_T];
#pragma unroll
    for (int c = 0; c < CO_T; ++c) acc[c] = 0.f;
    for (int ci = 0; ci < Cin; ++ci) {
        const float* xr = xb + (size_t)ci * L;
        for (int j = 0; j < K; ++j) {
            const int ti = t - pad + j * dil;
            const float xv = (ti >= 0 && ti < L) ? xr[ti] : 0.f;
#pragma unroll
            for (int c = 0; c < CO_T; ++c) acc[c] = fmaf(w[((size_t)(co0 + c) * Cin + ci) * K + j], xv, acc[c]);
        }
    }
#pragma unroll
    for (int c = 0; c < CO_T; ++c) {
        const int co = co0 + c;
        float v = acc[c] + bias[co];
        if (alpha) v = v * alpha[co] + beta[co];
        v = apply_act(v, act);
        const size_t o = ((size_t)b * Cout + co) * Lo + t;
        if (res) v = v + res[o];
        y[o] = v;
    }
}

// ---------------------------------------------------------------------------
namespace {
constexpr int kConvTT = 4;
constexpr int kConvTQ = 2;

template <int KS, int CO_T>
int32_t conv_dispatch(const float* x, const float* w, const float* b, const float* alpha,
                      const float* beta, const float* res, int act, bool xt, int B, int Cin,
                      int Cout, int L, float* y, hipStream_t st) {
    dim3 grid(cdiv(L, 256 * kConvTT), Cout / CO_T, B);
    if (xt) {
        if (res) return fail(M2_E_ARG, "conv: transposed input with residual is not supported");
        hipLaunchKernelGGL((conv_kernel<KS, CO_T, kConvTT, false, true>), grid, dim3(256), 0, st, x, w, b, alpha, beta, res, Cin, Cout, L, act, y);
    } else if (res) {
        hipLaunchKernelGGL((conv_kernel<KS, CO_T, kConvTT, true, false>), grid, dim3(256), 0, st, x, w, b, alpha, beta, res, Cin, Cout, L, act, y);
    } else {
        hipLaunchKernelGGL((conv_kernel<KS, CO_T, kConvTT, false, false>), grid, dim3(256), 0, st, x, w, b, alpha, beta, res, Cin, Cout, L, act, y);
    }
    M2_LAUNCHED("conv_kernel");
    return M2_OK;
}

template <int KS>
int32_t conv_pick(const float* x, const float* w, const float* b, const float* alpha,
                  const float* beta, const float* res, int act, bool xt, int B, int Cin, int Cout,
                  int L, float* y, hipStream_t st) {
    if (Cout % 8 == 0) return conv_dispatch<KS, 8>(x, w, b, alpha, beta, res, act, xt, B, Cin, Cout, L, y, st);
    if (Cout % 4 == 0) return conv_dispatch<KS, 4>(x, w, b, alpha, beta, res, act, xt, B, Cin, Cout, L, y, st);
    if (Cout % 2 == 0) return conv_dispatch<KS, 2>(x, w, b, alpha, beta, res, act, xt, B, Cin, Cout, L, y, st);
    return conv_dispatch<KS, 1>(x, w, b, alpha, beta, res, act, xt, B, Cin, Cout, L, y, st);
}

template <int R, int CO_T>
int32_t convT_launch(const float* x, const float* w, const float* b, int act, int B, int Cin,
                     int Cout, int L, float* y, hipStream_t st) {
    dim3 grid(cdiv(L, 256 * kConvTQ), Cout / CO_T, B);
    hipLaunchKernelGGL((convT_kernel<R, CO_T, kConvTQ>), grid, dim3(256), 0, st, x, w, b, Cin, Cout, L, act, y);
    M2_LAUNCHED("convT_kernel");
    return M2_OK;
}

template <int R>
int32_t convT_dispatch(const float* x, const float* w, const float* b, int act, int B, int Cin,
                       int Cout, int L, float* y, hipStream_t st) {
    if (Cout % 8 == 0) return convT_launch<R, 8>(x, w, b, act, B, Cin, Cout, L, y, st);
    if (Cout % 4 == 0) return convT_launch<R, 4>(x, w, b, act, B, Cin, Cout, L, y, st);
    if (Cout % 2 == 0) return convT_launch<R, 2>(x, w, b, act, B, Cin, Cout, L, y, st);
    return convT_launch<R, 1>(x, w, b, act, B, Cin, Cout, L, y, st);
}
}  // namespace

int32_t launch_conv(const float* x, const float* w, const float* b, const float* alpha,
                    const float* beta, const float* res, int ksize, int act, bool x_transposed,
                    int B, int Cin, int Cout, int L, float* y, hipStream_t st) {
    M2_CHECK_SHAPE(Cin > 0 && Cout > 0, "conv: empty channels");
    M2_CHECK_ARG((alpha == nullptr) == (beta == nullptr), "conv: alpha and beta go together");
    if (B == 0 || L == 0) return M2_OK;
    if (ksize == 3) return conv_pick<3>(x, w, b, alpha, beta, res, act, x_transposed, B, Cin, Cout, L, y, st);
    if (ksize == 1) return conv_pick<1>(x, w, b, alpha, beta, res, act, x_transposed, B, Cin, Cout, L, y, st);
    return fail(M2_E_SHAPE, "conv: kernel size must be 1 or 3");
}

int32_t launch_conv_general(const float* x, const float* w, const float* b, const float* alpha, const float* beta,
                            const float* res, int ksize, int dil, int pad, int act, int B, int Cin, int Cout, int L,
                            float* y, hipStream_t st) {
    M2_CHECK_SHAPE(Cin > 0 && Cout > 0 && ksize > 0 && dil > 0 && pad >= 0, "conv: bad kernel geometry");
    M2_CHECK_ARG((alpha == nullptr) == (beta == nullptr), "conv: alpha and beta go together");
    const long lo = (long)L + 2L * pad - (long)dil * (ksize - 1);
    M2_CHECK_SHAPE(lo >= 0 && lo <= INT32_MAX, "conv: output length out of range");
    const int Lo = (int)lo;
    M2_CHECK_SHAPE(!res || Lo == L, "conv: a residual needs the output length to equal the input length");
    if (B == 0 || Lo == 0) return M2_OK;
    const int cot = Cout % 4 == 0 ? 4 : (Cout % 2 == 0 ? 2 : 1);
    const dim3 grid(cdiv(Lo, 256), Cout / cot, B);
    if (cot == 4)
        hipLaunchKernelGGL((conv_general_kernel<4>), grid, dim3(256), 0, st, x, w, b, alpha, beta, res, Cin, Cout, L,
                           Lo, ksize, dil, pad, act, y);
    else if (cot == 2)
        hipLaunchKernelGGL((conv_general_kernel<2>), grid, dim3(256), 0, st, x, w, b, alpha, beta, res, Cin, Cout, L,
                           Lo, ksize, dil, pad, act, y);
    else
        hipLaunchKernelGGL((conv_general_kernel<1>), grid, dim3(256), 0, st, x, w, b, alpha, beta, res, Cin, Cout, L,
                           Lo, ksize, dil, pad, act, y);
    M2_LAUNCHED("conv_general_kernel");
    return M2_OK;
}

int32_t launch_convT(const float* x, const float* w, const float* b, int rate, int act, int B,
                     int Cin, int Cout, int L, float* y, hipStream_t st) {
    M2_CHECK_SHAPE(Cin > 0 && Cout > 0, "convT: empty channels");
    if (B == 0 || L == 0) return M2_OK;
    switch (rate) {
        case 2: return convT_dispatch<2>(x, w, b, act, B, Cin, Cout, L, y, st);
        case 4: return convT_dispatch<4>(x, w, b, act, B, Cin, Cout, L, y, st);
        default: return fail(M2_E_SHAPE, "convT: upsample rate must be 2 or 4");
    }
}

}  // namespace m2
