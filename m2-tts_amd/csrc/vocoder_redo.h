// The range policy's local redo ("fallback", m2_set_range_policy): a tail
// workgroup whose own audio samples came out non-finite on the split-f16 path
// recomputes exactly those frames in fp32 from the mel, inside the same launch.
//
// The split path needs every operand below 65520 (f16 max after rounding); an
// input or activation beyond it becomes +-inf and the non-finite value reaches
// the audio ("Range guard").  The pipelined tail kernels
// see their own output samples in registers, so each workgroup knows whether
// its strip of audio is finite.  With a VocRedo in the launch, a workgroup
// whose strip is not re-runs the reference's layer sequence for the strip's
// frames (/root/reference/src/models/tts_model.py:279-297: input_conv, then
// per rate leaky(ConvT), LightweightResBlock components.py:196-200, then
// tanh(output_conv)) in fp32 by direct convolution, in windows of FW frames
// widened by kRedoHalo frames each side (the vocoder's receptive field: the
// streamed vocoder's kVocHalo), each layer's activations of the window held
// in the workgroup's LDS; positions outside the utterance are the reference's
// zero padding, positions outside the window only reach the halo frames,
// which are not stored.  No other launch, no host wait: a call whose audio is
// finite costs one workgroup barrier per tail workgroup.
#pragma once
#include "m2_common.h"

namespace m2 {

constexpr int kRedoHalo = 3;  // frames; == kVocHalo (m2_runtime.hip)

// The vocoder's fp32 weights in the reference layouts (model buffer).
struct VocRedoW {
    int M = 0, C = 0;                       // mel channels, vocoder channels
    const float *wi = nullptr, *bi = nullptr;  // input_conv: [C][M][3], [C]
    const float *wt[4] = {}, *bt[4] = {};      // upsamples.k: [c][c / 2][2 R], [c / 2]
    const float *w1[4] = {}, *b1[4] = {};      // resblocks.k.conv1: [c][c][3], [c]
    const float *w2[4] = {}, *b2[4] = {};      // resblocks.k.conv2
    const float *wo = nullptr, *bo = nullptr;  // output_conv: [1][C / 16][3], [1]
};

// What a tail launch needs for the local redo (null rw: no redo).
struct VocRedo {
    const VocRedoW* rw = nullptr;  // device copy (m2_model)
    const float* mel = nullptr;    // the call's mel, [B][M][T] or, trans, [B][T][M]
    int trans = 0;
};

// LDS floats the redo needs for windows of FW output frames (two activation
// buffers of the widest stage: 4 C floats per window frame).
__host__ __device__ constexpr int redo_lds_floats(int C, int FW) { return 2 * 4 * C * (FW + 2 * kRedoHalo); }

namespace redo {
constexpr int kRates[4] = {4, 4, 2, 2};

__device__ __forceinline__ float leaky(float x) { return x > 0.f ? x : kLeaky * x; }

// One conv1d (kernel 3, padding 1) over n window positions whose first is
// absolute position a0 of a signal of length L: y[co][j] = b[co] +
// sum_ci,k w[co][ci][k] x[ci][j + k - 1] (x = 0 outside the window and the
// signal), then leaky (ACT 1), or added to y (ACT 2: the ResBlock residual).
template <int ACT>
__device__ void conv3(const float* __restrict__ w, const float* __restrict__ b, const float* x, float* y, int cin,
                      int cout, int n, int a0, int L) {
    for (int idx = threadIdx.x; idx < cout * n; idx += blockDim.x) {
        const int co = idx / n, j = idx - co * n;
        float acc = b[co];
        const float* wr = w + (size_t)co * cin * 3;
        for (int k = 0; k < 3; ++k) {
            const int jj = j + k - 1, t = a0 + jj;
            if (jj < 0 || jj >= n || t < 0 || t >= L) continue;
            for (int ci = 0; ci < cin; ++ci) acc = fmaf(wr[ci * 3 + k], x[ci * n + jj], acc);
        }
        if constexpr (ACT == 1) y[idx] = leaky(acc);
        else if constexpr (ACT == 2) y[idx] += acc;
        else y[idx] = acc;
    }
}

// ConvTranspose1d(cin, cin / 2, 2 R, stride R, padding R / 2) + leaky: output
// t reads x[q] with tap t + R / 2 - q R in [0, 2 R), i.e. q = floor((t + R / 2)
// / R) (tap k0) and q - 1 (tap k0 + R).  x holds nin positions from a0.
__device__ void convT(const float* __restrict__ w, const float* __restrict__ b, const float* x, float* y, int cin,
                      int R, int nin, int a0, int Lin) {
    const int cout = cin / 2, n = nin * R;
    for (int idx = threadIdx.x; idx < cout * n; idx += blockDim.x) {
        const int co = idx / n, j = idx - co * n;
        const int t = a0 * R + j, qa = (t + R / 2) / R, k0 = t + R / 2 - qa * R;
        float acc = b[co];
        for (int tap = 0; tap < 2; ++tap) {
            const int q = qa - tap, qr = q - a0, k = k0 + tap * R;
            if (qr < 0 || qr >= nin || q < 0 || q >= Lin) continue;
            for (int ci = 0; ci < cin; ++ci) acc = fmaf(w[((size_t)ci * cout + co) * 2 * R + k], x[ci * nin + qr], acc);
        }
        y[idx] = leaky(acc);
    }
}
}  // namespace redo

// Frames [f0, f1) of utterance b (T frames): audio samples [64 f0, 64 f1) of
// arow (= audio + b 64 T), recomputed in fp32.  lds: lds_floats >=
// redo_lds_floats(C, 1).  Every thread of the workgroup calls it.
__device__ inline void redo_frames(const VocRedoW& w, const float* __restrict__ mel, bool trans, int T, int b,
                                   int f0, int f1, float* __restrict__ arow, float* lds, int lds_floats) {
    const int C = w.C, M = w.M;
    const int FW = lds_floats / (8 * C) - 2 * kRedoHalo;  // output frames per window
    const float* mb = mel + (size_t)b * M * T;
    for (int g0 = f0; g0 < f1; g0 += FW) {
        const int g1 = min(f1, g0 + FW), w0 = max(0, g0 - kRedoHalo), w1 = min(T, g1 + kRedoHalo), W = w1 - w0;
        float* X = lds;
        float* Y = lds + 4 * C * (FW + 2 * kRedoHalo);
        __syncthreads();  // the previous window's last readers are done
        // input_conv: C x W positions from the mel (real mel outside the window)
        for (int idx = threadIdx.x; idx < C * W; idx += blockDim.x) {
            const int co = idx / W, j = idx - co * W, t = w0 + j;
            float acc = w.bi[co];
            const float* wr = w.wi + (size_t)co * M * 3;
            for (int k = 0; k < 3; ++k) {
                const int tt = t + k - 1;
                if (tt < 0 || tt >= T) continue;
                for (int ci = 0; ci < M; ++ci)
                    acc = fmaf(wr[ci * 3 + k], trans ? mb[(size_t)tt * M + ci] : mb[(size_t)ci * T + tt], acc);
            }
            X[idx] = acc;
        }
        int c = C, r = 1;  // channels and resolution of the signal in X
        for (int s = 0; s < 4; ++s) {
            const int R = redo::kRates[s], nin = W * r;
            __syncthreads();
            redo::convT(w.wt[s], w.bt[s], X, Y, c, R, nin, w0 * r, T * r);
            c /= 2;
            r *= R;
            const int n = W * r;
            __syncthreads();
            redo::conv3<1>(w.w1[s], w.b1[s], Y, X, c, c, n, w0 * r, T * r);  // h = leaky(conv1(a)) into X
            __syncthreads();
            redo::conv3<2>(w.w2[s], w.b2[s], X, Y, c, c, n, w0 * r, T * r);  // a += conv2(h), in place in Y
            float* t = X;  // the stage's output becomes the next input
            X = Y;
            Y = t;
        }
        __syncthreads();
        // tanh(output_conv) for the window's centre frames [g0, g1)
        const int n = W * 64, j0 = 64 * (g0 - w0), j1 = 64 * (g1 - w0);
        for (int j = j0 + (int)threadIdx.x; j < j1; j += blockDim.x) {
            float acc = w.bo[0];
            for (int k = 0; k < 3; ++k) {
                const int jj = j + k - 1, t = 64 * w0 + jj;
                if (jj < 0 || jj >= n || t < 0 || t >= 64 * T) continue;
                for (int ci = 0; ci < c; ++ci) acc = fmaf(w.wo[ci * 3 + k], X[ci * n + jj], acc);
            }
            arow[64 * (size_t)w0 + j] = tanhf(acc);
        }
    }
    __syncthreads();
}

}  // namespace m2
