// Fused vocoder: packed-weight table and launcher (vocoder_fused.hip).
#pragma once
#include <functional>
#include <vector>

#include "m2_common.h"

namespace m2 {

// Vocoder weights in MFMA A-fragment order (pack_conv3 / pack_convT) plus the
// raw output_conv weight; all device pointers.
struct VocW {
    const float *wi, *bi;
    const float *wt[4], *bt[4];
    const float *w1[4], *b1[4], *w2[4], *b2[4];
    const float *wo, *bo;
};

bool vocoder_fused_supported(int M, int C);

// mark(kernel_index 0..2, begin): measurement hook around the head / mid / tail launches.
int32_t launch_vocoder_fused(const float* mel, bool trans, int M, int C, int B, int T, const VocW& w, float* U1,
                             float* U2, float* audio, hipStream_t st, const std::function<void(int, bool)>& mark);

constexpr int kVocKernels = 3;
extern const char* const kVocKernelNames[kVocKernels];

// Host-side packing into A-fragment order for v_mfma_f32_16x16x4_f32, k-steps
// padded to KSP = roundup(KS, 4), layout [mb][s/4][lane][s%4] holding
// A[row = mb*16 + (lane&15)][kk = 4*s + (lane>>4)].
// conv3:  A[co][k*Cin + ci] = W[co][ci][k]            (W: [Cout][Cin][3])
// convT:  per phase ph, A[co][tap*Cin + ci] = W[ci][co][k_tap(ph)]   (W: [Cin][Cout][2R])
std::vector<float> pack_conv3(const float* W, int Cout, int Cin);
std::vector<float> pack_convT(const float* W, int Cin, int Cout, int R);

}  // namespace m2
