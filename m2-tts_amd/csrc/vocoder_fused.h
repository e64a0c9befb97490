// Fused vocoder: packed-weight table and launcher (vocoder_fused.hip).
#pragma once
#include <cstdint>
#include <functional>
#include <vector>

#include "m2_common.h"
#include "vocoder_redo.h"

namespace m2 {

// Vocoder weights in MFMA A-fragment order (pack_conv3 / pack_convT) plus the
// raw output_conv weight; all device pointers.
struct VocW {
    const float *wi, *bi;
    const float *wt[4], *bt[4];
    const float *w1[4], *b1[4], *w2[4], *b2[4];
    const float *wo, *bo;
    // stage1's 8-channel tail layers in the two-phase forms (M2_F32_PAIR):
    // ConvT4 (pack_convT2_paired) and ResBlock4's convs (pack_conv3_2p);
    // null when the last stage does not have 8 channels
    const float *wt4p = nullptr, *w1p = nullptr, *w2p = nullptr;
    // stage1's input conv composed into ConvT1 (M2_F32_COMP): packed weights
    // (pack_f32_head_comp), per-phase bias [4][C/2] and edge tables
    // (pack_x3_head_comp's, MP = M); null otherwise
    const float *hcw = nullptr, *hcb = nullptr, *hce = nullptr;
    // device word; when set, the call is the range policy's on-device redo
    // of a split-path call whose audio came out non-finite: ONE persistent
    // launch (voc_redo_kernel) whose workgroups return at once unless it is
    // non-zero, with guard_queue its 4 zeroed work-queue words
    const int* guard = nullptr;
    const unsigned* guard_queue = nullptr;
    // device frame count (dev_frames); T of the launch = capacity when set
    const int32_t* dT = nullptr;
};

bool vocoder_fused_supported(int M, int C);

// mark(kernel_index 0..2, begin): measurement hook around the head / mid / tail launches.
int32_t launch_vocoder_fused(const float* mel, bool trans, int M, int C, int B, int T, const VocW& w, float* U1,
                             float* U2, float* audio, hipStream_t st, const std::function<void(int, bool)>& mark);

constexpr int kVocKernels = 3;
extern const char* const kVocKernelNames[kVocKernels];
extern const char* const kVocX3KernelNames[kVocKernels];

// Host-side packing into A-fragment order for v_mfma_f32_16x16x4_f32, k-steps
// padded to KSP = roundup(KS, 4), layout [mb][s/4][lane][s%4] holding
// A[row = mb*16 + (lane&15)][kk = 4*s + (lane>>4)].
// conv3:  A[co][k*Cin + ci] = W[co][ci][k]            (W: [Cout][Cin][3])
// convT:  per phase ph, A[co][tap*Cin + ci] = W[ci][co][k_tap(ph)]   (W: [Cin][Cout][2R])
std::vector<float> pack_conv3(const float* W, int Cout, int Cin);
std::vector<float> pack_convT(const float* W, int Cin, int Cout, int R);
std::vector<float> pack_convT2_paired(const float* W, int Cin);  // Cout = 8, R = 2
std::vector<float> pack_f32_head_comp(const float* Win, const float* WT, int M, int C);
std::vector<float> pack_conv3_2p(const float* W);                 // 8 -> 8 channels

// ---------------------------------------------------------------------------
// Split-f16 vocoder (vocoder_x3.hip): conv / convT weights packed as f16
// hi/lo pairs in v_mfma_f32_16x16x32_f16 A-fragment order; biases and the
// output conv stay fp32.
typedef unsigned int vx_u32x4 __attribute__((ext_vector_type(4)));

// fp32 -> (hi, lo) f16 pair, hi = f16(v), lo = f16(v - hi): the activation
// format of every split-f16 buffer (LDS rows, U1, U2) and of the packed
// weights.  lo is unscaled and may be an f16 subnormal, an absolute error of
// at most 2^-25 per value (whole-vocoder waveform RMS 3e-7 vs fp64, against
// 1.6e-7 for plain fp32: tools/probe/split_sim.py).  One v_cvt_pk_f16_f32
// per pair for hi and one v_fma_mix{lo,hi}_f16 per value for lo (v - hi
// rounded once).
// Range: hi rounds to nearest even, so |v| >= 65520 (past the f16 range)
// gives hi = inf and lo = v - inf = NaN, and the NaN propagates through every
// later MFMA, activation and split to the output: a split path's result is
// either exact to the bound above or non-finite, never silently wrong (a
// round-toward-zero hi would saturate at 65504 and lose precision quietly
// for 65504 < |v| < 131024).  The vocoder's last kernel flags non-finite
// audio (m2_model_check / M2_E_RANGE; the fallback policy re-runs the call
// on the exact-f32 kernels).
// hi comes from a compiler-visible conversion (one v_cvt_pk_f16_f32): it is
// the first reader of MFMA results in most epilogues, and only an instruction
// the compiler sees gets the MFMA -> VALU wait states in front of it (an
// inline-asm reader straight after the MFMA would read its stale destination
// registers); the fma_mix halves below follow it.
__device__ __forceinline__ void split2u(float v0, float v1, unsigned& hi, unsigned& lo) {
    typedef float f2_t __attribute__((ext_vector_type(2)));
    typedef _Float16 h2_t __attribute__((ext_vector_type(2)));
    hi = __builtin_bit_cast(unsigned, __builtin_convertvector(f2_t{v0, v1}, h2_t));
    asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hi), "v"(v0));
    asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hi), "v"(v1));
}

// max(x, y) as a bare v_max_f32: fmaxf (and fmed3 with inf, which the
// compiler turns back into it) adds a NaN-quieting v_max(x, x) per MFMA result.
__device__ __forceinline__ float vmax(float x, float y) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

// leaky_relu(x, 0.1) of four accumulator values: two packed multiplies and
// four bare max (== x > 0 ? x : 0.1x, as act_t<ACT_LEAKY>).
__device__ __forceinline__ void leaky4(float (&v)[4]) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 s0 = f2{v[0], v[1]} * kLeaky, s1 = f2{v[2], v[3]} * kLeaky;
    v[0] = vmax(v[0], s0.x);
    v[1] = vmax(v[1], s0.y);
    v[2] = vmax(v[2], s1.x);
    v[3] = vmax(v[3], s1.y);
}
struct VocX {
    const vx_u32x4* wi;
    const float* bi;
    const vx_u32x4* wt[4];
    const float* bt[4];
    const vx_u32x4* w1[4];
    const float* b1[4];
    const vx_u32x4* w2[4];
    const float* b2[4];
    const float *wo, *bo;
    // pipelined stage1 tail (vocoder_tailp.hip); null = the x3 tail kernel
    const vx_u32x4* tp;
    const float* tpb;
    // pipelined stage1 mid stage (vocoder_midp.hip); null = the x3 mid kernel
    const vx_u32x4* mp;
    const float* mpb;
    // pipelined stage2 tail (vocoder_tailp2.hip); null = the x3 tail kernel
    const vx_u32x4* tp2;
    const float* tp2b;
    // stage1 head with input_conv composed into ConvT1 (vocoder_x3.hip,
    // head_convT1c_planar): weights, per-phase bias, edge tables; null = the
    // two layers
    const vx_u32x4* hc;
    const float* hcb;
    const float* hce;
    // set to 1 (vector store) by the last kernel when an audio sample is not
    // finite; host-mapped (m2_model_check), or a device word of the range
    // policy's on-device redo
    int* rflag;
    // zeroed by the head kernel's first thread when set (the on-device redo's
    // other flag word, whose last readers ran in the previous call)
    int* rclear = nullptr;
    // the redo's four work-queue words (VocW::guard_queue), zeroed with rclear:
    // a redo launch that stopped early cannot leave them claimed for the next
    unsigned* rqueue = nullptr;
    // x3 head: issue priority by wave age (M2_X3_HEAD_PRIO=1: the younger
    // waves of each SIMD higher; measured level at stage1 B=32 in both
    // orders, profiles/r06/r06z16_head_prio.txt: an A/B switch only)
    int head_prio = 0;
    // device frame count (dev_frames): when set, the T passed to the launches
    // is the capacity their grids cover
    const int32_t* dT = nullptr;
    // range policy "fallback" on the pipelined tails (tailp / tailp2): the
    // fp32 weights of their in-launch local redo (vocoder_redo.h; device
    // copy), else null
    const VocRedoW* redo_w = nullptr;
};

// Non-finite output check of the split path's last kernel: any NaN among the
// four values -> *flag = 1 (rare path; the host reads and clears it).
__device__ __forceinline__ void flag_nonfinite4(float a, float b, float c, float d, int* flag) {
    if (flag && ((a != a) | (b != b) | (c != c) | (d != d))) *reinterpret_cast<volatile int*>(flag) = 1;
}
// The same, also raising the workgroup's LDS word lflag (the pipelined tails'
// local redo, vocoder_redo.h).
__device__ __forceinline__ void flag_nonfinite4(float a, float b, float c, float d, int* flag, int* lflag) {
    if ((a != a) | (b != b) | (c != c) | (d != d)) {
        if (flag) *reinterpret_cast<volatile int*>(flag) = 1;
        *reinterpret_cast<volatile int*>(lflag) = 1;
    }
}

// Pipelined stage1 tail (vocoder_tailp.hip): ConvT3, ResBlock3, ConvT4,
// ResBlock4 and output_conv in polyphase form over the columns q of U2.
// Layer l (0..6) has nmb(l) m-blocks of 16 rows and nkb(l) k-blocks of 32.
// A k-block's B fragment is one of the layer's nfrag(l) fragments,
// frag(l, mb, kb); fslot(l, f, g) is what lane group g reads for fragment f:
// column offset dq and input octet of the layer's input ring.  Fragments are
// shared between the m-blocks of a layer wherever their taps allow, so one
// wave doing both m-blocks reads each fragment once; a slot an m-block does
// not use carries zero weights (its dense polyphase matrix is zero there).
// The same tables pack the weights (host) and address the fragments (device).
namespace tp {
struct Slot {
    int dq, oct;
};
constexpr int kLayers = 7, kUnits = 22;
// The composed ResBlock4-conv2 + output_conv layer (six-layer form): weight
// units after the 22 of the seven-layer form, its bias (rows 0..3) and the
// edge terms (vL[8], vR[8], kL, kR) after the seven layers' biases.
constexpr int kOutcUnit0 = kUnits, kOutcUnits = 4, kOutcBias = kLayers * 32, kOutcCorr = kOutcBias + 32;
constexpr int kBiasFloats = kOutcCorr + 32;
// Fragment f, lane group g: 0, 1 on ring R5 (ResBlock4's intermediate h),
// 2, 3 on ring R4 (ConvT4's output x); slots of f = 3 repeated in f = 2 carry
// zero weights.
constexpr Slot outc_slot(int f, int g) {
    return f == 0 || f == 2 ? Slot{0, g}
                            : (f == 1 ? (g < 2 ? Slot{-1, 2 + g} : Slot{1, g - 2})
                                      : (g == 0 ? Slot{-1, 3} : (g == 1 ? Slot{1, 0} : Slot{0, g})));
}
constexpr int nmb(int l) { return l == 6 ? 1 : 2; }
constexpr int nkb(int l) { return (l == 4 || l == 5) ? 1 : 2; }
// ConvT4 (layer 3): output phases 1 and 2 read column q only (t3 = 2q, 2q + 1),
// phases 0 and 3 also its neighbours, so its m-block 0 holds phases 1, 2 (one
// k-block) and m-block 1 phases 0, 3 (two); MFMA row R holds the dense
// (phase, channel) row prow(l, R).  Weight units keep nkb(l) per m-block.
constexpr int nkbm(int l, int mb) { return l == 3 && mb == 0 ? 1 : nkb(l); }
constexpr int prow(int l, int R) { return l != 3 ? R : (R < 16 ? R + 8 : (R < 24 ? R - 16 : R)); }
constexpr int nfrag(int l) { return l == 0 ? 3 : 2; }
constexpr int unit0(int l) { return l <= 4 ? 4 * l : (l == 5 ? 18 : 20); }
// ConvT3: phase 0 reads columns q, q-1 (fragments 0, 1), phase 1 q+1, q (2, 0);
// ResBlock4 convs: m-block (phases p, p+1) reads phases p-1 .. p+2, one
// fragment per m-block; the others: whole column q, then the neighbours.
constexpr int frag(int l, int mb, int kb) {
    return l == 0 ? (mb == 0 ? kb : (kb == 0 ? 2 : 0)) : ((l == 4 || l == 5) ? mb : kb);
}
constexpr Slot fslot(int l, int f, int g) {
    if (l == 0) return Slot{f == 0 ? 0 : (f == 1 ? -1 : 1), g};
    if (l == 4 || l == 5)
        return f == 0 ? (g == 0 ? Slot{-1, 3} : Slot{0, g - 1}) : (g == 3 ? Slot{1, 0} : Slot{0, g + 1});
    if (f == 0) return Slot{0, g};  // the whole column q
    if (l == 6)  // output conv: phase 0 also reads (q-1, phase 3), phase 3 (q+1, phase 0); g 2, 3: (q, g) again
        return g == 0 ? Slot{-1, 3} : (g == 1 ? Slot{1, 0} : Slot{0, g});
    // 2 phases of 16 channels: phase 0 also reads (q-1, phase 1), phase 1 (q+1, phase 0)
    return g < 2 ? Slot{-1, 2 + g} : Slot{1, g - 2};
}
constexpr Slot kslot(int l, int mb, int kb, int g) { return fslot(l, frag(l, mb, kb), g); }
}  // namespace tp


// Pipelined stage1 mid stage (vocoder_midp.hip): ConvT2 (layer 0), ResBlock2
// conv1 / conv2 (layers 1, 2) in polyphase form over the columns q of U1, 8
// m-blocks (phase s = mb / 2) per layer; mslot(l, s, kb, g) as tp::kslot.
namespace mp {
struct MSlot {
    int dq, oct;
};
constexpr int kUnits = 80;
constexpr int mkb(int l) { return l == 0 ? 4 : 3; }
constexpr int munit0(int l) { return l == 0 ? 0 : (l == 1 ? 32 : 56); }
constexpr MSlot mslot(int l, int s, int kb, int g) {
    if (l == 0)  // ConvT2: phases 0, 1 read columns q, q-1; phases 2, 3 read q+1, q (64 ch: 2 k-blocks each)
        return MSlot{kb < 2 ? (s < 2 ? 0 : 1) : (s < 2 ? -1 : 0), 4 * (kb & 1) + g};
    const int pp = s + kb - 1, dq = pp < 0 ? -1 : pp / 4;  // tap t2 + kb - 1: phase pp mod 4 of column q + dq
    return MSlot{dq, 4 * (pp - 4 * dq) + g};
}
}  // namespace mp
struct MidpSrc {
    const float *wt, *bt, *w1, *b1, *w2, *b2;
};
bool pack_midp(const MidpSrc& s, std::vector<uint16_t>* w, std::vector<float>* bias, bool* range_ok);
// dT (dev_frames): when set, L1 is the capacity (4 x capacity frames)
int32_t launch_vocoder_midp(const void* U1, int L1, int B, const vx_u32x4* W, const float* bias, void* U2,
                            hipStream_t st, const int32_t* dT = nullptr);
extern const char* const kVocMidpKernelName;

// Raw fp32 reference weights of the five tail modules (host pointers).
struct TailpSrc {
    const float *wt3, *bt3, *w31, *b31, *w32, *b32, *wt4, *bt4, *w41, *b41, *w42, *b42, *wo, *bo;
};
// false when a layer's non-zero weights do not fit the slot table (cannot
// happen for the stage1 shapes; the x3 tail is kept then).
bool pack_tailp(const TailpSrc& s, std::vector<uint16_t>* w, std::vector<float>* bias, bool* range_ok);
// rd.rw set: range policy "fallback" - a workgroup whose audio strip is not
// finite recomputes it in fp32 inside the launch (vocoder_redo.h).
int32_t launch_vocoder_tailp(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                             int* rflag, hipStream_t st, const int32_t* dT = nullptr, const VocRedo& rd = VocRedo{});
extern const char* const kVocTailpKernelName;
// The same five modules at stage2 widths (C = 256: U2 64 channels) for the
// pipelined stage2 tail (vocoder_tailp2.hip, two waves per layer).
bool pack_tailp2(const TailpSrc& s, std::vector<uint16_t>* w, std::vector<float>* bias, bool* range_ok);
int32_t launch_vocoder_tailp2(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                              int* rflag, hipStream_t st, const int32_t* dT = nullptr, const VocRedo& rd = VocRedo{});
extern const char* const kVocTailp2KernelName;

bool vocoder_x3_supported(int M, int C);
int vocoder_x3_mel_pad(int M);  // input-conv channel count after padding to the k-block layout
// U1/U2: workspace for the intermediates (same bytes as fp32 [B][C/2][4T] / [B][C/4][16T]).
int32_t launch_vocoder_x3(const float* mel, bool trans, int M, int C, int B, int T, const VocX& w, void* U1, void* U2,
                          float* audio, hipStream_t st, const std::function<void(int, bool)>& mark);
// range_ok is cleared when a weight is outside the f16 range (|w| >= 65504).
// res: ResBlock conv2 - for 8/16 channels the residual x is folded into the
// GEMM as an identity block on the padding octets (vocoder_x3.hip, mma_x3).
constexpr bool res_fold_channels(int C) { return C == 8 || C == 16; }
std::vector<uint16_t> pack_x3_conv3(const float* W, int Cout, int Cin, int CinPad, bool* range_ok, bool res);
std::vector<uint16_t> pack_x3_convT(const float* W, int Cin, int Cout, int R, bool* range_ok);
// input_conv o ConvT1 (R = 4) for the stage1 head; false when the shapes do not fit
bool pack_x3_head_comp(const float* Win, const float* bin, const float* WT, const float* bT, int M, int MP, int C,
                       std::vector<uint16_t>* w, std::vector<float>* bias, std::vector<float>* edge, bool* range_ok);

}  // namespace m2
