// Fused SimpleVocoder for gfx950 (tts_model.py:279-297).
//
// Three launches per vocoder pass instead of fourteen:
//   head  : input_conv(M->C, k3) -> ConvT1(x4)+leaky -> ResBlock1        mel  -> U1 [B][C/2][4T]
//   mid   : ConvT2(x4)+leaky -> ResBlock2                                 U1   -> U2 [B][C/4][16T]
//   tail  : ConvT3(x2)+leaky -> ResBlock3 -> ConvT4(x2)+leaky -> ResBlock4
//           -> output_conv(k3) -> tanh                                    U2   -> audio [B][1][64T]
// Each workgroup owns one utterance and one window of positions and runs its
// whole layer chain out of LDS; the window is widened by the exact receptive
// field of the chain (k3 conv: +-1, ConvT(k=2r,s=r,p=r/2): one extra input
// frame each side), so every kept output is the same arithmetic as the
// unfused layer.  Positions outside [0, L) of every layer are stored as 0,
// which is the zero padding the next conv sees in the reference.
// The tail is where fusion pays most: its layers have 8-32 channels (1-12
// FLOP/B unfused), fused the tail reads 32 ch of U2 and writes one sample row.
//
// Every conv / transposed conv is an implicit GEMM on the exact-f32 MFMA
// v_mfma_f32_16x16x4_f32 (64 FLOP/clk/SIMD = the fp32 peak): rows = output
// channels (A = packed weights, streamed from L2, one f32 per lane per MFMA),
// columns = 16 positions (B = activations in LDS: lanes 0-15 read 16
// consecutive positions of one channel row, lanes 16-63 the next 3 rows; rows
// are padded to a stride = 16 mod 32 floats so the two 32-lane halves of a
// ds_read_b32 hit disjoint banks).  K = (tap, channel).  ConvT is r GEMMs,
// one per output phase, each with K = 2 taps x Cin (the 2-tap polyphase form).
#include <algorithm>
#include <cstdlib>
#include <functional>

#include "m2_common.h"
#include "vocoder_fused.h"

namespace m2 {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// An LDS activation window: row stride P (floats), absolute position of col 0.
struct LB {
    float* p;
    int P;
    int start;
};

constexpr int rup16(int n) { return (n + 15) / 16 * 16; }
// Row stride >= cols with stride = 16 (mod 32): conflict-free B-operand reads.
constexpr int pstride(int cols) { return ((cols + 15) / 32) * 32 + 16; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
// Compact row stride (multiple of 4, >= cols): up to 4-lane 2-way conflicts
// between the two 16-lane halves of a read, in exchange for LDS capacity.
constexpr int cstride(int cols) { return (cols + 3) / 4 * 4 + ((((cols + 3) / 4 * 4) % 32 == 0) ? 4 : 0); }
constexpr int stride_for(int cols, bool compact) { return compact ? cstride(cols) : pstride(cols); }

// ---------------------------------------------------------------------------
// acc[n] += sum_s A(s) * B(s, n) over KS = NTAP*KC k-steps for NT 16-wide
// column tiles.  A: packed weights, k-steps padded to KSP (multiple of 4),
// laid out [s/4][lane][s%4] so one global_load_dwordx4 per lane fetches 4
// k-steps (1 KiB per wave-instruction).  B(s, n) = bp[(s % KC)*4*P +
// (s / KC)*OFFSTEP + n*16] from LDS (P, OFFSTEP compile-time: every B read
// is a ds_read with an immediate offset off one per-item base address).  Register double buffer over k-blocks of
// KB steps: block i+1's loads are in flight while block i's KB*NT MFMAs run
// (KB = 8: 2 KiB of weights per wave in flight - the weight stream from L2 is
// latency-bound, so bytes in flight set its rate; measured on the round-6
// stage1 tree as a separate build, processes alternated: 1.5 % slower than
// KB = 4, profiles/r06/r06z10_kb8.txt).  Loads of tiles past `nt` re-read the
// last live tile (no branch; nothing is stored from them).
#ifndef M2_KB8
#define M2_KB8 0
#endif
template <int KS>
struct KPlan {
    static constexpr int KSP = (KS + 3) / 4 * 4;
    static constexpr int KB = (KSP <= 8) ? KSP : ((KS % 8 == 0 && M2_KB8) ? 8 : 4);
    static constexpr int NB = KSP / KB;
};

template <int KC, int NTAP, int NT, int P, int OFFSTEP, int CS = 16>
__device__ __forceinline__ void mma_run(const float* __restrict__ wp, const float* __restrict__ bp, int nt,
                                        f32x4 (&acc)[NT]) {
    constexpr int KS = NTAP * KC;
    using KP = KPlan<KS>;
    constexpr int KB = KP::KB, NB = KP::NB;
    f32x4 a[2][KB / 4];
    auto load = [&](int blk, f32x4 (&aa)[KB / 4]) {
#pragma unroll
        for (int q = 0; q < KB / 4; ++q) aa[q] = *reinterpret_cast<const f32x4*>(wp + (blk * (KB / 4) + q) * 256);
        __builtin_amdgcn_sched_barrier(0);
    };
    // One k-block: all B reads first (one LDS round trip per block), then the
    // KB*NT MFMAs.  sched_barrier pins the order: hipcc otherwise sinks the
    // next block's weight loads to the end of the block and interleaves
    // ds_read -> lgkmcnt(0) -> 2 MFMAs, exposing an LDS round trip per pair.
    auto compute = [&](int blk, const f32x4 (&aa)[KB / 4]) {
        float bv[KB][NT];
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            const int s = blk * KB + i;
            if (NB > 1 || s < KS) {
                const float* br = bp + (s % KC) * 4 * P + (s / KC) * OFFSTEP;
#pragma unroll
                for (int n = 0; n < NT; ++n) bv[i][n] = (n < nt) ? br[n * CS] : 0.f;
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < KB; ++i) {
            if (NB > 1 || blk * KB + i < KS) {
#pragma unroll
                for (int n = 0; n < NT; ++n)
                    if (n < nt) acc[n] = mfma16(aa[i / 4][i % 4], bv[i][n], acc[n]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    static_assert(NB == 1 || KS % KB == 0, "multi-block K must be a multiple of the block");
    load(0, a[0]);
    int blk = 0;
#pragma unroll 1
    for (; blk + 2 < NB; blk += 2) {
        load(blk + 1, a[1]);
        compute(blk, a[0]);
        load(blk + 2, a[0]);
        compute(blk + 1, a[1]);
    }
    if (blk + 1 < NB) {
        load(blk + 1, a[1]);
        compute(blk, a[0]);
        compute(blk + 1, a[1]);
    } else {
        compute(blk, a[0]);
    }
}

// Work distribution inside a layer.  Dynamic (-DM2_STATIC_SCHED=0): each wave takes the
// next item from an LDS counter - waves sharing a SIMD progress at different
// rates (issue arbitration favours the older wave), so a static item->wave
// map leaves the SIMD idle behind the slowest wave at every layer barrier.
// Static (default, 1-3 % faster measured on MI355X): item = wave, wave + nwaves, ...
#ifndef M2_STATIC_SCHED
#define M2_STATIC_SCHED 1
#endif
__device__ __forceinline__ int first_item(int* ctr) {
    if (M2_STATIC_SCHED) return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int v = 0;
    if ((threadIdx.x & 63) == 0) v = atomicAdd(ctr, 1);
    return __builtin_amdgcn_readfirstlane(__shfl(v, 0));
}
__device__ __forceinline__ int next_item(int* ctr, int item) {
    if (M2_STATIC_SCHED) return item + (blockDim.x >> 6);
    return first_item(ctr);
}

// Conv1d(k=3, pad=1) over an LDS window: abs positions [a0, a0+npos), all
// COUT channels.  Epilogue: +bias, act, (+ residual read from `out` in place),
// 0 outside [0, L).  Packed weights: Wp[mb][s][lane] = W[mb*16 + (lane&15)]
// [ci][k] with k*CIN + ci = 4*s + (lane>>4)  (zero rows for co >= COUT).
template <int CIN, int COUT, int NT, int ACT, bool RES, int PIN>
__device__ __forceinline__ void lconv3(const float* __restrict__ Wp, const float* __restrict__ bias, LB in,
                                       LB out, int a0, int npos, int L, int* ctr) {
    static_assert(CIN % 4 == 0, "CIN must be a multiple of 4");
    constexpr int KC = CIN / 4, KS = 3 * KC, MB = (COUT + 15) / 16;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ntiles = (npos + 15) >> 4;
    const int nch = (ntiles + NT - 1) / NT;
    for (int item = first_item(ctr); item < MB * nch; item = next_item(ctr, item)) {
        const int mb = item % MB, tile0 = (item / MB) * NT;
        const int nt = min(NT, ntiles - tile0);
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = mb * 16 + lk * 4 + r;
            bv[r] = co < COUT ? bias[co] : 0.f;  // issued before the MFMA loop: latency hidden
        }
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_run<KC, 3, NT, PIN, 1>(Wp + (size_t)mb * KPlan<KS>::KSP * 64 + lane * 4,
                                   in.p + lk * PIN + (a0 + tile0 * 16 + li - in.start - 1), nt, acc);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            if (n < nt) {
                const int j = (tile0 + n) * 16 + li;
                const int t = a0 + j;
                if (j < npos) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int co = mb * 16 + lk * 4 + r;
                        if (co < COUT) {
                            float v = act_t<ACT>(acc[n][r] + bv[r]);
                            float* o = out.p + co * out.P + (t - out.start);
                            if (RES) v += *o;
                            *o = (t >= 0 && t < L) ? v : 0.f;
                        }
                    }
                }
            }
        }
    }
}

// leaky(ConvTranspose1d(k=2R, stride R, pad R/2)) over an LDS window: input
// positions q in [q0, q0+nq) produce outputs t = q*R + ph, ph < R.  Phase ph
// reads taps (q, q-1) if ph + R/2 < R else (q+1, q).  Packed weights:
// Wp[ph][mb][s][lane] = W[ci][mb*16 + (lane&15)][k_tap] with
// tap*CIN + ci = 4*s + (lane>>4).
template <int CIN, int COUT, int R, int NT, int PIN>
__device__ __forceinline__ void lconvT(const float* __restrict__ Wp, const float* __restrict__ bias, LB in,
                                       LB out, int q0, int nq, int L, int* ctr) {
    static_assert(CIN % 4 == 0, "CIN must be a multiple of 4");
    constexpr int KC = CIN / 4, KS = 2 * KC, MB = (COUT + 15) / 16, PAD = R / 2;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ntiles = (nq + 15) >> 4;
    const int nch = (ntiles + NT - 1) / NT;
    for (int item = first_item(ctr); item < R * MB * nch; item = next_item(ctr, item)) {
        const int ph = item % R, rest = item / R;
        const int mb = rest % MB, tile0 = (rest / MB) * NT;
        const int nt = min(NT, ntiles - tile0);
        const int d0 = (ph + PAD < R) ? 0 : 1;  // tap 0 offset; tap 1 is d0 - 1
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = mb * 16 + lk * 4 + r;
            bv[r] = co < COUT ? bias[co] : 0.f;
        }
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_run<KC, 2, NT, PIN, -1>(Wp + (size_t)(ph * MB + mb) * KPlan<KS>::KSP * 64 + lane * 4,
                                    in.p + lk * PIN + (q0 + tile0 * 16 + li - in.start + d0), nt, acc);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            if (n < nt) {
                const int j = (tile0 + n) * 16 + li;
                const int t = (q0 + j) * R + ph;
                if (j < nq) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int co = mb * 16 + lk * 4 + r;
                        if (co < COUT) {
                            const float v = act_t<ACT_LEAKY>(acc[n][r] + bv[r]);
                            out.p[co * out.P + (t - out.start)] = (t >= 0 && t < L) ? v : 0.f;
                        }
                    }
                }
            }
        }
    }
}

// The head's input conv composed into ConvT1 (stage1 exact-f32, the default;
// M2_F32_COMP=0 runs the input conv as its own layer; B=32 T=500 0.1959 ->
// 0.1847 ms per call alternated in one process, within 1.3e-6 of the
// two-layer form, profiles/r06/r06z7_comp.txt):
// u = leaky(Wc * mel + bc[ph]) with Wc[ph] = W_T[ph] o W_in a 4-tap transposed
// conv straight from the mel window (taps kk: mel frame q + d0 + 1 - kk), the
// weights composed on the host in double (pack_f32_head_comp; the split head's
// composition, vocoder_x3.hip).  The input conv's own zero padding (a0 = 0 at
// frames -1 and T) is not what the composed form sees there, so the outputs
// reading a0[-1] (q = 0, ph < 2) or a0[T] (q = T - 1, ph >= 2) subtract
// corr[ph][co] (head_f32_corr) before the activation.  Per-phase bias
// bc[ph * C1 + co].
template <int M, int COUT, int NT, int PIN>
__device__ __forceinline__ void lconvT1c(const float* __restrict__ Wp, const float* __restrict__ bias, LB in, LB out,
                                         int q0, int nq, int T, const float* corr, int* ctr) {
    constexpr int R = 4, KC = M / 4, KS = 4 * KC, MB = (COUT + 15) / 16, PAD = R / 2;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ntiles = (nq + 15) >> 4;
    const int nch = (ntiles + NT - 1) / NT;
    const int L = 4 * T;
    for (int item = first_item(ctr); item < R * MB * nch; item = next_item(ctr, item)) {
        const int ph = item % R, rest = item / R;
        const int mb = rest % MB, tile0 = (rest / MB) * NT;
        const int nt = min(NT, ntiles - tile0);
        const int d0 = (ph + PAD < R) ? 0 : 1;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = bias[ph * COUT + mb * 16 + lk * 4 + r];
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_run<KC, 4, NT, PIN, -1>(Wp + (size_t)(ph * MB + mb) * KPlan<KS>::KSP * 64 + lane * 4,
                                    in.p + lk * PIN + (q0 + tile0 * 16 + li - in.start + d0 + 1), nt, acc);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            if (n < nt) {
                const int j = (tile0 + n) * 16 + li;
                const int q = q0 + j, t = q * R + ph;
                if (j < nq) {
                    const bool edge = corr && (ph < 2 ? q == 0 : q == T - 1);
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int co = mb * 16 + lk * 4 + r;
                        float v = acc[n][r] + bv[r];
                        if (edge) v -= corr[ph * COUT + co];
                        v = act_t<ACT_LEAKY>(v);
                        out.p[co * out.P + (t - out.start)] = (t >= 0 && t < L) ? v : 0.f;
                    }
                }
            }
        }
    }
}

// corr[ph][co] = sum_m E[ph][co][m] mel[m][frame] + e[ph][co], frame 0 for
// ph < 2 (left edge: a0[-1]) and T - 1 for ph >= 2 (right edge: a0[T]), the
// terms the composed form adds where the reference's ConvT1 sees a0's zero
// padding (E, e: pack_x3_head_comp's edge tables at MP = M).
template <int M, int C1>
__device__ __forceinline__ void head_f32_corr(const float* __restrict__ E, LB mel, int T, bool left, bool right,
                                              float* corr) {
    for (int i = threadIdx.x; i < 4 * C1; i += blockDim.x) {
        const int ph = i / C1;
        const bool use = ph < 2 ? left : right;
        float v = 0.f;
        if (use) {
            const int f = ph < 2 ? 0 : T - 1;
            const float* x = mel.p + (f - mel.start);
            const float* e = E + (size_t)i * M;
            v = E[(size_t)4 * C1 * M + i];
            for (int m = 0; m < M; ++m) v = fmaf(e[m], x[m * mel.P], v);
        }
        corr[i] = v;
    }
}

// Two-phase forms of the 8-channel layers (stage1's ConvT4 and ResBlock4,
// the default; M2_F32_PAIR=0 runs them phase by phase): an 8-channel output
// fills half of a 16-row m-block, so two output phases share one: row
// (p, co) = 8p + co.  The tail's MFMAs per window 5,056 -> 4,300 (W3 = 500);
// the exact-f32 vocoder at B=32 T=500 0.2089 -> 0.1983 ms per call, one
// process alternated (profiles/r06/r06z3_pair.txt), within 5.9e-7 of the
// phase-by-phase form and of the oracle's bound (test_gpu_f32_forms.py).
// ConvT4 paired: leaky(ConvTranspose1d(k=4, stride 2, pad 1)) as a k3 conv
// over its input positions q whose 16 output rows are (phase, channel),
// output t = 2q + p: 12 k-steps per 16 columns instead of 2 x 8
// (pack_convT2_paired: out[2q] = x[q] W1 + x[q-1] W3, out[2q+1] = x[q+1] W0 + x[q] W2).
template <int CIN, int NT, int PIN>
__device__ __forceinline__ void lconvT2p(const float* __restrict__ Wp, const float* __restrict__ bias, LB in,
                                         LB out, int q0, int nq, int L, int* ctr) {
    static_assert(CIN % 4 == 0, "CIN must be a multiple of 4");
    constexpr int KC = CIN / 4;
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ntiles = (nq + 15) >> 4;
    const int nch = (ntiles + NT - 1) / NT;
    for (int item = first_item(ctr); item < nch; item = next_item(ctr, item)) {
        const int tile0 = item * NT;
        const int nt = min(NT, ntiles - tile0);
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = bias[(lk * 4 + r) & 7];
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_run<KC, 3, NT, PIN, 1>(Wp + lane * 4, in.p + lk * PIN + (q0 + tile0 * 16 + li - in.start - 1), nt, acc);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            if (n < nt) {
                const int j = (tile0 + n) * 16 + li;
                if (j < nq) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = lk * 4 + r, ph = row >> 3, co = row & 7;
                        const int t = 2 * (q0 + j) + ph;
                        const float v = act_t<ACT_LEAKY>(acc[n][r] + bv[r]);
                        out.p[co * out.P + (t - out.start)] = (t >= 0 && t < L) ? v : 0.f;
                    }
                }
            }
        }
    }
}

// ResBlock4's k3 convs in the two-phase form: column j covers positions
// a0 + 2j + p (p = 0, 1), K = taps at a0 + 2j - 1 .. a0 + 2j + 2 x 8 input
// channels (8 k-steps per 32 positions instead of 12).  The B reads step two
// positions per lane, so the windows these read take an odd row stride
// (ostride: conflict-free 32-lane groups).  Packed by pack_conv3_2p.
template <int NT, int ACT, bool RES, int PIN>
__device__ __forceinline__ void lconv3_2p(const float* __restrict__ Wp, const float* __restrict__ bias, LB in,
                                          LB out, int a0, int npos, int L, int* ctr) {
    constexpr int KC = 2;  // 8 input channels
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    const int ncol = (npos + 1) >> 1;
    const int ntiles = (ncol + 15) >> 4;
    const int nch = (ntiles + NT - 1) / NT;
    for (int item = first_item(ctr); item < nch; item = next_item(ctr, item)) {
        const int tile0 = item * NT;
        const int nt = min(NT, ntiles - tile0);
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = bias[(lk * 4 + r) & 7];
        f32x4 acc[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_run<KC, 4, NT, PIN, 1, 32>(Wp + lane * 4, in.p + lk * PIN + (a0 + 2 * (tile0 * 16 + li) - in.start - 1), nt,
                                       acc);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            if (n < nt) {
                const int j = (tile0 + n) * 16 + li;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = lk * 4 + r, p = row >> 3, co = row & 7;
                    const int jj = 2 * j + p, t = a0 + jj;
                    if (jj < npos) {
                        float v = act_t<ACT>(acc[n][r] + bv[r]);
                        float* o = out.p + co * out.P + (t - out.start);
                        if (RES) v += *o;
                        *o = (t >= 0 && t < L) ? v : 0.f;
                    }
                }
            }
        }
    }
}

// Global [rows][Lg] (or [Lg][rows] when TRANS) -> LDS window cols [0, ncols),
// zero outside [0, Lg).
template <bool TRANS>
__device__ __forceinline__ void gload(const float* __restrict__ g, int rows, int Lg, LB dst, int ncols) {
    const int n = rows * ncols;
#pragma unroll 2
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        int r, c;
        if (TRANS) { c = i / rows; r = i - c * rows; }
        else { r = i / ncols; c = i - r * ncols; }
        const int t = dst.start + c;
        float v = 0.f;
        if (t >= 0 && t < Lg) v = TRANS ? g[(size_t)t * rows + r] : g[(size_t)r * Lg + t];
        dst.p[r * dst.P + c] = v;
    }
}

// LDS window -> global [rows][Lg], abs positions [a0, a0+n) clipped to Lg.
__device__ __forceinline__ void gstore(float* __restrict__ g, int rows, int Lg, LB src, int a0, int n) {
    const int m = rows * n;
#pragma unroll 2
    for (int i = threadIdx.x; i < m; i += blockDim.x) {
        const int r = i / n, c = i - r * n;
        const int t = a0 + c;
        if (t < Lg) g[(size_t)r * Lg + t] = src.p[r * src.P + (t - src.start)];
    }
}

// ---------------------------------------------------------------------------
// Window plans.  All column counts are exact receptive-field arithmetic; the
// capacities also cover the garbage columns a 16-wide MFMA tile computes past
// the last needed position (those columns are never stored).
template <int M, int C, int TF, bool CP = false>
struct HeadPlan {
    static constexpr int C1 = C / 2;
    static constexpr int MEL_N = TF + 6;           // frames [f0-3, f0+TF+3)
    static constexpr int A0_N = TF + 4;            // input conv out  [f0-2, f0+TF+2)
    static constexpr int NQ = TF + 2;              // ConvT1 inputs   [f0-1, f0+TF+1)
    static constexpr int H_N = 4 * TF + 2;         // RB1 conv1 out   [4f0-1, 4f0+4TF+1)
    static constexpr int O_N = 4 * TF;             // RB1 out         [4f0, 4f0+4TF)
    static constexpr int P_MEL = stride_for(cmax(MEL_N, rup16(A0_N) + 2), CP);
    static constexpr int P_A0 = stride_for(cmax(A0_N, rup16(NQ) + 2), CP);
    static constexpr int P_U = stride_for(cmax(4 * NQ, rup16(H_N) + 4), CP);
    static constexpr int P_H = stride_for(cmax(H_N, rup16(O_N) + 2), CP);
    static constexpr int R0 = cmax(M * P_MEL + C * P_A0, C1 * P_H);
    static constexpr int R1 = C1 * P_U;
    static constexpr int LDS_FLOATS = R0 + R1;
};

template <int CI, int W>
struct MidPlan {  // U1 (CI ch, res 4) -> U2 (CI/2 ch, res 16); W res-4 positions
    static constexpr int CO = CI / 2;
    static constexpr int IN_N = W + 4;             // [p0-2, p0+W+2)
    static constexpr int NQ = W + 2;               // ConvT2 inputs [p0-1, p0+W+1)
    static constexpr int H_N = 4 * W + 2;          // [4p0-1, 4p0+4W+1)
    static constexpr int O_N = 4 * W;              // [4p0, 4p0+4W)
    static constexpr int P_IN = pstride(cmax(IN_N, rup16(NQ) + 2));
    static constexpr int P_U = pstride(cmax(4 * NQ, rup16(H_N) + 4));
    static constexpr int P_H = pstride(cmax(H_N, rup16(O_N) + 2));
    static constexpr int R0 = cmax(CI * P_IN, CO * P_H);
    static constexpr int R1 = CO * P_U;
    static constexpr int LDS_FLOATS = R0 + R1;
};

// Odd row stride >= cols (the two-phase layers' stride-2 B reads).
constexpr int ostride(int cols) { return ((cols + 15) / 32) * 32 + 17; }
template <int CI, int W, bool PAIR = false>
struct TailPlan {  // U2 (CI ch, res 16) -> audio (res 64); W res-16 positions
    static constexpr int C3 = CI / 2, C4 = CI / 4;
    static constexpr int IN_N = W + 8;             // [p0-4, p0+W+4)
    static constexpr int NQ3 = W + 6;              // ConvT3 inputs [p0-3, p0+W+3) -> U3 [2p0-6, ..)
    static constexpr int H3_N = 2 * W + 8;         // [2p0-4, 2p0+2W+4)
    static constexpr int O3_N = 2 * W + 6;         // [2p0-3, 2p0+2W+3)
    static constexpr int NQ4 = 2 * W + 4;          // ConvT4 inputs [2p0-2, 2p0+2W+2) -> U4 [4p0-4, ..)
    static constexpr int H4_N = 4 * W + 4;         // [4p0-2, 4p0+4W+2)
    static constexpr int O4_N = 4 * W + 2;         // [4p0-1, 4p0+4W+1)
    static constexpr int A_N = 4 * W;              // audio [4p0, 4p0+4W)
    static constexpr int P_IN = pstride(cmax(IN_N, rup16(NQ3) + 2));
    static constexpr int P_U3 = pstride(cmax(2 * NQ3, cmax(rup16(H3_N) + 3, rup16(NQ4) + 5)));
    static constexpr int P_H3 = pstride(cmax(H3_N, rup16(O3_N) + 2));
    // (PAIR: the two-phase ResBlock4 reads up to 2 x 16 columns past its last
    // needed position pair)
    static constexpr int P_U4 = PAIR ? ostride(cmax(2 * NQ4, 4 * W + 40)) : pstride(cmax(2 * NQ4, rup16(H4_N) + 3));
    static constexpr int P_H4 = PAIR ? ostride(cmax(H4_N, 4 * W + 40)) : pstride(cmax(H4_N, rup16(O4_N) + 2));
    // region A: U2in -> H3 -> U4 ; region B: U3 -> H4
    static constexpr int RA = cmax(CI * P_IN, cmax(C3 * P_H3, C4 * P_U4));
    static constexpr int RB = cmax(C3 * P_U3, C4 * P_H4);
    static constexpr int LDS_FLOATS = RA + RB;
};

// ---------------------------------------------------------------------------
// Tiling configurations.  WAVES waves per workgroup; NT_* = 16-position tiles
// per work item of each layer, chosen so every layer splits into a multiple
// of WAVES items; MINW = launch-bounds waves per SIMD (VGPR cap).
struct CfgS1W8 {  // stage1: 8 waves, <= 74 KB LDS (2 workgroups / CU)
    static constexpr int M = 64, C = 128, TF = 28, W2 = 60, W3 = 240, WAVES = 8, MINW = 5;
    static constexpr bool CP = false;
    static constexpr int NT_IN = 2, NT_T1 = 2, NT_R1 = 4, NT_T2 = 4, NT_R2 = 4, NT_T3 = 4, NT_R3 = 4, NT_T4 = 4, NT_R4 = 4;
};
struct CfgS1W16 {  // stage1: 16 waves, one workgroup per CU (152/132/131 KB LDS)
    static constexpr int M = 64, C = 128, TF = 63, W2 = 125, W3 = 500, WAVES = 16, MINW = 4;
    static constexpr bool CP = false;
    static constexpr int NT_IN = 3, NT_T1 = 5, NT_R1 = 4, NT_T2 = 4, NT_R2 = 4, NT_T3 = 4, NT_R3 = 4, NT_T4 = 8, NT_R4 = 8;
};
struct CfgS1W16s {  // CfgS1W16 with ~2-3 smaller work items per wave for the dynamic schedule
    static constexpr int M = 64, C = 128, TF = 63, W2 = 125, W3 = 500, WAVES = 16, MINW = 4;
    static constexpr bool CP = false;
    static constexpr int NT_IN = 2, NT_T1 = 2, NT_R1 = 2, NT_T2 = 2, NT_R2 = 2, NT_T3 = 2, NT_R3 = 2, NT_T4 = 4, NT_R4 = 4;
};
// The 16-wave tiling's mid and tail as two 8-wave workgroups per CU (the
// windows halved: 1,024 workgroups at B=32 T=500, two rounds as before), so
// one workgroup's layer barriers overlap the other's MFMA chains (M2_F32_MT).
// Measured in one process, B=32 T=500 with the two-phase tail layers
// (profiles/r06/r06z3_mt.txt): the tail 0.1986 -> 0.1948 ms per call (the
// default, M2_F32_MT=2); the mid 0.228 (its 63-position windows re-read
// twice the halo).
struct CfgS1T8 {
    static constexpr int M = 64, C = 128, TF = 28, W2 = 63, W3 = 250, WAVES = 8, MINW = 5;
    static constexpr bool CP = false;
    static constexpr int NT_IN = 2, NT_T1 = 2, NT_R1 = 4, NT_T2 = 4, NT_R2 = 4, NT_T3 = 4, NT_R3 = 4, NT_T4 = 4, NT_R4 = 4;
};
struct CfgS2W8 {
    static constexpr int M = 80, C = 256, TF = 12, W2 = 28, W3 = 120, WAVES = 8, MINW = 5;
    static constexpr bool CP = false;
    static constexpr int NT_IN = 2, NT_T1 = 2, NT_R1 = 4, NT_T2 = 4, NT_R2 = 4, NT_T3 = 4, NT_R3 = 4, NT_T4 = 4, NT_R4 = 4;
};
struct CfgTinyW8 {  // M2TTSModel(hidden 32, mel 32, vocoder 64) as in the reference smoke tests
    static constexpr int M = 32, C = 64, TF = 28, W2 = 60, W3 = 240, WAVES = 8, MINW = 5;
    static constexpr bool CP = false;
    static constexpr int NT_IN = 2, NT_T1 = 2, NT_R1 = 4, NT_T2 = 4, NT_R2 = 4, NT_T3 = 4, NT_R3 = 4, NT_T4 = 4, NT_R4 = 4;
};

// Diagnostic build only (-DM2_STAMPS): per-wave s_memtime stamps at phase
// boundaries, [kernel][workgroup][wave][16]; never part of the product build.
#ifdef M2_STAMPS
__device__ unsigned long long g_stamps[3][4096][16][16];
#define STAMP(K, i)                                                                                      \
    do {                                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        unsigned long long _t;                                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                      \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        const int _wg = blockIdx.y * gridDim.x + blockIdx.x;                                             \
        if ((threadIdx.x & 63) == 0 && _wg < 4096) g_stamps[K][_wg][threadIdx.x >> 6][i] = _t;           \
    } while (0)
#else
#define STAMP(K, i) \
    do {            \
    } while (0)
#endif

// The three kernels' bodies are device functions of the window (bx, b), so
// the guarded redo below can run them from one persistent launch.
// COMP: the input conv composed into ConvT1 (lconvT1c), one layer and one
// barrier fewer.
template <class Cfg, bool TRANS, bool COMP = false>
__device__ __forceinline__ void voc_head_body(int bx, int b, const float* __restrict__ mel, int T, const VocW& w,
                                              float* __restrict__ U1) {
    constexpr int M = Cfg::M, C = Cfg::C, TF = Cfg::TF;
    using Pl = HeadPlan<M, C, TF, Cfg::CP>;
    constexpr int C1 = Pl::C1;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int f0 = bx * TF;
    if (w.dT) {  // speculative launch: T was the capacity
        T = dev_frames(w.dT, T);
        if (f0 >= T) return;
    }
    __shared__ int ctr[8];  // per-layer work counters (32 B: keeps the dynamic LDS base 16-B aligned)
    if (threadIdx.x < 8) ctr[threadIdx.x] = 0;
    LB melw{lds, Pl::P_MEL, f0 - 3};
    LB a0w{lds + M * Pl::P_MEL, Pl::P_A0, f0 - 2};
    LB hw{lds, Pl::P_H, 4 * f0 - 1};
    LB uw{lds + Pl::R0, Pl::P_U, 4 * f0 - 4};
    STAMP(0, 0);
    gload<TRANS>(mel + (size_t)b * M * T, M, T, melw, Pl::MEL_N);
    STAMP(0, 1);
    __syncthreads();
    STAMP(0, 2);
    if constexpr (COMP) {
        // the edge terms (workgroup-uniform: the windows holding frame 0 or T - 1)
        const bool left = f0 == 0, right = T - 1 >= f0 - 1 && T - 1 <= f0 + TF;
        float* corr = a0w.p;  // the a0 rows are not used by the composed form
        if (left || right) {
            head_f32_corr<M, C1>(w.hce, melw, T, left, right, corr);
            __syncthreads();
        }
        STAMP(0, 3);
        STAMP(0, 4);
        lconvT1c<M, C1, Cfg::NT_T1, Pl::P_MEL>(w.hcw, w.hcb, melw, uw, f0 - 1, Pl::NQ, T, (left || right) ? corr : nullptr,
                                              ctr + 1);
    } else {
        lconv3<M, C, Cfg::NT_IN, ACT_NONE, false, Pl::P_MEL>(w.wi, w.bi, melw, a0w, f0 - 2, Pl::A0_N, T, ctr + 0);
        STAMP(0, 3);
        __syncthreads();
        STAMP(0, 4);
        lconvT<C, C1, 4, Cfg::NT_T1, Pl::P_A0>(w.wt[0], w.bt[0], a0w, uw, f0 - 1, Pl::NQ, 4 * T, ctr + 1);
    }
    STAMP(0, 5);
    __syncthreads();
    STAMP(0, 6);
    lconv3<C1, C1, Cfg::NT_R1, ACT_LEAKY, false, Pl::P_U>(w.w1[0], w.b1[0], uw, hw, 4 * f0 - 1, Pl::H_N, 4 * T, ctr + 2);
    STAMP(0, 7);
    __syncthreads();
    STAMP(0, 8);
    lconv3<C1, C1, Cfg::NT_R1, ACT_NONE, true, Pl::P_H>(w.w2[0], w.b2[0], hw, uw, 4 * f0, Pl::O_N, 4 * T, ctr + 3);
    STAMP(0, 9);
    __syncthreads();
    STAMP(0, 10);
    gstore(U1 + (size_t)b * C1 * 4 * T, C1, 4 * T, uw, 4 * f0, Pl::O_N);
    STAMP(0, 11);
}

template <class Cfg>
__device__ __forceinline__ void voc_mid_body(int bx, int b, const float* __restrict__ U1, int L1, const VocW& w,
                                             float* __restrict__ U2) {
    constexpr int CI = Cfg::C / 2, W = Cfg::W2;
    using Pl = MidPlan<CI, W>;
    constexpr int CO = Pl::CO;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int p0 = bx * W;
    if (w.dT) {  // speculative launch: L1 was the capacity
        L1 = 4 * dev_frames(w.dT, L1 / 4);
        if (p0 >= L1) return;
    }
    __shared__ int ctr[8];  // per-layer work counters (32 B: keeps the dynamic LDS base 16-B aligned)
    if (threadIdx.x < 8) ctr[threadIdx.x] = 0;
    const int L2 = 4 * L1;
    LB inw{lds, Pl::P_IN, p0 - 2};
    LB hw{lds, Pl::P_H, 4 * p0 - 1};
    LB uw{lds + Pl::R0, Pl::P_U, 4 * p0 - 4};
    STAMP(1, 0);
    gload<false>(U1 + (size_t)b * CI * L1, CI, L1, inw, Pl::IN_N);
    STAMP(1, 1);
    __syncthreads();
    STAMP(1, 2);
    lconvT<CI, CO, 4, Cfg::NT_T2, Pl::P_IN>(w.wt[1], w.bt[1], inw, uw, p0 - 1, Pl::NQ, L2, ctr + 0);
    STAMP(1, 3);
    __syncthreads();
    STAMP(1, 4);
    lconv3<CO, CO, Cfg::NT_R2, ACT_LEAKY, false, Pl::P_U>(w.w1[1], w.b1[1], uw, hw, 4 * p0 - 1, Pl::H_N, L2, ctr + 1);
    STAMP(1, 5);
    __syncthreads();
    STAMP(1, 6);
    lconv3<CO, CO, Cfg::NT_R2, ACT_NONE, true, Pl::P_H>(w.w2[1], w.b2[1], hw, uw, 4 * p0, Pl::O_N, L2, ctr + 2);
    STAMP(1, 7);
    __syncthreads();
    STAMP(1, 8);
    gstore(U2 + (size_t)b * CO * L2, CO, L2, uw, 4 * p0, Pl::O_N);
    STAMP(1, 9);
}

// PAIR: ConvT4 and ResBlock4 in the two-phase forms (8-channel stages only).
template <class Cfg, bool PAIR = false>
__device__ __forceinline__ void voc_tail_body(int bx, int b, const float* __restrict__ U2, int L2, const VocW& w,
                                              float* __restrict__ audio) {
    constexpr int CI = Cfg::C / 4, W = Cfg::W3;
    static_assert(!PAIR || CI / 4 == 8, "two-phase tail layers need 8 channels");
    using Pl = TailPlan<CI, W, PAIR>;
    constexpr int C3 = Pl::C3, C4 = Pl::C4;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int p0 = bx * W;
    if (w.dT) {  // speculative launch: L2 was the capacity
        L2 = 16 * dev_frames(w.dT, L2 / 16);
        if (p0 >= L2) return;
    }
    __shared__ int ctr[8];  // per-layer work counters (32 B: keeps the dynamic LDS base 16-B aligned)
    if (threadIdx.x < 8) ctr[threadIdx.x] = 0;
    const int L3 = 2 * L2, L4 = 4 * L2;
    float* ra = lds;
    float* rb = lds + Pl::RA;
    LB inw{ra, Pl::P_IN, p0 - 4};
    LB u3{rb, Pl::P_U3, 2 * p0 - 6};
    LB h3{ra, Pl::P_H3, 2 * p0 - 4};
    LB u4{ra, Pl::P_U4, 4 * p0 - 4};
    LB h4{rb, Pl::P_H4, 4 * p0 - 2};
    STAMP(2, 0);
    gload<false>(U2 + (size_t)b * CI * L2, CI, L2, inw, Pl::IN_N);
    __syncthreads();
    STAMP(2, 1);
    lconvT<CI, C3, 2, Cfg::NT_T3, Pl::P_IN>(w.wt[2], w.bt[2], inw, u3, p0 - 3, Pl::NQ3, L3, ctr + 0);
    STAMP(2, 2);
    __syncthreads();
    STAMP(2, 3);
    lconv3<C3, C3, Cfg::NT_R3, ACT_LEAKY, false, Pl::P_U3>(w.w1[2], w.b1[2], u3, h3, 2 * p0 - 4, Pl::H3_N, L3, ctr + 1);
    STAMP(2, 4);
    __syncthreads();
    STAMP(2, 5);
    lconv3<C3, C3, Cfg::NT_R3, ACT_NONE, true, Pl::P_H3>(w.w2[2], w.b2[2], h3, u3, 2 * p0 - 3, Pl::O3_N, L3, ctr + 2);
    STAMP(2, 6);
    __syncthreads();
    STAMP(2, 7);
    // (PAIR: half the column tiles per item, so the phase-merged layers keep
    // every wave busy)
    if constexpr (PAIR)
        lconvT2p<C3, cmax(1, Cfg::NT_T4 / 2), Pl::P_U3>(w.wt4p, w.bt[3], u3, u4, 2 * p0 - 2, Pl::NQ4, L4, ctr + 3);
    else
        lconvT<C3, C4, 2, Cfg::NT_T4, Pl::P_U3>(w.wt[3], w.bt[3], u3, u4, 2 * p0 - 2, Pl::NQ4, L4, ctr + 3);
    STAMP(2, 8);
    __syncthreads();
    STAMP(2, 9);
    if constexpr (PAIR)
        lconv3_2p<cmax(1, Cfg::NT_R4 / 2), ACT_LEAKY, false, Pl::P_U4>(w.w1p, w.b1[3], u4, h4, 4 * p0 - 2, Pl::H4_N, L4, ctr + 4);
    else
        lconv3<C4, C4, Cfg::NT_R4, ACT_LEAKY, false, Pl::P_U4>(w.w1[3], w.b1[3], u4, h4, 4 * p0 - 2, Pl::H4_N, L4,
                                                                ctr + 4);
    STAMP(2, 10);
    __syncthreads();
    STAMP(2, 11);
    if constexpr (PAIR)
        lconv3_2p<cmax(1, Cfg::NT_R4 / 2), ACT_NONE, true, Pl::P_H4>(w.w2p, w.b2[3], h4, u4, 4 * p0 - 1, Pl::O4_N, L4, ctr + 5);
    else
        lconv3<C4, C4, Cfg::NT_R4, ACT_NONE, true, Pl::P_H4>(w.w2[3], w.b2[3], h4, u4, 4 * p0 - 1, Pl::O4_N, L4,
                                                              ctr + 5);
    STAMP(2, 12);
    __syncthreads();
    STAMP(2, 13);
    // output_conv (C4 -> 1, k3) + tanh: VALU, one position per thread, coalesced stores.
    float* arow = audio + (size_t)b * L4;
    const float bo = w.bo[0];
    for (int j = threadIdx.x; j < Pl::A_N; j += blockDim.x) {
        const int t = 4 * p0 + j;
        if (t < L4) {
            const float* x = u4.p + (t - 1 - u4.start);
            float acc = 0.f;
#pragma unroll
            for (int ci = 0; ci < C4; ++ci) {
                acc = fmaf(w.wo[ci * 3 + 0], x[ci * u4.P + 0], acc);
                acc = fmaf(w.wo[ci * 3 + 1], x[ci * u4.P + 1], acc);
                acc = fmaf(w.wo[ci * 3 + 2], x[ci * u4.P + 2], acc);
            }
            arow[t] = tanhf(acc + bo);
        }
    }
    STAMP(2, 14);
}

template <class Cfg, bool TRANS, bool COMP = false>
__global__ __launch_bounds__(Cfg::WAVES * 64, Cfg::MINW) void voc_head_kernel(const float* __restrict__ mel, int T,
                                                                             VocW w, float* __restrict__ U1) {
    voc_head_body<Cfg, TRANS, COMP>(blockIdx.x, blockIdx.y, mel, T, w, U1);
}
template <class Cfg>
__global__ __launch_bounds__(Cfg::WAVES * 64, Cfg::MINW) void voc_mid_kernel(const float* __restrict__ U1, int L1,
                                                                            VocW w, float* __restrict__ U2) {
    voc_mid_body<Cfg>(blockIdx.x, blockIdx.y, U1, L1, w, U2);
}
template <class Cfg, bool PAIR = false>
__global__ __launch_bounds__(Cfg::WAVES * 64, Cfg::MINW) void voc_tail_kernel(const float* __restrict__ U2, int L2,
                                                                             VocW w, float* __restrict__ audio) {
    voc_tail_body<Cfg, PAIR>(blockIdx.x, blockIdx.y, U2, L2, w, audio);
}

// The range policy's on-device redo (m2_set_range_policy "fallback"): ONE
// launch after the split-f16 kernels.  Every workgroup returns at once unless
// the call's flag word (*w.guard) is raised; then the workgroups claim the
// exact-f32 head, mid and tail windows from one ordered queue (q[0]) and a
// mid (tail) window waits until every head (mid) window is published (q[1],
// q[2]).  A workgroup only ever waits for windows claimed before its own, by
// workgroups already running, so any number of resident workgroups finishes
// (no co-residency assumption).  Publication: every wave's stores are written
// back (agent-scope release fence) before the count; a waiter acquires after
// it (U1 / U2 cross XCDs, whose L2s are not coherent).  The four words are
// zeroed by the call's first (x3 head) kernel (VocX::rqueue), so a redo that
// stopped early cannot leave the next one's queue claimed.
__device__ __forceinline__ void redo_publish(unsigned* c) {
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(c, 1u);
}
__device__ __forceinline__ void redo_wait(unsigned* c, unsigned n) {
    if (threadIdx.x == 0)
        while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    __threadfence();
}
// Compiled for one workgroup per CU (WAVES / 4 waves per SIMD): the three
// bodies in one loop need more registers than each kernel's own occupancy
// target leaves (at MINW they spilled 52-73 VGPRs), and the redo's speed
// matters less than the split kernels' (it runs only for out-of-range calls).
template <class Cfg, bool TRANS, bool PAIR = false, bool COMP = false>
__global__ __launch_bounds__(Cfg::WAVES * 64, Cfg::WAVES / 4) void voc_redo_kernel(const float* __restrict__ mel, int B,
                                                                             int T, VocW w, float* __restrict__ U1,
                                                                             float* __restrict__ U2,
                                                                             float* __restrict__ audio,
                                                                             unsigned* __restrict__ q) {
    if (*w.guard == 0) return;  // the split-f16 result is finite: nothing to redo
    const int hx = (T + Cfg::TF - 1) / Cfg::TF, mx = (4 * T + Cfg::W2 - 1) / Cfg::W2, tx = (16 * T + Cfg::W3 - 1) / Cfg::W3;
    const int nh = hx * B, nm = mx * B, nt = tx * B;
    __shared__ int item;
    for (;;) {
        __syncthreads();  // the previous window is done with LDS and `item`
        if (threadIdx.x == 0) item = (int)atomicAdd(q, 1u);
        __syncthreads();
        const int i = item;
        if (i >= nh + nm + nt) break;
        if (i < nh) {
            voc_head_body<Cfg, TRANS, COMP>(i % hx, i / hx, mel, T, w, U1);
            redo_publish(q + 1);
        } else if (i < nh + nm) {
            redo_wait(q + 1, (unsigned)nh);
            voc_mid_body<Cfg>((i - nh) % mx, (i - nh) / mx, U1, 4 * T, w, U2);
            redo_publish(q + 2);
        } else {
            redo_wait(q + 2, (unsigned)nm);
            voc_tail_body<Cfg, PAIR>((i - nh - nm) % tx, (i - nh - nm) / tx, U2, 16 * T, w, audio);
        }
    }
}

// ---------------------------------------------------------------------------
namespace {
template <typename K>
int32_t set_lds(K kernel, size_t bytes) {
    M2_CHECK_SHAPE(bytes <= 160 * 1024, "fused vocoder: LDS plan exceeds 160 KiB");
    M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes));
    return M2_OK;
}

template <class Cfg, bool PAIR = false, bool COMP = false>
int32_t voc_redo(const float* mel, bool trans, int B, int T, const VocW& w, float* U1, float* U2, float* audio,
                 hipStream_t st) {
    using HP = HeadPlan<Cfg::M, Cfg::C, Cfg::TF, Cfg::CP>;
    using MP = MidPlan<Cfg::C / 2, Cfg::W2>;
    using TP = TailPlan<Cfg::C / 4, Cfg::W3, PAIR>;
    constexpr int threads = Cfg::WAVES * 64;
    constexpr size_t lds = 4 * (size_t)std::max(std::max(HP::LDS_FLOATS, MP::LDS_FLOATS), TP::LDS_FLOATS);
    static int full = 0, cus = 0;
    if (!full) {
        int32_t rc;
        if ((rc = set_lds(voc_redo_kernel<Cfg, false, PAIR, COMP>, lds))) return rc;
        if ((rc = set_lds(voc_redo_kernel<Cfg, true, PAIR, COMP>, lds))) return rc;
        int occ = 0, dev = 0;
        M2_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, voc_redo_kernel<Cfg, false, PAIR, COMP>, threads, lds));
        M2_HIP(hipGetDevice(&dev));
        M2_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
        cus = std::max(1, cus);
        full = std::max(1, occ) * cus;
    }
    // workgroups of the (usually empty) launch: one per CU by default; the
    // ordered queue needs no co-residency, so any count is correct
    // (M2_REDO_GRID=n forces n, 0 = every resident slot)
    const int grid = sw().redo_grid < 0 ? cus : (sw().redo_grid == 0 ? full : sw().redo_grid);
    unsigned* q = const_cast<unsigned*>(reinterpret_cast<const unsigned*>(w.guard_queue));
    if (trans)
        hipLaunchKernelGGL((voc_redo_kernel<Cfg, true, PAIR, COMP>), dim3(grid), dim3(threads), lds, st, mel, B, T, w, U1, U2, audio,
                           q);
    else
        hipLaunchKernelGGL((voc_redo_kernel<Cfg, false, PAIR, COMP>), dim3(grid), dim3(threads), lds, st, mel, B, T, w, U1, U2,
                           audio, q);
    M2_LAUNCHED("voc_redo_kernel");
    return M2_OK;
}

// The redo's tiling: the 8-wave form of the stage (every stage1 tiling packs
// the same weights and writes the same U1 / U2 / audio), so it gets up to 256
// VGPRs per lane at one workgroup per CU.
template <class Cfg> struct RedoCfg { using type = Cfg; };
template <> struct RedoCfg<CfgS1W16> { using type = CfgS1W8; };
template <> struct RedoCfg<CfgS1W16s> { using type = CfgS1W8; };

// MCfg / TCfg: the mid's / tail's tiling (windows W2 / W3, waves), by
// default the head's.
// PAIR: the tail's 8-channel layers in the two-phase forms (lconvT2p /
// lconv3_2p), in the guarded redo as well.
template <class Cfg, class MCfg = Cfg, class TCfg = Cfg, bool PAIR = false, bool COMP = false>
int32_t voc_fused(const float* mel, bool trans, int B, int T, const VocW& w, float* U1, float* U2, float* audio,
                  hipStream_t st, const std::function<void(int, bool)>& mark) {
    if (w.guard) return voc_redo<typename RedoCfg<Cfg>::type, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st);
    using HP = HeadPlan<Cfg::M, Cfg::C, Cfg::TF, Cfg::CP>;
    using MP = MidPlan<MCfg::C / 2, MCfg::W2>;
    using TP = TailPlan<TCfg::C / 4, TCfg::W3, PAIR>;
    constexpr int threads = Cfg::WAVES * 64;
    static bool attr = false;
    if (!attr) {
        int32_t rc;
        if ((rc = set_lds(voc_head_kernel<Cfg, false, COMP>, HP::LDS_FLOATS * 4))) return rc;
        if ((rc = set_lds(voc_head_kernel<Cfg, true, COMP>, HP::LDS_FLOATS * 4))) return rc;
        if ((rc = set_lds(voc_mid_kernel<MCfg>, MP::LDS_FLOATS * 4))) return rc;
        if ((rc = set_lds(voc_tail_kernel<TCfg, PAIR>, TP::LDS_FLOATS * 4))) return rc;
        attr = true;
    }
    mark(0, true);
    if (trans)
        hipLaunchKernelGGL((voc_head_kernel<Cfg, true, COMP>), dim3(cdiv(T, Cfg::TF), B), dim3(threads), HP::LDS_FLOATS * 4,
                           st, mel, T, w, U1);
    else
        hipLaunchKernelGGL((voc_head_kernel<Cfg, false, COMP>), dim3(cdiv(T, Cfg::TF), B), dim3(threads), HP::LDS_FLOATS * 4,
                           st, mel, T, w, U1);
    mark(0, false);
    M2_LAUNCHED("voc_head_kernel");
    mark(1, true);
    hipLaunchKernelGGL((voc_mid_kernel<MCfg>), dim3(cdiv(4 * T, MCfg::W2), B), dim3(MCfg::WAVES * 64), MP::LDS_FLOATS * 4,
                       st, U1, 4 * T, w, U2);
    mark(1, false);
    M2_LAUNCHED("voc_mid_kernel");
    mark(2, true);
    hipLaunchKernelGGL((voc_tail_kernel<TCfg, PAIR>), dim3(cdiv(16 * T, TCfg::W3), B), dim3(TCfg::WAVES * 64),
                       TP::LDS_FLOATS * 4, st, U2, 16 * T, w, audio);
    mark(2, false);
    M2_LAUNCHED("voc_tail_kernel");
    return M2_OK;
}

template <bool PAIR, bool COMP>
int32_t s1_fused(const float* mel, bool trans, int B, int T, const VocW& w, float* U1, float* U2, float* audio,
                 hipStream_t st, const std::function<void(int, bool)>& mark, bool w16, int plan) {
    if (plan == 3)
        return voc_fused<CfgS1W16s, CfgS1W16s, CfgS1W16s, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st, mark);
    if (w16) {
        switch (sw().f32_mt) {
            case 1:
                return voc_fused<CfgS1W16, CfgS1T8, CfgS1W16, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st, mark);
            case 2:
                return voc_fused<CfgS1W16, CfgS1W16, CfgS1T8, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st, mark);
            case 3:
                return voc_fused<CfgS1W16, CfgS1T8, CfgS1T8, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st, mark);
            case 4:  // the mid's items halved (two per wave), the tail on half windows: 0.1843 ->
                     // 0.1894 ms alternated (profiles/r06/r06z14_mid_items.txt), a switch only
                return voc_fused<CfgS1W16, CfgS1W16s, CfgS1T8, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st, mark);
            default:
                return voc_fused<CfgS1W16, CfgS1W16, CfgS1W16, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st,
                                                                           mark);
        }
    }
    return voc_fused<CfgS1W8, CfgS1W8, CfgS1W8, PAIR, COMP>(mel, trans, B, T, w, U1, U2, audio, st, mark);
}
}  // namespace

bool vocoder_fused_supported(int M, int C) {
    return (M == 64 && C == 128) || (M == 80 && C == 256) || (M == 32 && C == 64);
}

int32_t launch_vocoder_fused(const float* mel, bool trans, int M, int C, int B, int T, const VocW& w, float* U1,
                             float* U2, float* audio, hipStream_t st,
                             const std::function<void(int, bool)>& mark) {
    if (B == 0 || T == 0) return M2_OK;
    const int plan = sw().voc_plan;
    if (M == 64 && C == 128) {
        // Workgroup rounds: one 16-wave WG per CU; 8-wave WGs pair up.  Pick the
        // tiling whose workgroup count wastes the least of its last round.
        const int n16 = B * cdiv(T, CfgS1W16::TF), n8 = B * cdiv(T, CfgS1W8::TF);
        const double waste16 = (double)cdiv(n16, 256) * 256 / n16, waste8 = (double)cdiv(n8, 512) * 512 / n8;
        const bool w16 = plan == 2 || (plan < 0 && waste16 <= waste8);
        const bool pair = sw().f32_pair && w.wt4p, comp = sw().f32_comp && w.hcw;
        if (pair && comp) return s1_fused<true, true>(mel, trans, B, T, w, U1, U2, audio, st, mark, w16, plan);
        if (pair) return s1_fused<true, false>(mel, trans, B, T, w, U1, U2, audio, st, mark, w16, plan);
        if (comp) return s1_fused<false, true>(mel, trans, B, T, w, U1, U2, audio, st, mark, w16, plan);
        return s1_fused<false, false>(mel, trans, B, T, w, U1, U2, audio, st, mark, w16, plan);
    }
    if (M == 80 && C == 256) {
        if (sw().f32_comp && w.hcw)
            return voc_fused<CfgS2W8, CfgS2W8, CfgS2W8, false, true>(mel, trans, B, T, w, U1, U2, audio, st, mark);
        return voc_fused<CfgS2W8>(mel, trans, B, T, w, U1, U2, audio, st, mark);
    }
    if (M == 32 && C == 64) return voc_fused<CfgTinyW8>(mel, trans, B, T, w, U1, U2, audio, st, mark);
    return fail(M2_E_SHAPE, "fused vocoder: unsupported (mel_channels, vocoder_channels)");
}

#ifdef M2_STAMPS
extern "C" int32_t m2_debug_stamps(void* host, size_t bytes) {
    return (int32_t)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes < sizeof(g_stamps) ? bytes : sizeof(g_stamps));
}
#endif

const char* const kVocKernelNames[kVocKernels] = {
    "voc_head_kernel (input_conv + ConvT1 + ResBlock1)",
    "voc_mid_kernel (ConvT2 + ResBlock2)",
    "voc_tail_kernel (ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv)"};

// Index of A-fragment element (m-block mb, k-step s, lane) in the packed
// layout [mb][s/4][lane][s%4] with KSP (k-steps rounded up to 4) per m-block.
static inline size_t apack_index(int mb, int s, int lane, int KSP) {
    return (((size_t)mb * (KSP / 4) + s / 4) * 64 + lane) * 4 + (s % 4);
}

std::vector<float> pack_conv3(const float* W, int Cout, int Cin) {
    const int MB = (Cout + 15) / 16, KS = 3 * Cin / 4, KSP = (KS + 3) / 4 * 4;
    std::vector<float> out((size_t)MB * KSP * 64, 0.f);
    for (int mb = 0; mb < MB; ++mb)
        for (int s = 0; s < KS; ++s)
            for (int lane = 0; lane < 64; ++lane) {
                const int co = mb * 16 + (lane & 15), kk = 4 * s + (lane >> 4);
                const int k = kk / Cin, ci = kk % Cin;
                if (co < Cout) out[apack_index(mb, s, lane, KSP)] = W[((size_t)co * Cin + ci) * 3 + k];
            }
    return out;
}

// input_conv o ConvT1 for the exact-f32 head (lconvT1c), composed in double:
// Wc(ph, co, m, kk) as pack_x3_head_comp, packed [ph][mb][s][lane][s % 4] with
// K index kk * M + m (4 taps x M mel channels).
std::vector<float> pack_f32_head_comp(const float* Win, const float* WT, int M, int C) {
    const int C1 = C / 2, R = 4, P = R / 2, MB = (C1 + 15) / 16, KS = M, KSP = (KS + 3) / 4 * 4;
    auto kj = [&](int ph, int j) {
        const int k0 = (ph + P < R) ? ph + P : ph + P - R, k1 = (ph + P < R) ? ph + P + R : ph + P;
        return j ? k1 : k0;
    };
    std::vector<double> wc((size_t)R * C1 * M * 4, 0.0);  // [ph][co][m][kk]
    for (int ph = 0; ph < R; ++ph)
        for (int co = 0; co < C1; ++co)
            for (int j = 0; j < 2; ++j) {
                const int k = kj(ph, j);
                for (int ci = 0; ci < C; ++ci) {
                    const double a = WT[((size_t)ci * C1 + co) * 2 * R + k];
                    for (int tin = 0; tin < 3; ++tin) {
                        const int kk = j + 2 - tin;
                        for (int m = 0; m < M; ++m)
                            wc[(((size_t)ph * C1 + co) * M + m) * 4 + kk] += a * (double)Win[((size_t)ci * M + m) * 3 + tin];
                    }
                }
            }
    std::vector<float> out((size_t)R * MB * KSP * 64, 0.f);
    for (int ph = 0; ph < R; ++ph)
        for (int mb = 0; mb < MB; ++mb)
            for (int s = 0; s < KS; ++s)
                for (int lane = 0; lane < 64; ++lane) {
                    const int co = mb * 16 + (lane & 15), k = 4 * s + (lane >> 4), kk = k / M, m = k % M;
                    if (co < C1) out[apack_index(ph * MB + mb, s, lane, KSP)] = (float)wc[(((size_t)ph * C1 + co) * M + m) * 4 + kk];
                }
    return out;
}

// Two-phase ConvT4 (lconvT2p): ConvTranspose1d(k=4, s=2, p=1), W [Cin][8][4],
// as a k3 conv over input positions with rows (phase, co): tap d = k - 1,
// out[2q] = x[q] W1 + x[q-1] W3, out[2q+1] = x[q+1] W0 + x[q] W2.
std::vector<float> pack_convT2_paired(const float* W, int Cin) {
    std::vector<float> d((size_t)16 * Cin * 3, 0.f);  // [row][ci][k] as pack_conv3 reads it
    for (int co = 0; co < 8; ++co)
        for (int ci = 0; ci < Cin; ++ci) {
            const float* w = W + ((size_t)ci * 8 + co) * 4;
            d[((size_t)co * Cin + ci) * 3 + 0] = w[3];
            d[((size_t)co * Cin + ci) * 3 + 1] = w[1];
            d[((size_t)(8 + co) * Cin + ci) * 3 + 1] = w[2];
            d[((size_t)(8 + co) * Cin + ci) * 3 + 2] = w[0];
        }
    return pack_conv3(d.data(), 16, Cin);
}

// Two-phase 8-channel k3 conv (lconv3_2p), W [8][8][3]: A[row = 8p + co]
// [kk = 8 tap + ci] = W[co][ci][tap - p] for tap - p in 0..2 (tap t reads
// position a0 + 2j + t - 1).
std::vector<float> pack_conv3_2p(const float* W) {
    const int KS = 8, KSP = 8;
    std::vector<float> out((size_t)KSP * 64, 0.f);
    for (int s = 0; s < KS; ++s)
        for (int lane = 0; lane < 64; ++lane) {
            const int row = lane & 15, p = row >> 3, co = row & 7, kk = 4 * s + (lane >> 4);
            const int tap = kk / 8, ci = kk % 8, k = tap - p;
            if (k >= 0 && k <= 2) out[apack_index(0, s, lane, KSP)] = W[((size_t)co * 8 + ci) * 3 + k];
        }
    return out;
}

std::vector<float> pack_convT(const float* W, int Cin, int Cout, int R) {
    const int MB = (Cout + 15) / 16, KS = 2 * Cin / 4, P = R / 2, KSP = (KS + 3) / 4 * 4;
    std::vector<float> out((size_t)R * MB * KSP * 64, 0.f);
    for (int ph = 0; ph < R; ++ph) {
        const int k0 = (ph + P < R) ? ph + P : ph + P - R;  // tap 0: x[q] or x[q+1]
        const int k1 = (ph + P < R) ? ph + P + R : ph + P;  // tap 1: x[q-1] or x[q]
        for (int mb = 0; mb < MB; ++mb)
            for (int s = 0; s < KS; ++s)
                for (int lane = 0; lane < 64; ++lane) {
                    const int co = mb * 16 + (lane & 15), kk = 4 * s + (lane >> 4);
                    const int tap = kk / Cin, ci = kk % Cin;
                    const int k = tap ? k1 : k0;
                    if (co < Cout) out[apack_index(ph * MB + mb, s, lane, KSP)] = W[((size_t)ci * Cout + co) * 2 * R + k];
                }
    }
    return out;
}

}  // namespace m2
