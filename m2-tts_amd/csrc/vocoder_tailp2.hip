// Pipelined SimpleVocoder tail for stage2 (C = 256; tts_model.py:279-297, the
// last two upsampling stages): ConvT3 (64 -> 32 channels, x2) + leaky,
// ResBlock3, ConvT4 (32 -> 16, x2) + leaky, ResBlock4, output_conv (16 -> 1)
// + tanh, split-f16 arithmetic (vocoder_x3.hip).  The stage1 design of
// vocoder_tailp.hip at twice the channels: every signal is a 64-row column
// over the columns q of U2 (64 channels at 16T):
//   u3 (ConvT3 out, ResBlock3)  2 phases x 32 channels, row 32 p3 + c
//   u4 (ConvT4 out, ResBlock4)  4 phases x 16 channels, row 16 p4 + c
//   audio                       4 phases x 1 channel
// and every layer is a k3-over-q convolution of 64 output rows (4 m-blocks)
// whose K is a list of (dq, input octet) slots (tp2::kslot).  A layer's
// weights (8-16 fragment pairs per m-block pair) no longer fit one wave, so
// each layer runs on two waves of two m-blocks each, paired so that a wave's
// m-blocks read the same B fragments where the slots allow:
//   ConvT3    wave w = output phase w (both read columns q and q -1 / q + 1)
//   ResBlock3 wave w = phase w (taps (dq, phase) of t3 - 1, t3, t3 + 1)
//   ConvT4    wave 0 = phases 1, 2 (both read column q only), wave 1 = 0, 3
//   ResBlock4 wave w = phases 2w, 2w + 1 (16-channel units p-1 .. p+2 of the
//             unit sequence (q-1, 3), (q, 0..3), (q+1, 0), two per fragment)
//   output_conv one wave, one m-block (rows 0-3 = the 4 audio phases)
// 13 layer waves + 1 loader wave, one workgroup per CU (104 KB of rings).
// Pipeline protocol, warm-up chunk, zero columns outside [0, L2), lean
// epilogues and the identity-A residual MFMAs are those of vocoder_tailp.hip.
// Default (NL = 6): ResBlock4's conv2 and output_conv composed into one layer
// on one wave (outc2_role; the stage1 tail's outc_role at 16 channels): 11
// layer waves + the loader, 92 KB of rings, one pipeline step fewer.
// M2_TAILP2_SEVEN=1 keeps the seven-layer form.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "m2_common.h"
#include "vocoder_fused.h"

namespace m2 {
namespace tp2 {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef vx_u32x4 u32x4;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS rings: R0 = U2, R(l+1) = output of layer l; a ring row is one column as
// a 128-B hi row (64 f16) in the hi plane and a 128-B lo row kLoOff(n) bytes
// later.  Octet o of row r sits at 16 * (o ^ (r & 7)): every fragment read
// (ds_read_b128), residual read and epilogue store (ds_write_b128) of the
// kernel is then bank-conflict free (tools/probe/tailp2_banks.py models them
// all).  R6 holds 3 chunks of 16 columns (its only reader is one step behind
// the writer; R0 too with the register loader), the others 4.
// TAILP2_DMA (default): U2 into R0 by LDS-DMA, one chunk ahead, R0 4 chunks
// (loader_role_dma below; TAILP2_DMA=0 keeps the register loader, R0 3 chunks).
// Alternated twice on one box (profiles/r06/r06t_tail2_dma_ab/): tail2
// 19.38 / 19.51 -> 18.97 / 18.84 us at B=8 T=500, 146.0 / 146.4 -> 145.4 /
// 145.4 us at B=16 T=2600; 174 tests green (r06t_tests.log).
#ifndef TAILP2_DMA
#define TAILP2_DMA 1
#endif
constexpr int kRingRows[7] = {TAILP2_DMA ? 64 : 48, 64, 64, 64, 64, 64, 48};
constexpr int kRingOff(int n) { return n == 0 ? 0 : kRingOff(n - 1) + kRingRows[n - 1] * 256; }
constexpr int kLoOff(int n) { return kRingRows[n] * 128; }
constexpr int kPeriod(int n) { return kRingRows[n] / 16; }
static_assert(kRingOff(7) <= 160 * 1024, "one workgroup per CU");
// NL = 7: layers 0-5 two waves each, output conv one, loader one (14 waves);
// NL = 6: layers 0-4 two waves each, the composed layer one, loader one (12),
// plus the composed layer's edge-term slot (8 floats) after the rings.
constexpr int kCorrSlot = kRingOff(6);
constexpr int ring_bytes(int nl) { return nl == 6 ? kCorrSlot + 32 : kRingOff(7); }
// after the rings: the workgroup's non-finite-audio word (the local redo,
// vocoder_redo.h); the redo itself reuses the rings' bytes
constexpr int kFlagOff(int nl) { return ring_bytes(nl); }
constexpr int lds_bytes(int nl) { return ring_bytes(nl) + 16; }
constexpr int nwaves(int nl) { return nl == 6 ? 12 : 14; }

__device__ __forceinline__ unsigned ring_at(int n, int row, int oct) {
    return kRingOff(n) + row * 128 + 16 * (oct ^ (row & 7));
}
__device__ __forceinline__ int ring_row(int n, int j, int c) {
    const int r = 16 * j + c, R = kRingRows[n];
    return r < 0 ? r + R : (r >= R ? r - R : r);
}

__device__ __forceinline__ f32x4 mfma_h(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float tanh_fast(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)); }

constexpr int off_l(int l) { return l + 1; }
constexpr int last_step(int nch, int nl) { return nch - 1 + off_l(nl - 1); }

template <int V>
using ic = std::integral_constant<int, V>;

// ---------------------------------------------------------------------------
// Slot tables (shared by the packer and the kernel).
struct Slot {
    int dq, oct;
};
constexpr int kLayers = 7;
constexpr int nwv(int l) { return l == 6 ? 1 : 2; }   // waves of layer l
constexpr int nmbw(int l) { return l == 6 ? 1 : 2; }  // m-blocks per wave
constexpr int nkb(int l) { return l == 0 ? 4 : ((l == 1 || l == 2 || l == 6) ? 3 : 2); }
constexpr int unit0(int l) { return l == 0 ? 0 : unit0(l - 1) + nwv(l - 1) * nmbw(l - 1) * nkb(l - 1); }
constexpr int kUnits = unit0(kLayers);
constexpr int unit_of(int l, int w, int m, int kb) { return unit0(l) + (w * nmbw(l) + m) * nkb(l) + kb; }
// dense m-block (output rows 16 d .. 16 d + 15) of wave w's m-block m
constexpr int dmb(int l, int w, int m) { return l == 3 ? (w == 0 ? 1 + m : (m == 0 ? 0 : 3)) : nmbw(l) * w + m; }
constexpr int fdiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }
// 16-channel units of a 4-phase signal around column q: (q-1, 3), (q, 0..3), (q+1, 0)
constexpr Slot s4unit(int j) { return j == 0 ? Slot{-1, 3} : (j == 5 ? Slot{1, 0} : Slot{0, j - 1}); }
constexpr Slot kslot(int l, int w, int m, int kb, int g) {
    if (l == 0)  // phase w: columns (q, q-1) for phase 0, (q+1, q) for phase 1; 64 channels = 2 k-blocks each
        return Slot{kb < 2 ? (w == 0 ? 0 : 1) : (w == 0 ? -1 : 0), 4 * (kb & 1) + g};
    if (l == 1 || l == 2) {  // phase w, tap t3 + kb - 1: phase pp mod 2 of column q + floor(pp / 2)
        const int pp = w + kb - 1, dq = fdiv(pp, 2);
        return Slot{dq, 4 * (pp - 2 * dq) + g};
    }
    if (l == 3) {  // ConvT4 output phase s reads two (column, phase) slots of u3
        const int s = dmb(l, w, m);
        const int dq = s == 0 ? (kb == 0 ? 0 : -1) : (s == 3 ? (kb == 0 ? 1 : 0) : 0);
        const int ph = (s == 0 || s == 3) ? kb : 1 - kb;  // s0: (q,0) (q-1,1); s1, s2: (q,1) (q,0); s3: (q+1,0) (q,1)
        return Slot{dq, 4 * ph + g};
    }
    // ResBlock4 convs (phase p = 2w + m reads units p .. p+2) and the output conv
    // (all units): k-block kb of a wave = unit pair gi = (l == 6 ? kb : w + kb)
    const int gi = l == 6 ? kb : w + kb;
    const Slot u = s4unit(2 * gi + g / 2);
    return Slot{u.dq, 2 * u.oct + (g & 1)};
}
// The wave's distinct B fragments: ConvT4 wave 1 (phases 0, 3) reads four, one
// pair per m-block; every other wave's m-blocks share theirs (one per k-block).
constexpr int nfrag(int l, int w) { return (l == 3 && w == 1) ? 4 : nkb(l); }
constexpr int frag_of(int l, int w, int m, int kb) { return (l == 3 && w == 1) ? 2 * m + kb : kb; }
constexpr Slot fslot(int l, int w, int f, int g) {
    return (l == 3 && w == 1) ? kslot(l, w, f / 2, f % 2, g) : kslot(l, w, 0, f, g);
}
// The composed ResBlock4-conv2 + output_conv layer (outc2_role): fragments
// 0-3 on ring R5 (ResBlock4's intermediate h; the k5 taps of the 4 output
// phases read the 16-channel units (q-1, 2), (q-1, 3), (q, 0..3), (q+1, 0),
// (q+1, 1), two per fragment), 4-6 on ring R4 (ConvT4's output x; the output
// conv's units).  Weight units after kUnits, its bias (rows 0-3) after the
// seven layers' biases, then the edge terms vL[16], vR[16], kL, kR.
constexpr int kOutcF = 7, kOutcUnit0 = kUnits, kOutcBias = kLayers * 64, kOutcCorr = kOutcBias + 64;
constexpr int kBiasFloats = kOutcCorr + 64;
constexpr Slot outc_hunit(int j) { return j < 2 ? Slot{-1, 2 + j} : (j < 6 ? Slot{0, j - 2} : Slot{1, j - 6}); }
constexpr Slot outc_slot(int f, int g) {
    if (f >= 4) return kslot(6, 0, 0, f - 4, g);
    const Slot u = outc_hunit(2 * f + g / 2);
    return Slot{u.dq, 2 * u.oct + (g & 1)};
}

// One wave: layer L, half W (m-blocks dmb(L, W, 0..NMB-1)).  As in
// vocoder_tailp.hip's layer_role: weights and biases in VGPRs for the whole
// strip, LDS addresses precomputed per ring phase (the step loop is unrolled by
// the lcm of the ring periods), one fp32 accumulator per m-block for the three
// split products, identity-A MFMAs for the ResBlock residual.
template <int L, int W, int NL>
__device__ __forceinline__ void layer_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                           const u32x4* __restrict__ W_, const float* __restrict__ bias,
                                           float* __restrict__ arow, int* rflag) {
    constexpr int NMB = nmbw(L), NKB = nkb(L), NF = nfrag(L, W);
    constexpr bool RES = L == 2 || L == 5;
    constexpr int PI = kPeriod(L), PO = L < 6 ? kPeriod(L + 1) : 1, PX = RES ? kPeriod(L - 1) : 1;
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    u32x4 a[NMB][NKB][2];
    float bv[NMB][4];
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const int u = unit_of(L, W, m, kb);
            a[m][kb][0] = W_[u * 128 + lane];
            a[m][kb][1] = W_[u * 128 + 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[m][r] = bias[L * 64 + (NMB * W + m) * 16 + 4 * g + r];  // MFMA row order
    }
    unsigned radr[NF][PI], xadr[PX], oadr[PO];
#pragma unroll
    for (int j = 0; j < PI; ++j)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const Slot sl = fslot(L, W, f, g);
            radr[f][j] = ring_at(L, ring_row(L, j, li + sl.dq - 1), sl.oct);
        }
    // residual x: the block input (ring R(L-1), two columns ahead), octets 4W .. 4W+3
#pragma unroll
    for (int j = 0; j < PX; ++j) xadr[j] = RES ? ring_at(L - 1, ring_row(L - 1, j, li - 2), 4 * W + g) : 0u;
    // epilogue: lane group g stores the hi (g even) / lo (g odd) octet 2 d + (g >> 1)
    // of m-block d = dmb(L, W, m); the m-blocks' addresses differ by an XOR of
    // 32 (d ^ d0) in the octet field (the swizzle is an XOR on bits 4-6)
#pragma unroll
    for (int j = 0; j < PO; ++j)
        oadr[j] = L < 6 ? (g & 1) * kLoOff(L + 1) + ring_at(L + 1, ring_row(L + 1, j, li), 2 * dmb(L, W, 0) + (g >> 1))
                        : 0u;
    u32x4 aid[NMB];  // identity A of m-block m: row li takes fragment row 16 m + li = 8 g + e
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (_Float16)(16 * m + li == 8 * g + e ? 1.f : 0.f);
        aid[m] = __builtin_bit_cast(u32x4, v);
    }
    const int sL = qa + NL - 1 - L;  // first column of chunk 0
    auto work = [&](int k, auto jc) {
        constexpr int kk = decltype(jc)::value;
        constexpr int ji = kk % PI, jx = kk % PX, jo = kk % PO;
        u32x4 bh[NF], bl[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            bh[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][ji]);
            bl[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][ji] + kLoOff(L));
        }
        u32x4 xh, xl;
        if constexpr (RES) {
            xh = *reinterpret_cast<const u32x4*>(lds + xadr[jx]);
            xl = *reinterpret_cast<const u32x4*>(lds + xadr[jx] + kLoOff(L - 1));
        }
        f32x4 acc[NMB];
#pragma unroll
        for (int m = 0; m < NMB; ++m) acc[m] = f32x4{bv[m][0], bv[m][1], bv[m][2], bv[m][3]};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                for (int m = 0; m < NMB; ++m) {
                    const int f = frag_of(L, W, m, kb);
                    acc[m] = mfma_h(a[m][kb][pr == 2], pr == 1 ? bl[f] : bh[f], acc[m]);
                }
        if constexpr (RES) {
#pragma unroll
            for (int m = 0; m < NMB; ++m) acc[m] = mfma_h(aid[m], xh, acc[m]);
#pragma unroll
            for (int m = 0; m < NMB; ++m) acc[m] = mfma_h(aid[m], xl, acc[m]);
        }
        const int x0 = sL + 16 * k;
        if constexpr (L == NL - 1) {
            // rows 0..3 (lane group 0) = audio samples 4x .. 4x+3
            const int x = x0 + li;
            if (g == 0 && k >= 0 && x >= 0 && x < L2) {
                float4 o;
                o.x = tanh_fast(acc[0][0]);
                o.y = tanh_fast(acc[0][1]);
                o.z = tanh_fast(acc[0][2]);
                o.w = tanh_fast(acc[0][3]);
                *reinterpret_cast<float4*>(arow + 4 * (size_t)x) = o;
                flag_nonfinite4(o.x, o.y, o.z, o.w, rflag, reinterpret_cast<int*>(lds + kFlagOff(NL)));
            }
        } else {
            auto epilogue = [&](auto zc) {
                constexpr bool ZERO = decltype(zc)::value;
                float v[NMB][4];
#pragma unroll
                for (int m = 0; m < NMB; ++m) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[m][r] = acc[m][r];
                    if constexpr (!RES) leaky4(v[m]);
                }
                if constexpr (ZERO) {
                    const int x = x0 + li;
                    const bool out = x < 0 || x >= L2;
#pragma unroll
                    for (int m = 0; m < NMB; ++m)
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[m][r] = out ? 0.f : v[m][r];
                    if constexpr (L == 4 && NL == 6) {
                        // outc2_role's edge terms: wave 0's m-block 0 is phase 0
                        // (h[:, 0] at column 0), wave 1's m-block 1 phase 3
                        // (h[:, L4 - 1] at column L2 - 1); lane group g holds
                        // channels 4g .. 4g + 3 and adds its products (group 0
                        // also kL / kR) into slot 4W + g.  (Opaque pointer: the
                        // constants load in this rare branch, not hoisted.)
                        const float* cp = bias + kOutcCorr;
                        asm volatile("" : "+s"(cp));
                        if (W == 0 ? x == 0 : x == L2 - 1) {
                            const float* cv = cp + 16 * W + 4 * g;
                            float d = g == 0 ? cp[32 + W] : 0.f;
#pragma unroll
                            for (int r = 0; r < 4; ++r) d = fmaf(cv[r], v[W][r], d);
                            *reinterpret_cast<float*>(lds + kCorrSlot + 4 * (4 * W + g)) = d;
                        }
                    }
                }
#pragma unroll
                for (int m = 0; m < NMB; ++m) {
                    unsigned h0, h1, l0, l1;
                    split2u(v[m][0], v[m][1], h0, l0);
                    split2u(v[m][2], v[m][3], h1, l1);
                    const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
                    const unsigned mx = 32u * (unsigned)(dmb(L, W, m) ^ dmb(L, W, 0));
                    *reinterpret_cast<u32x4*>(lds + (oadr[jo] ^ mx)) = u32x4{s0[0], s1[0], s0[1], s1[1]};
                }
            };
            // (layer 4 of the six-layer form also takes it for a chunk that
            // starts at column 0 or ends at L2: outc2_role's edge terms)
            constexpr int EW = L == 4 && NL == 6 ? 1 : 0;
            if (edge && (x0 < EW || x0 + 16 > L2 - EW)) epilogue(std::true_type{});  // wave-uniform
            else epilogue(std::false_type{});
        }
    };
    const int LAST = last_step(nch, NL);
    auto step = [&](int s, auto jc) {
        if (s <= LAST) {
            const int k = s - off_l(L);
            if (k >= -1 && k < nch) work(k, jc);
            step_barrier();
        }
    };
    constexpr int U = (PI == 3 || PO == 3 || PX == 3) ? 12 : 4;
    constexpr int J0 = ((-1 - off_l(L)) % U + U) % U;
    auto iter = [&](int s, auto... i) { (step(s + decltype(i)::value, ic<(J0 + decltype(i)::value) % U>{}), ...); };
#pragma unroll 1
    for (int s = -1; s <= LAST; s += U) {
        if constexpr (U == 4)
            iter(s, ic<0>{}, ic<1>{}, ic<2>{}, ic<3>{});
        else
            iter(s, ic<0>{}, ic<1>{}, ic<2>{}, ic<3>{}, ic<4>{}, ic<5>{}, ic<6>{}, ic<7>{}, ic<8>{}, ic<9>{},
                 ic<10>{}, ic<11>{});
    }
}

// ResBlock4 conv2 + output_conv composed (NL = 6; vocoder_tailp.hip's
// outc_role at 16 channels): audio = tanh(Wc * h + Wo * x + bo') with
// Wc = Wo o W2 a k5 conv on ResBlock4's intermediate h (ring R5) and Wo on
// ConvT4's output x (ring R4, two columns ahead); 7 k-blocks = 21 MFMAs on one
// wave, in place of ResBlock4 conv2 (two waves of 2 x 2 x 3 + 4) and the
// output conv (9).  The utterance's two edge samples subtract the y the
// reference pads with zeros (terms from layer 4, LDS slot kCorrSlot).
__device__ __forceinline__ void outc2_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                           const u32x4* __restrict__ W_, const float* __restrict__ bias,
                                           float* __restrict__ arow, int* rflag) {
    constexpr int L = 5, NL = 6, NF = kOutcF, P = 4;
    static_assert(kRingRows[4] == 64 && kRingRows[5] == 64, "64-row rings");
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    u32x4 a[NF][2];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        a[f][0] = W_[(kOutcUnit0 + f) * 128 + lane];
        a[f][1] = W_[(kOutcUnit0 + f) * 128 + 64 + lane];
    }
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bias[kOutcBias + 4 * g + r];
    // one VGPR per fragment: on a 64-row ring (8 KB planes) the address of
    // ring phase j is (rbase + 2048 j) & 8191 past the ring (the swizzle reads
    // row bits 0-2 only)
    unsigned rbase[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const Slot sl = outc_slot(f, g);
        rbase[f] = f < 4 ? ring_at(5, ring_row(5, 0, li + sl.dq - 1), sl.oct) - kRingOff(5)
                         : ring_at(4, ring_row(4, 0, li + sl.dq - 2), sl.oct) - kRingOff(4);
    }
    auto radr = [&](int f, int j) { return (f < 4 ? kRingOff(5) : kRingOff(4)) + ((rbase[f] + 2048u * j) & 8191u); };
    auto work = [&](int k, auto jc) {
        constexpr int j = decltype(jc)::value;
        u32x4 bh[NF], bl[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            bh[f] = *reinterpret_cast<const u32x4*>(lds + radr(f, j));
            bl[f] = *reinterpret_cast<const u32x4*>(lds + radr(f, j) + (f < 4 ? kLoOff(5) : kLoOff(4)));
        }
        f32x4 acc = f32x4{bv[0], bv[1], bv[2], bv[3]};
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr) acc = mfma_h(a[f][pr == 2], pr == 1 ? bl[f] : bh[f], acc);
        const int x0 = qa + 16 * k, x = x0 + li;
        float v[4] = {acc[0], acc[1], acc[2], acc[3]};
        if (edge && (x0 <= 0 || x0 + 16 >= L2)) {  // wave-uniform
            const f32x4 e0 = *reinterpret_cast<const f32x4*>(lds + kCorrSlot);
            const f32x4 e1 = *reinterpret_cast<const f32x4*>(lds + kCorrSlot + 16);
            if (x == 0) v[0] -= (e0[0] + e0[1]) + (e0[2] + e0[3]);
            if (x == L2 - 1) v[3] -= (e1[0] + e1[1]) + (e1[2] + e1[3]);
        }
        if (g == 0 && k >= 0 && x >= 0 && x < L2) {
            float4 o;
            o.x = tanh_fast(v[0]);
            o.y = tanh_fast(v[1]);
            o.z = tanh_fast(v[2]);
            o.w = tanh_fast(v[3]);
            *reinterpret_cast<float4*>(arow + 4 * (size_t)x) = o;
            flag_nonfinite4(o.x, o.y, o.z, o.w, rflag, reinterpret_cast<int*>(lds + kFlagOff(NL)));
        }
    };
    const int LAST = last_step(nch, NL);
    auto step = [&](int s, auto jc) {
        if (s <= LAST) {
            const int k = s - off_l(L);
            if (k >= 0 && k < nch) work(k, jc);  // chunk -1 feeds no later layer
            step_barrier();
        }
    };
    constexpr int J0 = ((-1 - off_l(L)) % P + P) % P;
#pragma unroll 1
    for (int s = -1; s <= LAST; s += P) {
        step(s, ic<J0 % P>{});
        step(s + 1, ic<(J0 + 1) % P>{});
        step(s + 2, ic<(J0 + 2) % P>{});
        step(s + 3, ic<(J0 + 3) % P>{});
    }
}

// U2 rows (256 B: hi[64] lo[64]) into ring R0, two chunks ahead: chunk c =
// columns [qa + 7 + 16c, +16), zero outside [0, L2).  Lane (r = lane >> 4, pc =
// lane & 15) moves 16 B of columns r, r + 4, r + 8, r + 12 (pc < 8: hi octet pc,
// else lo octet pc - 8); loads unconditional (clamped) so their waits are counted.
template <int NL, bool EDGE>
__device__ __forceinline__ void loader_role(unsigned char* lds, int qa, int L2, int nch,
                                            const unsigned char* __restrict__ u2) {
    const int lane = threadIdx.x & 63, r = lane >> 4, pc = lane & 15;
    auto fetch = [&](int c, u32x4 (&v)[4]) {
#pragma unroll
        for (int h = 0; h < 4; ++h) {
            int col = qa + NL + 16 * c + r + 4 * h;
            if (EDGE) col = min(max(col, 0), L2 - 1);
            v[h] = *reinterpret_cast<const u32x4*>(u2 + (size_t)col * 256 + pc * 16);
        }
    };
    u32x4 buf[3][4];
    unsigned wadr[3][4];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int h = 0; h < 4; ++h) wadr[j][h] = (pc >> 3) * kLoOff(0) + ring_at(0, ring_row(0, j, r + 4 * h), pc & 7);
    auto step = [&](int s, auto jc, u32x4 (&cur)[4], u32x4 (&ahead)[4]) {
        constexpr int j = decltype(jc)::value;
        fetch(min(s + 2, nch - 1), ahead);
        if (s < nch) {
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                const int col = qa + NL + 16 * s + r + 4 * h;
                const bool in = !EDGE || (col >= 0 && col < L2);
                const u32x4 z{0u, 0u, 0u, 0u};
                *reinterpret_cast<u32x4*>(lds + wadr[j][h]) = in ? cur[h] : z;
            }
        }
        step_barrier();
    };
    fetch(-1, buf[0]);
    fetch(0, buf[1]);
    int s = -1;
#pragma unroll 1
    for (; s + 2 <= last_step(nch, NL); s += 3) {
        step(s, ic<2>{}, buf[0], buf[2]);
        step(s + 1, ic<0>{}, buf[1], buf[0]);
        step(s + 2, ic<1>{}, buf[2], buf[1]);
    }
#pragma unroll 1
    for (; s <= last_step(nch, NL); ++s) step_barrier();
}

// TAILP2_DMA: U2 rows into ring R0 by LDS-DMA (as vocoder_tailp.hip's
// loader_role_dma).  A chunk's hi plane is 16 rows x 128 B = two 1-KB
// buffer_load_dwordx4 ... lds (rows 8i .. 8i + 7: lane l fills row 8i + l / 8,
// slot l % 8, i.e. octet (l % 8) ^ (row & 7)), its lo plane two more; columns
// outside [0, L2) are out of the descriptor's range and land as zeros.  Chunk
// c + 1 goes into the slot of chunk c - 3 at the top of step c, and chunk c
// must have landed before step c's barrier (vmcnt(4)).
template <int NL>
__device__ __forceinline__ void loader_role_dma(unsigned char* lds, int qa, int L2, int nch,
                                                const unsigned char* __restrict__ u2) {
    static_assert(NL > 0 && kRingRows[0] == 64, "4-chunk R0");
    const int lane = threadIdx.x & 63, r8 = lane >> 3;
    [[maybe_unused]] const int oct = (lane & 7) ^ (r8 & 7);
    // descriptor from the strip's first column to the utterance's end (small
    // 32-bit offsets at any length; columns before 0 only in the first strip)
    const int c0 = max(0, qa + NL - 16);
    [[maybe_unused]] const auto rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(u2) + (size_t)c0 * 256, 0, (int)min((long)(L2 - c0) * 256, 0x7fffffffL),
        0x00020000);
    auto dma = [&](int c) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass of hipcc does not know this builtin)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int voff = (qa + NL + 16 * c + 8 * i + r8 - c0) * 256 + 16 * oct;  // out of range -> 0
            unsigned char* dst = lds + kRingOff(0) + 2048 * (c & 3) + 1024 * i;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, voff, 0,
                                                     0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + kLoOff(0)),
                                                     16, voff + 128, 0, 0, 0);
        }
#endif
    };
    dma(-1);
#pragma unroll 1
    for (int s = -1; s <= last_step(nch, NL); ++s) {
        if (s + 1 < nch) {
            dma(s + 1);
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        step_barrier();
    }
}

template <int NL>
__global__ __launch_bounds__(nwaves(NL) * 64, 1) void tailp2_kernel(const unsigned char* __restrict__ U2, int L2,
                                                                     int nch, const u32x4* __restrict__ W,
                                                                     const float* __restrict__ bias,
                                                                     float* __restrict__ audio, int* rflag,
                                                                     const int32_t* __restrict__ dT, VocRedo rd) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = blockIdx.y, qa = blockIdx.x * 16 * nch;
    if (dT) {  // speculative launch: L2 was the capacity
        L2 = 16 * dev_frames(dT, L2 / 16);
        if (qa >= L2) return;
    }
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool edge = qa < 32 || qa + 16 * nch + 32 > L2;
    float* arow = audio + (size_t)b * 4 * L2;
    int* const lflag = reinterpret_cast<int*>(lds + kFlagOff(NL));
    if (threadIdx.x == 0) *lflag = 0;  // before the first epilogue: the pipeline's step barriers order it
    // later layers: younger waves, the step waits for the slowest role
    if (w >= 10) __builtin_amdgcn_s_setprio(3);
    else if (w >= 6) __builtin_amdgcn_s_setprio(2);
    else if (w >= 2) __builtin_amdgcn_s_setprio(1);
    const unsigned char* u2 = U2 + (size_t)b * L2 * 256;
    switch (w) {
        case 0: layer_role<0, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 1: layer_role<0, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 2: layer_role<1, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 3: layer_role<1, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 4: layer_role<2, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 5: layer_role<2, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 6: layer_role<3, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 7: layer_role<3, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 8: layer_role<4, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 9: layer_role<4, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 10:
            if constexpr (NL == 7) layer_role<5, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag);
            else outc2_role(lds, qa, L2, nch, edge, W, bias, arow, rflag);
            break;
        case 11:
            if constexpr (NL == 7) {
                layer_role<5, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag);
                break;
            }
            [[fallthrough]];
        case 12:
            if constexpr (NL == 7) {
                if (w == 12) {
                    layer_role<6, 0, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag);
                    break;
                }
            }
            [[fallthrough]];
        default:
            if constexpr (TAILP2_DMA) loader_role_dma<NL>(lds, qa, L2, nch, u2);
            else if (edge) loader_role<NL, true>(lds, qa, L2, nch, u2);
            else loader_role<NL, false>(lds, qa, L2, nch, u2);
            break;
    }
    if (rd.rw) {  // range policy "fallback": this strip's audio again in fp32 if it is not finite
        __syncthreads();
        if (*lflag)
            redo_frames(*rd.rw, rd.mel, rd.trans, L2 / 16, b, qa / 16, min(L2, qa + 16 * nch) / 16, arow,
                        reinterpret_cast<float*>(lds), ring_bytes(NL) / 4);
    }
}

template <int NL>
int32_t launch_nl(int nch, const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                  int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    static bool attr = false;
    if (!attr) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(tailp2_kernel<NL>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes(NL)));
        attr = true;
    }
    hipLaunchKernelGGL((tailp2_kernel<NL>), dim3(cdiv(L2, 16 * nch), B), dim3(nwaves(NL) * 64), lds_bytes(NL), st,
                       static_cast<const unsigned char*>(U2), L2, nch, W, bias, audio, rflag, dT, rd);
    M2_LAUNCHED("tailp2_kernel");
    return M2_OK;
}

}  // namespace tp2

const char* const kVocTailp2KernelName =
    "tailp2_kernel (stage2 ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv, pipelined)";

int32_t launch_vocoder_tailp2(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                              int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    if (B == 0 || L2 == 0) return M2_OK;
    // Strip length (chunks of 16 columns): the one minimising rounds x (nch +
    // NL pipeline steps) at one workgroup per CU, any length from 8 to 256
    // (the kernel takes it at run time: 16 x 2600 gets 256 strips of 163
    // chunks, one round, where the instantiated lengths of round 4 gave 224
    // strips of 192).  M2_TAILP2_NCH forces one; M2_TAILP2_SEVEN=1 the
    // seven-layer form (switch table, m2_common.h).
    const bool seven = sw().tailp2_seven;
    const int nl = seven ? 7 : 6;
    int nch = sw().tailp2_nch > 0 ? std::min(sw().tailp2_nch, 4096) : 0;
    if (!nch) {
        const long chunks = cdiv(L2, 16);
        long best = -1;
        for (int n = 8; n <= 256; ++n) {
            const long wgs = (long)cdiv((int)chunks, n) * B, rounds = (wgs + 255) / 256, cost = rounds * (n + nl);
            if (best < 0 || cost < best) best = cost, nch = n;
        }
    }
    return seven ? tp2::launch_nl<7>(nch, U2, L2, B, W, bias, audio, rflag, st, dT, rd)
                 : tp2::launch_nl<6>(nch, U2, L2, B, W, bias, audio, rflag, st, dT, rd);
}

// ---------------------------------------------------------------------------
// Host packing: each layer as a dense polyphase matrix Wd[row][dq + 1][input
// row] (64 x 3 x 64), cut into (wave, m-block, k-block) fragment pairs along
// tp2::kslot: A[row = lane & 15][slot g = lane >> 4, element e] =
// Wd[16 dmb + (lane & 15)][dq + 1][8 oct + e], zero on a slot the m-block
// already read.  Every non-zero of Wd must sit on a slot.
namespace {

int floordiv2(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

struct Dense64 {
    std::vector<float> w = std::vector<float>(64 * 3 * 64, 0.f);
    float& at(int row, int dq, int in) { return w[(row * 3 + dq + 1) * 64 + in]; }
};

// ConvTranspose1d(k=4, stride 2, pad 1), W [Cin][Cout][4], on a Pin-phase input
// -> 2 Pin phases of Cout channels: out[2i] = x[i] W1 + x[i-1] W3,
// out[2i+1] = x[i+1] W0 + x[i] W2 (tts_model.py:255-263).
void dense_convT2(Dense64& d, const float* W, int Pin, int Cin, int Cout) {
    const int taps[2][2][2] = {{{0, 1}, {-1, 3}}, {{1, 0}, {0, 2}}};
    for (int pin = 0; pin < Pin; ++pin)
        for (int s = 0; s < 2; ++s)
            for (int j = 0; j < 2; ++j) {
                const int pp = pin + taps[s][j][0], dq = floordiv2(pp, Pin), p2 = pp - dq * Pin, kk = taps[s][j][1];
                for (int co = 0; co < Cout; ++co)
                    for (int ci = 0; ci < Cin; ++ci)
                        d.at((2 * pin + s) * Cout + co, dq, p2 * Cin + ci) += W[((size_t)ci * Cout + co) * 4 + kk];
            }
}

// Conv1d(k=3, pad 1), W [Cout][Cin][3], on a P-phase signal.
void dense_conv3(Dense64& d, const float* W, int P, int Cin, int Cout) {
    for (int p = 0; p < P; ++p)
        for (int k = 0; k < 3; ++k) {
            const int pp = p + k - 1, dq = floordiv2(pp, P), p2 = pp - dq * P;
            for (int co = 0; co < Cout; ++co)
                for (int ci = 0; ci < Cin; ++ci) d.at(p * Cout + co, dq, p2 * Cin + ci) += W[((size_t)co * Cin + ci) * 3 + k];
        }
}

void put_split(std::vector<uint16_t>& out, size_t idx, float v, bool* range_ok) {
    if (!(std::fabs(v) < 65504.f)) *range_ok = false;
    const _Float16 h = (_Float16)v;
    const _Float16 l = (_Float16)(v - (float)h);
    uint16_t hb, lb;
    std::memcpy(&hb, &h, 2);
    std::memcpy(&lb, &l, 2);
    out[idx] = hb;
    out[idx + 64 * 8] = lb;
}

}  // namespace

bool pack_outc2(const TailpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok);

bool pack_tailp2(const TailpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok) {
    using namespace tp2;
    Dense64 d[kLayers];
    dense_convT2(d[0], s.wt3, 1, 64, 32);
    dense_conv3(d[1], s.w31, 2, 32, 32);
    dense_conv3(d[2], s.w32, 2, 32, 32);
    dense_convT2(d[3], s.wt4, 2, 32, 16);
    dense_conv3(d[4], s.w41, 4, 16, 16);
    dense_conv3(d[5], s.w42, 4, 16, 16);
    dense_conv3(d[6], s.wo, 4, 16, 1);
    const int nrows[kLayers] = {64, 64, 64, 64, 64, 64, 4};
    // every non-zero dense weight must be read by some slot of its m-block
    for (int l = 0; l < kLayers; ++l)
        for (int w = 0; w < nwv(l); ++w)
            for (int m = 0; m < nmbw(l); ++m)
                for (int rr = 0; rr < 16; ++rr) {
                    const int row = 16 * dmb(l, w, m) + rr;
                    if (row >= nrows[l]) continue;
                    for (int dq = -1; dq <= 1; ++dq)
                        for (int in = 0; in < 64; ++in) {
                            if (d[l].at(row, dq, in) == 0.f) continue;
                            bool found = false;
                            for (int kb = 0; kb < nkb(l) && !found; ++kb)
                                for (int g = 0; g < 4; ++g) {
                                    const Slot sl = kslot(l, w, m, kb, g);
                                    if (sl.dq == dq && sl.oct == in / 8) found = true;
                                }
                            if (!found) return false;
                        }
                }
    wout->assign((size_t)(kUnits + kOutcF) * 2 * 64 * 8, 0);
    for (int l = 0; l < kLayers; ++l)
        for (int w = 0; w < nwv(l); ++w)
            for (int m = 0; m < nmbw(l); ++m)
                for (int kb = 0; kb < nkb(l); ++kb) {
                    const int u = unit_of(l, w, m, kb);
                    for (int lane = 0; lane < 64; ++lane) {
                        const int row = 16 * dmb(l, w, m) + (lane & 15), g = lane >> 4;
                        const Slot sl = kslot(l, w, m, kb, g);
                        bool dup = false;  // a (dq, octet) this m-block already reads in an earlier slot
                        for (int j = 0; j < kb * 4 + g; ++j) {
                            const Slot o = kslot(l, w, m, j / 4, j % 4);
                            dup = dup || (o.dq == sl.dq && o.oct == sl.oct);
                        }
                        for (int e = 0; e < 8; ++e) {
                            float v = 0.f;
                            if (row < nrows[l] && !dup) v = d[l].at(row, sl.dq, 8 * sl.oct + e);
                            put_split(*wout, (((size_t)u * 2) * 64 + lane) * 8 + e, v, range_ok);
                        }
                    }
                }
    // biases in MFMA row order: [layer][wave][m-block][16 rows]
    bout->assign(kBiasFloats, 0.f);
    const float* bsrc[kLayers] = {s.bt3, s.b31, s.b32, s.bt4, s.b41, s.b42, s.bo};
    const int cper[kLayers] = {32, 32, 32, 16, 16, 16, 1};
    for (int l = 0; l < kLayers; ++l)
        for (int w = 0; w < nwv(l); ++w)
            for (int m = 0; m < nmbw(l); ++m)
                for (int rr = 0; rr < 16; ++rr) {
                    const int row = 16 * dmb(l, w, m) + rr;
                    if (row < nrows[l]) (*bout)[l * 64 + (nmbw(l) * w + m) * 16 + rr] = bsrc[l][row % cper[l]];
                }
    return pack_outc2(s, wout, bout, range_ok);
}

// The composed layer (outc2_role), in double: audio[t] = tanh(bo' + sum_d
// Wo[c][d] x[c][t+d] + sum_j Wc[c'][j] h[c'][t+j]), Wc[c'][j] = sum_{d+e=j}
// sum_c Wo[c][d] W2[c][c'][e], bo' = bo + sum_d sum_c Wo[c][d] b2[c]; rows =
// the 4 output phases, input row p2 * 16 + c at column q + dq.  Edge terms as
// in vocoder_tailp.hip's pack_outc.
bool pack_outc2(const TailpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok) {
    using namespace tp2;
    constexpr int C = 16;
    std::vector<double> dh(4 * 3 * 64, 0.0), dx(4 * 3 * 64, 0.0);
    auto at = [](std::vector<double>& d, int p, int dq, int in) -> double& { return d[(p * 3 + dq + 1) * 64 + in]; };
    auto wo = [&](int c, int k) { return (double)s.wo[c * 3 + k]; };
    auto w2 = [&](int c, int ci, int k) { return (double)s.w42[(c * C + ci) * 3 + k]; };
    for (int p = 0; p < 4; ++p)
        for (int d = -1; d <= 1; ++d)
            for (int c = 0; c < C; ++c) {
                const int tx = p + d, qx = floordiv2(tx, 4);
                at(dx, p, qx, (tx - 4 * qx) * C + c) += wo(c, d + 1);
                for (int e = -1; e <= 1; ++e)
                    for (int ci = 0; ci < C; ++ci) {
                        const int th = p + d + e, qh = floordiv2(th, 4);
                        at(dh, p, qh, (th - 4 * qh) * C + ci) += wo(c, d + 1) * w2(c, ci, e + 1);
                    }
            }
    for (int p = 0; p < 4; ++p)
        for (int dq = -1; dq <= 1; ++dq)
            for (int in = 0; in < 64; ++in)
                for (int src = 0; src < 2; ++src) {
                    if (at(src ? dx : dh, p, dq, in) == 0.0) continue;
                    bool found = false;
                    for (int f = src ? 4 : 0; f < (src ? kOutcF : 4); ++f)
                        for (int g = 0; g < 4; ++g) {
                            const Slot sl = outc_slot(f, g);
                            found = found || (sl.dq == dq && sl.oct == in / 8);
                        }
                    if (!found) return false;
                }
    for (int f = 0; f < kOutcF; ++f)
        for (int lane = 0; lane < 64; ++lane) {
            const int row = lane & 15, g = lane >> 4;
            const Slot sl = outc_slot(f, g);
            for (int e = 0; e < 8; ++e) {
                double v = 0.0;
                if (row < 4) v = at(f < 4 ? dh : dx, row, sl.dq, 8 * sl.oct + e);
                put_split(*wout, (((size_t)(kOutcUnit0 + f) * 2) * 64 + lane) * 8 + e, (float)v, range_ok);
            }
        }
    double bo = s.bo[0], kl = 0.0, kr = 0.0;
    for (int c = 0; c < C; ++c) {
        for (int k = 0; k < 3; ++k) bo += wo(c, k) * s.b42[c];
        kl += wo(c, 0) * s.b42[c];
        kr += wo(c, 2) * s.b42[c];
    }
    for (int r = 0; r < 4; ++r) (*bout)[kOutcBias + r] = (float)bo;
    for (int ci = 0; ci < C; ++ci) {
        double vl = 0.0, vr = 0.0;
        for (int c = 0; c < C; ++c) {
            vl += wo(c, 0) * w2(c, ci, 2);
            vr += wo(c, 2) * w2(c, ci, 0);
        }
        (*bout)[kOutcCorr + ci] = (float)vl;
        (*bout)[kOutcCorr + 16 + ci] = (float)vr;
    }
    (*bout)[kOutcCorr + 32] = (float)kl;
    (*bout)[kOutcCorr + 33] = (float)kr;
    return true;
}

}  // namespace m2
