// Fused SimpleVocoder on the f16 MFMA with a three-product split (gfx950).
//
// Same three launches and the same exact-halo windows as vocoder_fused.hip
// (head: input_conv -> ConvT1 -> ResBlock1, mid: ConvT2 -> ResBlock2, tail:
// ConvT3 -> ResBlock3 -> ConvT4 -> ResBlock4 -> output_conv -> tanh), but the
// GEMMs run on v_mfma_f32_16x16x32_f16 (16 cycles for 16K FLOP, 16x the
// FLOP rate of the f32 MFMA) with every fp32 operand x carried as two halves
//     x_hi = f16(x),  x_lo = f16(x - x_hi)        (split2u, vocoder_fused.h)
// and every product as
//     a.b ~= a_hi.b_hi + (a_hi.b_lo + a_lo.b_hi)
// accumulated in fp32 (two accumulators per tile, summed in the epilogue).
// The dropped a_lo.b_lo term is 2^-22 relative, and each half-product is
// exact in the fp32 accumulator, so the result carries fp32-level error:
// simulated over the whole stage1/stage2 vocoder (tools/probe/split_sim.py)
// the waveform RMS error vs fp64 is 3e-7 against 1.5e-7 for plain fp32
// convolution (plain f16 operands: 3.1e-4, outside the 1e-4 bound).  Three
// MFMAs per product leave 16/3 = 5.3x the exact-f32 MFMA rate.  Range: |x| and
// |w| must stay below 65504 (f16 max); weights are checked at model creation.
//
// Data layout.  Activations live position-major: one row per position holding
// hi[C] then lo[C] (f16), rows padded to a stride RS with RS/16 = 2 (mod 4) so
// the 16-lane groups of a ds_read_b128 hit 16 distinct 16-B bank quads.  An
// MFMA B fragment (lane = position j, 8 consecutive channels of one tap) is
// one ds_read_b128 for the hi half and one for the lo half.  The global
// intermediates U1 [B][4T] and U2 [B][16T] use the same row format (4*C
// bytes per position, the bytes of an fp32 tensor), so the next kernel copies
// rows without converting.  Weights are packed per (phase, m-block, k-block of
// 32) as [hi|lo][lane][8 halves]: two global_load_dwordx4 per lane.
// K order: k-block kb, lane group g = lane>>4 covers octet o = 4kb+g of the
// (tap, channel/8) sequence; any k order shared by A and B gives the same sum.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <functional>

#include "m2_common.h"
#include "vocoder_fused.h"

namespace m2 {
namespace x3 {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef vx_u32x4 u32x4;
typedef float f32x4 __attribute__((ext_vector_type(4)));


__device__ __forceinline__ f32x4 mfma_h(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

// Row stride in bytes for C channels: >= 4C, multiple of 16, (RS/16) % 4 == 2
// (C = 8: 32 B, 2-way conflicts between rows 8 apart are accepted).
constexpr int rs_for(int C) {
    int u = (4 * C + 15) / 16;
    if (C <= 8) return u * 16;
    while (u % 4 != 2) ++u;
    return u * 16;
}
constexpr int rup16(int n) { return (n + 15) / 16 * 16; }
constexpr int cmax(int a, int b) { return a > b ? a : b; }

// An LDS activation window: rows of RS bytes, absolute position of row 0.
struct XW {
    unsigned char* p;
    int start;
};

__device__ __forceinline__ void split4(const float (&v)[4], h4& hi, h4& lo) {
    unsigned h0, h1, l0, l1;
    split2u(v[0], v[1], h0, l0);
    split2u(v[2], v[3], h1, l1);
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    hi = __builtin_bit_cast(h4, u32x2{h0, h1});
    lo = __builtin_bit_cast(h4, u32x2{l0, l1});
}

template <int CIN, int NTAP>
constexpr int nkb_of() { return (NTAP * (CIN / 8) + 3) / 4; }

// ---------------------------------------------------------------------------
// acc[n] += A_hi.B_hi + A_hi.B_lo + A_lo.B_hi over all k-blocks, for
// NT 16-position tiles (NT compile-time: no per-tile guards, which would
// make the MFMA chain conditional code and blow up register allocation).
// wp: this lane's A slot of k-block 0 (u32x4 units, k-block stride 128 =
// hi + lo).  bp: LDS row of this lane's position for tap 0 and k-block 0,
// before the lane-group offset.  Tap k reads row bp + k*STEP (STEP = +1 for
// conv3 [t-1, t, t+1], -1 for the ConvT taps).
// XR (residual fold, 8- and 16-channel ResBlock conv2): the padding octets
// of the last k-block read the block input x at the output row (xr) and the
// packed weights hold the identity there, so the GEMM itself adds x.
// NMB m-blocks (weight rows WS u32x4 apart) share every B fragment read.
// a: the weight-fragment pipeline (PD k-blocks in flight).  PRE: the caller
// already issued the loads of k-blocks 0 .. PD-1 (the previous layer's item
// did, before its epilogue and the barrier); wp_next (PD == 4, NMB == 1): once
// this item's last MFMA is issued, start the next item's first PD k-blocks.
template <int CIN, int NTAP, int NMB, int PDM = 4>
constexpr int pd_of() {
    constexpr int NKB = (NTAP * (CIN / 8) + 3) / 4;
    return NKB < PDM / NMB ? NKB : PDM / NMB;
}
// TB: tap k's rows start at tb[k] (this lane's row and lane-group chunk, the
// plane swizzle applied) instead of bp + k*STEP*RSI - the phase-planar
// layouts of the head.
// BP: see below.
template <int CIN, int NTAP, int STEP, int RSI, int NT, bool XR, int NMB, int WS, bool PRE, bool TB = false,
          int PDM = 4, int BP = 0>
__device__ __forceinline__ void mma_x3(const u32x4* __restrict__ wp, const unsigned char* bp,
                                       const unsigned char* xr, f32x4 (&acc)[NMB][NT],
                                       u32x4 (&a)[pd_of<CIN, NTAP, NMB, PDM>()][NMB][2], const u32x4* wp_next,
                                       const unsigned char* const* tb = nullptr) {
    constexpr int NOCT = CIN / 8, NK = NTAP * NOCT, NKB = (NK + 3) / 4;
    static_assert(CIN % 8 == 0 && (NOCT <= 2 || NOCT % 4 == 0), "channel count must be 8, 16 or a multiple of 32");
    static_assert(!XR || 4 * NKB - NK == NOCT, "residual fold needs exactly one row of padding octets");
    constexpr int Q = NOCT >= 4 ? 4 : NOCT;     // lane groups per tap row
    constexpr int TPK = NOCT >= 4 ? 0 : 4 / Q;  // taps per k-block when a tap row has < 4 octets
    auto koff = [](int kb) {
        const int tap = NOCT >= 4 ? kb / (NOCT / 4) : kb * TPK;
        const int col = NOCT >= 4 ? (kb % (NOCT / 4)) * 64 : 0;
        return tap * STEP * RSI + col;
    };
    const int g = (threadIdx.x & 63) >> 4;
    const unsigned char* bl = bp + (g / Q) * STEP * RSI + (g % Q) * 16;
    // Last k-block: padding octets (zero weights) re-read octet 0's bytes -
    // inside the window and finite - or, with XR, x's octet (o - NK).
    const int o_last = 4 * (NKB - 1) + g;
    const unsigned char* b_last = o_last < NK ? bl + koff(NKB - 1)
                                              : (XR ? xr + (o_last - NK) * 16 : bp + koff(NKB - 1));
    // Weight fragments stream PD k-blocks ahead (PD = all of them up to
    // PDM / NMB): one L2 round trip per item rather than one per k-block (a
    // k-block is only 3*NT*NMB MFMAs, shorter than an L2 hit), at most
    // 8 * PDM VGPRs in flight (PDM = 4 where the register budget is 128 per
    // wave, the config's PDM where it is 256: the stage2 kernels).
    constexpr int PD = pd_of<CIN, NTAP, NMB, PDM>();
    if (!PRE)
#pragma unroll
    for (int kb = 0; kb < PD; ++kb)
#pragma unroll
        for (int m = 0; m < NMB; ++m) {
            a[kb][m][0] = wp[m * WS + kb * 128];
            a[kb][m][1] = wp[m * WS + kb * 128 + 64];
        }
    auto bbase = [&](int kb) {
        if constexpr (TB) {
            static_assert(NOCT >= 4 && !XR, "tap bases: whole octet rows only");
            return tb[kb / (NOCT / 4)] + (kb % (NOCT / 4)) * 64;  // tb: the lane group's chunk included
        } else {
            return kb == NKB - 1 ? b_last : bl + koff(kb);
        }
    };
    // BP 1: k-block kb + 1's B fragments are read from LDS before k-block
    // kb's MFMAs are issued (two register buffers, 8 NT more VGPRs), so their
    // LDS latency hides behind the MFMAs instead of sitting before each
    // k-block's first; BP 2: only the hi fragments one k-block ahead (4 NT
    // more VGPRs).  Taken where it measured faster (the stage2 head, CfgS2).
    constexpr int NBH = BP ? 2 : 1, NBL = BP == 1 ? 2 : 1;
    u32x4 bh[NBH][NT], blo[NBL][NT];
    auto readh = [&](int kb, int q) {
        const unsigned char* b0 = bbase(kb);
#pragma unroll
        for (int n = 0; n < NT; ++n) bh[q][n] = *reinterpret_cast<const u32x4*>(b0 + n * 16 * RSI);
    };
    auto readl = [&](int kb, int q) {
        const unsigned char* b0 = bbase(kb);
#pragma unroll
        for (int n = 0; n < NT; ++n) blo[q][n] = *reinterpret_cast<const u32x4*>(b0 + n * 16 * RSI + 2 * CIN);
    };
    if constexpr (BP) readh(0, 0);
    if constexpr (BP == 1) readl(0, 0);
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
        const int q = BP ? (kb & 1) : 0, ql = BP == 1 ? (kb & 1) : 0;
        if constexpr (BP == 2) readl(kb, 0);
        if constexpr (BP) {
            if (kb + 1 < NKB) {
                readh(kb + 1, (kb + 1) & 1);
                if constexpr (BP == 1) readl(kb + 1, (kb + 1) & 1);
            }
        } else {
            readh(kb, 0);
            readl(kb, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < NMB; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = mfma_h(a[kb % PD][m][0], bh[q][n], acc[m][n]);
#pragma unroll
        for (int m = 0; m < NMB; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = mfma_h(a[kb % PD][m][0], blo[ql][n], acc[m][n]);
#pragma unroll
        for (int m = 0; m < NMB; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = mfma_h(a[kb % PD][m][1], bh[q][n], acc[m][n]);
        if (kb + PD < NKB) {
#pragma unroll
            for (int m = 0; m < NMB; ++m) {
                a[kb % PD][m][0] = wp[m * WS + (kb + PD) * 128];
                a[kb % PD][m][1] = wp[m * WS + (kb + PD) * 128 + 64];
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (PD == 4 && NMB == 1) {
        if (wp_next) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb) {
                a[kb][0][0] = wp_next[kb * 128];
                a[kb][0][1] = wp_next[kb * 128 + 64];
            }
        }
    }
}


// Epilogue for one tile (acc already holds the bias): v = act(acc)
// [+ residual read back from `out`], 0 outside [0, L) (only
// evaluated for tiles that reach past an edge), split and stored as hi/lo.
// Executed by every lane (the permlane16 swap reads the partner lane group);
// `store` says whether this lane's 16 B are written.  After the swap lane group
// 0 (2) holds the hi halves of channels 0-7 (8-15) of the m-block and group 1
// (3) the lo halves: one ds_write_b128 per lane instead of two ds_write_b64
// (2-way instead of 4-way bank conflicts on RS/16 = 2 mod 4 rows).
// GO: the tile goes straight to global rows of 4*COUT bytes (gout, absolute
// position t, t < L only) instead of back into `out` (the residual is still
// read from `out`).
template <int COUT, int RSO, int ACT, bool RES, bool GO>
__device__ __forceinline__ void store_tile(const f32x4& acc, XW out, int t, int co0, int L,
                                           bool edge, bool store, unsigned char* gout) {
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = acc[r];
    if constexpr (ACT == ACT_LEAKY) leaky4(v);
    else static_assert(ACT == ACT_NONE, "x3 layers: leaky or none");
    unsigned char* rowp = out.p + (t - out.start) * RSO;
    if (RES) {
        const unsigned char* row = rowp + co0 * 2;
        const h4 hi = *reinterpret_cast<const h4*>(row), lo = *reinterpret_cast<const h4*>(row + 2 * COUT);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)hi[r] + (float)lo[r];
    }
    if (!GO && edge && (t < 0 || t >= L)) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = 0.f;
    }
    unsigned h0, h1, l0, l1;
    split2u(v[0], v[1], h0, l0);
    split2u(v[2], v[3], h1, l1);
    const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
    const int g = (threadIdx.x & 63) >> 4;
    const int off = 2 * (co0 - 4 * g + 8 * (g >> 1)) + (g & 1) * 2 * COUT;
    if constexpr (GO) {
        if (store && t < L)
            *reinterpret_cast<u32x4*>(gout + (size_t)t * 4 * COUT + off) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    } else if (store) {
        *reinterpret_cast<u32x4*>(rowp + off) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    }
}

// Does 3-tap packing fold the ResBlock residual into the GEMM (see mma_x3)?
// Must agree with the host packer (res_fold_channels in vocoder_fused.h).
template <int C>
constexpr bool kFold = res_fold_channels(C);

// One work item: NTT tiles of NMB (phase, m-block) rows (consecutive m-blocks
// of one phase, co0 .. co0 + 16 NMB, sharing the B fragments) starting at
// tile0.  Output position of column j (relative to the layer's first input
// q0 / a0): t = (p0 + j) * RR + ph (RR = 1, ph = 0 for conv3).
// corr (the composed stage2 head): per-(phase, channel) terms subtracted from
// the outputs of input column qe (an utterance edge), before the activation.
template <int CIN, int COUT, int NTAP, int STEP, int RSI, int RSO, int NTT, int ACT, bool RES, bool XR, int RR,
          int JMAX, int NMB, bool PRE, bool GO = false, int PDM = 4, int BP = 0>
__device__ __forceinline__ void run_item(const u32x4* __restrict__ wp, const float* __restrict__ bias,
                                         const unsigned char* bp, const unsigned char* xr, XW out, int co0, int p0,
                                         int ph, int tile0, int L, u32x4 (&a)[pd_of<CIN, NTAP, NMB, PDM>()][NMB][2],
                                         const u32x4* wp_next, unsigned char* gout = nullptr,
                                         const unsigned char* corr = nullptr, int qe = 0) {
    constexpr int WS = nkb_of<CIN, NTAP>() * 128;  // u32x4 between consecutive m-blocks' weights
    f32x4 acc[NMB][NTT];
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
        f32x4 bv;
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = co0 + 16 * m + r < COUT ? bias[co0 + 16 * m + r] : 0.f;
#pragma unroll
        for (int n = 0; n < NTT; ++n) acc[m][n] = bv;
    }
    mma_x3<CIN, NTAP, STEP, RSI, NTT, XR, NMB, WS, PRE, false, PDM, BP>(wp, bp, xr, acc, a, wp_next);
    const bool edge = (p0 + tile0 * 16) * RR < 0 || (p0 + (tile0 + NTT) * 16) * RR > L;
    const int li = threadIdx.x & 15, g = (threadIdx.x & 63) >> 4;
    if (corr) {  // wave-uniform
#pragma unroll
        for (int n = 0; n < NTT; ++n)
            if (qe >= p0 + (tile0 + n) * 16 && qe < p0 + (tile0 + n) * 16 + 16 && p0 + (tile0 + n) * 16 + li == qe) {
#pragma unroll
                for (int m = 0; m < NMB; ++m) {
                    const f32x4 c = *reinterpret_cast<const f32x4*>(corr + 4 * (ph * COUT + co0 + 16 * m));
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[m][n][r] -= c[r];
                }
            }
    }
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
        const int cm = co0 + 16 * m;
        const bool rows_ok = cm - 4 * g + 8 * (g >> 1) < COUT;  // after the swap: this lane's 8 channels
#pragma unroll
        for (int n = 0; n < NTT; ++n) {
            const int j = (tile0 + n) * 16 + li;
            const bool col_ok = ((tile0 + n + 1) * 16 <= JMAX) || j < JMAX;
            store_tile<COUT, RSO, ACT, RES, GO>(acc[m][n], out, (p0 + j) * RR + ph, cm, L, edge, rows_ok && col_ok,
                                                gout);
        }
    }
}

// Work items of a layer: (row, chunk) with each row's NTILES split into
// NCH = ceil(NTILES / NT) chunks whose sizes differ by at most one tile
// (25 tiles, NT 4: seven chunks of 3-4 rather than six of 4 and one of 1),
// dealt round-robin over the waves.  Chunk sizes are compile-time (QLO or
// QLO + 1): two instantiations of the item body, no per-tile guards.
template <int NTILES, int NT>
struct Chunks {
    static constexpr int NCH = (NTILES + NT - 1) / NT, QLO = NTILES / NCH, QHI = QLO + (NTILES % NCH ? 1 : 0);
    __device__ static int lo(int k) { return k * NTILES / NCH; }
};

// Weight-fragment hand-off between the layers of a kernel in which every wave
// does exactly one item per layer (the stage1 head): the loads of the next
// layer's first four k-blocks are issued right after the current item's last
// MFMA, so they are in flight during its epilogue and the barrier.
typedef u32x4 APipe[4][1][2];

// Work items of a layer: (m-block group, chunk) for conv3, (phase, m-block
// group, chunk) for the transposed convs; NMB m-blocks per item share the B
// reads.  ONE (= the wave count, one item each): the wave's item is its index, its
// first k-blocks' weights were loaded into `ap` by the previous layer, and it
// starts the loads of `wp_next` (the next layer's item) into `ap`.
template <int CIN, int COUT, int NT, int NPOS, int NMB>
struct Conv3Items {
    static constexpr int MB = (COUT + 15) / 16, NKB = nkb_of<CIN, 3>(), MG = MB / NMB;
    static_assert(MB % NMB == 0, "m-block groups");
    using CH = Chunks<(NPOS + 15) / 16, NT>;
    static constexpr int N = MG * CH::NCH;
    __device__ static const u32x4* wp(const u32x4* Wp, int item) {
        return Wp + (size_t)(item % MG) * NMB * NKB * 128 + (threadIdx.x & 63);
    }
};
template <int CIN, int COUT, int R, int NT, int NQ, int NMB>
struct ConvTItems {
    static constexpr int MB = (COUT + 15) / 16, NKB = nkb_of<CIN, 2>(), MG = MB / NMB;
    static_assert(MB % NMB == 0, "m-block groups");
    using CH = Chunks<(NQ + 15) / 16, NT>;
    static constexpr int N = R * MG * CH::NCH;
    __device__ static const u32x4* wp(const u32x4* Wp, int item) {
        const int rg = item % (R * MG), ph = rg / MG, mb = (rg - ph * MG) * NMB;
        return Wp + (size_t)(ph * MB + mb) * NKB * 128 + (threadIdx.x & 63);
    }
};

// Conv1d(k=3, pad=1): abs positions [a0, a0+NPOS) of `out` from `in`.
// RES: out += conv(in) (ResBlock conv2, x = out), folded into the GEMM for
// 8/16 channels, read back in the epilogue otherwise.
// GO: store the output tiles to global rows (gout) instead of `out`.
template <int CIN, int COUT, int NT, int ACT, bool RES, int RSI, int RSO, int NPOS, int NMB = 1, int ONE = 0,
          bool GO = false, int PDM = 4, int BP = 0>
__device__ __forceinline__ void xconv3(const u32x4* __restrict__ Wp, const float* __restrict__ bias, XW in, XW out,
                                       int a0, int L, APipe* ap = nullptr, const u32x4* wp_next = nullptr,
                                       unsigned char* gout = nullptr) {
    using IT = Conv3Items<CIN, COUT, NT, NPOS, NMB>;
    using CH = typename IT::CH;
    constexpr int MG = IT::MG;
    constexpr bool FOLD = RES && kFold<CIN>;
    static_assert(!FOLD || (CIN == COUT && RSI == RSO), "folded residual: x has the conv's input layout");
    static_assert(!ONE || (IT::N == ONE && NMB == 1 && pd_of<CIN, 3, 1>() == 4), "one item per wave");
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    auto body = [&](int item, auto pre) {
        constexpr bool PRE = decltype(pre)::value;
        const int mb = (item % MG) * NMB, k = item / MG;
        const int tile0 = CH::lo(k), nt = CH::lo(k + 1) - tile0;
        const int co0 = mb * 16 + 4 * g;
        const int p = a0 + tile0 * 16 + li;  // this lane's output position in tile 0
        const u32x4* wp = IT::wp(Wp, item);
        const unsigned char* bp = in.p + (p - 1 - in.start) * RSI;
        const unsigned char* xr = out.p + (p - out.start) * RSO;
        u32x4 al[pd_of<CIN, 3, NMB, PDM>()][NMB][2];
        auto& a = [&]() -> auto& {
            if constexpr (PRE) return *ap;
            else return al;
        }();
        if (nt == CH::QHI)
            run_item<CIN, COUT, 3, 1, RSI, RSO, CH::QHI, ACT, RES && !FOLD, FOLD, 1, NPOS, NMB, PRE, GO, PDM, BP>(
                wp, bias, bp, xr, out, co0, a0, 0, tile0, L, a, wp_next, gout);
        else
            run_item<CIN, COUT, 3, 1, RSI, RSO, CH::QLO, ACT, RES && !FOLD, FOLD, 1, NPOS, NMB, PRE, GO, PDM, BP>(
                wp, bias, bp, xr, out, co0, a0, 0, tile0, L, a, wp_next, gout);
    };
    if constexpr (ONE) {
        body(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), std::true_type{});
    } else {
#pragma unroll 1
        for (int item = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); item < IT::N; item += blockDim.x >> 6)
            body(item, std::false_type{});
    }
}

// leaky(ConvTranspose1d(k=2R, stride R, pad R/2)): inputs q in [q0, q0+NQ)
// give outputs t = q*R + ph.  Phase ph reads taps (q, q-1) if ph + R/2 < R,
// else (q+1, q): B base row q + d0, tap k at row q + d0 - k.
template <int CIN, int COUT, int R, int NT, int RSI, int RSO, int NQ, int NMB = 1, int ONE = 0, int PDM = 4>
__device__ __forceinline__ void xconvT(const u32x4* __restrict__ Wp, const float* __restrict__ bias, XW in, XW out,
                                       int q0, int L, APipe* ap = nullptr, const u32x4* wp_next = nullptr) {
    using IT = ConvTItems<CIN, COUT, R, NT, NQ, NMB>;
    using CH = typename IT::CH;
    constexpr int MG = IT::MG, PAD = R / 2;
    static_assert(!ONE || (IT::N == ONE && NMB == 1 && pd_of<CIN, 2, 1>() == 4), "one item per wave");
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    auto body = [&](int item, auto pre) {
        constexpr bool PRE = decltype(pre)::value;
        const int rg = item % (R * MG), k = item / (R * MG);  // rg = ph*MG + m-block group
        const int ph = rg / MG, mb = (rg - ph * MG) * NMB;
        const int tile0 = CH::lo(k), nt = CH::lo(k + 1) - tile0;
        const int d0 = (ph + PAD < R) ? 0 : 1;
        const int co0 = mb * 16 + 4 * g;
        const u32x4* wp = IT::wp(Wp, item);
        const unsigned char* bp = in.p + (q0 + tile0 * 16 + li + d0 - in.start) * RSI;
        u32x4 al[pd_of<CIN, 2, NMB, PDM>()][NMB][2];
        auto& a = [&]() -> auto& {
            if constexpr (PRE) return *ap;
            else return al;
        }();
        if (nt == CH::QHI)
            run_item<CIN, COUT, 2, -1, RSI, RSO, CH::QHI, ACT_LEAKY, false, false, R, NQ, NMB, PRE, false, PDM>(
                wp, bias, bp, nullptr, out, co0, q0, ph, tile0, L, a, wp_next);
        else
            run_item<CIN, COUT, 2, -1, RSI, RSO, CH::QLO, ACT_LEAKY, false, false, R, NQ, NMB, PRE, false, PDM>(
                wp, bias, bp, nullptr, out, co0, q0, ph, tile0, L, a, wp_next);
    };
    if constexpr (ONE) {
        body(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6), std::true_type{});
    } else {
#pragma unroll 1
        for (int item = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); item < IT::N; item += blockDim.x >> 6)
            body(item, std::false_type{});
    }
}

// The composed input_conv o ConvT1 on the generic item path (the stage2
// head): head_convT1c_planar's layer over (phase, m-block, chunk) items, 4
// mel taps (frames q + d0 + 1 - k), per-phase bias, edge terms from `corr`.
template <int MP, int COUT, int NT, int RSI, int RSO, int NQ, int PDM = 4, int BP = 0>
__device__ __forceinline__ void xconvT1c(const u32x4* __restrict__ Wp, const float* __restrict__ bias,
                                         const unsigned char* corr, XW mel, XW out, int q0, int T) {
    constexpr int R = 4, MB = (COUT + 15) / 16, NKB = nkb_of<MP, 4>();
    using CH = Chunks<(NQ + 15) / 16, NT>;
    constexpr int N = R * MB * CH::NCH;
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
#pragma unroll 1
    for (int item = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); item < N; item += blockDim.x >> 6) {
        const int rg = item % (R * MB), k = item / (R * MB), ph = rg / MB, mb = rg - ph * MB;
        const int tile0 = CH::lo(k), nt = CH::lo(k + 1) - tile0, d0 = ph < 2 ? 0 : 1, co0 = mb * 16 + 4 * g;
        const u32x4* wp = Wp + (size_t)(ph * MB + mb) * NKB * 128 + lane;
        const unsigned char* bp = mel.p + (q0 + tile0 * 16 + li + d0 + 1 - mel.start) * RSI;
        const int qe = ph < 2 ? 0 : T - 1;
        u32x4 al[pd_of<MP, 4, 1, PDM>()][1][2];
        if (nt == CH::QHI)
            run_item<MP, COUT, 4, -1, RSI, RSO, CH::QHI, ACT_LEAKY, false, false, R, NQ, 1, false, false, PDM, BP>(
                wp, bias + ph * COUT, bp, nullptr, out, co0, q0, ph, tile0, 4 * T, al, nullptr, nullptr, corr, qe);
        else
            run_item<MP, COUT, 4, -1, RSI, RSO, CH::QLO, ACT_LEAKY, false, false, R, NQ, 1, false, false, PDM, BP>(
                wp, bias + ph * COUT, bp, nullptr, out, co0, q0, ph, tile0, 4 * T, al, nullptr, nullptr, corr, qe);
    }
}

// Edge terms of the composed stage2 head: thread v (4 x COUT threads) sums
// E[v][0..M) . mel[edge] + e[v] into corr (the windows holding an edge only).
template <int M, int MP, int COUT, int RSM>
__device__ __forceinline__ void head_edge_terms_s2(const float* __restrict__ hce, XW mel, int T, bool left,
                                                   bool right, unsigned char* corr) {
    const int v = threadIdx.x, ph = v / COUT;
    if (v >= 4 * COUT) return;
    const bool need = ph < 2 ? left : right;
    float d = 0.f;
    if (need) {
        const unsigned char* row = mel.p + ((ph < 2 ? 0 : T - 1) - mel.start) * RSM;
        d = hce[4 * COUT * MP + v];
#pragma unroll
        for (int o = 0; o < M / 8; ++o) {
            const h8 hi = *reinterpret_cast<const h8*>(row + 16 * o);
            const h8 lo = *reinterpret_cast<const h8*>(row + 2 * MP + 16 * o);
            const float4 e0 = *reinterpret_cast<const float4*>(hce + (size_t)v * MP + 8 * o);
            const float4 e1 = *reinterpret_cast<const float4*>(hce + (size_t)v * MP + 8 * o + 4);
            const float e[8] = {e0.x, e0.y, e0.z, e0.w, e1.x, e1.y, e1.z, e1.w};
#pragma unroll
            for (int i = 0; i < 8; ++i) d = fmaf(e[i], (float)hi[i] + (float)lo[i], d);
        }
    }
    *reinterpret_cast<float*>(corr + 4 * v) = d;
}

// ---------------------------------------------------------------------------
// Phase-planar head (stage1, one item per wave).  ConvT1's output u (x4) and
// ResBlock1's hidden h are kept as 4 planes of 64 rows, plane p = positions
// t = 4q + p for q in [qs(p), qs(p) + 64): u: qs = f0 - 1 for p >= 2, else
// f0; h: qs = f0 - 1 for p = 3, else f0 - exactly the positions the next
// layer reads.  Against the position-major layout (ConvT1 NQ = 65 inputs =
// 5 tiles per phase, outputs 4 rows apart) this is 4 tiles per phase (20 %
// fewer ConvT1 MFMAs) and conflict-free epilogue stores (consecutive lanes,
// consecutive rows); the ResBlock1 convs become per-phase GEMMs whose three
// taps read rows of the neighbouring planes (mma_x3 with tap bases).
// Plane rows are swizzled: row r's 16-B chunks c and c ^ 1 trade places when
// bit 2 of r is set (plane_sw).  A tile's epilogue writes rows li of one
// chunk per lane group, 8 consecutive lanes per ds_write_b128 pass; at a row
// stride of 18 chunks rows r and r + 4 met in the same banks (2-way); the
// swizzle moves rows 4-7 by 4 banks.  The B-fragment reads (4 lane groups
// of 16, chunks c0 + g) stay conflict-free: the bit only permutes the chunk
// pairs of one k-block, per lane, and folds into the tap bases.
__device__ __forceinline__ int plane_sw(int r) { return (r >> 2) & 1; }
__device__ __forceinline__ int qs_u(int p, int f0) { return f0 - (p >= 2 ? 1 : 0); }
__device__ __forceinline__ int qs_h(int p, int f0) { return f0 - (p == 3 ? 1 : 0); }
constexpr int kPlane = 64;

// Epilogue of one tile into an explicit plane row (rowp, swizzle bit rsw) or
// straight to global (GO); the residual, if any, is read from plane row xrow
// (swizzle bit xsw).
template <int COUT, int ACT, bool RES, bool GO>
__device__ __forceinline__ void store_row(const f32x4& acc, unsigned char* rowp, const unsigned char* xrow, int co0,
                                          bool zero, bool store, unsigned char* gout, int t, int rsw, int xsw = 0) {
    const int g = (threadIdx.x & 63) >> 4;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = acc[r];
    if constexpr (ACT == ACT_LEAKY) leaky4(v);
    if constexpr (RES) {  // channels co0 .. co0 + 3: chunk co0 / 8, half g & 1
        const unsigned char* row = xrow + 2 * (co0 - 4 * g) + 16 * ((g >> 1) ^ xsw) + 8 * (g & 1);
        const h4 hi = *reinterpret_cast<const h4*>(row), lo = *reinterpret_cast<const h4*>(row + 2 * COUT);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += (float)hi[r] + (float)lo[r];
    }
    if (zero) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = 0.f;
    }
    unsigned h0, h1, l0, l1;
    split2u(v[0], v[1], h0, l0);
    split2u(v[2], v[3], h1, l1);
    const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
    const int off = 2 * (co0 - 4 * g) + (g & 1) * 2 * COUT;
    if (store) {
        if constexpr (GO)
            *reinterpret_cast<u32x4*>(gout + (size_t)t * 4 * COUT + off + 16 * (g >> 1)) =
                u32x4{s0[0], s1[0], s0[1], s1[1]};
        else
            *reinterpret_cast<u32x4*>(rowp + off + 16 * ((g >> 1) ^ rsw)) = u32x4{s0[0], s1[0], s0[1], s1[1]};
    }
}

// ConvT1 (x4, k 8, pad 2) + leaky from the position-major inconv output (in,
// frames f0-2 ..) into the u planes; item = wave = (phase, m-block).
template <int CIN, int COUT, int RSI, int RSO>
__device__ __forceinline__ void head_convT1_planar(const u32x4* __restrict__ Wp, const float* __restrict__ bias,
                                                   XW in, unsigned char* u, int f0, int L, APipe* ap,
                                                   const u32x4* wp_next) {
    constexpr int MB = COUT / 16, NKB = nkb_of<CIN, 2>(), NT = 4;
    const int item = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ph = item / MB, mb = item - ph * MB;
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4, co0 = mb * 16 + 4 * g;
    const int qs = qs_u(ph, f0), d0 = ph < 2 ? 0 : 1;  // taps (q + d0, q + d0 - 1)
    const u32x4* wp = Wp + (size_t)(ph * MB + mb) * NKB * 128 + lane;
    const unsigned char* bp = in.p + (qs + li + d0 - in.start) * RSI;
    f32x4 acc[1][NT];
    f32x4 bv;
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bias[co0 + r];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[0][n] = bv;
    mma_x3<CIN, 2, -1, RSI, NT, false, 1, NKB * 128, true>(wp, bp, nullptr, acc, *ap, wp_next);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int t = 4 * (qs + 16 * n + li) + ph;
        store_row<COUT, ACT_LEAKY, false, false>(acc[0][n], u + (ph * kPlane + 16 * n + li) * RSO, nullptr, co0,
                                                 t < 0 || t >= L, true, nullptr, t, plane_sw(li));
    }
}

// input_conv composed into ConvT1 (stage1 head, round 2): the input conv
// (k3, no activation) feeds only ConvT1, which is linear before its leaky, so
// u = leaky(Wc * mel + bc[ph]) with Wc[ph] = W_T[ph] o W_in a 4-tap transposed
// conv straight from the mel window (output phase ph at input column q reads
// mel frames q + d0 + 1 - k, k = 0..3, d0 = 0 for ph < 2 else 1): K = 4 x 64
// mel channels, the same 8 k-blocks as ConvT1's 2 x 128, and no input-conv
// layer (its MFMAs, barrier and LDS round trip) at all.  The reference's
// ConvT1 sees zeros at input frames -1 and T, where the composed form sees
// the input conv of the zero-padded mel (b_in + W_in[.,.,2] mel[0] /
// b_in + W_in[.,.,0] mel[T-1]); outputs t = 0, 1 and 4T - 2, 4T - 1 subtract
// that term: E[ph][co][m] . mel[edge] + e[ph][co] (hce: [4][C1][MP] then
// [4][C1], fp32; phases 0, 1 left edge, 2, 3 right edge).  The edge windows
// of an utterance compute those 256 sums cooperatively before the layer
// (head_edge_terms: their table loads issued at kernel start) into an LDS
// table `corr` that the lanes holding the edge outputs read (null elsewhere).
// (A per-lane loop over the table in the epilogue made the edge windows the
// kernel's critical path.)  Bias bc: [4][C1] (it depends on the phase).
// The composed head's edge terms, all 1024 threads of an edge window: thread
// t sums 16 of the 64 products of value v = t / 4 (= ph * COUT + co); four
// adjacent lanes reduce by shuffles.  ev: this thread's 16 table entries,
// loaded at kernel start (head_edge_load).
template <int MP, int COUT>
__device__ __forceinline__ void head_edge_load(const float* __restrict__ hce, float4 (&ev)[4], float& eb) {
    static_assert(4 * COUT * 4 == 1024 && MP == 64, "1024 threads: 4 phases x COUT values x 4 parts of 16");
    const int t = threadIdx.x, v = t >> 2, part = t & 3;
#pragma unroll
    for (int i = 0; i < 4; ++i) ev[i] = *reinterpret_cast<const float4*>(hce + (size_t)v * MP + 16 * part + 4 * i);
    eb = hce[4 * COUT * MP + v];
}
template <int MP, int COUT, int RSM>
__device__ __forceinline__ void head_edge_terms(const float4 (&ev)[4], float eb, XW mel, int T, bool left, bool right,
                                                unsigned char* corr) {
    const int t = threadIdx.x, v = t >> 2, part = t & 3, ph = v / COUT;
    const bool need = ph < 2 ? left : right;  // wave-uniform (16 waves, 4 per phase)
    float d = 0.f;
    if (need) {
        const unsigned char* row = mel.p + ((ph < 2 ? 0 : T - 1) - mel.start) * RSM + 2 * 16 * part;
        const float e[16] = {ev[0].x, ev[0].y, ev[0].z, ev[0].w, ev[1].x, ev[1].y, ev[1].z, ev[1].w,
                             ev[2].x, ev[2].y, ev[2].z, ev[2].w, ev[3].x, ev[3].y, ev[3].z, ev[3].w};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const h8 hi = *reinterpret_cast<const h8*>(row + 16 * h);
            const h8 lo = *reinterpret_cast<const h8*>(row + 2 * MP + 16 * h);
#pragma unroll
            for (int i = 0; i < 8; ++i) d = fmaf(e[8 * h + i], (float)hi[i] + (float)lo[i], d);
        }
    }
    d += __shfl_xor(d, 1);
    d += __shfl_xor(d, 2);
    if (part == 0) *reinterpret_cast<float*>(corr + 4 * v) = need ? d + eb : 0.f;
}

template <int MP, int COUT, int RSM, int RSO>
__device__ __forceinline__ void head_convT1c_planar(const u32x4* __restrict__ Wp, const float* __restrict__ bias,
                                                    const unsigned char* corr, XW mel, unsigned char* u, int f0,
                                                    int T, APipe* ap, const u32x4* wp_next) {
    constexpr int MB = COUT / 16, NKB = nkb_of<MP, 4>(), NT = 4;
    static_assert(NKB == 8 && pd_of<MP, 4, 1>() == 4, "the ConvT1 weight pipeline shape");
    const int item = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int ph = item / MB, mb = item - ph * MB;
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4, co0 = mb * 16 + 4 * g;
    const int qs = qs_u(ph, f0), d0 = ph < 2 ? 0 : 1;  // taps: mel frames q + d0 + 1 - k
    const u32x4* wp = Wp + (size_t)(ph * MB + mb) * NKB * 128 + lane;
    const unsigned char* bp = mel.p + (qs + li + d0 + 1 - mel.start) * RSM;
    f32x4 acc[1][NT];
    f32x4 bv;
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bias[ph * COUT + co0 + r];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[0][n] = bv;
    mma_x3<MP, 4, -1, RSM, NT, false, 1, NKB * 128, true>(wp, bp, nullptr, acc, *ap, wp_next);
    const int L = 4 * T, qe = ph < 2 ? 0 : T - 1;  // the input column of this phase's edge outputs
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int q = qs + 16 * n + li, t = 4 * q + ph;
        if (corr && qe >= qs + 16 * n && qe < qs + 16 * n + 16) {  // wave-uniform: a tile with an edge output
            if (q == qe) {
                const f32x4 c = *reinterpret_cast<const f32x4*>(corr + 4 * (ph * COUT + co0));
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[0][n][r] -= c[r];
            }
        }
        store_row<COUT, ACT_LEAKY, false, false>(acc[0][n], u + (ph * kPlane + 16 * n + li) * RSO, nullptr, co0,
                                                 t < 0 || t >= L, true, nullptr, t, plane_sw(li));
    }
}

// ResBlock1 conv (k3, pad 1) between planes: input planes start at qsi(p),
// output plane p covers q in [qso(p), +64).  CONV2: + x from the u planes,
// stored straight to U1 (t < L and q < f0 + tf only); else leaky into the
// h planes (0 outside [0, L)).
template <int C, int RS, bool CONV2>
__device__ __forceinline__ void head_rb1_planar(const u32x4* __restrict__ Wp, const float* __restrict__ bias,
                                                const unsigned char* in, unsigned char* out,
                                                const unsigned char* x, int f0, int tf, int L, APipe* ap,
                                                const u32x4* wp_next, unsigned char* gout) {
    constexpr int MB = C / 16, NKB = nkb_of<C, 3>(), NT = 4;
    const int item = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int p = item / MB, mb = item - p * MB;
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4, co0 = mb * 16 + 4 * g;
    const int qo = CONV2 ? f0 : qs_h(p, f0);
    const unsigned char* tb[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int pd = p + d - 1, dq = pd < 0 ? -1 : (pd > 3 ? 1 : 0), pi = pd - 4 * dq;
        const int qsi = CONV2 ? qs_h(pi, f0) : qs_u(pi, f0);
        const int r = qo + dq - qsi + li;  // row in plane pi (>= 0)
        tb[d] = in + (pi * kPlane + r) * RS + 16 * (g ^ plane_sw(r));
    }
    const u32x4* wp = Wp + (size_t)mb * NKB * 128 + lane;
    f32x4 acc[1][NT];
    f32x4 bv;
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bias[co0 + r];
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[0][n] = bv;
    mma_x3<C, 3, 1, RS, NT, false, 1, NKB * 128, true, true>(wp, nullptr, nullptr, acc, *ap, wp_next, tb);
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const int q = qo + 16 * n + li, t = 4 * q + p;
        if constexpr (CONV2) {
            const int xr = q - qs_u(p, f0);
            store_row<C, ACT_NONE, true, true>(acc[0][n], nullptr, x + (p * kPlane + xr) * RS, co0, false,
                                               q < f0 + tf && t < L, gout, t, 0, plane_sw(xr));
        } else {
            store_row<C, ACT_LEAKY, false, false>(acc[0][n], out + (p * kPlane + 16 * n + li) * RS, nullptr, co0,
                                                  t < 0 || t >= L, true, nullptr, t, plane_sw(li));
        }
    }
}

// ---------------------------------------------------------------------------
// Global <-> LDS.  Trip counts are compile-time (NTHR threads, N rows) so
// every thread issues all its global loads before the first LDS store.
// mel -> window rows [0, N) (abs start + r), MP channels (zero past M).
template <bool TRANS, int M, int MP, int RS, int N, int NTHR>
__device__ __forceinline__ void gload_mel(const float* __restrict__ g, int T, XW dst) {
    if (TRANS) {  // [T][M]: an item = 8 channels of one frame (two 16-B loads); consecutive threads take
                  // consecutive frames, so the LDS stores are the [M][T] branch's b128 pattern (was 16
                  // threads per frame row with 8-B hi / lo stores: [B,T,M] 0.2 us/step behind [B,M,T] in
                  // tools/probe/mel_layout_ab.py, now level)
        constexpr int OCT = MP / 8, TOT = N * OCT, IT = (TOT + NTHR - 1) / NTHR;
        float4 x[IT][2];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = threadIdx.x + k * NTHR;
            const int o = i / N, r = i - o * N, t = dst.start + r;
            const bool in = i < TOT && t >= 0 && t < T;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int c = 8 * o + 4 * h;
                x[k][h] = make_float4(0.f, 0.f, 0.f, 0.f);
                if (in && c < M) x[k][h] = *reinterpret_cast<const float4*>(g + (size_t)t * M + c);
            }
        }
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = threadIdx.x + k * NTHR;
            if (i < TOT) {
                const int o = i / N, r = i - o * N;
                unsigned hh[4], ll[4];
                split2u(x[k][0].x, x[k][0].y, hh[0], ll[0]);
                split2u(x[k][0].z, x[k][0].w, hh[1], ll[1]);
                split2u(x[k][1].x, x[k][1].y, hh[2], ll[2]);
                split2u(x[k][1].z, x[k][1].w, hh[3], ll[3]);
                unsigned char* row = dst.p + r * RS + 16 * o;
                *reinterpret_cast<u32x4*>(row) = u32x4{hh[0], hh[1], hh[2], hh[3]};
                *reinterpret_cast<u32x4*>(row + 2 * MP) = u32x4{ll[0], ll[1], ll[2], ll[3]};
            }
        }
    } else {  // [M][T]: an item = 8 channels of one frame; consecutive threads take consecutive frames
        constexpr int OCT = MP / 8, TOT = N * OCT, IT = (TOT + NTHR - 1) / NTHR;
        float x[IT][8];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = threadIdx.x + k * NTHR;
            const int o = i / N, r = i - o * N, t = dst.start + r;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const int c = 8 * o + e;
                x[k][e] = (i < TOT && t >= 0 && t < T && c < M) ? g[(size_t)c * T + t] : 0.f;
            }
        }
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = threadIdx.x + k * NTHR;
            if (i < TOT) {
                const int o = i / N, r = i - o * N;
                unsigned hh[4], ll[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) split2u(x[k][2 * e], x[k][2 * e + 1], hh[e], ll[e]);
                unsigned char* row = dst.p + r * RS + 16 * o;
                *reinterpret_cast<u32x4*>(row) = u32x4{hh[0], hh[1], hh[2], hh[3]};
                *reinterpret_cast<u32x4*>(row + 2 * MP) = u32x4{ll[0], ll[1], ll[2], ll[3]};
            }
        }
    }
}

// rows of 4C bytes (hi|lo) at global positions [start, start+N), zero outside [0, Lg)
template <int C, int RS, int N, int NTHR>
__device__ __forceinline__ void gload_rows(const unsigned char* __restrict__ g, int Lg, XW dst) {
    constexpr int Q = C / 4, TOT = N * Q, IT = (TOT + NTHR - 1) / NTHR;  // 16-B chunks
    u32x4 v[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int i = threadIdx.x + k * NTHR;
        const int r = i / Q, q = i - r * Q, t = dst.start + r;
        v[k] = u32x4{0u, 0u, 0u, 0u};
        if (i < TOT && t >= 0 && t < Lg) v[k] = *reinterpret_cast<const u32x4*>(g + (size_t)t * 4 * C + q * 16);
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int i = threadIdx.x + k * NTHR;
        const int r = i / Q, q = i - r * Q;
        if (i < TOT) *reinterpret_cast<u32x4*>(dst.p + r * RS + q * 16) = v[k];
    }
}

template <int C, int RS, int N, int NTHR>
__device__ __forceinline__ void gstore_rows(unsigned char* __restrict__ g, int Lg, XW src, int a0) {
    constexpr int Q = C / 4, TOT = N * Q, IT = (TOT + NTHR - 1) / NTHR;
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int i = threadIdx.x + k * NTHR;
        const int r = i / Q, q = i - r * Q, t = a0 + r;
        if (i < TOT && t < Lg)
            *reinterpret_cast<u32x4*>(g + (size_t)t * 4 * C + q * 16) =
                *reinterpret_cast<const u32x4*>(src.p + (t - src.start) * RS + q * 16);
    }
}

// ---------------------------------------------------------------------------
// Window plans (rows; the same receptive-field arithmetic as the f32 plans).
// Two LDS regions per kernel, A then B, with buffers aliased by lifetime.
// Region-A buffers are sized to the rows actually written; the garbage
// columns of a partial 16-wide tile may read past them into region B, which
// only feeds columns that are never stored (an MFMA output column depends
// on its own B column only).  Region-B buffers keep the full read extent.
template <int MP, int C, int TF, bool PL = false>
struct HeadPlan {  // A: a0 | h   B: mel | u
    static constexpr int C1 = C / 2;
    static constexpr int RS_M = rs_for(MP), RS_C = rs_for(C), RS_1 = rs_for(C1);
    static constexpr int MEL_N = TF + 6, A0_N = TF + 4, NQ = TF + 2, H_N = 4 * TF + 2, O_N = 4 * TF;
    static constexpr int CAP_MEL = cmax(MEL_N, rup16(A0_N) + 2);
    static constexpr int CAP_U = cmax(4 * NQ, rup16(H_N) + 4);
    // PL: the phase-planar path keeps h and u as 4 planes of 64 rows
    static constexpr int RA = cmax(A0_N * RS_C, cmax(H_N, PL ? 4 * 64 : 0) * RS_1);
    static constexpr int LDS_BYTES = RA + cmax(CAP_MEL * RS_M, cmax(CAP_U, PL ? 4 * 64 + 4 : 0) * RS_1);
};

template <int CI, int W>
struct MidPlan {  // A: in | h   B: u
    static constexpr int CO = CI / 2;
    static constexpr int RS_I = rs_for(CI), RS_O = rs_for(CO);
    static constexpr int IN_N = W + 4, NQ = W + 2, H_N = 4 * W + 2, O_N = 4 * W;
    static constexpr int CAP_U = cmax(4 * NQ, rup16(H_N) + 4);
    static constexpr int RA = cmax(IN_N * RS_I, H_N * RS_O);
    static constexpr int LDS_BYTES = RA + CAP_U * RS_O;
};

template <int CI, int W>
struct TailPlan {  // A: in | h3 | u4   B: u3 | h4
    static constexpr int C3 = CI / 2, C4 = CI / 4;
    static constexpr int RS_I = rs_for(CI), RS_3 = rs_for(C3), RS_4 = rs_for(C4);
    static constexpr int IN_N = W + 8, NQ3 = W + 6, H3_N = 2 * W + 8, O3_N = 2 * W + 6;
    static constexpr int NQ4 = 2 * W + 4, H4_N = 4 * W + 4, O4_N = 4 * W + 2, A_N = 4 * W;
    static constexpr int CAP_U3 = cmax(2 * NQ3, cmax(rup16(H3_N) + 3, rup16(NQ4) + 5));
    static constexpr int CAP_H4 = cmax(H4_N, rup16(O4_N) + 2);
    static constexpr int RA = cmax(IN_N * RS_I, cmax(H3_N * RS_3, 2 * NQ4 * RS_4));
    static constexpr int LDS_BYTES = RA + cmax(CAP_U3 * RS_3, CAP_H4 * RS_4);
};

// Tilings.  Per kernel: waves per workgroup (*W), window (TF frames / W2 /
// W3 positions), launch-bound waves per SIMD (*MIN: 4 -> <= 128 VGPRs), and
// NT_* = tile-chunk size per layer, chosen so each layer's items come to a
// multiple of the wave count.  Stage1 at B=32, T=500 (bench): head 8 x 32 =
// 256 workgroups (one per CU), mid 16 x 32 = 512 (two rounds), tail 48 x 32 =
// 1536 at two per CU (three full rounds).
#ifndef X3_HEAD_TF  // head tiling experiments (tools/probe): frames per window, waves, tile chunks
#define X3_HEAD_TF 63
#define X3_HEAD_HW 16
#define X3_NT_IN 3
#define X3_NT_T1 5
#define X3_NT_R1 4
#define X3_G_T1 1
#define X3_G_R1 1
#endif
#ifndef X3_PLANAR  // stage1 head: phase-planar ConvT1 / ResBlock1 (0: position-major x3 layers)
#define X3_PLANAR 1
#endif
struct CfgS1 {
    static constexpr int PDM = 4;
    static constexpr int M = 64, MP = 64, C = 128;
    static constexpr int TF = X3_HEAD_TF, HW = X3_HEAD_HW, HMIN = 4;
    static constexpr int W2 = 125, MW = 16, MMIN = 4;
    static constexpr int W3 = 168, TW = 8, TMIN = 4;
    static constexpr int NT_IN = X3_NT_IN, NT_T1 = X3_NT_T1, NT_R1 = X3_NT_R1, NT_T2 = 4, NT_R2 = 4, NT_T3 = 3,
                         NT_R3 = 3, NT_T4 = 3, NT_R4 = 6;
    // head ConvT1 / ResBlock1: m-blocks per item sharing B (2: half the B reads)
    static constexpr int G_T1 = X3_G_T1, G_R1 = X3_G_R1;
};
#ifndef X3S2_TF  // stage2 tiling experiments (tools/probe/s2_tiles.sh)
#define X3S2_TF 16
#define X3S2_NT_R1 5
#endif
#ifndef X3S2_W2
#define X3S2_W2 30
#define X3S2_NT_R2 4
#endif
#ifndef X3S2_W3
#define X3S2_W3 120
#define X3S2_NT_T3 4
#define X3S2_NT_R3 4
#endif
#ifndef X3S2_HW  // stage2 head waves per workgroup (tiling experiments)
#define X3S2_HW 8
#endif
#ifndef X3S2_HBP  // stage2 head: B-fragment reads one k-block ahead (CfgS2::HBP, mma_x3 BP)
#define X3S2_HBP 1
#endif
#ifndef X3S2W_HBP  // the 16-wave stage2 head of large grids (CfgS2H24::HBP)
#define X3S2W_HBP 2
#endif
#ifndef X3S2W_TF  // the 16-wave stage2 head's window (CfgS2H24::TF)
#define X3S2W_TF 24
#endif
#ifndef X3S2A_W2  // the small-grid stage2 mid window (CfgS2Alt::W2)
#define X3S2A_W2 33
#endif
#ifndef X3S2_PDM  // stage2 weight-fragment k-blocks in flight per item (mma_x3)
#define X3S2_PDM 4
#endif
struct CfgS2 {
    static constexpr int M = 80, MP = 96, C = 256;
    static constexpr int TF = X3S2_TF, HW = X3S2_HW, HMIN = 2;
    static constexpr int W2 = X3S2_W2, MW = 8, MMIN = 2;
    static constexpr int W3 = X3S2_W3, TW = 8, TMIN = 2;
    static constexpr int NT_IN = 2, NT_T1 = 2, NT_R1 = X3S2_NT_R1, NT_T2 = 4, NT_R2 = X3S2_NT_R2, NT_T3 = X3S2_NT_T3,
                         NT_R3 = X3S2_NT_R3, NT_T4 = 4, NT_R4 = 4;
    static constexpr int G_T1 = 1, G_R1 = 1;
    // weight k-blocks in flight per item (8 VGPRs each).  4, as stage1: 8 and
    // 12 (the 256-VGPR budget of 8 waves at one workgroup per CU allows them)
    // measured level or slower - head 25.8 / 26.3 / 27.0 us at 8x500, mid
    // 184.2 / 184.4 / 185.2 us at 16x2600 (profiles/r04/r04b_pdm_pipeline_ab.txt):
    // the stage2 head and mid are not bound by the latency of their weight
    // stream
    static constexpr int PDM = X3S2_PDM;
    // head B fragments one k-block ahead (mma_x3 BP; 116 -> 156 VGPRs, one
    // workgroup per CU either way): head 26.5 -> 25.0 us at 8x500; in the mid
    // kernels it measured slower (24.0 -> 26.0 us at 8x500, 186 -> 212 us at
    // 16x2600: 4 -> 3 waves per SIMD), in the 16-wave H24 head level (172 ->
    // 175 us, spills; its hi-only form, BP 2, 173.6 -> 171.5 us: CfgS2H24) -
    // profiles/r05/r05g_bpipe_ab.txt, r05r_head_bp2_ab.txt
    static constexpr int HBP = X3S2_HBP;
};
// Stage2 mid / tail tilings for small grids (run<CfgS2> picks per call): at
// B=8, T=500 the default windows make 576 mid workgroups (1.1 rounds of 512
// slots at two per CU) and 536 tail workgroups (2.1 rounds of 256 at one
// per CU); 32 / 125 make 504 and 512 (one and two full rounds), at 1.20x /
// 1.075x the time per workgroup (5-tile chunks where 4 were enough).
// Measured B=8 T=500: mid 26.4 -> 22.9 us, tail 35.5 -> 26.1 us; large grids
// keep the defaults (tools/probe/s2_tiles.sh).  Since round 5 the windows
// are 30 and 33 positions (same tiles, fewer workgroups: below).
struct CfgS2Alt : CfgS2 {
    static constexpr int W2 = X3S2A_W2, NT_R2 = 5;
    static constexpr int W3 = 125, NT_T3 = 5, NT_R3 = 5;
};
constexpr double kAltMidCost = 1.20, kAltTailCost = 1.075;
// Stage2 head windows of 24 frames for large grids (composed head: less
// weight streaming per frame; 16x2600 0.569 -> 0.548 ms, 64x500 0.430 ->
// 0.421 ms per vocoder step, but 8x500 0.072 -> 0.075 ms: 168 workgroups
// leave CUs idle), taken when the 16-frame grid has >= 1024 workgroups.
// 16 waves per workgroup there (more latency hiding at one workgroup per CU:
// head 140.8 -> 135.2 us at 64x500, 170.6 -> 165.4 at 16x2600; at 8x500 the
// 16-frame, 8-wave head stays, tools/probe/s2_tiles.sh with X3S2_HW=16).
struct CfgS2H24 : CfgS2 {
    static constexpr int TF = X3S2W_TF, HW = 16;
    static constexpr int PDM = 4;  // 16 waves: 128 VGPRs per wave
    static constexpr int HBP = X3S2W_HBP;
};
constexpr long kS2WideHeadWGs = 1024;  // in 16-frame windows
// Each window's layers run whole 16-row m-tiles: the head's ResBlock1 covers
// 4 TF + 2 rows (16 and 19 frames: 5 tiles, 24 and 27: 7), the mid's
// ResBlock2 4 W + 2 and its ConvT2 W + 2 rows per phase (28 and 30
// positions: 8 and 2 tiles, 32 and 33: 10 with NT_R2 = 5, and 3).  So the
// 19 / 27-frame heads and the 30 / 33-position mids cost what the 16 / 24 /
// 28 / 32 ones do per workgroup and make fewer workgroups; run<CfgS2> takes
// the fewer rounds of workgroup slots, the smaller window when the rounds tie.
// Bit-identical audio either way (every output sums the same products in the
// same order).  Alternated twice (profiles/r05/r05ab_windows_ab.txt): head
// 38.9 -> 27.2 us at 16x262 (272 -> 224 workgroups: one round of 256),
// 146.3 -> 132.9 at 128x262, 141.2 -> 128.0 at 64x500; mid 184.4 -> 176.6 us
// at 16x2600, 149.1 -> 145.2 at 128x262, 26.7 -> 25.2 at 16x262 (W33:
// 512 workgroups, one round of two per CU).
struct CfgS2T19 : CfgS2 {
    static constexpr int TF = 19;
};
struct CfgS2H27 : CfgS2H24 {
    static constexpr int TF = 27;
};

// Diagnostic build only (-DM2_STAMPS): per-wave s_memtime stamps at phase
// boundaries, [kernel][workgroup][wave][16] (tools/probe/stamps.py --x3).
#ifdef M2_STAMPS
__device__ unsigned long long g_x3_stamps[3][4096][16][16];
#define XSTAMP(K, i)                                                                                     \
    do {                                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        unsigned long long _t;                                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                      \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        const int _wg = blockIdx.y * gridDim.x + blockIdx.x;                                             \
        if ((threadIdx.x & 63) == 0 && _wg < 4096) g_x3_stamps[K][_wg][threadIdx.x >> 6][i] = _t;        \
    } while (0)
// s_memrealtime (100 MHz) into slot i: with an s_memtime pair of the same
// wave it gives the shader clock over that interval (tools/probe/stamps.py)
#define XSTAMP_RT(K, i)                                                                                  \
    do {                                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        unsigned long long _t;                                                                           \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                  \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        const int _wg = blockIdx.y * gridDim.x + blockIdx.x;                                             \
        if ((threadIdx.x & 63) == 0 && _wg < 4096) g_x3_stamps[K][_wg][threadIdx.x >> 6][i] = _t;        \
    } while (0)
#else
#define XSTAMP(K, i) \
    do {             \
    } while (0)
#define XSTAMP_RT(K, i) \
    do {                \
    } while (0)
#endif

// Window x and utterance y of a head workgroup, XCD-aware: workgroups go to
// the 8 XCDs round-robin by linear id, and with x fastest the 8 windows of an
// utterance land on 8 different XCDs, each of which fetches the mel lines
// its window shares with its neighbours ([M][T] rows: a 69-frame window of a
// channel row spans 3-4 lines of 128 B): FETCH_SIZE grew 0.22 MB per
// utterance against 0.13 MB of mel at T = 500 (profiles/r04/r04c_head_fetch_*).
// With B a multiple of 8 XCD k could take every window of utterances
// b = k mod 8, so shared lines are fetched once per utterance: FETCH 9.66 ->
// 7.71 MB per launch at B=32 ((FETCH - the 2.7 MB of weights per 8 XCDs) /
// mel 1.7 -> 1.22), but the headline step +0.3 % (0.07158 / 0.07148 /
// 0.07172 vs 0.07145 / 0.07138 / 0.07123 ms alternated,
// profiles/r04/r04h_head_*, r04k_headline_xcd_ab.txt): the over-read lines
// are served by the Infinity Cache, and the plain order spreads an
// utterance's edge windows over the XCDs.  Kept as a build option
// (-DX3_HEAD_XCD=1); the plain order is the default.
#ifndef X3_HEAD_XCD
#define X3_HEAD_XCD 0
#endif
__device__ __forceinline__ void head_tile(int& x, int& y) {
    x = blockIdx.x;
    y = blockIdx.y;
    if (X3_HEAD_XCD && (gridDim.y & 7) == 0) {
        const int L = blockIdx.y * gridDim.x + blockIdx.x, k = L & 7, s = L >> 3, nx = gridDim.x;
        y = 8 * (s / nx) + k;
        x = s - (s / nx) * nx;
    }
}

// The stage1 head runs ConvT1 / ResBlock1 phase-planar when one item per wave
// covers them: planes of 64 rows hold TF + 2 <= 65 input columns and the
// (phase, m-block) items of the C/2-channel layers number exactly HW.
template <class Cfg>
constexpr bool head_planar() {
    return X3_PLANAR && Cfg::TF + 1 <= 64 && 4 * (Cfg::C / 2 / 16) == Cfg::HW && Cfg::G_T1 == 1 && Cfg::G_R1 == 1;
}

// COMP (stage1 planar head): input_conv composed into ConvT1
// (head_convT1c_planar; w.hc / w.hcb / w.hce).
template <class Cfg, bool TRANS, bool COMP = false>
__global__ __launch_bounds__(Cfg::HW * 64, Cfg::HMIN) void x3_head_kernel(const float* __restrict__ mel, int T,
                                                                            VocX w, unsigned char* __restrict__ U1) {
    if (w.rclear && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < 5) {
        if (threadIdx.x == 0) *reinterpret_cast<volatile int*>(w.rclear) = 0;
        else if (w.rqueue) reinterpret_cast<volatile unsigned*>(w.rqueue)[threadIdx.x - 1] = 0u;
    }
    if (w.head_prio == 1) {  // waves w, w + 4, ... share a SIMD; age favours the older ones
        const int pr = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >> 2;
        if (pr == 1) __builtin_amdgcn_s_setprio(1);
        else if (pr == 2) __builtin_amdgcn_s_setprio(2);
        else if (pr >= 3) __builtin_amdgcn_s_setprio(3);
    }
    constexpr int M = Cfg::M, MP = Cfg::MP, C = Cfg::C, TF = Cfg::TF;
    int wx, wy;
    head_tile(wx, wy);
    if (w.dT) {  // speculative launch: T was the capacity
        T = dev_frames(w.dT, T);
        if (wx * TF >= T) return;
    }
    using Pl = HeadPlan<MP, C, TF, head_planar<Cfg>()>;
    constexpr int C1 = Pl::C1;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = wy, f0 = wx * TF;
    XW a0w{lds, f0 - 2};
    XW hw{lds, 4 * f0 - 1};
    XW melw{lds + Pl::RA, f0 - 3};
    XW uw{lds + Pl::RA, 4 * f0 - 4};
    constexpr int NW = Cfg::HW;
    using I0 = Conv3Items<MP, C, Cfg::NT_IN, Pl::A0_N, 1>;
    using I1 = ConvTItems<C, C1, 4, Cfg::NT_T1, Pl::NQ, Cfg::G_T1>;
    using I2 = Conv3Items<C1, C1, Cfg::NT_R1, Pl::H_N, Cfg::G_R1>;
    using I3 = Conv3Items<C1, C1, Cfg::NT_R1, Pl::O_N, Cfg::G_R1>;
    // One item per wave in every layer (stage1): weight fragments handed
    // from layer to layer across the barriers (APipe).
    constexpr bool ONE = Cfg::G_T1 == 1 && Cfg::G_R1 == 1 && I0::N == NW && I1::N == NW && I2::N == NW &&
                         I3::N == NW && pd_of<MP, 3, 1>() == 4 && pd_of<C, 2, 1>() == 4 && pd_of<C1, 3, 1>() == 4;
    // phase-planar ConvT1 / ResBlock1: planes of 64 rows hold TF + 2 <= 65
    // input columns, one item per wave = (phase, m-block)
    constexpr bool PLANAR = ONE && head_planar<Cfg>();
    XSTAMP_RT(0, 14);
    XSTAMP(0, 0);
    if constexpr (COMP && !PLANAR) {
        // stage2: the composed layer on the generic item path; the mel window
        // in region A (the u rows it feeds are region B), edge terms after it
        static_assert(!ONE, "generic path");
        static_assert(Pl::CAP_MEL * Pl::RS_M + 4 * 4 * C1 <= Pl::RA, "mel window + edge terms in region A");
        static_assert(4 * C1 <= Cfg::HW * 64, "one thread per edge term");
        const XW melA{lds, f0 - 3};
        unsigned char* corr = lds + Pl::CAP_MEL * Pl::RS_M;
        // ConvT1's input columns here are [f0 - 1, f0 + TF]
        const bool left = f0 == 0, right = T - 1 >= f0 - 1 && T - 1 <= f0 + TF;
        gload_mel<TRANS, M, MP, Pl::RS_M, Pl::MEL_N, Cfg::HW * 64>(mel + (size_t)b * M * T, T, melA);
        XSTAMP(0, 1);
        __syncthreads();
        if (left || right) {
            head_edge_terms_s2<M, MP, C1, Pl::RS_M>(w.hce, melA, T, left, right, corr);
            __syncthreads();
        }
        XSTAMP(0, 2);
        XSTAMP(0, 3);
        XSTAMP(0, 4);
        xconvT1c<MP, C1, Cfg::NT_T1, Pl::RS_M, Pl::RS_1, Pl::NQ, Cfg::PDM, Cfg::HBP>(w.hc, w.hcb, (left || right) ? corr : nullptr, melA,
                                                              uw, f0 - 1, T);
        XSTAMP(0, 5);
        __syncthreads();
        XSTAMP(0, 6);
        xconv3<C1, C1, Cfg::NT_R1, ACT_LEAKY, false, Pl::RS_1, Pl::RS_1, Pl::H_N, 1, 0, false, Cfg::PDM, Cfg::HBP>(w.w1[0], w.b1[0], uw, hw, 4 * f0 - 1,
                                                                                 4 * T);
        XSTAMP(0, 7);
        __syncthreads();
        XSTAMP(0, 8);
        xconv3<C1, C1, Cfg::NT_R1, ACT_NONE, true, Pl::RS_1, Pl::RS_1, Pl::O_N, 1, 0, true, Cfg::PDM, Cfg::HBP>(
            w.w2[0], w.b2[0], hw, uw, 4 * f0, 4 * T, nullptr, nullptr, U1 + (size_t)b * 4 * T * 4 * C1);
        XSTAMP(0, 9);
        return;
    } else if constexpr (COMP) {
        static_assert(PLANAR, "the composed head runs on the phase-planar path");
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        constexpr int MB1 = C1 / 16;
        APipe ap;
        const u32x4* wp0 = w.hc + (size_t)wv * nkb_of<MP, 4>() * 128 + (threadIdx.x & 63);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            ap[kb][0][0] = wp0[kb * 128];
            ap[kb][0][1] = wp0[kb * 128 + 64];
        }
        // the mel window goes to region A (the u planes it feeds are written
        // into region B in the same phase; the h planes overwrite it later)
        static_assert(Pl::CAP_MEL * Pl::RS_M + 4 * 4 * C1 <= Pl::RA, "mel window + edge terms in region A");
        const XW melA{lds, f0 - 3};
        unsigned char* corr = lds + Pl::CAP_MEL * Pl::RS_M;
        // the windows holding an utterance edge (workgroup-uniform)
        const bool left = f0 == 0, right = T - 1 >= f0 - 1 && T - 1 < f0 + TF;
        float4 ev[4];
        float eb = 0.f;
        if (left || right) head_edge_load<MP, C1>(w.hce, ev, eb);
        gload_mel<TRANS, M, MP, Pl::RS_M, Pl::MEL_N, Cfg::HW * 64>(mel + (size_t)b * M * T, T, melA);
        XSTAMP(0, 1);
        __syncthreads();
        if (left || right) {
            head_edge_terms<MP, C1, Pl::RS_M>(ev, eb, melA, T, left, right, corr);
            __syncthreads();
        }
        XSTAMP(0, 2);
        XSTAMP(0, 3);  // (no input-conv layer)
        XSTAMP(0, 4);
        unsigned char* up = lds + Pl::RA;
        unsigned char* hp = lds;
        head_convT1c_planar<MP, C1, Pl::RS_M, Pl::RS_1>(
            w.hc, w.hcb, (left || right) ? corr : nullptr, melA, up, f0, T, &ap,
            w.w1[0] + (size_t)(wv % MB1) * nkb_of<C1, 3>() * 128 + (threadIdx.x & 63));
        XSTAMP(0, 5);
        __syncthreads();
        XSTAMP(0, 6);
        head_rb1_planar<C1, Pl::RS_1, false>(w.w1[0], w.b1[0], up, hp, nullptr, f0, TF, 4 * T, &ap,
                                             w.w2[0] + (size_t)(wv % MB1) * nkb_of<C1, 3>() * 128 +
                                                 (threadIdx.x & 63),
                                             nullptr);
        XSTAMP(0, 7);
        __syncthreads();
        XSTAMP(0, 8);
        head_rb1_planar<C1, Pl::RS_1, true>(w.w2[0], w.b2[0], hp, nullptr, up, f0, TF, 4 * T, &ap, nullptr,
                                            U1 + (size_t)b * 4 * T * 4 * C1);
        XSTAMP(0, 9);
        XSTAMP_RT(0, 15);
        return;
    } else if constexpr (ONE) {
        const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        APipe ap;
        const u32x4* wp0 = I0::wp(w.wi, wv);
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            ap[kb][0][0] = wp0[kb * 128];
            ap[kb][0][1] = wp0[kb * 128 + 64];
        }
        gload_mel<TRANS, M, MP, Pl::RS_M, Pl::MEL_N, Cfg::HW * 64>(mel + (size_t)b * M * T, T, melw);
        XSTAMP(0, 1);
        __syncthreads();
        XSTAMP(0, 2);
        if constexpr (PLANAR) {
            // phase-planar ConvT1 / ResBlock1 (u planes in region B, h planes in region A)
            unsigned char* up = lds + Pl::RA;
            unsigned char* hp = lds;
            xconv3<MP, C, Cfg::NT_IN, ACT_NONE, false, Pl::RS_M, Pl::RS_C, Pl::A0_N, 1, NW>(
                w.wi, w.bi, melw, a0w, f0 - 2, T, &ap, w.wt[0] + (size_t)wv * nkb_of<C, 2>() * 128 + (threadIdx.x & 63));
            XSTAMP(0, 3);
            __syncthreads();
            XSTAMP(0, 4);
            constexpr int MB1 = C1 / 16;
            head_convT1_planar<C, C1, Pl::RS_C, Pl::RS_1>(w.wt[0], w.bt[0], a0w, up, f0, 4 * T, &ap,
                                                        w.w1[0] + (size_t)(wv % MB1) * nkb_of<C1, 3>() * 128 +
                                                            (threadIdx.x & 63));
            XSTAMP(0, 5);
            __syncthreads();
            XSTAMP(0, 6);
            head_rb1_planar<C1, Pl::RS_1, false>(w.w1[0], w.b1[0], up, hp, nullptr, f0, TF, 4 * T, &ap,
                                                 w.w2[0] + (size_t)(wv % MB1) * nkb_of<C1, 3>() * 128 +
                                                     (threadIdx.x & 63),
                                                 nullptr);
            XSTAMP(0, 7);
            __syncthreads();
            XSTAMP(0, 8);
            head_rb1_planar<C1, Pl::RS_1, true>(w.w2[0], w.b2[0], hp, nullptr, up, f0, TF, 4 * T, &ap, nullptr,
                                                U1 + (size_t)b * 4 * T * 4 * C1);
            XSTAMP(0, 9);
            XSTAMP_RT(0, 15);
            return;
        }
        xconv3<MP, C, Cfg::NT_IN, ACT_NONE, false, Pl::RS_M, Pl::RS_C, Pl::A0_N, 1, NW>(
            w.wi, w.bi, melw, a0w, f0 - 2, T, &ap, I1::wp(w.wt[0], wv));
        XSTAMP(0, 3);
        __syncthreads();
        XSTAMP(0, 4);
        xconvT<C, C1, 4, Cfg::NT_T1, Pl::RS_C, Pl::RS_1, Pl::NQ, 1, NW>(w.wt[0], w.bt[0], a0w, uw, f0 - 1, 4 * T,
                                                                     &ap, I2::wp(w.w1[0], wv));
        XSTAMP(0, 5);
        __syncthreads();
        XSTAMP(0, 6);
        xconv3<C1, C1, Cfg::NT_R1, ACT_LEAKY, false, Pl::RS_1, Pl::RS_1, Pl::H_N, 1, NW>(
            w.w1[0], w.b1[0], uw, hw, 4 * f0 - 1, 4 * T, &ap, I3::wp(w.w2[0], wv));
        XSTAMP(0, 7);
        __syncthreads();
        XSTAMP(0, 8);
        // ResBlock1 conv2 + x straight to U1 (rows of hi[C1] lo[C1]): no LDS
        // round trip, no last barrier, no separate store phase
        xconv3<C1, C1, Cfg::NT_R1, ACT_NONE, true, Pl::RS_1, Pl::RS_1, Pl::O_N, 1, NW, true>(
            w.w2[0], w.b2[0], hw, uw, 4 * f0, 4 * T, &ap, nullptr, U1 + (size_t)b * 4 * T * 4 * C1);
        XSTAMP(0, 9);
        XSTAMP_RT(0, 15);
        return;
    } else {
        gload_mel<TRANS, M, MP, Pl::RS_M, Pl::MEL_N, Cfg::HW * 64>(mel + (size_t)b * M * T, T, melw);
        XSTAMP(0, 1);
        __syncthreads();
        XSTAMP(0, 2);
        xconv3<MP, C, Cfg::NT_IN, ACT_NONE, false, Pl::RS_M, Pl::RS_C, Pl::A0_N>(w.wi, w.bi, melw, a0w, f0 - 2, T);
        XSTAMP(0, 3);
        __syncthreads();
        XSTAMP(0, 4);
        xconvT<C, C1, 4, Cfg::NT_T1, Pl::RS_C, Pl::RS_1, Pl::NQ, Cfg::G_T1>(w.wt[0], w.bt[0], a0w, uw, f0 - 1,
                                                                            4 * T);
        XSTAMP(0, 5);
        __syncthreads();
        XSTAMP(0, 6);
        xconv3<C1, C1, Cfg::NT_R1, ACT_LEAKY, false, Pl::RS_1, Pl::RS_1, Pl::H_N, Cfg::G_R1>(w.w1[0], w.b1[0], uw,
                                                                                            hw, 4 * f0 - 1, 4 * T);
        XSTAMP(0, 7);
        __syncthreads();
        XSTAMP(0, 8);
        xconv3<C1, C1, Cfg::NT_R1, ACT_NONE, true, Pl::RS_1, Pl::RS_1, Pl::O_N, Cfg::G_R1>(w.w2[0], w.b2[0], hw, uw,
                                                                                           4 * f0, 4 * T);
    }
    XSTAMP(0, 9);
    __syncthreads();
    XSTAMP(0, 10);
    gstore_rows<C1, Pl::RS_1, Pl::O_N, Cfg::HW * 64>(U1 + (size_t)b * 4 * T * 4 * C1, 4 * T, uw, 4 * f0);
    XSTAMP(0, 11);
}

template <class Cfg>
__global__ __launch_bounds__(Cfg::MW * 64, Cfg::MMIN) void x3_mid_kernel(const unsigned char* __restrict__ U1,
                                                                           int L1, VocX w,
                                                                           unsigned char* __restrict__ U2) {
    constexpr int CI = Cfg::C / 2, W = Cfg::W2;
    using Pl = MidPlan<CI, W>;
    constexpr int CO = Pl::CO;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = blockIdx.y, p0 = blockIdx.x * W;
    if (w.dT) {  // speculative launch: L1 was the capacity
        L1 = 4 * dev_frames(w.dT, L1 / 4);
        if (p0 >= L1) return;
    }
    const int L2 = 4 * L1;
    XW inw{lds, p0 - 2};
    XW hw{lds, 4 * p0 - 1};
    XW uw{lds + Pl::RA, 4 * p0 - 4};
    XSTAMP(1, 0);
    gload_rows<CI, Pl::RS_I, Pl::IN_N, Cfg::MW * 64>(U1 + (size_t)b * L1 * 4 * CI, L1, inw);
    XSTAMP(1, 1);
    __syncthreads();
    XSTAMP(1, 2);
    xconvT<CI, CO, 4, Cfg::NT_T2, Pl::RS_I, Pl::RS_O, Pl::NQ, 1, 0, Cfg::PDM>(w.wt[1], w.bt[1], inw, uw, p0 - 1, L2);
    XSTAMP(1, 3);
    __syncthreads();
    XSTAMP(1, 4);
    xconv3<CO, CO, Cfg::NT_R2, ACT_LEAKY, false, Pl::RS_O, Pl::RS_O, Pl::H_N, 1, 0, false, Cfg::PDM>(w.w1[1], w.b1[1], uw, hw, 4 * p0 - 1, L2);
    XSTAMP(1, 5);
    __syncthreads();
    XSTAMP(1, 6);
    xconv3<CO, CO, Cfg::NT_R2, ACT_NONE, true, Pl::RS_O, Pl::RS_O, Pl::O_N, 1, 0, false, Cfg::PDM>(w.w2[1], w.b2[1], hw, uw, 4 * p0, L2);
    XSTAMP(1, 7);
    __syncthreads();
    XSTAMP(1, 8);
    gstore_rows<CO, Pl::RS_O, Pl::O_N, Cfg::MW * 64>(U2 + (size_t)b * L2 * 4 * CO, L2, uw, 4 * p0);
    XSTAMP(1, 9);
}

template <class Cfg>
__global__ __launch_bounds__(Cfg::TW * 64, Cfg::TMIN) void x3_tail_kernel(const unsigned char* __restrict__ U2,
                                                                            int L2, VocX w,
                                                                            float* __restrict__ audio) {
    constexpr int CI = Cfg::C / 4, W = Cfg::W3;
    using Pl = TailPlan<CI, W>;
    constexpr int C3 = Pl::C3, C4 = Pl::C4;
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int b = blockIdx.y, p0 = blockIdx.x * W;
    if (w.dT) {  // speculative launch: L2 was the capacity
        L2 = 16 * dev_frames(w.dT, L2 / 16);
        if (p0 >= L2) return;
    }
    const int L3 = 2 * L2, L4 = 4 * L2;
    unsigned char* ra = lds;
    unsigned char* rb = lds + Pl::RA;
    XW inw{ra, p0 - 4};
    XW u3{rb, 2 * p0 - 6};
    XW h3{ra, 2 * p0 - 4};
    XW u4{ra, 4 * p0 - 4};
    XW h4w{rb, 4 * p0 - 2};
    XSTAMP(2, 0);
    gload_rows<CI, Pl::RS_I, Pl::IN_N, Cfg::TW * 64>(U2 + (size_t)b * L2 * 4 * CI, L2, inw);
    XSTAMP(2, 1);
    __syncthreads();
    XSTAMP(2, 2);
    xconvT<CI, C3, 2, Cfg::NT_T3, Pl::RS_I, Pl::RS_3, Pl::NQ3, 1, 0, Cfg::PDM>(w.wt[2], w.bt[2], inw, u3, p0 - 3, L3);
    XSTAMP(2, 3);
    __syncthreads();
    XSTAMP(2, 4);
    xconv3<C3, C3, Cfg::NT_R3, ACT_LEAKY, false, Pl::RS_3, Pl::RS_3, Pl::H3_N, 1, 0, false, Cfg::PDM>(w.w1[2], w.b1[2], u3, h3, 2 * p0 - 4, L3);
    XSTAMP(2, 5);
    __syncthreads();
    XSTAMP(2, 6);
    xconv3<C3, C3, Cfg::NT_R3, ACT_NONE, true, Pl::RS_3, Pl::RS_3, Pl::O3_N, 1, 0, false, Cfg::PDM>(w.w2[2], w.b2[2], h3, u3, 2 * p0 - 3, L3);
    XSTAMP(2, 7);
    __syncthreads();
    XSTAMP(2, 8);
    xconvT<C3, C4, 2, Cfg::NT_T4, Pl::RS_3, Pl::RS_4, Pl::NQ4, 1, 0, Cfg::PDM>(w.wt[3], w.bt[3], u3, u4, 2 * p0 - 2, L4);
    XSTAMP(2, 9);
    __syncthreads();
    XSTAMP(2, 10);
    xconv3<C4, C4, Cfg::NT_R4, ACT_LEAKY, false, Pl::RS_4, Pl::RS_4, Pl::H4_N, 1, 0, false, Cfg::PDM>(w.w1[3], w.b1[3], u4, h4w, 4 * p0 - 2, L4);
    XSTAMP(2, 11);
    __syncthreads();
    XSTAMP(2, 12);
    xconv3<C4, C4, Cfg::NT_R4, ACT_NONE, true, Pl::RS_4, Pl::RS_4, Pl::O4_N, 1, 0, false, Cfg::PDM>(w.w2[3], w.b2[3], h4w, u4, 4 * p0 - 1, L4);
    XSTAMP(2, 13);
    __syncthreads();
    XSTAMP(2, 14);
    // output_conv (C4 -> 1, k3) + tanh on the VALU, one sample per thread.
    float* arow = audio + (size_t)b * L4;
    const float bo = w.bo[0];
    for (int j = threadIdx.x; j < Pl::A_N; j += blockDim.x) {
        const int t = 4 * p0 + j;
        if (t < L4) {
            const unsigned char* x = u4.p + (t - 1 - u4.start) * Pl::RS_4;
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const _Float16* hr = reinterpret_cast<const _Float16*>(x + k * Pl::RS_4);
#pragma unroll
                for (int ci = 0; ci < C4; ++ci)
                    acc = fmaf(w.wo[ci * 3 + k], (float)hr[ci] + (float)hr[C4 + ci], acc);
            }
            const float o = tanhf(acc + bo);
            arow[t] = o;
            flag_nonfinite4(o, 0.f, 0.f, 0.f, w.rflag);
        }
    }
    XSTAMP(2, 15);
}

template <typename K>
int32_t set_lds(K kernel, size_t bytes) {
    M2_CHECK_SHAPE(bytes <= 160 * 1024, "x3 vocoder: LDS plan exceeds 160 KiB");
    M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                               (int)bytes));
    return M2_OK;
}

// Workgroup slots of the device for a kernel (CUs x its occupancy), queried
// once per kernel: the vocoder calls this on every launch decision.
template <typename K>
long grid_slots(K kernel, int threads, size_t lds) {
    int ncu = 0, dev = 0, per = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(kernel), threads, lds) !=
            hipSuccess || per <= 0)
        per = 1;
    return (long)per * ncu;
}
inline long rounds_of(long n, long slots) { return (n + slots - 1) / slots; }

template <class Cfg>
int32_t run(const float* mel, bool trans, int B, int T, const VocX& w, void* U1, void* U2, float* audio,
            hipStream_t st, const std::function<void(int, bool)>& mark) {
    using HP = HeadPlan<Cfg::MP, Cfg::C, Cfg::TF, head_planar<Cfg>()>;
    using HP24 = HeadPlan<CfgS2H24::MP, CfgS2H24::C, CfgS2H24::TF, false>;
    using HP19 = HeadPlan<CfgS2T19::MP, CfgS2T19::C, CfgS2T19::TF, false>;
    using HP27 = HeadPlan<CfgS2H27::MP, CfgS2H27::C, CfgS2H27::TF, false>;
    using MP = MidPlan<Cfg::C / 2, Cfg::W2>;
    using TP = TailPlan<Cfg::C / 4, Cfg::W3>;
    constexpr bool S2 = std::is_same<Cfg, CfgS2>::value;
    using MPA = MidPlan<CfgS2Alt::C / 2, CfgS2Alt::W2>;
    using TPA = TailPlan<CfgS2Alt::C / 4, CfgS2Alt::W3>;
    static bool attr = false;
    if (!attr) {
        int32_t rc;
        if ((rc = set_lds(x3_head_kernel<Cfg, false>, HP::LDS_BYTES))) return rc;
        if ((rc = set_lds(x3_head_kernel<Cfg, true>, HP::LDS_BYTES))) return rc;
        if ((rc = set_lds(x3_head_kernel<Cfg, false, true>, HP::LDS_BYTES))) return rc;
        if ((rc = set_lds(x3_head_kernel<Cfg, true, true>, HP::LDS_BYTES))) return rc;
        if ((rc = set_lds(x3_mid_kernel<Cfg>, MP::LDS_BYTES))) return rc;
        if ((rc = set_lds(x3_tail_kernel<Cfg>, TP::LDS_BYTES))) return rc;
        if constexpr (S2) {
            if ((rc = set_lds(x3_head_kernel<CfgS2H24, false, true>, HP24::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_head_kernel<CfgS2H24, true, true>, HP24::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_head_kernel<CfgS2T19, false, true>, HP19::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_head_kernel<CfgS2T19, true, true>, HP19::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_head_kernel<CfgS2H27, false, true>, HP27::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_head_kernel<CfgS2H27, true, true>, HP27::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_mid_kernel<CfgS2Alt>, MPA::LDS_BYTES))) return rc;
            if ((rc = set_lds(x3_tail_kernel<CfgS2Alt>, TPA::LDS_BYTES))) return rc;
        }
        attr = true;
    }
    bool alt_mid = false, alt_tail = false;
    if constexpr (S2) {
        static const long sm0 = grid_slots(x3_mid_kernel<Cfg>, Cfg::MW * 64, MP::LDS_BYTES),
                          sm1 = grid_slots(x3_mid_kernel<CfgS2Alt>, Cfg::MW * 64, MPA::LDS_BYTES),
                          st0 = grid_slots(x3_tail_kernel<Cfg>, Cfg::TW * 64, TP::LDS_BYTES),
                          st1 = grid_slots(x3_tail_kernel<CfgS2Alt>, Cfg::TW * 64, TPA::LDS_BYTES);
        if (!w.mp && sw().s2_mid_alt >= 0)
            alt_mid = sw().s2_mid_alt == 1;
        else if (!w.mp)
            alt_mid = rounds_of((long)cdiv(4 * T, CfgS2Alt::W2) * B, sm1) * kAltMidCost <
                      (double)rounds_of((long)cdiv(4 * T, Cfg::W2) * B, sm0);
        if (!w.tp && !w.tp2)
            alt_tail = rounds_of((long)cdiv(16 * T, CfgS2Alt::W3) * B, st1) * kAltTailCost <
                       (double)rounds_of((long)cdiv(16 * T, Cfg::W3) * B, st0);
    }
    auto* u1 = static_cast<unsigned char*>(U1);
    auto* u2 = static_cast<unsigned char*>(U2);
    mark(0, true);
    // the composed input_conv o ConvT1 head when packed (stage1; 22.1 -> 19.7
    // us, profiles/ab/r02l_head_comp.txt); M2_HEAD_INCONV=1 runs the two
    // layers (A/B and test switch, m2_common.h switch table)
    const bool comp = w.hc && !sw().head_inconv;
    const dim3 hg(cdiv(T, Cfg::TF), B), hb(Cfg::HW * 64);
    // stage2, composed head: the 16-wave heads (24 / 27 frames) on large
    // grids, the 8-wave heads (16 / 19) below; within a pair the fewer rounds
    // of workgroup slots, the smaller window on a tie (M2_S2_HEAD_TF forces)
    int hv = 16;
    if constexpr (S2) {
        static const long s16 = grid_slots(x3_head_kernel<Cfg, false, true>, Cfg::HW * 64, HP::LDS_BYTES),
                          s19 = grid_slots(x3_head_kernel<CfgS2T19, false, true>, CfgS2T19::HW * 64, HP19::LDS_BYTES),
                          s24 = grid_slots(x3_head_kernel<CfgS2H24, false, true>, CfgS2H24::HW * 64, HP24::LDS_BYTES),
                          s27 = grid_slots(x3_head_kernel<CfgS2H27, false, true>, CfgS2H27::HW * 64, HP27::LDS_BYTES);
        auto rounds = [&](int tf, long slots) { return rounds_of((long)cdiv(T, tf) * B, slots); };
        if (sw().s2_head_tf)
            hv = sw().s2_head_tf;
        else if ((long)cdiv(T, 16) * B >= kS2WideHeadWGs)
            hv = rounds(27, s27) < rounds(24, s24) ? 27 : 24;
        else
            hv = rounds(19, s19) < rounds(16, s16) ? 19 : 16;
    }
    auto head = [&](auto cfg) {
        using HC = decltype(cfg);
        using HPc = HeadPlan<HC::MP, HC::C, HC::TF, false>;
        const dim3 g(cdiv(T, HC::TF), B), b(HC::HW * 64);
        if (trans)
            hipLaunchKernelGGL((x3_head_kernel<HC, true, true>), g, b, HPc::LDS_BYTES, st, mel, T, w, u1);
        else
            hipLaunchKernelGGL((x3_head_kernel<HC, false, true>), g, b, HPc::LDS_BYTES, st, mel, T, w, u1);
    };
    if (S2 && comp && hv != 16) {
        if constexpr (S2) {
            if (hv == 19)
                head(CfgS2T19{});
            else if (hv == 24)
                head(CfgS2H24{});
            else
                head(CfgS2H27{});
        }
    } else if (comp && trans)
        hipLaunchKernelGGL((x3_head_kernel<Cfg, true, true>), hg, hb, HP::LDS_BYTES, st, mel, T, w, u1);
    else if (comp)
        hipLaunchKernelGGL((x3_head_kernel<Cfg, false, true>), hg, hb, HP::LDS_BYTES, st, mel, T, w, u1);
    if (!comp && trans)
        hipLaunchKernelGGL((x3_head_kernel<Cfg, true>), hg, hb, HP::LDS_BYTES, st, mel, T, w, u1);
    else if (!comp)
        hipLaunchKernelGGL((x3_head_kernel<Cfg, false>), hg, hb, HP::LDS_BYTES, st, mel, T, w, u1);
    mark(0, false);
    M2_LAUNCHED("x3_head_kernel");
    mark(1, true);
    if (w.mp) {  // stage1: the pipelined mid stage (vocoder_midp.hip)
        const int32_t rc = launch_vocoder_midp(u1, 4 * T, B, w.mp, w.mpb, u2, st, w.dT);
        if (rc) return rc;
    } else if (S2 && alt_mid) {
        hipLaunchKernelGGL((x3_mid_kernel<CfgS2Alt>), dim3(cdiv(4 * T, CfgS2Alt::W2), B), dim3(Cfg::MW * 64),
                           MPA::LDS_BYTES, st, u1, 4 * T, w, u2);
        M2_LAUNCHED("x3_mid_kernel");
    } else {
        hipLaunchKernelGGL((x3_mid_kernel<Cfg>), dim3(cdiv(4 * T, Cfg::W2), B), dim3(Cfg::MW * 64), MP::LDS_BYTES, st,
                           u1, 4 * T, w, u2);
        M2_LAUNCHED("x3_mid_kernel");
    }
    mark(1, false);
    mark(2, true);
    if (w.tp2) {  // stage2: the pipelined tail (vocoder_tailp2.hip)
        const int32_t rc = launch_vocoder_tailp2(u2, 16 * T, B, w.tp2, w.tp2b, audio, w.rflag, st, w.dT,
                                                 VocRedo{w.redo_w, mel, trans});
        mark(2, false);
        return rc;
    }
    if (w.tp) {  // stage1: the pipelined tail (vocoder_tailp.hip)
        const int32_t rc =
            launch_vocoder_tailp(u2, 16 * T, B, w.tp, w.tpb, audio, w.rflag, st, w.dT, VocRedo{w.redo_w, mel, trans});
        mark(2, false);
        return rc;
    }
    if (S2 && alt_tail)
        hipLaunchKernelGGL((x3_tail_kernel<CfgS2Alt>), dim3(cdiv(16 * T, CfgS2Alt::W3), B), dim3(Cfg::TW * 64),
                           TPA::LDS_BYTES, st, u2, 16 * T, w, audio);
    else
        hipLaunchKernelGGL((x3_tail_kernel<Cfg>), dim3(cdiv(16 * T, Cfg::W3), B), dim3(Cfg::TW * 64), TP::LDS_BYTES, st,
                           u2, 16 * T, w, audio);
    mark(2, false);
    M2_LAUNCHED("x3_tail_kernel");
    return M2_OK;
}

}  // namespace x3

const char* const kVocX3KernelNames[kVocKernels] = {
    "x3_head_kernel (input_conv + ConvT1 + ResBlock1)",
    "x3_mid_kernel (ConvT2 + ResBlock2)",
    "x3_tail_kernel (ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv)"};

#ifdef M2_STAMPS
extern "C" int32_t m2_debug_stamps_x3(void* host, size_t bytes) {
    return (int32_t)hipMemcpyFromSymbol(host, HIP_SYMBOL(x3::g_x3_stamps),
                                        bytes < sizeof(x3::g_x3_stamps) ? bytes : sizeof(x3::g_x3_stamps));
}
#endif

bool vocoder_x3_supported(int M, int C) { return (M == 64 && C == 128) || (M == 80 && C == 256); }

int vocoder_x3_mel_pad(int M) { return M == 80 ? 96 : M; }

int32_t launch_vocoder_x3(const float* mel, bool trans, int M, int C, int B, int T, const VocX& w, void* U1, void* U2,
                          float* audio, hipStream_t st, const std::function<void(int, bool)>& mark) {
    if (B == 0 || T == 0) return M2_OK;
    if (M == 64 && C == 128) return x3::run<x3::CfgS1>(mel, trans, B, T, w, U1, U2, audio, st, mark);
    if (M == 80 && C == 256) return x3::run<x3::CfgS2>(mel, trans, B, T, w, U1, U2, audio, st, mark);
    return fail(M2_E_SHAPE, "x3 vocoder: unsupported (mel_channels, vocoder_channels)");
}

// ---------------------------------------------------------------------------
// Host packing: [group = phase*MB + mb][kb][hi|lo][lane][8 halves] with
// A[co = mb*16 + (lane&15)][octet o = 4kb + (lane>>4), element e] =
// W(ph, co, ci = (o % NOCT)*8 + e, tap = o / NOCT); zero for co >= Cout or o >= NK.
namespace {
void put(std::vector<uint16_t>& out, size_t idx, float v, bool* range_ok) {
    if (!(std::fabs(v) < 65504.f)) *range_ok = false;
    const _Float16 h = (_Float16)v;
    const _Float16 l = (_Float16)(v - (float)h);
    uint16_t hb, lb;
    std::memcpy(&hb, &h, 2);
    std::memcpy(&lb, &l, 2);
    out[idx] = hb;
    out[idx + 64 * 8] = lb;
}

template <typename Wf>
std::vector<uint16_t> pack_x3(int NPH, int Cout, int Cin, int NTAP, Wf W, bool* range_ok) {
    const int MB = (Cout + 15) / 16, NOCT = Cin / 8, NK = NTAP * NOCT, NKB = (NK + 3) / 4;
    std::vector<uint16_t> out((size_t)NPH * MB * NKB * 2 * 64 * 8, 0);
    for (int ph = 0; ph < NPH; ++ph)
        for (int mb = 0; mb < MB; ++mb)
            for (int kb = 0; kb < NKB; ++kb)
                for (int lane = 0; lane < 64; ++lane) {
                    const int co = mb * 16 + (lane & 15), o = 4 * kb + (lane >> 4);
                    if (co >= Cout || o >= NK) continue;
                    const int tap = o / NOCT;
                    for (int e = 0; e < 8; ++e) {
                        const int ci = (o % NOCT) * 8 + e;
                        const size_t idx = ((((size_t)(ph * MB + mb) * NKB + kb) * 2) * 64 + lane) * 8 + e;
                        put(out, idx, W(ph, co, ci, tap), range_ok);
                    }
                }
    return out;
}
}  // namespace

std::vector<uint16_t> pack_x3_conv3(const float* W, int Cout, int Cin, int CinPad, bool* range_ok, bool res) {
    std::vector<uint16_t> out = pack_x3(
        1, Cout, CinPad, 3,
        [&](int, int co, int ci, int tap) { return ci < Cin ? W[((size_t)co * Cin + ci) * 3 + tap] : 0.f; }, range_ok);
    if (res && res_fold_channels(Cin)) {
        // Identity on the padding octets of the last k-block (x octet o - NK):
        // hi = 1.0 (0x3c00), lo = 0.
        const int NOCT = Cin / 8, NK = 3 * NOCT, NKB = (NK + 3) / 4, kb = NKB - 1;
        for (int lane = 0; lane < 64; ++lane) {
            const int co = lane & 15, o = 4 * kb + (lane >> 4);
            if (o < NK || co >= Cout) continue;
            for (int e = 0; e < 8; ++e)
                if ((o - NK) * 8 + e == co) out[(((size_t)kb * 2) * 64 + lane) * 8 + e] = 0x3c00;
        }
    }
    return out;
}

// input_conv o ConvT1 for the composed stage1 head (head_convT1c_planar), in
// double: Wc(ph, co, m, k) = sum_{j = 0, 1; tin = j + 2 - k in [0, 2]} sum_ci
// W_T[ci][co][kj(ph)] W_in[ci][m][tin] (ConvT tap j: input frame q + d0 - j,
// kernel index kj; input-conv tap tin: mel frame i - 1 + tin); bc[ph][co] =
// b_T[co] + sum_j sum_ci W_T[ci][co][kj] b_in[ci]; edge tables E[ph][co][m] =
// sum_ci W_T[ci][co][k_edge] W_in[ci][m][2 (ph < 2) | 0], e[ph][co] = sum_ci
// W_T[ci][co][k_edge] b_in[ci], k_edge = k1 (frame -1) for ph < 2, k0 (frame T).
bool pack_x3_head_comp(const float* Win, const float* bin, const float* WT, const float* bT, int M, int MP, int C,
                       std::vector<uint16_t>* w, std::vector<float>* bias, std::vector<float>* edge, bool* range_ok) {
    const int C1 = C / 2, R = 4, P = R / 2;
    if (MP % 8 || MP < M) return false;
    auto kj = [&](int ph, int j) {
        const int k0 = (ph + P < R) ? ph + P : ph + P - R, k1 = (ph + P < R) ? ph + P + R : ph + P;
        return j ? k1 : k0;
    };
    auto wt = [&](int ci, int co, int k) { return (double)WT[((size_t)ci * C1 + co) * 2 * R + k]; };
    auto wi = [&](int ci, int m, int k) { return m < M ? (double)Win[((size_t)ci * M + m) * 3 + k] : 0.0; };
    std::vector<double> wc((size_t)R * C1 * MP * 4, 0.0);  // [ph][co][m][k]
    for (int ph = 0; ph < R; ++ph)
        for (int co = 0; co < C1; ++co)
            for (int j = 0; j < 2; ++j) {
                const int k = kj(ph, j);
                for (int ci = 0; ci < C; ++ci) {
                    const double a = wt(ci, co, k);
                    for (int tin = 0; tin < 3; ++tin) {
                        const int kk = j + 2 - tin;  // composed tap: mel frame q + d0 + 1 - kk
                        for (int m = 0; m < M; ++m) wc[(((size_t)ph * C1 + co) * MP + m) * 4 + kk] += a * wi(ci, m, tin);
                    }
                }
            }
    *w = pack_x3(R, C1, MP, 4, [&](int ph, int co, int m, int k) { return (float)wc[(((size_t)ph * C1 + co) * MP + m) * 4 + k]; },
                 range_ok);
    bias->assign((size_t)R * C1, 0.f);
    edge->assign((size_t)R * C1 * MP + (size_t)R * C1, 0.f);
    for (int ph = 0; ph < R; ++ph)
        for (int co = 0; co < C1; ++co) {
            double b = bT[co];
            for (int j = 0; j < 2; ++j)
                for (int ci = 0; ci < C; ++ci) b += wt(ci, co, kj(ph, j)) * bin[ci];
            (*bias)[(size_t)ph * C1 + co] = (float)b;
            const int ke = kj(ph, ph < 2 ? 1 : 0), tin = ph < 2 ? 2 : 0;
            double e = 0.0;
            for (int ci = 0; ci < C; ++ci) e += wt(ci, co, ke) * bin[ci];
            (*edge)[(size_t)R * C1 * MP + (size_t)ph * C1 + co] = (float)e;
            for (int m = 0; m < M; ++m) {
                double v = 0.0;
                for (int ci = 0; ci < C; ++ci) v += wt(ci, co, ke) * wi(ci, m, tin);
                (*edge)[((size_t)ph * C1 + co) * MP + m] = (float)v;
            }
        }
    return true;
}

std::vector<uint16_t> pack_x3_convT(const float* W, int Cin, int Cout, int R, bool* range_ok) {
    const int P = R / 2;
    return pack_x3(R, Cout, Cin, 2,
                   [&](int ph, int co, int ci, int tap) {
                       const int k0 = (ph + P < R) ? ph + P : ph + P - R;  // tap 0: x[q] or x[q+1]
                       const int k1 = (ph + P < R) ? ph + P + R : ph + P;  // tap 1: x[q-1] or x[q]
                       return W[((size_t)ci * Cout + co) * 2 * R + (tap ? k1 : k0)];
                   },
                   range_ok);
}

}  // namespace m2
