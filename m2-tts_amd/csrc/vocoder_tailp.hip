// Pipelined SimpleVocoder tail for stage1 (tts_model.py:279-297, the last two
// upsampling stages): ConvT3 (32 -> 16, x2) + leaky, ResBlock3, ConvT4
// (16 -> 8, x2) + leaky, ResBlock4, output_conv (8 -> 1) + tanh, with the
// split-f16 arithmetic of vocoder_x3.hip (every fp32 operand as f16 hi/lo,
// three v_mfma_f32_16x16x32_f16 per product, fp32 accumulate).
//
// Polyphase form.  Everything is indexed by the column q of the tail's input
// U2 (32 channels at 16T).  ConvT3's output u3 (16 channels at t3 = 2q + p3)
// is stored as a 32-row column (p3, channel); ConvT4's output u4 (8 channels
// at t4 = 4q + p4) as a 32-row column (p4, channel); the audio as a 4-row
// column.  In this form every layer is a k3-over-q convolution with 32 output
// rows = two 16-row m-blocks, whose K is a list of (dq, input octet) slots
// (tp::kslot): a k=3 conv on a P-phase signal reads tap t+d at column
// q + floor((p+d)/P), phase (p+d) mod P.  The 8-channel layers fill all 16
// rows of an m-block (two phases), where the natural layout fills 8;
// ConvT4 pairs phases 1, 2 (which read column q only: one k-block) and 0, 3
// (tp::prow), 9 MFMAs per step instead of 12.
//
// Round 2 (default): ResBlock4's conv2 and output_conv are one composed layer
// (outc_role below), so 6 layers, 7 waves and 7 pipeline steps of fill; the
// description below is of the 7-layer form (M2_TAILP_SEVEN=1), which the
// 6-layer one follows for its first five layers.
//
// Systolic pipeline.  One workgroup owns a strip of 16*nch columns of one
// utterance and runs 8 waves with fixed roles: a loader wave streams U2 into
// an LDS ring, and each of the 7 layers is done by one wave for all its
// m-blocks (which share B fragments, tp::frag, so each is read from LDS once),
// with their weights (2 KB per (m-block, k-block) fragment pair) and biases
// held in VGPRs for the whole strip.  In step s the wave of layer l computes
// chunk k = s - l - 1 (16 columns) from the ring its producer wrote in steps
// s-1 and s-2; one s_barrier per step.  Rings hold 3 chunks where the only
// reader is one layer down (a producer writing chunk k+1 never meets its
// consumer reading chunks k and k-1) and 4 where a residual reader two layers
// down also reads them (R1, R4).  Layer l's chunk k covers
// columns [qa + 6 - l + 16k, +16): each layer lags its input by one column,
// the receptive field of its k3 taps, so chunk k of layer l+1 needs exactly
// chunks k and k-1 of layer l.  Chunk -1 is the warm-up: its leftmost columns
// read never-written ring rows and are garbage, but an MFMA output column
// depends on its own B column only, and layer l is valid from column
// qa - 8 + l of chunk -1 on while later layers need it from qa - 6 + l.
// Columns outside [0, L2) store 0 (the next conv's zero padding).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "m2_common.h"
#include "vocoder_fused.h"

namespace m2 {
namespace tp {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef vx_u32x4 u32x4;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// LDS rings.  R0 = U2 input, R(l+1) = output of layer l (l = 0..5); a ring
// row is one column: 32 rows x (hi, lo) f16 kept as a hi plane and a lo plane
// of 64-B rows (the lo plane kLoOff(n) bytes after the hi plane, so a
// fragment's lo read is its hi read plus an immediate offset).  Within a 64-B
// row octet o sits at 16 * (o ^ ((row >> 1) & 3)): with lane li on row r0 + li
// that makes every B-fragment read (ds_read_b128, 16-lane groups) and every
// epilogue store (ds_write_b128, 8 consecutive rows) bank-conflict free
// without padding (tools/probe/tailp_banks.py).  The swizzle depends on row
// bits 1-2 only, so it does not change from chunk to chunk.  Rings hold 4
// chunks of 16 columns (3 for R6, whose only reader is one step behind its
// writer, and for R0 with the register loader; R1 and R4 also feed a residual
// reader two layers down): three workgroups per CU.
// TAILP_DMA (default): the loader moves U2 into R0 by LDS-DMA (buffer_load
// ... lds: L2 -> LDS, no VGPR staging, no ds_write), one chunk ahead, so R0
// holds 4 chunks (TAILP_DMA=0 keeps the register loader
// and a 3-chunk R0).  Alternated twice on one box (profiles/r06/
// r06s_tail_dma_ab/): tail 21.85 / 21.76 -> 21.46 / 21.47 us under
// rocprofv3 at B=32 (-1.6 %; the loader's two ds_write_b128 per step were
// 2 KB of the ~12 KB each chunk writes into LDS), 141 tail / range /
// stress / streaming / parity tests green (r06s_tests.log).
#ifndef TAILP_DMA
#define TAILP_DMA 1
#endif
constexpr int kRingRows[7] = {TAILP_DMA ? 64 : 48, 64, 64, 64, 64, 64, 48};
constexpr int kRingOff(int n) { return n == 0 ? 0 : kRingOff(n - 1) + kRingRows[n - 1] * 128; }
constexpr int kLoOff(int n) { return kRingRows[n] * 64; }
constexpr int kPeriod(int n) { return kRingRows[n] / 16; }  // chunks per ring (3 or 4)
// NL computing layers use rings R0 .. R(NL-1) and NL + 1 waves (one per layer
// + the loader): NL = 7 53,248 B, NL = 6 (outc_role) 47,120 B.
// NL = 6 also keeps the outc edge-term slot (4 floats) after the rings.
constexpr int kCorrSlot = kRingOff(6);
constexpr int ring_bytes(int nl) { return nl == 6 ? kCorrSlot + 16 : kRingOff(nl); }
// after the rings: the workgroup's non-finite-audio word (the local redo,
// vocoder_redo.h); the redo itself reuses the rings' bytes
constexpr int kFlagOff(int nl) { return ring_bytes(nl); }
constexpr int lds_bytes(int nl) { return ring_bytes(nl) + 16; }
constexpr int nwaves(int nl) { return nl + 1; }
static_assert(lds_bytes(6) * 3 <= 160 * 1024, "three workgroups per CU");
static_assert(TAILP_DMA || lds_bytes(7) * 3 <= 160 * 1024, "three workgroups per CU");
#ifdef M2_STAMPS
constexpr int NWAVES = 8;  // stamp buffer size (the larger variant)
#endif

// Byte offset of (row, octet) in ring n's hi plane; row in [0, kRingRows[n]).
__device__ __forceinline__ unsigned ring_at(int n, int row, int oct) {
    return kRingOff(n) + row * 64 + 16 * (oct ^ ((row >> 1) & 3));
}
// Row of column offset c (-2 .. 16) of the chunk in ring phase j.
__device__ __forceinline__ int ring_row(int n, int j, int c) {
    const int r = 16 * j + c, R = kRingRows[n];
    return r < 0 ? r + R : (r >= R ? r - R : r);
}

__device__ __forceinline__ f32x4 mfma_h(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

// LDS hand-off between roles: the step's ds_writes complete, then the
// workgroup barrier.  No vmcnt wait (the loader's prefetches stay in flight),
// and the "memory" clobber keeps the compiler from moving LDS accesses across.
// (An LDS-flag protocol that lets the roles run decoupled measured slower:
// 48 vs 35.5 us, its polls sit on every hand-off of the chain.)
__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Diagnostic build only (-DM2_STAMPS): per-wave s_memtime at the start of
// every step (after the barrier) and before its barrier, [workgroup][wave]
// [step + 1][2]; [62] kernel entry, [63] exit (tools/probe/stamps_tailp.py).
#ifdef M2_STAMPS
__device__ unsigned long long g_tp_stamps[1024][NWAVES][64][2];
#define TPSTAMP(i, j)                                                                                  \
    do {                                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        unsigned long long _t;                                                                         \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        const int _wg = blockIdx.y * gridDim.x + blockIdx.x;                                           \
        if ((threadIdx.x & 63) == 0 && _wg < 1024 && (i) < 64) g_tp_stamps[_wg][threadIdx.x >> 6][(i)][(j)] = _t; \
    } while (0)
#else
#define TPSTAMP(i, j) \
    do {              \
    } while (0)
#endif

// tanh(x) = 1 - 2 / (1 + e^{2x}) on v_exp_f32 / v_rcp_f32: absolute error
// ~1e-7 (saturates to +-1 through inf / 0), against ~40 instructions for tanhf.
__device__ __forceinline__ float tanh_fast(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)); }

// Layer l computes chunk k in step k + l + 1; the last step is layer 6's
// chunk nch - 1.  (Staggered epilogues, where some layers store chunk k one
// step after computing it, measured slower and were dropped.)
// NL = number of computing layers: 7 (ResBlock4 conv2 and output_conv as two
// layers) or 6 (the two composed into one, outc_role below).
constexpr int off_l(int l) { return l + 1; }
constexpr int last_step(int nch, int nl) { return nch - 1 + off_l(nl - 1); }

template <int V>
using ic = std::integral_constant<int, V>;

// One wave per layer (all NMB m-blocks).  Everything lane-dependent that does
// not change along the strip is precomputed: the weights, biases and the LDS
// addresses of the fragment reads, residual reads and epilogue stores for the
// four ring phases j = k mod 4 (the step loop is unrolled by four, so j is a
// compile-time index).  Per step and m-block the epilogue is then leaky (a
// packed multiply and two max), the split (3 VALU per pair), two permlane16
// swaps and one ds_write_b128; the zeroing of columns outside [0, L2) is a
// scalar branch taken only by chunks that straddle an utterance end.
template <int L, int NMB, int NL>
__device__ __forceinline__ void layer_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                           const u32x4* __restrict__ W, const float* __restrict__ bias,
                                           float* __restrict__ arow, int* rflag) {
    constexpr int NKB = nkb(L), NF = nfrag(L);
    // ResBlock conv2: + x (the ConvT output, ring R(L-1), two columns ahead),
    // added by two more MFMAs per m-block with an identity A (x hi, x lo) on
    // one more shared fragment: 4 MFMA issues instead of 24 VALU per step.
    constexpr bool RES = L == 2 || L == 5;
    constexpr int ACT = RES ? ACT_NONE : ACT_LEAKY;  // layer 6: tanh below
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    // Fragment f is read iff one of this wave's (m-block, k-block) uses it.
    auto used = [](int f) {
        bool u = false;
        for (int m = 0; m < NMB; ++m)
            for (int kb = 0; kb < nkbm(L, m); ++kb) u = u || frag(L, m, kb) == f;
        return u;
    };
    u32x4 a[NMB][NKB][2];
    float bv[NMB][4];
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
#pragma unroll
        for (int kb = 0; kb < nkbm(L, m); ++kb) {
            const int u = unit0(L) + m * NKB + kb;
            a[m][kb][0] = W[u * 128 + lane];
            a[m][kb][1] = W[u * 128 + 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[m][r] = bias[L * 32 + m * 16 + 4 * g + r];  // packed in MFMA row order
    }
    // Input ring R(L) holds layer L-1's columns one column ahead of layer L's,
    // the residual ring R(L-1) two columns ahead.  Addresses for each ring
    // phase (chunk index mod the ring's chunk count).
    constexpr int PI = kPeriod(L), PO = L < 6 ? kPeriod(L + 1) : 1, PX = RES ? kPeriod(L - 1) : 1;
    unsigned radr[NF][PI], xadr[PX], oadr[PO];
#pragma unroll
    for (int j = 0; j < PI; ++j)
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            const Slot sl = fslot(L, f, g);
            radr[f][j] = ring_at(L, ring_row(L, j, li + sl.dq - 1), sl.oct);
        }
#pragma unroll
    for (int j = 0; j < PX; ++j) xadr[j] = RES ? ring_at(L - 1, ring_row(L - 1, j, li - 2), g) : 0u;
    // epilogue: after the permlane16 swap lane group g stores the hi (g even)
    // or lo (g odd) octet of rows 8(g >> 1) .. +7 of each m-block: ring octet
    // 2m + (g >> 1) (address oadr ^ 32m); ConvT4's permuted m-blocks hold
    // octets 1, 2 (phases 1, 2) and 0, 3 (address oadr ^ 16)
    constexpr unsigned MX = L == 3 ? 16u : 32u;
    const int obase = L == 3 ? 1 + (g >> 1) : (g >> 1);
#pragma unroll
    for (int j = 0; j < PO; ++j)
        oadr[j] = L < 6 ? (g & 1) * kLoOff(L + 1) + ring_at(L + 1, ring_row(L + 1, j, li), obase) : 0u;
    // identity A of m-block m: row li takes input row 16m + li = 8g + e
    u32x4 aid[NMB];
#pragma unroll
    for (int m = 0; m < NMB; ++m) {
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (_Float16)(16 * m + li == 8 * g + e ? 1.f : 0.f);
        aid[m] = __builtin_bit_cast(u32x4, v);
    }
    const int sL = qa + NL - 1 - L;  // first column of chunk 0
    auto work = [&](int k, auto jc) {
        constexpr int kk = decltype(jc)::value;  // k mod lcm of the ring periods
        constexpr int ji = kk % PI, jx = kk % PX, jo = kk % PO;
        u32x4 bh[NF], bl[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f)
            if (used(f)) {
                bh[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][ji]);
                bl[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][ji] + kLoOff(L));
            }
        u32x4 xh, xl;
        if constexpr (RES) {
            xh = *reinterpret_cast<const u32x4*>(lds + xadr[jx]);
            xl = *reinterpret_cast<const u32x4*>(lds + xadr[jx] + kLoOff(L - 1));
        }
        // hi*hi, hi*lo and lo*hi into one fp32 accumulator per m-block
        f32x4 acc[NMB];
#pragma unroll
        for (int m = 0; m < NMB; ++m) acc[m] = f32x4{bv[m][0], bv[m][1], bv[m][2], bv[m][3]};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                for (int m = 0; m < NMB; ++m)
                    if (kb < nkbm(L, m)) {
                        const int f = frag(L, m, kb);
                        acc[m] = mfma_h(a[m][kb][pr == 2], pr == 1 ? bl[f] : bh[f], acc[m]);
                    }
        if constexpr (RES) {
#pragma unroll
            for (int m = 0; m < NMB; ++m) acc[m] = mfma_h(aid[m], xh, acc[m]);
#pragma unroll
            for (int m = 0; m < NMB; ++m) acc[m] = mfma_h(aid[m], xl, acc[m]);
        }
        const int x0 = sL + 16 * k;  // this chunk's first column
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
            // Both m-blocks in one basic block (the compiler interleaves their
            // dependent VALU chains); chunks that straddle an utterance end
            // take the copy that zeroes columns outside [0, L2).
            auto epilogue = [&](auto zc) {
                constexpr bool ZERO = decltype(zc)::value;
                float v[NMB][4];
#pragma unroll
                for (int m = 0; m < NMB; ++m) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[m][r] = acc[m][r];
                    if constexpr (ACT == ACT_LEAKY) leaky4(v[m]);
                }
                if constexpr (ZERO) {
                    const int x = x0 + li;
                    const bool out = x < 0 || x >= L2;
#pragma unroll
                    for (int m = 0; m < NMB; ++m)
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[m][r] = out ? 0.f : v[m][r];
                    if constexpr (L == 4 && NL == 6) {
                        // outc_role's edge terms: lane group g holds channels
                        // 4(g & 1) .. +3 of phase 2m + (g >> 1) in m-block m, so
                        // groups 0, 1 have h[:, 0] at column 0 and groups 2, 3
                        // h[:, L4 - 1] at column L2 - 1 (m-block 1); each adds
                        // its four products (group 0 / 2 also kL / kR) into
                        // slot g.  (Opaque pointer: the 18 constants are loaded
                        // in this rare branch, not hoisted into VGPRs.)
                        const float* cp = bias + kOutcCorr;
                        asm volatile("" : "+s"(cp));
                        const bool right = g >= 2;
                        if (right ? x == L2 - 1 : x == 0) {
                            const float* cv = cp + (right ? 8 + 4 * (g - 2) : 4 * g);
                            float d = g == 0 ? cp[16] : (g == 2 ? cp[17] : 0.f);
#pragma unroll
                            for (int r = 0; r < 4; ++r) d = fmaf(cv[r], right ? v[1][r] : v[0][r], d);
                            *reinterpret_cast<float*>(lds + kCorrSlot + 4 * g) = d;
                        }
                    }
                }
#pragma unroll
                for (int m = 0; m < NMB; ++m) {
                    unsigned h0, h1, l0, l1;
                    split2u(v[m][0], v[m][1], h0, l0);
                    split2u(v[m][2], v[m][3], h1, l1);
                    // Lane groups 0/1 (and 2/3) hold channels 0-3 / 4-7 (8-11 /
                    // 12-15) of the m-block; one permlane16 swap per dword gives
                    // group 0 the hi octet of channels 0-7 and group 1 its lo
                    // octet (groups 2/3: channels 8-15), so each lane stores one
                    // 16-B chunk (ds_write_b128) instead of two 8-B halves.
                    const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
                    const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
                    *reinterpret_cast<u32x4*>(lds + (oadr[jo] ^ (MX * m))) = u32x4{s0[0], s1[0], s0[1], s1[1]};
                }
            };
            // (layer 4 of the six-layer form also takes it for a chunk that
            // starts at column 0 or ends at L2: outc_role's edge terms)
            constexpr int EW = L == 4 && NL == 6 ? 1 : 0;
            if (edge && (x0 < EW || x0 + 16 > L2 - EW)) epilogue(std::true_type{});  // wave-uniform
            else epilogue(std::false_type{});
        }
    };
    const int LAST = last_step(nch, NL);
    auto step = [&](int s, auto jc) {
        if (s <= LAST) {
            TPSTAMP(s + 1, 0);
            const int k = s - off_l(L);
            if (k >= -1 && k < nch) work(k, jc);
            TPSTAMP(s + 1, 1);
            step_barrier();
        }
    };
    // step s handles chunk k = s - L - 1; the loop is unrolled by U, the lcm
    // of the periods of the rings this layer touches, so every ring phase is a
    // compile-time index: copy i of the iteration starting at step s sees
    // k mod U = (J0 + i) mod U.
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

// ResBlock4 conv2 and output_conv composed into one layer (NL = 6): the
// resblock's output y = conv2(h) + b2 + x feeds only the output conv, which
// is linear, so audio = tanh(Wc * h + Wo * x + bo') with Wc = Wo o W2 (a k5
// conv on h, ResBlock4's intermediate, ring R5) and Wo (k3 on x, ConvT4's
// output, ring R4, two columns ahead like a residual read).  On the 4-phase
// column form both still span columns q-1 .. q+1: fragments 0, 1 read R5
// (tp::fslot of the 2-phase layers: (q, 0..3), (q-1, 2|3), (q+1, 0|1)),
// fragments 2, 3 read R4 (those of output_conv), 4 k-blocks = 12 MFMAs per
// chunk against 10 + 6 for the two layers, one pipeline step and one wave
// fewer.  The reference zero-pads y, not h: the composed form sees a y at
// t = -1 and t = L4 (b2 + conv2 of the edge sample), so the two edge samples
// of an utterance subtract that term (kL + vL . h[:, 0], kR + vR . h[:, L4-1])
// before tanh.  Layer 4 computes those two sums from its fp32 outputs in the
// epilogue of the chunk that holds the column and leaves them in an LDS slot
// (kCorrSlot; one writer per strip, read at least one step later), so this
// role, at the 80-VGPR budget with its four fragment pairs, adds one read.
__device__ __forceinline__ void outc_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                          const u32x4* __restrict__ W, const float* __restrict__ bias,
                                          float* __restrict__ arow, int* rflag) {
    constexpr int L = 5, NL = 6, NF = 4, P = 4;  // rings R4 and R5 both hold 4 chunks
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    u32x4 a[NF][2];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        a[f][0] = W[(kOutcUnit0 + f) * 128 + lane];
        a[f][1] = W[(kOutcUnit0 + f) * 128 + 64 + lane];
    }
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = bias[kOutcBias + 4 * g + r];
    // Fragment addresses as one VGPR each: on a 64-row ring the row of ring
    // phase j is (c + 16 j) mod 64 and the swizzle depends on row bits 1-2
    // only, so ring_at(n, ring_row(n, j, c), o) - kRingOff(n) =
    // (rbase + 1024 j) & 4095 with rbase its j = 0 value (four VGPRs instead
    // of sixteen: this role holds four weight fragment pairs).
    static_assert(kRingRows[4] == 64 && kRingRows[5] == 64, "64-row rings");
    unsigned rbase[NF];
#pragma unroll
    for (int f = 0; f < NF; ++f) {
        const Slot sl = outc_slot(f, g);
        // R5 holds layer 4's columns one ahead of this layer's, R4 layer 3's two
        rbase[f] = f < 2 ? ring_at(5, ring_row(5, 0, li + sl.dq - 1), sl.oct) - kRingOff(5)
                         : ring_at(4, ring_row(4, 0, li + sl.dq - 2), sl.oct) - kRingOff(4);
    }
    auto radr = [&](int f, int j) { return (f < 2 ? kRingOff(5) : kRingOff(4)) + ((rbase[f] + 1024u * j) & 4095u); };
    auto work = [&](int k, auto jc) {
        constexpr int j = decltype(jc)::value;
        u32x4 bh[NF], bl[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            bh[f] = *reinterpret_cast<const u32x4*>(lds + radr(f, j));
            bl[f] = *reinterpret_cast<const u32x4*>(lds + radr(f, j) + (f < 2 ? kLoOff(5) : kLoOff(4)));
        }
        const int x0 = qa + 16 * k, x = x0 + li;
        f32x4 acc = f32x4{bv[0], bv[1], bv[2], bv[3]};
#pragma unroll
        for (int f = 0; f < NF; ++f)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr) acc = mfma_h(a[f][pr == 2], pr == 1 ? bl[f] : bh[f], acc);
        float v[4] = {acc[0], acc[1], acc[2], acc[3]};
        if (edge && (x0 <= 0 || x0 + 16 >= L2)) {  // wave-uniform
            // the edge terms layer 4 left in the slot (written in an earlier step)
            const f32x4 e = *reinterpret_cast<const f32x4*>(lds + kCorrSlot);
            if (x == 0) v[0] -= e[0] + e[1];
            if (x == L2 - 1) v[3] -= e[2] + e[3];
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

// U2 rows (128 B: hi[32] lo[32], the mid kernel's output format) into ring R0,
// two chunks ahead: chunk c = columns [qa + 7 + 16c, +16), zero outside [0, L2).
// EDGE: the strip's columns (with the prologue / epilogue chunks) may leave
// [0, L2); interior strips skip the clamps and the zero selects.
template <int NL, bool EDGE>
__device__ __forceinline__ void loader_role(unsigned char* lds, int qa, int L2, int nch,
                                            const unsigned char* __restrict__ u2) {
    const int lane = threadIdx.x & 63, r = lane >> 3, pc = lane & 7;
    // Every step issues its two loads unconditionally (column clamped into the
    // utterance, zeroed when written) so the compiler can count them: the
    // write of chunk s then waits with vmcnt(4) for its own loads only, not
    // for the two younger chunks still in flight.
    auto fetch = [&](int c, u32x4 (&v)[2]) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int col = qa + NL + 16 * c + r + 8 * h;
            if (EDGE) col = min(max(col, 0), L2 - 1);
            v[h] = *reinterpret_cast<const u32x4*>(u2 + (size_t)col * 128 + pc * 16);
        }
    };
    // Three register buffers used in rotation by a loop unrolled by three, so
    // no register that a load in flight writes is ever copied (a copy would
    // wait for that load).
    u32x4 buf[3][2];
    // R0 has 3 chunks: chunk s sits in ring phase s mod 3 (the loop below is
    // unrolled by three, so copy i writes phase (i + 2) mod 3).  Lanes pc 0-3
    // carry hi octets, 4-7 lo octets.
    unsigned wadr[3][2];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int h = 0; h < 2; ++h) wadr[j][h] = (pc >> 2) * kLoOff(0) + ring_at(0, ring_row(0, j, r + 8 * h), pc & 3);
    auto step = [&](int s, auto jc, u32x4 (&cur)[2], u32x4 (&ahead)[2]) {
        constexpr int j = decltype(jc)::value;
        fetch(min(s + 2, nch - 1), ahead);  // past the strip: re-read the last chunk (an L2 hit)
        if (s < nch) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int col = qa + NL + 16 * s + r + 8 * h;
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
    for (; s + 2 <= last_step(nch, NL); s += 3) {  // covers every step with work (s <= nch - 1)
        step(s, ic<2>{}, buf[0], buf[2]);
        step(s + 1, ic<0>{}, buf[1], buf[0]);
        step(s + 2, ic<1>{}, buf[2], buf[1]);
    }
#pragma unroll 1
    for (; s <= last_step(nch, NL); ++s) step_barrier();
}

// TAILP_DMA: U2 rows into ring R0 by LDS-DMA.  One buffer_load_dwordx4 ...
// lds writes 64 lanes x 16 B = 1 KB at M0 + 16 x lane, i.e. exactly the 16
// rows (columns) of a chunk's hi plane (or lo plane) in ring phase c mod 4;
// lane l fills row l / 4, slot l % 4, so it loads the U2 octet ring_at
// places there (octet (l % 4) ^ ((row >> 1) & 3)).  The descriptor spans the
// utterance's L2 rows: columns before 0 or from L2 on are out of range and
// land as zeros (the next conv's zero padding), so edge and interior strips
// run the same code.  Chunk c + 1 is issued at the top of step c into the
// slot of chunk c - 3 (read for the last time in step c - 1, before that
// step's barrier); chunk c must have landed before step c's barrier
// (vmcnt(2): only chunk c + 1's two loads may still be in flight).
template <int NL>
__device__ __forceinline__ void loader_role_dma(unsigned char* lds, int qa, int L2, int nch,
                                                const unsigned char* __restrict__ u2) {
    static_assert(NL > 0 && kRingRows[0] == 64, "4-chunk R0");
    const int lane = threadIdx.x & 63, row = lane >> 2;
    [[maybe_unused]] const int oct = (lane & 3) ^ ((row >> 1) & 3);
    // the descriptor starts at the strip's first column (32-bit offsets stay
    // small for any utterance length) and ends at the utterance's last row;
    // columns before 0 only occur in the first strip, whose base is column 0
    const int c0 = max(0, qa + NL - 16);
    [[maybe_unused]] const auto rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(u2) + (size_t)c0 * 128, 0, (int)min((long)(L2 - c0) * 128, 0x7fffffffL),
        0x00020000);
    auto dma = [&](int c) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass of hipcc does not know this builtin)
        const int voff = (qa + NL + 16 * c + row - c0) * 128 + 16 * oct;  // < 0 or >= L2 rows: out of range -> 0
        unsigned char* dst = lds + kRingOff(0) + 1024 * (c & 3);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)dst, 16, voff, 0, 0,
                                                 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + kLoOff(0)), 16,
                                                 voff + 64, 0, 0, 0);
#endif
    };
    dma(-1);
#pragma unroll 1
    for (int s = -1; s <= last_step(nch, NL); ++s) {
        if (s + 1 < nch) {
            dma(s + 1);
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        step_barrier();
    }
}

// NCHC > 0: the strip length as a compile-time constant (the headline's 21,
// measured 0.45 us faster than the same length as an argument); 0: nch.
template <int NL, int NCHC>
__global__ __launch_bounds__(nwaves(NL) * 64, 6) void tailp_kernel(const unsigned char* __restrict__ U2, int L2,
                                                                    int nch_arg, const u32x4* __restrict__ W,
                                                                    const float* __restrict__ bias,
                                                                    float* __restrict__ audio, int* rflag,
                                                                    const int32_t* __restrict__ dT, VocRedo rd) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int nch = NCHC ? NCHC : nch_arg;
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
    TPSTAMP(62, 0);
    // Later layers get higher issue priority: they are the younger waves of
    // the workgroup and lose VALU arbitration on age (MI355X_MICROARCH.md, two
    // waves per SIMD), while the step waits for the slowest role (-1.5 %).
    // (Pairing the roles so that waves w and w + 4, which share a SIMD, carry
    // equal MFMA counts measured the same: the step is latency-bound.)
    if (w >= 5) __builtin_amdgcn_s_setprio(3);
    else if (w >= 3) __builtin_amdgcn_s_setprio(2);
    else if (w >= 1) __builtin_amdgcn_s_setprio(1);
    const unsigned char* u2 = U2 + (size_t)b * L2 * 128;
    switch (w) {
        case 0: layer_role<0, 2, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 1: layer_role<1, 2, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 2: layer_role<2, 2, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 3: layer_role<3, 2, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 4: layer_role<4, 2, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag); break;
        case 5:
            if constexpr (NL == 7) layer_role<5, 2, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag);
            else outc_role(lds, qa, L2, nch, edge, W, bias, arow, rflag);
            break;
        case 6:
            if constexpr (NL == 7) {
                layer_role<6, 1, NL>(lds, qa, L2, nch, edge, W, bias, arow, rflag);
                break;
            }
            [[fallthrough]];
        default:
            if constexpr (TAILP_DMA) loader_role_dma<NL>(lds, qa, L2, nch, u2);
            else if (edge) loader_role<NL, true>(lds, qa, L2, nch, u2);
            else loader_role<NL, false>(lds, qa, L2, nch, u2);
            break;
    }
    TPSTAMP(63, 0);
    if (rd.rw) {  // range policy "fallback": this strip's audio again in fp32 if it is not finite
        __syncthreads();
        if (*lflag)
            redo_frames(*rd.rw, rd.mel, rd.trans, L2 / 16, b, qa / 16, min(L2, qa + 16 * nch) / 16, arow,
                        reinterpret_cast<float*>(lds), ring_bytes(NL) / 4);
    }
}

template <int NL, int NCHC>
int32_t launch(int nch, const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
               int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    static bool attr = false;
    if (!attr) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(tailp_kernel<NL, NCHC>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes(NL)));
        attr = true;
    }
    hipLaunchKernelGGL((tailp_kernel<NL, NCHC>), dim3(cdiv(L2, 16 * nch), B), dim3(nwaves(NL) * 64), lds_bytes(NL),
                       st, static_cast<const unsigned char*>(U2), L2, nch, W, bias, audio, rflag, dT, rd);
    M2_LAUNCHED("tailp_kernel");
    return M2_OK;
}
template <int NL>
int32_t launch_nl(int nch, const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                  int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    return nch == 21 ? launch<NL, 21>(nch, U2, L2, B, W, bias, audio, rflag, st, dT, rd)
                     : launch<NL, 0>(nch, U2, L2, B, W, bias, audio, rflag, st, dT, rd);
}

}  // namespace tp

#ifdef M2_STAMPS
extern "C" int32_t m2_debug_stamps_tailp(void* host, size_t bytes) {
    return (int32_t)hipMemcpyFromSymbol(host, HIP_SYMBOL(tp::g_tp_stamps),
                                        bytes < sizeof(tp::g_tp_stamps) ? bytes : sizeof(tp::g_tp_stamps));
}
#endif

const char* const kVocTailpKernelName =
    "tailp_kernel (ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv, pipelined)";

int32_t launch_vocoder_tailp(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                             int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    if (B == 0 || L2 == 0) return M2_OK;
    // Strip length (16-column chunks per workgroup, a launch argument): the
    // one from 8 to 256 minimising rounds of 768 workgroups (three per CU) x
    // pipeline steps (stage1 B = 32, L2 = 8000: 24 strips of 21 chunks, one
    // round; B = 8: 63 strips of 8).  M2_TAILP_NCH forces one.
    const int nl = sw().tailp_seven ? 7 : 6;
    int nch = sw().tailp_nch > 0 ? std::min(sw().tailp_nch, 4096) : 0;
    if (!nch) {
        const long chunks = cdiv(L2, 16);
        long best = -1;
        for (int n = 8; n <= 256; ++n) {
            const long wgs = (long)cdiv((int)chunks, n) * B, rounds = (wgs + 767) / 768, cost = rounds * (n + nl + 1);
            if (best < 0 || cost < best) best = cost, nch = n;
        }
    }
    // M2_TAILP_SEVEN=1: ResBlock4 conv2 and the output conv as two layers
    // (the round-2 form; A/B and test switch, m2_common.h switch table).
    // (A wave -> role map that balances the MFMA load of the SIMDs — the
    // hardware puts wave w on SIMD c[(w + r) mod 4], c = (0, 2, 1, 3), with a
    // rotation r per co-resident workgroup, tools/probe/simd_map.hip — gave
    // classes of 18/21/16/12 MFMAs instead of 18/24/16/9 and measured the same:
    // the step is latency-bound, not bound by one SIMD's MFMA pipe.)
    const bool seven = sw().tailp_seven;
    return seven ? tp::launch_nl<7>(nch, U2, L2, B, W, bias, audio, rflag, st, dT, rd)
                 : tp::launch_nl<6>(nch, U2, L2, B, W, bias, audio, rflag, st, dT, rd);
}

// ---------------------------------------------------------------------------
// Host packing.  Each layer is first written as a dense polyphase matrix
// Wd[row][dq + 1][input row] (32 x 3 x 32), then cut into (m-block, k-block)
// fragment pairs along tp::kslot: A[row = mb*16 + (lane&15)][slot g = lane>>4,
// element e] = Wd[row][dq + 1][8*oct + e], zero on a repeated slot.  Every
// non-zero of Wd must sit on a slot.
namespace {

int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

struct Dense {
    std::vector<float> w = std::vector<float>(32 * 3 * 32, 0.f);
    float& at(int row, int dq, int in) { return w[(row * 3 + dq + 1) * 32 + in]; }
};

// ConvTranspose1d(k=4, stride 2, pad 1), W [Cin][Cout][4], on a Pin-phase input
// (Cin channels per phase) -> 2*Pin phases of Cout channels (tts_model.py:255-263):
// out[2i] = x[i] W1 + x[i-1] W3, out[2i+1] = x[i+1] W0 + x[i] W2.
void dense_convT2(Dense& d, const float* W, int Pin, int Cin, int Cout) {
    const int taps[2][2][2] = {{{0, 1}, {-1, 3}}, {{1, 0}, {0, 2}}};  // [s][j] = (input offset, kernel tap)
    for (int pin = 0; pin < Pin; ++pin)
        for (int s = 0; s < 2; ++s)
            for (int j = 0; j < 2; ++j) {
                const int pp = pin + taps[s][j][0], dq = floordiv(pp, Pin), p2 = pp - dq * Pin, kk = taps[s][j][1];
                for (int co = 0; co < Cout; ++co)
                    for (int ci = 0; ci < Cin; ++ci)
                        d.at((2 * pin + s) * Cout + co, dq, p2 * Cin + ci) += W[((size_t)ci * Cout + co) * 4 + kk];
            }
}

// Conv1d(k=3, pad 1), W [Cout][Cin][3], on a P-phase signal.
void dense_conv3(Dense& d, const float* W, int P, int Cin, int Cout) {
    for (int p = 0; p < P; ++p)
        for (int k = 0; k < 3; ++k) {
            const int pp = p + k - 1, dq = floordiv(pp, P), p2 = pp - dq * P;
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

bool pack_outc(const TailpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok);

bool pack_tailp(const TailpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok) {
    Dense d[tp::kLayers];
    dense_convT2(d[0], s.wt3, 1, 32, 16);
    dense_conv3(d[1], s.w31, 2, 16, 16);
    dense_conv3(d[2], s.w32, 2, 16, 16);
    dense_convT2(d[3], s.wt4, 2, 16, 8);
    dense_conv3(d[4], s.w41, 4, 8, 8);
    dense_conv3(d[5], s.w42, 4, 8, 8);
    dense_conv3(d[6], s.wo, 4, 8, 1);
    const int nrows[tp::kLayers] = {32, 32, 32, 32, 32, 32, 4};
    for (int l = 0; l < tp::kLayers; ++l)
        for (int R = 0; R < 32; ++R)  // MFMA row R computes dense row prow(l, R)
            for (int dq = -1; dq <= 1; ++dq)
                for (int in = 0; in < 32; ++in) {
                    const int row = tp::prow(l, R);
                    if (d[l].at(row, dq, in) == 0.f) continue;
                    bool missing = row < nrows[l];
                    for (int kb = 0; missing && kb < tp::nkbm(l, R / 16); ++kb)
                        for (int g = 0; g < 4; ++g) {
                            const tp::Slot sl = tp::kslot(l, R / 16, kb, g);
                            if (sl.dq == dq && sl.oct == in / 8) missing = false;
                        }
                    if (missing) return false;  // a non-zero weight that no slot reads
                }
    wout->assign((size_t)(tp::kUnits + tp::kOutcUnits) * 2 * 64 * 8, 0);
    for (int l = 0; l < tp::kLayers; ++l)
        for (int mb = 0; mb < tp::nmb(l); ++mb)
            for (int kb = 0; kb < tp::nkbm(l, mb); ++kb) {
                const int u = tp::unit0(l) + mb * tp::nkb(l) + kb;
                for (int lane = 0; lane < 64; ++lane) {
                    const int row = tp::prow(l, mb * 16 + (lane & 15)), g = lane >> 4;
                    const tp::Slot sl = tp::kslot(l, mb, kb, g);
                    // a (dq, octet) the m-block already reads in an earlier slot gets zeros
                    bool dup = false;
                    for (int j = 0; j < kb * 4 + g; ++j) {
                        const tp::Slot o = tp::kslot(l, mb, j / 4, j % 4);
                        dup = dup || (o.dq == sl.dq && o.oct == sl.oct);
                    }
                    for (int e = 0; e < 8; ++e) {
                        float v = 0.f;
                        if (row < nrows[l] && !dup) v = d[l].at(row, sl.dq, 8 * sl.oct + e);
                        put_split(*wout, (((size_t)u * 2) * 64 + lane) * 8 + e, v, range_ok);
                    }
                }
            }
    bout->assign(tp::kBiasFloats, 0.f);
    const float* bsrc[tp::kLayers] = {s.bt3, s.b31, s.b32, s.bt4, s.b41, s.b42, s.bo};
    const int cper[tp::kLayers] = {16, 16, 16, 8, 8, 8, 1};
    for (int l = 0; l < tp::kLayers; ++l)
        for (int R = 0; R < nrows[l]; ++R) (*bout)[l * 32 + R] = bsrc[l][tp::prow(l, R) % cper[l]];
    return pack_outc(s, wout, bout, range_ok);
}

// The composed ResBlock4-conv2 + output_conv layer (outc_role), in double:
// audio[t] = tanh(bo' + sum_d Wo[c][d] x[c][t+d] + sum_j Wc[c'][j] h[c'][t+j]),
// Wc[c'][j] = sum_{d+e=j} sum_c Wo[c][d] W2[c][c'][e], bo' = bo + sum_d sum_c
// Wo[c][d] b2[c]; on the 4-phase columns (row p = output phase, input row
// p2*8 + c at column q + dq).  Edge terms: the y the composed form sees at
// t = -1 is b2 + W2[.][.][2] h[., 0], at t = L4 it is b2 + W2[.][.][0] h[., L4-1].
namespace {
// The composed layer's dense matrices on the 4-phase columns (dh on ResBlock4's
// intermediate h, dx on ConvT4's output x: [output phase][dq + 1][input row]),
// its bias and the edge terms vL[8], vR[8], kL, kR.
struct OutcDense {
    double dh[4][3][32] = {}, dx[4][3][32] = {}, bo = 0.0, corr[18] = {};
};
OutcDense outc_dense(const TailpSrc& s) {
    OutcDense o;
    auto& dh = o.dh;
    auto& dx = o.dx;
    auto wo = [&](int c, int k) { return (double)s.wo[c * 3 + k]; };
    auto w2 = [&](int c, int ci, int k) { return (double)s.w42[(c * 8 + ci) * 3 + k]; };
    for (int p = 0; p < 4; ++p)
        for (int d = -1; d <= 1; ++d)
            for (int c = 0; c < 8; ++c) {
                const int tx = p + d, qx = floordiv(tx, 4);
                dx[p][qx + 1][(tx - 4 * qx) * 8 + c] += wo(c, d + 1);
                for (int e = -1; e <= 1; ++e)
                    for (int ci = 0; ci < 8; ++ci) {
                        const int th = p + d + e, qh = floordiv(th, 4);
                        dh[p][qh + 1][(th - 4 * qh) * 8 + ci] += wo(c, d + 1) * w2(c, ci, e + 1);
                    }
            }
    double bo = s.bo[0], kl = 0.0, kr = 0.0;
    for (int c = 0; c < 8; ++c) {
        for (int k = 0; k < 3; ++k) bo += wo(c, k) * s.b42[c];
        kl += wo(c, 0) * s.b42[c];
        kr += wo(c, 2) * s.b42[c];
    }
    o.bo = bo;
    for (int ci = 0; ci < 8; ++ci) {
        double vl = 0.0, vr = 0.0;
        for (int c = 0; c < 8; ++c) {
            vl += wo(c, 0) * w2(c, ci, 2);
            vr += wo(c, 2) * w2(c, ci, 0);
        }
        o.corr[ci] = vl;
        o.corr[8 + ci] = vr;
    }
    o.corr[16] = kl;
    o.corr[17] = kr;
    return o;
}
}  // namespace

bool pack_outc(const TailpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok) {
    const OutcDense o = outc_dense(s);
    const auto& dh = o.dh;
    const auto& dx = o.dx;
    // every non-zero on a slot (fragments 0, 1: h; 2, 3: x)
    for (int p = 0; p < 4; ++p)
        for (int dq = -1; dq <= 1; ++dq)
            for (int in = 0; in < 32; ++in)
                for (int src = 0; src < 2; ++src) {
                    if ((src ? dx : dh)[p][dq + 1][in] == 0.0) continue;
                    bool found = false;
                    for (int f = 2 * src; f < 2 * src + 2; ++f)
                        for (int g = 0; g < 4; ++g) {
                            const tp::Slot sl = tp::outc_slot(f, g);
                            found = found || (sl.dq == dq && sl.oct == in / 8);
                        }
                    if (!found) return false;
                }
    for (int f = 0; f < tp::kOutcUnits; ++f)
        for (int lane = 0; lane < 64; ++lane) {
            const int row = lane & 15, g = lane >> 4;
            const tp::Slot sl = tp::outc_slot(f, g);
            const bool dup = f == 3 && g >= 2;  // (q, 2), (q, 3) of x are read by fragment 2
            for (int e = 0; e < 8; ++e) {
                double v = 0.0;
                if (row < 4 && !dup) v = (f < 2 ? dh : dx)[row][sl.dq + 1][8 * sl.oct + e];
                put_split(*wout, (((size_t)(tp::kOutcUnit0 + f) * 2) * 64 + lane) * 8 + e, (float)v, range_ok);
            }
        }
    for (int r = 0; r < 4; ++r) (*bout)[tp::kOutcBias + r] = (float)o.bo;
    for (int i = 0; i < 18; ++i) (*bout)[tp::kOutcCorr + i] = (float)o.corr[i];
    return true;
}

}  // namespace m2
