// Register-hand-off stage1 vocoder tail (M2_TAILR=1): the layers of
// vocoder_tailp.hip's six-layer form (tts_model.py:279-297: ConvT3 + leaky,
// ResBlock3, ConvT4 + leaky, ResBlock4 conv1, then ResBlock4 conv2 composed
// with output_conv + tanh) in the same split-f16 arithmetic and polyphase
// column form, without the per-layer LDS hand-off.
//
// Why.  vocoder_tailp.hip gives every layer its own wave: a layer's output
// chunk goes through an LDS ring to the next wave, and all seven waves meet at
// a workgroup barrier every 16 columns, so each step waits for the slowest
// layer's LDS read -> MFMA -> epilogue -> LDS write chain (DESIGN.md section 4,
// "Why the tail sits near 0.2").  Here one wave runs several layers of a chunk
// back to back and hands a layer's output to the next in registers: the next
// layer's k3 taps are the same register block shifted by one or two columns,
// and the 16 columns of an MFMA tile are the 16 lanes of a DPP row, so a tap
// is a `row_shr` whose first columns come from the previous chunk's block
// (`row_ror` of it) - two DPP moves per dword, no LDS traffic, no barrier.
//
// Layout.  An MFMA accumulator holds rows 4g .. 4g + 3 of an m-block in lane
// group g (columns = lanes 0-15); a B fragment wants eight consecutive input
// rows (an "octet") per lane group.  After the split into f16 hi / lo pairs,
// one v_permlane32_swap and one v_permlane16_swap per dword pair regroup the
// two m-blocks' accumulators into a 32-row column block whose lane group g
// holds octet g - or, with the m-blocks swapped, octets (2, 3, 0, 1); layers
// whose next layer reads octets in another order compute their rows in an
// order that makes the regrouping produce it (tr::rrow, ConvT4).  The slot
// tables (vocoder_fused.h, tr::) then put one column shift on all four lane
// groups of a fragment wherever the taps allow, and a row-masked DPP (a shift
// for some lane groups only) where they do not.
//
// Work split.  Two waves per workgroup, a two-stage pipeline over the strip's
// chunks with one s_barrier per step:
//   wave 0 (front): ConvT3 (B fragments read from the U2 ring), ResBlock3
//     conv1 and conv2 in registers; writes ResBlock3's output to ring R.
//   wave 1 (back): streams U2 into its ring (global -> LDS, two chunks ahead),
//     ConvT4 (fragments from ring R), ResBlock4 conv1 and the composed output
//     layer in registers; tanh, audio store, non-finite flag.
// 128 threads, ~13 KB of rings, four workgroups (eight waves, two per SIMD) per
// CU; a strip of nch chunks takes nch + 3 steps.  Columns outside [0, L2) are
// zeroed in every layer's output (the next conv's zero padding), the composed
// layer's edge terms as in vocoder_tailp.hip.  Chunk -1 is the warm-up of the
// lagged layers (each layer's chunk sits one column left of its input's, the
// composed layer's x two), its first columns read the previous-chunk blocks,
// which start at zero (finite; only columns no later layer reads).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "m2_common.h"
#include "vocoder_fused.h"

namespace m2 {
namespace tr {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef vx_u32x4 u32x4;
typedef float f32x4 __attribute__((ext_vector_type(4)));

// LDS: two rings of 3 chunks (48 columns) of 32 rows x (hi, lo) f16 each, as
// vocoder_tailp.hip's rings (64-B hi rows, the lo plane kPlane bytes later,
// octet o of row r at 16 (o ^ ((r >> 1) & 3)): conflict-free reads and
// writes); the local redo's windows reuse the bytes below kRedoBytes; the
// edge-term slot and the non-finite word after them.
constexpr int kRows = 48;
constexpr int kPlane = kRows * 64;
constexpr int kU2Off = 0, kROff = 2 * kPlane;
constexpr int kRedoBytes = 36864;  // redo_frames' two window buffers for 3 frames at C = 128
constexpr int kCorrOff = kRedoBytes, kFlagOff = kRedoBytes + 16, kLdsBytes = kRedoBytes + 32;
static_assert(kROff + 2 * kPlane <= kRedoBytes, "rings below the redo region");
static_assert(4 * kLdsBytes <= 160 * 1024, "four workgroups per CU");
constexpr int kWaves = 2;

__device__ __forceinline__ unsigned ring_at(int base, int row, int oct) {
    return base + row * 64 + 16 * (oct ^ ((row >> 1) & 3));
}
// row of column c (-3 .. 15) of the chunk in ring slot j
__device__ __forceinline__ int ring_row(int j, int c) {
    const int r = 16 * j + c;
    return r < 0 ? r + kRows : (r >= kRows ? r - kRows : r);
}

__device__ __forceinline__ f32x4 mfma_h(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float tanh_fast(float x) { return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x)); }

template <int V>
using ic = std::integral_constant<int, V>;

#ifndef TR_DIAG  // diagnostic timing builds only: 1 = the front wave skips its layers, 2 = the back wave its
#define TR_DIAG 0
#endif

// A 32-row column block of 16 columns (or a B fragment): hi and lo planes.
struct Blk {
    u32x4 h, l;
};

template <int CTRL, int RM>
__device__ __forceinline__ u32x4 dpp4(u32x4 old, u32x4 src) {
    u32x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = (unsigned)__builtin_amdgcn_update_dpp((int)old[i], (int)src[i], CTRL, RM, 0xF, false);
    return r;
}
// `base` with the lane groups of RM replaced by `cur` shifted N columns right
// (lane li takes column li - N), its first N columns from `prev` (the previous
// chunk's columns 16 - N .. 15): row_ror of prev, then row_shr of cur, whose
// out-of-row lanes keep the rotated values.
template <int N, int RM>
__device__ __forceinline__ Blk shr(const Blk& base, const Blk& cur, const Blk& prev) {
    static_assert(N >= 1 && N <= 3, "column shifts 1..3");
    const Blk t{dpp4<0x120 + N, RM>(base.h, prev.h), dpp4<0x120 + N, RM>(base.l, prev.l)};
    return Blk{dpp4<0x110 + N, RM>(t.h, cur.h), dpp4<0x110 + N, RM>(t.l, cur.l)};
}

// The two m-blocks' activations (v[m][r]: row 16 m + 4 g + r, column li) as a
// column block: lane group g' holds the octet of m-block P's lane groups
// 2 (g' & 1), +1 (g' < 2) or m-block 1 - P's (g' >= 2), i.e. octets in the
// order (P lo, P hi, Q lo, Q hi).  Per dword pair (rows r, r + 1 of the
// m-blocks): permlane32_swap gathers the lower lane groups of both m-blocks
// into one register and the upper into the other, permlane16_swap then pairs
// each group with its neighbour's rows 4 .. 7.
template <int P>
__device__ __forceinline__ Blk to_block(const unsigned (&h)[2][2], const unsigned (&l)[2][2]) {
    constexpr int Q = 1 - P;
    Blk b;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
        auto a = __builtin_amdgcn_permlane32_swap(h[P][d], h[Q][d], false, false);
        auto c = __builtin_amdgcn_permlane16_swap(a[0], a[1], false, false);
        b.h[d] = c[0];
        b.h[d + 2] = c[1];
        a = __builtin_amdgcn_permlane32_swap(l[P][d], l[Q][d], false, false);
        c = __builtin_amdgcn_permlane16_swap(a[0], a[1], false, false);
        b.l[d] = c[0];
        b.l[d + 2] = c[1];
    }
    return b;
}

__device__ __forceinline__ void split_mb(const float (&v)[2][4], unsigned (&h)[2][2], unsigned (&l)[2][2]) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        split2u(v[m][0], v[m][1], h[m][0], l[m][0]);
        split2u(v[m][2], v[m][3], h[m][1], l[m][1]);
    }
}

// Activation, then zero columns outside [0, L2) when the chunk straddles an
// utterance end (wave-uniform test).
template <bool LEAKY>
__device__ __forceinline__ void activate(const f32x4 (&acc)[2], float (&v)[2][4], int x0, int L2, bool edge) {
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[m][r] = acc[m][r];
        if constexpr (LEAKY) leaky4(v[m]);
    }
    if (edge && (x0 < 0 || x0 + 16 > L2)) {
        const int x = x0 + (threadIdx.x & 15);
        const bool out = x < 0 || x >= L2;
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[m][r] = out ? 0.f : v[m][r];
    }
}

// Weights of (layer, m-block, k-block) for this lane: hi, lo A fragments.
__device__ __forceinline__ void load_unit(const u32x4* __restrict__ W, int u, int lane, u32x4 (&a)[2]) {
    a[0] = W[u * 128 + lane];
    a[1] = W[u * 128 + 64 + lane];
}

// One two-m-block layer: acc[m] = bias + sum over its k-blocks of the three
// split products (hi.hi, hi.lo, lo.hi) of fragment frag(L, m, kb).
template <int L, int NF>
__device__ __forceinline__ void layer_mma(const u32x4 (&a)[2][2][2], const float (&bv)[2][4], const Blk (&F)[NF],
                                          f32x4 (&acc)[2]) {
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[m] = f32x4{bv[m][0], bv[m][1], bv[m][2], bv[m][3]};
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int pr = 0; pr < 3; ++pr)
#pragma unroll
            for (int m = 0; m < 2; ++m)
                if (kb < nkbm(L, m)) {
                    const Blk& f = F[frag(L, m, kb)];
                    acc[m] = mfma_h(a[m][kb][pr == 2], pr == 1 ? f.l : f.h, acc[m]);
                }
}

// Wave 0: ConvT3, ResBlock3 conv1, conv2 (+ x).  Step s computes chunk
// s - 2: its U2 columns were stored by wave 1 in steps s - 2 and s - 1.
__device__ __forceinline__ void front_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                           const u32x4* __restrict__ W, const float* __restrict__ bias) {
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    u32x4 a[3][2][2][2];
    float bv[3][2][4];
#pragma unroll
    for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int m = 0; m < 2; ++m) {
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) load_unit(W, unit(l, m, kb), lane, a[l][m][kb]);
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[l][m][r] = bias[l * 32 + m * 16 + 4 * g + r];
        }
    // identity A of m-block m (ResBlock3's residual): row li takes input row 16m + li = 8g + e
    u32x4 aid[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (_Float16)(16 * m + li == 8 * g + e ? 1.f : 0.f);
        aid[m] = __builtin_bit_cast(u32x4, v);
    }
    // ConvT3's fragments from the U2 ring (ConvT3 lags U2 by one column), ring R's stores
    unsigned radr[3][3], oadr[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const Slot sl = fslot(0, f, g);
            radr[f][j] = ring_at(kU2Off, ring_row(j, li + sl.dq - 1), sl.oct);
        }
        // after the permlane16 swap lane group g stores the hi (g even) or lo
        // (g odd) octet 2m + (g >> 1) (address ^ 32 m)
        oadr[j] = (g & 1) * kPlane + ring_at(kROff, ring_row(j, li), g >> 1);
    }
    const Blk z{u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
    Blk p0 = z, p1 = z;  // previous chunk's ConvT3 / conv1 outputs
    auto work = [&](int k, auto jc) {
        constexpr int j = decltype(jc)::value;  // ring slot of chunk k
        const int x0 = qa + 5 + 16 * k;          // ConvT3's first column
        f32x4 acc[2];
        float v[2][4];
        unsigned h[2][2], l[2][2];
        // ConvT3
        Blk F[3];
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            F[f].h = *reinterpret_cast<const u32x4*>(lds + radr[f][j]);
            F[f].l = *reinterpret_cast<const u32x4*>(lds + radr[f][j] + kPlane);
        }
        layer_mma<0, 3>(a[0], bv[0], F, acc);
        activate<true>(acc, v, x0, L2, edge);
        split_mb(v, h, l);
        const Blk n0 = to_block<0>(h, l);
        // ResBlock3 conv1: columns q, q-1, q+1 of ConvT3's output
        F[0] = shr<1, 0xF>(n0, n0, p0);
        F[1] = shr<2, 0xF>(n0, n0, p0);
        F[2] = n0;
        p0 = n0;
        layer_mma<1, 3>(a[1], bv[1], F, acc);
        activate<true>(acc, v, x0 - 1, L2, edge);
        split_mb(v, h, l);
        const Blk n1 = to_block<0>(h, l);
        const Blk xr = F[1];  // ConvT3's output at conv2's columns (two to the left)
        // ResBlock3 conv2 + x (two identity-A MFMAs per m-block)
        F[0] = shr<1, 0xF>(n1, n1, p1);
        F[1] = shr<2, 0xF>(n1, n1, p1);
        F[2] = n1;
        p1 = n1;
        layer_mma<2, 3>(a[2], bv[2], F, acc);
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m] = mfma_h(aid[m], xr.h, acc[m]);
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m] = mfma_h(aid[m], xr.l, acc[m]);
        activate<false>(acc, v, x0 - 2, L2, edge);
        // to ring R in vocoder_tailp's layout: one 16-B hi or lo octet per lane and m-block
#pragma unroll
        for (int m = 0; m < 2; ++m) {
            unsigned h0, h1, l0, l1;
            split2u(v[m][0], v[m][1], h0, l0);
            split2u(v[m][2], v[m][3], h1, l1);
            const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
            *reinterpret_cast<u32x4*>(lds + (oadr[j] ^ (32u * m))) = u32x4{s0[0], s1[0], s0[1], s1[1]};
        }
    };
    const int last = nch + 2;
    auto step = [&](int s, auto jc) {
        if (s <= last) {
            const int k = s - 2;
            if (TR_DIAG != 1 && k >= -1 && k < nch) work(k, jc);
            step_barrier();
        }
    };
    // s = 3i + u: chunk s - 2 sits in ring slot (u + 1) mod 3
#pragma unroll 1
    for (int s = 0; s <= last; s += 3) {
        step(s, ic<1>{});
        step(s + 1, ic<2>{});
        step(s + 2, ic<0>{});
    }
}

// Wave 1: the U2 loader, ConvT4, ResBlock4 conv1, the composed output layer.
// Step s stores U2 chunk s - 1 and computes chunk s - 3 (ring R's chunk, written
// by wave 0 in step s - 1).
__device__ __forceinline__ void back_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                          const u32x4* __restrict__ W, const float* __restrict__ bias,
                                          const unsigned char* __restrict__ u2, float* __restrict__ arow,
                                          int* rflag) {
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    u32x4 a3[2][2][2], a4[2][1][2], a5[4][2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
            if (kb < nkbm(3, m)) load_unit(W, unit(3, m, kb), lane, a3[m][kb]);
        load_unit(W, unit(4, m, 0), lane, a4[m][0]);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) load_unit(W, unit(5, 0, f), lane, a5[f]);
    float b3[2][4], b4[2][4], b5[4];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            b3[m][r] = bias[3 * 32 + m * 16 + 4 * g + r];
            b4[m][r] = bias[4 * 32 + m * 16 + 4 * g + r];
        }
#pragma unroll
    for (int r = 0; r < 4; ++r) b5[r] = bias[5 * 32 + 4 * g + r];
    // ConvT4's fragments from ring R (one column lag)
    unsigned radr[2][3];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            const Slot sl = fslot(3, f, g);
            radr[f][j] = ring_at(kROff, ring_row(j, li + sl.dq - 1), sl.oct);
        }
    // loader: lane (r, pc) moves 16-B piece pc of the 128-B U2 rows of columns
    // r and r + 8 of a chunk (pieces 0-3 hi octets, 4-7 lo); chunk c = columns
    // qa + 6 + 16 c + [0, 16) (ConvT3's inputs), zero outside [0, L2)
    const int lr = lane >> 3, pc = lane & 7;
    unsigned wadr[3][2];
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) wadr[j][hh] = (pc >> 2) * kPlane + ring_at(kU2Off, ring_row(j, lr + 8 * hh), pc & 3);
    auto fetch = [&](int c, u32x4 (&buf)[2]) {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int col = min(max(qa + 6 + 16 * c + lr + 8 * hh, 0), L2 - 1);
            buf[hh] = *reinterpret_cast<const u32x4*>(u2 + (size_t)col * 128 + pc * 16);
        }
    };
    u32x4 ub[3][2];
    fetch(-1, ub[0]);
    fetch(0, ub[1]);
    const Blk z{u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
    Blk pr3 = z, pl3 = z, pw4 = z;  // previous chunk's ConvT4 output (two orders), ResBlock4 conv1 output
    const float* cp = bias + 6 * 32;  // the composed layer's edge terms vL[8], vR[8], kL, kR
    auto work = [&](int k, auto jc) {
        constexpr int j = decltype(jc)::value;  // ring R slot of chunk k
        const int x0 = qa + 2 + 16 * k;          // ConvT4's first column
        f32x4 acc[2];
        float v[2][4];
        unsigned h[2][2], l[2][2];
        // ConvT4 (rows: m-block 0 = phases 3, 0; m-block 1 = phases 1, 2)
        Blk F[2];
#pragma unroll
        for (int f = 0; f < 2; ++f) {
            F[f].h = *reinterpret_cast<const u32x4*>(lds + radr[f][j]);
            F[f].l = *reinterpret_cast<const u32x4*>(lds + radr[f][j] + kPlane);
        }
        layer_mma<3, 2>(a3, b3, F, acc);
        activate<true>(acc, v, x0, L2, edge);
        split_mb(v, h, l);
        const Blk r3 = to_block<0>(h, l);  // octets (3, 0, 1, 2)
        const Blk l3 = to_block<1>(h, l);  // octets (1, 2, 3, 0)
        // ResBlock4 conv1: m-block 0 reads (q-1, 3) (q, 0) (q, 1) (q, 2), m-block 1
        // (q, 1) (q, 2) (q, 3) (q+1, 0)
        Blk G[2];
        G[0] = shr<2, 0x1>(shr<1, 0xE>(r3, r3, pr3), r3, pr3);
        G[1] = shr<1, 0x7>(l3, l3, pl3);
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m] = f32x4{b4[m][0], b4[m][1], b4[m][2], b4[m][3]};
#pragma unroll
        for (int pr = 0; pr < 3; ++pr)
#pragma unroll
            for (int m = 0; m < 2; ++m) acc[m] = mfma_h(a4[m][0][pr == 2], pr == 1 ? G[m].l : G[m].h, acc[m]);
        const int x1 = x0 - 1;  // ResBlock4 conv1's first column
#pragma unroll
        for (int m = 0; m < 2; ++m) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[m][r] = acc[m][r];
            leaky4(v[m]);
        }
        if (edge && (x1 < 1 || x1 + 16 > L2 - 1)) {  // zero padding, and the composed layer's edge terms
            const int x = x1 + li;
            const bool out = x < 0 || x >= L2;
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[m][r] = out ? 0.f : v[m][r];
            // lane group g holds channels 4 (g & 1) .. + 3 of phase 2m + (g >> 1): groups 0, 1
            // h[:, 0] at column 0, groups 2, 3 h[:, L4 - 1] at column L2 - 1 (m-block 1)
            const float* cq = cp;
            asm volatile("" : "+s"(cq));
            const bool right = g >= 2;
            if (right ? x == L2 - 1 : x == 0) {
                const float* cv = cq + (right ? 8 + 4 * (g - 2) : 4 * g);
                float d = g == 0 ? cq[16] : (g == 2 ? cq[17] : 0.f);
#pragma unroll
                for (int r = 0; r < 4; ++r) d = fmaf(cv[r], right ? v[1][r] : v[0][r], d);
                *reinterpret_cast<float*>(lds + kCorrOff + 4 * g) = d;
            }
        }
        split_mb(v, h, l);
        const Blk w4 = to_block<1>(h, l);  // octets (2, 3, 0, 1)
        if (k >= 0) {  // chunk -1 feeds no later layer
            // the composed layer: h at q (shift 1), (q-1, 2|3 | q+1, 0|1); x at q
            // (shift 2), (q-1, 3), (q+1, 0) (lane groups 2, 3: zero weights)
            Blk O[4];
            O[0] = shr<1, 0xF>(w4, w4, pw4);
            O[1] = shr<2, 0x3>(w4, w4, pw4);
            O[2] = shr<2, 0xF>(r3, r3, pr3);
            O[3] = shr<3, 0x1>(G[0], r3, pr3);
            f32x4 ao{b5[0], b5[1], b5[2], b5[3]};
#pragma unroll
            for (int f = 0; f < 4; ++f)
#pragma unroll
                for (int pr = 0; pr < 3; ++pr) ao = mfma_h(a5[f][pr == 2], pr == 1 ? O[f].l : O[f].h, ao);
            const int xa = qa + 16 * k, x = xa + li;
            float o4[4] = {ao[0], ao[1], ao[2], ao[3]};
            if (edge && (xa <= 0 || xa + 16 >= L2)) {
                const f32x4 e = *reinterpret_cast<const f32x4*>(lds + kCorrOff);
                if (x == 0) o4[0] -= e[0] + e[1];
                if (x == L2 - 1) o4[3] -= e[2] + e[3];
            }
            if (g == 0 && x >= 0 && x < L2) {
                float4 o;
                o.x = tanh_fast(o4[0]);
                o.y = tanh_fast(o4[1]);
                o.z = tanh_fast(o4[2]);
                o.w = tanh_fast(o4[3]);
                *reinterpret_cast<float4*>(arow + 4 * (size_t)x) = o;
                flag_nonfinite4(o.x, o.y, o.z, o.w, rflag, reinterpret_cast<int*>(lds + kFlagOff));
            }
        }
        pr3 = r3;
        pl3 = l3;
        pw4 = w4;
    };
    const int last = nch + 2;
    // s = 3i + u: U2 chunk s - 1 goes to ring slot (u + 2) mod 3 from ub[u]
    // (loaded two steps earlier), chunk s + 1 is loaded into ub[(u + 2) mod 3];
    // chunk s - 3 sits in ring R slot u.
    auto step = [&](int s, auto jc, u32x4 (&cur)[2], u32x4 (&ahead)[2]) {
        constexpr int u = decltype(jc)::value;
        if (s <= last) {
            const int c = s - 1;
            fetch(min(c + 2, nch - 1), ahead);  // past the strip: the last chunk again (an L2 hit)
            if (c < nch) {
#pragma unroll
                for (int hh = 0; hh < 2; ++hh) {
                    const int col = qa + 6 + 16 * c + lr + 8 * hh;
                    const u32x4 zz{0u, 0u, 0u, 0u};
                    *reinterpret_cast<u32x4*>(lds + wadr[(u + 2) % 3][hh]) = col >= 0 && col < L2 ? cur[hh] : zz;
                }
            }
            const int k = s - 3;
            if (TR_DIAG != 2 && k >= -1 && k < nch) work(k, jc);
            step_barrier();
        }
    };
#pragma unroll 1
    for (int s = 0; s <= last; s += 3) {
        step(s, ic<0>{}, ub[0], ub[2]);
        step(s + 1, ic<1>{}, ub[1], ub[0]);
        step(s + 2, ic<2>{}, ub[2], ub[1]);
    }
}

__global__ __launch_bounds__(kWaves * 64, 2) void tailr_kernel(const unsigned char* __restrict__ U2, int L2, int nch,
                                                                const u32x4* __restrict__ W,
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
    int* const lflag = reinterpret_cast<int*>(lds + kFlagOff);
    if (threadIdx.x == 0) *lflag = 0;  // before the first audio store: the step barriers order it
    if (w == 0) front_role(lds, qa, L2, nch, edge, W, bias);
    else back_role(lds, qa, L2, nch, edge, W, bias, U2 + (size_t)b * L2 * 128, arow, rflag);
    if (rd.rw) {  // range policy "fallback": this strip's audio again in fp32 if it is not finite
        __syncthreads();
        if (*lflag)
            redo_frames(*rd.rw, rd.mel, rd.trans, L2 / 16, b, qa / 16, min(L2, qa + 16 * nch) / 16, arow,
                        reinterpret_cast<float*>(lds), kRedoBytes / 4);
    }
}

}  // namespace tr

const char* const kVocTailrKernelName =
    "tailr_kernel (ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv, register hand-off)";

int32_t launch_vocoder_tailr(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                             int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    if (B == 0 || L2 == 0) return M2_OK;
    static bool attr = false;
    if (!attr) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(tr::tailr_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, tr::kLdsBytes));
        attr = true;
    }
    // Strip length: about one round of four workgroups per CU (stage1 B = 32,
    // L2 = 8000: 32 strips of 16 chunks per utterance), at least 8 chunks
    // (each strip pays 3 steps of pipeline fill).
    const int chunks = cdiv(L2, 16);
    int nch = sw().tailr_nch;
    if (!nch) nch = std::max(8, cdiv(chunks, std::max(1, 4 * 256 / B)));
    hipLaunchKernelGGL(tr::tailr_kernel, dim3(cdiv(chunks, nch), B), dim3(tr::kWaves * 64), tr::kLdsBytes, st,
                       static_cast<const unsigned char*>(U2), L2, nch, W, bias, audio, rflag, dT, rd);
    M2_LAUNCHED("tailr_kernel");
    return M2_OK;
}

}  // namespace m2
