// Stage1 vocoder tail with three layers chained per wave (M2_TAILR=1): the
// six-layer form of vocoder_tailp.hip (tts_model.py:279-297: ConvT3 + leaky,
// ResBlock3, ConvT4 + leaky, ResBlock4 conv1, then ResBlock4 conv2 composed
// with output_conv + tanh), with its packed weights, slot tables, LDS ring
// format and per-chunk arithmetic - the same MFMA sequence per output, so the
// audio is bit-identical to it - on a different schedule.
//
// vocoder_tailp.hip gives each layer its own wave and advances all seven in
// lockstep, one workgroup barrier per 16-column chunk: every step waits for
// the slowest layer's LDS read -> MFMA -> epilogue -> LDS write chain and the
// barrier's skew ("Why the tail sits near 0.2").  Here a
// workgroup has two waves:
//   wave 0 (front): ConvT3, ResBlock3 conv1, conv2 (+ x) of chunk k in a row,
//     each layer reading the ring the previous one wrote a moment earlier
//     (the same wave: LDS operations complete in order, no barrier);
//   wave 1 (back): streams U2 into ring R0 (two chunks ahead), then ConvT4,
//     ResBlock4 conv1 and the composed output layer of chunk k - 1; tanh,
//     audio, non-finite flag.
// One s_barrier per step hands ring R3 (ResBlock3's output) and ring R0 from
// one wave to the other.  Six 3-chunk rings (36 KB, also the local redo's
// windows), four workgroups per CU: eight waves, each SIMD holding two
// independent three-layer chains.  A strip of nch chunks takes nch + 3 steps.
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

// Ring n (R0 = U2, R(l + 1) = output of layer l): 3 chunks = 48 columns of
// 32 rows x (hi, lo) f16, vocoder_tailp.hip's format (64-B hi rows, the lo
// plane kPlane bytes later, octet o of row r at 16 (o ^ ((r >> 1) & 3)):
// conflict-free fragment reads and epilogue writes).
constexpr int kRows = 48, kPlane = kRows * 64, kRing = 2 * kPlane;
constexpr int kRedoBytes = 6 * kRing;  // the rings; redo_frames' windows (3 frames at C = 128) reuse them
constexpr int kCorrOff = kRedoBytes, kFlagOff = kRedoBytes + 16, kLdsBytes = kRedoBytes + 32;
static_assert(4 * kLdsBytes <= 160 * 1024, "four workgroups per CU");

__device__ __forceinline__ unsigned ring_at(int n, int row, int oct) {
    return n * kRing + row * 64 + 16 * (oct ^ ((row >> 1) & 3));
}
// row of column c (-2 .. 15) of the chunk in ring slot j
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

// Layer L (0..4) of the six-layer form: both m-blocks, weights and biases in
// VGPRs for the strip, fragment / residual / store addresses per ring slot.
template <int L>
struct Layer {
    static constexpr int NKB = tp::nkb(L), NF = tp::nfrag(L);
    static constexpr bool RES = L == 2;  // ResBlock3 conv2: + x (ring R1, two columns ahead)
    u32x4 a[2][NKB][2];
    float bv[2][4];
    unsigned radr[NF][3], oadr[3], xadr[RES ? 3 : 1];
    u32x4 aid[RES ? 2 : 1];

    __device__ __forceinline__ void init(const u32x4* __restrict__ W, const float* __restrict__ bias) {
        const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
#pragma unroll
            for (int kb = 0; kb < NKB; ++kb)
                if (kb < tp::nkbm(L, m)) {
                    const int u = tp::unit0(L) + m * NKB + kb;
                    a[m][kb][0] = W[u * 128 + lane];
                    a[m][kb][1] = W[u * 128 + 64 + lane];
                }
#pragma unroll
            for (int r = 0; r < 4; ++r) bv[m][r] = bias[L * 32 + m * 16 + 4 * g + r];
        }
        // ring R(L) holds the previous layer's columns one ahead of this
        // layer's; the epilogue stores octet 2m + (g >> 1) (ConvT4: its
        // permuted m-blocks hold octets 1, 2 and 0, 3), hi or lo by g & 1
        const int obase = L == 3 ? 1 + (g >> 1) : (g >> 1);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                const tp::Slot sl = tp::fslot(L, f, g);
                radr[f][j] = ring_at(L, ring_row(j, li + sl.dq - 1), sl.oct);
            }
            oadr[j] = (g & 1) * kPlane + ring_at(L + 1, ring_row(j, li), obase);
            if constexpr (RES) xadr[j] = ring_at(L - 1, ring_row(j, li - 2), g);
        }
        if constexpr (RES) {  // identity A of m-block m: row li takes input row 16m + li = 8g + e
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                h8 v;
#pragma unroll
                for (int e = 0; e < 8; ++e) v[e] = (_Float16)(16 * m + li == 8 * g + e ? 1.f : 0.f);
                aid[m] = __builtin_bit_cast(u32x4, v);
            }
        }
    }

    // B fragments of chunk k (ring slot J); RES: x too (slot NF)
    struct Frags {
        u32x4 h[NF + RES], l[NF + RES];
    };
    template <int J>
    __device__ __forceinline__ Frags load(const unsigned char* lds) const {
        Frags F;
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            F.h[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J]);
            F.l[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J] + kPlane);
        }
        if constexpr (RES) {
            F.h[NF] = *reinterpret_cast<const u32x4*>(lds + xadr[J]);
            F.l[NF] = *reinterpret_cast<const u32x4*>(lds + xadr[J] + kPlane);
        }
        return F;
    }
    __device__ __forceinline__ void mma(const Frags& F, f32x4 (&acc)[2]) const {
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[m] = f32x4{bv[m][0], bv[m][1], bv[m][2], bv[m][3]};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    if (kb < tp::nkbm(L, m)) {
                        const int f = tp::frag(L, m, kb);
                        acc[m] = mfma_h(a[m][kb][pr == 2], pr == 1 ? F.l[f] : F.h[f], acc[m]);
                    }
        if constexpr (RES) {
#pragma unroll
            for (int m = 0; m < 2; ++m) acc[m] = mfma_h(aid[m], F.h[NF], acc[m]);
#pragma unroll
            for (int m = 0; m < 2; ++m) acc[m] = mfma_h(aid[m], F.l[NF], acc[m]);
        }
    }
    // the epilogue of chunk k (ring slot J): columns x0 .. x0 + 15 of this
    // layer's output into ring R(L + 1)
    template <int J>
    __device__ __forceinline__ void store(unsigned char* lds, const f32x4 (&acc)[2], int x0, int L2, bool edge,
                                          const float* cp) const {
        const int li = threadIdx.x & 15, g = (threadIdx.x & 63) >> 4;
        auto epilogue = [&](auto zc) {
            constexpr bool ZERO = decltype(zc)::value;
            float v[2][4];
#pragma unroll
            for (int m = 0; m < 2; ++m) {
#pragma unroll
                for (int r = 0; r < 4; ++r) v[m][r] = acc[m][r];
                if constexpr (!RES) leaky4(v[m]);
            }
            if constexpr (ZERO) {
                const int x = x0 + li;
                const bool out = x < 0 || x >= L2;
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[m][r] = out ? 0.f : v[m][r];
                if constexpr (L == 4) {
                    // the composed layer's edge terms (vocoder_tailp.hip layer 4):
                    // lane group g holds channels 4 (g & 1) .. + 3 of phase
                    // 2m + (g >> 1); groups 0, 1 h[:, 0] at column 0, groups 2,
                    // 3 h[:, L4 - 1] at column L2 - 1 (m-block 1)
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
            }
            constexpr unsigned MX = L == 3 ? 16u : 32u;
#pragma unroll
            for (int m = 0; m < 2; ++m) {
                unsigned h0, h1, l0, l1;
                split2u(v[m][0], v[m][1], h0, l0);
                split2u(v[m][2], v[m][3], h1, l1);
                const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
                const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
                *reinterpret_cast<u32x4*>(lds + (oadr[J] ^ (MX * m))) = u32x4{s0[0], s1[0], s0[1], s1[1]};
            }
        };
        constexpr int EW = L == 4 ? 1 : 0;  // layer 4 also for the chunks holding column 0 or L2 - 1
        if (edge && (x0 < EW || x0 + 16 > L2 - EW)) epilogue(std::true_type{});  // wave-uniform
        else epilogue(std::false_type{});
    }
};

// The composed ResBlock4-conv2 + output_conv layer (vocoder_tailp.hip
// outc_role): fragments 0, 1 on ring R5 (ResBlock4's intermediate, one column
// ahead), 2, 3 on ring R4 (ConvT4's output, two ahead).
struct Outc {
    u32x4 a[4][2];
    float bv[4];
    unsigned radr[4][3];

    __device__ __forceinline__ void init(const u32x4* __restrict__ W, const float* __restrict__ bias) {
        const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            a[f][0] = W[(tp::kOutcUnit0 + f) * 128 + lane];
            a[f][1] = W[(tp::kOutcUnit0 + f) * 128 + 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = bias[tp::kOutcBias + 4 * g + r];
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int f = 0; f < 4; ++f) {
                const tp::Slot sl = tp::outc_slot(f, g);
                radr[f][j] = f < 2 ? ring_at(5, ring_row(j, li + sl.dq - 1), sl.oct)
                                   : ring_at(4, ring_row(j, li + sl.dq - 2), sl.oct);
            }
    }

    struct Frags {
        u32x4 h[4], l[4];
    };
    template <int J>
    __device__ __forceinline__ Frags load(const unsigned char* lds) const {
        Frags F;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            F.h[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J]);
            F.l[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J] + kPlane);
        }
        return F;
    }
    __device__ __forceinline__ void mma(const Frags& F, f32x4& acc) const {
        acc = f32x4{bv[0], bv[1], bv[2], bv[3]};
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr) acc = mfma_h(a[f][pr == 2], pr == 1 ? F.l[f] : F.h[f], acc);
    }
    __device__ __forceinline__ void store(unsigned char* lds, const f32x4& acc, int x0, int L2, bool edge,
                                          float* __restrict__ arow, int* rflag) const {
        const int li = threadIdx.x & 15, g = (threadIdx.x & 63) >> 4;
        const int x = x0 + li;
        float v[4] = {acc[0], acc[1], acc[2], acc[3]};
        if (edge && (x0 <= 0 || x0 + 16 >= L2)) {  // wave-uniform
            const f32x4 e = *reinterpret_cast<const f32x4*>(lds + kCorrOff);
            if (x == 0) v[0] -= e[0] + e[1];
            if (x == L2 - 1) v[3] -= e[2] + e[3];
        }
        if (g == 0 && x >= 0 && x < L2) {
            float4 o;
            o.x = tanh_fast(v[0]);
            o.y = tanh_fast(v[1]);
            o.z = tanh_fast(v[2]);
            o.w = tanh_fast(v[3]);
            *reinterpret_cast<float4*>(arow + 4 * (size_t)x) = o;
            flag_nonfinite4(o.x, o.y, o.z, o.w, rflag, reinterpret_cast<int*>(lds + kFlagOff));
        }
    }
};

// U2 into ring R0: lane (r, pc) moves 16-B piece pc of the 128-B U2 rows of
// columns r and r + 8 of a chunk (pieces 0-3 hi octets, 4-7 lo); chunk c =
// columns qa + 6 + 16 c + [0, 16) (ConvT3's inputs), zero outside [0, L2).
// Step s = 3i + u stores chunk s - 1 into slot (u + 2) mod 3 from ub[u]
// (loaded two steps earlier) and loads chunk s + 1 into ub[(u + 2) mod 3]:
// no register a load in flight writes is ever copied.
struct Loader {
    const unsigned char* u2;
    int qa, L2, nch, lr, pc;
    unsigned wadr[3][2];
    u32x4 ub[3][2];

    __device__ __forceinline__ void fetch(int c, u32x4 (&buf)[2]) const {
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
            const int col = min(max(qa + 6 + 16 * c + lr + 8 * hh, 0), L2 - 1);
            buf[hh] = *reinterpret_cast<const u32x4*>(u2 + (size_t)col * 128 + pc * 16);
        }
    }
    __device__ __forceinline__ void init(const unsigned char* u2_, int qa_, int L2_, int nch_) {
        u2 = u2_;
        qa = qa_;
        L2 = L2_;
        nch = nch_;
        const int lane = threadIdx.x & 63;
        lr = lane >> 3;
        pc = lane & 7;
#pragma unroll
        for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int hh = 0; hh < 2; ++hh)
                wadr[j][hh] = (pc >> 2) * kPlane + ring_at(0, ring_row(j, lr + 8 * hh), pc & 3);
        fetch(-1, ub[0]);
        fetch(0, ub[1]);
    }
    template <int U>
    __device__ __forceinline__ void step(unsigned char* lds, int s) {
        const int c = s - 1;
        fetch(min(c + 2, nch - 1), ub[(U + 2) % 3]);  // past the strip: the last chunk again (an L2 hit)
        if (c < nch) {
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int col = qa + 6 + 16 * c + lr + 8 * hh;
                const u32x4 zz{0u, 0u, 0u, 0u};
                *reinterpret_cast<u32x4*>(lds + wadr[(U + 2) % 3][hh]) = col >= 0 && col < L2 ? ub[U][hh] : zz;
            }
        }
    }
};

// The step loop: step s = 3i + u (u compile-time, so every ring slot is a
// compile-time index), then the workgroup barrier; the last step is
// nch + kSkew + 1 (the composed layer's chunk nch - 1).
constexpr int kLast = 6;  // last step - nch
template <class Body>
__device__ __forceinline__ void run_steps(int nch, Body&& body) {
    const int last = nch + kLast;
    auto step = [&](int s, auto uc) {
        if (s <= last) {
            body(s, uc);
            step_barrier();
        }
    };
#pragma unroll 1
    for (int s = 0; s <= last; s += 3) {
        step(s, ic<0>{});
        step(s + 1, ic<1>{});
        step(s + 2, ic<2>{});
    }
}

// Skewed schedule: in step s each layer l works on its own chunk k_l (front:
// ConvT3 s - 2, conv1 s - 3, conv2 s - 4; back: ConvT4 s - 5, ResBlock4 conv1
// s - 6, the composed layer s - 7), whose inputs were all written in earlier
// steps, so a wave's three layers are independent within the step: all their
// fragment loads are issued first (before any store of the step: a ring slot
// a later layer still reads for its previous chunk's last columns may be
// rewritten in the same step, and LDS operations of one wave complete in
// order), then the three MFMA chains (six accumulators), then the epilogues.
// Layer l's chunk k starts at column qa + 5 - l + 16 k (the composed layer's
// at qa + 16 k); ring slot = k mod 3 = (u + 3 - offset mod 3) mod 3.
template <int OFF, int U>
using slot_of = ic<(U + 3 * 3 - OFF) % 3>;

__device__ __forceinline__ bool live(int k, int nch) { return k >= -1 && k < nch; }

// Wave 0: ConvT3 (chunk s - 2; its U2 columns stored by wave 1 in steps s - 2,
// s - 1), ResBlock3 conv1 (s - 3), conv2 (s - 4; ring R3 to wave 1).
__device__ __forceinline__ void front_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                           const u32x4* __restrict__ W, const float* __restrict__ bias) {
    Layer<0> l0;
    Layer<1> l1;
    Layer<2> l2;
    l0.init(W, bias);
    l1.init(W, bias);
    l2.init(W, bias);
    run_steps(nch, [&](int s, auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int j0 = slot_of<2, u>::value, j1 = slot_of<3, u>::value, j2 = slot_of<4, u>::value;
        const int k0 = s - 2, k1 = s - 3, k2 = s - 4;
        const bool a0 = live(k0, nch), a1 = live(k1, nch), a2 = live(k2, nch);
        if (a0 && a1 && a2) {  // the steady state: all three
            const auto F2 = l2.load<j2>(lds);
            const auto F1 = l1.load<j1>(lds);
            const auto F0 = l0.load<j0>(lds);
            f32x4 c0[2], c1[2], c2[2];
            l2.mma(F2, c2);
            l1.mma(F1, c1);
            l0.mma(F0, c0);
            l2.store<j2>(lds, c2, qa + 3 + 16 * k2, L2, edge, nullptr);
            l1.store<j1>(lds, c1, qa + 4 + 16 * k1, L2, edge, nullptr);
            l0.store<j0>(lds, c0, qa + 5 + 16 * k0, L2, edge, nullptr);
        } else {  // fill and drain: one layer at a time, loads before stores as above
            f32x4 c[2];
            const auto F2 = l2.load<j2>(lds);
            const auto F1 = l1.load<j1>(lds);
            const auto F0 = l0.load<j0>(lds);
            if (a2) {
                l2.mma(F2, c);
                l2.store<j2>(lds, c, qa + 3 + 16 * k2, L2, edge, nullptr);
            }
            if (a1) {
                l1.mma(F1, c);
                l1.store<j1>(lds, c, qa + 4 + 16 * k1, L2, edge, nullptr);
            }
            if (a0) {
                l0.mma(F0, c);
                l0.store<j0>(lds, c, qa + 5 + 16 * k0, L2, edge, nullptr);
            }
        }
    });
}

// Wave 1: the loader (U2 chunk s - 1), ConvT4 (chunk s - 5: ring R3's chunk
// written by wave 0 in step s - 1), ResBlock4 conv1 (s - 6), the composed
// layer (s - 7; chunk -1 feeds nothing).
__device__ __forceinline__ void back_role(unsigned char* lds, int qa, int L2, int nch, bool edge,
                                          const u32x4* __restrict__ W, const float* __restrict__ bias,
                                          const unsigned char* __restrict__ u2, float* __restrict__ arow,
                                          int* rflag) {
    Loader ld;
    ld.init(u2, qa, L2, nch);
    Layer<3> l3;
    Layer<4> l4;
    Outc oc;
    l3.init(W, bias);
    l4.init(W, bias);
    oc.init(W, bias);
    const float* cp = bias + tp::kOutcCorr;
    run_steps(nch, [&](int s, auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int j3 = slot_of<5, u>::value, j4 = slot_of<6, u>::value, j5 = slot_of<7, u>::value;
        const int k3 = s - 5, k4 = s - 6, k5 = s - 7;
        const bool a3 = live(k3, nch), a4 = live(k4, nch), a5 = k5 >= 0 && k5 < nch;
        // all loads of the step first (the composed layer's x reads ring R4's
        // slot ConvT4 rewrites in this step), then the loader's store
        const auto F5 = oc.load<j5>(lds);
        const auto F4 = l4.load<j4>(lds);
        const auto F3 = l3.load<j3>(lds);
        ld.template step<u>(lds, s);
        if (a3 && a4 && a5) {
            f32x4 c3[2], c4[2], c5;
            oc.mma(F5, c5);
            l4.mma(F4, c4);
            l3.mma(F3, c3);
            // ResBlock4 conv1 before the composed layer's epilogue: its edge terms
            oc.store(lds, c5, qa + 16 * k5, L2, edge, arow, rflag);
            l4.store<j4>(lds, c4, qa + 1 + 16 * k4, L2, edge, cp);
            l3.store<j3>(lds, c3, qa + 2 + 16 * k3, L2, edge, nullptr);
        } else {
            f32x4 c[2], c5;
            if (a5) {
                oc.mma(F5, c5);
                oc.store(lds, c5, qa + 16 * k5, L2, edge, arow, rflag);
            }
            if (a4) {
                l4.mma(F4, c);
                l4.store<j4>(lds, c, qa + 1 + 16 * k4, L2, edge, cp);
            }
            if (a3) {
                l3.mma(F3, c);
                l3.store<j3>(lds, c, qa + 2 + 16 * k3, L2, edge, nullptr);
            }
        }
    });
}

__global__ __launch_bounds__(128, 2) void tailr_kernel(const unsigned char* __restrict__ U2, int L2, int nch,
                                                        const u32x4* __restrict__ W, const float* __restrict__ bias,
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
    "tailr_kernel (ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv, skewed layers per wave)";

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
    // (each strip pays 7 steps of pipeline fill and drain).
    const int chunks = cdiv(L2, 16);
    int nch = sw().tailr_nch;
    if (!nch) nch = std::max(8, cdiv(chunks, std::max(1, 4 * 256 / B)));
    hipLaunchKernelGGL(tr::tailr_kernel, dim3(cdiv(chunks, nch), B), dim3(128), tr::kLdsBytes, st,
                       static_cast<const unsigned char*>(U2), L2, nch, W, bias, audio, rflag, dT, rd);
    M2_LAUNCHED("tailr_kernel");
    return M2_OK;
}

}  // namespace m2
