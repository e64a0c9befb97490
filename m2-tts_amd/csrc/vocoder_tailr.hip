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

    // chunk k (ring slot J): columns x0 .. x0 + 15 of this layer's output
    template <int J>
    __device__ __forceinline__ void work(unsigned char* lds, int x0, int L2, bool edge, const float* cp) const {
        const int li = threadIdx.x & 15, g = (threadIdx.x & 63) >> 4;
        u32x4 bh[NF], bl[NF];
#pragma unroll
        for (int f = 0; f < NF; ++f) {
            bh[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J]);
            bl[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J] + kPlane);
        }
        u32x4 xh, xl;
        if constexpr (RES) {
            xh = *reinterpret_cast<const u32x4*>(lds + xadr[J]);
            xl = *reinterpret_cast<const u32x4*>(lds + xadr[J] + kPlane);
        }
        f32x4 acc[2];
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
                        acc[m] = mfma_h(a[m][kb][pr == 2], pr == 1 ? bl[f] : bh[f], acc[m]);
                    }
        if constexpr (RES) {
#pragma unroll
            for (int m = 0; m < 2; ++m) acc[m] = mfma_h(aid[m], xh, acc[m]);
#pragma unroll
            for (int m = 0; m < 2; ++m) acc[m] = mfma_h(aid[m], xl, acc[m]);
        }
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

    template <int J>
    __device__ __forceinline__ void work(unsigned char* lds, int x0, int L2, bool edge, float* __restrict__ arow,
                                         int* rflag) const {
        const int li = threadIdx.x & 15, g = (threadIdx.x & 63) >> 4;
        u32x4 bh[4], bl[4];
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            bh[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J]);
            bl[f] = *reinterpret_cast<const u32x4*>(lds + radr[f][J] + kPlane);
        }
        f32x4 acc = f32x4{bv[0], bv[1], bv[2], bv[3]};
#pragma unroll
        for (int f = 0; f < 4; ++f)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr) acc = mfma_h(a[f][pr == 2], pr == 1 ? bl[f] : bh[f], acc);
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

// The step loop of role R of NW: step s = 3i + u computes chunk k = s - 2 - R
// (ring slot k mod 3 = (u + 1 - R) mod 3, a compile-time index), then the
// workgroup barrier; body(s, k, ic<u>, ic<slot>) with k in [-1, nch) or -2
// (nothing to compute).  The last role's chunk nch - 1 is done in step
// nch + NW - 1 + ... = nch + NW.
template <int R, int NW, class Body>
__device__ __forceinline__ void run_steps(int nch, Body&& body) {
    const int last = nch + NW;
    auto step = [&](int s, auto uc) {
        constexpr int u = decltype(uc)::value;
        if (s <= last) {
            int k = s - 2 - R;
            if (k < -1 || k >= nch) k = -2;
            body(s, k, uc, ic<(u + 4 - R) % 3>{});
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

// NW = 2.  Wave 0: ConvT3, ResBlock3 conv1, conv2 (+ x) of chunk s - 2 (its U2
// columns stored by wave 1 in steps s - 2 and s - 1).  Wave 1: the loader,
// ConvT4, ResBlock4 conv1 and the composed layer of chunk s - 3 (ring R3's
// chunk written by wave 0 in step s - 1).
// NW = 3.  Wave 0: ConvT3, conv1 (chunk s - 2); wave 1: conv2, ConvT4 (chunk
// s - 3; rings R1 / R2 from wave 0); wave 2: the loader, ResBlock4 conv1 and
// the composed layer (chunk s - 4; ring R4 from wave 1).  Layer l's chunk k
// starts at column qa + 5 - l + 16 k.
template <int NW>
__device__ __forceinline__ void role(int w, unsigned char* lds, int qa, int L2, int nch, bool edge,
                                     const u32x4* __restrict__ W, const float* __restrict__ bias,
                                     const unsigned char* __restrict__ u2, float* __restrict__ arow, int* rflag) {
    const float* cp = bias + tp::kOutcCorr;
    if (w == 0) {
        Layer<0> l0;
        Layer<1> l1;
        l0.init(W, bias);
        l1.init(W, bias);
        if constexpr (NW == 2) {
            Layer<2> l2;
            l2.init(W, bias);
            run_steps<0, NW>(nch, [&](int, int k, auto, auto jc) {
                constexpr int j = decltype(jc)::value;
                if (k == -2) return;
                l0.template work<j>(lds, qa + 5 + 16 * k, L2, edge, nullptr);
                l1.template work<j>(lds, qa + 4 + 16 * k, L2, edge, nullptr);
                l2.template work<j>(lds, qa + 3 + 16 * k, L2, edge, nullptr);
            });
        } else {
            run_steps<0, NW>(nch, [&](int, int k, auto, auto jc) {
                constexpr int j = decltype(jc)::value;
                if (k == -2) return;
                l0.template work<j>(lds, qa + 5 + 16 * k, L2, edge, nullptr);
                l1.template work<j>(lds, qa + 4 + 16 * k, L2, edge, nullptr);
            });
        }
    } else if (NW == 3 && w == 1) {
        Layer<2> l2;
        Layer<3> l3;
        l2.init(W, bias);
        l3.init(W, bias);
        run_steps<1, NW>(nch, [&](int, int k, auto, auto jc) {
            constexpr int j = decltype(jc)::value;
            if (k == -2) return;
            l2.template work<j>(lds, qa + 3 + 16 * k, L2, edge, nullptr);
            l3.template work<j>(lds, qa + 2 + 16 * k, L2, edge, nullptr);
        });
    } else {
        Loader ld;
        ld.init(u2, qa, L2, nch);
        Layer<4> l4;
        Outc oc;
        l4.init(W, bias);
        oc.init(W, bias);
        if constexpr (NW == 2) {
            Layer<3> l3;
            l3.init(W, bias);
            run_steps<1, NW>(nch, [&](int s, int k, auto uc, auto jc) {
                constexpr int u = decltype(uc)::value, j = decltype(jc)::value;
                ld.template step<u>(lds, s);
                if (k == -2) return;
                l3.template work<j>(lds, qa + 2 + 16 * k, L2, edge, nullptr);
                l4.template work<j>(lds, qa + 1 + 16 * k, L2, edge, cp);
                if (k >= 0) oc.template work<j>(lds, qa + 16 * k, L2, edge, arow, rflag);  // chunk -1 feeds nothing
            });
        } else {
            run_steps<2, NW>(nch, [&](int s, int k, auto uc, auto jc) {
                constexpr int u = decltype(uc)::value, j = decltype(jc)::value;
                ld.template step<u>(lds, s);
                if (k == -2) return;
                l4.template work<j>(lds, qa + 1 + 16 * k, L2, edge, cp);
                if (k >= 0) oc.template work<j>(lds, qa + 16 * k, L2, edge, arow, rflag);
            });
        }
    }
}

template <int NW>
__global__ __launch_bounds__(NW * 64, NW == 2 ? 2 : 3) void tailr_kernel(const unsigned char* __restrict__ U2, int L2,
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
    int* const lflag = reinterpret_cast<int*>(lds + kFlagOff);
    if (threadIdx.x == 0) *lflag = 0;  // before the first audio store: the step barriers order it
    role<NW>(w, lds, qa, L2, nch, edge, W, bias, U2 + (size_t)b * L2 * 128, arow, rflag);
    if (rd.rw) {  // range policy "fallback": this strip's audio again in fp32 if it is not finite
        __syncthreads();
        if (*lflag)
            redo_frames(*rd.rw, rd.mel, rd.trans, L2 / 16, b, qa / 16, min(L2, qa + 16 * nch) / 16, arow,
                        reinterpret_cast<float*>(lds), kRedoBytes / 4);
    }
}

template <int NW>
static int32_t launch(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio, int* rflag,
                      hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    static bool attr = false;
    if (!attr) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(tailr_kernel<NW>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
        attr = true;
    }
    // Strip length: about one round of four workgroups per CU (stage1 B = 32,
    // L2 = 8000: 32 strips of 16 chunks per utterance), at least 8 chunks
    // (each strip pays NW + 1 steps of pipeline fill).
    const int chunks = cdiv(L2, 16);
    int nch = sw().tailr_nch;
    if (!nch) nch = std::max(8, cdiv(chunks, std::max(1, 4 * 256 / B)));
    hipLaunchKernelGGL(tailr_kernel<NW>, dim3(cdiv(chunks, nch), B), dim3(NW * 64), kLdsBytes, st,
                       static_cast<const unsigned char*>(U2), L2, nch, W, bias, audio, rflag, dT, rd);
    M2_LAUNCHED("tailr_kernel");
    return M2_OK;
}

}  // namespace tr

const char* const kVocTailrKernelName =
    "tailr_kernel (ConvT3 + ResBlock3 + ConvT4 + ResBlock4 + output_conv, layers chained per wave)";

int32_t launch_vocoder_tailr(const void* U2, int L2, int B, const vx_u32x4* W, const float* bias, float* audio,
                             int* rflag, hipStream_t st, const int32_t* dT, const VocRedo& rd) {
    if (B == 0 || L2 == 0) return M2_OK;
    return sw().tailr == 3 ? tr::launch<3>(U2, L2, B, W, bias, audio, rflag, st, dT, rd)
                           : tr::launch<2>(U2, L2, B, W, bias, audio, rflag, st, dT, rd);
}

}  // namespace m2
