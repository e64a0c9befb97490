// One launch per pre-LN transformer layer (gfx950, split-f16 MFMA
// v_mfma_f32_16x16x32_f16).
//
// layer_kernel computes, for a tile of 16 rows (queries) of ONE utterance:
//   att = softmax(Q K^T * scale [+ -1e9 key mask]) V      both heads   (components.py:59-90)
//   o   = x + att . Wo^T + bo                                           (components.py:86, 136-137)
//   y   = o + W2 . relu(W1 . LN2(o) + b1) + b2                          (components.py:98-103, 139-140)
// and then, on the same tile, the next launch's row-local work: the next
// layer's LN1 -> QKV projection (components.py:55-56, 135), written straight
// into the attention layouts below, or the decoder's final LN -> mel
// projection (tts_model.py:225-228).  A stack of L layers is L + 1 launches
// (the first LN1 -> QKV builds its own input rows: first_kernel), where the
// three-launch form (ln_gemm / attention / post_attn, transformer_fused.hip)
// needs 2L + 1, and the attention no longer re-splits K and V per query
// block: the producing epilogue writes them as f16 hi/lo once.
//
// Attention layouts (TflBufs, one set per layer, ping-pong between layers),
// all in MFMA-fragment order: a 1-KB fragment holds the 16 B of each of the 64
// lanes of one v_mfma_f32_16x16x32_f16 operand, lane-contiguous, so every
// operand load of the consumer is one 1-KB contiguous wave read (a load of 16
// rows x 64 B - the row-major form - ran at 34 GB/s per CU against 82 GB/s
// contiguous from L2, tools/probe/l2bw.hip):
//   Q, K  [B*heads][npad/16 row blocks][KS k-steps][hi|lo][lane][8 f16]
//         [KT tail steps][hi|lo][lane < 32][8 f16]: lane (row li, group g) of
//         k-step ks holds dims 32 ks + 8 g .. + 7 of row 16 blk + li (the
//         operands of v_mfma_f32_16x16x32_f16); a head_dim that is an odd
//         multiple of 16 (48, 16) ends in a 16-dim tail step stored for lane
//         groups 0, 1 only (512 B per plane): the lanes of groups 2, 3 take
//         zeros from an out-of-range buffer offset, so no zero padding is
//         stored or read (the MFMAs still run K = 32: a K = 16 MFMA chained
//         with K = 32 ones on one accumulator gave wrong scores, the hazard
//         DESIGN.md notes in round 2); Q pre-scaled by scale * log2(e)
//         when the attention is unmasked (the score is then the raw dot
//         product, base 2);
//   V^T   [B*heads][npad/32 chunks][hd/16 blocks][hi|lo][lane][8 f16]: lane
//         (dim 16 t + li, group g) holds the chunk's keys at positions
//         8 g .. + 7, keys in the order the P^T fragment of the PV MFMA holds
//         them (key 16 u + 4 g + e at position 8 g + 4 u + e).
// K fragments are the A operand of S^T = K . Q^T (16 keys x 32 dims), Q
// fragments its B operand, V^T fragments the A operand of O^T += V^T . P^T.
// These are L2-resident reads (the previous launch wrote them); rows past N
// are zeros (the producing tiles write them).
//
// Workgroup = 8 waves, 16 rows of one utterance; the tiles of an utterance
// get workgroup ids on one XCD (workgroup L runs on XCD L % 8) so its K / V
// stay in that XCD's L2.  Attention: wave w = (head w / 4, key quarter w % 4)
// takes the 32-key chunks c = w % 4 (mod 4) with its own online-softmax state
// (the lazy rescaling of attention_split_kernel when unmasked); the four
// quarters merge through LDS.  GEMMs: wave w computes the 16-column blocks
// w, w + 8, ... as D^T = W . X^T (A = packed weights, B = split LDS rows), or
// as D = X . W^T for the V columns, whose lanes then hold 4 consecutive keys
// of one V^T row.  Arithmetic: every fp32 product as hi*hi + hi*lo + lo*hi
// on f16 halves, LayerNorms / softmax / residuals in fp32.
#include <cmath>
#include <cstdlib>

#include "m2_common.h"
#include "transformer_layer.h"
#include "vocoder_fused.h"  // split2u, vmax, vx_u32x4

namespace m2 {
namespace tfl {

// Diagnostic build only (-DTFL_STAMPS, tools/probe/tfl_stamps.py): per-wave
// s_memtime stamps at the phase boundaries of layer_kernel,
// [workgroup][wave][16]; slots 14 / 15 = s_memrealtime (100 MHz) at start / end.
#ifdef TFL_STAMPS
__device__ unsigned long long g_tfl_stamps[4096][8][16];
#define TSTAMP(i)                                                                                          \
    do {                                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        unsigned long long _t;                                                                             \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                        \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) g_tfl_stamps[blockIdx.x][threadIdx.x >> 6][i] = _t; \
    } while (0)
#define TSTAMP_RT(i)                                                                                       \
    do {                                                                                                   \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        unsigned long long _t;                                                                             \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
        __builtin_amdgcn_sched_barrier(0);                                                                 \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096) g_tfl_stamps[blockIdx.x][threadIdx.x >> 6][i] = _t; \
    } while (0)
#else
#define TSTAMP(i) \
    do {          \
    } while (0)
#define TSTAMP_RT(i) \
    do {             \
    } while (0)
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef vx_u32x4 u32x4;

// Diagnostic builds only (-DTFL_DIAG=bits, tools/runs): attention_qsplit2's
// lean path without 1 its global K / V loads after step 2, 2 its softmax
// VALU, 4 its LDS stores, 8 its QK^T MFMAs, 16 its PV MFMAs - the
// per-step time each piece holds (results are garbage; never the product).
#ifndef TFL_DIAG
#define TFL_DIAG 0
#endif
#ifndef TFL_STAGE_FIRST  // A/B builds: 0 = a step's staging after its K fragment reads
#define TFL_STAGE_FIRST 1  // (0: decoder layers +4.5 % at B=128 T=2600, profiles/r04/r04i_stage_order.txt)
#endif
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLazyT = 8.f;  // unmasked lazy rescale: weights stay <= 2^kLazyT
constexpr int TQ = 16;         // rows (queries) per workgroup
constexpr int NW = 8;          // waves per workgroup
constexpr int KC = 32;         // keys per chunk
constexpr int HEADS = 2;
constexpr int WPH = NW / HEADS;  // waves per head (key quarters)

__device__ __forceinline__ f32x4 mfma(u32x4 a, u32x4 b, f32x4 c) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}
// Byte offset of this lane's tail-step piece in a block (lane groups 0, 1),
// or one past any buffer record for groups 2, 3 (a raw buffer load there
// returns zeros).
__device__ __forceinline__ int tail_off(int lane) { return lane < 32 ? 16 * lane : 0x40000000; }

template <int HD>
struct Geo {
    static constexpr int KS = HD / 32, KT = (HD % 32) / 16, MT = HD / 16;
    static constexpr int KSA = KS > 0 ? KS : 1;  // array extent
    static constexpr int TAIL = KS * 2048;       // byte offset of the tail step (hi 512 B | lo 512 B)
    static constexpr int QKBLK = KS * 2048 + KT * 1024;  // bytes of a 16-row Q / K block
    static constexpr int VCH = MT * 2048;    // bytes of a V^T chunk (MT d-blocks x hi|lo x 1 KB)
    static constexpr int XW = 2 + 4 * MT;    // merge record per lane (m, lsum, acc)
};

constexpr int srs(int K) { return 4 * K + 32; }  // split LDS row bytes (RS/16 = 2 mod 4: conflict-free b128 reads)
constexpr int frs(int K) { return K + 4; }       // fp32 LDS row floats

__device__ __forceinline__ float grp4_max(float x) {  // over the 4 lanes of one query (l, l^16, l^32, l^48)
    x = vmax(x, __shfl_xor(x, 16));
    return vmax(x, __shfl_xor(x, 32));
}

// An n-block's weight strip (pack_bfrag_split: [nb][ks][hi|lo][lane][8 f16]).
template <int K>
struct Strip {
    u32x4 w[K / 32][2];
    __device__ __forceinline__ void load(const u32x4* __restrict__ Wp, int nb) {
        const u32x4* p = Wp + (size_t)nb * (K / 32) * 128 + (threadIdx.x & 63);
#pragma unroll
        for (int ks = 0; ks < K / 32; ++ks) {
            w[ks][0] = p[ks * 128];
            w[ks][1] = p[ks * 128 + 64];
        }
    }
};

// D^T = W . X^T over RB 16-row blocks of the LDS rows X (split, stride
// srs(K)): acc[rb] lane (row rb*16 + (lane & 15)) holds columns 4 (lane >> 4)
// + r of the block; every weight fragment feeds the RB blocks.
template <int K, int RB>
__device__ __forceinline__ void gemm_t(const unsigned char* X, const Strip<K>& st, f32x4 (&acc)[RB]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
        u32x4 xh[RB], xl[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const unsigned char* p = X + (rb * 16 + i) * srs(K) + 2 * (32 * ks + 8 * g);
            xh[rb] = *reinterpret_cast<const u32x4*>(p);
            xl[rb] = *reinterpret_cast<const u32x4*>(p + 2 * K);
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma(st.w[ks][0], xh[rb], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma(st.w[ks][0], xl[rb], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma(st.w[ks][1], xh[rb], acc[rb]);
    }
}
// D = X . W^T: acc[rb] lane holds rows rb*16 + 4 (lane >> 4) + r of column lane & 15.
template <int K, int RB>
__device__ __forceinline__ void gemm_n(const unsigned char* X, const Strip<K>& st, f32x4 (&acc)[RB]) {
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < K / 32; ++ks) {
        u32x4 xh[RB], xl[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const unsigned char* p = X + (rb * 16 + i) * srs(K) + 2 * (32 * ks + 8 * g);
            xh[rb] = *reinterpret_cast<const u32x4*>(p);
            xl[rb] = *reinterpret_cast<const u32x4*>(p + 2 * K);
        }
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma(xh[rb], st.w[ks][0], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma(xl[rb], st.w[ks][0], acc[rb]);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = mfma(xh[rb], st.w[ks][1], acc[rb]);
    }
}

// Four consecutive fp32 values -> their hi and lo f16 at p, p + 2K.
template <int K>
__device__ __forceinline__ void put_split4(unsigned char* p, float a, float b, float c, float d) {
    unsigned h0, h1, l0, l1;
    split2u(a, b, h0, l0);
    split2u(c, d, h1, l1);
    *reinterpret_cast<uint2*>(p) = uint2{h0, h1};
    *reinterpret_cast<uint2*>(p + 2 * K) = uint2{l0, l1};
}

// LayerNorm (eps 1e-5, biased variance, affine) of R fp32 LDS rows src into
// split rows dst: 8 lanes per row, two-pass as nn.LayerNorm; g, b in LDS.
template <int H, int R, int NT = NW * 64>
__device__ __forceinline__ void ln_rows(const float* src, unsigned char* dst, const float* g, const float* b) {
    constexpr int PER = H / 8;
    static_assert(PER % 4 == 0, "H multiple of 32");
#pragma unroll 1
    for (int x = threadIdx.x; x < 8 * R; x += NT) {
        const int row = x >> 3, part = x & 7;
        const float* xr = src + row * frs(H) + part * PER;
        float v[PER];
#pragma unroll
        for (int q = 0; q < PER / 4; ++q) {
            const float4 t = *reinterpret_cast<const float4*>(xr + 4 * q);
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < PER; ++k) s += v[k];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        s += __shfl_xor(s, 4);
        const float mean = s / (float)H;
        float var = 0.f;
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const float d = v[k] - mean;
            var += d * d;
        }
        var += __shfl_xor(var, 1);
        var += __shfl_xor(var, 2);
        var += __shfl_xor(var, 4);
        const float rstd = 1.0f / sqrtf(var / (float)H + kLnEps);
        unsigned char* yr = dst + row * srs(H) + 2 * part * PER;
#pragma unroll
        for (int q = 0; q < PER / 4; ++q) {
            float y[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = part * PER + 4 * q + e;
                y[e] = (v[4 * q + e] - mean) * rstd * g[k] + b[k];
            }
            put_split4<H>(yr + 8 * q, y[0], y[1], y[2], y[3]);
        }
    }
}

// Where a QKV projection's columns go (the attention layouts above).
struct QkvOut {
    unsigned char *q, *k, *v;
    int npad, nch;
    float qs;  // Q scale: scale * log2(e) for unmasked attention, else 1
};

// Q / K column block nb (< 2H/16) of the 16 rows t0.. (D^T accumulator).
template <int H, int HD>
__device__ __forceinline__ void store_qk(const QkvOut& o, int b, int t0, int N, int nb, f32x4 acc) {
    using G = Geo<HD>;
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int which = nb / (H / 16), c0 = (nb - which * (H / 16)) * 16;
    const int h = c0 / HD, dh = c0 - h * HD, d0 = dh + 4 * g;
    const int t = t0 + i;
    const bool live = t < N;
    const float sc = which == 0 ? o.qs : 1.f;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = live ? acc[r] * sc : 0.f;
    unsigned h0, h1, l0, l1;
    split2u(v[0], v[1], h0, l0);
    split2u(v[2], v[3], h1, l1);
    // fragment order: dims d0 .. d0+3 of row t are half (d0 % 8) / 4 of lane
    // ((d0 % 32) / 8) * 16 + t % 16 in k-step d0 / 32 of row block t / 16
    unsigned char* blk = (which ? o.k : o.q) + ((size_t)(b * HEADS + h) * (o.npad / 16) + t / 16) * G::QKBLK;
    if (d0 < 32 * G::KS) {
        unsigned char* ph = blk + (d0 / 32) * 2048 + ((((d0 & 31) >> 3) * 16 + (t & 15)) * 16) + ((d0 & 7) >> 2) * 8;
        *reinterpret_cast<uint2*>(ph) = uint2{h0, h1};
        *reinterpret_cast<uint2*>(ph + 1024) = uint2{l0, l1};
    } else {  // tail step: lane ((d0 - 32 KS) / 8) * 16 + t % 16, half (d0 % 8) / 4
        unsigned char* ph = blk + G::TAIL + (((d0 - 32 * G::KS) >> 3) * 16 + (t & 15)) * 16 + ((d0 & 7) >> 2) * 8;
        *reinterpret_cast<uint2*>(ph) = uint2{h0, h1};
        *reinterpret_cast<uint2*>(ph + 512) = uint2{l0, l1};
    }
}

// V column block nb (>= 2H/16) of the 16 rows t0.. (D accumulator: rows
// t0 + 4g + r, column lane & 15).
template <int H, int HD>
__device__ __forceinline__ void store_v(const QkvOut& o, int b, int t0, int N, int nb, f32x4 acc) {
    using G = Geo<HD>;
    const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    const int c = (nb - 2 * (H / 16)) * 16 + i;
    const int h = c / HD, d = c - h * HD;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (t0 + 4 * g + r < N) ? acc[r] : 0.f;
    unsigned h0, h1, l0, l1;
    split2u(v[0], v[1], h0, l0);
    split2u(v[2], v[3], h1, l1);
    // keys 16u + 4g + e (u = row block within the chunk) -> positions 8g + 4u + e:
    // half u of lane g * 16 + d % 16 of d-block d / 16
    unsigned char* pc = o.v + ((size_t)(b * HEADS + h) * o.nch + (t0 >> 5)) * G::VCH + (d >> 4) * 2048 +
                        (g * 16 + (d & 15)) * 16 + ((t0 >> 4) & 1) * 8;
    *reinterpret_cast<uint2*>(pc) = uint2{h0, h1};
    *reinterpret_cast<uint2*>(pc + 1024) = uint2{l0, l1};
}

// The QKV projection of the tile's LN rows Xn (16 RB rows from t0) into the
// attention layouts.
template <int H, int HD, int RB, int NWV = NW>
__device__ __forceinline__ void qkv_phase(const unsigned char* Xn, const u32x4* __restrict__ W, Strip<H>& cur,
                                          const QkvOut& o, int b, int t0, int N) {
    constexpr int NB = 3 * H / 16, NQK = 2 * H / 16;
    const int wave = threadIdx.x >> 6;
#pragma unroll 1
    for (int nb = wave; nb < NB; nb += NWV) {
        Strip<H> nxt;
        if (nb + NWV < NB) nxt.load(W, nb + NWV);
        f32x4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (nb < NQK) {
            gemm_t<H, RB>(Xn, cur, acc);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) store_qk<H, HD>(o, b, t0 + 16 * rb, N, nb, acc[rb]);
        } else {
            gemm_n<H, RB>(Xn, cur, acc);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) store_v<H, HD>(o, b, t0 + 16 * rb, N, nb, acc[rb]);
        }
        if (nb + NWV < NB) cur = nxt;
    }
}

// The 16-row tiles' QKV projection with every strip of the wave requested
// beforehand (qkv_strips): no strip load on the chain between the blocks.
template <int H>
struct QkvStrips {
    static constexpr int NB = 3 * H / 16, NK = (NB + NW - 1) / NW;
    Strip<H> s[NK];
    __device__ __forceinline__ void load(const u32x4* __restrict__ W) {
        const int wave = threadIdx.x >> 6;
#pragma unroll
        for (int k = 0; k < NK; ++k)
            if (wave + NW * k < NB) s[k].load(W, wave + NW * k);
    }
};
template <int H, int HD, int RB = 1>
__device__ __forceinline__ void qkv_phase_pre(const unsigned char* Xn, const QkvStrips<H>& sq, const QkvOut& o, int b,
                                              int t0, int N) {
    constexpr int NQK = 2 * H / 16;
    const int wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < QkvStrips<H>::NK; ++k) {
        const int nb = wave + NW * k;
        if (nb < QkvStrips<H>::NB) {
            f32x4 acc[RB];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (nb < NQK) {
                gemm_t<H, RB>(Xn, sq.s[k], acc);
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) store_qk<H, HD>(o, b, t0 + 16 * rb, N, nb, acc[rb]);
            } else {
                gemm_n<H, RB>(Xn, sq.s[k], acc);
#pragma unroll
                for (int rb = 0; rb < RB; ++rb) store_v<H, HD>(o, b, t0 + 16 * rb, N, nb, acc[rb]);
            }
        }
    }
}

// A tile wholly past the utterance's end: its rows of the next attention
// buffers are zeros (no GEMM).
template <int H, int HD, int RB, int NWV = NW>
__device__ __forceinline__ void zero_tile(const QkvOut& o, int b, int t0) {
    constexpr int NB = 3 * H / 16, NQK = 2 * H / 16;
    const f32x4 z4 = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int nb = threadIdx.x >> 6; nb < NB; nb += NWV)
        for (int rb = 0; rb < RB; ++rb) {
            if (nb < NQK) store_qk<H, HD>(o, b, t0 + 16 * rb, 0, nb, z4);
            else store_v<H, HD>(o, b, t0 + 16 * rb, 0, nb, z4);
        }
}

// Utterance and tile of this workgroup (TflQueue): a claim on the queue of
// the XCD the workgroup runs on - utterance b's tiles are in queue b % 8 - or,
// when that queue is empty, on the next non-empty one.  The grid has exactly
// one workgroup per tile and every queue scan ends with an empty queue, so
// every tile is claimed once whatever the placement (XCD affinity only makes
// it fast: a layer's K / V stay in the L2 of the XCD that wrote them).
__device__ __forceinline__ void claim_tile(int B, int ntile, unsigned* __restrict__ cnt, unsigned seq, int* sh,
                                           int* b, int* tile) {
    if (threadIdx.x == 0) {
        unsigned x;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        x &= 7;
        unsigned* mine = cnt + (seq & 1) * 256;
        if (blockIdx.x == 0)  // the next launch's set (the previous launch's, done by stream order)
            for (int y = 0; y < 8; ++y)
                __hip_atomic_store(cnt + ((seq + 1) & 1) * 256 + y * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int got = -1;
        for (int k = 0; k < 8 && got < 0; ++k) {
            const int y = (x + k) & 7;
            const int n = (y < B ? (B - 1 - y) / 8 + 1 : 0) * ntile;
            if (n == 0) continue;
            const int i = (int)__hip_atomic_fetch_add(mine + y * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (i < n) got = (y + 8 * (i / ntile)) * ntile + (i - (i / ntile) * ntile);
        }
        *sh = got;
    }
    __syncthreads();
    // wave-uniform in an SGPR: every address derived from b (the K / V buffer
    // descriptors in particular) stays scalar - a VGPR-held b turns each buffer
    // load into a readfirstlane waterfall loop
    const int it = __builtin_amdgcn_readfirstlane(*sh);
    *b = __builtin_amdgcn_readfirstlane(it / ntile);
    *tile = __builtin_amdgcn_readfirstlane(it - (it / ntile) * ntile);
}

// ---------------------------------------------------------------------------
// Attention of the tile's 16 RB queries (RB 16-query blocks share every K / V
// fragment), both heads, over all N keys.  Leaves the normalised output rows
// as split LDS rows A [16 RB][srs(H)] (the out projection's B operand).  The
// caller's `between` runs after the chunk loop, before the merge (the first
// GEMM's weight strip is requested there).
template <int H, int HD, bool MASKED, int RB, typename Between>
__device__ __forceinline__ void attention_tile(const unsigned char* __restrict__ qb, const unsigned char* __restrict__ kb,
                                               const unsigned char* __restrict__ vb, int b, int t0, int N, int npad,
                                               int len, float sl2, unsigned char* A, float* xs, Between between) {
    using G = Geo<HD>;
    constexpr int KS = G::KS, KSA = G::KSA, KT = G::KT, MT = G::MT, QKBLK = G::QKBLK, VCH = G::VCH, XW = G::XW;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, g = lane >> 4;
    const int h = wave / WPH, kq = wave - h * WPH;
    const int nch = npad / KC, nchl = (N + KC - 1) / KC;  // layout chunks, chunks holding live keys
    const size_t bh = (size_t)__builtin_amdgcn_readfirstlane(b * HEADS + h);

    // B = Q^T fragments: lane (query li of block qt, dims 32 ks + 8 g .. + 7)
    u32x4 qh[RB][KSA], ql[RB][KSA], qxh[RB], qxl[RB];
#pragma unroll
    for (int qt = 0; qt < RB; ++qt) {
        const unsigned char* qp = qb + (bh * (npad / 16) + t0 / 16 + qt) * QKBLK + 16 * lane;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            qh[qt][ks] = *reinterpret_cast<const u32x4*>(qp + 2048 * ks);
            ql[qt][ks] = *reinterpret_cast<const u32x4*>(qp + 2048 * ks + 1024);
        }
        if constexpr (KT) {
            const u32x4 z = u32x4{0u, 0u, 0u, 0u};
            qxh[qt] = lane < 32 ? *reinterpret_cast<const u32x4*>(qp + G::TAIL) : z;
            qxl[qt] = lane < 32 ? *reinterpret_cast<const u32x4*>(qp + G::TAIL + 512) : z;
        }
    }
    // Chunk c's K fragments and V^T fragments through a buffer descriptor whose
    // record count is 0 past the last chunk: the prefetch of a chunk that does
    // not exist is issued unconditionally (no branch around a load, so the
    // compiler's vmcnt waits stay graded) and reads zeros without traffic.
    const int loff = 16 * lane, toff = tail_off(lane);
    struct Frag {
        u32x4 kh[2][KSA], kl[2][KSA], kxh[2], kxl[2], vh[MT], vl[MT];
    };
    auto load = [&](Frag& f, int c) {
        const bool ok = c < nchl;
        const auto rk = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<unsigned char*>(kb) + (bh * (npad / 16) + (size_t)(ok ? c : 0) * 2) * QKBLK, 0,
            ok ? 2 * QKBLK : 0, 0x00020000);
        const auto rv = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<unsigned char*>(vb) + (bh * nch + (ok ? c : 0)) * VCH, 0, ok ? VCH : 0, 0x00020000);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                f.kh[u][ks] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, loff + u * QKBLK + 2048 * ks, 0, 0));
                f.kl[u][ks] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, loff + u * QKBLK + 2048 * ks + 1024, 0, 0));
            }
        if constexpr (KT)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f.kxh[u] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, toff, u * QKBLK + G::TAIL, 0));
                f.kxl[u] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, toff, u * QKBLK + G::TAIL + 512, 0));
            }
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            f.vh[t] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, loff + t * 2048, 0, 0));
            f.vl[t] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, loff + t * 2048 + 1024, 0, 0));
        }
    };

    f32x4 acc[RB][MT];
    float m[RB], lsum[RB];
#pragma unroll
    for (int qt = 0; qt < RB; ++qt) {
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        m[qt] = MASKED ? -INFINITY : 0.f;
        lsum[qt] = 0.f;
    }
    bool fresh = true;  // unmasked: no chunk processed yet (wave-uniform)

    auto process = [&](const Frag& f, int c) {
        float s[RB][2][4];  // key 32 c + 16 u + 4 g + r of query li of block qt (base-2 score)
#pragma unroll
        for (int qt = 0; qt < RB; ++qt) {
            const float nm = (MASKED || fresh) ? 0.f : -m[qt];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                f32x4 st = f32x4{nm, nm, nm, nm};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    st = mfma(f.kh[u][ks], qh[qt][ks], st);
                    st = mfma(f.kh[u][ks], ql[qt][ks], st);
                    st = mfma(f.kl[u][ks], qh[qt][ks], st);
                }
                if constexpr (KT) {
                    st = mfma(f.kxh[u], qxh[qt], st);
                    st = mfma(f.kxh[u], qxl[qt], st);
                    st = mfma(f.kxl[u], qxh[qt], st);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) s[qt][u][r] = st[r];
            }
        }
        const int k0 = c * KC;
        if constexpr (MASKED) {
            // scores * scale, masked keys exactly the -1e9 fill, keys past N -inf
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = k0 + 16 * u + 4 * g + r;
#pragma unroll
                    for (int qt = 0; qt < RB; ++qt)
                        s[qt][u][r] = key < len ? s[qt][u][r] * sl2 : (key < N ? kMaskFill * kLog2e : -INFINITY);
                }
        } else if (N - k0 < KC) {  // the last chunk: keys past N score -inf (wave-uniform)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int qt = 0; qt < RB; ++qt)
                        s[qt][u][r] = k0 + 16 * u + 4 * g + r < N ? s[qt][u][r] : -INFINITY;
        }
        float cmax[RB];
#pragma unroll
        for (int qt = 0; qt < RB; ++qt)
            cmax[qt] = fmaxf(fmaxf(fmaxf(s[qt][0][0], s[qt][0][1]), fmaxf(s[qt][0][2], s[qt][0][3])),
                             fmaxf(fmaxf(s[qt][1][0], s[qt][1][1]), fmaxf(s[qt][1][2], s[qt][1][3])));
        if constexpr (MASKED) {
#pragma unroll
            for (int qt = 0; qt < RB; ++qt) {
                const float mn = vmax(m[qt], grp4_max(cmax[qt]));
                const float corr = __builtin_amdgcn_exp2f(m[qt] - mn);  // m = -inf on the first chunk -> 0
                lsum[qt] *= corr;
#pragma unroll
                for (int t = 0; t < MT; ++t) acc[qt][t] *= corr;
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[qt][u][r] -= mn;
                m[qt] = mn;
            }
        } else {
            bool up = fresh;
#pragma unroll
            for (int qt = 0; qt < RB; ++qt) up = up || cmax[qt] > kLazyT;
            if (__builtin_amdgcn_ballot_w64(up) != 0) {  // wave-uniform: move the base
#pragma unroll
                for (int qt = 0; qt < RB; ++qt) {
                    const float cm = grp4_max(cmax[qt]);  // finite: every chunk has a live key
                    const float d = fresh ? cm : vmax(cm, 0.f);
                    m[qt] += d;
                    if (!fresh) {
                        const float corr = __builtin_amdgcn_exp2f(-d);
                        lsum[qt] *= corr;
#pragma unroll
                        for (int t = 0; t < MT; ++t) acc[qt][t] *= corr;
                    }
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[qt][u][r] -= d;
                }
            }
            fresh = false;
        }
        u32x4 bh4[RB], bl4[RB];
#pragma unroll
        for (int qt = 0; qt < RB; ++qt) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    s[qt][u][r] = __builtin_amdgcn_exp2f(s[qt][u][r]);
                    lsum[qt] += s[qt][u][r];
                }
            // B = P^T: lane (query li) holds keys 4g + e (u = 0) and 16 + 4g + e (u = 1)
            unsigned ph[4], pl[4];
            split2u(s[qt][0][0], s[qt][0][1], ph[0], pl[0]);
            split2u(s[qt][0][2], s[qt][0][3], ph[1], pl[1]);
            split2u(s[qt][1][0], s[qt][1][1], ph[2], pl[2]);
            split2u(s[qt][1][2], s[qt][1][3], ph[3], pl[3]);
            bh4[qt] = u32x4{ph[0], ph[1], ph[2], ph[3]};
            bl4[qt] = u32x4{pl[0], pl[1], pl[2], pl[3]};
        }
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int qt = 0; qt < RB; ++qt) {
                acc[qt][t] = mfma(f.vh[t], bh4[qt], acc[qt][t]);
                acc[qt][t] = mfma(f.vh[t], bl4[qt], acc[qt][t]);
                acc[qt][t] = mfma(f.vl[t], bh4[qt], acc[qt][t]);
            }
    };

    // chunks kq, kq + 4, ... through a two-slot register ring.  The scheduling
    // barriers keep each slot's loads in program order (slot 0 before slot 1),
    // so the wait at the top of an iteration is for the older slot only.  (A
    // three-slot ring for the 16-row tiles measured slower: B=8 decoder
    // attention 12.2k -> 18.6k cycles, profiles/r05/r05ae_*.)
    const int nj = kq < nchl ? (nchl - kq + WPH - 1) / WPH : 0;
    Frag f0, f1;
    load(f0, kq);
    __builtin_amdgcn_sched_barrier(0);
    load(f1, kq + WPH);
    __builtin_amdgcn_sched_barrier(0);
    // (The head-1 waves, the younger of each SIMD pair, finish their
    // quarters ~4k cycles after the head-0 waves at B=8 T=500 - phase stamps,
    // profiles/r06/r06at_stamps.txt - and the merge waits for them; the two
    // waves of a SIMD taking the issue priority in turn, one chunk each,
    // measured level: r06au_*.)
#pragma unroll 1
    for (int j = 0; j < nj; j += 2) {
        process(f0, kq + WPH * j);
        __builtin_amdgcn_sched_barrier(0);
        load(f0, kq + WPH * (j + 2));
        __builtin_amdgcn_sched_barrier(0);
        if (j + 1 < nj) process(f1, kq + WPH * (j + 1));  // wave-uniform
        __builtin_amdgcn_sched_barrier(0);
        load(f1, kq + WPH * (j + 3));
        __builtin_amdgcn_sched_barrier(0);
    }
    TSTAMP(1);
    between();

    // merge the four key quarters of each head through LDS
    if (!MASKED && fresh) {  // this wave processed no chunk
#pragma unroll
        for (int qt = 0; qt < RB; ++qt) m[qt] = -INFINITY;
    }
#pragma unroll
    for (int qt = 0; qt < RB; ++qt) {
        float* xw = xs + ((wave * RB + qt) * 64 + lane) * XW;
        xw[0] = m[qt];
        xw[1] = lsum[qt];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) xw[2 + 4 * t + r] = acc[qt][t][r];
    }
    __syncthreads();
    if (kq < MT) {  // wave (h, j = kq): output dims 16 j .. 16 j + 15 of head h
        const int j = kq;
#pragma unroll
        for (int qt = 0; qt < RB; ++qt) {
            float mi[WPH], mx = -INFINITY;
#pragma unroll
            for (int q = 0; q < WPH; ++q) {
                mi[q] = xs[(((h * WPH + q) * RB + qt) * 64 + lane) * XW];
                mx = vmax(mx, mi[q]);
            }
            float ls = 0.f, o[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < WPH; ++q) {
                const float* xq = xs + (((h * WPH + q) * RB + qt) * 64 + lane) * XW;
                const float fq = __builtin_amdgcn_exp2f(mi[q] - mx);
                ls += xq[1] * fq;
#pragma unroll
                for (int r = 0; r < 4; ++r) o[r] += xq[2 + 4 * j + r] * fq;
            }
            ls += __shfl_xor(ls, 16);
            ls += __shfl_xor(ls, 32);
            const float inv = 1.0f / ls;
            put_split4<H>(A + (16 * qt + li) * srs(H) + 2 * (h * HD + 16 * j + 4 * g), o[0] * inv, o[1] * inv,
                          o[2] * inv, o[3] * inv);
        }
    }
    __syncthreads();
    TSTAMP(2);
}

// ---------------------------------------------------------------------------
// Attention of a 64-row tile for large grids: wave w = (head w / 4, query
// block w % 4) owns 16 queries of one head over ALL keys (its own online
// softmax, no merge), and the workgroup stages the K and V^T fragments of
// both heads in LDS once per 64 keys (two 32-key chunks: one 1-KB contiguous
// wave read per piece, 6 per thread for head_dim 48), shared by the four waves
// of a head.  The key-quarter form above reads every K / V byte from L2 once
// per 16 or 32 queries and is bound by the CU's L2 read rate (~37 B/clk,
// tools/probe/l2bw.hip); this one reads it once per 64 queries and then from
// LDS.  Per 64 keys: the QK^T MFMAs of both chunks (four independent
// accumulators), one softmax update, the PV MFMAs; two LDS buffers and one
// register set - keys 64 (p + 2) are in flight from L2 while p is computed and
// p + 1 goes to LDS; one barrier per 64 keys.  Leaves the normalised rows in A
// (split, stride srs(H)); `ring` is 2 * 2 chunks.
template <int HD>
struct QsGeo {
    using G = Geo<HD>;
    static constexpr int KB = 2 * G::QKBLK;      // one head's K of a chunk (two 16-key blocks)
    static constexpr int HB = KB + G::VCH;       // one head's K and V^T
    static constexpr int CB = 2 * HB;            // a chunk, both heads
    static constexpr int SB = 2 * CB;            // 64 keys
    static constexpr int PPT = SB / (16 * NW * 64);  // 16-B pieces per thread
    static_assert(CB % (16 * NW * 64) == 0, "chunk bytes a multiple of one 512-thread b128 round");
};

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// A raw buffer descriptor of a wave-uniform base address (the staging loads
// of the query-split attention: per-lane offset in a VGPR, step in an SGPR).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const unsigned char* base) {
    const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)base);
    const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)((uintptr_t)base >> 32));
    void* p = reinterpret_cast<void*>(((unsigned long long)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7ffffff0, 0x00020000);
}
// Lean unmasked softmax: true when a weight of the step exceeds 2^kLazyT,
// read from the f16 hi halves of P (8 packed words).  The weights are >= 0,
// so an f16 hi half orders as its bit pattern: packed u16 maxima compared with
// the bits of 2^kLazyT, which also catches +inf (0x7C00) and NaN (0x7Exx).
// (The earlier f16 form - packed f16 maxima converted to f32 and compared -
// missed a +inf hi half on gfx950: a weight past 65504, i.e. a later chunk's
// score more than 16 above the base, went unmoved and the output became NaN;
// tests/test_gpu_range.py::test_attention_scores_past_f16_range.)
__device__ __forceinline__ bool p_hi_exceeds(u32x4 a, u32x4 b) {
    typedef unsigned short u2 __attribute__((ext_vector_type(2)));
    auto h = [](unsigned w) { return __builtin_bit_cast(u2, w); };
    u2 mx = __builtin_elementwise_max(h(a[0]), h(a[1]));
    mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(h(a[2]), h(a[3])));
    mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(h(b[0]), h(b[1])));
    mx = __builtin_elementwise_max(mx, __builtin_elementwise_max(h(b[2]), h(b[3])));
    static_assert(kLazyT == 8.f, "the bit pattern below is f16 2^8");
    constexpr unsigned short lim = 0x5C00;  // f16 256.0
    return mx.x > lim || mx.y > lim;
}

// LEAN (M2_TFL_QS2=4): the lean softmax of attention_qsplit2 (C = -m
// accumulators when unmasked, row sums by MFMA on an all-ones fragment).
template <int H, int HD, bool MASKED, bool LEAN = false>
__device__ __forceinline__ void attention_qsplit(const unsigned char* __restrict__ qb, const unsigned char* __restrict__ kb,
                                                 const unsigned char* __restrict__ vb, int b, int t0, int N, int npad,
                                                 int len, float sl2, unsigned char* A, unsigned char* ring) {
    using G = Geo<HD>;
    using Q = QsGeo<HD>;
    constexpr int KS = G::KS, KSA = G::KSA, KT = G::KT, MT = G::MT, QKBLK = G::QKBLK, CB = Q::CB, SB = Q::SB;
    constexpr int PPT = Q::PPT;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, g = lane >> 4;
    const int h = wave / WPH, qblk = wave - h * WPH;
    const int nch = npad / KC, nsc = (N + 2 * KC - 1) / (2 * KC);  // layout chunks (even), 64-key steps

    // B = Q^T fragments of this wave's 16 queries
    u32x4 qh[KSA], ql[KSA], qxh, qxl;
    {
        const unsigned char* qp =
            qb + ((size_t)(b * HEADS + h) * (npad / 16) + t0 / 16 + qblk) * QKBLK + 16 * lane;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            qh[ks] = *reinterpret_cast<const u32x4*>(qp + 2048 * ks);
            ql[ks] = *reinterpret_cast<const u32x4*>(qp + 2048 * ks + 1024);
        }
        if constexpr (KT) {
            const u32x4 z = u32x4{0u, 0u, 0u, 0u};
            qxh = lane < 32 ? *reinterpret_cast<const u32x4*>(qp + G::TAIL) : z;
            qxl = lane < 32 ? *reinterpret_cast<const u32x4*>(qp + G::TAIL + 512) : z;
        }
    }
    // the global source of piece i (16 B) of 64-key step 0: [chunk][head][K blocks | V^T chunk],
    // through a buffer descriptor of its region (a wave's 1-KB piece lies in
    // one K or V^T region): per-lane offset fixed, the step's advance scalar
    __amdgpu_buffer_rsrc_t rsrc[PPT];
    int sstep[PPT];  // bytes from one 64-key step to the next for that piece
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int o = 16 * (tid + NW * 64 * i), j = o / CB, oc = o - j * CB, hh = oc / Q::HB, r = oc - hh * Q::HB;
        const size_t bh = (size_t)b * HEADS + hh;
        const bool isk = r < Q::KB;
        const unsigned char* base = isk ? kb + (bh * (npad / 16) + 2 * j) * QKBLK + (r & ~1023)
                                        : vb + (bh * nch + j) * G::VCH + ((r - Q::KB) & ~1023);
        rsrc[i] = wave_rsrc(base);
        sstep[i] = __builtin_amdgcn_readfirstlane(isk ? 4 * QKBLK : 2 * G::VCH);
    }
    u32x4 pre[PPT];
    auto gload = [&](int p) {
#pragma unroll
        for (int i = 0; i < PPT; ++i)
            pre[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc[i], 16 * lane, p * sstep[i], 0));
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < PPT; ++i) *reinterpret_cast<u32x4*>(ring + buf * SB + 16 * (tid + NW * 64 * i)) = pre[i];
    };

    f32x4 acc[MT], lacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = MASKED ? -INFINITY : 0.f, lsum = 0.f;
    bool fresh = true;
    const u32x4 ones = u32x4{0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u};  // f16 1.0 x 8

    // keys 64 p + 32 j + 16 u + 4 g + r, j = chunk of the step, u = 16-key block
    auto process = [&](const unsigned char* sb, int p) {
        float s[2][2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const unsigned char* kp = sb + j * CB + h * Q::HB + u * QKBLK + 16 * lane;
                const float c0 = (LEAN && !MASKED && !fresh) ? -m : 0.f;
                f32x4 st = f32x4{c0, c0, c0, c0};
#pragma unroll
                for (int ks = 0; ks < KS; ++ks) {
                    const u32x4 kh = *reinterpret_cast<const u32x4*>(kp + 2048 * ks);
                    const u32x4 kl = *reinterpret_cast<const u32x4*>(kp + 2048 * ks + 1024);
                    st = mfma(kh, qh[ks], st);
                    st = mfma(kh, ql[ks], st);
                    st = mfma(kl, qh[ks], st);
                }
                if constexpr (KT) {  // lanes of groups 2, 3 read other tail bytes: their Q operand is zero
                    const u32x4 kxh = *reinterpret_cast<const u32x4*>(kp + G::TAIL);
                    const u32x4 kxl = *reinterpret_cast<const u32x4*>(kp + G::TAIL + 512 - 512 * (lane >> 5));
                    st = mfma(kxh, qxh, st);
                    st = mfma(kxh, qxl, st);
                    st = mfma(kxl, qxh, st);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) s[j][u][r] = st[r];
            }
        const int k0 = p * 2 * KC;
        if constexpr (MASKED) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int key = k0 + 32 * j + 16 * u + 4 * g + r;
                        s[j][u][r] = key < len ? s[j][u][r] * sl2 : (key < N ? kMaskFill * kLog2e : -INFINITY);
                    }
        } else if (N - k0 < 2 * KC) {  // the last step: keys past N score -inf (wave-uniform)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        s[j][u][r] = k0 + 32 * j + 16 * u + 4 * g + r < N ? s[j][u][r] : -INFINITY;
        }
        auto step_max = [&]() {
            float c = s[0][0][0];
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) c = fmaxf(c, s[j][u][r]);
            return c;
        };
        if constexpr (LEAN && !MASKED) {
            // as attention_qsplit2's lean form: the base from the first step's
            // maximum, later moves detected on the f16 hi halves of P
            if (fresh) {  // wave-uniform
                const float cm = grp4_max(step_max());  // finite: the step's first chunk has a live key
                m = cm;
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[j][u][r] -= cm;
                fresh = false;
            }
            u32x4 bh4[2], bl4[2];
            auto exp_split = [&]() {
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    float e[2][4];
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) e[u][r] = __builtin_amdgcn_exp2f(s[j][u][r]);
                    unsigned ph[4], pl[4];
                    split2u(e[0][0], e[0][1], ph[0], pl[0]);
                    split2u(e[0][2], e[0][3], ph[1], pl[1]);
                    split2u(e[1][0], e[1][1], ph[2], pl[2]);
                    split2u(e[1][2], e[1][3], ph[3], pl[3]);
                    bh4[j] = u32x4{ph[0], ph[1], ph[2], ph[3]};
                    bl4[j] = u32x4{pl[0], pl[1], pl[2], pl[3]};
                }
            };
            exp_split();
            if (__builtin_amdgcn_ballot_w64(p_hi_exceeds(bh4[0], bh4[1])) != 0) {  // wave-uniform: move the base
                const float d = vmax(grp4_max(step_max()), 0.f);
                m += d;
                const float corr = __builtin_amdgcn_exp2f(-d);
                lacc *= corr;
#pragma unroll
                for (int t = 0; t < MT; ++t) acc[t] *= corr;
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[j][u][r] -= d;
                exp_split();
            }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                lacc = mfma(ones, bh4[j], lacc);
                lacc = mfma(ones, bl4[j], lacc);
                const unsigned char* vp = sb + j * CB + h * Q::HB + Q::KB + 16 * lane;
#pragma unroll
                for (int t = 0; t < MT; ++t) {
                    const u32x4 vh = *reinterpret_cast<const u32x4*>(vp + t * 2048);
                    const u32x4 vl = *reinterpret_cast<const u32x4*>(vp + t * 2048 + 1024);
                    acc[t] = mfma(vh, bh4[j], acc[t]);
                    acc[t] = mfma(vh, bl4[j], acc[t]);
                    acc[t] = mfma(vl, bh4[j], acc[t]);
                }
            }
            return;
        }
        const float cmax = step_max();
        if constexpr (MASKED) {
            const float mn = vmax(m, grp4_max(cmax));
            const float corr = __builtin_amdgcn_exp2f(m - mn);
            lsum *= corr;
            if constexpr (LEAN) lacc *= corr;
#pragma unroll
            for (int t = 0; t < MT; ++t) acc[t] *= corr;
            m = mn;
        } else if constexpr (LEAN) {
            // scores relative to the base already (attention_qsplit2's LEAN form)
            if (__builtin_amdgcn_ballot_w64(fresh || cmax > kLazyT) != 0) {
                const float cm = grp4_max(cmax);  // finite: the step's first chunk has a live key
                const float d = fresh ? cm : vmax(cm, 0.f);
                m += d;
                if (!fresh) {
                    const float corr = __builtin_amdgcn_exp2f(-d);
                    lacc *= corr;
#pragma unroll
                    for (int t = 0; t < MT; ++t) acc[t] *= corr;
                }
#pragma unroll
                for (int jj = 0; jj < 2; ++jj)
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[jj][u][r] -= d;
            }
            fresh = false;
        } else {
            // lazy base (attention_split_kernel): move it only on the first step or
            // when a score exceeds it by more than 2^kLazyT (wave-uniform)
            const float rel = cmax - m;
            if (__builtin_amdgcn_ballot_w64(fresh || rel > kLazyT) != 0) {
                const float cm = grp4_max(cmax);  // finite: the step's first chunk has a live key
                const float mn = fresh ? cm : vmax(cm, m);
                if (!fresh) {
                    const float corr = __builtin_amdgcn_exp2f(m - mn);
                    lsum *= corr;
#pragma unroll
                    for (int t = 0; t < MT; ++t) acc[t] *= corr;
                }
                m = mn;
            }
            fresh = false;
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (LEAN && !MASKED) {
                        s[j][u][r] = __builtin_amdgcn_exp2f(s[j][u][r]);
                    } else {
                        s[j][u][r] = __builtin_amdgcn_exp2f(s[j][u][r] - m);
                        if constexpr (!LEAN) lsum += s[j][u][r];
                    }
                }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            unsigned ph[4], pl[4];
            split2u(s[j][0][0], s[j][0][1], ph[0], pl[0]);
            split2u(s[j][0][2], s[j][0][3], ph[1], pl[1]);
            split2u(s[j][1][0], s[j][1][1], ph[2], pl[2]);
            split2u(s[j][1][2], s[j][1][3], ph[3], pl[3]);
            const u32x4 bh4 = u32x4{ph[0], ph[1], ph[2], ph[3]}, bl4 = u32x4{pl[0], pl[1], pl[2], pl[3]};
            if constexpr (LEAN) {
                lacc = mfma(ones, bh4, lacc);
                lacc = mfma(ones, bl4, lacc);
            }
            const unsigned char* vp = sb + j * CB + h * Q::HB + Q::KB + 16 * lane;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const u32x4 vh = *reinterpret_cast<const u32x4*>(vp + t * 2048);
                const u32x4 vl = *reinterpret_cast<const u32x4*>(vp + t * 2048 + 1024);
                acc[t] = mfma(vh, bh4, acc[t]);
                acc[t] = mfma(vh, bl4, acc[t]);
                acc[t] = mfma(vl, bh4, acc[t]);
            }
        }
    };

    gload(0);
    lstore(0);
    if (1 < nsc) gload(1);
    lds_barrier();
    // (Head 0's waves at a higher issue priority than the head-1 wave of the
    // same query block on their SIMD, so that one wave's MFMA phase could fall
    // on the other's softmax phase: no change at B=64 T=500, B=16 T=2600 or
    // stage1 B=32, in-process A/B, profiles/r03/ab/r03x_ab.txt.)
#pragma unroll 1
    for (int p = 0; p < nsc; ++p) {
        // step p from buffer p & 1; p + 1 goes to the other buffer, p + 2 is requested
        if (p + 1 < nsc) lstore((p + 1) & 1);
        if (p + 2 < nsc) gload(p + 2);
        process(ring + (p & 1) * SB, p);
        lds_barrier();
    }
    TSTAMP(1);
    if constexpr (LEAN) {
        lsum = lacc[0];  // complete over the keys already
    } else {
        lsum += __shfl_xor(lsum, 16);
        lsum += __shfl_xor(lsum, 32);
    }
    const float inv = 1.0f / lsum;
#pragma unroll
    for (int t = 0; t < MT; ++t)
        put_split4<H>(A + (16 * qblk + li) * srs(H) + 2 * (h * HD + 16 * t + 4 * g), acc[t][0] * inv, acc[t][1] * inv,
                      acc[t][2] * inv, acc[t][3] * inv);
}

// The same 64-row tile with each wave on TWO 16-query blocks and ONE 32-key
// chunk of every 64-key step: wave w = (head w / 4, query pair (w / 2) % 2,
// chunk w % 2).  Every K / V^T fragment a wave reads from LDS then feeds the
// MFMAs of both query blocks, so the workgroup reads half the LDS bytes per
// step of attention_qsplit (8 waves x one chunk instead of 8 waves x both
// chunks of its head); the MFMA count is the same.  Each wave keeps an online
// softmax per query block over its chunks; the two chunk waves of a (head,
// query pair) merge through LDS at the end (each finalises one block).  A
// chunk wholly past N is skipped (wave-uniform), so a wave may see no key:
// its record then carries m = -inf and weight 0.
template <int V>
struct CI {
    static constexpr int value = V;
};

// LEAN (M2_TFL_QS2=3): the softmax with fewer VALU instructions per step -
// unmasked, the QK^T MFMAs start from C = -m (scores arrive relative to the
// lazy base: no subtraction before exp2), and the row sums come from two more
// MFMAs on a constant all-ones A fragment (P_hi + P_lo summed by the matrix
// core, already complete over the chunk's keys) instead of 16 adds per step.
template <int H, int HD, bool MASKED, bool LEAN = false>
__device__ __forceinline__ void attention_qsplit2(const unsigned char* __restrict__ qb, const unsigned char* __restrict__ kb,
                                                  const unsigned char* __restrict__ vb, int b, int t0, int N, int npad,
                                                  int len, float sl2, unsigned char* A, unsigned char* ring) {
    using G = Geo<HD>;
    using Q = QsGeo<HD>;
    constexpr int KS = G::KS, KSA = G::KSA, KT = G::KT, MT = G::MT, QKBLK = G::QKBLK, CB = Q::CB, SB = Q::SB;
    constexpr int PPT = Q::PPT, RW = 2 + 4 * MT;  // merge record floats per lane
    static_assert(NW * RW * 64 * 4 <= 2 * SB, "merge records fit the ring");
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, g = lane >> 4;
    const int h = wave >> 2, qp = (wave >> 1) & 1, j = wave & 1;
    const int nch = npad / KC, nsc = (N + 2 * KC - 1) / (2 * KC);

    // B = Q^T fragments of this wave's two 16-query blocks 2 qp, 2 qp + 1
    u32x4 qh[2][KSA], ql[2][KSA], qxh[2], qxl[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
        const unsigned char* qp8 =
            qb + ((size_t)(b * HEADS + h) * (npad / 16) + t0 / 16 + 2 * qp + qq) * QKBLK + 16 * lane;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            qh[qq][ks] = *reinterpret_cast<const u32x4*>(qp8 + 2048 * ks);
            ql[qq][ks] = *reinterpret_cast<const u32x4*>(qp8 + 2048 * ks + 1024);
        }
        if constexpr (KT) {
            const u32x4 z = u32x4{0u, 0u, 0u, 0u};
            qxh[qq] = lane < 32 ? *reinterpret_cast<const u32x4*>(qp8 + G::TAIL) : z;
            qxl[qq] = lane < 32 ? *reinterpret_cast<const u32x4*>(qp8 + G::TAIL + 512) : z;
        }
    }
    // the staging of a 64-key step into LDS: as attention_qsplit, but every
    // piece through a buffer descriptor of its region (a wave's 1-KB piece
    // lies in one K or V^T region: the region bytes are multiples of 1 KB),
    // so a step's loads take the per-lane offset from a fixed VGPR and the
    // step's advance from an SGPR - no 64-bit address arithmetic per step
    __amdgpu_buffer_rsrc_t rsrc[PPT];
    int voff[PPT], sstep[PPT];
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
        const int o = 16 * (tid + NW * 64 * i), jj = o / CB, oc = o - jj * CB, hh = oc / Q::HB, r = oc - hh * Q::HB;
        const size_t bh = (size_t)b * HEADS + hh;
        const bool isk = r < Q::KB;
        const unsigned char* base = isk ? kb + (bh * (npad / 16) + 2 * jj) * QKBLK + (r & ~1023)
                                        : vb + (bh * nch + jj) * G::VCH + ((r - Q::KB) & ~1023);
        rsrc[i] = wave_rsrc(base);
        voff[i] = 16 * lane;
        sstep[i] = __builtin_amdgcn_readfirstlane(isk ? 4 * QKBLK : 2 * G::VCH);
    }
    u32x4 pre[PPT];
    auto gload = [&](int p) {
#pragma unroll
        for (int i = 0; i < PPT; ++i)
            pre[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc[i], voff[i], p * sstep[i], 0));
    };
    auto lstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < PPT; ++i) *reinterpret_cast<u32x4*>(ring + buf * SB + 16 * (tid + NW * 64 * i)) = pre[i];
    };

    f32x4 acc[2][MT], lacc[2];
    float m[2], lsum[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[qq][t] = f32x4{0.f, 0.f, 0.f, 0.f};
        m[qq] = MASKED ? -INFINITY : 0.f;
        lsum[qq] = 0.f;
        lacc[qq] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const u32x4 ones = u32x4{0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u};  // f16 1.0 x 8
    bool fresh = true;  // no chunk processed yet (wave-uniform)

    // keys 64 p + 32 j + 16 u + 4 g + r of query li of block qq
    // stage: the next steps' staging (LDS stores, global loads), issued
    // before this chunk's K fragment reads (TFL_STAGE_FIRST, the default) or
    // after them (measured slower)
    auto process = [&](const unsigned char* sb, int p, auto&& stage) {
        float s[2][2][4];
        u32x4 kf[2][KSA][2], kx[2][2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const unsigned char* kp = sb + j * CB + h * Q::HB + u * QKBLK + 16 * lane;
#pragma unroll
            for (int ks = 0; ks < KS * !(TFL_DIAG & 8); ++ks) {
                kf[u][ks][0] = *reinterpret_cast<const u32x4*>(kp + 2048 * ks);
                kf[u][ks][1] = *reinterpret_cast<const u32x4*>(kp + 2048 * ks + 1024);
            }
            if constexpr (KT && !(TFL_DIAG & 8)) {  // lanes of groups 2, 3 read other tail bytes: their Q operand is zero
                kx[u][0] = *reinterpret_cast<const u32x4*>(kp + G::TAIL);
                kx[u][1] = *reinterpret_cast<const u32x4*>(kp + G::TAIL + 512 - 512 * (lane >> 5));
            }
        }
        if constexpr (!TFL_STAGE_FIRST) stage();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x4 st[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            if constexpr (LEAN && !MASKED)
                if (!fresh)
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq) st[qq] = f32x4{-m[qq], -m[qq], -m[qq], -m[qq]};
#pragma unroll
            for (int ks = 0; ks < KS * !(TFL_DIAG & 8); ++ks) {
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    st[qq] = mfma(kf[u][ks][0], qh[qq][ks], st[qq]);
                    st[qq] = mfma(kf[u][ks][0], ql[qq][ks], st[qq]);
                    st[qq] = mfma(kf[u][ks][1], qh[qq][ks], st[qq]);
                }
            }
            if constexpr (KT && !(TFL_DIAG & 8)) {
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    st[qq] = mfma(kx[u][0], qxh[qq], st[qq]);
                    st[qq] = mfma(kx[u][0], qxl[qq], st[qq]);
                    st[qq] = mfma(kx[u][1], qxh[qq], st[qq]);
                }
            }
#pragma unroll
            for (int qq = 0; qq < 2; ++qq)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[qq][u][r] = st[qq][r];
        }
        const int k0 = p * 2 * KC + j * KC;
        if constexpr (MASKED) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int key = k0 + 16 * u + 4 * g + r;
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq)
                        s[qq][u][r] = key < len ? s[qq][u][r] * sl2 : (key < N ? kMaskFill * kLog2e : -INFINITY);
                }
        } else if (N - k0 < KC) {  // the chunk straddles N: keys past N score -inf (wave-uniform)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq)
                        s[qq][u][r] = k0 + 16 * u + 4 * g + r < N ? s[qq][u][r] : -INFINITY;
        }
        auto chunk_max = [&](int qq) {
            return fmaxf(fmaxf(fmaxf(s[qq][0][0], s[qq][0][1]), fmaxf(s[qq][0][2], s[qq][0][3])),
                         fmaxf(fmaxf(s[qq][1][0], s[qq][1][1]), fmaxf(s[qq][1][2], s[qq][1][3])));
        };
        if constexpr (LEAN && !MASKED) {
            // the scores arrive relative to the base.  First chunk: the base is
            // the chunk's maximum.  Later: the base moves only when some weight
            // exceeds 2^kLazyT, detected AFTER the exponentials on the f16 hi
            // halves of P (packed maxima: ~10 VALU in place of the ~23 of a
            // per-score maximum before them); then, rarely, the exponentials
            // are recomputed from the kept scores.
            if (fresh) {  // wave-uniform
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    const float cm = grp4_max(chunk_max(qq));  // finite: the chunk holds a key < N
                    m[qq] = cm;
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[qq][u][r] -= cm;
                }
                fresh = false;
            }
            u32x4 bh4[2], bl4[2];
            auto exp_split = [&]() {
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    float e[2][4];
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) e[u][r] = __builtin_amdgcn_exp2f(s[qq][u][r]);
                    unsigned ph[4], pl[4];
                    split2u(e[0][0], e[0][1], ph[0], pl[0]);
                    split2u(e[0][2], e[0][3], ph[1], pl[1]);
                    split2u(e[1][0], e[1][1], ph[2], pl[2]);
                    split2u(e[1][2], e[1][3], ph[3], pl[3]);
                    bh4[qq] = u32x4{ph[0], ph[1], ph[2], ph[3]};
                    bl4[qq] = u32x4{pl[0], pl[1], pl[2], pl[3]};
                }
            };
            if constexpr (TFL_DIAG & 2) {  // diagnostic: no softmax VALU (P = the scores' bits)
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    bh4[qq] = u32x4{__float_as_uint(s[qq][0][0]), __float_as_uint(s[qq][0][1]),
                                    __float_as_uint(s[qq][0][2]), __float_as_uint(s[qq][0][3])};
                    bl4[qq] = u32x4{__float_as_uint(s[qq][1][0]), __float_as_uint(s[qq][1][1]),
                                    __float_as_uint(s[qq][1][2]), __float_as_uint(s[qq][1][3])};
                }
            } else
                exp_split();
            if constexpr (!(TFL_DIAG & 2)) {
                if (__builtin_amdgcn_ballot_w64(p_hi_exceeds(bh4[0], bh4[1])) != 0) {  // wave-uniform: move the base
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq) {
                        const float d = vmax(grp4_max(chunk_max(qq)), 0.f);
                        m[qq] += d;
                        const float corr = __builtin_amdgcn_exp2f(-d);
                        lacc[qq] *= corr;
#pragma unroll
                        for (int t = 0; t < MT; ++t) acc[qq][t] *= corr;
#pragma unroll
                        for (int u = 0; u < 2; ++u)
#pragma unroll
                            for (int r = 0; r < 4; ++r) s[qq][u][r] -= d;
                    }
                    exp_split();
                }
            }
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                lacc[qq] = mfma(ones, bh4[qq], lacc[qq]);
                lacc[qq] = mfma(ones, bl4[qq], lacc[qq]);
            }
            const unsigned char* vp = sb + j * CB + h * Q::HB + Q::KB + 16 * lane;
#pragma unroll
            for (int t = 0; t < MT * !(TFL_DIAG & 16); ++t) {
                const u32x4 vh = *reinterpret_cast<const u32x4*>(vp + t * 2048);
                const u32x4 vl = *reinterpret_cast<const u32x4*>(vp + t * 2048 + 1024);
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    acc[qq][t] = mfma(vh, bh4[qq], acc[qq][t]);
                    acc[qq][t] = mfma(vh, bl4[qq], acc[qq][t]);
                    acc[qq][t] = mfma(vl, bh4[qq], acc[qq][t]);
                }
            }
            if constexpr ((TFL_DIAG & 16) != 0)  // keep P live
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) asm volatile("" ::"v"(bh4[qq]), "v"(bl4[qq]));
            return;
        }
        float cmax[2];
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) cmax[qq] = chunk_max(qq);
        if constexpr (MASKED) {
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const float mn = vmax(m[qq], grp4_max(cmax[qq]));  // finite: the chunk holds a key < N
                const float corr = __builtin_amdgcn_exp2f(m[qq] - mn);  // m = -inf on the first chunk -> 0
                lsum[qq] *= corr;
                if constexpr (LEAN) lacc[qq] *= corr;
#pragma unroll
                for (int t = 0; t < MT; ++t) acc[qq][t] *= corr;
                m[qq] = mn;
            }
        } else if constexpr (LEAN) {
            // scores relative to the base already: move it (and them) only on
            // the first chunk or when one exceeds it by more than 2^kLazyT
            bool up = fresh;
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) up = up || cmax[qq] > kLazyT;
            if (__builtin_amdgcn_ballot_w64(up) != 0) {
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    const float cm = grp4_max(cmax[qq]);  // finite: the chunk holds a key < N
                    const float d = fresh ? cm : vmax(cm, 0.f);
                    m[qq] += d;
                    if (!fresh) {
                        const float corr = __builtin_amdgcn_exp2f(-d);
                        lacc[qq] *= corr;
#pragma unroll
                        for (int t = 0; t < MT; ++t) acc[qq][t] *= corr;
                    }
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[qq][u][r] -= d;
                }
            }
        } else {
            // lazy base (attention_split_kernel): moved only on the first chunk or
            // when a score exceeds it by more than 2^kLazyT (wave-uniform)
            bool up = fresh;
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) up = up || cmax[qq] - m[qq] > kLazyT;
            if (__builtin_amdgcn_ballot_w64(up) != 0) {
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    const float cm = grp4_max(cmax[qq]);  // finite: the chunk holds a key < N
                    const float mn = fresh ? cm : vmax(cm, m[qq]);
                    if (!fresh) {
                        const float corr = __builtin_amdgcn_exp2f(m[qq] - mn);
                        lsum[qq] *= corr;
#pragma unroll
                        for (int t = 0; t < MT; ++t) acc[qq][t] *= corr;
                    }
                    m[qq] = mn;
                }
            }
        }
        fresh = false;
        u32x4 bh4[2], bl4[2];
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    if constexpr (LEAN && !MASKED) {
                        s[qq][u][r] = __builtin_amdgcn_exp2f(s[qq][u][r]);
                    } else {
                        s[qq][u][r] = __builtin_amdgcn_exp2f(s[qq][u][r] - m[qq]);
                        if constexpr (!LEAN) lsum[qq] += s[qq][u][r];
                    }
                }
            // B = P^T: lane (query li) holds keys 4g + e (u = 0) and 16 + 4g + e (u = 1)
            unsigned ph[4], pl[4];
            split2u(s[qq][0][0], s[qq][0][1], ph[0], pl[0]);
            split2u(s[qq][0][2], s[qq][0][3], ph[1], pl[1]);
            split2u(s[qq][1][0], s[qq][1][1], ph[2], pl[2]);
            split2u(s[qq][1][2], s[qq][1][3], ph[3], pl[3]);
            bh4[qq] = u32x4{ph[0], ph[1], ph[2], ph[3]};
            bl4[qq] = u32x4{pl[0], pl[1], pl[2], pl[3]};
        }
        if constexpr (LEAN)
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                lacc[qq] = mfma(ones, bh4[qq], lacc[qq]);
                lacc[qq] = mfma(ones, bl4[qq], lacc[qq]);
            }
        const unsigned char* vp = sb + j * CB + h * Q::HB + Q::KB + 16 * lane;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            const u32x4 vh = *reinterpret_cast<const u32x4*>(vp + t * 2048);
            const u32x4 vl = *reinterpret_cast<const u32x4*>(vp + t * 2048 + 1024);
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                acc[qq][t] = mfma(vh, bh4[qq], acc[qq][t]);
                acc[qq][t] = mfma(vh, bl4[qq], acc[qq][t]);
                acc[qq][t] = mfma(vl, bh4[qq], acc[qq][t]);
            }
        }
    };

    gload(0);
    lstore(0);
    if (1 < nsc) gload(1);
    lds_barrier();
#pragma unroll 1
    for (int p = 0; p < nsc; ++p) {
        // step p from buffer p & 1; p + 1 goes to the other buffer, p + 2 is requested
        auto stage = [&] {
            if (p + 1 < nsc) {
                if constexpr (!(TFL_DIAG & 4)) lstore((p + 1) & 1);
                else
#pragma unroll
                    for (int i = 0; i < PPT; ++i) asm volatile("" ::"v"(pre[i]));  // diagnostic: loads kept, no LDS stores
            }
            if (p + 2 < nsc && (!(TFL_DIAG & 1) || p < 2)) gload(p + 2);
        };
        const bool live = 2 * KC * p + KC * j < N;  // wave-uniform
        if (TFL_STAGE_FIRST || !live) stage();
        if (live) process(ring + (p & 1) * SB, p, stage);
        lds_barrier();
    }
    TSTAMP(1);
    if (fresh) {  // this wave saw no key
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) m[qq] = -INFINITY;
    }
    // merge the two chunk waves of (h, qp): wave j finalises block 2 qp + j and
    // hands its state of the other block to its partner (wave ^ 1).  The block
    // index is a compile-time constant in each branch (a runtime index into
    // the register arrays would move them to scratch or LDS).
    float* rec = reinterpret_cast<float*>(ring);
    auto put = [&](auto J) {
        constexpr int qo = 1 - decltype(J)::value;
        float* w = rec + (size_t)wave * RW * 64 + lane;
        w[0] = m[qo];
        w[64] = LEAN ? lacc[qo][0] : lsum[qo];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) w[(2 + 4 * t + r) * 64] = acc[qo][t][r];
    };
    auto fin = [&](auto J) {
        constexpr int qq = decltype(J)::value;
        const float* o = rec + (size_t)(wave ^ 1) * RW * 64 + lane;
        const float mo = o[0];
        const float mx = vmax(m[qq], mo);  // finite: chunk 0 of step 0 holds key 0 < N
        const float fm = __builtin_amdgcn_exp2f(m[qq] - mx), fo = __builtin_amdgcn_exp2f(mo - mx);
        float ls = (LEAN ? lacc[qq][0] : lsum[qq]) * fm + o[64] * fo;
        if constexpr (!LEAN) {  // lane-partial sums (keys 4g + r): add the four groups
            ls += __shfl_xor(ls, 16);
            ls += __shfl_xor(ls, 32);
        }
        const float inv = 1.0f / ls;
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = (acc[qq][t][r] * fm + o[(2 + 4 * t + r) * 64] * fo) * inv;
            put_split4<H>(A + (16 * (2 * qp + qq) + li) * srs(H) + 2 * (h * HD + 16 * t + 4 * g), v[0], v[1], v[2],
                          v[3]);
        }
    };
    if (j) put(CI<1>{});
    else put(CI<0>{});
    __syncthreads();
    if (j) fin(CI<1>{});
    else fin(CI<0>{});
}

// Key-quarter attention for 64-row tiles (M2_TFL_QS2=12; the default for
// unmasked layers).  Each wave owns four 16-query blocks of one head (every
// K / V^T fragment it holds feeds four blocks) and takes them through the lean
// softmax as two pairs (scores from C = -m, the base moved only when a
// weight's f16 hi half passes 2^kLazyT); all eight waves compute - two per
// SIMD, so one wave's softmax VALU meets the other's MFMAs.  Wave (h, kq)
// takes chunks kq, kq + 4, ... of head h (the key quarters of attention_tile)
// straight from L2 into registers by buffer loads: nothing in a chunk is
// shared between waves, so there is no staging, no ring and no barrier in the
// chunk loop.  One fragment set: chunk c's V^T is requested at the top of its
// iteration (first used by the first pair's PV), chunk c + 4's K right after
// the second pair's QK^T.  At head_dim 48 the 16-dim tail k-step is two MFMAs,
// not three: [k hi | k lo] . [q hi | q hi], then [k hi | (1, 1)] . [q lo | -m]
// - the second's lane group 2 carries the base, so the QK^T chain returns
// q.k - m from C = 0.  Row sums are per-lane fp32 sums of the exponentials,
// reduced over the query's four lane groups once, at the merge.  The four
// quarters of a head merge through LDS at the end, wave (h, kq) finalising
// block kq.
// Round 6, against the round-4/5 default (form 9: one computing wave per SIMD
// beside a staging wave that moved K / V into an LDS ring by LDS-DMA, one
// barrier per 64 keys; its computing wave's dependent chain per step was the
// bound, the MFMA pipe ~42 % busy): configs[4] step 8.67 -> 8.31 ms, B=16
// T=2600 -7.1 %, B=64 T=500 -2.6 %, decoder layers 1.35-1.44 -> 1.24-1.33 ms,
// MFMA busy 52 % (profiles/r06/r06ad_*, r06ae_pmc.txt); then the two-MFMA
// tail (three before: 92 -> 84 MFMAs per chunk; configs[4] step -1.4 %, B=16
// T=2600 -1.6 %, r06ai_*) and the VALU row sums (two MFMAs per block pair on
// an all-ones fragment before: 84 -> 76; layers 1,261 / 1,203 -> 1,241 /
// 1,179 us, step -2.0 %, r06aj_*, r06ak_*).  Measured and not kept: each wave
// moving its next chunk into a private LDS slot by LDS-DMA a whole iteration
// ahead (step 8.23 -> 8.54 ms, r06af_*); both pairs' QK^T before either
// softmax (+2.2 %), s_setprio 1 around each MFMA group (+0.7 %), both (+2.9 %;
// r06ag_*); a barrier of all eight waves every 1 / 2 / 4 / 8 chunks (+3.3 to
// +4.4 %, r06an_ab_lf.txt); the issue priority to whichever SIMD partner lags
// (each wave posting its chunk index in LDS: +0.6 % / +1.5 %, r06ap_*) - the
// older wave of each SIMD pair finishes its quarter ~11k cycles first
// (r06ao_stamps.txt), and neither evens that out for a gain.
template <int H, int HD, typename Between>
__device__ __forceinline__ void attention_quarters(const unsigned char* __restrict__ qb,
                                                   const unsigned char* __restrict__ kb,
                                                   const unsigned char* __restrict__ vb, int b, int t0, int N,
                                                   int npad, unsigned char* A, unsigned char* U,
                                                   Between between) {
    using G = Geo<HD>;
    constexpr int KS = G::KS, KSA = G::KSA, KT = G::KT, MT = G::MT, QKBLK = G::QKBLK, VCH = G::VCH, XW = G::XW;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, g = lane >> 4;
    const int h = wave / WPH, kq = wave - h * WPH;
    const int nch = npad / KC, nchl = (N + KC - 1) / KC;
    const size_t bh = (size_t)__builtin_amdgcn_readfirstlane(b * HEADS + h);

    u32x4 qh[4][KSA], ql[4][KSA], qxh[4], qxl[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
        const unsigned char* qp8 = qb + (bh * (npad / 16) + t0 / 16 + qq) * QKBLK + 16 * lane;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            qh[qq][ks] = *reinterpret_cast<const u32x4*>(qp8 + 2048 * ks);
            ql[qq][ks] = *reinterpret_cast<const u32x4*>(qp8 + 2048 * ks + 1024);
        }
        if constexpr (KT) {
            const u32x4 z = u32x4{0u, 0u, 0u, 0u};
            qxh[qq] = *reinterpret_cast<const u32x4*>(qp8 - 16 * lane + 16 * (lane & 31) + G::TAIL);  // both halves
            qxl[qq] = lane < 32 ? *reinterpret_cast<const u32x4*>(qp8 + G::TAIL + 512) : z;
        }
    }
    // chunk c's fragments through descriptors of its two K blocks / V^T chunk
    // (lane l reads 16 B at 16 l of each 1-KB piece: the layout the QKV
    // epilogues write)
    const int loff = 16 * lane, toff = tail_off(lane);
    u32x4 kf[2][KSA][2], kx[2][2], vf[MT][2];
    auto load_k = [&](int c) {
        const auto rk = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<unsigned char*>(kb) + (bh * (npad / 16) + (size_t)c * 2) * QKBLK, 0, 2 * QKBLK, 0x00020000);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                kf[u][ks][0] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, loff, u * QKBLK + 2048 * ks, 0));
                kf[u][ks][1] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, loff, u * QKBLK + 2048 * ks + 1024, 0));
            }
            if constexpr (KT) {
                kx[u][0] = __builtin_bit_cast(
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, loff, u * QKBLK + G::TAIL, 0));
                kx[u][1] = __builtin_bit_cast(  // hi | zeros
                    u32x4, __builtin_amdgcn_raw_buffer_load_b128(rk, toff, u * QKBLK + G::TAIL, 0));
            }
        }
    };
    auto load_v = [&](int c) {
        const auto rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(vb) + (bh * nch + c) * VCH, 0,
                                                          VCH, 0x00020000);
#pragma unroll
        for (int t = 0; t < MT; ++t) {
            vf[t][0] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, loff, t * 2048, 0));
            vf[t][1] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rv, loff, t * 2048 + 1024, 0));
        }
    };
    f32x4 acc[4][MT];
    float m[4] = {0.f, 0.f, 0.f, 0.f}, lsum[4] = {0.f, 0.f, 0.f, 0.f};  // lsum: per-lane partial row sums
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[qq][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    bool fresh = true;
    // QT (head_dim 48): the base rides in the tail's second MFMA, whose lane
    // groups 2, 3 carry no head dims (zeros loaded).  Lane group 2's first
    // two elements become A = (1, 1) (every key) and B = (hi, lo) of -m (its
    // query): the QK^T chain then delivers q.k - m itself, from C = 0 - no
    // per-step -m vector build.  The base is kept as the value those two f16
    // halves represent (hi + lo, exact in f32), so every use of m stays
    // consistent.
    constexpr bool QT = KT == 1 && KS >= 1;
    const bool g2 = (lane >> 4) == 2;
    auto set_base = [&](int qq, float mnew) {
        if constexpr (QT) {
            const _Float16 hi = (_Float16)(-mnew);
            const _Float16 lo = (_Float16)(-mnew - (float)hi);
            m[qq] = -((float)hi + (float)lo);
            const unsigned w = (unsigned)__builtin_bit_cast(unsigned short, hi) |
                               ((unsigned)__builtin_bit_cast(unsigned short, lo) << 16);
            if (g2) qxl[qq][0] = w;
        } else {
            m[qq] = mnew;
        }
    };
    auto c0 = [&](int qq) { return QT ? f32x4{0.f, 0.f, 0.f, 0.f} : f32x4{-m[qq], -m[qq], -m[qq], -m[qq]}; };

    // QK^T of blocks Q0, Q0 + 1 over the chunk in registers: s[qq][u][r] =
    // key 16 u + 4 g + r of query li of block Q0 + qq (base-2, minus the base)
    auto qk = [&](auto Q0c, float (&s)[2][2][4]) {
        constexpr int Q0 = decltype(Q0c)::value;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            f32x4 st[2] = {c0(Q0), c0(Q0 + 1)};
#pragma unroll
            for (int ks = 0; ks < KS; ++ks)
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    st[qq] = mfma(kf[u][ks][0], qh[Q0 + qq][ks], st[qq]);
                    st[qq] = mfma(kf[u][ks][0], ql[Q0 + qq][ks], st[qq]);
                    st[qq] = mfma(kf[u][ks][1], qh[Q0 + qq][ks], st[qq]);
                }
            if constexpr (KT)  // [k hi | k lo] . [q hi | q hi], then [k hi | (1, 1)] . [q lo | -m]
#pragma unroll
                for (int qq = 0; qq < 2; ++qq) {
                    st[qq] = mfma(kx[u][0], qxh[Q0 + qq], st[qq]);
                    st[qq] = mfma(kx[u][1], qxl[Q0 + qq], st[qq]);
                }
#pragma unroll
            for (int qq = 0; qq < 2; ++qq)
#pragma unroll
                for (int r = 0; r < 4; ++r) s[qq][u][r] = st[qq][r];
        }
    };
    // the lean softmax of blocks Q0, Q0 + 1 over chunk c and their PV
    auto smpv = [&](auto Q0c, int c, bool first, float (&s)[2][2][4]) {
        constexpr int Q0 = decltype(Q0c)::value;
        const int k0 = c * KC;
        if (N - k0 < KC) {  // the chunk straddles N (wave-uniform)
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int qq = 0; qq < 2; ++qq)
                        s[qq][u][r] = k0 + 16 * u + 4 * g + r < N ? s[qq][u][r] : -INFINITY;
        }
        auto chunk_max = [&](int qq) {
            return fmaxf(fmaxf(fmaxf(s[qq][0][0], s[qq][0][1]), fmaxf(s[qq][0][2], s[qq][0][3])),
                         fmaxf(fmaxf(s[qq][1][0], s[qq][1][1]), fmaxf(s[qq][1][2], s[qq][1][3])));
        };
        if (first) {  // the wave's first chunk: the base is its maximum (wave-uniform)
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                set_base(Q0 + qq, grp4_max(chunk_max(qq)));  // finite: the chunk holds a key < N
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[qq][u][r] -= m[Q0 + qq];
            }
        }
        u32x4 bh4[2], bl4[2];
        float esum[2];
        auto exp_split = [&]() {
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                float e[2][4];
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) e[u][r] = __builtin_amdgcn_exp2f(s[qq][u][r]);
                esum[qq] = ((e[0][0] + e[0][1]) + (e[0][2] + e[0][3])) + ((e[1][0] + e[1][1]) + (e[1][2] + e[1][3]));
                unsigned ph[4], pl[4];
                split2u(e[0][0], e[0][1], ph[0], pl[0]);
                split2u(e[0][2], e[0][3], ph[1], pl[1]);
                split2u(e[1][0], e[1][1], ph[2], pl[2]);
                split2u(e[1][2], e[1][3], ph[3], pl[3]);
                bh4[qq] = u32x4{ph[0], ph[1], ph[2], ph[3]};
                bl4[qq] = u32x4{pl[0], pl[1], pl[2], pl[3]};
            }
        };
        exp_split();
        if (__builtin_amdgcn_ballot_w64(p_hi_exceeds(bh4[0], bh4[1])) != 0) {  // rare: move the base
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                const float mold = m[Q0 + qq];
                set_base(Q0 + qq, mold + vmax(grp4_max(chunk_max(qq)), 0.f));
                const float d = m[Q0 + qq] - mold;
                const float corr = __builtin_amdgcn_exp2f(-d);
                lsum[Q0 + qq] *= corr;
#pragma unroll
                for (int t = 0; t < MT; ++t) acc[Q0 + qq][t] *= corr;
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[qq][u][r] -= d;
            }
            exp_split();
        }
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) lsum[Q0 + qq] += esum[qq];
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int qq = 0; qq < 2; ++qq) {
                acc[Q0 + qq][t] = mfma(vf[t][0], bh4[qq], acc[Q0 + qq][t]);
                acc[Q0 + qq][t] = mfma(vf[t][0], bl4[qq], acc[Q0 + qq][t]);
                acc[Q0 + qq][t] = mfma(vf[t][1], bh4[qq], acc[Q0 + qq][t]);
            }
    };

    const int nj = kq < nchl ? (nchl - kq + WPH - 1) / WPH : 0;  // this wave's chunks
    if (nj > 0) load_k(kq);
#pragma unroll 1
    for (int j = 0; j < nj; ++j) {
        const int c = kq + WPH * j;
        load_v(c);
        if constexpr (QT)  // lane group 2 of the second tail MFMA: A = (1, 1) (zeros loaded)
#pragma unroll
            for (int u = 0; u < 2; ++u) kx[u][1][0] |= g2 ? 0x3C003C00u : 0u;
        float s0[2][2][4], s2[2][2][4];
        qk(CI<0>{}, s0);
        smpv(CI<0>{}, c, fresh, s0);
        qk(CI<2>{}, s2);
        if (j + 1 < nj) load_k(c + WPH);  // wave-uniform: the K fragments are dead
        smpv(CI<2>{}, c, fresh, s2);
        fresh = false;
    }
    TSTAMP(1);
    if (fresh) {  // this wave saw no key
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) m[qq] = -INFINITY;
    }
    // merge: every wave leaves (m, row sum, acc) of its four blocks; wave
    // (h, kq) combines block kq over the head's four quarters
    float* rec = reinterpret_cast<float*>(U);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
        float* w = rec + (size_t)(wave * 4 + qq) * XW * 64 + lane;
        w[0] = m[qq];
        const float l = lsum[qq] + __shfl_xor(lsum[qq], 16);  // over the query's four lane groups
        w[64] = l + __shfl_xor(l, 32);
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) w[(2 + 4 * t + r) * 64] = acc[qq][t][r];
    }
    between();  // the caller's next loads, in flight across the merge
    __syncthreads();
    float mi[WPH], mx = -INFINITY;
#pragma unroll
    for (int q = 0; q < WPH; ++q) {
        mi[q] = rec[(size_t)((h * WPH + q) * 4 + kq) * XW * 64 + lane];
        mx = vmax(mx, mi[q]);  // finite: quarter 0 holds key 0 < N
    }
    float ls = 0.f, o[MT][4] = {};
#pragma unroll
    for (int q = 0; q < WPH; ++q) {
        const float* r0 = rec + (size_t)((h * WPH + q) * 4 + kq) * XW * 64 + lane;
        const float f = __builtin_amdgcn_exp2f(mi[q] - mx);
        ls += r0[64] * f;
#pragma unroll
        for (int t = 0; t < MT; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[t][r] += r0[(2 + 4 * t + r) * 64] * f;
    }
    const float inv = 1.0f / ls;
#pragma unroll
    for (int t = 0; t < MT; ++t)
        put_split4<H>(A + (16 * kq + li) * srs(H) + 2 * (h * HD + 16 * t + 4 * g), o[t][0] * inv, o[t][1] * inv,
                      o[t][2] * inv, o[t][3] * inv);
}

// ---------------------------------------------------------------------------
struct LArgs {
    int B, N, npad, ntile;
    const int32_t* dN;  // device frame count (dev_frames; N is then the capacity)
    unsigned* qcnt;
    unsigned qseq;
    float sl2;  // scale * log2(e)
    const int64_t* lengths;
    const float* x_in;
    float* x_out;
    const unsigned char *q, *k, *v;
    const u32x4 *Wo, *W1, *W2, *Wn;
    const float *bo, *g2, *b2n, *b1, *b2, *gn, *bn, *bn2;
    unsigned char *nq, *nk, *nv;
    float* z;
};

// RB = 1 (16-row tiles) while the grid fits one round of the CUs, else 2
// (32-row tiles: every K / V and weight fragment a workgroup reads serves
// twice the rows), 4 (64-row query-split tiles; QV picks the attention form).
#ifndef TFL_ONE  // A/B builds: 0 = the 16-row tiles compiled like the others
#define TFL_ONE 1
#endif
// 16-row tiles run only on grids of at most one workgroup per CU (tfl_rb):
// there they request every weight strip a phase ahead - both FFN1 strips of
// a wave before the attention merge, the FFN2 and QKV' strips before FFN1 -
// and the residual rows at the start (ONE; 232-236 VGPRs for H = 96, no
// scratch).  B=8 S=100 stage2, alternated twice: the six layer launches
// 78.2 -> 75.9 us; stage1 B=32 encoder layers 9.9 -> 9.0 and 7.7 -> 7.4 us
// (profiles/r05/r05af_*).
constexpr bool tfl_one(int rb) { return TFL_ONE && rb == 1; }
#ifndef TFL_PRE12  // A/B builds: 0 = form 12's tiles load each strip in the phase that uses it
#define TFL_PRE12 1
#endif
template <int H, bool MASKED, int NEXT, int NN, int RB, int QV = 1>
__global__ __launch_bounds__(512, 2) void layer_kernel(LArgs a) {
    static_assert(RB == 1 || RB == 2 || RB == 4, "16-, 32- or 64-row tiles");
    static_assert(QV != 12 || !MASKED, "the key-quarter form is unmasked-only");
    constexpr int HD = H / HEADS, F = 2 * H, TR = 16 * RB;
    constexpr bool ONE = tfl_one(RB);
    constexpr bool QS = RB == 4;                  // 64-row tiles: K / V staged in LDS
    // every weight strip requested a phase ahead (the registers are free once
    // the attention is done): the 16-row tiles, and form 12's 64-row tiles
    constexpr bool PRE = ONE || (TFL_PRE12 && QV == 12);
    __shared__ __attribute__((aligned(16))) unsigned char A[TR * srs(H)];   // att, then LN2(o), LN(y) (split)
    // the attention's scratch (key-quarter merge records / the K-V chunk ring)
    // and, after it, o / y (fp32, O) and relu(FFN1) (split, Hd)
    constexpr int OB = TR * frs(H) * 4, HB = TR * srs(F);
    constexpr int XB = QV == 12 ? NW * 4 * 64 * Geo<HD>::XW * 4  // form 12: merge records
                       : QS     ? 2 * QsGeo<HD>::SB
                                : NW * RB * 64 * Geo<HD>::XW * 4;
    __shared__ __attribute__((aligned(16))) unsigned char U[OB + HB > XB ? OB + HB : XB];
    float* const O = reinterpret_cast<float*>(U);
    unsigned char* const Hd = U + OB;
    float* const xs = reinterpret_cast<float*>(U);
    // the layer's vectors, read once into LDS (their L2 latency otherwise sits
    // in every LayerNorm and epilogue): bo | g2 | b2n | b1 [F] | b2 | gn | bn | bn2 [NN]
    constexpr int VO = 0, VG2 = H, VB2N = 2 * H, VB1 = 3 * H, VB2 = 3 * H + F, VGN = 4 * H + F, VBN = 5 * H + F,
                  VBN2 = 6 * H + F;
    __shared__ __attribute__((aligned(16))) float vec[6 * H + F + (NN > 0 ? NN : 4)];
    __shared__ int item;
    int b, tile;
    claim_tile(a.B, a.ntile, a.qcnt, a.qseq, &item, &b, &tile);
    const int t0 = tile * TR, N = a.dN ? dev_frames(a.dN, a.N) : a.N;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, gq = lane >> 4;
    const QkvOut qo{a.nq, a.nk, a.nv, a.npad, a.npad / KC, MASKED ? 1.f : a.sl2};
    if (t0 >= N) {
        if constexpr (NEXT == 1) zero_tile<H, HD, RB>(qo, b, t0);
        return;
    }
    for (int e = threadIdx.x; e < H; e += NW * 64) {
        vec[VO + e] = a.bo[e];
        vec[VG2 + e] = a.g2[e];
        vec[VB2N + e] = a.b2n[e];
        vec[VB2 + e] = a.b2[e];
        if constexpr (NEXT != 0) {
            vec[VGN + e] = a.gn[e];
            vec[VBN + e] = a.bn[e];
        }
    }
    for (int e = threadIdx.x; e < F; e += NW * 64) vec[VB1 + e] = a.b1[e];
    if constexpr (NEXT == 2)
        for (int e = threadIdx.x; e < NN; e += NW * 64) vec[VBN2 + e] = a.bn2[e];
    TSTAMP_RT(14);
    TSTAMP(0);
    int len = N;
    if constexpr (MASKED) len = (int)max((int64_t)0, min(a.lengths[b], (int64_t)N));  // mask[b, s] = s < lengths[b]
    Strip<H> so;
    Strip<H> s1, s1b;  // FFN1 strips (ONE: both of this wave's, requested before the merge)
    f32x4 xres = f32x4{0.f, 0.f, 0.f, 0.f};
    [[maybe_unused]] f32x4 xres4[RB];  // form 12: the residual rows, requested before the merge
    if constexpr (ONE) {  // the out projection's residual rows (here: measured 0.4 us better than beside Wo)
        if (wave < H / 16 && t0 + i < N)
            xres = *reinterpret_cast<const f32x4*>(a.x_in + ((size_t)b * N + t0 + i) * H + wave * 16 + 4 * gq);
    }
    if constexpr (QS) {
        if constexpr (QV == 12)
            attention_quarters<H, HD>(a.q, a.k, a.v, b, t0, N, a.npad, A, U, [&] {
                if (wave < F / 16) s1.load(a.W1, wave);  // both FFN1 strips of this wave
                if (wave + NW < F / 16) s1b.load(a.W1, wave + NW);
                if (wave < H / 16) {  // the out projection's strip and residual rows
                    so.load(a.Wo, wave);
#pragma unroll
                    for (int rb = 0; rb < RB; ++rb)
                        xres4[rb] = t0 + rb * 16 + i < N ? *reinterpret_cast<const f32x4*>(
                                                               a.x_in + ((size_t)b * N + t0 + rb * 16 + i) * H +
                                                               wave * 16 + 4 * gq)
                                                         : f32x4{0.f, 0.f, 0.f, 0.f};
                }
            });
        else if constexpr (QV == 3) attention_qsplit2<H, HD, MASKED, true>(a.q, a.k, a.v, b, t0, N, a.npad, len, a.sl2, A, U);
        else if constexpr (QV == 2) attention_qsplit2<H, HD, MASKED>(a.q, a.k, a.v, b, t0, N, a.npad, len, a.sl2, A, U);
        // (lean one-block form for the unmasked decoder only: masked, its MFMA
        // row sums moved the stage1 encoder's error at B=128 S=130 from under
        // to just over the tile tests' 2e-5 bound, for no measured gain)
        else if constexpr (QV == 4) attention_qsplit<H, HD, MASKED, !MASKED>(a.q, a.k, a.v, b, t0, N, a.npad, len, a.sl2, A, U);
        else attention_qsplit<H, HD, MASKED>(a.q, a.k, a.v, b, t0, N, a.npad, len, a.sl2, A, U);
        if (QV != 12 && wave < H / 16) so.load(a.Wo, wave);
        __syncthreads();
        TSTAMP(2);
    } else {
        attention_tile<H, HD, MASKED, RB>(a.q, a.k, a.v, b, t0, N, a.npad, len, a.sl2, A, xs, [&] {
            if (wave < H / 16) so.load(a.Wo, wave);
            if constexpr (ONE) {
                if (wave < F / 16) s1.load(a.W1, wave);
                if (wave + NW < F / 16) s1b.load(a.W1, wave + NW);
            }
        });
    }
    const size_t row0 = (size_t)b * N + t0;
    // o = x + att . Wo^T + bo
    if (wave < H / 16) {
        const int col = wave * 16 + 4 * gq;
        f32x4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = *reinterpret_cast<const f32x4*>(vec + VO + col);
        gemm_t<H, RB>(A, so, acc);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int rr = rb * 16 + i;
            f32x4 x = f32x4{0.f, 0.f, 0.f, 0.f};
            if constexpr (ONE) x = xres;
            else if constexpr (QV == 12) x = xres4[rb];
            else if (t0 + rr < N) x = *reinterpret_cast<const f32x4*>(a.x_in + (row0 + rr) * H + col);
            *reinterpret_cast<f32x4*>(O + rr * frs(H) + col) = x + acc[rb];
        }
    }
    Strip<F> s2;
    if constexpr (PRE) {
        if (wave < H / 16) s2.load(a.W2, wave);
    } else if (wave < F / 16) {
        s1.load(a.W1, wave);
    }
    __syncthreads();
    TSTAMP(3);
    ln_rows<H, TR>(O, A, vec + VG2, vec + VB2N);
    __syncthreads();
    TSTAMP(4);
    // h = relu(LN2(o) . W1^T + b1)
    auto ffn1 = [&](int nb, const Strip<H>& st) {
        const int col = nb * 16 + 4 * gq;
        f32x4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = *reinterpret_cast<const f32x4*>(vec + VB1 + col);
        gemm_t<H, RB>(A, st, acc);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
            put_split4<F>(Hd + (rb * 16 + i) * srs(F) + 2 * col, acc[rb][0] > 0.f ? acc[rb][0] : 0.f,
                          acc[rb][1] > 0.f ? acc[rb][1] : 0.f, acc[rb][2] > 0.f ? acc[rb][2] : 0.f,
                          acc[rb][3] > 0.f ? acc[rb][3] : 0.f);
    };
    // PRE: the QKV' strips of this wave, requested before FFN1 (the
    // final-projection strip for NEXT 2)
    QkvStrips<H> sq;
    if constexpr (PRE) {
        if constexpr (NEXT == 1) {
            sq.load(a.Wn);
        } else if constexpr (NEXT == 2) {
            if (wave < NN / 16) sq.s[0].load(a.Wn, wave);
        }
        static_assert(F / 16 <= 2 * NW, "two FFN1 blocks per wave at most");
        if (wave < F / 16) ffn1(wave, s1);
        if (wave + NW < F / 16) ffn1(wave + NW, s1b);
    } else {
#pragma unroll 1
        for (int nb = wave; nb < F / 16; nb += NW) {
            Strip<H> nxt;
            if (nb + NW < F / 16) nxt.load(a.W1, nb + NW);
            ffn1(nb, s1);
            if (nb + NW < F / 16) s1 = nxt;
        }
        if (wave < H / 16) s2.load(a.W2, wave);
    }
    __syncthreads();
    TSTAMP(5);
    // y = o + h . W2^T + b2
    if (wave < H / 16) {
        const int col = wave * 16 + 4 * gq;
        f32x4 acc[RB];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) acc[rb] = *reinterpret_cast<const f32x4*>(vec + VB2 + col);
        gemm_t<F, RB>(Hd, s2, acc);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
            const int rr = rb * 16 + i;
            const f32x4 y = *reinterpret_cast<const f32x4*>(O + rr * frs(H) + col) + acc[rb];
            if (t0 + rr < N) *reinterpret_cast<f32x4*>(a.x_out + (row0 + rr) * H + col) = y;
            if constexpr (NEXT != 0) *reinterpret_cast<f32x4*>(O + rr * frs(H) + col) = y;
        }
    }
    if constexpr (NEXT == 1) {
        Strip<H> sn;
        if (!PRE && wave < 3 * H / 16) sn.load(a.Wn, wave);
        __syncthreads();
        TSTAMP(6);
        ln_rows<H, TR>(O, A, vec + VGN, vec + VBN);
        __syncthreads();
        TSTAMP(7);
        if constexpr (PRE) {
            qkv_phase_pre<H, HD, RB>(A, sq, qo, b, t0, N);
        } else {
            qkv_phase<H, HD, RB>(A, a.Wn, sn, qo, b, t0, N);
        }
        TSTAMP(8);
        TSTAMP_RT(15);
    } else if constexpr (NEXT == 2) {
        Strip<H> sn;
        if constexpr (PRE) sn = sq.s[0];
        else if (wave < NN / 16) sn.load(a.Wn, wave);
        __syncthreads();
        TSTAMP(6);
        ln_rows<H, TR>(O, A, vec + VGN, vec + VBN);
        __syncthreads();
        TSTAMP(7);
#pragma unroll 1
        for (int nb = wave; nb < NN / 16; nb += NW) {
            Strip<H> nxt;
            if (nb + NW < NN / 16) nxt.load(a.Wn, nb + NW);
            const int col = nb * 16 + 4 * gq;
            f32x4 acc[RB];
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) acc[rb] = *reinterpret_cast<const f32x4*>(vec + VBN2 + col);
            gemm_t<H, RB>(A, sn, acc);
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) {
                const int rr = rb * 16 + i;
                if (t0 + rr < N) *reinterpret_cast<f32x4*>(a.z + (row0 + rr) * NN + col) = acc[rb];
            }
            if (nb + NW < NN / 16) sn = nxt;
        }
        TSTAMP(8);
        TSTAMP_RT(15);
    } else {
        TSTAMP(6);
        TSTAMP(7);
        TSTAMP(8);
        TSTAMP_RT(15);
    }
}

// ---------------------------------------------------------------------------
enum { SRC_X = 0, SRC_EMBED = 1, SRC_EXPAND = 2 };
struct FArgs {
    int B, N, npad, ntile;
    const int32_t* dN;  // device frame count (dev_frames; N is then the capacity)
    unsigned* qcnt;
    unsigned qseq;
    float sl2;
    const float* x_in;
    const int64_t* ids;
    const float *emb, *pe;
    int vocab;
    float escale;
    const int64_t* lengths;
    uint8_t* mask;
    const float* enc;
    const int32_t* cum;
    int S;
    int32_t* post;
    int32_t post_seq;
    float* x_out;
    const float *g, *bln;
    const u32x4* W;
    unsigned char *q, *k, *v;
};

#ifndef FK_MINW  // A/B builds: waves per SIMD the first launch is compiled for
#define FK_MINW 2
#endif
// Waves per first-launch workgroup: 64-row tiles (the very large grids) run
// 4 waves, so two workgroups share a CU at 189 VGPRs and one tile's latency
// chain (prefix sums -> search -> gather -> LN -> QKV -> stores) overlaps the
// other's: configs[4]'s frame-expansion launch 210 -> 192 us; the small grids'
// 16- and 32-row tiles keep 8 (4 there: B=8 6.3 -> 7.5 us,
// profiles/r04/r04af_*).
#ifndef FK_NW4  // A/B builds: waves of the 64-row-tile workgroups
#define FK_NW4 4
#endif
constexpr int fk_nw(int rb) { return rb == 4 ? FK_NW4 : NW; }
template <int H, int SRC, bool MASKED, int RB>
__global__ __launch_bounds__(fk_nw(RB) * 64, FK_MINW) void first_kernel(FArgs a) {
    constexpr int HD = H / HEADS, H4 = H / 4, TR = 16 * RB, FNW = fk_nw(RB);
    __shared__ __attribute__((aligned(16))) float O[TR * frs(H)];
    __shared__ __attribute__((aligned(16))) unsigned char A[TR * srs(H)];
    __shared__ __attribute__((aligned(16))) float vec[2 * H];
    __shared__ int sp[TR];
    __shared__ int item;
    if (a.post && blockIdx.x == 0 && threadIdx.x == 0) {  // the frame count for the host (TflFirst::post)
        __hip_atomic_store(a.post + 1, max(1, *a.dN), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(a.post, a.post_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    int b, tile;
    claim_tile(a.B, a.ntile, a.qcnt, a.qseq, &item, &b, &tile);
    const int t0 = tile * TR, N = a.dN ? dev_frames(a.dN, a.N) : a.N;
    const int wave = threadIdx.x >> 6;
    const QkvOut qo{a.q, a.k, a.v, a.npad, a.npad / KC, MASKED ? 1.f : a.sl2};
    if (t0 >= N) {
        zero_tile<H, HD, RB, FNW>(qo, b, t0);
        return;
    }
    // 16-row tiles (tfl_one): all of the wave's QKV strips at the start
    constexpr bool ONE = tfl_one(RB) && FNW == NW;
    Strip<H> sq;
    QkvStrips<H> sqa;
    if constexpr (ONE) sqa.load(a.W);
    else if (wave < 3 * H / 16) sq.load(a.W, wave);
    for (int e = threadIdx.x; e < H; e += FNW * 64) {
        vec[e] = a.g[e];
        vec[H + e] = a.bln[e];
    }
    if constexpr (SRC == SRC_EXPAND) {
        // source phoneme of each frame: the smallest s with cum[s + 1] > t (-1:
        // past the total); the utterance's prefix sums are searched in LDS
        // (one coalesced load instead of a chain of dependent L2 reads)
        constexpr int CS = 1024;
        __shared__ int32_t cs[CS];
        const int32_t* cg = a.cum + (size_t)b * (a.S + 1);
        const bool in_lds = a.S + 1 <= CS;
        if (in_lds)
            for (int k = threadIdx.x; k <= a.S; k += FNW * 64) cs[k] = cg[k];
        __syncthreads();
        if (threadIdx.x < TR) {
            const int32_t* c = in_lds ? cs : cg;
            const int t = t0 + threadIdx.x;
            int v = -1;
            if (t < N && t < c[a.S]) {
                int lo = 0, hi = a.S - 1;
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (c[mid + 1] > t) hi = mid;
                    else lo = mid + 1;
                }
                v = b * a.S + lo;
            }
            sp[threadIdx.x] = v;
        }
        __syncthreads();
    }
    for (int idx = threadIdx.x; idx < TR * H4; idx += FNW * 64) {
        const int r = idx / H4, c = (idx - r * H4) * 4, t = t0 + r;
        const size_t row = (size_t)b * N + t;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (t < N) {
            if constexpr (SRC == SRC_X) {
                v = *reinterpret_cast<const float4*>(a.x_in + row * H + c);
            } else if constexpr (SRC == SRC_EMBED) {
                // tts_model.py:78-80: E[id] * sqrt(H) + pe[t]; ids outside the table read zeros
                const int64_t id = a.ids[row];
                float4 e = make_float4(0.f, 0.f, 0.f, 0.f);
                if (id >= 0 && id < a.vocab) e = *reinterpret_cast<const float4*>(a.emb + id * H + c);
                const float4 p = *reinterpret_cast<const float4*>(a.pe + (size_t)t * H + c);
                v = make_float4(__builtin_fmaf(e.x, a.escale, p.x), __builtin_fmaf(e.y, a.escale, p.y),
                                __builtin_fmaf(e.z, a.escale, p.z), __builtin_fmaf(e.w, a.escale, p.w));
                if (a.mask && c == 0) a.mask[row] = (int64_t)t < a.lengths[b] ? 1 : 0;  // components.py:236-240
            } else {
                const int q = sp[r];
                if (q >= 0) v = *reinterpret_cast<const float4*>(a.enc + (size_t)q * H + c);
            }
            if constexpr (SRC != SRC_X) *reinterpret_cast<float4*>(a.x_out + row * H + c) = v;
        }
        *reinterpret_cast<float4*>(O + r * frs(H) + c) = v;
    }
    __syncthreads();
    ln_rows<H, TR, FNW * 64>(O, A, vec, vec + H);
    __syncthreads();
    if constexpr (ONE) qkv_phase_pre<H, HD>(A, sqa, qo, b, t0, N);
    else qkv_phase<H, HD, RB, FNW>(A, a.W, sq, qo, b, t0, N);
}

}  // namespace tfl

#ifdef TFL_STAMPS
extern "C" int32_t m2_debug_stamps_tfl(void* host, size_t bytes) {
    return (int32_t)hipMemcpyFromSymbol(host, HIP_SYMBOL(tfl::g_tfl_stamps),
                                        bytes < sizeof(tfl::g_tfl_stamps) ? bytes : sizeof(tfl::g_tfl_stamps));
}
#endif

// ---------------------------------------------------------------------------
bool tfl_supported(int H, int heads) { return heads == 2 && (H == 32 || H == 64 || H == 96); }

bool tfl_proj_supported(int H, int NN) {
    return (H == 32 && (NN == 32 || NN == 64)) || (H == 64 && (NN == 64 || NN == 80)) ||
           (H == 96 && (NN == 80 || NN == 96));
}

// a multiple of 64 so that 16-, 32- and 64-row tiles all cover [0, npad) exactly
int tfl_npad(int N) { return (N + 63) / 64 * 64; }

namespace {
void tfl_sizes(int B, int N, int H, int heads, size_t* qk, size_t* v) {
    const int HD = H / heads, npad = tfl_npad(N);
    *qk = align_up((size_t)B * heads * (npad / 16) * ((HD / 32) * 2048 + ((HD % 32) / 16) * 1024), 256);
    *v = align_up((size_t)B * heads * (npad / tfl::KC) * (HD / 16) * 2048, 256);
}
}  // namespace

size_t tfl_bytes(int B, int N, int H, int heads) {
    size_t qk, v;
    tfl_sizes(B, N, H, heads, &qk, &v);
    return 2 * qk + v;
}

void tfl_carve(unsigned char* base, int B, int N, int H, int heads, TflBufs* out) {
    size_t qk, v;
    tfl_sizes(B, N, H, heads, &qk, &v);
    *out = TflBufs{base, base + qk, base + 2 * qk};
}

namespace {
// Rows per workgroup of the layer launches: 64 (query-split attention, K / V
// staged in LDS) once the 64-row tiles alone fill the 256 CUs; else 16 while
// one round of the CUs holds the 16-row grid, else 32.  M2_TFL_RB=1|2|4
// forces one.  The first (LN1 -> QKV) launch has no attention: at most 32.
int tfl_rb(int B, int N) {
    if (sw().tfl_rb) return sw().tfl_rb;
    const long tiles16 = (long)B * (tfl_npad(N) / tfl::TQ);
    return tiles16 >= 4 * 256 ? 4 : (tiles16 > 256 ? 2 : 1);
}
// 64-row tiles: two query blocks per wave with the lean softmax
// (attention_qsplit2<..., LEAN>) at head_dim 48 (stage2: B=128 T=2600 step
// -1.5 %, B=16 T=2600 -1.9 %, B=64 T=500 -0.8 % against the plain two-block
// form, which was itself -0.7 % at B=128 T=2600 against one block; the lean
// one-block form +2.2 % at B=16 T=2600), the lean one-block form below
// (stage1 B=32: -0.7 % against the plain one-block form; two blocks +0.3 to
// +0.6 %; in-process A/Bs, profiles/r03/r03ab_*, r03ad_ab.txt, r03aj_ab.txt,
// r03al_ab.txt).  Round 4: at head_dim 48 the wave-specialised form with
// LDS-DMA staging (attention_qsplit_ws<..., DMA>; masked launches keep the
// lean two-block form): against the ping-pong form (6), itself -0.9 % on the
// long-form step against the lean two-block form (3): long-form step -1.5 %,
// B=16 T=2600 -1.1 %, B=64 T=500 level (in-process A/Bs,
// profiles/r04/r04j_*, r04l_*, r04m_*, r04n_*); at head_dim 32 it is slower
// than the lean one-block form (stage1 B=32 +0.5 %, B=128 +1.4 %).  Measured
// and not kept (removed in round 5): the software-pipelined form (5, level or
// slower, r04d / r04e), the wave-specialised form with register staging (7,
// between 6 and 9) and with its regions interleaved by group barriers (8,
// +3 %; 10).  Round 6: the key-quarter form (12, attention_quarters) for
// every unmasked layer - at head_dim 48 it replaces 9 (configs[4] step -4.2 %,
// B=16 T=2600 -7.1 %, B=64 T=500 -2.6 %; 9 removed, history keeps it), at
// head_dim 32 the lean one-block form (stage1 B=128 S=130 -3.2 %, B=32 S=520
// -9.1 %; profiles/r06/r06ad_*, r06ah_*).  Masked layers, and layers whose
// scores may leave the f16 range (12's base is an f16 pair), keep the
// previous default: 3 at head_dim 48, 4 below.  M2_TFL_QS2=0|2|3|4|12 forces
// a form (switch table, m2_common.h): 0 / 2 one / two query blocks, 3 / 4 the
// same with the lean softmax, 12 the key-quarter form (unmasked layers).
int tfl_qs2(int H) {
    if (sw().tfl_qs2 >= 0) return sw().tfl_qs2;
    return 12;
}
int tfl_ntile(int N, int rb) { return (tfl_npad(N) + tfl::TQ * rb - 1) / (tfl::TQ * rb); }
dim3 tfl_grid(int B, int N, int rb) { return dim3(B * tfl_ntile(N, rb)); }
float tfl_sl2(int H) {
    const float scale = (float)(1.0 / std::sqrt((double)(H / tfl::HEADS)));  // components.py:52, fp32 at the mul
    return scale * tfl::kLog2e;
}
}  // namespace

int32_t launch_tfl_first(const TflFirst& f, int B, int N, int H, int heads, bool masked, float* x_out,
                         const float* g, const float* bln, const float* Wqkv, const TflBufs& out, TflQueue q,
                         hipStream_t st) {
    M2_CHECK_SHAPE(tfl_supported(H, heads), "tfl: unsupported (hidden_dim, heads)");
    M2_CHECK_ARG(q.cnt, "tfl: no work-queue counters");
    // every launch must run: its workgroups zero the NEXT launch's work-queue
    // counter set (TflQueue), so an empty launch that returned M2_OK would
    // leave that set stale (callers return before an empty batch)
    if (B == 0 || N == 0) return fail(M2_E_INTERNAL, "tfl: empty launch (no work-queue hand-off)");
    tfl::FArgs a{};
    a.B = B;
    a.N = N;
    a.npad = tfl_npad(N);
    // rows per workgroup: the layers' choice up to 32, 64 for grids of >= 8
    // rounds of 16-row tiles (latency-bound rounds; with 8-wave workgroups
    // 64-row tiles made stage2 B=64 1.4 % slower, profiles/r03/ab/r03x_ab.txt,
    // with the 4-wave ones (fk_nw) 0.5-1.7 % faster, r04ag_s2_b64_first_rb);
    // M2_TFL_FIRST_RB=1|2|4 forces one (switch table, m2_common.h)
    int rb = tfl_rb(B, N) > 1 ? 2 : 1;
    if ((long)B * (tfl_npad(N) / tfl::TQ) >= 8L * 256) rb = 4;
    if (sw().tfl_first_rb) rb = sw().tfl_first_rb;
    if (masked && sw().tfl_rb_masked) rb = sw().tfl_rb_masked;
    if (!masked && sw().tfl_rb_unmasked) rb = sw().tfl_rb_unmasked;
    a.ntile = tfl_ntile(N, rb);
    a.qcnt = q.cnt;
    a.qseq = q.seq;
    a.sl2 = tfl_sl2(H);
    a.x_in = f.x_in;
    a.ids = f.ids;
    a.emb = f.emb;
    a.pe = f.pe;
    a.vocab = f.vocab;
    a.escale = f.escale;
    a.lengths = f.lengths;
    a.mask = f.lengths ? f.mask : nullptr;
    a.enc = f.enc;
    a.cum = f.cum;
    a.S = f.S;
    a.dN = f.dN;
    a.post = f.dN ? f.post : nullptr;
    a.post_seq = f.post_seq;
    a.x_out = x_out;
    a.g = g;
    a.bln = bln;
    a.W = reinterpret_cast<const vx_u32x4*>(Wqkv);
    a.q = out.q;
    a.k = out.k;
    a.v = out.v;
    const dim3 grid = tfl_grid(B, N, rb), blk(tfl::fk_nw(rb) * 64);
#define M2_TFF(HH, SS, MM)                                                                      \
    if (H == HH && f.src == SS && masked == MM) {                                               \
        if (rb == 4) hipLaunchKernelGGL((tfl::first_kernel<HH, SS, MM, 4>), grid, blk, 0, st, a);  \
        else if (rb == 2) hipLaunchKernelGGL((tfl::first_kernel<HH, SS, MM, 2>), grid, blk, 0, st, a);  \
        else hipLaunchKernelGGL((tfl::first_kernel<HH, SS, MM, 1>), grid, blk, 0, st, a);          \
        M2_LAUNCHED("tfl first_kernel");                                                        \
        return M2_OK;                                                                           \
    }
#define M2_TFF_H(HH)                  \
    M2_TFF(HH, tfl::SRC_X, false)     \
    M2_TFF(HH, tfl::SRC_X, true)      \
    M2_TFF(HH, tfl::SRC_EMBED, false) \
    M2_TFF(HH, tfl::SRC_EMBED, true)  \
    M2_TFF(HH, tfl::SRC_EXPAND, false)
    M2_TFF_H(32)
    M2_TFF_H(64)
    M2_TFF_H(96)
#undef M2_TFF_H
#undef M2_TFF
    return fail(M2_E_SHAPE, "tfl first layer: unsupported (hidden_dim, row source, mask)");
}

int32_t launch_tfl_layer(const TflLayer& w, int B, int N, int H, int heads, bool masked, const int64_t* lengths,
                         const float* x_in, float* x_out, const TflBufs& in, int next, const TflBufs& out, int NN,
                         float* z, TflQueue q, hipStream_t st, const int32_t* dN) {
    M2_CHECK_SHAPE(tfl_supported(H, heads), "tfl: unsupported (hidden_dim, heads)");
    M2_CHECK_ARG(!masked || lengths, "tfl: masked attention needs lengths");
    M2_CHECK_ARG(q.cnt, "tfl: no work-queue counters");
    // every launch must run: its workgroups zero the NEXT launch's work-queue
    // counter set (TflQueue), so an empty launch that returned M2_OK would
    // leave that set stale (callers return before an empty batch)
    if (B == 0 || N == 0) return fail(M2_E_INTERNAL, "tfl: empty launch (no work-queue hand-off)");
    auto u4 = [](const float* p) { return reinterpret_cast<const vx_u32x4*>(p); };
    tfl::LArgs a{};
    a.B = B;
    a.N = N;
    a.dN = dN;
    a.npad = tfl_npad(N);
    const int rb = masked && sw().tfl_rb_masked     ? sw().tfl_rb_masked
                   : !masked && sw().tfl_rb_unmasked ? sw().tfl_rb_unmasked
                                                     : tfl_rb(B, N);
    a.ntile = tfl_ntile(N, rb);
    a.qcnt = q.cnt;
    a.qseq = q.seq;
    a.sl2 = tfl_sl2(H);
    a.lengths = lengths;
    a.x_in = x_in;
    a.x_out = x_out;
    a.q = in.q;
    a.k = in.k;
    a.v = in.v;
    a.Wo = u4(w.Wo);
    a.W1 = u4(w.W1);
    a.W2 = u4(w.W2);
    a.Wn = u4(w.Wn);
    a.bo = w.bo;
    a.g2 = w.g2;
    a.b2n = w.b2n;
    a.b1 = w.b1;
    a.b2 = w.b2;
    a.gn = w.gn;
    a.bn = w.bn;
    a.bn2 = w.bn2;
    a.nq = out.q;
    a.nk = out.k;
    a.nv = out.v;
    a.z = z;
    const dim3 grid = tfl_grid(B, N, rb), blk(tfl::NW * 64);
    // form 12 is unmasked-only, and at head_dim 48 keeps the softmax base as
    // an f16 pair: a masked launch, or a layer whose scores may leave the f16
    // range, runs the previous default instead (the lean two-block form 3 at
    // head_dim 48, the one-block form 4 below)
    int qs2 = tfl_qs2(H);
    if (qs2 == 12 && (masked || w.wide_scores)) qs2 = H / tfl::HEADS >= 48 ? 3 : 4;
#define M2_TFL(HH, MM, NX, NNN)                                                                 \
    if (H == HH && masked == MM && next == NX && (NX != 2 || NN == NNN)) {                      \
        if constexpr (!MM) {                                                                    \
            if (rb == 4 && qs2 == 12) {                                                         \
                hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 4, 12>), grid, blk, 0, st, a); \
                M2_LAUNCHED("tfl layer_kernel");                                                \
                return M2_OK;                                                                   \
            }                                                                                   \
        }                                                                                       \
        if (rb == 4 && qs2 == 4) hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 4, 4>), grid, blk, 0, st, a);  \
        else if (rb == 4 && qs2 == 3) hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 4, 3>), grid, blk, 0, st, a);  \
        else if (rb == 4 && qs2 == 2) hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 4, 2>), grid, blk, 0, st, a);  \
        else if (rb == 4) hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 4>), grid, blk, 0, st, a);  \
        else if (rb == 2) hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 2>), grid, blk, 0, st, a);  \
        else hipLaunchKernelGGL((tfl::layer_kernel<HH, MM, NX, NNN, 1>), grid, blk, 0, st, a);          \
        M2_LAUNCHED("tfl layer_kernel");                                                        \
        return M2_OK;                                                                           \
    }
#define M2_TFL_H(HH, P0, P1)     \
    M2_TFL(HH, false, 0, 0)      \
    M2_TFL(HH, false, 1, 0)      \
    M2_TFL(HH, true, 0, 0)       \
    M2_TFL(HH, true, 1, 0)       \
    M2_TFL(HH, false, 2, P0)     \
    M2_TFL(HH, false, 2, P1)
    M2_TFL_H(32, 32, 64)
    M2_TFL_H(64, 64, 80)
    M2_TFL_H(96, 80, 96)
#undef M2_TFL_H
#undef M2_TFL
    return fail(M2_E_SHAPE, "tfl layer: unsupported (hidden_dim, mask, next, projection width)");
}

}  // namespace m2
