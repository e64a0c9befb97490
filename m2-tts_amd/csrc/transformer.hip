// Transformer kernels for the text encoder and the mel decoder (gfx950).
//
//   embed_pe_kernel    TextEncoder embed*sqrt(H) + pe           tts_model.py:78-80
//   layer_norm_kernel  nn.LayerNorm(eps 1e-5)                   tts_model.py:87,223
//   linear_kernel      [LN ->] x.W^T + b [-> relu] [+ residual] components.py:55-56,98-103,131-140
//   attention_kernel   softmax(QK^T*scale, -1e9 key mask).V     components.py:72-86
//
// All fp32.  The GEMMs run on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32,
// 64 FLOP/clk/SIMD = the fp32 vector peak, one rounding per product).
#include <cstdlib>
#include <type_traits>

#include "m2_common.h"
#include "vocoder_fused.h"  // split2u: fp32 -> (hi, lo) f16

namespace m2 {

typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// x[b,s,:] = E[ids[b,s],:] * sqrt(H) + pe[s,:]
// Out-of-range ids read a zero row (the reference would raise in nn.Embedding).
// With lengths != nullptr the same launch writes the padding mask
// mask[b,s] = s < lengths[b] (components.py:236-240; the encoder's first
// kernel, one launch fewer per inference).
__global__ void embed_pe_kernel(const int64_t* __restrict__ ids, const float* __restrict__ emb,
                                const float* __restrict__ pe, int R, int S, int H, int vocab,
                                float emb_scale, float* __restrict__ out, const int64_t* __restrict__ lengths,
                                uint8_t* __restrict__ mask) {
    const int total = R * H;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int r = i / H, h = i - r * H;
        const int64_t id = ids[r];
        const float e = (id >= 0 && id < vocab) ? emb[id * H + h] : 0.f;
        const int s = r % S;
        out[i] = e * emb_scale + pe[s * H + h];
        if (lengths && h == 0) mask[r] = (int64_t)s < lengths[r / S] ? 1 : 0;
    }
}

// ---------------------------------------------------------------------------
// One wave per row; two-pass mean / biased variance, as nn.LayerNorm.
__global__ __launch_bounds__(256) void layer_norm_kernel(const float* __restrict__ x,
                                                         const float* __restrict__ g,
                                                         const float* __restrict__ b, int R,
                                                         int K, float* __restrict__ y) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= R) return;
    const float* xr = x + (size_t)row * K;
    float mean, rstd;
    ln_row_stats(xr, K, lane, mean, rstd);
    float* yr = y + (size_t)row * K;
    for (int k = lane; k < K; k += 64) yr[k] = ln_apply(xr[k], mean, rstd, g[k], b[k]);
}

// ---------------------------------------------------------------------------
// y[R,N] = act(LN?(x)[R,K] . W[N,K]^T + bias) (+ res[R,N])
//
// Workgroup = 4 waves, output tile 64 rows x 64 cols; wave (wr,wc) owns a
// 32x32 sub-tile accumulated by K/2 v_mfma_f32_32x32x2_f32.  X and W tiles
// are staged in LDS with rows padded by 4 floats (16 B), so the per-lane
// float4 operand reads of 32 different rows hit distinct bank quads.
// k-order: at step s, lane half h supplies k = h*K/2 + s for BOTH operands,
// so each lane streams its k range with float4 reads (any consistent k
// permutation is a valid order for the sum).  Needs K % 8 == 0, K <= 256.
constexpr int LIN_TILE = 64;

__global__ __launch_bounds__(256) void linear_kernel(
    const float* __restrict__ x, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ w, const float* __restrict__ bias, const float* res, int act, int R,
    int K, int N, float* y) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const int KP = K + 4;
    float* Xs = lds;                    // [64][KP]
    float* Ws = lds + LIN_TILE * KP;    // [64][KP]
    float* stats = Ws + LIN_TILE * KP;  // [64][2] mean, rstd
    const int tid = threadIdx.x;
    const int r0 = blockIdx.x * LIN_TILE, c0 = blockIdx.y * LIN_TILE;
    const int K4 = K >> 2;

    for (int i = tid; i < LIN_TILE * K4; i += 256) {
        const int row = i / K4, c4 = i - row * K4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + row < R) v = *reinterpret_cast<const float4*>(x + (size_t)(r0 + row) * K + 4 * c4);
        *reinterpret_cast<float4*>(Xs + row * KP + 4 * c4) = v;
        float4 u = make_float4(0.f, 0.f, 0.f, 0.f);
        if (c0 + row < N) u = *reinterpret_cast<const float4*>(w + (size_t)(c0 + row) * K + 4 * c4);
        *reinterpret_cast<float4*>(Ws + row * KP + 4 * c4) = u;
    }
    __syncthreads();

    if (gamma != nullptr) {
        // 4 lanes per row: partial sums then a 4-lane butterfly.
        const int row = tid >> 2, part = tid & 3;
        const float* xr = Xs + row * KP;
        float s = 0.f;
        for (int k = part; k < K; k += 4) s += xr[k];
        s += __shfl_xor(s, 1);
        s += __shfl_xor(s, 2);
        const float mean = s / (float)K;
        float v = 0.f;
        for (int k = part; k < K; k += 4) { float d = xr[k] - mean; v += d * d; }
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        if (part == 0) { stats[2 * row] = mean; stats[2 * row + 1] = 1.0f / sqrtf(v / (float)K + kLnEps); }
        __syncthreads();
        for (int i = tid; i < LIN_TILE * K; i += 256) {
            const int rr = i / K, k = i - rr * K;
            float* p = Xs + rr * KP + k;
            *p = (*p - stats[2 * rr]) * stats[2 * rr + 1] * gamma[k] + beta[k];
        }
        __syncthreads();
    }

    const int wave = tid >> 6, lane = tid & 63;
    const int wr = wave >> 1, wc = wave & 1;
    if (c0 + wc * 32 >= N) return;  // whole sub-tile past the last column
    const int li = lane & 31, h = lane >> 5;
    const float* ap = Xs + (wr * 32 + li) * KP + h * (K >> 1);
    const float* bp = Ws + (wc * 32 + li) * KP + h * (K >> 1);
    f32x16 acc = {};
    for (int s = 0; s < (K >> 1); s += 4) {
        const float4 a = *reinterpret_cast<const float4*>(ap + s);
        const float4 bb = *reinterpret_cast<const float4*>(bp + s);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bb.x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bb.y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bb.z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bb.w, acc, 0, 0, 0);
    }
    const int col = c0 + wc * 32 + li;
    if (col >= N) return;
    const float bv = bias ? bias[col] : 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = r0 + wr * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (row < R) {
            float v = acc[reg] + bv;
            if (act == ACT_RELU) v = v > 0.f ? v : 0.f;
            const size_t o = (size_t)row * N + col;
            if (res) v = res[o] + v;
            y[o] = v;
        }
    }
}

// ---------------------------------------------------------------------------
// Attention core on the exact-f32 MFMA (v_mfma_f32_16x16x4_f32), flash-style.
//
// Workgroup = 4 waves = 64 queries of one (utterance, head); keys stream
// through LDS in chunks of 64.  Each wave owns 16 queries and works on the
// TRANSPOSED problem so that no register shuffles sit between the two GEMMs:
//   S^T[key][q] = K . Q^T    A = K rows from LDS, B = Q (registers, whole loop)
//   O^T[d][q]  += V^T . P^T  A = V^T rows from LDS, B = P^T straight from the
//                            S^T accumulators
// A 16x16 accumulator lane holds column q = lane&15 and rows 4*(lane>>4)+r, so
// after S^T a lane owns keys {4g + r} of ONE query (g = lane>>4): exactly the
// B operand of the PV product when k-step r takes keys {4g + r : g} (a fixed
// permutation of the 16 keys, applied to V^T's reads as well).  QK^T uses the
// k-order d = 16t + 4g + c so both operands are float4 reads.  Softmax
// statistics are per query, i.e. per lane: the running max is reduced over
// the 4 lane groups (2 xor-shuffles) once per 64-key chunk; the running sum
// stays a per-lane partial until the end.
// Scores are (q.k) * scale with masked keys set to exactly -1e9 as the
// reference does (a fully masked row becomes a uniform average, as there);
// keys past N get weight 0.  components.py:72-86
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int ATT_KC = 64;  // keys per LDS chunk

// Softmax in base 2: scores are carried as (q.k)*scale*log2(e) and
// exponentiated with v_exp_f32 (exp2); a masked key's -1e9 becomes
// -1e9*log2(e) (still exp -> 0, and equal across a fully masked row).
constexpr float kLog2e = 1.4426950408889634f;

template <int HD>
__global__ __launch_bounds__(256) void attention_kernel(const float* __restrict__ qkv,
                                                        const uint8_t* __restrict__ key_mask,
                                                        int N, int H, float scale,
                                                        float* __restrict__ out) {
    static_assert(HD % 16 == 0, "head_dim must be a multiple of 16");
    constexpr int KSTR = HD + 4;       // Ks row stride (floats)
    constexpr int VSTR = ATT_KC + 4;   // Vt row stride
    constexpr int NT = HD / 16;        // 16-wide d tiles
    constexpr int IT = ATT_KC * (HD / 4) / 256;  // float4 of K (and of V) per thread per chunk
    // Two chunk buffers: chunk c+1 is fetched into registers while chunk c is
    // consumed, then stored into the other buffer - one barrier per chunk.
    __shared__ __attribute__((aligned(16))) float Ks[2][ATT_KC * KSTR];
    __shared__ __attribute__((aligned(16))) float Vt[2][HD * VSTR];
    __shared__ float Mk[2][ATT_KC];
    const int b = blockIdx.z, hh = blockIdx.y;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, g = lane >> 4;
    const size_t row3 = (size_t)3 * H;
    const float* base = qkv + (size_t)b * N * row3 + hh * HD;
    const int qi = blockIdx.x * 64 + wave * 16 + li;
    const float sl2 = scale * kLog2e;

    float4 kr[IT], vr[IT];
    float mkr = 0.f;
    auto fetch = [&](int j0) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256, key = i / (HD / 4), d4 = i - key * (HD / 4), j = j0 + key;
            kr[it] = vr[it] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (j < N) {
                kr[it] = *reinterpret_cast<const float4*>(base + j * row3 + H + 4 * d4);
                vr[it] = *reinterpret_cast<const float4*>(base + j * row3 + 2 * H + 4 * d4);
            }
        }
        if (tid < ATT_KC) {
            const int j = j0 + tid;
            // 0: live key, 1: masked (score -1e9), 2: past the end (weight 0)
            mkr = j >= N ? 2.f : ((key_mask && key_mask[(size_t)b * N + j] == 0) ? 1.f : 0.f);
        }
    };
    auto stash = [&](int buf) {
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = tid + it * 256, key = i / (HD / 4), d4 = i - key * (HD / 4);
            *reinterpret_cast<float4*>(&Ks[buf][key * KSTR + 4 * d4]) = kr[it];
            Vt[buf][(4 * d4 + 0) * VSTR + key] = vr[it].x;
            Vt[buf][(4 * d4 + 1) * VSTR + key] = vr[it].y;
            Vt[buf][(4 * d4 + 2) * VSTR + key] = vr[it].z;
            Vt[buf][(4 * d4 + 3) * VSTR + key] = vr[it].w;
        }
        if (tid < ATT_KC) Mk[buf][tid] = mkr;
    };

    fetch(0);
    float4 q[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
        q[t] = qi < N ? *reinterpret_cast<const float4*>(base + qi * row3 + 16 * t + 4 * g)
                      : make_float4(0.f, 0.f, 0.f, 0.f);
    f32x4 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, lsum = 0.f;
    stash(0);
    __syncthreads();

    const int nch = (N + ATT_KC - 1) / ATT_KC;
#pragma unroll 1
    for (int c = 0; c < nch; ++c) {
        const int buf = c & 1;
        if (c + 1 < nch) fetch((c + 1) * ATT_KC);
        const float* K = Ks[buf];
        const float* V = Vt[buf];
        const float* MK = Mk[buf];
        float s[4][4];  // [16-key block][r]: key 16*kb + 4*g + r of query li (base-2 scores)
        float cmax = -INFINITY;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            f32x4 st = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float4 a = *reinterpret_cast<const float4*>(K + (16 * kb + li) * KSTR + 16 * t + 4 * g);
                st = mfma16(a.x, q[t].x, st);
                st = mfma16(a.y, q[t].y, st);
                st = mfma16(a.z, q[t].z, st);
                st = mfma16(a.w, q[t].w, st);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const float mk = MK[16 * kb + 4 * g + r];
                const float v = st[r] * sl2;
                s[kb][r] = mk == 0.f ? v : (mk == 1.f ? kMaskFill * kLog2e : -INFINITY);
                cmax = fmaxf(cmax, s[kb][r]);
            }
        }
        cmax = fmaxf(cmax, __shfl_xor(cmax, 16));
        cmax = fmaxf(cmax, __shfl_xor(cmax, 32));
        const float mn = fmaxf(m, cmax);
        const float corr = exp2f(m - mn);  // m = -inf on the first chunk -> 0
        lsum *= corr;
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] *= corr;
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                s[kb][r] = exp2f(s[kb][r] - mn);
                lsum += s[kb][r];
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const float4 v = *reinterpret_cast<const float4*>(V + (16 * t + li) * VSTR + 16 * kb + 4 * g);
                acc[t] = mfma16(v.x, s[kb][0], acc[t]);
                acc[t] = mfma16(v.y, s[kb][1], acc[t]);
                acc[t] = mfma16(v.z, s[kb][2], acc[t]);
                acc[t] = mfma16(v.w, s[kb][3], acc[t]);
            }
        }
        m = mn;
        if (c + 1 < nch) {
            stash(buf ^ 1);  // the other buffer was last read in chunk c-1, before the previous barrier
            __syncthreads();
        }
    }
    lsum += __shfl_xor(lsum, 16);
    lsum += __shfl_xor(lsum, 32);
    if (qi >= N) return;
    const float inv = 1.0f / lsum;
    float* orow = out + ((size_t)b * N + qi) * H + hh * HD;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) orow[16 * t + 4 * g + r] = acc[t][r] * inv;
}

// ---------------------------------------------------------------------------
// The same attention core on split-f16 MFMA (v_mfma_f32_16x16x32_f16, 16x the
// f32 MFMA's rate): every fp32 operand as hi = f16(x), lo = f16(x - hi) and
// every product as hi*hi + hi*lo + lo*hi in one fp32 accumulator, the
// vocoder's arithmetic (~2^-22 relative per product).  Same
// tiling and transposed formulation as attention_kernel; K and V^T are split
// once, when a chunk is stashed in LDS (hi and lo planes per row), Q once per
// wave, P per 32-key k-step in registers.
//   S^T = K . Q^T: A = K rows (lane: 8 head dims of one key), B = Q^T (lane:
//     8 head dims of its query); head dims padded to 32 per k-step.
//   O^T += V^T . P^T: a 32-key k-step takes key blocks 2j and 2j+1, whose S^T
//     accumulators give lane group g keys {32j + 4g + e, 32j + 16 + 4g + e}
//     (e < 4) of its query: exactly the B fragment, provided V^T's columns are
//     stored in that order (key 32j + 16h + 4g + e at column 32j + 8g + 4h + e).
// Row strides 160 / 288 B (RS/16 = 2 mod 4): conflict-free ds_read_b128.
template <int V>
using ic_ = std::integral_constant<int, V>;
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(const F& f) {
    if constexpr (I < N) {
        f(ic_<I>{});
        static_for<N, I + 1>(f);
    }
}
// Diagnostic build only (-DATT_STAMPS): per-wave s_memtime stamps at phase
// boundaries of attention_split_kernel, [workgroup][wave][16]; slots 14 / 15
// = s_memrealtime (100 MHz) at start / end (tools/probe/att_stamps.py).
#ifdef ATT_STAMPS
__device__ unsigned long long g_att_stamps[2048][8][16];
#define ASTAMP(i)                                                                                        \
    do {                                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        unsigned long long _t;                                                                           \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                      \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048) g_att_stamps[blockIdx.x][threadIdx.x >> 6][i] = _t; \
    } while (0)
#define ASTAMP_RT(i)                                                                                     \
    do {                                                                                                 \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        unsigned long long _t;                                                                           \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                  \
        __builtin_amdgcn_sched_barrier(0);                                                               \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 2048) g_att_stamps[blockIdx.x][threadIdx.x >> 6][i] = _t; \
    } while (0)
#else
#define ASTAMP(i) \
    do {          \
    } while (0)
#define ASTAMP_RT(i) \
    do {             \
    } while (0)
#endif

// Key split: a workgroup is 8 waves = 4 query groups x 2 key halves; the
// key-half-0 waves take the even 64-key chunks, the key-half-1 waves the odd
// ones, each with its own online-softmax state, merged through LDS at the end
// (flash-decoding inside the workgroup).  Twice the waves per query of the
// 4-wave form at the same LDS per wave: the per-chunk latency chain (LDS ->
// MFMA -> softmax -> MFMA) is what bounds this kernel.
// max over the four lanes l, l ^ 16, l ^ 32, l ^ 48 (the 16-lane groups of
// one query).  (A permlane16/32_swap form gave wrong maxima in the masked
// head_dim-48 instance - tools/probe/att_check.py - and the lazy path below
// needs this only on the chunks that move the base.)
__device__ __forceinline__ float grp4_max(float x) {
    x = vmax(x, __shfl_xor(x, 16));
    return vmax(x, __shfl_xor(x, 32));
}
// lazy-rescale threshold (base-2 units): weights stay <= 2^kLazyT
constexpr float kLazyT = 8.f;

template <int HD>
struct AttSplit {
    static constexpr int KS = (HD + 31) / 32, DP = 32 * KS;  // QK^T k-steps, padded head dim
    static constexpr int KRS = 4 * DP + 32;                    // K row: hi[DP] lo[DP] f16 + pad
    static constexpr int VRS = 4 * ATT_KC + 32;                // V^T row: hi[64 keys] lo[64] + pad
    static constexpr int KBUF = ATT_KC * KRS, VBUF = HD * VRS, MBUF = ATT_KC * 8;
    static constexpr int NBUF = 4;                             // 2 chunk pairs: one read, one being stashed
    static constexpr int LDS = NBUF * (KBUF + VBUF + MBUF);
};

__device__ __forceinline__ f32x4 mfma_f16(vx_u32x4 a, vx_u32x4 b, f32x4 c) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

// QT query tiles of 16 per wave (64 * QT queries per workgroup): every K / V
// fragment read from LDS feeds QT tiles, and every K / V byte a workgroup
// stages serves QT times as many queries (all K and V of an (utterance,
// head) pass through each of its query blocks' workgroups).  The launcher
// picks QT = 2 while the grid keeps a workgroup per CU.
// MASKED = false (the decoder, mask=None): Q is pre-scaled by
// scale * log2(e) before it is split, so a score is the raw MFMA dot product
// (no per-key (scale, fill) table, no fma per score); only the keys past N in
// the last chunk are set to -inf.  MASKED: the per-key (scale, add) table.
// The instruction budget matters: per 64-key chunk a wave issues 3 x
// (4 KS + 2 MT) MFMAs against ~200 VALU (PMC, tools/probe/att_pmc.sh), so
// address arithmetic is kept to uniform chunk bases plus per-lane 32-bit
// offsets fixed for the whole kernel.
template <int HD, int QT, bool MASKED>
__global__ __launch_bounds__(512, (HD <= 32 && QT == 1) ? 4 : 2) void attention_split_kernel(
    const float* __restrict__ qkv, const uint8_t* __restrict__ key_mask, int N, int H, float scale,
    float* __restrict__ out, int nqb, int heads, int ngroups) {
    using P = AttSplit<HD>;
    constexpr int KS = P::KS, DP = P::DP, KRS = P::KRS, VRS = P::VRS;
    constexpr int MT = HD / 16;                  // 16-row d blocks of O^T
    constexpr int IT = ATT_KC * (HD / 4) / 256;  // float4 of K per thread per chunk (256 threads per chunk)
    static_assert(HD % 16 == 0 && ATT_KC * (HD / 4) % 256 == 0, "head_dim");
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    unsigned char* const Ks0 = smem;
    unsigned char* const Vt0 = smem + P::NBUF * P::KBUF;
    // MASKED: per key (scale, add): live (scale*log2e, 0), masked (0,
    // -1e9*log2e), past the end (0, -inf): the base-2 score is one fma
    float2* const Mk0 = reinterpret_cast<float2*>(smem + P::NBUF * (P::KBUF + P::VBUF));
    // XCD-aware workgroup order: workgroup L runs on XCD L % 8 (each XCD has
    // its own L2), so the nqb query blocks of one (utterance, head) - which
    // all stream the same K and V - are given ids on the same XCD.
    const int L = blockIdx.x, xcd = L & 7, r = L >> 3;
    const int grp = xcd + 8 * (r / nqb), qb = r - (r / nqb) * nqb;
    if (grp >= ngroups) return;  // padding of the last round (ngroups % 8 != 0)
    ASTAMP_RT(14);
    ASTAMP(0);
    const int b = grp / heads, hh = grp - b * heads;
    const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, g = lane >> 4;
    const int qg = wave & 3, kh = wave >> 2;  // query group, key half
    const int ct = tid & 255, ch = wave >> 2;  // fetch / stash: thread within a chunk, chunk of the pair
    const int row3 = 3 * H;
    const int q0 = qb * 64 * QT + qg * 16 * QT + li;  // query of tile qt: q0 + 16 qt
    const float sl2 = scale * kLog2e;

    if constexpr (DP > HD) {  // zero the padded head dims of every K buffer once
        for (int i = tid; i < P::NBUF * ATT_KC; i += 512) {
            unsigned char* r = Ks0 + i * KRS;
            for (int d = HD; d < DP; d += 4) {
                *reinterpret_cast<uint2*>(r + 2 * d) = uint2{0u, 0u};
                *reinterpret_cast<uint2*>(r + 2 * DP + 2 * d) = uint2{0u, 0u};
            }
        }
    }
    // Chunk pairs stream through registers PF pairs ahead of their stash.
    // K: thread = (key, head-dim quad), quads fastest (128-B rows); V: thread
    // = (key pair, quad), pairs fastest, so the transposed stores (two keys'
    // f16 in one dword of a V^T row) hit 32 distinct banks.  Loads are
    // buffer loads through a per-chunk descriptor (base = the chunk's first
    // row, records = the rows left before N): per-lane byte offsets fixed for
    // the whole kernel, no address arithmetic per load (the VALU issue is what
    // bounds this loop), and rows past N read as zeros (they score -inf).
    // Every load is unconditional: a load inside a branch makes the compiler
    // wait for it at once (s_waitcnt vmcnt(0) at the join), which serialised
    // the prologue's loads (tools/probe/att_stamps.py).
    // PF = 2 pairs ahead; requesting every pair of N <= 512 in the prologue
    // (4 register slots) measured 5 % slower: the loop is VALU-issue bound.
    constexpr int PF = 2;
    constexpr int NQ4 = HD / 4, ITV = (32 * NQ4 + 255) / 256;
    const float* ubase = qkv + (size_t)b * N * row3;  // this utterance's rows
    const int hoff = hh * HD;
    int kvo[IT], vvo[ITV][2];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int i = ct + it * 256, key = i / NQ4, d4 = i - key * NQ4;
        kvo[it] = 4 * (key * row3 + H + hoff + 4 * d4);
    }
#pragma unroll
    for (int it = 0; it < ITV; ++it) {
        const int i = ct + it * 256, pr = i & 31, d4 = i >> 5;  // lanes past the quads load, are not stashed
#pragma unroll
        for (int h = 0; h < 2; ++h) vvo[it][h] = 4 * ((2 * pr + h) * row3 + 2 * H + hoff + 4 * (d4 < NQ4 ? d4 : 0));
    }
    float4 kr[PF][IT], vr[PF][ITV][2];
    int mraw[PF];
    const int nch = (N + ATT_KC - 1) / ATT_KC, npair = (nch + 1) / 2;
    auto fetch = [&](int pr_, auto sc) {  // chunk 2 pr_ + ch
        constexpr int sl = decltype(sc)::value;
        const int j0 = (2 * pr_ + ch) * ATT_KC;
        const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ubase) + (size_t)j0 * row3, 0,
                                                          4 * max(N - j0, 0) * row3, 0x00020000);
#pragma unroll
        for (int it = 0; it < IT; ++it)
            kr[sl][it] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, kvo[it], 0, 0));
#pragma unroll
        for (int it = 0; it < ITV; ++it)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                vr[sl][it][h] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, vvo[it][h], 0, 0));
        if constexpr (MASKED) mraw[sl] = key_mask[(size_t)b * N + min(j0 + (ct & (ATT_KC - 1)), N - 1)];
    };
    auto stash = [&](int buf, int pr_, auto sc) {  // this thread's chunk of pair pr_ into buffer buf
        constexpr int sl = decltype(sc)::value;
        unsigned char* Kb = Ks0 + buf * P::KBUF;
        unsigned char* Vb = Vt0 + buf * P::VBUF;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int i = ct + it * 256, key = i / NQ4, d4 = i - key * NQ4;
            unsigned h0, h1, l0, l1;
            split2u(kr[sl][it].x, kr[sl][it].y, h0, l0);
            split2u(kr[sl][it].z, kr[sl][it].w, h1, l1);
            unsigned char* kp = Kb + key * KRS + 8 * d4;
            *reinterpret_cast<uint2*>(kp) = uint2{h0, h1};
            *reinterpret_cast<uint2*>(kp + 2 * DP) = uint2{l0, l1};
        }
#pragma unroll
        for (int it = 0; it < ITV; ++it) {
            const int i = ct + it * 256, pr = i & 31, d4 = i >> 5;
            if (d4 < NQ4) {
                // keys 2pr, 2pr + 1 sit next to each other in the permuted column order
                const int key = 2 * pr;
                const int pk = (key & 32) | (((key >> 2) & 3) << 3) | (((key >> 4) & 1) << 2) | (key & 3);
                const float4 v0 = vr[sl][it][0], v1 = vr[sl][it][1];
                const float a[4] = {v0.x, v0.y, v0.z, v0.w}, c[4] = {v1.x, v1.y, v1.z, v1.w};
                unsigned char* vp = Vb + 4 * d4 * VRS + 2 * pk;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    unsigned hi, lo;
                    split2u(a[e], c[e], hi, lo);
                    *reinterpret_cast<unsigned*>(vp + e * VRS) = hi;
                    *reinterpret_cast<unsigned*>(vp + e * VRS + 2 * ATT_KC) = lo;
                }
            }
        }
        if constexpr (MASKED) {
            if (ct < ATT_KC) {
                const int j = (2 * pr_ + ch) * ATT_KC + ct;
                Mk0[buf * ATT_KC + ct] = j >= N ? make_float2(0.f, -INFINITY)
                                                : (mraw[sl] == 0 ? make_float2(0.f, kMaskFill * kLog2e)
                                                                 : make_float2(sl2, 0.f));
            }
        }
    };

    // B = Q^T: lane (query li, group g) holds head dims 32 ks + 8 g .. + 7;
    // unmasked: pre-scaled by scale * log2(e) (the score is then the dot).
    // Q rows (past N: zeros, never stored) are requested before the first
    // K / V pairs and converted after them.
    float4 qr[QT][KS][2];
    {
        const auto rq = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ubase), 0, 4 * N * row3, 0x00020000);
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int qo = 4 * ((q0 + 16 * qt) * row3 + hoff + 32 * ks + 8 * g);
                qr[qt][ks][0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rq, qo, 0, 0));
                qr[qt][ks][1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rq, qo + 16, 0, 0));
            }
    }
    static_for<PF>([&](auto kc) { fetch(decltype(kc)::value, kc); });  // unconditional (zero rows past N)
    const float qsc = MASKED ? 1.f : sl2;
    vx_u32x4 qh[QT][KS], ql[QT][KS];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const float q8[8] = {qr[qt][ks][0].x, qr[qt][ks][0].y, qr[qt][ks][0].z, qr[qt][ks][0].w,
                                 qr[qt][ks][1].x, qr[qt][ks][1].y, qr[qt][ks][1].z, qr[qt][ks][1].w};
            float v[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = 32 * ks + 8 * g + e < HD ? q8[e] * qsc : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                unsigned hi, lo;
                split2u(v[2 * e], v[2 * e + 1], hi, lo);
                qh[qt][ks][e] = hi;
                ql[qt][ks][e] = lo;
            }
        }
    f32x4 acc[QT][MT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[qt][t] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[QT], lsum[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        m[qt] = MASKED ? -INFINITY : 0.f;
        lsum[qt] = 0.f;
    }
    bool fresh = true;  // unmasked: no chunk processed yet by this wave (wave-uniform)
    ASTAMP(1);
    stash(ch, 0, ic_<0>{});
    __syncthreads();
    ASTAMP(2);

    // chunk c of this wave (2p + kh) from buffer buf
    // MASKED (the encoder): per-key (scale, fill) table, eager online softmax.
    // Unmasked (the decoder): lazy rescaling - the scores are accumulated
    // relative to the running base m (the QK MFMAs start from C = -m) and m
    // moves only on the wave's first chunk or when a score exceeds it by more
    // than kLazyT, so most chunks take no subtraction per score and no
    // rescale of acc / lsum.  Exact up to rounding: numerator and lsum share
    // the base, every weight 2^(s - m) stays <= 2^kLazyT.
    auto process = [&](int buf, int c) {
        const unsigned char* K = Ks0 + buf * P::KBUF;
        const unsigned char* V = Vt0 + buf * P::VBUF;
        const float2* MK = Mk0 + buf * ATT_KC;
        const int lim = N - c * ATT_KC;  // keys 16 kb + 4 g + r >= lim are past the end
        float s[QT][4][4];  // [tile][16-key block][r]: key 16*kb + 4*g + r of query li (base-2 scores)
        float cmax[QT];
        f32x4 c0[QT];
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            cmax[qt] = -INFINITY;
            const float nm = (MASKED || fresh) ? 0.f : -m[qt];
            c0[qt] = f32x4{nm, nm, nm, nm};
        }
#pragma unroll
        for (int kb = 0; kb < 4; ++kb) {
            f32x4 st[QT];
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) st[qt] = c0[qt];
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const unsigned char* kp = K + (16 * kb + li) * KRS + 2 * (32 * ks + 8 * g);
                const vx_u32x4 ah = *reinterpret_cast<const vx_u32x4*>(kp);
                const vx_u32x4 al = *reinterpret_cast<const vx_u32x4*>(kp + 2 * DP);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) st[qt] = mfma_f16(ah, qh[qt][ks], st[qt]);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) st[qt] = mfma_f16(ah, ql[qt][ks], st[qt]);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) st[qt] = mfma_f16(al, qh[qt][ks], st[qt]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                float2 mk = make_float2(1.f, 0.f);
                if constexpr (MASKED) mk = MK[16 * kb + 4 * g + r];
#pragma unroll
                for (int qt = 0; qt < QT; ++qt)
                    // masked: 0 * dot + fill, exactly the fill
                    s[qt][kb][r] = MASKED ? __builtin_fmaf(st[qt][r], mk.x, mk.y) : st[qt][r];
            }
        }
        if constexpr (!MASKED) {
            if (lim < ATT_KC) {  // the last chunk: keys past N score -inf (wave-uniform branch)
#pragma unroll
                for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int qt = 0; qt < QT; ++qt)
                            s[qt][kb][r] = 16 * kb + 4 * g + r < lim ? s[qt][kb][r] : -INFINITY;
            }
        }
        // row maximum: v_max3 over compiler-visible fmaxf (the first readers of
        // the MFMA results must be instructions the compiler sees, so it puts
        // the MFMA -> VALU wait states in front of them)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt)
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
                cmax[qt] = fmaxf(fmaxf(fmaxf(cmax[qt], s[qt][kb][0]), s[qt][kb][1]), fmaxf(s[qt][kb][2], s[qt][kb][3]));
        if constexpr (MASKED) {
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) {
                const float mn = vmax(m[qt], grp4_max(cmax[qt]));
                // raw v_exp_f32 (results below 2^-126 flush to 0: weights that small
                // vanish next to the row's maximum weight 1 anyway)
                const float corr = __builtin_amdgcn_exp2f(m[qt] - mn);  // m = -inf on the first chunk -> 0
                lsum[qt] *= corr;
#pragma unroll
                for (int t = 0; t < MT; ++t) acc[qt][t] *= corr;
#pragma unroll
                for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                    for (int r = 0; r < 4; ++r) s[qt][kb][r] -= mn;
                m[qt] = mn;
            }
        } else {
            bool up = fresh;
#pragma unroll
            for (int qt = 0; qt < QT; ++qt) up = up || cmax[qt] > kLazyT;
            if (__builtin_amdgcn_ballot_w64(up) != 0) {  // wave-uniform: move the base
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    const float cm = grp4_max(cmax[qt]);  // finite: a processed chunk has a live key
                    const float d = fresh ? cm : vmax(cm, 0.f);
                    m[qt] += d;
                    if (!fresh) {
                        const float corr = __builtin_amdgcn_exp2f(-d);
                        lsum[qt] *= corr;
#pragma unroll
                        for (int t = 0; t < MT; ++t) acc[qt][t] *= corr;
                    }
#pragma unroll
                    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[qt][kb][r] -= d;
                }
            }
            fresh = false;
        }
        vx_u32x4 bh[QT][2], bl[QT][2];  // B = P^T of tile qt, 32-key half j
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
            for (int kb = 0; kb < 4; ++kb)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    s[qt][kb][r] = __builtin_amdgcn_exp2f(s[qt][kb][r]);
                    lsum[qt] += s[qt][kb][r];
                }
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                unsigned ph[4], pl[4];  // keys 32j + 4g + e (e < 4), 32j + 16 + 4g + e - 4
                split2u(s[qt][2 * j][0], s[qt][2 * j][1], ph[0], pl[0]);
                split2u(s[qt][2 * j][2], s[qt][2 * j][3], ph[1], pl[1]);
                split2u(s[qt][2 * j + 1][0], s[qt][2 * j + 1][1], ph[2], pl[2]);
                split2u(s[qt][2 * j + 1][2], s[qt][2 * j + 1][3], ph[3], pl[3]);
                bh[qt][j] = vx_u32x4{ph[0], ph[1], ph[2], ph[3]};
                bl[qt][j] = vx_u32x4{pl[0], pl[1], pl[2], pl[3]};
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const unsigned char* vp = V + (16 * t + li) * VRS + 2 * (32 * j + 8 * g);
                const vx_u32x4 vh = *reinterpret_cast<const vx_u32x4*>(vp);
                const vx_u32x4 vl = *reinterpret_cast<const vx_u32x4*>(vp + 2 * ATT_KC);
#pragma unroll
                for (int qt = 0; qt < QT; ++qt) {
                    acc[qt][t] = mfma_f16(vh, bh[qt][j], acc[qt][t]);
                    acc[qt][t] = mfma_f16(vh, bl[qt][j], acc[qt][t]);
                    acc[qt][t] = mfma_f16(vl, bh[qt][j], acc[qt][t]);
                }
            }
    };
    // pair p: buffers 2 (p & 1) + {0, 1}; registers of slot p % PF (unrolled by PF)
    auto pair = [&](int p, auto sc) {
        constexpr int sl = decltype(sc)::value;
        if (2 * p + kh < nch) process(2 * (p & 1) + kh, 2 * p + kh);  // wave-uniform
        if (p + 1 < npair) {
            // the other buffer pair was last read in pair p-1, before the previous barrier
            stash(2 * ((p + 1) & 1) + ch, p + 1, ic_<(sl + 1) % PF>{});
            if (p + PF < npair) fetch(p + PF, ic_<sl>{});  // slot sl is free again
        }
        __syncthreads();
#ifdef ATT_STAMPS
        if (p < 9) ASTAMP(3 + p);
#endif
    };
#pragma unroll 1
    for (int p = 0; p < npair; p += PF)
        static_for<PF>([&](auto kc) {
            if (p + decltype(kc)::value < npair) pair(p + decltype(kc)::value, kc);
        });
    // merge the two key halves: kh 1 hands (m, lsum partial, acc) to kh 0 via LDS
    constexpr int XW = 2 + 4 * MT;
    float* xs = reinterpret_cast<float*>(smem) + (qg * 64 + lane) * (QT * XW);
    if (!MASKED && fresh) {  // this wave processed no chunk (kh 1 of a one-chunk utterance)
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) m[qt] = -INFINITY;
    }
    if (kh == 1) {
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) {
            xs[qt * XW] = m[qt];
            xs[qt * XW + 1] = lsum[qt];
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) xs[qt * XW + 2 + 4 * t + r] = acc[qt][t][r];
        }
    }
    __syncthreads();
    ASTAMP(12);
    if (kh == 1) return;
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
        const float mb = xs[qt * XW], mt = vmax(m[qt], mb);
        const float fa = __builtin_amdgcn_exp2f(m[qt] - mt), fb = __builtin_amdgcn_exp2f(mb - mt);
        float ls = lsum[qt] * fa + xs[qt * XW + 1] * fb;
        ls += __shfl_xor(ls, 16);
        ls += __shfl_xor(ls, 32);
        const int qi = q0 + 16 * qt;
        if (qi < N) {
            const float inv = 1.0f / ls;
            float* orow = out + ((size_t)b * N + qi) * H + hh * HD;
#pragma unroll
            for (int t = 0; t < MT; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    orow[16 * t + 4 * g + r] = (acc[qt][t][r] * fa + xs[qt * XW + 2 + 4 * t + r] * fb) * inv;
        }
    }
    ASTAMP(13);
    ASTAMP_RT(15);
}

#ifdef ATT_STAMPS
extern "C" int32_t m2_debug_stamps_att(void* host, size_t bytes) {
    return (int32_t)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_att_stamps),
                                        bytes < sizeof(g_att_stamps) ? bytes : sizeof(g_att_stamps));
}
#endif

template <int HD, int QT, bool MASKED>
static int32_t launch_att_split_qt(int N, int heads, int B, const float* qkv, const uint8_t* mask, int H, float scale,
                                   float* out, hipStream_t st) {
    static_assert(4 * 64 * QT * (2 + 4 * (HD / 16)) * 4 <= AttSplit<HD>::LDS, "merge area inside the buffers");
    const int nqb = cdiv(N, 64 * QT), ngroups = heads * B;
    const dim3 g1(8 * nqb * ((ngroups + 7) / 8));
    static bool attr = false;
    if (!attr) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(attention_split_kernel<HD, QT, MASKED>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, AttSplit<HD>::LDS));
        attr = true;
    }
    hipLaunchKernelGGL((attention_split_kernel<HD, QT, MASKED>), g1, dim3(512), AttSplit<HD>::LDS, st, qkv, mask, N,
                       H, scale, out, nqb, heads, ngroups);
    M2_LAUNCHED("attention_split_kernel");
    return M2_OK;
}

// QT = 2 halves the K/V bytes each query costs; taken for head_dim <= 32
// while the grid keeps at least one workgroup per CU (M2_ATT_QT=1/2 forces
// one).  tools/probe/att_bench.py, us per launch, QT=1 -> 2: 32x500x64
// 19.0 -> 17.6; hd 48 at QT 2 spills (64x500x96 58.9 -> 301).
template <int HD>
static int32_t launch_att_split(dim3 grid, const float* qkv, const uint8_t* mask, int N, int H, float scale,
                                float* out, hipStream_t st) {
    const int heads = (int)grid.y, B = (int)grid.z;
    const int forced = sw().att_qt;
    // head_dim > 32: two tiles' registers spill past the 256-VGPR cap (400-432
    // B/lane of scratch, 6-8x slower), so those instances are not compiled and
    // M2_ATT_QT=2 is refused for them
    if constexpr (HD <= 32) {
        const bool qt2 = forced ? forced == 2 : (long)cdiv(N, 128) * heads * B >= 256;
        if (qt2) {
            if (mask) return launch_att_split_qt<HD, 2, true>(N, heads, B, qkv, mask, H, scale, out, st);
            return launch_att_split_qt<HD, 2, false>(N, heads, B, qkv, mask, H, scale, out, st);
        }
    } else if (forced == 2) {
        return fail(M2_E_SHAPE, "attention: M2_ATT_QT=2 is not available for head_dim > 32 (it spills)");
    }
    if (mask) return launch_att_split_qt<HD, 1, true>(N, heads, B, qkv, mask, H, scale, out, st);
    return launch_att_split_qt<HD, 1, false>(N, heads, B, qkv, mask, H, scale, out, st);
}

// Any head_dim (the standalone MultiHeadAttention with head_dim outside the
// MFMA instances 16 / 32 / 48 / 64, components.py:42-90): one query per lane,
// the reference's max-subtracted softmax computed online in fp32, the query
// row and its output accumulator in LDS (head_dim <= 256).
__global__ __launch_bounds__(64) void attention_generic_kernel(const float* __restrict__ qkv,
                                                               const uint8_t* __restrict__ key_mask, int N, int H,
                                                               int hd, float scale, float* __restrict__ out) {
    extern __shared__ float gsm[];
    const int b = blockIdx.z, h = blockIdx.y, tid = threadIdx.x, q = blockIdx.x * 64 + tid;
    float* qs = gsm + tid * hd;
    float* as = gsm + 64 * hd + tid * hd;
    const float* base = qkv + (size_t)b * N * 3 * H;
    if (q >= N) return;
    for (int d = 0; d < hd; ++d) {
        qs[d] = base[(size_t)q * 3 * H + h * hd + d];
        as[d] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int j = 0; j < N; ++j) {
        const float* kr = base + (size_t)j * 3 * H + H + h * hd;
        const float* vr = kr + H;
        float dot = 0.f;
        for (int d = 0; d < hd; ++d) dot = fmaf(qs[d], kr[d], dot);
        float sc = dot * scale;
        if (key_mask && key_mask[(size_t)b * N + j] == 0) sc = kMaskFill;
        const float mn = fmaxf(m, sc);
        const float corr = expf(m - mn), pj = expf(sc - mn);
        l = l * corr + pj;
        for (int d = 0; d < hd; ++d) as[d] = fmaf(pj, vr[d], as[d] * corr);
        m = mn;
    }
    const float inv = 1.0f / l;
    float* orow = out + ((size_t)b * N + q) * H + h * hd;
    for (int d = 0; d < hd; ++d) orow[d] = as[d] * inv;
}

// ---------------------------------------------------------------------------
// Host launchers (used by the runtime and by the standalone C entry points).
int32_t launch_embed_pe(const int64_t* ids, const float* emb, const float* pe, int B, int S, int H,
                        int vocab, float* out, const int64_t* lengths, uint8_t* mask, hipStream_t st) {
    const int total = B * S * H;
    const int grid = std::min(cdiv(total, 256), 4096);
    const float scale = (float)std::sqrt((double)H);  // python float H**0.5, cast to fp32 by the mul
    hipLaunchKernelGGL(embed_pe_kernel, dim3(grid), dim3(256), 0, st, ids, emb, pe, B * S, S, H,
                       vocab, scale, out, lengths, mask);
    M2_LAUNCHED("embed_pe_kernel");
    return M2_OK;
}

int32_t launch_embed_pe_scaled(const int64_t* ids, const float* emb, const float* pe, int B, int S,
                               int H, int vocab, float scale, float* out, hipStream_t st) {
    const int total = B * S * H;
    if (total == 0) return M2_OK;
    const int grid = std::min(cdiv(total, 256), 4096);
    hipLaunchKernelGGL(embed_pe_kernel, dim3(grid), dim3(256), 0, st, ids, emb, pe, B * S, S, H,
                       vocab, scale, out, nullptr, nullptr);
    M2_LAUNCHED("embed_pe_kernel");
    return M2_OK;
}

__global__ void add_pe_kernel(const float* __restrict__ x, const float* __restrict__ pe, int R,
                              int S, int H, float* __restrict__ y) {
    const int total = R * H;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
        const int r = i / H, h = i - r * H;
        y[i] = x[i] + pe[(r % S) * H + h];
    }
}

int32_t launch_add_pe(const float* x, const float* pe, int B, int S, int H, float* y, hipStream_t st) {
    const int total = B * S * H;
    if (total == 0) return M2_OK;
    hipLaunchKernelGGL(add_pe_kernel, dim3(std::min(cdiv(total, 256), 4096)), dim3(256), 0, st, x,
                       pe, B * S, S, H, y);
    M2_LAUNCHED("add_pe_kernel");
    return M2_OK;
}

int32_t launch_layer_norm(const float* x, const float* g, const float* b, int R, int K, float* y,
                          hipStream_t st) {
    if (R == 0) return M2_OK;
    hipLaunchKernelGGL(layer_norm_kernel, dim3(cdiv(R, 4)), dim3(256), 0, st, x, g, b, R, K, y);
    M2_LAUNCHED("layer_norm_kernel");
    return M2_OK;
}

int32_t launch_linear(const float* x, const float* gamma, const float* beta, const float* w,
                      const float* bias, const float* res, int act, int R, int K, int N, float* y,
                      hipStream_t st) {
    M2_CHECK_SHAPE(K % 8 == 0 && K <= 256 && K > 0, "linear: K must be a multiple of 8 and <= 256");
    if (R == 0 || N == 0) return M2_OK;
    const size_t lds = sizeof(float) * (2 * LIN_TILE * (K + 4) + 2 * LIN_TILE);
    static bool attr_set = false;
    if (!attr_set) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(linear_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    hipLaunchKernelGGL(linear_kernel, dim3(cdiv(R, LIN_TILE), cdiv(N, LIN_TILE)), dim3(256), lds,
                       st, x, gamma, beta, w, bias, res, act, R, K, N, y);
    M2_LAUNCHED("linear_kernel");
    return M2_OK;
}

int32_t launch_attention(const float* qkv, const uint8_t* mask, int B, int N, int H, int heads,
                         float* out, hipStream_t st, bool force_f32) {
    M2_CHECK_SHAPE(heads > 0 && H % heads == 0, "attention: H % heads != 0");
    const int hd = H / heads;
    if (B == 0 || N == 0) return M2_OK;
    const float scale = (float)(1.0 / std::sqrt((double)hd));  // components.py:52 (self.scale), fp32 at the mul
    dim3 grid(cdiv(N, 64), heads, B);
    // split-f16 MFMA by default; M2_ATT_F32=1: the exact-f32 MFMA kernel
    // (switch table, m2_common.h)
    const bool f32 = force_f32 || sw().att_f32;
    // float4 reads of q/k/v rows in the MFMA kernels: H and the head offsets 16-B aligned
    if (H % 4 != 0 || (hd != 16 && hd != 32 && hd != 48 && hd != 64)) {  // no MFMA instance: the generic kernel
        M2_CHECK_SHAPE(hd <= 256, "attention: head_dim must be at most 256");
        const size_t lds = (size_t)2 * 64 * hd * sizeof(float);
        static bool attr = false;
        if (!attr) {
            M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(attention_generic_kernel),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, 2 * 64 * 256 * 4));
            attr = true;
        }
        hipLaunchKernelGGL(attention_generic_kernel, grid, dim3(64), lds, st, qkv, mask, N, H, hd, scale, out);
        M2_LAUNCHED("attention_generic_kernel");
        return M2_OK;
    }
    if (!f32) switch (hd) {
            case 16: return launch_att_split<16>(grid, qkv, mask, N, H, scale, out, st);
            case 32: return launch_att_split<32>(grid, qkv, mask, N, H, scale, out, st);
            case 48: return launch_att_split<48>(grid, qkv, mask, N, H, scale, out, st);
            case 64: return launch_att_split<64>(grid, qkv, mask, N, H, scale, out, st);
            default: break;
        }
    switch (hd) {
        case 16: hipLaunchKernelGGL(attention_kernel<16>, grid, dim3(256), 0, st, qkv, mask, N, H, scale, out); break;
        case 32: hipLaunchKernelGGL(attention_kernel<32>, grid, dim3(256), 0, st, qkv, mask, N, H, scale, out); break;
        case 48: hipLaunchKernelGGL(attention_kernel<48>, grid, dim3(256), 0, st, qkv, mask, N, H, scale, out); break;
        case 64: hipLaunchKernelGGL(attention_kernel<64>, grid, dim3(256), 0, st, qkv, mask, N, H, scale, out); break;
        default: return fail(M2_E_SHAPE, "attention: head_dim must be 16, 32, 48 or 64");
    }
    M2_LAUNCHED("attention_kernel");
    return M2_OK;
}

}  // namespace m2
