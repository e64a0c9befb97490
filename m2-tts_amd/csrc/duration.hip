// Duration predictor and length regulator (gfx950).
//
//   duration_kernel   DurationPredictor: 2x[Conv1d k3 -> BN(eval) -> ReLU],
//                     Conv1d k1 -> softplus                tts_model.py:99-117,
//                                                          components.py:163-174,214-223
//   lr_count_kernel   int(trunc(d)) per phoneme, per-utterance prefix sums,
//                     totals and batch max                  tts_model.py:146-166
//   lr_expand_kernel  frame -> phoneme gather + zero pad / truncate
//                                                           tts_model.py:146-178
// The reference's regulator is a Python double loop with one host sync per
// phoneme; here it is one scan kernel and one gather kernel, and the only
// host round trip left is the caller's read of T_max to size the output.
#include <algorithm>
#include <cstdlib>

#include "m2_common.h"

namespace m2 {

// ---------------------------------------------------------------------------
// One workgroup (8 waves) per (utterance, 14-phoneme tile): 8 x 32 = 256
// workgroups at B=32, S=100, one per CU.  Both k=3 convs are GEMMs on the
// exact-f32 MFMA (v_mfma_f32_16x16x4_f32): rows = 16 positions (one 16-row
// block), columns = 16 output channels per wave (n-block nb = wave; H=128
// has 8), K = (tap, channel) = 3H.  A = activation rows in LDS (stride H+2:
// a ds_read_b32 half-wave of 16 rows x 2 k-lanes hits 32 banks), B = conv
// weights packed in B-fragment order (m2_model_create; L2-resident).  conv1
// covers positions [s0-1, s0+15) so conv2 can produce [s0, s0+14) (14 of its
// 16 rows; outside [0,S) conv1 stores the zero padding conv2 sees).
// Epilogue: +bias, BatchNorm (alpha = gamma/sqrt(var+eps), beta' = beta -
// mean*alpha, the inference form PyTorch's CPU batch_norm evaluates), ReLU.
// Then the k=1 projection (one wave per phoneme) and softplus.  The encoder
// output is read in its [B,S,H] layout (the reference's transpose(1,2) is a
// view).  (Was 4 waves x 30-phoneme tiles, two row blocks per wave: 128
// workgroups with 2x longer per-wave MFMA chains, 15.5 us at B=32.)
constexpr int DUR_TS = 14;
constexpr int DUR_WAVES = 8;

typedef float dur_f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) unsigned gu32;  // global (never flat) agent-scope accesses

// The frame count fused into the duration kernel (duration_kernel<H, LN, true>)
struct DurCount {
    float scale;
    int32_t *cum, *T, *Tmax;
    unsigned* ticket;  // zero between calls (the last workgroup resets it)
    int32_t* mbox;     // host-mapped (seq, T_max) mailbox or null
    int32_t seq;
};

__device__ __forceinline__ int frames_from(float d, float scale) {
    const float v = d * scale;                       // fp32 product, as dur*scale
    if (!(v >= 1.0f)) return 0;                      // also NaN -> 0
    return v >= 1073741824.f ? 1073741824 : (int)v;  // int() truncates toward zero
}

__device__ __forceinline__ int frames_of(const void* dur, int is_int, float scale, size_t i) {
    if (is_int) {
        const int v = static_cast<const int32_t*>(dur)[i];
        return v > 0 ? v : 0;
    }
    return frames_from(static_cast<const float*>(dur)[i], scale);
}

// This wave's weight fragments of one conv (n-block = wave), requested at
// kernel start so their L2 round trips overlap the encoder-row loads and the
// LayerNorm instead of sitting between the barriers (H <= 128: one n-block
// per wave).
template <int H>
struct DurW {
    float4 w[3 * H / 16];
};
template <int H>
__device__ __forceinline__ void dur_wload(const float4* __restrict__ Wp, DurW<H>& r) {
    static_assert(H / 16 <= DUR_WAVES, "one n-block per wave");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave < H / 16) {
        const float4* wp = Wp + (size_t)wave * (3 * H / 16) * 64 + lane;
#pragma unroll
        for (int k = 0; k < 3 * H / 16; ++k) r.w[k] = wp[k * 64];
    }
}

template <int H, int RBK>
__device__ __forceinline__ void dur_conv_mfma(const float* in, const DurW<H>& W, const float* __restrict__ b,
                                              const float* __restrict__ a, const float* __restrict__ c, float* out,
                                              int pos0, int S) {
    constexpr int XS = H + 2;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    if (wave < H / 16) {
        const int nb = wave;
        // RBK 16-position row blocks share every weight fragment (independent
        // accumulation chains)
        dur_f32x4 acc[RBK];
#pragma unroll
        for (int rb = 0; rb < RBK; ++rb) acc[rb] = dur_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 3; ++tap) {
#pragma unroll
            for (int s4 = 0; s4 < H / 16; ++s4) {
                const float4 w = W.w[tap * (H / 16) + s4];
                const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int rb = 0; rb < RBK; ++rb)
                        acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            in[(16 * rb + i + tap) * XS + g + (4 * s4 + q) * 4], wv[q], acc[rb], 0, 0, 0);
            }
        }
        const int co = nb * 16 + i;
        const float bb = b[co], aa = a[co], cc = c[co];
#pragma unroll
        for (int rb = 0; rb < RBK; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * rb + 4 * g + r, s = pos0 + row;
                float v = (acc[rb][r] + bb) * aa + cc;
                v = v > 0.f ? v : 0.f;
                out[row * XS + co] = (s >= 0 && s < S) ? v : 0.f;
            }
    }
}

// Split-f16 form of the convs (the inference path's fused-LayerNorm
// launches when the model's static range bound allows, m2_model_create):
// every fp32 operand as f16 hi + lo, three v_mfma_f32_16x16x32_f16 per 32-deep
// K step (hi.hi + lo.hi + hi.lo, fp32 accumulate) - 48 cycles of matrix core
// per K step where the exact-f32 MFMA needs 8 x 32.  Activation rows in LDS
// as [hi: H f16 | lo: H f16 | 32 B pad] (stride dur_rs(H): conflict-free
// ds_read_b128 of 16 rows); the weights (pack_bfrag_split of [co][tap*H + ci])
// are the B operand: lane (output channel co, k-group g) holds 8 K elements.
typedef unsigned dur_u32x4 __attribute__((ext_vector_type(4)));
constexpr int dur_rs(int H) { return 4 * H + 32; }
template <int H>
struct DurWS {
    dur_u32x4 w[3 * H / 32][2];
};
template <int H>
__device__ __forceinline__ void dur_wload_split(const float* __restrict__ Wp, DurWS<H>& r) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (wave < H / 16) {
        const dur_u32x4* p = reinterpret_cast<const dur_u32x4*>(Wp) + (size_t)wave * (3 * H / 32) * 128 + lane;
#pragma unroll
        for (int ks = 0; ks < 3 * H / 32; ++ks) {
            r.w[ks][0] = p[ks * 128];
            r.w[ks][1] = p[ks * 128 + 64];
        }
    }
}
__device__ __forceinline__ dur_f32x4 dur_mfma16(dur_u32x4 a, dur_u32x4 b, dur_f32x4 c) {
    typedef _Float16 h8 __attribute__((ext_vector_type(8)));
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}
// One value as f16 hi / lo halves at row p, column k of a split row buffer.
template <int H>
__device__ __forceinline__ void dur_put_split(unsigned char* rows, int p, int k, float v) {
    const _Float16 hi = (_Float16)v, lo = (_Float16)(v - (float)hi);
    *reinterpret_cast<_Float16*>(rows + p * dur_rs(H) + 2 * k) = hi;
    *reinterpret_cast<_Float16*>(rows + p * dur_rs(H) + 2 * H + 2 * k) = lo;
}
// The conv of dur_conv_mfma on split rows `in`; out: split rows (SPLIT_OUT,
// conv1 -> conv2's input) or fp32 rows of stride H + 2 (conv2 -> projection).
template <int H, int RBK, bool SPLIT_OUT>
__device__ __forceinline__ void dur_conv_split(const unsigned char* in, const DurWS<H>& W, const float* __restrict__ b,
                                               const float* __restrict__ a, const float* __restrict__ c, void* out,
                                               int pos0, int S) {
    constexpr int KS = 3 * H / 32, KPT = H / 32;  // K steps, K steps per tap
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
    if (wave < H / 16) {
        const int nb = wave;
        dur_f32x4 acc[RBK];
#pragma unroll
        for (int rb = 0; rb < RBK; ++rb) acc[rb] = dur_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int tap = ks / KPT, ci0 = 32 * (ks - tap * KPT);
            dur_u32x4 xh[RBK], xl[RBK];
#pragma unroll
            for (int rb = 0; rb < RBK; ++rb) {
                const unsigned char* p = in + (16 * rb + i + tap) * dur_rs(H) + 2 * (ci0 + 8 * g);
                xh[rb] = *reinterpret_cast<const dur_u32x4*>(p);
                xl[rb] = *reinterpret_cast<const dur_u32x4*>(p + 2 * H);
            }
#pragma unroll
            for (int rb = 0; rb < RBK; ++rb) acc[rb] = dur_mfma16(xh[rb], W.w[ks][0], acc[rb]);
#pragma unroll
            for (int rb = 0; rb < RBK; ++rb) acc[rb] = dur_mfma16(xl[rb], W.w[ks][0], acc[rb]);
#pragma unroll
            for (int rb = 0; rb < RBK; ++rb) acc[rb] = dur_mfma16(xh[rb], W.w[ks][1], acc[rb]);
        }
        const int co = nb * 16 + i;
        const float bb = b[co], aa = a[co], cc = c[co];
#pragma unroll
        for (int rb = 0; rb < RBK; ++rb)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * rb + 4 * g + r, s = pos0 + row;
                float v = (acc[rb][r] + bb) * aa + cc;
                v = v > 0.f ? v : 0.f;
                v = (s >= 0 && s < S) ? v : 0.f;
                if constexpr (SPLIT_OUT) dur_put_split<H>(static_cast<unsigned char*>(out), row, co, v);
                else static_cast<float*>(out)[row * (H + 2) + co] = v;
            }
    }
}

__device__ __forceinline__ int32_t sat32(long long v) { return (int32_t)min(v, (long long)INT32_MAX); }

// The length regulator's frame count run by the duration kernel's last
// workgroup: the same arithmetic as lr_count_kernel<true> - frames_from per
// phoneme, 64-bit prefix sums saturated at INT32_MAX into cum[b, 0..S], totals
// T[b], Tmax, the ticket reset for the next call and the optional host mailbox
// post.  The durations were stored sc1 by the other workgroups of this launch,
// so every load of them is an sc1 load; the whole batch's frame counts are
// fetched in one pass (8 loads in flight per lane) into LDS, then one wave per
// utterance scans them.  B * S <= kDurCountMax.
constexpr int kDurCountMax = 8192;
__device__ __forceinline__ float dur_ld(const float* d, size_t i) {
    return __uint_as_float(__hip_atomic_load((gu32*)(d + i), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ void count_frames(const float* __restrict__ dur, int B, int S, const DurCount& dc) {
    __shared__ int32_t fr[kDurCountMax];
    __shared__ long long wmax[DUR_WAVES];
    constexpr int NT = 64 * DUR_WAVES, U = 8;
    const int n = B * S, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (int i0 = threadIdx.x; i0 < n; i0 += U * NT) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i0 + u * NT < n ? dur_ld(dur, (size_t)i0 + u * NT) : 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i0 + u * NT < n) fr[i0 + u * NT] = frames_from(v[u], dc.scale);
    }
    __syncthreads();
    const int per = (S + 63) / 64, lo = min(S, lane * per), hi = min(S, lo + per);
    long long mx = 0;
    for (int b = wave; b < B; b += DUR_WAVES) {
        const int32_t* f = fr + b * S;
        long long sum = 0;
        for (int s = lo; s < hi; ++s) sum += f[s];
        long long inc = sum;  // inclusive scan over the wave's lanes
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const long long v = __shfl_up(inc, off);
            if (lane >= off) inc += v;
        }
        long long run = inc - sum;
        int32_t* c = dc.cum + (size_t)b * (S + 1);
        if (lane == 0) c[0] = 0;
        for (int s = lo; s < hi; ++s) {
            run += f[s];
            c[s + 1] = sat32(run);
        }
        const long long total = __shfl(inc, 63);
        if (lane == 0) dc.T[b] = sat32(total);
        mx = max(mx, total);
    }
    if (lane == 0) wmax[wave] = mx;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 0; w < DUR_WAVES; ++w) mx = max(mx, wmax[w]);
        const int32_t tm = sat32(mx);
        *dc.Tmax = tm;
        __hip_atomic_store((gu32*)dc.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dc.mbox) {  // null: T_max stays on the device (m2_inference_front_dev)
            __hip_atomic_store(dc.mbox + 1, tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(dc.mbox, dc.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// LN: `enc` is the encoder's last layer output BEFORE its final LayerNorm
// (tts_model.py:87); each workgroup normalises its rows while loading them
// (one wave per row, the halo rows redundantly) and stores its own 14
// normalised rows to enc_out - the encoder output the length regulator
// expands - in place of a separate layer_norm_kernel launch.
// PERS (large grids, no fused count): a grid of at most one workgroup per CU
// walks the tiles (tile t: utterance t / ntx, phonemes (t % ntx) * TS ..),
// loading both convs' weight fragments once instead of once per tile - at
// B=128 S=520 the 2,304 30-phoneme tiles streamed 0.44 MB of split weights
// each (1 GB per launch from L2).
template <int H, bool LN, bool COUNT, int RBK, bool SPL = false, bool PERS = false>
__global__ __launch_bounds__(64 * DUR_WAVES) void duration_kernel(
    const float* __restrict__ enc, int S, const float4* __restrict__ w1, const float* __restrict__ b1,
    const float* __restrict__ a1, const float* __restrict__ c1, const float4* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ a2, const float* __restrict__ c2,
    const float* __restrict__ pw, const float* __restrict__ pb, float* __restrict__ dur,
    const float* __restrict__ lng, const float* __restrict__ lnb, float* __restrict__ enc_out, DurCount dc,
    int ntiles) {
    static_assert(!(PERS && COUNT), "the fused count's ticket counts workgroups of a one-tile-each grid");
    constexpr int XS = H + 2, NT = 64 * DUR_WAVES;
    constexpr int TS = 16 * RBK - 2, NX = TS + 4;  // phonemes per tile, input rows with the halo
    static_assert(!SPL || LN, "the split convs take the fused LayerNorm's bounded rows");
    // SPL: X and Y1 as split rows (stride dur_rs(H) bytes) in the same arrays
    constexpr int XF = SPL ? (dur_rs(H) + 3) / 4 : XS;  // floats per row of X / Y1
    __shared__ __attribute__((aligned(16))) float X[NX * XF];   // positions s0-2 .. s0+TS+1
    __shared__ __attribute__((aligned(16))) float Y1[NX * XF];  // s0-1 .. s0+TS (+2 zero rows read by conv2's unused rows)
    __shared__ float Y2[16 * RBK * XS];  // s0 .. s0+TS-1 (+2 unused)
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    DurW<H> W1, W2;
    DurWS<H> V1, V2;
    if constexpr (SPL) {
        dur_wload_split<H>(reinterpret_cast<const float*>(w1), V1);
        dur_wload_split<H>(reinterpret_cast<const float*>(w2), V2);
    } else {
        dur_wload<H>(w1, W1);
        dur_wload<H>(w2, W2);
    }
    auto tile = [&](const int b, const int s0) {
    const float* e = enc + (size_t)b * S * H;
    if constexpr (LN) {
        // every row of this wave is loaded before the first is normalised (one
        // memory round trip per wave instead of one per row)
        constexpr int NR = (NX + DUR_WAVES - 1) / DUR_WAVES, KP = (H + 63) / 64;
        float xv[NR][KP];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int p = wave + j * DUR_WAVES, s = s0 - 2 + p;
            const float* xr = e + (size_t)min(max(s, 0), S - 1) * H;
#pragma unroll
            for (int q = 0; q < KP; ++q) xv[j][q] = (lane + 64 * q < H) ? xr[lane + 64 * q] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int p = wave + j * DUR_WAVES, s = s0 - 2 + p;
            if (p >= NX) break;
            float* d = X + p * XF;
            if (s >= 0 && s < S) {
                float mean, rstd;
                ln_row_stats_regs<KP>(xv[j], H, lane, mean, rstd);
                float* yo = (p >= 2 && p < 2 + TS) ? enc_out + ((size_t)b * S + s) * H : nullptr;
#pragma unroll
                for (int q = 0; q < KP; ++q) {
                    const int k = lane + 64 * q;
                    if (k < H) {
                        const float y = ln_apply(xv[j][q], mean, rstd, lng[k], lnb[k]);
                        if constexpr (SPL) dur_put_split<H>(reinterpret_cast<unsigned char*>(X), p, k, y);
                        else d[k] = y;
                        if (yo) yo[k] = y;
                    }
                }
            } else {
                for (int k = lane; k < H; k += 64) {
                    if constexpr (SPL) dur_put_split<H>(reinterpret_cast<unsigned char*>(X), p, k, 0.f);
                    else d[k] = 0.f;
                }
            }
        }
    } else {
        for (int idx = tid; idx < NX * (H / 4); idx += NT) {
            const int p = idx / (H / 4), c4 = (idx - p * (H / 4)) * 4, s = s0 - 2 + p;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (s >= 0 && s < S) v = *reinterpret_cast<const float4*>(e + (size_t)s * H + c4);
            float* d = X + p * XS + c4;
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        }
    }
    for (int idx = tid; idx < 2 * XF; idx += NT) Y1[16 * RBK * XF + idx] = 0.f;
    __syncthreads();
    if constexpr (SPL) {
        dur_conv_split<H, RBK, true>(reinterpret_cast<const unsigned char*>(X), V1, b1, a1, c1, Y1, s0 - 1, S);
        __syncthreads();
        dur_conv_split<H, RBK, false>(reinterpret_cast<const unsigned char*>(Y1), V2, b2, a2, c2, Y2, s0, S);
    } else {
        dur_conv_mfma<H, RBK>(X, W1, b1, a1, c1, Y1, s0 - 1, S);
        __syncthreads();
        dur_conv_mfma<H, RBK>(Y1, W2, b2, a2, c2, Y2, s0, S);
    }
    __syncthreads();
    // k=1 projection H -> 1: one wave per phoneme, shuffle reduction.
    for (int p = wave; p < TS; p += DUR_WAVES) {
        const int s = s0 + p;
        float acc = 0.f;
        for (int ci = lane; ci < H; ci += 64) acc = fmaf(pw[ci], Y2[p * XS + ci], acc);
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0 && s < S) {
            const float x = acc + pb[0];
            // F.softplus(beta=1, threshold=20)
            const float d = x > 20.f ? x : log1pf(expf(x));
            if constexpr (COUNT)  // write-through (sc1): the last workgroup reads it in this launch
                __hip_atomic_store((gu32*)(dur + (size_t)b * S + s), __float_as_uint(d), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            else
                dur[(size_t)b * S + s] = d;
        }
    }
    };
    if constexpr (PERS) {
        const int ntx = (S + TS - 1) / TS;
#pragma unroll 1
        for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
            tile(t / ntx, (t % ntx) * TS);
            __syncthreads();  // the next tile's rows overwrite X / Y1 / Y2
        }
    } else {
        tile(blockIdx.y, blockIdx.x * TS);
    }
    if constexpr (COUNT) {
        // hand-off to the last workgroup (MI355X_MICROARCH.md, inter-workgroup
        // visibility, table row 1): every storing wave drains its sc1 stores,
        // the barrier orders them before lane 0's ticket add, and the workgroup
        // whose add returns the last ticket reads every duration with sc1 loads
        // (no fences: no L2 write-back per workgroup, which made round 1's
        // fused form slower than the separate count kernel)
        // This hand-off relies on gfx950's cache behaviour, not on the C++
        // memory model: sc1 stores write through to the device-coherent
        // level and retire in order before s_waitcnt vmcnt(0) returns, and sc1
        // loads bypass the non-coherent caches; the relaxed atomics carry no
        // ordering of their own.  Other targets must use lr_count_kernel.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "duration_kernel<COUNT=true>: the fused frame count's hand-off is written for gfx950 only"
#endif
        __shared__ int last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
            last = __hip_atomic_fetch_add((gu32*)dc.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   gridDim.x * gridDim.y - 1;
        __syncthreads();
        if (last) count_frames(dur, gridDim.y, S, dc);
    }
}

// ---------------------------------------------------------------------------
// One wave per utterance: n[s] = max(0, trunc(d[s]*scale)) for ceil(S/64)
// consecutive phonemes per lane, a shuffle scan of the lanes' sums (no LDS,
// no barrier: was 256 threads and a Hillis-Steele scan in LDS, 16 barriers,
// 6.0 us at stage1 B=32 S=100), exclusive prefix sums into cum[b, 0..S],
// T[b] = cum[b, S]; atomicMax into Tmax (zeroed by the launcher's memset node).


// SYNC: no pre-zeroed Tmax / atomicMax: the last workgroup to finish (a
// ticket counter, reset by that workgroup for the next call) reduces the
// totals, stores Tmax and posts (seq, Tmax) to a host-mapped mailbox with
// system-scope stores (Tmax first, then seq with release order), which the
// host polls instead of a device->host copy and a stream synchronisation.
// Frame counts are clamped to 2^30 per phoneme and summed in 64 bits; the
// stored prefix sums and totals saturate at INT32_MAX (the host rejects a
// T_max above m2's frame limit with M2_E_SHAPE instead of wrapping).
template <bool SYNC>
__global__ __launch_bounds__(64) void lr_count_kernel(const void* __restrict__ dur, int is_int, float scale, int S,
                                                      int32_t* __restrict__ cum, int32_t* __restrict__ T,
                                                      int32_t* __restrict__ Tmax, unsigned* __restrict__ ticket,
                                                      int32_t* __restrict__ mbox, int32_t seq) {
    const int b = blockIdx.x, lane = threadIdx.x;
    const int per = (S + 63) / 64, lo = min(S, lane * per), hi = min(S, lo + per);
    const size_t base = (size_t)b * S;
    long long sum = 0;
    for (int s = lo; s < hi; ++s) sum += frames_of(dur, is_int, scale, base + s);
    long long inc = sum;  // inclusive scan over the lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const long long v = __shfl_up(inc, off);
        if (lane >= off) inc += v;
    }
    long long run = inc - sum;  // exclusive prefix of this lane's phonemes
    int32_t* c = cum + (size_t)b * (S + 1);
    if (lane == 0) c[0] = 0;
    for (int s = lo; s < hi; ++s) {
        run += frames_of(dur, is_int, scale, base + s);
        c[s + 1] = sat32(run);
    }
    const int32_t total = sat32(__shfl(inc, 63));
    if constexpr (!SYNC) {
        if (lane == 0) {
            T[b] = total;
            atomicMax(Tmax, total);
        }
    } else {
        bool last = false;
        if (lane == 0) {
            __hip_atomic_store(T + b, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __atomic_thread_fence(__ATOMIC_RELEASE);  // totals before the ticket
            last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
        }
        if (__shfl(last ? 1 : 0, 0)) {  // every other workgroup's total is visible
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (all lanes: lane 0's ticket was the acquire)
            long long m = 0;
            for (int i = lane; i < (int)gridDim.x; i += 64)
                m = max(m, (long long)__hip_atomic_load(T + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) m = max(m, __shfl_xor(m, off));
            if (lane == 0) {
                const int32_t tm = sat32(m);
                *Tmax = tm;
                __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (mbox) {  // null: T_max stays on the device (m2_inference_front_dev)
                    __hip_atomic_store(mbox + 1, tm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(mbox, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
}

// Frame gather: a workgroup owns LR_TF frames of one utterance.  The
// utterance's prefix sums go to LDS once, one thread per frame finds its
// phoneme there (binary search: smallest s with cum[s+1] > t; frames at or
// past cum[S] are zero padding), then the whole workgroup copies the rows in
// 16-B pieces.  (Was one wave per frame searching global memory: 7 dependent
// L2 round trips per frame.)
constexpr int LR_TF = 64;

__global__ __launch_bounds__(256) void lr_expand_kernel(const float* __restrict__ enc,
                                                        const int32_t* __restrict__ cum, int S,
                                                        int H, int T_out, float* __restrict__ out) {
    extern __shared__ int32_t cs[];  // [S + 1] prefix sums, then [LR_TF] source phoneme per frame
    int32_t* src = cs + S + 1;
    const int b = blockIdx.y, t0 = blockIdx.x * LR_TF, tid = threadIdx.x;
    const int32_t* c = cum + (size_t)b * (S + 1);
    for (int i = tid; i <= S; i += 256) cs[i] = c[i];
    __syncthreads();
    if (tid < LR_TF) {
        const int t = t0 + tid;
        int sp = -1;
        if (t < T_out && t < cs[S]) {
            int lo = 0, hi = S - 1;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (cs[mid + 1] > t) hi = mid; else lo = mid + 1;
            }
            sp = lo;
        }
        src[tid] = sp;
    }
    __syncthreads();
    const int nf = min(LR_TF, T_out - t0);
    if ((H & 3) == 0) {
        const int H4 = H / 4;
        for (int i = tid; i < nf * H4; i += 256) {
            const int f = i / H4, c4 = i - f * H4, sp = src[f];
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (sp >= 0) v = *reinterpret_cast<const float4*>(enc + ((size_t)b * S + sp) * H + 4 * c4);
            *reinterpret_cast<float4*>(out + ((size_t)b * T_out + t0 + f) * H + 4 * c4) = v;
        }
    } else {
        for (int i = tid; i < nf * H; i += 256) {
            const int f = i / H, h = i - f * H, sp = src[f];
            out[((size_t)b * T_out + t0 + f) * H + h] = sp >= 0 ? enc[((size_t)b * S + sp) * H + h] : 0.f;
        }
    }
}

// ---------------------------------------------------------------------------
// p: w1 (packed), b1, alpha1, beta1, w2 (packed), b2, alpha2, beta2, proj_w, proj_b
namespace {
int32_t duration_launch(const float* enc, int B, int S, int H, const float* const* p, float* dur, hipStream_t st,
                        const float* ln_g, const float* ln_b, float* enc_out, const DurCount* dc,
                        const float* const* wsplit) {
    if (B == 0 || S == 0) return M2_OK;
    // 14-phoneme tiles (one 16-position row block per wave) while they fit one
    // round of the CUs; beyond, 30-phoneme tiles (two row blocks sharing each
    // weight fragment): half the workgroups, each streaming the same weights.
    // M2_DUR_RB=1|2 forces one (switch table, m2_common.h).
    int rbk = (long)B * cdiv(S, DUR_TS) > 256 ? 2 : 1;
    if (sw().dur_rb) rbk = sw().dur_rb;
    dim3 grid(cdiv(S, 16 * rbk - 2), B);
    const dim3 blk(64 * DUR_WAVES);
    // persistent tiles (PERS) past two rounds of the CUs, without the fused
    // count (M2_DUR_PERS=0 never)
    const int ntiles = (int)grid.x * B;
    static int ncu = 0;
    if (!ncu) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
    }
    // (not at H = 128: both convs' weight fragments held for the whole walk
    // spill there; its tiles keep one tile per workgroup)
    const bool pers = !dc && sw().dur_pers && ntiles > 2 * ncu && H <= 96;
    if (pers) grid = dim3(ncu, 1);
    auto f4 = [](const float* q) { return reinterpret_cast<const float4*>(q); };
    const DurCount none{};
    // split-f16 convs: the fused-LayerNorm (inference) launches of a model
    // whose static bound allows them (wsplit = its split weight packs)
    const bool spl = wsplit && enc_out;
#define M2_DUR_K(HH, LL, CC, RR, SP, PP)                                                                            \
    hipLaunchKernelGGL((duration_kernel<HH, LL, CC, RR, SP, PP>), grid, blk, 0, st, enc, S,                      \
                       f4(SP ? wsplit[0] : p[0]), p[1], p[2], p[3], f4(SP ? wsplit[1] : p[4]), p[5], p[6], p[7],    \
                       p[8], p[9], dur, LL ? ln_g : nullptr, LL ? ln_b : nullptr, LL ? enc_out : nullptr,           \
                       dc ? *dc : none, ntiles)
#define M2_DUR_L(HH, LL, CC, RR, SP)                      \
    do {                                                  \
        if constexpr (!CC && HH <= 96) {                  \
            if (pers) M2_DUR_K(HH, LL, CC, RR, SP, true); \
            else M2_DUR_K(HH, LL, CC, RR, SP, false);     \
        } else {                                          \
            M2_DUR_K(HH, LL, CC, RR, SP, false);          \
        }                                                 \
    } while (0)
#define M2_DUR_R(HH, LL, CC, SP)                      \
    if (rbk == 2) M2_DUR_L(HH, LL, CC, 2, SP);        \
    else M2_DUR_L(HH, LL, CC, 1, SP)
#define M2_DUR(HH)                                                      \
    case HH:                                                            \
        if (enc_out && dc) {                                            \
            if (spl) M2_DUR_R(HH, true, true, true);                    \
            else M2_DUR_R(HH, true, true, false);                       \
        } else if (enc_out) {                                           \
            if (spl) M2_DUR_R(HH, true, false, true);                   \
            else M2_DUR_R(HH, true, false, false);                      \
        } else if (dc) M2_DUR_R(HH, false, true, false);                \
        else M2_DUR_R(HH, false, false, false);                         \
        break;
    switch (H) {
        M2_DUR(32)
        M2_DUR(64)
        M2_DUR(96)
        M2_DUR(128)
        default: return fail(M2_E_SHAPE, "duration: hidden_dim must be 32, 64, 96 or 128");
    }
#undef M2_DUR_R
#undef M2_DUR
#undef M2_DUR_L
#undef M2_DUR_K
    M2_LAUNCHED("duration_kernel");
    return M2_OK;
}
}  // namespace

// p: w1 (packed), b1, alpha1, beta1, w2 (packed), b2, alpha2, beta2, proj_w, proj_b
int32_t launch_duration(const float* enc, int B, int S, int H, const float* const* p, float* dur, hipStream_t st,
                        const float* ln_g, const float* ln_b, float* enc_out, const float* const* wsplit) {
    return duration_launch(enc, B, S, H, p, dur, st, ln_g, ln_b, enc_out, nullptr, wsplit);
}

// The same launch with the length regulator's count (lr_count_kernel<true>'s
// outputs: cum, T, Tmax, ticket reset, mailbox post) run by its last
// workgroup - one launch fewer per inference.  0 < B * S <= kDurCountMax.
bool duration_count_fusable(int B, int S) { return B > 0 && S > 0 && (long)B * S <= kDurCountMax; }

int32_t launch_duration_count(const float* enc, int B, int S, int H, const float* const* p, float* dur,
                              hipStream_t st, const float* ln_g, const float* ln_b, float* enc_out, float scale,
                              int32_t* cum, int32_t* T, int32_t* Tmax, unsigned* ticket, int32_t* mbox, int32_t seq,
                              const float* const* wsplit) {
    M2_CHECK_ARG(B > 0 && S > 0 && (long)B * S <= kDurCountMax, "duration + count: batch too large to fuse");
    const DurCount dc{scale, cum, T, Tmax, ticket, mbox, seq};
    return duration_launch(enc, B, S, H, p, dur, st, ln_g, ln_b, enc_out, &dc, wsplit);
}

int32_t launch_lr_count(const void* dur, int is_int, float scale, int B, int S, int32_t* cum,
                        int32_t* T, int32_t* Tmax, hipStream_t st) {
    M2_HIP(hipMemsetAsync(Tmax, 0, sizeof(int32_t), st));
    if (B == 0) return M2_OK;
    hipLaunchKernelGGL(lr_count_kernel<false>, dim3(B), dim3(64), 0, st, dur, is_int, scale, S, cum, T,
                       Tmax, nullptr, nullptr, 0);
    M2_LAUNCHED("lr_count_kernel");
    return M2_OK;
}

int32_t launch_lr_count_sync(const void* dur, int is_int, float scale, int B, int S, int32_t* cum, int32_t* T,
                             int32_t* Tmax, unsigned* ticket, int32_t* mbox, int32_t seq, hipStream_t st) {
    hipLaunchKernelGGL(lr_count_kernel<true>, dim3(B), dim3(64), 0, st, dur, is_int, scale, S, cum, T, Tmax,
                       ticket, mbox, seq);
    M2_LAUNCHED("lr_count_kernel");
    return M2_OK;
}

int32_t launch_lr_expand(const float* enc, const int32_t* cum, int B, int S, int H, int T_out,
                         float* out, hipStream_t st) {
    if (B == 0 || T_out == 0) return M2_OK;
    const size_t lds = ((size_t)S + 1 + LR_TF) * sizeof(int32_t);
    M2_CHECK_SHAPE(lds <= 64 * 1024, "length_regulator: too many phonemes per utterance");
    hipLaunchKernelGGL(lr_expand_kernel, dim3(cdiv(T_out, LR_TF), B), dim3(256), lds, st, enc, cum, S, H,
                       T_out, out);
    M2_LAUNCHED("lr_expand_kernel");
    return M2_OK;
}

}  // namespace m2
