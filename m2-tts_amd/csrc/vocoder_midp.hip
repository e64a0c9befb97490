// Pipelined SimpleVocoder mid stage for stage1 (tts_model.py:279-297, the
// second upsampling stage): ConvT2 (64 -> 32 channels, x4, k 8, pad 2) +
// leaky, ResBlock2 (conv1 + leaky, conv2 + residual), split-f16 arithmetic
// (vocoder_x3.hip).  Reads U1 (the head kernel's output, rows of hi[64] lo[64]
// per position at 4T) and writes U2 (rows of hi[32] lo[32] at 16T), the
// formats of the x3 mid kernel it replaces.
//
// Polyphase form over the columns q of U1: ConvT2's output u2 (32 channels at
// t2 = 4q + s) is a 128-row column (phase s, channel) = 8 m-blocks of 16
// rows, m-block 2s + h holding channels 16h .. 16h+15 of phase s.
//   ConvT2, phase s:  s < 2: x[q] W[s+2] + x[q-1] W[s+6]
//                     s > 1: x[q+1] W[s-2] + x[q] W[s+2]
//     -> K = 2 taps x 64 channels = 4 k-blocks (tap, octet half).
//   ResBlock2 convs, phase s: taps t2-1, t2, t2+1 = phase (s+d) mod 4 of
//     column q + floor((s+d)/4), d = -1, 0, 1 -> K = 3 k-blocks, one whole
//     32-channel phase each: no padding.
// The two m-blocks of one phase read the same K slots, so one wave owns a
// phase (both m-blocks) and every B fragment it reads feeds two MFMA tiles.
//
// Systolic pipeline, one workgroup per CU (88 KB of LDS rings): a loader wave
// streams U1 into ring R0, 4 waves (one per phase) per layer compute 16
// columns per step each, one s_barrier per step, weights (8 / 6 fragment pairs
// per wave) in VGPRs for the whole strip - the structure of vocoder_tailp.hip
// (ring protocol, warm-up chunk -1, zero columns outside [0, L1), permlane16
// swapped 16-B epilogue stores).  The conv2 waves add the residual (ring R1,
// ConvT2's output) in the epilogue and store U2 rows straight to global.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "m2_common.h"
#include "vocoder_fused.h"

namespace m2 {
namespace mp {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef vx_u32x4 u32x4;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int RROWS = 64;               // 4 chunks of 16 columns
constexpr int RS0 = 288;                // R0 row: 256 B (hi[64] lo[64]) + pad, RS/16 = 2 mod 4
constexpr int RS1 = 544;                // R1/R2 row: 512 B (hi[128] lo[128]) + pad
constexpr int R0_OFF = 0, R1_OFF = RROWS * RS0, R2_OFF = R1_OFF + RROWS * RS1;
constexpr int LDS_BYTES = R2_OFF + RROWS * RS1;
constexpr int NWAVES = 13;              // 4 phases x 3 layers + 1 loader (wave 12)

// Byte offset of 16-B unit u in row `row` of ring R1 / R2 (stride RS1): units
// swap pairwise (u ^ 1) in rows 4-7 of every 8.  With RS1 / 16 = 2 (mod 4) the
// B-fragment and residual reads (ds_read_b128, 16-lane groups) were already
// conflict-free but the epilogue stores (ds_write_b128: 8 consecutive rows,
// 32 banks) hit two-way conflicts; the swap makes all three conflict-free
// (tools/probe/midp_banks.py models every access of the kernel).
__device__ __forceinline__ unsigned r12_at(int row, int u) { return row * RS1 + 16 * (u ^ ((row >> 2) & 1)); }

__device__ __forceinline__ f32x4 mfma_h(u32x4 a, u32x4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(h8, a), __builtin_bit_cast(h8, b), c, 0, 0, 0);
}

__device__ __forceinline__ void step_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int V>
using ic = std::integral_constant<int, V>;

// Layer L (0 ConvT2, 1 conv1, 2 conv2) of phase S: both m-blocks 2S, 2S+1.
// As in vocoder_tailp.hip: one fp32 accumulator per m-block for the three
// split products, LDS addresses precomputed for the four ring phases
// j = k mod 4 (step loop unrolled by four), leaky as a packed multiply and
// bare max, zeroing as a wave-uniform branch on chunks that straddle an
// utterance end, and conv2's residual (ConvT2's output, ring R1, two columns
// ahead: channels 32S .. 32S+31 = one fragment shared by both m-blocks) as
// two identity-A MFMAs per m-block instead of 24 VALU.
template <int L, int S>
__device__ __forceinline__ void layer_role(unsigned char* lds, int qa, int L1, int nch, bool edge,
                                           const u32x4* __restrict__ W, const float* __restrict__ bias,
                                           unsigned char* __restrict__ u2row) {
    constexpr int NKB = mkb(L);
    constexpr int IN_OFF = L == 0 ? R0_OFF : (L == 1 ? R1_OFF : R2_OFF);
    constexpr int LO_IN = L == 0 ? 128 : 256;           // lo half offset in an input row
    const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
    u32x4 a[2][NKB][2];
    float bv[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const int u = munit0(L) + (2 * S + h) * NKB + kb;
            a[h][kb][0] = W[u * 128 + lane];
            a[h][kb][1] = W[u * 128 + 64 + lane];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[h][r] = bias[L * 128 + 32 * S + 16 * h + 4 * g + r];
    }
    unsigned radr[NKB][4], xadr[4], oadr[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            const MSlot sl = mslot(L, S, kb, g);  // the input ring runs one column ahead of this layer
            const int row = (16 * j + li + sl.dq - 1) & (RROWS - 1);
            radr[kb][j] = IN_OFF + (L == 0 ? row * RS0 + sl.oct * 16 : r12_at(row, sl.oct));
        }
        xadr[j] = R1_OFF + r12_at((16 * j + li - 2) & (RROWS - 1), 4 * S + g);
        // unit 4S + 16 (g & 1) + (g >> 1) (+ 2h below: bit 1, so the swap of bit 0 commutes)
        oadr[j] = (L == 0 ? R1_OFF : R2_OFF) + r12_at((16 * j + li) & (RROWS - 1), 4 * S + 16 * (g & 1) + (g >> 1));
    }
    u32x4 aid[2];  // identity A of m-block h: row li takes fragment row 16h + li = 8g + e
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        h8 v;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (_Float16)(16 * h + li == 8 * g + e ? 1.f : 0.f);
        aid[h] = __builtin_bit_cast(u32x4, v);
    }
    const int sL = qa + 2 - L;
    auto work = [&](int k, auto jc) {
        constexpr int j = decltype(jc)::value;
        u32x4 bh[NKB], bl[NKB];
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb) {
            bh[kb] = *reinterpret_cast<const u32x4*>(lds + radr[kb][j]);
            bl[kb] = *reinterpret_cast<const u32x4*>(lds + radr[kb][j] + LO_IN);
        }
        u32x4 xh, xl;
        if constexpr (L == 2) {
            xh = *reinterpret_cast<const u32x4*>(lds + xadr[j]);
            xl = *reinterpret_cast<const u32x4*>(lds + xadr[j] + 256);
        }
        f32x4 acc[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[h] = f32x4{bv[h][0], bv[h][1], bv[h][2], bv[h][3]};
#pragma unroll
        for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
            for (int pr = 0; pr < 3; ++pr)
#pragma unroll
                for (int h = 0; h < 2; ++h) acc[h] = mfma_h(a[h][kb][pr == 2], pr == 1 ? bl[kb] : bh[kb], acc[h]);
        if constexpr (L == 2) {
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[h] = mfma_h(aid[h], xh, acc[h]);
#pragma unroll
            for (int h = 0; h < 2; ++h) acc[h] = mfma_h(aid[h], xl, acc[h]);
        }
        const int x0 = sL + 16 * k;  // this chunk's first column
        const bool straddle = edge && (x0 < 0 || x0 + 16 > L1);  // wave-uniform
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[h][r];
            if constexpr (L < 2) {
                leaky4(v);
                if (straddle) {
                    const int x = x0 + li;
                    if (x < 0 || x >= L1) {
#pragma unroll
                        for (int r = 0; r < 4; ++r) v[r] = 0.f;
                    }
                }
            }
            unsigned h0, h1, l0, l1;
            split2u(v[0], v[1], h0, l0);
            split2u(v[2], v[3], h1, l1);
            // lane groups 0/1 (2/3): channels 0-7 (8-15) of the m-block as
            // one 16-B hi chunk (group 0/2) and one lo chunk (group 1/3)
            const auto s0 = __builtin_amdgcn_permlane16_swap(h0, l0, false, false);
            const auto s1 = __builtin_amdgcn_permlane16_swap(h1, l1, false, false);
            const u32x4 val{s0[0], s1[0], s0[1], s1[1]};
            if constexpr (L < 2) {
                *reinterpret_cast<u32x4*>(lds + oadr[j] + 32 * h) = val;
            } else {
                const int x = x0 + li;
                if (k >= 0 && x >= 0 && x < L1)  // U2 row of position 4x + S
                    *reinterpret_cast<u32x4*>(u2row + ((size_t)4 * x + S) * 128 + 32 * h + 64 * (g & 1) +
                                              16 * (g >> 1)) = val;
            }
        }
    };
    const int LAST = nch + 2;  // conv2 computes chunk nch - 1 in step nch + 2
    auto step = [&](int s, auto jc) {
        if (s <= LAST) {
            const int k = s - (L + 1);
            if (k >= -1 && k < nch) work(k, jc);
            step_barrier();
        }
    };
    constexpr int J0 = (-1 - (L + 1)) & 3;  // ring phase of step -1's chunk
#pragma unroll 1
    for (int s = -1; s <= LAST; s += 4) {
        step(s, ic<J0>{});
        step(s + 1, ic<(J0 + 1) & 3>{});
        step(s + 2, ic<(J0 + 2) & 3>{});
        step(s + 3, ic<(J0 + 3) & 3>{});
    }
}

// U1 rows (256 B) into ring R0, two chunks ahead: chunk c = columns
// [qa + 3 + 16c, +16), zero outside [0, L1).  Four 16-B pieces per lane per
// chunk, loads issued unconditionally (clamped) so their waits are counted.
template <bool EDGE>
__device__ __forceinline__ void loader_role(unsigned char* lds, int qa, int L1, int nch,
                                            const unsigned char* __restrict__ u1) {
    const int lane = threadIdx.x & 63, cr = lane >> 4, pc = lane & 15;
    auto fetch = [&](int c, u32x4 (&v)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            int col = qa + 3 + 16 * c + 4 * j + cr;
            if (EDGE) col = min(max(col, 0), L1 - 1);
            v[j] = *reinterpret_cast<const u32x4*>(u1 + (size_t)col * 256 + pc * 16);
        }
    };
    u32x4 buf[3][4];
    auto step = [&](int s, u32x4 (&cur)[4], u32x4 (&ahead)[4]) {
        fetch(min(s + 2, nch - 1), ahead);
        if (s < nch) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int col = qa + 3 + 16 * s + 4 * j + cr;
                const bool in = !EDGE || (col >= 0 && col < L1);
                const u32x4 z{0u, 0u, 0u, 0u};
                *reinterpret_cast<u32x4*>(lds + R0_OFF + ((16 * s + 4 * j + cr) & (RROWS - 1)) * RS0 + pc * 16) =
                    in ? cur[j] : z;
            }
        }
        step_barrier();
    };
    fetch(-1, buf[0]);
    fetch(0, buf[1]);
    int s = -1;
#pragma unroll 1
    for (; s + 2 <= nch + 2; s += 3) {
        step(s, buf[0], buf[2]);
        step(s + 1, buf[1], buf[0]);
        step(s + 2, buf[2], buf[1]);
    }
#pragma unroll 1
    for (; s <= nch + 2; ++s) step_barrier();
}

// MIDP_DMA (default): U1 rows into ring R0 by LDS-DMA (as the tails'
// loader_role_dma): a chunk's 16 ring rows are 16 x RS0 = 4,608 contiguous
// bytes (hi[64] lo[64] + 32 B of padding per row), written by five
// buffer_load_dwordx4 ... lds of 64 lanes x 16 B (the fifth by lanes 0-31
// only: EXEC-masked lanes write nothing, so the next chunk's rows are left
// alone).  Lane l of instruction i fills 16-B unit u = 64 i + l of the
// chunk: row u / 18, unit u % 18 of the row - units 0-15 are the U1 row's
// 16-B pieces in order, 16-17 the padding (loaded out of range: zeros).
// Columns outside [0, L1) are out of the descriptor's range and land as
// zeros.  Chunk c + 1 is issued at the top of step c into the slot of chunk
// c - 3; chunk c has landed before step c's barrier (vmcnt(5)).
// Measured level, so not the default (MIDP_DMA=1 builds it): midp 19.74 /
// 20.14 us against 19.83 / 19.86 us with the register loader, alternated on
// one box, 169 tests green on it (profiles/r06/r06u_mid_dma_ab/,
// r06u_tests.log) - the mid's loader is not on its step's critical path.
#ifndef MIDP_DMA
#define MIDP_DMA 0
#endif
__device__ __forceinline__ void loader_role_dma(unsigned char* lds, int qa, int L1, int nch,
                                                const unsigned char* __restrict__ u1) {
    static_assert(RROWS == 64 && RS0 == 288, "4-chunk R0 of 288-B rows");
    const int lane = threadIdx.x & 63;
    // descriptor from the strip's first column to the utterance's end
    const int c0 = max(0, qa + 3 - 16);
    [[maybe_unused]] const auto rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<unsigned char*>(u1) + (size_t)c0 * 256, 0, (int)min((long)(L1 - c0) * 256, 0x7fffffffL),
        0x00020000);
    // per instruction i: this lane's row in the chunk and byte in the U1 row (-1: padding)
    int urow[5], ubyte[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const int u = 64 * i + lane;
        urow[i] = u / 18;
        ubyte[i] = u % 18 < 16 ? 16 * (u % 18) : -1;
    }
    [[maybe_unused]] auto dma = [&](int c) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass of hipcc does not know this builtin)
        unsigned char* dst = lds + R0_OFF + (c & 3) * 16 * RS0;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const int col = qa + 3 + 16 * c + urow[i] - c0;
            const int voff = ubyte[i] < 0 ? -1 : col * 256 + ubyte[i];  // < 0 / past L1: out of range -> 0
            if (i < 4 || lane < 32)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + 1024 * i),
                                                         16, voff, 0, 0, 0);
        }
#endif
    };
    dma(-1);
#pragma unroll 1
    for (int s = -1; s <= nch + 2; ++s) {
        if (s + 1 < nch) {
            dma(s + 1);
            asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        step_barrier();
    }
}

// NCHC > 0: the strip length as a compile-time constant (the headline's 16); 0: nch.
template <int NCHC>
__global__ __launch_bounds__(NWAVES * 64, 4) void midp_kernel(const unsigned char* __restrict__ U1, int L1, int nch_arg,
                                                               const u32x4* __restrict__ W,
                                                               const float* __restrict__ bias,
                                                               unsigned char* __restrict__ U2,
                                                               const int32_t* __restrict__ dT) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    const int nch = NCHC ? NCHC : nch_arg;
    const int b = blockIdx.y, qa = blockIdx.x * 16 * nch;
    if (dT) {  // speculative launch: L1 was the capacity
        L1 = 4 * dev_frames(dT, L1 / 4);
        if (qa >= L1) return;
    }
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool edge = qa < 16 || qa + 16 * nch + 16 > L1;
    unsigned char* u2row = U2 + (size_t)b * 4 * L1 * 128;
    if (w >= 8) __builtin_amdgcn_s_setprio(2);  // later layers: younger waves, the step waits for them
    else if (w >= 4) __builtin_amdgcn_s_setprio(1);
    switch (w) {
        case 0: layer_role<0, 0>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 1: layer_role<0, 1>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 2: layer_role<0, 2>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 3: layer_role<0, 3>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 4: layer_role<1, 0>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 5: layer_role<1, 1>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 6: layer_role<1, 2>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 7: layer_role<1, 3>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 8: layer_role<2, 0>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 9: layer_role<2, 1>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 10: layer_role<2, 2>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        case 11: layer_role<2, 3>(lds, qa, L1, nch, edge, W, bias, u2row); break;
        default:
            if constexpr (MIDP_DMA) loader_role_dma(lds, qa, L1, nch, U1 + (size_t)b * L1 * 256);
            else if (edge) loader_role<true>(lds, qa, L1, nch, U1 + (size_t)b * L1 * 256);
            else loader_role<false>(lds, qa, L1, nch, U1 + (size_t)b * L1 * 256);
            break;
    }
}

template <int NCHC>
int32_t launch(int nch, const void* U1, int L1, int B, const vx_u32x4* W, const float* bias, void* U2,
               hipStream_t st, const int32_t* dT) {
    static bool attr = false;
    if (!attr) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(midp_kernel<NCHC>),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
        attr = true;
    }
    hipLaunchKernelGGL(midp_kernel<NCHC>, dim3(cdiv(L1, 16 * nch), B), dim3(NWAVES * 64), LDS_BYTES, st,
                       static_cast<const unsigned char*>(U1), L1, nch, W, bias, static_cast<unsigned char*>(U2), dT);
    M2_LAUNCHED("midp_kernel");
    return M2_OK;
}

}  // namespace mp

const char* const kVocMidpKernelName = "midp_kernel (ConvT2 + ResBlock2, pipelined)";

int32_t launch_vocoder_midp(const void* U1, int L1, int B, const vx_u32x4* W, const float* bias, void* U2,
                            hipStream_t st, const int32_t* dT) {
    if (B == 0 || L1 == 0) return M2_OK;
    // Strip length (16-column chunks of U1 per workgroup, a launch argument):
    // the one from 4 to 256 minimising rounds of 256 workgroups (one per CU)
    // x pipeline steps (stage1 B = 32, L1 = 2000: 8 strips of 16 chunks, one
    // round; the round-4 sweep at 8 / 16 / 32 measured 23.1 / 20.0 / 29.9 us).
    // M2_MIDP_NCH forces one.
    int nch = sw().midp_nch > 0 ? std::min(sw().midp_nch, 4096) : 0;
    if (!nch) {
        const long chunks = cdiv(L1, 16);
        long best = -1;
        for (int n = 4; n <= 256; ++n) {
            const long wgs = (long)cdiv((int)chunks, n) * B, rounds = (wgs + 255) / 256, cost = rounds * (n + 4);
            if (best < 0 || cost < best) best = cost, nch = n;
        }
    }
    return nch == 16 ? mp::launch<16>(nch, U1, L1, B, W, bias, U2, st, dT)
                     : mp::launch<0>(nch, U1, L1, B, W, bias, U2, st, dT);
}

// ---------------------------------------------------------------------------
// Host packing: dense polyphase matrices Wd[row][dq + 1][input row] (128 x 3 x
// 128) cut into (m-block, k-block) fragment pairs along mp::mslot, unscaled
// hi/lo halves (split2u's format).
namespace {

int floordiv(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

struct Dense {
    std::vector<float> w = std::vector<float>(128 * 3 * 128, 0.f);
    float& at(int row, int dq, int in) { return w[(row * 3 + dq + 1) * 128 + in]; }
};

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

bool pack_midp(const MidpSrc& s, std::vector<uint16_t>* wout, std::vector<float>* bout, bool* range_ok) {
    Dense d[3];
    // ConvTranspose1d(64 -> 32, k 8, stride 4, pad 2), W [64][32][8]
    // (tts_model.py:255-263): out[4m + s] = x[m] W[s+2] + (s < 2 ? x[m-1] W[s+6] : x[m+1] W[s-2]).
    for (int sp = 0; sp < 4; ++sp)
        for (int co = 0; co < 32; ++co)
            for (int ci = 0; ci < 64; ++ci) {
                d[0].at(32 * sp + co, 0, ci) += s.wt[((size_t)ci * 32 + co) * 8 + sp + 2];
                if (sp < 2) d[0].at(32 * sp + co, -1, ci) += s.wt[((size_t)ci * 32 + co) * 8 + sp + 6];
                else d[0].at(32 * sp + co, 1, ci) += s.wt[((size_t)ci * 32 + co) * 8 + sp - 2];
            }
    // Conv1d(32 -> 32, k 3, pad 1), W [32][32][3], on the 4-phase signal.
    const float* wc[2] = {s.w1, s.w2};
    for (int l = 1; l <= 2; ++l)
        for (int sp = 0; sp < 4; ++sp)
            for (int k = 0; k < 3; ++k) {
                const int pp = sp + k - 1, dq = floordiv(pp, 4), p2 = pp - dq * 4;
                for (int co = 0; co < 32; ++co)
                    for (int ci = 0; ci < 32; ++ci)
                        d[l].at(32 * sp + co, dq, 32 * p2 + ci) += wc[l - 1][((size_t)co * 32 + ci) * 3 + k];
            }
    for (int l = 0; l < 3; ++l)
        for (int row = 0; row < 128; ++row)
            for (int dq = -1; dq <= 1; ++dq)
                for (int in = 0; in < 128; ++in) {
                    if (d[l].at(row, dq, in) == 0.f) continue;
                    bool missing = true;
                    for (int kb = 0; missing && kb < mp::mkb(l); ++kb)
                        for (int g = 0; g < 4; ++g) {
                            const mp::MSlot sl = mp::mslot(l, row / 32, kb, g);
                            if (sl.dq == dq && sl.oct == in / 8) missing = false;
                        }
                    if (missing) return false;
                }
    wout->assign((size_t)mp::kUnits * 2 * 64 * 8, 0);
    for (int l = 0; l < 3; ++l)
        for (int mb = 0; mb < 8; ++mb)
            for (int kb = 0; kb < mp::mkb(l); ++kb) {
                const int u = mp::munit0(l) + mb * mp::mkb(l) + kb;
                for (int lane = 0; lane < 64; ++lane) {
                    const int row = mb * 16 + (lane & 15);
                    const mp::MSlot sl = mp::mslot(l, mb / 2, kb, lane >> 4);
                    for (int e = 0; e < 8; ++e)
                        put_split(*wout, (((size_t)u * 2) * 64 + lane) * 8 + e, d[l].at(row, sl.dq, 8 * sl.oct + e),
                                  range_ok);
                }
            }
    bout->assign(3 * 128, 0.f);
    const float* bsrc[3] = {s.bt, s.b1, s.b2};
    for (int l = 0; l < 3; ++l)
        for (int row = 0; row < 128; ++row) (*bout)[l * 128 + row] = bsrc[l][row % 32];
    return true;
}

}  // namespace m2
