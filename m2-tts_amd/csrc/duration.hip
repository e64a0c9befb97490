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

#include "m2_common.h"

namespace m2 {

// ---------------------------------------------------------------------------
// One workgroup per (utterance, 16-phoneme tile).  The encoder rows of the
// tile plus a 2-phoneme halo each side are staged in LDS; conv1 is evaluated
// on the tile +-1 (positions outside [0,S) are the zero padding conv2 sees),
// conv2 on the tile, then the k=1 projection and softplus.  The encoder
// output is read in its [B,S,H] layout (the reference's transpose(1,2) is a
// view).  BatchNorm uses alpha = gamma/sqrt(var+eps), beta' = beta -
// mean*alpha, the inference form PyTorch's CPU batch_norm evaluates.
// Conv weights arrive packed [ci][k][co] (m2_model_create) and are staged in
// LDS one layer at a time (3*H*H floats: 48 KiB at H=64, 108 KiB at H=96):
// the inner loop is then LDS-only - lanes (consecutive co) read consecutive
// weights, the activation rows are float4 broadcasts.  The whole predictor is
// ~0.2 GFLOP at B=32, S=100; what matters is not waiting on L2 per FMA.
constexpr int DUR_TS = 16;

// out[p][co] (+)= sum_{ci in chunk, k} W[ci][k][co] * in[p + k][ci] for p in
// [0, np), with the weight rows of channels [ci0, ci0 + cc) staged in Ws.
__device__ __forceinline__ void dur_conv_chunk(const float* in, const float* Ws, int H, int np, int ci0,
                                               int cc, bool first, float* out) {
    for (int i = threadIdx.x; i < np * H; i += 256) {
        const int p = i / H, co = i - p * H;
        const float* x0 = in + p * H + ci0;
        const float* w0 = Ws + co;
        float acc = first ? 0.f : out[i];
        for (int ci = 0; ci < cc; ci += 4) {
            const float4 u0 = *reinterpret_cast<const float4*>(x0 + ci);
            const float4 u1 = *reinterpret_cast<const float4*>(x0 + H + ci);
            const float4 u2 = *reinterpret_cast<const float4*>(x0 + 2 * H + ci);
            acc = fmaf(w0[0], u0.x, acc); acc = fmaf(w0[H], u1.x, acc); acc = fmaf(w0[2 * H], u2.x, acc);
            w0 += 3 * H;
            acc = fmaf(w0[0], u0.y, acc); acc = fmaf(w0[H], u1.y, acc); acc = fmaf(w0[2 * H], u2.y, acc);
            w0 += 3 * H;
            acc = fmaf(w0[0], u0.z, acc); acc = fmaf(w0[H], u1.z, acc); acc = fmaf(w0[2 * H], u2.z, acc);
            w0 += 3 * H;
            acc = fmaf(w0[0], u0.w, acc); acc = fmaf(w0[H], u1.w, acc); acc = fmaf(w0[2 * H], u2.w, acc);
            w0 += 3 * H;
        }
        out[i] = acc;
    }
}

// One conv layer: weights streamed through LDS in chunks of `cc` input
// channels (all of them at once for H <= 108), then bias, BN, ReLU, and zero
// for rows whose position pos0 + p is outside [0, S).
__device__ __forceinline__ void dur_conv(const float* in, float* Ws, const float* __restrict__ w, int H, int cc,
                                         int np, int pos0, int S, const float* __restrict__ b,
                                         const float* __restrict__ a, const float* __restrict__ c,
                                         float* out) {
    for (int ci0 = 0; ci0 < H; ci0 += cc) {
        const int n = 3 * min(cc, H - ci0) * H;
        const float* src = w + (size_t)ci0 * 3 * H;
        __syncthreads();  // previous chunk's readers are done with Ws
        for (int i = threadIdx.x * 4; i < n; i += 256 * 4)
            *reinterpret_cast<float4*>(Ws + i) = *reinterpret_cast<const float4*>(src + i);
        __syncthreads();
        dur_conv_chunk(in, Ws, H, np, ci0, min(cc, H - ci0), ci0 == 0, out);
    }
    for (int i = threadIdx.x; i < np * H; i += 256) {
        const int p = i / H, co = i - p * H, s = pos0 + p;
        float v = (out[i] + b[co]) * a[co] + c[co];
        v = v > 0.f ? v : 0.f;
        out[i] = (s >= 0 && s < S) ? v : 0.f;
    }
}

__global__ __launch_bounds__(256) void duration_kernel(
    const float* __restrict__ enc, int S, int H, int cc, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ a2,
    const float* __restrict__ c2, const float* __restrict__ pw, const float* __restrict__ pb,
    float* __restrict__ dur) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* X = lds;                          // [TS+4][H]  s0-2 .. s0+TS+1
    float* Y1 = X + (DUR_TS + 4) * H;        // [TS+2][H]  s0-1 .. s0+TS
    float* Y2 = Y1 + (DUR_TS + 2) * H;       // [TS][H]    s0   .. s0+TS-1
    float* Ws = Y2 + DUR_TS * H;             // [3*cc][H]  weight chunk
    const int b = blockIdx.y, s0 = blockIdx.x * DUR_TS, tid = threadIdx.x;
    const float* e = enc + (size_t)b * S * H;

    for (int i = tid; i < (DUR_TS + 4) * H; i += 256) {
        const int p = i / H, c = i - p * H, s = s0 - 2 + p;
        X[i] = (s >= 0 && s < S) ? e[(size_t)s * H + c] : 0.f;
    }
    dur_conv(X, Ws, w1, H, cc, DUR_TS + 2, s0 - 1, S, b1, a1, c1, Y1);
    dur_conv(Y1, Ws, w2, H, cc, DUR_TS, s0, S, b2, a2, c2, Y2);
    __syncthreads();
    // k=1 projection H -> 1: one wave per phoneme, shuffle reduction.
    const int lane = tid & 63, wave = tid >> 6;
    for (int p = wave; p < DUR_TS; p += 4) {
        const int s = s0 + p;
        float acc = 0.f;
        for (int ci = lane; ci < H; ci += 64) acc = fmaf(pw[ci], Y2[p * H + ci], acc);
        for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
        if (lane == 0 && s < S) {
            const float x = acc + pb[0];
            // F.softplus(beta=1, threshold=20)
            dur[(size_t)b * S + s] = x > 20.f ? x : log1pf(expf(x));
        }
    }
}

// ---------------------------------------------------------------------------
// One workgroup per utterance: n[s] = max(0, trunc(d[s]*scale)); exclusive
// scan into cum[b, 0..S]; T[b] = cum[b,S]; atomicMax into Tmax (zeroed by the
// launcher's memset node).
__device__ __forceinline__ int frames_of(const void* dur, int is_int, float scale, size_t i) {
    if (is_int) {
        const int v = static_cast<const int32_t*>(dur)[i];
        return v > 0 ? v : 0;
    }
    const float v = static_cast<const float*>(dur)[i] * scale;  // fp32 product, as dur*scale
    if (!(v >= 1.0f)) return 0;                                   // also NaN -> 0
    return v >= 1073741824.f ? 1073741824 : (int)v;               // int() truncates toward zero
}

__global__ __launch_bounds__(256) void lr_count_kernel(const void* __restrict__ dur, int is_int,
                                                       float scale, int S, int32_t* __restrict__ cum,
                                                       int32_t* __restrict__ T,
                                                       int32_t* __restrict__ Tmax) {
    __shared__ int part[256];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int chunk = (S + 255) / 256;
    const int lo = min(S, tid * chunk), hi = min(S, lo + chunk);
    const size_t base = (size_t)b * S;
    int sum = 0;
    for (int s = lo; s < hi; ++s) sum += frames_of(dur, is_int, scale, base + s);
    part[tid] = sum;
    __syncthreads();
    // Hillis-Steele inclusive scan over the 256 partials.
    for (int off = 1; off < 256; off <<= 1) {
        const int v = tid >= off ? part[tid - off] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = part[tid] - sum;  // exclusive prefix of this thread's chunk
    int32_t* c = cum + (size_t)b * (S + 1);
    if (tid == 0) c[0] = 0;
    for (int s = lo; s < hi; ++s) {
        run += frames_of(dur, is_int, scale, base + s);
        c[s + 1] = run;
    }
    if (tid == 255) {
        T[b] = part[255];
        atomicMax(Tmax, part[255]);
    }
}

// One wave per output frame; binary search of the frame in cum[b].
__global__ __launch_bounds__(256) void lr_expand_kernel(const float* __restrict__ enc,
                                                        const int32_t* __restrict__ cum, int S,
                                                        int H, int T_out, float* __restrict__ out) {
    const int b = blockIdx.y;
    const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (t >= T_out) return;
    const int32_t* c = cum + (size_t)b * (S + 1);
    float* o = out + ((size_t)b * T_out + t) * H;
    if (t >= c[S]) {
        for (int h = lane; h < H; h += 64) o[h] = 0.f;
        return;
    }
    int lo = 0, hi = S - 1;  // smallest s with c[s+1] > t
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (c[mid + 1] > t) hi = mid; else lo = mid + 1;
    }
    const float* e = enc + ((size_t)b * S + lo) * H;
    for (int h = lane; h < H; h += 64) o[h] = e[h];
}

// ---------------------------------------------------------------------------
int32_t launch_duration(const float* enc, int B, int S, int H, const float* const* p, float* dur,
                        hipStream_t st) {
    if (B == 0 || S == 0) return M2_OK;
    // LDS: activations (3*TS+6)*H + a weight chunk of cc input channels 3*cc*H.
    const size_t act = (size_t)(3 * DUR_TS + 6) * H;
    const size_t room = 160 * 1024 / sizeof(float);
    M2_CHECK_SHAPE(H % 4 == 0 && act + 12 * (size_t)H <= room, "duration: hidden_dim must be a multiple of 4 and <= 630");
    const int cc = (int)std::min<size_t>((size_t)H, (room - act) / (3 * (size_t)H) / 4 * 4);
    const size_t lds = sizeof(float) * (act + 3 * (size_t)cc * H);
    static bool attr_set = false;
    if (!attr_set) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(duration_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    hipLaunchKernelGGL(duration_kernel, dim3(cdiv(S, DUR_TS), B), dim3(256), lds, st, enc, S, H, cc,
                       p[0], p[1], p[2], p[3], p[4], p[5], p[6], p[7], p[8], p[9], dur);
    M2_LAUNCHED("duration_kernel");
    return M2_OK;
}

int32_t launch_lr_count(const void* dur, int is_int, float scale, int B, int S, int32_t* cum,
                        int32_t* T, int32_t* Tmax, hipStream_t st) {
    M2_HIP(hipMemsetAsync(Tmax, 0, sizeof(int32_t), st));
    if (B == 0) return M2_OK;
    hipLaunchKernelGGL(lr_count_kernel, dim3(B), dim3(256), 0, st, dur, is_int, scale, S, cum, T,
                       Tmax);
    M2_LAUNCHED("lr_count_kernel");
    return M2_OK;
}

int32_t launch_lr_expand(const float* enc, const int32_t* cum, int B, int S, int H, int T_out,
                         float* out, hipStream_t st) {
    if (B == 0 || T_out == 0) return M2_OK;
    hipLaunchKernelGGL(lr_expand_kernel, dim3(cdiv(T_out, 4), B), dim3(256), 0, st, enc, cum, S, H,
                       T_out, out);
    M2_LAUNCHED("lr_expand_kernel");
    return M2_OK;
}

}  // namespace m2
