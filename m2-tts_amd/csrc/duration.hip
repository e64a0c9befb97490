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
#include "m2_common.h"

namespace m2 {

// ---------------------------------------------------------------------------
// One workgroup per (utterance, 32-phoneme tile).  The encoder rows of the
// tile plus a 2-phoneme halo each side are staged in LDS; conv1 is evaluated
// on the tile +-1 (positions outside [0,S) are the zero padding conv2 sees),
// conv2 on the tile, then the k=1 projection and softplus.  The encoder
// output is read in its [B,S,H] layout (the reference's transpose(1,2) is a
// view).  BatchNorm uses alpha = gamma/sqrt(var+eps), beta' = beta -
// mean*alpha, the inference form PyTorch's CPU batch_norm evaluates.
// Conv weights arrive packed [ci][k][co] (m2_model_create) so the lanes of a
// wave - consecutive output channels - read consecutive weights.
constexpr int DUR_TS = 32;

__global__ __launch_bounds__(256) void duration_kernel(
    const float* __restrict__ enc, int S, int H, const float* __restrict__ w1,
    const float* __restrict__ b1, const float* __restrict__ a1, const float* __restrict__ c1,
    const float* __restrict__ w2, const float* __restrict__ b2, const float* __restrict__ a2,
    const float* __restrict__ c2, const float* __restrict__ pw, const float* __restrict__ pb,
    float* __restrict__ dur) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* X = lds;                          // [TS+4][H]  s0-2 .. s0+TS+1
    float* Y1 = X + (DUR_TS + 4) * H;        // [TS+2][H]  s0-1 .. s0+TS
    float* Y2 = Y1 + (DUR_TS + 2) * H;       // [TS][H]    s0   .. s0+TS-1
    const int b = blockIdx.y, s0 = blockIdx.x * DUR_TS, tid = threadIdx.x;
    const float* e = enc + (size_t)b * S * H;

    for (int i = tid; i < (DUR_TS + 4) * H; i += 256) {
        const int p = i / H, c = i - p * H, s = s0 - 2 + p;
        X[i] = (s >= 0 && s < S) ? e[(size_t)s * H + c] : 0.f;
    }
    __syncthreads();
    for (int i = tid; i < (DUR_TS + 2) * H; i += 256) {
        const int p = i / H, co = i - p * H, s = s0 - 1 + p;
        float v = 0.f;
        if (s >= 0 && s < S) {
            float acc = 0.f;
            for (int ci = 0; ci < H; ++ci) {
                const float* wr = w1 + (size_t)ci * 3 * H + co;
                acc = fmaf(wr[0], X[(p + 0) * H + ci], acc);
                acc = fmaf(wr[H], X[(p + 1) * H + ci], acc);
                acc = fmaf(wr[2 * H], X[(p + 2) * H + ci], acc);
            }
            v = (acc + b1[co]) * a1[co] + c1[co];
            v = v > 0.f ? v : 0.f;
        }
        Y1[i] = v;
    }
    __syncthreads();
    for (int i = tid; i < DUR_TS * H; i += 256) {
        const int p = i / H, co = i - p * H;
        float acc = 0.f;
        for (int ci = 0; ci < H; ++ci) {
            const float* wr = w2 + (size_t)ci * 3 * H + co;
            acc = fmaf(wr[0], Y1[(p + 0) * H + ci], acc);
            acc = fmaf(wr[H], Y1[(p + 1) * H + ci], acc);
            acc = fmaf(wr[2 * H], Y1[(p + 2) * H + ci], acc);
        }
        const float v = (acc + b2[co]) * a2[co] + c2[co];
        Y2[i] = v > 0.f ? v : 0.f;
    }
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
    const size_t lds = sizeof(float) * (3 * DUR_TS + 6) * H;
    M2_CHECK_SHAPE(lds <= 160 * 1024, "duration: hidden_dim too large");
    static bool attr_set = false;
    if (!attr_set) {
        M2_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(duration_kernel),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        attr_set = true;
    }
    hipLaunchKernelGGL(duration_kernel, dim3(cdiv(S, DUR_TS), B), dim3(256), lds, st, enc, S, H,
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
