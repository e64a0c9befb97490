// Microbenchmark: efficiency of the fused vocoder's MFMA inner loop
// (v_mfma_f32_16x16x4_f32, A streamed from global, B from LDS) in isolation.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_probe.hip -o tools/probe/mfma_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NT, int MODE>  // MODE 0: A global + B LDS; 1: A reg + B LDS; 2: A global + B reg; 3: A reg + B reg
__global__ __launch_bounds__(512) void probe(const float* __restrict__ W, float* out, int iters) {
    __shared__ float lds[64 * 272];
    const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
    for (int i = threadIdx.x; i < 64 * 272; i += blockDim.x) lds[i] = (float)(i & 7) * 0.25f;
    __syncthreads();
    f32x4 acc[NT];
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0, 0, 0, 0};
    const float* wp = W + ((threadIdx.x >> 6) * 64 + lane) * 4;
    const float* bp = lds + lk * 272 + li;
    f32x4 a0 = *reinterpret_cast<const f32x4*>(wp), a1 = *reinterpret_cast<const f32x4*>(wp + 256);
    for (int it = 0; it < iters; ++it) {
        const int blk = it & 3;
        f32x4 n0, n1;
        if (MODE == 0 || MODE == 2) {
            n0 = *reinterpret_cast<const f32x4*>(wp + ((blk + 1) & 3) * 2048);
            n1 = *reinterpret_cast<const f32x4*>(wp + ((blk + 1) & 3) * 2048 + 256);
        }
        float bv[8][NT];
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
            for (int n = 0; n < NT; ++n)
                bv[i][n] = (MODE < 2) ? bp[(i % 4) * 4 * 272 + (i / 4) + n * 16 + blk] : (float)(i + n + it);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float av = i < 4 ? a0[i] : a1[i - 4];
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[i][n], acc[n], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (MODE == 0 || MODE == 2) { a0 = n0; a1 = n1; }
    }
    float s = 0;
    for (int n = 0; n < NT; ++n) s += acc[n][0] + acc[n][1] + acc[n][2] + acc[n][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NT, int MODE>
void run(const float* W, float* out, int blocks, int iters) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL((probe<NT, MODE>), dim3(blocks), dim3(512), 0, 0, W, out, iters);
    hipEventRecord(a);
    hipLaunchKernelGGL((probe<NT, MODE>), dim3(blocks), dim3(512), 0, 0, W, out, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    const double mfma = (double)blocks * 8 * iters * 8 * NT;
    const double tf = mfma * 2048 / (ms * 1e-3) / 1e12;
    printf("NT=%d mode=%d blocks=%d: %.3f ms, %.1f TF/s (%.0f%% of 157.3)\n", NT, MODE, blocks, ms, tf, tf / 157.3 * 100);
}

int main() {
    float *W, *out;
    hipMalloc(&W, 4 << 20); hipMalloc(&out, 16 << 20);
    { std::vector<float> h(1 << 20); unsigned x = 12345; for (auto& v : h) { x = x * 1664525u + 1013904223u; v = ((x >> 8) & 0xffff) / 65536.0f - 0.5f; } hipMemcpy(W, h.data(), 4 << 20, hipMemcpyHostToDevice); }
    for (int blocks : {256, 512, 1024}) {
        run<2, 0>(W, out, blocks, 2000); run<4, 0>(W, out, blocks, 1000);
        run<2, 1>(W, out, blocks, 2000); run<4, 1>(W, out, blocks, 1000);
        run<4, 2>(W, out, blocks, 1000); run<4, 3>(W, out, blocks, 1000);
    }
    return 0;
}
