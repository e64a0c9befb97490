// Semantics probe: v_mfma_f32_16x16x16_f16 chained with v_mfma_f32_16x16x32_f16
// on one accumulator (the one-launch layers' 48-dim QK^T: a 16-dim tail step
// and a 32-dim step).  D = A0 B0 (K=16) + A1 B1 (K=32), checked on the host.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/mfma_mix.hip -o tools/probe/mfma_mix.bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

// A0 [16][16], B0 [16 k][16 n], A1 [16][32], B1 [32][16] row-major f16; D [16][16]
template <int ORDER>
__global__ void k(const _Float16* A0, const _Float16* B0, const _Float16* A1, const _Float16* B1, float* D) {
    const int l = threadIdx.x, li = l & 15, g = l >> 4;
    h4 a0, b0;
    h8 a1, b1;
    for (int j = 0; j < 4; ++j) {
        a0[j] = A0[li * 16 + 4 * g + j];
        b0[j] = B0[(4 * g + j) * 16 + li];
    }
    for (int j = 0; j < 8; ++j) {
        a1[j] = A1[li * 32 + 8 * g + j];
        b1[j] = B1[(8 * g + j) * 16 + li];
    }
    f4 c = {0.f, 0.f, 0.f, 0.f};
    if (ORDER == 0) {
        c = __builtin_amdgcn_mfma_f32_16x16x16f16(a0, b0, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, c, 0, 0, 0);
    } else if (ORDER == 1) {
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x16f16(a0, b0, c, 0, 0, 0);
    } else if (ORDER == 2) {
        c = __builtin_amdgcn_mfma_f32_16x16x16f16(a0, b0, c, 0, 0, 0);
    } else {
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1, c, 0, 0, 0);
    }
    for (int r = 0; r < 4; ++r) D[(4 * g + r) * 16 + li] = c[r];
}

int main() {
    std::vector<_Float16> A0(256), B0(256), A1(512), B1(512);
    srand(1);
    auto rnd = [] { return (_Float16)((rand() % 2001 - 1000) / 1000.f); };
    for (auto& x : A0) x = rnd();
    for (auto& x : B0) x = rnd();
    for (auto& x : A1) x = rnd();
    for (auto& x : B1) x = rnd();
    _Float16 *dA0, *dB0, *dA1, *dB1;
    float* dD;
    hipMalloc(&dA0, 512); hipMalloc(&dB0, 512); hipMalloc(&dA1, 1024); hipMalloc(&dB1, 1024); hipMalloc(&dD, 1024);
    hipMemcpy(dA0, A0.data(), 512, hipMemcpyHostToDevice);
    hipMemcpy(dB0, B0.data(), 512, hipMemcpyHostToDevice);
    hipMemcpy(dA1, A1.data(), 1024, hipMemcpyHostToDevice);
    hipMemcpy(dB1, B1.data(), 1024, hipMemcpyHostToDevice);
    for (int order = 0; order < 4; ++order) {
        if (order == 0) hipLaunchKernelGGL(k<0>, 1, 64, 0, 0, dA0, dB0, dA1, dB1, dD);
        if (order == 1) hipLaunchKernelGGL(k<1>, 1, 64, 0, 0, dA0, dB0, dA1, dB1, dD);
        if (order == 2) hipLaunchKernelGGL(k<2>, 1, 64, 0, 0, dA0, dB0, dA1, dB1, dD);
        if (order == 3) hipLaunchKernelGGL(k<3>, 1, 64, 0, 0, dA0, dB0, dA1, dB1, dD);
        std::vector<float> D(256);
        hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost);
        double err = 0;
        for (int i = 0; i < 16; ++i)
            for (int j = 0; j < 16; ++j) {
                double ref = 0;
                if (order != 3)
                    for (int q = 0; q < 16; ++q) ref += (double)A0[i * 16 + q] * (double)B0[q * 16 + j];
                if (order != 2)
                    for (int q = 0; q < 32; ++q) ref += (double)A1[i * 32 + q] * (double)B1[q * 16 + j];
                err = fmax(err, fabs(ref - D[i * 16 + j]));
            }
        printf("order %d (%s): max |err| %.3g\n", order,
               order == 0 ? "x16 then x32" : order == 1 ? "x32 then x16" : order == 2 ? "x16 only" : "x32 only", err);
    }
    return 0;
}
