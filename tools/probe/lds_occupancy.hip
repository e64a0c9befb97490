// How many 512-thread workgroups per CU co-reside as a function of dynamic LDS?
// (occupancy API answer + a timing probe: 1024 WGs of a fixed ~50 us spin).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ __launch_bounds__(512) void spin(float* out, long long cycles) {
    extern __shared__ float lds[];
    const long long t0 = clock64();
    float acc = 0.f;
    while (clock64() - t0 < cycles) acc += lds[threadIdx.x & 63];
    if (acc == 12345.f) out[0] = acc;
}

int main() {
    float* out;
    hipMalloc(&out, 64);
    hipFuncSetAttribute((const void*)spin, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    for (int kb : {32, 48, 56, 60, 64, 66, 68, 70, 72, 74, 76, 78, 80, 96}) {
        size_t bytes = (size_t)kb * 1024;
        int nb = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, spin, 512, bytes);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipLaunchKernelGGL(spin, dim3(512), dim3(512), bytes, 0, out, 100000LL);
        hipEventRecord(a);
        hipLaunchKernelGGL(spin, dim3(512), dim3(512), bytes, 0, out, 100000LL);  // 512 WGs
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        printf("LDS %3d KB: occupancy API %d WG/CU; 512 WGs x 100k-cycle spin: %.3f ms\n", kb, nb, ms);
    }
    return 0;
}
