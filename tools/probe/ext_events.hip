// Event timing of one kernel between two others on one stream: hipEventRecord
// around the launch vs the start / stop events of hipExtLaunchKernelGGL,
// against the kernel's own duration (s_memrealtime at 100 MHz, first start to
// last end over its workgroups).  A kernel of 768 workgroups spinning a fixed
// number of cycles stands in for the vocoder tail.
//   hipcc --offload-arch=gfx950 -O2 tools/probe/ext_events.hip -o /tmp/ext_events
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e = (x);                                                   \
        if (e != hipSuccess) {                                                \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));                \
            return 1;                                                         \
        }                                                                     \
    } while (0)

__global__ void spin(long long cycles, unsigned long long* span) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const long long c0 = clock64();
    while (clock64() - c0 < cycles) {
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if (span && threadIdx.x == 0) {
        atomicMin(span, t0);
        atomicMax(span + 1, t1);
    }
}

int main() {
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned long long* span;
    CK(hipMalloc(&span, 16));
    hipEvent_t a, b;
    CK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
    CK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
    const dim3 g(768), blk(448);
    const long long cyc = 40000;  // ~20 us at ~2 GHz
    std::vector<float> rec, ext;
    std::vector<double> own_rec, own_ext;
    for (int it = 0; it < 60; ++it) {
        for (int mode = 0; mode < 2; ++mode) {
            const unsigned long long init[2] = {~0ull, 0ull};
            CK(hipMemcpyAsync(span, init, 16, hipMemcpyHostToDevice, st));
            hipLaunchKernelGGL(spin, g, blk, 0, st, cyc, nullptr);
            if (mode == 0) {
                CK(hipEventRecord(a, st));
                hipLaunchKernelGGL(spin, g, blk, 0, st, cyc, span);
                CK(hipEventRecord(b, st));
            } else {
                hipExtLaunchKernelGGL(spin, g, blk, 0, st, a, b, 0, cyc, span);
            }
            hipLaunchKernelGGL(spin, g, blk, 0, st, cyc, nullptr);
            CK(hipStreamSynchronize(st));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, a, b));
            unsigned long long h[2];
            CK(hipMemcpy(h, span, 16, hipMemcpyDeviceToHost));
            const double own = (double)(h[1] - h[0]) / 100.0;  // us at 100 MHz
            if (it >= 10) {
                (mode ? ext : rec).push_back(ms * 1000.f);
                (mode ? own_ext : own_rec).push_back(own);
            }
        }
    }
    auto med = [](auto v) { std::sort(v.begin(), v.end()); return (double)v[v.size() / 2]; };
    std::printf("hipEventRecord pair : events %.2f us, kernel's own span %.2f us\n", med(rec), med(own_rec));
    std::printf("hipExtLaunchKernel  : events %.2f us, kernel's own span %.2f us\n", med(ext), med(own_ext));
    return 0;
}
