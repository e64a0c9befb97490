// Which SIMD does each wave of a workgroup land on?  Workgroups shaped like
// tailp_kernel (7 or 8 waves, 47-53 KB of dynamic LDS: three per CU) record
// HW_ID (SIMD, CU, SE) and XCC_ID per wave while all of them are resident;
// the host prints, per CU, the SIMD of wave w for each co-resident workgroup
// and the per-SIMD wave counts.   hipcc --offload-arch=gfx950 -O2 simd_map.hip -o /tmp/simd_map
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ void probe(unsigned* out, int nw) {
    extern __shared__ unsigned char lds[];
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        out[(blockIdx.x * nw + w) * 2] = hw;
        out[(blockIdx.x * nw + w) * 2 + 1] = xcc;
    }
    lds[threadIdx.x] = (unsigned char)hw;
    // stay resident ~50 us so the whole grid is co-resident
    const long long t0 = clock64();
    while (clock64() - t0 < 100000) __builtin_amdgcn_s_sleep(2);
    __syncthreads();
    if (lds[(threadIdx.x + 64) % blockDim.x] == 0xff) out[0] = 0;
}

int main(int argc, char** argv) {
    const int nw = argc > 1 ? atoi(argv[1]) : 7, lds = argc > 2 ? atoi(argv[2]) : 47120, grid = 768;
    unsigned* d;
    hipMalloc(&d, grid * nw * 8);
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    hipLaunchKernelGGL(probe, dim3(grid), dim3(nw * 64), lds, 0, d, nw);
    if (hipDeviceSynchronize() != hipSuccess) { printf("fail\n"); return 1; }
    std::vector<unsigned> h(grid * nw * 2);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    // key: (xcc, se, sh, cu) -> list of (wg, [simd per wave])
    std::map<unsigned, std::vector<std::pair<int, std::vector<int>>>> cus;
    for (int b = 0; b < grid; ++b) {
        unsigned hw0 = h[(b * nw) * 2], x = h[(b * nw) * 2 + 1] & 0xf;
        unsigned key = (x << 16) | (((hw0 >> 13) & 7) << 8) | (((hw0 >> 12) & 1) << 4) | ((hw0 >> 8) & 0xf);
        std::vector<int> s;
        for (int w = 0; w < nw; ++w) s.push_back((h[(b * nw + w) * 2] >> 4) & 3);
        cus[key].push_back({b, s});
    }
    int shown = 0;
    std::map<std::vector<int>, int> hist;  // sorted per-SIMD wave counts per CU
    std::map<std::vector<int>, int> firstpat;
    for (auto& [k, v] : cus) {
        std::vector<int> cnt(4, 0);
        for (auto& [b, s] : v) for (int q : s) cnt[q]++;
        hist[cnt]++;
        for (auto& [b, s] : v) firstpat[s]++;
        if (shown++ < 6) {
            printf("cu %06x:", k);
            for (auto& [b, s] : v) { printf("  wg%3d[", b); for (int q : s) printf("%d", q); printf("]"); }
            printf("  per-simd %d %d %d %d\n", cnt[0], cnt[1], cnt[2], cnt[3]);
        }
    }
    printf("CUs %zu\n", cus.size());
    for (auto& [c, n] : hist) printf("per-simd waves %d %d %d %d : %d CUs\n", c[0], c[1], c[2], c[3], n);
    for (auto& [s, n] : firstpat) { printf("wave->simd "); for (int q : s) printf("%d", q); printf(" : %d WGs\n", n); }
    return 0;
}
