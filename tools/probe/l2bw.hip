// Per-CU read bandwidth of L2-resident data (the one-launch transformer
// layer's K / V and weight reads): every workgroup of a 256-workgroup grid
// (one per CU) reads `per_wg` bytes of a buffer that all workgroups on its
// XCD share (workgroup L reads slice L % 8), 16-B loads, `inflight` loads per
// lane in flight.  Prints GB/s per CU and chip-wide.
//   hipcc --offload-arch=gfx950 -O3 tools/probe/l2bw.hip -o tools/probe/l2bw.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ROWS = 0: a wave-instruction reads 1 KB contiguous (lane i: element base + i);
// ROWS = 1: 16 rows of 64 B, rows 256 B apart (lane (i, g): row i, 16 g) -
// the one-launch layer's K-fragment pattern; a wave covers 4 such blocks
// (the row's 4 x 64 B) before moving on.  ROWS = 2: that pattern, each
// workgroup of an XCD starting k/32 of the way into the slice; ROWS = 3:
// contiguous 1 KB with that rotated start (time-skewed readers of one
// shared buffer: the query-split attention's K / V stream).
template <int INF, int ROWS>
__global__ __launch_bounds__(512) void rd(const u32x4* __restrict__ buf, size_t slice_elems, int per_wg_elems,
                                          unsigned* __restrict__ out) {
    const u32x4* p = buf + (size_t)(blockIdx.x & 7) * slice_elems;
    unsigned acc = 0;
    const int stride = blockDim.x * INF;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int base = threadIdx.x; base < per_wg_elems; base += stride) {
        u32x4 v[INF];
#pragma unroll
        for (int i = 0; i < INF; ++i) {
            int e = base + i * blockDim.x;
            if (ROWS == 1 || ROWS == 2) {
                const int ins = (base - threadIdx.x) / 64 + w + i * (blockDim.x / 64);  // wave-instruction index
                const int blk = ins >> 2, part = ins & 3;                               // 16-row block, 64-B column
                e = blk * 256 + (lane & 15) * 16 + part * 4 + (lane >> 4);              // 16-B elements
            }
            if (ROWS >= 2) {  // rotated start: workgroup k of an XCD begins k/32 of the way in
                const int rot = (int)(((long long)(blockIdx.x >> 3) * per_wg_elems / 32) & ~63);
                e = e < per_wg_elems ? (e + rot) % per_wg_elems : e;
            }
            v[i] = e < per_wg_elems ? p[e] : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int i = 0; i < INF; ++i) acc ^= v[i].x + v[i].y + v[i].z + v[i].w;
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

int main(int argc, char** argv) {
    const int per_wg = argc > 1 ? atoi(argv[1]) : 448 * 1024;
    const int grid = argc > 2 ? atoi(argv[2]) : 256;
    const int threads = argc > 3 ? atoi(argv[3]) : 512;
    const size_t slice = (per_wg + 15) / 16;
    u32x4* buf;
    unsigned* out;
    hipMalloc(&buf, slice * 8 * 16);
    hipMalloc(&out, 4096 * 4);
    hipMemset(buf, 1, slice * 8 * 16);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int inf : {4, 8, 16, -4, -8, 104, 108, 116, 204, 208, 216}) {
        auto launch = [&] {
            if (inf == 4) hipLaunchKernelGGL((rd<4, 0>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 8) hipLaunchKernelGGL((rd<8, 0>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 16) hipLaunchKernelGGL((rd<16, 0>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == -4) hipLaunchKernelGGL((rd<4, 1>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == -8) hipLaunchKernelGGL((rd<8, 1>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == -16) hipLaunchKernelGGL((rd<16, 1>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 104) hipLaunchKernelGGL((rd<4, 2>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 108) hipLaunchKernelGGL((rd<8, 2>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 116) hipLaunchKernelGGL((rd<16, 2>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 204) hipLaunchKernelGGL((rd<4, 3>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 208) hipLaunchKernelGGL((rd<8, 3>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
            if (inf == 216) hipLaunchKernelGGL((rd<16, 3>), dim3(grid), dim3(threads), 0, 0, buf, slice, (int)slice, out);
        };
        for (int i = 0; i < 50; ++i) launch();
        hipDeviceSynchronize();
        const int n = 200;
        hipEventRecord(a);
        for (int i = 0; i < n; ++i) launch();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double us = ms * 1e3 / n;
        const double per_cu = (double)per_wg / (us * 1e-6) / 1e9;
        printf("per_wg %d B, grid %d x %d threads, %s, %2d loads/lane in flight: %.2f us/launch, %.1f GB/s per WG, %.2f TB/s chip\n",
               per_wg, grid, threads,
               inf > 200 ? "rotated contiguous 1 KB" : inf > 100 ? "rotated 16 rows x 64 B" : inf > 0 ? "contiguous 1 KB" : "16 rows x 64 B",
               inf > 200 ? inf - 200 : inf > 100 ? inf - 100 : inf > 0 ? inf : -inf, us, per_cu,
               per_cu * grid / 1e3);
    }
    return 0;
}
