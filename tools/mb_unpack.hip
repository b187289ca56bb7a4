// Microbenchmark: rank 0's GRAY8 -> RGBA8 expansion of a c4 frame (3840 x 2160) and its floors.
//   memset    hipMemsetAsync of the 33 MB RGBA8 image (write-only floor)
//   copy      hipMemcpyAsync device to device of 33 MB
//   rows<Q>   one workgroup of 256 lanes per image row, Q 4-pixel quads per lane per step (the product's kernel: Q = 4)
//   flat<Q>   a flat grid, Q quads per lane, no row loop (rows still looked up per quad)
// Each variant: 20 warm launches, then 200 timed back to back on one stream (events); prints JSON lines.
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_unpack.hip -o tools/_mb_unpack
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                      \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

constexpr int W = 3840, H = 2160, NR = 8, HB = 8;
constexpr int SLAB = 272;

__device__ __forceinline__ uint4 gray4(uint32_t g) {
    uint4 o;
    o.x = (g & 0xffu) * 0x010101u | 0xff000000u;
    o.y = ((g >> 8) & 0xffu) * 0x010101u | 0xff000000u;
    o.z = ((g >> 16) & 0xffu) * 0x010101u | 0xff000000u;
    o.w = (g >> 24) * 0x010101u | 0xff000000u;
    return o;
}

__device__ __forceinline__ const uint32_t* src_row(const uint8_t* g, int j) {
    const int band = j / HB, within = j - band * HB, rank = band % NR, lb = band / NR;
    return reinterpret_cast<const uint32_t*>(g + ((size_t)rank * SLAB + (size_t)lb * HB + within) * W);
}

template <int Q>
__global__ __launch_bounds__(256) void rows_kernel(const uint8_t* __restrict__ g, uint4* __restrict__ d) {
    const int j = blockIdx.x;
    const uint32_t* s = src_row(g, j);
    uint4* o = d + (size_t)j * (W / 4);
    constexpr int groups = W / 4;
    for (int q0 = threadIdx.x; q0 < groups; q0 += Q * 256) {
        uint32_t a[Q];
#pragma unroll
        for (int u = 0; u < Q; ++u) {
            const int q = q0 + u * 256;
            a[u] = q < groups ? s[q] : 0;
        }
#pragma unroll
        for (int u = 0; u < Q; ++u) {
            const int q = q0 + u * 256;
            if (q < groups) o[q] = gray4(a[u]);
        }
    }
}

template <int Q>
__global__ __launch_bounds__(256) void flat_kernel(const uint8_t* __restrict__ g, uint4* __restrict__ d, int nquads) {
    const int base = (blockIdx.x * 256) * Q + threadIdx.x;
    uint32_t a[Q];
#pragma unroll
    for (int u = 0; u < Q; ++u) {
        const int q = base + u * 256;
        a[u] = 0;
        if (q < nquads) {
            const int j = q / (W / 4), x = q - j * (W / 4);
            a[u] = src_row(g, j)[x];
        }
    }
#pragma unroll
    for (int u = 0; u < Q; ++u) {
        const int q = base + u * 256;
        if (q < nquads) d[q] = gray4(a[u]);
    }
}

int main() {
    uint8_t* g = nullptr;
    uint4* d = nullptr;
    uint8_t* d2 = nullptr;
    const size_t out_bytes = (size_t)W * H * 4;
    CK(hipMalloc(&g, (size_t)NR * SLAB * W));
    CK(hipMalloc(&d, out_bytes));
    CK(hipMalloc(&d2, out_bytes));
    CK(hipMemset(g, 7, (size_t)NR * SLAB * W));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int nquads = W * H / 4;
    auto run = [&](const char* name, auto launch) -> int {
        for (int k = 0; k < 20; ++k) launch();
        CK(hipStreamSynchronize(st));
        CK(hipEventRecord(e0, st));
        for (int k = 0; k < 200; ++k) launch();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"variant\": \"%s\", \"us\": %.3f}\n", name, ms * 1e3 / 200);
        return 0;
    };
    run("memset", [&] { (void)hipMemsetAsync(d, 0, out_bytes, st); });
    run("copy", [&] { (void)hipMemcpyAsync(d2, d, out_bytes, hipMemcpyDeviceToDevice, st); });
    run("rows1", [&] { hipLaunchKernelGGL(rows_kernel<1>, dim3(H), dim3(256), 0, st, g, d); });
    run("rows4", [&] { hipLaunchKernelGGL(rows_kernel<4>, dim3(H), dim3(256), 0, st, g, d); });
    run("flat1", [&] { hipLaunchKernelGGL(flat_kernel<1>, dim3((nquads + 255) / 256), dim3(256), 0, st, g, d, nquads); });
    run("flat2", [&] { hipLaunchKernelGGL(flat_kernel<2>, dim3((nquads + 511) / 512), dim3(256), 0, st, g, d, nquads); });
    run("flat4", [&] { hipLaunchKernelGGL(flat_kernel<4>, dim3((nquads + 1023) / 1024), dim3(256), 0, st, g, d, nquads); });
    run("flat8", [&] { hipLaunchKernelGGL(flat_kernel<8>, dim3((nquads + 2047) / 2048), dim3(256), 0, st, g, d, nquads); });
    run("empty_rows", [&] { hipLaunchKernelGGL(rows_kernel<4>, dim3(1), dim3(256), 0, st, g, d); });
    CK(hipGetLastError());
    return 0;
}
