// mb_hostwrite.hip — how fast a kernel's stores reach pinned host memory over PCIe, by store shape (diagnostic for the
// draw() path: could the render kernel store its GRAY8 frame straight into the caller's pinned buffer?).
// A 1920 x 1080 GRAY8 frame (2,073,600 B) written by one launch in each pattern, into device memory, coherent pinned
// host memory (hipHostMallocDefault) and non-coherent pinned host memory; prints one JSON line per (pattern, target)
// with the kernel time (HIP events, median of REPS launches) and the rate.
//   tile8x8    one-wave workgroup per 8 x 8 tile, 1 B per lane: 8 rows x 8 B (the render kernel's GRAY8 store)
//   row64      one wave per 64 x 1 pixels: 64 contiguous bytes
//   tile32x8   a 256-thread workgroup's 32 x 8 tile staged in LDS: 8 rows x 32 B, 4 B per lane
//   tile64x8   a 512-thread workgroup's 64 x 8 tile staged in LDS, one wave stores it: 8 rows x 64 B, 8 B per lane
//   copy16     the copy kernel: 16 B per lane, contiguous (1 KB per wave store)
// Build: hipcc -O3 --offload-arch=gfx950 tools/mb_hostwrite.hip -o tools/_mb_hostwrite
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e_ = (x);                                                      \
        if (e_ != hipSuccess) {                                                   \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

constexpr int W = 1920, H = 1080;

__global__ __launch_bounds__(64) void k_tile8x8(uint8_t* __restrict__ dst) {
    const int tx = blockIdx.x, ty = blockIdx.y, l = threadIdx.x;
    const int i = tx * 8 + (l & 7), j = ty * 8 + (l >> 3);
    if (i < W && j < H) dst[(size_t)j * W + i] = (uint8_t)(i ^ j);
}

__global__ __launch_bounds__(64) void k_row64(uint8_t* __restrict__ dst) {
    const int i = blockIdx.x * 64 + threadIdx.x, j = blockIdx.y;
    if (i < W) dst[(size_t)j * W + i] = (uint8_t)(i ^ j);
}

__global__ __launch_bounds__(256) void k_tile32x8(uint8_t* __restrict__ dst) {
    __shared__ uint8_t t[8][32];
    const int l = threadIdx.x, w = l >> 6, ll = l & 63;
    const int cx = w * 8 + (ll & 7), cy = ll >> 3;
    const int i0 = blockIdx.x * 32, j0 = blockIdx.y * 8;
    t[cy][cx] = (uint8_t)((i0 + cx) ^ (j0 + cy));
    __syncthreads();
    if (l < 64) {                                 // 8 rows x 32 B: 4 B per lane, lanes 0..63
        const int r = l >> 3, c = (l & 7) * 4;
        if (j0 + r < H) *reinterpret_cast<uint32_t*>(dst + (size_t)(j0 + r) * W + i0 + c) =
            *reinterpret_cast<const uint32_t*>(&t[r][c]);
    }
}

__global__ __launch_bounds__(512) void k_tile64x8(uint8_t* __restrict__ dst) {
    __shared__ uint8_t t[8][64];
    const int l = threadIdx.x, w = l >> 6, ll = l & 63;
    const int cx = w * 8 + (ll & 7), cy = ll >> 3;
    const int i0 = blockIdx.x * 64, j0 = blockIdx.y * 8;
    t[cy][cx] = (uint8_t)((i0 + cx) ^ (j0 + cy));
    __syncthreads();
    if (l < 64) {                                 // 8 rows x 64 B: 8 B per lane
        const int r = l >> 3, c = (l & 7) * 8;
        if (j0 + r < H) *reinterpret_cast<uint2*>(dst + (size_t)(j0 + r) * W + i0 + c) =
            *reinterpret_cast<const uint2*>(&t[r][c]);
    }
}

__global__ __launch_bounds__(256) void k_copy16(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t n) {
    const size_t n16 = n >> 4;
    for (size_t k = (size_t)blockIdx.x * 256 + threadIdx.x; k < n16; k += (size_t)gridDim.x * 256)
        reinterpret_cast<uint4*>(dst)[k] = reinterpret_cast<const uint4*>(src)[k];
}

int main() {
    const size_t n = (size_t)W * H;
    const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 50;
    uint8_t *d_buf, *d_src, *h_coh, *h_nc, *m_coh, *m_nc;
    CK(hipMalloc(&d_buf, n));
    CK(hipMalloc(&d_src, n));
    CK(hipMemset(d_src, 7, n));
    CK(hipHostMalloc(&h_coh, n, hipHostMallocDefault));
    CK(hipHostMalloc(&h_nc, n, hipHostMallocNonCoherent));
    CK(hipHostGetDevicePointer((void**)&m_coh, h_coh, 0));
    CK(hipHostGetDevicePointer((void**)&m_nc, h_nc, 0));
    struct Target { const char* name; uint8_t* p; } targets[] = {{"device", d_buf}, {"host_coherent", m_coh},
                                                              {"host_noncoherent", m_nc}};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char* pats[] = {"tile8x8", "row64", "tile32x8", "tile64x8", "copy16_16wg", "copy16_256wg", "copy16_2048wg"};
    for (const char* pat : pats) {
        for (const Target& T : targets) {
            auto launch = [&]() {
                std::string p = pat;
                if (p == "tile8x8") hipLaunchKernelGGL(k_tile8x8, dim3(W / 8, H / 8), dim3(64), 0, 0, T.p);
                else if (p == "row64") hipLaunchKernelGGL(k_row64, dim3(W / 64, H), dim3(64), 0, 0, T.p);
                else if (p == "tile32x8") hipLaunchKernelGGL(k_tile32x8, dim3(W / 32, H / 8), dim3(256), 0, 0, T.p);
                else if (p == "tile64x8") hipLaunchKernelGGL(k_tile64x8, dim3(W / 64, H / 8), dim3(512), 0, 0, T.p);
                else if (p == "copy16_16wg") hipLaunchKernelGGL(k_copy16, dim3(16), dim3(256), 0, 0, d_src, T.p, n);
                else if (p == "copy16_256wg") hipLaunchKernelGGL(k_copy16, dim3(256), dim3(256), 0, 0, d_src, T.p, n);
                else hipLaunchKernelGGL(k_copy16, dim3(2048), dim3(256), 0, 0, d_src, T.p, n);
            };
            for (int r = 0; r < 3; ++r) launch();
            CK(hipDeviceSynchronize());
            std::vector<float> ms;
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0, 0));
                launch();
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float t = 0;
                CK(hipEventElapsedTime(&t, e0, e1));
                ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const float med = ms[ms.size() / 2];
            printf("{\"pattern\": \"%s\", \"target\": \"%s\", \"us\": %.2f, \"min_us\": %.2f, \"GBps\": %.1f}\n", pat,
                   T.name, med * 1e3, ms[0] * 1e3, n / (med * 1e-3) / 1e9);
        }
    }
    // correctness spot check of the last host pattern
    CK(hipDeviceSynchronize());
    printf("{\"check\": %d}\n", (int)h_coh[12345]);
    return 0;
}
