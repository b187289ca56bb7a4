// tools/mb_persist.hip — does the per-pixel floor of rt_render_kernel come from dispatching 32,400 short
// workgroups?  (not product code)  The empty-scene work of one c2 frame (primary ray, FP64 normalize,
// RGBA32F + RGBA8 stores) with three launch shapes:
//   wg64       one 64-thread workgroup per 8 x 8 tile (the render kernel's default)
//   wg256      one 256-thread workgroup per 32 x 8 tile
//   persistN   N waves per SIMD resident, each loops over 8 x 8 tiles (static stride or atomic counter)
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/mb_persist.hip -o tools/_mbp
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

struct P {
    double eye[3], look[3], right[3], upp[3], pitch;
    int bx, by, W, H, tiles_x, ntiles;
};

__device__ __forceinline__ void pixel(const P& p, int i, int j, float4* out32, uchar4* out8, int work) {
    double a = p.pitch * (double)(i + p.bx), b = p.pitch * (double)(j + p.by);
    double sx = (p.look[0] + a * p.right[0]) + b * p.upp[0];
    double sy = (p.look[1] + a * p.right[1]) + b * p.upp[1];
    double sz = (p.look[2] + a * p.right[2]) + b * p.upp[2];
    double dx = sx - p.eye[0], dy = sy - p.eye[1], dz = sz - p.eye[2];
    double v = 0.0;
    for (int w = 0; w < work; ++w) {
        double l = sqrt(dx * dx + dy * dy + dz * dz);
        dx = dx / l, dy = dy / l, dz = dz / l;
        v += dx + dy + dz;
    }
    if (i < p.W && j < p.H) {
        size_t k = (size_t)j * p.W + i;
        out32[k] = make_float4((float)v, (float)dx, (float)dy, 1.0f);
        out8[k] = make_uchar4((unsigned char)(int)(v * 7.0), 0, 0, 255);
    }
}

template <int WORK>
__global__ __launch_bounds__(64) void wg64(P p, float4* o32, uchar4* o8) {
    const int lane = threadIdx.x;
    const int tx = blockIdx.x % p.tiles_x, ty = blockIdx.x / p.tiles_x;
    pixel(p, tx * 8 + (lane & 7), ty * 8 + (lane >> 3), o32, o8, WORK);
}

template <int WORK>
__global__ __launch_bounds__(256) void wg256(P p, float4* o32, uchar4* o8) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tx32 = (p.W + 31) / 32;
    const int tx = blockIdx.x % tx32, ty = blockIdx.x / tx32;
    pixel(p, tx * 32 + wave * 8 + (lane & 7), ty * 8 + (lane >> 3), o32, o8, WORK);
}

template <int WORK>
__global__ __launch_bounds__(64) void persist_static(P p, float4* o32, uchar4* o8) {
    const int lane = threadIdx.x;
    for (int t = blockIdx.x; t < p.ntiles; t += gridDim.x) {
        const int tx = t % p.tiles_x, ty = t / p.tiles_x;
        pixel(p, tx * 8 + (lane & 7), ty * 8 + (lane >> 3), o32, o8, WORK);
    }
}

template <int WORK>
__global__ __launch_bounds__(64) void persist_atomic(P p, float4* o32, uchar4* o8, unsigned* ctr) {
    const int lane = threadIdx.x;
    for (;;) {
        unsigned t = 0;
        if (lane == 0) t = atomicAdd(&ctr[0], 1u);
        t = __shfl(t, 0);
        if (t >= (unsigned)p.ntiles) break;
        const int tx = t % p.tiles_x, ty = t / p.tiles_x;
        pixel(p, tx * 8 + (lane & 7), ty * 8 + (lane >> 3), o32, o8, WORK);
    }
    // last wave out resets the counters for the next launch (stream order)
    if (lane == 0) {
        __threadfence();
        unsigned d = atomicAdd(&ctr[1], 1u);
        if (d == gridDim.x - 1) {
            ctr[0] = 0;
            ctr[1] = 0;
            __threadfence();
        }
    }
}

int main() {
    P p{};
    double eye[3] = {0, 100, 200}, look[3] = {0, 0, -160};
    for (int c = 0; c < 3; ++c) p.eye[c] = eye[c], p.look[c] = look[c];
    p.right[0] = 1;
    p.upp[1] = 0.96, p.upp[2] = 0.27;
    p.pitch = 500.0 / 1920;
    p.bx = -960, p.by = -540, p.W = 1920, p.H = 1080;
    p.tiles_x = p.W / 8;
    p.ntiles = p.tiles_x * ((p.H + 7) / 8);
    float4* o32;
    uchar4* o8;
    unsigned* ctr;
    hipMalloc(&o32, (size_t)p.W * p.H * 16);
    hipMalloc(&o8, (size_t)p.W * p.H * 4);
    hipMalloc(&ctr, 8);
    hipMemset(ctr, 0, 8);
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    auto timeit = [&](const char* name, int work, auto launch) {
        launch();
        hipDeviceSynchronize();
        float best = 1e9;
        for (int round = 0; round < 5; ++round) {
            hipEventRecord(e0);
            for (int r = 0; r < 50; ++r) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            best = fminf(best, ms * 1000 / 50);
        }
        printf("{\"kernel\": \"%s\", \"work\": %d, \"us\": %.2f}\n", name, work, best);
    };
    const int tiles256 = ((p.W + 31) / 32) * ((p.H + 7) / 8);
#define RUN(WORK)                                                                                         \
    timeit("wg64", WORK, [&] { wg64<WORK><<<p.ntiles, 64>>>(p, o32, o8); });                              \
    timeit("wg256", WORK, [&] { wg256<WORK><<<tiles256, 256>>>(p, o32, o8); });                           \
    for (int w : {4, 8, 16}) {                                                                            \
        char nm[64];                                                                                      \
        snprintf(nm, 64, "static%d", w);                                                                  \
        timeit(nm, WORK, [&] { persist_static<WORK><<<cus * 4 * w, 64>>>(p, o32, o8); });                 \
        snprintf(nm, 64, "atomic%d", w);                                                                  \
        timeit(nm, WORK, [&] { persist_atomic<WORK><<<cus * 4 * w, 64>>>(p, o32, o8, ctr); });            \
    }
    RUN(0)
    RUN(1)
    RUN(4)
    return 0;
}
