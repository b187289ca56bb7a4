// Refill probe (diagnostic): do one-wave workgroups of very different lengths keep every wave slot busy?  Each wave
// sleeps for the duration the same dispatch position took in a traced render launch (tools/wave_trace.py:
// tools/_var/<cfg>_durations.bin, float microseconds in dispatch order), then records {start, end, HW_ID}.  Per
// footprint (dynamic LDS bytes, VGPRs) it prints the launch span, the ideal span (sum of durations / wave slots) and
// the mean resident waves per CU — whether idle slots come from the durations themselves or from a resource the
// footprint holds (e.g. LDS).
// build: hipcc -O3 --offload-arch=gfx950 tools/mb_refill.cpp -o tools/_var/mb_refill
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <map>
#include <vector>

template <int NV>
__global__ __launch_bounds__(64) void sleeper(const float* __restrict__ dur_us, uint64_t* rec) {
    extern __shared__ char lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (NV == 72) asm volatile("" ::: "v71", "s93");
    if constexpr (NV == 64) asm volatile("" ::: "v63", "s93");
    if constexpr (NV == 32) asm volatile("" ::: "v31", "s63");
    const size_t w = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    const uint64_t ticks = (uint64_t)(dur_us[w] * 100.0f);          // s_memrealtime: 100 MHz
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
    if (threadIdx.x == 0) {
        lds[0] = 1;
        rec[3 * w] = t0;
        rec[3 * w + 1] = __builtin_amdgcn_s_memrealtime();
        rec[3 * w + 2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                         ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
    }
}

// Persistent variant: a fixed grid of one-wave workgroups (the resident maximum) takes dispatch positions from atomic
// counters — one per XCD (QPX = 1: queue j hands out j, j + 8, ... as the hardware dispatcher deals positions to XCD j)
// or one for the whole device (QPX = 0) — and fetches its next position while it sleeps the current one.
template <int QPX>
__global__ __launch_bounds__(64) void sleeper_persistent(const float* __restrict__ dur_us, uint64_t* rec, int n,
                                                         unsigned* counters) {
    const unsigned xcc = QPX ? (__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) & 7) : 0;
    const unsigned stride = QPX ? 8 : 1;
    unsigned k = 0;
    if (threadIdx.x == 0) k = atomicAdd(&counters[xcc * 16], 1u);
    k = __builtin_amdgcn_readfirstlane(k);
    while (true) {
        const unsigned w = xcc + stride * k;
        if (w >= (unsigned)n) break;
        unsigned next = 0;
        if (threadIdx.x == 0) next = atomicAdd(&counters[xcc * 16], 1u);     // in flight while this one sleeps
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t ticks = (uint64_t)(dur_us[w] * 100.0f);
        while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(4);
        if (threadIdx.x == 0) {
            rec[3 * w] = t0;
            rec[3 * w + 1] = __builtin_amdgcn_s_memrealtime();
            rec[3 * w + 2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                             ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
        }
        k = __builtin_amdgcn_readfirstlane(next);
    }
}

static void report(const char* cfg, int n, const std::vector<uint64_t>& h, int NV, size_t lds, int slots_per_simd,
                   double sum_us, const char* mode);

template <int NV>
static void run(const char* cfg, const float* d_dur, int n, int gx, uint64_t* d_rec, std::vector<uint64_t>& h,
                size_t lds, int slots_per_simd, double sum_us) {
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(sleeper<NV>, dim3(gx, n / gx), dim3(64), lds, 0, d_dur, d_rec);
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); exit(1); }
    }
    hipMemcpy(h.data(), d_rec, h.size() * 8, hipMemcpyDeviceToHost);
    report(cfg, n, h, NV, lds, slots_per_simd, sum_us, "grid");
}

static void report(const char* cfg, int n, const std::vector<uint64_t>& h, int NV, size_t lds, int slots_per_simd,
                   double sum_us, const char* mode) {
    uint64_t t0 = ~0ull, t1 = 0;
    std::map<uint64_t, double> busy;
    for (int w = 0; w < n; ++w) {
        t0 = std::min(t0, h[3 * w]);
        t1 = std::max(t1, h[3 * w + 1]);
        const uint64_t hw = h[3 * w + 2], id = hw & 0xffffffffu, xcc = (hw >> 32) & 0xf;
        const uint64_t cu = (xcc << 16) | (((id >> 13) & 7) << 8) | ((id >> 8) & 0xf);
        busy[cu] += (h[3 * w + 1] - h[3 * w]) * 0.01;
    }
    const double span = (t1 - t0) * 0.01;
    double mean = 0;
    for (auto& kv : busy) mean += kv.second / span;
    mean /= busy.size();
    const double ideal = sum_us / (busy.size() * 4.0 * slots_per_simd);
    std::printf("{\"durations\": \"%s\", \"mode\": \"%s\", \"vgprs\": %d, \"lds\": %zu, \"span_us\": %.1f, "
                "\"ideal_span_us\": %.1f, \"mean_resident_per_cu\": %.2f, \"cus\": %zu}\n", cfg, mode, NV, lds, span, ideal,
                mean, busy.size());
}

template <int QPX>
static void run_persistent(const char* cfg, const float* d_dur, int n, uint64_t* d_rec, unsigned* d_cnt,
                           std::vector<uint64_t>& h, int slots_per_simd, double sum_us, int cus) {
    const int grid = cus * 4 * slots_per_simd;
    for (int rep = 0; rep < 2; ++rep) {
        hipMemset(d_cnt, 0, 8 * 16 * 4);
        hipMemset(d_rec, 0, h.size() * 8);
        hipLaunchKernelGGL(sleeper_persistent<QPX>, dim3(grid), dim3(64), 0, 0, d_dur, d_rec, n, d_cnt);
        if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); exit(1); }
    }
    hipMemcpy(h.data(), d_rec, h.size() * 8, hipMemcpyDeviceToHost);
    report(cfg, n, h, 72, 0, slots_per_simd, sum_us, QPX ? "persistent_per_xcd_queue" : "persistent_one_queue");
}

int main(int argc, char** argv) {
    const char* cfg = argc > 1 ? argv[1] : "c5";
    const int gx = argc > 2 ? atoi(argv[2]) : 960;
    char path[256];
    std::snprintf(path, sizeof path, "tools/_var/%s_durations.bin", cfg);
    FILE* f = std::fopen(path, "rb");
    if (!f) { std::printf("missing %s\n", path); return 1; }
    std::vector<float> dur;
    float x;
    while (std::fread(&x, 4, 1, f) == 1) dur.push_back(x);
    std::fclose(f);
    const int n = (int)dur.size();
    double sum = 0;
    for (float v : dur) sum += v;
    float* d_dur;
    uint64_t* d_rec;
    hipMalloc(&d_dur, n * 4);
    hipMemcpy(d_dur, dur.data(), n * 4, hipMemcpyHostToDevice);
    hipMalloc(&d_rec, (size_t)n * 3 * 8);
    std::vector<uint64_t> h((size_t)n * 3);
    for (size_t lds : {(size_t)0, (size_t)4608, (size_t)9216}) {
        run<72>(cfg, d_dur, n, gx, d_rec, h, lds, 7, sum);
    }
    run<64>(cfg, d_dur, n, gx, d_rec, h, 0, 7, sum);
    run<32>(cfg, d_dur, n, gx, d_rec, h, 0, 8, sum);
    unsigned* d_cnt;
    hipMalloc(&d_cnt, 8 * 16 * 4);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    run_persistent<1>(cfg, d_dur, n, d_rec, d_cnt, h, 7, sum, prop.multiProcessorCount);
    run_persistent<0>(cfg, d_dur, n, d_rec, d_cnt, h, 7, sum, prop.multiProcessorCount);
    hipFree(d_cnt);
    hipFree(d_dur);
    hipFree(d_rec);
    return 0;
}
