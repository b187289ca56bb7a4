// Wave-slot probe (diagnostic): how many one-wave workgroups the hardware keeps resident per SIMD for a
// given VGPR / LDS footprint.  Each wave spins ~30 us, then lane 0 records {start, end, HW_ID}; the host
// reports the largest wave slot id seen and the peak concurrent waves per SIMD.
// build: hipcc -O3 --offload-arch=gfx950 tools/mb_slots.cpp -o tools/_var/mb_slots
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <map>
#include <vector>

template <int NV>
__global__ __launch_bounds__(64) void spin(uint64_t* rec, uint64_t ticks) {
    extern __shared__ char lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    // claim VGPRs v0 .. v(NV-1): the kernel descriptor then reserves NV registers per lane
    if constexpr (NV == 32) asm volatile("" ::: "v31");
    if constexpr (NV == 64) asm volatile("" ::: "v63");
    if constexpr (NV == 71) asm volatile("" ::: "v70");
    if constexpr (NV == 72) asm volatile("" ::: "v71");
    if constexpr (NV == 80) asm volatile("" ::: "v79");
    if constexpr (NV == 171) asm volatile("" ::: "v70", "s99");   // 71 VGPRs and 100 SGPRs (the c2 kernel)
    // 71 VGPRs and NV - 1000 SGPRs (next_free_sgpr): where the SGPR budget costs the seventh wave
    if constexpr (NV == 1080) asm volatile("" ::: "v70", "s79");
    if constexpr (NV == 1088) asm volatile("" ::: "v70", "s87");
    if constexpr (NV == 1090) asm volatile("" ::: "v70", "s89");
    if constexpr (NV == 1092) asm volatile("" ::: "v70", "s91");
    if constexpr (NV == 1094) asm volatile("" ::: "v70", "s93");
    if constexpr (NV == 1096) asm volatile("" ::: "v70", "s95");
    if constexpr (NV == 1098) asm volatile("" ::: "v70", "s97");
    // 63 VGPRs (8 waves by VGPRs) and NV - 2000 SGPRs: where the SGPR budget costs the eighth / seventh wave (r04)
    if constexpr (NV == 2064) asm volatile("" ::: "v62", "s63");
    if constexpr (NV == 2072) asm volatile("" ::: "v62", "s71");
    if constexpr (NV == 2080) asm volatile("" ::: "v62", "s79");
    if constexpr (NV == 2084) asm volatile("" ::: "v62", "s83");
    if constexpr (NV == 2088) asm volatile("" ::: "v62", "s87");
    if constexpr (NV == 2092) asm volatile("" ::: "v62", "s91");
    if constexpr (NV == 2096) asm volatile("" ::: "v62", "s95");
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        lds[0] = 1;
        const size_t w = blockIdx.x;
        rec[3 * w] = t0;
        rec[3 * w + 1] = __builtin_amdgcn_s_memrealtime();
        rec[3 * w + 2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                         ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
    }
}

template <int NV>
static void run(uint64_t* d, std::vector<uint64_t>& h, int n, size_t lds) {
    hipLaunchKernelGGL(spin<NV>, dim3(n), dim3(64), lds, 0, d, (uint64_t)3000);
    if (hipDeviceSynchronize() != hipSuccess) { std::printf("launch failed\n"); return; }
    hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::map<uint64_t, std::vector<std::pair<uint64_t, int>>> ev;
    int maxwid = 0;
    for (int w = 0; w < n; ++w) {
        const uint64_t hw = h[3 * w + 2], id = hw & 0xffffffffu, xcc = (hw >> 32) & 0xf;
        maxwid = std::max(maxwid, (int)(id & 0xf));
        const uint64_t key = (xcc << 16) | (((id >> 13) & 7) << 8) | (((id >> 8) & 0xf) << 2) | ((id >> 4) & 3);
        ev[key].push_back({h[3 * w], 1});
        ev[key].push_back({h[3 * w + 1], -1});
    }
    int peak = 0;
    double mean_peak = 0;
    for (auto& kv : ev) {
        auto& v = kv.second;
        std::sort(v.begin(), v.end(), [](auto a, auto b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
        int c = 0, p = 0;
        for (auto& e : v) { c += e.second; p = std::max(p, c); }
        peak = std::max(peak, p);
        mean_peak += p;
    }
    std::printf("{\"vgprs\": %d, \"lds\": %zu, \"simds\": %zu, \"max_wave_slot_id\": %d, \"peak_per_simd\": %d, "
                "\"mean_peak_per_simd\": %.2f}\n", NV, lds, ev.size(), maxwid, peak, mean_peak / ev.size());
}

int main() {
    const int n = 256 * 4 * 10;
    uint64_t* d;
    hipMalloc(&d, (size_t)n * 3 * 8);
    std::vector<uint64_t> h((size_t)n * 3);
    for (size_t lds : {(size_t)4608}) {
        run<71>(d, h, n, lds);
        run<171>(d, h, n, lds);
        run<1080>(d, h, n, lds);
        run<1088>(d, h, n, lds);
        run<1090>(d, h, n, lds);
        run<1092>(d, h, n, lds);
        run<1094>(d, h, n, lds);
        run<1096>(d, h, n, lds);
        run<1098>(d, h, n, lds);
        run<2064>(d, h, n, lds);
        run<2072>(d, h, n, lds);
        run<2080>(d, h, n, lds);
        run<2084>(d, h, n, lds);
        run<2088>(d, h, n, lds);
        run<2092>(d, h, n, lds);
        run<2096>(d, h, n, lds);
    }
    hipFree(d);
    return 0;
}
