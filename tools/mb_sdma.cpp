// mb_sdma.cpp — can a frame's device-to-host copy run on a copy (SDMA) engine instead of a blit kernel?  (diagnostic for
// the draw() path: the blit / copy kernels share the CUs with the next frame's render and slow it.)
// A 1920 x 1080 GRAY8 frame (2,073,600 B) from hipMalloc memory into hipHostMalloc memory:
//   hip        hipMemcpyAsync (the runtime's choice of engine)
//   hsa        hsa_amd_memory_async_copy (the HSA runtime's choice)
//   sdma<k>    hsa_amd_memory_async_copy_on_engine on SDMA engine k (each engine hsa_amd_memory_copy_engine_status
//              reports free), forced onto the engine
// each alone, and each while a busy kernel (all CUs, ~VALU spin) runs, whose own time is reported beside.
// One JSON line per case: median microseconds of REPS copies.
// build: hipcc -O3 --offload-arch=gfx950 tools/mb_sdma.cpp -o tools/_var/mb_sdma -lhsa-runtime64
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } \
    } while (0)
#define HK(x)                                                                               \
    do {                                                                                    \
        hsa_status_t s_ = (x);                                                              \
        if (s_ != HSA_STATUS_SUCCESS) { const char* m = nullptr; hsa_status_string(s_, &m);  \
            fprintf(stderr, "%s: %s\n", #x, m ? m : "?"); exit(1); }                         \
    } while (0)

static hsa_agent_t g_gpu{0}, g_cpu{0};
static hsa_status_t find_agents(hsa_agent_t a, void*) {
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU && g_gpu.handle == 0) g_gpu = a;
    if (t == HSA_DEVICE_TYPE_CPU && g_cpu.handle == 0) g_cpu = a;
    return HSA_STATUS_SUCCESS;
}

__global__ void busy(float* out, int iters) {
    float x = threadIdx.x * 1e-3f, y = 1.0f;
    for (int i = 0; i < iters; ++i) { x = fmaf(x, 0.999f, y); y = fmaf(y, 1.0001f, -x * 1e-6f); }
    if (x == 12345.0f) out[0] = y;
}

__global__ void fire(int64_t* v) {
    if (threadIdx.x == 0) __hip_atomic_store(v, (int64_t)0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const size_t n = 1920 * 1080;
    const int reps = getenv("REPS") ? atoi(getenv("REPS")) : 30;
    void *d_src, *h_dst;
    float* d_out;
    CK(hipSetDevice(0));
    CK(hipMalloc(&d_src, n));
    CK(hipMalloc(&d_out, 64));
    CK(hipMemset(d_src, 5, n));
    CK(hipHostMalloc(&h_dst, n, hipHostMallocDefault));
    HK(hsa_init());
    HK(hsa_iterate_agents(find_agents, nullptr));
    uint32_t mask = 0;
    HK(hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &mask));
    printf("{\"sdma_engines_free_mask\": %u}\n", mask);
    hsa_signal_t sig;
    HK(hsa_signal_create(1, 0, nullptr, &sig));
    hipStream_t ks;
    CK(hipStreamCreateWithFlags(&ks, hipStreamNonBlocking));
    hipEvent_t k0, k1;
    CK(hipEventCreate(&k0));
    CK(hipEventCreate(&k1));

    struct Case { std::string name; std::function<void()> copy; };
    std::vector<Case> cases;
    cases.push_back({"hip", [&] { CK(hipMemcpyAsync(h_dst, d_src, n, hipMemcpyDeviceToHost, 0)); CK(hipStreamSynchronize(0)); }});
    cases.push_back({"hsa", [&] {
        hsa_signal_store_relaxed(sig, 1);
        HK(hsa_amd_memory_async_copy(h_dst, g_cpu, d_src, g_gpu, n, 0, nullptr, sig));
        while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {}
    }});
    for (int k = 0; k < 16; ++k) {
        if (!(mask & (1u << k)) || k >= (getenv("ENGINES") ? atoi(getenv("ENGINES")) : 16)) continue;
        const hsa_amd_sdma_engine_id_t eng = (hsa_amd_sdma_engine_id_t)(1u << k);
        cases.push_back({"sdma" + std::to_string(k), [&, eng] {
            hsa_signal_store_relaxed(sig, 1);
            HK(hsa_amd_memory_async_copy_on_engine(h_dst, g_cpu, d_src, g_gpu, n, 0, nullptr, sig, eng, true));
            while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {}
        }});
    }
    // the frame in halves on two engines at once (one completion signal counting both): does PCIe take more than one
    // engine's rate?
    {
        int e0 = -1, e1 = -1;
        for (int k = 0; k < 16; ++k)
            if (mask & (1u << k)) { if (e0 < 0) e0 = k; else if (e1 < 0) e1 = k; }
        if (e1 >= 0) {
            const hsa_amd_sdma_engine_id_t a = (hsa_amd_sdma_engine_id_t)(1u << e0), b = (hsa_amd_sdma_engine_id_t)(1u << e1);
            cases.push_back({"sdma" + std::to_string(e0) + "+" + std::to_string(e1) + "_halves", [&, a, b] {
                hsa_signal_store_relaxed(sig, 2);
                HK(hsa_amd_memory_async_copy_on_engine(h_dst, g_cpu, d_src, g_gpu, n / 2, 0, nullptr, sig, a, true));
                HK(hsa_amd_memory_async_copy_on_engine((char*)h_dst + n / 2, g_cpu, (char*)d_src + n / 2, g_gpu, n - n / 2,
                                                       0, nullptr, sig, b, true));
                while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE) != 0) {}
            }});
        }
    }
    // busy kernel alone
    const int iters = getenv("ITERS") ? atoi(getenv("ITERS")) : 20000;
    auto run_busy = [&] { hipLaunchKernelGGL(busy, dim3(256 * 16), dim3(256), 0, ks, d_out, iters); };
    std::vector<double> kb;
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(k0, ks));
        run_busy();
        CK(hipEventRecord(k1, ks));
        CK(hipEventSynchronize(k1));
        float ms;
        CK(hipEventElapsedTime(&ms, k0, k1));
        kb.push_back(ms * 1e3);
    }
    printf("{\"busy_kernel_alone_us\": %.1f}\n", median(kb));
    for (auto& c : cases) {
        for (int r = 0; r < 3; ++r) c.copy();
        std::vector<double> t;
        for (int r = 0; r < reps; ++r) {
            auto a = std::chrono::steady_clock::now();
            c.copy();
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
        }
        // the same copies while the busy kernel runs: copy time, and the kernel's own time
        std::vector<double> tb, kt;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(k0, ks));
            run_busy();
            CK(hipEventRecord(k1, ks));
            int m = 0;
            while (hipEventQuery(k1) == hipErrorNotReady && m < 1000) {
                auto a = std::chrono::steady_clock::now();
                c.copy();
                tb.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
                ++m;
            }
            CK(hipEventSynchronize(k1));
            float ms;
            CK(hipEventElapsedTime(&ms, k0, k1));
            kt.push_back(ms * 1e3);
        }
        printf("{\"copy\": \"%s\", \"us\": %.1f, \"min_us\": %.1f, \"GBps\": %.1f, \"us_beside_busy_kernel\": %.1f, "
               "\"copies_beside\": %zu, \"busy_kernel_us_with_copies\": %.1f, \"check\": %d}\n",
               c.name.c_str(), median(t), *std::min_element(t.begin(), t.end()), n / median(t) / 1e3,
               tb.empty() ? -1.0 : median(tb), tb.size(), median(kt), (int)((unsigned char*)h_dst)[777]);
    }
    // GPU-triggered (the draw() design): a kernel writes the frame into d_src on a HIP stream, the stream then stores 0
    // into an HSA signal (GPU_ONLY, so its value pointer may be written) — writer 1: hipStreamWriteValue64, writer 2: a
    // one-wave kernel's system-scope store — and an SDMA copy queued beforehand with that signal as its dependency moves
    // the frame once it fires.  Checked byte for byte; a dependency that never fires is released from the host after
    // 100 ms (reported), so no copy is left waiting.
    for (int writer = 1; writer <= 2 && mask; ++writer) {
        int k = 0;
        while (!(mask & (1u << k))) ++k;
        const hsa_amd_sdma_engine_id_t eng = (hsa_amd_sdma_engine_id_t)(1u << k);
        hsa_signal_t dep;
        HK(hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &dep));
        volatile hsa_signal_value_t* dep_ptr = nullptr;
        HK(hsa_amd_signal_value_pointer(dep, &dep_ptr));
        hsa_signal_store_screlease(dep, 1);             // can this writer fire it at all?
        hipError_t we = writer == 1 ? hipStreamWriteValue64(ks, (void*)dep_ptr, 0, 0) : hipSuccess;
        if (writer == 2) { hipLaunchKernelGGL(fire, dim3(1), dim3(64), 0, ks, (int64_t*)dep_ptr); we = hipGetLastError(); }
        const hipError_t se = hipStreamSynchronize(ks);
        printf("{\"writer\": %d, \"queue\": \"%s\", \"sync\": \"%s\", \"fired\": %d}\n", writer, hipGetErrorString(we),
               hipGetErrorString(se), (int)(hsa_signal_load_scacquire(dep) == 0));
        fflush(stdout);
        if (we != hipSuccess || se != hipSuccess || hsa_signal_load_scacquire(dep) != 0) {
            (void)hipGetLastError();
            HK(hsa_signal_destroy(dep));
            continue;
        }
        std::vector<double> t;
        int bad = 0, released = 0;
        for (int r = 0; r < reps; ++r) {
            hsa_signal_store_relaxed(dep, 1);
            hsa_signal_store_relaxed(sig, 1);
            const unsigned char v = (unsigned char)(r + 1);
            auto a = std::chrono::steady_clock::now();
            HK(hsa_amd_memory_async_copy_on_engine(h_dst, g_cpu, d_src, g_gpu, n, 1, &dep, sig, eng, true));
            CK(hipMemsetAsync(d_src, v, n, ks));                                 // "the render"
            if (writer == 1) CK(hipStreamWriteValue64(ks, (void*)dep_ptr, 0, 0));
            else hipLaunchKernelGGL(fire, dim3(1), dim3(64), 0, ks, (int64_t*)dep_ptr);
            const auto deadline = std::chrono::steady_clock::now() + std::chrono::milliseconds(100);
            while (hsa_signal_load_scacquire(sig) != 0) {
                if (std::chrono::steady_clock::now() > deadline) {                // never fired: release it
                    hsa_signal_store_screlease(dep, 0);
                    ++released;
                    while (hsa_signal_load_scacquire(sig) != 0) {}
                    break;
                }
            }
            t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
            CK(hipStreamSynchronize(ks));
            for (size_t q = 0; q < n; q += 4099) bad += ((unsigned char*)h_dst)[q] != v;
        }
        printf("{\"copy\": \"sdma%d_after_stream\", \"writer\": %d, \"us_issue_to_done\": %.1f, \"min_us\": %.1f, "
               "\"mismatches\": %d, \"released_by_host\": %d}\n", k, writer, median(t), *std::min_element(t.begin(), t.end()),
               bad, released);
        HK(hsa_signal_destroy(dep));
    }
    HK(hsa_signal_destroy(sig));
    return 0;
}
