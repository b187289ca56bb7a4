// TEST INFRASTRUCTURE: host-side phase timing of rt_render_screen (build / resolve) on the CPU, with the
// device entry points of san_stubs.cpp (rays traced by the oracle, synchronously inside the build phase).
// make prof && RT_SCREEN_PROFILE=1 ./_build/screen_prof [W H]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../include/rt_api.h"

int main(int argc, char** argv) {
    const int W = argc > 2 ? atoi(argv[1]) : 500, H = argc > 2 ? atoi(argv[2]) : 500;
    rt_ctx* ctx = nullptr;
    if (rt_ctx_create(0, &ctx)) return 1;
    const char* sq[4] = {"b6", "b4", "d7", "a7"};
    int32_t ty[4] = {0, 1, 3, 2};
    rt_sphere sb[4];
    rt_mesh mb[4];
    rt_light l;
    rt_scene s;
    if (rt_load_scene(sq, ty, 4, &s, sb, 4, mb, 4, &l)) return 1;
    rt_camera cam;
    rt_camera_init_reference(&cam, W, H, 1.0);
    std::vector<double> rgb((size_t)W * H * 3);
    std::vector<uint8_t> ns((size_t)W * H);
    uint64_t calls = 0;
    const auto t0 = std::chrono::steady_clock::now();
    int rc = rt_render_screen(ctx, &s, &cam, W, H, 5, RT_RAND_GLIBC, 1u, rgb.data(), nullptr, ns.data(), &calls);
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    long long n = 0;
    for (uint8_t v : ns) n += v;
    printf("rc %d, %lld samples, %llu rand calls, %.3f s total (oracle tracing included)\n", rc, n,
           (unsigned long long)calls, t);
    rt_ctx_destroy(ctx);
    return rc;
}
