// san_main.cpp — TEST INFRASTRUCTURE: drives the host half of the C ABI (csrc/rt_host.cpp), the faithful
// rayTraceScreen chain (csrc/rt_screen.cpp, traced through san_stubs.cpp) and the oracle (oracle/rt_oracle.c)
// under -fsanitize=address,undefined.  Checks results as it goes; prints "sanitize ok" at the end.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "../../ray_tracer_fragment_shader_amd/csrc/rt_internal.hpp"

extern "C" {
int oracle_local_rows(int H, const rt_rows* r);
int oracle_render(const rt_scene* d, const rt_camera* c, int W, int H, int depth, const rt_rows* rows, double* rgb,
                  uint32_t* raycount, int nthreads);
int oracle_intersect(const rt_scene* d, const double* starts, const double* ends, int n, rt_hit* hits);
int oracle_render_screen(const rt_scene* d, const double eye[3], const double look[3], const double up[3],
                         int bottom_x, int bottom_y, int W, int H, int depth, int rng_kind, uint32_t seed,
                         double* rgb, uint8_t* nsamples, uint64_t* rand_calls);
}

static int g_fail = 0;
#define CHECK(cond)                                                                   \
    do {                                                                              \
        if (!(cond)) {                                                                \
            std::fprintf(stderr, "%s:%d: check failed: %s\n", __FILE__, __LINE__, #cond); \
            ++g_fail;                                                                 \
        }                                                                             \
    } while (0)

static unsigned g_rng = 12345;
static int rnd(int n) {
    g_rng = g_rng * 1103515245u + 12345u;
    return (int)((g_rng >> 8) % (unsigned)n);
}

// Row bands: every image row of every frame belongs to exactly one (rank, local row).
static void check_bands() {
    const int Hs[] = {1, 2, 7, 97, 133, 1080, 2160};
    for (int H : Hs)
        for (int G = 1; G <= 9; ++G)
            for (int hb : {1, 3, 8, 15, 16, 400})
                for (int frames : {1, 2, 3}) {
                    std::vector<int> seen((size_t)H * frames, 0);
                    for (int r = 0; r < G; ++r) {
                        rt_rows rows = {hb, G, r, frames};
                        int nl = -1;
                        CHECK(rt_local_rows(H, &rows, &nl) == RT_OK);
                        CHECK(nl == oracle_local_rows(H, &rows));
                        for (int lr = 0; lr < nl; ++lr) {
                            int j = -1;
                            CHECK(rt_global_row(H, &rows, lr, &j) == RT_OK);
                            if (j >= 0 && j < H * frames) ++seen[j];
                        }
                        int j = 0;
                        CHECK(rt_global_row(H, &rows, nl, &j) == RT_EINVAL);
                    }
                    for (int v : seen) CHECK(v == 1);
                    int band = 0, slab = 0;
                    CHECK(rt_band_plan(H, G, 0, &band, &slab) == RT_OK);
                    CHECK(band >= 1 && slab >= 1);
                }
    rt_rows bad = {0, 2, 0, 1};
    int nl;
    CHECK(rt_local_rows(10, &bad, &nl) == RT_EINVAL);
}

static void check_squares_and_scenes() {
    for (char r = 'a'; r <= 'h'; ++r)
        for (char c = '1'; c <= '8'; ++c) {
            char sq[3] = {r, c, 0};
            double p[3];
            CHECK(rt_convert_string_coordinate(sq, p) == RT_OK);
            CHECK(std::fabs(p[0]) <= 140 && p[1] == 60 && std::fabs(p[2]) <= 140);
        }
    CHECK(rt_convert_string_coordinate("a", nullptr) == RT_EINVAL);
    // random boards through loadScene, including undersized buffers and duplicate squares
    for (int it = 0; it < 300; ++it) {
        int n = rnd(40);
        std::vector<std::string> sq(n);
        std::vector<const char*> p(n);
        std::vector<int32_t> ty(n);
        for (int k = 0; k < n; ++k) {
            sq[k] = std::string(1, (char)('a' + rnd(8))) + (char)('1' + rnd(8));
            p[k] = sq[k].c_str();
            ty[k] = rnd(6);
        }
        const int cap = rnd(3) == 0 ? rnd(5) : 64;
        std::vector<rt_sphere> sb(cap > 0 ? cap : 1);
        std::vector<rt_mesh> mb(cap > 0 ? cap : 1);
        rt_scene s;
        rt_light l;
        int rc = rt_load_scene(p.data(), ty.data(), n, &s, sb.data(), cap, mb.data(), cap, &l);
        CHECK(rc == RT_OK || rc == RT_EUNSUPPORTED || rc == RT_EINVAL);
        if (rc == RT_EINVAL) continue;
        CHECK(s.n_spheres <= cap && s.n_meshes <= cap);
        std::vector<unsigned char> blob;
        int b = rt_build_dev_scene(&s, &blob);
        CHECK(b == RT_OK || b == RT_EUNSUPPORTED);
        // oracle frames of the same scene at a tiny size, banded
        rt_camera cam;
        CHECK(rt_camera_init_reference(&cam, 9, 7, 30.0) == RT_OK);
        rt_rows rows = {2, 3, it % 3, 1 + it % 2};
        const int nl = oracle_local_rows(7, &rows);
        std::vector<double> rgb((size_t)nl * 9 * 3);
        std::vector<uint32_t> rcnt((size_t)nl * 9);
        CHECK(oracle_render(&s, &cam, 9, 7, rnd(8), &rows, rgb.data(), rcnt.data(), 1) == RT_OK);
    }
    // spheres at the limits, every material flag, the empty scene
    rt_scene s;
    CHECK(rt_scene_init_reference(&s) == RT_OK);
    std::vector<rt_sphere> big(RT_MAX_SPHERES);
    for (int k = 0; k < RT_MAX_SPHERES; ++k) {
        big[k].center[0] = rnd(300) - 150.0;
        big[k].center[1] = rnd(100);
        big[k].center[2] = rnd(300) - 150.0;
        big[k].radius = 1 + rnd(30);
    }
    rt_light lights[RT_MAX_LIGHTS];
    for (auto& l : lights) {
        for (int q = 0; q < 3; ++q) l.color[q] = 0.5, l.position[q] = rnd(400) - 200.0;
    }
    s.spheres = big.data();
    s.n_spheres = RT_MAX_SPHERES;
    s.lights = lights;
    s.n_lights = RT_MAX_LIGHTS;
    std::vector<unsigned char> blob;
    CHECK(rt_build_dev_scene(&s, &blob) == RT_OK);
    s.n_spheres = RT_MAX_SPHERES + 1;
    CHECK(rt_build_dev_scene(&s, &blob) == RT_EINVAL);
    s.n_spheres = 0;
    s.n_lights = 0;
    s.has_board = 0;
    CHECK(rt_build_dev_scene(&s, &blob) == RT_OK);
    CHECK(rt_build_dev_scene(nullptr, &blob) == RT_EINVAL);
    // intersections of random rays with a mesh board
    const char* sq[4] = {"b6", "b4", "d7", "a7"};
    int32_t ty[4] = {0, 1, 3, 2};
    rt_sphere sb[4];
    rt_mesh mb[4];
    rt_light l;
    CHECK(rt_load_scene(sq, ty, 4, &s, sb, 4, mb, 4, &l) == RT_OK);
    std::vector<double> a(3 * 512), e(3 * 512);
    for (auto& v : a) v = rnd(500) - 250.0;
    for (size_t k = 0; k < e.size(); ++k) e[k] = a[k] + rnd(200) - 100.0;
    std::vector<rt_hit> hits(512);
    CHECK(oracle_intersect(&s, a.data(), e.data(), 512, hits.data()) == RT_OK);
}

static void check_ppm() {
    for (int ch : {3, 4})
        for (int W : {1, 3, 5, 17}) {
            const int H = 3;
            std::vector<uint8_t> px((size_t)W * H * ch);
            for (auto& v : px) v = (uint8_t)rnd(256);
            const char* path = "san_out.ppm";
            CHECK(rt_write_ppm(path, px.data(), W, H, ch) == RT_OK);
            FILE* f = std::fopen(path, "rb");
            CHECK(f != nullptr);
            if (!f) continue;
            std::vector<uint8_t> buf(64 + px.size());
            size_t n = std::fread(buf.data(), 1, buf.size(), f);
            std::fclose(f);
            char hdr[32];
            int hl = std::snprintf(hdr, sizeof(hdr), "P6 %d %d 255\n", W, H);
            CHECK(n == (size_t)hl + (size_t)W * H * 3);
            CHECK(std::memcmp(buf.data(), hdr, hl) == 0);
            std::remove(path);
        }
    uint8_t one[4] = {0, 0, 0, 0};
    CHECK(rt_write_ppm("san_out.ppm", one, 1, 1, 2) == RT_EINVAL);
}

// The speculative chunked rayTraceScreen chain against the serial restatement, bit for bit.
static void check_screen() {
    rt_ctx* ctx = nullptr;
    CHECK(rt_ctx_create(0, &ctx) == RT_OK);
    const char* sq[4] = {"b6", "b4", "d7", "a7"};
    int32_t ty[4] = {0, 1, 3, 2};
    rt_sphere sb[4];
    rt_mesh mb[4];
    rt_light l;
    rt_scene s;
    CHECK(rt_load_scene(sq, ty, 4, &s, sb, 4, mb, 4, &l) == RT_OK);
    // (120 x 90: enough object edges for chunks that break, so queued continuations are dropped — r04's two
    // chunks in flight)
    const int sizes[][3] = {{1, 1, 2}, {13, 7, 2}, {40, 3, 2}, {24, 24, 2}, {120, 90, 1}};
    for (auto& wh : sizes)
        for (int kind : {RT_RAND_GLIBC, RT_RAND_MSVC}) {
            if (kind == RT_RAND_MSVC && wh[2] < 2) continue;
            const int W = wh[0], H = wh[1];
            rt_camera cam;
            CHECK(rt_camera_init_reference(&cam, W, H, 1.0) == RT_OK);
            std::vector<double> rgb((size_t)W * H * 3), want(rgb.size());
            std::vector<uint8_t> rgba((size_t)W * H * 4), ns((size_t)W * H), want_ns(ns.size());
            uint64_t calls = 0, want_calls = 0;
            CHECK(rt_render_screen(ctx, &s, &cam, W, H, 5, kind, 7u, rgb.data(), rgba.data(), ns.data(), &calls) ==
                  RT_OK);
            CHECK(oracle_render_screen(&s, cam.eye, cam.look_at, cam.up, cam.bottom_x, cam.bottom_y, W, H, 5, kind,
                                       7u, want.data(), want_ns.data(), &want_calls) == RT_OK);
            CHECK(std::memcmp(rgb.data(), want.data(), rgb.size() * sizeof(double)) == 0);
            CHECK(ns == want_ns);
            CHECK(calls == want_calls);
        }
    rt_camera cam;
    rt_camera_init_reference(&cam, 4, 4, 1.0);
    CHECK(rt_render_screen(ctx, &s, &cam, 4, 4, 5, 9, 1u, nullptr, nullptr, nullptr, nullptr) == RT_EINVAL);
    CHECK(rt_render_screen(ctx, &s, &cam, 0, 4, 5, 0, 1u, nullptr, nullptr, nullptr, nullptr) == RT_EINVAL);
    rt_ctx_destroy(ctx);
}

int main() {
    check_bands();
    check_squares_and_scenes();
    check_ppm();
    check_screen();
    if (g_fail) {
        std::fprintf(stderr, "%d check(s) failed\n", g_fail);
        return 1;
    }
    std::printf("sanitize ok\n");
    return 0;
}
