// rt_cli.cpp — `rt_render`: the reference application's frame flow on the MI355X path.
//
// Reference flow (Hw4/MySdlApplication.cpp): onInit -> initScene2 (stdin dialogue, :1430-1493) ->
// loadScene (:1495-1539) -> every frame draw() (:1541-1563) -> rayTraceScreen -> GL points; a screenshot
// would go through writePpmScreenshot (Hw4/ppm.cpp:15-25).  Here: the same dialogue (or a canonical
// scene) -> rt_load_scene -> rt_render (one HIP launch) -> RGBA8 -> rt_write_ppm.  No SDL/GL window:
// the image goes to a PPM file (the output path the reference already has).
//
//   rt_render --config c2 --out c2.ppm            canonical scene
//   rt_render --config demo --out demo.ppm        initScene's demo (tetrahedron, sphere, cube), 500x500
//   rt_render --stdin --width 500 --height 500 --pitch 1 --out app.ppm < answers.txt
//                                                  initScene2's questions answered on stdin
//   rt_render --config demo --faithful glibc|msvc [--seed S] --out demo_ref.ppm
//                                                  rayTraceScreen exactly as the app runs it (jitter, up to
//                                                  16 adaptive samples, colour carry-over): rt_render_screen
//   rt_render --config c4 --gpus 8 [--band H] [--repeat K] --out c4.ppm
//                                                  one frame's rows split over 8 GPUs (rt_group, RCCL gather to
//                                                  GPU 0); with fewer GPUs than --gpus the
//                                                  contexts share devices and the gather is a device copy
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../include/rt_api.h"

namespace {

struct Options {
    std::string config = "c2";
    std::string out = "frame.ppm";
    bool from_stdin = false;
    int width = 0, height = 0, depth = -1, device = 0;
    double pitch = 0;
    int faithful = -1;                       // RT_RAND_GLIBC / RT_RAND_MSVC: rt_render_screen
    unsigned seed = 1;
    int gpus = 0;                            // > 0: rt_group over this many ranks (rt_render_multi)
    int band = 0;                            // band height (0: auto)
    int repeat = 1;                          // frames rendered (the last one is written)
};

[[noreturn]] void die(const std::string& what, int code) {
    std::fprintf(stderr, "rt_render: %s failed (%d): %s\n", what.c_str(), code, rt_last_error());
    std::exit(1);
}

void check(int code, const char* what) {
    if (code != RT_OK) die(what, code);
}

// initScene2 (:1430-1493): "(a) light, (b) tetrahedron, (c) cube, (d) sphere, (e) cylinder, (f) cone",
// then a square "a1-h8", then "yes/no" for another object.  Returns the boardMap entries in input order.
void read_dialogue(std::vector<std::string>* squares, std::vector<int32_t>* types) {
    std::string tmp;
    bool finished = false;
    while (!finished) {
        bool answered = false;
        while (!answered) {
            std::cout << "Please select the type of object to add:\n"
                      << "(a) light, (b) tetrahedron, (c) cube, (d) sphere, (e) cylinder, (f) cone" << std::endl;
            if (!(std::cin >> tmp)) return;
            answered = tmp.size() <= 1;
            int type = tmp[0] - 'a';
            if (type >= 0 && type < 6) {
                std::cout << "Please enter the position: (a1-h8)" << std::endl;
                if (!(std::cin >> tmp)) return;
                squares->push_back(tmp);
                types->push_back(type);
            } else {
                answered = false;
            }
        }
        answered = false;
        while (!answered) {
            std::cout << "Would you like to add another object? (yes/no)" << std::endl;
            if (!(std::cin >> tmp)) return;
            if (tmp == "no" || tmp == "n") finished = answered = true;
            else if (tmp == "yes" || tmp == "y") answered = true;
        }
    }
}

struct Canonical {
    int w, h, nsph, nl, depth;
};

Canonical canonical(const std::string& c) {
    if (c == "c1") return {640, 480, 3, 1, 0};
    if (c == "c2") return {1920, 1080, 8, 1, 1};
    if (c == "c3" || c == "c4") return {3840, 2160, 8, 2, 2};
    if (c == "c5") return {7680, 4320, 64, 2, 3};
    std::fprintf(stderr, "rt_render: unknown config %s\n", c.c_str());
    std::exit(2);
}

void hip_check(hipError_t e, const char* what) {
    if (e != hipSuccess) {
        std::fprintf(stderr, "rt_render: %s failed: %s\n", what, hipGetErrorString(e));
        std::exit(1);
    }
}

// --gpus N: one context per rank on device q % (devices), one rt_group, rt_render_multi into an RGBA8 image
// on rank 0's device (draw()'s frame, MySdlApplication.cpp:1541-1563, with its rows split over the GPUs).
int render_multi(const Options& o, const rt_scene& scene, const rt_camera& cam, int W, int H, int depth) {
    int ndev = 0;
    check(rt_device_count(&ndev), "rt_device_count");
    std::vector<rt_ctx*> ctxs(o.gpus, nullptr);
    for (int q = 0; q < o.gpus; ++q) {
        check(rt_ctx_create(q % ndev, &ctxs[q]), "rt_ctx_create");
        check(rt_set_scene(ctxs[q], &scene), "rt_set_scene");
    }
    rt_group* g = nullptr;
    check(rt_group_create(ctxs.data(), o.gpus, RT_TRANSPORT_AUTO, &g), "rt_group_create");
    int transport = 0, band = 0, slab = 0;
    check(rt_group_info(g, nullptr, nullptr, nullptr, &transport), "rt_group_info");
    check(rt_band_plan(H, o.gpus, o.band, &band, &slab), "rt_band_plan");
    hip_check(hipSetDevice(0), "hipSetDevice");
    uint8_t* d8 = nullptr;
    hip_check(hipMalloc(&d8, (size_t)W * H * 4), "hipMalloc");
    hipStream_t st = nullptr;
    hip_check(hipStreamCreate(&st), "hipStreamCreate");
    check(rt_render_multi(g, &cam, W, H, depth, o.band, RT_OUT_RGBA8, nullptr, d8, st), "rt_render_multi");
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");                  // first frame (setup)
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < o.repeat; ++k)
        check(rt_render_multi(g, &cam, W, H, depth, o.band, RT_OUT_RGBA8, nullptr, d8, st), "rt_render_multi");
    hip_check(hipStreamSynchronize(st), "hipStreamSynchronize");
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / o.repeat;
    std::vector<uint8_t> rgba8((size_t)W * H * 4);
    hip_check(hipMemcpy(rgba8.data(), d8, rgba8.size(), hipMemcpyDeviceToHost), "hipMemcpy");
    check(rt_write_ppm(o.out.c_str(), rgba8.data(), W, H, 4), "rt_write_ppm");
    std::printf("rt_render: %dx%d depth %d over %d ranks (%d device(s), band %d rows, %s gather to rank 0) -> %s | "
                "%.3f ms per frame over %d frame(s)\n", W, H, depth, o.gpus, std::min(ndev, o.gpus), band,
                transport == RT_TRANSPORT_RCCL ? "RCCL" : "device-copy", o.out.c_str(), ms, o.repeat);
    rt_group_destroy(g);
    (void)hipFree(d8);
    (void)hipStreamDestroy(st);
    for (auto* c : ctxs) rt_ctx_destroy(c);
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    Options o;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&]() -> std::string {
            if (i + 1 >= argc) { std::fprintf(stderr, "missing value for %s\n", a.c_str()); std::exit(2); }
            return argv[++i];
        };
        if (a == "--config") o.config = next();
        else if (a == "--out") o.out = next();
        else if (a == "--stdin") o.from_stdin = true;
        else if (a == "--width") o.width = std::atoi(next().c_str());
        else if (a == "--height") o.height = std::atoi(next().c_str());
        else if (a == "--depth") o.depth = std::atoi(next().c_str());
        else if (a == "--pitch") o.pitch = std::atof(next().c_str());
        else if (a == "--device") o.device = std::atoi(next().c_str());
        else if (a == "--faithful") o.faithful = next() == "msvc" ? RT_RAND_MSVC : RT_RAND_GLIBC;
        else if (a == "--seed") o.seed = (unsigned)std::strtoul(next().c_str(), nullptr, 10);
        else if (a == "--gpus") o.gpus = std::atoi(next().c_str());
        else if (a == "--band") o.band = std::atoi(next().c_str());
        else if (a == "--repeat") o.repeat = std::max(1, std::atoi(next().c_str()));
        else { std::fprintf(stderr, "usage: rt_render [--config c1|c2|c3|c5|demo | --stdin] [--width W --height H "
                                    "--pitch P --depth B] [--device N] [--faithful glibc|msvc [--seed S]] "
                                    "[--gpus N [--band H]] [--repeat K] [--out file.ppm]\n"); return 2; }
    }

    rt_scene scene;
    std::vector<rt_sphere> spheres(RT_MAX_SPHERES);
    std::vector<rt_mesh> meshes(RT_MAX_MESHES);
    std::vector<rt_light> lights(2);
    int W, H, depth;
    double pitch;
    if (o.from_stdin) {
        std::vector<std::string> sq;
        std::vector<int32_t> ty;
        read_dialogue(&sq, &ty);
        std::vector<const char*> csq;
        for (auto& s : sq) csq.push_back(s.c_str());
        check(rt_load_scene(csq.data(), ty.data(), (int)csq.size(), &scene, spheres.data(), RT_MAX_SPHERES,
                            meshes.data(), RT_MAX_MESHES, &lights[0]),
              "rt_load_scene");
        W = o.width > 0 ? o.width : 500;                    // g_windowWidth/Height (:570)
        H = o.height > 0 ? o.height : 500;
        depth = o.depth >= 0 ? o.depth : 5;                 // MAX_DEPTH (:48)
        pitch = o.pitch > 0 ? o.pitch : 1.0;                // rayTraceScreen's unit pixel step
    } else if (o.config == "demo") {
        // initScene (MySdlApplication.cpp:1387-1428): light b6, tetrahedron b4, sphere d7 (r 20),
        // cube a7, inserted in that order after the board; the app's 500x500 window, MAX_DEPTH 5.
        check(rt_scene_init_reference(&scene), "rt_scene_init_reference");
        check(rt_convert_string_coordinate("d7", spheres[0].center), "rt_convert_string_coordinate");
        spheres[0].radius = 20.0;
        meshes[0] = rt_mesh{RT_MESH_TETRAHEDRON, 0, {0, 0, 0}, 40.0};
        meshes[1] = rt_mesh{RT_MESH_CUBE, 1, {0, 0, 0}, 40.0};
        check(rt_convert_string_coordinate("b4", meshes[0].position), "rt_convert_string_coordinate");
        check(rt_convert_string_coordinate("a7", meshes[1].position), "rt_convert_string_coordinate");
        check(rt_light_position_from_square("b6", lights[0].position), "rt_light_position_from_square");
        for (int q = 0; q < 3; ++q) lights[0].color[q] = 1.0;
        scene.n_spheres = 1;
        scene.spheres = spheres.data();
        scene.n_meshes = 2;
        scene.meshes = meshes.data();
        scene.n_lights = 1;
        scene.lights = lights.data();
        W = o.width > 0 ? o.width : 500;
        H = o.height > 0 ? o.height : 500;
        depth = o.depth >= 0 ? o.depth : 5;
        pitch = o.pitch > 0 ? o.pitch : 1.0;
    } else {
        Canonical c = canonical(o.config);
        check(rt_scene_init_reference(&scene), "rt_scene_init_reference");
        static const char* kSq[8] = {"d7", "b2", "f5", "h8", "c4", "e2", "g6", "a5"};
        int n = 0;
        if (c.nsph == 64) {
            for (int r = 0; r < 8; ++r)
                for (int cc = 0; cc < 8; ++cc) {
                    char s[3] = {(char)('a' + r), (char)('1' + cc), 0};
                    check(rt_convert_string_coordinate(s, spheres[n].center), "rt_convert_string_coordinate");
                    spheres[n].center[0] += 0.0;
                    spheres[n].center[1] += (double)(((r + cc) % 3) * 25);
                    spheres[n].center[2] += 0.0;
                    spheres[n].radius = 10.0;
                    ++n;
                }
        } else {
            for (; n < c.nsph; ++n) {
                check(rt_convert_string_coordinate(kSq[n], spheres[n].center), "rt_convert_string_coordinate");
                spheres[n].radius = 20.0;
            }
        }
        const char* lsq[2] = {"b6", "g3"};
        const double lcol[2] = {1.0, 0.5};
        for (int k = 0; k < c.nl; ++k) {
            check(rt_light_position_from_square(lsq[k], lights[k].position), "rt_light_position_from_square");
            for (int q = 0; q < 3; ++q) lights[k].color[q] = lcol[k];
        }
        scene.n_spheres = n;
        scene.spheres = spheres.data();
        scene.n_lights = c.nl;
        scene.lights = lights.data();
        W = o.width > 0 ? o.width : c.w;
        H = o.height > 0 ? o.height : c.h;
        depth = o.depth >= 0 ? o.depth : c.depth;
        pitch = o.pitch > 0 ? o.pitch : 500.0 / W;          // canonical framing
    }

    rt_camera cam;
    check(rt_camera_init_reference(&cam, W, H, pitch), "rt_camera_init_reference");
    rt_ctx* ctx = nullptr;
    check(rt_ctx_create(o.device, &ctx), "rt_ctx_create");
    std::vector<uint8_t> rgba8((size_t)W * H * 4);
    if (o.faithful >= 0) {
        uint64_t calls = 0;
        std::vector<uint8_t> ns((size_t)W * H);
        check(rt_render_screen(ctx, &scene, &cam, W, H, depth, o.faithful, o.seed, nullptr, rgba8.data(), ns.data(),
                               &calls), "rt_render_screen");
        check(rt_write_ppm(o.out.c_str(), rgba8.data(), W, H, 4), "rt_write_ppm");
        unsigned long long samples = 0;
        for (uint8_t v : ns) samples += v;
        std::printf("rt_render: %dx%d depth %d faithful rayTraceScreen (%s rand, seed %u) -> %s | %llu samples, "
                    "%llu rand() calls\n", W, H, depth, o.faithful == RT_RAND_MSVC ? "msvc" : "glibc", o.seed,
                    o.out.c_str(), samples, (unsigned long long)calls);
        rt_ctx_destroy(ctx);
        return 0;
    }
    if (o.gpus > 0) {
        rt_ctx_destroy(ctx);
        return render_multi(o, scene, cam, W, H, depth);
    }
    rt_stats st;
    const auto t0 = std::chrono::steady_clock::now();
    for (int k = 0; k < o.repeat; ++k)
        check(rt_render(ctx, &scene, &cam, W, H, depth, nullptr, nullptr, rgba8.data(), nullptr, &st), "rt_render");
    const double per_call_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() /
                               o.repeat;
    check(rt_write_ppm(o.out.c_str(), rgba8.data(), W, H, 4), "rt_write_ppm");
    const uint64_t rays = st.primary_rays + st.reflect_rays + st.shadow_rays;
    std::printf("rt_render: %dx%d depth %d -> %s | rays %llu (primary %llu, reflect %llu, shadow %llu) | kernel %.3f ms"
                " | %.1f Mray/s\n",
                W, H, depth, o.out.c_str(), (unsigned long long)rays, (unsigned long long)st.primary_rays,
                (unsigned long long)st.reflect_rays, (unsigned long long)st.shadow_rays, st.kernel_ms,
                rays / (st.kernel_ms * 1e3));
    if (o.repeat > 1) std::printf("rt_render: %d calls, %.3f ms per call (host to host)\n", o.repeat, per_call_ms);
    rt_ctx_destroy(ctx);
    return 0;
}
