// rt_screen.cpp — reference-faithful rayTraceScreen on the GPU: rt_render_screen.
//
// rayTraceScreen (/root/reference/Hw4/MySdlApplication.cpp:1251-1324) is a serial chain: the colour
// average is carried from pixel to pixel (:1283, never reset), a pixel takes samples until the
// convergence test passes (:1294-1311, at most 16), and every sample draws three rand() values
// (randomUnit, :1148-1169), so where pixel p's samples sit in the rand() stream depends on the sample
// counts of all earlier pixels.  The expensive part — one rayTraceRay per sample — is independent once
// that position is known.  So:
//   * the host predicts each pixel's sample count (from the resolved pixel below it, else the last resolved
//     pixel: counts are 2 in converged background and 16 on objects), which places every pixel of a chunk at
//     a predicted stream position; the GPU forms the jittered rays of a window of stream positions around
//     each prediction from the chunk's randomUnit() values and traces them (rt_trace_rays_dev, the
//     bit-exact rayTraceRay);
//   * the host then walks the chunk in order with the reference's own convergence arithmetic (FP64, same
//     operation order, -ffp-contract=off), reading each sample's colour at its actual stream position.  When
//     the actual position leaves a pixel's window the rest of the chunk is dropped and the next chunk starts
//     there.
// The result is the reference's frame bit for bit (tests: oracle_render_screen, and the reference's own
// rand() consumption, tests/golden/screen.json).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "rt_internal.hpp"

namespace {

struct V3 {
    double x, y, z;
};
inline V3 v3(double x, double y, double z) { return V3{x, y, z}; }
inline V3 v3(const double* p) { return V3{p[0], p[1], p[2]}; }
inline V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }     // :196-197
inline V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }     // :199-200
inline V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }       // :1118-1131
inline V3 cross(V3 a, V3 b) { return v3(a.y * b.z - b.y * a.z, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
inline double length(V3 a) { return std::sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }   // :174
inline V3 normalize(V3 a) {                                                           // :175
    double l = length(a);
    return v3(a.x / l, a.y / l, a.z / l);
}

// rand(): glibc's TYPE_3 additive feedback generator (RAND_MAX 2^31 - 1) or the MSVC CRT LCG (32767).
struct Rand {
    int kind;
    uint32_t lcg;
    int32_t r[34];
    int i = 0;
    Rand(int k, uint32_t seed) : kind(k), lcg(seed) {
        if (kind == RT_RAND_GLIBC) {                                  // srandom_r, TYPE_3
            std::vector<int32_t> t(344);
            t[0] = (int32_t)(seed ? seed : 1);
            for (int q = 1; q < 31; ++q) {
                int64_t v = (16807LL * t[q - 1]) % 2147483647LL;
                t[q] = (int32_t)(v < 0 ? v + 2147483647LL : v);
            }
            for (int q = 31; q < 34; ++q) t[q] = t[q - 31];
            for (int q = 34; q < 344; ++q) t[q] = (int32_t)((uint32_t)t[q - 31] + (uint32_t)t[q - 3]);
            for (int q = 0; q < 34; ++q) r[q] = t[310 + q];
        }
    }
    int next() {
        if (kind == RT_RAND_MSVC) {
            lcg = lcg * 214013u + 2531011u;
            return (int)((lcg >> 16) & 0x7fff);
        }
        int32_t v = (int32_t)((uint32_t)r[(i + 3) % 34] + (uint32_t)r[(i + 31) % 34]);
        r[i] = v;
        i = (i + 1) % 34;
        return (int)((uint32_t)v >> 1);
    }
    double max() const { return kind == RT_RAND_MSVC ? 32767.0 : 2147483647.0; }
};

// The stream of randomUnit() results (:1148-1169), generated on demand and kept from the first sample
// not yet consumed by a resolved pixel.
struct Jitter {
    Rand rng;
    uint64_t base = 0;                     // sample index of q.front()
    std::deque<V3> q;
    std::deque<uint32_t> calls;            // rand() calls of each sample
    uint64_t consumed_calls = 0;
    Jitter(int kind, uint32_t seed) : rng(kind, seed) {}
    const V3& at(uint64_t s) {
        while (base + q.size() <= s) {
            const double den = rng.max() + 1.0;
            V3 v = v3(0.0, 0.0, 0.0);
            uint32_t c = 0;
            while (v.x == 0 && v.y == 0 && v.z == 0) {                // vec.isZero() (:1160, :173)
                double z = (double)rng.next() / den - .5;            // Point(rand, rand, rand): the
                double y = (double)rng.next() / den - .5;            // arguments are evaluated right to
                double x = (double)rng.next() / den - .5;            // left (g++ and MSVC)
                c += 3;
                v = v3(x, y, z);
            }
            q.push_back(normalize(v));                               // vec.normalize() (:1166)
            calls.push_back(c);
        }
        return q[s - base];
    }
    void consume_until(uint64_t s) {       // samples [base, s) now belong to resolved pixels
        while (base < s) {
            at(base);
            consumed_calls += calls.front();
            q.pop_front();
            calls.pop_front();
            ++base;
        }
    }
};

inline unsigned char to_u8(double c) {
    double v = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c);
    return (unsigned char)(int)std::floor(v * 255.0 + 0.5);
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HostBuf {
    void* p = nullptr;
    ~HostBuf() {
        if (p) (void)hipHostFree(p);
    }
};
struct Stream {
    hipStream_t s = nullptr;
    ~Stream() {
        if (s) (void)hipStreamDestroy(s);
    }
};

}  // namespace

extern "C" int rt_render_screen(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, int W, int H, int depth,
                                int rand_kind, uint32_t seed, double* rgb64f, uint8_t* rgba8, uint8_t* samples,
                                uint64_t* rand_calls) {
    if (!ctx || !scene || !cam) return rt_fail(RT_EINVAL, "rt_render_screen: null argument");
    if (W <= 0 || H <= 0 || (long long)W * H > (1LL << 31)) return rt_fail(RT_EINVAL, "rt_render_screen: bad size");
    if (depth < 0 || depth > RT_MAX_DEPTH) return rt_fail(RT_EINVAL, "rt_render_screen: depth out of range");
    if (rand_kind != RT_RAND_GLIBC && rand_kind != RT_RAND_MSVC)
        return rt_fail(RT_EINVAL, "rt_render_screen: unknown rand_kind");
    int rc = rt_set_scene(ctx, scene);
    if (rc) return rc;

    const double kSamples = 16.0;                                    // SUPER_SAMPLE_NUMBER (:52)
    const double small = scene->small_number;                        // SMALL_NUMBER (:50)
    const V3 camera = v3(cam->eye), lookAt = v3(cam->look_at);
    const V3 lookDirection = lookAt - camera;                        // :1270
    const V3 right = normalize(cross(lookDirection, v3(cam->up)));   // :1271-1273
    const V3 rightOffset = (double)W * right;                        // :1274
    const V3 up = normalize(cross(right, lookDirection));            // :1276-1277
    V3 walk = (lookAt + (double)cam->bottom_x * right) + (double)cam->bottom_y * up;   // :1279

    // Speculation with windows (r03).  Each pixel's sample count is predicted from the pixel below it (its
    // row is resolved; object edges move little from row to row) or, in the first row, from the last resolved
    // pixel, which gives every pixel of a chunk a predicted first stream index.  The GPU traces, for every
    // pixel, the samples of a window of kWin stream indices either side of its predicted range, so the chunk
    // keeps resolving while the actual stream position drifts by up to kWin from the prediction (a count that
    // differs at an object edge no longer ends the chunk).  The jittered rays are formed on the device from the
    // chunk's randomUnit() values (rt_screen_form_ends): the host generates each stream value once and sends
    // 24 bytes per value instead of the rays.  Simulated on the reference's own sample counts (demo frame):
    // 759 round trips instead of 2,515, for ~85 traced samples per pixel instead of 7.
    const int kMaxRays = 1 << 19, kMaxPix = 4096, kWin = 28;
    const int kMaxJit = kMaxPix * 16 + 2 * kWin + 16;
    static_assert(16 + 2 * kWin <= kScreenMaxWindow, "window exceeds the ray-formation workgroup");
    DevBuf d_start, d_end;
    HostBuf h_rgb, h_pix, h_jit;
    void* d_rgb = nullptr;
    void* d_pix = nullptr;
    void* d_jit = nullptr;
    Stream st;
    const size_t ray_bytes = (size_t)kMaxRays * 3 * sizeof(double);
    const unsigned mapped = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e = hipStreamCreateWithFlags(&st.s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&d_start.p, ray_bytes);
    if (e == hipSuccess) e = hipMalloc(&d_end.p, ray_bytes);
    if (e == hipSuccess) e = hipHostMalloc(&h_rgb.p, ray_bytes, mapped);
    if (e == hipSuccess) e = hipHostMalloc(&h_pix.p, (size_t)kMaxPix * sizeof(ScreenPix), mapped);
    if (e == hipSuccess) e = hipHostMalloc(&h_jit.p, (size_t)kMaxJit * 3 * sizeof(double), mapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d_rgb, h_rgb.p, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d_pix, h_pix.p, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&d_jit, h_jit.p, 0);
    if (e != hipSuccess) return rt_fail(RT_ENOMEM, std::string("rt_render_screen: ") + hipGetErrorString(e));
    const double cam_p[3] = {camera.x, camera.y, camera.z};
    rc = rt_fill_points(static_cast<double*>(d_start.p), kMaxRays, cam_p, st.s);
    if (rc) return rc;
    const double* hr = static_cast<const double*>(h_rgb.p);
    ScreenPix* hp = static_cast<ScreenPix*>(h_pix.p);
    double* hj = static_cast<double*>(h_jit.p);

    Jitter jit(rand_kind, seed);
    V3 avgColor = v3(0.0, 0.0, 0.0);                                 // :1283, carried across pixels
    const long long P = (long long)W * H;
    long long p = 0;                                                 // first unresolved pixel (raster order)
    uint64_t S = 0;                                                  // its first sample in the stream
    int chunk = 64;
    std::vector<uint8_t> counts((size_t)P, 0);                       // resolved sample counts (predictions)
    std::vector<V3> sp(kMaxPix);
    // RT_SCREEN_PROFILE=1: host build / GPU round trip / resolve times and chunk counts on stderr.
    const bool prof = getenv("RT_SCREEN_PROFILE") != nullptr;
    using clk = std::chrono::steady_clock;
    double t_build = 0, t_gpu = 0, t_res = 0;
    long long n_chunks = 0, n_rays = 0;
    while (p < P) {
        const auto c0 = clk::now();
        // Chunk: pixels p .. p+m-1 with their predicted counts and sample windows.
        int m = (int)std::min<long long>(chunk, P - p);
        V3 w = walk;
        int total = 0, jmax = 0;
        long long spred = 0;                                         // predicted first sample, relative to S
        for (int q = 0; q < m; ++q) {
            const long long pix = p + q;
            const int pred = (pix - W >= 0 && pix - W < p) ? counts[pix - W] : (p > 0 ? counts[p - 1] : 16);
            const long long lo = std::max(0LL, spred - kWin), hi = spred + pred + kWin;
            const int len = (int)(hi - lo);
            if (total + len > kMaxRays || hi > kMaxJit) {
                m = q;
                break;
            }
            sp[q] = w;
            hp[q].sp[0] = w.x, hp[q].sp[1] = w.y, hp[q].sp[2] = w.z;
            hp[q].base = (int32_t)lo, hp[q].len = len, hp[q].off = total, hp[q].pad = 0;
            total += len;
            jmax = std::max(jmax, (int)hi);
            spred += pred;
            w = w + right;                                           // screenPt += right (:1315)
            if ((int)(pix % W) == W - 1) w = (w - rightOffset) + up; // :1320-1321
        }
        for (int k = 0; k < jmax; ++k) {                             // randomUnit() values S .. S + jmax - 1
            const V3& v = jit.at(S + (uint64_t)k);
            hj[3 * k] = v.x, hj[3 * k + 1] = v.y, hj[3 * k + 2] = v.z;
        }
        const auto c1 = clk::now();
        // One round trip: form the rays, trace them (colours straight into host memory), synchronise.
        rc = rt_screen_form_ends(static_cast<const ScreenPix*>(d_pix), m, static_cast<const double*>(d_jit),
                                 static_cast<double*>(d_end.p), st.s);
        if (rc) return rc;
        rc = rt_trace_rays_dev(ctx, static_cast<const double*>(d_start.p), static_cast<const double*>(d_end.p), total,
                               depth, static_cast<double*>(d_rgb), nullptr, st.s);
        if (rc) return rc;
        // While the GPU traces: generate the stream values the next chunk will need (rand() + normalize are
        // the host's largest share of a round trip), so its build only copies them.
        (void)jit.at(S + 2 * (uint64_t)jmax + 64);
        e = hipStreamSynchronize(st.s);
        if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render_screen: ") + hipGetErrorString(e));

        const auto c2 = clk::now();
        // Resolve in order with the reference's loop (:1294-1311), each sample read from its pixel's window.
        int q = 0;
        long long A = 0;                                             // actual first sample of pixel q, relative to S
        bool broke = false;
        for (; q < m; ++q) {
            const ScreenPix& X = hp[q];
            if (A < X.base) {                                        // the stream ran behind the window
                broke = true;
                break;
            }
            const V3 a0 = avgColor;
            double k;
            int n = 0;
            bool need_more = false;
            for (k = 0.0; k < kSamples; k++) {
                const long long idx = A + n - X.base;
                if (idx >= X.len) { need_more = true; break; }       // ... or ran past it
                const double* c = hr + 3 * (X.off + idx);
                ++n;
                const V3 color = v3(c[0], c[1], c[2]);
                const V3 oldWeightedColor = (k + 1.0) * avgColor;
                avgColor = avgColor + color;                         // avgColor += color
                const V3 weightedColor = k * avgColor;
                if (length(weightedColor - oldWeightedColor) < small * k * (k + 1)) break;
            }
            if (need_more) {
                avgColor = a0;
                broke = true;
                break;
            }
            avgColor = v3(avgColor.x / k, avgColor.y / k, avgColor.z / k);   // avgColor /= k (:1310)
            const long long pix = p + q;
            if (rgb64f) {
                rgb64f[3 * pix] = avgColor.x, rgb64f[3 * pix + 1] = avgColor.y, rgb64f[3 * pix + 2] = avgColor.z;
            }
            if (rgba8) {
                rgba8[4 * pix] = to_u8(avgColor.x), rgba8[4 * pix + 1] = to_u8(avgColor.y);
                rgba8[4 * pix + 2] = to_u8(avgColor.z), rgba8[4 * pix + 3] = 255;
            }
            if (samples) samples[pix] = (uint8_t)n;
            counts[pix] = (uint8_t)n;
            A += n;
            walk = sp[q] + right;
            if ((int)(pix % W) == W - 1) walk = (walk - rightOffset) + up;
        }
        // (q >= 1: pixel p's window starts at its own first sample and holds >= 16 + kWin samples)
        p += q;
        S += (uint64_t)A;
        jit.consume_until(S);
        chunk = broke ? std::max(16, chunk / 2) : std::min(kMaxPix, chunk * 2);
        if (prof) {
            const auto c3 = clk::now();
            t_build += std::chrono::duration<double>(c1 - c0).count();
            t_gpu += std::chrono::duration<double>(c2 - c1).count();
            t_res += std::chrono::duration<double>(c3 - c2).count();
            ++n_chunks;
            n_rays += total;
        }
    }
    if (prof)
        fprintf(stderr, "rt_render_screen: %lld chunks, %lld rays traced; build %.1f ms, gpu %.1f ms, resolve %.1f ms\n",
                n_chunks, n_rays, t_build * 1e3, t_gpu * 1e3, t_res * 1e3);
    if (rand_calls) *rand_calls = jit.consumed_calls;
    return RT_OK;
}
