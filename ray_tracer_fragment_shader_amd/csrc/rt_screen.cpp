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
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
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

// rand(): glibc's TYPE_3 additive feedback generator (RAND_MAX 2^31 - 1) or the MSVC CRT LCG (32767), produced
// in blocks: the glibc state is the last 34 outputs of r[n] = r[n - 31] + r[n - 3] (mod 2^32), result r[n] >> 1.
struct Rand {
    static constexpr int kHist = 34, kBlock = 4096;
    int kind;
    uint32_t lcg;
    uint32_t h[kHist + kBlock];                                      // history, then the block's raw values
    int32_t out[kBlock];
    int pos = kBlock;                                                // next unread entry of out
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
            for (int q = 0; q < kHist; ++q) h[q] = (uint32_t)t[310 + q];
        }
    }
    void refill() {
        if (kind == RT_RAND_MSVC) {
            for (int k = 0; k < kBlock; ++k) {
                lcg = lcg * 214013u + 2531011u;
                out[k] = (int32_t)((lcg >> 16) & 0x7fff);
            }
        } else {
            for (int k = kHist; k < kHist + kBlock; ++k) h[k] = h[k - 31] + h[k - 3];
            for (int k = 0; k < kBlock; ++k) out[k] = (int32_t)(h[kHist + k] >> 1);
            std::memcpy(h, h + kBlock, sizeof(uint32_t) * kHist);
        }
        pos = 0;
    }
    int next() {
        if (pos == kBlock) refill();
        return out[pos++];
    }
    double max() const { return kind == RT_RAND_MSVC ? 32767.0 : 2147483647.0; }
};

// The stream of randomUnit() results (:1148-1169), generated ahead in batches into one flat array and kept
// from the first sample not yet consumed by a resolved pixel.
struct Jitter {
    Rand rng;
    uint64_t base = 0;                     // sample index of xyz[0]
    std::vector<double> xyz;               // 3 per sample
    std::vector<uint32_t> calls;           // rand() calls of each sample
    size_t n = 0;                          // samples generated from base on (the arrays hold more room)
    uint64_t cons = 0;                     // first sample not yet consumed
    uint64_t consumed_calls = 0;
    Jitter(int kind, uint32_t seed) : rng(kind, seed) {}
    // samples up to index s (exclusive) generated
    void ensure(uint64_t s) {
        if (base + n >= s) return;
        const size_t want = (size_t)(s - base) + 2048;               // a batch ahead
        if (calls.size() < want) {
            xyz.resize(3 * (want + want / 2));
            calls.resize(want + want / 2);
        }
        // rand() / (RAND_MAX + 1.0) divides by a power of two: the product with its reciprocal is the same double.
        const double inv = 1.0 / (rng.max() + 1.0);
        const int32_t half = (int32_t)((rng.max() + 1.0) / 2);       // the draw that makes a coordinate exactly 0
        constexpr int kB = 512;
        int32_t X[kB], Y[kB], Z[kB];
        while (n < want) {
            const int cnt = (int)std::min<size_t>(kB, want - n);
            for (int k = 0; k < cnt; ++k) {                          // the draws (integer work, in order)
                uint32_t c = 0;
                int32_t z, y, x;
                do {                                                 // vec.isZero() (:1160, :173): draw again
                    z = rng.next();                                  // Point(rand, rand, rand): the arguments
                    y = rng.next();                                  // are evaluated right to left (g++, MSVC)
                    x = rng.next();
                    c += 3;
                } while (x == half && y == half && z == half);
                X[k] = x, Y[k] = y, Z[k] = z;
                calls[n + k] = c;
            }
            double* o = &xyz[3 * n];
            for (int k = 0; k < cnt; ++k) {                          // randomUnit(): (r / den - .5), normalize()
                const double x = (double)X[k] * inv - .5, y = (double)Y[k] * inv - .5, z = (double)Z[k] * inv - .5;
                const double l = std::sqrt(x * x + y * y + z * z);   // length() (:174)
                o[3 * k] = x / l, o[3 * k + 1] = y / l, o[3 * k + 2] = z / l;   // (:175)
            }
            n += cnt;
        }
    }
    const double* at(uint64_t s) {         // the sample's x, y, z (valid until the next ensure / consume)
        ensure(s + 1);
        return &xyz[3 * (size_t)(s - base)];
    }
    void consume_until(uint64_t s) {       // samples [cons, s) now belong to resolved pixels
        ensure(s);
        for (uint64_t q = cons; q < s; ++q) consumed_calls += calls[(size_t)(q - base)];
        cons = std::max(cons, s);
        const size_t k = (size_t)(cons - base);
        if (k > 4096 && k > n / 2) {       // drop the consumed front (amortised)
            std::memmove(xyz.data(), xyz.data() + 3 * k, sizeof(double) * 3 * (n - k));
            std::memmove(calls.data(), calls.data() + k, sizeof(uint32_t) * (n - k));
            base += k;
            n -= k;
        }
    }
};

// length(d) < t (:1307) without the square root where the squares decide: s = |d|^2 is computed exactly as
// length() computes it, and sqrt is correctly rounded and monotonic, so s < t^2 (1 - 2^-40) (t^2 itself within 2^-53)
// puts sqrt(s) below t (1 - 2^-42), which rounds below t, and s > t^2 (1 + 2^-40) puts it above; only between the
// two (and for t <= 0, inf or NaN operands, where both comparisons fail) is the square root taken.
// tt must be a normal double for its 2^-53 relative error (t^2 in the subnormal range has a far larger one, and the
// 2^-40 margins would no longer hold): below DBL_MIN the square root decides.
inline bool converged(V3 d, double t) {
    const double s = d.x * d.x + d.y * d.y + d.z * d.z;
    if (t > 0.0 && t * t >= 0x1p-1022) {
        const double tt = t * t;
        if (s < tt * (1.0 - 0x1p-40)) return true;
        if (s > tt * (1.0 + 0x1p-40)) return false;
    }
    return std::sqrt(s) < t;
}

inline unsigned char to_u8(double c) {
    double v = c < 0.0 ? 0.0 : (c > 1.0 ? 1.0 : c);
    return (unsigned char)(int)std::floor(v * 255.0 + 0.5);
}

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

struct ScreenBuf {                                                    // one chunk's stream and mapped buffers
    Stream st;
    std::vector<double> sp;                                          // host: screen point of each pixel (x, y, z)
    HostBuf h_rgb, h_pix, h_jit;
    void* d_rgb = nullptr;
    void* d_pix = nullptr;
    void* d_jit = nullptr;
    hipEvent_t done = nullptr;                                       // recorded after the chunk's trace
    ~ScreenBuf() {
        if (done) (void)hipEventDestroy(done);
    }
};
struct ScreenWs {                                                    // chunks in flight + the rays' start
    uint32_t seq = 0;                                                // the last chunk's sequence number
    static constexpr int kAheadMax = 2;                              // continuations queued behind a chunk
    static constexpr int kSets = 2 * kAheadMax + 1;                  // in flight + draining
    HostBuf h_cam;
    void* d_cam = nullptr;
    ScreenBuf buf[kSets];
};
// A chunk's pixel table, then its first-pixel table (one entry per kScreenBlock rays).
constexpr size_t kPixBytes = (size_t)kScreenMaxPix * sizeof(ScreenPix);
constexpr size_t kDoneOffset = kPixBytes + (size_t)kScreenMaxBlocks * sizeof(int32_t);   // per-workgroup done words
constexpr size_t kPixTableBytes = kDoneOffset + (size_t)kScreenMaxBlocks * sizeof(uint32_t);

// A buffer set's stream, event and mapped buffers, allocated on the set's first use (the default pipeline uses
// three of the kSets).
hipError_t alloc_set(ScreenBuf& b) {
    const size_t ray_bytes = (size_t)kScreenMaxRays * 3 * sizeof(double);
    const unsigned mapped = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e = hipSuccess;                                       // (a set left half-built by a failure resumes)
    if (!b.st.s) e = hipStreamCreateWithFlags(&b.st.s, hipStreamNonBlocking);
    b.sp.resize(3 * (size_t)kScreenMaxPix);
    if (e == hipSuccess && !b.h_rgb.p) e = hipHostMalloc(&b.h_rgb.p, ray_bytes, mapped);
    if (e == hipSuccess && !b.h_pix.p) {
        e = hipHostMalloc(&b.h_pix.p, kPixTableBytes, mapped);
        if (e == hipSuccess) std::memset(static_cast<char*>(b.h_pix.p) + kDoneOffset, 0, kScreenMaxBlocks * sizeof(uint32_t));
    }
    if (e == hipSuccess && !b.h_jit.p) e = hipHostMalloc(&b.h_jit.p, (size_t)kScreenMaxJit * 3 * sizeof(double), mapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&b.d_rgb, b.h_rgb.p, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&b.d_pix, b.h_pix.p, 0);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&b.d_jit, b.h_jit.p, 0);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&b.done, hipEventDisableTiming);
    return e;
}

std::unique_ptr<ScreenWs> alloc_ws() {
    std::unique_ptr<ScreenWs> w(new ScreenWs());
    const unsigned mapped = hipHostMallocMapped | hipHostMallocCoherent;
    hipError_t e = hipHostMalloc(&w->h_cam.p, 3 * sizeof(double), mapped);
    if (e == hipSuccess) e = hipHostGetDevicePointer(&w->d_cam, w->h_cam.p, 0);
    if (e != hipSuccess) return nullptr;
    return w;
}

std::mutex g_ws_mu;
// Idle workspaces by context.  Allocated once and never destroyed: a context still alive at process exit leaks its
// workspace instead of calling hipEventDestroy / hipHostFree / hipStreamDestroy from static destruction, after the
// HIP runtime may have begun tearing down.
auto& g_ws = *new std::unordered_map<const rt_ctx*, std::unique_ptr<ScreenWs>>();

std::unique_ptr<ScreenWs> take_ws(const rt_ctx* ctx) {
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        auto it = g_ws.find(ctx);
        if (it != g_ws.end() && it->second) {
            std::unique_ptr<ScreenWs> w = std::move(it->second);
            g_ws.erase(it);
            return w;
        }
    }
    return alloc_ws();
}

void give_ws(const rt_ctx* ctx, std::unique_ptr<ScreenWs> w) {
    std::lock_guard<std::mutex> lk(g_ws_mu);
    auto& slot = g_ws[ctx];
    if (!slot) slot = std::move(w);                                  // else: freed here (a concurrent call's)
}

}  // namespace

void rt_screen_release(const rt_ctx* ctx) {
    std::unique_ptr<ScreenWs> w;
    {
        std::lock_guard<std::mutex> lk(g_ws_mu);
        auto it = g_ws.find(ctx);
        if (it == g_ws.end()) return;
        w = std::move(it->second);
        g_ws.erase(it);
    }
}

extern "C" int rt_render_screen(rt_ctx* ctx, const rt_scene* scene, const rt_camera* cam, int W, int H, int depth,
                                int rand_kind, uint32_t seed, double* rgb64f, uint8_t* rgba8, uint8_t* samples,
                                uint64_t* rand_calls) {
    if (!ctx || !scene || !cam) return rt_fail(RT_EINVAL, "rt_render_screen: null argument");
    if (W <= 0 || H <= 0 || (long long)W * H > (1LL << 31)) return rt_fail(RT_EINVAL, "rt_render_screen: bad size");
    if (depth < 0 || depth > RT_MAX_DEPTH) return rt_fail(RT_EINVAL, "rt_render_screen: depth out of range");
    if (rand_kind != RT_RAND_GLIBC && rand_kind != RT_RAND_MSVC)
        return rt_fail(RT_EINVAL, "rt_render_screen: unknown rand_kind");
    // Everything below (the cached workspace's streams, events and mapped buffers, the trace launches) belongs to the
    // context's device, whatever device the caller has current (rt_set_scene returns early for an unchanged scene
    // without selecting it); the caller's device is restored on return.
    struct DeviceGuard {
        int prev = -1;
        explicit DeviceGuard(int dev) {
            if (hipGetDevice(&prev) != hipSuccess) prev = -1;
            (void)hipSetDevice(dev);
        }
        ~DeviceGuard() {
            if (prev >= 0) (void)hipSetDevice(prev);
        }
    } device_guard(rt_ctx_device(ctx));
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
    // chunk's randomUnit() values by the trace launch itself (rt_trace_screen_dev): the host generates each stream
    // value once and sends 24 bytes per value instead of the rays, and a chunk is one launch.  Simulated on the
    // reference's own sample counts (demo frame): 759 round trips instead of 2,515, for ~85 traced samples per pixel
    // instead of 7 (tools/screen_sim.py replays the schedule).
    //
    // Two chunks in flight (r04).  While the GPU traces chunk c, the host builds and queues chunk c + 1 as the
    // continuation of c's prediction chain (the pixels below it that lie in c use c's predicted counts; its
    // stream base is c's predicted end minus kWin), then waits for c and resolves it.  When c resolves to its
    // end, c + 1 is already traced or tracing: the host's build and resolution overlap the GPU's round trip
    // instead of following it.  When c breaks, c + 1 is dropped and a chunk starts at the break, as before.
    // Chunks go to three buffer sets, each with its own stream: a dropped continuation finishes on its stream
    // beside the restarted chain instead of ahead of it, and its set is reused once it is done.  Resolution is
    // unchanged: every pixel reads its samples at its actual stream position, or breaks.
    const int kMaxRays = kScreenMaxRays, kMaxPix = kScreenMaxPix;
    const int kMaxJit = kScreenMaxJit;
    constexpr int kWinMax = (kScreenMaxWindow - 16) / 2;
    static_assert(kScreenMaxJit >= kScreenMaxPix * 16 + 2 * kWinMax + 16, "stream-value buffer too small");
    // RT_SCREEN_WIN (A/B): the window half-width kWin (stream positions either side of a pixel's predicted range).
    // 56 (the most a pixel table entry holds): fewer restarts for twice the traced colours; in-process A/B against
    // r03's 28, demo -9.6%, c2 scene -14% (20: +33%; 36/44: -1 to -13%; 72/96/120 with larger tables: +2 to +34%).
    int kWin = kWinMax;
    if (const char* ev = getenv("RT_SCREEN_WIN")) kWin = std::min(std::max(atoi(ev), 16), kWinMax);
    // The buffers live in the context between calls (allocating ~40 MB of device and mapped host memory
    // per frame cost more than a quarter of a demo frame); a call running concurrently on the same context
    // allocates its own.
    std::unique_ptr<ScreenWs> ws = take_ws(ctx);
    if (!ws) return rt_fail(RT_ENOMEM, "rt_render_screen: workspace allocation failed");
    struct Give {                                                    // on every return: the streams' work is
        rt_ctx* ctx;                                                 // done, then the workspace goes back
        std::unique_ptr<ScreenWs>& ws;
        ~Give() {
            for (ScreenBuf& b : ws->buf)
                if (b.st.s) (void)hipStreamSynchronize(b.st.s);
            give_ws(ctx, std::move(ws));
        }
    } give{ctx, ws};
    ScreenBuf* buf = ws->buf;
    double* hc = static_cast<double*>(ws->h_cam.p);                  // the rays' start: the camera
    hc[0] = camera.x, hc[1] = camera.y, hc[2] = camera.z;

    Jitter jit(rand_kind, seed);
    V3 avgColor = v3(0.0, 0.0, 0.0);                                 // :1283, carried across pixels
    const long long P = (long long)W * H;
    long long p = 0;                                                 // first unresolved pixel (raster order)
    uint64_t S = 0;                                                  // its first sample in the stream
    int chunk = 64;
    std::vector<uint8_t> counts((size_t)P, 0);                       // resolved sample counts (predictions)
    std::vector<uint8_t> pcount((size_t)P, 0);                       // predicted counts of queued pixels
    // RT_SCREEN_PROFILE=1: host build / GPU wait / resolve times and chunk counts on stderr.
    const bool prof = getenv("RT_SCREEN_PROFILE") != nullptr;
    // RT_SCREEN_NEXT (A/B): size of the queued continuation as a multiple of the current chunk size (0: none, one
    // chunk in flight as in r03).
    int next_mul = 1;
    if (const char* ev = getenv("RT_SCREEN_NEXT")) next_mul = std::max(0, atoi(ev));
    // RT_SCREEN_AHEAD (A/B): continuations kept queued behind the chunk being resolved (1: r04's two chunks in flight).
    int ahead = 1;
    if (const char* ev = getenv("RT_SCREEN_AHEAD")) ahead = atoi(ev);
    ahead = next_mul > 0 ? std::min(std::max(ahead, 1), ScreenWs::kAheadMax) : 0;
    // RT_SCREEN_NEXT_MIN: continuations only once the chunk size has grown to at least this many pixels (a run of
    // clean chunks); after a break the chain waits for each chunk before queueing the next.  Two thirds of the
    // continuations queued behind every chunk were dropped (583 of 886 on the demo frame), and their building and
    // tracing cost more than they saved: in-process A/B (tools/screen_ab.py), against none at all, demo -9%,
    // c2 scene -6% with continuations from the maximum chunk size (4,096 pixels) on; from 0 pixels +1–3%.
    // RT_SCREEN_MAX_CHUNK (A/B): the largest chunk (pixels); a chunk is waited for whole before it is resolved.
    // (Smaller caps, with continuations from the cap on, measured slower: 2,048 ±1%, 1,024 +2–3%, 512 +5–12%.)
    int max_chunk = kMaxPix;
    if (const char* ev = getenv("RT_SCREEN_MAX_CHUNK")) max_chunk = std::min(std::max(16, atoi(ev)), kMaxPix);
    int next_min = max_chunk;
    if (const char* ev = getenv("RT_SCREEN_NEXT_MIN")) next_min = std::max(0, atoi(ev));
    // RT_SCREEN_PROGRESSIVE=1 (A/B): resolve a chunk while it is traced, each pixel once the workgroups holding its
    // rays have published per-workgroup done words (a system-scope release after their colour stores).  Bit-exact,
    // but demo +4.7%, c2 scene -0.4% against waiting for the whole chunk (in-process A/B): the releases cost what the
    // overlap saves.  Off.
    bool progressive = false;
    // RT_SCREEN_PREFETCH: resolve prefetches the colours of the pixel this many ahead at its predicted position (the
    // GPU wrote them over PCIe: every pixel's first read would miss the host's caches).  0: off.
    // RT_SCREEN_SHRINK (A/B): the chunk size is divided by this after a break (and doubles after a clean chunk); 2
    // measured fastest (1: x4-5, every break re-traces a maximum chunk; 4: +3-4%; 8: +5-9%).
    int shrink = 2;
    if (const char* ev = getenv("RT_SCREEN_SHRINK")) shrink = std::max(1, atoi(ev));
    int prefetch = 8;
    if (const char* ev = getenv("RT_SCREEN_PREFETCH")) prefetch = std::max(0, atoi(ev));
    if (const char* ev = getenv("RT_SCREEN_PROGRESSIVE")) progressive = atoi(ev) != 0;
    using clk = std::chrono::steady_clock;
    double t_build = 0, t_gen = 0, t_gpu = 0, t_res = 0;
    const auto t_start = clk::now();
    long long n_chunks = 0, n_rays = 0, n_dropped = 0;

    // A queued chunk: pixels p0 .. p0+m-1, windows relative to stream index S0.
    struct Chunk {
        int b = 0;                                                   // buffer set
        long long p0 = 0;
        int m = 0;
        uint64_t S0 = 0;
        long long spred_end = 0;                                     // predicted start of pixel p0+m, rel. to S0
        uint64_t jend = 0;                                           // its stream values: S0 .. jend - 1
        V3 walk_end = v3(0.0, 0.0, 0.0);                             // screen point of pixel p0+m
        uint32_t seq = 0;                                            // its workgroups' done value
    };
    // Build chunk (pixels p0.., at most `want`) into buffer set b and queue its round trip.  pred_start: the
    // predicted first sample of pixel p0 (absolute); the chunk's base is pred_start - kWin, at least `floor`.
    auto queue = [&](Chunk& c, int b, long long p0, uint64_t pred_start, uint64_t floor, V3 w0, int want) -> int {
        const auto c0 = clk::now();
        ScreenBuf& B = buf[b];
        ScreenPix* hp = static_cast<ScreenPix*>(B.h_pix.p);
        int32_t* hf = reinterpret_cast<int32_t*>(static_cast<char*>(B.h_pix.p) + kPixBytes);
        double* hj = static_cast<double*>(B.h_jit.p);
        c.b = b;
        c.p0 = p0;
        c.S0 = std::max<uint64_t>(floor, pred_start > (uint64_t)kWin ? pred_start - kWin : 0);
        double* sp = B.sp.data();
        int m = (int)std::min<long long>(want, P - p0);
        V3 w = w0;
        int total = 0, jmax = 0, nb = 0;
        long long spred = (long long)pred_start - (long long)c.S0;  // predicted first sample, relative to S0
        for (int q = 0; q < m; ++q) {
            const long long pix = p0 + q;
            const long long below = pix - W;
            const int pred = below >= 0 ? (below < p ? counts[below] : pcount[below]) : (p > 0 ? counts[p - 1] : 16);
            const long long lo = std::max(0LL, spred - kWin), hi = std::max(lo, spred + pred + kWin);
            const int len = (int)(hi - lo);
            if (total + len > kMaxRays || hi > kMaxJit) {
                m = q;
                break;
            }
            pcount[pix] = (uint8_t)pred;
            sp[3 * q] = w.x, sp[3 * q + 1] = w.y, sp[3 * q + 2] = w.z;
            hp[q].sp[0] = w.x, hp[q].sp[1] = w.y, hp[q].sp[2] = w.z;
            hp[q].base = (int32_t)lo, hp[q].len = len, hp[q].off = total, hp[q].pad = 0;
            for (; nb * kScreenBlock < total + len; ++nb) hf[nb] = q;  // workgroups whose first ray is q's
            total += len;
            jmax = std::max(jmax, (int)hi);
            spred += pred;
            w = w + right;                                           // screenPt += right (:1315)
            if ((int)(pix % W) == W - 1) w = (w - rightOffset) + up; // :1320-1321
        }
        c.m = m;
        c.spred_end = spred;
        c.jend = c.S0 + (uint64_t)jmax;
        c.walk_end = w;
        if (jmax > 0)                                                // randomUnit() values S0 .. S0 + jmax - 1
            std::memcpy(hj, jit.at(c.S0 + (uint64_t)(jmax - 1)) - 3 * (size_t)(jmax - 1), sizeof(double) * 3 * jmax);
        // One round trip: one launch forms the rays and traces them (colours straight into host memory).
        c.seq = ++ws->seq ? ws->seq : ++ws->seq;                     // (never 0: the words start at 0)
        const int r = rt_trace_screen_dev(ctx, static_cast<const double*>(ws->d_cam),
                                          static_cast<const ScreenPix*>(B.d_pix),
                                          reinterpret_cast<const int32_t*>(static_cast<const char*>(B.d_pix) + kPixBytes),
                                          m, static_cast<const double*>(B.d_jit), total, depth,
                                          static_cast<double*>(B.d_rgb),
                                          progressive ? reinterpret_cast<uint32_t*>(static_cast<char*>(B.d_pix) + kDoneOffset)
                                                      : nullptr,
                                          c.seq,
                                          B.st.s);
        if (r) return r;
        const hipError_t er = hipEventRecord(B.done, B.st.s);
        if (er != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render_screen: ") + hipGetErrorString(er));
        if (prof) {
            t_build += std::chrono::duration<double>(clk::now() - c0).count();
            ++n_chunks;
            n_rays += total;
        }
        return RT_OK;
    };

    // A buffer set no queued chunk uses, preferably one whose last chunk is done (dropped continuations drain on
    // their own streams while the chain goes on in the other sets).
    bool in_use[ScreenWs::kSets] = {};
    auto pick = [&](int* out) -> int {
        int idle = -1, fresh = -1;
        for (int b = 0; b < ScreenWs::kSets; ++b) {
            if (in_use[b]) continue;
            if (!buf[b].done) {                                  // never used
                if (fresh < 0) fresh = b;
                continue;
            }
            const hipError_t q = hipEventQuery(buf[b].done);
            if (q == hipSuccess) {
                *out = b;
                return RT_OK;
            }
            if (q != hipErrorNotReady) return rt_fail(RT_EHIP, std::string("rt_render_screen: ") + hipGetErrorString(q));
            if (idle < 0) idle = b;
        }
        if (fresh >= 0) {
            const hipError_t q = alloc_set(buf[fresh]);
            if (q != hipSuccess) return rt_fail(RT_ENOMEM, std::string("rt_render_screen: ") + hipGetErrorString(q));
            *out = fresh;
            return RT_OK;
        }
        const hipError_t q = hipEventSynchronize(buf[idle].done);   // (kSets > 1 + kAheadMax: one exists)
        if (q != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render_screen: ") + hipGetErrorString(q));
        *out = idle;
        return RT_OK;
    };    auto queue_in_free = [&](std::deque<Chunk>& fl, long long p0, uint64_t pred_start, uint64_t floor, V3 w0,
                             int want) -> int {
        int b = 0;
        int r = pick(&b);
        if (!r) {
            fl.emplace_back();
            r = queue(fl.back(), b, p0, pred_start, floor, w0, want);
            if (!r) in_use[b] = true;
        }
        return r;
    };

    std::deque<Chunk> fl;                                            // chunks in flight, oldest first
    if ((rc = queue_in_free(fl, 0, 0, 0, walk, chunk))) return rc;
    while (p < P) {
        // continuations of the prediction chain, queued behind the chunk about to be resolved
        while ((int)fl.size() < 1 + ahead && chunk >= next_min && fl.back().p0 + fl.back().m < P) {
            const Chunk t = fl.back();
            if ((rc = queue_in_free(fl, t.p0 + t.m, t.S0 + (uint64_t)t.spred_end, S, t.walk_end,
                                    std::min(chunk * next_mul, max_chunk))))
                return rc;
        }
        // While the GPU traces: generate the stream values the following chunk will need (rand() + normalize
        // are the host's largest share of a round trip), so its build only copies them.
        const auto cg = clk::now();
        jit.ensure(fl.back().jend + (fl.back().jend - fl.back().S0) + 64);
        const auto c1 = clk::now();
        const Chunk cur = fl.front();
        // Resolve while the chunk is still being traced: a pixel's colours are read once the workgroups holding its
        // rays have published their done words (release at system scope after their colour stores).
        const volatile uint32_t* dw =
            reinterpret_cast<const volatile uint32_t*>(static_cast<const char*>(buf[cur.b].h_pix.p) + kDoneOffset);
        int ready = -1;                                              // workgroups 0 .. ready are done
        if (!progressive) {
            const hipError_t q = hipEventSynchronize(buf[cur.b].done);
            if (q != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render_screen: ") + hipGetErrorString(q));
            ready = kScreenMaxBlocks;
        }
        double t_spin = 0.0;
        auto wait_rays = [&](int last_ray) -> int {
            const int w = last_ray / kScreenBlock;
            if (ready >= w) return RT_OK;
            const auto s0 = clk::now();
            for (unsigned spins = 1; ready < w; ++spins) {
                if (dw[ready + 1] == cur.seq) {
                    ++ready;
                    continue;
                }
                if (spins % 4096 == 0) {                             // the launch failed or ended without the word
                    const hipError_t q = hipEventQuery(buf[cur.b].done);
                    if (q == hipSuccess && dw[ready + 1] != cur.seq)
                        return rt_fail(RT_EHIP, "rt_render_screen: a workgroup finished without its done word");
                    if (q != hipSuccess && q != hipErrorNotReady)
                        return rt_fail(RT_EHIP, std::string("rt_render_screen: ") + hipGetErrorString(q));
                }
            }
            std::atomic_thread_fence(std::memory_order_acquire);
            t_spin += std::chrono::duration<double>(clk::now() - s0).count();
            return RT_OK;
        };
        const auto c2 = clk::now();

        // Resolve cur in order with the reference's loop (:1294-1311), each sample read from its pixel's window.
        const double* hr = static_cast<const double*>(buf[cur.b].h_rgb.p);
        const ScreenPix* hp = static_cast<const ScreenPix*>(buf[cur.b].h_pix.p);
        int q = 0;
        long long A = (long long)S - (long long)cur.S0;               // actual first sample of pixel q, rel. to S0
        bool broke = A < 0;
        for (; q < cur.m && !broke; ++q) {
            const ScreenPix& X = hp[q];
            if ((rc = wait_rays(X.off + X.len - 1))) return rc;
            if (prefetch && q + prefetch < cur.m) {                   // the predicted samples of pixel q + prefetch
                const ScreenPix& Y = hp[q + prefetch];
                const double* y = hr + 3 * (size_t)(Y.off + std::min(Y.len - 1, kWin));
                __builtin_prefetch(y);
                __builtin_prefetch(y + 8);
            }
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
                if (converged(weightedColor - oldWeightedColor, small * k * (k + 1))) break;
            }
            if (need_more) {
                avgColor = a0;
                broke = true;
                break;
            }
            avgColor = v3(avgColor.x / k, avgColor.y / k, avgColor.z / k);   // avgColor /= k (:1310)
            const long long pix = cur.p0 + q;
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
            walk = v3(&buf[cur.b].sp[3 * q]) + right;
            if ((int)(pix % W) == W - 1) walk = (walk - rightOffset) + up;
        }
        p = cur.p0 + q;
        if (q > 0) S = cur.S0 + (uint64_t)A;                         // (q == 0: nothing resolved, S unchanged)
        jit.consume_until(S);
        if (prof) {
            t_gen += std::chrono::duration<double>(c1 - cg).count();
            t_gpu += std::chrono::duration<double>(c2 - c1).count() + t_spin;     // waiting for done words
            t_res += std::chrono::duration<double>(clk::now() - c2).count() - t_spin;
        }
        in_use[cur.b] = false;
        fl.pop_front();
        if (!broke && q == cur.m) {
            chunk = std::min(max_chunk, chunk * 2);
            if (fl.empty() && p < P && (rc = queue_in_free(fl, p, S, S, walk, chunk))) return rc;
            continue;
        }
        // cur broke at pixel p: the queued continuations are dropped (each finishes on its own stream, beside the
        // restarted chain, not ahead of it) and the chain restarts there
        chunk = std::max(16, chunk / shrink);
        n_dropped += (long long)fl.size();
        for (const Chunk& d : fl) in_use[d.b] = false;
        fl.clear();
        if (p < P && (rc = queue_in_free(fl, p, S, S, walk, chunk))) return rc;
    }
    if (prof)
        fprintf(stderr, "rt_render_screen: %lld chunks (%lld dropped), %lld rays traced; build %.1f ms, %llu stream values "
                "%.1f ms, gpu wait %.1f ms, resolve %.1f ms; loop %.1f ms\n", n_chunks, n_dropped, n_rays, t_build * 1e3,
                (unsigned long long)(jit.base + jit.n), t_gen * 1e3, t_gpu * 1e3, t_res * 1e3, std::chrono::duration<double>(clk::now() - t_start).count() * 1e3);
    if (rand_calls) *rand_calls = jit.consumed_calls;
    return RT_OK;
}
