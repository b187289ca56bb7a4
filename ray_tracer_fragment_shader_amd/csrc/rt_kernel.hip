// rt_kernel.hip — MI355X (gfx950) kernels and the device half of the C ABI (include/rt_api.h).
//
// Kernels
//   rt_render_kernel<B, LDS, MINW, TRANSP, CULL, WG>  one work-item per pixel, FP64, iterative bounce loop
//                             (rt_device.hpp); CULL: wave-level sphere culling for >= kConeMin spheres.
//                             Default: one-wave workgroups (WG = 64), each owning an 8 x 8 pixel tile
//                             (square tiles keep a wave's rays coherent, so the __any early-out and the
//                             culling masks work for whole waves).  The scene (bounding sphere, board,
//                             materials, lights, spheres) is read through the scalar cache; the A/B
//                             variants with 256-thread workgroups (32 x 8 tiles) copy it into LDS once per
//                             workgroup (LDS = 1) or stage the output tile in LDS for 32-pixel row stores.
//                             Per-level colours wait in LDS slots; stores go out per wave (8 rows of
//                             128 B of RGBA32F).
//   rt_trace_rays_kernel<B>   rayTraceRay on an arbitrary ray list (parity / fuzz entry point).
//   rt_intersect_kernel       g_scene.intersection on an arbitrary ray list (primitive KATs).
//   rt_unshuffle_kernel       multi-GPU: gathered row bands -> image order.
//
// Reference: /root/reference/Hw4/MySdlApplication.cpp (rayTraceScreen :1251-1324, rayTraceRay
// :1184-1249, intersection code :611-823, :1084-1113).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_diag.h"
#include "rt_device.hpp"
#include "rt_internal.hpp"

using namespace rt;

#ifndef RT_WAVE_TRACE
#define RT_WAVE_TRACE 0
#endif
// __launch_bounds__ minimum waves per EU of the depth <= 3 render kernels.  0 (default): 6 for depth <= 2
// (<= 80 VGPRs, no spills since the bounce loop stopped carrying the previous ray through the light loop),
// 5 for depth 3 (<= 96 VGPRs; 6 would spill 8 B/lane).
#ifndef RT_MINW
#define RT_MINW 0
#endif
#ifndef RT_NT_STORES
#define RT_NT_STORES 0                         // 1: non-temporal RGBA32F/RGBA8 stores (A/B)
#endif
#ifndef RT_WG_FAST
#define RT_WG_FAST 64                          // workgroup of the default render kernels: 64 (8 x 8) or 128 (16 x 8)
#endif
#ifndef RT_MINW_CULL
#define RT_MINW_CULL 5                         // the culling variant (>= kConeMin spheres): 87 VGPRs, no spills
#endif

namespace {

constexpr int kTileW = 32;   // workgroup tile: 32 columns ...
constexpr int kTileH = 8;    // ... x 8 rows = 256 pixels
constexpr int kThreads = 256;
static_assert(kThreads == kSlotStride, "one LDS colour slot column per work-item");

// LDS bytes of trace()'s per-level slots for depth B: 3 doubles (+ the material id when TRANSP) per level
// and work-item of a `wg`-thread workgroup.
__host__ __device__ constexpr int slot_bytes(int B, bool transp, int wg = kSlotStride) {
    return (B + 1) * (3 * 8 + (transp ? 4 : 0)) * wg;
}

struct RenderParams {
    double eye[3];
    double look[3];
    double right[3];
    double upp[3];
    double pitch;
    int32_t bottom_x, bottom_y;
    int32_t width, height;
    int32_t local_rows;                        // over all frames
    int32_t frame_rows;                        // local rows per frame
    int32_t frames;
    int32_t band_height, n_ranks, rank;
    int32_t lds_bytes;
    int32_t np;
    int32_t nl;
    int32_t wg_staging;                        // 1: stage the 32 x 8 tile in LDS behind a workgroup barrier
    float look32[3], right32[3], upp32[3], eye32[3], pitch32;   // FP32 camera for primary_cone_mask
    float cone_slack;                          // its error bound (render_params)
    const int32_t* tile_rows;                  // dispatch order of tile rows (nullptr: bottom to top)
    uint32_t* row_cost;                        // calibration render: per tile row, sum of wave times (100 MHz)
    int32_t tile_rows_n;                       // tile rows of this launch
};

constexpr int kGridY = 32768;                  // grid.y per grid.z slice

// Image row (within its frame) of local row lr; local rows are frame-major (rt_rows.frames).
__device__ __forceinline__ int global_row_of(const RenderParams& P, int lr) {
    if (P.frames > 1) lr %= P.frame_rows;
    if (P.n_ranks <= 1) return lr;
    int band = lr / P.band_height, within = lr - band * P.band_height;
    return (band * P.n_ranks + P.rank) * P.band_height + within;
}

// Copy the scene record into LDS, 16 B per work-item per step.
__device__ __forceinline__ void stage_scene(char* dst, const DevScene* __restrict__ src, int bytes) {
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (int k = threadIdx.x; k < (bytes >> 4); k += kThreads) d[k] = s[k];
}

// floor(clamp(c, 0, 1) * 255 + 0.5) (RGBA8 definition).  fmax/fmin (v_max/v_min_f64) clamp
// exactly like the comparisons; NaN becomes 0 (the conversion of a NaN is 0 on the device as well).
__device__ __forceinline__ unsigned char to_u8(double c) {
    double v = fmin(fmax(c, 0.0), 1.0);
    return (unsigned char)(int)floor(v * 255.0 + 0.5);
}

#if RT_WAVE_TRACE
// Diagnostic build only (tools/wave_trace.py): per workgroup {start, end} shader-clock stamps and HW_ID.
__device__ uint64_t* g_wtrace = nullptr;
#endif

template <int B, int LDS, int MINW, bool TRANSP, bool CULL, int WG = kThreads, bool TREE = false>
__global__ __launch_bounds__(WG, MINW) void rt_render_kernel(const DevScene* __restrict__ gscene,
                                                             RenderParams P, float4* __restrict__ out32,
                                                             uchar4* __restrict__ out8,
                                                             double* __restrict__ out64,
                                                             uint32_t* __restrict__ outrc) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
#if RT_WAVE_TRACE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const uint64_t t_cal = P.row_cost ? __builtin_amdgcn_s_memrealtime() : 0;
    // LDS: [header | DevSphere[np] | DevSpherePrim[np]] (LDS = 1), the per-level colour slots of trace()
    // (slot_bytes), then the output staging tile (12 KB, RT_WG_STAGING only).
    // The scene record is broadcast into LDS once per workgroup; the FP32 filter images stay in global
    // memory and are read with wave-uniform indices (scalar loads, SGPR operands).
    int off = 0;
    const DevScene* S = gscene;
    if (LDS) {
        stage_scene(smem, gscene, P.lds_bytes);
        S = reinterpret_cast<const DevScene*>(smem);
        off = P.lds_bytes;
    }
    double* slot = reinterpret_cast<double*>(smem + off) + tid;
    int* mslot = reinterpret_cast<int*>(smem + off + 3 * 8 * (B + 1) * WG) + tid;
    off += slot_bytes(B, TRANSP, WG);
    float4* st32 = reinterpret_cast<float4*>(smem + off);                              // [8][32] 4 KB
    double* st64 = reinterpret_cast<double*>(smem + off + 4096);                        // [8][32][3] 6 KB
    uint32_t* strc = reinterpret_cast<uint32_t*>(smem + off + 4096 + 6144);             // [8][32] 1 KB
    uchar4* st8 = reinterpret_cast<uchar4*>(smem + off + 4096 + 6144 + 1024);           // [8][32] 1 KB
    if (LDS) __syncthreads();
    const SceneView V = view_of(S, gscene, P.np, P.nl);
    const d3 eye = ld3(P.eye);

    const int wave = tid >> 6, lane = tid & 63;
    // The 32 x 8 tile (WG = 256) is cut into 4 wave blocks of 8 x 8 pixels (square blocks keep a wave's
    // rays coherent; 16 x 4 and 32 x 2 blocks measured no faster, and 32 x 2 slower at c5); WG = 64: one
    // wave, one 8 x 8 tile.
    constexpr int bw = 8, bh = 8, TW = WG / 8;
    const int bx0 = wave * bw, by0 = 0;
    const int cx = bx0 + (lane & 7);               // column inside the tile
    const int cy = lane >> 3;                      // row inside the tile
    const int tx = blockIdx.x;                      // 2-D grid: tiles_x x tiles_y
    const int gy = (int)(blockIdx.z * kGridY + blockIdx.y);    // tile rows beyond kGridY go to grid.z
    const int ty = P.tile_rows ? P.tile_rows[gy] : gy;
    if ((unsigned)ty >= (unsigned)P.tile_rows_n) return;        // padding of the last grid.z slice
    const int i = tx * TW + cx;
    const int lr = ty * kTileH + cy;
    const bool valid = i < P.width && lr < P.local_rows;

    // Per-wave sphere culling (all lanes active here).  The block's rows must be contiguous image rows.
    uint64_t cone = ~0ull;
    if (P.np >= kConeMin) {
        // Within one frame global_row_of is increasing, so jb - ja == 7 means 8 consecutive rows.
        const int lr0 = ty * kTileH + by0, ja = global_row_of(P, lr0), jb = global_row_of(P, lr0 + bh - 1);
        const bool one_frame = P.frames <= 1 || lr0 / P.frame_rows == (lr0 + bh - 1) / P.frame_rows;
        const float hx = 0.5f * (float)(bw - 1), hy = 0.5f * (float)(bh - 1);
        if (one_frame && jb - ja == bh - 1)
            cone = primary_cone_mask(V, P.look32, P.right32, P.upp32, P.eye32, P.pitch32,
                                     (float)(tx * TW + bx0 + P.bottom_x) + hx, (float)(ja + P.bottom_y) + hy,
                                     sqrtf(hx * hx + hy * hy), P.cone_slack, lane);
    }

    // Every lane traces (trace() reduces over the wave): lanes outside the frame trace a clamped pixel
    // and store nothing.
    uint32_t seg = 0, sh = 0;
    const int ic = i < P.width ? i : P.width - 1, lrc = lr < P.local_rows ? lr : P.local_rows - 1;
    const int j = global_row_of(P, lrc);
    const d3 right = ld3(P.right), upp = ld3(P.upp);
    // Primary ray Line(camera, sp), SURVEY.md Appendix B (basis: rayTraceScreen :1270-1279).
    const d3 sp = add(add(ld3(P.look), scl(P.pitch * (double)(ic + P.bottom_x), right)),
                      scl(P.pitch * (double)(j + P.bottom_y), upp));
    const d3 bdP = sub(ld3(V.S->bc), eye);                  // bounding-sphere deltaP for p0 = camera
    d3 col;
    if constexpr (TREE)
        col = trace_tree<B>(V, eye, sp, &seg, &sh);
    else
        col = trace<B, true, TRANSP, CULL, WG>(V, eye, sp, bdP, dot(bdP, bdP), cone, &seg, &sh, slot, mslot);

    if (WG != kThreads || !P.wg_staging) {
        // Direct stores: each wave writes its 8 x 8 block as 8 row segments (128 B of RGBA32F each) and
        // retires without waiting at a workgroup barrier for slower waves of the tile.
        if (valid) {
            const size_t k = (size_t)lr * P.width + i;
#if RT_NT_STORES
            if (out32) {
                float* o = reinterpret_cast<float*>(out32 + k);
                __builtin_nontemporal_store((float)col.x, o);
                __builtin_nontemporal_store((float)col.y, o + 1);
                __builtin_nontemporal_store((float)col.z, o + 2);
                __builtin_nontemporal_store(1.0f, o + 3);
            }
#else
            if (out32) out32[k] = make_float4((float)col.x, (float)col.y, (float)col.z, 1.0f);
#endif
            if (out64) { out64[3 * k] = col.x; out64[3 * k + 1] = col.y; out64[3 * k + 2] = col.z; }
            if (outrc) outrc[k] = seg | (sh << 16);
#if RT_NT_STORES
            if (out8) {
                const uint32_t px = (uint32_t)to_u8(col.x) | ((uint32_t)to_u8(col.y) << 8) |
                                    ((uint32_t)to_u8(col.z) << 16) | (255u << 24);
                __builtin_nontemporal_store(px, reinterpret_cast<uint32_t*>(out8 + k));
            }
#else
            if (out8) out8[k] = make_uchar4(to_u8(col.x), to_u8(col.y), to_u8(col.z), 255);
#endif
        }
        if (P.row_cost && tid == 0)
            atomicAdd(P.row_cost + ty, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cal));
#if RT_WAVE_TRACE
        if (g_wtrace && tid == 0) {
            const size_t w = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
            g_wtrace[3 * w] = t_start;
            g_wtrace[3 * w + 1] = __builtin_amdgcn_s_memrealtime();
            g_wtrace[3 * w + 2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                                  ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
        }
#endif
        return;
    }
    // Stage through LDS, then store whole tile rows.
    const int ts = cy * kTileW + cx;
    if (out32) st32[ts] = make_float4((float)col.x, (float)col.y, (float)col.z, 1.0f);
    if (out64) { st64[3 * ts] = col.x; st64[3 * ts + 1] = col.y; st64[3 * ts + 2] = col.z; }
    if (outrc) strc[ts] = seg | (sh << 16);
    if (out8) st8[ts] = make_uchar4(to_u8(col.x), to_u8(col.y), to_u8(col.z), 255);
    __syncthreads();
    const int oy = tid >> 5, ox = tid & 31;
    const int gi = tx * kTileW + ox, glr = ty * kTileH + oy;
    if (gi < P.width && glr < P.local_rows) {
        const size_t k = (size_t)glr * P.width + gi;
        if (out32) out32[k] = st32[tid];
        if (out64) {
            out64[3 * k] = st64[3 * tid];
            out64[3 * k + 1] = st64[3 * tid + 1];
            out64[3 * k + 2] = st64[3 * tid + 2];
        }
        if (outrc) outrc[k] = strc[tid];
        if (out8) out8[k] = st8[tid];
    }
    if (P.row_cost && tid == 0) atomicAdd(P.row_cost + ty, (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cal));
}

// Tile-row dispatch order from a calibration render's per-row costs: rows by decreasing cost (ties by
// index), so the longest rows are dispatched first and the cheap ones fill the tail (longest-processing-
// time-first list scheduling).  One workgroup, bitonic sort of (~cost, row) keys in LDS; n <= kOrderMax.
constexpr int kOrderMax = 8192;
constexpr int kRecalibrate = 8;                // renders of a moving camera per re-timing of the tile rows
__global__ __launch_bounds__(1024) void rt_order_kernel(const uint32_t* __restrict__ cost, int n,
                                                        int32_t* __restrict__ order) {
    __shared__ uint64_t key[kOrderMax];
    int m = 1;
    while (m < n) m <<= 1;
    for (int k = threadIdx.x; k < m; k += blockDim.x)
        key[k] = k < n ? ((uint64_t)(~cost[k]) << 32) | (uint32_t)k : ~0ull;
    __syncthreads();
    for (int size = 2; size <= m; size <<= 1) {
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int k = threadIdx.x; k < m; k += blockDim.x) {
                const int o = k ^ stride;
                if (o > k) {
                    const bool up = (k & size) == 0;
                    const uint64_t a = key[k], b = key[o];
                    if ((a > b) == up) { key[k] = b; key[o] = a; }
                }
            }
            __syncthreads();
        }
    }
    for (int k = threadIdx.x; k < n; k += blockDim.x) order[k] = (int32_t)(key[k] & 0xffffffffu);
}

// Per-eye primary-ray sphere data (run by rt_render_dev when the camera eye changes): deltaP = C - eye
// and dot(deltaP, deltaP) exactly as Shape::intersection computes them for p0 = camera (:740, :750), and
// the FP32 filter image f32(deltaP), c0 = (r2 - dd) + K (S0^2 + r2) rounded up, S0 = max|deltaP_i|.
// Filter error < 35 eps32 S0^2 + 2 eps32 r2 << K (S0^2 + r2), K = 256 eps32.  Padding spheres have
// r2 = -inf, hence c0 = -inf: always rejected.
__global__ __launch_bounds__(kThreads) void rt_prepare_kernel(DevScene* __restrict__ g, double ex, double ey,
                                                              double ez) {
    const int np = g->n_padded;
    DevSphere* sph = reinterpret_cast<DevSphere*>(g + 1);
    DevSpherePrim* prim = reinterpret_cast<DevSpherePrim*>(sph + np);
    DevSphereF* sphf = reinterpret_cast<DevSphereF*>(prim + np);
    DevSpherePrimF* primf = reinterpret_cast<DevSpherePrimF*>(sphf + np);
    DevSphereCone* cone = reinterpret_cast<DevSphereCone*>(primf + np);
    const d3 eye = mk(ex, ey, ez);
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k == 0) {
        g->eye[0] = ex; g->eye[1] = ey; g->eye[2] = ez;
        // board plane numerator for p0 = eye, as board_hit computes it (:657)
        g->board_num = dot(ld3(g->tri[0].n), sub(ld3(g->tri[0].v0), eye));
    }
    if (k >= np) return;
    d3 dP = sub(ld3(sph[k].c), eye);
    double dd = dot(dP, dP);
    DevSpherePrim pp;
    pp.dP[0] = dP.x; pp.dP[1] = dP.y; pp.dP[2] = dP.z;
    pp.dd = dd;
    prim[k] = pp;
    double s0 = fmax(fabs(dP.x), fmax(fabs(dP.y), fabs(dP.z)));
    double r2 = sph[k].r2;
    double c0 = (r2 - dd) + (double)kFilterK * (s0 * s0 + r2);
    DevSpherePrimF f;
    f.dx = (float)dP.x; f.dy = (float)dP.y; f.dz = (float)dP.z;
    f.c0 = __double2float_ru(c0);
    primf[k] = f;
    // Cone of directions from the eye that can hit sphere k (primary_cone_mask).  r' covers the FP64
    // test's rounding (disc error < 4 ulp of 3 D^2 < D^2 2^-48): r'^2 = r2 (1 + 2^-20) + D^2 2^-46.
    DevSphereCone cn;
    if (!(r2 >= 0.0)) {                                     // padding: never kept
        cn.vx = cn.vy = cn.vz = 1e30f;
        cn.chord = 0.0f;
    } else {
        double D = sqrt(dd);
        double rp = sqrt(r2 * (1.0 + 0x1p-20) + dd * 0x1p-46);
        double sn = rp / D;
        if (!(sn < 0.999)) {                                // eye inside / at the sphere: always kept
            cn.vx = cn.vy = cn.vz = 0.0f;
            cn.chord = 4.0f;
        } else {
            double ch = sn * sqrt(2.0 / (1.0 + sqrt(1.0 - sn * sn))) + 0x1p-20;
            cn.vx = (float)(dP.x / D); cn.vy = (float)(dP.y / D); cn.vz = (float)(dP.z / D);
            cn.chord = __double2float_ru(ch);
        }
    }
    cone[k] = cn;
}

// Eye-independent reciprocals of the division shortcuts (run by rt_set_scene): rcp_core of the checker
// square and of every triangle's den, with the compiler's own Newton steps (rt_device.hpp div_core).
__global__ __launch_bounds__(kThreads) void rt_scene_init_kernel(DevScene* __restrict__ g) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k == 0) g->rsquare = rcp_core(g->square);
    if (k < 2) g->tri[k].rden = g->tri[k].fast ? rcp_core(g->tri[k].den) : 0.0;
    const SceneView V = view_of(g, g, g->n_padded, g->n_lights);
    if (k < g->n_tris) {
        DevTri* t = const_cast<DevTri*>(V.tri) + k;
        t->rden = t->fast ? rcp_core(t->den) : 0.0;
    }
}

template <int B, bool TRANSP, bool TREE = false>
__global__ __launch_bounds__(kThreads) void rt_trace_rays_kernel(const DevScene* __restrict__ S,
                                                                 const double* __restrict__ starts,
                                                                 const double* __restrict__ ends, int n,
                                                                 double* __restrict__ rgb,
                                                                 uint32_t* __restrict__ rc) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // Every lane traces (trace() reduces over the wave); lanes past n repeat ray n - 1 and store nothing.
    const int k = blockIdx.x * kThreads + threadIdx.x, kk = k < n ? k : n - 1;
    uint32_t seg = 0, sh = 0;
    const SceneView V = view_of(S, S, S->n_padded, S->n_lights);
    double* slot = reinterpret_cast<double*>(smem) + threadIdx.x;
    int* mslot = reinterpret_cast<int*>(smem + 3 * 8 * (B + 1) * kSlotStride) + threadIdx.x;
    d3 c;
    if constexpr (TREE)
        c = trace_tree<B>(V, ld3(starts + 3 * kk), ld3(ends + 3 * kk), &seg, &sh);
    else
        c = trace<B, false, TRANSP, false>(V, ld3(starts + 3 * kk), ld3(ends + 3 * kk), mk(0.0, 0.0, 0.0), 0.0,
                                           ~0ull, &seg, &sh, slot, mslot);
    if (k >= n) return;
    if (rgb) { rgb[3 * k] = c.x; rgb[3 * k + 1] = c.y; rgb[3 * k + 2] = c.z; }
    if (rc) rc[k] = seg | (sh << 16);
}

__global__ __launch_bounds__(kThreads) void rt_intersect_kernel(const DevScene* __restrict__ S,
                                                                const double* __restrict__ starts,
                                                                const double* __restrict__ ends, int n,
                                                                rt_hit* __restrict__ hits) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const SceneView V = view_of(S, S, S->n_padded, S->n_lights);
    Ray r;
    r.p0 = ld3(starts + 3 * k);
    d3 d = sub(ld3(ends + 3 * k), r.p0);
    set_dir(&r, d, unit(d));
    set_origin_f32(S, &r);
    d3 p;
    int kind = closest_hit<true>(V, r, &p);
    rt_hit h;
    h.hit = kind >= 0;
    h.material = -1;
    for (int q = 0; q < 3; ++q) {
        h.point[q] = 0.0; h.normal[q] = 0.0; h.reflected_end[q] = 0.0; h.transmitted_end[q] = 0.0;
    }
    if (kind >= 0) {
        d3 n, pe;
        int mat;
        surface(V, kind, p, r.u, &n, &mat, &pe);
        d3 pt = transmitted_end(V, kind, mat, p, r.u, n);
        h.transmitted_end[0] = pt.x; h.transmitted_end[1] = pt.y; h.transmitted_end[2] = pt.z;
        h.material = mat;
        h.point[0] = p.x; h.point[1] = p.y; h.point[2] = p.z;
        h.normal[0] = n.x; h.normal[1] = n.y; h.normal[2] = n.z;
        h.reflected_end[0] = pe.x; h.reflected_end[1] = pe.y; h.reflected_end[2] = pe.z;
    }
    hits[k] = h;
}

// One workgroup per image row; copies the row from its rank's slab (rank 0's from src0 when given: the
// group's root does not send its own slab to itself), 16 bytes per work-item step when rows are 16-byte
// multiples (RGBA8 rows of W % 4 == 0, every RGBA32F row), else 4.
template <int VEC>
__global__ __launch_bounds__(kThreads) void rt_unshuffle_kernel(const uint32_t* __restrict__ src,
                                                                const uint32_t* __restrict__ src0,
                                                                uint32_t* __restrict__ dst, int row_words,
                                                                int height, int band_height, int n_ranks,
                                                                int slab_rows) {
    const int j = blockIdx.x;
    if (j >= height) return;
    const int band = j / band_height;
    const int rank = band % n_ranks;
    const int lr = (band / n_ranks) * band_height + (j - band * band_height);
    const uint32_t* s = (rank == 0 && src0) ? src0 + (size_t)lr * row_words
                                            : src + ((size_t)rank * slab_rows + lr) * row_words;
    uint32_t* d = dst + (size_t)j * row_words;
    if (VEC == 4) {
        const uint4* s4 = reinterpret_cast<const uint4*>(s);
        uint4* d4 = reinterpret_cast<uint4*>(d);
        for (int w = threadIdx.x; w < (row_words >> 2); w += kThreads) d4[w] = s4[w];
    } else {
        for (int w = threadIdx.x; w < row_words; w += kThreads) d[w] = s[w];
    }
}

// rt_render's ray statistics: sums of the per-pixel counters (primary+reflect segments, shadow rays) into
// sums[0], sums[1] (zeroed by the caller), so only 16 bytes cross PCIe instead of 4 bytes per pixel.
__global__ __launch_bounds__(kThreads) void rt_raysum_kernel(const uint32_t* __restrict__ rc, size_t n,
                                                             unsigned long long* __restrict__ sums) {
    unsigned long long seg = 0, sh = 0;
    for (size_t k = (size_t)blockIdx.x * kThreads + threadIdx.x; k < n; k += (size_t)gridDim.x * kThreads) {
        const uint32_t v = rc[k];
        seg += v & 0xffffu;
        sh += v >> 16;
    }
    for (int o = 32; o > 0; o >>= 1) {
        seg += __shfl_down(seg, o);
        sh += __shfl_down(sh, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(sums, seg);
        atomicAdd(sums + 1, sh);
    }
}

// Diagnostics (include/rt_diag.h): the exact-arithmetic fast paths of rt_device.hpp beside the compiler's
// IEEE sequences, on caller-supplied operands.  op 0: per vector v (3 doubles) -> 9 doubles
// [divs(v, len(v)), len(v), unit(v), |v| from unit(), len_fast(v)]; op 1: per pair (a, b) -> 2 doubles
// [a / b, div_core(a, b, rcp_core(b))].
__global__ __launch_bounds__(kThreads) void rt_probe_math_kernel(int op, const double* __restrict__ in, int n,
                                                                 double* __restrict__ out) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    if (op == 1) {                                          // (a, b) -> [a / b, div_core(a, b, rcp_core(b))]
        const double a = in[2 * k], b = in[2 * k + 1];
        out[2 * k] = a / b;
        out[2 * k + 1] = div_core(a, b, rcp_core(b));
        return;
    }
    const d3 v = mk(in[3 * k], in[3 * k + 1], in[3 * k + 2]);
    double* o = out + 9 * (size_t)k;
    const double l0 = len(v);
    const d3 u0 = divs(v, l0);
    double l1;
    const d3 u1 = unit(v, &l1);
    o[0] = u0.x, o[1] = u0.y, o[2] = u0.z, o[3] = l0;
    o[4] = u1.x, o[5] = u1.y, o[6] = u1.z, o[7] = l1;
    o[8] = len_fast(v);
}

// ------------------------------------------------------------------------------------------------
// Template dispatch.
// RT_MAX_B < 7 (experiment builds only, tools/variants.sh): deeper kernels are not instantiated.
#ifndef RT_MAX_B
#define RT_MAX_B 7
#endif
// MINW = 0: the depth-dependent default of RT_MINW (6 for depth <= 2, else 5).
template <int B, int LDS, int MINW, bool TRANSP, bool CULL, int WG, bool TREE>
hipError_t launch_render_one(dim3 grid, size_t lds, hipStream_t st, const DevScene* s, const RenderParams& P,
                             float4* o32, uchar4* o8, double* o64, uint32_t* orc) {
    constexpr int MW = MINW != 0 ? MINW : (B <= 2 ? 6 : 5);
    if constexpr (B > RT_MAX_B) {
        return hipErrorInvalidValue;
    } else {
        if (lds > 65536) {
            hipError_t e = hipFuncSetAttribute((const void*)rt_render_kernel<B, LDS, MW, TRANSP, CULL, WG, TREE>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL((rt_render_kernel<B, LDS, MW, TRANSP, CULL, WG, TREE>), grid, dim3(WG), lds, st, s, P, o32, o8,
                           o64, orc);
        return hipGetLastError();
    }
}

template <int LDS, int MINW, bool TRANSP, bool CULL = false, int WG = kThreads, bool TREE = false>
hipError_t launch_render_lds(int depth, dim3 grid, size_t lds, hipStream_t st, const DevScene* s,
                             const RenderParams& P, float4* o32, uchar4* o8, double* o64, uint32_t* orc) {
#define RT_CASE(b) \
    case b: return launch_render_one<b, LDS, MINW, TRANSP, CULL, WG, TREE>(grid, lds, st, s, P, o32, o8, o64, orc);
    switch (depth) {
        RT_CASE(0) RT_CASE(1) RT_CASE(2) RT_CASE(3) RT_CASE(4) RT_CASE(5) RT_CASE(6) RT_CASE(7)
        default: return hipErrorInvalidValue;
    }
#undef RT_CASE
}

template <bool TRANSP, bool TREE = false>
hipError_t launch_trace_rays(int depth, dim3 grid, hipStream_t st, const DevScene* s, const double* a,
                             const double* b, int n, double* rgb, uint32_t* rc) {
#define RT_CASE(k)                                                                                      \
    case k:                                                                                             \
        hipLaunchKernelGGL((rt_trace_rays_kernel<k, TRANSP, TREE>), grid, dim3(kThreads), TREE ? 0 : slot_bytes(k, TRANSP), st, s, \
                           a, b, n, rgb, rc);                                                           \
        break;
    switch (depth) {
        RT_CASE(0) RT_CASE(1) RT_CASE(2) RT_CASE(3) RT_CASE(4) RT_CASE(5) RT_CASE(6) RT_CASE(7)
        default: return hipErrorInvalidValue;
    }
#undef RT_CASE
    return hipGetLastError();
}

}  // namespace

// ================================================================================================
// C ABI — device half.

struct rt_ctx {
    int device = 0;
    DevScene* d_scene = nullptr;
    size_t scene_cap = 0;
    int scene_bytes = 0;
    int lds_bytes = 0;
    int n_padded = 0;
    int n_lights = 0;
    bool scene_set = false;
    bool transparent = false;                  // some material is transparent: TRANSP kernel variants
    bool tree = false;                         // some material transmits and reflects: TREE kernel variants
    bool eye_valid = false;                    // the device *Prim arrays hold data for `eye`
    bool ever_captured = false;                // a render was captured into a hipGraph: replays may rewrite
                                               // the per-eye data, so every later render re-prepares it
    double eye[3] = {0, 0, 0};
    std::vector<unsigned char> blob;           // host image of d_scene (rt_set_scene skips an unchanged scene)
    int min_waves = 5;                         // >= 5: the RT_MINW / RT_MINW_CULL launch bounds for depth <= 3 (measured faster
                                               // than no bound: tools/ab.py); RT_MIN_WAVES=0 disables
    int use_lds = 0;                           // RT_SCENE_IN_LDS=1: header + exact records in LDS (A/B: tools/ab.py)
    int wg_staging = 0;                        // RT_WG_STAGING=1: LDS-staged 32-pixel row stores (A/B)
    // Adaptive tile-row order (rt_order_kernel): the first render of a new (scene, camera, size, rows,
    // depth, outputs) view uses the identity order; the second render of the same view is a calibration
    // render that also times its tile rows; later renders dispatch the rows by decreasing time.  A render
    // of another camera with the same frame shape (size, rows, depth, outputs, scene) reuses the last
    // calibrated order — row costs change slowly with the camera — and every kRecalibrate-th such render
    // re-times the rows under it, so a moving camera keeps a longest-first order without paying for a
    // calibration every frame.  Any order is a permutation of the tile rows: images never depend on it.
    // order_mode (rt_diag_tile_order): 0 adaptive, 1 bottom-to-top.
    int32_t* d_tile_rows = nullptr;
    uint32_t* d_row_cost = nullptr;
    int n_tile_rows = 0;                       // capacity of both (kOrderMax, allocated by rt_ctx_create)
    using ViewKey = std::array<unsigned char, sizeof(rt_camera) + 6 * sizeof(int) + sizeof(rt_rows) + sizeof(uint64_t)>;
    bool order_valid = false;                  // d_tile_rows holds the order of view `order_key`
    ViewKey order_key{};
    bool seen_valid = false;                   // `seen_key`: the last view rendered once in identity order
    ViewKey seen_key{};
    int stale = 0;                             // renders of other cameras since the order was calibrated
    int order_mode = 0;
    uint64_t scene_gen = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // rt_render's device buffers (grow-only, reused across calls): rgba32f, rgba8, rgb64f, raycount, sums
    void* d_out[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    size_t out_cap[5] = {0, 0, 0, 0, 0};
};

#define RT_HIP(call)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) return rt_fail(RT_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

#if RT_WAVE_TRACE
extern "C" int rt_debug_wave_trace(void* dev_buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_wtrace), &dev_buf, sizeof(dev_buf)) == hipSuccess ? RT_OK : RT_EHIP;
}
#endif

extern "C" int rt_device_count(int* count) {
    if (!count) return rt_fail(RT_EINVAL, "rt_device_count: null pointer");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        return rt_fail(RT_EHIP, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
    }
    *count = n;
    return RT_OK;
}

extern "C" int rt_ctx_create(int device, rt_ctx** out) {
    if (!out) return rt_fail(RT_EINVAL, "rt_ctx_create: null out");
    *out = nullptr;
    int n = 0;
    int rc = rt_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n) return rt_fail(RT_EHIP, "rt_ctx_create: no HIP device " + std::to_string(device));
    RT_HIP(hipSetDevice(device));
    rt_ctx* c = new rt_ctx();
    c->device = device;
    if (const char* e = getenv("RT_SCENE_IN_LDS")) c->use_lds = atoi(e) != 0;
    if (const char* e = getenv("RT_MIN_WAVES")) c->min_waves = atoi(e);
    if (const char* e = getenv("RT_WG_STAGING")) c->wg_staging = atoi(e) != 0;
    if (const char* e = getenv("RT_TILE_ORDER")) c->order_mode = atoi(e) == 1 ? 1 : 0;   // 1: bottom-to-top (A/B)
    if (hipMalloc(&c->d_tile_rows, sizeof(int32_t) * kOrderMax) != hipSuccess ||
        hipMalloc(&c->d_row_cost, sizeof(uint32_t) * kOrderMax) != hipSuccess) {
        rt_ctx_destroy(c);
        return rt_fail(RT_ENOMEM, "rt_ctx_create: hipMalloc of the tile-row order failed");
    }
    c->n_tile_rows = kOrderMax;
    if (hipMemset(c->d_tile_rows, 0, sizeof(int32_t) * kOrderMax) != hipSuccess) {
        rt_ctx_destroy(c);
        return rt_fail(RT_EHIP, "rt_ctx_create: hipMemset of the tile-row order failed");
    }
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess) {
        delete c;
        return rt_fail(RT_EHIP, "rt_ctx_create: hipEventCreate failed");
    }
    *out = c;
    return RT_OK;
}

int rt_ctx_device(const rt_ctx* c) { return c ? c->device : -1; }

extern "C" int rt_ctx_destroy(rt_ctx* c) {
    if (!c) return RT_OK;
    (void)hipSetDevice(c->device);
    if (c->d_scene) (void)hipFree(c->d_scene);
    if (c->d_tile_rows) (void)hipFree(c->d_tile_rows);
    if (c->d_row_cost) (void)hipFree(c->d_row_cost);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (void* p : c->d_out)
        if (p) (void)hipFree(p);
    delete c;
    return RT_OK;
}

extern "C" int rt_set_scene(rt_ctx* c, const rt_scene* scene) {
    if (!c) return rt_fail(RT_EINVAL, "rt_set_scene: null context");
    std::vector<unsigned char> blob;
    int rc = rt_build_dev_scene(scene, &blob);
    if (rc) return rc;
    // An unchanged scene (same flattened record, byte for byte) keeps the device copy, the per-eye data
    // and the tile-row order: rt_render calls this every frame.
    if (c->scene_set && blob == c->blob) return RT_OK;
    RT_HIP(hipSetDevice(c->device));
    // Renders still in flight on any stream of this device read d_scene: wait for them before it changes.
    RT_HIP(hipDeviceSynchronize());
    c->scene_set = false;
    if (blob.size() > c->scene_cap) {
        if (c->d_scene) RT_HIP(hipFree(c->d_scene));
        c->d_scene = nullptr;
        c->scene_cap = 0;
        if (hipMalloc(&c->d_scene, blob.size()) != hipSuccess)
            return rt_fail(RT_ENOMEM, "rt_set_scene: hipMalloc failed");
        c->scene_cap = blob.size();
    }
    RT_HIP(hipMemcpy(c->d_scene, blob.data(), blob.size(), hipMemcpyHostToDevice));
    c->scene_bytes = (int)blob.size();
    const rt::DevScene* h = reinterpret_cast<const rt::DevScene*>(blob.data());
    hipLaunchKernelGGL(rt_scene_init_kernel, dim3((unsigned)((std::max(h->n_tris, 2) + kThreads - 1) / kThreads)),
                       dim3(kThreads), 0, nullptr, c->d_scene);
    RT_HIP(hipGetLastError());
    RT_HIP(hipDeviceSynchronize());
    c->lds_bytes = h->lds_bytes;
    c->n_padded = h->n_padded;
    c->n_lights = h->n_lights;
    c->transparent = h->transparent != 0 || h->n_meshes > 0;   // FULL kernel variants
    c->tree = h->tree != 0;
    c->eye_valid = false;
    c->scene_set = true;
    c->blob.swap(blob);
    ++c->scene_gen;
    return RT_OK;
}

static int render_params(const rt_ctx* c, const rt_camera* cam, int W, int H, int depth, const rt_rows* rows,
                         RenderParams* P) {
    if (!c) return rt_fail(RT_EINVAL, "render: null context");
    if (!c->scene_set) return rt_fail(RT_EINVAL, "render: rt_set_scene has not been called");
    if (!cam) return rt_fail(RT_EINVAL, "render: null camera");
    if (W <= 0 || H <= 0 || (long long)W * H > (1LL << 31)) return rt_fail(RT_EINVAL, "render: bad image size");
    if (depth < 0 || depth > RT_MAX_DEPTH) return rt_fail(RT_EINVAL, "render: depth out of range [0, 7]");
    int nl = 0;
    int rc = rt_local_rows(H, rows, &nl);
    if (rc) return rc;
    memset(P, 0, sizeof(*P));
    double right[3], upp[3];
    rt_camera_basis(cam, right, upp);
    for (int q = 0; q < 3; ++q) {
        P->eye[q] = cam->eye[q];
        P->look[q] = cam->look_at[q];
        P->right[q] = right[q];
        P->upp[q] = upp[q];
    }
    P->pitch = cam->pitch;
    P->bottom_x = cam->bottom_x;
    P->bottom_y = cam->bottom_y;
    P->width = W;
    P->height = H;
    P->local_rows = nl;
    bool banded = rows && rows->n_ranks > 1;
    P->band_height = banded ? rows->band_height : H;
    P->n_ranks = banded ? rows->n_ranks : 1;
    P->rank = banded ? rows->rank : 0;
    P->frames = (rows && rows->frames > 1) ? rows->frames : 1;
    P->frame_rows = nl / P->frames;
    P->lds_bytes = c->lds_bytes;
    P->np = c->n_padded;
    P->nl = c->n_lights;
    P->wg_staging = c->wg_staging;
    // FP32 camera for the per-wave cone culling, and the bound on its error as a chord distance: every
    // FP32 coordinate is below M in magnitude and carries < 16 roundings, and |sp - eye| >= |look - eye|
    // (right, up' are orthogonal to look - eye), so direction errors are < 64 eps32 M / |look - eye|.
    double M = 1.0, D2 = 0.0;
    for (int q = 0; q < 3; ++q) {
        P->look32[q] = (float)P->look[q];
        P->right32[q] = (float)P->right[q];
        P->upp32[q] = (float)P->upp[q];
        P->eye32[q] = (float)P->eye[q];
        M = std::max(M, std::fabs(P->look[q]) + std::fabs(P->eye[q]));
        D2 += (P->look[q] - P->eye[q]) * (P->look[q] - P->eye[q]);
    }
    P->pitch32 = (float)P->pitch;
    M += std::fabs(P->pitch) * (std::abs((double)P->bottom_x) + std::abs((double)P->bottom_y) + W + H + 16.0);
    const double slack = 0x1p-16 + 64.0 * 0x1p-24 * M / std::sqrt(D2);
    P->cone_slack = (D2 > 0.0 && slack < 0.25) ? (float)slack : 8.0f;   // 8: keep every sphere
    return RT_OK;
}

extern "C" int rt_render_dev(rt_ctx* c, const rt_camera* cam, int W, int H, int depth, const rt_rows* rows,
                             float* rgba32f, uint8_t* rgba8, double* rgb64f, uint32_t* raycount, void* stream) {
    RenderParams P;
    int rc = render_params(c, cam, W, H, depth, rows, &P);
    if (rc) return rc;
    if (P.local_rows == 0) return RT_OK;
    RT_HIP(hipSetDevice(c->device));
    // One-wave workgroups (8 x 8 tiles) by default: measured faster than 256-thread workgroups (32 x 8
    // tiles) at every config (c2 -1%, c3 -3%, c5 -12%: a finished wave's slot is refilled without
    // waiting for three siblings).  The A/B variants that share a workgroup-wide LDS copy (scene in LDS,
    // staged row stores) keep 256 threads.
    const bool big = c->use_lds || c->wg_staging;
    const int tw = big ? kTileW : RT_WG_FAST / 8;
    const int tiles_x = (W + tw - 1) / tw;
    const int tiles_y = (P.local_rows + kTileH - 1) / kTileH;
    P.tile_rows_n = tiles_y;
    hipStream_t st = (hipStream_t)stream;
    // A render captured into a hipGraph must be self-contained: it always prepares its eye's data and uses
    // the identity tile-row order (the context's order buffer belongs to whatever view it last calibrated).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    const bool capturing = cap != hipStreamCaptureStatusNone;
    if (capturing) c->ever_captured = true;
    bool calibrate = false;
    rt_ctx::ViewKey key{};
    if (!capturing && c->order_mode == 0 && tiles_y <= c->n_tile_rows) {
        // Key of the frame's work: camera, size, outputs, row plan, depth and scene generation.
        unsigned char* kp = key.data();                 // fixed size: no host allocation per render
        memcpy(kp, cam, sizeof(rt_camera)); kp += sizeof(rt_camera);
        // which outputs are written changes the rows' relative cost (an RGB64F parity render writes
        // 24 B per pixel): each output set gets its own calibration
        const int outs = (rgba32f ? 1 : 0) | (rgba8 ? 2 : 0) | (rgb64f ? 4 : 0) | (raycount ? 8 : 0);
        const int ints[6] = {W, H, depth, tiles_x, tiles_y, outs};
        memcpy(kp, ints, sizeof(ints)); kp += sizeof(ints);
        if (rows) memcpy(kp, rows, sizeof(rt_rows));
        kp += sizeof(rt_rows);
        memcpy(kp, &c->scene_gen, sizeof(uint64_t));
        constexpr size_t kCam = sizeof(rt_camera);
        const bool same_shape = c->order_valid &&
                                memcmp(key.data() + kCam, c->order_key.data() + kCam, key.size() - kCam) == 0;
        if (c->order_valid && key == c->order_key) {
            P.tile_rows = c->d_tile_rows;
        } else if (same_shape) {
            P.tile_rows = c->d_tile_rows;               // another camera: the last calibrated order
            if (++c->stale >= kRecalibrate) {           // ... re-timed every kRecalibrate-th render
                RT_HIP(hipMemsetAsync(c->d_row_cost, 0, sizeof(uint32_t) * tiles_y, st));
                P.row_cost = c->d_row_cost;
                calibrate = true;
                c->order_valid = false;
            }
        } else if (c->seen_valid && key == c->seen_key) {
            RT_HIP(hipMemsetAsync(c->d_row_cost, 0, sizeof(uint32_t) * tiles_y, st));
            P.row_cost = c->d_row_cost;                 // calibration render (identity order)
            calibrate = true;
            c->order_valid = false;                     // rt_order_kernel rewrites d_tile_rows below
        } else {
            c->seen_key = key;                          // first render of this view: identity order
            c->seen_valid = true;
        }
    }
    dim3 grid((unsigned)tiles_x, (unsigned)std::min(tiles_y, kGridY), (unsigned)((tiles_y + kGridY - 1) / kGridY));
    const size_t lds64 = slot_bytes(depth, c->transparent, 64);
    const size_t lds256 = (c->wg_staging ? 4096 + 6144 + 1024 + 1024 : 0) + slot_bytes(depth, c->transparent);
    hipError_t e;
    // Primary-ray sphere data for this eye (stream-ordered; only when the eye changes, or always once graphs
    // that carry their own prepare launch exist).
    if (capturing || c->ever_captured || !c->eye_valid || memcmp(c->eye, cam->eye, sizeof(c->eye)) != 0) {
        c->eye_valid = false;
        dim3 pg((unsigned)((std::max(c->n_padded, 1) + kThreads - 1) / kThreads));
        hipLaunchKernelGGL(rt_prepare_kernel, pg, dim3(kThreads), 0, st, c->d_scene, cam->eye[0], cam->eye[1],
                           cam->eye[2]);
        e = hipGetLastError();
        if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_prepare_kernel: ") + hipGetErrorString(e));
        memcpy(c->eye, cam->eye, sizeof(c->eye));
        c->eye_valid = true;
    }
    const bool cull = c->n_padded >= kConeMin, mw5 = c->min_waves >= 5 && depth <= 3;
    float4* o32 = reinterpret_cast<float4*>(rgba32f);
    uchar4* o8 = reinterpret_cast<uchar4*>(rgba8);
    if (c->tree)
        e = launch_render_lds<0, 1, true, false, 64, true>(depth, grid, 0, st, c->d_scene, P, o32, o8, rgb64f, raycount);
    else if (c->transparent)
        e = launch_render_lds<0, 1, true, false, 64>(depth, grid, lds64, st, c->d_scene, P, o32, o8, rgb64f, raycount);
    else if (c->use_lds)
        e = launch_render_lds<1, 1, false, false, kThreads>(depth, grid, c->lds_bytes + lds256, st, c->d_scene, P,
                                                             o32, o8, rgb64f, raycount);
    else if (c->wg_staging)
        e = (mw5 ? launch_render_lds<0, RT_MINW, false, false, kThreads> : launch_render_lds<0, 1, false, false, kThreads>)(
                depth, grid, lds256, st, c->d_scene, P, o32, o8, rgb64f, raycount);
    else {
        // >= kConeMin spheres: the wave-culling variant (secondary and shadow rays, rt_device.hpp CULL).
        auto launch = cull ? (mw5 ? launch_render_lds<0, RT_MINW_CULL, false, true, RT_WG_FAST>
                                  : launch_render_lds<0, 1, false, true, RT_WG_FAST>)
                           : (mw5 ? launch_render_lds<0, RT_MINW, false, false, RT_WG_FAST>
                                  : launch_render_lds<0, 1, false, false, RT_WG_FAST>);
        e = launch(depth, grid, slot_bytes(depth, false, RT_WG_FAST), st, c->d_scene, P, o32, o8, rgb64f, raycount);
    }
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render_kernel launch: ") + hipGetErrorString(e));
    if (calibrate) {
        hipLaunchKernelGGL(rt_order_kernel, dim3(1), dim3(1024), 0, st, c->d_row_cost, tiles_y, c->d_tile_rows);
        e = hipGetLastError();
        if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_order_kernel: ") + hipGetErrorString(e));
        c->order_key = key;                             // only once the order kernel is queued
        c->order_valid = true;
        c->stale = 0;
    }
    return RT_OK;
}

// Grow-only device buffer k of the context (rt_render's outputs).
static int ctx_buffer(rt_ctx* c, int k, size_t bytes, void** out) {
    if (bytes > c->out_cap[k]) {
        if (c->d_out[k]) (void)hipFree(c->d_out[k]);
        c->d_out[k] = nullptr;
        c->out_cap[k] = 0;
        if (hipMalloc(&c->d_out[k], bytes) != hipSuccess)
            return rt_fail(RT_ENOMEM, "rt_render: hipMalloc of output buffers failed");
        c->out_cap[k] = bytes;
    }
    *out = c->d_out[k];
    return RT_OK;
}

extern "C" int rt_render(rt_ctx* c, const rt_scene* scene, const rt_camera* cam, int W, int H, int depth,
                         const rt_rows* rows, float* rgba32f, uint8_t* rgba8, double* rgb64f, rt_stats* stats) {
    if (!c) return rt_fail(RT_EINVAL, "rt_render: null context");
    int rc = rt_set_scene(c, scene);                    // no device work when the scene is unchanged
    if (rc) return rc;
    RenderParams P;
    rc = render_params(c, cam, W, H, depth, rows, &P);
    if (rc) return rc;
    RT_HIP(hipSetDevice(c->device));
    const size_t npx = (size_t)P.local_rows * W;
    void* d[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    const size_t bytes[5] = {npx * 16, npx * 4, npx * 24, npx * 4, 2 * sizeof(unsigned long long)};
    const bool want[5] = {rgba32f != nullptr, rgba8 != nullptr, rgb64f != nullptr, stats != nullptr, stats != nullptr};
    for (int k = 0; k < 5; ++k)
        if (want[k] && npx > 0 && (rc = ctx_buffer(c, k, bytes[k], &d[k])) != RT_OK) return rc;
    hipError_t e = hipEventRecord(c->ev0, nullptr);
    if (e == hipSuccess) {
        rc = rt_render_dev(c, cam, W, H, depth, rows, (float*)d[0], (uint8_t*)d[1], (double*)d[2], (uint32_t*)d[3],
                           nullptr);
        if (rc) return rc;
        e = hipEventRecord(c->ev1, nullptr);
    }
    if (e == hipSuccess && stats && npx > 0) {
        e = hipMemsetAsync(d[4], 0, bytes[4], nullptr);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(rt_raysum_kernel, dim3((unsigned)std::min<size_t>((npx + kThreads - 1) / kThreads, 1024)),
                               dim3(kThreads), 0, nullptr, (const uint32_t*)d[3], npx, (unsigned long long*)d[4]);
            e = hipGetLastError();
        }
    }
    if (e == hipSuccess && rgba32f && npx) e = hipMemcpy(rgba32f, d[0], bytes[0], hipMemcpyDeviceToHost);
    if (e == hipSuccess && rgba8 && npx) e = hipMemcpy(rgba8, d[1], bytes[1], hipMemcpyDeviceToHost);
    if (e == hipSuccess && rgb64f && npx) e = hipMemcpy(rgb64f, d[2], bytes[2], hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess && stats) {
        unsigned long long sums[2] = {0, 0};
        if (npx) e = hipMemcpy(sums, d[4], sizeof(sums), hipMemcpyDeviceToHost);
        stats->primary_rays = npx;
        stats->reflect_rays = sums[0] - npx;
        stats->shadow_rays = sums[1];
        float ms = 0.f;
        if (e == hipSuccess && npx) e = hipEventElapsedTime(&ms, c->ev0, c->ev1);
        stats->kernel_ms = ms;
    }
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render: ") + hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_trace_rays_dev(rt_ctx* c, const double* starts, const double* ends, int n, int depth,
                                 double* rgb64f, uint32_t* raycount, void* stream) {
    if (!c || !c->scene_set) return rt_fail(RT_EINVAL, "rt_trace_rays_dev: no context/scene");
    if (n < 0 || (n > 0 && (!starts || !ends))) return rt_fail(RT_EINVAL, "rt_trace_rays_dev: bad rays");
    if (depth < 0 || depth > RT_MAX_DEPTH) return rt_fail(RT_EINVAL, "rt_trace_rays_dev: depth out of range");
    if (n == 0) return RT_OK;
    RT_HIP(hipSetDevice(c->device));
    dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
    hipError_t e = (c->tree ? launch_trace_rays<true, true>
                    : c->transparent ? launch_trace_rays<true> : launch_trace_rays<false>)(
        depth, grid, (hipStream_t)stream, c->d_scene, starts, ends, n, rgb64f, raycount);
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_trace_rays_kernel: ") + hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_intersect_dev(rt_ctx* c, const double* starts, const double* ends, int n, rt_hit* hits,
                                void* stream) {
    if (!c || !c->scene_set) return rt_fail(RT_EINVAL, "rt_intersect_dev: no context/scene");
    if (n < 0 || (n > 0 && (!starts || !ends || !hits))) return rt_fail(RT_EINVAL, "rt_intersect_dev: bad rays");
    if (n == 0) return RT_OK;
    RT_HIP(hipSetDevice(c->device));
    dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
    hipLaunchKernelGGL(rt_intersect_kernel, grid, dim3(kThreads), 0, (hipStream_t)stream, c->d_scene, starts, ends,
                       n, hits);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_intersect_kernel: ") + hipGetErrorString(e));
    return RT_OK;
}

int rt_unshuffle_dev_ex(const void* gathered, const void* rank0_slab, void* image, int W, int H, int elem_bytes,
                        int band_height, int n_ranks, int slab_rows, void* stream) {
    if (!gathered || !image) return rt_fail(RT_EINVAL, "rt_unshuffle_dev: null buffer");
    if (W <= 0 || H <= 0 || band_height <= 0 || n_ranks <= 0 || slab_rows < 0)
        return rt_fail(RT_EINVAL, "rt_unshuffle_dev: bad geometry");
    if (elem_bytes <= 0 || ((long long)W * elem_bytes) % 4 != 0)
        return rt_fail(RT_EINVAL, "rt_unshuffle_dev: row bytes must be a multiple of 4");
    rt_rows r = {band_height, n_ranks, 0, 0};
    for (int q = 0; q < n_ranks; ++q) {
        int nl = 0;
        r.rank = q;
        rt_local_rows(H, &r, &nl);
        if (nl > slab_rows) return rt_fail(RT_EINVAL, "rt_unshuffle_dev: slab_rows smaller than a rank's rows");
    }
    const int row_words = (int)(((long long)W * elem_bytes) / 4);
    const bool vec = row_words % 4 == 0 && ((uintptr_t)gathered | (uintptr_t)rank0_slab | (uintptr_t)image) % 16 == 0;
    auto k = vec ? rt_unshuffle_kernel<4> : rt_unshuffle_kernel<1>;
    hipLaunchKernelGGL(k, dim3((unsigned)H), dim3(kThreads), 0, (hipStream_t)stream, (const uint32_t*)gathered,
                       (const uint32_t*)rank0_slab, (uint32_t*)image, row_words, H, band_height, n_ranks, slab_rows);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_unshuffle_kernel: ") + hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_unshuffle_dev(const void* gathered, void* image, int W, int H, int elem_bytes, int band_height,
                                int n_ranks, int slab_rows, void* stream) {
    return rt_unshuffle_dev_ex(gathered, nullptr, image, W, H, elem_bytes, band_height, n_ranks, slab_rows, stream);
}

// Diagnostics (include/rt_diag.h): tile-row dispatch order of later renders: 0 adaptive (default), 1
// bottom-to-top.
extern "C" int rt_diag_tile_order(rt_ctx* c, int mode) {
    if (!c || (mode != 0 && mode != 1)) return rt_fail(RT_EINVAL, "rt_diag_tile_order: bad args");
    c->order_mode = mode;
    c->order_valid = false;
    c->seen_valid = false;
    return RT_OK;
}

// Diagnostics (include/rt_diag.h): registers and scratch of the render kernel instance rt_render_dev
// launches for `depth` and scene kind `variant` (0 spheres + board, 1 >= kConeMin spheres (CULL),
// 2 meshes / transparency, 3 ray trees) — the tests assert the default instances never spill.
template <int B>
static const void* render_kernel_of(int variant) {
    constexpr int kFast = B <= 3 ? (RT_MINW != 0 ? RT_MINW : (B <= 2 ? 6 : 5)) : 1;
    constexpr int kCull = B <= 3 ? RT_MINW_CULL : 1;
    switch (variant) {
        case 0: return (const void*)rt_render_kernel<B, 0, kFast, false, false, RT_WG_FAST, false>;
        case 1: return (const void*)rt_render_kernel<B, 0, kCull, false, true, RT_WG_FAST, false>;
        case 2: return (const void*)rt_render_kernel<B, 0, 1, true, false, 64, false>;
        case 3: return (const void*)rt_render_kernel<B, 0, 1, true, false, 64, true>;
        default: return nullptr;
    }
}

extern "C" int rt_diag_kernel_resources(int depth, int variant, int* vgprs, int* scratch_bytes) {
    if (depth < 0 || depth > RT_MAX_B || variant < 0 || variant > 3 || !vgprs || !scratch_bytes)
        return rt_fail(RT_EINVAL, "rt_diag_kernel_resources: bad arguments");
    const void* f = nullptr;
    switch (depth) {
        case 0: f = render_kernel_of<0>(variant); break;
        case 1: f = render_kernel_of<1>(variant); break;
        case 2: f = render_kernel_of<2>(variant); break;
        case 3: f = render_kernel_of<3>(variant); break;
#if RT_MAX_B >= 7
        case 4: f = render_kernel_of<4>(variant); break;
        case 5: f = render_kernel_of<5>(variant); break;
        case 6: f = render_kernel_of<6>(variant); break;
        case 7: f = render_kernel_of<7>(variant); break;
#endif
    }
    hipFuncAttributes a;
    RT_HIP(hipFuncGetAttributes(&a, f));
    *vgprs = a.numRegs;
    *scratch_bytes = (int)a.localSizeBytes;
    return RT_OK;
}

extern "C" int rt_probe_math_dev(int op, const double* in, int n, double* out, void* stream) {
    if (op != 0 && op != 1) return rt_fail(RT_EINVAL, "rt_probe_math_dev: unknown op");
    if (n < 0 || (n > 0 && (!in || !out))) return rt_fail(RT_EINVAL, "rt_probe_math_dev: bad buffers");
    if (n == 0) return RT_OK;
    hipLaunchKernelGGL(rt_probe_math_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       (hipStream_t)stream, op, in, n, out);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_probe_math_kernel: ") + hipGetErrorString(e));
    return RT_OK;
}
