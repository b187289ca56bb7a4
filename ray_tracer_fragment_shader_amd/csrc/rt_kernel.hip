// rt_kernel.hip — MI355X (gfx950) kernels and the device half of the C ABI (include/rt_api.h).
//
// Kernels (the render and ray-list kernels are templates in rt_render.hpp, instantiated per depth in
// rt_render_b<B>.hip; the rest live here)
//   rt_render_kernel<...>     one work-item per pixel, FP64, iterative bounce loop (rt_render.hpp)
//   rt_trace_rays_kernel<B>   rayTraceRay on an arbitrary ray list (rt_render.hpp)
//   rt_prepare_kernel         per-eye sphere data, board numerator and cull flag (once per camera eye)
//   rt_scene_init_kernel      device-side reciprocals of constant divisors (once per scene)
//   rt_rowsum_kernel, rt_order_kernel, rt_disp_kernel
//                             the dispatch table of a calibrated view: tile rows (or tiles, hipCUB radix sort)
//                             longest first from a calibration render's per-tile wave times
//   rt_intersect_kernel       g_scene.intersection on an arbitrary ray list (primitive KATs)
//   rt_unpack_kernel          multi-GPU: gathered row bands -> image order, packed pixels -> RGBA
//   rt_raysum_kernel          rt_render's ray statistics
//
// Reference: /root/reference/Hw4/MySdlApplication.cpp (rayTraceScreen :1251-1324, rayTraceRay
// :1184-1249, intersection code :611-823, :1084-1113).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/rt_api.h"
#include "../../include/rt_diag.h"
#include "rt_internal.hpp"
#include "rt_render.hpp"

using namespace rt;

namespace {

using namespace rtk;

#if RT_WAVE_TRACE
uint64_t* g_wtrace = nullptr;                  // diagnostic build only (tools/wave_trace.py)
#endif

// Tile-row dispatch order from a calibration render's per-row costs: rows by decreasing cost (ties by
// index), so the longest rows are dispatched first and the cheap ones fill the tail (longest-processing-
// time-first list scheduling).  One workgroup, bitonic sort of (~cost, row) keys in LDS; n <= kOrderMax.
constexpr int kOrderMax = 8192;
#ifndef RT_CONE_CACHE_DEFAULT
#define RT_CONE_CACHE_DEFAULT 1
#endif
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

// Per tile row, the sum of its tiles' wave times (the row order's cost); one workgroup per row.
__global__ __launch_bounds__(256) void rt_rowsum_kernel(const uint32_t* __restrict__ tile_cost, int tiles_x,
                                                        uint32_t* __restrict__ row_cost) {
    __shared__ uint32_t part[256];
    uint32_t acc = 0;
    for (int x = threadIdx.x; x < tiles_x; x += 256) acc += tile_cost[(size_t)blockIdx.x * tiles_x + x];
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) part[threadIdx.x] += part[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) row_cost[blockIdx.x] = part[0];
}

__global__ __launch_bounds__(256) void rt_iota_kernel(int32_t* __restrict__ v, int n) {
    const int k = blockIdx.x * 256 + threadIdx.x;
    if (k < n) v[k] = k;
}

// The dispatch table of a calibrated view: position L (linear workgroup id, L = gy * tiles_x + bx) traces tile
// by_pos[L] (tile order: tile indices by decreasing calibrated time) or, row order (by_pos = nullptr), tile column
// tile_col(bx, gy) of tile row row_order[gy]; with the calibration render's per-tile primary cone masks when
// `cone` (else 0).  Stored at cone_slot(L): grouped by the XCD workgroup L runs on.
__global__ __launch_bounds__(256) void rt_disp_kernel(const int32_t* __restrict__ row_order,
                                                      const int32_t* __restrict__ by_pos,
                                                      const uint64_t* __restrict__ cone, int tiles_x, int tiles_y,
                                                      DispRec* __restrict__ disp) {
    const size_t k = (size_t)blockIdx.x * 256 + threadIdx.x, n = (size_t)tiles_x * tiles_y;
    if (k >= n) return;
    int tx, ty;
    if (by_pos) {
        const int t = by_pos[k];
        ty = t / tiles_x;
        tx = t - ty * tiles_x;
    } else {
        const int gy = (int)(k / tiles_x), bx = (int)(k - (size_t)gy * tiles_x);
        ty = row_order[gy];
        tx = tile_col(bx, gy, tiles_x);
    }
    const uint64_t m = cone ? cone[(size_t)ty * tiles_x + tx] : 0;
    DispRec r;
    r.cone_lo = (uint32_t)m;
    r.cone_hi = (uint32_t)(m >> 32);
    r.tile = ((uint32_t)ty << 16) | (uint32_t)tx;
    r.pad = 0;
    disp[cone_slot(k, n)] = r;
}

// Per-eye primary-ray sphere data (run by rt_render_dev when the camera eye changes): deltaP = C - eye
// and dot(deltaP, deltaP) exactly as Shape::intersection computes them for p0 = camera (:740, :750), and
// the FP32 filter image f32(deltaP), c0 = (r2 - dd) + K (S0^2 + r2) rounded up, S0 = max|deltaP_i|.
// Filter error < 35 eps32 S0^2 + 2 eps32 r2 << K (S0^2 + r2), K = 256 eps32.  Padding spheres have
// r2 = -inf, hence c0 = -inf: always rejected.
__global__ __launch_bounds__(kThreads) void rt_prepare_kernel(DevScene* __restrict__ g, double ex, double ey,
                                                              double ez) {
    const int np = g->n_padded, ns = g->n_stride;
    DevSphere* sph = reinterpret_cast<DevSphere*>(g + 1);
    DevSpherePrim* prim = reinterpret_cast<DevSpherePrim*>(sph + ns);
    DevSphereF* sphf = reinterpret_cast<DevSphereF*>(prim + ns);
    DevSpherePrimF* primf = reinterpret_cast<DevSpherePrimF*>(sphf + ns);
    DevSphereCone* cone = reinterpret_cast<DevSphereCone*>(primf + ns);
    const d3 eye = mk(ex, ey, ez);
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k == 0) {
        g->eye[0] = ex; g->eye[1] = ey; g->eye[2] = ez;
        // board plane numerator for p0 = eye, as board_hit computes it (:657)
        g->board_num = dot(ld3(g->tri[0].n), sub(ld3(g->tri[0].v0), eye));
        g->hits_ok = hits_ok_from(g, eye);      // hit points of rays from this eye skip the cull (hits_inside)
        // A primary ray that hits an object passes g_scene's cull when every object lies within R - 1 of bc
        // (hits_inside) and the eye is at least R + 1 away: the line then passes within R - 1 of bc, so its exact
        // disc >= R^2 - (R - 1)^2 = 2R - 1, and the eye being outside the bound puts the entry root at
        // s >= D - R >= 1 (the hit lies ahead of the eye, past the entry); the FP64 rounding of disc and s is
        // ~2^-49 (D^2 + R^2) and ~2^-50 (D + R), far below 2R - 1 and 1 - eps for D <= 2^20 (R + 1).  (s >= 1 clears the
        // reference's |s| < eps cull only for eps < 1: required explicitly, as hits_inside does through inner2.)
        const double bx = eye.x - g->bc[0], by = eye.y - g->bc[1], bz = eye.z - g->bc[2];
        const double D2 = bx * bx + by * by + bz * bz, R1 = sqrt(g->br2) + 1.0;
        g->prim_bound_ok = (g->bound_on != 0) & (g->hits_inside != 0) & (g->eps < 0.5) &
                           (D2 >= R1 * R1 * (1.0 + 0x1p-30)) & (D2 <= R1 * R1 * 0x1p40);
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
    const SceneView V = view_of(g, g, g->n_padded, g->n_stride, g->n_lights);
    if (k < g->n_tris) {
        DevTri* t = const_cast<DevTri*>(V.tri) + k;
        t->rden = t->fast ? rcp_core(t->den) : 0.0;
    }
}

__global__ __launch_bounds__(kThreads) void rt_intersect_kernel(const DevScene* __restrict__ S,
                                                                const double* __restrict__ starts,
                                                                const double* __restrict__ ends, int n,
                                                                rt_hit* __restrict__ hits) {
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= n) return;
    const SceneView V = view_of(S, S, S->n_padded, S->n_stride, S->n_lights);
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

// Row of the gathered buffer that holds image row j: rank = band % n_ranks, local row within its slab.  Rank 0's
// rows come from src0 when given (the group's root does not send its own slab to itself).
__device__ __forceinline__ const uint8_t* gathered_row(const uint8_t* src, const uint8_t* src0, int j, int band_height,
                                                       int n_ranks, int slab_rows, size_t row_bytes) {
    const int band = j / band_height;
    const int rank = band % n_ranks;
    const int lr = (band / n_ranks) * band_height + (j - band * band_height);
    return (rank == 0 && src0) ? src0 + (size_t)lr * row_bytes : src + ((size_t)rank * slab_rows + lr) * row_bytes;
}

// One workgroup per image row; copies the row from its rank's slab, 16 bytes per work-item step when rows are
// 16-byte multiples (RGBA8 rows of W % 4 == 0, every RGBA32F row), else 4.
template <int VEC>
__global__ __launch_bounds__(kThreads) void rt_unshuffle_kernel(const uint32_t* __restrict__ src,
                                                                const uint32_t* __restrict__ src0,
                                                                uint32_t* __restrict__ dst, int row_words,
                                                                int height, int band_height, int n_ranks,
                                                                int slab_rows) {
    const int j = blockIdx.x;
    if (j >= height) return;
    const uint32_t* s = reinterpret_cast<const uint32_t*>(
        gathered_row(reinterpret_cast<const uint8_t*>(src), reinterpret_cast<const uint8_t*>(src0), j, band_height,
                     n_ranks, slab_rows, (size_t)row_words * 4));
    uint32_t* d = dst + (size_t)j * row_words;
    if (VEC == 4) {
        const uint4* s4 = reinterpret_cast<const uint4*>(s);
        uint4* d4 = reinterpret_cast<uint4*>(d);
        for (int w = threadIdx.x; w < (row_words >> 2); w += kThreads) d4[w] = s4[w];
    } else {
        for (int w = threadIdx.x; w < row_words; w += kThreads) d[w] = s[w];
    }
}

// Unshuffle + expand packed rows into RGBA images (the wire formats of rt_render_multi, include/rt_api.h):
//   kUnpackGray8: GRAY8 -> RGBA8 (g, g, g, 255);  kUnpackRgb8: RGB8 -> RGBA8 (r, g, b, 255);
//   kUnpackGray32f: GRAY32F -> RGBA32F (v, v, v, 1).
// Exact: the render kernel writes these very bytes into the RGBA images (achromatic scenes: R = G = B bit for
// bit).  VEC (16-byte aligned buffers, W % 4 == 0): 4 — 4 pixels per work-item step, 16-byte stores; 16 — a byte
// wire format: the same 16-byte stores, four steps per lane unrolled with their loads issued first, so a
// 4K row is one round trip per lane instead of four dependent ones (DESIGN §7 has the times).
constexpr int kUnpackGray8 = 0, kUnpackRgb8 = 1, kUnpackGray32f = 2;
__device__ __forceinline__ uint4 gray4_rgba(uint32_t g) {
    uint4 o;
    o.x = (g & 0xffu) * 0x010101u | 0xff000000u;
    o.y = ((g >> 8) & 0xffu) * 0x010101u | 0xff000000u;
    o.z = ((g >> 16) & 0xffu) * 0x010101u | 0xff000000u;
    o.w = (g >> 24) * 0x010101u | 0xff000000u;
    return o;
}
// three little-endian words r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3 -> four RGBA8 pixels
__device__ __forceinline__ uint4 rgb4_rgba(uint32_t a, uint32_t b, uint32_t c) {
    uint4 o;
    o.x = (a & 0xffffffu) | 0xff000000u;
    o.y = (a >> 24) | ((b & 0xffffu) << 8) | 0xff000000u;
    o.z = (b >> 16) | ((c & 0xffu) << 16) | 0xff000000u;
    o.w = (c >> 8) | 0xff000000u;
    return o;
}
template <int MODE, int VEC>
__global__ __launch_bounds__(kThreads) void rt_unpack_kernel(const uint8_t* __restrict__ src,
                                                             const uint8_t* __restrict__ src0,
                                                             uint8_t* __restrict__ dst, int W, int height,
                                                             int band_height, int n_ranks, int slab_rows) {
    const int j = blockIdx.x;
    if (j >= height) return;
    constexpr size_t in_px = MODE == kUnpackGray8 ? 1 : MODE == kUnpackRgb8 ? 3 : 4;
    constexpr size_t out_px = MODE == kUnpackGray32f ? 16 : 4;
    const uint8_t* s = gathered_row(src, src0, j, band_height, n_ranks, slab_rows, (size_t)W * in_px);
    uint8_t* d = dst + (size_t)j * W * out_px;
    if (VEC == 16 && MODE != kUnpackGray32f) {
        // four 4-pixel quads per lane, kThreads apart (every load and store instruction covers a contiguous run of the
        // row), the four loads issued before the first store
        const int groups = W >> 2;
        uint4* d4 = reinterpret_cast<uint4*>(d);
        for (int q0 = threadIdx.x; q0 < groups; q0 += 4 * kThreads) {
            uint32_t a[4], b[4], c[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * kThreads;
                if (q < groups) {
                    if (MODE == kUnpackGray8) {
                        a[u] = reinterpret_cast<const uint32_t*>(s)[q];
                    } else {
                        const uint32_t* s3 = reinterpret_cast<const uint32_t*>(s) + 3 * q;
                        a[u] = s3[0];
                        b[u] = s3[1];
                        c[u] = s3[2];
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int q = q0 + u * kThreads;
                if (q < groups) d4[q] = MODE == kUnpackGray8 ? gray4_rgba(a[u]) : rgb4_rgba(a[u], b[u], c[u]);
            }
        }
        return;
    }
    if (VEC) {
        const int groups = W >> 2;
        for (int q = threadIdx.x; q < groups; q += kThreads) {
            if (MODE == kUnpackGray8) {
                reinterpret_cast<uint4*>(d)[q] = gray4_rgba(reinterpret_cast<const uint32_t*>(s)[q]);
            } else if (MODE == kUnpackRgb8) {
                const uint32_t* s3 = reinterpret_cast<const uint32_t*>(s) + 3 * q;
                reinterpret_cast<uint4*>(d)[q] = rgb4_rgba(s3[0], s3[1], s3[2]);
            } else {
                const float4 v = reinterpret_cast<const float4*>(s)[q];
                float4* o = reinterpret_cast<float4*>(d) + 4 * q;
                o[0] = make_float4(v.x, v.x, v.x, 1.0f);
                o[1] = make_float4(v.y, v.y, v.y, 1.0f);
                o[2] = make_float4(v.z, v.z, v.z, 1.0f);
                o[3] = make_float4(v.w, v.w, v.w, 1.0f);
            }
        }
        return;
    }
    for (int x = threadIdx.x; x < W; x += kThreads) {
        if (MODE == kUnpackGray8) {
            const uint8_t g = s[x];
            d[4 * x] = g; d[4 * x + 1] = g; d[4 * x + 2] = g; d[4 * x + 3] = 255;
        } else if (MODE == kUnpackRgb8) {
            d[4 * x] = s[3 * x]; d[4 * x + 1] = s[3 * x + 1]; d[4 * x + 2] = s[3 * x + 2]; d[4 * x + 3] = 255;
        } else {
            float v;
            memcpy(&v, s + 4 * (size_t)x, 4);
            const float4 o = make_float4(v, v, v, 1.0f);
            memcpy(d + 16 * (size_t)x, &o, 16);
        }
    }
}

// rt_render's ray statistics: sums of the per-pixel counters (primary+reflect segments, shadow rays) into
// sums[0], sums[1] (zeroed by the caller), so only 16 bytes cross PCIe instead of 4 bytes per pixel.
// Device -> pinned host frame (rt_host_alloc memory, mapped into the device's address space): a copy kernel
// whose 16-byte stores cross PCIe straight into the host buffer.  On the render stream it needs no cross-stream
// hand-off; on the copy stream it overlaps the next frame's render (rt_ctx::copy_mode has the measurements).
__global__ __launch_bounds__(kThreads) void rt_copy_out_kernel(const uint8_t* __restrict__ src,
                                                               uint8_t* __restrict__ dst, size_t n) {
    const size_t n16 = n >> 4;
    const size_t step = (size_t)gridDim.x * kThreads;
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (size_t k = (size_t)blockIdx.x * kThreads + threadIdx.x; k < n16; k += step) d[k] = s[k];
    if (blockIdx.x == 0 && threadIdx.x < (n & 15)) dst[(n16 << 4) + threadIdx.x] = src[(n16 << 4) + threadIdx.x];
}

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
    int n_stride = 0;
    int n_lights = 0;
    bool scene_set = false;
    bool transparent = false;                  // some material is transparent: TRANSP kernel variants
    bool tree = false;                         // some material transmits and reflects: TREE kernel variants
    bool achromatic = false;                   // R = G = B everywhere (rt_scene_achromatic): GRAY formats allowed
    bool eye_valid = false;                    // the device *Prim arrays hold data for `eye`
    bool ever_captured = false;                // a render was captured into a hipGraph: replays may rewrite
                                               // the per-eye data, so every later render re-prepares it
    double eye[3] = {0, 0, 0};
    std::vector<unsigned char> blob;           // host image of d_scene (rt_set_scene skips an unchanged scene)
    int min_waves = 5;                         // >= 5: the RT_MINW / RT_MINW_CULL launch bounds for depth <= 3 (measured faster
                                               // than no bound: tools/ab.py); RT_MIN_WAVES=0 disables
    int use_lds = 0;                           // RT_SCENE_IN_LDS=1: header + exact records in LDS (A/B: tools/ab.py)
    int wg_staging = 0;                        // RT_WG_STAGING=1: LDS-staged 32-pixel row stores (A/B)
    // Where the packed host frames' device-to-host copy runs (r04, tools/copy_ab.py and tools/copy_trace.py on MI355X,
    // c2 GRAY8, 2.07 MB into pinned memory; us per frame, medians of 5 interleaved rounds x 60 frames):
    //                                              synchronous   pipelined (wait f-1)   (wait f-2)
    //   copy kernel behind the render (rs)             84-85         74-75               74-75
    //   copy kernel on the copy stream (cs), 16 WGs    100           74                  66
    //                                     4 / 8 WGs    122 / 108     111 / 77            111 / 64
    //   hipMemcpyAsync on the copy stream              106-107       59 / 95 / 290       59 / 95 / 290
    // The runtime executes that hipMemcpyAsync as its own blit kernel (__amd_rocclr_copyBuffer in the kernel trace, no
    // SDMA transfer in the memory-copy trace, whatever GPU_FORCE_BLIT_COPY_SIZE / ROC_ENABLE_LARGE_BAR /
    // HSA_ENABLE_SDMA / GPU_BLIT_ENGINE_TYPE say), and its pipelined rate settles in one of three states per process
    // (59, 95 or 290 us) — so the product uses its own copy kernel for both calls: behind the render on `rs` for
    // rt_render_packed, on `cs` with 16 workgroups (a copy beside the next render takes CUs from it: fewer
    // workgroups leave it more) after a cross-stream event for rt_render_packed_async.
    // r05: the HSA runtime does reach the SDMA engines (hsa_amd_memory_async_copy_on_engine; tools/mb_sdma.cpp: engines
    // 0-3 move the frame at 44.5 GB/s, 46 us, and take nothing from a kernel running beside them), and a copy queued
    // with a dependency signal that the render stream fires starts without the host (copy_mode 3, sd_* below).
    // tools/copy_ab.py, same box, 60 frames x 5 rounds:   synchronous   pipelined (wait f-1)   (wait f-2)
    //   copy kernel behind the render (rs)                    79.3          69.9                  70.2
    //   copy kernel on the copy stream (cs), 16 WGs           95.2          85.3                  85.7
    //   SDMA engine behind the render                         81.6          49.6                  49.5
    // So rt_render_packed_async defaults to the SDMA engine for page-locked buffers (the copy stream for others or
    // when no engine is free) and rt_render_packed to the copy kernel behind the render.  RT_COPY_MODE (1: rs, 0: cs,
    // 2: the kernel stores straight into the pinned buffer — 290 us: single-byte stores over PCIe, 3: SDMA),
    // RT_COPY_KERNEL (0: hipMemcpyAsync) and RT_COPY_BLOCKS override (A/B; -1 / 0: the defaults above).
    int copy_mode = -1;
    int copy_kernel = -1;
    int copy_blocks = 0;                       // RT_COPY_BLOCKS: workgroups of the copy kernel (0: the defaults above)
    // Adaptive tile-row order (rt_order_kernel): the first render of a new (scene, camera, size, rows,
    // depth, outputs) view uses the identity order; the second render of the same view is a calibration
    // render that also times its tile rows; later renders dispatch the rows by decreasing time.  A render
    // of another camera with the same frame shape (size, rows, depth, outputs, scene) reuses the last
    // calibrated order and every kRecalibrate-th such render re-times the rows under it when RT_MOVING_ORDER=1; by
    // default (r06) it renders in identity order (moving_order below).  Any order is a permutation of the tile rows:
    // images never depend on it.
    // order_mode (rt_diag_tile_order): 0 adaptive, 1 bottom-to-top.
    int32_t* d_tile_rows = nullptr;            // row order: tile rows by decreasing calibrated time
    uint32_t* d_row_cost = nullptr;            // ... their times (rt_rowsum_kernel)
    int n_tile_rows = 0;                       // capacity of both (kOrderMax, allocated by rt_ctx_create)
    // The view's dispatch table (rt_disp_kernel) and what builds it, per tile (view_cap tiles each): the calibration
    // render's wave times (d_tile_cost) and cone masks (d_cone_tile), and the tile order's radix-sort buffers.
    // order_policy (RT_ORDER_POLICY): 0 tile rows longest first (r01-r04), 1 tiles longest first.
    DispRec* d_disp = nullptr;
    uint32_t* d_tile_cost = nullptr;
    uint32_t* d_sort_keys = nullptr;
    int32_t* d_sort_in = nullptr;
    int32_t* d_sort_out = nullptr;
    void* d_sort_tmp = nullptr;
    size_t sort_tmp_bytes = 0;
    size_t view_cap = 0;
    int order_policy = 0;
    using ViewKey = std::array<unsigned char, sizeof(rt_camera) + 6 * sizeof(int) + sizeof(rt_rows) + sizeof(uint64_t)>;
    bool order_valid = false;                  // d_tile_rows holds the order of view `order_key`
    ViewKey order_key{};
    bool seen_valid = false;                   // `seen_key`: the last view rendered once in identity order
    ViewKey seen_key{};
    int stale = 0;                             // renders of other cameras since the order was calibrated
    // r06: a moving camera renders in identity order (RT_MOVING_ORDER=1: the last calibrated order, re-timed every
    // RT_RECALIBRATE-th render, 8 by default then — the r03-r05 policy).  tools/moving_probe.py, c2 orbit, 3 frames in
    // flight: identity 22.8 us per frame, the static view's order kept 24.2, re-timed every 8th render 26.9 (the
    // re-timing's order kernels stall the context's stream; the static view's row costs are not the orbit's).
    int moving_order = 0;
    int recalibrate = kRecalibrate;
    int order_mode = 0;
    // Primary cone masks of the calibrated view (scenes with >= kPrimaryConeMin spheres): the calibration render
    // writes each tile's mask (d_cone_tile), rt_disp_kernel puts them in the dispatch table, and later renders of
    // exactly that view (order_key) read them instead of recomputing them.  Renders of another camera compute their
    // own.  One-wave (8 x 8 tile) variants only.  Ordering against renders on other streams: view_ev and the reader
    // tracking below.
    uint64_t* d_cone_tile = nullptr;
    bool cone_valid = false;                   // d_disp holds the masks of view order_key
    // r06: the culling kernels' level masks of view order_key, lmask_stride per tile (rt_device.hpp LevelMasks),
    // written by its calibration render (grow-only, lmask_cap masks); RT_LEVEL_MASKS=0: computed in every render
    uint64_t* d_lmask = nullptr;
    size_t lmask_cap = 0;
    int lmask_stride = 0;
    bool lmask_valid = false;
    bool level_masks = true;
    // Cross-stream ordering of the per-view state: the per-eye records inside d_scene (rt_prepare_kernel) and the
    // calibration buffers (d_row_cost, d_tile_rows, d_tile_cost, d_cone_tile, d_disp).  Every render reads the per-eye
    // records; a render that prepares a new eye or calibrates also writes.  A writer records view_ev on its stream
    // after its last write; a render on another stream first waits for view_ev on the GPU (read-after-write,
    // write-after-write).  Renders are tracked by stream: a writer drains the device first when renders were queued
    // on a stream other than its own since the last drain (write-after-read); same-stream renders are ordered by
    // the stream, so one stream per context (the benchmark's layout) never waits or drains.
    hipEvent_t view_ev = nullptr;
    hipStream_t view_st = nullptr;
    bool view_rec = false;                     // view_ev was recorded (on view_st)
    hipStream_t reader_st = nullptr;           // the stream of the renders queued since the last drain ...
    bool readers = false;                      // ... (any)
    bool readers_multi = false;                // ... on more than one stream
    int cone_cache = RT_CONE_CACHE_DEFAULT;    // RT_CONE_CACHE=0: always compute the masks in the kernel (A/B)
    bool achro_off = false;                    // RT_ACHRO_OFF=1: the three-channel kernels for achromatic scenes (A/B)
    uint64_t scene_gen = 0;
    uint64_t scene_hash = 0;                   // FNV-1a of `blob` (rt_ctx_scene_id)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // The host-buffer calls (rt_render, rt_render_packed, rt_render_packed_async) run on the context's own
    // streams: renders on `rs` (blocking w.r.t. the null stream, like the null-stream renders it replaced), the
    // device-to-host copies on `cs`, so an asynchronous frame's copy overlaps the next frame's render.
    hipStream_t rs = nullptr, cs = nullptr;
    // rt_render_packed_async frame t uses slot t % kSlots (device buffer 5 + slot): up to kSlots - 1 frames of
    // latency behind the one being queued
    static constexpr int kSlots = 3;
    hipEvent_t rendered[kSlots] = {};          // slot b's packed frame is in its device buffer
    hipEvent_t copied[kSlots] = {};            // slot b's packed frame is in its host buffer
    bool copied_rec[kSlots] = {};
    bool copied_cs[kSlots] = {};               // ... by a copy on the copy stream (else on the render stream)
    // copy_mode 3: the frame leaves on a copy (SDMA) engine — no CUs taken from the next render.  Per slot, the
    // render stream stores 0 into sd_dep (hipStreamWriteValue64 on the HSA signal's value) once the frame is in its
    // device buffer; the SDMA copies, queued with sd_dep as their dependency, then move it, each decrementing its
    // own completion signal sd_done[slot][half] (one signal per engine copy, initialised to 1).
    bool sd_tried = false, sd_ok = false;
    hsa_agent_t sd_gpu{0}, sd_cpu{0};
    uint32_t sd_engine = 0, sd_engine2 = 0;            // the two lowest free engines (sd_engine2 = 0: only one)
    int sd_split = 2;                                   // RT_SDMA_SPLIT: engines a frame's copy is split over (1, 2)
    hsa_signal_t sd_dep[kSlots] = {}, sd_done[kSlots][2] = {};
    volatile hsa_signal_value_t* sd_dep_ptr[kSlots] = {};
    hipEvent_t sd_fired[kSlots] = {};                   // recorded on rs right after slot b's sdma_fire
    bool sd_pending[kSlots] = {};
    int sd_copies[kSlots] = {};                         // engine copies queued for slot b (1 or 2)
    int sd_writer = 0;                                  // sdma_fire: 1 stream write-value, 2 signal kernel
    int sd_writer_req = 0;                              // RT_SDMA_WRITER (A/B): 1 or 2 forces the writer, 0 tries 2 then 1
    int sd_wait_ms = 5000;                              // RT_SDMA_WAIT_MS: how often sdma_wait re-checks a slow render
    int last_copy_mode = -1;                            // the mode the last packed frame took (rt_diag_copy_path)
    uint64_t ticket = 0;                       // rt_render_packed_async frames queued so far
    // rt_render's device buffers (grow-only, reused across calls): rgba32f, rgba8, rgb64f, raycount, sums,
    // packed slot 0, packed slot 1
    static constexpr int kBufs = 5 + kSlots;
    void* d_out[kBufs] = {};
    size_t out_cap[kBufs] = {};
};

#define RT_HIP(call)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) return rt_fail(RT_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

#if RT_WAVE_TRACE
extern "C" int rt_debug_wave_trace(void* dev_buf) {
    g_wtrace = reinterpret_cast<uint64_t*>(dev_buf);
    return RT_OK;
}
#endif

#if RT_COUNTERS
// Diagnostic build only (tools/counters.py): point the uploaded scene's event counters at `dev_buf`
// (kCntCount uint64 on the context's device); call after rt_set_scene.
extern "C" int rt_debug_counters(rt_ctx* c, void* dev_buf) {
    if (!c || !c->scene_set) return rt_fail(RT_EINVAL, "rt_debug_counters: no scene");
    RT_HIP(hipSetDevice(c->device));
    RT_HIP(hipMemcpy(&c->d_scene->counters, &dev_buf, sizeof(dev_buf), hipMemcpyHostToDevice));
    return RT_OK;
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

// The per-tile view buffers (dispatch table, tile times, cone masks, sort buffers) of a context.
static void rt_free_view_bufs(rt_ctx* c) {
    void* bufs[] = {c->d_disp, c->d_tile_cost, c->d_cone_tile, c->d_sort_keys, c->d_sort_in, c->d_sort_out,
                    c->d_sort_tmp};
    for (void* b : bufs)
        if (b) (void)hipFree(b);
    c->d_disp = nullptr;
    c->d_tile_cost = c->d_sort_keys = nullptr;
    c->d_cone_tile = nullptr;
    c->d_sort_in = c->d_sort_out = nullptr;
    c->d_sort_tmp = nullptr;
    c->sort_tmp_bytes = 0;
    c->view_cap = 0;
}

// ... grown to hold `tiles` tiles (the caller has drained the device: renders may read the old ones).  False (and no
// buffers) when the device is out of memory: the view then keeps the identity order.
static bool rt_grow_view_bufs(rt_ctx* c, size_t tiles) {
    if (tiles <= c->view_cap) return true;
    rt_free_view_bufs(c);
    const size_t slots = cone_slots(tiles);
    bool ok = hipMalloc(&c->d_disp, slots * sizeof(DispRec)) == hipSuccess &&
              hipMalloc(&c->d_tile_cost, tiles * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&c->d_cone_tile, tiles * sizeof(uint64_t)) == hipSuccess &&
              hipMalloc(&c->d_sort_keys, tiles * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&c->d_sort_in, tiles * sizeof(int32_t)) == hipSuccess &&
              hipMalloc(&c->d_sort_out, tiles * sizeof(int32_t)) == hipSuccess;
    if (ok) {
        size_t tmp = 0;
        ok = hipcub::DeviceRadixSort::SortPairsDescending(nullptr, tmp, c->d_tile_cost, c->d_sort_keys, c->d_sort_in,
                                                          c->d_sort_out, (int)tiles) == hipSuccess &&
             hipMalloc(&c->d_sort_tmp, tmp) == hipSuccess;
        c->sort_tmp_bytes = tmp;
    }
    if (!ok) {
        (void)hipGetLastError();
        rt_free_view_bufs(c);
        return false;
    }
    c->view_cap = tiles;
    return true;
}

static int sdma_wait(rt_ctx* c, int b);   // below, with the SDMA path

extern "C" int rt_ctx_destroy(rt_ctx* c) {
    if (!c) return RT_OK;
    (void)hipSetDevice(c->device);
    rt_screen_release(c);
    if (c->rs) (void)hipStreamSynchronize(c->rs);
    if (c->cs) (void)hipStreamSynchronize(c->cs);
    if (c->d_scene) (void)hipFree(c->d_scene);
    if (c->d_tile_rows) (void)hipFree(c->d_tile_rows);
    if (c->d_row_cost) (void)hipFree(c->d_row_cost);
    rt_free_view_bufs(c);
    if (c->d_lmask) (void)hipFree(c->d_lmask);
    if (c->sd_ok) {
        for (int b = 0; b < rt_ctx::kSlots; ++b) {
            (void)sdma_wait(c, b);                     // (the render stream has drained: its signal has fired)
            hsa_signal_destroy(c->sd_dep[b]);
            hsa_signal_destroy(c->sd_done[b][0]);
            hsa_signal_destroy(c->sd_done[b][1]);
            (void)hipEventDestroy(c->sd_fired[b]);
        }
        hsa_shut_down();
    }
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->view_ev) (void)hipEventDestroy(c->view_ev);
    for (int b = 0; b < rt_ctx::kSlots; ++b) {
        if (c->rendered[b]) (void)hipEventDestroy(c->rendered[b]);
        if (c->copied[b]) (void)hipEventDestroy(c->copied[b]);
    }
    if (c->rs) (void)hipStreamDestroy(c->rs);
    if (c->cs) (void)hipStreamDestroy(c->cs);
    for (void* p : c->d_out)
        if (p) (void)hipFree(p);
    delete c;
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
    if (const char* e = getenv("RT_COPY_MODE")) c->copy_mode = std::min(std::max(atoi(e), -1), 3);
    if (const char* e = getenv("RT_SDMA_SPLIT")) c->sd_split = std::min(std::max(atoi(e), 1), 2);
    if (const char* e = getenv("RT_SDMA_WRITER")) c->sd_writer_req = std::min(std::max(atoi(e), 0), 2);
    if (const char* e = getenv("RT_SDMA_WAIT_MS")) c->sd_wait_ms = std::max(atoi(e), 0);
    if (const char* e = getenv("RT_MOVING_ORDER")) c->moving_order = atoi(e) != 0;
    if (const char* e = getenv("RT_RECALIBRATE")) c->recalibrate = std::max(atoi(e), 0);
    if (const char* e = getenv("RT_COPY_BLOCKS")) c->copy_blocks = std::max(atoi(e), 0);
    if (const char* e = getenv("RT_COPY_KERNEL")) c->copy_kernel = std::min(std::max(atoi(e), -1), 1);
    if (const char* e = getenv("RT_CONE_CACHE")) c->cone_cache = atoi(e) != 0;
    if (const char* e = getenv("RT_LEVEL_MASKS")) c->level_masks = atoi(e) != 0;
    if (const char* e = getenv("RT_ORDER_POLICY")) c->order_policy = std::min(std::max(atoi(e), 0), 1);
    if (const char* e = getenv("RT_ACHRO_OFF")) c->achro_off = atoi(e) != 0;
    if (hipMalloc(&c->d_tile_rows, sizeof(int32_t) * kOrderMax) != hipSuccess ||
        hipMalloc(&c->d_row_cost, sizeof(uint32_t) * kOrderMax) != hipSuccess) {
        rt_ctx_destroy(c);
        return rt_fail(RT_ENOMEM, "rt_ctx_create: hipMalloc of the tile-row order failed");
    }
    c->n_tile_rows = kOrderMax;
    bool ok = hipMemset(c->d_tile_rows, 0, sizeof(int32_t) * kOrderMax) == hipSuccess &&
              hipEventCreate(&c->ev0) == hipSuccess && hipEventCreate(&c->ev1) == hipSuccess &&
              hipEventCreateWithFlags(&c->view_ev, hipEventDisableTiming) == hipSuccess &&
              hipStreamCreateWithFlags(&c->rs, hipStreamDefault) == hipSuccess &&
              hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking) == hipSuccess;
    for (int b = 0; b < rt_ctx::kSlots && ok; ++b)
        ok = hipEventCreateWithFlags(&c->rendered[b], hipEventDisableTiming) == hipSuccess &&
             hipEventCreateWithFlags(&c->copied[b], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        rt_ctx_destroy(c);
        return rt_fail(RT_EHIP, "rt_ctx_create: stream/event creation failed");
    }
    *out = c;
    return RT_OK;
}

int rt_ctx_device(const rt_ctx* c) { return c ? c->device : -1; }

int rt_ctx_achromatic(const rt_ctx* c) { return c && c->scene_set && c->achromatic ? 1 : 0; }

void rt_ctx_scene_id(const rt_ctx* c, uint64_t* gen, uint64_t* fingerprint) {
    *gen = c && c->scene_set ? c->scene_gen : 0;
    *fingerprint = c && c->scene_set ? c->scene_hash : 0;
}

extern "C" int rt_set_scene(rt_ctx* c, const rt_scene* scene) {
    if (!c) return rt_fail(RT_EINVAL, "rt_set_scene: null context");
    std::vector<unsigned char> blob;
    int rc = rt_build_dev_scene(scene, &blob);
    if (rc) return rc;
    // An unchanged scene (same flattened record, byte for byte) keeps the device copy, the per-eye data
    // and the tile-row order: rt_render calls this every frame.
    if (c->scene_set && blob == c->blob) return RT_OK;
    int achromatic = 0;
    rc = rt_scene_achromatic(scene, &achromatic);
    if (rc) return rc;
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
    c->n_stride = h->n_stride;
    c->n_lights = h->n_lights;
    c->transparent = h->transparent != 0 || h->n_meshes > 0;   // FULL kernel variants
    c->tree = h->tree != 0;
    c->achromatic = achromatic != 0;
    c->eye_valid = false;
    c->scene_set = true;
    c->blob.swap(blob);
    c->scene_hash = rt_blob_fingerprint(c->blob);
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
    P->ns = c->n_stride;
    P->nl = c->n_lights;
    P->wg_staging = c->wg_staging;
#if RT_WAVE_TRACE
    P->wtrace = g_wtrace;
#endif
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

static bool float_format(int f) { return f == RT_PIXEL_RGBA32F || f == RT_PIXEL_GRAY32F; }
static bool byte_format(int f) { return f == RT_PIXEL_RGBA8 || f == RT_PIXEL_RGB8 || f == RT_PIXEL_GRAY8; }

// The device render behind rt_render_dev / rt_render_dev_packed: the float image (fmt_f) and the byte image
// (fmt_8) in their formats, the FP64 colour and the ray counters, each nullable.
static int render_dev_impl(rt_ctx* c, const rt_camera* cam, int W, int H, int depth, const rt_rows* rows,
                           int fmt_f, void* pf, int fmt_8, void* p8, double* rgb64f, uint32_t* raycount,
                           void* stream) {
    RenderParams P;
    int rc = render_params(c, cam, W, H, depth, rows, &P);
    if (rc) return rc;
    if ((pf && !float_format(fmt_f)) || (p8 && !byte_format(fmt_8)))
        return rt_fail(RT_EINVAL, "render: bad pixel format for the float / byte image");
    if (((pf && fmt_f == RT_PIXEL_GRAY32F) || (p8 && fmt_8 == RT_PIXEL_GRAY8)) && !c->achromatic)
        return rt_fail(RT_EINVAL, "render: GRAY pixel formats need an achromatic scene (rt_scene_achromatic)");
    P.fmt_f = fmt_f == RT_PIXEL_GRAY32F ? kFmtF_GRAY : kFmtF_RGBA;
    P.fmt_8 = fmt_8 == RT_PIXEL_GRAY8 ? kFmt8_GRAY : fmt_8 == RT_PIXEL_RGB8 ? kFmt8_RGB : kFmt8_RGBA;
    const bool packed = (pf && P.fmt_f != kFmtF_RGBA) || (p8 && P.fmt_8 != kFmt8_RGBA);
    if (packed) P.wg_staging = 0;                   // the LDS-staged stores (A/B variant) write RGBA only
    if (P.local_rows == 0) return RT_OK;
    RT_HIP(hipSetDevice(c->device));
    // One-wave workgroups (8 x 8 tiles) by default: measured faster than 256-thread workgroups (32 x 8
    // tiles) at every config (c2 -1%, c3 -3%, c5 -12%: a finished wave's slot is refilled without
    // waiting for three siblings).  The A/B variants that share a workgroup-wide LDS copy (scene in LDS,
    // staged row stores) keep 256 threads.
    const bool big = !packed && (c->use_lds || c->wg_staging);    // packed formats: one-wave variants only
    const int tw = big ? kTileW : RT_WG_FAST / 8;
    const int tiles_x = (W + tw - 1) / tw;
    const int tiles_y = (P.local_rows + kTileH - 1) / kTileH;
    P.tile_rows_n = tiles_y;
    P.tiles_x = tiles_x;
    hipStream_t st = (hipStream_t)stream;
    // A render captured into a hipGraph must be self-contained: it always prepares its eye's data and uses
    // the identity tile-row order (the context's order buffer belongs to whatever view it last calibrated).
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    RT_HIP(hipStreamIsCapturing(st, &cap));
    const bool capturing = cap != hipStreamCaptureStatusNone;
    if (capturing) c->ever_captured = true;
    bool calibrate = false, cone_calib = false, lm_calib = false;
    // level masks per tile (opaque scenes, one-wave tiles): B ray masks + (B + 1) nl shadow masks.  The culling
    // kernels compute them in their calibration render; for the fast kernels' scenes (< kConeMin spheres) a culling
    // kernel writes them in a launch of its own right after the calibration render (no image outputs), and later
    // renders skip the filter batches they rule out
    const bool opaque_tiles = !c->tree && !c->transparent && !big && RT_WG_FAST == 64;
    const bool cull_kernel = c->n_padded >= kConeMin && opaque_tiles;
    int lm_stride = opaque_tiles && c->level_masks && c->cone_cache ? depth + (depth + 1) * c->n_lights : 0;
    if (lm_stride > kLevelMaskSlotsMax) lm_stride = 0;
    rt_ctx::ViewKey key{};
    // (dispatch records pack the tile as ty << 16 | tx)
    if (!capturing && c->order_mode == 0 && tiles_y <= c->n_tile_rows && tiles_x < 65536 && tiles_y < 65536) {
        // Key of the frame's work: camera, size, outputs, row plan, depth and scene generation.
        unsigned char* kp = key.data();                 // fixed size: no host allocation per render
        memcpy(kp, cam, sizeof(rt_camera)); kp += sizeof(rt_camera);
        // which outputs are written (and in which format) changes the rows' relative cost (an RGB64F parity
        // render writes 24 B per pixel): each output set gets its own calibration
        const int outs = (pf ? 1 : 0) | (p8 ? 2 : 0) | (rgb64f ? 4 : 0) | (raycount ? 8 : 0) | (P.fmt_f << 4) |
                         (P.fmt_8 << 6);
        const int ints[6] = {W, H, depth, tiles_x, tiles_y, outs};
        memcpy(kp, ints, sizeof(ints)); kp += sizeof(ints);
        if (rows) memcpy(kp, rows, sizeof(rt_rows));
        kp += sizeof(rt_rows);
        memcpy(kp, &c->scene_gen, sizeof(uint64_t));
        constexpr size_t kCam = sizeof(rt_camera);
        const bool same_shape = c->order_valid &&
                                memcmp(key.data() + kCam, c->order_key.data() + kCam, key.size() - kCam) == 0;
        if (c->order_valid && key == c->order_key) {
            P.disp = c->d_disp;
            // (the cached masks hold one mask per one-wave 8 x 8 tile: the 256-thread A/B variants never read them)
            P.cone_use = c->cone_valid && !big ? 1 : 0;
            if (c->lmask_valid && lm_stride > 0 && c->lmask_stride == lm_stride) {   // this view's level masks
                P.lmask_in = c->d_lmask;
                P.lmask_stride = lm_stride;
            }
        } else if (same_shape && c->moving_order) {
            P.disp = c->d_disp;                         // another camera: the last calibrated order, its own masks
            if (c->recalibrate > 0 && ++c->stale >= c->recalibrate) {   // ... re-timed every recalibrate-th render
                calibrate = true;
                c->order_valid = false;
            }
        } else if (c->seen_valid && key == c->seen_key) {   // (by default a moving camera's views come here: the
                                                            // first render of a view in identity order, its second
                                                            // the calibration — a camera that stops is calibrated)
            calibrate = true;                           // calibration render (identity order)
            c->order_valid = false;                     // rt_disp_kernel rewrites d_disp below
            // the calibration records one mask per tile from lane 0 of its wave: one-wave workgroups only
            cone_calib = c->cone_cache && c->n_padded >= kPrimaryConeMin && !c->tree && !c->transparent && !big &&
                         RT_WG_FAST == 64;
            lm_calib = cone_calib && lm_stride > 0;
        } else {
            c->seen_key = key;                          // first render of this view: identity order
            c->seen_valid = true;
        }
    }
    const bool prepare = capturing || c->ever_captured || !c->eye_valid || memcmp(c->eye, cam->eye, sizeof(c->eye)) != 0;
    const size_t tiles = (size_t)tiles_x * tiles_y;
    if (!capturing) {                                   // (a captured render carries its own prepare launch)
        // read-after-write / write-after-write: the last write of the view state was queued on another stream
        if (c->view_rec && c->view_st != st) RT_HIP(hipStreamWaitEvent(st, c->view_ev, 0));
        if (prepare || calibrate) {
            // write-after-read: renders queued on other streams may still read what this render rewrites (or frees)
            if ((c->readers && (c->readers_multi || c->reader_st != st)) || (calibrate && tiles > c->view_cap) ||
                (lm_calib && tiles * (size_t)lm_stride > c->lmask_cap))
                RT_HIP(hipDeviceSynchronize());
            c->readers = c->readers_multi = false;      // same-stream renders are ordered before the rewrite
        }
        if (!c->readers) {                              // this render reads the view state on st
            c->readers = true;
            c->reader_st = st;
        } else if (c->reader_st != st) {
            c->readers_multi = true;
        }
    }
    if (calibrate) {
        // the calibration render writes every tile's wave time (and, a static view's, its cone mask); the buffers
        // grow here (the device was drained above)
        c->cone_valid = false;
        c->lmask_valid = false;
        if (!rt_grow_view_bufs(c, tiles)) {             // out of memory: identity order, masks in the kernel
            calibrate = cone_calib = lm_calib = false;
            P.disp = nullptr;
            P.cone_use = 0;
        } else {
            P.tile_cost = c->d_tile_cost;
            if (cone_calib) P.cone_out = c->d_cone_tile;
        }
        if (lm_calib && tiles * (size_t)lm_stride > c->lmask_cap) {     // (the device was drained above)
            if (c->d_lmask) (void)hipFree(c->d_lmask);
            c->d_lmask = nullptr;
            c->lmask_cap = 0;
            if (hipMalloc(&c->d_lmask, tiles * (size_t)lm_stride * sizeof(uint64_t)) == hipSuccess)
                c->lmask_cap = tiles * (size_t)lm_stride;
            else
                (void)hipGetLastError();                // out of memory: the masks stay in the kernel
        }
        if (lm_calib && c->d_lmask) {
            if (cull_kernel) {                          // (fast scenes: the mask launch below writes them)
                P.lmask_out = c->d_lmask;
                P.lmask_stride = lm_stride;
            }
        } else {
            lm_calib = false;
        }
    }
    const dim3 grid((unsigned)tiles_x, (unsigned)std::min(tiles_y, kGridY), (unsigned)((tiles_y + kGridY - 1) / kGridY));
    hipError_t e;
    // Primary-ray sphere data for this eye (stream-ordered; only when the eye changes, or always once graphs
    // that carry their own prepare launch exist).
    if (prepare) {
        c->eye_valid = false;
        dim3 pg((unsigned)((std::max(c->n_padded, 1) + kThreads - 1) / kThreads));
        hipLaunchKernelGGL(rt_prepare_kernel, pg, dim3(kThreads), 0, st, c->d_scene, cam->eye[0], cam->eye[1],
                           cam->eye[2]);
        e = hipGetLastError();
        if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_prepare_kernel: ") + hipGetErrorString(e));
        memcpy(c->eye, cam->eye, sizeof(c->eye));
        c->eye_valid = true;
    }
    RenderLaunch L;
    // achromatic opaque scenes: the one-channel instances (rt_device.hpp shade ACHRO; RT_ACHRO_OFF=1 for A/B)
    L.achro = c->achromatic && !c->transparent && !c->tree && !c->achro_off;
    L.grid = grid;
    L.stream = st;
    L.scene = c->d_scene;
    L.P = P;
    L.o32 = pf;
    L.o8 = p8;
    L.o64 = rgb64f;
    L.orc = raycount;
    const bool cull = c->n_padded >= kConeMin, mw5 = c->min_waves >= 5 && depth <= 3;
    if (c->tree) {
        L.variant = kVarTree;
        L.lds = 0;
    } else if (c->transparent) {
        L.variant = kVarTransp;
        L.lds = slot_bytes(depth, true, 64);
    } else if (c->use_lds) {
        L.variant = kVarLds;
        L.lds = c->lds_bytes + slot_bytes(depth, false);
    } else if (c->wg_staging) {
        L.variant = mw5 ? kVarStaging : kVarStagingAnyW;
        L.lds = 4096 + 6144 + 1024 + 1024 + slot_bytes(depth, false);
    } else {
        // >= kConeMin spheres: the wave-culling variant (secondary and shadow rays, rt_device.hpp CULL).
        L.variant = cull ? (mw5 ? kVarCull : kVarCullAnyW) : (mw5 ? kVarFast : kVarFastAnyW);
        L.lds = slot_bytes(depth, false, RT_WG_FAST, cull);
    }
    if (packed) {                                       // the instances with runtime pixel-format stores
        if (c->tree) L.variant = kVarTreePacked;
        else if (c->transparent) L.variant = kVarTranspPacked;
        else L.variant = cull ? kVarCullPacked : kVarFastPacked;
        if (!c->tree && !c->transparent) L.lds = slot_bytes(depth, false, RT_WG_FAST, cull);
    }
    switch (depth) {
        case 0: e = launch_render<0>(L); break;
        case 1: e = launch_render<1>(L); break;
        case 2: e = launch_render<2>(L); break;
        case 3: e = launch_render<3>(L); break;
        case 4: e = launch_render<4>(L); break;
        case 5: e = launch_render<5>(L); break;
        case 6: e = launch_render<6>(L); break;
        default: e = launch_render<7>(L); break;
    }
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_render_kernel launch: ") + hipGetErrorString(e));
    if (lm_calib && !cull_kernel) {
        // a fast kernel's scene: the level masks of the view from a culling kernel that stores nothing else (identity
        // order, its own primary cone masks, no image) — stream-ordered before the renders that read them
        RenderLaunch M = L;
        M.P.lmask_out = c->d_lmask;
        M.P.lmask_in = nullptr;
        M.P.lmask_stride = lm_stride;
        M.P.disp = nullptr;
        M.P.cone_use = 0;
        M.P.cone_out = nullptr;
        M.P.tile_cost = nullptr;
        M.o32 = M.o8 = nullptr;
        M.o64 = nullptr;
        M.orc = nullptr;
        M.variant = mw5 ? kVarCull : kVarCullAnyW;
        M.lds = slot_bytes(depth, false, RT_WG_FAST, true);
        switch (depth) {
            case 0: e = launch_render<0>(M); break;
            case 1: e = launch_render<1>(M); break;
            case 2: e = launch_render<2>(M); break;
            case 3: e = launch_render<3>(M); break;
            case 4: e = launch_render<4>(M); break;
            case 5: e = launch_render<5>(M); break;
            case 6: e = launch_render<6>(M); break;
            default: e = launch_render<7>(M); break;
        }
        if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("level-mask launch: ") + hipGetErrorString(e));
    }
    if (calibrate) {
        // the dispatch table of this view (stream-ordered after the calibration render, which wrote the tile times)
        const dim3 tg((unsigned)((tiles + 255) / 256));
        const uint64_t* cones = cone_calib ? c->d_cone_tile : nullptr;
        if (c->order_policy == 1) {                     // tiles longest first
            hipLaunchKernelGGL(rt_iota_kernel, tg, dim3(256), 0, st, c->d_sort_in, (int)tiles);
            size_t tmp = c->sort_tmp_bytes;
            e = hipcub::DeviceRadixSort::SortPairsDescending(c->d_sort_tmp, tmp, c->d_tile_cost, c->d_sort_keys,
                                                             c->d_sort_in, c->d_sort_out, (int)tiles, 0, 32, st);
            if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("tile order sort: ") + hipGetErrorString(e));
            hipLaunchKernelGGL(rt_disp_kernel, tg, dim3(256), 0, st, nullptr, c->d_sort_out, cones, tiles_x, tiles_y,
                               c->d_disp);
        } else {                                        // tile rows longest first
            hipLaunchKernelGGL(rt_rowsum_kernel, dim3((unsigned)tiles_y), dim3(256), 0, st, c->d_tile_cost, tiles_x,
                               c->d_row_cost);
            hipLaunchKernelGGL(rt_order_kernel, dim3(1), dim3(1024), 0, st, c->d_row_cost, tiles_y, c->d_tile_rows);
            hipLaunchKernelGGL(rt_disp_kernel, tg, dim3(256), 0, st, c->d_tile_rows, nullptr, cones, tiles_x, tiles_y,
                               c->d_disp);
        }
        e = hipGetLastError();
        if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("dispatch table: ") + hipGetErrorString(e));
        c->order_key = key;                             // only once the order kernel is queued
        c->order_valid = true;
        c->cone_valid = cone_calib;
        c->lmask_valid = lm_calib;
        c->lmask_stride = lm_calib ? lm_stride : 0;
        c->stale = 0;
    }
    if ((prepare || calibrate) && !capturing) {
        RT_HIP(hipEventRecord(c->view_ev, st));         // later renders on other streams wait for these writes
        c->view_st = st;
        c->view_rec = true;
    }
    return RT_OK;
}

extern "C" int rt_render_dev(rt_ctx* c, const rt_camera* cam, int W, int H, int depth, const rt_rows* rows,
                             float* rgba32f, uint8_t* rgba8, double* rgb64f, uint32_t* raycount, void* stream) {
    return render_dev_impl(c, cam, W, H, depth, rows, RT_PIXEL_RGBA32F, rgba32f, RT_PIXEL_RGBA8, rgba8, rgb64f,
                           raycount, stream);
}

extern "C" int rt_render_dev_packed(rt_ctx* c, const rt_camera* cam, int W, int H, int depth, const rt_rows* rows,
                                    int float_format, void* float_pixels, int byte_format, void* byte_pixels,
                                    void* stream) {
    return render_dev_impl(c, cam, W, H, depth, rows, float_format, float_pixels, byte_format, byte_pixels, nullptr,
                           nullptr, stream);
}

// Grow-only device buffer k of the context (rt_render's outputs).
static int ctx_buffer(rt_ctx* c, int k, size_t bytes, void** out) {
    if (bytes > c->out_cap[k]) {
        // the buffer may still be read by a copy (or written by a render) queued on the context's streams
        RT_HIP(hipStreamSynchronize(c->rs));
        RT_HIP(hipStreamSynchronize(c->cs));
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

// Ray statistics of a render with per-pixel counters d_rc (npx pixels) into *stats (the stream must be done).
static int read_stats(rt_ctx* c, size_t npx, const unsigned long long* d_sums, rt_stats* stats) {
    unsigned long long sums[2] = {0, 0};
    if (npx) RT_HIP(hipMemcpy(sums, d_sums, sizeof(sums), hipMemcpyDeviceToHost));
    stats->primary_rays = npx;
    stats->reflect_rays = sums[0] - npx;
    stats->shadow_rays = sums[1];
    float ms = 0.f;
    if (npx) RT_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    stats->kernel_ms = ms;
    return RT_OK;
}

// rt_host_alloc's pinned allocations (host base -> size, device mapping): host frames that land in one are
// copied by rt_copy_out_kernel, everything else by hipMemcpyAsync (pageable memory is staged by HIP).
static std::mutex g_pinned_mu;
static std::map<uintptr_t, std::pair<size_t, uintptr_t>> g_pinned;

static void* pinned_device_ptr(const void* host, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_pinned_mu);
    const uintptr_t h = (uintptr_t)host;
    auto it = g_pinned.upper_bound(h);
    if (it == g_pinned.begin()) return nullptr;
    --it;
    if (h + bytes > it->first + it->second.first) return nullptr;
    return (void*)(it->second.second + (h - it->first));
}

// The device address of any page-locked host buffer (rt_host_alloc's, or one the caller pinned elsewhere, e.g. a
// torch pin_memory() tensor): the runtime's pointer attributes; nullptr for pageable memory.
static void* host_device_ptr(const void* host, size_t bytes) {
    if (void* d = pinned_device_ptr(host, bytes)) return d;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, host) != hipSuccess) {
        (void)hipGetLastError();                                     // pageable: not an error of this call
        return nullptr;
    }
    return a.type == hipMemoryTypeHost ? a.devicePointer : nullptr;
}

constexpr unsigned kCopyStreamBlocks = 16;     // copy kernel beside a render: workgroups (rt_ctx::copy_mode)

// A copy kernel into rt_host_alloc memory (else hipMemcpyAsync); max_blocks: its workgroups (0: one per 4 KB, up to
// 1024).  RT_COPY_KERNEL / RT_COPY_BLOCKS override.
static int copy_to_host(rt_ctx* c, void* host, const void* dev, size_t bytes, hipStream_t st, unsigned max_blocks = 0) {
    if (!bytes) return RT_OK;
    void* dmap = host_device_ptr(host, bytes);
    const bool kernel = c->copy_kernel != 0;
    if (dmap && kernel && ((uintptr_t)dmap | (uintptr_t)dev) % 16 == 0) {
        unsigned blocks = (unsigned)std::min<size_t>((bytes / 16 + kThreads - 1) / kThreads + 1, 1024);
        if (c->copy_blocks > 0) max_blocks = (unsigned)c->copy_blocks;
        if (max_blocks > 0) blocks = std::min(blocks, max_blocks);
        hipLaunchKernelGGL(rt_copy_out_kernel, dim3(blocks), dim3(kThreads), 0, st, (const uint8_t*)dev,
                           (uint8_t*)dmap, bytes);
        RT_HIP(hipGetLastError());
        return RT_OK;
    }
    RT_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, st));
    return RT_OK;
}

static int queue_raysum(rt_ctx* c, size_t npx, uint32_t* d_rc, unsigned long long* d_sums) {
    RT_HIP(hipMemsetAsync(d_sums, 0, 2 * sizeof(unsigned long long), c->rs));
    hipLaunchKernelGGL(rt_raysum_kernel, dim3((unsigned)std::min<size_t>((npx + kThreads - 1) / kThreads, 1024)),
                       dim3(kThreads), 0, c->rs, (const uint32_t*)d_rc, npx, d_sums);
    RT_HIP(hipGetLastError());
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
    RT_HIP(hipEventRecord(c->ev0, c->rs));
    rc = rt_render_dev(c, cam, W, H, depth, rows, (float*)d[0], (uint8_t*)d[1], (double*)d[2], (uint32_t*)d[3], c->rs);
    if (rc) return rc;
    RT_HIP(hipEventRecord(c->ev1, c->rs));
    if (stats && npx > 0 && (rc = queue_raysum(c, npx, (uint32_t*)d[3], (unsigned long long*)d[4]))) return rc;
    // asynchronous copies on the render stream (rt_host_alloc memory: a copy kernel; other memory: hipMemcpyAsync),
    // one synchronisation of that stream (not of the device: other streams' work is not waited for)
    void* host[3] = {rgba32f, rgba8, rgb64f};
    for (int k = 0; k < 3; ++k)
        if (host[k] && npx && (rc = copy_to_host(c, host[k], d[k], bytes[k], c->rs))) return rc;
    RT_HIP(hipStreamSynchronize(c->rs));
    if (stats) return read_stats(c, npx, (const unsigned long long*)d[4], stats);
    return RT_OK;
}

// ---- copy_mode 3: device-to-host frames on an SDMA engine (HSA runtime, hsa_amd_memory_async_copy_on_engine) ----
struct SdmaAgents {
    uint32_t domain = 0, bdf = 0;
    hsa_agent_t gpu{0}, cpu{0};
};
static hsa_status_t sdma_find_agent(hsa_agent_t a, void* data) {
    SdmaAgents* f = static_cast<SdmaAgents*>(data);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && f->cpu.handle == 0) f->cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU) {
        uint32_t dom = 0, bdf = 0;
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
        hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
        if (dom == f->domain && bdf == f->bdf) f->gpu = a;
    }
    return HSA_STATUS_SUCCESS;
}

__global__ void __launch_bounds__(64) rt_signal_fire_kernel(int64_t* value) {
    if (threadIdx.x == 0) __hip_atomic_store(value, (int64_t)0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Queue "slot b's frame is in its device buffer" on the render stream: store 0 into sd_dep[b] (writer 1: the
// stream's write-value operation, 2: a one-wave kernel behind the render).
static hipError_t sdma_fire(rt_ctx* c, int b, int writer) {
    if (writer == 1) return hipStreamWriteValue64(c->rs, (void*)c->sd_dep_ptr[b], 0, 0);
    hipLaunchKernelGGL(rt_signal_fire_kernel, dim3(1), dim3(64), 0, c->rs, (int64_t*)c->sd_dep_ptr[b]);
    return hipGetLastError();
}

// The context's GPU agent (matched to its HIP device by PCI domain / bus / device / function), a CPU agent, a free SDMA
// engine between them and the per-slot signals; false (once, remembered) when any of it is missing.
static bool sdma_init(rt_ctx* c) {
    if (c->sd_tried) return c->sd_ok;
    c->sd_tried = true;
    char bus[64] = {};
    unsigned dom = 0, b = 0, d = 0, f = 0;
    if (hipDeviceGetPCIBusId(bus, sizeof bus, c->device) != hipSuccess ||
        sscanf(bus, "%x:%x:%x.%x", &dom, &b, &d, &f) != 4 || hsa_init() != HSA_STATUS_SUCCESS)
        return false;
    SdmaAgents ag;
    ag.domain = dom;
    ag.bdf = (b << 8) | (d << 3) | f;
    uint32_t mask = 0;
    if (hsa_iterate_agents(sdma_find_agent, &ag) != HSA_STATUS_SUCCESS || !ag.gpu.handle || !ag.cpu.handle ||
        hsa_amd_memory_copy_engine_status(ag.cpu, ag.gpu, &mask) != HSA_STATUS_SUCCESS || mask == 0) {
        hsa_shut_down();
        return false;
    }
    // sd_dep is waited on by the copy engine only (GPU_ONLY: the one kind whose value a stream or kernel may store)
    bool ok = true;
    for (int k = 0; k < rt_ctx::kSlots && ok; ++k)
        ok = hsa_amd_signal_create(1, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &c->sd_dep[k]) == HSA_STATUS_SUCCESS &&
             hsa_signal_create(0, 0, nullptr, &c->sd_done[k][0]) == HSA_STATUS_SUCCESS &&
             hsa_signal_create(0, 0, nullptr, &c->sd_done[k][1]) == HSA_STATUS_SUCCESS &&
             hsa_amd_signal_value_pointer(c->sd_dep[k], &c->sd_dep_ptr[k]) == HSA_STATUS_SUCCESS &&
             hipEventCreateWithFlags(&c->sd_fired[k], hipEventDisableTiming) == hipSuccess;
    // how the render stream fires it: a one-wave kernel's system-scope store, else the stream's own write
    // (hipStreamWriteValue64); each is tried once on slot 0's signal and must be seen from the host.  (r06: the kernel
    // first — the same speed, profiles/r06/ab/copy_ab_sdma_writer.json — and a plain store into memory the HSA runtime
    // allocated, where the write-value hands the runtime a pointer it did not allocate.)
    if (ok) {
        c->sd_writer = 0;
        for (int w : {2, 1}) {
            if (c->sd_writer) break;
            if (c->sd_writer_req && w != c->sd_writer_req) continue;
            hsa_signal_store_screlease(c->sd_dep[0], 1);
            if (sdma_fire(c, 0, w) == hipSuccess && hipStreamSynchronize(c->rs) == hipSuccess &&
                hsa_signal_load_scacquire(c->sd_dep[0]) == 0)
                c->sd_writer = w;
            (void)hipGetLastError();
        }
        ok = c->sd_writer != 0;
    }
    if (!ok) {
        for (int k = 0; k < rt_ctx::kSlots; ++k) {
            if (c->sd_dep[k].handle) hsa_signal_destroy(c->sd_dep[k]);
            for (int h = 0; h < 2; ++h)
                if (c->sd_done[k][h].handle) hsa_signal_destroy(c->sd_done[k][h]);
            if (c->sd_fired[k]) (void)hipEventDestroy(c->sd_fired[k]);
            c->sd_fired[k] = nullptr;
        }
        hsa_shut_down();
        return false;
    }
    c->sd_gpu = ag.gpu;
    c->sd_cpu = ag.cpu;
    c->sd_engine = mask & (~mask + 1);                 // the lowest free engine
    const uint32_t rest = mask & ~c->sd_engine;
    c->sd_engine2 = rest & (~rest + 1);                 // and the next (0: none)
    c->sd_ok = true;
    return true;
}

// Wait until slot b's SDMA copies are done.  Elapsed time alone is not a failure: a deep frame may still be queued
// behind others on the render stream.  Every sd_wait_ms the render stream's progress is checked (sd_fired, recorded
// right after the frame's sdma_fire): while that event is pending the render is running, and once it has completed the
// dependency has fired and the engines finish the copy — both keep waiting.  Only a render stream that reports an
// error (its write never comes) has its dependency released by hand, so the engines are not left waiting; the stream
// is then drained before the slot is reused, so no stale write of this frame can release a later frame's copy early.
static int sdma_wait(rt_ctx* c, int b) {
    if (!c->sd_pending[b]) return RT_OK;
    // (the wait's timeout is a hint in timestamp ticks and may return early: the deadline is kept here)
    uint64_t freq = 0;
    if (hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &freq) != HSA_STATUS_SUCCESS || freq == 0) freq = 1000000000;
    const auto period = std::chrono::milliseconds(c->sd_wait_ms);
    auto done_by = [&](std::chrono::steady_clock::time_point deadline) {
        for (int h = 0; h < c->sd_copies[b]; ++h) {
            hsa_signal_value_t v = 1;
            for (;;) {
                // the wait's hint: at most 100 ms and no later than the deadline (0 at RT_SDMA_WAIT_MS=0: a poll)
                const auto left = std::chrono::duration_cast<std::chrono::nanoseconds>(
                    deadline - std::chrono::steady_clock::now()).count();
                const uint64_t hint = left <= 0 ? 0 : std::min<uint64_t>(freq / 10, (uint64_t)((double)left * 1e-9 * freq));
                v = hsa_signal_wait_scacquire(c->sd_done[b][h], HSA_SIGNAL_CONDITION_LT, 1, hint, HSA_WAIT_STATE_BLOCKED);
                if (v < 1 || std::chrono::steady_clock::now() >= deadline) break;
            }
            if (v >= 1) return false;
        }
        return true;
    };
    hipError_t q = hipSuccess;
    for (;;) {
        if (done_by(std::chrono::steady_clock::now() + period)) {
            c->sd_pending[b] = false;
            return RT_OK;
        }
        q = hipEventQuery(c->sd_fired[b]);
        if (q != hipSuccess && q != hipErrorNotReady) break;       // the render stream failed
    }
    (void)hipGetLastError();
    hsa_signal_store_screlease(c->sd_dep[b], 0);
    for (int h = 0; h < c->sd_copies[b]; ++h)
        hsa_signal_wait_scacquire(c->sd_done[b][h], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    (void)hipStreamSynchronize(c->rs);
    (void)hipGetLastError();
    c->sd_pending[b] = false;
    return rt_fail(RT_EHIP, std::string("rt_render_packed: the frame's render failed before its SDMA copy: ") +
                                hipGetErrorString(q));
}

// rt_render_packed / rt_render_packed_async: one image in `format`, copied to host memory.
// async: the copy goes to an SDMA engine (or, for pageable memory, the copy kernel on the copy stream; pipelined frames:
// it runs beside the next render), else behind the render on the render stream (see rt_ctx::copy_mode).
static int render_packed_queue(rt_ctx* c, const rt_scene* scene, const rt_camera* cam, int W, int H, int depth,
                               int format, void* host, int slot, bool with_stats, size_t* npx_out, void** sums,
                               bool async) {
    if (!c) return rt_fail(RT_EINVAL, "rt_render_packed: null context");
    if (!host) return rt_fail(RT_EINVAL, "rt_render_packed: null host buffer");
    int pb = 0;
    int rc = rt_pixel_bytes(format, &pb);
    if (rc) return rc;
    rc = rt_set_scene(c, scene);
    if (rc) return rc;
    RenderParams P;
    rc = render_params(c, cam, W, H, depth, nullptr, &P);
    if (rc) return rc;
    RT_HIP(hipSetDevice(c->device));
    const size_t npx = (size_t)W * H;
    *npx_out = npx;
    void* px = nullptr;
    void* rcb = nullptr;
    // RT_COPY_MODE=2 (A/B): the kernel stores the frame straight into the pinned host buffer (mapped into the
    // device's address space), no device buffer and no copy; 3: an SDMA engine copies it (rt_ctx sd_*)
    int mode = c->copy_mode >= 0 ? c->copy_mode : (async ? 3 : 1);
    // (the engine needs page-locked host memory: pageable buffers take the copy-kernel / hipMemcpyAsync path; it is
    // given the buffer's device-side address, which for memory registered after allocation may differ from `host`)
    void* const hdev = mode == 3 ? host_device_ptr(host, npx * pb) : nullptr;
    if (mode == 3 && (!hdev || !sdma_init(c))) mode = async ? 0 : 1;
    // the slot's device buffer: an SDMA copy of an earlier frame may still read it (whatever this call's mode)
    if ((rc = sdma_wait(c, slot))) return rc;
    c->last_copy_mode = mode;
    void* direct = mode == 2 ? pinned_device_ptr(host, npx * pb) : nullptr;
    if (direct) px = direct;
    else if ((rc = ctx_buffer(c, 5 + slot, npx * pb, &px))) return rc;
    if (with_stats && ((rc = ctx_buffer(c, 3, npx * 4, &rcb)) || (rc = ctx_buffer(c, 4, 16, sums)))) return rc;
    const hipStream_t cs = mode != 0 ? c->rs : c->cs;
    // mode 3: the copy in halves on two engines when two are free (r05, tools/copy_ab.py: 49.3 vs 50.3 us per
    // pipelined c2 GRAY8 frame), each half decrementing sd_done.  (Rendering a synchronous frame in two row chunks,
    // each copied as soon as it is in its buffer, measured no faster: 83.9 vs 83.1 us — the chunks are two views to
    // the per-view tile-order and cone caches, and each copy's start after its signal costs ~8 us.)
    const size_t nbytes = npx * pb;
    const size_t half = c->sd_engine2 && c->sd_split >= 2 && nbytes >= 65536 ? nbytes / 2 & ~(size_t)255 : 0;
    if (mode == 3) {                                    // before the render is queued: it fires sd_dep
        hsa_signal_store_relaxed(c->sd_dep[slot], 1);
        hsa_signal_store_relaxed(c->sd_done[slot][0], 1);
        hsa_signal_store_relaxed(c->sd_done[slot][1], 1);
    }
    // the slot's device buffer is free once its previous frame's copy has left (ordered by the stream when that
    // copy ran on the render stream)
    if (c->copied_rec[slot] && c->copied_cs[slot]) RT_HIP(hipStreamWaitEvent(c->rs, c->copied[slot], 0));
    if (with_stats) RT_HIP(hipEventRecord(c->ev0, c->rs));
    const bool f = float_format(format);
    rc = render_dev_impl(c, cam, W, H, depth, nullptr, f ? format : RT_PIXEL_RGBA32F, f ? px : nullptr,
                         f ? RT_PIXEL_RGBA8 : format, f ? nullptr : px, nullptr, (uint32_t*)rcb, c->rs);
    if (rc) return rc;
    if (with_stats) RT_HIP(hipEventRecord(c->ev1, c->rs));
    if (with_stats && (rc = queue_raysum(c, npx, (uint32_t*)rcb, (unsigned long long*)*sums))) return rc;
    if (mode == 3) {
        RT_HIP(sdma_fire(c, slot, c->sd_writer));      // the frame is in px
        RT_HIP(hipEventRecord(c->sd_fired[slot], c->rs));
        const hsa_status_t hs = hsa_amd_memory_async_copy_on_engine(
            hdev, c->sd_cpu, px, c->sd_gpu, half ? half : nbytes, 1, &c->sd_dep[slot], c->sd_done[slot][0],
            (hsa_amd_sdma_engine_id_t)c->sd_engine, true);
        if (hs != HSA_STATUS_SUCCESS) {
            RT_HIP(hipStreamSynchronize(c->rs));
            return rt_fail(RT_EHIP, "rt_render_packed: hsa_amd_memory_async_copy_on_engine failed");
        }
        c->sd_pending[slot] = true;                     // (the first copy is queued: its slot must be waited for)
        c->sd_copies[slot] = 1;
        if (half) {
            const hsa_status_t h2 = hsa_amd_memory_async_copy_on_engine(
                (char*)hdev + half, c->sd_cpu, (char*)px + half, c->sd_gpu, nbytes - half, 1, &c->sd_dep[slot],
                c->sd_done[slot][1], (hsa_amd_sdma_engine_id_t)c->sd_engine2, true);
            if (h2 != HSA_STATUS_SUCCESS) {
                (void)sdma_wait(c, slot);
                return rt_fail(RT_EHIP, "rt_render_packed: hsa_amd_memory_async_copy_on_engine failed");
            }
            c->sd_copies[slot] = 2;
        }
        c->copied_rec[slot] = false;
        return RT_OK;
    }
    if (cs != c->rs) {
        // the copy runs on the copy stream, so it overlaps the next frame's render
        RT_HIP(hipEventRecord(c->rendered[slot], c->rs));
        RT_HIP(hipStreamWaitEvent(cs, c->rendered[slot], 0));
    }
    if (!direct && (rc = copy_to_host(c, host, px, npx * pb, cs, mode == 0 ? kCopyStreamBlocks : 0))) return rc;
    RT_HIP(hipEventRecord(c->copied[slot], cs));
    c->copied_rec[slot] = true;
    c->copied_cs[slot] = cs != c->rs;
    return RT_OK;
}

extern "C" int rt_render_packed(rt_ctx* c, const rt_scene* scene, const rt_camera* cam, int W, int H, int depth,
                                int format, void* host_pixels, rt_stats* stats) {
    size_t npx = 0;
    void* sums = nullptr;
    if (!c) return rt_fail(RT_EINVAL, "rt_render_packed: null context");
    const uint64_t t = c->ticket + 1;                   // issued only once the frame is queued
    int rc = render_packed_queue(c, scene, cam, W, H, depth, format, host_pixels, (int)(t % rt_ctx::kSlots), stats != nullptr,
                                 &npx, &sums, false);
    if (rc) return rc;
    c->ticket = t;
    if (c->sd_pending[t % rt_ctx::kSlots]) {
        if ((rc = sdma_wait(c, (int)(t % rt_ctx::kSlots)))) return rc;
    } else {
        RT_HIP(hipEventSynchronize(c->copied[t % rt_ctx::kSlots]));
    }
    if (stats) {
        RT_HIP(hipStreamSynchronize(c->rs));
        return read_stats(c, npx, (const unsigned long long*)sums, stats);
    }
    return RT_OK;
}

extern "C" int rt_render_packed_async(rt_ctx* c, const rt_scene* scene, const rt_camera* cam, int W, int H,
                                      int depth, int format, void* host_pixels, uint64_t* ticket) {
    size_t npx = 0;
    void* sums = nullptr;
    if (!c) return rt_fail(RT_EINVAL, "rt_render_packed_async: null context");
    const uint64_t t = c->ticket + 1;
    int rc = render_packed_queue(c, scene, cam, W, H, depth, format, host_pixels, (int)(t % rt_ctx::kSlots), false, &npx,
                                 &sums, true);
    if (rc) return rc;
    c->ticket = t;
    if (ticket) *ticket = t;
    return RT_OK;
}

extern "C" int rt_ctx_wait(rt_ctx* c, uint64_t ticket) {
    if (!c) return rt_fail(RT_EINVAL, "rt_ctx_wait: null context");
    if (ticket > c->ticket) return rt_fail(RT_EINVAL, "rt_ctx_wait: ticket not issued");
    RT_HIP(hipSetDevice(c->device));
    if (ticket == 0) {                                  // everything queued on the context's streams
        RT_HIP(hipStreamSynchronize(c->rs));
        RT_HIP(hipStreamSynchronize(c->cs));
        for (int b = 0; b < rt_ctx::kSlots; ++b) {
            const int rc = sdma_wait(c, b);
            if (rc) return rc;
        }
        return RT_OK;
    }
    // slot (ticket % kSlots) holds this frame's copy or a later one's (which the GPU orders after it)
    const int sl = (int)(ticket % rt_ctx::kSlots);
    if (c->sd_pending[sl]) return sdma_wait(c, sl);
    if (c->copied_rec[sl]) RT_HIP(hipEventSynchronize(c->copied[sl]));
    return RT_OK;
}

extern "C" int rt_diag_copy_path(rt_ctx* c, int* mode, int* writer) {
    if (!c) return rt_fail(RT_EINVAL, "rt_diag_copy_path: null context");
    if (mode) *mode = c->last_copy_mode;
    if (writer) *writer = c->sd_ok ? c->sd_writer : 0;
    return RT_OK;
}

extern "C" int rt_host_alloc(size_t bytes, void** out) {
    if (!out || bytes == 0) return rt_fail(RT_EINVAL, "rt_host_alloc: bad arguments");
    *out = nullptr;
    // RT_HOST_NONCOHERENT=1 (A/B): non-coherent pinned memory (the GPU may cache its writes until the kernel ends)
    const char* nc = getenv("RT_HOST_NONCOHERENT");
    RT_HIP(hipHostMalloc(out, bytes, nc && atoi(nc) ? hipHostMallocNonCoherent : hipHostMallocDefault));
    void* dmap = nullptr;
    if (hipHostGetDevicePointer(&dmap, *out, 0) != hipSuccess || !dmap) dmap = nullptr;
    if (dmap) {                                         // host frames in it are copied by rt_copy_out_kernel
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned[(uintptr_t)*out] = {bytes, (uintptr_t)dmap};
    }
    return RT_OK;
}

extern "C" int rt_host_free(void* p) {
    if (!p) return RT_OK;
    {
        std::lock_guard<std::mutex> lk(g_pinned_mu);
        g_pinned.erase((uintptr_t)p);
    }
    RT_HIP(hipHostFree(p));
    return RT_OK;
}

constexpr size_t kScreenLdsMax = 64 * 1024;       // screen chunks: scene record in LDS when it fits beside the slots

static int trace_rays_launch(rt_ctx* c, const double* starts, const double* ends, int n, int depth, double* rgb64f,
                             uint32_t* raycount, hipStream_t st, const ScreenArgs& sa) {
    RT_HIP(hipSetDevice(c->device));
    const dim3 grid((unsigned)((n + kThreads - 1) / kThreads));
    const int v = c->tree ? 2 : c->transparent ? 1 : 0;
    hipError_t e;
    switch (depth) {
        case 0: e = launch_trace_rays<0>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        case 1: e = launch_trace_rays<1>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        case 2: e = launch_trace_rays<2>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        case 3: e = launch_trace_rays<3>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        case 4: e = launch_trace_rays<4>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        case 5: e = launch_trace_rays<5>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        case 6: e = launch_trace_rays<6>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
        default: e = launch_trace_rays<7>(v, grid, st, c->d_scene, starts, ends, n, rgb64f, raycount, sa); break;
    }
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_trace_rays_kernel: ") + hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_trace_rays_dev(rt_ctx* c, const double* starts, const double* ends, int n, int depth,
                                 double* rgb64f, uint32_t* raycount, void* stream) {
    if (!c || !c->scene_set) return rt_fail(RT_EINVAL, "rt_trace_rays_dev: no context/scene");
    if (n < 0 || (n > 0 && (!starts || !ends))) return rt_fail(RT_EINVAL, "rt_trace_rays_dev: bad rays");
    if (depth < 0 || depth > RT_MAX_DEPTH) return rt_fail(RT_EINVAL, "rt_trace_rays_dev: depth out of range");
    if (n == 0) return RT_OK;
    return trace_rays_launch(c, starts, ends, n, depth, rgb64f, raycount, (hipStream_t)stream, ScreenArgs{});
}

int rt_trace_screen_dev(rt_ctx* c, const double cam[3], const ScreenPix* pix, const int32_t* first, int m,
                        const double* jit, int n, int depth, double* rgb64f, uint32_t* done, uint32_t seq,
                        void* stream) {
    if (!c || !c->scene_set) return rt_fail(RT_EINVAL, "rt_trace_screen_dev: no context/scene");
    if (depth < 0 || depth > RT_MAX_DEPTH) return rt_fail(RT_EINVAL, "rt_trace_screen_dev: depth out of range");
    if (n <= 0 || m <= 0) return RT_OK;
    ScreenArgs sa;
    sa.pix = pix, sa.m = m, sa.first = first, sa.jit = jit, sa.done = done, sa.seq = seq;
    // RT_SCREEN_LDS=0 (A/B): the scene record read from global memory instead of LDS
    static const bool lds = !getenv("RT_SCREEN_LDS") || atoi(getenv("RT_SCREEN_LDS")) != 0;
    const size_t slots = c->tree ? 0 : slot_bytes(depth, c->transparent, kScreenBlock);
    if (lds && c->scene_bytes % 8 == 0 && (size_t)c->scene_bytes + slots <= kScreenLdsMax) sa.scene_lds = c->scene_bytes;
    return trace_rays_launch(c, cam, nullptr, n, depth, rgb64f, nullptr, (hipStream_t)stream, sa);
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

static int check_band_geometry(const char* who, const void* gathered, const void* image, int W, int H,
                               int band_height, int n_ranks, int slab_rows) {
    if (!gathered || !image) return rt_fail(RT_EINVAL, std::string(who) + ": null buffer");
    if (W <= 0 || H <= 0 || band_height <= 0 || n_ranks <= 0 || slab_rows < 0)
        return rt_fail(RT_EINVAL, std::string(who) + ": bad geometry");
    rt_rows r = {band_height, n_ranks, 0, 0};
    for (int q = 0; q < n_ranks; ++q) {
        int nl = 0;
        r.rank = q;
        rt_local_rows(H, &r, &nl);
        if (nl > slab_rows) return rt_fail(RT_EINVAL, std::string(who) + ": slab_rows smaller than a rank's rows");
    }
    return RT_OK;
}

int rt_unshuffle_dev_ex(const void* gathered, const void* rank0_slab, void* image, int W, int H, int elem_bytes,
                        int band_height, int n_ranks, int slab_rows, void* stream) {
    int rc = check_band_geometry("rt_unshuffle_dev", gathered, image, W, H, band_height, n_ranks, slab_rows);
    if (rc) return rc;
    if (elem_bytes <= 0 || ((long long)W * elem_bytes) % 4 != 0)
        return rt_fail(RT_EINVAL, "rt_unshuffle_dev: row bytes must be a multiple of 4");
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

// RT_UNPACK_VEC4=1 (A/B): the 4-pixel steps for byte formats too (r05's kernel)
static const bool g_unpack_vec4 = [] {
    const char* e = getenv("RT_UNPACK_VEC4");
    return e && atoi(e) != 0;
}();

int rt_unpack_dev_ex(const void* gathered, const void* rank0_slab, void* image, int W, int H, int src_format,
                     int dst_format, int band_height, int n_ranks, int slab_rows, void* stream) {
    int sb = 0, db = 0;
    int rc = rt_pixel_bytes(src_format, &sb);
    if (!rc) rc = rt_pixel_bytes(dst_format, &db);
    if (rc) return rc;
    if (src_format == dst_format)
        return rt_unshuffle_dev_ex(gathered, rank0_slab, image, W, H, sb, band_height, n_ranks, slab_rows, stream);
    rc = check_band_geometry("rt_unpack_dev", gathered, image, W, H, band_height, n_ranks, slab_rows);
    if (rc) return rc;
    int mode;
    if (src_format == RT_PIXEL_GRAY8 && dst_format == RT_PIXEL_RGBA8) mode = kUnpackGray8;
    else if (src_format == RT_PIXEL_RGB8 && dst_format == RT_PIXEL_RGBA8) mode = kUnpackRgb8;
    else if (src_format == RT_PIXEL_GRAY32F && dst_format == RT_PIXEL_RGBA32F) mode = kUnpackGray32f;
    else return rt_fail(RT_EINVAL, "rt_unpack_dev: unsupported format pair");
    const bool al16 = ((uintptr_t)gathered | (uintptr_t)rank0_slab | (uintptr_t)image) % 16 == 0;
    const int vec = !al16 || W % 4 != 0 ? 0 : mode != kUnpackGray32f && !g_unpack_vec4 ? 16 : 4;
    const uint8_t* g = (const uint8_t*)gathered;
    const uint8_t* g0 = (const uint8_t*)rank0_slab;
    uint8_t* im = (uint8_t*)image;
    const hipStream_t st = (hipStream_t)stream;
    const dim3 grid((unsigned)H), blk(kThreads);
#define RT_UNPACK(M, V) hipLaunchKernelGGL((rt_unpack_kernel<M, V>), grid, blk, 0, st, g, g0, im, W, H, band_height, \
                                           n_ranks, slab_rows)
    if (mode == kUnpackGray8) {
        if (vec == 16) RT_UNPACK(kUnpackGray8, 16); else if (vec) RT_UNPACK(kUnpackGray8, 4); else RT_UNPACK(kUnpackGray8, 0);
    } else if (mode == kUnpackRgb8) {
        if (vec == 16) RT_UNPACK(kUnpackRgb8, 16); else if (vec) RT_UNPACK(kUnpackRgb8, 4); else RT_UNPACK(kUnpackRgb8, 0);
    } else {
        if (vec) RT_UNPACK(kUnpackGray32f, 4); else RT_UNPACK(kUnpackGray32f, 0);
    }
#undef RT_UNPACK
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return rt_fail(RT_EHIP, std::string("rt_unpack_kernel: ") + hipGetErrorString(e));
    return RT_OK;
}

extern "C" int rt_unpack_dev(const void* gathered, void* image, int W, int H, int src_format, int dst_format,
                             int band_height, int n_ranks, int slab_rows, void* stream) {
    return rt_unpack_dev_ex(gathered, nullptr, image, W, H, src_format, dst_format, band_height, n_ranks, slab_rows,
                            stream);
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
extern "C" int rt_diag_kernel_resources(int depth, int variant, int* vgprs, int* scratch_bytes) {
    if (depth < 0 || depth > RT_MAX_B || variant < 0 || variant > 5 || !vgprs || !scratch_bytes)
        return rt_fail(RT_EINVAL, "rt_diag_kernel_resources: bad arguments");
    const void* f = nullptr;
    switch (depth) {
        case 0: f = render_kernel_ptr<0>(variant); break;
        case 1: f = render_kernel_ptr<1>(variant); break;
        case 2: f = render_kernel_ptr<2>(variant); break;
        case 3: f = render_kernel_ptr<3>(variant); break;
        case 4: f = render_kernel_ptr<4>(variant); break;
        case 5: f = render_kernel_ptr<5>(variant); break;
        case 6: f = render_kernel_ptr<6>(variant); break;
        default: f = render_kernel_ptr<7>(variant); break;
    }
    if (!f) return rt_fail(RT_EINVAL, "rt_diag_kernel_resources: kernel not built");
    hipFuncAttributes a;
    RT_HIP(hipFuncGetAttributes(&a, f));
    *vgprs = a.numRegs;
    *scratch_bytes = (int)a.localSizeBytes;
    return RT_OK;
}

// Workgroups of the render kernel (depth, variant as above) the runtime places per CU with `lds_bytes` of
// dynamic LDS (hipOccupancyMaxActiveBlocksPerMultiprocessor).
extern "C" int rt_diag_kernel_occupancy(int depth, int variant, int lds_bytes, int* blocks_per_cu) {
    if (depth < 0 || depth > RT_MAX_B || variant < 0 || variant > 5 || lds_bytes < 0 || !blocks_per_cu)
        return rt_fail(RT_EINVAL, "rt_diag_kernel_occupancy: bad arguments");
    const void* f = nullptr;
    switch (depth) {
        case 0: f = render_kernel_ptr<0>(variant); break;
        case 1: f = render_kernel_ptr<1>(variant); break;
        case 2: f = render_kernel_ptr<2>(variant); break;
        case 3: f = render_kernel_ptr<3>(variant); break;
        case 4: f = render_kernel_ptr<4>(variant); break;
        case 5: f = render_kernel_ptr<5>(variant); break;
        case 6: f = render_kernel_ptr<6>(variant); break;
        default: f = render_kernel_ptr<7>(variant); break;
    }
    if (!f) return rt_fail(RT_EINVAL, "rt_diag_kernel_occupancy: kernel not built");
    RT_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks_per_cu, f, RT_WG_FAST, (size_t)lds_bytes));
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
