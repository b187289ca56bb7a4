// rt_render.hpp — the per-pixel render kernel and the ray-list kernel (templates), shared by rt_kernel.hip
// (the C ABI) and the per-depth instance files rt_render_b<B>.hip.  The bounce depth B is a template
// parameter (the bounce loop is unrolled); each depth's instances live in their own translation unit so the
// eight depths compile in parallel (one file with all of them took > 5 minutes of one core).
//
//   rt_render_kernel<B, LDS, MINW, TRANSP, CULL, WG, TREE>  one work-item per pixel, FP64, iterative bounce
//                             loop (rt_device.hpp).  Default: one-wave workgroups (WG = 64), each owning an
//                             8 x 8 pixel tile (square tiles keep a wave's rays coherent, so the __any early-out
//                             and the culling masks work for whole waves).  The scene is read through the
//                             scalar cache; the A/B variants with 256-thread workgroups (32 x 8 tiles) copy it
//                             into LDS once per workgroup (LDS = 1) or stage the output tile in LDS for 32-pixel
//                             row stores.  Per-level colours wait in LDS slots; stores go out per wave.
//   rt_trace_rays_kernel<B>   rayTraceRay on an arbitrary ray list (parity / fuzz / faithful-screen entry).
//
// Output pixel formats (RenderParams::fmt_f / fmt_8, wave-uniform): the float image is RGBA32F (16 B/px) or
// GRAY32F (4 B/px, the R channel: only for scenes proven achromatic, where R = G = B bit for bit); the byte
// image is RGBA8 (4 B/px), RGB8 (3 B/px) or GRAY8 (1 B/px, achromatic scenes).  The packed formats cut the
// bytes a frame moves over xGMI (rt_render_multi) or PCIe (rt_render_packed).
//
// Reference: /root/reference/Hw4/MySdlApplication.cpp (rayTraceScreen :1251-1324, rayTraceRay :1184-1249,
// intersection code :611-823, :1084-1113).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>

#include "../../include/rt_api.h"
#include "rt_device.hpp"

#ifndef RT_WAVE_TRACE
#define RT_WAVE_TRACE 0
#endif
#ifndef RT_ABLATE
#define RT_ABLATE 0                            // instruction-count ablation builds (tools/ablate.sh): 1 prologue, 2 no stores
#endif
// __launch_bounds__ minimum waves per EU of the depth <= 3 render kernels.  0 (default): 6 for depth <= 2
// (<= 80 VGPRs, no spills since the bounce loop stopped carrying the previous ray through the light loop),
// 5 for depth 3 (<= 96 VGPRs; 6 would spill 8 B/lane).
#ifndef RT_MINW
#define RT_MINW 0
#endif
#ifndef RT_NT_STORES
#define RT_NT_STORES 1                         // non-temporal RGBA32F/RGBA8 stores (0: A/B)
#endif
#ifndef RT_WG_FAST
#define RT_WG_FAST 64                          // workgroup of the default render kernels: 64 (8 x 8) or 128 (16 x 8)
#endif
// RT_PIX_RECOMPUTE=1: the store recomputes the pixel position from an opaque copy of the thread index instead of
// keeping it live through trace(): 2 VGPRs fewer in the culling kernels, but c3 +2.9% (same-box A/B), so off.
#ifndef RT_PIX_RECOMPUTE
#define RT_PIX_RECOMPUTE 0
#endif
// ... but in the 7-wave culling kernels it is what keeps the pixel position out of scratch (12 B/lane spilled at
// the prologue and reloaded for the stores otherwise): on for them.
#ifndef RT_PIX_RECOMPUTE_CULL
#define RT_PIX_RECOMPUTE_CULL 1
#endif
// The culling variant (>= kConeMin spheres): 7 waves per SIMD (72 VGPRs, 94 SGPRs with 30 spilled to VGPR lanes,
// 12 B/lane of scratch), which its LDS allows since the last level's colour stays in registers (RT_CULL_LAST_REG:
// 4.5 KB per workgroup at depth 3).  c5 -2.6% serial, -3.9% with 3 frames in flight against the same code at 6
// waves (77 VGPRs, no scratch; in-process A/B).
#ifndef RT_MINW_CULL
#define RT_MINW_CULL 7
#endif
// (depth 2 spills 12 B/lane at 7 waves even with the store position recomputed: 6 waves there, 75 VGPRs, no scratch)
__host__ __device__ constexpr int cull_min_waves(int B) { return B == 2 && RT_MINW_CULL > 6 ? 6 : RT_MINW_CULL; }
// Default launch-bound waves per SIMD of the fast kernels by depth: 6 up to depth 2, 5 from depth 3.  The bound
// is a floor: the depth 1 and 2 kernels come out at 63 / 67 VGPRs under it (8 / 7 waves by VGPRs; the c2 kernel
// accumulates its colour in LDS, shade ACC) and their SGPR cap (rt_render_kernel_sg, 96) gives them 7 waves per
// SIMD on the hardware; r03's bound of 7 made the compiler trade SGPR spills (v_writelane) for the same VGPRs and
// ran c2 +2.3% slower (same-box A/B).
__host__ __device__ constexpr int kDefaultMinWaves(int B) { return B <= 2 ? 6 : 5; }
// RT_MAX_B < 7 (experiment builds only, tools/variants.sh): deeper kernels are not instantiated.
#ifndef RT_MAX_B
#define RT_MAX_B 7
#endif
// Per-tile cache of the culling kernels' level masks (rt_device.hpp LevelMasks); 0: always computed (A/B builds).
#ifndef RT_LEVEL_MASKS
#define RT_LEVEL_MASKS 1
#endif
// The most mask slots per tile the cache holds (B ray masks + (B + 1) nl shadow masks); beyond it the masks are computed.
constexpr int kLevelMaskSlotsMax = 24;

namespace rtk {

using namespace rt;

constexpr int kTileW = 32;   // workgroup tile of the 256-thread variants: 32 columns ...
constexpr int kTileH = 8;    // ... x 8 rows = 256 pixels
constexpr int kThreads = 256;
static_assert(kThreads == kSlotStride, "one LDS colour slot column per work-item");
constexpr int kGridY = 32768;                  // grid.y per grid.z slice

// Pixel formats of the kernel's two images (include/rt_api.h RT_PIXEL_*).
constexpr int kFmtF_RGBA = 0, kFmtF_GRAY = 1;                // float image
constexpr int kFmt8_RGBA = 0, kFmt8_RGB = 1, kFmt8_GRAY = 2;  // byte image

// LDS bytes of trace()'s per-level slots for depth B: 3 doubles per colour slot (colour_slots: one per level,
// plus one for the parked continuation when the colour accumulates in LDS) and the material id per level when
// TRANSP, per work-item of a `wg`-thread workgroup.
__host__ __device__ constexpr int slot_bytes(int B, bool transp, int wg = kSlotStride, bool cull = false) {
    return (colour_slots(B, transp, cull) * 3 * 8 + (transp ? (B + 1) * 4 : 0)) * wg;
}

// Image tile column traced at grid column bx of dispatch row gy.  The dispatcher sends workgroup L = gy * tiles_x + bx
// to XCD L mod 8; with tiles_x a multiple of 8 (every benchmark width) XCD j would trace the same image columns
// (j mod 8) in every row — a fixed vertical stripe set whose cost depends on the scene (c2: XCDs ending 31.9 to
// 35.7 us into a 35.7-us launch, wave trace).  RT_XCD_SWIZZLE=1 rotates the columns by gy mod 8, handing each XCD
// every column class over 8 rows: the XCDs then end within 1.5 us of each other, but c2 runs +1.3% serial, +0.6% in
// flight (c3, c5 within 0.6%; in-process A/B) — the stripes were not what held the launch's end.  Off.
#ifndef RT_XCD_SWIZZLE
#define RT_XCD_SWIZZLE 0
#endif
__host__ __device__ __forceinline__ int tile_col(int bx, int gy, int tiles_x) {
#if RT_XCD_SWIZZLE
    const int rot = (gy & 7) < tiles_x ? (gy & 7) : 0;
    const int c = bx + rot;
    return c >= tiles_x ? c - tiles_x : c;
#else
    (void)gy;
    (void)tiles_x;
    return bx;
#endif
}

// Slot of dispatch position L (linear workgroup id) in the dispatch table of n positions: grouped by L mod 8, the XCD
// the round-robin dispatcher sends workgroup L to (up to a per-launch rotation), so each XCD reads a contiguous run
// of the table and no L2 line is fetched by more than one XCD.
#ifndef RT_DISP32
#define RT_DISP32 0
#endif
__host__ __device__ __forceinline__ size_t cone_slot(size_t L, size_t n) { return (L & 7) * ((n + 7) >> 3) + (L >> 3); }
__host__ __device__ __forceinline__ size_t cone_slots(size_t n) { return ((n + 7) >> 3) << 3; }

// One dispatch position of a calibrated view (rt_kernel.hip rt_disp_kernel): the tile its workgroup traces
// (ty << 16 | tx) and that tile's primary cone mask (valid when RenderParams::cone_use).  The table is indexed by
// cone_slot(position): one 16-byte scalar load per wave brings both.
struct alignas(16) DispRec {
    uint32_t cone_lo, cone_hi;
    uint32_t tile;
    uint32_t pad;
};

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
    int32_t fmt_f;                             // kFmtF_*: float image format
    int32_t fmt_8;                             // kFmt8_*: byte image format
    float look32[3], right32[3], upp32[3], eye32[3], pitch32;   // FP32 camera for primary_cone_mask
    float cone_slack;                          // its error bound (render_params)
    const DispRec* disp;                       // dispatch table (nullptr: identity order; the kernel reads its argument)
    uint32_t* tile_cost;                       // calibration render: each tile's wave time (100 MHz), by tile
    int32_t tile_rows_n;                       // tile rows of this launch
    int32_t tiles_x;                           // tiles per tile row (= grid.x)
    uint64_t* wtrace;                          // RT_WAVE_TRACE builds: per-wave {start, end, HW_ID}
    int32_t cone_use;                          // 1: disp's cone masks are this view's (cached primary cone masks)
    uint64_t* cone_out;                        // calibration render: each tile's mask, by tile (or nullptr)
    int32_t ns;                                // stride of the scene's per-sphere arrays (DevScene::n_stride)
    // Per-tile level masks (rt_device.hpp LevelMasks; culling kernels, one-wave tiles): lmask_stride slots per tile,
    // written by the calibration render (lmask_out) and read by later renders of exactly that view (lmask_in)
    uint64_t* lmask_out;
    const uint64_t* lmask_in;
    int32_t lmask_stride;
};

// The dispatch table's geometry, scalar arguments right after the table, so that gfx950's kernarg preload
// (-mllvm -amdgpu-kernarg-preload-count=4, Makefile KERNARG_PRELOAD) can hand both to the wave in SGPRs and its
// first memory access is its dispatch record.  Measured (r05, tools/ab_libs.py, 9 rounds): preloading 4 or 6
// dwords within +-0.8% of none at c2 / c3 / c5 (and the preloaded registers cost 20 more SGPR spills), so off.
struct DispGeom {
    int32_t tiles_x;                           // tiles per tile row (= grid.x)
    int32_t n;                                 // dispatch positions with a record (tile rows x tiles_x)
};

// The render kernels' arguments, in order: the kernel-argument segment lays them out as this struct (each at its
// natural alignment), which late_outputs() relies on.  (The kernels take them as separate parameters: one
// by-value struct parameter measured +11 VGPRs in the culling kernel.)
struct RenderArgs {
    const DispRec* disp;                       // dispatch table (nullptr: identity order)
    int32_t tiles_x, n_disp;                   // its DispGeom (scalars: aggregates are not preloaded)
    const DevScene* scene;
    RenderParams P;
    void* o32;                                 // float image (RGBA32F / GRAY32F) or nullptr
    void* o8;                                  // byte image (RGBA8 / RGB8 / GRAY8) or nullptr
    double* o64;                               // RGB64F parity image or nullptr
    uint32_t* orc;                             // per-pixel ray counters or nullptr
};

// The output pointers, read from the kernel-argument segment where the stores need them: scalar loads behind an
// opaque copy of the segment pointer, so the compiler cannot hoist them to the kernel's start and hold 8 SGPRs
// through the whole trace (the SGPR budget of a seventh wave per SIMD).
struct RenderOuts {
    void* o32;
    void* o8;
    double* o64;
    uint32_t* orc;
};
__device__ __forceinline__ RenderOuts late_outputs() {
    typedef const __attribute__((address_space(4))) char* kptr;
    typedef void* const __attribute__((address_space(4)))* kpp;
    kptr ka = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    RenderOuts o;
    o.o32 = *(kpp)(ka + offsetof(RenderArgs, o32));
    o.o8 = *(kpp)(ka + offsetof(RenderArgs, o8));
    o.o64 = (double*)*(kpp)(ka + offsetof(RenderArgs, o64));
    o.orc = (uint32_t*)*(kpp)(ka + offsetof(RenderArgs, orc));
    return o;
}

}  // namespace rtk

// The level-mask arrays of the render (RenderParams::lmask_in / lmask_out, rt_device.hpp LevelMasks), read from the
// kernel-argument segment where a mask is needed (behind an opaque copy of the segment pointer, as late_outputs).
namespace rt {
using rtk::RenderArgs;
using rtk::RenderParams;
__device__ __forceinline__ const uint64_t* level_masks_in() {
    typedef const __attribute__((address_space(4))) char* kptr;
    typedef const uint64_t* const __attribute__((address_space(4)))* kpp;
    kptr ka = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    return *(kpp)(ka + offsetof(RenderArgs, P) + offsetof(RenderParams, lmask_in));
}
__device__ __forceinline__ uint64_t* level_masks_out() {
    typedef const __attribute__((address_space(4))) char* kptr;
    typedef uint64_t* const __attribute__((address_space(4)))* kpp;
    kptr ka = (kptr)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(ka));
    return *(kpp)(ka + offsetof(RenderArgs, P) + offsetof(RenderParams, lmask_out));
}
}  // namespace rt

namespace rtk {

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

// Store pixel k of the two images in their formats.  PACKED = false: RGBA32F / RGBA8 only (the benchmark
// kernels: the runtime format branches cost c3 8% through the whole kernel's register allocation, same-box
// A/B); PACKED = true: fmt_f / fmt_8 are kernel arguments (scalar branches).
template <bool PACKED>
__device__ __forceinline__ void store_pixel(const RenderParams& P, size_t k, d3 col, void* __restrict__ out32,
                                            void* __restrict__ out8) {
    if (out32) {
        if (PACKED && P.fmt_f == kFmtF_GRAY) {
            reinterpret_cast<float*>(out32)[k] = (float)col.x;
        } else {
#if RT_NT_STORES
            float* o = reinterpret_cast<float*>(out32) + 4 * k;
            __builtin_nontemporal_store((float)col.x, o);
            __builtin_nontemporal_store((float)col.y, o + 1);
            __builtin_nontemporal_store((float)col.z, o + 2);
            __builtin_nontemporal_store(1.0f, o + 3);
#else
            reinterpret_cast<float4*>(out32)[k] = make_float4((float)col.x, (float)col.y, (float)col.z, 1.0f);
#endif
        }
    }
    if (out8) {
        if (PACKED && P.fmt_8 == kFmt8_GRAY) {
            reinterpret_cast<uint8_t*>(out8)[k] = to_u8(col.x);
        } else if (PACKED && P.fmt_8 == kFmt8_RGB) {
            uint8_t* o = reinterpret_cast<uint8_t*>(out8) + 3 * k;
            o[0] = to_u8(col.x);
            o[1] = to_u8(col.y);
            o[2] = to_u8(col.z);
        } else {
#if RT_NT_STORES
            const uint32_t px = (uint32_t)to_u8(col.x) | ((uint32_t)to_u8(col.y) << 8) |
                                ((uint32_t)to_u8(col.z) << 16) | (255u << 24);
            __builtin_nontemporal_store(px, reinterpret_cast<uint32_t*>(out8) + k);
#else
            reinterpret_cast<uchar4*>(out8)[k] = make_uchar4(to_u8(col.x), to_u8(col.y), to_u8(col.z), 255);
#endif
        }
    }
}

template <int B, int LDS, int MINW, bool TRANSP, bool CULL, int WG = kThreads, bool TREE = false,
          bool PACKED = false, bool FIX64 = false, bool ACHRO = false>
__device__ __forceinline__ void render_body(const DevScene* __restrict__ gscene, RenderParams P,
                                            const DispRec* __restrict__ disp, DispGeom geom) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x;
#if RT_WAVE_TRACE
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
#endif
    const uint64_t t_cal = __builtin_amdgcn_s_memrealtime();   // used by calibration renders (P.tile_cost)
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
    int* mslot = reinterpret_cast<int*>(smem + off + 3 * 8 * colour_slots(B, TRANSP, CULL) * WG) + tid;
    off += slot_bytes(B, TRANSP, WG, CULL);
    float4* st32 = reinterpret_cast<float4*>(smem + off);                              // [8][32] 4 KB
    double* st64 = reinterpret_cast<double*>(smem + off + 4096);                        // [8][32][3] 6 KB
    uint32_t* strc = reinterpret_cast<uint32_t*>(smem + off + 4096 + 6144);             // [8][32] 1 KB
    uchar4* st8 = reinterpret_cast<uchar4*>(smem + off + 4096 + 6144 + 1024);           // [8][32] 1 KB
    if (LDS) __syncthreads();
    // the fast kernels (scenes with np < kConeMin) see the fixed array stride as a constant
    constexpr bool kFixed = !LDS && !TRANSP && !CULL && !TREE && WG == RT_WG_FAST && RT_WG_FAST != kThreads;
    // (FIX64: the culling instance for scenes whose arrays have the stride kCullStride, see rt_layout.hpp)
    const SceneView V = view_of(S, gscene, P.np, kFixed ? kFastStride : FIX64 ? kCullStride : P.ns, P.nl);
    const d3 eye = ld3(P.eye);

    const int wave = tid >> 6, lane = tid & 63;
    // The 32 x 8 tile (WG = 256) is cut into 4 wave blocks of 8 x 8 pixels (square blocks keep a wave's
    // rays coherent; 16 x 4 and 32 x 2 blocks measured no faster, and 32 x 2 slower at c5); WG = 64: one
    // wave, one 8 x 8 tile.
    constexpr int bw = 8, bh = 8, TW = WG / 8;
    const int bx0 = wave * bw, by0 = 0;
    const int cx = bx0 + (lane & 7);               // column inside the tile
    const int cy = lane >> 3;                      // row inside the tile
    const int bxd = blockIdx.x;                     // 2-D grid: tiles_x x tiles_y
    const int gy = (int)(blockIdx.z * kGridY + blockIdx.y);    // tile rows beyond kGridY go to grid.z
    // The tile of this dispatch position and (cached views) its primary cone mask: one 16-byte record of the
    // dispatch table (a const __restrict__ kernel argument: a scalar load issued beside the other argument loads),
    // or the identity order.  Padding positions of the last grid.z slice trace a clamped tile and store nothing (no
    // early return: a branch here kept the compiler from issuing the scene loads until the tile had arrived).
    int tx = tile_col(bxd, gy, P.tiles_x), ty_raw = gy;
    uint64_t cone_cached = 0;
    if (disp) {
#if RT_DISP32
        // (32-bit index arithmetic: a frame's dispatch positions number < 2^31; cone_slot's value, fewer scalar ops
        // on the chain to the wave's first dependent load)
        const uint32_t n = (uint32_t)geom.n, Lp = (uint32_t)gy * (uint32_t)geom.tiles_x + (uint32_t)bxd;
        const uint32_t Lc = Lp < n ? Lp : n - 1;
        const DispRec rec = disp[(Lc & 7u) * ((n + 7u) >> 3) + (Lc >> 3)];   // (padding positions: in bounds, unused)
#else
        const size_t n = (size_t)geom.n, Lp = (size_t)gy * geom.tiles_x + bxd;
        const DispRec rec = disp[cone_slot(Lp < n ? Lp : n - 1, n)];   // (padding positions: in bounds, unused)
#endif
        asm volatile("" ::"s"(rec.cone_lo), "s"(rec.cone_hi), "s"(rec.tile));
        cone_cached = (uint64_t)rec.cone_lo | ((uint64_t)rec.cone_hi << 32);
        tx = (int)(rec.tile & 0xffffu);
        ty_raw = Lp < n ? (int)(rec.tile >> 16) : P.tile_rows_n;
    }
    const bool pad = (unsigned)ty_raw >= (unsigned)P.tile_rows_n;
    const int ty = pad ? P.tile_rows_n - 1 : ty_raw;
    // the stores' tile row: past every local row for padding positions (their bounds check fails), so no flag
    // needs to live through the trace
    const int ty_st = pad ? (1 << 27) : ty_raw;
    const int i = tx * TW + cx;
    const int lr = ty * kTileH + cy;
    const bool valid = i < P.width && lr < P.local_rows && !pad;
    (void)valid;                                   // (the direct stores recompute it from i_e, lr_e)
#if RT_WAVE_TRACE >= 2
    asm volatile("" ::"s"(ty));
    const uint64_t t_ty = __builtin_amdgcn_s_memrealtime();   // the tile row has arrived
#endif

    // Per-wave sphere culling (all lanes active here).  The block's rows must be contiguous image rows.
    uint64_t cone = ~0ull;
    RT_COUNT(V.S, kCntWaves, 1);
    if (P.np >= kPrimaryConeMin && P.cone_use) {
        // the mask this view's calibration render computed for this tile, in its dispatch record (rt_disp_kernel):
        // no cone phase
        cone = cone_cached;
    } else if (P.np >= kPrimaryConeMin) {
        // Within one frame global_row_of is increasing, so jb - ja == 7 means 8 consecutive rows.
        const int lr0 = ty * kTileH + by0, ja = global_row_of(P, lr0), jb = global_row_of(P, lr0 + bh - 1);
        const bool one_frame = P.frames <= 1 || lr0 / P.frame_rows == (lr0 + bh - 1) / P.frame_rows;
        const float hx = 0.5f * (float)(bw - 1), hy = 0.5f * (float)(bh - 1);
        if (one_frame && jb - ja == bh - 1)
            cone = primary_cone_mask(V, P.look32, P.right32, P.upp32, P.eye32, P.pitch32,
                                     (float)(tx * TW + bx0 + P.bottom_x) + hx, (float)(ja + P.bottom_y) + hy,
                                     sqrtf(hx * hx + hy * hy), P.cone_slack, lane);
        RT_COUNT(V.S, kCntConeKept, __popcll(cone & sphere_bits(V.np)));
        if (P.cone_out && tid == 0 && !pad) P.cone_out[(size_t)ty * P.tiles_x + tx] = cone;   // lane 0, vector store
    }
#if RT_WAVE_TRACE >= 2
    asm volatile("" ::"s"(cone));
    const uint64_t t_cone = __builtin_amdgcn_s_memrealtime();   // the primary cone mask is known
#endif

    // Every lane traces (trace() reduces over the wave): lanes outside the frame trace a clamped pixel
    // and store nothing.
    uint32_t seg = 0, sh = 0;
    const int ic = i < P.width ? i : P.width - 1, lrc = lr < P.local_rows ? lr : P.local_rows - 1;
    const int j = global_row_of(P, lrc);
    const d3 right = ld3(P.right), upp = ld3(P.upp);
    // Primary ray Line(camera, sp), SURVEY.md Appendix B (basis: rayTraceScreen :1270-1279).
    const d3 sp = add(add(ld3(P.look), scl(P.pitch * (double)(ic + P.bottom_x), right)),
                      scl(P.pitch * (double)(j + P.bottom_y), upp));
#if RT_WAVE_TRACE
    const uint64_t t_mid = __builtin_amdgcn_s_memrealtime();   // prologue done: the primary ray is formed
#endif
#if RT_ABLATE == 1
    // (instruction-count ablation builds only, tools/ablate.sh: the prologue alone — no trace, no stores)
    asm volatile("" ::"v"(sp.x), "v"(sp.y), "v"(sp.z), "s"(cone));
    return;
#endif
    d3 col;
    LevelMasks lm{-1};
    if (RT_LEVEL_MASKS && !TRANSP && !TREE && P.lmask_stride > 0 && !pad) lm.tile = (ty * P.tiles_x + tx) * P.lmask_stride;
    if constexpr (TREE)
        col = trace_tree<B>(V, eye, sp, &seg, &sh);
    else
        col = trace<B, true, TRANSP, CULL, WG, ACHRO>(V, eye, sp, cone, &seg, &sh, slot, mslot, lm);
#if RT_WAVE_TRACE >= 2
    asm volatile("" ::"v"(col.x), "v"(col.y), "v"(col.z));
    const uint64_t t_trace = __builtin_amdgcn_s_memrealtime();   // trace() done, the stores next
#endif
#if RT_ABLATE == 2
    asm volatile("" ::"v"(col.x), "v"(col.y), "v"(col.z), "v"(seg), "v"(sh));   // (ablation: trace, no stores)
    return;
#endif

    if (WG != kThreads || !P.wg_staging) {
        // Direct stores: each wave writes its 8 x 8 block as 8 row segments (128 B of RGBA32F each) and
        // retires without waiting at a workgroup barrier for slower waves of the tile.
        int tid_e = tid;
#if RT_PIX_RECOMPUTE
        asm volatile("" : "+v"(tid_e));
#else
        if constexpr (CULL && RT_PIX_RECOMPUTE_CULL) asm volatile("" : "+v"(tid_e));
#endif
        const int lane_e = tid_e & 63;
        const int i_e = tx * TW + (tid_e >> 6) * bw + (lane_e & 7), lr_e = ty_st * kTileH + (lane_e >> 3);
        if (i_e < P.width && lr_e < P.local_rows) {
            const RenderOuts O = late_outputs();
            const size_t k = (size_t)lr_e * P.width + i_e;
            store_pixel<PACKED>(P, k, col, O.o32, O.o8);
            if (O.o64) { O.o64[3 * k] = col.x; O.o64[3 * k + 1] = col.y; O.o64[3 * k + 2] = col.z; }
            if (O.orc) O.orc[k] = seg | (sh << 16);
        }
        if (P.tile_cost && tid == 0 && ty_st < P.tile_rows_n)
            P.tile_cost[(size_t)ty_st * P.tiles_x + tx] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cal);
#if RT_WAVE_TRACE
        if (P.wtrace && tid == 0) {
            const size_t w = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
            P.wtrace[4 * w] = t_start;
            P.wtrace[4 * w + 1] = __builtin_amdgcn_s_memrealtime();
            P.wtrace[4 * w + 3] = t_mid;
#if RT_WAVE_TRACE >= 2
            P.wtrace[4 * (size_t)P.tile_rows_n * gridDim.x + 3 * w] = t_ty;
            P.wtrace[4 * (size_t)P.tile_rows_n * gridDim.x + 3 * w + 1] = t_cone;
            P.wtrace[4 * (size_t)P.tile_rows_n * gridDim.x + 3 * w + 2] = t_trace;
#endif
            P.wtrace[4 * w + 2] = (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11)) |
                                  ((uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11)) << 32);
        }
#endif
        return;
    }
    // Stage through LDS, then store whole tile rows (RGBA formats only: the host routes packed formats to the
    // direct-store variants).
    const RenderOuts O = late_outputs();
    void* const out32 = O.o32;
    void* const out8 = O.o8;
    double* const out64 = O.o64;
    uint32_t* const outrc = O.orc;
    const int ts = cy * kTileW + cx;
    if (out32) st32[ts] = make_float4((float)col.x, (float)col.y, (float)col.z, 1.0f);
    if (out64) { st64[3 * ts] = col.x; st64[3 * ts + 1] = col.y; st64[3 * ts + 2] = col.z; }
    if (outrc) strc[ts] = seg | (sh << 16);
    if (out8) st8[ts] = make_uchar4(to_u8(col.x), to_u8(col.y), to_u8(col.z), 255);
    __syncthreads();
    const int oy = tid >> 5, ox = tid & 31;
    const int gi = tx * kTileW + ox, glr = ty * kTileH + oy;
    if (gi < P.width && glr < P.local_rows && !pad) {                     // (A/B variant: pad kept)
        const size_t k = (size_t)glr * P.width + gi;
        if (out32) reinterpret_cast<float4*>(out32)[k] = st32[tid];
        if (out64) {
            out64[3 * k] = st64[3 * tid];
            out64[3 * k + 1] = st64[3 * tid + 1];
            out64[3 * k + 2] = st64[3 * tid + 2];
        }
        if (outrc) outrc[k] = strc[tid];
        if (out8) reinterpret_cast<uchar4*>(out8)[k] = st8[tid];
    }
    if (P.tile_cost && tid == 0 && !pad)
        P.tile_cost[(size_t)ty * P.tiles_x + tx] = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t_cal);
}

// (out32 .. outrc are read by late_outputs() from the argument segment, not through the parameters.)
// The parameter list must match RenderArgs field for field: kernarg_offsets_match below checks it at compile time.
template <int B, int LDS, int MINW, bool TRANSP, bool CULL, int WG = kThreads, bool TREE = false,
          bool PACKED = false, bool FIX64 = false, bool ACHRO = false>
__global__ __launch_bounds__(WG, MINW) void rt_render_kernel(const DispRec* __restrict__ disp, int32_t tiles_x, int32_t n_disp,
                                                             const DevScene* __restrict__ gscene, RenderParams P,
                                                             void* out32, void* out8, double* out64, uint32_t* outrc) {
    render_body<B, LDS, MINW, TRANSP, CULL, WG, TREE, PACKED, FIX64, ACHRO>(gscene, P, disp, DispGeom{tiles_x, n_disp});
}

// The same kernel with its SGPRs capped at RT_FAST_SGPRS (amdgpu_num_sgpr: a constant, hence a kernel of its
// own).  The hardware fits 7 one-wave workgroups per SIMD only up to 96 SGPRs per wave (the compiler's
// TotalSGPRs, VCC and friends included) and 8 only up to 78 (tools/mb_slots.cpp: 71 VGPRs with 96 SGPRs -> 7
// waves, 98 -> 6; 63 VGPRs with 78 -> 8, 86 -> 7) — the compiler's occupancy estimate assumes a larger SGPR file.
// r03: the cap cost 19 SGPR spills (+1.1%), so it was off.  r04: with the output pointers read at the stores
// (late_outputs), the fixed array stride of the fast kernels and the bounding-sphere delta formed where it is
// tested, the uncapped c2 kernel needs 98 SGPRs / 62 VGPRs and the capped one 94 / 63 with 2 spills: 7 waves per
// SIMD, c2 -1.7% and c3 -2.5% against the uncapped build (same-box in-process A/B, tools/ab_libs.py); a cap of 80
// (8 waves, 14 spills) ran +0.8%.
#ifndef RT_FAST_SGPRS
#define RT_FAST_SGPRS 96
#endif
// (the same parameter list as rt_render_kernel: RenderArgs, checked below)
template <int B, int MINW, bool CULL, bool PACKED, bool ACHRO = false>
__global__ __launch_bounds__(RT_WG_FAST, MINW) __attribute__((amdgpu_num_sgpr(RT_FAST_SGPRS)))
void rt_render_kernel_sg(const DispRec* __restrict__ disp, int32_t tiles_x, int32_t n_disp,
                         const DevScene* __restrict__ gscene, RenderParams P, void* out32, void* out8, double* out64,
                         uint32_t* outrc) {
    render_body<B, 0, MINW, false, CULL, RT_WG_FAST, false, PACKED, false, ACHRO>(gscene, P, disp, DispGeom{tiles_x, n_disp});
}

// r05: the achromatic depth-2 fast kernel (c3) fits 63 VGPRs, so a cap of 78 SGPRs gives it 8 waves per SIMD (58
// SGPRs spilled to VGPR lanes): c3 -1.2% against the 96-SGPR instance (tools/ab_libs.py, 9 rounds, same frames); the
// same cap on the depth-1 kernel (c2) ran +2.5%, so only depth RT_SG8_B takes it.
#ifndef RT_FAST8_SGPRS
#define RT_FAST8_SGPRS 78
#endif
// r06: off (-1).  After the r06 scalar-stream cuts the plain depth-2 instance needs 94 SGPRs and 64 VGPRs with no
// spills — 7 waves per SIMD on the hardware (8 need <= 78 SGPRs, above; the compiler reports 8) — and measured c3
// -0.9% serial, -3.1% in flight against the capped 8-wave one with its 58 spilled SGPRs
// (profiles/r06/ab/ab_libs_nosg8*.jsonl).
#ifndef RT_SG8_B
#define RT_SG8_B -1
#endif
#ifndef RT_SG8_MINW
#define RT_SG8_MINW 8                          // r06: the 8-wave kernel asks for 8 waves (<= 64 VGPRs) explicitly
#endif
template <int B, int MINW, bool CULL, bool PACKED, bool ACHRO = true>
__global__ __launch_bounds__(RT_WG_FAST, (RT_SG8_MINW > MINW ? RT_SG8_MINW : MINW)) __attribute__((amdgpu_num_sgpr(RT_FAST8_SGPRS)))
void rt_render_kernel_sg8(const DispRec* __restrict__ disp, int32_t tiles_x, int32_t n_disp,
                          const DevScene* __restrict__ gscene, RenderParams P, void* out32, void* out8, double* out64,
                          uint32_t* outrc) {
    render_body<B, 0, MINW, false, CULL, RT_WG_FAST, false, PACKED, false, ACHRO>(gscene, P, disp, DispGeom{tiles_x, n_disp});
}
template <int B, bool ACHRO>
constexpr bool use_sg8() { return ACHRO && B == RT_SG8_B && RT_FAST8_SGPRS > 0; }

// late_outputs() reads the output pointers at offsetof(RenderArgs, ...) of the kernel-argument segment, which lays the
// kernels' parameters out in order, each at its natural alignment.  The offsets of both kernels' actual parameter
// lists are computed here from their types and compared with RenderArgs: adding, reordering or re-typing a parameter
// (or a RenderParams change that moves the pointers) fails to compile instead of storing through a wrong pointer.
template <typename... A>
struct KernargLayout {
    static constexpr size_t offset(size_t i) {
        constexpr size_t sz[] = {sizeof(A)...}, al[] = {alignof(A)...};
        size_t off = 0;
        for (size_t k = 0;; ++k) {
            off = (off + al[k] - 1) / al[k] * al[k];
            if (k == i) return off;
            off += sz[k];
        }
    }
};
template <typename... A>
constexpr bool kernarg_offsets_match(void (*)(A...)) {
    using K = KernargLayout<A...>;
    return sizeof...(A) == 9 && K::offset(0) == offsetof(RenderArgs, disp) &&
           K::offset(1) == offsetof(RenderArgs, tiles_x) && K::offset(2) == offsetof(RenderArgs, n_disp) &&
           K::offset(3) == offsetof(RenderArgs, scene) && K::offset(4) == offsetof(RenderArgs, P) &&
           K::offset(5) == offsetof(RenderArgs, o32) && K::offset(6) == offsetof(RenderArgs, o8) &&
           K::offset(7) == offsetof(RenderArgs, o64) && K::offset(8) == offsetof(RenderArgs, orc);
}
static_assert(kernarg_offsets_match(&rt_render_kernel<1, 0, 1, false, false>),
              "rt_render_kernel's parameters must lay out as RenderArgs (late_outputs)");
static_assert(kernarg_offsets_match(&rt_render_kernel_sg<1, 1, false, false>),
              "rt_render_kernel_sg's parameters must lay out as RenderArgs (late_outputs)");
static_assert(kernarg_offsets_match(&rt_render_kernel_sg8<1, 1, false, false>),
              "rt_render_kernel_sg8's parameters must lay out as RenderArgs (late_outputs)");

// rayTraceRay on a list of rays Line(starts[k], ends[k]).  Rays from arbitrary starts: whether their hit
// points may skip the bounding-sphere cull is decided per ray (hits_ok_from).
// Screen mode (spix != nullptr, rt_render_screen's chunks): every ray starts at starts[0..2] (the camera) and ends at
// its pixel's screen point + 0.5 * its jitter value (MSA:1296), formed here instead of by a launch of its own.
template <int B, bool TRANSP, bool TREE = false, int WG = kThreads>
__global__ __launch_bounds__(WG) void rt_trace_rays_kernel(const DevScene* __restrict__ S,
                                                                 const double* __restrict__ starts,
                                                                 const double* __restrict__ ends, int n,
                                                                 double* __restrict__ rgb,
                                                                 uint32_t* __restrict__ rc,
                                                                 const ScreenPix* __restrict__ spix, int sm,
                                                                 const int32_t* __restrict__ sfirst,
                                                                 const double* __restrict__ sjit, int scene_lds,
                                                                 uint32_t* __restrict__ sdone, uint32_t sseq) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // Every lane traces (trace() reduces over the wave); lanes past n repeat ray n - 1 and store nothing.
    const int k = blockIdx.x * WG + threadIdx.x, kk = k < n ? k : n - 1;
    uint32_t seg = 0, sh = 0;
    // scene_lds > 0 (small launches: rt_render_screen's chunks): the whole scene record is copied into LDS first —
    // one burst of loads instead of a cold-cache round trip per record on the rays' dependent chain.  (The slots
    // behind it stay 8-byte aligned: scene_lds is a multiple of 8.)
    int off = 0;
    if (scene_lds > 0) {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(S);
        uint32_t* dst = reinterpret_cast<uint32_t*>(smem);
        for (int q = threadIdx.x; q < (scene_lds >> 2); q += WG) dst[q] = src[q];
        __syncthreads();
        S = reinterpret_cast<const DevScene*>(smem);
        off = scene_lds;
    }
    SceneView V = view_of(S, S, S->n_padded, S->n_stride, S->n_lights);
    d3 p0, p1;
    if (spix) {
        p0 = ld3(starts);
        int q = sfirst[blockIdx.x];                         // the pixel of the workgroup's first ray (WG = kScreenBlock)
        while (q + 1 < sm && spix[q + 1].off <= kk) ++q;
        const ScreenPix& X = spix[q];
        const double* J = sjit + 3 * (size_t)(X.base + (kk - X.off));
        p1 = d3{X.sp[0] + 0.5 * J[0], X.sp[1] + 0.5 * J[1], X.sp[2] + 0.5 * J[2]};
    } else {
        p0 = ld3(starts + 3 * kk);
        p1 = ld3(ends + 3 * kk);
    }
    V.hits_ok = hits_ok_from(S, p0);
    double* slot = reinterpret_cast<double*>(smem + off) + threadIdx.x;
    int* mslot = reinterpret_cast<int*>(smem + off + 3 * 8 * colour_slots(B, TRANSP) * WG) + threadIdx.x;
    d3 c;
    if constexpr (TREE)
        c = trace_tree<B>(V, p0, p1, &seg, &sh);
    else
        c = trace<B, false, TRANSP, false, WG>(V, p0, p1, ~0ull, &seg, &sh, slot, mslot);
    if (k < n) {
        if (rgb) { rgb[3 * k] = c.x; rgb[3 * k + 1] = c.y; rgb[3 * k + 2] = c.z; }
        if (rc) rc[k] = seg | (sh << 16);
    }
    if (sdone) {                                        // screen chunks: this workgroup's colours are out
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) __hip_atomic_store(sdone + blockIdx.x, sseq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// The screen-mode arguments of a trace launch (all null: a plain ray list).
struct ScreenArgs {
    const ScreenPix* pix = nullptr;
    int m = 0;
    const int32_t* first = nullptr;
    const double* jit = nullptr;
    int scene_lds = 0;                 // bytes of the scene record copied into LDS (multiple of 4; 0: none)
    uint32_t* done = nullptr;          // per-workgroup completion words (rt_trace_screen_dev)
    uint32_t seq = 0;
};

// Render-kernel variants rt_render_dev chooses between (rt_kernel.hip).
enum RenderVariant {
    kVarFast = 0,          // spheres + board (the benchmark kernels), launch bounds RT_MINW (depth <= 3)
    kVarFastAnyW,          // ... no occupancy bound (depth > 3, or RT_MIN_WAVES < 5)
    kVarCull,              // >= kConeMin spheres: per-wave culling, RT_MINW_CULL (depth <= 3)
    kVarCullAnyW,
    kVarTransp,            // meshes / transparent materials (FULL)
    kVarTree,              // ray trees (trace_tree)
    kVarLds,               // A/B: scene in LDS, 256-thread workgroups
    kVarStaging,           // A/B: LDS-staged row stores, 256-thread workgroups, RT_MINW
    kVarStagingAnyW,
    // packed pixel formats (rt_render_dev_packed: GRAY / RGB images), one per scene kind
    kVarFastPacked,
    kVarCullPacked,
    kVarTranspPacked,
    kVarTreePacked,
    kVarCount
};

struct RenderLaunch {
    int variant;
    bool achro;                                // achromatic scene: the one-channel instances (opaque variants)
    dim3 grid;
    size_t lds;
    hipStream_t stream;
    const DevScene* scene;
    RenderParams P;
    void* o32;
    void* o8;
    double* o64;
    uint32_t* orc;
};

// Defined once per depth B in rt_render_b<B>.hip.
template <int B>
hipError_t launch_render(const RenderLaunch& L);
template <int B>
hipError_t launch_trace_rays(int variant /* 0 opaque, 1 FULL, 2 tree */, dim3 grid, hipStream_t st,
                             const DevScene* s, const double* a, const double* b, int n, double* rgb, uint32_t* rc,
                             const ScreenArgs& sa);
template <int B>
const void* render_kernel_ptr(int variant);   // rt_diag_kernel_resources: 0 fast, 1 cull, 2 FULL, 3 tree

#define RT_DECLARE_DEPTH(B)                                                                                   \
    template <>                                                                                                \
    hipError_t launch_render<B>(const RenderLaunch& L);                                                        \
    template <>                                                                                                \
    hipError_t launch_trace_rays<B>(int, dim3, hipStream_t, const DevScene*, const double*, const double*, int,   \
                                    double*, uint32_t*, const ScreenArgs&);                                    \
    template <>                                                                                                \
    const void* render_kernel_ptr<B>(int);
RT_DECLARE_DEPTH(0) RT_DECLARE_DEPTH(1) RT_DECLARE_DEPTH(2) RT_DECLARE_DEPTH(3)
RT_DECLARE_DEPTH(4) RT_DECLARE_DEPTH(5) RT_DECLARE_DEPTH(6) RT_DECLARE_DEPTH(7)
#undef RT_DECLARE_DEPTH

// Body of the per-depth instance files.
template <int B, int LDS, int MINW, bool TRANSP, bool CULL, int WG, bool TREE, bool PACKED = false, bool FIX64 = false,
          bool ACHRO = false>
hipError_t launch_render_one(const RenderLaunch& L) {
    auto kern = rt_render_kernel<B, LDS, MINW, TRANSP, CULL, WG, TREE, PACKED, FIX64, ACHRO>;
    if (L.lds > 65536) {
        hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(kern, L.grid, dim3(WG), L.lds, L.stream, L.P.disp, L.P.tiles_x, L.P.tile_rows_n * L.P.tiles_x, L.scene, L.P, L.o32, L.o8, L.o64, L.orc);
    return hipGetLastError();
}

// The SGPR-capped fast kernel (rt_render_kernel_sg) for the depths whose fast kernels fit 7 waves by VGPRs (c2: 63,
// c3: 67).
#ifndef RT_SG_MAX_B
#define RT_SG_MAX_B 2
#endif
template <int B, int MINW, bool PACKED, bool ACHRO = false>
hipError_t launch_render_sg(const RenderLaunch& L) {
    if constexpr (use_sg8<B, ACHRO>())
        hipLaunchKernelGGL((rt_render_kernel_sg8<B, MINW, false, PACKED, ACHRO>), L.grid, dim3(RT_WG_FAST), L.lds,
                           L.stream, L.P.disp, L.P.tiles_x, L.P.tile_rows_n * L.P.tiles_x, L.scene, L.P, L.o32, L.o8, L.o64, L.orc);
    else
        hipLaunchKernelGGL((rt_render_kernel_sg<B, MINW, false, PACKED, ACHRO>), L.grid, dim3(RT_WG_FAST), L.lds,
                           L.stream, L.P.disp, L.P.tiles_x, L.P.tile_rows_n * L.P.tiles_x, L.scene, L.P, L.o32, L.o8, L.o64, L.orc);
    return hipGetLastError();
}

// The achromatic (one-channel, rt_device.hpp shade ACHRO) instances: the benchmark depths' fast and culling kernels.
#ifndef RT_ACHRO
#define RT_ACHRO 1
#endif
#ifndef RT_ACHRO_MAX_B
#define RT_ACHRO_MAX_B 3
#endif

template <int B>
hipError_t launch_render_impl(const RenderLaunch& L) {
    if constexpr (B > RT_MAX_B) {
        return hipErrorInvalidValue;
    } else {
        constexpr int MW = RT_MINW != 0 ? RT_MINW : kDefaultMinWaves(B);
        constexpr bool kAchro = RT_ACHRO && B <= RT_ACHRO_MAX_B;
        if constexpr (kAchro) {
            if (L.achro) {
                switch (L.variant) {
                    case kVarFast:
                        if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0) return launch_render_sg<B, MW, false, true>(L);
                        return launch_render_one<B, 0, MW, false, false, RT_WG_FAST, false, false, false, true>(L);
                    case kVarCull:
                        if (RT_CULL_FIX64 && L.P.ns == kCullStride)
                            return launch_render_one<B, 0, cull_min_waves(B), false, true, RT_WG_FAST, false, false, true,
                                                     true>(L);
                        return launch_render_one<B, 0, cull_min_waves(B), false, true, RT_WG_FAST, false, false, false,
                                                 true>(L);
                    case kVarFastPacked:
                        if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0) return launch_render_sg<B, MW, true, true>(L);
                        return launch_render_one<B, 0, MW, false, false, RT_WG_FAST, false, true, false, true>(L);
                    case kVarCullPacked:
                        if (RT_CULL_FIX64 && L.P.ns == kCullStride)
                            return launch_render_one<B, 0, cull_min_waves(B), false, true, RT_WG_FAST, false, true, true,
                                                     true>(L);
                        return launch_render_one<B, 0, cull_min_waves(B), false, true, RT_WG_FAST, false, true, false,
                                                 true>(L);
                    default: break;                     // the other variants: three channels
                }
            }
        }
        switch (L.variant) {
            case kVarFast:
                if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0) return launch_render_sg<B, MW, false>(L);
                return launch_render_one<B, 0, MW, false, false, RT_WG_FAST, false>(L);
            case kVarFastAnyW: return launch_render_one<B, 0, 1, false, false, RT_WG_FAST, false>(L);
            case kVarCull:
                if (RT_CULL_FIX64 && L.P.ns == kCullStride)
                    return launch_render_one<B, 0, cull_min_waves(B), false, true, RT_WG_FAST, false, false, true>(L);
                return launch_render_one<B, 0, cull_min_waves(B), false, true, RT_WG_FAST, false>(L);
            case kVarCullAnyW:
                if (RT_CULL_FIX64 && L.P.ns == kCullStride)
                    return launch_render_one<B, 0, 1, false, true, RT_WG_FAST, false, false, true>(L);
                return launch_render_one<B, 0, 1, false, true, RT_WG_FAST, false>(L);
            case kVarTransp: return launch_render_one<B, 0, 1, true, false, 64, false>(L);
            case kVarTree: return launch_render_one<B, 0, 1, true, false, 64, true>(L);
            case kVarLds: return launch_render_one<B, 1, 1, false, false, kThreads, false>(L);
            case kVarStaging: return launch_render_one<B, 0, MW, false, false, kThreads, false>(L);
            case kVarStagingAnyW: return launch_render_one<B, 0, 1, false, false, kThreads, false>(L);
            case kVarFastPacked:
                if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0) return launch_render_sg<B, MW, true>(L);
                return launch_render_one<B, 0, (B <= 3 ? MW : 1), false, false, RT_WG_FAST, false, true>(L);
            case kVarCullPacked:
                if (RT_CULL_FIX64 && L.P.ns == kCullStride)
                    return launch_render_one<B, 0, (B <= 3 ? cull_min_waves(B) : 1), false, true, RT_WG_FAST, false, true,
                                             true>(L);
                return launch_render_one<B, 0, (B <= 3 ? cull_min_waves(B) : 1), false, true, RT_WG_FAST, false, true>(L);
            case kVarTranspPacked: return launch_render_one<B, 0, 1, true, false, 64, false, true>(L);
            case kVarTreePacked: return launch_render_one<B, 0, 1, true, false, 64, true, true>(L);
            default: return hipErrorInvalidValue;
        }
    }
}

template <int B>
hipError_t launch_trace_rays_impl(int variant, dim3 grid, hipStream_t st, const DevScene* s, const double* a,
                                  const double* b, int n, double* rgb, uint32_t* rc, const ScreenArgs& sa) {
    if constexpr (B > RT_MAX_B) {
        return hipErrorInvalidValue;
    } else {
        const size_t lds = (size_t)sa.scene_lds;
        if (sa.pix) {                                   // screen chunks: kScreenBlock-thread workgroups
            constexpr int W = kScreenBlock;
            const dim3 g((unsigned)((n + W - 1) / W));
            if (variant == 2)
                hipLaunchKernelGGL((rt_trace_rays_kernel<B, true, true, W>), g, dim3(W), lds, st, s, a, b, n, rgb, rc,
                                   sa.pix, sa.m, sa.first, sa.jit, sa.scene_lds, sa.done, sa.seq);
            else if (variant == 1)
                hipLaunchKernelGGL((rt_trace_rays_kernel<B, true, false, W>), g, dim3(W), lds + slot_bytes(B, true, W),
                                   st, s, a, b, n, rgb, rc, sa.pix, sa.m, sa.first, sa.jit, sa.scene_lds, sa.done, sa.seq);
            else
                hipLaunchKernelGGL((rt_trace_rays_kernel<B, false, false, W>), g, dim3(W), lds + slot_bytes(B, false, W),
                                   st, s, a, b, n, rgb, rc, sa.pix, sa.m, sa.first, sa.jit, sa.scene_lds, sa.done, sa.seq);
            return hipGetLastError();
        }
        if (variant == 2)
            hipLaunchKernelGGL((rt_trace_rays_kernel<B, true, true>), grid, dim3(kThreads), lds, st, s, a, b, n, rgb, rc,
                               sa.pix, sa.m, sa.first, sa.jit, sa.scene_lds, sa.done, sa.seq);
        else if (variant == 1)
            hipLaunchKernelGGL((rt_trace_rays_kernel<B, true, false>), grid, dim3(kThreads), lds + slot_bytes(B, true),
                               st, s, a, b, n, rgb, rc, sa.pix, sa.m, sa.first, sa.jit, sa.scene_lds, sa.done, sa.seq);
        else
            hipLaunchKernelGGL((rt_trace_rays_kernel<B, false, false>), grid, dim3(kThreads), lds + slot_bytes(B, false),
                               st, s, a, b, n, rgb, rc, sa.pix, sa.m, sa.first, sa.jit, sa.scene_lds, sa.done, sa.seq);
        return hipGetLastError();
    }
}

template <int B>
const void* render_kernel_ptr_impl(int variant) {
    if constexpr (B > RT_MAX_B) {
        return nullptr;
    } else {
        constexpr int kFast = B <= 3 ? (RT_MINW != 0 ? RT_MINW : kDefaultMinWaves(B)) : 1;
        constexpr int kCull = B <= 3 ? cull_min_waves(B) : 1;
        switch (variant) {
            case 0:
                if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0) return (const void*)rt_render_kernel_sg<B, kFast, false, false>;
                return (const void*)rt_render_kernel<B, 0, kFast, false, false, RT_WG_FAST, false>;
            case 1: return (const void*)rt_render_kernel<B, 0, kCull, false, true, RT_WG_FAST, false, false, (bool)RT_CULL_FIX64>;
            case 2: return (const void*)rt_render_kernel<B, 0, 1, true, false, 64, false>;
            case 3: return (const void*)rt_render_kernel<B, 0, 1, true, false, 64, true>;
            case 4:                                     // the achromatic (one-channel) instances of 0 and 1
                if constexpr (RT_ACHRO && B <= RT_ACHRO_MAX_B) {
                    if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0 && use_sg8<B, true>())
                        return (const void*)rt_render_kernel_sg8<B, kFast, false, false, true>;
                    else if constexpr (B <= RT_SG_MAX_B && RT_FAST_SGPRS > 0)
                        return (const void*)rt_render_kernel_sg<B, kFast, false, false, true>;
                    else return (const void*)rt_render_kernel<B, 0, kFast, false, false, RT_WG_FAST, false, false, false, true>;
                }
                return nullptr;
            case 5:
                if constexpr (RT_ACHRO && B <= RT_ACHRO_MAX_B)
                    return (const void*)rt_render_kernel<B, 0, kCull, false, true, RT_WG_FAST, false, false,
                                                         (bool)RT_CULL_FIX64, true>;
                return nullptr;
            default: return nullptr;
        }
    }
}

}  // namespace rtk

// One line per instance file: the depth-B definitions of the three declarations above.
#define RT_RENDER_INSTANCES(B)                                                                                  \
    namespace rtk {                                                                                            \
    template <>                                                                                                \
    hipError_t launch_render<B>(const RenderLaunch& L) { return launch_render_impl<B>(L); }                    \
    template <>                                                                                                \
    hipError_t launch_trace_rays<B>(int v, dim3 g, hipStream_t st, const DevScene* s, const double* a,         \
                                    const double* b, int n, double* rgb, uint32_t* rc, const ScreenArgs& sa) { \
        return launch_trace_rays_impl<B>(v, g, st, s, a, b, n, rgb, rc, sa);                                   \
    }                                                                                                          \
    template <>                                                                                                \
    const void* render_kernel_ptr<B>(int v) { return render_kernel_ptr_impl<B>(v); }                           \
    }
