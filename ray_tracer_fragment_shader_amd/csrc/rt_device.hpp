// rt_device.hpp — FP64 device math and the per-ray tracer of the MI355X path.
//
// Every value that reaches the image is computed with the reference's exact IEEE binary64 operation
// order; the file is compiled with -ffp-contract=off so no a*b+c is fused.
// Citations are into /root/reference/Hw4/MySdlApplication.cpp.
//
// Restatement choices, each bit-identical to the reference (argued at its use):
//  * u = normalize(end - start) is computed once per ray, not once per child (Line::direction :258-263
//    recomputes the same expression on the same inputs);
//  * the closest-hit search keeps (distance, child, point); normal / reflection / material are computed
//    once for the winner (pure functions of the winner's point);
//  * the board's two triangles share vertex 0 and normal, so the plane step (m, p, w) is done once;
//  * shadow rays stop at the first blocker (any-hit): rayTraceRay reads only intersects() and the
//    blocker's transparency (:1221), and the GPU path only accepts opaque materials;
//  * the recursion (:1238-1247) is a loop; with opacity (1,1,1) the colour of level k is
//    local[k] + colour[k+1], so the frame colour is the right-nested sum local[0] + (local[1] + ...);
//  * for primary rays p0 = eye for every pixel, so deltaP = C - eye and dot(deltaP, deltaP) (:740, :750)
//    are computed once per workgroup, with the same operations, instead of once per ray;
// and work-skipping tests that are exact:
//  * FP32 sphere filter: a sphere is skipped only when an FP32 evaluation of the discriminant with a
//    proven error margin shows disc < 0, i.e. the FP64 test would report a miss (sphere_reject32);
//  * board: m = num/nd and s = A/den, t = B/den are divided only when the sign of the operands leaves the
//    quotient's sign test open (board_hit);
//  * bounding sphere: an origin with |o - c|^2 < (R-1)^2 provably passes the cull (bound_pass);
//  * shadow rays: a sphere is tested only if the ray's line through the light can meet it (light-cone
//    records, occluded);
//  * per-wave culling (>= kConeMin spheres): spheres no ray of the wave can reach, by a conservative
//    bound on the wave's rays (primary_cone_mask, ray_bundle_mask, shadow_bundle_mask);
// and exact arithmetic shortcuts:
//  * |v| and v / |v| without the scale/fixup steps of the IEEE sequences where they are identities, one
//    reciprocal shared by the three quotients (unit, len_fast).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.hpp"

// 1 (r06): the exact sqrt / quotient fast paths run unconditionally and their rare slow paths sit behind one
// wave-uniform ballot branch (sqrt_fast, div_const, unit) instead of an exec-mask region per call site — fewer
// scalar-stream instructions (in-process A/B c2 -4.5%, c3 -3.9%, c5 -5.5%, profiles/r06/ab; r02 measured +-0.8%).
#ifndef RT_FAST_FALLBACK
#define RT_FAST_FALLBACK 1
#endif
// 1: the exact tests of a filter batch visit its spheres in a loop the whole wave runs (record index
// wave-uniform: scalar loads, SGPR operands; lanes whose filter rejected a sphere are masked off);
// 0: each lane walks its own surviving spheres (per-lane index: vector loads).
#ifndef RT_UNIFORM_PRIMARY
#define RT_UNIFORM_PRIMARY 1
#endif
#ifndef RT_UNIFORM_SECONDARY
#define RT_UNIFORM_SECONDARY 1
#endif
#ifndef RT_UNIFORM_SHADOW
#define RT_UNIFORM_SHADOW 0
#endif
// 1: the fast (non-CULL) bounce loop keeps the continuation's unit direction live through the light loop;
// 0: it is recomputed after it (fewer live registers).
#ifndef RT_KEEP_NU
#define RT_KEEP_NU 0
#endif
// 1: the fast loop also parks the continuation's unit direction (computed before the light loop) in the
// next level's LDS slot instead of recomputing it after the light loop (RT_KEEP_NU without the registers).
#ifndef RT_PARK_NU
#define RT_PARK_NU 1
#endif
// The same for the CULL variant's levels (and its end - start, in this level's slot).
#ifndef RT_PARK_NU_CULL
#define RT_PARK_NU_CULL 1
#endif
// The fast loop parks the continuation's end - start in the level's (still empty) LDS colour slot while
// the light loop runs (fewer live registers) and reloads it for the next ray: at depth >= RT_PARK_ND_MIN_B.
#ifndef RT_PARK_ND_MIN_B
#define RT_PARK_ND_MIN_B RT_SKIP_FAST_MIN_B
#endif
// 1: rays that start at a hit point skip the bounding-sphere cull when the host proved every hit point
// lies inside its shortcut radius (DevScene::hits_inside).
#ifndef RT_HITS_INSIDE
#define RT_HITS_INSIDE 1
#endif
// 1: the bounce loop of trace() is unrolled (one copy of the level code per level); 0: a loop (one copy).
#ifndef RT_UNROLL_LEVELS
#define RT_UNROLL_LEVELS 1
#endif
// A/B only: 0 reads the per-eye flag from the scene header at each use (wrong for ray lists)
#ifndef RT_HITS_VIEW
#define RT_HITS_VIEW 1
#endif
// 1: rays that start at a board hit skip the board test, rays that start at a sphere hit that sphere's test
// (certain misses, origin_skip).
#ifndef RT_BOARD_SKIP
#define RT_BOARD_SKIP 1
#endif
#ifndef RT_SELF_SKIP
#define RT_SELF_SKIP 1
#endif
// The skips in the fast (non-CULL) bounce loop from this depth on (they always run in the CULL variant).
// There they come with the continuation parked in LDS across the light loop (RT_PARK_ND): without it the
// extra live state spilled 12 B/lane at 6 waves/SIMD (c2 HBM writes 1.01x -> 1.22x); with it no spills,
// c3 (depth 2) -1.2 to -1.9%, c2 (depth 1) +0.7 to +1.1% (r02, in-process A/B) — hence depth >= 2 until r04.  The
// 7-wave depth-1 kernel (94 SGPRs, 65 VGPRs, no scratch) gains from them: c2 -1.9% serial, -0.5% with 3 frames
// in flight (r04, in-process A/B; the skips alone -1.4%, the parking alone +0.8%) — hence depth >= 1.
// 1: closest-hit distances are computed only when two candidates meet (take_closer).
#ifndef RT_LAZY_DIST
#define RT_LAZY_DIST 1
#endif
// 1: primary rays that hit an object skip the bounding-sphere cull when the eye's per-eye flag proves they pass it.
#ifndef RT_PRIM_BOUND_SKIP
#define RT_PRIM_BOUND_SKIP 1
#endif
// 1: the reference's board is decided by the hit point's position in its square where that is certain (board_hit).
#ifndef RT_BOARD_POS
#define RT_BOARD_POS 1
#endif
// 1: primary rays of waves whose cone mask keeps no sphere normalise their direction only where they hit the board.
#ifndef RT_LAZY_PRIMARY_U
#define RT_LAZY_PRIMARY_U 1
#endif
#ifndef RT_SKIP_FAST_MIN_B
#define RT_SKIP_FAST_MIN_B 1
#endif

// 1: diagnostic build (tools/counters.py): wave-level event counters in DevScene::counters.
#ifndef RT_COUNTERS
#define RT_COUNTERS 0
#endif

namespace rt {

// Counter slots of RT_COUNTERS builds.
enum Counter {
    kCntWaves = 0, kCntConeKept, kCntRayMasks, kCntRayKept, kCntShadowMasks, kCntShadowKept, kCntExactRay,
    kCntExactShadow, kCntBoardShadow, kCntLevels, kCntExactPrimary, kCntFilterRay, kCntFilterShadow,
    // active lanes (sum over the counted wave events) of the same events, and of the culling levels' live / hit lanes
    kCntLanesFilterRay, kCntLanesExactRay, kCntLanesFilterShadow, kCntLanesExactShadow, kCntLanesLevelAlive,
    kCntLanesLevelHit, kCntCount
};

struct d3 {
    double x, y, z;
};

__device__ __forceinline__ d3 mk(double x, double y, double z) { return d3{x, y, z}; }
__device__ __forceinline__ d3 add(d3 a, d3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }     // :196-197
__device__ __forceinline__ d3 sub(d3 a, d3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }     // :199-200
__device__ __forceinline__ d3 scl(double s, d3 a) { return mk(s * a.x, s * a.y, s * a.z); }       // :1118-1131
__device__ __forceinline__ d3 had(d3 a, d3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }     // :192-193
__device__ __forceinline__ double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }   // :189-190
__device__ __forceinline__ double len(d3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }  // :174
__device__ __forceinline__ d3 divs(d3 a, double l) { return mk(a.x / l, a.y / l, a.z / l); }      // :175
__device__ __forceinline__ d3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }

// ------------------------------------------------------------------------------------------------
// Exact fast paths for |v| and v / |v|.
// The compiler lowers IEEE sqrt and division on gfx950 to these sequences (lib/isa/rt_kernel.s):
//   sqrt(x): x < 2^-767 is scaled by 2^256; y = rsq(x); g = x y; h = y / 2; r = fma(-h, g, 1/2);
//            g = fma(g, r, g); d = fma(-g, g, x); h = fma(h, r, h); g = fma(d, h, g); d = fma(-g, g, x);
//            g = fma(d, h, g); unscale; x in {+0, -0, +inf} returns x.
//   a / b:   b' = div_scale(b); r = rcp(b'); e = fma(-b', r, 1); r = fma(r, e, r); e = fma(-b', r, 1);
//            r = fma(r, e, r); a' = div_scale(a); q = a' r; e = fma(-b', q, a'); q = div_fmas(e, r, q);
//            div_fixup(q, b, a).
// For operands away from the scaling and special-value thresholds the scale, class and fixup steps are
// identities (fixup returns |q| with the sign of a XOR b; for a = +-0 it returns that signed zero), so
// the remaining operations, run here explicitly, give the same bits.  Each fast path checks its
// operands and takes the compiler's sequence otherwise:
//   sqrt_core: 2^-700 <= x <= 2^700 (no scaling: x >= 2^-767; finite, nonzero);
//   unit():    s = |v|^2 in [2^-700, 2^700], so l = sqrt(s) in [2^-350, 2^350] (l and 1/l normal), and
//              every component 0 or |v_i| >= 2^-500 (no numerator scaling: |v_i| >= 2^-969, quotient
//              >= 2^-850 normal, |v_i| <= l (1 + 2^-50) so exponent(v_i) - exponent(l) <= 1 < 768).
//              The three quotients share the reciprocal r (it depends on b only) — the compiler emits
//              it three times — and l > 0 makes the fixup's sign that of v_i (copysign).
// tests/test_gpu_parity.py::test_math_fast_paths checks both against the compiler's sqrt and division
// (and numpy's binary64) on adversarial operands through rt_probe_math_dev (include/rt_diag.h).
__device__ __forceinline__ double sqrt_core(double x) {
    double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    double r = fma(-h, g, 0.5);
    g = fma(g, r, g);
    double d = fma(-g, g, x);
    h = fma(h, r, h);
    g = fma(d, h, g);
    d = fma(-g, g, x);
    return fma(d, h, g);
}

// The range checks are evaluated without short-circuits (& and | on bools: compares combined in SGPR
// masks, no exec-mask branches), and the rare fallback is one wave-uniform branch taken only when some lane
// needs it (RT_FAST_FALLBACK).
__device__ __forceinline__ bool sqrt_fast_ok(double x) { return (x >= 0x1p-700) & (x <= 0x1p+700); }

// True when some active lane of the wave has `bad` set (the fast paths' fallback branch).
__device__ __forceinline__ bool any_lane(bool bad) { return __ballot(bad) != 0; }

__device__ __forceinline__ double rcp_core(double b) {
    double r = __builtin_amdgcn_rcp(b);
    double e = fma(-b, r, 1.0);
    r = fma(r, e, r);
    e = fma(-b, r, 1.0);
    return fma(r, e, r);
}

__device__ __forceinline__ double div_core(double a, double b, double r) {
    double q = a * r;
    double e = fma(-b, q, a);
    return fma(e, r, q);
}

__device__ __forceinline__ bool num_fast_ok(double a) { return (a == 0.0) | (fabs(a) >= 0x1p-500); }

// a / b for a constant b with r = rcp_core(b) precomputed on the device (rt_scene_init_kernel).  `fast`
// (host): |b| in [2^-200, 2^200]; then for |a| in [2^-500, 2^500] the quotient's exponent is within
// [-700, 700] and exponent(a) - exponent(b) <= 700 < 768, so the sequence's div_scale steps are identities
// and div_core is the IEEE quotient bit for bit (fast paths above); other operands (zero, tiny, huge,
// NaN) take the compiler's division.
__device__ __forceinline__ double div_const(double a, double b, double r, int32_t fast) {
#if RT_FAST_FALLBACK
    const double aa = fabs(a);
    const bool ok = (fast != 0) & (aa >= 0x1p-500) & (aa <= 0x1p+500);
    double q = div_core(a, b, r);
    if (any_lane(!ok)) q = ok ? q : a / b;
    return q;
#else
    const double aa = fabs(a);
    if (fast && aa >= 0x1p-500 && aa <= 0x1p+500) return div_core(a, b, r);
    return a / b;
#endif
}

// The compiler's IEEE sqrt sequence on gfx950, restated op for op (same bits for every input): x below 2^-767
// is scaled by 2^256, sqrt_core, the result scaled by 2^-128, and +-0 / +inf return the (scaled) input.  Its
// constants (256, -128, the class mask) come from opaque SGPR moves: the compiler's own expansion hoisted them
// out of the bounce loop into three VGPRs held across the whole kernel for this rarely taken path, which cost
// the register headroom of a seventh wave per SIMD at c2.
// RT_SQRT_IEEE_ASM=0 (experiment builds): the compiler's sqrt() instead; the c5 culling kernel then needs
// 83 VGPRs (5 waves per SIMD) and runs +6% (same-box A/B).
#ifndef RT_SQRT_IEEE_ASM
#define RT_SQRT_IEEE_ASM 1
#endif
__device__ __forceinline__ double sqrt_ieee(double x) {
#if !RT_SQRT_IEEE_ASM
    return sqrt(x);
#endif
    int up, down, cls;
    asm volatile("s_mov_b32 %0, 0x100" : "=s"(up));
    asm volatile("s_mov_b32 %0, 0xffffff80" : "=s"(down));
    asm volatile("s_mov_b32 %0, 0x260" : "=s"(cls));          // class: -0, +0, +inf
    const bool small = x < 0x1p-767;
    const double xs = __builtin_amdgcn_ldexp(x, small ? up : 0);
    const double g = __builtin_amdgcn_ldexp(sqrt_core(xs), small ? down : 0);
    return __builtin_amdgcn_class(xs, cls) ? xs : g;
}

// sqrt(x), bit-identical, with the fast sequence when it applies.
__device__ __forceinline__ double sqrt_fast(double x) {
#if RT_FAST_FALLBACK
    const bool ok = sqrt_fast_ok(x);
    double y = sqrt_core(x);
    if (any_lane(!ok)) y = ok ? y : sqrt_ieee(x);
    return y;
#else
    return sqrt_fast_ok(x) ? sqrt_core(x) : sqrt_ieee(x);
#endif
}

// |a| (= len(a), :174).
__device__ __forceinline__ double len_fast(d3 a) { return sqrt_fast(a.x * a.x + a.y * a.y + a.z * a.z); }

// u = a / |a| component-wise (= divs(a, len(a)), :174-175, Line::direction :258-263); *l = |a|.
__device__ __forceinline__ d3 unit(d3 a, double* l) {
    double s = a.x * a.x + a.y * a.y + a.z * a.z;
#if RT_FAST_FALLBACK
    const bool ok = sqrt_fast_ok(s) & num_fast_ok(a.x) & num_fast_ok(a.y) & num_fast_ok(a.z);
    double L = sqrt_core(s);
    double r = rcp_core(L);
    d3 u = mk(copysign(div_core(a.x, L, r), a.x), copysign(div_core(a.y, L, r), a.y),
              copysign(div_core(a.z, L, r), a.z));
    if (any_lane(!ok)) {
        if (!ok) {
            L = sqrt_ieee(s);
            u = divs(a, L);
        }
    }
    *l = L;
    return u;
#else
    if (sqrt_fast_ok(s) && num_fast_ok(a.x) && num_fast_ok(a.y) && num_fast_ok(a.z)) {
        double L = sqrt_core(s);
        double r = rcp_core(L);
        *l = L;
        return mk(copysign(div_core(a.x, L, r), a.x), copysign(div_core(a.y, L, r), a.y),
                  copysign(div_core(a.z, L, r), a.z));
    }
    double L = sqrt_ieee(s);
    *l = L;
    return divs(a, L);
#endif
}

__device__ __forceinline__ d3 unit(d3 a) {
    double l;
    return unit(a, &l);
}

// Where the kernels read the scene from.  `S`, `sph`, `prim` (header and FP64 exact records) live in
// LDS in the render kernel (or in global memory for the ray-list kernels); the FP32 filter images `sphf`,
// `primf` are always read from global memory with wave-uniform indices, i.e. through the scalar cache
// into SGPR operands.
// One count per wave (from its first active lane) in RT_COUNTERS builds.
#define RT_COUNT(S, slot, v)                                                                                   \
    do {                                                                                                       \
        if (RT_COUNTERS && (S)->counters && __lane_id() == __builtin_ctzll(__ballot(1)))                       \
            atomicAdd((S)->counters + (slot), (unsigned long long)(v));                                        \
    } while (0)
// ... of the lanes active at this point (lane utilisation = lanes / (64 x events))
// (the ballot is taken before RT_COUNT narrows the wave to one lane)
#define RT_COUNT_BALLOT(S, slot, pred)                                                                         \
    do {                                                                                                       \
        if (RT_COUNTERS) {                                                                                     \
            const unsigned long long n_ = __popcll(__ballot(pred));                                            \
            RT_COUNT(S, slot, n_);                                                                             \
        }                                                                                                      \
    } while (0)
#define RT_COUNT_LANES(S, slot) RT_COUNT_BALLOT(S, slot, 1)

struct SceneView {
    const DevScene* S;
    const DevSphere* sph;
    const DevSpherePrim* prim;
    const DevSphereF* sphf;
    const DevSpherePrimF* primf;
    const DevSphereCone* cone;       // [np] primary-ray cones (per eye)
    const DevSphereLightF* lightf;   // [nl][np] shadow-ray cone filter
    const DevMesh* mesh;             // global, wave-uniform reads
    const DevTri* tri;
    int np;                          // padded sphere count (wave-uniform)
    int ns;                          // stride of the per-sphere arrays (a constant in the fast kernels)
    int nl;                          // light count (wave-uniform)
    int nm;                          // mesh count (wave-uniform)
    int hits_ok;                     // rays from this kernel's hit points may skip the bounding-sphere cull
};

// Whether the hit points of rays from origin p0 (and of every later level) lie inside the bounding-sphere
// shortcut radius: the host proved that every object lies within R - 1 of bc with a slack that covers the
// rounding of hit points computed from origins up to sqrt(hits_lim2) away (DevScene::hits_lim2, rt_host.cpp).
// NaN origins fail the compare.
__device__ __forceinline__ int hits_ok_from(const DevScene* S, d3 p0) {
    const double dx = p0.x - S->bc[0], dy = p0.y - S->bc[1], dz = p0.z - S->bc[2];
    return (S->hits_inside != 0) & (dx * dx + dy * dy + dz * dz <= S->hits_lim2);
}

// hdr: header copy the kernel reads (LDS or global); g: the global record (for the filter images).  ns: the
// arrays' stride (DevScene::n_stride; the fast kernels pass the constant kFastStride, so every record address is
// the scene pointer plus a constant).
__device__ __forceinline__ SceneView view_of(const DevScene* hdr, const DevScene* g, int np, int ns, int nl) {
    SceneView v;
    v.S = hdr;
    v.np = np;
    v.ns = ns;
    v.nl = nl;
    v.sph = reinterpret_cast<const DevSphere*>(hdr + 1);
    v.prim = reinterpret_cast<const DevSpherePrim*>(v.sph + ns);
    const DevSphere* gsph = reinterpret_cast<const DevSphere*>(g + 1);
    const DevSpherePrim* gprim = reinterpret_cast<const DevSpherePrim*>(gsph + ns);
    v.sphf = reinterpret_cast<const DevSphereF*>(gprim + ns);
    v.primf = reinterpret_cast<const DevSpherePrimF*>(v.sphf + ns);
    v.cone = reinterpret_cast<const DevSphereCone*>(v.primf + ns);
    v.lightf = reinterpret_cast<const DevSphereLightF*>(v.cone + ns);
    v.mesh = reinterpret_cast<const DevMesh*>(v.lightf + (size_t)nl * ns);
    v.nm = g->n_meshes;
    v.tri = reinterpret_cast<const DevTri*>(v.mesh + v.nm);
    v.hits_ok = hdr->hits_ok;        // for the camera eye (rt_prepare_kernel); ray lists set it per ray
    return v;
}

// Hit kinds: -1 miss, 0 board, 1 + k sphere k, kMeshKind + 16 m + t mesh m's triangle t.
constexpr int kMeshKind = 1 << 20;

// A ray Line(p0, p0 + d) with u = normalize(d), plus its FP32 filter image.
struct Ray {
    d3 p0, d, u;
    float px, py, pz;    // f32(p0 - bound centre)
    float ux, uy, uz;    // f32(u)
    float mP;            // 4K * max|p_i|^2 (the ray's share of the filter margin)
};

__device__ __forceinline__ void set_origin_f32(const DevScene* S, Ray* r) {
    r->px = (float)(r->p0.x - S->bc[0]);
    r->py = (float)(r->p0.y - S->bc[1]);
    r->pz = (float)(r->p0.z - S->bc[2]);
    float sp = fmaxf(fabsf(r->px), fmaxf(fabsf(r->py), fabsf(r->pz)));
    r->mP = 4.0f * kFilterK * sp * sp;
}

__device__ __forceinline__ void set_dir(Ray* r, d3 d, d3 u) {
    r->d = d;
    r->u = u;
    r->ux = (float)u.x;
    r->uy = (float)u.y;
    r->uz = (float)u.z;
}

// ------------------------------------------------------------------------------------------------
// g_scene bounding-sphere cull (:747-758): miss iff disc < 0 or |s| < eps.
// Shortcut: if dd = |bc - p0|^2 < (R-1)^2 the cull passes.  Proof: m = R^2 - dd >= 2R - 1 > 0, so
// disc = uD^2 + m > 0 and s = uD - sqrt(disc) < 0 with |s| = m / (sqrt(uD^2 + m) + uD) >= m / (R + |dP|)
// >= (2R - 1) / (2R - 1) = 1 >> eps (sqrt(uD^2 + m) <= R since uD^2 <= dd); FP64 rounding is ~1e-13.
__device__ __forceinline__ bool bound_pass_dp(const DevScene* S, d3 dP, double dd, d3 u) {
    if (!S->bound_on) return true;
    if (dd < S->inner2) return true;
    double uD = dot(u, dP);
    double disc = uD * uD - dd + S->br2;
    if (disc < 0) return false;
    double s = uD - sqrt_fast(disc);
    return !(fabs(s) < S->eps);
}

__device__ __forceinline__ bool bound_pass(const DevScene* S, d3 p0, d3 u) {
    if (!S->bound_on) return true;
    d3 dP = sub(ld3(S->bc), p0);
    return bound_pass_dp(S, dP, dot(dP, dP), u);
}

// CheckerBoard -> Quad -> Triangle T1 then T2, first hit wins (:1097, :817, :611-707).
// d = end - start (unnormalised, :647).  Returns the hit point in *p.  PRIMARY: p0 is the camera eye and
// the numerator n . (v0 - eye) was computed for it by rt_prepare_kernel with the same operations.
// RT_BOARD_FLAT=1: the same decisions with one divergent region per outcome instead of one per early return (the
// sign tests and the numerator evaluated for every lane, the position decision and the exact triangles folded into
// one hit flag): fewer exec-mask save / restore pairs in the scalar stream (DESIGN.md §9, c2 SALU attribution).
#ifndef RT_BOARD_FLAT
#define RT_BOARD_FLAT 1
#endif
#if RT_BOARD_FLAT
template <bool PRIMARY = false>
__device__ __forceinline__ bool board_hit(const DevScene* S, d3 p0, d3 d, d3* p) {
    const DevTri& T = S->tri[0];
    d3 n = ld3(T.n);
    double nd = dot(n, d);                                  // :648
    d3 v0 = ld3(T.v0);
    double num = PRIMARY ? S->board_num : dot(n, sub(v0, p0));   // :657 numerator
    // :651 and the sign half of :659 (m = num / nd <= 0 misses), as in the branchy version below
    const bool live = !(fabs(nd) < S->eps) & !((num == 0.0) | ((num < 0.0) != (nd < 0.0)));
    bool hit = false;
    if (live) {
        double m = num / nd;                                // :657
#if RT_BOARD_FLAT >= 2
        // (:659's m < eps folded into the decision below: one region less; the hit point of such a lane is unused)
        const bool far_enough = !(m < S->eps);
        {
#else
        if (!(m < S->eps)) {                                // :659
#endif
            d3 q = add(p0, scl(m, d));                      // :665
            d3 w = sub(q, v0);                              // :667
            bool decided = false;
#if RT_BOARD_POS
            if (S->board_fast) {                            // (the position decision of the branchy version)
                const double wx = w.x, wz = w.z, lo = S->board_lo, hi = S->board_hi, diag = fabs(wx - wz);
                const double far = S->board_far, out = S->board_out, ax = fabs(wx), az = fabs(wz);
                const bool in = (wx >= lo) & (wz >= lo) & (wx <= hi) & (wz <= hi) & (diag >= lo);
                const bool outside = (ax <= far) & (az <= far) & ((wx <= -lo) | (wz <= -lo) | (wx >= out) | (wz >= out));
                hit = in;
                decided = in | outside;
            }
#endif
#if RT_BOARD_FLAT >= 2
            hit &= far_enough;
            decided |= !far_enough;
#endif
            if (!decided) {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const DevTri& Tt = S->tri[t];
                    double wu = dot(w, ld3(Tt.u));          // :670
                    double wv = dot(w, ld3(Tt.v));          // :671
                    double A = Tt.uv * wv - Tt.vv * wu;
                    double B = Tt.uv * wu - Tt.uu * wv;
                    if (!hit & !(A > Tt.thr || B > Tt.thr)) {
                        double s = div_const(A, Tt.den, Tt.rden, Tt.fast);   // :673
                        double tt = div_const(B, Tt.den, Tt.rden, Tt.fast);  // :674
                        hit = (s >= 0) & (tt >= 0) & (s + tt <= 1);          // :676
                    }
                }
            }
            if (hit) *p = q;
        }
    }
    return hit;
}
#else
template <bool PRIMARY = false>
__device__ __forceinline__ bool board_hit(const DevScene* S, d3 p0, d3 d, d3* p) {
    const DevTri& T = S->tri[0];
    d3 n = ld3(T.n);
    double nd = dot(n, d);                                  // :648
    if (fabs(nd) < S->eps) return false;                    // :651
    d3 v0 = ld3(T.v0);
    double num = PRIMARY ? S->board_num : dot(n, sub(v0, p0));   // :657 numerator
    // m = num / nd is <= 0 (hence < eps, a miss at :659) when num == 0 or the signs differ.  NaNs fall
    // through to the division and miss there, as in the reference.
    if (num == 0.0 || ((num < 0.0) != (nd < 0.0))) return false;
    double m = num / nd;                                    // :657 (its denominator recomputed: same value)
    if (m < S->eps) return false;                           // :659
    d3 q = add(p0, scl(m, d));                              // :665
    d3 w = sub(q, v0);                                      // :667
#if RT_BOARD_POS
    // The reference's board (host: board_fast) decided by the position of w in its square, where that is certain.
    // With L the side, T1 = (P1, P2, P3) and T2 = (P1, P3, P4) give, in exact arithmetic on the computed w,
    //   T1: s = (wx - wz) / L, t = wz / L;   T2: s = wx / L, t = (wz - wx) / L
    // (uu, uv, vv, den are exact for an integer L <= 2^12, the products with u's and v's zero components vanish),
    // and the reference's rounded s, t (:670-674) err by less than E = 64 u (|wx| + |wz|) / L + 4 u (u = 2^-53: two
    // roundings per dot product, three in A and B, one quotient).  For |wx|, |wz| <= far = 2^24 L, E < 2^-22 + 2^-51;
    // the margin delta = L 2^-19 keeps every decision below at least delta / (2L) = 2^-20 > 2E + u |s + t| away:
    //  * delta <= wx, wz <= L - delta and |wx - wz| >= delta: the triangle on w's side of the diagonal has
    //    s, t >= delta / L and s + t <= 1 - delta / L — it passes (:676), a hit at q;
    //  * wx <= -delta, wz <= -delta, wx >= L + delta or wz >= L + delta: each triangle fails one of its three tests
    //    by >= delta / (2L) (e.g. wx <= -delta: T2's s < 0, and T1's s + t = wx / L < 0 puts s or t below -delta/(2L)).
    // Everything else — within delta of an edge or the diagonal, |w| beyond `far`, NaN — takes the exact tests.
    if (S->board_fast) {
        const double wx = w.x, wz = w.z, lo = S->board_lo, hi = S->board_hi, diag = fabs(wx - wz);
        if ((wx >= lo) & (wz >= lo) & (wx <= hi) & (wz <= hi) & (diag >= lo)) {
            *p = q;
            return true;
        }
        const double far = S->board_far, out = S->board_out, ax = fabs(wx), az = fabs(wz);
        if ((ax <= far) & (az <= far) & ((wx <= -lo) | (wz <= -lo) | (wx >= out) | (wz >= out))) return false;
    }
#endif
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const DevTri& Tt = S->tri[t];
        double wu = dot(w, ld3(Tt.u));                      // :670
        double wv = dot(w, ld3(Tt.v));                      // :671
        double A = Tt.uv * wv - Tt.vv * wu;
        double B = Tt.uv * wu - Tt.uu * wv;
        // den < 0 (host-checked, else thr = +inf): A > thr = |den| 2^-1070 makes A/den negative and nonzero,
        // so s >= 0 fails without dividing; likewise B for t.
        if (A > Tt.thr || B > Tt.thr) continue;
        double s = div_const(A, Tt.den, Tt.rden, Tt.fast);  // :673
        double tt = div_const(B, Tt.den, Tt.rden, Tt.fast); // :674
        if (s >= 0 && tt >= 0 && s + tt <= 1) {             // :676
            *p = q;
            return true;
        }
    }
    return false;
}

#endif

// Tests that a ray starting at the hit point q of the previous level certainly misses (exact skips):
//  * the board, when q is a board hit of a ray from p0.  The board normal is exactly (0, -1, 0) (host-
//    checked), so num = n . (v0 - q) = -(v0.y - q.y) with q.y = p0.y + m0 d0.y rounded, m0 = num0 / nd0
//    rounded: |num| <= 2^-50 (3 |p0.y| + 5 |v0.y| + 1) < eps^2 / 2 whenever |p0.y| <= board_skip_y
//    (host).  board_hit misses unless |nd| >= eps, and then |m| = |num / nd| (1 + 2^-53) < eps: the m < eps
//    test (:659) misses.
//  * sphere k, when q is a hit of sphere k.  Any ray from q has dP = C - q, dd = |dP|^2 (computed here with
//    the same operations) and |uD| <= sqrt(dd) (1 + 2^-50), so disc = fl(fl(uD^2 - dd) + r2) is within
//    E = 2^-49 (dd + r2) of uD^2 + g, g = r2 - dd.  uD < 0 gives s < 0; otherwise
//    |s| <= sqrt(|g| + E) + 2^-51 sqrt(dd + r2) < eps when |g| + E < eps^2 / 4 (self_eps2): the near root
//    misses (:754, :767) — the reference never uses the far root.
// NaN / inf operands fail the compares (no skip).  Returns -1 (no skip), 0 (board) or 1 + k (sphere k).
__device__ __forceinline__ int origin_skip(const SceneView& V, int kind, d3 p0, d3 q) {
    const DevScene* S = V.S;
    if (RT_BOARD_SKIP && kind == 0) return fabs(p0.y) <= S->board_skip_y ? 0 : -1;
    if (RT_SELF_SKIP && kind >= 1 && kind < kMeshKind) {
        const DevSphere& sp = V.sph[kind - 1];
        const d3 dP = sub(ld3(sp.c), q);
        const double dd = dot(dP, dP);
        return fabs(sp.r2 - dd) + 0x1p-49 * (dd + sp.r2) < S->self_eps2 ? kind : -1;
    }
    return -1;
}

// Clears sphere `self` (origin_skip - 1) from the pass bits of the batch starting at k0.
__device__ __forceinline__ uint32_t drop_self(uint32_t pass, int self, int k0) {
    return (unsigned)(self - k0) < (unsigned)kChunk ? pass & ~(1u << (self - k0)) : pass;
}

// Triangle::intersection (:611-707) on a mesh triangle, with the same division-skipping sign tests as
// board_hit.  d = end - start (unnormalised).
__device__ __forceinline__ bool tri_hit(const DevTri& T, d3 p0, d3 d, double eps, d3* p) {
    if (T.degenerate != 0.0) return false;                  // :633-637
    d3 n = ld3(T.n);
    double nd = dot(n, d);                                  // :648
    if (fabs(nd) < eps) return false;                       // :651
    d3 v0 = ld3(T.v0);
    double num = dot(n, sub(v0, p0));
    if (num == 0.0 || ((num < 0.0) != (nd < 0.0))) return false;
    double m = num / nd;                                    // :657
    if (m < eps) return false;                              // :659
    d3 q = add(p0, scl(m, d));                              // :665
    d3 w = sub(q, v0);                                      // :667
    double wu = dot(w, ld3(T.u));
    double wv = dot(w, ld3(T.v));
    double A = T.uv * wv - T.vv * wu;
    double B = T.uv * wu - T.uu * wv;
    if (A > T.thr || B > T.thr) return false;
    double s = div_const(A, T.den, T.rden, T.fast);         // :673
    double tt = div_const(B, T.den, T.rden, T.fast);        // :674
    if (s >= 0 && tt >= 0 && s + tt <= 1) {                 // :676
        *p = q;
        return true;
    }
    return false;
}

// A mesh's own bounding-sphere cull (Shape::intersection with radius > 0, :747-758).
__device__ __forceinline__ bool mesh_bound(const DevMesh& M, d3 p0, d3 u, double eps) {
    d3 dP = sub(ld3(M.bc), p0);
    double dd = dot(dP, dP);
    if (dd < M.inner2) return true;
    double uD = dot(u, dP);
    double disc = uD * uD - dd + M.br2;
    if (disc < 0) return false;
    double s = uD - sqrt_fast(disc);
    return !(fabs(s) < eps);
}

// The mesh's closest sub-object hit (strict <, in sub-object order; a cube face is a Quad: its second
// triangle is tested only if the first misses, :817).  Returns the triangle index or -1.
__device__ __forceinline__ int mesh_closest_tri(const SceneView& V, const DevMesh& M, d3 p0, d3 d, double eps,
                                                double* mbest, d3* mq) {
    int mt = -1;
    *mbest = -1.0;
    for (int f = 0; f < M.nfaces; ++f) {
        int t = M.tri0 + f * M.per_face;
        d3 q;
        bool h = tri_hit(V.tri[t], p0, d, eps, &q);
        if (!h && M.per_face == 2) {
            ++t;
            h = tri_hit(V.tri[t], p0, d, eps, &q);
        }
        if (h) {
            double dist = len_fast(sub(q, p0));
            if (dist < *mbest || *mbest < 0.0) {
                *mbest = dist;
                mt = t;
                *mq = q;
            }
        }
    }
    return mt;
}

// Position of a hit kind in g_scene's child list (only evaluated on exact distance ties).
__device__ __forceinline__ int child_of(const SceneView& V, int kind) {
    const int hb = V.S->has_board ? 1 : 0;
    if (kind == 0) return 0;
    if (kind >= kMeshKind) return V.mesh[(kind - kMeshKind) >> 4].child;
    const int k = kind - 1;
    int before = 0;
    for (int m = 0; m < V.nm; ++m) before += (V.mesh[m].child - hb - m) <= k ? 1 : 0;
    return hb + k + before;
}

// Meshes after the board and the spheres: (distance, child index) order = the reference's ordered
// strict-< walk over the child list.
__device__ __forceinline__ void meshes_closest(const SceneView& V, const Ray& r, double eps, int* kind,
                                               double* best, d3* hp) {
    for (int m = 0; m < V.nm; ++m) {
        const DevMesh& M = V.mesh[m];
        if (!mesh_bound(M, r.p0, r.u, eps)) continue;
        double mbest;
        d3 mq;
        int t = mesh_closest_tri(V, M, r.p0, r.d, eps, &mbest, &mq);
        if (t < 0) continue;
        // (a deferred distance of the current candidate, take_closer, is computed here)
        if (RT_LAZY_DIST && *kind >= 0 && *best < 0.0) *best = len_fast(sub(*hp, r.p0));
        if (mbest < *best || *kind < 0 || (mbest == *best && M.child < child_of(V, *kind))) {
            *best = mbest;
            *kind = kMeshKind + 16 * m + (t - M.tri0);
            *hp = mq;
        }
    }
}

// FP32 filter: true only if disc = uD^2 - |dP|^2 + r^2 < 0 is certain.
// Error budget (eps32 = 2^-24; S >= |c_i| + |p_i| per component, c, p relative to the bound centre):
// |d(dx)| <= 2 eps32 S; |d(uD)| <= 10.4 eps32 S; |d(uD^2)| <= 36 eps32 S^2; |d(dd)| <= 21 eps32 S^2;
// fma roundings <= 6 eps32 S^2 + eps32 r^2; total < 64 eps32 (S^2 + r^2) = (K/4)(S^2 + r^2).
// The margin folded into rm + mP is 4K(sC^2 + sp^2) + K r^2 >= 2K S^2 + K r^2, so a negative FP32
// value implies a negative exact discriminant.  Inf/NaN compare false and fall through to FP64.
__device__ __forceinline__ bool sphere_reject32(const DevSphereF& f, const Ray& r) {
    float dx = f.cx - r.px, dy = f.cy - r.py, dz = f.cz - r.pz;
    float e = f.rm + r.mP;
    e = fmaf(-dx, dx, e);
    e = fmaf(-dy, dy, e);
    e = fmaf(-dz, dz, e);
    float uD = r.ux * dx;
    uD = fmaf(r.uy, dy, uD);
    uD = fmaf(r.uz, dz, uD);
    return fmaf(uD, uD, e) < 0.0f;
}

// Sphere (:747-772), exact FP64: candidate point if disc >= 0 and s >= eps.
__device__ __forceinline__ bool sphere_hit_dp(d3 dP, double dd, double r2, d3 p0, d3 u, double eps, d3* p) {
    double uD = dot(u, dP);                                 // :749
    double disc = uD * uD - dd + r2;                        // :750
    if (disc < 0) return false;                             // :754
    double s = uD - sqrt_fast(disc);                             // :752
    if (s < eps) return false;                              // covers |s| < eps (:754) and s < eps (:767)
    *p = add(p0, scl(s, u));                                // :762
    return true;
}

__device__ __forceinline__ bool sphere_hit(const DevSphere& sp, d3 p0, d3 u, double eps, d3* p) {
    d3 dP = sub(ld3(sp.c), p0);                             // :740
    return sphere_hit_dp(dP, dot(dP, dP), sp.r2, p0, u, eps, p);
}

// Bits of the spheres a 64-bit mask may name: k < min(np, 64).
__device__ __forceinline__ uint64_t sphere_bits(int np) { return np >= 64 ? ~0ull : ((1ull << np) - 1); }

// The closest-hit update (:811-818) for candidate q of kind k: the reference keeps the first candidate and then
// one with a strictly smaller Euclidean distance |q - p0|.  Distances are compared only when two candidates meet,
// so they are computed only then (RT_LAZY_DIST): the first candidate's is deferred — *best < 0 with *kind >= 0
// means "not computed yet" — and a ray with a single candidate (most board and sphere hits) computes none.  The
// same comparisons on the same values: kind and hit point are unchanged, bit for bit (a NaN distance compares false
// either way, and a computed NaN best is never recomputed: NaN < 0 is false).
__device__ __forceinline__ void take_closer(d3 p0, d3 q, int k, int* kind, double* best, d3* hp) {
#if RT_LAZY_DIST
    if (*kind < 0) {
        *kind = k;
        *hp = q;
        return;
    }
    if (*best < 0.0) *best = len_fast(sub(*hp, p0));
    const double dist = len_fast(sub(q, p0));                // :811-812
    if (dist < *best) {                                      // :813
        *best = dist;
        *kind = k;
        *hp = q;
    }
#else
    const double dist = len_fast(sub(q, p0));
    if (dist < *best || *best < 0.0) {
        *best = dist;
        *kind = k;
        *hp = q;
    }
#endif
}

// Closest hit of g_scene (:796-821): Euclidean distance |p - p0|, strict <, board (child 0) first.
// kind: -1 miss, 0 board, 1 + k sphere k.
// Spheres go in batches of kChunk: the FP32 filter of the whole batch is evaluated branch-free (records
// in SGPRs), then each lane runs the exact FP64 test only on its own surviving spheres, in increasing k,
// so the strict-< closest-hit order of the reference is unchanged.  Padding spheres never survive.
#ifndef RT_SEC_PREFETCH
#define RT_SEC_PREFETCH 0
#endif
__device__ __forceinline__ void sphere_batch_closest(const SceneView& V, const Ray& r, int k0, double eps,
                                                     int* kind, double* best, d3* hp, int self = -1) {
    uint32_t pass = 0;
#if RT_SEC_PREFETCH
    // the batch's exact-test records requested with its filter records (one wait for all)
    DevSphere sp4[kChunk];
#pragma unroll
    for (int j = 0; j < kChunk; ++j) sp4[j] = V.sph[k0 + j];
    asm volatile("" ::"s"(sp4[0].r2), "s"(sp4[1].r2), "s"(sp4[2].r2), "s"(sp4[3].r2));
#endif
#pragma unroll
    for (int j = 0; j < kChunk; ++j) pass |= (sphere_reject32(V.sphf[k0 + j], r) ? 0u : 1u) << j;
    pass = drop_self(pass, self, k0);                       // r starts on sphere `self`: a certain miss
#if RT_UNIFORM_SECONDARY
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
        if (!(pass & (1u << j))) continue;                  // skipped by the wave when no lane needs it
        const int k = k0 + j;
#if RT_SEC_PREFETCH
        {
            d3 q;
            if (sphere_hit(sp4[j], r.p0, r.u, eps, &q)) take_closer(r.p0, q, 1 + k, kind, best, hp);
            continue;
        }
#endif
#else
    while (pass) {
        const int k = k0 + __builtin_ctz(pass);
        pass &= pass - 1;
#endif
        d3 q;
        if (sphere_hit(V.sph[k], r.p0, r.u, eps, &q)) take_closer(r.p0, q, 1 + k, kind, best, hp);   // :811-813
    }
}

// `mask` (np >= kConeMin): spheres k < 64 this wave's rays may hit (ray_bundle_mask); the rest of the
// first 64 are skipped.  Spheres are visited in increasing k either way.
// skip = origin_skip of r's origin: 0 skips the board test, 1 + k sphere k's (certain misses).
// from_hit: r starts at a hit point, which passes the cull when S->hits_inside (host-proven).
template <bool FULL, bool CULL = false>
__device__ __forceinline__ int closest_hit(const SceneView& V, const Ray& r, d3* hp, uint64_t mask = ~0ull,
                                           int skip = -1, bool from_hit = false) {
    const DevScene* S = V.S;
    if (!(RT_HITS_INSIDE && from_hit && (RT_HITS_VIEW ? V.hits_ok : S->hits_ok)) && !bound_pass(S, r.p0, r.u)) return -1;
    int kind = -1;
    double best = -1.0;
    if (S->has_board && skip != 0) {
        d3 q;
        if (board_hit(S, r.p0, r.d, &q)) take_closer(r.p0, q, 0, &kind, &best, hp);
    }
    const double eps = S->eps;
    int k0 = 0;
    if (CULL && V.np >= kConeMin) {
        for (uint64_t m = mask & sphere_bits(V.np); m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            RT_COUNT(S, kCntFilterRay, 1);
            RT_COUNT_LANES(S, kCntLanesFilterRay);
#if RT_PRIM_PREFETCH
            // the exact test's record with the filter's (one wait for both, as in primary_sphere)
            const DevSphereF sf = V.sphf[k];
            const DevSphere sp = V.sph[k];
            asm volatile("" ::"s"(sf.rm), "s"(sp.r2));
            if (k == skip - 1 || sphere_reject32(sf, r)) continue;
#else
            if (k == skip - 1 || sphere_reject32(V.sphf[k], r)) continue;
            const DevSphere& sp = V.sph[k];
#endif
            RT_COUNT(S, kCntExactRay, 1);
            RT_COUNT_LANES(S, kCntLanesExactRay);
            d3 q;
            if (sphere_hit(sp, r.p0, r.u, eps, &q)) take_closer(r.p0, q, 1 + k, &kind, &best, hp);   // :811-813
        }
        k0 = 64;
    }
    for (; k0 < V.np; k0 += kChunk) {
        // (a batch none of whose spheres the mask keeps is missed by every ray of the wave: the cached masks of the
        // fast kernels, LevelMasks; ~0 otherwise)
        if (k0 < 64 && ((mask >> k0) & ((1ull << kChunk) - 1)) == 0) continue;
        sphere_batch_closest(V, r, k0, eps, &kind, &best, hp, skip - 1);
    }
    if (FULL) meshes_closest(V, r, eps, &kind, &best, hp);
    return kind;
}

// Closest hit of a primary ray Line(eye, sp): deltaP and |deltaP|^2 per sphere were computed for this
// eye by rt_prepare_kernel with the reference's operations (:740, :750).  A miss of the bounding-sphere
// cull makes the whole g_scene a miss, whatever the children say, so it can be tested after them.
// One sphere of a primary ray: FP32 filter on the per-eye image, then the exact test (:747-772) and the
// strict-< closest-hit update (:811-813).
#ifndef RT_PRIM_PREFETCH
#define RT_PRIM_PREFETCH 0
#endif
__device__ __forceinline__ void primary_sphere(const SceneView& V, const Ray& r, int k, double eps, int* kind,
                                               double* best, d3* hp) {
    const DevSpherePrimF f = V.primf[k];
#if RT_PRIM_PREFETCH
    // The exact test's records are requested with the filter's (scalar loads, one wait for all): a sphere that
    // passes the filter then costs no second round trip to memory.
    const DevSpherePrim pp = V.prim[k];
    const double r2 = V.sph[k].r2;
    asm volatile("" ::"s"(f.c0), "s"(pp.dd), "s"(r2));
#endif
    float uD = r.ux * f.dx;
    uD = fmaf(r.uy, f.dy, uD);
    uD = fmaf(r.uz, f.dz, uD);
    if (fmaf(uD, uD, f.c0) < 0.0f) return;                  // certain disc < 0
#if !RT_PRIM_PREFETCH
    const DevSpherePrim& pp = V.prim[k];
    const double r2 = V.sph[k].r2;
#endif
    d3 q;
    RT_COUNT(V.S, kCntExactPrimary, 1);
    if (sphere_hit_dp(ld3(pp.dP), pp.dd, r2, r.p0, r.u, eps, &q)) take_closer(r.p0, q, 1 + k, kind, best, hp);
}

// Closest hit of a primary ray Line(eye, sp): deltaP and |deltaP|^2 per sphere were computed for this
// eye by rt_prepare_kernel with the reference's operations (:740, :750).  A miss of the bounding-sphere
// cull makes the whole g_scene a miss, whatever the children say, so it can be tested after them.  `cone` (np >= kConeMin): bit k
// set when sphere k < 64 may be hit by some ray of this wave (primary_cone_mask); the others are
// provably missed and skipped.  Spheres are still visited in increasing k (tie order unchanged).
// lazy_u (wave-uniform; trace): no sphere of the wave's cone mask is left (<= 64 spheres, all covered by the
// mask) and the scene has no meshes, so only
// the board can be hit and the direction u = unit(d) (the board test uses d) is computed here for the lanes that
// hit it — the rest miss and never read it.
template <bool FULL>
__device__ __forceinline__ int closest_hit_primary(const SceneView& V, Ray& r, uint64_t cone, d3* hp,
                                                   bool lazy_u = false) {
    const DevScene* S = V.S;
    int kind = -1;
    double best = -1.0;
    if (S->has_board) {
        d3 q;
        if (board_hit<true>(S, r.p0, r.d, &q)) take_closer(r.p0, q, 0, &kind, &best, hp);
    }
    const double eps = S->eps;
    int k0 = 0;
    if (V.np >= kPrimaryConeMin) {
        for (uint64_t m = cone & sphere_bits(V.np); m; m &= m - 1)
            primary_sphere(V, r, __builtin_ctzll(m), eps, &kind, &best, hp);
        k0 = 64;
    }
    for (; k0 < V.np; k0 += kChunk) {
        uint32_t pass = 0;
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const DevSpherePrimF& f = V.primf[k0 + j];
            float uD = r.ux * f.dx;
            uD = fmaf(r.uy, f.dy, uD);
            uD = fmaf(r.uz, f.dz, uD);
            pass |= (fmaf(uD, uD, f.c0) < 0.0f ? 0u : 1u) << j;   // < 0: certain disc < 0
        }
#if RT_UNIFORM_PRIMARY
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            if (!(pass & (1u << j))) continue;
            const int k = k0 + j;
#else
        while (pass) {
            const int k = k0 + __builtin_ctz(pass);
            pass &= pass - 1;
#endif
            const DevSpherePrim& pp = V.prim[k];
            d3 q;
            if (sphere_hit_dp(ld3(pp.dP), pp.dd, V.sph[k].r2, r.p0, r.u, eps, &q)) take_closer(r.p0, q, 1 + k, &kind, &best, hp);
        }
    }
    if (FULL) meshes_closest(V, r, eps, &kind, &best, hp);
    if (lazy_u && kind >= 0) set_dir(&r, r.d, unit(r.d));
    // The bounding-sphere cull (:747-758) only turns hits into misses, so it is evaluated last and only
    // for rays that hit something: waves of background rays skip it.
    // (deltaP = bc - eye, computed here for the waves that need it rather than held from the kernel's start)
    // (prim_bound_ok, per eye: every primary hit passes it — proof at rt_prepare_kernel)
    if (kind >= 0 && !(RT_PRIM_BOUND_SKIP && S->prim_bound_ok)) {
        const d3 bdP = sub(ld3(S->bc), r.p0);               // :740 with p0 = camera
        if (!bound_pass_dp(S, bdP, dot(bdP, bdP), r.u)) kind = -1;
    }
    return kind;
}

// chord(phi) = |x - y| for unit vectors at angle phi = asin(s): s sqrt(2 / (1 + sqrt(1 - s^2))).
__device__ __host__ __forceinline__ float chord_of_sin(float s) {
    return s * sqrtf(2.0f / (1.0f + sqrtf(fmaxf(0.0f, 1.0f - s * s))));
}

// FP32 square root and reciprocal of the wave-culling tests (RT_FAST_MASK = 1): the hardware instructions
// (v_sqrt_f32, v_rcp_f32, 1 ulp: relative error < 2^-22 on normal operands) instead of the correctly rounded
// sequences (scaling, Newton and fixup steps around them: ~10 instructions each).  The culling tests only need
// conservative bounds, and their margins (R inflated by 2^-12 relative, chord limits by 2^-14 absolute, shadow
// cones by 2^-16 in cos) are > 2^6 times the extra error; 0, +inf and NaN keep their meaning (sqrt(0) = 0,
// rcp(+inf) = 0, NaN propagates and fails the `>` compares, i.e. keeps the sphere).
#ifndef RT_FAST_MASK
#define RT_FAST_MASK 1                         // same-box A/B: c5 -5.7%, c2/c3 +-1%
#endif
__device__ __forceinline__ float msqrt(float x) {
#if RT_FAST_MASK
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
__device__ __forceinline__ float mrcp(float x) {
#if RT_FAST_MASK
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
__device__ __forceinline__ float mdiv(float a, float b) {
#if RT_FAST_MASK
    return a * __builtin_amdgcn_rcpf(b);
#else
    return a / b;
#endif
}
__device__ __forceinline__ float mchord_of_sin(float s) {
    return s * msqrt(mdiv(2.0f, 1.0f + msqrt(fmaxf(0.0f, 1.0f - s * s))));
}

// Per-wave culling of primary rays (V.np >= kConeMin; all 64 lanes must be active).  The wave's rays go
// from the eye through the screen points of its bw x bh block, all within R = half_diag pitch of the
// block centre c (half_diag = |((bw - 1) / 2, (bh - 1) / 2)|), hence (exact geometry) within angle asin(R / |c - eye|) of a = unit(c - eye): chord
// distance |u - a| <= rho.  A ray that hits sphere k has |u - v_k| <= chord_k (DevSphereCone, rounded
// up, radius inflated for FP64 rounding), so |a - v_k| <= rho + chord_k + slack, where `slack` (host,
// RenderParams) bounds the FP32 error of a and of the test itself.  Lane j evaluates sphere j; the
// ballot is the mask of spheres this wave must test.  NaNs keep the sphere.
__device__ __forceinline__ uint64_t primary_cone_mask(const SceneView& V, const float look[3],
                                                      const float right[3], const float upp[3],
                                                      const float eye[3], float pitch, float ci, float cj,
                                                      float half_diag, float slack, int lane) {
    const float a_r = pitch * ci, a_u = pitch * cj;
    float dx = fmaf(a_u, upp[0], fmaf(a_r, right[0], look[0])) - eye[0];
    float dy = fmaf(a_u, upp[1], fmaf(a_r, right[1], look[1])) - eye[1];
    float dz = fmaf(a_u, upp[2], fmaf(a_r, right[2], look[2])) - eye[2];
    const float dn = msqrt(fmaf(dx, dx, fmaf(dy, dy, dz * dz)));
    const float sn = mdiv((half_diag * 1.001f) * pitch, dn);
    if (!(sn < 0.5f)) return ~0ull;                         // eye too close to the screen: no culling
    const float rho = mchord_of_sin(sn) + slack;
    const float idn = mrcp(dn);
    dx *= idn, dy *= idn, dz *= idn;
    bool keep = false;
    if (lane < V.np) {
        const DevSphereCone& c = V.cone[lane];
        const float ex = dx - c.vx, ey = dy - c.vy, ez = dz - c.vz;
        const float lim = rho + c.chord;
        keep = !(fmaf(ex, ex, fmaf(ey, ey, ez * ez)) > lim * lim);
    }
    return __ballot(keep);
}

// ------------------------------------------------------------------------------------------------
// Wave-level culling of secondary and shadow rays (np >= kConeMin).  Called with all 64 lanes active;
// `on` marks the lanes whose ray the mask must cover.  Lane j evaluates sphere j (< 64) against the
// wave's bundle; the ballot is the mask of spheres to test.  Lanes whose ray has a non-finite
// coordinate widen the bundle to everything (the reference reports NaN rays as hits).

// max over the 64 lanes (DPP: quad permutes, row mirrors, row broadcasts; GFX9 encodings).
template <int CTRL, int ROWS = 0xF>
__device__ __forceinline__ float dpp_f32(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWS, 0xF, false));
}

__device__ __forceinline__ float wave_max(float v) {
    v = fmaxf(v, dpp_f32<0xB1>(v));                          // quad_perm [1,0,3,2]
    v = fmaxf(v, dpp_f32<0x4E>(v));                          // quad_perm [2,3,0,1]
    v = fmaxf(v, dpp_f32<0x141>(v));                         // row_half_mirror
    v = fmaxf(v, dpp_f32<0x140>(v));                         // row_mirror
    v = fmaxf(v, dpp_f32<0x142, 0xA>(v));                    // row_bcast:15 -> rows 1, 3
    v = fmaxf(v, dpp_f32<0x143, 0xC>(v));                    // row_bcast:31 -> rows 2, 3
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float lane_f32(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ float inf_if_nan(float v) { return v >= 0.0f ? v : __builtin_inff(); }

// Reflected / transmitted rays (p_l, u_l): o, a = origin and direction of the first `on` lane,
// rho_o >= |p_l - o|, rho_d >= |u_l - a| (chord).  A ray that hits sphere k (exact FP64 test) passes
// within r' of C_k (r'^2 = r^2 (1 + 2^-20) + D^2 2^-46 covers the test's rounding), so the ray from o
// with the same direction passes within R = r' + rho_o: either |C_k - o| <= R, or the angle between u_l
// and v = unit(C_k - o) is at most asin(R / |C_k - o|), i.e. |a - v| <= rho_d + chord(R / |C_k - o|).
// FP32 coordinates carry < 2^-20 relative error; R gets 2^-12 (|o| + |C| + 1) absolute and the chord
// test 2^-14 of slack.
#ifndef RT_CHEAP_BUNDLE
#define RT_CHEAP_BUNDLE 0
#endif
__device__ __forceinline__ uint64_t ray_bundle_part(const SceneView& V, bool on, const Ray& r, int f) {
    const int lane = __lane_id();
    const float ox = lane_f32(r.px, f), oy = lane_f32(r.py, f), oz = lane_f32(r.pz, f);
    const float ax = lane_f32(r.ux, f), ay = lane_f32(r.uy, f), az = lane_f32(r.uz, f);
    // squared spreads reduced, one square root on the maxima (sqrt is monotonic: the same rho as the max
    // of per-lane roots, with two transcendental instructions per lane fewer)
    float dp = 0.0f, du = 0.0f;
    if (on) {
        const float px = r.px - ox, py = r.py - oy, pz = r.pz - oz;
        const float ux = r.ux - ax, uy = r.uy - ay, uz = r.uz - az;
        dp = inf_if_nan(fmaf(px, px, fmaf(py, py, pz * pz)));
        du = inf_if_nan(fmaf(ux, ux, fmaf(uy, uy, uz * uz)));
    }
    const float rho_o = msqrt(wave_max(dp)), rho_d = msqrt(wave_max(du));
    if (!(rho_d < 1.0f) || !(rho_o < 1e30f)) return ~0ull;   // spread too wide: no culling
    bool keep = false;
    if (lane < V.np) {
        const DevSphereF& c = V.sphf[lane];
        if (c.rm >= 0.0f) {                                   // padding spheres: rm = -inf
            const float vx = c.cx - ox, vy = c.cy - oy, vz = c.cz - oz;
            const float D2 = fmaf(vx, vx, fmaf(vy, vy, vz * vz));
            const float D = msqrt(D2);
            const float Dm = D + rho_o;
            const float scale = fmaxf(fabsf(ox), fmaxf(fabsf(oy), fabsf(oz))) +
                                fmaxf(fabsf(c.cx), fmaxf(fabsf(c.cy), fabsf(c.cz))) + 1.0f;
            const float R = (msqrt(fmaf(c.rm, 1.0f + 0x1p-20f, Dm * Dm * 0x1p-46f)) + rho_o) * (1.0f + 0x1p-12f) +
                            0x1p-12f * scale;
#if RT_CHEAP_BUNDLE
            // The same cone test without the chord's two square roots and the reciprocal of D: for s = R / D <= 0.9,
            // chord(asin s) = s sqrt(2 / (1 + sqrt(1 - s^2))) <= s (1 + s^2 / 4) (equal at s = 0, 1.2% above the
            // chord at s = 0.9; the gap only grows towards 0.9), so |a - v / D| <= rho_d + chord + 2^-14 follows from
            // |a D - v| <= rho_d D + R (1 + s^2 / 4) + 2^-14 D (both sides times D > 0).  s > 0.9 (D < R / 0.9):
            // kept, as D <= R is.  FP32 errors of a D - v (< 2^-21 D) and of s^2 (mrcp: 2^-22 relative) stay far
            // inside the 2^-14 D slack.
            if (!(D * 0.9f > R)) {
                keep = true;
            } else {
                const float s2 = (R * R) * mrcp(D2);
                const float limD = fmaf(rho_d + 0x1p-14f, D, R * fmaf(0.25f, s2, 1.0f));
                const float ex = fmaf(ax, D, -vx), ey = fmaf(ay, D, -vy), ez = fmaf(az, D, -vz);
                keep = !(fmaf(ex, ex, fmaf(ey, ey, ez * ez)) > limD * limD);
            }
#else
            if (!(D > R)) {
                keep = true;
            } else {
                const float iD = mrcp(D);
                const float lim = rho_d + mchord_of_sin(R * iD) + 0x1p-14f;
                const float ex = ax - vx * iD, ey = ay - vy * iD, ez = az - vz * iD;
                keep = !(fmaf(ex, ex, fmaf(ey, ey, ez * ez)) > lim * lim);
            }
#endif
        }
    }
    const uint64_t kept = __ballot(keep);
    RT_COUNT(V.S, kCntRayMasks, 1);
    RT_COUNT(V.S, kCntRayKept, __popcll(kept & sphere_bits(V.np)));
    return kept;
}

// 1: a wave whose rays fan out (a sphere's silhouette: mirror rays off the board beside grazing reflections
// off the sphere) is covered by two bundles — the lanes within chord 0.9 of the first lane's direction (always
// narrow enough to cull) and the rest — and the mask is their union (each part is conservative for its lanes);
// 0: one bundle, no culling once the directions spread past chord 1.
#ifndef RT_BUNDLE_SPLIT
#define RT_BUNDLE_SPLIT 1
#endif
__device__ __forceinline__ uint64_t ray_bundle_mask(const SceneView& V, bool on, const Ray& r) {
    const uint64_t onm = __ballot(on);
    if (!onm) return 0;
    const int f = __builtin_ctzll(onm);
#if RT_BUNDLE_SPLIT
    const float ax = lane_f32(r.ux, f), ay = lane_f32(r.uy, f), az = lane_f32(r.uz, f);
    const float ux = r.ux - ax, uy = r.uy - ay, uz = r.uz - az;
    const bool near = on && fmaf(ux, ux, fmaf(uy, uy, uz * uz)) < 0.81f;     // NaN: not near
    uint64_t m = ray_bundle_part(V, near, r, f);
    const bool rest = on && !near;
    const uint64_t restm = __ballot(rest);
    if (restm) m |= ray_bundle_part(V, rest, r, __builtin_ctzll(restm));
    return m;
#else
    return ray_bundle_part(V, on, r, f);
#endif
}

// Shadow rays to light li: every ray lies on a line through the light, with direction w_l = u_l.
// a = w of the first `on` lane, rho >= |w_l - a|.  The light record gives v_k and c_k <= cos(phi_k),
// so a line through L that meets sphere k has |w -+ v_k| <= chord_k = sqrt(2 - 2 c_k) for one sign, and
// then |a -+ v_k| <= rho + chord_k (+ 2^-14 for FP32).  c_k = -inf: always kept; +inf (padding): never.
__device__ __forceinline__ uint64_t shadow_bundle_mask(const SceneView& V, bool on, const Ray& r, int li) {
    const int lane = __lane_id();
    const uint64_t onm = __ballot(on);
    if (!onm) return 0;
    const int f = __builtin_ctzll(onm);
    const float ax = lane_f32(r.ux, f), ay = lane_f32(r.uy, f), az = lane_f32(r.uz, f);
    float du = 0.0f;
    if (on) {
        const float ux = r.ux - ax, uy = r.uy - ay, uz = r.uz - az;
        du = inf_if_nan(fmaf(ux, ux, fmaf(uy, uy, uz * uz)));      // squared (see ray_bundle_mask)
    }
    const float rho = msqrt(wave_max(du));
    if (!(rho < 1.0f)) return ~0ull;
    bool keep = false;
    if (lane < V.np) {
        const DevSphereLightF& c = V.lightf[li * V.ns + lane];
        if (c.c <= 1.0f) {
            const float lim = rho + msqrt(fmaxf(0.0f, 2.0f - 2.0f * c.c)) + 0x1p-14f;
            const float l2 = lim * lim;
            const float ex = ax - c.vx, ey = ay - c.vy, ez = az - c.vz;
            const float fx = ax + c.vx, fy = ay + c.vy, fz = az + c.vz;
            keep = !(fmaf(ex, ex, fmaf(ey, ey, ez * ez)) > l2) || !(fmaf(fx, fx, fmaf(fy, fy, fz * fz)) > l2);
        }
    }
    const uint64_t kept = __ballot(keep);
    RT_COUNT(V.S, kCntShadowMasks, 1);
    RT_COUNT(V.S, kCntShadowKept, __popcll(kept & sphere_bits(V.np)));
    return kept;
}

// Shadow test: intersects() of g_scene.intersection(Line(pt, Lpos)) (:1216-1221), any hit.
// Spheres are filtered with the light's cone records: the ray lies on a line through light `li`, which
// meets sphere k only if |u . v_k| >= cos(phi_k) (host builder, rt_host.cpp).  FP32 error of the lane's
// dot product: |f32(u) - u|, |f32(v_k) - v_k| <= sqrt(3) 2^-24 and three roundings, < 7 * 2^-24 in all,
// far inside the 2^-16 folded into c_k; the FP64 hit test's own rounding moves the line by ~1e-13
// relative, likewise covered.  A NaN direction is not rejected (it compares false), as the FP64 test
// reports NaN rays as hits.
// RT_OCCL_FLAT=1: the same any-hit test with a per-lane flag instead of returns from inside the sphere loops (a lane
// that found a blocker leaves the loops; the board is tested by the lanes still unblocked).  occluded<.., FLAT> picks
// the form per instance (shade: the three-channel culling kernels keep the returns — the flag form spills 32 VGPRs
// to scratch in their depth-3 instance).
#ifndef RT_OCCL_FLAT
#define RT_OCCL_FLAT 1
#endif
template <bool FULL, bool CULL = false>
__device__ __forceinline__ bool occluded_flag(const SceneView& V, const Ray& r, int li, uint64_t mask = ~0ull,
                                              int skip = -1) {
    const DevScene* S = V.S;
    if (!(RT_HITS_INSIDE && (RT_HITS_VIEW ? V.hits_ok : S->hits_ok)) && !bound_pass(S, r.p0, r.u)) return false;   // shadow rays start at hits
    const double eps = S->eps;
    const DevSphereLightF* lf = V.lightf + li * V.ns;
    bool blocked = false;
    int k0 = 0;
    if (CULL && V.np >= kConeMin) {                               // mask: shadow_bundle_mask
        for (uint64_t m = mask & sphere_bits(V.np); m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            const DevSphereLightF& f = lf[k];
            float t = r.ux * f.vx;
            t = fmaf(r.uy, f.vy, t);
            t = fmaf(r.uz, f.vz, t);
            RT_COUNT(S, kCntFilterShadow, 1);
            RT_COUNT_LANES(S, kCntLanesFilterShadow);
            if (blocked | (fabsf(t) < f.c) | (k == skip - 1)) continue;
            RT_COUNT(S, kCntExactShadow, 1);
            RT_COUNT_LANES(S, kCntLanesExactShadow);
            d3 q;
            blocked = sphere_hit(V.sph[k], r.p0, r.u, eps, &q);
        }
        k0 = 64;
    }
    for (; k0 < V.np; k0 += kChunk) {
        if (k0 < 64 && ((mask >> k0) & ((1ull << kChunk) - 1)) == 0) continue;   // (cached masks, as closest_hit)
        uint32_t pass = 0;
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const DevSphereLightF& f = lf[k0 + j];
            float t = r.ux * f.vx;
            t = fmaf(r.uy, f.vy, t);
            t = fmaf(r.uz, f.vz, t);
            pass |= (fabsf(t) < f.c ? 0u : 1u) << j;
        }
        pass = blocked ? 0u : drop_self(pass, skip - 1, k0);
        while (pass) {
            const int k = k0 + __builtin_ctz(pass);
            d3 q;
            blocked = sphere_hit(V.sph[k], r.p0, r.u, eps, &q);
            pass = blocked ? 0u : pass & (pass - 1);
        }
    }
    if (S->has_board && skip != 0 && !blocked) {
        d3 q;
        RT_COUNT(S, kCntBoardShadow, 1);
        blocked = board_hit(S, r.p0, r.d, &q);
    }
    for (int m = 0; FULL && m < V.nm; ++m) {
        const DevMesh& M = V.mesh[m];
        if (blocked || !mesh_bound(M, r.p0, r.u, eps)) continue;
        for (int t = M.tri0; t < M.tri0 + M.nfaces * M.per_face && !blocked; ++t) {
            d3 q;
            blocked = tri_hit(V.tri[t], r.p0, r.d, eps, &q);
        }
    }
    return blocked;
}

template <bool FULL, bool CULL = false>
__device__ __forceinline__ bool occluded_ret(const SceneView& V, const Ray& r, int li, uint64_t mask = ~0ull,
                                             int skip = -1) {
    const DevScene* S = V.S;
    if (!(RT_HITS_INSIDE && (RT_HITS_VIEW ? V.hits_ok : S->hits_ok)) && !bound_pass(S, r.p0, r.u)) return false;   // shadow rays start at hits
    const double eps = S->eps;
    const DevSphereLightF* lf = V.lightf + li * V.ns;
    int k0 = 0;
    if (CULL && V.np >= kConeMin) {                               // mask: shadow_bundle_mask
        for (uint64_t m = mask & sphere_bits(V.np); m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            const DevSphereLightF& f = lf[k];
            float t = r.ux * f.vx;
            t = fmaf(r.uy, f.vy, t);
            t = fmaf(r.uz, f.vz, t);
            RT_COUNT(S, kCntFilterShadow, 1);
            RT_COUNT_LANES(S, kCntLanesFilterShadow);
            if (fabsf(t) < f.c || k == skip - 1) continue;
            RT_COUNT(S, kCntExactShadow, 1);
            RT_COUNT_LANES(S, kCntLanesExactShadow);
            d3 q;
            if (sphere_hit(V.sph[k], r.p0, r.u, eps, &q)) return true;
        }
        k0 = 64;
    }
    for (; k0 < V.np; k0 += kChunk) {
        if (k0 < 64 && ((mask >> k0) & ((1ull << kChunk) - 1)) == 0) continue;   // (cached masks, as closest_hit)
        uint32_t pass = 0;
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            const DevSphereLightF& f = lf[k0 + j];
            float t = r.ux * f.vx;
            t = fmaf(r.uy, f.vy, t);
            t = fmaf(r.uz, f.vz, t);
            pass |= (fabsf(t) < f.c ? 0u : 1u) << j;
        }
        pass = drop_self(pass, skip - 1, k0);
#if RT_UNIFORM_SHADOW
#pragma unroll
        for (int j = 0; j < kChunk; ++j) {
            if (!(pass & (1u << j))) continue;
            const int k = k0 + j;
#else
        while (pass) {
            const int k = k0 + __builtin_ctz(pass);
            pass &= pass - 1;
#endif
            d3 q;
            if (sphere_hit(V.sph[k], r.p0, r.u, eps, &q)) return true;
        }
    }
    if (S->has_board && skip != 0) {
        d3 q;
        RT_COUNT(S, kCntBoardShadow, 1);
        if (board_hit(S, r.p0, r.d, &q)) return true;
    }
    for (int m = 0; FULL && m < V.nm; ++m) {
        const DevMesh& M = V.mesh[m];
        if (!mesh_bound(M, r.p0, r.u, eps)) continue;
        for (int t = M.tri0; t < M.tri0 + M.nfaces * M.per_face; ++t) {
            d3 q;
            if (tri_hit(V.tri[t], r.p0, r.d, eps, &q)) return true;
        }
    }
    return false;
}

template <bool FULL, bool CULL = false, bool FLAT = RT_OCCL_FLAT>
__device__ __forceinline__ bool occluded(const SceneView& V, const Ray& r, int li, uint64_t mask = ~0ull,
                                         int skip = -1) {
    if constexpr (FLAT) return occluded_flag<FULL, CULL>(V, r, li, mask, skip);
    else return occluded_ret<FULL, CULL>(V, r, li, mask, skip);
}

// Material of a hit (checker parity for the board, :1101-1111).
// (int)(x / square) for the checker, both quotients sharing one reciprocal r = rcp_core(square) (the
// compiler's own Newton steps): for |x| in [2^-969, 2^500] and a normal `square` div_core is the IEEE
// quotient bit for bit (fast paths above); below that the quotient is < 2^-400 and truncates to 0 either
// way, hit points on the board never exceed it, and NaN stays NaN (converted to 0 either way).
// MESH = false: the caller's closest hits never name a mesh triangle (the opaque kernels' closest_hit<false> tests no
// meshes), so that branch is compiled out (RT_MESH_STATIC).
#ifndef RT_MESH_STATIC
#define RT_MESH_STATIC 1
#endif
template <bool MESH = true>
__device__ __forceinline__ int material_of(const SceneView& V, int kind, d3 p) {
    const DevScene* S = V.S;
    if (kind == 0) {
        d3 q = add(sub(p, ld3(S->coff)), mk(S->half, 0.0, S->half));
        const double r = S->rsquare;                        // rcp_core(square), rt_scene_init_kernel
        int squareSum = (int)div_core(q.x, S->square, r) + (int)div_core(q.z, S->square, r);
        return (squareSum & 1) == 0 ? 0 : 1;
    }
    if (MESH && kind >= kMeshKind) return V.mesh[(kind - kMeshKind) >> 4].mat;
    return 2;
}

// Shadow test when some material is transparent: the closest blocker decides (:1219-1221).
__device__ __forceinline__ bool occluded_transparent(const SceneView& V, const Ray& r) {
    d3 p;
    int kind = closest_hit<true>(V, r, &p, ~0ull, -1, true);        // shadow rays start at hits
    if (kind < 0) return false;
    return V.S->mat[material_of(V, kind, p)].transparent == 0;
}

// Transmitted ray end p + t (:685-699, :780-791) with the refraction of the object's own material: the
// board's triangles carry Material() (refraction 1, :291-293, :838-841), spheres and meshes theirs.
__device__ __forceinline__ d3 transmitted_end(const SceneView& V, int kind, int mat, d3 p, d3 u, d3 n) {
    double rr = kind == 0 ? 1.0 : V.S->mat[mat].refr;
    d3 t = mk(0.0, 0.0, 0.0);
    double cti = dot(u, n);                                 // :690
    double modulus = 1 - rr * rr * (1 - cti * cti);         // :691
    if (modulus > 0) {
        double ctr = sqrt_ieee(modulus);
        t = sub(scl(rr, u), scl(ctr + rr * cti, n));        // :696
    }
    return add(p, t);                                       // Line(p, p + t) (:699)
}

// Surface data of a hit: normal, material id, reflected end point p + r (:679-683, :774-778, :1101-1111).
#ifndef RT_CENTER_UNIFORM
#define RT_CENTER_UNIFORM 0
#endif
template <bool MESH = true>
__device__ __forceinline__ void surface(const SceneView& V, int kind, d3 p, d3 u, d3* n, int* mat, d3* pe) {
    const DevScene* S = V.S;
    if (kind == 0) {
        *n = ld3(S->tri[0].n);
    } else if (MESH && kind >= kMeshKind) {
        const DevMesh& M = V.mesh[(kind - kMeshKind) >> 4];
        *n = ld3(V.tri[M.tri0 + ((kind - kMeshKind) & 15)].n);
    } else {
#if RT_CENTER_UNIFORM
        // the centres of the spheres this wave hit, one scalar load per distinct sphere (the first remaining
        // lane's), instead of a per-lane vector load
        d3 c = mk(0.0, 0.0, 0.0);
        bool todo = true;
        for (;;) {
            const uint64_t m = __ballot(todo);
            if (m == 0) break;
            const int k = __builtin_amdgcn_readlane(kind, (int)__builtin_ctzll(m));
            if (todo && kind == k) {
                c = ld3(V.sph[k - 1].c);
                todo = false;
            }
        }
#else
        d3 c = ld3(V.sph[kind - 1].c);
#endif
        d3 dp = sub(p, c);                                  // directionP0 (:763)
        *n = unit(dp);                                      // :774-775
    }
    *mat = material_of<MESH>(V, kind, p);
    d3 r = sub(u, scl(2 * dot(u, *n), *n));                 // :682 / :777
    *pe = add(p, r);                                        // Line(p, p + r)
}

// Per-tile cache of the culling masks of every level (r06, RT_LEVEL_MASKS): a static view's rays are the same bits in
// every frame, so the wave-uniform masks ray_bundle_mask and shadow_bundle_mask compute from them are a pure function
// of the view, like the primary cone mask of the dispatch record.  The view's calibration render stores them per tile
// (`out`, lane 0), later renders of exactly that view read them (`in`) instead of computing them: slot l - 1 holds
// level l's ray mask (l = 1 .. B), slot B + l nl + i the shadow mask of light i at level l.  A mask is stored only
// where the wave computes it (a level every lane missed before is never reached, in either render).  Both null: the
// masks are computed (moving cameras, the calibration's first render, scenes with too many slots).  The wave keeps
// only its tile's first slot; the two arrays' addresses are read from the kernel arguments where a mask is needed
// (level_masks_in / _out, rt_render.hpp), so no pointer is held in SGPRs through the trace.
struct LevelMasks {
    int tile;                                  // first slot of this wave's tile (tile * slots per tile), -1: none
};
__device__ __forceinline__ const uint64_t* level_masks_in();
__device__ __forceinline__ uint64_t* level_masks_out();

// Local illumination of one hit over all lights (:1213-1228).  ks = |u . rdir|, u = incoming ray
// direction, rdir = reflectedRay().direction() (:1225).  `hit` marks the lanes whose colour is wanted.  CULL: called by all
// lanes of the wave, the light loop stays converged for shadow_bundle_mask; otherwise only by hit lanes.
// FULL: meshes may be present and materials may be transparent (closest-hit shadows, :1219-1221).
// ACC: the colour is accumulated in LDS at acc[0], acc[SS], acc[2 SS] (starting at 0, the same additions in the
// same order) instead of in registers live across every light's shadow test; the return value is then unused.
#ifndef RT_MAT_UNIFORM
#define RT_MAT_UNIFORM 0
#endif
// ACHRO (an achromatic scene, rt_scene_achromatic: every light colour and every material term an object uses has
// R = G = B): the three channels are the same operations on equal values, so only R is computed and the colour is
// (R, R, R) — bit for bit the reference's (G and B are R's operations repeated).  Not with FULL (transparency weights).
template <bool FULL, bool CULL, bool ACC = false, int SS = 256, bool ACHRO = false>
__device__ __forceinline__ d3 shade(const SceneView& V, bool hit, d3 p, d3 n, int mat, double ks,
                                    int skip = -1, double* acc = nullptr, const LevelMasks* lm = nullptr,
                                    int lslot = 0) {
    static_assert(!(ACHRO && FULL), "achromatic shading is for opaque scenes");
    const DevScene* S = V.S;
    d3 color = mk(0.0, 0.0, 0.0);
    if (ACC) {
        acc[0] = 0.0;
        if (!ACHRO) {
            acc[SS] = 0.0;
            acc[2 * SS] = 0.0;
        }
    }
    Ray sr;
    sr.p0 = p;
    if (FULL) set_origin_f32(S, &sr);                       // closest-hit shadows use the ray filter
    for (int i = 0; i < V.nl; ++i) {
        d3 lpos = ld3(S->light[i].pos);
        d3 sd = sub(lpos, p);                               // shadowRay end - start (:1216)
        double dl;                                          // shadowRay.length()
        d3 sdir = unit(sd, &dl);                            // shadowRay.direction()
        set_dir(&sr, sd, sdir);
        const double kd = fabs(dot(n, sdir));               // before the shadow test: fewer live registers
        uint64_t m = ~0ull;
        const int t = lm ? lm->tile : -1;
        if (CULL && !FULL && (V.np >= kConeMin || t >= 0)) {
            // (light i's shadow mask at this level: cached per tile for a calibrated static view, LevelMasks; also
            // computed for a fast scene when this render writes the cache)
            const uint64_t* in = t >= 0 ? level_masks_in() : nullptr;
            if (in) {
                m = in[t + lslot + i];
            } else {
                m = shadow_bundle_mask(V, hit, sr, i);
                uint64_t* out = t >= 0 ? level_masks_out() : nullptr;
                if (out && __lane_id() == 0) out[t + lslot + i] = m;
            }
        } else if (!CULL && !FULL && t >= 0) {
            // fast kernels: the cached mask lets occluded skip the filter batches no ray of the wave can meet
            const uint64_t* in = level_masks_in();
            if (in) m = in[t + lslot + i];
        }
        bool lit = false;
        if (hit)
            lit = !(FULL ? occluded_transparent(V, sr)
                         : occluded<false, CULL, RT_OCCL_FLAT && (ACHRO || !CULL)>(V, sr, i, m, skip));
        if (lit && ACHRO) {                                 // R only (same operations as below, channel x)
            const double a = S->att / (S->att + dl * dl);   // attenuation (:1181)
            const double lc = a * S->light[i].col[0];       // :1223
            const DevMat& M = S->mat[mat];
            const double term = (M.amb[0] * lc + kd * (M.diff[0] * lc)) + ks * (M.spec[0] * lc);   // :1224-1226
            if (ACC) acc[0] = acc[0] + term;
            else color.x = color.x + term;
        } else if (lit) {
            double a = S->att / (S->att + dl * dl);         // attenuation (:1181)
            d3 lC = scl(a, ld3(S->light[i].col));           // :1223
#if RT_MAT_UNIFORM
            // Opaque scenes use materials 0-2 (board squares, spheres): each one some lit lane needs is read with
            // scalar loads (wave-uniform address) and selected per lane, instead of a per-lane vector load.
            d3 amb = mk(0.0, 0.0, 0.0), dif = amb, spc = amb;
            if (!FULL) {
#pragma unroll
                for (int m = 0; m < 3; ++m) {
                    if (__ballot(mat == m) == 0) continue;
                    const DevMat& M = S->mat[m];
                    if (mat == m) {
                        amb = ld3(M.amb);
                        dif = ld3(M.diff);
                        spc = ld3(M.spec);
                    }
                }
            } else {
                const DevMat& M = S->mat[mat];
                amb = ld3(M.amb);
                dif = ld3(M.diff);
                spc = ld3(M.spec);
            }
            d3 term = add(add(had(amb, lC), scl(kd, had(dif, lC))), scl(ks, had(spc, lC)));
#else
            const DevMat& M = S->mat[mat];                  // material terms loaded only when lit
            d3 term = add(add(had(ld3(M.amb), lC), scl(kd, had(ld3(M.diff), lC))), scl(ks, had(ld3(M.spec), lC)));
#endif
            if (ACC) {                                      // :1224-1226, in LDS
                acc[0] = acc[0] + term.x;
                acc[SS] = acc[SS] + term.y;
                acc[2 * SS] = acc[2 * SS] + term.z;
            } else {
                color = add(color, term);                   // :1224-1226
            }
        }
    }
    return ACHRO ? mk(color.x, color.x, color.x) : color;
}

// The fast loop (non-CULL, opaque) at depth 1 accumulates each level's colour in its LDS slot (shade ACC), which
// frees the 6 VGPRs the colour held across the light loop (c2: 7 waves per SIMD without spills); the continuation
// parked across that loop then needs one extra slot (slot B + 1).  Deeper kernels keep the colour in registers:
// the extra slot would cost them LDS occupancy (B = 2 at 7 waves: 172 KB per CU).
#ifndef RT_ACC_LDS_MAX_B
#define RT_ACC_LDS_MAX_B 1
#endif
__host__ __device__ constexpr bool acc_lds(int B, bool transp) { return !transp && B >= 1 && B <= RT_ACC_LDS_MAX_B; }
// The culling variant keeps its last level's colour in registers (RT_CULL_LAST_REG): B colour slots instead of
// B + 1, so depth 3 needs 4.5 KB of LDS per one-wave workgroup instead of 6 KB — 35 workgroups per CU instead of
// 26, i.e. room for a seventh wave per SIMD.
#ifndef RT_CULL_LAST_REG
#define RT_CULL_LAST_REG 1
#endif
__host__ __device__ constexpr int colour_slots(int B, bool transp, bool cull = false) {
    return cull && RT_CULL_LAST_REG && !transp ? B : B + 1 + (acc_lds(B, transp) ? 1 : 0);
}

// rayTraceRay(g_scene, lights, Line(p0, p1), color, B) with color starting at 0 (:1184-1249), as a loop.
// Every hit of a non-tree scene spawns exactly one continuation (host-checked; ray trees: trace_tree): the
// reflected ray (opacity != 0) or the transmitted ray (transparency != 0 and |transparency| > eps), weighted
// by that vector (:1238-1247),
// so the colour is the right-nested local[0] + w[0] % (local[1] + w[1] % (...)).  TRANSP = false: all
// materials opaque, no meshes, w = (1,1,1) (multiplication by 1.0 is exact) and any-hit shadows.
// PRIMARY: p0 is the camera and V.prim/V.primf hold its per-sphere data;
// cone = primary_cone_mask of the wave (used when np >= kConeMin).
// seg / shadow count the rays actually traced.
// CULL (>= kConeMin spheres): called by all 64 lanes of a wave, the culling masks reduce over it.
// The per-level colours
// local[k] (and, TRANSP, the level's material for w[k]) wait in LDS until the right-nested sum, not in registers: slot[(3k + c) kSlotStride],
// mslot[k kSlotStride], component-major so a wave's 64 lanes touch 64 consecutive words.
constexpr int kSlotStride = 256;

// The continuation of a hit at level lvl (:1238-1247), computed before the light loop: its end - start
// (the transmitted ray's when the material transmits, else the reflected ray's rd) and the material id.
template <bool TRANSP>
__device__ __forceinline__ d3 continuation(const SceneView& V, int kind, int mat, d3 p, d3 n, d3 u, d3 rd) {
    if (TRANSP && V.S->mat[mat].transmit) return sub(transmitted_end(V, kind, mat, p, u, n), p);   // Line(p, p + t)
    return rd;                                                                                       // Line(p, p + r)
}

// A hit at level lvl: park its colour (and, TRANSP, its material for the weight w) in LDS.
template <bool TRANSP, int SS = kSlotStride, bool ACHRO = false>
__device__ __forceinline__ void park_level(int lvl, int mat, d3 c, double* slot, int* mslot) {
    double* sl = slot + 3 * lvl * SS;
    sl[0] = c.x;
    if (!ACHRO) {                                           // (achromatic: G = B = R)
        sl[SS] = c.y;
        sl[2 * SS] = c.z;
    }
    if (TRANSP) mslot[lvl * SS] = mat;
}

// The next level's ray for EVERY lane: Line(p, p + nd) for lanes that hit; lanes that did not get a zero
// ray (they are not alive at the next level and never trace it).  Assigning it unconditionally ends the
// live range of the previous ray at the hit test, so it is not carried through the light loop (the
// compiler cannot see that a lane which did not hit never reads its ray again).  u = unit(nd) is
// recomputed here (same operations, same bits) rather than kept live through the light loop.
__device__ __forceinline__ void next_ray(bool hit, d3 p, d3 nd, Ray* r) {
    d3 nu = nd;
    if (hit) nu = unit(nd);                                 // not for the zero rays: unit(0) is the slow path
    r->p0 = p;
    set_dir(r, nd, nu);
}

// As above with the continuation's unit direction kept from before the light loop (RT_KEEP_NU).
__device__ __forceinline__ void next_ray(d3 p, d3 nd, d3 nu, Ray* r) {
    r->p0 = p;
    set_dir(r, nd, nu);
}

// One bounce level of the CULL variant, run by all lanes of the wave (ray_bundle_mask and shade's
// shadow_bundle_mask reduce over it).  Returns false when no lane hit (the bounce loop ends).
template <int B, bool TRANSP, int SS = kSlotStride, bool ACHRO = false>
__device__ __forceinline__ bool cull_level(const SceneView& V, int lvl, bool first, bool alive, uint64_t cone, Ray* r, int* levels,
                                           double* slot, int* mslot, int* skip, bool lazy_u, d3* last,
                                           const LevelMasks& lm) {
    // the last level's colour stays in registers (RT_CULL_LAST_REG): slot B does not exist, so the continuation
    // of level B - 1 parks only its end - start and recomputes its unit direction after the light loop
    constexpr bool kLastReg = RT_CULL_LAST_REG && !TRANSP;
    uint64_t smask = ~0ull;
    RT_COUNT(V.S, kCntLevels, 1);
    if (!first) {
        set_origin_f32(V.S, r);
        if (V.np >= kConeMin || lm.tile >= 0) {
            const uint64_t* in = lm.tile >= 0 ? level_masks_in() : nullptr;
            if (in) {
                smask = in[lm.tile + lvl - 1];              // this tile's level-lvl ray mask (calibrated view)
            } else {
                smask = ray_bundle_mask(V, alive, *r);
                uint64_t* out = lm.tile >= 0 ? level_masks_out() : nullptr;
                if (out && __lane_id() == 0) out[lm.tile + lvl - 1] = smask;
            }
        }
    }
    d3 p = mk(0.0, 0.0, 0.0);
    int kind = -1;
    if (alive) {
        kind = first ? closest_hit_primary<TRANSP>(V, *r, cone, &p, lazy_u)
                     : closest_hit<TRANSP, true>(V, *r, &p, smask, TRANSP ? -1 : *skip, lvl > 0);
    }
    const bool hit = kind >= 0;
    RT_COUNT_BALLOT(V.S, kCntLanesLevelAlive, alive);
    RT_COUNT_BALLOT(V.S, kCntLanesLevelHit, hit);
    *skip = TRANSP ? -1 : origin_skip(V, kind, r->p0, p);      // this hit's rays start at p
    if (!__any(hit)) return false;
    d3 n = mk(0.0, 0.0, 0.0), nd = n;
    int mat = 0;
    double ks = 0.0;
    // (depth >= 3 only: at depth 2 the register allocation of this variant came out worse, 96 VGPRs + spills)
    constexpr bool kParkCull = RT_PARK_NU_CULL && B >= 3;
    double* psl = slot + 3 * lvl * SS;                      // this level's colour slot, written after shade
    if (hit) {
        d3 pe;
        surface<TRANSP || !RT_MESH_STATIC>(V, kind, p, r->u, &n, &mat, &pe);
        const d3 rd = sub(pe, p);                           // reflectedRay = Line(p, p + r)
        const d3 rdir = unit(rd);                           // reflectedRay.direction()
        ks = fabs(dot(r->u, rdir));                         // |u . reflectedRay.direction()|
        nd = continuation<TRANSP>(V, kind, mat, p, n, r->u, rd);
        if (kParkCull && lvl < B) {
            // the continuation (end - start and unit direction) waits in this and the next level's LDS
            // slots across the light loop: no registers, no unit() after it (as in the fast loop)
            psl[0] = nd.x;
            psl[SS] = nd.y;
            psl[2 * SS] = nd.z;
            if (!(kLastReg && lvl == B - 1)) {
                const d3 nu = (TRANSP && V.S->mat[mat].transmit) ? unit(nd) : rdir;
                psl[3 * SS] = nu.x;
                psl[4 * SS] = nu.y;
                psl[5 * SS] = nu.z;
            }
            asm volatile("" ::: "memory");
        }
    }
    const d3 c = shade<TRANSP, true, false, 256, ACHRO>(V, hit, p, n, mat, ks, *skip, nullptr, &lm, B + lvl * V.nl);
    d3 nu = nd;
    if (hit) {
        if (kParkCull && lvl < B) {
            asm volatile("" ::: "memory");
            nd = mk(psl[0], psl[SS], psl[2 * SS]);
            // (opaque: nd is the reflected ray's end - start, so unit(nd) is rdir, the same operations)
            if (kLastReg && lvl == B - 1) nu = unit(nd);
            else nu = mk(psl[3 * SS], psl[4 * SS], psl[5 * SS]);
        }
        if (kLastReg && lvl == B) *last = c;
        else park_level<TRANSP, SS, ACHRO>(lvl, mat, c, slot, mslot);
        *levels = lvl + 1;
    }
    if (lvl < B) {
        if (kParkCull) next_ray(p, nd, nu, r);
        else next_ray(hit, p, nd, r);
    }
    return true;
}

template <int B, bool PRIMARY, bool TRANSP, bool CULL, int SS = kSlotStride, bool ACHRO = false>
__device__ __forceinline__ d3 trace(const SceneView& V, d3 p0, d3 p1, uint64_t cone,
                                    uint32_t* seg, uint32_t* shadow, double* slot, int* mslot,
                                    LevelMasks lm = LevelMasks{-1}) {
    const DevScene* S = V.S;
    int levels = 0;
    Ray r;
    r.p0 = p0;
    d3 d = sub(p1, p0);
    // A primary ray of a wave whose cone mask keeps no sphere can only hit the board: its direction is computed
    // by closest_hit_primary for the lanes that hit (sky waves skip the normalisation).
    // (spheres past the first 64 are not in the mask: scenes with more always normalise)
    const bool lazy_u = RT_LAZY_PRIMARY_U && PRIMARY && !TRANSP && V.np >= kPrimaryConeMin && V.np <= 64 &&
                        (cone & sphere_bits(V.np)) == 0;
    if (lazy_u) r.d = d;
    else set_dir(&r, d, unit(d));
    // rays traced (seg, shadow) follow from `levels`: every lane traces levels 0 .. min(levels, B), nl shadow rays per hit
    int skip = -1;                                          // origin_skip of r's origin
    d3 last = mk(0.0, 0.0, 0.0);                            // CULL, RT_CULL_LAST_REG: level B's colour
    constexpr bool kLastReg = CULL && RT_CULL_LAST_REG && !TRANSP;
    constexpr bool kSkip = !TRANSP && B >= RT_SKIP_FAST_MIN_B;  // fast loop: origin skips from this depth
    constexpr bool kPark = B >= RT_PARK_ND_MIN_B;
#if RT_UNROLL_LEVELS
#pragma unroll
#else
#pragma unroll 1
#endif
    for (int lvl = 0; lvl <= B; ++lvl) {
        const bool alive = lvl == 0 || levels == lvl;
        if (!__any(alive)) break;                           // the whole wave has missed: early out
        const bool first = PRIMARY && lvl == 0;
        if (CULL) {
            if (!cull_level<B, TRANSP, SS, ACHRO>(V, lvl, first, alive, cone, &r, &levels, slot, mslot,
                                           &skip, lazy_u, &last, lm))
                break;
        } else {
            d3 p = mk(0.0, 0.0, 0.0);
            int kind = -1;
            if (alive) {
                if (first) {
                    kind = closest_hit_primary<TRANSP>(V, r, cone, &p, lazy_u);
                } else {
                    set_origin_f32(S, &r);
                    uint64_t rm = ~0ull;                    // this tile's cached level-lvl ray mask (LevelMasks)
                    if (!TRANSP && lm.tile >= 0) {
                        const uint64_t* in = level_masks_in();
                        if (in) rm = in[lm.tile + lvl - 1];
                    }
                    kind = closest_hit<TRANSP>(V, r, &p, rm, TRANSP ? -1 : skip, lvl > 0);
                }
            }
            const bool hit = kind >= 0;
            skip = kSkip ? origin_skip(V, kind, r.p0, p) : -1;   // this hit's rays start at p
            d3 nd = mk(0.0, 0.0, 0.0);
#if RT_KEEP_NU || RT_PARK_NU
            d3 nu = nd;
#endif
            if (hit) {
                d3 n, pe;
                int mat;
                surface<TRANSP || !RT_MESH_STATIC>(V, kind, p, r.u, &n, &mat, &pe);
                const d3 rd = sub(pe, p);                   // reflectedRay = Line(p, p + r)
                const d3 rdir = unit(rd);                   // reflectedRay.direction()
                const double ks = fabs(dot(r.u, rdir));     // |u . reflectedRay.direction()|
                nd = continuation<TRANSP>(V, kind, mat, p, n, r.u, rd);
#if RT_KEEP_NU && !RT_PARK_NU
                nu = (TRANSP && V.S->mat[mat].transmit) ? unit(nd) : rdir;
#endif
                double* psl = slot + 3 * lvl * SS;          // this level's colour slot, written after shade
#if RT_PARK_NU
                // ... and the continuation's unit direction in the next level's slot (written after that
                // level's shade): no recomputation of unit(nd) after the light loop, no live registers
                if (lvl < B) {
                    const d3 nu = (TRANSP && V.S->mat[mat].transmit) ? unit(nd) : rdir;
                    double* nsl = psl + 3 * SS;
                    nsl[0] = nu.x;
                    nsl[SS] = nu.y;
                    nsl[2 * SS] = nu.z;
                }
#endif
                // with the colour accumulated in this level's slot (kAcc), the end - start waits in slot lvl + 2
                constexpr bool kAcc = acc_lds(B, TRANSP);
                double* ndsl = kAcc ? psl + 6 * SS : psl;
                if ((kPark || RT_PARK_NU) && lvl < B) {
                    ndsl[0] = nd.x;
                    ndsl[SS] = nd.y;
                    ndsl[2 * SS] = nd.z;
                    asm volatile("" ::: "memory");          // keep it in LDS across the light loop
                }
                const d3 c = shade<TRANSP, false, kAcc, SS, ACHRO>(V, true, p, n, mat, ks, skip, psl, &lm, B + lvl * V.nl);
                if ((kPark || RT_PARK_NU) && lvl < B) {
                    asm volatile("" ::: "memory");
                    nd = mk(ndsl[0], ndsl[SS], ndsl[2 * SS]);
#if RT_PARK_NU
                    nu = mk(psl[3 * SS], psl[4 * SS], psl[5 * SS]);
#endif
                }
                if (!kAcc) park_level<TRANSP, SS, ACHRO>(lvl, mat, c, slot, mslot);
                levels = lvl + 1;
            }
#if RT_KEEP_NU || RT_PARK_NU
            if (lvl < B) next_ray(p, nd, nu, &r);
#else
            if (lvl < B) next_ray(hit, p, nd, &r);
#endif
        }
    }
    d3 acc = mk(0.0, 0.0, 0.0);
#pragma unroll 1
    for (int lvl = levels - 1; lvl >= 0; --lvl) {
        const double* sl = slot + 3 * lvl * SS;
        d3 c;
        if (kLastReg && lvl == B) c = last;             // (RT_CULL_LAST_REG: level B's colour in registers)
        else if (ACHRO) c = mk(sl[0], sl[0], sl[0]);
        else c = mk(sl[0], sl[SS], sl[2 * SS]);
        if (lvl == levels - 1) acc = c;
        else acc = TRANSP ? add(c, had(ld3(S->mat[mslot[lvl * SS]].w), acc)) : add(c, acc);
    }
    *seg = (uint32_t)(levels < B + 1 ? levels + 1 : B + 1);
    *shadow = (uint32_t)(V.nl * levels);
    return acc;
}

// ------------------------------------------------------------------------------------------------
// Ray trees (scenes with a material that both transmits and reflects, :1238-1247): rayTraceRay recurses
// into the transmitted child, then the reflected child, and adds each child's colour weighted by T and by
// 1 - T to the node's own colour, in that order.  Depth-first walk with an explicit per-lane node stack
// (node k = the ray at recursion depth B - k on the current path; dynamically indexed, so it lives in
// scratch memory — this path is for the rare tree scenes, the single-continuation scenes never run it).
// A child that misses is skipped: the reference adds w % (0,0,0) = +-0 to a colour that is never -0 (it
// starts at +0 and only sums), which leaves it unchanged.  General closest_hit for every ray (the primary
// shortcuts give the same bits), closest-hit shadows (FULL).
struct TreeNode {
    d3 p, td, rd;                      // hit point, transmitted and reflected ray (end - start)
    d3 acc;                            // the node's colour so far: local, then + T % child_T, + (1-T) % child_R
    int mat;
    int state;                         // 0: transmitted child next, 1: reflected child next, 2: done
};

// Trace Line(a, a + d) as node k: closest hit, local colour; false on a miss.
__device__ __forceinline__ bool tree_eval(const SceneView& V, d3 a, d3 d, TreeNode* node, uint32_t* nseg,
                                          uint32_t* nsh) {
    Ray r;
    r.p0 = a;
    set_dir(&r, d, unit(d));
    set_origin_f32(V.S, &r);
    ++*nseg;
    d3 p;
    const int kind = closest_hit<true>(V, r, &p);
    if (kind < 0) return false;
    d3 n, pe;
    int mat;
    surface(V, kind, p, r.u, &n, &mat, &pe);
    const d3 rd = sub(pe, p);                               // reflectedRay = Line(p, p + r)
    const double ks = fabs(dot(r.u, unit(rd)));             // |u . reflectedRay.direction()|
    node->acc = shade<true, false>(V, true, p, n, mat, ks);
    *nsh += V.nl;
    node->p = p;
    node->rd = rd;
    node->td = V.S->mat[mat].transmit ? sub(transmitted_end(V, kind, mat, p, r.u, n), p) : mk(0.0, 0.0, 0.0);
    node->mat = mat;
    node->state = 0;
    return true;
}

template <int B>
__device__ __forceinline__ d3 trace_tree(const SceneView& V, d3 p0, d3 p1, uint32_t* seg, uint32_t* shadow) {
    TreeNode st[B + 1];
    uint32_t nseg = 0, nsh = 0;
    d3 col = mk(0.0, 0.0, 0.0);
    if (tree_eval(V, p0, sub(p1, p0), &st[0], &nseg, &nsh)) {
        int k = 0;
        for (;;) {
            TreeNode& f = st[k];
            if (k < B) {                                    // depth B - k > 0: children (:1230)
                const DevMat& M = V.S->mat[f.mat];
                if (f.state == 0) {
                    f.state = 1;
                    if (M.transmit && tree_eval(V, f.p, f.td, &st[k + 1], &nseg, &nsh)) {
                        ++k;
                        continue;
                    }
                }
                if (f.state == 1) {
                    f.state = 2;
                    if (M.reflect && tree_eval(V, f.p, f.rd, &st[k + 1], &nseg, &nsh)) {
                        ++k;
                        continue;
                    }
                }
            }
            if (k == 0) break;
            TreeNode& pa = st[k - 1];                       // f is pa's child: T (state 1) or R (state 2)
            const DevMat& PM = V.S->mat[pa.mat];
            pa.acc = add(pa.acc, had(pa.state == 1 ? ld3(PM.wt) : ld3(PM.wo), f.acc));   // :1241, :1246
            --k;
        }
        col = st[0].acc;
    }
    *seg = nseg;
    *shadow = nsh;
    return col;
}

}  // namespace rt
