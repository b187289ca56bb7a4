// rt_layout.hpp — the device scene record (plain C++, shared by the host builder and the kernels).
//
// Layout in HBM (one allocation per rt_ctx):
//   DevScene header
//   DevSphere[ns]       FP64 exact data                 ┐ copied into LDS once per workgroup
//   DevSpherePrim[ns]   primary-ray FP64 data (per eye)  ┘ (lds_bytes)
//   DevSphereF[ns]      FP32 filter image               ┐ read through the scalar cache (SGPR operands),
//   DevSpherePrimF[ns]  primary-ray FP32 filter (per eye)│ one batch of kChunk records per s_load group
//   DevSphereCone[ns]   primary-ray cone of each sphere (per eye): per-wave culling
//   DevSphereLightF[nl][ns]  shadow-ray FP32 cone filter ┘ per light (line through the light)
//   DevMesh[nm]         tetrahedra / cubes: bounding sphere, triangle range, material, child index
//   DevTri[nt]          their triangles (world vertex 0, u, v, n, uv, uu, vv, den)
// np = n_spheres rounded up to kChunk; the padding spheres have r2 = -inf and filter terms = -inf, so
// they are rejected by the filter and can never hit.  ns = the arrays' stride: np, except for scenes the fast
// (non-culling) kernels render (np < kConeMin), whose arrays all have the fixed stride kFastStride — those kernels
// then address every record at a constant offset from the scene pointer instead of holding six array pointers
// in SGPRs (the SGPR budget of a seventh wave per SIMD).  The two *Prim arrays and DevSphereCone depend on
// the camera eye and are (re)written on the device by rt_prepare_kernel whenever rt_render_dev sees a
// new eye.
#pragma once

#include <stdint.h>

namespace rt {

constexpr int kChunk = 4;              // spheres per branch-free filter batch
#ifndef RT_CONE_MIN
#define RT_CONE_MIN 16
#endif
constexpr int kConeMin = RT_CONE_MIN;   // per-wave culling (primary cones, ray and shadow bundles) from this many (padded) spheres
constexpr int kFastStride = kConeMin - kChunk;   // the array stride of every scene with np < kConeMin
// Scenes of kConeMin .. 64 (padded) spheres — the culling kernels' — have the fixed stride 64, which their kernel
// instance sees as a constant (RT_CULL_FIX64; more spheres: stride np, the general instance).
#ifndef RT_CULL_FIX64
#define RT_CULL_FIX64 1
#endif
constexpr int kCullStride = 64;
inline constexpr int sphere_stride(int np) {
    return np < kConeMin ? kFastStride : (RT_CULL_FIX64 && np <= kCullStride ? kCullStride : np);
}
// The primary-ray cone mask is one ballot per wave (fast FP32 math): from 8 spheres it beats the per-sphere
// FP32 filter batches it replaces (same-box A/B: c2 -0.8%, c3 -1.9%; from 4 spheres c1 +3.7%).
#ifndef RT_PRIMARY_CONE_MIN
#define RT_PRIMARY_CONE_MIN 8
#endif
constexpr int kPrimaryConeMin = RT_PRIMARY_CONE_MIN;   // the primary-ray cone mask alone (every kernel variant)

// FP32 filter margin factor: 256 unit roundoffs of binary32.  The filter's own error is below
// 64 * 2^-24 * (S^2 + r^2) (error budget in rt_device.hpp, sphere_reject32), so a margin of
// 4K(sC^2 + sp^2) + K r^2 >= 2K S^2 + K r^2 leaves a factor >= 4 of slack.
constexpr float kFilterK = 256.0f / 16777216.0f;

struct alignas(16) DevTri {            // Triangle after its ctor (:406-433), vertex 0 in world space
    double v0[3];                      // (zero + (board_p + scene_pos)) + vertex0   (:640-641, :739)
    double u[3], v[3], n[3];
    double uv, uu, vv, den;
    double thr;                        // |den| * 2^-1070: A > thr  =>  A/den < 0 and nonzero
    double degenerate;                 // 1.0: this triangle never intersects (:633-637)
    double rden;                       // rcp_core(den), computed on the device (rt_scene_init_kernel)
    int32_t fast;                      // 1: |den| in [2^-200, 2^200], quotients A/den may use rden
    int32_t pad;
};

struct alignas(16) DevMat {            // the colour terms rayTraceRay reads (:1224-1226) and its continuation
    double amb[3], diff[3], spec[3];
    double w[3];                       // weight of the child colour: transparency (transmit) or 1 - T (reflect)
    double wt[3];                      // ray trees: weight of the transmitted child, T (:1241)
    double wo[3];                      // ray trees: weight of the reflected child, 1 - T (:1246)
    double refr;                       // refraction ratio (transmitted ray, :686-697)
    int32_t transmit;                  // 1: transmitted ray (:1238-1242), 0: reflected ray (:1243-1247)
    int32_t transparent;               // transparency != 0: a shadow blocker of this material lets light pass (:1221)
    int32_t reflect;                   // opacity != 0: a reflected ray (:1243); with transmit: both (a ray tree)
    int32_t pad;
};

struct alignas(16) DevMesh {           // Tetrahedron / Cube Shape (:863-950)
    double bc[3];                      // _position + positionOffset (:739)
    double br2;                        // radius^2, radius = sqrt(3)*edge/2
    double inner2;                     // (radius - 1)^2 or -1 (bound-cull shortcut, as for g_scene)
    int32_t tri0;                      // first DevTri
    int32_t nfaces;                    // faces: 1 triangle each (tetrahedron) or 2 = Quad, first hit (cube)
    int32_t per_face;                  // 1 or 2
    int32_t mat;                       // material index (3 tetrahedron, 4 cube)
    int32_t child;                     // index in g_scene's child list (closest-hit tie order)
    int32_t pad;
};

struct alignas(16) DevLight {
    double pos[3];
    double col[3];
};

struct alignas(16) DevSphere {         // world centre = _position + positionOffset (:739), r*r (:750)
    double c[3];
    double r2;
};

struct alignas(16) DevSpherePrim {     // primary rays: deltaP = C - eye and dot(deltaP, deltaP) (:740, :750)
    double dP[3];
    double dd;
};

struct alignas(16) DevSphereF {        // FP32 filter: centre - bound centre, r2 + 4K*sC^2 + K*r2 (rounded up)
    float cx, cy, cz, rm;
};

struct alignas(16) DevSpherePrimF {    // FP32 filter for primary rays: f32(dP), r2 - dd + K*(S0^2 + r2)
    float dx, dy, dz, c0;
};

struct alignas(16) DevSphereCone {     // primary rays: f32(unit(C - eye)) and the chord radius of the
    float vx, vy, vz, chord;           // sphere's cone of directions seen from the eye (rounded up)
};

struct alignas(16) DevSphereLightF {   // shadow rays to light i: f32(unit(C - L)) and cos(phi) - margin,
    float vx, vy, vz, c;               // phi = asin(r / |C - L|); c = -inf: always test, +inf: never (padding)
};

struct alignas(16) DevScene {
    double bc[3];                      // g_scene position + (0,0,0)                     (:739)
    double br2;                        // g_scene radius squared                          (:750)
    double inner2;                     // (radius - 1)^2: origins with |o - bc|^2 < inner2 pass the cull
    double eps;                        // SMALL_NUMBER
    double att;                        // ATTENUATION_FACTOR
    double coff[3];                    // checker offset = positionOffset of CheckerBoard (:1101)
    double half;                       // BOARD_HALF_SIZE
    double square;                     // SQUARE_EDGE_SIZE
    double rsquare;                    // rcp_core(square), computed on the device (rt_scene_init_kernel)
    double board_skip_y;               // rays starting at a board hit whose ray came from |y| <= this provably
                                       // miss the board (rt_device.hpp origin_skip); -1: never skipped
    double self_eps2;                  // eps^2 / 4: sphere self-test skip threshold (origin_skip)
    double hits_lim2;                  // hits_inside holds for rays whose level-0 origin o has |o - bc|^2 <= this
    double board_num;                  // n . (v0 - eye) of the board plane for the camera `eye` (per eye)
    // Board decided by position (board_fast, rt_device.hpp board_hit): margin delta, L - delta, L + delta and the
    // range |w| <= far within which the decisions' error bound holds (w = hit point - vertex 0, L = board side)
    double board_lo, board_hi, board_out, board_far;
    double eye[3];                     // camera the *Prim arrays and board_num were computed for
    int32_t bound_on;                  // g_scene radius > 0
    int32_t has_board;
    int32_t n_spheres;                 // real spheres
    int32_t n_padded;                  // np: n_spheres rounded up to kChunk
    int32_t n_stride;                  // ns: stride of the per-sphere arrays (sphere_stride(np))
    int32_t n_lights;
    int32_t lds_bytes;                 // header + DevSphere[np] + DevSpherePrim[np]
    int32_t n_meshes;
    int32_t n_tris;
    int32_t transparent;               // some material is transparent: closest-hit shadows, weighted children
    int32_t tree;                      // some material transmits AND reflects: ray-tree kernels (trace_tree)
    int32_t hits_inside;               // every hit point lies within (R - 1) of bc: rays from hits pass the cull
    int32_t hits_ok;                   // hits_inside for the camera eye (rt_prepare_kernel, per eye)
    int32_t board_fast;                // the reference's board, exactly: barycentric tests decided by position
    int32_t prim_bound_ok;             // per eye: every primary ray that hits an object passes the cull (rt_prepare_kernel)
    unsigned long long* counters;      // RT_COUNTERS builds (tools/counters.py): per-wave event counters, else null
    DevTri tri[2];                     // board triangles T1 = (P1,P2,P3), T2 = (P1,P3,P4)   (:840-841)
    DevMat mat[5];                     // 0 white square, 1 black square, 2 sphere, 3 tetrahedron, 4 cube
    DevLight light[16];
};

inline constexpr int padded_spheres(int n) { return (n + kChunk - 1) / kChunk * kChunk; }

inline constexpr int lds_bytes_for(int n) {
    return (int)(sizeof(DevScene) +
                 (sizeof(DevSphere) + sizeof(DevSpherePrim)) * (unsigned)sphere_stride(padded_spheres(n)));
}

inline constexpr int scene_bytes_for(int n, int n_meshes = 0, int n_tris = 0, int n_lights = 0) {
    return lds_bytes_for(n) +
           (int)((sizeof(DevSphereF) + sizeof(DevSpherePrimF) + sizeof(DevSphereCone) +
                  sizeof(DevSphereLightF) * (unsigned)n_lights) *
                 (unsigned)sphere_stride(padded_spheres(n))) +
           (int)(sizeof(DevMesh) * (unsigned)n_meshes + sizeof(DevTri) * (unsigned)n_tris);
}

}  // namespace rt

// rt_render_screen's chunk (rt_screen.cpp), read by the screen mode of rt_trace_rays_kernel: one pixel's screen point
// and the window of jitter-stream samples traced for it (stream indices base .. base + len - 1, relative to the
// chunk's first stream index), whose rays are ray indices off .. off + len - 1 of the launch.
struct ScreenPix {
    double sp[3];
    int32_t base, len, off, pad;
};
constexpr int kScreenMaxWindow = 128;          // len <= this (the window half-width kWin <= 56)
// (64-thread workgroups — one wave per CU for a small chunk — measured the same GPU wait per chunk as 256: the
// latency is the trace's own instruction chain, not CU sharing)
#ifndef RT_SCREEN_WG
#define RT_SCREEN_WG 256
#endif
constexpr int kScreenBlock = RT_SCREEN_WG;     // rays per first-pixel table entry (the screen trace launch's workgroup)
