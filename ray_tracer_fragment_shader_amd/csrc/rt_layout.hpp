// rt_layout.hpp — the device scene record (plain C++, shared by the host builder and the kernels).
//
// Layout in HBM (one allocation per rt_ctx, uploaded by rt_set_scene):
//   DevScene header | DevSphere[n] (FP64 exact data) | DevSphereF[n] (FP32 filter data)
// Per workgroup the kernel copies the record into LDS and appends, computed in its prologue for the
// frame's camera, DevSpherePrim[n] | DevSpherePrimF[n] (primary-ray data, see rt_device.hpp).
#pragma once

#include <stdint.h>

namespace rt {

// FP32 filter margin factor: 256 unit roundoffs of binary32.  The filter's own error is below
// 64 * 2^-24 * (S^2 + r^2) (error budget in rt_device.hpp, sphere_reject32), so a margin of
// 4K(sC^2 + sp^2) + K r^2 >= 2K S^2 + K r^2 leaves a factor >= 4 of slack.
constexpr float kFilterK = 256.0f / 16777216.0f;

struct alignas(16) DevTri {            // Triangle after its ctor (:406-433), vertex 0 in world space
    double v0[3];                      // (zero + (board_p + scene_pos)) + vertex0   (:640-641, :739)
    double u[3], v[3], n[3];
    double uv, uu, vv, den;
    double thr;                        // |den| * 2^-1070: A > thr  =>  A/den < 0 and nonzero
    double pad;
};

struct alignas(16) DevMat {            // the three colour terms rayTraceRay reads (:1224-1226)
    double amb[3], diff[3], spec[3];
    double pad;
};

struct alignas(16) DevLight {
    double pos[3];
    double col[3];
};

struct alignas(16) DevSphere {         // world centre = _position + positionOffset (:739), r*r (:750)
    double c[3];
    double r2;
};

struct alignas(16) DevSphereF {        // FP32 filter: centre - bound centre, r2 + 4K*sC^2 + K*r2 (rounded up)
    float cx, cy, cz, rm;
};

struct alignas(16) DevSpherePrim {     // primary rays: deltaP = C - eye and dot(deltaP, deltaP) (:740, :750)
    double dP[3];
    double dd;
};

struct alignas(16) DevSpherePrimF {    // FP32 filter for primary rays: f32(dP), r2 - dd + K*(S0^2 + r2)
    float dx, dy, dz, c0;
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
    int32_t bound_on;                  // g_scene radius > 0
    int32_t has_board;
    int32_t n_spheres;
    int32_t n_lights;
    DevTri tri[2];                     // board triangles T1 = (P1,P2,P3), T2 = (P1,P3,P4)   (:840-841)
    DevMat mat[3];                     // 0 white square, 1 black square, 2 sphere
    DevLight light[16];
    // followed by n_spheres DevSphere, then n_spheres DevSphereF
};

inline constexpr int scene_bytes_for(int n_spheres) {
    return (int)(sizeof(DevScene) + (sizeof(DevSphere) + sizeof(DevSphereF)) * (unsigned)n_spheres);
}

inline constexpr int prim_bytes_for(int n_spheres) {
    return (int)((sizeof(DevSpherePrim) + sizeof(DevSpherePrimF)) * (unsigned)n_spheres);
}

}  // namespace rt
