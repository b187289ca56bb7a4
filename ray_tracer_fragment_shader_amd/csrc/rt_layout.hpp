// rt_layout.hpp — the device scene record (plain C++, shared by host builder and kernels).
#pragma once

#include <stdint.h>

namespace rt {

// Device scene: the flat, precomputed form of g_scene.  Built on the host (rt_kernel.hip, build_scene)
// with the reference's operation order for every precomputed quantity.
struct alignas(16) DevTri {            // Triangle after its ctor (:406-433), vertex 0 in world space
    double v0[3];                      // (zero + (board_p + scene_pos)) + vertex0   (:640-641, :739)
    double u[3], v[3], n[3];
    double uv, uu, vv, den;
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

struct alignas(16) DevScene {
    double bc[3];                      // g_scene position + (0,0,0)                     (:739)
    double br2;                        // g_scene radius squared                          (:750)
    double eps;                        // SMALL_NUMBER
    double att;                        // ATTENUATION_FACTOR
    double coff[3];                    // checker offset = positionOffset of CheckerBoard (:1101)
    double half;                       // BOARD_HALF_SIZE
    double square;                     // SQUARE_EDGE_SIZE
    double pad0;
    int32_t bound_on;                  // g_scene radius > 0
    int32_t has_board;
    int32_t n_spheres;
    int32_t n_lights;
    DevTri tri[2];                     // board triangles T1 = (P1,P2,P3), T2 = (P1,P3,P4)   (:840-841)
    DevMat mat[3];                     // 0 white square, 1 black square, 2 sphere
    DevLight light[16];
    // followed by n_spheres DevSphere
};

}  // namespace rt
