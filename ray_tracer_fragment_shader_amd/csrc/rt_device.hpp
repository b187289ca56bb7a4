// rt_device.hpp — FP64 device math and the per-ray tracer of the MI355X path.
//
// Every operation keeps the reference's exact IEEE binary64 operation order (Appendix A of SURVEY.md);
// the file is compiled with -ffp-contract=off so no a*b+c is fused.  Citations are into
// /root/reference/Hw4/MySdlApplication.cpp.
//
// Restatement choices that are bit-identical to the reference (each argued at its use):
//  * the ray direction u = normalize(end - start) is computed once per ray, not once per child
//    (Line::direction :258-263 recomputes the same expression on the same inputs);
//  * the closest-hit search keeps only (distance, child, point); normal / reflection / material are
//    computed once for the winner (they are pure functions of the winner's point);
//  * the board's two triangles share vertex 0 and normal, so the plane step (m, p, w) is done once;
//  * shadow rays stop at the first blocker (any-hit): rayTraceRay reads only intersects() and the
//    blocker's transparency (:1221), and the GPU path only accepts opaque materials;
//  * the recursion (:1238-1247) becomes a loop; the colour of level k is local[k] + colour[k+1] with
//    opacity (1,1,1), so the frame colour is the right-nested sum local[0] + (local[1] + (...)).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_layout.hpp"

namespace rt {

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

__device__ __forceinline__ const DevSphere* spheres_of(const DevScene* s) {
    return reinterpret_cast<const DevSphere*>(s + 1);
}

__device__ __forceinline__ d3 ld3(const double* p) { return mk(p[0], p[1], p[2]); }

// ------------------------------------------------------------------------------------------------
// g_scene bounding-sphere cull (:747-758): miss iff disc < 0 or |s| < eps.
__device__ __forceinline__ bool bound_pass(const DevScene* S, d3 p0, d3 u) {
    if (!S->bound_on) return true;
    d3 dP = sub(ld3(S->bc), p0);
    double uD = dot(u, dP);
    double disc = uD * uD - dot(dP, dP) + S->br2;
    if (disc < 0) return false;
    double s = uD - sqrt(disc);
    return !(fabs(s) < S->eps);
}

// CheckerBoard -> Quad -> Triangle T1 then T2, first hit wins (:1097, :817, :611-707).
// d = end - start (unnormalised, :647).  Returns the hit point in *p.
__device__ __forceinline__ bool board_hit(const DevScene* S, d3 p0, d3 d, d3* p) {
    const DevTri& T = S->tri[0];
    d3 n = ld3(T.n);
    double nd = dot(n, d);                                  // :648
    if (fabs(nd) < S->eps) return false;                    // :651
    d3 v0 = ld3(T.v0);
    double m = dot(n, sub(v0, p0)) / nd;                    // :657 (denominator recomputed there: same value)
    if (m < S->eps) return false;                           // :659
    d3 q = add(p0, scl(m, d));                              // :665
    d3 w = sub(q, v0);                                      // :667
#pragma unroll
    for (int t = 0; t < 2; ++t) {
        const DevTri& Tt = S->tri[t];
        double wu = dot(w, ld3(Tt.u));
        double wv = dot(w, ld3(Tt.v));
        double s = (Tt.uv * wv - Tt.vv * wu) / Tt.den;      // :673
        double tt = (Tt.uv * wu - Tt.uu * wv) / Tt.den;     // :674
        if (s >= 0 && tt >= 0 && s + tt <= 1) {             // :676
            *p = q;
            return true;
        }
    }
    return false;
}

// Sphere (:747-772): candidate point if disc >= 0 and s >= eps (|s| < eps or s < eps -> miss).
__device__ __forceinline__ bool sphere_hit(const DevSphere& sp, d3 p0, d3 u, double eps, d3* p) {
    d3 dP = sub(ld3(sp.c), p0);
    double uD = dot(u, dP);
    double disc = uD * uD - dot(dP, dP) + sp.r2;
    if (disc < 0) return false;
    double s = uD - sqrt(disc);
    if (s < eps) return false;                              // covers |s| < eps (:754) and s < eps (:767)
    *p = add(p0, scl(s, u));                                // :762
    return true;
}

// Closest hit of g_scene (:796-821): Euclidean distance |p - p0|, strict <, board (child 0) first.
// kind: -1 miss, 0 board, 1 + k sphere k.
__device__ __forceinline__ int closest_hit(const DevScene* S, const DevSphere* sph, d3 p0, d3 d, d3 u,
                                           d3* hp) {
    if (!bound_pass(S, p0, u)) return -1;
    int kind = -1;
    double best = -1.0;
    if (S->has_board) {
        d3 q;
        if (board_hit(S, p0, d, &q)) {
            kind = 0;
            best = len(sub(q, p0));
            *hp = q;
        }
    }
    const int ns = S->n_spheres;
    const double eps = S->eps;
    for (int k = 0; k < ns; ++k) {
        d3 q;
        if (sphere_hit(sph[k], p0, u, eps, &q)) {
            double dist = len(sub(q, p0));                  // :811-812
            if (dist < best || best < 0.0) {                // :813
                best = dist;
                kind = 1 + k;
                *hp = q;
            }
        }
    }
    return kind;
}

// Shadow test: intersects() of g_scene.intersection(Line(pt, Lpos)) (:1216-1221), any hit.
__device__ __forceinline__ bool occluded(const DevScene* S, const DevSphere* sph, d3 p0, d3 d, d3 u) {
    if (!bound_pass(S, p0, u)) return false;
    const int ns = S->n_spheres;
    const double eps = S->eps;
    for (int k = 0; k < ns; ++k) {
        d3 q;
        if (sphere_hit(sph[k], p0, u, eps, &q)) return true;
    }
    if (S->has_board) {
        d3 q;
        if (board_hit(S, p0, d, &q)) return true;
    }
    return false;
}

// Surface data of a hit: normal, material id, reflected end point p + r (:679-683, :774-778, :1101-1111).
__device__ __forceinline__ void surface(const DevScene* S, const DevSphere* sph, int kind, d3 p, d3 u,
                                        d3* n, int* mat, d3* pe) {
    if (kind == 0) {
        *n = ld3(S->tri[0].n);
        d3 q = add(sub(p, ld3(S->coff)), mk(S->half, 0.0, S->half));
        int squareSum = (int)(q.x / S->square) + (int)(q.z / S->square);
        *mat = (squareSum & 1) == 0 ? 0 : 1;
    } else {
        d3 c = ld3(sph[kind - 1].c);
        d3 dp = sub(p, c);
        *n = divs(dp, len(dp));
        *mat = 2;
    }
    d3 r = sub(u, scl(2 * dot(u, *n), *n));
    *pe = add(p, r);
}

// Local illumination of one hit over all lights (:1213-1228).  u = incoming ray direction,
// rdir = reflectedRay().direction().  Returns the number of shadow rays traced.
__device__ __forceinline__ d3 shade(const DevScene* S, const DevSphere* sph, d3 p, d3 n, int mat, d3 u,
                                    d3 rdir) {
    const DevMat& M = S->mat[mat];
    d3 amb = ld3(M.amb), dif = ld3(M.diff), spc = ld3(M.spec);
    double ks = fabs(dot(u, rdir));
    d3 color = mk(0.0, 0.0, 0.0);
    const int nl = S->n_lights;
    for (int i = 0; i < nl; ++i) {
        d3 lpos = ld3(S->light[i].pos);
        d3 sd = sub(lpos, p);                               // shadowRay end - start
        double dl = len(sd);                                // shadowRay.length()
        d3 sdir = divs(sd, dl);                             // shadowRay.direction()
        if (!occluded(S, sph, p, sd, sdir)) {
            double a = S->att / (S->att + dl * dl);         // attenuation (:1181)
            d3 lC = scl(a, ld3(S->light[i].col));
            d3 term = add(add(had(amb, lC), scl(fabs(dot(n, sdir)), had(dif, lC))), scl(ks, had(spc, lC)));
            color = add(color, term);
        }
    }
    return color;
}

// rayTraceRay(g_scene, lights, Line(p0, p1), color, B) with color starting at 0 (:1184-1249),
// iterative.  seg / shadow count the rays actually traced.
template <int B>
__device__ __forceinline__ d3 trace(const DevScene* S, const DevSphere* sph, d3 p0, d3 p1, uint32_t* seg,
                                    uint32_t* shadow) {
    d3 local[B + 1];
    int levels = 0;
    d3 d = sub(p1, p0);
    d3 u = divs(d, len(d));
    uint32_t nseg = 0, nsh = 0;
#pragma unroll
    for (int lvl = 0; lvl <= B; ++lvl) {
        local[lvl] = mk(0.0, 0.0, 0.0);
        bool alive = lvl == 0 || levels == lvl;
        if (!__any(alive)) break;                           // the whole wave has missed: early out
        if (alive) {
            ++nseg;
            d3 p;
            int kind = closest_hit(S, sph, p0, d, u, &p);
            if (kind >= 0) {
                d3 n, pe;
                int mat;
                surface(S, sph, kind, p, u, &n, &mat, &pe);
                d3 rd = sub(pe, p);                         // reflectedRay = Line(p, p + r)
                d3 rdir = divs(rd, len(rd));
                local[lvl] = shade(S, sph, p, n, mat, u, rdir);
                nsh += S->n_lights;
                levels = lvl + 1;
                p0 = p;                                     // next level traces the reflected ray
                d = rd;
                u = rdir;
            }
        }
    }
    d3 acc = mk(0.0, 0.0, 0.0);
#pragma unroll
    for (int lvl = B; lvl >= 0; --lvl) {
        if (lvl < levels) acc = (lvl == levels - 1) ? local[lvl] : add(local[lvl], acc);
    }
    *seg = nseg;
    *shadow = nsh;
    return acc;
}

}  // namespace rt
