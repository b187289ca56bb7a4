// tools/microbench.hip — where the per-pixel floor of rt_render_kernel comes from (not product code).
// Each kernel uses the render kernel's grid (32 x 8 tiles, 256 threads, 8 x 8 per wave) on a 1920 x 1080
// frame and writes one uchar4 per pixel; they add the primary-ray steps one at a time:
//   store    the write alone
//   gen      + sp = (look + pitch (i+bx) right) + pitch (j+by) up, d = sp - eye
//   norm     + u = d / |d| (FP64 sqrt + 3 IEEE divisions)
//   norm1    + u = d * (1 / |d|) (one division)
//   bound    + the bounding-sphere test (dot, sqrt)
// Build: hipcc -O3 -ffp-contract=off --offload-arch=gfx950 tools/microbench.hip -o tools/_mb
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

struct P {
    double eye[3], look[3], right[3], upp[3], pitch, bc[3], br2, eps;
    int bx, by, W, H;
};

template <int MODE>
__global__ __launch_bounds__(256) void k(P p, uchar4* __restrict__ out) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int tiles_x = (p.W + 31) / 32;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int i = tx * 32 + wave * 8 + (lane & 7), j = ty * 8 + (lane >> 3);
    if (i >= p.W || j >= p.H) return;
    double v = 0.0;
    if (MODE >= 1) {
        double a = p.pitch * (double)(i + p.bx), b = p.pitch * (double)(j + p.by);
        double sx = (p.look[0] + a * p.right[0]) + b * p.upp[0];
        double sy = (p.look[1] + a * p.right[1]) + b * p.upp[1];
        double sz = (p.look[2] + a * p.right[2]) + b * p.upp[2];
        double dx = sx - p.eye[0], dy = sy - p.eye[1], dz = sz - p.eye[2];
        v = dx + dy + dz;
        if (MODE >= 2) {
            double l = sqrt(dx * dx + dy * dy + dz * dz);
            double ux, uy, uz;
            if (MODE == 3) {
                double r = 1.0 / l;
                ux = dx * r, uy = dy * r, uz = dz * r;
            } else {
                ux = dx / l, uy = dy / l, uz = dz / l;
            }
            v = ux + uy + uz;
            if (MODE >= 4) {
                double px = p.bc[0] - p.eye[0], py = p.bc[1] - p.eye[1], pz = p.bc[2] - p.eye[2];
                double dd = px * px + py * py + pz * pz;
                double uD = ux * px + uy * py + uz * pz;
                double disc = uD * uD - dd + p.br2;
                v = disc < 0 ? -1.0 : (fabs(uD - sqrt(disc)) < p.eps ? -2.0 : v);
            }
        }
    }
    out[(size_t)j * p.W + i] = make_uchar4((unsigned char)(int)(v * 7.0), 0, 0, 255);
}

int main() {
    P p{};
    double eye[3] = {0, 100, 200}, look[3] = {0, 0, -160};
    for (int c = 0; c < 3; ++c) p.eye[c] = eye[c], p.look[c] = look[c];
    p.right[0] = 1;
    p.upp[1] = 0.96, p.upp[2] = 0.27;
    p.pitch = 500.0 / 1920;
    p.bx = -960, p.by = -540, p.W = 1920, p.H = 1080;
    p.bc[2] = -160, p.br2 = 3 * 160.0 * 160.0, p.eps = 1e-12;
    uchar4* out;
    hipMalloc(&out, (size_t)p.W * p.H * 4);
    dim3 grid((p.W / 32) * ((p.H + 7) / 8));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char* names[] = {"store", "gen", "norm", "norm1", "bound"};
    for (int round = 0; round < 3; ++round) {
        for (int m = 0; m < 5; ++m) {
            auto launch = [&]() {
                switch (m) {
                    case 0: k<0><<<grid, 256>>>(p, out); break;
                    case 1: k<1><<<grid, 256>>>(p, out); break;
                    case 2: k<2><<<grid, 256>>>(p, out); break;
                    case 3: k<3><<<grid, 256>>>(p, out); break;
                    default: k<4><<<grid, 256>>>(p, out); break;
                }
            };
            launch();
            hipEventRecord(e0);
            for (int r = 0; r < 50; ++r) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            if (round == 2) printf("{\"kernel\": \"%s\", \"us\": %.2f}\n", names[m], ms * 1000 / 50);
        }
    }
    return 0;
}
