// Host check of eigh3_min (NVT2's Jacobi solve) against eigh3 (the LAPACK ssyevd port) on NVT-like tensors:
// T = mean of n nᵀ over 32 unit normals drawn around one, two or three directions (flat / edge / corner) with
// noise, plus random SPD matrices.  Reports the max eigenvalue difference, the worst |y_jacobi . y_lapack| of the
// smallest eigenvector (sign-free), and class disagreements.
//   hipcc -O2 -std=c++17 -ffp-contract=off -I../include -I../normal-guided-pointcloud-denoiser_amd/csrc \
//         eigh_min_check.cpp -o /tmp/eigh_min_check && /tmp/eigh_min_check
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
#include "pcd_device.h"
using namespace pcd;
int main() {
    std::mt19937 rng(7);
    std::normal_distribution<float> nd(0.f, 1.f);
    double max_dw = 0, min_dot = 1;
    long cls_diff = 0, n = 0;
    for (int it = 0; it < 2000000; ++it) {
        const int kind = it % 4;
        const float noise = (it / 4 % 5) * 0.05f;
        Vec3 dirs[3];
        for (int d = 0; d < 3; ++d) {
            Vec3 v = v3(nd(rng), nd(rng), nd(rng));
            const float l = std::sqrt(sq3(v));
            dirs[d] = (1.f / l) * v;
        }
        double t[6] = {0, 0, 0, 0, 0, 0};
        for (int j = 0; j < 32; ++j) {
            Vec3 v;
            if (kind == 3) v = v3(nd(rng), nd(rng), nd(rng));
            else v = dirs[j % (kind + 1)] + noise * v3(nd(rng), nd(rng), nd(rng));
            const float l = std::sqrt(sq3(v));
            v = (1.f / l) * v;
            t[0] += v.x * v.x; t[1] += v.x * v.y; t[2] += v.x * v.z; t[3] += v.y * v.y; t[4] += v.y * v.z; t[5] += v.z * v.z;
        }
        Sym3 T{(float)(t[0] / 32), (float)(t[1] / 32), (float)(t[2] / 32), (float)(t[3] / 32), (float)(t[4] / 32),
               (float)(t[5] / 32)};
        float w1[3], V[3][3], w2[3];
        Vec3 y;
        eigh3(T, w1, V);
        eigh3_min(T, w2, y);
        for (int k = 0; k < 3; ++k) max_dw = std::fmax(max_dw, std::fabs((double)w1[k] - w2[k]));
        // smallest eigenvector: only meaningful when it is separated from the middle one
        if (w1[1] - w1[0] > 1e-3f) {
            const double dt = std::fabs((double)V[0][0] * y.x + (double)V[1][0] * y.y + (double)V[2][0] * y.z);
            min_dot = std::fmin(min_dot, dt);
        }
        cls_diff += classify(w1, 0.2f, nullptr) != classify(w2, 0.2f, nullptr);
        ++n;
    }
    std::printf("n=%ld max|dw|=%.3g min|y.y_lapack| (gap>1e-3)=%.9f class differences=%ld (%.5f %%)\n", n, max_dw,
                min_dot, cls_diff, 100.0 * cls_diff / n);
    return 0;
}
