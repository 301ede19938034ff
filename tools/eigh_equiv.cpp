// Bit-for-bit check of the constant-index ssteqr3 (pcd_device.h) against LAPACK's general loop (ssteqr3_generic)
// over random, NVT-like, degenerate and non-finite 3x3 symmetric matrices (host build, not a unit test):
//   hipcc -O2 -std=c++17 -ffp-contract=off -DPCD_EIGH_GENERIC -I../include -I../normal-guided-pointcloud-denoiser_amd/csrc \
//         tools/eigh_equiv.cpp -o /tmp/eigh_equiv && /tmp/eigh_equiv 2000000
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "pcd_device.h"

using namespace pcd;

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 rng(12345);
    std::normal_distribution<float> N01(0.f, 1.f);
    std::uniform_real_distribution<float> U(0.f, 1.f);
    long bad = 0;
    for (long it = 0; it < n; ++it) {
        Sym3 A;
        const int kind = (int)(it % 7);
        if (kind == 0) {                      // random symmetric
            A = Sym3{N01(rng), N01(rng), N01(rng), N01(rng), N01(rng), N01(rng)};
        } else if (kind <= 3) {               // NVT-like: mean of n nᵀ over 1..3 normal clusters
            float a[6] = {0, 0, 0, 0, 0, 0};
            const int cl = kind, cnt = 1 + (int)(U(rng) * 32);
            float cn[3][3];
            for (int c = 0; c < cl; ++c) for (int q = 0; q < 3; ++q) cn[c][q] = N01(rng);
            const float noise = U(rng) < 0.3f ? 0.f : powf(10.f, -1.f - 5.f * U(rng));
            for (int t = 0; t < cnt; ++t) {
                const int c = t % cl;
                float v[3] = {cn[c][0] + noise * N01(rng), cn[c][1] + noise * N01(rng), cn[c][2] + noise * N01(rng)};
                const float L = sqrtf(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
                for (int q = 0; q < 3; ++q) v[q] /= L;
                a[0] += v[0] * v[0]; a[1] += v[0] * v[1]; a[2] += v[0] * v[2];
                a[3] += v[1] * v[1]; a[4] += v[1] * v[2]; a[5] += v[2] * v[2];
            }
            A = Sym3{a[0] / cnt, a[1] / cnt, a[2] / cnt, a[3] / cnt, a[4] / cnt, a[5] / cnt};
        } else if (kind == 4) {               // sparse / diagonal / repeated entries
            float a[6];
            for (int q = 0; q < 6; ++q) {
                const float r = U(rng);
                a[q] = r < 0.4f ? 0.f : r < 0.6f ? 1.f : r < 0.7f ? -0.f : N01(rng);
            }
            A = Sym3{a[0], a[1], a[2], a[3], a[4], a[5]};
        } else if (kind == 5) {               // extreme scales
            const float sc = powf(10.f, -40.f + 80.f * U(rng));
            A = Sym3{sc * N01(rng), sc * N01(rng), sc * N01(rng), sc * N01(rng), sc * N01(rng), sc * N01(rng)};
        } else {                              // a few non-finite entries
            float a[6];
            for (int q = 0; q < 6; ++q) {
                const float r = U(rng);
                a[q] = r < 0.05f ? NAN : r < 0.1f ? INFINITY : N01(rng);
            }
            A = Sym3{a[0], a[1], a[2], a[3], a[4], a[5]};
        }
        float w0[3], V0[3][3], w1[3], V1[3][3];
        eigh3<0>(A, w0, V0);
        eigh3<1>(A, w1, V1);
        // equal bit for bit, except that any NaN matches any NaN (non-finite inputs: NaN sign/payload is free)
        auto same = [](const float* a, const float* b, int m) {
            for (int q = 0; q < m; ++q)
                if (!(std::isnan(a[q]) && std::isnan(b[q])) && memcmp(a + q, b + q, sizeof(float))) return false;
            return true;
        };
        if (!same(w0, w1, 3) || !same(&V0[0][0], &V1[0][0], 9)) {
            if (bad < 5)
                printf("mismatch kind %d: A = %a %a %a %a %a %a  w0 %a %a %a  w1 %a %a %a\n", kind, A.a00, A.a01,
                       A.a02, A.a11, A.a12, A.a22, w0[0], w0[1], w0[2], w1[0], w1[1], w1[2]);
            ++bad;
        }
    }
    printf("%ld matrices, %ld mismatches\n", n, bad);
    return bad != 0;
}
