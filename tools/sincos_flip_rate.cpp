// How often the device fp64 sincos (pt_math.h pt_sincos: π/2 reduction in double-double + fdlibm
// kernels, within 1 ulp of glibc) changes a float the reference would build, at the real call sites
// ("extend check_sincos to random radii and to the call sites' float expressions").
// The reference calls Math.Sin and Math.Cos separately (the oracle: glibc sin / cos, not sincos).
// Sites, each with the float expressions of pt_device.h / pt_math.h:
//   RUV    Vector.RandomUnitVector (Vector.cs:339-347): mk(r·sin a, r·cos a, z), r = sqrt(1 − z²)
//   WB     Ray.WeightedBounce (Ray.cs:28-35): muls(s, √u·cos θ), muls(t, √u·sin θ), θ = 2πv, s, t unit floats
//   CONE   Util.Cone (Util.cs:17-32): m1, m2 = sin, cos θ' (θ' = θ(1 − 2acos(u)/π), θ ≤ 1.2),
//          muls(s, m1·cos a), muls(t, m1·sin a), muls(dir, m2), a = 2πv
// A "flip" is a call whose float outputs differ in any bit.  (acos is not compared: OCML's and
// glibc's acos cannot both run here; the two sides use glibc's acos.)
// usage: g++ -O2 -std=c++17 -ffp-contract=off -fno-builtin-sin -fno-builtin-cos -I ptsharp_amd/csrc \
//          -o /tmp/sfr tools/sincos_flip_rate.cpp && /tmp/sfr [calls per site]
#define PT_DEVICE_SINCOS 1
#include "pt_math.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

using pt::v3;
static bool same(v3 a, v3 b) { return !std::memcmp(&a, &b, sizeof a); }
static v3 unit(std::mt19937_64& g) {
    std::normal_distribution<double> N;
    double x = N(g), y = N(g), z = N(g), l = std::sqrt(x * x + y * y + z * z);
    return pt::mk(x / l, y / l, z / l);
}
int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 100000000L;
    std::mt19937_64 g(7);
    auto U = [&]() { return (double)(g() >> 11) * (1.0 / 9007199254740992.0); };
    long flips[3] = {0, 0, 0}, sc_ulp[2] = {0, 0};
    for (long i = 0; i < n; i++) {
        // RUV
        {
            const double z = U() * 2.0 - 1.0, a = U() * 2.0 * pt::kPi, r = std::sqrt(1.0 - z * z);
            double ds, dc;
            pt::pt_sincos(a, &ds, &dc);
            const double ls = std::sin(a), lc = std::cos(a);
            sc_ulp[0] += ds != ls; sc_ulp[1] += dc != lc;
            flips[0] += !same(pt::mk(r * ds, r * dc, z), pt::mk(r * ls, r * lc, z));
        }
        // WeightedBounce
        {
            const double u = U(), v = U(), radius = std::sqrt(u), th = 2 * pt::kPi * v;
            const v3 s = unit(g), t = unit(g), nn = unit(g);
            double ds, dc;
            pt::pt_sincos(th, &ds, &dc);
            const double ls = std::sin(th), lc = std::cos(th);
            auto wb = [&](double st, double ct) {
                return pt::add(pt::add(pt::add(pt::zero3(), pt::muls(s, radius * ct)), pt::muls(t, radius * st)),
                               pt::muls(nn, std::sqrt(1 - u)));
            };
            flips[1] += !same(wb(ds, dc), wb(ls, lc));
        }
        // Cone
        {
            const double theta0 = U() * 1.2, u = U(), v = U();
            const double th = theta0 * (1 - (2 * std::acos(u) / pt::kPi)), a = v * 2 * pt::kPi;
            const v3 s = unit(g), t = unit(g), dir = unit(g);
            double dm1, dm2, dsa, dca;
            pt::pt_sincos(th, &dm1, &dm2);
            pt::pt_sincos(a, &dsa, &dca);
            auto cone = [&](double m1, double m2, double sa, double ca) {
                return pt::normalize(pt::add(pt::add(pt::add(pt::zero3(), pt::muls(s, m1 * ca)), pt::muls(t, m1 * sa)),
                                             pt::muls(dir, m2)));
            };
            flips[2] += !same(cone(dm1, dm2, dsa, dca), cone(std::sin(th), std::cos(th), std::sin(a), std::cos(a)));
        }
    }
    std::printf("calls per site: %ld\n", n);
    std::printf("sin / cos last-bit differences (RUV arguments, [0, 2pi)): %.3g / %.3g per call\n",
                (double)sc_ulp[0] / n, (double)sc_ulp[1] / n);
    const char* names[3] = {"RandomUnitVector", "WeightedBounce", "Cone"};
    for (int k = 0; k < 3; k++)
        std::printf("%-17s float outputs differ: %ld of %ld calls (%.3g per call)\n", names[k], flips[k], n,
                    (double)flips[k] / n);
    return 0;
}
