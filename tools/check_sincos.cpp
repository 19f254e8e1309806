// Host check of the device fp64 sincos (ptsharp_amd/csrc/pt_math.h pt_sincos, restated here
// for g++): ulp distance to glibc's sin / cos over 2e7 arguments in [0, 2π] and [0, 1.2], and
// whether r·sin / r·cos rounded to float ever differ.
// usage: g++ -O2 -ffp-contract=off -fno-builtin-sin -fno-builtin-cos -o /tmp/cs tools/check_sincos.cpp && /tmp/cs
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>
static inline void ksc(double x, double y, double& s, double& c) {
    const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03, S3 = -1.98412698298579493134e-04,
                 S4 = 2.75573137070700676789e-06, S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
    const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03, C3 = 2.48015872894767294178e-05,
                 C4 = -2.75573143513906633035e-07, C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
    double z = x * x, w = z * z;
    double r = S2 + z * (S3 + z * S4) + z * w * (S5 + z * S6);
    double v = z * x;
    s = x - ((z * (0.5 * y - v * r) - y) - v * S1);
    double rc = z * (C1 + z * (C2 + z * C3)) + w * w * (C4 + z * (C5 + z * C6));
    double hz = 0.5 * z;
    double ww = 1.0 - hz;
    c = ww + (((1.0 - ww) - hz) + (z * rc - x * y));
}
static inline void my_sincos(double x, double* sp, double* cp) {
    const double hi = 1.5707963267948966, lo = 6.123233995736766e-17, tpi = 0.63661977236758134;
    double k = std::rint(x * tpi);
    double ph = k * hi;
    double pe = std::fma(k, hi, -ph);
    double r = x - ph;
    double cc = pe + k * lo;
    double y0 = r - cc;
    double y1 = (r - y0) - cc;
    double s, c;
    ksc(y0, y1, s, c);
    int q = (int)k & 3;
    double so = (q & 1) ? c : s, co = (q & 1) ? s : c;
    if (q == 1 || q == 2) co = -co;
    if (q >= 2) so = -so;
    *sp = so; *cp = co;
}
static int64_t ulpd(double a, double b) { int64_t ia, ib; memcpy(&ia,&a,8); memcpy(&ib,&b,8); if (ia<0) ia = INT64_MIN - ia; if (ib<0) ib = INT64_MIN - ib; return ia>ib?ia-ib:ib-ia; }
int main() {
    std::mt19937_64 g(1);
    int64_t maxs = 0, maxc = 0, diffs = 0, diffc = 0, fdiff = 0;
    const long N = 20000000;
    for (long i = 0; i < N; i++) {
        double u = (double)(g() >> 11) * (1.0 / 9007199254740992.0);
        double x = u * 2.0 * 3.141592653589793;
        if (i % 4 == 1) x = u * 1.2;
        if (i % 4 == 2) x = (double)(float)(u*2*3.141592653589793);
        double s1, c1, s2, c2;
        s1 = sin(x); c1 = cos(x);
        my_sincos(x, &s2, &c2);
        int64_t a = ulpd(s1, s2), b = ulpd(c1, c2);
        maxs = a > maxs ? a : maxs; maxc = b > maxc ? b : maxc;
        diffs += a != 0; diffc += b != 0;
        double r = 0.7312345;
        if ((float)(r * s1) != (float)(r * s2) || (float)(r * c1) != (float)(r * c2)) fdiff++;
    }
    printf("max ulp sin %lld cos %lld, differing sin %lld cos %lld of %ld, float-result diffs %lld\n",
           (long long)maxs, (long long)maxc, (long long)diffs, (long long)diffc, N, (long long)fdiff);
    // special points
    double xs[] = {0.0, 1e-300, 1.5707963267948966, 3.141592653589793, 4.71238898038469, 6.283185307179586, 0.7853981633974483};
    for (double x : xs) { double s, c; my_sincos(x, &s, &c); printf("%.17g: %.17g %.17g | %.17g %.17g\n", x, s, c, sin(x), cos(x)); }
}
