// Host check of the Volume marches (ptsharp_amd/csrc/pt_ext.h vol_t / vol_build_runs / t_after):
// vol_t (the per-lane march) and the cooperative march with its strided pass over runs of uniform
// cells (emulated lane by lane) against the reference loop of
// Volume.Intersect (Volume.cs:168-197) restated here position by position, on seeded volumes
// (smooth blobs with noise and exact-zero regions, the reference's narrow windows, Sample's
// y-from-z slip) and seeded rays, bit for bit; and t_after against k repeated additions.
// usage: vol_skip_check [rays per volume]   (exit status 1 on any difference)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <random>
#include <vector>

#include "../../ptsharp_amd/csrc/pt_ext.h"

using namespace pt;

// Volume.Intersect as written: every position sampled
static double naive_t(const DevVolume& v, v3 o, v3 d) {
    double tmin, tmax;
    box_span(v.bmin, v.bmax, o, d, tmin, tmax);
    double step = (double)(1.0f / 512.0f);
    const double start = net_max(step, tmin);
    int sign = -1, iters = 0;
    auto sg_at = [&](double t) { return vol_sign_of(v, vol_sample(v, (double)add(o, muls(d, t)).x, 0, (double)add(o, muls(d, t)).z)); };
    for (double t = start; t <= tmax && iters < (1 << 24); t += step, iters++) {
        const int s = sg_at(t);
        if (s == 0 || (sign >= 0 && s != sign)) {
            t -= step;
            step /= 64;
            t += step;
            for (int i = 0; i < 64; i++) {
                if (sg_at(t) == 0) return t - step;
                t += step;
            }
        }
        sign = s;
    }
    return kHitInf;
}

// pt_device.h coop_vol_t with its strided pass over uniform runs (kVolStride) and the table
// Sign (vol_sign_fast), its 64 lanes as loops: lane r of a round takes the r-th position.
static int sign_fast(const DevVolume& v, v3 o, v3 d, double t) {
    const int s = vol_key_sign(v, vol_key(v, o, d, t));
    if (s > 0) return s;
    return vol_sign(v, add(o, muls(d, t)));
}
static bool box_sign(const DevVolume& v, VolKey a, VolKey b, int sign) {
    const int x0 = std::min(a.x, b.x), y0 = std::min(a.y, b.y), z0 = std::min(a.z, b.z);
    const int nx = std::max(a.x, b.x) - x0, ny = std::max(a.y, b.y) - y0, nz = std::max(a.z, b.z) - z0;
    if (nx > 1 || ny > 1 || nz > 1) return false;
    for (int c = 0; c < 8; c++) {
        const int dx = c & 1, dy = (c >> 1) & 1, dz = c >> 2;
        if (dx > nx || dy > ny || dz > nz) continue;
        if (vol_key_sign(v, VolKey{x0 + dx, y0 + dy, z0 + dz}) != sign) return false;
    }
    return true;
}
static double coop_emul(const DevVolume& v, v3 o, v3 d, int S) {
    const int nact = 64;
    double tmin, tmax;
    box_span(v.bmin, v.bmax, o, d, tmin, tmax);
    double step = (double)(1.0f / 512.0f);
    double t = net_max(step, tmin);
    int sign = -1, iters = 0;
    for (;;) {
        while (S > 0) {
            const VolKey k0 = vol_key(v, o, d, t);
            const int s0 = vol_key_sign(v, k0);
            if (s0 <= 0 || (sign >= 0 && s0 != sign)) break;
            int f = nact;
            VolKey kp = k0;
            for (int r = 0; r < nact; r++) {
                const int off = (r + 1) * S;
                const double tr = t_after(t, step, off);
                const bool valid = tr <= tmax && iters + off < (1 << 24);
                const VolKey kr = vol_key(v, o, d, tr);
                if (!(valid && box_sign(v, kp, kr, s0))) { f = r; break; }
                kp = kr;
            }
            if (f == 0) break;
            const int k = f * S + 1;
            t = t_after(t, step, k);
            iters += k;
            sign = s0;
            if (f < nact) break;
        }
        double tk[64];
        int sg[64];
        bool valid[64];
        for (int r = 0; r < nact; r++) {
            tk[r] = t_after(t, step, r);
            valid[r] = tk[r] <= tmax && iters + r < (1 << 24);
            sg[r] = valid[r] ? sign_fast(v, o, d, tk[r]) : 0;
        }
        int ke = -1;
        for (int r = 0; r < nact && ke < 0; r++) {
            const int prev = r == 0 ? sign : sg[r - 1];
            if (valid[r] && (sg[r] == 0 || (prev >= 0 && sg[r] != prev))) ke = r;
        }
        if (ke < 0) {
            for (int r = 0; r < nact; r++)
                if (!valid[r]) return kHitInf;
            t = tk[nact - 1] + step;
            sign = sg[nact - 1];
            iters += nact;
            continue;
        }
        double tr = tk[ke];
        const int sge = sg[ke];
        tr -= step;
        step /= 64;
        tr += step;
        for (int j = 0; j < 64; j++) {
            if (sign_fast(v, o, d, tr) == 0) return tr - step;
            tr += step;
        }
        t = tr + step;   // the outer loop's t += step, with the refined step
        sign = sge;
        iters += ke + 1;
    }
}

int main(int argc, char** argv) {
    const int rays = argc > 1 ? atoi(argv[1]) : 20000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::normal_distribution<double> N(0.0, 1.0);
    long long bad = 0, total = 0, hits = 0, cbad = 0, sbad = 0;
    double t_skip = 0, t_naive = 0;
    // t_after against repeated addition, across binade crossings
    for (int i = 0; i < 200000; i++) {
        const double step = (i & 1) ? (double)(1.0f / 512.0f) : (double)(1.0f / 512.0f) / 64;
        double t = std::ldexp(U(rng), (int)(U(rng) * 8) - 3) + step;
        const long long k = (long long)(U(rng) * 3000);
        double r = t;
        for (long long j = 0; j < k; j++) r += step;
        if (t_after(t, step, k) != r) {
            if (bad < 5) printf("t_after(%.17g, %g, %lld) = %.17g, repeated %.17g\n", t, step, k, t_after(t, step, k), r);
            bad++;
        }
    }
    printf("t_after: 200000 cases, %lld differences\n", bad);
    {   // vol_zdiv (the reciprocal and two corrections) against the division: fp32 positions and
        // random doubles over zscales with random, all-ones and few-bit significands
        long long zbad = 0, zn = 0;
        std::mt19937_64 g(99);
        for (int s = 0; s < 600; s++) {
            double zs;
            if (s < 3) zs = s == 0 ? 3.4 / 0.9765625 : s == 1 ? (double)(3.4f / 0.9765625f) : 0.37;
            else {
                uint64_t mant = g() & 0x000FFFFFFFFFFFFFull;
                if (s % 3 == 1) mant = 0x000FFFFFFFFFFFFFull - (g() % 64);
                if (s % 3 == 2) mant &= ~((1ull << (g() % 52)) - 1);
                const uint64_t u = mant | ((uint64_t)(1023 + (int)(g() % 16) - 8) << 52);
                memcpy(&zs, &u, 8);
            }
            DevVolume zv{};
            zv.zscale = zs;
            zv.zinv = vol_zinv(zs);
            for (int i = 0; i < 100000; i++) {
                double z;
                if (i & 1) {
                    uint32_t u = (uint32_t)g();
                    u = (u & 0x807FFFFFu) | ((uint32_t)(127 - 40 + (int)(g() % 50)) << 23);
                    float f;
                    memcpy(&f, &u, 4);
                    z = f;
                } else {
                    uint64_t u = g();
                    u = (u & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 60 + (int)(g() % 120)) << 52);
                    memcpy(&z, &u, 8);
                }
                zn++;
                if (vol_zdiv(zv, z) != z / zs) {
                    if (zbad < 5) printf("vol_zdiv(%a) by %a: %a, division %a\n", z, zs, vol_zdiv(zv, z), z / zs);
                    zbad++;
                }
            }
        }
        printf("vol_zdiv against the division: %lld cases, %lld differences\n", zn, zbad);
        bad += zbad;
    }
    // the last volume has 256 narrow windows: a cell above all of them has Sign 257, past the run
    // table's int8 (stored as "no shortcut")
    const int dims[][3] = {{32, 32, 16}, {16, 16, 8}, {48, 48, 24}, {7, 5, 3}, {9, 7, 4}};
    const double zscales[] = {3.4 / 0.9765625, 1.0, 0.37};
    int vi = 0;
    for (const auto& dm : dims)
        for (double zs : zscales) {
            const int w = dm[0], h = dm[1], dd = dm[2];
            std::vector<double> data((size_t)w * h * dd);
            for (int z = 0; z < dd; z++)
                for (int y = 0; y < h; y++)
                    for (int x = 0; x < w; x++) {   // volume_slices-like: blob + noise, clipped, 8-bit
                        const double X = 2.0 * x / (w - 1) - 1, Y = 2.0 * y / (h - 1) - 1, Z = 2.0 * z / (dd - 1) - 1;
                        const double r2 = X * X + 1.3 * Y * Y + 0.8 * Z * Z;
                        double f = 0.75 * std::exp(-1.5 * r2) + 0.08 * N(rng);
                        if ((vi & 1) && X > 0.3) f = 0;   // exact-zero slab
                        f = std::fmin(std::fmax(std::round(f * 255), 0.0), 255.0) / 255;
                        data[(size_t)x + (size_t)y * w + (size_t)z * w * h] = f;
                    }
            std::vector<DevWindow> win;
            if (dm[0] == 9) {
                for (int i = 0; i < 256; i++) {
                    const double lo = (double)(0.001f + 0.0002f * (float)i);
                    win.push_back(DevWindow{lo, (double)((float)lo + 0.00005f), i, 0});
                }
            } else {
                for (int i = 0; i < 5; i++) {
                    const double lo = (double)(0.2f + 0.1f * (float)i);
                    win.push_back(DevWindow{lo, (double)((float)lo + 0.01f), i, 0});
                }
            }
            DevVolume v{};
            v.data = data.data();
            v.windows = win.data();
            v.w = w; v.h = h; v.d = dd; v.nwin = (int)win.size();
            v.zscale = zs;
            v.zinv = vol_zinv(zs);   // the device's Sample arithmetic (vol_zdiv); naive_t divides (vref)
            const float bmn[3] = {-1, -1, -0.2f}, bmx[3] = {1, 1, 1};
            for (int k = 0; k < 3; k++) { v.bmin[k] = bmn[k]; v.bmax[k] = bmx[k]; }
            std::vector<int8_t> runs((size_t)(w + 1) * (h + 1) * (dd + 1));
            vol_build_runs(v, runs.data(), v.zero_sign);
            v.runs = runs.data();
            // the device's cell-major corners (vol_build_cells): vol_t, vol_sign_at and the emulated cooperative
            // march read them, the loop as written (naive_t, vref) reads the grid
            std::vector<double> cells(8 * runs.size());
            vol_build_cells(v, cells.data());
            v.cells = cells.data();
            long long uni = 0;
            for (int8_t r : runs) uni += r != 0;
            long long vbad = 0;
            for (int i = 0; i < rays; i++) {
                v3 o, dir;
                const int kind = i % 5;
                o = v3{(float)(U(rng) * 4 - 2), (float)(U(rng) * 4 - 2), (float)(U(rng) * 3 - 1.2)};
                v3 aim{(float)(U(rng) * 2 - 1), (float)(U(rng) * 2 - 1), (float)(U(rng) * 1.2 - 0.2)};
                dir = normalize(sub(aim, o));
                if (kind == 1) dir = normalize(v3{dir.x, dir.y, 0.0f});    // d.z = 0
                if (kind == 2) dir = normalize(v3{0.0f, dir.y, dir.z});    // d.x = 0
                if (kind == 3) o = aim;                                   // origin inside the box
                if (kind == 4) {   // grazing: nearly parallel to the x planes, origin on a lattice plane
                    dir = normalize(v3{(float)(1e-6 * (U(rng) - 0.5)), dir.y, dir.z});
                    if (i & 8) o.x = (float)(2.0 * (int)(U(rng) * w) / w - 1.0);
                }
                if (!(dir.x == dir.x)) continue;
                uint32_t n = 0;
                const auto c0 = std::chrono::steady_clock::now();
                const double a = vol_t(v, o, dir, &n);
                const auto c1 = std::chrono::steady_clock::now();
                DevVolume vref = v;
                vref.zinv = 0.0;
                vref.cells = nullptr;
                const double b = naive_t(vref, o, dir);
                const auto c2 = std::chrono::steady_clock::now();
                t_skip += std::chrono::duration<double>(c1 - c0).count();
                t_naive += std::chrono::duration<double>(c2 - c1).count();
                {   // pt_ext.h vol_sign_at (the device march's Sign) against the key and the sample taken apart
                    double tmn, tmx;
                    box_span(v.bmin, v.bmax, o, dir, tmn, tmx);
                    if (tmx > tmn)
                        for (int j = 0; j < 16; j++) {
                            const double t = std::fmax(tmn, 0.0) + (tmx - std::fmax(tmn, 0.0)) * U(rng);
                            if (vol_sign_at(v, o, dir, t) != sign_fast(v, o, dir, t)) {
                                if (sbad < 5) printf("vol %d ray %d t %.17g: vol_sign_at %d, key / sample %d\n", vi, i, t,
                                                     vol_sign_at(v, o, dir, t), sign_fast(v, o, dir, t));
                                sbad++;
                            }
                        }
                }
                for (int S : {8, 16, 32}) {
                    const double c = coop_emul(v, o, dir, S);
                    if (c != b && !(c != c && b != b)) {
                        if (cbad < 5) printf("vol %d ray %d stride %d: coop %.17g naive %.17g\n", vi, i, S, c, b);
                        cbad++;
                    }
                }
                total++;
                hits += b < kHitInf;
                if (a != b && !(a != a && b != b)) {
                    if (vbad < 5)
                        printf("vol %d ray %d: vol_t %.17g naive %.17g  o=(%a,%a,%a) d=(%a,%a,%a)\n", vi, i, a, b, o.x, o.y, o.z,
                               dir.x, dir.y, dir.z);
                    vbad++;
                }
            }
            printf("volume %dx%dx%d zscale %.4g: %lld of %zu cells uniform, zero sign %d, %d rays, %lld differences\n", w, h,
                   dd, zs, uni, runs.size(), v.zero_sign, rays, vbad);
            bad += vbad;
            vi++;
        }
    printf("vol_sign_at against the key and the sample taken apart: %lld differences\n", sbad);
    printf("cooperative march with the strided pass (strides 8, 16, 32), emulated: %lld differences\n", cbad);
    bad += cbad;
    printf("%lld rays, %lld hits, %lld differences; vol_t %.3f s, the loop as written %.3f s\n", total, hits, bad, t_skip,
           t_naive);
    return bad ? 1 : 0;
}
