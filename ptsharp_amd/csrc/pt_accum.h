// pt_accum.h — order-independent accumulation of path contributions (both engines).
//
// RenderParallel sums a pixel's spp sample colours in fp64 (Renderer.cs:292-306) and each
// sample is the recursion's fp64 sum of emission, environment and direct-light terms
// (Sampler.cs:55-145).  On the GPU the terms of one pixel arrive from many threads in an
// order set by queue-slot atomics, so an fp64 atomic sum differs in its last bits from
// run to run.  Here every term x (fp64) is split into integers before it is added:
//
//     s = x·2^12,  hi = floor(s) (int64),  lo = round((s − hi)·2^40) ∈ [0, 2^40]
//
// and a pixel keeps Σhi and Σlo per channel in two 64-bit words.  Integer addition is
// associative, so the sums — and the fp64 value made from them at finalize,
// (Σhi + ⌊Σlo/2^40⌋)·2^-12 + (Σlo mod 2^40)·2^-52 — are the same bits whatever order the
// terms arrive in, on any engine, rank split or run.  Resolution 2^-52 absolute per term;
// Σlo cannot wrap before 2^24 terms per pixel per pass.  Terms with |x| ≥ 2^39, or not
// finite, go to an fp64 side sum instead (only pathological scenes produce them; a NaN or
// an infinity then propagates as it does in the reference).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace pt {

constexpr double kFixHiScale = 4096.0;                   // 2^12
constexpr double kFixLoScale = 1099511627776.0;          // 2^40
constexpr double kFixBig = 549755813888.0;               // |x| ≥ 2^39: side sum
constexpr double kFixMagicHi = 6755399441055744.0;       // 1.5·2^52: an integer f with |f| < 2^51 is bits(f + M) − bits(M)
constexpr double kFixMagicLo = 4503599627370496.0;       // 2^52: round(y) for y ∈ [0, 2^40] is the low mantissa of y + 2^52
constexpr unsigned long long kFixLoMask = (1ull << 40) - 1ull;
constexpr int kFixWords = 6;                             // {Σhi r, g, b, Σlo r, g, b}

// Accumulators of n pixels (or samples): w [n][6] 64-bit words, big [n][3] fp64.
struct FixAcc {
    unsigned long long* w;
    double* big;
};

struct Fix {
    long long hi;
    unsigned long long lo;
};

__device__ __forceinline__ bool fix_ok(double x) { return fabs(x) < kFixBig; }   // false for NaN too

// x with fix_ok(x): s = x·2^12 and f = floor(s) are exact (|s| < 2^51), s − f is exact (its
// bits are s's fraction bits) and so is the scaling by 2^40; only the lo rounding rounds
// (to nearest even, like rint).  The integers come out of the mantissa of a magic-number
// sum (no fp64 → int64 conversion, which gfx950 does not have as one instruction).
__device__ __forceinline__ Fix to_fix(double x) {
    const double s = x * kFixHiScale;
    const double f = floor(s);
    const long long hi = __double_as_longlong(f + kFixMagicHi) - __double_as_longlong(kFixMagicHi);
    const unsigned long long lo =
        (unsigned long long)(__double_as_longlong((s - f) * kFixLoScale + kFixMagicLo) - __double_as_longlong(kFixMagicLo));
    return Fix{hi, lo};
}

__device__ __forceinline__ double fix_value(long long hi, unsigned long long lo) {
    const long long h = hi + (long long)(lo >> 40);
    return (double)h * (1.0 / kFixHiScale) + (double)(lo & kFixLoMask) * (1.0 / (kFixHiScale * kFixLoScale));
}

// Per-lane register accumulator (the megakernel's samples).
struct FixReg {
    long long hi[3];
    unsigned long long lo[3];
    double big[3];
};
__device__ __forceinline__ void fixreg_clear(FixReg& a) {
    for (int k = 0; k < 3; k++) { a.hi[k] = 0; a.lo[k] = 0; a.big[k] = 0.0; }
}
__device__ __forceinline__ void fixreg_add(FixReg& a, int k, double x) {
    if (x == 0.0) return;
    if (!fix_ok(x)) { a.big[k] += x; return; }
    const Fix f = to_fix(x);
    a.hi[k] += f.hi;
    a.lo[k] += f.lo;
}
__device__ __forceinline__ void fixreg_add3(FixReg& a, double r, double g, double b) {
    fixreg_add(a, 0, r);
    fixreg_add(a, 1, g);
    fixreg_add(a, 2, b);
}
__device__ __forceinline__ double fixreg_value(const FixReg& a, int k) { return fix_value(a.hi[k], a.lo[k]) + a.big[k]; }

// One lane's term into accumulator i (non-returning 64-bit integer atomics at L2).
__device__ __forceinline__ void fix_add_lane(const FixAcc& A, size_t i, double r, double g, double b) {
    unsigned long long* w = A.w + kFixWords * i;
    const double x[3] = {r, g, b};
    for (int k = 0; k < 3; k++) {
        if (x[k] == 0.0) continue;
        if (!fix_ok(x[k])) { atomicAdd(A.big + 3 * i + k, x[k]); continue; }
        const Fix f = to_fix(x[k]);
        if (f.hi) atomicAdd(w + k, (unsigned long long)f.hi);
        if (f.lo) atomicAdd(w + 3 + k, f.lo);
    }
}

// Wave-aggregated fix_add_lane: lanes of a wave often add to the same accumulator (a
// pixel's samples sit in consecutive queue slots), and same-address atomics serialise at
// L2.  Lanes are grouped into runs of equal `idx` (segment ids from a ballot of run heads);
// each run's integer terms are summed by a segmented suffix scan over shuffles (exact, so
// the lane order inside a run does not matter) and the run's head issues the atomics.
// Wave-uniform call; lanes with has = false add nothing.
// Returns the number of runs (atomic sets) the wave issued.
__device__ __forceinline__ uint32_t fix_add_wave(const FixAcc& A, uint32_t idx, bool has, double r, double g, double b) {
    if (__ballot(has) == 0ull) return 0u;   // wave-uniform: nothing to add
    const int lane = threadIdx.x & 63;
    const double x[3] = {r, g, b};
    bool big = false;
    long long hi[3];
    unsigned long long lo[3];
    for (int k = 0; k < 3; k++) {
        hi[k] = 0; lo[k] = 0;
        if (!has || x[k] == 0.0) continue;
        if (!fix_ok(x[k])) { big = true; continue; }
        const Fix f = to_fix(x[k]);
        hi[k] = f.hi; lo[k] = f.lo;
    }
    if (big) {   // rare: the side sum, per lane
        for (int k = 0; k < 3; k++)
            if (x[k] != 0.0 && !fix_ok(x[k])) atomicAdd(A.big + 3 * (size_t)idx + k, x[k]);
    }
    // Runs are taken over the lanes that add: a lane without a term does not split its
    // neighbours' run (it adds zero to the run it sits in).  Head = an adding lane whose previous
    // adding lane has another idx (or none).
    const uint64_t adders = __ballot(has);
    const uint64_t below = adders & ((1ull << lane) - 1ull);
    const int prev_lane = below ? 63 - __builtin_clzll(below) : lane;
    const uint32_t prev = __shfl(idx, prev_lane, 64);
    const bool head = has && (below == 0ull || prev != idx);
    const uint64_t heads = __ballot(head);
    // A run spans its head to its last adder; lanes without a term inside that span belong to it
    // (they pass sums through), the others to no run (a segment id of their own).
    const uint64_t above = adders & ~((2ull << lane) - 1ull);
    const int nxt = above ? __builtin_ctzll(above) : 64;
    const bool inside = has || (below != 0ull && nxt < 64 && !((heads >> nxt) & 1ull));
    const int seg = inside ? __popcll(heads & (~0ull >> (63 - lane))) : -1 - lane;
    for (int off = 1; off < 64; off <<= 1) {   // suffix sums within a run
        const int so = __shfl_down(seg, off, 64);
        const bool take = lane + off < 64 && so == seg;
        if (__ballot(take) == 0ull) break;     // every run spans at most `off` lanes: sums complete
        for (int k = 0; k < 3; k++) {
            const long long uh = __shfl_down(hi[k], off, 64);
            const unsigned long long ul = __shfl_down(lo[k], off, 64);
            if (take) { hi[k] += uh; lo[k] += ul; }
        }
    }
    if (head) {
        unsigned long long* w = A.w + kFixWords * (size_t)idx;
        for (int k = 0; k < 3; k++) {
            if (hi[k]) atomicAdd(w + k, (unsigned long long)hi[k]);
            if (lo[k]) atomicAdd(w + 3 + k, lo[k]);
        }
    }
    return (uint32_t)__popcll(heads);
}

// Value of accumulator i (then cleared for the next pass).
__device__ __forceinline__ void fix_take(const FixAcc& A, size_t i, double out[3]) {
    unsigned long long* w = A.w + kFixWords * i;
    double* bg = A.big + 3 * i;
    for (int k = 0; k < 3; k++) {
        out[k] = fix_value((long long)w[k], w[3 + k]) + bg[k];
        w[k] = 0ull; w[3 + k] = 0ull; bg[k] = 0.0;
    }
}

}  // namespace pt
