// pt_accum.h — order-independent accumulation of path contributions (both engines).
//
// RenderParallel sums a pixel's spp sample colours in fp64 (Renderer.cs:292-306) and each
// sample is the recursion's fp64 sum of emission, environment and direct-light terms
// (Sampler.cs:55-145).  On the GPU the terms of one pixel arrive from many threads in an
// order set by queue-slot atomics, so an fp64 atomic sum differs in its last bits from
// run to run.  Here every term x (fp64) becomes an integer first,
//
//     V = round(x·2^44)   (|x| < 2^19, so |V| < 2^63),
//
// and a pixel keeps, per channel, the 128-bit sum T = Σ V as a 64-bit low word (one
// returning integer atomic per term) and a 64-bit high word that only sees the rare carry
// out of the low word (the atomic's returned old value tells exactly which add wrapped).
// Integer addition is associative, so T — and the fp64 value made from it at finalize,
// T·2^-44 — is the same bits whatever order the terms arrive in, on any engine, rank split
// or run.  Resolution 2^-44 (5.7e-14) absolute per term.  Terms with |x| ≥ 2^19, or not
// finite, go to an fp64 side sum instead (only pathological scenes produce them; a NaN or
// an infinity then propagates as it does in the reference).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace pt {

constexpr double kFixHiScale = 4096.0;                   // 2^12: V = floor(x·2^12)·2^32 + round(frac·2^32)
constexpr double kFixLoScale = 4294967296.0;             // 2^32
constexpr double kFixBig = 524288.0;                     // |x| ≥ 2^19: side sum
constexpr double kFixWave = 8192.0;                      // |x| < 2^13: |V| < 2^57, 64 of them sum without overflow
constexpr double kFixMagicLo = 4503599627370496.0;       // 2^52: round(y), y ∈ [0, 2^32], is the low mantissa of y + 2^52
constexpr int kFixWords = 3;                             // words per accumulator in w (hi: its own array, the same stride)

// Accumulators of n pixels (or samples), channel-planar: the low words w [3][n], the high words
// hi [3][n] (touched only by a carry out of the low word, so the atomics' working set is w alone),
// big [3][n] fp64.  Planar because integer atomics execute at the memory side, one request per
// 64-B segment a wave instruction touches (MI355X_MICROARCH.md "Global float atomics": 64 rows ≈17×
// slower than 256 contiguous bytes): a wave adding channel k for 64 consecutive accumulators touches
// 512 contiguous bytes (8 segments) here, against 24 segments with the three channels interleaved
// ([n][3], 24 B per accumulator).  `n` is the plane stride.
struct FixAcc {
    unsigned long long* w;
    unsigned long long* hi;
    double* big;
    uint64_t n;
};
__device__ __forceinline__ size_t fix_at(const FixAcc& A, size_t i, int k) { return (size_t)k * A.n + i; }

__device__ __forceinline__ bool fix_ok(double x) { return fabs(x) < kFixBig; }   // false for NaN too

// x with fix_ok(x): s = x·2^12 and floor(s) are exact and |floor(s)| < 2^31 (a native fp64 →
// int32 conversion), s − floor(s) ∈ [0, 1) is exact (its bits are s's fraction bits), its scaling
// by 2^32 is exact, and only the magic-number sum rounds (to nearest even, like llrint).
__device__ __forceinline__ long long to_fix(double x) {
    const double s = x * kFixHiScale;
    const double f = floor(s);
    const long long lo =
        __double_as_longlong((s - f) * kFixLoScale + kFixMagicLo) - __double_as_longlong(kFixMagicLo);
    return (long long)(int)f * 4294967296ll + lo;
}

// T = hi·2^64 + lo (hi signed) → T·2^-44.  When T fits 64 signed bits (hi is lo's sign
// extension: every sum of a few terms, negative ones included) it is converted in one step; the
// two-word form would round a negative T's lo (near 2^64) to a multiple of 2^11 first and then
// cancel it against hi·2^64, losing most of the 2^-44 resolution.
__device__ __forceinline__ double fix_value(long long hi, unsigned long long lo) {
    if (hi == ((long long)lo >> 63)) return (double)(long long)lo * (1.0 / 17592186044416.0);
    return (double)hi * 1048576.0 + (double)lo * (1.0 / 17592186044416.0);
}

// Per-lane register accumulator (the megakernel's samples): the same 128-bit sums.
struct FixReg {
    unsigned long long lo[3];
    long long hi[3];
    double big[3];
};
__device__ __forceinline__ void fixreg_clear(FixReg& a) {
    for (int k = 0; k < 3; k++) { a.lo[k] = 0; a.hi[k] = 0; a.big[k] = 0.0; }
}
__device__ __forceinline__ void fixreg_add(FixReg& a, int k, double x) {
    if (x == 0.0) return;
    if (!fix_ok(x)) { a.big[k] += x; return; }
    const long long v = to_fix(x);
    const unsigned long long old = a.lo[k];
    a.lo[k] = old + (unsigned long long)v;
    a.hi[k] += (v < 0 ? -1 : 0) + (a.lo[k] < old ? 1 : 0);
}
__device__ __forceinline__ void fixreg_add3(FixReg& a, double r, double g, double b) {
    fixreg_add(a, 0, r);
    fixreg_add(a, 1, g);
    fixreg_add(a, 2, b);
}
__device__ __forceinline__ double fixreg_value(const FixReg& a, int k) { return fix_value(a.hi[k], a.lo[k]) + a.big[k]; }

// v (a fixed-point sum, as a signed 64-bit value) into channel k of accumulator i: one
// returning atomic on the low word; the high word gets the carry (and v's sign extension).
__device__ __forceinline__ void fix_atomic(const FixAcc& A, size_t i, int k, long long v) {
    const unsigned long long old = atomicAdd(A.w + fix_at(A, i, k), (unsigned long long)v);
    const unsigned long long now = old + (unsigned long long)v;
    const long long dh = (v < 0 ? -1 : 0) + (now < old ? 1 : 0);
    if (dh) atomicAdd(A.hi + fix_at(A, i, k), (unsigned long long)dh);
}

// One lane's term into accumulator i.
__device__ __forceinline__ void fix_add_lane(const FixAcc& A, size_t i, double r, double g, double b) {
    const double x[3] = {r, g, b};
    for (int k = 0; k < 3; k++) {
        if (x[k] == 0.0) continue;
        if (!fix_ok(x[k])) { atomicAdd(A.big + fix_at(A, i, k), x[k]); continue; }
        fix_atomic(A, i, k, to_fix(x[k]));
    }
}

// Wave-aggregated fix_add_lane: lanes of a wave often add to the same accumulator (a
// pixel's samples sit in consecutive queue slots), and same-address atomics serialise at
// the memory side.  The adding lanes are grouped into runs of equal `idx`; each run's
// integer terms are summed by a segmented suffix scan over shuffles (exact, so the lane
// order inside a run does not matter) and the run's head issues the atomics.  A lane with
// a term of 2^13 or more adds it on its own (a run's sum must stay inside 63 bits).
// Wave-uniform call; lanes with has = false add nothing.  Returns the runs issued.
// A block's LDS table of run sums (k_wf_nee_accum): open addressing on the accumulator index,
// TABLE entries of {key, three 64-bit sums}.  Terms below kFixLds (|V| < 2^50) only, so a
// window of up to 2^12 of them per key sums without overflow; the block flushes the table
// into the 128-bit accumulators (fix_atomic) after each window.
constexpr double kFixLds = 64.0;
constexpr uint32_t kLdsFree = 0xFFFFFFFFu;
struct LdsFix {
    uint32_t* key;               // [n], kLdsFree = free
    unsigned long long* sum;     // [n][3]
    uint32_t mask;               // n - 1 (n a power of two)
};
// A run's sums into the table; false if its probe sequence is full (the caller adds globally).
__device__ __forceinline__ bool lds_fix_add(const LdsFix& T, uint32_t idx, const long long v[3]) {
    // the index itself (linear probing): the flush walks the table in slot order, so neighbouring
    // accumulators' atomics leave in one wave instruction (8-B lanes on few 64-B segments; a
    // multiplicative hash scattered them, one segment per lane: C5 nee_accum 115 -> 88 ms, r05nee).
    // Each 512-index block is shifted by 8 slots per block: pixels a row apart differ by W,
    // and with idx alone rows 4 apart collided at W = 1920, 2 apart at 3840, every row at a power-of-two
    // width; runs of one row stay contiguous.
#ifndef PT_ACC_ROWSHIFT
#define PT_ACC_ROWSHIFT 1   // 0: the index alone (round 5; A/B builds)
#endif
    const uint32_t home = PT_ACC_ROWSHIFT ? idx + (idx >> 9) * 8u : idx;
    for (uint32_t p = 0; p < 8u; p++) {
        const uint32_t sl = (home + p) & T.mask;
        const uint32_t k = atomicCAS(T.key + sl, kLdsFree, idx);
        if (k == kLdsFree || k == idx) {
            for (int c = 0; c < 3; c++)
                if (v[c]) atomicAdd(T.sum + 3u * sl + c, (unsigned long long)v[c]);
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ uint32_t fix_add_wave(const FixAcc& A, uint32_t idx, bool has, double r, double g, double b,
                                                 const LdsFix* T = nullptr) {
    if (__ballot(has) == 0ull) return 0u;   // wave-uniform: nothing to add
    const int lane = threadIdx.x & 63;
    const double x[3] = {r, g, b};
    const double lim = T ? kFixLds : kFixWave;
    bool alone = false;
    long long v[3];
    for (int k = 0; k < 3; k++) {
        v[k] = 0;
        if (!has || x[k] == 0.0) continue;
        if (!(fabs(x[k]) < lim)) { alone = true; continue; }
        v[k] = to_fix(x[k]);
    }
    if (alone) {   // rare: large (or side-sum) terms, added per lane
        for (int k = 0; k < 3; k++)
            if (x[k] != 0.0 && !(fabs(x[k]) < lim)) {
                if (!fix_ok(x[k])) atomicAdd(A.big + fix_at(A, idx, k), x[k]);
                else fix_atomic(A, idx, k, to_fix(x[k]));
            }
    }
    // Runs are taken over the lanes that add: a lane without a term does not split its
    // neighbours' run.  Head = an adding lane whose previous adding lane has another idx (or none).
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
            const long long u = __shfl_down(v[k], off, 64);
            if (take) v[k] += u;
        }
    }
    if (head && (v[0] | v[1] | v[2]) && !(T && lds_fix_add(*T, idx, v))) {
        for (int k = 0; k < 3; k++)
            if (v[k]) fix_atomic(A, idx, k, v[k]);
    }
    return (uint32_t)__popcll(heads);
}

// Value of accumulator i (then cleared for the next pass).
__device__ __forceinline__ void fix_take(const FixAcc& A, size_t i, double out[3]) {
    for (int k = 0; k < 3; k++) {
        const size_t j = fix_at(A, i, k);
        out[k] = fix_value((long long)A.hi[j], A.w[j]) + A.big[j];
        A.w[j] = 0ull; A.hi[j] = 0ull; A.big[j] = 0.0;
    }
}

}  // namespace pt
