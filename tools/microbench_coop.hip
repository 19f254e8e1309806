// Cooperative vs per-lane node fetch (BVH-traversal-like dependent chase over random
// 128-B nodes).  per-lane: every lane loads its own node with 7 x 16-B loads (64 distinct
// lines per load instruction).  coop: the 8 lanes of a group load the group's nodes, one
// node per instruction (8 lanes x 16 B = one line, 8 lines per instruction), stage them
// through LDS and each lane reads its own node back (7 x ds_read_b128; rows XOR-swizzled).
// STAGE = nodes staged at once per wave (64: one pass; 32: two passes of half the lanes, half
// the LDS).  Every kernel also holds STK bytes of LDS per thread (the traversal stack), so
// occupancy is the real kernel's.  Working sets: L2-resident, a "tree" set (79 MB, 60 % of
// the steps in a 2 MB hot set: the measured L2 hit rate of the closest-hit kernel) and 96 MB
// uniform.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench_coop tools/microbench_coop.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}

__global__ void k_fill(uint32_t* b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = hash32((uint32_t)i * 0x9E3779B9u + 12345u);
}

__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// next node: with a hot mask, 10 of 16 steps stay in the hot set
__device__ __forceinline__ uint32_t next_idx(uint32_t x, int s, uint32_t mask, uint32_t hot) {
    const uint32_t h = hash32(x ^ (uint32_t)s);
    return ((h >> 28) < 10u ? h & hot : h) & mask;
}

template <int WAVES, int STK>
__global__ __launch_bounds__(256, WAVES) void k_lane(const uint4* __restrict__ buf, uint32_t mask, uint32_t hot, int steps,
                                                     int active, uint32_t* out) {
    __shared__ uint32_t stk[STK / 4 * 256];
    const uint32_t lane = threadIdx.x & 63u, gid = blockIdx.x * 256u + threadIdx.x;
    uint32_t idx = hash32(gid) & mask, acc = 0;
    stk[threadIdx.x] = gid;
    if (lane < (uint32_t)active) {
        for (int s = 0; s < steps; s++) {
            const uint4* p = buf + (size_t)idx * 8;
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) x ^= fold(p[k]);
            acc += x;
            idx = next_idx(x, s, mask, hot);
        }
    }
    out[gid] = acc + stk[(threadIdx.x * 7) & 255];
}

template <int WAVES, int STAGE, int STK>
__global__ __launch_bounds__(256, WAVES) void k_coop(const uint4* __restrict__ buf, uint32_t mask, uint32_t hot, int steps,
                                                     int active, uint32_t* out) {
    __shared__ uint4 stage[4][STAGE * 8];
    __shared__ uint32_t stk[STK / 4 * 256];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, gid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t grp = lane & ~7u, piece = lane & 7u;
    uint4* st = stage[wave];
    stk[threadIdx.x] = gid;
    uint32_t idx = hash32(gid) & mask, acc = 0;
    const bool on = lane < (uint32_t)active;
    for (int s = 0; s < steps; s++) {
        uint32_t x = 0;
        uint4 v[8];   // every load issued before any LDS hand-off: one memory round trip per step
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t src = grp + (uint32_t)j;
            const uint32_t nidx = __shfl(idx, (int)src, 64);
            v[j] = make_uint4(0u, 0u, 0u, 0u);
            if (src < (uint32_t)active && piece < 7) v[j] = buf[(size_t)nidx * 8 + piece];
        }
#pragma unroll
        for (int h = 0; h < 64 / STAGE; h++) {
            // pass h stages the nodes of lanes with (lane & 7) in [h*STAGE/8, (h+1)*STAGE/8)
#pragma unroll
            for (int j = 0; j < STAGE / 8; j++) {
                const uint32_t row = (grp >> 3) * (STAGE / 8) + (uint32_t)j;   // staging row of lane grp + h*STAGE/8 + j
                if (piece < 7) st[row * 8 + (piece ^ (row & 7u))] = v[h * (STAGE / 8) + j];
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
            const uint32_t mj = piece - (uint32_t)(h * (STAGE / 8));
            if (on && mj < (uint32_t)(STAGE / 8)) {
                const uint32_t row = (grp >> 3) * (STAGE / 8) + mj;
#pragma unroll
                for (int k = 0; k < 7; k++) x ^= fold(st[row * 8 + ((uint32_t)k ^ (row & 7u))]);
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
        }
        acc += x;
        idx = next_idx(x, s, mask, hot);
    }
    out[gid] = acc + stk[(threadIdx.x * 7) & 255];
}

template <class F>
static void timeit(const char* name, F launch, double lane_steps, int cus) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    launch();
    CK(hipGetLastError());
    CK(hipEventRecord(a));
    for (int r = 0; r < 3; r++) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 3;
    printf("%-44s %.3f ms  lane-steps %.2f G/s  CU-cycles per lane-step %.2f\n", name, ms, lane_steps / ms / 1e6,
           (ms * 1e-3 * 2.4e9 * cus) / lane_steps);
    fflush(stdout);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const size_t maxb = (size_t)96 << 20;
    uint4* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, maxb));
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)buf, maxb / 4);
    CK(hipDeviceSynchronize());
    struct WS { const char* name; size_t bytes; size_t hot; };
    const WS ws[3] = {{"L2-resident 2 MB", (size_t)2 << 20, 0}, {"tree 79 MB (60 % in 2 MB)", (size_t)79 << 20, (size_t)2 << 20},
                      {"uniform 96 MB", (size_t)96 << 20, 0}};
    const int steps = 256;
    auto pmask = [](size_t w) { uint32_t m = 1; while ((size_t)m * 2 <= w / 128) m *= 2; return m - 1; };
    for (const WS& w : ws) {
        const uint32_t mask = pmask(w.bytes), hot = w.hot ? pmask(w.hot) : 0xFFFFFFFFu;
        printf("working set %s\n", w.name);
        for (int active : {64, 40}) {
            char nm[96];
            auto run = [&](const char* tag, int waves, auto kern) {
                const int blocks = cus * waves;
                const double ls = (double)blocks * 4 * active * steps;
                snprintf(nm, sizeof nm, "%s waves=%d active=%d", tag, waves, active);
                timeit(nm, [&] { hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, buf, mask, hot, steps, active, out); },
                       ls, cus);
            };
            run("per-lane (stack 64B)", 6, k_lane<6, 64>);
            run("coop stage64 (stack 64B)", 3, k_coop<3, 64, 64>);
            run("coop stage32 (stack 64B)", 5, k_coop<5, 32, 64>);
            run("coop stage32 (stack 32B)", 6, k_coop<6, 32, 32>);
            run("coop stage16 (stack 64B)", 6, k_coop<6, 16, 64>);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
