// Cooperative vs per-lane node fetch (BVH-traversal-like dependent chase over random
// 128-B nodes).  per-lane: every lane loads its own node with 7 x 16-B loads (64 distinct
// lines per load instruction).  coop: the 8 lanes of a group load the 8 nodes of the
// group, one node per instruction (8 lanes x 16 B = one line, 8 lines per instruction),
// stage them through LDS and each lane reads its own node back (7 x ds_read_b128).
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

template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_lane(const uint4* __restrict__ buf, uint32_t mask, int steps, int active,
                                                     uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u, gid = blockIdx.x * 256u + threadIdx.x;
    uint32_t idx = hash32(gid) & mask, acc = 0;
    if (lane < (uint32_t)active) {
        for (int s = 0; s < steps; s++) {
            const uint4* p = buf + (size_t)idx * 8;
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) x ^= fold(p[k]);
            acc += x;
            idx = (x ^ (uint32_t)s) & mask;
        }
    }
    out[gid] = acc;
}

constexpr int kRow = 9;   // uint4 per staged node row (8 + 1 pad: rows start on different banks)

template <int WAVES>
__global__ __launch_bounds__(256, WAVES) void k_coop(const uint4* __restrict__ buf, uint32_t mask, int steps, int active,
                                                     uint32_t* out) {
    __shared__ uint4 stage[4][64 * kRow];
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6, gid = blockIdx.x * 256u + threadIdx.x;
    const uint32_t grp = lane & ~7u, piece = lane & 7u;
    uint4* st = stage[wave];
    uint32_t idx = hash32(gid) & mask, acc = 0;
    const bool on = lane < (uint32_t)active;
    for (int s = 0; s < steps; s++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t src = grp + (uint32_t)j;                 // node of lane src
            const uint32_t nidx = __shfl(idx, (int)src, 64);
            if (src < (uint32_t)active && piece < 7) st[src * kRow + piece] = buf[(size_t)nidx * 8 + piece];
        }
        __builtin_amdgcn_s_waitcnt(0);   // wave-local LDS hand-off: own writes, then reads
        __builtin_amdgcn_wave_barrier();
        uint32_t x = 0;
        if (on) {
#pragma unroll
            for (int k = 0; k < 7; k++) x ^= fold(st[lane * kRow + k]);
        }
        __builtin_amdgcn_wave_barrier();
        acc += x;
        idx = (x ^ (uint32_t)s) & mask;
    }
    out[gid] = acc;
}

template <class F>
static void timeit(const char* name, F launch, double lane_steps, int cus) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    launch();
    CK(hipEventRecord(a));
    for (int r = 0; r < 3; r++) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 3;
    printf("%-34s %.3f ms  lane-steps %.2f G/s  CU-cycles per lane-step %.2f\n", name, ms, lane_steps / ms / 1e6,
           (ms * 1e-3 * 2.4e9 * cus) / lane_steps);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const size_t maxb = (size_t)1 << 30;
    uint4* buf;
    uint32_t* out;
    CK(hipMalloc(&buf, maxb));
    CK(hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(uint32_t)));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, (uint32_t*)buf, maxb / 4);
    CK(hipDeviceSynchronize());
    const size_t ws[3] = {(size_t)2 << 20, (size_t)96 << 20, maxb};
    const int steps = 256;
    for (size_t w : ws) {
        uint32_t mask = 1;
        while (mask * 2 <= w / 128) mask *= 2;
        mask -= 1;
        printf("working set %.0f MB\n", w / 1048576.0);
        for (int active : {64, 26}) {
            char nm[64];
            for (int waves : {4, 7}) {
                const int blocks = cus * waves;
                const double ls = (double)blocks * 4 * active * steps;
                snprintf(nm, sizeof nm, "per-lane  waves=%d active=%d", waves, active);
                if (waves == 4)
                    timeit(nm, [&] { hipLaunchKernelGGL(k_lane<4>, dim3(blocks), dim3(256), 0, 0, buf, mask, steps, active, out); }, ls, cus);
                else
                    timeit(nm, [&] { hipLaunchKernelGGL(k_lane<7>, dim3(blocks), dim3(256), 0, 0, buf, mask, steps, active, out); }, ls, cus);
            }
            const int blocks = cus * 4;
            const double ls = (double)blocks * 4 * active * steps;
            snprintf(nm, sizeof nm, "coop      waves=4 active=%d", active);
            timeit(nm, [&] { hipLaunchKernelGGL(k_coop<4>, dim3(blocks), dim3(256), 0, 0, buf, mask, steps, active, out); }, ls, cus);
        }
    }
    CK(hipDeviceSynchronize());
    return 0;
}
