// Dependent random-gather microbenchmark (one lane = one pointer chase, like a BVH
// traversal step): each step loads K 16-B pieces of one record (record = STRIDE x 16 B)
// and derives the next record from the data.  Prints lane-steps/s, wave-instructions/s
// per CU and lines/s per CU, to tell whether a divergent traversal is bound by vector
// memory instructions, by distinct cache lines, or by active lanes.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/microbench_gather tools/microbench_gather.hip
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

template <int K, int STRIDE>
__global__ __launch_bounds__(256) void k_chase(const uint4* __restrict__ buf, uint32_t mask, int steps, int active,
                                              uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    uint32_t idx = hash32(gid) & mask, acc = 0;
    if (lane < (uint32_t)active) {
        for (int s = 0; s < steps; s++) {
            const uint4* p = buf + (size_t)idx * STRIDE;
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < K; k++) {
                const uint4 v = p[k];
                x ^= v.x ^ v.y ^ v.z ^ v.w;
            }
            acc += x;
            idx = (x ^ (uint32_t)s) & mask;
        }
    }
    out[gid] = acc;
}

// G lanes share one 128-B record: lane reads its W-byte piece at offset (lane % G) * W;
// the group xor-reduces its pieces (shuffles) to pick the next record.
template <int G, int W>
__global__ __launch_bounds__(256) void k_group(const uint8_t* __restrict__ buf, uint32_t mask, int steps,
                                              uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    uint32_t idx = hash32(gid / G) & mask, acc = 0;
    for (int s = 0; s < steps; s++) {
        const uint8_t* p = buf + (size_t)idx * 128 + (lane % G) * W;
        uint32_t x;
        if (W == 16) { const uint4 v = *(const uint4*)p; x = v.x ^ v.y ^ v.z ^ v.w; }
        else if (W == 8) { const uint2 v = *(const uint2*)p; x = v.x ^ v.y; }
        else x = *(const uint32_t*)p;
#pragma unroll
        for (int o = 1; o < G; o *= 2) x ^= __shfl_xor(x, o);
        acc += x;
        idx = (x ^ (uint32_t)s) & mask;
    }
    out[gid] = acc;
}

// Throughput form of k_group: K independent 16-B loads per step, each from a different
// record, with G lanes sharing each record (64/G distinct lines per wave-instruction).
template <int G, int K>
__global__ __launch_bounds__(256) void k_group_tp(const uint8_t* __restrict__ buf, uint32_t mask, int steps,
                                                 uint32_t* out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t gid = blockIdx.x * 256u + threadIdx.x;
    uint32_t idx = hash32(gid / G) & mask, acc = 0;
    for (int s = 0; s < steps; s++) {
        uint32_t x = 0;
#pragma unroll
        for (int j = 0; j < K; j++) {
            const uint4 v = *(const uint4*)(buf + (size_t)((idx + j * 40503u) & mask) * 128 + (lane % G) * 16);
            x ^= v.x ^ v.y ^ v.z ^ v.w;
        }
#pragma unroll
        for (int o = 1; o < G; o *= 2) x ^= __shfl_xor(x, o);
        acc += x;
        idx = (x ^ (uint32_t)s) & mask;
    }
    out[gid] = acc;
}

template <int G, int K>
static void run_group_tp(const void* buf, size_t bytes, uint32_t* out, int cus) {
    uint32_t mask = 1;
    while (mask * 2 <= bytes / 128) mask *= 2;
    mask -= 1;
    const int blocks = cus * 7, steps = 128;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_group_tp<G, K>), dim3(blocks), dim3(256), 0, 0, (const uint8_t*)buf, mask, steps, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < 3; r++)
        hipLaunchKernelGGL((k_group_tp<G, K>), dim3(blocks), dim3(256), 0, 0, (const uint8_t*)buf, mask, steps, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 3;
    const double waves = (double)blocks * 4, wave_instr = waves * steps * K;
    const double cyc = 1.0 / (wave_instr / cus / (ms * 1e-3 * 2.4e9));
    printf("group_tp G=%d K=%d ws=%6.0fMB  %.3f ms  cycles/wave-instr/CU %.1f  lines/instr %d  cycles/line %.2f  "
           "records(128B)/CU/cycle %.3f\n", G, K, bytes / 1048576.0, ms, cyc, 64 / G, cyc / (64 / G),
           (64.0 / G) / cyc);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

template <int G, int W>
static void run_group(const void* buf, size_t bytes, uint32_t* out, int cus) {
    uint32_t mask = 1;
    while (mask * 2 <= bytes / 128) mask *= 2;
    mask -= 1;
    const int blocks = cus * 7, steps = 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_group<G, W>), dim3(blocks), dim3(256), 0, 0, (const uint8_t*)buf, mask, steps, out);
    CK(hipEventRecord(a));
    for (int r = 0; r < 3; r++)
        hipLaunchKernelGGL((k_group<G, W>), dim3(blocks), dim3(256), 0, 0, (const uint8_t*)buf, mask, steps, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= 3;
    const double waves = (double)blocks * 4, wave_instr = waves * steps;
    const double cyc = 1.0 / (wave_instr / cus / (ms * 1e-3 * 2.4e9));
    printf("group G=%d W=%2dB ws=%6.0fMB  %.3f ms  cycles/wave-instr/CU %.1f  distinct lines/instr %d  B/CU/cycle %.1f\n",
           G, W, bytes / 1048576.0, ms, cyc, 64 / G, 64.0 * W / cyc);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

template <int K, int STRIDE>
static void run(uint4* buf, size_t bytes, int waves_per_simd, int active, uint32_t* out, int cus) {
    const uint32_t records = (uint32_t)(bytes / (16 * STRIDE));
    uint32_t mask = 1;
    while (mask * 2 <= records) mask *= 2;
    mask -= 1;
    const int blocks = cus * waves_per_simd;   // 4 waves per block = one per SIMD
    const int steps = 256;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_chase<K, STRIDE>), dim3(blocks), dim3(256), 0, 0, buf, mask, steps, active, out);
    CK(hipEventRecord(a));
    const int reps = 3;
    for (int r = 0; r < reps; r++)
        hipLaunchKernelGGL((k_chase<K, STRIDE>), dim3(blocks), dim3(256), 0, 0, buf, mask, steps, active, out);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    ms /= reps;
    const double waves = (double)blocks * 4;
    const double lane_steps = waves * active * steps;
    const double wave_instr = waves * steps * K;
    const double lines = lane_steps * ((K * 16 + 127) / 128);
    printf("K=%d stride=%3dB ws=%6.0fMB waves/SIMD=%d active=%2d  %.3f ms  lane-steps %.2f G/s  "
           "wave-VMEM/CU/cycle(2.4GHz) %.4f  lines/CU/cycle %.3f  ns/step/wave %.0f\n",
           K, 16 * STRIDE, bytes / 1048576.0, waves_per_simd, active, ms, lane_steps / ms / 1e6,
           wave_instr / cus / (ms * 1e-3 * 2.4e9), lines / cus / (ms * 1e-3 * 2.4e9),
           ms * 1e6 / steps);
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
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
    printf("CUs %d\n", cus);
    if (argc > 1) {   // "chase": K of a 128-B record's eight 16-B pieces per dependent step, 6 waves per SIMD
        for (size_t w : {(size_t)96 << 20, maxb}) {
            run<1, 8>(buf, w, 6, 64, out, cus);
            run<2, 8>(buf, w, 6, 64, out, cus);
            run<4, 8>(buf, w, 6, 64, out, cus);
            run<6, 8>(buf, w, 6, 64, out, cus);
            run<7, 8>(buf, w, 6, 64, out, cus);
            run<8, 8>(buf, w, 6, 64, out, cus);
            run<4, 4>(buf, w, 6, 64, out, cus);
        }
        CK(hipDeviceSynchronize());
        return 0;
    }
    const size_t ws[3] = {(size_t)2 << 20, (size_t)96 << 20, maxb};
    for (size_t w : ws) {
        run_group_tp<1, 8>(buf, w, out, cus);
        run_group_tp<2, 8>(buf, w, out, cus);
        run_group_tp<4, 8>(buf, w, out, cus);
        run_group_tp<8, 8>(buf, w, out, cus);
        run_group_tp<8, 16>(buf, w, out, cus);
        run_group_tp<8, 4>(buf, w, out, cus);
    }
    for (size_t w : ws) {
        run_group<1, 4>(buf, w, out, cus);
        run_group<1, 8>(buf, w, out, cus);
        run_group<1, 16>(buf, w, out, cus);
        run_group<2, 16>(buf, w, out, cus);
        run_group<4, 16>(buf, w, out, cus);
        run_group<8, 16>(buf, w, out, cus);
        run_group<8, 8>(buf, w, out, cus);
        run_group<16, 8>(buf, w, out, cus);
        run_group<32, 4>(buf, w, out, cus);
        run_group<4, 4>(buf, w, out, cus);
        run<1, 8>(buf, w, 7, 64, out, cus);
        run<2, 8>(buf, w, 7, 64, out, cus);
        run<4, 8>(buf, w, 7, 64, out, cus);
        run<7, 8>(buf, w, 7, 64, out, cus);
        run<8, 8>(buf, w, 7, 64, out, cus);
        run<4, 4>(buf, w, 7, 64, out, cus);
        run<7, 8>(buf, w, 7, 16, out, cus);
        run<7, 8>(buf, w, 7, 32, out, cus);
        run<7, 8>(buf, w, 4, 64, out, cus);
        run<7, 8>(buf, w, 8, 64, out, cus);
        run<6, 8>(buf, w, 7, 64, out, cus);
        run<8, 16>(buf, w, 7, 64, out, cus);
    }
    CK(hipDeviceSynchronize());
    return 0;
}
