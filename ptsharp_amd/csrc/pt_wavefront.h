// pt_wavefront.h — HBM queues of the wavefront engine (pt_wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_scene.h"

namespace pt {

// Ray queues are double-buffered by depth parity; every array is float4 /
// uint64 SoA so each lane moves 16 B per access.
struct WfQueues {
    float4* q_o[2];      // {origin.xyz, pixel}
    float4* q_d[2];      // {direction.xyz, depth | emission << 8}
    float4* q_t[2];      // {throughput.rgb, -}
    uint64_t* q_k[2];    // RNG node key of the vertex the ray leads to
    uint4* hits;         // {t (fp64 bits), kind, record}
    float4* s_o;         // shadow rays: {origin.xyz, pixel}
    float4* s_d;         // {direction.xyz, light index}
    float4* s_c;         // {contribution if visible, -}
    uint32_t* counts;    // [0],[1] ray queues, [2] shadow queue, [3] overflow flag
    uint32_t cap;        // entries per ray queue
    uint32_t s_cap;      // shadow queue entries
    double* acc;         // [P][3] per-pixel sum of this pass' sample colours
};

struct WfPlan {
    uint64_t chunk;            // camera samples per chunk
    uint32_t root_children;    // ⌊√FH⌋² · modes at depth 0
    uint32_t children;         // modes at depth >= 1 (1, or 2 under SpecularModeAll)
    uint32_t lights_per_child; // 1, or #lights under LightModeAll
    uint32_t trace_blocks;     // grid caps (grid-stride loops)
    uint32_t shade_blocks;
};

// Optional per-launch timing hook (hipEvent pairs recorded around each kernel; pt_api.hip).
struct LaunchTimer {
    virtual void begin(int kernel_class) = 0;
    virtual void end(int kernel_class) = 0;
    virtual ~LaunchTimer() = default;
};

hipError_t wavefront_pass(const DevScene& S, const DevCamera& cam, const DevSampler& smp, const DevPass& P,
                          const DevBuffer& B, const WfQueues& Q, const WfPlan& plan, bool count, hipStream_t stream,
                          LaunchTimer* timer);

}  // namespace pt
