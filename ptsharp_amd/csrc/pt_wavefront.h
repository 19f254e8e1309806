// pt_wavefront.h — HBM queues of the wavefront engine (pt_wavefront.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pt_accum.h"
#include "pt_scene.h"

namespace pt {

// Ray queues are double-buffered by depth parity; every array is float4 /
// uint64 SoA so each lane moves 16 B per access.  Every queue is split into
// kParts partitions, one per XCD group (blocks b, b + 8, ... share an XCD and
// its L2): group g consumes partition g and appends the children and NEE
// requests it makes to partition g of the next queues, so each XCD's L2 keeps
// working on one region of the image at every depth, and the reservation
// atomics spread over kParts counter words.
constexpr int kParts = 8;
constexpr uint32_t kNoRecord = 0xFFFFFFFFu;
struct WfQueues {
    float4* q_o[2];      // {origin.xyz, pixel}
    float4* q_d[2];      // {direction.xyz, depth | emission << 8}
    double2* q_t[2];     // {throughput.r, throughput.g} (fp64, as the reference's Colour)
    ulonglong2* q_k[2];  // {RNG node key of the vertex the ray leads to, throughput.b (fp64 bits)}
    uint4* hits;         // {t (fp64 bits), kind, record}
    uint4* sdfq;         // split closest hit: {slot, SDF record, best world t (fp64 bits)} (k_wf_sdf_hits)
    uint4* sdfq_sh;      // split shadow rays: {slot, SDF record, the light's t (fp64 bits)} (k_wf_sdf_shadow)
    // Volume records deferred the same way (one per sdfq / sdfq_sh entry, kNoRecord: none; the entry's
    // SDF record may be kNoRecord too): k_wf_vol_hits / k_wf_vol_shadow march them before the SDF
    // kernels run, lowering the entry's t when the Volume is nearer.  Null: no Volume in the scene.
    uint32_t* volq;
    uint32_t* volq_sh;
    // Routed split (DevScene::route): the slots of the rays whose segment reaches a §8f row-4 shape's box,
    // per partition (pcap / spcap entries each): only these go through the FULL analytic half
    uint32_t* hq;        // closest-hit rays (k_wf_trace_lanes → k_wf_trace<.., SPLIT>)
    uint32_t* hq_sh;     // shadow rays (k_wf_shadow_lanes → k_wf_shadow<.., SPLIT>; one shadow pass at a time)
    // Shadow rays (a diffuse child's sampleLights, set up by k_wf_shade), two sets by depth
    // parity (set q holds the shadow rays counted in pair word q), so the shadow pass and the
    // light-term accumulation of depth d can run beside the closest-hit and shade passes of d + 1.
    float4* n_o[2];      // {origin.xyz, pixel}
    float4* n_n[2];      // {direction.xyz, light index | kDead: no ray cast (diffuse <= 0)}
    double2* n_w[2];     // two per entry, {r, g} {b, pixel (bits)}: throughput·weight·light colour·coverage (fp64),
                         // added if the light is visible
    uint8_t* n_lit[2];   // per entry: 1 = the light is the nearest hit (k_wf_shadow*), read by k_wf_nee_accum
    uint32_t* counts;    // counter slots, each kCountStride words apart (see count_word below):
                         // slot q·kParts+g = {rays, NEE requests} of partition g of ray queue q
                         // (one packed 64-bit word, reserved together); slot kFetchSlot + k·kParts + g
                         // = work-fetch cursor of kernel k (0 trace, 1 shade, 2 + q shadow set q) in
                         // partition g; slots kKeptSlot + q = rays of queue q with shading work (k_wf_trace)
    unsigned long long* overflow;   // set to 1 when a queue overflowed: a word of the pass' counters
                                    // (DevBuffer::counters[kOverflowCounter]), read back with them
    uint32_t cap;        // entries per ray queue (kParts partitions of pcap)
    uint32_t s_cap;      // NEE queue entries (kParts partitions of spcap)
    uint32_t pcap, spcap;
    FixAcc acc;          // [P] per-pixel sum of this pass' sample colours (pt_accum.h: order-independent)
    uint32_t* ovf;       // closest-hit traversal stack entries beyond kLdsStack: [kStackMax - kLdsStack][kWfMaxThreads]
    uint32_t* ovf_sh;    // the same for the shadow kernels, which may run beside a closest-hit kernel (side stream)
    FixAcc acc_s;        // [chunk] per-sample accumulators of the adaptive / firefly phases
    // k_wf_shadow_lanes' tail (helper hand-off): 0 as in a render, from the queue's drain on; 1 (PT_SHADOW_TAIL=early,
    // tests) a wave refills only when all its lanes are idle and its idle lanes help from the first claim on, so
    // the hand-off protocol runs throughout the pass instead of in each wave's last rays
    int32_t tail_early;
};

// Every counter sits on a line of its own: returning atomics execute at the memory side,
// one line at a time, so cursors packed into one 128-B line serialise every partition's
// claims on one channel.  kCountStride words (4 B each) between slots.
constexpr int kCountStride = 64;
static_assert(kCountStride >= 2, "a slot holds a packed 64-bit pair");
constexpr int kFetchSlot = 2 * kParts;   // 8 cursors (k = 0..7) per partition
constexpr int kKeptSlot = 10 * kParts;   // two slots (depth parity): rays k_wf_trace left work for k_wf_shade
constexpr int kSdfSlot = 10 * kParts + 2;   // entries of Q.sdfq
constexpr int kSdfShSlot = 10 * kParts + 3;   // two slots (shadow set q): entries of Q.sdfq_sh
constexpr int kHeavySlot = 10 * kParts + 5;     // kParts slots: entries of Q.hq per partition
constexpr int kHeavyShSlot = 11 * kParts + 5;  // 2 x kParts slots (shadow set q): entries of Q.hq_sh per partition
constexpr int kEndSlot = 13 * kParts + 5;
constexpr int count_word(int slot) { return slot * kCountStride; }
constexpr int kFetchWord = count_word(kFetchSlot);
constexpr int kCountWords = count_word(kEndSlot);
constexpr int kChunkResetWords = kCountWords;   // every slot is zeroed per chunk
constexpr int kOverflowCounter = 15;            // DevBuffer::counters word of WfQueues::overflow

// work-fetch cursor of kernel k (0 trace, 1 shade, 2 + q shadow rays of set q, 4 the analytic phase
// of a split closest hit, 5 + q that of split shadow rays of set q; pt_wavefront.hip "split"; 7 the FULL
// shade of a routed shade, DevScene::shade_route) in partition g
constexpr int fetch_word(int k, int g) { return count_word(kFetchSlot + k * kParts + g); }
constexpr int kept_word(int q) { return count_word(kKeptSlot + q); }
constexpr int kSdfWord = count_word(kSdfSlot);
// Every counter a depth's kernels append to is zeroed by a kernel ahead of them on the same stream
// (k_wf_shade's block 0: the next closest hit's heavy queue, the shadow set it writes), never by a
// hipMemsetAsync: a fill kernel queued behind the other stream's persistent grid waits for a free CU
// and holds its stream (C5: 500 such fills per pass, 0.47 ms each).
constexpr int sdf_sh_word(int q) { return count_word(kSdfShSlot + q); }
constexpr int heavy_word(int g) { return count_word(kHeavySlot + g); }
constexpr int heavy_sh_word(int q, int g) { return count_word(kHeavyShSlot + q * kParts + g); }

#ifndef PT_LDS_STACK
#define PT_LDS_STACK 16
#endif
constexpr int kLdsStack = PT_LDS_STACK;          // LDS stack entries per lane (traversal kernels)
constexpr uint32_t kWfMaxBlocks = 256 * 8;        // grid cap of the traversal kernels

// k_wf_camera deals a chunk's camera samples to the partitions in runs of deal_run 256-sample
// blocks, the runs round-robin (pt_wavefront.hip): one block (16 pixels' samples) per run.  Runs of
// one 32x32 tile's samples, so that each XCD traces compact patches of the scene, measured slower
// (C4 5899 → 5831 Mrays/s; profiles/r03e_ab_deal.txt).
__host__ __device__ inline uint32_t deal_run(int32_t) { return 1u; }
// Camera samples the fullest partition receives from a chunk of `samples`.
__host__ __device__ inline uint64_t deal_group_max(uint64_t samples, int32_t spp_launch) {
    const uint64_t run = deal_run(spp_launch), nblk = (samples + 255) / 256, nruns = (nblk + run - 1) / run;
    return (nruns + kParts - 1) / kParts * run * 256;
}
constexpr uint32_t kWfMaxThreads = kWfMaxBlocks * 256;

struct WfPlan {
    uint64_t chunk;            // camera samples per chunk
    uint64_t chunk_extra;      // camera samples per chunk of the adaptive / firefly phases (>= chunk: their
                               // queues and per-sample accumulators are sized for it)
    uint32_t root_children;    // ⌊√FH⌋² · modes at depth 0
    uint32_t children;         // modes at depth >= 1 (1, or 2 under SpecularModeAll)
    uint32_t lights_per_child; // shadow-ray slots per diffuse child: 1, or #lights under LightModeAll
    uint32_t trace_blocks;     // persistent grids: resident capacity of each kernel (lockstep traversal,
    uint32_t shade_blocks;     // shade, lockstep shadow; the refill and FULL traversal kernels below)
    uint32_t shadow_blocks;
    uint32_t lanes_trace_blocks, lanes_shadow_blocks, full_trace_blocks, full_shadow_blocks;
    uint32_t linear_trace_blocks, linear_shadow_blocks;   // k_wf_trace_linear / k_wf_shadow_linear (resident)
    int32_t shade_form;        // k_wf_shade form: 0 chosen per depth from the kept count, 1 direct, 2 SCAN
                               // (PT_SHADE_FORM=direct|scan in the environment; tests)
    int32_t lanes;             // refill traversal kernels: -1 by BVH size, 0 never, 1 always
                               // (PT_LANES=0|1 in the environment; tests)
    int32_t linear;            // linear kernels (few analytic records, no triangles): -1 where they apply, 0 never
                               // (PT_LINEAR=0 in the environment; tests)
    // Optional second stream: each depth's shadow pass runs there, beside the next depth's
    // closest-hit pass (independent queues), so one fills the other's ramp and tail.
    // ev_main orders shade(d) → shadow(d); ev_side[q], recorded after the light terms of
    // shadow set q were added, orders them before shade(d + 2) rewrites set q.  Null: one stream.
    hipStream_t side;
    hipEvent_t ev_main, ev_side[2];
};

// Optional per-launch timing hook (hipEvent pairs recorded around each kernel on the
// stream it runs on; pt_api.hip).
struct LaunchTimer {
    virtual void begin(int kernel_class, hipStream_t s) = 0;
    virtual void end(int kernel_class, hipStream_t s) = 0;
    virtual ~LaunchTimer() = default;
};

hipError_t wavefront_pass(const DevScene& S, const DevCamera& cam, const DevSampler& smp, const DevPass& P,
                          const DevBuffer& B, const WfQueues& Q, const WfPlan& plan, bool count, hipStream_t stream,
                          LaunchTimer* timer);

// Extra-sample phase of a pass: `entries` pixels (tile order, or `plist`), K samples each,
// sample indices sample_base + 0..K-1.  `firefly`: 0 every sample AddSample'd, camera jitter
// NextDouble() (RenderParallel's adaptive loop; Render's adaptive loop); 1 RenderParallel's
// firefly loop: stop at the first IsFirefly sample (`snap`: M at the start of the phase),
// pixels that took all K samples without a stop are appended to next_list (count in
// *next_count, a device word); 2 Render's firefly loop: every sample AddSample'd, jitter
// (x + NextDouble()) · (1.0f / w) (Renderer.cs:184-185).
enum ExtraMode : int { EXTRA_ADD = 0, EXTRA_FIREFLY_STOP = 1, EXTRA_ADD_SCALED = 2 };
hipError_t wavefront_extra(const DevScene& S, const DevCamera& cam, const DevSampler& smp, const DevPass& P,
                           const DevBuffer& B, const WfQueues& Q, const WfPlan& plan, bool count, hipStream_t stream,
                           LaunchTimer* timer, int firefly, int32_t K, uint32_t sample_base, uint64_t entries,
                           const uint32_t* plist, const double* snap, uint32_t* next_list, uint32_t* next_count);

// Persistent grid sizes (resident capacity on this device) of the traversal / shade kernels.
hipError_t wavefront_grids(WfPlan& plan);

// Pixels of the pass whose StandardDeviation().MaxComponent() exceeds 1 (kind 0: the firefly
// candidates, Renderer.cs:179,426) or is at least 1 (kind 1: Render's adaptive branch, where
// AdaptiveSamples · (int)clamp(v / 1, 0, 1)^1 is nonzero, Renderer.cs:155-158) into plist;
// *count = how many (device word).
hipError_t select_pixels(const DevPass& P, const DevBuffer& B, int kind, uint32_t* plist, uint32_t* count,
                         hipStream_t stream);

}  // namespace pt
