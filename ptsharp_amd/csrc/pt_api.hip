// pt_api.hip — C-ABI implementation of libptsharp_hip.so (include/ptsharp_hip.h).
//
// Host runtime around the gfx950 render kernels: scene flattening and BVH
// build (replacing Scene.Compile / Tree.NewTree, Scene.cs:48-68), HBM-resident
// Welford buffer (Renderer.PBuffer, Renderer.cs:20), pass launch and timing
// (RenderParallel + its stopwatch, Renderer.cs:199-213,470), ray statistics
// (Scene.rays, Scene.cs:70-79), and the multi-GPU Buffer gather over RCCL.
// No exception crosses the ABI: every entry point returns a pt_status and
// leaves a thread-local message for pt_last_error (the OIDN convention,
// OIDN.cs:85-86).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/ptsharp_hip.h"
#include "pt_bvh.h"
#include "pt_device.h"
#include "pt_math.h"
#include "pt_scene.h"
#include "pt_wavefront.h"

#pragma clang fp contract(off)

namespace pt {
// After a gather the root's Buffer holds every rank's tiles; before its next pass adds to
// its own tiles (and before a firefly snapshot is all-reduced) the other ranks' pixels are
// cleared again, so every context's Buffer holds exactly its own tiles between gathers.
__global__ __launch_bounds__(256) void k_clear_foreign(DevBuffer B, int32_t width, int32_t height, int32_t tiles_x,
                                                       const uint8_t* own) {
    const size_t P = (size_t)width * (size_t)height;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (size_t)gridDim.x * blockDim.x) {
        const int x = (int)(i % (size_t)width), y = (int)(i / (size_t)width);
        if (own[(y >> 5) * tiles_x + (x >> 5)]) continue;
        B.n[i] = 0;
        for (int k = 0; k < 3; k++) { B.m[3 * i + k] = 0.0; B.v[3 * i + k] = 0.0; }
    }
}
// Packed tiles (pt_read_tiles / pt_write_tiles, the tile-compacted gather): entry s of a run
// is pixel (s & 31, (s >> 5) & 31) of tile ids[s >> 10], row-major inside the tile; pack
// copies {M, V, N} out (zeros outside the image), unpack writes a run into the Buffer.
__global__ __launch_bounds__(256) void k_tiles_pack(DevBuffer B, int32_t width, int32_t height, int32_t tiles_x,
                                                    const int32_t* ids, uint32_t nt, double* pm, double* pv,
                                                    int32_t* pn, int unpack) {
    const size_t total = (size_t)nt * 1024u;
    for (size_t s = (size_t)blockIdx.x * blockDim.x + threadIdx.x; s < total; s += (size_t)gridDim.x * blockDim.x) {
        const int tile = ids[s >> 10];
        const int x = (tile % tiles_x) * 32 + (int)(s & 31u), y = (tile / tiles_x) * 32 + (int)((s >> 5) & 31u);
        const bool in = x < width && y < height;
        const size_t i = (size_t)y * (size_t)width + (size_t)x;
        if (unpack) {
            if (!in) continue;
            B.n[i] = pn[s];
            for (int k = 0; k < 3; k++) { B.m[3 * i + k] = pm[3 * s + k]; B.v[3 * i + k] = pv[3 * s + k]; }
        } else {
            pn[s] = in ? B.n[i] : 0;
            for (int k = 0; k < 3; k++) { pm[3 * s + k] = in ? B.m[3 * i + k] : 0.0; pv[3 * s + k] = in ? B.v[3 * i + k] : 0.0; }
        }
    }
}
__global__ void k_iota(int32_t* a, int32_t n) {
    for (int32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a[i] = i;
}
hipError_t launch_render_pass(const DevScene& S, const DevCamera& cam, const DevSampler& smp, const DevPass& P,
                              const DevBuffer& B, int num_tiles, bool count, hipStream_t stream);
hipError_t launch_intersect(const DevScene& S, uint32_t n, const float* o3, const float* d3, const double* tl,
                            double* out_t, int32_t* out_kind, hipStream_t stream);
}

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}

#define PT_HIP(call)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess)                                                                         \
            return fail(PT_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));               \
    } while (0)

struct DeviceArray {
    void* ptr = nullptr;
    size_t bytes = 0;
    void release() { if (ptr) (void)hipFree(ptr); ptr = nullptr; bytes = 0; }
};

// hipEvent pairs around each launch of a pass (PT_PASS_KERNEL_TIMING): device
// time per kernel class, read after the pass' final synchronisation.
struct EventTimer : pt::LaunchTimer {
    std::vector<hipEvent_t> pool;
    std::vector<int> cls;
    size_t used = 0;
    hipStream_t stream = nullptr;
    bool failed = false;
    void reset(hipStream_t s) { stream = s; used = 0; cls.clear(); failed = false; }
    void record(int c, bool is_begin, hipStream_t s) {
        if (used == pool.size()) {
            hipEvent_t e;
            if (hipEventCreate(&e) != hipSuccess) { failed = true; return; }
            pool.push_back(e);
        }
        if (hipEventRecord(pool[used], s ? s : stream) != hipSuccess) failed = true;
        if (is_begin) cls.push_back(c);
        used++;
    }
    void begin(int c, hipStream_t s) override { record(c, true, s); }
    void end(int c, hipStream_t s) override { record(c, false, s); }
    hipError_t collect(double* ms, uint32_t* launches) {
        for (size_t i = 0; i + 1 < used; i += 2) {
            float t = 0.f;
            hipError_t e = hipEventElapsedTime(&t, pool[i], pool[i + 1]);
            if (e != hipSuccess) return e;
            ms[cls[i / 2]] += t;
            launches[cls[i / 2]]++;
        }
        return hipSuccess;
    }
    void destroy() { for (auto e : pool) (void)hipEventDestroy(e); pool.clear(); }
};

struct TriBvhBuild;
struct Ctx {
    int device = 0;
    int width = 0, height = 0;
    hipStream_t stream = nullptr;
    hipStream_t side = nullptr;                          // shadow passes (pt::WfPlan::side)
    hipEvent_t ev_main = nullptr, ev_side[2] = {nullptr, nullptr};
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    // Welford buffer
    double* d_m = nullptr;
    double* d_v = nullptr;
    int32_t* d_n = nullptr;
    unsigned long long* d_counters = nullptr;   // [pt::kCounterAllocWords] the pass' counters (pt::DevBuffer::counters)
    unsigned long long* h_counters = nullptr;   // [pt::kCounterAllocWords] pinned: their read-back
    int32_t* d_tiles = nullptr;
    int32_t tiles_cap = 0;
    std::vector<int32_t> h_tiles;               // the tile list in d_tiles (uploaded when it changes)
    // scene
    bool has_scene = false;
    std::vector<DeviceArray> scene_arrays;
    pt::DevScene S{};
    // stats
    pt_stats stats{};
    // RCCL
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    bool gathered = false;          // other ranks' tiles are in the Buffer (a gather, pt_write_tiles) until the next pass
    bool loaded = false;            // pt_write_buffer put a whole checkpoint in (foreign pixels once the context has a communicator)
    uint8_t* d_own = nullptr;       // [tiles] 1 = a tile of this context's last tile list
    int32_t pass_tiles = 0;         // tiles of the last pass (0: the whole image); their ids are in d_tiles
    // tile-compacted gather workspace (allocated by the first gather): ids, M, V, N of up to
    // every tile of the image, the rank counts, and the ids 0..tiles-1 of a whole-image rank
    int32_t* g_ids = nullptr;
    double* g_m = nullptr;
    double* g_v = nullptr;
    int32_t* g_n = nullptr;
    int32_t* g_cnts = nullptr;      // [nranks + 1]: all ranks' tile counts, then this rank's
    int32_t* g_all = nullptr;
    // wavefront queues (allocated on first use, grown on demand)
    pt::WfQueues Q{};
    std::vector<DeviceArray> wf_arrays;
    uint32_t wf_cap = 0, wf_scap = 0;
    bool wf_two_sets = false;      // a second shadow-ray set allocated (the side stream's shadow passes need it)
    int32_t acc_passes = 0;        // passes of per-pixel accumulators allocated (a batch needs one set per pass)
    uint32_t wf_max_cap = 0;       // queue capacity bound (wf_max_cap()), once per context
    // adaptive / firefly phases (allocated on first use, with the queues)
    uint32_t* d_plist = nullptr;   // [P] firefly candidates (ping-pong with d_plist2 over the rounds)
    uint32_t* d_plist2 = nullptr;
    uint32_t* d_fcount = nullptr;  // [2] list lengths
    double* d_snap = nullptr;      // [P][3] M at the start of the firefly phase
    pt::FixAcc acc_s{};            // [acc_s_cap] per-sample accumulators (own allocation; Q.acc_s points at it)
    uint64_t acc_s_cap = 0;
    int last_engine = 0;
    pt::WfPlan grids{};            // persistent grid sizes (pt::wavefront_grids), once per context
    EventTimer timer;
    double tri_build_ms = 0;       // last upload: host time to build (or wait for, or find) the triangle BVH
    std::shared_ptr<const TriBvhBuild> tri_build;   // that build, shared with the other contexts of its geometry
                                                    // (released at the next upload and at pt_destroy)
};

// Queue capacity bound (entries per queue).  A pass is rendered in chunks of camera
// samples whose widest depth fits the queues; every chunk pays the fill and drain of
// 16 persistent launches, so fewer, larger chunks are faster (C4, 16 spp per pass: 8
// chunks of 32M-entry queues 2574 Mrays/s, 2 chunks 2809, one chunk 2853).  The bound is
// the largest power of two whose queues (209 B per entry: two extension queues of o, d, throughput r g,
// key + throughput b, the hits, one shadow set) fit half of the device's memory and half of its free memory,
// clamped to [2^20, 2^29] entries (2^29: 112 GB of the MI355X's 288 GB: C2's 33M camera samples × 16 children
// in one chunk).  A chunk small enough for the side stream (kSideStreamMaxRays) keeps a second shadow set
// (ensure_wavefront), within the same budget.
constexpr uint32_t kWfMinCapLimit = 1u << 20, kWfMaxCapLimit = 1u << 29;
#ifndef PT_SDF_LDS_MAX
#define PT_SDF_LDS_MAX 16384   // LDS bytes k_wf_sdf_* may stage the SDF programs in; 0: never
#endif
#ifndef PT_VOL_LDS_MAX
#define PT_VOL_LDS_MAX 40960   // LDS bytes k_wf_vol_* may stage the scene's one Volume in (its uniform-cell table); 0: never
#endif
#ifndef PT_VOL_CELLS_MAX
#define PT_VOL_CELLS_MAX (1ull << 30)   // bytes of cell-major Volume corners (8 per cell) a scene may hold; 0: none
#endif
#ifndef PT_EXTRA_CHUNK_MAX
#define PT_EXTRA_CHUNK_MAX (64ull << 20)   // camera samples per chunk of the adaptive / firefly phases, at most (round 6: 32M → 64M with the 2^29-entry queues, C5 +1.8 %, profiles/r06ec_ab_extra_chunk.txt)
#endif
#ifndef PT_VOL_DEFER
#define PT_VOL_DEFER 1   // split traversal: Volumes deferred to k_wf_vol_hits / k_wf_vol_shadow (0: marched in place)
#endif
constexpr double kSideStreamMaxRays = (double)(64ull << 20);   // a chunk's widest depth, extension rays
// Outside this budget, for row-4 scenes only (counted in, they halved C4-sized queues from 2^28 to 2^27
// entries and split the pass in two chunks, -3 %): the two deferred-record queues of a scene with SDF
// shapes or Volumes (sdfq, sdfq_sh: 32 B per entry), with Volumes their record words (volq, volq_sh: 8 B),
// and under the routed split the heavy queues (hq, hq_sh: 8 B).  At most 48 B per entry, 17 % over the
// 274 B: 12.9 GB at 2^28 entries, inside the three quarters of the device the budget leaves free.
constexpr size_t kWfBytesPerEntry = 2 * (16 + 16 + 16 + 16) + 16 + (64 + 1);

// PT_WF_MAX_CAP (entries, environment) lowers the bound: tests use it to force many chunks.
uint32_t wf_max_cap(Ctx* c) {
    if (c->wf_max_cap) return c->wf_max_cap;
    if (const char* env = std::getenv("PT_WF_MAX_CAP")) {
        const unsigned long long v = std::strtoull(env, nullptr, 10);
        uint32_t cap = kWfMaxCapLimit;
        while (cap > (uint32_t)pt::kParts * 1024u && cap > v) cap >>= 1;
        return c->wf_max_cap = cap;
    }
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = total_b = (size_t)kWfMinCapLimit * kWfBytesPerEntry * 4;
    const size_t budget = std::min(total_b / 2, free_b / 2);   // and at most half of what is free now
    uint32_t cap = kWfMaxCapLimit;
    while (cap > kWfMinCapLimit && (size_t)cap * kWfBytesPerEntry > budget) cap >>= 1;
    c->wf_max_cap = cap;
    return cap;
}

void free_wavefront(Ctx* c) {
    for (auto& a : c->wf_arrays) a.release();
    c->wf_arrays.clear();
    c->Q = pt::WfQueues{};
    c->wf_cap = c->wf_scap = 0;
    c->wf_two_sets = false;
    c->acc_passes = 0;
    c->d_plist = nullptr;
    c->d_plist2 = nullptr;
    c->d_fcount = nullptr;
    c->d_snap = nullptr;
    if (c->acc_s.w) { (void)hipFree(c->acc_s.w); (void)hipFree(c->acc_s.hi); (void)hipFree(c->acc_s.big); }
    c->acc_s = pt::FixAcc{};
    c->acc_s_cap = 0;
}

template <class T>
int wf_alloc(Ctx* c, T** out, size_t n) {
    DeviceArray a;
    a.bytes = n * sizeof(T);
    hipError_t e = hipMalloc(&a.ptr, a.bytes);
    if (e != hipSuccess) return fail(PT_ERR_OUT_OF_MEMORY, std::string("hipMalloc wavefront queues: ") + hipGetErrorString(e));
    c->wf_arrays.push_back(a);
    *out = (T*)a.ptr;
    return PT_OK;
}

// two_sets: the shadow passes run on the side stream beside the next depth (pt::WfPlan::side), so the shadow rays
// of depth d and d + 1 live at once, in sets by depth parity; on one stream a depth's shadow rays are consumed
// before the next depth's shade writes its own, and both sets are the same memory.
int ensure_wavefront(Ctx* c, uint32_t cap, uint32_t scap, int32_t acc_passes, bool two_sets) {
    // the split traversal's deferred-record queues (pt_wavefront.hip k_wf_vol_* / k_wf_sdf_*)
    const bool want_sdf = c->S.num_sdf > 0 || (PT_VOL_DEFER && c->S.num_vol > 0);
    const bool want_vol = PT_VOL_DEFER && c->S.num_vol > 0;
    const bool want_heavy = c->S.route != 0;  // the routed split's queues of rays that reach a row-4 shape's box
    if (c->wf_cap >= cap && c->wf_scap >= scap && c->Q.acc.w && c->acc_passes >= acc_passes && (!two_sets || c->wf_two_sets) &&
        (!want_sdf || c->Q.sdfq) && (!want_vol || c->Q.volq) &&
        (!want_heavy || c->Q.hq))
        return PT_OK;
    cap = std::max(cap, c->wf_cap);
    scap = std::max(scap, c->wf_scap);
    acc_passes = std::max(acc_passes, c->acc_passes);
    two_sets = two_sets || c->wf_two_sets;
    free_wavefront(c);
    pt::WfQueues Q{};
    int rc;
    for (int q = 0; q < 2; q++) {
        if ((rc = wf_alloc(c, &Q.q_o[q], cap))) return rc;
        if ((rc = wf_alloc(c, &Q.q_d[q], cap))) return rc;
        if ((rc = wf_alloc(c, &Q.q_t[q], cap))) return rc;
        if ((rc = wf_alloc(c, &Q.q_k[q], cap))) return rc;
    }
    if ((rc = wf_alloc(c, &Q.hits, cap))) return rc;
    if (want_sdf && (rc = wf_alloc(c, &Q.sdfq, cap))) return rc;
    if (want_vol && (rc = wf_alloc(c, &Q.volq, cap))) return rc;
    for (int q = 0; q < (two_sets ? 2 : 1); q++) {   // shadow-ray sets by depth parity
        if ((rc = wf_alloc(c, &Q.n_o[q], scap))) return rc;
        if ((rc = wf_alloc(c, &Q.n_n[q], scap))) return rc;
        if ((rc = wf_alloc(c, &Q.n_w[q], 2 * (size_t)scap))) return rc;
        if ((rc = wf_alloc(c, &Q.n_lit[q], scap))) return rc;
    }
    if (!two_sets) {   // one stream: set 1 is set 0's memory
        Q.n_o[1] = Q.n_o[0];
        Q.n_n[1] = Q.n_n[0];
        Q.n_w[1] = Q.n_w[0];
        Q.n_lit[1] = Q.n_lit[0];
    }
    if (want_sdf && (rc = wf_alloc(c, &Q.sdfq_sh, scap))) return rc;   // one shadow pass at a time uses it
    if (want_vol && (rc = wf_alloc(c, &Q.volq_sh, scap))) return rc;
    if (want_heavy && (rc = wf_alloc(c, &Q.hq, cap))) return rc;
    if (want_heavy && (rc = wf_alloc(c, &Q.hq_sh, scap))) return rc;   // one shadow pass at a time uses it
    if ((rc = wf_alloc(c, &Q.counts, pt::kCountWords))) return rc;
    Q.overflow = c->d_counters + pt::kOverflowCounter;
    // spill columns: one region for the closest-hit kernels, one for the shadow kernels (they
    // can run at the same time on the side stream)
    const size_t ovf_words = (size_t)(pt::kStackMax - pt::kLdsStack) * pt::kWfMaxThreads;
    if ((rc = wf_alloc(c, &Q.ovf, 2 * ovf_words))) return rc;
    Q.ovf_sh = Q.ovf + ovf_words;
    // per-pixel accumulators of one pass, or of each pass of a batch (pt_pass_params.passes)
    size_t P = (size_t)c->width * (size_t)c->height * (size_t)acc_passes;
    if ((rc = wf_alloc(c, &Q.acc.w, P * pt::kFixWords))) return rc;
    if ((rc = wf_alloc(c, &Q.acc.hi, P * pt::kFixWords))) return rc;
    if ((rc = wf_alloc(c, &Q.acc.big, P * 3))) return rc;
    Q.acc.n = P;   // channel-planar (pt_accum.h FixAcc)
    PT_HIP(hipMemsetAsync(Q.acc.w, 0, P * pt::kFixWords * sizeof(unsigned long long), c->stream));
    PT_HIP(hipMemsetAsync(Q.acc.hi, 0, P * pt::kFixWords * sizeof(unsigned long long), c->stream));
    PT_HIP(hipMemsetAsync(Q.acc.big, 0, P * 3 * sizeof(double), c->stream));
    PT_HIP(hipMemsetAsync(Q.counts, 0, pt::kCountWords * sizeof(uint32_t), c->stream));
    Q.cap = cap;
    Q.s_cap = scap;
    Q.pcap = cap / pt::kParts;
    Q.spcap = scap / pt::kParts;
    c->Q = Q;
    c->wf_cap = cap;
    c->wf_scap = scap;
    c->wf_two_sets = two_sets;
    c->acc_passes = acc_passes;
    return PT_OK;
}

// Buffers of the adaptive / firefly phases: per-sample accumulators for one chunk
// of camera samples, the candidate list and the M snapshot.
int ensure_extra(Ctx* c, uint64_t chunk) {
    if (c->acc_s.w && c->acc_s_cap >= chunk) { c->Q.acc_s = c->acc_s; return PT_OK; }
    int rc;
    const size_t P = (size_t)c->width * (size_t)c->height;
    if (!c->d_plist) {
        if ((rc = wf_alloc(c, &c->d_plist, P))) return rc;
        if ((rc = wf_alloc(c, &c->d_plist2, P))) return rc;
        if ((rc = wf_alloc(c, &c->d_fcount, 2))) return rc;
        if ((rc = wf_alloc(c, &c->d_snap, P * 3))) return rc;
    }
    if (c->acc_s.w) {
        (void)hipFree(c->acc_s.w); (void)hipFree(c->acc_s.hi); (void)hipFree(c->acc_s.big);
        c->acc_s = pt::FixAcc{}; c->acc_s_cap = 0;
    }
    c->Q.acc_s = pt::FixAcc{};
    if (hipMalloc(&c->acc_s.w, chunk * pt::kFixWords * sizeof(unsigned long long)) != hipSuccess)
        return fail(PT_ERR_OUT_OF_MEMORY, "hipMalloc per-sample accumulators");
    if (hipMalloc(&c->acc_s.hi, chunk * pt::kFixWords * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&c->acc_s.big, chunk * 3 * sizeof(double)) != hipSuccess) {
        (void)hipFree(c->acc_s.w);
        if (c->acc_s.hi) (void)hipFree(c->acc_s.hi);
        c->acc_s = pt::FixAcc{};
        return fail(PT_ERR_OUT_OF_MEMORY, "hipMalloc per-sample accumulators");
    }
    c->acc_s_cap = chunk;
    c->acc_s.n = chunk;
    PT_HIP(hipMemsetAsync(c->acc_s.w, 0, chunk * pt::kFixWords * sizeof(unsigned long long), c->stream));
    PT_HIP(hipMemsetAsync(c->acc_s.hi, 0, chunk * pt::kFixWords * sizeof(unsigned long long), c->stream));
    PT_HIP(hipMemsetAsync(c->acc_s.big, 0, chunk * 3 * sizeof(double), c->stream));
    c->Q.acc_s = c->acc_s;
    return PT_OK;
}

template <class T>
int upload(Ctx* c, const std::vector<T>& host, const T** out) {
    *out = nullptr;
    if (host.empty()) return PT_OK;
    DeviceArray a;
    a.bytes = host.size() * sizeof(T);
    hipError_t e = hipMalloc(&a.ptr, a.bytes);
    if (e != hipSuccess) return fail(PT_ERR_OUT_OF_MEMORY, std::string("hipMalloc scene: ") + hipGetErrorString(e));
    c->scene_arrays.push_back(a);
    PT_HIP(hipMemcpyAsync(a.ptr, host.data(), a.bytes, hipMemcpyHostToDevice, c->stream));
    *out = (const T*)a.ptr;
    return PT_OK;
}

void free_scene(Ctx* c) {
    for (auto& a : c->scene_arrays) a.release();
    c->scene_arrays.clear();
    c->S = pt::DevScene{};
    c->has_scene = false;
}

inline float4 f4(float x, float y, float z, float w) { return make_float4(x, y, z, w); }
inline float u2f(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
inline pt::v3 ld3(const float* p) { return pt::v3{p[0], p[1], p[2]}; }

// Conservative AABB padding for the fp32 slab test (see k_render_pass).
inline void pad_box(float* lo, float* hi) {
    for (int k = 0; k < 3; k++) {
        float m = std::max(std::fabs(lo[k]), std::fabs(hi[k]));
        float e = m * 2.0e-6f + 1e-30f;
        lo[k] = lo[k] - e;
        hi[k] = hi[k] + e;
    }
}

// Analytic shapes tested linearly by the refill traversal kernels when there are at most this many
// (pt_scene.h ana_linear); 0: always through the analytic BVH.
#ifndef PT_ANA_LINEAR
#define PT_ANA_LINEAR 8
#endif
#ifndef PT_SHADE_ROUTE
#define PT_SHADE_ROUTE 1   // the routed shade (pt_scene.h shade_route); 0: every vertex of a FULL scene through the FULL shade
#endif
#ifndef PT_ROUTE
#define PT_ROUTE 1   // the routed split traversal (pt_scene.h route); 0: every ray through the FULL analytic half
#endif

// BVH2 → 4-wide nodes (pt_bvh.h collapse_bvh4) as device float4 rows.  The
// collapse keeps every path's pushes within the kStackMax-entry traversal stack.
// The triangle BVH: a binned-SAH BVH2 with kTriBins bins per axis and leaves of at most 3 triangles
// (one leaf chunk), collapsed to 4-wide nodes by the SAH-optimal dynamic program (pt_bvh.h
// collapse_bvh4_sah, a triangle test priced at kTriCost traversal steps).  Against 32 bins and the
// greedy collapse: C4 nodes per closest-hit ray 8.51 → 8.27, 6025 → 6065 Mrays/s (profiles/r04ab1_*).
// Making SAH's leaf decision always take a full chunk (3 triangles) measured slower.
constexpr int kTriBins = 128;
constexpr double kTriCost = 0.5;
int pack_nodes(const pt::BvhResult& b, std::vector<float4>& out, int32_t& num_nodes, bool sah = false) {
    pt::Bvh4Result r;
    if (sah) pt::collapse_bvh4_sah(b, pt::kStack4Budget, r, 1.0, kTriCost, 3);
    else pt::collapse_bvh4(b, pt::kStack4Budget, r);
    if (r.stack_need > pt::kStack4Budget) return fail(PT_ERR_UNSUPPORTED, "BVH4 traversal stack bound exceeded");
    out.resize(r.words.size() / 4);
    std::memcpy(out.data(), r.words.data(), r.words.size() * sizeof(uint32_t));
    num_nodes = (int32_t)r.nodes();
    return PT_OK;
}

// ---- The triangle BVH, built once per process for identical geometry (Scene.Compile compiles a scene
// once, Scene.cs:48-68; the reference has one Tree per Scene).  N contexts of one process (the .NET group
// host, bench.py --gpus N) upload the same scene: the first pt_upload_scene builds the BVH (1.1 s at 1M
// triangles on the host), the others wait for that build and upload its bytes.  The key is the triangle
// count, the build parameters and two independent 64-bit hashes of the triangles' vertices in the
// upload's order; the last two builds are kept.
struct TriBvhBuild {
    std::vector<uint32_t> order;      // BVH position -> index into tri_src
    std::vector<float4> nodes, chunks;
    int32_t num_nodes = 0;
    float box[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int rc = PT_OK;
    std::string err;
};
struct TriBvhKey {
    uint64_t n = 0, h1 = 0, h2 = 0;
    bool operator==(const TriBvhKey& o) const { return n == o.n && h1 == o.h1 && h2 == o.h2; }
};
struct TriBvhCache {
    std::mutex mu;
    std::vector<std::pair<TriBvhKey, std::shared_future<std::shared_ptr<const TriBvhBuild>>>> entries;
    int64_t builds = 0, hits = 0;
};
TriBvhCache& tri_bvh_cache() {
    static TriBvhCache c;
    return c;
}
// A finished build that no context holds (only the cache's own reference): evictable.  Builds held by live
// contexts and builds in progress are never evicted, so neither a host-only pt_scene_bvh_digest nor another
// scene's upload can push out the build a context of this process would reuse.
bool tri_bvh_evictable(const std::shared_future<std::shared_ptr<const TriBvhBuild>>& f) {
    if (f.wait_for(std::chrono::seconds(0)) != std::future_status::ready) return false;
    return f.get().use_count() <= 1;
}
constexpr size_t kTriBvhSpare = 2;   // unreferenced finished builds kept for a later upload of the same geometry
TriBvhKey tri_bvh_key(const pt_scene_desc* d, const std::vector<int32_t>& tri_src) {
    TriBvhKey k;
    k.n = (uint64_t)tri_src.size() ^ ((uint64_t)kTriBins << 40) ^ ((uint64_t)(kTriCost * 1024) << 52);
    uint64_t a = 0x243F6A8885A308D3ull, b = 0x13198A2E03707344ull;
    auto mix = [](uint64_t x) {
        x ^= x >> 33; x *= 0xFF51AFD7ED558CCDull; x ^= x >> 33; x *= 0xC4CEB9FE1A85EC53ull; x ^= x >> 33;
        return x;
    };
    for (int32_t s : tri_src) {
        uint32_t w[9];
        std::memcpy(w, d->tri_v1 + 3 * (size_t)s, 12);
        std::memcpy(w + 3, d->tri_v2 + 3 * (size_t)s, 12);
        std::memcpy(w + 6, d->tri_v3 + 3 * (size_t)s, 12);
        for (int j = 0; j < 9; j++) {
            a = (a ^ w[j]) * 0x100000001B3ull;          // FNV-1a over 32-bit words
            b = mix(b + w[j] + 0x9E3779B97F4A7C15ull);  // a splitmix chain
        }
    }
    k.h1 = a;
    k.h2 = b;
    return k;
}
std::shared_ptr<const TriBvhBuild> build_tri_bvh(const pt_scene_desc* d, const std::vector<int32_t>& tri_src) {
    auto out = std::make_shared<TriBvhBuild>();
    const size_t nt = tri_src.size();
    std::vector<float> bmin(nt * 3), bmax(nt * 3);
    for (size_t i = 0; i < nt; i++) {
        int s = tri_src[i];
        for (int k = 0; k < 3; k++) {
            float a = d->tri_v1[3 * s + k], b = d->tri_v2[3 * s + k], cc = d->tri_v3[3 * s + k];
            bmin[3 * i + k] = std::fmin(std::fmin(a, b), cc);
            bmax[3 * i + k] = std::fmax(std::fmax(a, b), cc);
        }
        pad_box(&bmin[3 * i], &bmax[3 * i]);
    }
    pt::BvhResult tb;
    pt::build_bvh(bmin.data(), bmax.data(), (int64_t)nt, 0, tb, 3, false, kTriBins);   // leaves fit one chunk
    std::vector<float4> tri_recs(nt * 3);
    for (size_t i = 0; i < nt; i++) {
        int s = tri_src[tb.order[i]];
        pt::v3 v1 = ld3(d->tri_v1 + 3 * s), v2 = ld3(d->tri_v2 + 3 * s), v3_ = ld3(d->tri_v3 + 3 * s);
        pt::v3 e1 = pt::sub(v2, v1), e2 = pt::sub(v3_, v1);  // Triangle.cs:97-98
        tri_recs[3 * i + 0] = f4(v1.x, v1.y, v1.z, e1.x);
        tri_recs[3 * i + 1] = f4(e1.y, e1.z, e2.x, e2.y);
        tri_recs[3 * i + 2] = f4(e2.z, 0.f, 0.f, 0.f);
    }
    // 8-wide nodes with quantized child boxes (pt_bvh.h collapse_bvh8q), leaf chunks (one
    // 128-B line per leaf: the first record in word 0, up to three {v1, e1, e2})
    pt::Bvh8Result b8;
    pt::collapse_bvh8q(tb, pt::kStackMax, b8, 1.0, kTriCost, 3);
    if (b8.stack_need > pt::kStackMax) {
        out->rc = fail(PT_ERR_UNSUPPORTED, "BVH8 traversal stack bound exceeded");
        out->err = g_last_error;
        return out;
    }
    if (b8.chunk_first.size() > 0x1FFFFFFFu) {
        out->rc = fail(PT_ERR_UNSUPPORTED, "too many triangle leaves");
        out->err = g_last_error;
        return out;
    }
    out->nodes.resize(b8.words.size() / 4);
    std::memcpy(out->nodes.data(), b8.words.data(), b8.words.size() * sizeof(uint32_t));
    out->num_nodes = (int32_t)b8.nodes();
    out->chunks.resize(8 * b8.chunk_first.size());
    for (size_t ci = 0; ci < b8.chunk_first.size(); ci++) {
        float w[32] = {0.f};
        const uint32_t first = b8.chunk_first[ci], cnt = b8.chunk_count[ci];
        const uint32_t w0 = first | ((cnt - 1u) << 29);   // the first record, the count - 1 in bits 29-30
        std::memcpy(&w[0], &w0, 4);
        for (uint32_t t = 0; t < cnt; t++) {
            const float* rf = reinterpret_cast<const float*>(&tri_recs[3 * (size_t)(first + t)]);
            for (int j = 0; j < 9; j++) w[1 + 9 * t + j] = rf[j];
        }
        std::memcpy(&out->chunks[8 * ci], w, sizeof w);
    }
    if (!out->nodes.empty()) {   // root box = union of the root node's children (their quantized boxes)
        const uint32_t* w = b8.words.data();
        for (int ax = 0; ax < 3; ax++) { out->box[ax] = INFINITY; out->box[3 + ax] = -INFINITY; }
        for (int k = 0; k < (int)(w[3] >> 28); k++) {
            float lo[3], hi[3];
            pt::bvh8_child_box(w, k, lo, hi);
            for (int ax = 0; ax < 3; ax++) {
                out->box[ax] = std::min(out->box[ax], lo[ax]);
                out->box[3 + ax] = std::max(out->box[3 + ax], hi[ax]);
            }
        }
    }
    out->order = std::move(tb.order);
    return out;
}
// The build for this geometry: the cached one, one in progress on another thread (waited for), or a new one.
std::shared_ptr<const TriBvhBuild> tri_bvh_shared(const pt_scene_desc* d, const std::vector<int32_t>& tri_src) {
    const TriBvhKey key = tri_bvh_key(d, tri_src);
    TriBvhCache& C = tri_bvh_cache();
    std::promise<std::shared_ptr<const TriBvhBuild>> mine;
    std::shared_future<std::shared_ptr<const TriBvhBuild>> theirs;
    {
        std::lock_guard<std::mutex> lk(C.mu);
        for (auto& e : C.entries)
            if (e.first == key) { theirs = e.second; break; }
        if (theirs.valid()) {
            C.hits++;
        } else {
            C.builds++;
            C.entries.emplace_back(key, mine.get_future().share());
            // oldest first, only the evictable ones, down to kTriBvhSpare of them
            size_t spare = 0;
            for (auto& e : C.entries) spare += tri_bvh_evictable(e.second) ? 1 : 0;
            for (size_t i = 0; i < C.entries.size() && spare > kTriBvhSpare;) {
                if (tri_bvh_evictable(C.entries[i].second)) {
                    C.entries.erase(C.entries.begin() + (long)i);
                    spare--;
                } else {
                    i++;
                }
            }
        }
    }
    if (theirs.valid()) {
        std::shared_ptr<const TriBvhBuild> r = theirs.get();   // waits while another thread builds it
        if (r->rc == PT_OK) return r;
        return build_tri_bvh(d, tri_src);                        // that build failed: this thread's own error
    }
    std::shared_ptr<const TriBvhBuild> r = build_tri_bvh(d, tri_src);
    mine.set_value(r);
    if (r->rc != PT_OK) {   // a failed build is not kept
        std::lock_guard<std::mutex> lk(C.mu);
        for (size_t i = 0; i < C.entries.size(); i++)
            if (C.entries[i].first == key) { C.entries.erase(C.entries.begin() + (long)i); break; }
    }
    return r;
}

// A context lets go of its build (next upload, pt_destroy): the last context of a geometry takes its cache entry
// along, so the host memory (tens of MB at 1M triangles) lives as long as a context uses it.
void tri_bvh_release(Ctx* c) {
    if (!c->tri_build) return;
    TriBvhCache& C = tri_bvh_cache();
    std::lock_guard<std::mutex> lk(C.mu);
    for (size_t i = 0; i < C.entries.size(); i++) {
        auto& f = C.entries[i].second;
        if (f.wait_for(std::chrono::seconds(0)) == std::future_status::ready && f.get() == c->tri_build &&
            f.get().use_count() <= 2) {   // the cache's reference and this context's
            C.entries.erase(C.entries.begin() + (long)i);
            break;
        }
    }
    c->tri_build.reset();
}

// Box of a light shape as Box.Center / Box.OuterRadius compute it (Box.cs:316-324).
void light_sphere_of_box(pt::v3 mn, pt::v3 mx, pt::DevLight& L) {
    pt::v3 center = pt::add(mn, pt::mul(pt::sub(mx, mn), pt::mk(0.5, 0.5, 0.5)));
    L.center[0] = center.x; L.center[1] = center.y; L.center[2] = center.z;
    L.radius = (double)pt::lengthf(pt::sub(mn, center));
}

// ---- §8f row 4 host side: SDF tree → postfix program, boxes (IShape.BoundingBox)
struct HostBox { pt::v3 mn, mx; };
inline HostBox box_extend(const HostBox& a, const HostBox& b) { return HostBox{pt::vmin(a.mn, b.mn), pt::vmax(a.mx, b.mx)}; }
inline HostBox box_mul(const double* m, const HostBox& b) { HostBox r; pt::mat_box(m, b.mn, b.mx, r.mn, r.mx); return r; }
inline void rows12(const double* m16, double* out) { for (int k = 0; k < 12; k++) out[k] = m16[k]; }

// SDF.BoundingBox per node (SDF.cs:136-139, 191-195, 214-219, 280-284, 313-318, 344-353, 374-382, 413-434, 470-476, 509-530, 555-558)
HostBox sdf_box(const pt_scene_desc* d, int ni) {
    const pt_sdf_node& n = d->sdf_nodes[ni];
    const double* P = n.params;
    switch (n.op) {
        case PT_SDF_SPHERE: { double r = P[0]; return HostBox{pt::mk(-r, -r, -r), pt::mk(r, r, r)}; }
        case PT_SDF_CUBE: {
            double x = (double)(float)P[0] / 2, y = (double)(float)P[1] / 2, z = (double)(float)P[2] / 2;
            return HostBox{pt::mk(-x, -y, -z), pt::mk(x, y, z)};
        }
        case PT_SDF_CYLINDER: { double r = P[0], h = P[1] / 2; return HostBox{pt::mk(-r, -h, -r), pt::mk(r, h, r)}; }
        case PT_SDF_CAPSULE: {
            pt::v3 A = pt::mk(P[0], P[1], P[2]), B = pt::mk(P[3], P[4], P[5]);
            pt::v3 a = pt::vmin(A, B), b = pt::vmax(A, B);
            double r = P[6];   // SubScalar / AddScalar
            return HostBox{pt::mk((double)a.x - r, (double)a.y - r, (double)a.z - r),
                           pt::mk((double)b.x + r, (double)b.y + r, (double)b.z + r)};
        }
        case PT_SDF_TORUS: { double a = P[1], b = P[1] + P[0]; return HostBox{pt::mk(-b, -b, a), pt::mk(b, b, a)}; }
        case PT_SDF_TRANSFORM: return box_mul(n.matrix, sdf_box(d, d->sdf_children[n.first_child]));
        case PT_SDF_SCALE: {
            double f = (double)(float)P[0];   // new Matrix().Scale(new Vector(f, f, f))
            const double m[16] = {f, 0, 0, 0, 0, f, 0, 0, 0, 0, f, 0, 0, 0, 0, 1};
            return box_mul(m, sdf_box(d, d->sdf_children[n.first_child]));
        }
        case PT_SDF_UNION:
        case PT_SDF_INTERSECTION: {
            HostBox r{pt::zero3(), pt::zero3()};
            for (int i = 0; i < n.num_children; i++) {
                HostBox b = sdf_box(d, d->sdf_children[n.first_child + i]);
                r = i == 0 ? b : box_extend(r, b);
            }
            return r;
        }
        case PT_SDF_DIFFERENCE:
            return n.num_children > 0 ? sdf_box(d, d->sdf_children[n.first_child]) : HostBox{pt::zero3(), pt::zero3()};
        default: return HostBox{pt::zero3(), pt::zero3()};   // RepeatSDF: new Box()
    }
}

// Postfix program of an SDF tree (pt_ext.h SdfOp): SDF.Evaluate's recursion unrolled.
struct SdfCompiler {
    const pt_scene_desc* d;
    std::vector<pt::DevSdfIns> prog;
    std::vector<double> params;
    int ps = 0, vs = 0, max_ps = 0, max_vs = 0;
    void emit(int op, const double* P, int np) {
        prog.push_back(pt::DevSdfIns{op, (int32_t)params.size()});
        for (int k = 0; k < np; k++) params.push_back(P[k]);
        if (np == 0) params.push_back(0.0);
    }
    void value() { vs++; max_vs = std::max(max_vs, vs); }
    void node(int ni) {
        const pt_sdf_node& n = d->sdf_nodes[ni];
        const double* P = n.params;
        auto child = [&](int k) { return d->sdf_children[n.first_child + k]; };
        switch (n.op) {
            case PT_SDF_SPHERE: emit(pt::SDF_LEAF_SPHERE, P, 2); value(); return;
            case PT_SDF_CUBE: {   // Size is a Vector: its halves are taken from the fp32 values
                const double q[3] = {(double)(float)P[0], (double)(float)P[1], (double)(float)P[2]};
                emit(pt::SDF_LEAF_CUBE, q, 3); value(); return;
            }
            case PT_SDF_CYLINDER: emit(pt::SDF_LEAF_CYLINDER, P, 2); value(); return;
            case PT_SDF_CAPSULE: emit(pt::SDF_LEAF_CAPSULE, P, 8); value(); return;
            case PT_SDF_TORUS: emit(pt::SDF_LEAF_TORUS, P, 4); value(); return;
            case PT_SDF_TRANSFORM:
            case PT_SDF_SCALE:
            case PT_SDF_REPEAT: {
                if (n.op == PT_SDF_TRANSFORM) {
                    double inv[12];
                    rows12(n.inverse, inv);
                    emit(pt::SDF_PUSH_TRANSFORM, inv, 12);
                } else if (n.op == PT_SDF_SCALE) {
                    emit(pt::SDF_PUSH_SCALE, P, 1);
                } else {
                    const double st[3] = {(double)(float)P[0], (double)(float)P[1], (double)(float)P[2]};
                    emit(pt::SDF_PUSH_REPEAT, st, 3);
                }
                ps++;
                max_ps = std::max(max_ps, ps);
                node(child(0));
                emit(pt::SDF_POP_POINT, nullptr, 0);
                ps--;
                if (n.op == PT_SDF_SCALE) emit(pt::SDF_MUL, P, 1);
                return;
            }
            default: {   // Union / Difference / Intersection: fold over the children in order
                const int fold = n.op == PT_SDF_UNION ? pt::SDF_UNION : n.op == PT_SDF_DIFFERENCE ? pt::SDF_DIFFERENCE
                                                                                               : pt::SDF_INTERSECTION;
                if (n.num_children == 0) { emit(pt::SDF_CONST0, nullptr, 0); value(); return; }
                node(child(0));
                for (int k = 1; k < n.num_children; k++) {
                    node(child(k));
                    emit(fold, nullptr, 0);
                    vs--;
                }
            }
        }
    }
};

// A volume view over host (validation / light registration) or device data.
pt::DevVolume dev_volume(const pt_volume& v, const double* data, const pt::DevWindow* windows) {
    pt::DevVolume o{};
    o.data = data; o.windows = windows;
    o.w = v.w; o.h = v.h; o.d = v.d; o.nwin = v.num_windows; o.zscale = v.zscale; o.zinv = pt::vol_zinv(v.zscale);
    for (int k = 0; k < 3; k++) { o.bmin[k] = v.box_min[k]; o.bmax[k] = v.box_max[k]; }
    return o;
}

int validate_scene(const pt_scene_desc* d) {
    if (!d) return fail(PT_ERR_INVALID_ARG, "scene is NULL");
    if (d->num_materials <= 0 || !d->materials) return fail(PT_ERR_INVALID_ARG, "scene has no materials");
    if (d->num_shapes < 0 || (d->num_shapes > 0 && (!d->shape_kind || !d->shape_index)))
        return fail(PT_ERR_INVALID_ARG, "shape arrays missing");
    auto chk_mat = [&](const int32_t* m, int n) {
        for (int i = 0; i < n; i++) if (m[i] < 0 || m[i] >= d->num_materials) return false;
        return true;
    };
    if (d->num_spheres > 0 && (!d->sphere_center || !d->sphere_radius || !d->sphere_material ||
                               !chk_mat(d->sphere_material, d->num_spheres)))
        return fail(PT_ERR_INVALID_ARG, "bad sphere arrays");
    if (d->num_cubes > 0 && (!d->cube_min || !d->cube_max || !d->cube_material || !chk_mat(d->cube_material, d->num_cubes)))
        return fail(PT_ERR_INVALID_ARG, "bad cube arrays");
    if (d->num_planes > 0 && (!d->plane_point || !d->plane_normal || !d->plane_material ||
                              !chk_mat(d->plane_material, d->num_planes)))
        return fail(PT_ERR_INVALID_ARG, "bad plane arrays");
    if (d->num_triangles > 0 && (!d->tri_v1 || !d->tri_v2 || !d->tri_v3 || !d->tri_n1 || !d->tri_n2 || !d->tri_n3 ||
                                 !d->tri_material || !chk_mat(d->tri_material, d->num_triangles)))
        return fail(PT_ERR_INVALID_ARG, "bad triangle arrays");
    if (d->num_meshes > 0 && (!d->mesh_first || !d->mesh_count)) return fail(PT_ERR_INVALID_ARG, "bad mesh arrays");
    if (d->num_textures < 0 || (d->num_textures > 0 && !d->textures)) return fail(PT_ERR_INVALID_ARG, "bad texture arrays");
    for (int i = 0; i < d->num_textures; i++) {
        const pt_texture& t = d->textures[i];
        if (t.width < 2 || t.height < 2 || !t.data)   // BilinearSample reads x0 + 1 / y0 + 1 (Texture.cs:198-206)
            return fail(PT_ERR_INVALID_ARG, "texture " + std::to_string(i) + ": needs data and width, height >= 2");
    }
    auto chk_tex = [&](int32_t t) { return t >= 0 && t <= d->num_textures; };
    for (int i = 0; i < d->num_materials; i++) {
        const pt_material& m = d->materials[i];
        if (!chk_tex(m.texture) || !chk_tex(m.normal_texture) || !chk_tex(m.bump_texture) || !chk_tex(m.gloss_texture))
            return fail(PT_ERR_INVALID_ARG, "material " + std::to_string(i) + ": texture reference out of range");
    }
    if (!chk_tex(d->env_texture)) return fail(PT_ERR_INVALID_ARG, "env_texture out of range");
    // §8f row 4
    if (d->num_sdf_nodes < 0 || (d->num_sdf_nodes > 0 && (!d->sdf_nodes || !d->sdf_children)))
        return fail(PT_ERR_INVALID_ARG, "bad SDF node arrays");
    for (int i = 0; i < d->num_sdf_nodes; i++) {
        const pt_sdf_node& n = d->sdf_nodes[i];
        if (n.op < PT_SDF_SPHERE || n.op > PT_SDF_REPEAT) return fail(PT_ERR_INVALID_ARG, "SDF node " + std::to_string(i) + ": bad op");
        const bool one = n.op == PT_SDF_TRANSFORM || n.op == PT_SDF_SCALE || n.op == PT_SDF_REPEAT;
        const bool many = n.op >= PT_SDF_UNION && n.op <= PT_SDF_INTERSECTION;
        if ((one && n.num_children != 1) || (!one && !many && n.num_children != 0) || n.num_children < 0)
            return fail(PT_ERR_INVALID_ARG, "SDF node " + std::to_string(i) + ": wrong number of children");
        for (int k = 0; k < n.num_children; k++) {
            int c = d->sdf_children[n.first_child + k];
            if (c < 0 || c >= i) return fail(PT_ERR_INVALID_ARG, "SDF node " + std::to_string(i) + ": children must precede their parent");
        }
    }
    if (d->num_sdf_shapes < 0 || (d->num_sdf_shapes > 0 && !d->sdf_shapes)) return fail(PT_ERR_INVALID_ARG, "bad SDF shapes");
    for (int i = 0; i < d->num_sdf_shapes; i++)
        if (d->sdf_shapes[i].root < 0 || d->sdf_shapes[i].root >= d->num_sdf_nodes ||
            d->sdf_shapes[i].material < 0 || d->sdf_shapes[i].material >= d->num_materials)
            return fail(PT_ERR_INVALID_ARG, "SDF shape " + std::to_string(i) + ": bad root or material");
    if (d->num_volumes < 0 || (d->num_volumes > 0 && !d->volumes)) return fail(PT_ERR_INVALID_ARG, "bad volumes");
    for (int i = 0; i < d->num_volumes; i++) {
        const pt_volume& v = d->volumes[i];
        if (v.w < 1 || v.h < 1 || v.d < 1 || !v.data || v.num_windows < 0 || (v.num_windows > 0 && !v.windows))
            return fail(PT_ERR_INVALID_ARG, "volume " + std::to_string(i) + ": bad grid or windows");
        for (int k = 0; k < v.num_windows; k++)
            if (v.windows[k].material < 0 || v.windows[k].material >= d->num_materials)
                return fail(PT_ERR_INVALID_ARG, "volume " + std::to_string(i) + ": window material out of range");
    }
    if (d->num_transformed < 0 || (d->num_transformed > 0 && !d->transformed)) return fail(PT_ERR_INVALID_ARG, "bad transformed shapes");
    for (int i = 0; i < d->num_transformed; i++) {
        const pt_transformed_shape& x = d->transformed[i];
        int lim = x.shape_kind == PT_SHAPE_SPHERE ? d->num_spheres : x.shape_kind == PT_SHAPE_CUBE ? d->num_cubes
                : x.shape_kind == PT_SHAPE_PLANE ? d->num_planes : x.shape_kind == PT_SHAPE_SDF ? d->num_sdf_shapes
                : x.shape_kind == PT_SHAPE_VOLUME ? d->num_volumes : x.shape_kind == PT_SHAPE_MESH ? d->num_meshes : -1;
        if (lim < 0) return fail(PT_ERR_UNSUPPORTED, "transformed shape " + std::to_string(i) + ": inner kind not on the GPU path");
        if (x.shape_index < 0 || x.shape_index >= lim) return fail(PT_ERR_INVALID_ARG, "transformed shape " + std::to_string(i) + ": inner index out of range");
    }
    if (d->num_triangles > 0 && ((d->tri_t1 != nullptr) != (d->tri_t2 != nullptr) || (d->tri_t1 != nullptr) != (d->tri_t3 != nullptr)))
        return fail(PT_ERR_INVALID_ARG, "tri_t1/t2/t3 must be all set or all NULL");
    for (int i = 0; i < d->num_shapes; i++) {
        int k = d->shape_kind[i], j = d->shape_index[i];
        int lim = k == PT_SHAPE_SPHERE ? d->num_spheres : k == PT_SHAPE_CUBE ? d->num_cubes
                : k == PT_SHAPE_PLANE ? d->num_planes : k == PT_SHAPE_TRIANGLE ? d->num_triangles
                : k == PT_SHAPE_MESH ? d->num_meshes : k == PT_SHAPE_SDF ? d->num_sdf_shapes
                : k == PT_SHAPE_VOLUME ? d->num_volumes : k == PT_SHAPE_TRANSFORMED ? d->num_transformed : -1;
        if (lim < 0) return fail(PT_ERR_UNSUPPORTED, "unsupported shape kind " + std::to_string(k));
        if (j < 0 || j >= lim) return fail(PT_ERR_INVALID_ARG, "shape index out of range at shape " + std::to_string(i));
        if (k == PT_SHAPE_MESH) {
            int64_t f = d->mesh_first[j], n = d->mesh_count[j];
            if (f < 0 || n < 0 || f + n > d->num_triangles) return fail(PT_ERR_INVALID_ARG, "mesh range out of bounds");
        }
    }
    return PT_OK;
}

}  // namespace

extern "C" {

int pt_get_version(void) { return PT_ABI_VERSION; }

const char* pt_last_error(void) { return g_last_error.c_str(); }

int pt_device_count(int32_t* out_count) {
    if (!out_count) return fail(PT_ERR_INVALID_ARG, "out_count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) { *out_count = 0; return fail(PT_ERR_NO_DEVICE, hipGetErrorString(e)); }
    *out_count = n;
    return PT_OK;
}

int pt_create(const pt_device_opts* opts, void** out_ctx) {
    if (!opts || !out_ctx) return fail(PT_ERR_INVALID_ARG, "NULL argument");
    *out_ctx = nullptr;
    if (opts->width <= 1 || opts->height <= 1) return fail(PT_ERR_INVALID_ARG, "width/height must be > 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(PT_ERR_NO_DEVICE, "no HIP device");
    if (opts->device < 0 || opts->device >= ndev) return fail(PT_ERR_INVALID_ARG, "device ordinal out of range");
    Ctx* c = new (std::nothrow) Ctx();
    if (!c) return fail(PT_ERR_OUT_OF_MEMORY, "context allocation");
    c->device = opts->device;
    c->width = opts->width;
    c->height = opts->height;
    auto cleanup = [&](int code) { pt_destroy(c); return code; };
    if (hipSetDevice(c->device) != hipSuccess) return cleanup(fail(PT_ERR_HIP, "hipSetDevice"));
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) return cleanup(fail(PT_ERR_HIP, "stream"));
    if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess)
        return cleanup(fail(PT_ERR_HIP, "events"));
    if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_main, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_side[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_side[1], hipEventDisableTiming) != hipSuccess)
        return cleanup(fail(PT_ERR_HIP, "side stream"));
    size_t P = (size_t)c->width * (size_t)c->height;
    if (hipMalloc(&c->d_m, P * 3 * sizeof(double)) != hipSuccess || hipMalloc(&c->d_v, P * 3 * sizeof(double)) != hipSuccess ||
        hipMalloc(&c->d_n, P * sizeof(int32_t)) != hipSuccess ||
        hipMalloc(&c->d_counters, pt::kCounterAllocWords * sizeof(unsigned long long)) != hipSuccess ||
        hipHostMalloc(&c->h_counters, pt::kCounterAllocWords * sizeof(unsigned long long), hipHostMallocDefault) != hipSuccess)
        return cleanup(fail(PT_ERR_OUT_OF_MEMORY, "buffer allocation"));
    int rc = pt_reset_buffer(c);
    if (rc != PT_OK) return cleanup(rc);
    *out_ctx = c;
    return PT_OK;
}

int pt_reset_buffer(void* ctx) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    PT_HIP(hipSetDevice(c->device));
    size_t P = (size_t)c->width * (size_t)c->height;
    PT_HIP(hipMemsetAsync(c->d_m, 0, P * 3 * sizeof(double), c->stream));
    PT_HIP(hipMemsetAsync(c->d_v, 0, P * 3 * sizeof(double), c->stream));
    PT_HIP(hipMemsetAsync(c->d_n, 0, P * sizeof(int32_t), c->stream));
    PT_HIP(hipStreamSynchronize(c->stream));
    c->stats.rays_total = 0;
    c->stats.total_ms = 0;
    c->stats.passes = 0;
    return PT_OK;
}

int pt_upload_scene(void* ctx, const pt_scene_desc* d) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    int rc = validate_scene(d);
    if (rc != PT_OK) return rc;
    PT_HIP(hipSetDevice(c->device));
    auto t0 = std::chrono::steady_clock::now();
    free_scene(c);

    std::vector<pt::DevMaterial> mats((size_t)d->num_materials);
    for (int i = 0; i < d->num_materials; i++) {
        const pt_material& m = d->materials[i];
        pt::DevMaterial& o = mats[(size_t)i];
        for (int k = 0; k < 3; k++) o.color[k] = m.color[k];
        o.emittance = m.emittance;
        o.tint = m.tint;
        o.transparent = m.transparent;
        o.index = m.index;
        o.gloss = m.gloss;
        o.reflectivity = m.reflectivity;
        o.tex = m.texture - 1; o.ntex = m.normal_texture - 1; o.btex = m.bump_texture - 1; o.gtex = m.gloss_texture - 1;
        o.bump_multiplier = m.bump_multiplier;
    }
    // textures: one fp64 texel array in HBM, DevTexture views into it
    std::vector<size_t> tex_off((size_t)std::max(d->num_textures, 0));
    size_t texels = 0;
    for (int i = 0; i < d->num_textures; i++) {
        tex_off[(size_t)i] = texels;
        texels += 3 * (size_t)d->textures[i].width * (size_t)d->textures[i].height;
    }
    std::vector<double> tex_data(texels);
    for (int i = 0; i < d->num_textures; i++)
        std::memcpy(tex_data.data() + tex_off[(size_t)i], d->textures[i].data,
                    3 * (size_t)d->textures[i].width * (size_t)d->textures[i].height * sizeof(double));

    // --- gather primitives in Scene.Shapes order
    std::vector<int32_t> ana_kind, ana_scene;     // analytic prims (sphere, cube, SDF, volume, transformed)
    std::vector<int32_t> tri_src;                  // source triangle index per BVH triangle
    std::vector<int32_t> plane_scene;
    for (int i = 0; i < d->num_shapes; i++) {
        int k = d->shape_kind[i], j = d->shape_index[i];
        if (k == PT_SHAPE_PLANE) plane_scene.push_back(j);
        else if (k == PT_SHAPE_TRIANGLE) tri_src.push_back(j);
        else if (k == PT_SHAPE_MESH) for (int t = 0; t < d->mesh_count[j]; t++) tri_src.push_back(d->mesh_first[j] + t);
        else { ana_kind.push_back(k); ana_scene.push_back(j); }
    }
    if ((int64_t)tri_src.size() >= (int64_t)(1u << 29) || ana_kind.size() >= (1u << 29))
        return fail(PT_ERR_UNSUPPORTED, "more than 2^29 primitives");

    // --- §8f row 4 tables: SDF programs, volumes, transformed shapes
    mats.push_back(pt::DevMaterial{});   // `new Material()` (Volume.MaterialAt's fallback)
    for (auto& m : mats.back().color) m = 0.0;
    mats.back().tex = mats.back().ntex = mats.back().btex = mats.back().gtex = -1;
    const int32_t default_mat = d->num_materials;
    SdfCompiler sdfc{d};
    std::vector<pt::DevSdfShape> sdf_shapes((size_t)std::max(d->num_sdf_shapes, 0));
    std::vector<HostBox> sdf_boxes(sdf_shapes.size());
    for (size_t i = 0; i < sdf_shapes.size(); i++) {
        pt::DevSdfShape& o = sdf_shapes[i];
        o.begin = (int32_t)sdfc.prog.size();
        sdfc.ps = sdfc.vs = 0;
        sdfc.node(d->sdf_shapes[i].root);
        o.len = (int32_t)sdfc.prog.size() - o.begin;
        o.mat = d->sdf_shapes[i].material;
        int leaves = 0, folds = 0;   // a chain: one leaf, no fold (pt_ext.h sdf_eval_chain)
        for (int k = o.begin; k < o.begin + o.len; k++) {
            const int op = sdfc.prog[(size_t)k].op;
            if (op <= pt::SDF_LEAF_TORUS) leaves++;
            if (op == pt::SDF_UNION || op == pt::SDF_DIFFERENCE || op == pt::SDF_INTERSECTION || op == pt::SDF_CONST0) folds++;
        }
        o.chain = (leaves == 1 && folds == 0) ? 1 : 0;
        sdf_boxes[i] = sdf_box(d, d->sdf_shapes[i].root);   // SDFShape.BoundingBox (SDF.cs:100-103)
        o.bmin[0] = sdf_boxes[i].mn.x; o.bmin[1] = sdf_boxes[i].mn.y; o.bmin[2] = sdf_boxes[i].mn.z;
        o.bmax[0] = sdf_boxes[i].mx.x; o.bmax[1] = sdf_boxes[i].mx.y; o.bmax[2] = sdf_boxes[i].mx.z;
    }
    if (sdfc.max_ps + 1 > pt::kSdfStack || sdfc.max_vs > pt::kSdfStack)
        return fail(PT_ERR_UNSUPPORTED, "SDF tree nested deeper than the device evaluator's stacks");
    std::vector<pt::DevWindow> windows;
    std::vector<size_t> vol_off, win_off;
    size_t voxels = 0;
    for (int i = 0; i < d->num_volumes; i++) {
        const pt_volume& v = d->volumes[i];
        vol_off.push_back(voxels);
        win_off.push_back(windows.size());
        voxels += (size_t)v.w * v.h * v.d;
        for (int k = 0; k < v.num_windows; k++)
            windows.push_back(pt::DevWindow{v.windows[k].lo, v.windows[k].hi, v.windows[k].material, 0});
    }
    std::vector<double> vox(voxels);
    for (int i = 0; i < d->num_volumes; i++)
        std::memcpy(vox.data() + vol_off[(size_t)i], d->volumes[i].data,
                    (size_t)d->volumes[i].w * d->volumes[i].h * d->volumes[i].d * sizeof(double));
    // host views (Scene.Add's MaterialAt(new Vector()) for light registration)
    auto host_volume = [&](int i) { return dev_volume(d->volumes[i], vox.data() + vol_off[(size_t)i], windows.data() + win_off[(size_t)i]); };
    // uniform-cell tables of the march skip (pt_ext.h vol_build_runs), one per volume
    std::vector<int8_t> vol_runs;
    std::vector<size_t> runs_off;
    std::vector<int32_t> zero_sign((size_t)std::max(d->num_volumes, 0));
    for (int i = 0; i < d->num_volumes; i++) {
        const pt_volume& v = d->volumes[i];
        runs_off.push_back(vol_runs.size());
        vol_runs.resize(vol_runs.size() + (size_t)(v.w + 1) * (v.h + 1) * (v.d + 1));
        pt::vol_build_runs(host_volume(i), vol_runs.data() + runs_off.back(), zero_sign[(size_t)i]);
    }
    // cell-major corners of the march (pt_ext.h vol_build_cells), per volume while they stay within
    // PT_VOL_CELLS_MAX bytes in all; cells_off = -1: the march reads the grid
    std::vector<double> vol_cells;
    std::vector<int64_t> cells_off((size_t)std::max(d->num_volumes, 0), -1);
    const char* cells_env = std::getenv("PT_VOL_CELLS");   // "0" at upload: the march reads the grid (tests)
    for (int i = 0; i < d->num_volumes && !(cells_env && !std::strcmp(cells_env, "0")); i++) {
        const pt_volume& v = d->volumes[i];
        const size_t n = 8 * (size_t)(v.w + 1) * (v.h + 1) * (v.d + 1);
        if ((vol_cells.size() + n) * sizeof(double) > (size_t)PT_VOL_CELLS_MAX) continue;
        cells_off[(size_t)i] = (int64_t)vol_cells.size();
        vol_cells.resize(vol_cells.size() + n);
        pt::vol_build_cells(host_volume(i), vol_cells.data() + cells_off[(size_t)i]);
    }
    const pt::v3 origin = pt::zero3();
    // IShape.BoundingBox of a shape that can be analytic or inner (exact, as the reference computes it)
    auto shape_box = [&](int k, int j) -> HostBox {
        switch (k) {
            case PT_SHAPE_SPHERE: {
                const float* cc = d->sphere_center + 3 * j;
                double r = d->sphere_radius[j];
                return HostBox{pt::mk((double)cc[0] - r, (double)cc[1] - r, (double)cc[2] - r),
                               pt::mk((double)cc[0] + r, (double)cc[1] + r, (double)cc[2] + r)};
            }
            case PT_SHAPE_CUBE: return HostBox{ld3(d->cube_min + 3 * j), ld3(d->cube_max + 3 * j)};
            case PT_SHAPE_PLANE: return HostBox{pt::mk(-1e9, -1e9, -1e9), pt::mk(1e9, 1e9, 1e9)};
            case PT_SHAPE_SDF: return sdf_boxes[(size_t)j];
            case PT_SHAPE_VOLUME: return HostBox{ld3(d->volumes[j].box_min), ld3(d->volumes[j].box_max)};
            case PT_SHAPE_MESH: {   // Mesh.BoundingBox (Mesh.cs:88-120)
                const int f = d->mesh_first[j], n = d->mesh_count[j];
                if (n <= 0) return HostBox{pt::zero3(), pt::zero3()};
                HostBox b{ld3(d->tri_v1 + 3 * f), ld3(d->tri_v1 + 3 * f)};
                for (int t = f; t < f + n; t++) {
                    b.mn = pt::vmin(pt::vmin(pt::vmin(b.mn, ld3(d->tri_v1 + 3 * t)), ld3(d->tri_v2 + 3 * t)), ld3(d->tri_v3 + 3 * t));
                    b.mx = pt::vmax(pt::vmax(pt::vmax(b.mx, ld3(d->tri_v1 + 3 * t)), ld3(d->tri_v2 + 3 * t)), ld3(d->tri_v3 + 3 * t));
                }
                return b;
            }
        }
        return HostBox{pt::zero3(), pt::zero3()};
    };
    // IShape.MaterialAt(p) of an analytic / inner shape
    auto shape_mat = [&](int k, int j, pt::v3 p) -> int32_t {
        switch (k) {
            case PT_SHAPE_SPHERE: return d->sphere_material[j];
            case PT_SHAPE_CUBE: return d->cube_material[j];
            case PT_SHAPE_PLANE: return d->plane_material[j];
            case PT_SHAPE_SDF: return d->sdf_shapes[j].material;
            case PT_SHAPE_VOLUME: { pt::DevVolume v = host_volume(j); return pt::vol_material(v, p, default_mat); }
        }
        return default_mat;
    };
    // analytic-format record of a shape (top level: ana_recs; inner of a transformed shape: ext_recs)
    auto make_rec = [&](int k, int j, int32_t ext_mat, float4* r) {
        if (k == PT_SHAPE_SPHERE) {
            const float* cc = d->sphere_center + 3 * j;
            uint64_t rb; double rad = d->sphere_radius[j]; std::memcpy(&rb, &rad, 8);
            r[0] = f4(cc[0], cc[1], cc[2], u2f(pt::KIND_SPHERE));
            r[1] = f4(0.f, 0.f, 0.f, u2f((uint32_t)j));
            r[2] = f4(u2f((uint32_t)d->sphere_material[j]), u2f((uint32_t)(rb & 0xFFFFFFFFu)), u2f((uint32_t)(rb >> 32)), 0.f);
        } else if (k == PT_SHAPE_CUBE) {
            const float* mn = d->cube_min + 3 * j; const float* mx = d->cube_max + 3 * j;
            r[0] = f4(mn[0], mn[1], mn[2], u2f(pt::KIND_CUBE));
            r[1] = f4(mx[0], mx[1], mx[2], u2f((uint32_t)j));
            r[2] = f4(u2f((uint32_t)d->cube_material[j]), 0.f, 0.f, 0.f);
        } else if (k == PT_SHAPE_PLANE) {
            const float* pp = d->plane_point + 3 * j; const float* nn = d->plane_normal + 3 * j;
            r[0] = f4(pp[0], pp[1], pp[2], u2f(pt::KIND_PLANE));
            r[1] = f4(nn[0], nn[1], nn[2], u2f((uint32_t)j));
            r[2] = f4(u2f((uint32_t)d->plane_material[j]), 0.f, 0.f, 0.f);
        } else {   // SDF / volume / transformed: the shape lives in its table, `ext_mat` = MaterialAt(origin)
            const int32_t kind = k == PT_SHAPE_SDF ? pt::KIND_SDF : k == PT_SHAPE_VOLUME ? pt::KIND_VOLUME : pt::KIND_XFORM;
            r[0] = f4(0.f, 0.f, 0.f, u2f((uint32_t)kind));
            r[1] = f4(0.f, 0.f, 0.f, u2f((uint32_t)j));
            r[2] = f4(u2f((uint32_t)ext_mat), u2f((uint32_t)j), 0.f, 0.f);
        }
    };
    // instanced meshes: one object-space BVH4 per distinct inner mesh (BLAS), records in their own arrays
    std::vector<pt::DevBlas> blas;
    std::vector<float4> blas_nodes, blas_recs, blas_shade, blas_uv;
    std::vector<int32_t> blas_of_mesh((size_t)std::max(d->num_meshes, 0), -1);
    for (int i = 0; i < d->num_transformed; i++) {
        const pt_transformed_shape& x = d->transformed[i];
        if (x.shape_kind != PT_SHAPE_MESH || blas_of_mesh[(size_t)x.shape_index] >= 0) continue;
        const int f = d->mesh_first[x.shape_index], n = d->mesh_count[x.shape_index];
        std::vector<float> lo((size_t)n * 3), hi((size_t)n * 3);
        for (int t = 0; t < n; t++)
            for (int k = 0; k < 3; k++) {
                float a = d->tri_v1[3 * (f + t) + k], b = d->tri_v2[3 * (f + t) + k], cc = d->tri_v3[3 * (f + t) + k];
                lo[3 * (size_t)t + k] = std::fmin(std::fmin(a, b), cc);
                hi[3 * (size_t)t + k] = std::fmax(std::fmax(a, b), cc);
            }
        for (int t = 0; t < n; t++) pad_box(&lo[3 * (size_t)t], &hi[3 * (size_t)t]);
        pt::BvhResult bb;
        pt::build_bvh(lo.data(), hi.data(), (int64_t)n, 0, bb);
        std::vector<float4> nodes;
        int32_t nn = 0;
        if ((rc = pack_nodes(bb, nodes, nn))) return rc;
        pt::DevBlas B{(int32_t)(blas_nodes.size() / 8), nn, (int32_t)(blas_recs.size() / 3), 0};
        blas_nodes.insert(blas_nodes.end(), nodes.begin(), nodes.end());
        for (int t = 0; t < n; t++) {
            const int src = f + (int)bb.order[(size_t)t];
            pt::v3 v1 = ld3(d->tri_v1 + 3 * src), v2 = ld3(d->tri_v2 + 3 * src), v3_ = ld3(d->tri_v3 + 3 * src);
            pt::v3 e1 = pt::sub(v2, v1), e2 = pt::sub(v3_, v1);
            blas_recs.push_back(f4(v1.x, v1.y, v1.z, e1.x));
            blas_recs.push_back(f4(e1.y, e1.z, e2.x, e2.y));
            blas_recs.push_back(f4(e2.z, 0.f, 0.f, 0.f));
            const float* n1 = d->tri_n1 + 3 * src; const float* n2 = d->tri_n2 + 3 * src; const float* n3 = d->tri_n3 + 3 * src;
            blas_shade.push_back(f4(n1[0], n1[1], n1[2], n2[0]));
            blas_shade.push_back(f4(n2[1], n2[2], n3[0], n3[1]));
            blas_shade.push_back(f4(n3[2], u2f((uint32_t)d->tri_material[src]), 0.f, 0.f));
            const float zero[3] = {0.f, 0.f, 0.f};
            const float* t1 = d->tri_t1 ? d->tri_t1 + 3 * src : zero;
            const float* t2 = d->tri_t2 ? d->tri_t2 + 3 * src : zero;
            const float* t3 = d->tri_t3 ? d->tri_t3 + 3 * src : zero;
            blas_uv.push_back(f4(t1[0], t1[1], t2[0], t2[1]));
            blas_uv.push_back(f4(t3[0], t3[1], 0.f, 0.f));
        }
        blas_of_mesh[(size_t)x.shape_index] = (int32_t)blas.size();
        blas.push_back(B);
    }
    std::vector<pt::DevXform> xforms((size_t)std::max(d->num_transformed, 0));
    std::vector<float4> ext_recs(xforms.size() * 3);
    std::vector<HostBox> xform_boxes(xforms.size()), xform_bvh_boxes(xforms.size());
    // Hits of marched shapes can sit just outside their box (SDF: start 1e-4 and a 1e-3 jump back;
    // Volume: one step of 1/512 before the box): the BVH boxes are widened by that much.
    auto march_pad = [](int k) { return k == PT_SHAPE_SDF ? 2e-3 : k == PT_SHAPE_VOLUME ? 4.0 / 512 : 0.0; };
    for (size_t i = 0; i < xforms.size(); i++) {
        const pt_transformed_shape& x = d->transformed[i];
        pt::DevXform& o = xforms[i];
        rows12(x.matrix, o.m);
        rows12(x.inverse, o.inv);
        o.kind = x.shape_kind == PT_SHAPE_SDF ? pt::KIND_SDF : x.shape_kind == PT_SHAPE_VOLUME ? pt::KIND_VOLUME
               : x.shape_kind == PT_SHAPE_MESH ? pt::KIND_MESH : x.shape_kind;
        o.rec = x.shape_kind == PT_SHAPE_MESH ? blas_of_mesh[(size_t)x.shape_index] : (int32_t)i;
        if (x.shape_kind != PT_SHAPE_MESH)
            make_rec(x.shape_kind, x.shape_index, shape_mat(x.shape_kind, x.shape_index, origin), &ext_recs[3 * i]);
        HostBox ib = shape_box(x.shape_kind, x.shape_index);
        xform_boxes[i] = box_mul(x.matrix, ib);   // TransformedShape.BoundingBox (TransformedShape.cs:36-39)
        const double mp = march_pad(x.shape_kind);
        HostBox pb{pt::mk((double)ib.mn.x - mp, (double)ib.mn.y - mp, (double)ib.mn.z - mp),
                   pt::mk((double)ib.mx.x + mp, (double)ib.mx.y + mp, (double)ib.mx.z + mp)};
        xform_bvh_boxes[i] = box_mul(x.matrix, pb);
    }
    auto shape_mat_any = [&](int k, int j, pt::v3 p) -> int32_t {   // including TransformedShape.MaterialAt
        if (k == PT_SHAPE_TRANSFORMED) return shape_mat(d->transformed[j].shape_kind, d->transformed[j].shape_index, p);
        return shape_mat(k, j, p);
    };

    // --- triangle BVH (built once per process for the same geometry: tri_bvh_shared)
    const size_t nt = tri_src.size();
    const auto tbuild_t0 = std::chrono::steady_clock::now();
    const std::shared_ptr<const TriBvhBuild> tbv = tri_bvh_shared(d, tri_src);
    tri_bvh_release(c);   // the previous upload's build
    if (tbv->rc == PT_OK) c->tri_build = tbv;
    c->tri_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tbuild_t0).count();
    if (tbv->rc != PT_OK) return fail(tbv->rc, tbv->err);
    std::vector<float4> tri_recs(nt * 3), tri_shade(nt * 3);
    const bool want_uv = d->num_textures > 0 && nt > 0;   // texture coordinates only matter with textures
    std::vector<float4> tri_uv(want_uv ? nt * 2 : 0);
    for (size_t i = 0; i < nt; i++) {
        int s = tri_src[tbv->order[i]];
        pt::v3 v1 = ld3(d->tri_v1 + 3 * s), v2 = ld3(d->tri_v2 + 3 * s), v3_ = ld3(d->tri_v3 + 3 * s);
        pt::v3 e1 = pt::sub(v2, v1), e2 = pt::sub(v3_, v1);  // Triangle.cs:97-98
        tri_recs[3 * i + 0] = f4(v1.x, v1.y, v1.z, e1.x);
        tri_recs[3 * i + 1] = f4(e1.y, e1.z, e2.x, e2.y);
        tri_recs[3 * i + 2] = f4(e2.z, 0.f, 0.f, 0.f);
        const float* n1 = d->tri_n1 + 3 * s; const float* n2 = d->tri_n2 + 3 * s; const float* n3 = d->tri_n3 + 3 * s;
        tri_shade[3 * i + 0] = f4(n1[0], n1[1], n1[2], n2[0]);
        tri_shade[3 * i + 1] = f4(n2[1], n2[2], n3[0], n3[1]);
        tri_shade[3 * i + 2] = f4(n3[2], u2f((uint32_t)d->tri_material[s]), 0.f, 0.f);
        if (want_uv) {
            const float zero[3] = {0.f, 0.f, 0.f};
            const float* t1 = d->tri_t1 ? d->tri_t1 + 3 * s : zero;
            const float* t2 = d->tri_t2 ? d->tri_t2 + 3 * s : zero;
            const float* t3 = d->tri_t3 ? d->tri_t3 + 3 * s : zero;
            tri_uv[2 * i + 0] = f4(t1[0], t1[1], t2[0], t2[1]);
            tri_uv[2 * i + 1] = f4(t3[0], t3[1], 0.f, 0.f);
        }
    }
    const std::vector<float4>& tri_nodes = tbv->nodes;
    const int32_t tri_num_nodes = tbv->num_nodes;
    const std::vector<float4>& tri_chunks = tbv->chunks;
    float tri_box[6];
    std::memcpy(tri_box, tbv->box, sizeof tri_box);

    // --- analytic BVH (spheres, cubes, SDF shapes, volumes, transformed shapes)
    const size_t na = ana_kind.size();
    std::vector<float> amin(na * 3), amax(na * 3);
    for (size_t i = 0; i < na; i++) {
        int k = ana_kind[i], j = ana_scene[i];
        if (k == PT_SHAPE_SPHERE) {
            double r = d->sphere_radius[j];
            for (int q = 0; q < 3; q++) {
                double cc = d->sphere_center[3 * j + q];
                amin[3 * i + q] = std::nextafter((float)(cc - r), -INFINITY);
                amax[3 * i + q] = std::nextafter((float)(cc + r), INFINITY);
            }
        } else {
            HostBox b = k == PT_SHAPE_TRANSFORMED ? xform_bvh_boxes[(size_t)j] : shape_box(k, j);
            const double mp = k == PT_SHAPE_TRANSFORMED ? 0.0 : march_pad(k);
            const float lo[3] = {b.mn.x, b.mn.y, b.mn.z}, hi[3] = {b.mx.x, b.mx.y, b.mx.z};
            for (int q = 0; q < 3; q++) {
                amin[3 * i + q] = (float)((double)lo[q] - mp);
                amax[3 * i + q] = (float)((double)hi[q] + mp);
            }
        }
        pad_box(&amin[3 * i], &amax[3 * i]);
    }
    pt::BvhResult ab;
    pt::build_bvh(amin.data(), amax.data(), (int64_t)na, 0, ab);
    std::vector<float4> ana_recs(na * 3);
    // position in ana_recs of each shape (first occurrence), per kind: Sampler's identity test
    std::vector<std::vector<int32_t>> ana_pos(8);
    const int32_t counts[8] = {d->num_spheres, d->num_cubes, 0, 0, 0, d->num_sdf_shapes, d->num_volumes, d->num_transformed};
    for (int k = 0; k < 8; k++) ana_pos[(size_t)k].assign((size_t)std::max(counts[k], 0), -1);
    for (size_t i = 0; i < na; i++) {
        size_t src = ab.order[i];
        int k = ana_kind[src], j = ana_scene[src];
        make_rec(k, j, shape_mat_any(k, j, origin), &ana_recs[3 * i]);
        if (ana_pos[(size_t)k][(size_t)j] < 0) ana_pos[(size_t)k][(size_t)j] = (int32_t)i;
    }
    // the row-4 records (SDF shapes, volumes, transformed shapes) with their BVH boxes, in record order:
    // what the routed split's refill kernels test against a ray's segment (pt_scene.h route)
    std::vector<float4> heavy;
    for (size_t i = 0; i < na; i++) {
        const size_t src = ab.order[i];
        const int k = ana_kind[src];
        if (k != PT_SHAPE_SDF && k != PT_SHAPE_VOLUME && k != PT_SHAPE_TRANSFORMED) continue;
        heavy.push_back(f4(amin[3 * src], amin[3 * src + 1], amin[3 * src + 2], u2f((uint32_t)i)));
        heavy.push_back(f4(amax[3 * src], amax[3 * src + 1], amax[3 * src + 2], 0.f));
    }
    std::vector<float4> ana_nodes;
    int32_t ana_num_nodes = 0;
    if ((rc = pack_nodes(ab, ana_nodes, ana_num_nodes))) return rc;

    // --- planes
    std::vector<float4> planes(plane_scene.size() * 2);
    std::vector<int32_t> plane_pos_of_scene(d->num_planes > 0 ? d->num_planes : 0, -1);
    for (size_t i = 0; i < plane_scene.size(); i++) {
        int j = plane_scene[i];
        const float* p = d->plane_point + 3 * j; const float* n = d->plane_normal + 3 * j;
        planes[2 * i] = f4(p[0], p[1], p[2], u2f((uint32_t)d->plane_material[j]));
        planes[2 * i + 1] = f4(n[0], n[1], n[2], u2f((uint32_t)j));
        if (plane_pos_of_scene[(size_t)j] < 0) plane_pos_of_scene[(size_t)j] = (int32_t)i;
    }

    // --- lights, Scene.Add order (Scene.cs:29-38): MaterialAt(new Vector()).Emittance > 0
    std::vector<pt::DevLight> lights;
    for (int i = 0; i < d->num_shapes; i++) {
        int k = d->shape_kind[i], j = d->shape_index[i];
        int mat = k == PT_SHAPE_TRIANGLE ? d->tri_material[j] : k == PT_SHAPE_MESH ? -1 : shape_mat_any(k, j, origin);
        if (mat < 0 || mat >= d->num_materials || !(d->materials[mat].emittance > 0)) continue;  // Mesh: `default`
        pt::DevLight L{};
        L.kind = k; L.mat = mat; L.phantom = 0;
        if (k == PT_SHAPE_SPHERE) {   // Sampler.cs:218-223
            L.index = ana_pos[PT_SHAPE_SPHERE][(size_t)j];
            const float* cc = d->sphere_center + 3 * j;
            L.center[0] = cc[0]; L.center[1] = cc[1]; L.center[2] = cc[2];
            L.radius = d->sphere_radius[j];
        } else if (k == PT_SHAPE_PLANE) {
            L.index = plane_pos_of_scene[(size_t)j];
            light_sphere_of_box(pt::mk(-1e9, -1e9, -1e9), pt::mk(1e9, 1e9, 1e9), L);  // Plane.BoundingBox
        } else if (k == PT_SHAPE_TRIANGLE) {  // a directly-added struct Triangle: never passes the identity test
            L.index = -1; L.phantom = 1;
            pt::v3 a = ld3(d->tri_v1 + 3 * j), b = ld3(d->tri_v2 + 3 * j), cc = ld3(d->tri_v3 + 3 * j);
            light_sphere_of_box(pt::vmin(pt::vmin(a, b), cc), pt::vmax(pt::vmax(a, b), cc), L);
        } else {   // Cube, SDFShape, Volume: class shapes; TransformedShape: a struct, never identical
            const int32_t kind = k == PT_SHAPE_CUBE ? pt::KIND_CUBE : k == PT_SHAPE_SDF ? pt::KIND_SDF
                               : k == PT_SHAPE_VOLUME ? pt::KIND_VOLUME : pt::KIND_XFORM;
            L.kind = kind;
            L.index = ana_pos[(size_t)k][(size_t)j];
            L.phantom = k == PT_SHAPE_TRANSFORMED;
            HostBox b = k == PT_SHAPE_TRANSFORMED ? xform_boxes[(size_t)j] : shape_box(k, j);   // light.BoundingBox()
            light_sphere_of_box(b.mn, b.mx, L);
        }
        lights.push_back(L);
    }

    pt::DevScene S{};
    std::memcpy(S.tri_box, tri_box, sizeof tri_box);
    {   // the traversal lines: [ana_nodes | tri_nodes | tri_chunks], 8 float4 per node / chunk
        std::vector<float4> lines;
        lines.reserve(ana_nodes.size() + tri_nodes.size() + tri_chunks.size());
        lines.insert(lines.end(), ana_nodes.begin(), ana_nodes.end());
        lines.insert(lines.end(), tri_nodes.begin(), tri_nodes.end());
        lines.insert(lines.end(), tri_chunks.begin(), tri_chunks.end());
        if (lines.size() >= 0xFFFFFFFFull) return fail(PT_ERR_UNSUPPORTED, "more than 2^29 BVH lines");   // 32-bit piece offsets
        rc = upload(c, lines, &S.lines); if (rc) return rc;
        S.lines_n = (uint32_t)(lines.size() / 8);
        S.tri_node_line0 = (uint32_t)(ana_nodes.size() / 8);
        S.tri_chunk_line0 = (uint32_t)((ana_nodes.size() + tri_nodes.size()) / 8);
        S.ana_nodes = ana_nodes.empty() ? nullptr : S.lines;
        S.tri_nodes = tri_nodes.empty() ? nullptr : S.lines + 8 * (size_t)S.tri_node_line0;
        S.tri_chunks = tri_chunks.empty() ? nullptr : S.lines + 8 * (size_t)S.tri_chunk_line0;
    }
    // one 128-B shading record per triangle (pt_scene.h tri_rstride): what k_wf_shade reads
    // for a triangle hit is one line instead of two or three
    std::vector<float4> tri_sh(nt * 8, f4(0.f, 0.f, 0.f, 0.f));
    for (size_t i = 0; i < nt; i++) {
        for (int k = 0; k < 3; k++) tri_sh[8 * i + k] = tri_recs[3 * i + k];
        for (int k = 0; k < 3; k++) tri_sh[8 * i + 3 + k] = tri_shade[3 * i + k];
        if (want_uv)
            for (int k = 0; k < 2; k++) tri_sh[8 * i + 6 + k] = tri_uv[2 * i + k];
    }
    const float4* d_tri_sh = nullptr;
    rc = upload(c, tri_sh, &d_tri_sh); if (rc) return rc;
    S.tri_recs = d_tri_sh;
    S.tri_shade = d_tri_sh ? d_tri_sh + 3 : nullptr;
    S.tri_uv = d_tri_sh && want_uv ? d_tri_sh + 6 : nullptr;
    S.tri_rstride = 8;
    S.tri_ustride = 8;
    rc = upload(c, ana_recs, &S.ana_recs); if (rc) return rc;
    rc = upload(c, planes, &S.planes); if (rc) return rc;
    rc = upload(c, mats, &S.mats); if (rc) return rc;
    rc = upload(c, lights, &S.lights); if (rc) return rc;
    const double* d_tex = nullptr;
    rc = upload(c, tex_data, &d_tex); if (rc) return rc;
    std::vector<pt::DevTexture> texs((size_t)std::max(d->num_textures, 0));
    for (int i = 0; i < d->num_textures; i++)
        texs[(size_t)i] = pt::DevTexture{d_tex + tex_off[(size_t)i], d->textures[i].width, d->textures[i].height};
    rc = upload(c, texs, &S.texs); if (rc) return rc;
    S.env_tex = d->env_texture - 1;
    S.env_angle = d->env_texture_angle;
    rc = upload(c, sdfc.prog, &S.sdf_prog); if (rc) return rc;
    rc = upload(c, sdfc.params, &S.sdf_params); if (rc) return rc;
    {   // the SDF programs, staged in LDS by the SDF queue kernels when small (pt_wavefront.hip stage_sdf)
        const size_t need = sdfc.prog.size() * sizeof(pt::DevSdfIns) + sdfc.params.size() * sizeof(double);
        S.sdf_prog_n = (int32_t)sdfc.prog.size();
        S.sdf_lds = (!sdfc.prog.empty() && need <= (size_t)PT_SDF_LDS_MAX) ? (int32_t)need : 0;
    }
    rc = upload(c, sdf_shapes, &S.sdf_shapes); if (rc) return rc;
    const double* d_vox = nullptr;
    const pt::DevWindow* d_win = nullptr;
    rc = upload(c, vox, &d_vox); if (rc) return rc;
    rc = upload(c, windows, &d_win); if (rc) return rc;
    const int8_t* d_runs = nullptr;
    rc = upload(c, vol_runs, &d_runs); if (rc) return rc;
    const double* d_cells = nullptr;
    rc = upload(c, vol_cells, &d_cells); if (rc) return rc;
    std::vector<pt::DevVolume> vols;
    for (int i = 0; i < d->num_volumes; i++) {
        vols.push_back(dev_volume(d->volumes[i], d_vox + vol_off[(size_t)i], d_win ? d_win + win_off[(size_t)i] : nullptr));
        vols.back().runs = d_runs ? d_runs + runs_off[(size_t)i] : nullptr;
        vols.back().zero_sign = zero_sign[(size_t)i];
        vols.back().cells = cells_off[(size_t)i] >= 0 ? d_cells + cells_off[(size_t)i] : nullptr;
    }
    rc = upload(c, vols, &S.volumes); if (rc) return rc;
    S.vol_lds = 0;
    const char* lds_env = std::getenv("PT_VOL_LDS");   // "0" at upload: no staging (tests)
    if (d->num_volumes == 1 && !vol_runs.empty() && !(lds_env && !std::strcmp(lds_env, "0"))) {   // k_wf_vol_* stage it in LDS (pt_wavefront.hip stage_vol)
        const size_t need = pt::kVolLdsHeader + (((size_t)d->volumes[0].num_windows * sizeof(pt::DevWindow) + 15) & ~(size_t)15) +
                            ((vol_runs.size() + 15) & ~(size_t)15);
        if (need <= (size_t)PT_VOL_LDS_MAX) S.vol_lds = (int32_t)need;
    }
    rc = upload(c, xforms, &S.xforms); if (rc) return rc;
    rc = upload(c, ext_recs, &S.ext_recs); if (rc) return rc;
    rc = upload(c, blas, &S.blas); if (rc) return rc;
    rc = upload(c, blas_nodes, &S.blas_nodes); if (rc) return rc;
    rc = upload(c, blas_recs, &S.blas_recs); if (rc) return rc;
    rc = upload(c, blas_shade, &S.blas_shade); if (rc) return rc;
    rc = upload(c, blas_uv, &S.blas_uv); if (rc) return rc;
    S.default_mat = default_mat;
    S.full_geom = (d->num_sdf_shapes > 0 || d->num_volumes > 0 || d->num_transformed > 0) ? 1 : 0;
    S.full = (d->num_textures > 0 || S.full_geom) ? 1 : 0;
    S.tri_num_nodes = tri_num_nodes;
    S.ana_num_nodes = ana_num_nodes;
    S.ana_count = (int32_t)na;
    // C4's floor cube and two light spheres: a linear test of 3 records at refill costs less than a BVH
    // node step (seven loads through the texture path) and leaf record loads per ray
    S.ana_linear = (na > 0 && na <= (size_t)PT_ANA_LINEAR && !S.full_geom) ? 1 : 0;
    S.num_sdf = d->num_sdf_shapes;
    S.num_vol = d->num_volumes;
    S.lights_lean = 1;
    for (const pt::DevLight& L : lights)
        if (!L.phantom && (L.kind == pt::KIND_SDF || L.kind == pt::KIND_VOLUME || L.kind == pt::KIND_XFORM)) S.lights_lean = 0;
    // Routed split (C5's kind of scene: the 1M-triangle mesh, a floor cube, light spheres, one SDF shape and
    // one transformed Volume): only the rays whose segment reaches a row-4 box take the FULL kernels
    // (environment PT_ROUTE=0 at upload: every ray through the FULL analytic half, as a -DPT_ROUTE=0 build;
    // tests compare the two, whose only possible difference is the exact-t tie order of DESIGN.md §5)
    const char* route_env = std::getenv("PT_ROUTE");
    const bool route_on = PT_ROUTE && !(route_env && !std::strcmp(route_env, "0"));
    S.route = (route_on && S.full_geom && S.lights_lean && na <= (size_t)PT_ANA_LINEAR && !heavy.empty() &&
               tri_num_nodes > 64) ? 1 : 0;
    S.heavy_count = (int32_t)(heavy.size() / 2);
    bool mat_tex = false;
    for (const auto& m : mats) mat_tex = mat_tex || m.tex >= 0 || m.ntex >= 0 || m.btex >= 0 || m.gtex >= 0;
    S.shade_route = (PT_SHADE_ROUTE && S.full && !mat_tex && S.lights_lean) ? 1 : 0;   // (a Volume light's colour is FULL work)
    rc = upload(c, heavy, &S.heavy); if (rc) return rc;
    S.num_planes = (int32_t)plane_scene.size();
    S.num_lights = (int32_t)lights.size();
    S.num_mats = (int32_t)mats.size();
    for (int k = 0; k < 3; k++) S.env[k] = d->env_color[k];
    PT_HIP(hipStreamSynchronize(c->stream));
    c->S = S;
    c->has_scene = true;
    c->stats.bvh_nodes = (uint64_t)tri_num_nodes + (uint64_t)ana_num_nodes;
    c->stats.traversal_bytes = (tri_nodes.size() + tri_chunks.size() + ana_nodes.size() + ana_recs.size()) * sizeof(float4);
    c->stats.bvh_bytes = (tri_nodes.size() + tri_chunks.size() + ana_nodes.size()) * sizeof(float4) +
                         (tri_sh.size() + ana_recs.size()) * sizeof(float4);
    c->stats.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return PT_OK;
}

// Passes one batch may hold: its accumulator sets (pt::kFixWords 64-bit words + 3 fp64 side sums per
// pixel and pass) within an eighth of the device's memory.  PT_BATCH_MAX_PASSES (environment, tests)
// lowers it.
static int32_t batch_passes_max(Ctx* c) {
    const size_t per_pass = (size_t)c->width * (size_t)c->height *
                            (2 * pt::kFixWords * sizeof(unsigned long long) + 3 * sizeof(double));
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || total_b == 0) total_b = (size_t)8 << 30;
    int64_t k = (int64_t)std::max<size_t>(1, (total_b / 8) / std::max<size_t>(per_pass, 1));
    if (const char* env = std::getenv("PT_BATCH_MAX_PASSES")) k = std::min<int64_t>(k, std::max(1LL, std::atoll(env)));
    return (int32_t)std::min<int64_t>(k, INT32_MAX);
}

static int render_pass_impl(Ctx* c, const pt_camera* camera, const pt_sampler* sampler, const pt_pass_params* pass,
                            pt_trace_counters* counted) {
    if (!c || !camera || !sampler || !pass) return fail(PT_ERR_INVALID_ARG, "NULL argument");
    if (!c->has_scene) return fail(PT_ERR_NO_SCENE, "pt_render_pass before pt_upload_scene");
    if (pass->spp <= 0) return fail(PT_ERR_INVALID_ARG, "spp must be >= 1");
    if (sampler->first_hit_samples <= 0 || sampler->max_bounces < 0) return fail(PT_ERR_INVALID_ARG, "bad sampler");
    if (sampler->specular_mode == PT_SPEC_ALL && sampler->max_bounces > 32)
        return fail(PT_ERR_UNSUPPORTED, "SpecularModeAll with MaxBounces > 32");
    if (sampler->light_mode < 0 || sampler->light_mode > 1 || sampler->specular_mode < 0 || sampler->specular_mode > 2)
        return fail(PT_ERR_INVALID_ARG, "bad light/specular mode");
    PT_HIP(hipSetDevice(c->device));
    const int tiles_x = (c->width + 31) / 32, tiles_y = (c->height + 31) / 32;
    int num_tiles = tiles_x * tiles_y;
    const int32_t* d_tiles = nullptr;
    if (pass->num_tiles > 0) {
        if (!pass->tiles) return fail(PT_ERR_INVALID_ARG, "tiles is NULL");
        if (pass->num_tiles > c->tiles_cap) {
            if (c->d_tiles) (void)hipFree(c->d_tiles);
            c->d_tiles = nullptr;
            c->h_tiles.clear();
            PT_HIP(hipMalloc(&c->d_tiles, (size_t)pass->num_tiles * sizeof(int32_t)));
            c->tiles_cap = pass->num_tiles;
        }
        // the same list pass after pass (a rank's tiles): uploaded once
        if (c->h_tiles.size() != (size_t)pass->num_tiles ||
            std::memcmp(c->h_tiles.data(), pass->tiles, (size_t)pass->num_tiles * sizeof(int32_t))) {
            // ids in range, none twice (a tile listed twice would be rendered into its pixels twice)
            if (int rc = pt_tile_lists_check(pass->tiles, pass->num_tiles, tiles_x * tiles_y)) return rc;
            c->h_tiles.assign(pass->tiles, pass->tiles + pass->num_tiles);
            PT_HIP(hipMemcpyAsync(c->d_tiles, c->h_tiles.data(), (size_t)pass->num_tiles * sizeof(int32_t),
                                  hipMemcpyHostToDevice, c->stream));
        }
        d_tiles = c->d_tiles;
        num_tiles = pass->num_tiles;
    }
    c->pass_tiles = pass->num_tiles > 0 ? pass->num_tiles : 0;
    pt::DevCamera cam;
    std::memcpy(cam.p, camera->p, sizeof cam.p); std::memcpy(cam.u, camera->u, sizeof cam.u);
    std::memcpy(cam.v, camera->v, sizeof cam.v); std::memcpy(cam.w, camera->w, sizeof cam.w);
    cam.m = camera->m; cam.focal_distance = camera->focal_distance; cam.aperture_radius = camera->aperture_radius;
    pt::DevSampler smp{sampler->first_hit_samples, sampler->max_bounces, sampler->direct_lighting, sampler->soft_shadows,
                       sampler->light_mode, sampler->specular_mode};
    pt::DevPass P{c->width, c->height, pass->spp, pass->stratified, pass->seed, pass->pass_index, tiles_x, d_tiles,
                  num_tiles};
    P.acc_stride = (uint32_t)((size_t)c->width * (size_t)c->height);
    pt::DevBuffer B{c->d_m, c->d_v, c->d_n, c->d_counters};
    // ---- engine choice and wavefront plan
    const int n_root = (int)std::sqrt((double)sampler->first_hit_samples);
    const int nm_root = (sampler->specular_mode != PT_SPEC_NAIVE) ? 2 : 1;
    const int nm = sampler->specular_mode == PT_SPEC_ALL ? 2 : 1;
    pt::WfPlan plan{};
    if (const char* f = std::getenv("PT_SHADE_FORM")) plan.shade_form = !std::strcmp(f, "direct") ? 1 : !std::strcmp(f, "scan") ? 2 : 0;
    plan.lanes = -1;
    if (const char* f = std::getenv("PT_LANES")) plan.lanes = !std::strcmp(f, "0") ? 0 : !std::strcmp(f, "1") ? 1 : -1;
    plan.linear = -1;
    if (const char* f = std::getenv("PT_LINEAR")) plan.linear = !std::strcmp(f, "0") ? 0 : -1;
    plan.root_children = (uint32_t)std::max(1, n_root * n_root * nm_root);
    plan.children = (uint32_t)nm;
    plan.lights_per_child = (uint32_t)(sampler->light_mode == PT_LIGHT_ALL ? std::max(1, c->S.num_lights) : 1);
    if (!c->grids.trace_blocks) PT_HIP(pt::wavefront_grids(c->grids));
    plan.trace_blocks = c->grids.trace_blocks;
    plan.shade_blocks = c->grids.shade_blocks;
    plan.shadow_blocks = c->grids.shadow_blocks;
    plan.lanes_trace_blocks = c->grids.lanes_trace_blocks;
    plan.lanes_shadow_blocks = c->grids.lanes_shadow_blocks;
    plan.full_trace_blocks = c->grids.full_trace_blocks;
    plan.full_shadow_blocks = c->grids.full_shadow_blocks;
    plan.linear_trace_blocks = c->grids.linear_trace_blocks;
    plan.linear_shadow_blocks = c->grids.linear_shadow_blocks;
    const bool extra = pass->adaptive_samples > 0 || pass->firefly_samples > 0;
    const bool serial = (pass->flags & PT_PASS_SERIAL) != 0;   // Renderer.Render's extra phases (NumCPU == 1)
    // pt_pass_params.passes: K consecutive passes.  Plain RenderParallel passes run as one batch
    // (one launch sequence over all K passes' camera samples, so a small share — one rank's tiles
    // of a multi-GPU frame — fills the GPU like a whole frame); the others pass by pass.
    const int32_t batch = pass->passes > 1 ? pass->passes : 1;
    if (batch > 1 && counted) return fail(PT_ERR_INVALID_ARG, "counted passes run one at a time (passes = 1)");
    const bool batchable = batch > 1 && !extra && !serial && !pass->stratified && pass->engine != PT_ENGINE_MEGAKERNEL &&
                           (uint64_t)P.acc_stride * (uint64_t)batch <= 0xFFFFFFFFull;
    // A batch keeps one set of per-pixel accumulators per pass (72 B per pixel): the sets of one launch
    // sequence stay within an eighth of the device's memory; a larger K runs as consecutive sub-batches,
    // each bit-identical to its passes run one by one (4K at K = 500 would ask for ~300 GB).
    const int32_t sub = batchable ? std::min(batch, batch_passes_max(c)) : 1;
    if (batchable && sub == batch) P.passes = batch;
    const uint64_t cam_samples = (uint64_t)num_tiles * 1024u * (uint64_t)(pass->stratified ? 1 : pass->spp) *
                                 (uint64_t)P.passes;
    double growth = 1.0;   // queue growth beyond depth 1 (SpecularModeAll doubles every depth)
    if (nm == 2) growth = std::ldexp(1.0, std::min(std::max(sampler->max_bounces - 1, 0), 60));
    const double per_sample = (double)plan.root_children * growth;   // extension rays per camera sample (widest depth)
    const double per_sample_nee = per_sample * (double)plan.lights_per_child;  // shadow-ray slots per camera sample
    // Queues are kParts partitions.  Camera samples are dealt to the XCD groups in
    // 256-sample blocks, so a group gets at most ceil(ceil(chunk/256)/kParts)·256 of
    // them, and everything it appends stays in its own partition.
    const double pmax = (double)(wf_max_cap(c) / pt::kParts);
    const int32_t spp_launch = pass->stratified ? 1 : pass->spp;
    auto group_max = [&](uint64_t ch) { return (double)pt::deal_group_max(ch, spp_launch); };
    uint64_t chunk = (uint64_t)std::min<double>((double)cam_samples,
                                                std::floor(pmax / per_sample_nee / 256.0) * 256.0 * pt::kParts);
    // the deal's runs can give one partition a little more than an eighth: shrink until it fits
    {
        const uint64_t step = (uint64_t)pt::deal_run(spp_launch) * 256u * pt::kParts;
        while (chunk > step && group_max(chunk) * std::max(1.0, per_sample_nee) > pmax) chunk -= step;
        while (chunk > 256 && group_max(chunk) * std::max(1.0, per_sample_nee) > pmax) chunk -= 256;
        const uint64_t tile = (uint64_t)pt::deal_run(spp_launch) * 256u;   // chunks of whole tiles where they fit
        if (chunk < cam_samples && chunk >= tile) chunk = chunk / tile * tile;
    }
    if (pass->adaptive_samples < 0 || pass->firefly_samples < 0) return fail(PT_ERR_INVALID_ARG, "negative extra samples");
    // The adaptive / firefly phases' chunks: as many of their camera samples as the queues may hold (the main
    // loop's chunk is bounded by its own samples: C5's 1-spp pass at 4K gave the 32-sample adaptive phase 32
    // chunks of 8.3M), up to PT_EXTRA_CHUNK_MAX samples, whole tiles' worth of entries.
    uint64_t chunk_extra = chunk;
    if (extra && !serial) {
        const uint64_t k = (uint64_t)std::max(pass->adaptive_samples, 1);
        const uint64_t all = (uint64_t)num_tiles * 1024u * k;
        uint64_t ce = (uint64_t)std::min<double>((double)std::min<uint64_t>(all, (uint64_t)PT_EXTRA_CHUNK_MAX),
                                                 std::floor(pmax / per_sample_nee / 256.0) * 256.0 * pt::kParts);
        const uint64_t step = (uint64_t)pt::deal_run(spp_launch) * 256u * pt::kParts;
        while (ce > step && group_max(ce) * std::max(1.0, per_sample_nee) > pmax) ce -= step;
        while (ce > 256 && group_max(ce) * std::max(1.0, per_sample_nee) > pmax) ce -= 256;
        ce = ce / (1024u * k) * (1024u * k);   // whole tiles of entries
        if (ce > chunk_extra) chunk_extra = ce;
    }
    int engine = pass->engine;
    if (engine == PT_ENGINE_AUTO)
        engine = extra || chunk >= 4096 || chunk >= cam_samples ? PT_ENGINE_WAVEFRONT : PT_ENGINE_MEGAKERNEL;
    if (engine == PT_ENGINE_MEGAKERNEL && extra)
        return fail(PT_ERR_UNSUPPORTED, "adaptive / firefly phases run on the wavefront engine");
    if (engine == PT_ENGINE_WAVEFRONT && chunk < 1)
        return fail(PT_ERR_UNSUPPORTED, "wavefront queues cannot hold one camera sample of this sampler (use the megakernel)");
    if (engine != PT_ENGINE_WAVEFRONT && engine != PT_ENGINE_MEGAKERNEL) return fail(PT_ERR_INVALID_ARG, "bad engine");
    if (batch > 1 && !(P.passes > 1 && engine == PT_ENGINE_WAVEFRONT)) {
        // not one batch: the K passes one after another (or sub-batches of `sub` passes), the stats summed
        const int32_t step = (sub > 1 && engine == PT_ENGINE_WAVEFRONT) ? sub : 1;
        pt_pass_params one = *pass;
        pt_stats sum = c->stats;
        uint64_t rays = 0, shadow = 0, handoffs = 0;
        double ms = 0.0;
        for (int32_t k = 0; k < batch; k += step) {
            one.pass_index = pass->pass_index + (uint32_t)k;
            one.passes = std::min(step, batch - k);
            if (int rc = render_pass_impl(c, camera, sampler, &one, nullptr)) return rc;
            rays += c->stats.rays;
            shadow += c->stats.shadow_rays;
            handoffs += c->stats.tail_handoffs;
            ms += c->stats.last_pass_ms;
            for (int j = 0; j < PT_K_SLOTS; j++) {
                sum.kernel_ms[j] = (k ? sum.kernel_ms[j] : 0.0) + c->stats.kernel_ms[j];
                sum.kernel_launches[j] = (k ? sum.kernel_launches[j] : 0) + c->stats.kernel_launches[j];
            }
        }
        std::memcpy(c->stats.kernel_ms, sum.kernel_ms, sizeof sum.kernel_ms);
        std::memcpy(c->stats.kernel_launches, sum.kernel_launches, sizeof sum.kernel_launches);
        c->stats.rays = rays;
        c->stats.shadow_rays = shadow;
        c->stats.tail_handoffs = handoffs;
        c->stats.last_pass_ms = ms;
        return PT_OK;
    }
    if (engine == PT_ENGINE_WAVEFRONT) {
        plan.chunk = chunk;
        plan.chunk_extra = chunk_extra;
        // Shadow passes on the side stream, beside the next depth's closest-hit pass, when a
        // chunk's widest depth is small enough for the launches' fill and drain to matter (one
        // rank's 1/8 share of C4 passed one at a time, 33M rays: +6.5 %); a full C4 frame (265M)
        // runs 0.3 % slower that way and C2's 16-child chunks (268M) 6.2 % slower (10632 vs 11332
        // Mrays/s, profiles/r03c_c2_*.json): they keep one stream.  The bound is on rays, not
        // camera samples (round 2 used 20M camera samples, which sent C2 to the side stream).
        // PT_SIDE_STREAM=0|1 (environment; tests) forces one stream or the side stream.
        bool side = (double)chunk * per_sample <= kSideStreamMaxRays;
        if (const char* f = std::getenv("PT_SIDE_STREAM")) side = !std::strcmp(f, "1") ? true : !std::strcmp(f, "0") ? false : side;
        if (side) {
            plan.side = c->side;
            plan.ev_main = c->ev_main;
            plan.ev_side[0] = c->ev_side[0];
            plan.ev_side[1] = c->ev_side[1];
        }
        const double group_samples = group_max(chunk_extra);   // (>= chunk's)
        const double need = group_samples * per_sample;   // a partition's widest depth
        const uint32_t pcap = (uint32_t)std::min(pmax, std::max(8192.0, std::max(group_samples, need)));
        const uint32_t spcap = (uint32_t)std::min(pmax, std::max(8192.0, group_samples * per_sample_nee));
        uint32_t cap = pcap * pt::kParts, scap = spcap * pt::kParts;
        int rc = ensure_wavefront(c, cap, scap, P.passes, side);
        if (rc) return rc;
        if ((uint64_t)pass->adaptive_samples > chunk)
            return fail(PT_ERR_UNSUPPORTED, "adaptive samples exceed one wavefront chunk");
        if (serial && (uint64_t)pass->firefly_samples > chunk)
            return fail(PT_ERR_UNSUPPORTED, "firefly samples exceed one wavefront chunk");
        if (extra && (rc = ensure_extra(c, chunk_extra))) return rc;
    }
    c->last_engine = engine;
    if (c->gathered || (c->loaded && c->comm)) {
        c->gathered = false;
        c->loaded = false;
        if (pass->num_tiles > 0) {
            const int ntiles = tiles_x * tiles_y;
            std::vector<uint8_t> own((size_t)ntiles, 0);
            for (int i = 0; i < pass->num_tiles; i++) own[(size_t)pass->tiles[i]] = 1;
            if (!c->d_own) PT_HIP(hipMalloc(&c->d_own, (size_t)ntiles));
            PT_HIP(hipMemcpyAsync(c->d_own, own.data(), (size_t)ntiles, hipMemcpyHostToDevice, c->stream));
            hipLaunchKernelGGL(pt::k_clear_foreign, dim3(2048), dim3(256), 0, c->stream, B, c->width, c->height, tiles_x,
                               (const uint8_t*)c->d_own);
            PT_HIP(hipGetLastError());
            PT_HIP(hipStreamSynchronize(c->stream));   // `own` is a host temporary
        }
    }
    const bool timing = (pass->flags & PT_PASS_KERNEL_TIMING) != 0;
    c->timer.reset(c->stream);
    PT_HIP(hipMemsetAsync(c->d_counters, 0, (counted ? pt::kCounterAllocWords : pt::kCounterWords) * sizeof(unsigned long long),
                          c->stream));   // and the overflow flag; a counted pass' march clock slots too
    // a counted pass also counts the Volume / SDFShape march steps (counters 9, 10); the launches
    // take the scene by value, so the pointer is cleared again whichever way this call returns
    struct MarchScope {
        pt::DevScene& S;
        ~MarchScope() { S.march = nullptr; }
    } march_scope{c->S};
    c->S.march = counted ? c->d_counters + 9 : nullptr;
    PT_HIP(hipEventRecord(c->ev0, c->stream));
    if (engine == PT_ENGINE_WAVEFRONT) {
        pt::LaunchTimer* tm = timing ? &c->timer : nullptr;
        // PT_SHADOW_TAIL=early (environment; tests): k_wf_shadow_lanes hands stack entries to idle lanes from
        // the first claim on, so the tail protocol runs all pass long (pt_stats.tail_handoffs counts it)
        const char* tail_env = std::getenv("PT_SHADOW_TAIL");
        c->Q.tail_early = (tail_env && !std::strcmp(tail_env, "early")) ? 1 : 0;
        PT_HIP(pt::wavefront_pass(c->S, cam, smp, P, B, c->Q, plan, counted != nullptr, c->stream, tm));
        if (serial) {
            // Renderer.Render (Renderer.cs:80-198): after a pixel's main samples, AdaptiveSamples
            // individual samples if its σmax ≥ 1 (:153-175), then FireflySamples individual samples
            // if its σmax then exceeds 1 (:177-191).  Each decision reads the pixel's own Buffer
            // only, so the phases run over all pixels, one after the other.
            const int32_t K[2] = {pass->adaptive_samples, pass->firefly_samples};
            const uint32_t base[2] = {pt::kAdaptiveSampleBase, pt::kFireflySampleBase};
            for (int ph = 0; ph < 2; ph++) {
                if (K[ph] <= 0) continue;
                PT_HIP(pt::select_pixels(P, B, ph == 0 ? 1 : 0, c->d_plist, c->d_fcount, c->stream));
                uint32_t nsel = 0;
                PT_HIP(hipMemcpyAsync(&nsel, c->d_fcount, sizeof nsel, hipMemcpyDeviceToHost, c->stream));
                PT_HIP(hipStreamSynchronize(c->stream));
                PT_HIP(pt::wavefront_extra(c->S, cam, smp, P, B, c->Q, plan, counted != nullptr, c->stream, tm,
                                           ph == 0 ? pt::EXTRA_ADD : pt::EXTRA_ADD_SCALED, K[ph], base[ph], nsel,
                                           c->d_plist, nullptr, nullptr, nullptr));
            }
        }
        if (!serial && pass->adaptive_samples > 0)  // Renderer.cs:340-410
            PT_HIP(pt::wavefront_extra(c->S, cam, smp, P, B, c->Q, plan, counted != nullptr, c->stream, tm, 0,
                                       pass->adaptive_samples, pt::kAdaptiveSampleBase, (uint64_t)num_tiles * 1024u,
                                       nullptr, nullptr, nullptr, nullptr));
        if (!serial && pass->firefly_samples > 0) {  // Renderer.cs:412-470
            PT_HIP(pt::select_pixels(P, B, 0, c->d_plist, c->d_fcount, c->stream));
            uint32_t nsel = 0;
            PT_HIP(hipMemcpyAsync(&nsel, c->d_fcount, sizeof nsel, hipMemcpyDeviceToHost, c->stream));
            const size_t npx = (size_t)c->width * (size_t)c->height;
            PT_HIP(hipMemcpyAsync(c->d_snap, c->d_m, npx * 3 * sizeof(double), hipMemcpyDeviceToDevice, c->stream));
            if (c->comm) {
                // neighbours on other ranks' tiles: the disjoint M buffers sum to the full frame
                ncclResult_t r = ncclAllReduce(c->d_snap, c->d_snap, npx * 3, ncclFloat64, ncclSum, c->comm, c->stream);
                if (r != ncclSuccess) return fail(PT_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
            }
            PT_HIP(hipStreamSynchronize(c->stream));
            // Renderer.cs:430-445 traces a candidate's samples one after another and stops at the first
            // IsFirefly sample: rounds of one sample per still-active pixel, so exactly those samples are
            // traced (and counted in Scene.rays), no more.
            uint32_t* list = c->d_plist;
            uint32_t* next = c->d_plist2;
            for (int j = 0; j < pass->firefly_samples && nsel > 0; j++) {
                PT_HIP(hipMemsetAsync(c->d_fcount + 1, 0, sizeof(uint32_t), c->stream));
                PT_HIP(pt::wavefront_extra(c->S, cam, smp, P, B, c->Q, plan, counted != nullptr, c->stream, tm,
                                           pt::EXTRA_FIREFLY_STOP, 1,
                                           pt::kFireflySampleBase + (uint32_t)j, nsel, list, c->d_snap, next,
                                           c->d_fcount + 1));
                PT_HIP(hipMemcpyAsync(&nsel, c->d_fcount + 1, sizeof nsel, hipMemcpyDeviceToHost, c->stream));
                PT_HIP(hipStreamSynchronize(c->stream));
                std::swap(list, next);
            }
        }
    } else {
        if (timing) c->timer.begin(PT_K_MEGAKERNEL, c->stream);
        PT_HIP(pt::launch_render_pass(c->S, cam, smp, P, B, num_tiles, counted != nullptr, c->stream));
        if (timing) c->timer.end(PT_K_MEGAKERNEL, c->stream);
    }
    PT_HIP(hipEventRecord(c->ev1, c->stream));
    if (c->timer.failed) return fail(PT_ERR_HIP, "hipEventRecord (kernel timing) failed");
    const unsigned long long* ctr = c->h_counters;
    PT_HIP(hipMemcpyAsync(c->h_counters, c->d_counters, (counted ? pt::kCounterAllocWords : pt::kCounterWords) * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost, c->stream));
    PT_HIP(hipStreamSynchronize(c->stream));
    if (engine == PT_ENGINE_WAVEFRONT && ctr[pt::kOverflowCounter])
        return fail(PT_ERR_OUT_OF_MEMORY, "wavefront queue overflow (pass results are incomplete)");
    float ms = 0.f;
    PT_HIP(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    // counters: [0..2] closest-hit rays/nodes/prims, [3] shading fetches, [4..6] shadow rays/nodes/prims
    const uint64_t rays = ctr[0] + ctr[4];
    c->stats.rays = rays;
    c->stats.shadow_rays = ctr[4];
    c->stats.tail_handoffs = engine == PT_ENGINE_WAVEFRONT ? ctr[11] : 0;
    c->stats.rays_total += rays;
    c->stats.last_pass_ms = ms;
    c->stats.total_ms += ms;
    c->stats.passes += (uint64_t)P.passes;
    for (int k = 0; k < PT_K_SLOTS; k++) { c->stats.kernel_ms[k] = 0.0; c->stats.kernel_launches[k] = 0; }
    if (timing) PT_HIP(c->timer.collect(c->stats.kernel_ms, c->stats.kernel_launches));
    if (counted) {
        counted->rays = rays;
        counted->nodes_visited = ctr[1] + ctr[5];
        counted->prims_tested = ctr[2] + ctr[6];
        counted->shading_fetches = ctr[3];
        counted->shadow_rays = ctr[4];
        counted->shadow_nodes = ctr[5];
        counted->shadow_prims = ctr[6];
        counted->lit_shadow_rays = ctr[7];
        counted->accum_runs = ctr[8];
        counted->volume_samples = ctr[9];
        counted->sdf_evals = ctr[10];
        for (int k = 0; k < 8; k++) {
            counted->march_clock[k] = 0;
            for (int j = 0; j < pt::kMarchSlots; j++) counted->march_clock[k] += ctr[pt::kMarchClockWord + 8 * j + k];
        }
    }
    return PT_OK;
}

int pt_render_pass(void* ctx, const pt_camera* camera, const pt_sampler* sampler, const pt_pass_params* pass) {
    return render_pass_impl((Ctx*)ctx, camera, sampler, pass, nullptr);
}

int pt_render_pass_counted(void* ctx, const pt_camera* camera, const pt_sampler* sampler, const pt_pass_params* pass,
                           pt_trace_counters* out) {
    if (!out) return fail(PT_ERR_INVALID_ARG, "out is NULL");
    return render_pass_impl((Ctx*)ctx, camera, sampler, pass, out);
}

int pt_synchronize(void* ctx) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    PT_HIP(hipSetDevice(c->device));
    PT_HIP(hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_read_buffer(void* ctx, double* out_m, double* out_v, int32_t* out_n) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    PT_HIP(hipSetDevice(c->device));
    size_t P = (size_t)c->width * (size_t)c->height;
    if (out_m) PT_HIP(hipMemcpyAsync(out_m, c->d_m, P * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (out_v) PT_HIP(hipMemcpyAsync(out_v, c->d_v, P * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    if (out_n) PT_HIP(hipMemcpyAsync(out_n, c->d_n, P * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    PT_HIP(hipStreamSynchronize(c->stream));
    return PT_OK;
}

int pt_write_buffer(void* ctx, const double* m, const double* v, const int32_t* n) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    PT_HIP(hipSetDevice(c->device));
    size_t P = (size_t)c->width * (size_t)c->height;
    if (m) PT_HIP(hipMemcpyAsync(c->d_m, m, P * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (v) PT_HIP(hipMemcpyAsync(c->d_v, v, P * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
    if (n) PT_HIP(hipMemcpyAsync(c->d_n, n, P * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    PT_HIP(hipStreamSynchronize(c->stream));
    // The loaded Buffer may hold other ranks' pixels (every rank loads the whole checkpoint): on a
    // context that is part of a communicator the next tile-subset pass clears them first, as after a
    // gather, so a firefly snapshot's all-reduce and a later gather see each pixel on its owner only.
    // A lone context keeps them (a host resuming a frame and then rendering it tile subset by tile
    // subset keeps every restored pixel).
    c->loaded = true;
    return PT_OK;
}

static int tile_workspace(Ctx* c);

// Host copies of a tile list's packed {M, V, N} (see k_tiles_pack for the order).
static int tiles_io(void* ctx, const int32_t* tiles, int32_t num_tiles, double* m, double* v, int32_t* n, bool write) {
    Ctx* c = (Ctx*)ctx;
    if (!c || (num_tiles > 0 && (!tiles || !m || !v || !n))) return fail(PT_ERR_INVALID_ARG, "NULL argument");
    if (num_tiles < 0) return fail(PT_ERR_INVALID_ARG, "num_tiles < 0");
    const int32_t all = ((c->width + 31) / 32) * ((c->height + 31) / 32);
    if (num_tiles > all) return fail(PT_ERR_INVALID_ARG, "more tiles than the image has");
    for (int32_t i = 0; i < num_tiles; i++)
        if (tiles[i] < 0 || tiles[i] >= all) return fail(PT_ERR_INVALID_ARG, "tile id out of range");
    if (num_tiles == 0) return PT_OK;
    PT_HIP(hipSetDevice(c->device));
    int rc = tile_workspace(c);
    if (rc) return rc;
    const size_t s = (size_t)num_tiles * 1024u;
    PT_HIP(hipMemcpyAsync(c->g_ids, tiles, (size_t)num_tiles * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
    if (write) {
        PT_HIP(hipMemcpyAsync(c->g_m, m, s * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
        PT_HIP(hipMemcpyAsync(c->g_v, v, s * 3 * sizeof(double), hipMemcpyHostToDevice, c->stream));
        PT_HIP(hipMemcpyAsync(c->g_n, n, s * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
        c->gathered = true;   // foreign tiles written (a host-transport gather): cleared before the next subset pass
    }
    pt::DevBuffer B{c->d_m, c->d_v, c->d_n, c->d_counters};
    hipLaunchKernelGGL(pt::k_tiles_pack, dim3(2048), dim3(256), 0, c->stream, B, c->width, c->height,
                       (c->width + 31) / 32, c->g_ids, (uint32_t)num_tiles, c->g_m, c->g_v, c->g_n, write ? 1 : 0);
    PT_HIP(hipGetLastError());
    if (!write) {
        PT_HIP(hipMemcpyAsync(m, c->g_m, s * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        PT_HIP(hipMemcpyAsync(v, c->g_v, s * 3 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        PT_HIP(hipMemcpyAsync(n, c->g_n, s * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    }
    PT_HIP(hipStreamSynchronize(c->stream));
    return PT_OK;
}
int pt_read_tiles(void* ctx, const int32_t* tiles, int32_t num_tiles, double* out_m, double* out_v, int32_t* out_n) {
    return tiles_io(ctx, tiles, num_tiles, out_m, out_v, out_n, false);
}
int pt_write_tiles(void* ctx, const int32_t* tiles, int32_t num_tiles, const double* m, const double* v,
                   const int32_t* n) {
    return tiles_io(ctx, tiles, num_tiles, const_cast<double*>(m), const_cast<double*>(v), const_cast<int32_t*>(n), true);
}

// pt_intersect / pt_occluded: the rays to the device, one launch of k_intersect, the answers back.
static int ray_queries(void* ctx, int64_t n, const float* origins, const float* dirs, const double* t_light,
                       int32_t flags, double* out_t, int32_t* out_i) {
    Ctx* c = (Ctx*)ctx;
    if (!c || (n > 0 && (!origins || !dirs || !out_i || (!t_light && !out_t)))) return fail(PT_ERR_INVALID_ARG, "NULL argument");
    if (n < 0 || n > (int64_t)1 << 30) return fail(PT_ERR_INVALID_ARG, "n out of range [0, 2^30]");
    if (flags & ~(PT_MARCH_LANE | PT_MARCH_WAVE) || (flags & PT_MARCH_LANE && flags & PT_MARCH_WAVE))
        return fail(PT_ERR_INVALID_ARG, "flags: PT_MARCH_LANE or PT_MARCH_WAVE, not both");
    if (!c->has_scene) return fail(PT_ERR_NO_SCENE, "no scene uploaded");
    if (n == 0) return PT_OK;
    PT_HIP(hipSetDevice(c->device));
    const size_t N = (size_t)n;
    const size_t bytes = N * (6 * sizeof(float) + sizeof(double) + sizeof(double) + sizeof(int32_t));
    unsigned char* d = nullptr;
    hipError_t e = hipMalloc(&d, bytes);
    if (e != hipSuccess) return fail(PT_ERR_OUT_OF_MEMORY, std::string("hipMalloc ray queries: ") + hipGetErrorString(e));
    float* d_o = (float*)d;
    float* d_d = d_o + 3 * N;
    double* d_tl = (double*)(d_d + 3 * N);   // 8-B aligned: 24·N bytes precede it
    double* d_t = d_tl + N;
    int32_t* d_i = (int32_t*)(d_t + N);
    pt::DevScene S = c->S;
    if (flags & PT_MARCH_LANE) S.coop_min_lanes = 65;   // fewer than 65 active lanes: always
    if (flags & PT_MARCH_WAVE) S.coop_min_lanes = 1;    // every wave with a pending Volume marches it together
    int rc = PT_OK;
    auto step = [&](hipError_t err, const char* what) {
        if (rc == PT_OK && err != hipSuccess) rc = fail(PT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(err));
    };
    step(hipMemcpyAsync(d_o, origins, 3 * N * sizeof(float), hipMemcpyHostToDevice, c->stream), "origins");
    step(hipMemcpyAsync(d_d, dirs, 3 * N * sizeof(float), hipMemcpyHostToDevice, c->stream), "dirs");
    if (t_light) step(hipMemcpyAsync(d_tl, t_light, N * sizeof(double), hipMemcpyHostToDevice, c->stream), "t_light");
    if (rc == PT_OK) step(pt::launch_intersect(S, (uint32_t)N, d_o, d_d, t_light ? d_tl : nullptr, d_t, d_i, c->stream), "k_intersect");
    if (rc == PT_OK && out_t && !t_light) step(hipMemcpyAsync(out_t, d_t, N * sizeof(double), hipMemcpyDeviceToHost, c->stream), "out_t");
    if (rc == PT_OK) step(hipMemcpyAsync(out_i, d_i, N * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream), "out");
    step(hipStreamSynchronize(c->stream), "hipStreamSynchronize");
    (void)hipFree(d);
    return rc;
}
int pt_intersect(void* ctx, int64_t n, const float* origins, const float* dirs, int32_t flags, double* out_t,
                 int32_t* out_kind) {
    if (!out_t) return fail(PT_ERR_INVALID_ARG, "out_t is NULL");
    return ray_queries(ctx, n, origins, dirs, nullptr, flags, out_t, out_kind);
}
int pt_occluded(void* ctx, int64_t n, const float* origins, const float* dirs, const double* t_max, int32_t flags,
                int32_t* out_blocked) {
    if (n > 0 && !t_max) return fail(PT_ERR_INVALID_ARG, "t_max is NULL");
    return ray_queries(ctx, n, origins, dirs, t_max, flags, nullptr, out_blocked);
}

int pt_scene_bvh_digest(const pt_scene_desc* d, uint64_t out[4]) {
    if (!out) return fail(PT_ERR_INVALID_ARG, "out is NULL");
    const int rc = validate_scene(d);
    if (rc != PT_OK) return rc;
    std::vector<int32_t> tri_src;
    for (int i = 0; i < d->num_shapes; i++) {   // pt_upload_scene's triangle order
        const int k = d->shape_kind[i], j = d->shape_index[i];
        if (k == PT_SHAPE_TRIANGLE) tri_src.push_back(j);
        else if (k == PT_SHAPE_MESH) for (int t = 0; t < d->mesh_count[j]; t++) tri_src.push_back(d->mesh_first[j] + t);
    }
    const std::shared_ptr<const TriBvhBuild> b = tri_bvh_shared(d, tri_src);
    if (b->rc != PT_OK) return fail(b->rc, b->err);
    uint64_t h = 0xCBF29CE484222325ull;
    auto eat = [&](const void* p, size_t n) {
        const unsigned char* q = (const unsigned char*)p;
        for (size_t i = 0; i < n; i++) h = (h ^ q[i]) * 0x100000001B3ull;
    };
    eat(b->order.data(), b->order.size() * sizeof(uint32_t));
    eat(b->nodes.data(), b->nodes.size() * sizeof(float4));
    eat(b->chunks.data(), b->chunks.size() * sizeof(float4));
    out[0] = h;
    out[1] = (uint64_t)(b->nodes.size() + b->chunks.size()) * sizeof(float4);
    TriBvhCache& C = tri_bvh_cache();
    std::lock_guard<std::mutex> lk(C.mu);
    out[2] = (uint64_t)C.builds;
    out[3] = (uint64_t)C.hits;
    return PT_OK;
}

int pt_stats_get(void* ctx, pt_stats* out) {
    Ctx* c = (Ctx*)ctx;
    if (!c || !out) return fail(PT_ERR_INVALID_ARG, "NULL argument");
    *out = c->stats;
    return PT_OK;
}

void pt_destroy(void* ctx) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    tri_bvh_release(c);
    free_scene(c);
    free_wavefront(c);
    if (c->d_m) (void)hipFree(c->d_m);
    if (c->d_v) (void)hipFree(c->d_v);
    if (c->d_n) (void)hipFree(c->d_n);
    if (c->d_counters) (void)hipFree(c->d_counters);
    if (c->h_counters) (void)hipHostFree(c->h_counters);
    if (c->d_tiles) (void)hipFree(c->d_tiles);
    if (c->d_own) (void)hipFree(c->d_own);
    for (void* p : {(void*)c->g_ids, (void*)c->g_m, (void*)c->g_v, (void*)c->g_n, (void*)c->g_cnts, (void*)c->g_all})
        if (p) (void)hipFree(p);
    c->timer.destroy();
    if (c->ev_main) (void)hipEventDestroy(c->ev_main);
    for (hipEvent_t e : c->ev_side) if (e) (void)hipEventDestroy(e);
    if (c->side) (void)hipStreamDestroy(c->side);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

// ------------------------------------------------------------------ RCCL
int pt_comm_unique_id(uint8_t out_id[128]) {
    if (!out_id) return fail(PT_ERR_INVALID_ARG, "out_id is NULL");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return fail(PT_ERR_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::memcpy(out_id, &id, 128);
    return PT_OK;
}

int pt_comm_init(void* ctx, int32_t nranks, int32_t rank, const uint8_t id[128]) {
    Ctx* c = (Ctx*)ctx;
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(PT_ERR_INVALID_ARG, "bad comm arguments");
    PT_HIP(hipSetDevice(c->device));
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    ncclUniqueId uid;
    std::memcpy(&uid, id, 128);
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) return fail(PT_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    c->nranks = nranks;
    c->rank = rank;
    return PT_OK;
}

// ---- the gather's host-side arithmetic (pure functions, exported: hosts and CPU tests check them)
// Where each rank's packed tiles land in the root's receive buffers: rank p (not the root, with
// tiles) at tile offset out_offsets[p] (entries × 1024 pixels; M/V × 3072 doubles), in rank order;
// −1 for the root and for ranks with no tiles.  The counts are one pass' tile lists, which the
// ranks keep disjoint, so they cannot sum past the image's tiles.
int pt_gather_layout(int32_t nranks, int32_t root, const int32_t* counts, int32_t image_tiles,
                     int64_t* out_offsets, int64_t* out_total) {
    if (nranks < 1 || !counts || !out_offsets || !out_total || image_tiles < 0)
        return fail(PT_ERR_INVALID_ARG, "gather layout: bad arguments");
    if (root < 0 || root >= nranks) return fail(PT_ERR_INVALID_ARG, "gather layout: root out of range");
    int64_t sum = 0;
    for (int32_t p = 0; p < nranks; p++) {
        if (counts[p] < 0 || counts[p] > image_tiles)
            return fail(PT_ERR_INVALID_ARG, "gather layout: rank " + std::to_string(p) + " reports " +
                                                std::to_string(counts[p]) + " tiles of " + std::to_string(image_tiles));
        sum += counts[p];
    }
    if (sum > image_tiles)   // disjoint lists never hold more tiles than the image
        return fail(PT_ERR_INVALID_ARG, "gather: the ranks' tile lists overlap (more tiles than the image has)");
    int64_t off = 0;
    for (int32_t p = 0; p < nranks; p++) {
        if (p == root || counts[p] == 0) { out_offsets[p] = -1; continue; }
        out_offsets[p] = off;
        off += counts[p];
    }
    *out_total = off;
    return PT_OK;
}

// Every id in [0, image_tiles) and none twice (a tile on two ranks would be written twice, the
// last sender's copy replacing the others).
int pt_tile_lists_check(const int32_t* ids, int64_t n, int32_t image_tiles) {
    if (n < 0 || (n > 0 && !ids) || image_tiles < 0) return fail(PT_ERR_INVALID_ARG, "tile list: bad arguments");
    std::vector<uint8_t> seen((size_t)image_tiles, 0);
    for (int64_t i = 0; i < n; i++) {
        const int32_t t = ids[i];
        if (t < 0 || t >= image_tiles)
            return fail(PT_ERR_INVALID_ARG, "tile id " + std::to_string(t) + " out of range [0, " +
                                                std::to_string(image_tiles) + ")");
        if (seen[(size_t)t]) return fail(PT_ERR_INVALID_ARG, "tile " + std::to_string(t) + " listed twice");
        seen[(size_t)t] = 1;
    }
    return PT_OK;
}

// Every rank rendered a disjoint tile set into a zero-initialised full-frame
// buffer, so a sum-reduce onto `root` is the gather.
// Tile-compacted gather: every rank but the root packs the {M, V, N} of its
// tiles (the last pass' list) and sends them with the tile ids; the root writes them into
// its Buffer.  The ranks' tiles are disjoint, so this equals a sum-reduce of the full frames
// at ≈1/N of their bytes per rank (1080p, 8 ranks: 13.6 MB instead of 108 MB).  Two steps:
// the tile counts (one all-gather), then the grouped sends and receives.
static int tile_workspace(Ctx* c) {
    const int32_t tiles = ((c->width + 31) / 32) * ((c->height + 31) / 32);
    const size_t slots = (size_t)tiles * 1024u;
    if (!c->g_ids) {
        PT_HIP(hipMalloc(&c->g_ids, (size_t)tiles * sizeof(int32_t)));
        PT_HIP(hipMalloc(&c->g_m, slots * 3 * sizeof(double)));
        PT_HIP(hipMalloc(&c->g_v, slots * 3 * sizeof(double)));
        PT_HIP(hipMalloc(&c->g_n, slots * sizeof(int32_t)));
        PT_HIP(hipMalloc(&c->g_all, (size_t)tiles * sizeof(int32_t)));
        hipLaunchKernelGGL(pt::k_iota, dim3(64), dim3(256), 0, c->stream, c->g_all, tiles);
        PT_HIP(hipGetLastError());
    }
    return PT_OK;
}
static int gather_prepare(Ctx* c) {
    const int32_t tiles = ((c->width + 31) / 32) * ((c->height + 31) / 32);
    int rc = tile_workspace(c);
    if (rc) return rc;
    if (!c->g_cnts) PT_HIP(hipMalloc(&c->g_cnts, (size_t)(c->nranks + 1) * sizeof(int32_t)));
    const int32_t mine = c->pass_tiles > 0 ? c->pass_tiles : tiles;
    PT_HIP(hipMemcpyAsync(c->g_cnts + c->nranks, &mine, sizeof mine, hipMemcpyHostToDevice, c->stream));
    PT_HIP(hipStreamSynchronize(c->stream));   // `mine` is a host temporary
    return PT_OK;
}
static const int32_t* own_ids(Ctx* c) { return c->pass_tiles > 0 ? c->d_tiles : c->g_all; }
static int32_t own_count(Ctx* c) {
    return c->pass_tiles > 0 ? c->pass_tiles : ((c->width + 31) / 32) * ((c->height + 31) / 32);
}
// The rank's sends (not root) or receives (root) of step 2; inside a group.  Non-root ranks
// pack first (same stream, so the sends follow the packing).
static ncclResult_t gather_issue(Ctx* c, int32_t root, const std::vector<int32_t>& cnts,
                                 const std::vector<int64_t>& offs) {
    const int tiles_x = (c->width + 31) / 32;
    if (c->rank != root) {
        const int32_t nt = own_count(c);
        if (nt == 0) return ncclSuccess;
        pt::DevBuffer B{c->d_m, c->d_v, c->d_n, c->d_counters};
        hipLaunchKernelGGL(pt::k_tiles_pack, dim3(2048), dim3(256), 0, c->stream, B, c->width, c->height, tiles_x,
                           own_ids(c), (uint32_t)nt, c->g_m, c->g_v, c->g_n, 0);
        if (hipGetLastError() != hipSuccess) return ncclUnhandledCudaError;
        const size_t s = (size_t)nt * 1024u;
        ncclResult_t r = ncclSend(own_ids(c), (size_t)nt, ncclInt32, root, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclSend(c->g_m, s * 3, ncclFloat64, root, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclSend(c->g_v, s * 3, ncclFloat64, root, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclSend(c->g_n, s, ncclInt32, root, c->comm, c->stream);
        return r;
    }
    for (int p = 0; p < c->nranks; p++) {
        if (offs[(size_t)p] < 0) continue;   // the root, or a rank without tiles (pt_gather_layout)
        const size_t off = (size_t)offs[(size_t)p], nt = (size_t)cnts[(size_t)p], s = nt * 1024u;
        ncclResult_t r = ncclRecv(c->g_ids + off, nt, ncclInt32, p, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->g_m + off * 3072u, s * 3, ncclFloat64, p, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->g_v + off * 3072u, s * 3, ncclFloat64, p, c->comm, c->stream);
        if (r == ncclSuccess) r = ncclRecv(c->g_n + off * 1024u, s, ncclInt32, p, c->comm, c->stream);
        if (r != ncclSuccess) return r;
    }
    return ncclSuccess;
}
// The root checks the received tile ids against each other and its own list (a duplicate means
// two ranks rendered one tile: refused before anything is written), then writes them into its Buffer.
static int gather_finish(Ctx* c, int32_t root, int64_t total) {
    if (c->rank == root) {
        if (total > 0) {
            std::vector<int32_t> ids((size_t)total);
            PT_HIP(hipMemcpyAsync(ids.data(), c->g_ids, (size_t)total * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
            PT_HIP(hipStreamSynchronize(c->stream));
            const int32_t image = ((c->width + 31) / 32) * ((c->height + 31) / 32);
            if (c->pass_tiles > 0) ids.insert(ids.end(), c->h_tiles.begin(), c->h_tiles.end());
            else for (int32_t t = 0; t < image; t++) ids.push_back(t);   // the root rendered the whole image
            if (pt_tile_lists_check(ids.data(), (int64_t)ids.size(), image))
                return fail(PT_ERR_INVALID_ARG, std::string("gather: the ranks' tile lists overlap (") + g_last_error + ")");
            pt::DevBuffer B{c->d_m, c->d_v, c->d_n, c->d_counters};
            hipLaunchKernelGGL(pt::k_tiles_pack, dim3(2048), dim3(256), 0, c->stream, B, c->width, c->height,
                               (c->width + 31) / 32, c->g_ids, (uint32_t)total, c->g_m, c->g_v, c->g_n, 1);
            PT_HIP(hipGetLastError());
        }
        c->gathered = true;
    }
    PT_HIP(hipStreamSynchronize(c->stream));
    return PT_OK;
}
static int gather_counts(Ctx* c, int32_t root, std::vector<int32_t>& cnts, std::vector<int64_t>& offs, int64_t& total) {
    cnts.assign((size_t)c->nranks, 0);
    offs.assign((size_t)c->nranks, -1);
    PT_HIP(hipMemcpy(cnts.data(), c->g_cnts, (size_t)c->nranks * sizeof(int32_t), hipMemcpyDeviceToHost));
    const int32_t tiles = ((c->width + 31) / 32) * ((c->height + 31) / 32);
    return pt_gather_layout(c->nranks, root, cnts.data(), tiles, offs.data(), &total);
}

int pt_comm_gather(void* ctx, int32_t root) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    if (!c->comm) return fail(PT_ERR_RCCL, "pt_comm_init not called");
    if (root < 0 || root >= c->nranks) return fail(PT_ERR_INVALID_ARG, "root out of range");
    PT_HIP(hipSetDevice(c->device));
    int rc = gather_prepare(c);
    if (rc) return rc;
    ncclResult_t r = ncclAllGather(c->g_cnts + c->nranks, c->g_cnts, 1, ncclInt32, c->comm, c->stream);
    if (r != ncclSuccess) return fail(PT_ERR_RCCL, std::string("ncclAllGather: ") + ncclGetErrorString(r));
    PT_HIP(hipStreamSynchronize(c->stream));
    std::vector<int32_t> cnts;
    std::vector<int64_t> offs;
    int64_t total = 0;
    if ((rc = gather_counts(c, root, cnts, offs, total))) return rc;   // every rank sees the same counts
    r = ncclGroupStart();
    if (r == ncclSuccess) r = gather_issue(c, root, cnts, offs);
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return fail(PT_ERR_RCCL, std::string("gather send/recv: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    return gather_finish(c, root, total);
}

// One communicator over G contexts of this process (one per device), formed by one call:
// the single-process multi-GPU form a .NET host uses.
int pt_comm_init_all(void* const* ctxs, int32_t n) {
    if (!ctxs || n < 1) return fail(PT_ERR_INVALID_ARG, "bad context list");
    std::vector<int> devs((size_t)n);
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        if (!c) return fail(PT_ERR_INVALID_ARG, "NULL context in the list");
        for (int j = 0; j < i; j++)
            if (((Ctx*)ctxs[j])->device == c->device) return fail(PT_ERR_INVALID_ARG, "two contexts on one device");
        devs[(size_t)i] = c->device;
    }
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    }
    std::vector<ncclComm_t> comms((size_t)n, nullptr);
    ncclResult_t r = ncclCommInitAll(comms.data(), n, devs.data());
    if (r != ncclSuccess) return fail(PT_ERR_RCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        c->comm = comms[(size_t)i];
        c->nranks = n;
        c->rank = i;
    }
    return PT_OK;
}

// The group's gathers issued from one thread inside one RCCL group (each context's
// reduce on its own stream), then every stream synchronised.
int pt_comm_gather_all(void* const* ctxs, int32_t n, int32_t root) {
    if (!ctxs || n < 1) return fail(PT_ERR_INVALID_ARG, "bad context list");
    if (root < 0 || root >= n) return fail(PT_ERR_INVALID_ARG, "root out of range");
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        if (!c || !c->comm || c->nranks != n || c->rank != i)
            return fail(PT_ERR_RCCL, "contexts are not the group pt_comm_init_all formed (in that order)");
    }
    int rc;
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        PT_HIP(hipSetDevice(c->device));
        if ((rc = gather_prepare(c))) return rc;
    }
    ncclResult_t r = ncclGroupStart();   // step 1: the tile counts, every context in one group
    for (int i = 0; i < n && r == ncclSuccess; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        if (hipSetDevice(c->device) != hipSuccess) { r = ncclInvalidUsage; break; }
        r = ncclAllGather(c->g_cnts + c->nranks, c->g_cnts, 1, ncclInt32, c->comm, c->stream);
    }
    ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return fail(PT_ERR_RCCL, std::string("ncclAllGather (group): ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    std::vector<std::vector<int32_t>> cnts((size_t)n);
    std::vector<std::vector<int64_t>> offs((size_t)n);
    std::vector<int64_t> total((size_t)n, 0);
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        PT_HIP(hipSetDevice(c->device));
        PT_HIP(hipStreamSynchronize(c->stream));
        if ((rc = gather_counts(c, root, cnts[(size_t)i], offs[(size_t)i], total[(size_t)i]))) return rc;
    }
    r = ncclGroupStart();   // step 2: the sends and receives
    for (int i = 0; i < n && r == ncclSuccess; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        if (hipSetDevice(c->device) != hipSuccess) { r = ncclInvalidUsage; break; }
        r = gather_issue(c, root, cnts[(size_t)i], offs[(size_t)i]);
    }
    r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
        return fail(PT_ERR_RCCL, std::string("gather send/recv (group): ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
    for (int i = 0; i < n; i++) {
        Ctx* c = (Ctx*)ctxs[i];
        PT_HIP(hipSetDevice(c->device));
        if ((rc = gather_finish(c, root, total[(size_t)i]))) return rc;
    }
    return PT_OK;
}

int pt_comm_destroy(void* ctx) {
    Ctx* c = (Ctx*)ctx;
    if (!c) return fail(PT_ERR_INVALID_ARG, "ctx is NULL");
    if (c->comm) { ncclCommDestroy(c->comm); c->comm = nullptr; }
    c->nranks = 1; c->rank = 0;
    return PT_OK;
}

}  // extern "C"
