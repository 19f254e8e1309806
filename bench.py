#!/usr/bin/env python3
"""bench.py — Msamples/s (Scene.Intersect calls per second, BASELINE.json metric)
of PTSharp's render hot path on MI355X.

Workload (BASELINE.json configs[3], the north-star target): a seeded
1,000,000-triangle mesh in Example.bunny's scene (floor cube, two light spheres,
NewSampler(4,4), SpecularModeFirst), 1920x1080.  One step = one
Renderer.RenderParallel pass at --spp samples per pixel; K steps accumulate
K·spp samples per pixel (default 64 × 16 = 1024 spp).  N > 1: the image's 32x32
tiles are dealt round-robin to ranks, the scene is replicated, and the Welford
Buffer is gathered onto rank 0 over RCCL at the end of the timed region (strong
scaling: the image is fixed).  Two launch forms: under torch.distributed.run
(WORLD_SIZE set) one process per GPU joined by pt_comm_init; without a launcher,
`--gpus N` makes this one process drive devices 0..N-1 — N contexts joined by
pt_comm_init_all, one host thread per device, pt_comm_gather_all — the form the
.NET host's HipRendererGroup uses (Renderer.cs:257-333 spreads one frame over the
whole machine from one process).

Rank 0 prints one JSON line (driver contract), with `roofline` for the closest-hit
kernel and `cpu_baseline` (the oracle port timed on this host).

--workload c3 / c2 measure the other GPU configs of BASELINE.json the same way (not the
driver's line): C3 = the 69,451-triangle mesh in the same frame (L2 roofline of its dominant
kernel), C2 = the gopher 3-sphere scene, NewSampler(16,16), no triangle BVH, and C5 = the mixed 4K
scene: both VALU-issue-bound (fp64 sampler math; fp64 marches), priced by the pass' measured VALU issue
cycles per ray (PMC instruction mix by kind, profiles/pmc_valu_mix_<workload>.json) against 1024 SIMDs
at 2.4 GHz, with the measured fp32 / fp64 FLOP rates beside it.

Roofline: the closest-hit kernel's algorithmic bytes (per ray: 128 B per
BVH8 node fetch, 36 B per primitive test, 44 B ray in + hit out) over its HIP-event time,
against the L2 bandwidth (≈34.5 TB/s, MI355X_MICROARCH.md §L2).  The BVH nodes and leaf
chunks (~62 MB at 1M triangles) live in L2 and the 256 MB Infinity Cache, so HBM is not the
binding bound (the same bytes over 8 TB/s gave a fraction above 1 in round 1).  `traffic`
is the measured L2↔fabric bytes per launch (rocprofv3 FETCH_SIZE×2 + WRITE_SIZE, which
count Infinity-Cache hits too; profiles/pmc_traffic.json), set beside the compulsory bytes
(every ray's queue entry read once, its hit written once, the traversal footprint once).
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/s (rays×bounces/s) at 1920×1080×1024spp; PSNR vs C# ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)
L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md §L2 (per-XCD L2s, aggregate)
FP32_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md (FP32 vector peak)
# FP64 vector peak: half the FP32 rate (a wave64 fp64 FMA issues over 4 cycles against 2 for
# fp32, MI355X_MICROARCH.md "issue cost"; AMD's MI355X specification: 78.6 TFLOP/s)
FP64_PEAK_TFLOPS = 78.6
# VALU issue peak: 1024 SIMDs (256 CUs x 4) each issuing one cycle's work per cycle at 2.4 GHz, in
# T SIMD-cycles/s.  C2 and C5 are priced by their measured VALU issue cycles (tools/gpu_valu_mix.sh ->
# profiles/pmc_valu_mix_*.json): a flop model (round 4: 60 fp32 flops per shading) missed the fp64
# sincos / acos / sqrt chains that are most of their work.
VALU_ISSUE_PEAK = 1024 * 2.4e9 / 1e12
WORKLOADS = {
    "c4": "C4: 1M-triangle mesh in Example.bunny's scene, 1920x1080, NewSampler(4,4) SpecularModeFirst",
    "c3": "C3: 69,451-triangle mesh in Example.bunny's scene, 1920x1080, NewSampler(4,4) SpecularModeFirst",
    "c2": "C2: gopher 3-sphere scene (Example.cs:1542-1564, mesh replaced by two spheres), 1920x1080, "
          "NewSampler(16,16), no triangle BVH",
    "c5": "C5: mixed scene (the C4 1M-triangle frame + SDF torus + voxel Volume + environment texture), "
          "3840x2160, RenderParallel with AdaptiveSamples",
}
# per-workload defaults of --steps / --warmup / --spp / --width / --height / --adaptive: C5's 4K pass
# with AdaptiveSamples 32 traces 33 camera samples per pixel (≈5 G rays) per step
DEFAULTS = {"c5": dict(steps=2, warmup=1, spp=1, width=3840, height=2160, adaptive=32)}
DEFAULT = dict(steps=64, warmup=2, spp=16, width=1920, height=1080, adaptive=0)

# Algorithmic bytes per unit (SURVEY.md §8d with this BVH's node): per ray 128 B per node fetched (the
# triangle BVH's 8-wide node: origin, steps, child bases and counts 32 B + eight quantized child boxes 96 B;
# round 4's BVH4 node was 112 B: four 24-B boxes and four refs), 36 B per primitive tested (v0, e1, e2),
# 28 B ray in + 16 B hit out, and 40 B (three normals + material id) per closest-hit shading fetch.
B_NODE, B_PRIM, B_RAY, B_SHADE = 128, 36, 28 + 16, 40


def _gloo_gather(r, dist, rank, world, mine):
    """pt_comm_gather's protocol over gloo (tile counts, then each rank's packed tiles to rank 0,
    written into its Buffer with pt_write_tiles): the fallback if the RCCL gather fails."""
    import torch
    cnts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(cnts, torch.tensor([len(mine)], dtype=torch.int64))
    if rank != 0:
        dist.send(torch.from_numpy(np.ascontiguousarray(mine, np.int32)), dst=0)
        for a in r.ReadTiles(mine):
            dist.send(torch.from_numpy(np.ascontiguousarray(a)), dst=0)
        return
    for p in range(1, world):
        n = int(cnts[p][0])
        ids = torch.zeros(n, dtype=torch.int32)
        dist.recv(ids, src=p)
        parts = [torch.zeros((n, 32, 32, 3), dtype=torch.float64), torch.zeros((n, 32, 32, 3), dtype=torch.float64),
                 torch.zeros((n, 32, 32), dtype=torch.int32)]
        for x in parts:
            dist.recv(x, src=p)
        r.WriteTiles(ids.numpy(), *(x.numpy() for x in parts))


GATHER_WATCHDOG_S = 300.0


def library_id(path=None):
    """First 16 hex digits of the product library's SHA-256: bench lines and the stored counter profiles
    (profiles/pmc_*.json) carry it, so a profile taken on another build is flagged, not silently reused."""
    import hashlib
    path = path or os.path.join(ROOT, "ptsharp_amd", "libptsharp_hip.so")
    try:
        with open(path, "rb") as f:
            return hashlib.sha256(f.read()).hexdigest()[:16]
    except OSError:
        return None


def scale_block(contexts, gather_ms, elapsed_s):
    """What an N-GPU line needs to explain itself: every context's rays, device time
    of its passes (hipEvent) and wall time of its timed passes, the gather's wall time after the
    last pass, the slowest context and its share of the timed region, and the imbalance (slowest
    over mean wall).  contexts: [{"rank", "device", "rays", "kernel_ms", "render_ms"}]."""
    render = [float(c["render_ms"]) for c in contexts]
    slow = max(range(len(contexts)), key=lambda k: render[k]) if contexts else None
    mean = sum(render) / len(render) if render else 0.0
    return {
        "contexts": [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in c.items()} for c in contexts],
        "gather_ms": None if gather_ms is None else round(gather_ms, 3),
        "render_ms_max": round(max(render), 3) if render else None,
        "render_ms_mean": round(mean, 3) if render else None,
        "slowest_rank": None if slow is None else contexts[slow]["rank"],
        "slowest_share_of_elapsed": round(render[slow] / (elapsed_s * 1e3), 4) if render and elapsed_s > 0 else None,
        "imbalance": round(max(render) / mean, 4) if render and mean > 0 else None,
        "rays_total": int(sum(int(c["rays"]) for c in contexts)),
    }


def _watchdog(seconds, what):
    """Ends the process with status 3 if `what` has not finished within `seconds` (cancel() when it has)."""
    import threading

    def fire():
        print(f"{what} did not finish within {seconds:.0f} s on this rank; exiting", file=sys.stderr, flush=True)
        os._exit(3)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def _gather_check(r, dist, rank, world, mine):
    """Every rank's own tiles (pt_read_tiles, as it rendered them) to rank 0 over gloo; rank 0 reads
    the same tiles from its gathered Buffer and compares bit for bit.  Returns the verdict on rank 0."""
    import torch
    parts = [np.ascontiguousarray(a) for a in r.ReadTiles(mine)] if len(mine) else []
    cnts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(cnts, torch.tensor([len(mine)], dtype=torch.int64))
    if rank != 0:
        if len(mine):
            dist.send(torch.from_numpy(np.ascontiguousarray(mine, np.int32)), dst=0)
            for a in parts:
                dist.send(torch.from_numpy(a), dst=0)
        return None
    bad, checked = 0, len(mine)
    for p in range(1, world):
        n = int(cnts[p][0])
        if n == 0:
            continue
        ids = torch.zeros(n, dtype=torch.int32)
        dist.recv(ids, src=p)
        sent = [torch.zeros((n, 32, 32, 3), dtype=torch.float64), torch.zeros((n, 32, 32, 3), dtype=torch.float64),
                torch.zeros((n, 32, 32), dtype=torch.int32)]
        for x in sent:
            dist.recv(x, src=p)
        got = r.ReadTiles(ids.numpy())
        bad += sum(int(not np.array_equal(g, x.numpy())) for g, x in zip(got, sent))
        checked += n
    return {"tiles": checked, "bit_exact": bad == 0,
            "what": "rank 0's Buffer after the gather vs each rank's own pt_read_tiles, {M, V, N}"}


def _group_gather_check(rs, W, H, tiles_for_rank):
    """The one-process form's check: context 0's Buffer after pt_comm_gather_all against every other
    context's own pt_read_tiles of its tile list, bit for bit."""
    bad, checked = 0, 0
    for k, x in enumerate(rs):
        ids = tiles_for_rank(W, H, k, len(rs))
        if not len(ids):
            continue
        got = rs[0].ReadTiles(ids)
        mine = x.ReadTiles(ids)
        bad += sum(int(not np.array_equal(g, m)) for g, m in zip(got, mine))
        checked += len(ids)
    return {"tiles": checked, "bit_exact": bad == 0,
            "what": "context 0's Buffer after pt_comm_gather_all vs each context's own pt_read_tiles, {M, V, N}"}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="GPUs of this node; under torch.distributed.run (WORLD_SIZE set) one per process, "
                        "otherwise this one process drives devices 0..N-1 (pt_comm_init_all, one host thread each)")
    p.add_argument("--steps", type=int, default=None, help="timed steps (default 64; c5: 2)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2; c5: 1)")
    p.add_argument("--spp", type=int, default=None, help="samples per pixel per step (pass; default 16, c5: 1)")
    p.add_argument("--width", type=int, default=None, help="default 1920 (c5: 3840)")
    p.add_argument("--height", type=int, default=None, help="default 1080 (c5: 2160)")
    p.add_argument("--adaptive", type=int, default=None,
                   help="Renderer.AdaptiveSamples (Renderer.cs:340-410; default 0, c5: 32 as Example.cs:355,412)")
    p.add_argument("--firefly", type=int, default=0,
                   help="Renderer.FireflySamples (Renderer.cs:412-470; Example.bunny sets 32, Example.cs:1100): per pass, "
                        "pixels whose deviation exceeds 1 take up to N more samples, stopping at the first firefly")
    p.add_argument("--workload", choices=sorted(WORKLOADS), default="c4")
    p.add_argument("--tris", type=int, default=None, help="mesh triangles (default: 1,000,000 for c4, 69,451 for c3)")
    p.add_argument("--seed", type=int, default=1234)
    p.add_argument("--mesh-source", choices=["obj", "generator"], default="obj",
                   help="c3/c4 mesh: written as OBJ and loaded through pt_obj_load (default), or in memory")
    p.add_argument("--cpu-seconds", type=float, default=15.0, help="CPU-baseline sample budget (0 = skip)")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--engine", choices=["auto", "mega", "wave"], default="auto")
    p.add_argument("--json-out", default=None)
    p.add_argument("--passes-per-call", type=int, default=0,
                   help="passes per pt_render_pass call (pt_pass_params.passes; 0 = auto: the number of tile "
                        "shares, so one rank's share of an N-GPU frame is batched N passes at a time)")
    p.add_argument("--shard", default=None, metavar="K/N",
                   help="render only rank K's tiles of an N-way split, in this one process (profiling the "
                        "per-rank workload of an N-GPU run on one GPU; value then counts this shard only)")
    p.add_argument("--group", action="store_true",
                   help="the one-process multi-GPU form even at --gpus 1 (a one-context pt_comm_init_all group)")
    a = p.parse_args(argv)
    for k, v in DEFAULTS.get(a.workload, DEFAULT).items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    if a.gpus < 1:
        p.error("--gpus must be >= 1")
    return a


def resolve_world(gpus, env, group_flag=False):
    """How this process takes part in an N-GPU run.  Returns (mode, world, rank, local_rank):
    'dist'  — launched by torch.distributed.run (WORLD_SIZE in env): one rank per process, --gpus is
              the launcher's business (the env wins);
    'group' — no launcher and --gpus N > 1 (or --group): this process creates N contexts on devices
              0..N-1, joins them with pt_comm_init_all and drives each from its own host thread
              (Renderer.cs:257-333's whole-machine parallelism; HipRendererGroup's form);
    'single' — one GPU, one context."""
    if env.get("WORLD_SIZE") is not None:
        world = int(env["WORLD_SIZE"])
        return ("dist" if world > 1 else "single"), world, int(env.get("RANK", "0")), int(env.get("LOCAL_RANK", "0"))
    if gpus > 1 or group_flag:
        return "group", int(gpus), 0, 0
    return "single", 1, 0, 0


def _each(rs, fn):
    """fn(i, rs[i]) for every local context, concurrently (one host thread per device: the library's
    calls release the GIL, and every entry point sets its context's device), results in order."""
    if len(rs) == 1:
        return [fn(0, rs[0])]
    import threading
    out, errs = [None] * len(rs), []

    def run(i):
        try:
            out[i] = fn(i, rs[i])
        except BaseException as e:   # re-raised on the calling thread
            errs.append((i, e))
    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(rs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        i, e = sorted(errs, key=lambda x: x[0])[0]
        raise RuntimeError(f"device {i}: {e}") from e
    return out


def main(argv=None):
    a = parse(argv)
    mode, world, rank, local = resolve_world(a.gpus, os.environ, a.group)
    if mode == "dist" and a.gpus not in (1, world):
        print(f"--gpus {a.gpus} ignored: WORLD_SIZE={world} (one rank per process)", file=sys.stderr, flush=True)
    dist = None
    if mode == "dist":
        import torch.distributed as dist  # control plane only (barrier, id broadcast, max/sum)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from ptsharp_amd import Renderer, _abi, scenes, tiles_for_rank

    # A rehearsal of the N-rank path on a box with fewer GPUs than ranks (ranks share devices):
    # RCCL cannot put two ranks on one GPU, so the tiles are gathered over gloo there, and said so.
    ndev = C.c_int32(0)
    _abi.load_library().pt_device_count(C.byref(ndev))
    if mode == "group" and ndev.value < world:
        print(f"bench.py --gpus {world}: this process sees {ndev.value} HIP device(s); the one-process form "
              f"needs one device per GPU requested", file=sys.stderr, flush=True)
        sys.exit(2)
    shared = mode == "dist" and ndev.value < world and not os.environ.get("PT_BENCH_FORCE_RCCL")
    rccl_ok = False
    local = local % max(ndev.value, 1)
    t_scene = time.perf_counter()
    obj_info = None
    if a.workload == "c2":
        scene, camera, sampler = scenes.gopher3()
    else:
        frame = scenes.mixed if a.workload == "c5" else scenes.bunny_frame
        if a.tris is None:
            a.tris = 69_451 if a.workload == "c3" else 1_000_000
        if a.mesh_source == "obj":
            # Example.bunny loads its mesh with OBJ.Load (Example.cs:1088): the seeded mesh is written as
            # an OBJ file and read back through pt_obj_load (OBJ.cs's quirks), as SURVEY.md §8d specifies
            import tempfile
            from ptsharp_amd.scene import OBJ
            with tempfile.TemporaryDirectory() as d:
                path = os.path.join(d, f"mesh{a.tris}.obj")
                tw = time.perf_counter()
                scenes.write_blob_obj(path, a.tris, seed=a.seed)
                tw = time.perf_counter() - tw
                size = os.path.getsize(path)
                t_scene = tl = time.perf_counter()   # scene setup from the OBJ load on (not the writer)
                mesh = OBJ.Load(path)
                tl = time.perf_counter() - tl
            obj_info = {"obj_bytes": size, "obj_write_s": round(tw, 3), "obj_load_s": round(tl, 3),
                   "obj_triangles": len(mesh.v1)}
            raw = {k: getattr(mesh, k).copy() for k in ("v1", "v2", "v3", "n1", "n2", "n3", "t1", "t2", "t3")}
            scene, camera, sampler = frame(a.tris, seed=a.seed, mesh=mesh)
        else:
            scene, camera, sampler = frame(a.tris, seed=a.seed)
    scene.Compile()
    t_scene = time.perf_counter() - t_scene
    if obj_info is not None:   # the OBJ round trip is exact: the loaded Triangle[] is the generator's, bit for bit
        gen = scenes.blob_mesh(a.tris, a.seed)
        obj_info["obj_equals_generator"] = all(np.array_equal(raw[k].view(np.uint32), getattr(gen, k).view(np.uint32))
                                          for k in raw)
        del gen, raw

    W, H = a.width, a.height
    # the contexts this process drives: one (single / dist), or one per device (group), local index 0 = rank 0
    ranks = list(range(world)) if mode == "group" else [rank]
    devices = list(range(world)) if mode == "group" else [local]
    rs = []
    for rk, dev in zip(ranks, devices):
        r = Renderer.NewRenderer(scene, camera, sampler, W, H, True, device=dev)
        r.SamplesPerPixel = a.spp
        r.AdaptiveSamples = a.adaptive
        r.FireflySamples = a.firefly
        r.Seed = a.seed
        r.Engine = {"auto": 0, "mega": 1, "wave": 2}[a.engine]
        if a.shard:
            k, nsh = (int(x) for x in a.shard.split("/"))
            r.Tiles = tiles_for_rank(W, H, k, nsh)
        if world > 1:
            r.Tiles = tiles_for_rank(W, H, rk, world)
        rs.append(r)
    r = rs[0]
    if mode == "group":
        Renderer.CommInitAll(rs)   # pt_comm_init_all: ncclCommInitAll over devices 0..N-1, one call
        rccl_ok = True
    elif mode == "dist" and not shared:
        obj = [Renderer.CommUniqueId() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ok = 1
        try:
            r.CommInit(world, rank, obj[0])
        except Exception as e:
            print(f"pt_comm_init failed ({e}); the tiles will be gathered over gloo", file=sys.stderr, flush=True)
            ok = 0
        import torch
        t_ok = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(t_ok, op=dist.ReduceOp.MIN)
        rccl_ok = bool(t_ok[0])
    # every device uploads its replica, from its own thread; the triangle BVH is built once for all of them
    # (pt_upload_scene shares one host build of identical geometry: pt_scene_bvh_digest)
    t_up = time.perf_counter()
    _each(rs, lambda i, x: x._ensure_scene())
    t_up = time.perf_counter() - t_up
    st = r.Stats()
    build_ms, bvh_bytes = st.build_ms, st.bvh_bytes
    upload_ms = [round(x.Stats().build_ms, 1) for x in rs]
    # closest-hit and shadow kernels the library runs on this scene: per-lane refill
    # (k_wf_*_lanes) above 64 triangle-BVH nodes (pt_wavefront.hip kLanesMinNodes); the bench scene's
    # analytic BVH (floor cube, two light spheres) is one node
    # (SDF shapes, volumes or transformed shapes: the FULL instantiations, pt_wavefront.hip depth_loop)
    fl = scene.Compile()
    fullg = any(fl.counts_ext[1:4])
    full = fullg or len(fl.texture_list) > 0 or fl.env_texture > 0   # (1-based texture slots, 0 = none)
    lanes = st.bvh_nodes - 1 > 64
    # (row-4 scenes with a mesh split each traversal: the lean refill kernel <false, true>, then the FULL
    # kernel <false, true, true> on the rays that reach a row-4 box, then the deferred Volume and SDF
    # records' kernels; the class times them together)
    split = fullg and lanes
    # a few spheres / cubes (at most 8) and planes (at most 8), no triangles: the linear kernels
    # (pt_wavefront.hip k_wf_trace_linear / k_wf_shadow_linear); lean shadow kernels read a scene's lights
    # from LDS (their <.., true> forms) when it has at most 16
    n_ana = len(fl.sphere_radius) + len(fl.cube_min)
    linear = not fullg and not lanes and fl.num_triangles == 0 and 0 < n_ana <= 8 and len(fl.plane_point) <= 8
    emits = np.array([m.emittance > 0 for m in fl.materials] + [False])
    n_lights = sum(int(emits[np.asarray(arr, dtype=np.int64)].sum()) for arr in
                   (fl.sphere_material, fl.cube_material, fl.plane_material, fl.tri_material) if len(arr))
    ldsl = ", true" if n_lights <= 16 else ""
    trace_name = ("k_wf_trace_lanes<false, true> + k_wf_trace<false, true, true> + k_wf_vol_hits + k_wf_sdf_hits"
                  if split else "k_wf_trace<false, true>" if fullg else "k_wf_trace_lanes<false, false>" if lanes
                  else "k_wf_trace_linear<false>" if linear else "k_wf_trace<false, false>")
    shadow_name = ("k_wf_shadow_lanes<false, true> + k_wf_shadow<false, true, true> + k_wf_vol_shadow + k_wf_sdf_shadow"
                   if split else "k_wf_shadow<false, true>" if fullg
                   else f"k_wf_shadow_lanes<false, false{', false' + ldsl if ldsl else ''}>" if lanes
                   else f"k_wf_shadow_linear<false{ldsl or ', false'}>" if linear
                   else f"k_wf_shadow<false, false{', false' + ldsl if ldsl else ''}>")
    shade_name = "k_wf_shade<false, true, *>" if full else "k_wf_shade<false, false, *>"

    # Passes per call: a rank's 1/N share of the frame is batched N passes per call (the Buffer is
    # the one separate passes leave, bit for bit), so every launch sees a whole frame's worth of
    # camera samples; a whole frame already fills the GPU (and the queues) in one pass.
    shares = world if world > 1 else (int(a.shard.split("/")[1]) if a.shard else 1)
    ppc = a.passes_per_call or max(1, min(shares, 8))

    def run_passes(x, k, timed=False):   # k passes on context x, ppc per call; per-call stats when timed
        done, rays_k, kms_k, kl_k, kern = 0, 0, np.zeros(_abi.K_SLOTS), np.zeros(_abi.K_SLOTS, np.int64), 0.0
        while done < k:
            m = min(ppc, k - done)
            if m == 1:
                x.RenderParallel()
            else:
                x.RenderPasses(m)
            done += m
            if timed:
                s = x.Stats()
                rays_k += s.rays
                kern += s.last_pass_ms
                kms_k += np.array(s.kernel_ms[:])
                kl_k += np.array(s.kernel_launches[:])
        return rays_k, kern, kms_k, kl_k

    # warm-up includes one full batch (its accumulators)
    _each(rs, lambda i, x: run_passes(x, max(a.warmup, ppc if a.warmup else 0)))
    # one instrumented (untimed) pass on rank 0's context: traversal counters → algorithmic bytes per
    # ray, per kernel (every rank's share is the same mix of rays)
    ctr = r.RenderCounted()
    ext_rays = ctr.rays - ctr.shadow_rays
    ext_nodes = ctr.nodes_visited - ctr.shadow_nodes
    ext_prims = ctr.prims_tested - ctr.shadow_prims
    bytes_ext = B_NODE * ext_nodes + B_PRIM * ext_prims + B_RAY * ext_rays
    bytes_sh = B_NODE * ctr.shadow_nodes + B_PRIM * ctr.shadow_prims + B_RAY * ctr.shadow_rays
    bytes_all = bytes_ext + bytes_sh + B_SHADE * ctr.shading_fetches
    _each(rs, lambda i, x: x.ResetBuffer())

    def timing_on(i, x):
        x.Flags = _abi.PASS_KERNEL_TIMING
        x.Synchronize()
    # ---------------- timed region (per-kernel hipEvent timing on the library's stream)
    _each(rs, timing_on)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()

    def timed_passes(i, x):   # this context's timed passes and their wall time (one host thread each)
        tc = time.perf_counter()
        res = run_passes(x, a.steps, timed=True)
        return res + ((time.perf_counter() - tc) * 1e3,)
    per = _each(rs, timed_passes)
    t_rendered = time.perf_counter()
    rays_local = [p[0] for p in per]
    rays, kernel_ms, kms, klaunch = per[0][:4]   # rank 0's kernels for the roofline
    gather = None
    if shared:   # no RCCL between ranks on one device: the same tile protocol over gloo
        _gloo_gather(r, dist, rank, world, tiles_for_rank(W, H, rank, world))
        gather = "gloo (rehearsal)"
    elif mode == "dist" and not rccl_ok:
        _gloo_gather(r, dist, rank, world, tiles_for_rank(W, H, rank, world))
        gather = "gloo (RCCL init failed)"
    elif mode == "group":
        dog = _watchdog(GATHER_WATCHDOG_S, "pt_comm_gather_all")
        Renderer.GatherAll(rs, 0)   # pt_comm_gather_all: every context's sends / receives in one RCCL group
        dog.cancel()
        gather = "rccl (one process, pt_comm_gather_all)"
    elif mode == "dist":
        # A failure inside the RCCL group on one rank would leave its peers blocked in the group:
        # the watchdog ends this process (non-zero) instead of letting the job hang.  A failure
        # every rank sees alike (the MIN below) falls back to the same protocol over gloo.
        dog = _watchdog(GATHER_WATCHDOG_S, "pt_comm_gather")
        ok = 1
        try:
            r.Gather(0)   # pt_comm_gather: tile-compacted send/recv over RCCL
        except Exception as e:   # then every rank takes the same protocol over gloo
            print(f"pt_comm_gather failed ({e}); gathering the tiles over gloo", file=sys.stderr, flush=True)
            ok = 0
        import torch
        t_ok = torch.tensor([ok], dtype=torch.int32)
        dist.all_reduce(t_ok, op=dist.ReduceOp.MIN)
        if int(t_ok[0]):
            gather = "rccl"
        else:
            _gloo_gather(r, dist, rank, world, tiles_for_rank(W, H, rank, world))
            gather = "gloo (RCCL gather failed)"
        dog.cancel()
    _each(rs, lambda i, x: x.Synchronize())
    t1 = time.perf_counter()
    gather_ms = (t1 - t_rendered) * 1e3 if gather else None
    if dist:
        dist.barrier()
    elapsed = t1 - t0
    mine = [{"rank": rk, "device": dev, "rays": int(p[0]), "kernel_ms": float(p[1]), "render_ms": float(p[4]),
             "gather_ms": None if gather_ms is None else float(gather_ms)} for rk, dev, p in zip(ranks, devices, per)]
    if dist:
        allc = [None] * world
        dist.all_gather_object(allc, mine)
        contexts = [c for lst in allc for c in lst]
    else:
        contexts = mine
    if dist:
        import torch
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])
        rr = torch.tensor([rays], dtype=torch.float64)
        dist.all_reduce(rr, op=dist.ReduceOp.SUM)
        total_rays = int(rr[0])
    else:
        total_rays = int(sum(rays_local))   # group: every device's rays, one clock around all of them

    gather_check = None
    if mode == "dist":
        # after the timed region: rank 0's gathered Buffer must hold every rank's tiles as that rank
        # rendered them (each rank's pt_read_tiles of its own list, sent over gloo), bit for bit
        dog = _watchdog(GATHER_WATCHDOG_S, "gather check")
        gather_check = _gather_check(r, dist, rank, world, tiles_for_rank(W, H, rank, world))
        dog.cancel()
    elif mode == "group":
        gather_check = _group_gather_check(rs, W, H, tiles_for_rank)

    if rank != 0:
        r.close()
        if dist:
            dist.barrier()
            dist.destroy_process_group()
        return
    for x in rs[1:]:
        x.close()

    value = total_rays / elapsed / 1e6
    lib_id = library_id()
    # camera samples traced per pixel per step: the pass' own, then AdaptiveSamples (Renderer.cs:355-372;
    # its second loop only fills pixelVariances, which nothing reads, and is not traced: DESIGN.md §1a)
    cam_spp = a.spp + a.adaptive
    # kernel names as rocprofv3 reports them (template arguments <COUNT, FULL>; the shade
    # class times both of its forms <COUNT, FULL, SCAN>, one of which returns at once; the
    # closest-hit class is k_wf_trace_lanes<COUNT> on triangle scenes)
    names = ["k_wf_camera", trace_name, shade_name, shadow_name,
             "k_wf_finalize", "k_render_pass<false, false>", "k_wf_nee_accum", "-"]
    # the closest-hit kernel is the dominant one by design (on a multi-GPU shard the shadow
    # passes run beside it on a second stream, so their event spans overlap it)
    # (C3 / C2: the kernel with the most time)
    dom = _abi.K_TRACE if klaunch[_abi.K_TRACE] and a.workload == "c4" else int(np.argmax(kms))
    # algorithmic bytes of the dominant kernel over the timed region: the counted pass' bytes per
    # ray of that kernel's ray class × the rays it traced (same scene/seed/spp → same ray mix)
    if dom == _abi.K_TRACE:
        per_ray, kind_rays = bytes_ext / max(ext_rays, 1), ext_rays
    elif dom == _abi.K_SHADOW:
        per_ray, kind_rays = bytes_sh / max(ctr.shadow_rays, 1), ctr.shadow_rays
    else:
        per_ray, kind_rays = bytes_all / max(ctr.rays, 1), ctr.rays
    frac_rays = kind_rays / max(ctr.rays, 1)
    dom_bytes = per_ray * rays * frac_rays
    avg_launch_ms = kms[dom] / max(klaunch[dom], 1)
    achieved_gbs = dom_bytes / (kms[dom] * 1e-3) / 1e9
    rays_per_launch = rays * frac_rays / max(klaunch[dom], 1)
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json" if a.workload == "c4" else f"pmc_traffic_{a.workload}.json")
    if os.path.exists(pmc):
        with open(pmc) as f:
            tj = json.load(f)
        if tj.get("kernel") == names[dom] and tj.get("workload_tris") == scene.Compile().num_triangles:
            traffic = round(tj["traffic_bytes_per_ray"] * rays_per_launch)
            traffic_src = {"tag": tj.get("tag"), "library": tj.get("library"),
                           "same_library": tj.get("library") is not None and tj.get("library") == library_id()}
    # compulsory bytes of one launch: each ray's queue entry (origin, direction: 32 B) read and its
    # hit (16 B) written once, the traversal footprint (BVH nodes + leaf chunks) read once
    compulsory = rays_per_launch * 48 + st.traversal_bytes
    out = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "launch": {"single": "one process", "dist": "torch.distributed.run, one process per GPU",
                   "group": "one process, one host thread per GPU (pt_comm_init_all)"}[mode],
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32/f64",
        "data": ("synthetic (seeded displaced-sphere mesh" + (", written as OBJ and loaded through pt_obj_load"
                                                               if obj_info else "")
                 + ("; seeded environment texture, SDF torus and 32x32x16 voxel Volume" if a.workload == "c5" else "")
                 + "; no model assets ship with the reference)") if a.workload != "c2"
        else "synthetic (analytic gopher3 scene)",
        "config": {
            "workload": WORKLOADS[a.workload],
            "width": W, "height": H, "spp_per_step": a.spp, "total_spp": a.spp * a.steps,
            "adaptive_samples": a.adaptive, **({"firefly_samples": a.firefly} if a.firefly else {}),
            "triangles": scene.Compile().num_triangles, "parallelism": f"tiles{world}" + (f" shard {a.shard}" if a.shard else "")
            + (f" (rehearsal: {world} ranks on {ndev.value} GPU(s))" if shared else "")
            + (f", gather {gather}" if gather else ""),
            "gather_check": gather_check,
            "passes_per_call": ppc,
            "camera_samples_per_s": round(W * H * cam_spp * a.steps / elapsed, 1),
            "rays_per_camera_sample": round(total_rays / (W * H * cam_spp * a.steps), 3),
            "shadow_ray_fraction": round(ctr.shadow_rays / max(ctr.rays, 1), 4),
            "lit_shadow_rays_per_step": int(ctr.lit_shadow_rays), "accum_runs_per_step": int(ctr.accum_runs),
            "engine": a.engine, "scene_build_s": round(t_scene, 3), "bvh_build_ms": round(build_ms, 1),
            "scene_upload_s": round(t_up, 3), "contexts_upload_ms": upload_ms,
            "mesh_source": None if a.workload == "c2" else a.mesh_source, **(obj_info or {}),
            "bvh_bytes": int(bvh_bytes),
            "kernel_ms_per_step": {names[k]: round(kms[k] / a.steps, 3) for k in range(_abi.K_SLOTS) if klaunch[k]},
        },
        # per-context rays / device time / wall time and the gather's own time (rank 0's clock for the gather)
        "scale_detail": scale_block(contexts, gather_ms if mode != "dist" else
                                    max((c["gather_ms"] or 0.0) for c in contexts) if gather else None, elapsed),
        "library": lib_id,
        "roofline": {
            "bound": "l2", "kernel": names[dom],
            "achieved": round(achieved_gbs, 2), "peak": L2_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved_gbs / L2_PEAK_GBS, 5), "traffic": traffic,
            "traffic_kind": "L2-fabric bytes per launch (FETCH_SIZE x2 + WRITE_SIZE; Infinity-Cache hits included), "
                            "profiles/pmc_traffic.json, same workload",
            "traffic_source": traffic_src,
            "compulsory_bytes_per_launch": round(compulsory),
            "traffic_over_compulsory": None if traffic is None else round(traffic / compulsory, 3),
            "traffic_frac_of_hbm_peak": None if traffic is None else
            round(traffic / (avg_launch_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "avg_launch_ms": round(float(avg_launch_ms), 4), "launches": int(klaunch[dom]),
            "bytes_per_launch": round(dom_bytes / max(klaunch[dom], 1)),
            "bytes_per_ray": round(per_ray, 2),
            "rays_per_launch": round(rays_per_launch),
            "nodes_per_ray": round((ext_nodes if dom == _abi.K_TRACE else ctr.nodes_visited) /
                                   max(ext_rays if dom == _abi.K_TRACE else ctr.rays, 1), 3),
            "prims_per_ray": round((ext_prims if dom == _abi.K_TRACE else ctr.prims_tested) /
                                   max(ext_rays if dom == _abi.K_TRACE else ctr.rays, 1), 3),
            "all_kernels_bytes_per_ray": round(bytes_all / max(ctr.rays, 1), 2),
            "pass_achieved_gbs": round(bytes_all / max(ctr.rays, 1) * rays / (kernel_ms * 1e-3) / 1e9, 2),
        },
    }

    def whole_traffic(rays_timed):   # C2 / C5 (kernel "whole pass"): L2-fabric bytes per step, all kernels
        pw = os.path.join(ROOT, "profiles", f"pmc_traffic_{a.workload}.json")
        if not os.path.exists(pw):
            return {"traffic": None}
        with open(pw) as f:
            tw = json.load(f)
        return {"traffic": round(tw["traffic_bytes_per_ray"] * rays_timed / a.steps),
                "traffic_kind": f"L2-fabric bytes per step, every kernel of the pass (FETCH_SIZE x2 + WRITE_SIZE; "
                                f"Infinity-Cache hits included), profiles/pmc_traffic_{a.workload}.json ({tw.get('tag')}), "
                                f"same workload"}

    def march_clock():   # C5: the cooperative Volume march's time by phase (counted pass, s_memtime per phase)
        mc = [int(x) for x in ctr.march_clock]
        dense, strided = max(mc[6], 1), max(mc[7], 1)
        total = sum(mc[:6])
        names = ("strided_pass", "table", "corners", "windows", "bookkeeping", "refinements")
        return {"cycles_per_dense_round": {k: round(mc[1 + i] / dense, 1) for i, k in enumerate(names[1:5])},
                "cycles_per_strided_round": round(mc[0] / strided, 1),
                "share": {k: round(mc[i] / max(total, 1), 4) for i, k in enumerate(names)},
                "dense_rounds": mc[6], "strided_rounds": mc[7],
                "note": "wave cycles (shader clock) summed over marching waves, counted pass (clock reads add ~10 %)"}

    def valu_roofline():   # C2 / C5: whole pass bound by VALU issue (measured instruction mix, profiles/)
        pv = os.path.join(ROOT, "profiles", f"pmc_valu_mix_{a.workload}.json")
        extra = {"nodes_per_ray": round(ctr.nodes_visited / max(ctr.rays, 1), 3),
                 **({"volume_samples_per_ray": round(ctr.volume_samples / max(ctr.rays, 1), 3),
                     "sdf_evals_per_ray": round(ctr.sdf_evals / max(ctr.rays, 1), 3),
                     "volume_march_clock": march_clock()} if a.workload == "c5" else {})}
        if not os.path.exists(pv):
            return {"bound": "valu_issue", "kernel": "whole pass", "achieved": None, "peak": VALU_ISSUE_PEAK,
                    "unit": "T SIMD-cycles/s", "frac": None, "note": f"{pv} missing (tools/gpu_valu_mix.sh)", **extra}
        with open(pv) as f:
            vm = json.load(f)
        if vm.get("library") != lib_id:
            # the stored instruction mix was measured on another build: not priced
            return {"bound": "valu_issue", "kernel": "whole pass", "achieved": None, "peak": VALU_ISSUE_PEAK,
                    "unit": "T SIMD-cycles/s", "frac": None, **whole_traffic(rays),
                    "mix_stale": True, "mix_library": vm.get("library"), "library": lib_id,
                    "note": f"{pv} ({vm.get('tag')}) was measured on library {vm.get('library')}, not this one "
                            f"({lib_id}): re-run tools/gpu_valu_mix.sh", **extra}
        pr = vm["per_ray"]
        sec = kernel_ms * 1e-3
        achieved = pr["valu_issue_cycles"] * rays / sec / 1e12
        f32 = pr["fp32_flops"] * rays / sec / 1e12
        f64 = pr["fp64_flops"] * rays / sec / 1e12
        # the counted pass' instantiations (COUNT = true) merged into their timed kernels'
        merged = {}
        for name, kv in vm["kernels"].items():
            if name.startswith(("k_wf_trace", "k_wf_shadow", "k_wf_shade")) and not name.startswith("k_wf_shade_miss"):
                name = name.replace("<true", "<false", 1)
            m = merged.setdefault(name, {"valu_issue_cycles": 0.0, "busy": 0.0})
            m["valu_issue_cycles"] += kv["valu_issue_cycles"]
            m["busy"] += kv["busy_cycles_per_xcd"]
        dom_k = max(merged.items(), key=lambda kv: kv[1]["valu_issue_cycles"])
        dom_k = (dom_k[0], {"valu_issue_frac": round(dom_k[1]["valu_issue_cycles"] / max(1024 * dom_k[1]["busy"], 1.0), 4)})
        return {
            "bound": "valu_issue", "kernel": "whole pass",
            "achieved": round(achieved, 5), "peak": VALU_ISSUE_PEAK, "unit": "T SIMD-cycles/s",
            "frac": round(achieved / VALU_ISSUE_PEAK, 5), **whole_traffic(rays),
            "valu_issue_cycles_per_ray": round(pr["valu_issue_cycles"], 2), "valu_insts_per_ray": round(pr["valu_insts"], 2),
            "f64_insts_per_ray": round(pr["f64_insts"], 2),
            "measured_fp32_tflops": round(f32, 4), "measured_fp32_frac": round(f32 / FP32_PEAK_TFLOPS, 5),
            "measured_fp64_tflops": round(f64, 4), "measured_fp64_frac": round(f64 / FP64_PEAK_TFLOPS, 5),
            "issue_model": "cycles per wave64 instruction: 2 (fp32 / int), 4 (fp64 add / mul / fma), 8 (fp32 transcendental), "
                           "16 (fp64 transcendental); peak = 1024 SIMDs x 2.4 GHz",
            "mix_source": f"profiles/pmc_valu_mix_{a.workload}.json ({vm.get('tag')}: SQ_INSTS_VALU and its per-kind "
                          f"counters, SQ_INSTS_VALU_FLOPS_FP32/FP64, same workload, same library {lib_id})",
            "dominant_kernel": dom_k[0], "dominant_kernel_valu_issue_frac_under_counters": dom_k[1]["valu_issue_frac"],
            "pass_valu_issue_frac_under_counters": vm.get("pass_valu_issue_frac_under_counters"),
            **extra,
        }

    def shade_roofline():   # C4: the shade kernel beside the closest-hit roofline (VALU issue and bytes per vertex)
        # algorithmic bytes per step: each vertex's queue entry (o, d, throughput, key: 64 B) and hit (16 B)
        # read, the closest hit's triangle record and shading normals (96 B) per shading fetch, each child
        # ray written (64 B: every closest-hit ray after the camera's) and each shadow request written
        # (o, n, two fp64 weight pairs: 64 B); scaled from the counted pass to the timed region's rays
        if not klaunch[_abi.K_SHADE]:
            return None
        cam_rays = W * H * cam_spp
        per_pass = (ext_rays * (64 + 16) + ctr.shading_fetches * 96 + max(ext_rays - cam_rays, 0) * 64
                    + ctr.shadow_rays * 64)
        scale = rays / max(ctr.rays, 1)   # timed rays over the counted pass' rays (same ray mix)
        sec = kms[_abi.K_SHADE] * 1e-3
        gbs = per_pass * scale / max(sec, 1e-12) / 1e9
        blk = {"kernel": names[_abi.K_SHADE], "ms_per_step": round(kms[_abi.K_SHADE] / a.steps, 3),
               "launches": int(klaunch[_abi.K_SHADE]),
               "bytes_per_vertex": round(per_pass / max(ext_rays, 1), 2), "vertices_per_step": round(ext_rays * scale / a.steps),
               "achieved": round(gbs, 2), "unit": "GB/s", "frac_of_l2_peak": round(gbs / L2_PEAK_GBS, 5),
               "frac_of_hbm_peak": round(gbs / HBM_PEAK_GBS, 5), "valu_issue_frac": None}
        pv = os.path.join(ROOT, "profiles", "pmc_valu_mix_c4.json")
        if os.path.exists(pv):
            with open(pv) as f:
                vm = json.load(f)
            ks = {k: v for k, v in vm.get("kernels", {}).items() if k.startswith("k_wf_shade") and "miss" not in k}
            if vm.get("library") == lib_id and ks:
                issue = sum(v["valu_issue_cycles"] for v in ks.values())
                busy = sum(v["busy_cycles_per_xcd"] for v in ks.values())
                blk["valu_issue_frac"] = round(issue / max(1024 * busy, 1.0), 4)
                # the mix's rays are all rays (closest hit + shadow) of the profiled passes: the same mix here
                blk["valu_issue_cycles_per_vertex"] = round(issue / max(vm.get("rays_profiled", 1), 1)
                                                            * ctr.rays / max(ext_rays, 1), 2)
                blk["mix_source"] = f"profiles/pmc_valu_mix_c4.json ({vm.get('tag')}), same library"
            else:
                blk["mix_stale"] = True
                blk["mix_library"] = vm.get("library")
        return blk

    if a.workload == "c4":
        out["roofline"]["shade"] = shade_roofline()
        # the same pass priced by VALU issue (the C2 / C5 lines' bound): the closest-hit kernel is bound by its
        # dependent loads and by VALU issue together (profiles/r06q_wave_states.txt), so both fractions are shown
        vi = valu_roofline()
        out["roofline"]["valu_issue"] = {k: vi[k] for k in (
            "achieved", "peak", "unit", "frac", "valu_issue_cycles_per_ray", "dominant_kernel",
            "dominant_kernel_valu_issue_frac_under_counters", "pass_valu_issue_frac_under_counters", "mix_source",
            "mix_stale", "note") if k in vi}

    if a.workload in ("c2", "c5"):
        # C2 (fp64 sampler math, 16 children per camera hit) and C5 (the fp64 Volume / SDF marches) are
        # bound by VALU issue, not by bytes: the pass' measured VALU issue cycles per ray (instruction mix
        # by kind from PMC counters, priced at each kind's issue cost) over the pass' kernel time, against
        # 1024 SIMDs issuing every cycle; the measured fp32 / fp64 FLOP rates beside it
        out["roofline"] = valu_roofline()

    # keys that do not apply to this run are left out rather than null (one GPU: no gather; C2: no mesh)
    for k in ("gather_check", "mesh_source"):
        if out["config"].get(k, 0) is None:
            del out["config"][k]

    # ---------------- CPU baseline + parity sample (rank 0, N = 1 only), at the timed configuration: the
    # full frame at the bench's own spp per pass (one chunk, as each timed step runs it), pass index 1 (the
    # first timed step's), against the oracle on a strided pixel set sized to ~cpu_seconds of CPU work
    # (C3 and C2 too: the same leg on their frames; C5's adaptive phase is checked by the GPU tests)
    if world == 1 and a.workload in ("c4", "c3", "c2") and a.adaptive == 0 and (a.cpu_seconds > 0 or not a.no_parity):
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib as O
        osc = O.OracleScene(scene)
        threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
        spp = a.spp
        # probe ~2048 pixels (~3 s on C4; C2's 16 children per camera hit and 16 bounces: 256), then size the
        # sample to the budget
        stride = max(1, (W * H) // (256 if a.workload == "c2" else 2048))
        tp = time.perf_counter()
        _, prays = O.render_pixels(osc, camera, sampler, W, H, spp, 0, W * H, stride, seed=a.seed, pass_index=1,
                                   threads=threads)
        tp = time.perf_counter() - tp
        print(f"cpu baseline probe: {(W * H + stride - 1) // stride} pixels x {spp} spp, {prays} rays in {tp:.1f}s",
              file=sys.stderr, flush=True)   # (progress: a long oracle leg is not a hung run)
        budget = max(a.cpu_seconds, 1.0)
        npx = max(64, min(W * H, int(((W * H + stride - 1) // stride) * budget / max(tp, 1e-3))))
        stride = max(1, (W * H) // npx)
        tc = time.perf_counter()
        obuf, crays = O.render_pixels(osc, camera, sampler, W, H, spp, 0, W * H, stride, seed=a.seed, pass_index=1,
                                      threads=threads)
        tc = time.perf_counter() - tc
        sampled = (W * H + stride - 1) // stride
        out["cpu_baseline"] = {
            "value": round(crays / tc / 1e6, 5), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"oracle/pt_oracle.cpp (k-d tree, recursive sampler, fp64 colour) on {sampled} pixels "
                      f"(every {stride}th of {W}x{H}) x {spp} spp, pass 1, {crays} rays in {tc:.1f}s",
        }
        out["gpu_vs_cpu"] = round(value / (crays / tc / 1e6), 1)
        if not a.no_parity:
            # the GPU renders the whole frame at the same spp, seed and pass index: the timed step's chunking
            r.ResetBuffer()
            r.SamplesPerPixel = spp
            r.FireflySamples = 0   # (render_pixels runs the main samples; --firefly's phase is checked by the GPU tests)
            r._pass = 0
            r.RenderParallel()
            g = r.ReadBuffer()
            idx = np.arange(0, W * H, stride)
            gm = g.M.reshape(-1, 3)[idx]
            om = obuf.M.reshape(-1, 3)[idx]
            gn, on = g.N.reshape(-1)[idx], obuf.N.reshape(-1)[idx]
            err = np.abs(gm - om)
            ok = (err <= 1e-3 * np.maximum(1.0, np.abs(om))).all(axis=1).mean()
            ok9 = (err <= 1e-9 * np.maximum(1.0, np.abs(om))).all(axis=1).mean()
            from parity import psnr8
            out["parity"] = {"vs": "oracle (seeded CPU restatement; C# Random.Shared is unseedable)",
                             "spp": spp, "pass_index": 1,
                             "gpu_render": f"full {W}x{H} frame at {spp} spp in one pt_render_pass, as each timed step",
                             "pixels": int(len(idx)), "frac_within_1e-3": round(float(ok), 6),
                             "frac_within_1e-9": round(float(ok9), 6), "n_equal": bool(np.array_equal(gn, on)),
                             "psnr_db": round(psnr8(gm[None], om[None]), 2), "max_abs_err": float(err.max())}
    r.close()
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
