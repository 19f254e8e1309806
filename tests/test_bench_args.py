"""bench.py's launch forms (no GPU needed): how `--gpus N` and the launcher's environment decide
between one process per GPU (torch.distributed.run), one process driving N devices
(pt_comm_init_all, one host thread each) and a single context; and the refusal when N exceeds
the devices this process sees."""
import os
import subprocess
import sys

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("gpus,env,group,want", [
    (1, {}, False, ("single", 1, 0, 0)),
    (8, {}, False, ("group", 8, 0, 0)),
    (2, {}, False, ("group", 2, 0, 0)),
    (1, {}, True, ("group", 1, 0, 0)),
    # under torch.distributed.run the env wins; --gpus is the launcher's business
    (8, {"WORLD_SIZE": "8", "RANK": "3", "LOCAL_RANK": "3"}, False, ("dist", 8, 3, 3)),
    (1, {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"}, False, ("dist", 4, 0, 0)),
    (4, {"WORLD_SIZE": "1"}, False, ("single", 1, 0, 0)),
])
def test_resolve_world(gpus, env, group, want):
    assert bench.resolve_world(gpus, env, group) == want


def test_parse_defaults_and_gpus_bound():
    a = bench.parse([])
    assert (a.gpus, a.steps, a.warmup, a.spp, a.width, a.height) == (1, 64, 2, 16, 1920, 1080)
    a = bench.parse(["--workload", "c5"])
    assert (a.steps, a.spp, a.width, a.height, a.adaptive) == (2, 1, 3840, 2160, 32)
    with pytest.raises(SystemExit):
        bench.parse(["--gpus", "0"])


def test_each_runs_every_context_and_raises():
    import threading
    together = threading.Barrier(4, timeout=30)   # passes only if the four calls run concurrently

    def f(i, x):
        together.wait()
        return i, x
    out = bench._each(list("abcd"), f)
    assert out == [(0, "a"), (1, "b"), (2, "c"), (3, "d")]

    def boom(i, x):
        if i == 2:
            raise ValueError("bad device")
        return i
    with pytest.raises(RuntimeError, match="device 2"):
        bench._each([0, 1, 2, 3], boom)


def test_group_refuses_more_gpus_than_devices():
    """`bench.py --gpus N` with no launcher and fewer than N devices exits non-zero with a message
    (this container has no device, so N = 2 is already too many)."""
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("host has a GPU")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 2
    assert "HIP device" in p.stderr


def test_scale_block_keys():
    """The per-context record of an N-GPU line (`scale_detail`): each context's rays, device and wall
    time, the gather's time, the slowest context and its share, the imbalance."""
    ctx = [{"rank": 0, "device": 0, "rays": 100, "kernel_ms": 9.0, "render_ms": 10.0, "gather_ms": 1.5},
           {"rank": 1, "device": 1, "rays": 120, "kernel_ms": 11.0, "render_ms": 12.0, "gather_ms": 1.5}]
    b = bench.scale_block(ctx, 1.5, 0.0135)
    for k in ("contexts", "gather_ms", "render_ms_max", "render_ms_mean", "slowest_rank",
              "slowest_share_of_elapsed", "imbalance", "rays_total"):
        assert k in b
    assert b["slowest_rank"] == 1 and b["rays_total"] == 220 and b["gather_ms"] == 1.5
    assert b["imbalance"] == round(12.0 / 11.0, 4)
    assert b["slowest_share_of_elapsed"] == round(12.0 / 13.5, 4)
    assert [c["rank"] for c in b["contexts"]] == [0, 1]
    one = bench.scale_block(ctx[:1], None, 0.011)
    assert one["gather_ms"] is None and one["imbalance"] == 1.0


def test_library_id_matches_file():
    import hashlib
    p = os.path.join(ROOT, "ptsharp_amd", "libptsharp_hip.so")
    if not os.path.exists(p):
        pytest.skip("library not built")
    assert bench.library_id() == hashlib.sha256(open(p, "rb").read()).hexdigest()[:16]
