"""The 8-wide quantized triangle BVH the library builds (ptsharp_amd/csrc/pt_bvh.cpp collapse_bvh8q), host
build (tests/native/bvh8_check.cpp): every primitive in exactly one leaf chunk, every node reached once,
the traversal stack within kStackMax on every path, every slot box on a primitive's path holding it, and
the device's fp32 fma slab test (pt_device.h node8_step, restated) never culling a box the exact test
enters, on random boxes (1 .. 200K, coincident clusters) and a far-off sphere with flat boxes."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


def test_bvh8_structure_boxes_and_slab_arithmetic():
    subprocess.run(["make", "-s", "-C", NATIVE, "bvh8_check"], check=True)
    r = subprocess.run([os.path.join(NATIVE, "_build", "bvh8_check"), "2000"], capture_output=True, text=True, timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("bvh8_check: 0 failures")
    assert r.stdout.count(" 0 culled by the quantized tree") == 9
