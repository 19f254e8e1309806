"""The Volume marches (ptsharp_amd/csrc/pt_ext.h vol_t / vol_build_runs / t_after), host build:
vol_t, the per-lane march, equals Volume.Intersect's loop as written
(Volume.cs:168-197, restated position by position in tests/native/vol_skip_check.cpp) bit for bit
on seeded volumes and rays, including grazing rays and rays along lattice planes; t_after equals
k repeated fp64 additions across binade crossings; and the GPU's cooperative march with its strided
pass over uniform runs (pt_device.h coop_vol_t, kVolStride; its 64 lanes emulated as loops) gives
the same t as the loop as written, at strides 8, 16 and 32; and the march's Sign with the key and the
sample sharing one scaling of the position (pt_ext.h vol_sign_at) equals the two taken apart."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")


def test_vol_skip_bit_identical():
    subprocess.run(["make", "-s", "-C", NATIVE, "vol_skip_check"], check=True)
    r = subprocess.run([os.path.join(NATIVE, "_build", "vol_skip_check"), "4000"], capture_output=True, text=True,
                       timeout=300)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "t_after: 200000 cases, 0 differences" in r.stdout
    assert "vol_zdiv against the division: 60000000 cases, 0 differences" in r.stdout
    assert "(strides 8, 16, 32), emulated: 0 differences" in r.stdout
    assert "vol_sign_at against the key and the sample taken apart: 0 differences" in r.stdout
    assert " 0 differences;" in r.stdout.splitlines()[-1]
