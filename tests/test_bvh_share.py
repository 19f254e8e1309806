"""The triangle BVH is built once per process for identical geometry (pt_scene_bvh_digest, host only):
contexts that upload the same scene (bench.py --gpus N in one process, the .NET HipRendererGroup) share
one host build and receive the same bytes; a context uploading while another builds waits for it."""
import ctypes as C
import threading

import numpy as np

from ptsharp_amd import _abi, scenes


def digest(flat):
    out = (C.c_uint64 * 4)()
    _abi.check(_abi.load_library().pt_scene_bvh_digest(C.byref(flat.desc), out), "pt_scene_bvh_digest")
    return tuple(out)


def test_same_scene_built_once_and_identical():
    s, _, _ = scenes.bunny_frame(20_000, seed=41)
    flat = s.Compile()
    d0 = digest(flat)
    d1 = digest(flat)
    assert d0[0] == d1[0] and d0[1] == d1[1] > 0
    assert d1[2] == d0[2] and d1[3] == d0[3] + 1   # the second is a reuse, not a build
    # a separately compiled copy of the same geometry (a second Scene object, as each rank's host builds)
    s2, _, _ = scenes.bunny_frame(20_000, seed=41)
    d2 = digest(s2.Compile())
    assert d2[0] == d0[0] and d2[2] == d0[2]


def test_concurrent_uploads_share_one_build():
    s, _, _ = scenes.bunny_frame(60_000, seed=43)
    flat = s.Compile()
    before = digest(scenes.bunny_frame(2_000, seed=44)[0].Compile())   # counters before
    res = [None] * 6
    def run(i):
        res[i] = digest(flat)
    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(res))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert len({r[0] for r in res}) == 1 and len({r[1] for r in res}) == 1
    builds = max(r[2] for r in res) - before[2]
    hits = max(r[3] for r in res) - before[3]
    assert builds == 1 and hits == len(res) - 1


def test_different_geometry_different_bvh():
    a = digest(scenes.bunny_frame(20_000, seed=41)[0].Compile())
    s, _, _ = scenes.bunny_frame(20_000, seed=41)
    b = digest(scenes.bunny_frame(20_000, seed=42)[0].Compile())
    assert a[0] != b[0]
    # one vertex moved by one ulp is another scene
    flat = s.Compile()
    v = np.ctypeslib.as_array(flat.desc.tri_v1, shape=(flat.desc.num_triangles * 3,))
    v[5] = np.nextafter(v[5], np.float32(np.inf))
    c = digest(flat)
    assert c[0] != a[0]
