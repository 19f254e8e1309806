"""pt_comm_gather's host-side arithmetic on CPU (no device): pt_gather_layout (where each rank's
packed tiles land in the root's receive buffers) and pt_tile_lists_check (ids in range, none twice),
and the whole tile-compacted protocol replayed with numpy on the library's own offsets, for uneven
tile counts, ranks with no tiles, roots other than 0 and more ranks than tiles.  The reference deals
disjoint 32x32 sub-tiles to its tasks (Renderer.cs:257-333); the gather must put every rank's tiles
back where they came from, bit for bit, or refuse."""
import ctypes as C

import numpy as np
import pytest

from ptsharp_amd import _abi, tiles_for_rank

lib = _abi.load_library()


def layout(counts, root, image_tiles):
    n = len(counts)
    cnt = np.ascontiguousarray(counts, np.int32)
    offs = (C.c_int64 * n)()
    total = C.c_int64(0)
    rc = lib.pt_gather_layout(n, root, cnt.ctypes.data_as(C.POINTER(C.c_int32)), image_tiles, offs, C.byref(total))
    return rc, list(offs), total.value


def lists_check(ids, image_tiles):
    a = np.ascontiguousarray(ids, np.int32)
    return lib.pt_tile_lists_check(a.ctypes.data_as(C.POINTER(C.c_int32)), len(a), image_tiles)


def pack(frame, ids, w, h):
    """k_tiles_pack's order: entry k = tile ids[k], 32x32 row-major, zeros outside the image."""
    tx = (w + 31) // 32
    out = np.zeros((len(ids), 32, 32) + frame.shape[2:], frame.dtype)
    for k, t in enumerate(ids):
        x0, y0 = (t % tx) * 32, (t // tx) * 32
        blk = frame[y0:y0 + 32, x0:x0 + 32]
        out[k, :blk.shape[0], :blk.shape[1]] = blk
    return out


def unpack(frame, ids, packed, w, h):
    tx = (w + 31) // 32
    for k, t in enumerate(ids):
        x0, y0 = (t % tx) * 32, (t // tx) * 32
        blk = frame[y0:y0 + 32, x0:x0 + 32]
        blk[...] = packed[k, :blk.shape[0], :blk.shape[1]]


def replay(w, h, lists, root, seed=0):
    """Each rank's frame holds values on its own tiles only; the root's receive buffers are laid out
    by pt_gather_layout, filled by every other rank's packed tiles, checked and unpacked; the
    result must equal the sum of the frames."""
    rng = np.random.default_rng(seed)
    tiles = ((w + 31) // 32) * ((h + 31) // 32)
    frames = []
    for ids in lists:
        m = np.zeros((h, w, 3))
        n = np.zeros((h, w), np.int32)
        own = np.zeros((h, w), bool)
        unpack(own, ids, np.ones((len(ids), 32, 32), bool), w, h)
        m[own] = rng.random((int(own.sum()), 3)) + 0.5
        n[own] = rng.integers(1, 9, int(own.sum()))
        frames.append((m, n))
    rc, offs, total = layout([len(x) for x in lists], root, tiles)
    assert rc == 0, lib.pt_last_error()
    assert total == sum(len(x) for p, x in enumerate(lists) if p != root)
    g_ids = np.full(max(total, 1), -1, np.int32)
    g_m = np.full((max(total, 1), 32, 32, 3), np.nan)
    g_n = np.full((max(total, 1), 32, 32), -7, np.int32)
    for p, ids in enumerate(lists):
        if p == root or not len(ids):
            assert offs[p] == -1
            continue
        o = offs[p]
        assert (g_ids[o:o + len(ids)] == -1).all(), "two ranks' blocks overlap in the receive buffer"
        g_ids[o:o + len(ids)] = ids
        g_m[o:o + len(ids)] = pack(frames[p][0], ids, w, h)
        g_n[o:o + len(ids)] = pack(frames[p][1], ids, w, h)
    recv = g_ids[:total]
    root_own = lists[root] if len(lists[root]) else []
    assert lists_check(np.concatenate([recv, np.asarray(root_own, np.int32)]), tiles) == 0
    m, n = frames[root][0].copy(), frames[root][1].copy()
    unpack(m, recv, g_m[:total], w, h)
    unpack(n, recv, g_n[:total], w, h)
    assert np.array_equal(m, sum(f[0] for f in frames))
    assert np.array_equal(n, sum(f[1] for f in frames))


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("root", [0, "last"])
def test_interleaved_tiles_every_root(world, root):
    w, h = 200, 150   # 7 x 5 tiles: uneven counts for 2, 3, 4 and 8 ranks, partial edge tiles
    root = world - 1 if root == "last" else root
    replay(w, h, [tiles_for_rank(w, h, r, world) for r in range(world)], root)


def test_more_ranks_than_tiles():
    w, h = 40, 40     # 2 x 2 tiles over 8 ranks: four ranks render nothing
    lists = [tiles_for_rank(w, h, r, 8) for r in range(8)]
    assert sum(len(x) == 0 for x in lists) == 4
    for root in (0, 5, 7):
        replay(w, h, lists, root)


def test_uneven_random_partition_with_empty_root():
    rng = np.random.default_rng(3)
    w, h = 333, 257
    tiles = ((w + 31) // 32) * ((h + 31) // 32)
    owner = rng.integers(1, 6, tiles)          # ranks 1..5 own everything; rank 0 (a root) and 6 nothing
    lists = [np.flatnonzero(owner == r).astype(np.int32) for r in range(7)]
    replay(w, h, lists, 0, seed=1)
    replay(w, h, lists, 6, seed=2)
    replay(w, h, lists, 3, seed=4)


def test_layout_offsets():
    rc, offs, total = layout([3, 0, 5, 2], 2, 16)
    assert rc == 0 and offs == [0, -1, -1, 3] and total == 5
    rc, offs, total = layout([4], 0, 4)
    assert rc == 0 and offs == [-1] and total == 0


@pytest.mark.parametrize("counts,root,tiles", [
    ([3, 3, 3], 0, 8),        # sums past the image: overlapping lists
    ([1, -1], 0, 8),          # negative count
    ([9, 0], 1, 8),           # one rank claims more than the image
    ([1, 1], 2, 8),           # root out of range
    ([1, 1], -1, 8),
])
def test_layout_refuses(counts, root, tiles):
    rc, _, _ = layout(counts, root, tiles)
    assert rc == _abi.PT_ERR_INVALID_ARG
    assert lib.pt_last_error()


def test_tile_lists_check():
    assert lists_check([0, 5, 3, 1], 6) == 0
    assert lists_check([], 6) == 0
    assert lists_check([0, 5, 3, 5], 6) == _abi.PT_ERR_INVALID_ARG
    assert b"listed twice" in lib.pt_last_error()
    assert lists_check([0, 6], 6) == _abi.PT_ERR_INVALID_ARG
    assert lists_check([-1], 6) == _abi.PT_ERR_INVALID_ARG
    # two interleaved ranks' lists are disjoint, the same list twice is not
    a, b = tiles_for_rank(200, 150, 0, 2), tiles_for_rank(200, 150, 1, 2)
    assert lists_check(np.concatenate([a, b]), 35) == 0
    assert lists_check(np.concatenate([a, a]), 35) == _abi.PT_ERR_INVALID_ARG
