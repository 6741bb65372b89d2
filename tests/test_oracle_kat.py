"""Pin the CPU oracle against the reference's own known-answer tests.

Restates utils/tests/voxel_hash_test.cu (Single :56-92, Multiple :94-126, Collision :128-180) and
utils/tests/voxel_mem_test.cu (Test1 :38-90) against oracle/tsdf_oracle.c. These are the only
golden facts the reference holds for this path.
"""
import numpy as np
import pytest

from _oracle import OracleGrid, hash_block

NUM_BUCKET = 1 << 21
BLOCK_LEN = 8


@pytest.fixture
def grid():
    g = OracleGrid(0.01, 0.06, num_block_bits=12)
    yield g
    g.close()


def test_hash_known_values():
    # voxel_hash_test.cu:133-135: three keys collide in the last bucket
    assert hash_block(33, 180, 42) == NUM_BUCKET - 1
    assert hash_block(61, 16, 170) == NUM_BUCKET - 1
    assert hash_block(63, 171, 45) == NUM_BUCKET - 1
    # sign-extended short -> uint, multiply mod 2^32
    assert hash_block(1, 1, 1) == 1592143
    assert hash_block(-1, -1, -1) == 505009
    assert hash_block(0, 0, 0) == 0


def test_single(grid):
    """voxel_hash_test.cu:56-92 VoxelHashTest.Single."""
    grid.hash_allocate([[1, 1, 1]])
    r = grid.hash_retrieve([[8, 8, 8]])
    assert grid.num_active_blocks() == 1
    assert tuple(r["block_pos_off"][0, :3]) == (1, 1, 1)
    r = grid.hash_retrieve([[0, 0, 0]])  # empty block -> default voxel
    assert r["rgbw"][0, 3] == 0
    grid.hash_allocate([[0, 0, 0]])
    for i in range(BLOCK_LEN):
        assert grid.hash_assign([[0, 0, i]], [[i, i, i, i]]) == 0
    assert grid.num_active_blocks() == 2
    for i in range(BLOCK_LEN):
        r = grid.hash_retrieve([[0, 0, i]])
        assert list(r["rgbw"][0]) == [i, i, i, i]


def test_multiple(grid):
    """voxel_hash_test.cu:94-126 VoxelHashTest.Multiple (128 diagonal blocks, one launch)."""
    keys = np.array([[i, i, i] for i in range(128)], np.int16)
    grid.hash_allocate(keys)
    assert grid.num_active_blocks() == 128
    pts = keys * BLOCK_LEN
    vox = np.array([[i, i, i, i] for i in range(128)], np.uint8)
    assert grid.hash_assign(pts, vox) == 0
    r = grid.hash_retrieve(pts)
    np.testing.assert_array_equal(r["rgbw"], vox)
    np.testing.assert_array_equal(r["block_pos_off"][:, :3], keys)


def test_collision(grid):
    """voxel_hash_test.cu:128-180 VoxelHashTest.Collision: one insertion per bucket per launch."""
    keys = np.array([[33, 180, 42], [61, 16, 170], [63, 171, 45], [0, 0, 0]], np.int16)
    grid.hash_allocate(keys)
    assert grid.num_active_blocks() == 2
    grid.hash_allocate(keys)
    assert grid.num_active_blocks() == 3
    grid.hash_allocate(keys)
    assert grid.num_active_blocks() == 4
    pts = keys * BLOCK_LEN
    vox = np.array([[i, i, i, i] for i in range(4)], np.uint8)
    assert grid.hash_assign(pts, vox) == 0
    r = grid.hash_retrieve(pts)
    np.testing.assert_array_equal(r["rgbw"], vox)
    # the third key went to the list: tail of the last bucket links (with wrap-around) to entry 2
    d = grid.dump(pool=False)
    last = 2 * NUM_BUCKET - 1
    assert d["entry_pos"][last, 3] == 3  # offset = 2 + 2^22 - (2^22 - 1)
    assert tuple(d["entry_pos"][2, :3]) == (63, 171, 45)


def test_collision_delete_chain(grid):
    """Delete through slot 0, list head and list element (voxel_hash.cu:122-171)."""
    keys = np.array([[33, 180, 42], [61, 16, 170], [63, 171, 45]], np.int16)
    for _ in range(3):
        grid.hash_allocate(keys)
    assert grid.num_active_blocks() == 3
    # head + element of the same bucket in one launch: only the first lock holder succeeds
    grid.hash_delete(keys[[1, 2]])
    assert grid.num_active_blocks() == 2
    r = grid.hash_retrieve(keys * BLOCK_LEN)
    assert list(r["block_idx"] >= 0) == [True, False, True]
    # the moved element now sits in the head slot (entry 2^22-1), the old element entry is free
    d = grid.dump(pool=False)
    assert tuple(d["entry_pos"][2 * NUM_BUCKET - 1, :3]) == (63, 171, 45)
    assert d["entry_pos"][2 * NUM_BUCKET - 1, 3] == 0
    assert d["entry_idx"][2] == -1
    grid.hash_delete(keys)  # slot 0 (lock free) + head (locked) in one launch
    assert grid.num_active_blocks() == 0


def test_mem_pool(grid):
    """voxel_mem_test.cu:38-90 VoxelMemTest.Test1."""
    idx = grid.pool_acquire(8)
    assert len(set(idx.tolist())) == 8
    for i, b in enumerate(idx):
        grid.pool_set_weight(b, i)
    for i, b in enumerate(idx):
        assert (grid.pool_get_weights(b) == i).all()
    grid.pool_release(idx)  # release does not clobber memory
    for i, b in enumerate(idx):
        assert (grid.pool_get_weights(b) == i).all()
    idx2 = grid.pool_acquire(8)  # acquire again clears the weights
    assert sorted(idx2.tolist()) == sorted(idx.tolist())
    for b in idx2:
        assert (grid.pool_get_weights(b) == 0).all()


def test_pool_lifo_order(grid):
    """AquireBlock pops heap[free-1] (voxel_mem.cu:38-41); initial heap[i] = i (:6-11)."""
    n = grid.num_blocks
    assert list(grid.pool_acquire(3)) == [n - 1, n - 2, n - 3]
    grid.pool_release(np.array([n - 2], np.int32))
    assert list(grid.pool_acquire(1)) == [n - 2]


def test_oracle_mesh_is_a_surface():
    """Oracle marching cubes on a small integrated stream: triangles exist, lie inside the
    allocated region (+1 voxel), and no vertex is farther than one voxel from a sample point
    with the sign change it interpolates (sanity of the restatement; parity unpinned)."""
    from tsdf_amd import synth
    cam = synth.camera(48, 36, synth.TUM_FR1)
    g = OracleGrid(0.02, 0.08, 11)
    try:
        for f in range(3):
            fr = synth.render(cam, 3 * f)
            g.integrate(fr["rgb"], fr["depth"], fr["ht"], fr["lt"], 4.0, cam.K, fr["q"], fr["t"])
        tris = g.extract_mesh(None, 0.99, 1)
        assert tris.shape[0] > 100 and np.isfinite(tris).all()
        d = g.dump(pool=False)
        blk = d["entry_pos"][d["entry_idx"] >= 0, :3].astype(np.float32) * 8 * 0.02
        lo, hi = blk.min(0) - 0.02, blk.max(0) + 8 * 0.02 + 0.03
        v = tris.reshape(-1, 3)
        assert (v >= lo).all() and (v <= hi).all()
        # each vertex lies on a grid edge: two of its coordinates sit on sample positions
        on_grid = np.isclose(np.mod(v - 0.01, 0.02), 0, atol=1e-5) | np.isclose(np.mod(v - 0.01, 0.02), 0.02, atol=1e-5)
        assert (on_grid.sum(1) >= 2).all()
    finally:
        g.close()
