"""The reference's own known-answer tests, run on the MI355X engine through the C ABI.

utils/tests/voxel_hash_test.cu (Single :56-92, Multiple :94-126, Collision :128-180) and
utils/tests/voxel_mem_test.cu (Test1 :38-90); every check is also compared against the oracle.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NUM_BUCKET = 1 << 21
BLOCK_LEN = 8


@pytest.fixture
def pair():
    import tsdf_amd
    from _oracle import OracleGrid
    eng = tsdf_amd.Engine(0.01, 0.06, max_width=64, max_height=64, num_block_bits=12)
    ora = OracleGrid(0.01, 0.06, 12)
    yield eng, ora
    eng.close()
    ora.close()


def same_state(eng, ora):
    a, b = eng.dump(pool=False), ora.dump(pool=False)
    assert np.array_equal(a["entry_pos"], b["entry_pos"])
    assert np.array_equal(a["entry_idx"], b["entry_idx"])
    assert np.array_equal(a["heap"], b["heap"]) and a["free"] == b["free"]


def test_hash_values():
    import tsdf_amd
    assert tsdf_amd.hash_block(33, 180, 42) == NUM_BUCKET - 1
    assert tsdf_amd.hash_block(61, 16, 170) == NUM_BUCKET - 1
    assert tsdf_amd.hash_block(63, 171, 45) == NUM_BUCKET - 1
    assert tsdf_amd.hash_block(1, 1, 1) == 1592143
    assert tsdf_amd.hash_block(-1, -1, -1) == 505009


def test_single(pair):
    eng, ora = pair
    eng.hash_allocate([[1, 1, 1]])
    r = eng.hash_retrieve([[8, 8, 8]])
    assert eng.num_active_blocks() == 1
    assert tuple(r["block_pos_off"][0, :3]) == (1, 1, 1)
    assert eng.hash_retrieve([[0, 0, 0]])["rgbw"][0, 3] == 0
    eng.hash_allocate([[0, 0, 0]])
    for i in range(BLOCK_LEN):
        assert eng.hash_assign([[0, 0, i]], [[i, i, i, i]]) == 0
    assert eng.num_active_blocks() == 2
    for i in range(BLOCK_LEN):
        assert list(eng.hash_retrieve([[0, 0, i]])["rgbw"][0]) == [i, i, i, i]
    ora.hash_allocate([[1, 1, 1]])
    ora.hash_allocate([[0, 0, 0]])
    same_state(eng, ora)


def test_multiple(pair):
    eng, ora = pair
    keys = np.array([[i, i, i] for i in range(128)], np.int16)
    eng.hash_allocate(keys)
    assert eng.num_active_blocks() == 128
    vox = np.array([[i, i, i, i] for i in range(128)], np.uint8)
    assert eng.hash_assign(keys * BLOCK_LEN, vox) == 0
    r = eng.hash_retrieve(keys * BLOCK_LEN)
    np.testing.assert_array_equal(r["rgbw"], vox)
    np.testing.assert_array_equal(r["block_pos_off"][:, :3], keys)
    ora.hash_allocate(keys)
    same_state(eng, ora)


def test_collision(pair):
    eng, ora = pair
    keys = np.array([[33, 180, 42], [61, 16, 170], [63, 171, 45], [0, 0, 0]], np.int16)
    for expect in (2, 3, 4):
        eng.hash_allocate(keys)
        ora.hash_allocate(keys)
        assert eng.num_active_blocks() == expect
        same_state(eng, ora)
    vox = np.array([[i, i, i, i] for i in range(4)], np.uint8)
    assert eng.hash_assign(keys * BLOCK_LEN, vox) == 0
    np.testing.assert_array_equal(eng.hash_retrieve(keys * BLOCK_LEN)["rgbw"], vox)


def test_delete_paths(pair):
    eng, ora = pair
    keys = np.array([[33, 180, 42], [61, 16, 170], [63, 171, 45]], np.int16)
    for _ in range(3):
        eng.hash_allocate(keys)
        ora.hash_allocate(keys)
    for batch in (keys[[1, 2]], keys, keys[[2]]):
        eng.hash_delete(batch)
        ora.hash_delete(batch)
        same_state(eng, ora)
    assert eng.num_active_blocks() == 0


def test_mem_pool(pair):
    eng, ora = pair
    idx = eng.pool_acquire(8)
    assert len(set(idx.tolist())) == 8
    for i, b in enumerate(idx):
        eng.pool_set_weight(b, i)
    for i, b in enumerate(idx):
        assert (eng.pool_get_weights(b) == i).all()
    eng.pool_release(idx)
    for i, b in enumerate(idx):
        assert (eng.pool_get_weights(b) == i).all()
    idx2 = eng.pool_acquire(8)
    assert sorted(idx2.tolist()) == sorted(idx.tolist())
    for b in idx2:
        assert (eng.pool_get_weights(b) == 0).all()
    np.testing.assert_array_equal(idx, ora.pool_acquire(8))
