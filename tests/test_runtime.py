"""Native host runtime (``_rt``): voxel generator, bit packing, binvox IO."""
import numpy as np
import pytest
import torch

from featurenet_amd import _native


@pytest.fixture(scope="module")
def rt():
    if not _native.runtime_available():
        pytest.skip("native runtime not built")
    return _native.runtime()


def test_generator_deterministic_and_labelled(rt):
    a, la = rt.generate_voxels(32, 32, 7)
    b, lb = rt.generate_voxels(32, 32, 7, threads=1)
    assert a.shape == (32, 32 ** 3 // 8) and a.dtype == np.uint8
    np.testing.assert_array_equal(a, b)          # thread count does not change the data
    np.testing.assert_array_equal(la, lb)
    assert la.min() >= 0 and la.max() < rt.NUM_FEATURE_CLASSES
    c, _ = rt.generate_voxels(32, 32, 8)
    assert not np.array_equal(a, c)


def test_generator_requested_labels_and_occupancy(rt):
    labels = np.arange(24, dtype=np.int64)
    bits, lab = rt.generate_voxels(24, 32, 0, labels=labels)
    np.testing.assert_array_equal(lab, labels)
    vox = rt.unpack_bits(bits, 24 * 32 ** 3).reshape(24, 32, 32, 32)   # flat bit stream
    fill = vox.reshape(24, -1).mean(1)
    assert np.all(fill > 0.05) and np.all(fill < 0.995)    # a stock block with a feature removed
    # different classes give different shapes
    assert len({vox[i].tobytes() for i in range(24)}) == 24


def test_pack_unpack_roundtrip_and_torch_unpack(rt):
    from featurenet_amd.training.data import unpack_voxels

    rng = np.random.default_rng(0)
    vox = (rng.random((3, 16 ** 3)) < 0.3).astype(np.uint8)
    packed = rt.pack_bits(vox).reshape(3, -1)          # flat LSB-first bit stream
    np.testing.assert_array_equal(rt.unpack_bits(packed, vox.size).reshape(vox.shape), vox)
    t = unpack_voxels(torch.as_tensor(packed), 16)
    np.testing.assert_array_equal(t.reshape(3, -1).float().numpy().astype(np.uint8), vox)


def test_binvox_roundtrip(rt, tmp_path):
    rng = np.random.default_rng(1)
    g = (rng.random((16, 16, 16)) < 0.4).astype(np.uint8)
    p = str(tmp_path / "a.binvox")
    rt.write_binvox(p, g, [1.0, 2.0, 3.0], 0.5)
    back, tr, sc = rt.read_binvox(p)
    np.testing.assert_array_equal(back, g)
    assert tuple(tr) == (1.0, 2.0, 3.0) and sc == pytest.approx(0.5)


def test_voxel_dataset_and_binvox_folder(rt, tmp_path):
    from featurenet_amd.training.data import binvox_folder, voxel_dataset

    ds = voxel_dataset(48, 16, size=32, seed=3)
    assert ds.packed and ds.num_classes == 24 and ds.input_shape[:3] == (32, 32, 32)
    for cls in ("hole", "slot"):
        (tmp_path / cls).mkdir()
        for i in range(2):
            rt.write_binvox(str(tmp_path / cls / f"{i}.binvox"), np.ones((8, 8, 8), np.uint8))
    x, y, names = binvox_folder(tmp_path)
    assert len(y) == 4 and sorted(names) == ["hole", "slot"]
