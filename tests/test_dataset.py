"""The disk-tracking data path: the generator
(data/disk/create_dataset.py) against trajectories the reference's own generator drew
(tests/golden/dataset.npz), the disc rasteriser, and the npz layout read back through
dataset.ToyDiskDataset.  Images are not pinned to the reference (it draws with cv2, absent
here): the rasteriser is checked for the disc's size, position and visibility count."""
import os
import types

import numpy as np
import pytest

from _util import group, load


def _example(tmp, T=6, n=4, file_size=500, width=128):
    from data.disk.create_dataset import ToyExample
    return ToyExample(types.SimpleNamespace(width=width, out_dir=str(tmp), name="t", num_examples=n,
                                            sequence_length=T, file_size=file_size))


@pytest.mark.parametrize("case", [0, 1, 2])
def test_trajectories_match_reference(case, tmp_path):
    fx = group(load("dataset.npz"), f"c{case}")
    nd, pn, seed = fx["cfg"]
    ex = _example(tmp_path)
    np.random.seed(int(seed))
    for n in range(2):
        v = ex._get_data(int(nd), float(pn))
        for k in ("start_state", "state", "q"):
            np.testing.assert_array_equal(np.asarray(v[k]), fx[f"s{n}/{k}"], err_msg=f"seq {n} {k}")
    # the generator consumed exactly the reference's number of draws
    assert np.random.uniform() == float(fx["next_uniform"])


def test_fill_circle_disc():
    from data.disk.create_dataset import fill_circle
    im = np.zeros((128, 128, 3))
    fill_circle(im, (64.7, 40.2), 7, (255, 0, 0))
    mask = (im[:, :, 0] == 255) & (im[:, :, 1] == 0)
    assert mask.sum() == 149  # the radius-7 disc of integer-centre rasterisers (cv2's too)
    ys, xs = np.nonzero(mask)
    assert (xs.min(), xs.max(), ys.min(), ys.max()) == (57, 71, 33, 47)  # centre (64, 40): x = column
    im2 = np.zeros((16, 16, 3))
    fill_circle(im2, (-3, 8), 7, (1, 2, 3))  # clipped at the frame edge
    assert (im2[:, :, 0] == 1).sum() == sum(1 for y in range(16) for x in range(16) if (x + 3) ** 2 + (y - 8) ** 2 <= 49)


def test_observation_visibility(tmp_path):
    ex = _example(tmp_path)
    im, vis = ex._observation_model(np.array([0.0, 0.0, 0.0, 0.0]), [])
    assert im.dtype == np.float32 and im.shape == (128, 128, 3) and vis == 149
    assert im[64, 64, 0] == 1.0 and im[64, 64, 1] == 0.0
    # a distractor drawn over the red disc hides part of it
    _, vis2 = ex._observation_model(np.array([0.0, 0.0, 0.0, 0.0]), [(5, np.array([3.0, 0.0, 0.0, 0.0]), 0)])
    assert 0 < vis2 < 149


def test_generate_and_load(tmp_path):
    from data.disk.create_dataset import main
    from dataset import ToyDiskDataset
    np.random.seed(3)
    # file_size = min(num_examples, --file-size) = 10: each file splits 8 / 1 / 1, and files are
    # written until 10 training sequences exist -> two files (the reference's loop)
    main(["--out-dir", str(tmp_path), "--num-examples", "10", "--sequence-length", "5", "--file-size", "10",
          "--num-distractors", "2"])
    files = sorted(os.listdir(tmp_path))
    name = "toy_pn=2.0_d=2_const"
    assert f"info_{name}.txt" in files and f"{name}0_train.npz" in files and f"{name}1_test.npz" in files
    info = open(os.path.join(tmp_path, f"info_{name}.txt")).read()
    assert "Num train: 16" in info and "Num val: 2" in info and "Num test: 2" in info
    tr = ToyDiskDataset(str(tmp_path), name, "train_data")  # the first file only (dataset.py:38-39)
    assert len(tr) == 8
    si, ss, im, st, q, vis = tr[0]
    assert si.shape == (128, 128, 3) and ss.shape == (4,) and im.shape == (5, 128, 128, 3)
    assert st.shape == (5, 4) and q.shape == (5, 4) and vis.shape == (5,)
    assert st.dtype == np.float32  # stored float64 (as the reference), read as float32
    np.testing.assert_array_equal(q[0], np.array([2.0, 2.0, 2.0, 2.0], np.float32))
    te = ToyDiskDataset(str(tmp_path), name, "test_data")
    va = ToyDiskDataset(str(tmp_path), name, "val_data")
    assert len(te) == 1 and len(va) == 1
    # the frames show the disc where the state says (visible count > 0 while it is in frame)
    for t in range(5):
        x, y = st[t, 0] + 64, st[t, 1] + 64
        if 8 <= x < 120 and 8 <= y < 120 and vis[t] > 0:
            assert im[t, int(y), int(x), 0] == 1.0
