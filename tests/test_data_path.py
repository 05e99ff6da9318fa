"""Data path: the oracle against the reference's own outputs
(tests/golden/data_golden.npz, made by tests/golden/make_golden_data.py), the host mirror of
DataAndDataset.py, and the HIP path (tpg_landmark_boxes + tpg_crop_normalize) against both.
Integer boxes and every output value are checked bit-exact."""
import os

import numpy as np
import pytest
import torch

from oracle import data_oracle as DO

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data_golden.npz")


@pytest.fixture(scope="module")
def gold():
    with np.load(GOLD, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def _ntest(g):
    return len([k for k in g if k.startswith("test:") and k.endswith(":u8_128")])


def _oracle_test_sample(g, k, pts_idx=DO.FIVE_PTS_IDX_REPAIRED):
    w, h = g["test:%d:wh" % k]
    lm5 = DO.rescale(DO.five_points(g["test:%d:lm68" % k], pts_idx), w, h)
    return DO.crop_normalize(g["test:%d:u8_128" % k], DO.crop_boxes(lm5))


def test_oracle_five_points(gold):
    lm = gold["five:lm68"]
    for i in range(len(lm)):
        np.testing.assert_array_equal(DO.five_points(lm[i], DO.FIVE_PTS_IDX_REFERENCE), gold["five:ref"][i])
        np.testing.assert_array_equal(DO.five_points(lm[i], DO.FIVE_PTS_IDX_REPAIRED), gold["five:r5"][i])
    assert np.isnan(gold["five:ref"][:, 4]).all()


def test_oracle_test_dataset(gold):
    for k in range(_ntest(gold)):
        crops = _oracle_test_sample(gold, k)
        for name in DO.PATCH_NAMES:
            np.testing.assert_array_equal(crops[name], gold["test:%d:%s" % (k, name)], err_msg="%d %s" % (k, name))
    np.testing.assert_array_equal(DO.to_unit(gold["test:0:u8_128"]), gold["test:0:img"])
    # the crops leave the image for sample 1 (eyes at the corner): the fill reads as -1
    assert (gold["test:1:left_eye"] == -1.0).any()


def test_oracle_reference_table_raises(gold):
    assert int(gold["test_raises"]) == 1
    w, h = gold["test:0:wh"]
    lm5 = DO.rescale(DO.five_points(gold["test:0:lm68"], DO.FIVE_PTS_IDX_REFERENCE), w, h)
    with pytest.raises(ValueError):
        DO.crop_boxes(lm5)


def test_oracle_multipie_names(gold):
    for k, n in enumerate(gold["names:list"]):
        paths, label = DO.multipie_paths(str(n))
        assert list(paths.values()) == [str(s) for s in gold["names:%d:opened" % k]]
        assert label == int(gold["names:%d:label" % k])


def test_host_mirror(gold, monkeypatch):
    """tp-gan_amd/DataAndDataset.py's host functions: process() on a PIL image and the
    TrainDataset file naming, against the reference's outputs."""
    from PIL import Image
    import DataAndDataset as DD
    for k in range(_ntest(gold)):
        w, h = gold["test:%d:wh" % k]
        lm5 = DO.rescale(DO.five_points(gold["test:%d:lm68" % k], DO.FIVE_PTS_IDX_REPAIRED), w, h)
        b = DD.process(Image.fromarray(gold["test:%d:u8_128" % k]), lm5.copy())
        for name in DD.PATCH_NAMES:
            got = (DD._to_tensor(b[name]) * 2.0 - 1.0).numpy()
            np.testing.assert_array_equal(got, gold["test:%d:%s" % (k, name)])
    opened = []
    monkeypatch.setattr(Image, "open", lambda p: opened.append(p) or Image.fromarray(np.zeros((2, 2, 3), np.uint8)))
    names = [str(n) for n in gold["names:list"]]
    ds = DD.TrainDataset(names)
    for k in range(len(names)):
        opened.clear()
        s = ds[k]
        assert opened == [str(v) for v in gold["names:%d:opened" % k]]
        assert s["label"] == int(gold["names:%d:label" % k])


# ---------------------------------------------------------------- GPU (through the C-ABI)

@pytest.mark.gpu
def test_gpu_face_batcher_golden(gpu, gold):
    import DataAndDataset as DD
    n = _ntest(gold)
    img = torch.from_numpy(np.stack([gold["test:%d:u8_128" % k] for k in range(n)])).to(gpu)
    lm = torch.from_numpy(np.stack([gold["test:%d:lm68" % k] for k in range(n)])).to(gpu)
    wh = np.stack([gold["test:%d:wh" % k] for k in range(n)]).astype(np.float64)
    scale = torch.from_numpy((128.0 / wh).astype(np.float32)).to(gpu)
    out = DD.FaceBatcher(gpu)(img, lm, scale)
    torch.cuda.synchronize()
    for k in range(n):
        for name in DD.PATCH_NAMES:
            np.testing.assert_array_equal(out[name][k].cpu().numpy(), gold["test:%d:%s" % (k, name)],
                                          err_msg="%d %s" % (k, name))
    np.testing.assert_array_equal(out["I128"][0].cpu().numpy(), gold["test:0:img"])


@pytest.mark.gpu
def test_gpu_landmarks_vs_oracle(gpu, gold):
    import DataAndDataset as DD
    rng = np.random.default_rng(5)
    B = 257
    lm = (rng.random((B, 68, 2)) * 160 - 16).astype(np.float32)
    lm[: B // 2] = np.floor(lm[: B // 2])
    scale = (rng.random((B, 2)) * 1.5 + 0.25).astype(np.float32)
    for table in (DD.FIVE_PTS_IDX_REPAIRED, DD.FIVE_PTS_IDX_REFERENCE):
        fb = DD.FaceBatcher(gpu, pts_idx=table)
        lm5, boxes, status = fb.landmark_boxes(torch.from_numpy(lm).to(gpu), torch.from_numpy(scale).to(gpu))
        lm5, boxes, status = lm5.cpu().numpy(), boxes.cpu().numpy(), status.cpu().numpy()
        for b in range(B):
            ref5 = DO.five_points(lm[b], table)
            ref5[:, 0] = (ref5[:, 0] * scale[b, 0]).astype(np.float32)
            ref5[:, 1] = (ref5[:, 1] * scale[b, 1]).astype(np.float32)
            np.testing.assert_array_equal(lm5[b], ref5)
            if table is DD.FIVE_PTS_IDX_REFERENCE:
                assert status[b] == 1
                continue
            assert status[b] == 0
            rb = DO.crop_boxes(ref5)
            np.testing.assert_array_equal(boxes[b], np.array([rb[n] for n in DD.PATCH_NAMES], np.int32))


@pytest.mark.gpu
def test_gpu_reference_table_raises(gpu, gold):
    import DataAndDataset as DD
    img = torch.from_numpy(gold["test:0:u8_128"][None]).to(gpu)
    lm = torch.from_numpy(gold["test:0:lm68"][None]).to(gpu)
    with pytest.raises(ValueError):
        DD.FaceBatcher(gpu, pts_idx=DD.FIVE_PTS_IDX_REFERENCE)(img, lm)


@pytest.mark.gpu
def test_gpu_crops_random_batch(gpu):
    """Large batch with faces anywhere (crops partly or wholly outside the image), f32 exact and
    bf16 equal to torch's round-to-nearest-even of the f32 values."""
    import DataAndDataset as DD
    rng = np.random.default_rng(11)
    B = 96
    img = (rng.random((B, 128, 128, 3)) * 256).astype(np.uint8)
    lm = (rng.random((B, 68, 2)) * 200 - 36).astype(np.float32)
    out = DD.FaceBatcher(gpu)(torch.from_numpy(img).to(gpu), torch.from_numpy(lm).to(gpu))
    outb = DD.FaceBatcher(gpu, dtype=torch.bfloat16)(torch.from_numpy(img).to(gpu), torch.from_numpy(lm).to(gpu))
    torch.cuda.synchronize()
    for b in range(0, B, 7):
        ref = DO.crop_normalize(img[b], DO.crop_boxes(DO.five_points(lm[b], DO.FIVE_PTS_IDX_REPAIRED)))
        for name in DD.PATCH_NAMES:
            np.testing.assert_array_equal(out[name][b].cpu().numpy(), ref[name])
            assert torch.equal(outb[name][b].cpu(), torch.from_numpy(ref[name]).to(torch.bfloat16))
        np.testing.assert_array_equal(out["I128"][b].cpu().numpy(), DO.to_unit(img[b]))


@pytest.mark.gpu
def test_gpu_normalize_all_bytes(gpu):
    import DataAndDataset as DD
    v = np.arange(256, dtype=np.uint8).reshape(1, 16, 16, 1).repeat(3, axis=3)
    got = DD.FaceBatcher(gpu).normalize(torch.from_numpy(v).to(gpu)).cpu().numpy()
    np.testing.assert_array_equal(got, DO.to_unit(v[0])[None])


@pytest.mark.gpu
def test_gpu_empty_batch(gpu):
    import DataAndDataset as DD
    fb = DD.FaceBatcher(gpu)
    out = fb(torch.zeros(0, 128, 128, 3, dtype=torch.uint8, device=gpu), torch.zeros(0, 68, 2, device=gpu))
    assert out["left_eye"].shape == (0, 3, 40, 40)


@pytest.mark.gpu
def test_gpu_face_batcher_rejects_host_tensors(gpu):
    """Raw pointers go to the kernels: CPU inputs (TrainDataset(raw=True), numpy) must raise,
    not hand the GPU a host address."""
    import DataAndDataset as DD
    fb = DD.FaceBatcher(gpu)
    img = torch.zeros(2, 128, 128, 3, dtype=torch.uint8)
    lm = torch.full((2, 68, 2), 64.0)
    with pytest.raises(ValueError, match="must be on"):
        fb(img, lm.to(gpu))
    with pytest.raises(ValueError, match="must be on"):
        fb(img.to(gpu), lm)
    with pytest.raises(ValueError, match="must be on"):
        fb.landmark_boxes(lm.to(gpu), torch.ones(2, 2))
    with pytest.raises(ValueError, match="must be on"):
        fb.normalize(img)
    out = DD.FaceBatcher("cuda")(img.to(gpu), lm.to(gpu))  # "cuda" means the current device
    assert out["I128"].device == gpu
