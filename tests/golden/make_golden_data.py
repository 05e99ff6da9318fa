"""Golden fixtures for the data path, made by running the REFERENCE's own
functions here (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_data.py

torchvision (imported by DataAndDataset.py:3 / UtilityMethods.py:9) is not installed: it is
stubbed, and transforms.ToTensor is given torchvision's documented u8 behaviour (HWC u8 ->
CHW float32 / 255).  Recorded:
  five:*      get_5_landmarks_pixal_position on float and integer landmark sets, with the
              reference's index table (last point NaN) and with R5 (index 54)
  test:*      TestDataset.__getitem__ end to end on images written to a temp dir (LANCZOS resize
              to 128, landmark rescale, process() crops, [-1, 1] tensors) with R5, plus the
              128x128 u8 image it cropped from, so the device path can start from the same bytes
  test_raises TestDataset with the reference's table raises ValueError (floor of NaN)
  names:*     the 14 paths TrainDataset.__getitem__ opens and its label
"""
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402


def _stub_torchvision():
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")

    class ToTensor:
        def __call__(self, pic):
            a = np.asarray(pic)
            if a.ndim == 2:
                a = a[:, :, None]
            return torch.from_numpy(a.copy()).permute(2, 0, 1).contiguous().to(torch.float32).div(255)

    tvt.ToTensor = ToTensor
    tv.transforms = tvt
    sys.modules.setdefault("torchvision", tv)
    sys.modules.setdefault("torchvision.transforms", tvt)
    sys.path.insert(0, REF)


def main():
    _stub_torchvision()
    import UtilityMethods as UM
    import DataAndDataset as DD

    rng = np.random.default_rng(20260117)
    rec = {}
    ref_idx = [list(v) for v in UM.five_pts_idx]
    # 1. five points
    lm_f = (rng.random((6, 68, 2)) * 250).astype(np.float32)
    lm_i = np.floor(rng.random((6, 68, 2)) * 250).astype(np.float32)
    lm = np.concatenate([lm_f, lm_i])
    rec["five:lm68"] = lm
    rec["five:ref"] = np.stack([UM.get_5_landmarks_pixal_position(x) for x in lm])
    UM.five_pts_idx[4] = [54, 54]
    rec["five:r5"] = np.stack([UM.get_5_landmarks_pixal_position(x) for x in lm])

    # 2. TestDataset end to end (R5 table), images of several sizes, faces near the borders
    sizes = [(128, 128), (150, 170), (96, 110), (200, 140)]
    with tempfile.TemporaryDirectory() as td:
        paths, lms = [], []
        for k, (w, h) in enumerate(sizes):
            img = (rng.random((h, w, 3)) * 256).astype(np.uint8)
            p = os.path.join(td, "face%d.png" % k)
            Image.fromarray(img).save(p)
            paths.append(p)
            base = rng.random((68, 2)) * np.array([w, h])
            if k == 1:
                base[36:48] = [[2.0, 3.0]] * 12  # eyes at the top-left corner: crops leave the image
            if k == 3:
                base[27:36] = [[w - 1.5, h - 0.5]] * 9
            lms.append(" ".join("%.3f" % v for v in base.astype(np.float32).reshape(-1)))
        ds = DD.TestDataset(paths, lms)
        for k in range(len(paths)):
            b = ds[k]
            for key in ("left_eye", "right_eye", "nose", "mouth", "img"):
                if key == "img" and k:
                    continue  # one whole-image tensor pins ToTensor*2-1; the rest is the same map
                rec["test:%d:%s" % (k, key)] = b[key].numpy()
            img = Image.open(paths[k])
            rec["test:%d:u8_128" % k] = np.asarray(img.resize((128, 128), Image.LANCZOS))
            rec["test:%d:lm68" % k] = np.array(lms[k].split(" "), np.float32).reshape(-1, 2)
            rec["test:%d:wh" % k] = np.array([img.width, img.height], np.int32)
        UM.five_pts_idx[4] = ref_idx[4]
        try:
            ds[0]
            rec["test_raises"] = np.array(0)
        except ValueError:
            rec["test_raises"] = np.array(1)

    # 3. Multi-PIE naming: record what TrainDataset opens
    names = ["/data/mpie/128x128/001_01_01_010_05.png", "root/session/128x128/250_02_01_140_11.png",
             "a/b/c/128x128/346_04_02_190_19.png"]
    opened = []

    def fake_open(p):
        opened.append(p)
        return Image.fromarray(np.zeros((2, 2, 3), np.uint8))

    real_open = DD.Image.open
    DD.Image.open = fake_open
    try:
        ds = DD.TrainDataset(names)
        for k, n in enumerate(names):
            opened.clear()
            b = ds[k]
            rec["names:%d:opened" % k] = np.array(list(opened))
            rec["names:%d:label" % k] = np.array(b["label"])
    finally:
        DD.Image.open = real_open
    rec["names:list"] = np.array(names)
    np.savez_compressed(os.path.join(HERE, "data_golden.npz"), **rec)
    print("wrote %d arrays" % len(rec))


if __name__ == "__main__":
    main()
