"""CPU restatement of the reference's data path — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may use this module, and only
as the checker.  Pinned to the reference by tests/golden/data_golden.npz
(tests/golden/make_golden_data.py runs the reference's own functions).

  five_points      UtilityMethods.get_5_landmarks_pixal_position (UtilityMethods.py:148-164)
  rescale          TestDataset's `lm[i][k] *= 128/img.width|height` (DataAndDataset.py:244-246)
  crop_boxes       process() (DataAndDataset.py:42-54): mouth midpoint, floor, PIL box
  crop_normalize   PIL crop (zero fill outside) + ToTensor + x*2-1 (DataAndDataset.py:51-54,252-255)
  multipie_paths   TrainDataset.__getitem__ file naming and label (DataAndDataset.py:200-226)
"""
import math

import numpy as np

FIVE_PTS_IDX_REFERENCE = [[36, 41], [42, 47], [27, 35], [48, 48], [68, 68]]  # UtilityMethods.py:148
FIVE_PTS_IDX_REPAIRED = [[36, 41], [42, 47], [27, 35], [48, 48], [54, 54]]   # R5: right mouth corner
PATCH_NAMES = ["left_eye", "right_eye", "nose", "mouth"]                       # DataAndDataset.py:33
PATCH_WH = {"left_eye": (40, 40), "right_eye": (40, 40), "nose": (40, 32), "mouth": (48, 32)}  # :35-40


def five_points(lm68, pts_idx=FIVE_PTS_IDX_REFERENCE):
    """(68, 2) float32 -> (5, 2) float32: per range, float32 row sums in index order / count
    (numpy's mean over axis 0); an empty slice gives NaN (UtilityMethods.py:160-164)."""
    x = np.asarray(lm68, np.float32)
    out = np.empty((5, 2), np.float32)
    for j, (a, b) in enumerate(pts_idx):
        rows = x[a:b + 1]
        if len(rows) == 0:
            out[j] = np.nan
            continue
        acc = np.zeros(2, np.float32)
        for r in rows:
            acc = (acc + r).astype(np.float32)
        out[j] = (acc / np.float32(len(rows))).astype(np.float32)
    return out


def rescale(lm5, width, height, size=128):
    """DataAndDataset.py:244-246: float32 points times the float32-rounded size/width (numpy 2
    casts the weak Python float to the array's float32)."""
    out = np.array(lm5, np.float32)
    out[:, 0] = (out[:, 0] * np.float32(size / width)).astype(np.float32)
    out[:, 1] = (out[:, 1] * np.float32(size / height)).astype(np.float32)
    return out


def crop_boxes(lm5):
    """process() :42-54 -> {name: (left, upper, right, lower)}; math.floor raises on NaN
    (ValueError), as the reference does."""
    p = np.array(lm5, np.float32)
    p[3, 0] = np.float32((p[3, 0] + p[4, 0]) / np.float32(2.0))
    p[3, 1] = np.float32((p[3, 1] + p[4, 1]) / np.float32(2.0))
    boxes = {}
    for i, name in enumerate(PATCH_NAMES):
        x, y = math.floor(p[i, 0]), math.floor(p[i, 1])
        w, h = PATCH_WH[name]
        boxes[name] = (x - w // 2 + 1, y - h // 2 + 1, x + w // 2 + 1, y + h // 2 + 1)
    return boxes


def crop_u8(img_hwc, box):
    """PIL Image.crop: pixels outside the image are 0."""
    l, u, r, d = box
    H, W, C = img_hwc.shape
    out = np.zeros((d - u, r - l, C), np.uint8)
    y0, y1, x0, x1 = max(u, 0), min(d, H), max(l, 0), min(r, W)
    if y1 > y0 and x1 > x0:
        out[y0 - u:y1 - u, x0 - l:x1 - l] = img_hwc[y0:y1, x0:x1]
    return out


def to_unit(img_hwc_u8):
    """ToTensor (u8 / 255 in float32, CHW) then * 2.0 - 1.0 (DataAndDataset.py:219-220)."""
    t = np.asarray(img_hwc_u8).astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    return (t * np.float32(2.0) - np.float32(1.0)).astype(np.float32)


def crop_normalize(img_hwc_u8, boxes):
    return {k: to_unit(crop_u8(img_hwc_u8, boxes[k])) for k in PATCH_NAMES}


def multipie_paths(path):
    """TrainDataset.__getitem__ (:202-215, 226): the 14 files one sample opens, and the label.
    The frontal view replaces the camera field (second-to-last '_' field) with '051'."""
    img_name = path.split("/")
    fr = path.split("_")
    fr[-2] = "051"
    fr = "_".join(fr).split("/")
    paths = {"img": "/".join(img_name),
             "img32": "/".join(img_name[:-2] + ["32x32", img_name[-1]]),
             "img64": "/".join(img_name[:-2] + ["64x64", img_name[-1]]),
             "img_frontal": "/".join(fr),
             "img32_frontal": "/".join(fr[:-2] + ["32x32", fr[-1]]),
             "img64_frontal": "/".join(fr[:-2] + ["64x64", fr[-1]])}
    for p in PATCH_NAMES:
        paths[p] = "/".join(img_name[:-2] + ["patch", p, img_name[-1]])
        paths[p + "_frontal"] = "/".join(fr[:-2] + ["patch", p, fr[-1]])
    label = int(path.split("/")[-1].split("_")[0])
    return paths, label
