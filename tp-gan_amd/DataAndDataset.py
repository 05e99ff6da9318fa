"""Data path of the reference (DataAndDataset.py), with the per-sample landmark -> crop ->
normalise work moved onto the GPU for whole batches.

Reference API kept (same names, arguments, return values, errors):
  process(img, landmarks_5pts)       DataAndDataset.py:10-56 (PIL crop on the host)
  PretrainDataset / TrainDataset / TestDataset   :60-256 (file IO stays on the host; torchvision
                                     is not installed, so ToTensor is `_to_tensor` below)

Device path (no per-sample Python, no host synchronisation unless `check=True`):
  FaceBatcher(device)(img_u8, lm68, scale=None) -> {"I128", "left_eye", "right_eye", "nose", "mouth"}
      img_u8  uint8 [B, H, W, 3] device tensor (the 128x128 faces, HWC as PIL stores them)
      lm68    float32 [B, 68, 2] device landmarks; scale float32 [B, 2] (TestDataset's 128/size)
    tpg_landmark_boxes computes the five points and the four PIL crop boxes per face and
    tpg_crop_normalize writes the image and the four patches, u8/255*2-1, in ONE launch.
  FaceBatcher.normalize(img_u8) -> the [-1, 1] image alone (TrainDataset's pre-cropped files:
    ship u8 over PCIe, 1/4 of the float32 bytes, normalise on the device).

The reference's five-point table ends with [68, 68] (UtilityMethods.py:148), past the 68
landmarks: the mouth's right corner is NaN and math.floor raises ValueError in process(), so
its TestDataset cannot return a sample.  FaceBatcher defaults to the repaired table (R5: index 54,
dlib's right mouth corner); pass pts_idx=FIVE_PTS_IDX_REFERENCE to get the
reference's behaviour, ValueError included (check=True).
"""
import ctypes
import math
import os

import numpy as np
import torch
from torch.utils.data import Dataset

import tpgan_lib as L
from UtilityMethods import get_5_landmarks_pixal_position

FIVE_PTS_IDX_REFERENCE = [[36, 41], [42, 47], [27, 35], [48, 48], [68, 68]]
FIVE_PTS_IDX_REPAIRED = [[36, 41], [42, 47], [27, 35], [48, 48], [54, 54]]
PATCH_NAMES = ["left_eye", "right_eye", "nose", "mouth"]
PATCH_SIZE = {"left_eye": (40, 40), "right_eye": (40, 40), "nose": (40, 32), "mouth": (48, 32)}  # (w, h)


def _to_tensor(pic):
    """torchvision ToTensor for u8 images: HWC u8 -> CHW float32 / 255."""
    a = np.asarray(pic)
    if a.ndim == 2:
        a = a[:, :, None]
    return torch.from_numpy(a.copy()).permute(2, 0, 1).contiguous().to(torch.float32).div(255)


def process(img, landmarks_5pts):
    """Crop the four landmark patches from a PIL image (DataAndDataset.py:10-56).
    landmarks_5pts (5, 2) is modified in place (row 3 becomes the mouth midpoint), as in the reference."""
    batch = {}
    landmarks_5pts[3, 0] = (landmarks_5pts[3, 0] + landmarks_5pts[4, 0]) / 2.0
    landmarks_5pts[3, 1] = (landmarks_5pts[3, 1] + landmarks_5pts[4, 1]) / 2.0
    for i, name in enumerate(PATCH_NAMES):
        x = math.floor(landmarks_5pts[i, 0])
        y = math.floor(landmarks_5pts[i, 1])
        w, h = PATCH_SIZE[name]
        batch[name] = img.crop((x - w // 2 + 1, y - h // 2 + 1, x + w // 2 + 1, y + h // 2 + 1))
    return batch


class PretrainDataset(Dataset):
    """(image [0, 1] CHW, 8 landmark coordinates) for the MobileNetV2 landmark pretraining
    (DataAndDataset.py:60-95)."""

    def __init__(self, txt_name, data_root_dir):
        self.labels = _getPretrainLabelGroups(txt_name, data_root_dir)
        self.image_names = _getPretrainImageFullPaths(data_root_dir)

    def __len__(self):
        return len(self.image_names)

    def __getitem__(self, idx):
        from PIL import Image
        img_path = self.image_names[idx]
        img_name = img_path.split("\\")[-1]
        with Image.open(img_path).convert("RGB") as img:
            image = _to_tensor(img)
        g = self.labels[img_name]
        return image, torch.tensor([g[0][0], g[0][1], g[1][0], g[1][1], g[2][0], g[2][1], g[3][0], g[3][1]],
                                   dtype=torch.float32)


def _getPretrainLabelGroups(txt_name, data_root_dir):
    """CelebA-style landmark file -> {name: [(lx, ly), (rx, ry), (nx, ny), (mx, my)]}, mouth =
    integer midpoint of the corners (DataAndDataset.py:97-153)."""
    out = {}
    with open(os.path.join(data_root_dir, txt_name)) as f:
        next(f)
        next(f)
        for line in f:
            p = line.split()
            v = [int(t) for t in p[1:11]]
            out[p[0]] = [(v[0], v[1]), (v[2], v[3]), (v[4], v[5]), ((v[6] + v[8]) // 2, (v[7] + v[9]) // 2)]
    return out


def _getPretrainImageFullPaths(data_root_path):
    """Every *.jpg under the root, os.walk order (DataAndDataset.py:155-176)."""
    out = []
    for root, _, files in os.walk(data_root_path):
        for fn in files:
            if fn.lower().endswith(".jpg"):
                out.append(os.path.join(root, fn))
    return out


def multipie_paths(path):
    """The files one Multi-PIE sample is made of, and its identity label (DataAndDataset.py:200-226):
    the frontal view replaces the camera field (second-to-last '_' field) with '051'."""
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
    return paths, int(path.split("/")[-1].split("_")[0])


class TrainDataset(Dataset):
    """Multi-PIE sample: 14 images in [-1, 1] and the identity label (DataAndDataset.py:179-227).
    raw=True returns the u8 HWC arrays instead, for FaceBatcher.normalize on the device."""

    def __init__(self, img_list, raw=False):
        super().__init__()
        self.img_list = img_list
        self.raw = raw

    def __len__(self):
        return len(self.img_list)

    def __getitem__(self, idx):
        from PIL import Image
        paths, label = multipie_paths(self.img_list[idx])
        batch = {}
        for k, p in paths.items():
            img = Image.open(p)
            batch[k] = np.asarray(img) if self.raw else _to_tensor(img) * 2.0 - 1.0
        batch["label"] = label
        return batch


class TestDataset(Dataset):
    """Profile image + 68 landmarks -> 128x128 image, patches, 64/32 images in [-1, 1]
    (DataAndDataset.py:230-256).  pts_idx selects the five-point table (reference: NaN mouth
    corner -> ValueError)."""

    def __init__(self, img_list, lm_list, pts_idx=None):
        super().__init__()
        self.img_list = img_list
        self.lm_list = lm_list
        self.pts_idx = pts_idx
        assert len(img_list) == len(lm_list)

    def __len__(self):
        return len(self.img_list)

    def __getitem__(self, idx):
        from PIL import Image
        import UtilityMethods as UM
        img = Image.open(self.img_list[idx])
        lm = np.array(self.lm_list[idx].split(" "), np.float32).reshape(-1, 2)
        saved = [list(v) for v in UM.five_pts_idx]
        if self.pts_idx is not None:
            UM.five_pts_idx[:] = [list(v) for v in self.pts_idx]
        try:
            lm = get_5_landmarks_pixal_position(lm)
        finally:
            UM.five_pts_idx[:] = saved
        for i in range(5):
            lm[i][0] *= 128 / img.width
            lm[i][1] *= 128 / img.height
        img = img.resize((128, 128), Image.LANCZOS)
        batch = process(img, lm)
        batch["img"] = img
        batch["img64"] = img.resize((64, 64), Image.LANCZOS)
        batch["img32"] = batch["img64"].resize((32, 32), Image.LANCZOS)
        for k in batch:
            batch[k] = _to_tensor(batch[k]) * 2.0 - 1.0
        return batch


class FaceBatcher:
    """Whole-batch landmark crops and [-1, 1] normalisation on the GPU (tpg_landmark_boxes +
    tpg_crop_normalize).  Outputs are logical NCHW tensors of `dtype` (float32 default, what the
    train step's batch holds)."""

    def __init__(self, device, dtype=torch.float32, pts_idx=FIVE_PTS_IDX_REPAIRED, check=True):
        self.lib = L.load()
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.dtype = dtype
        self.check = check
        self._idx = (ctypes.c_int32 * 10)(*[v for r in pts_idx for v in r])
        self._wh = (ctypes.c_int32 * 8)(*[v for n in PATCH_NAMES for v in PATCH_SIZE[n]])

    def _on_device(self, t, name):
        """The kernels take raw pointers: a tensor on another device (e.g. the CPU output of
        TrainDataset(raw=True) or numpy) would hand them a host address."""
        if t.device != self.device:
            raise ValueError("%s must be on %s (FaceBatcher's device), got %s" % (name, self.device, t.device))

    def landmark_boxes(self, lm68, scale=None):
        """-> (lm5 float32 [B, 5, 2], boxes int32 [B, 4, 4] (left, upper, right, lower), status int32 [B])."""
        if lm68.dtype != torch.float32 or lm68.dim() != 3 or lm68.shape[2] != 2:
            raise ValueError("lm68 must be float32 [B, npts, 2]")
        self._on_device(lm68, "lm68")
        if scale is not None:
            self._on_device(scale, "scale")
        lm68 = lm68.contiguous()
        B = lm68.shape[0]
        lm5 = torch.empty(B, 5, 2, dtype=torch.float32, device=self.device)
        boxes = torch.empty(B, 4, 4, dtype=torch.int32, device=self.device)
        status = torch.empty(B, dtype=torch.int32, device=self.device)
        if scale is not None:
            if scale.dtype != torch.float32 or tuple(scale.shape) != (B, 2):
                raise ValueError("scale must be float32 [B, 2]")
            scale = scale.contiguous()
        with torch.cuda.device(self.device):  # the launch goes to this device's current stream
            L.check(self.lib.tpg_landmark_boxes(B, lm68.shape[1], lm68.data_ptr(),
                                                scale.data_ptr() if scale is not None else None, self._idx, self._wh,
                                                lm5.data_ptr(), boxes.data_ptr(), status.data_ptr(), L.stream_ptr()))
        return lm5, boxes, status

    def _crop(self, img_u8, jobs, boxes):
        if img_u8.dtype != torch.uint8 or img_u8.dim() != 4:
            raise ValueError("img_u8 must be uint8 [B, H, W, C]")
        self._on_device(img_u8, "img_u8")
        B, H, W, C = img_u8.shape
        s = img_u8.stride()
        strides = (ctypes.c_int64 * 4)(s[0], s[3], s[1], s[2])  # logical (n, c, h, w)
        outs, hw, slots, res = (L.TpgTensor * len(jobs))(), (ctypes.c_int32 * (2 * len(jobs)))(), \
            (ctypes.c_int32 * len(jobs))(), {}
        for k, (name, h, w, slot) in enumerate(jobs):
            t = torch.empty(B, C, h, w, dtype=self.dtype, device=self.device)
            res[name] = t
            outs[k] = L.tt(t)
            hw[2 * k], hw[2 * k + 1], slots[k] = h, w, slot
        with torch.cuda.device(self.device):
            L.check(self.lib.tpg_crop_normalize(B, C, H, W, img_u8.data_ptr(), strides, len(jobs), outs, hw, slots,
                                                boxes.data_ptr() if boxes is not None else None, 16, L.stream_ptr()))
        return res

    def normalize(self, img_u8, name="I128"):
        B, H, W, C = img_u8.shape
        return self._crop(img_u8, [(name, H, W, -1)], None)[name]

    def __call__(self, img_u8, lm68, scale=None):
        lm5, boxes, status = self.landmark_boxes(lm68, scale)
        if self.check and bool((status != 0).any()):
            raise ValueError("cannot convert float NaN to integer (landmark point is NaN; five-point table %s)"
                             % list(self._idx))
        B, H, W, C = img_u8.shape
        jobs = [("I128", H, W, -1)] + [(n, PATCH_SIZE[n][1], PATCH_SIZE[n][0], i) for i, n in enumerate(PATCH_NAMES)]
        out = self._crop(img_u8, jobs, boxes)
        out["boxes"] = boxes
        return out
