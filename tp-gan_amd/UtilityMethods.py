"""Helpers of the reference (UtilityMethods.py) used around the hot path.

getOptimizer / set_requires_grad / save_model / save_optimizer / EMaC2I keep the
reference's names and behaviour (UtilityMethods.py:14-121).  The landmark helpers of
the data path (:123-164) are kept for import compatibility; resize_tensor uses PIL
directly instead of torchvision (not installed here).
"""
import os

import numpy as np
import torch
from torch import optim

from config import optimizer_param


def getOptimizer(model_parameters, optimizer_name="SGD") -> optim.Optimizer:
    """Optimizer by name from config.optimizer_param; unknown names give SGD (:14-41)."""
    params = list(model_parameters)
    lr, wd = optimizer_param["learning_rate"], optimizer_param["weight_decay"]
    table = {
        "SGD": lambda: optim.SGD(params, lr=lr, weight_decay=wd, momentum=optimizer_param["momentum"],
                                 nesterov=optimizer_param.get("nesterov", False)),
        "Adam": lambda: optim.Adam(params, lr=lr, weight_decay=wd),
        "RMSprop": lambda: optim.RMSprop(params, lr=lr, weight_decay=wd, momentum=optimizer_param["momentum"]),
        "Adagrad": lambda: optim.Adagrad(params, lr=lr, weight_decay=wd),
        "Adadelta": lambda: optim.Adadelta(params, lr=lr, weight_decay=wd),
    }
    return table.get(optimizer_name, table["SGD"])()


def set_requires_grad(parameters, isGrad):
    """Freeze / unfreeze parameters (:43-56); the G-step freezes D with it."""
    for param in parameters:
        param.requires_grad = isGrad


def save_model(model, dir, epoch):
    """torch.save(state_dict) to <dir>/model_epoch_<epoch>.pth (:58-76)."""
    fn = os.path.join(dir, f"model_epoch_{epoch}.pth")
    os.makedirs(os.path.dirname(fn), exist_ok=True)
    torch.save(model.state_dict(), fn)
    print(f"saved model {fn}")


def save_optimizer(optimizer, model, dir, epoch):
    """{optimizer, model, epoch} to <dir>/optimizer_epoch_<epoch>.pth (:78-103)."""
    fn = os.path.join(dir, f"optimizer_epoch_{epoch}.pth")
    os.makedirs(os.path.dirname(fn), exist_ok=True)
    torch.save({"optimizer": optimizer.state_dict(), "model": model.state_dict(), "epoch": epoch}, fn)
    print(f"Optimizer saved to {fn}")


def elementwise_multiply_and_cast_to_int(list_x, scalar):
    """[int(v * scalar) for v in list_x] (:109-121)."""
    return [int(v * scalar) for v in list_x]


def resize_tensor(x, size, interpolation=None):
    """Resize a [C, H, W] float image in [0, 1] through PIL bilinear (:123-145)."""
    from PIL import Image
    if interpolation is None:
        interpolation = Image.BILINEAR
    if isinstance(size, int):
        h, w = x.shape[-2:]
        size = (size, int(size * w / h)) if h <= w else (int(size * h / w), size)
    arr = (x.detach().cpu().clamp(0, 1).permute(1, 2, 0).numpy() * 255.0).round().astype(np.uint8)
    img = Image.fromarray(arr.squeeze(-1) if arr.shape[-1] == 1 else arr)
    img = img.resize((size[1], size[0]), interpolation)
    out = torch.from_numpy(np.asarray(img, dtype=np.float32) / 255.0)
    return out.unsqueeze(0) if out.dim() == 2 else out.permute(2, 0, 1)


# dlib 68-point index ranges of left eye, right eye, nose, left / right mouth corner.
# The reference's last entry is [68, 68], which is past the end (NaN mean, SURVEY.md
# C17); it is kept as written so the data path behaves like the reference.
five_pts_idx = [[36, 41], [42, 47], [27, 35], [48, 48], [68, 68]]


def get_5_landmarks_pixal_position(x):
    """Mean (x, y) of each five_pts_idx range -> (5, 2) float32 (:149-164)."""
    with np.errstate(invalid="ignore"), __import__("warnings").catch_warnings():
        __import__("warnings").simplefilter("ignore")
        return np.array([np.mean(x[a:b + 1], axis=0) for a, b in five_pts_idx], np.float32)
