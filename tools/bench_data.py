"""Measure the device data path against the HBM roofline.

    python tools/bench_data.py [--batch 256] [--iters 50]

FaceBatcher on a resident batch: tpg_landmark_boxes + tpg_crop_normalize (image + 4 patches,
float32 NCHW outputs).  Algorithmic bytes per face: the 128x128x3 u8 image read once (49,152 B)
+ the float32 image written (196,608 B) + the four float32 patches written ((40*40*2 + 40*32 +
48*32) * 3 * 4 = 72,192 B) = 317,952 B; landmarks (544 B in, 224 B out) are counted too.
Timed with HIP events on the launch stream; peak 8 TB/s (MI355X_MICROARCH.md).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tp-gan_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    import DataAndDataset as DD
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    B = a.batch
    img = torch.randint(0, 256, (B, 128, 128, 3), generator=g, dtype=torch.uint8).to(dev)
    lm = (torch.rand(B, 68, 2, generator=g) * 100 + 14).to(dev)
    fb = DD.FaceBatcher(dev, check=False)
    for _ in range(3):
        fb(img, lm)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.iters):
        fb(img, lm)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    per_face = 49152 + 196608 + 72192 + 544 + 224
    gbs = per_face * B / (ms * 1e-3) / 1e9
    print(json.dumps({"op": "FaceBatcher (tpg_landmark_boxes + tpg_crop_normalize)", "batch": B,
                      "ms_per_batch": round(ms, 4), "faces_per_s": round(B / (ms * 1e-3), 1),
                      "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                                   "frac": round(gbs / 8000.0, 4), "bytes_per_face": per_face}}))


if __name__ == "__main__":
    main()
