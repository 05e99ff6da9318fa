"""Golden fixtures for the identity-feature extractors, by running the REFERENCE's
MobileNetV2 (MobileNetV2.py:122-249) in float64 here (never on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_features.py

Weights come from oracle.det_init.det_module_state (names -> values, BatchNorm states
well-conditioned), so the fixtures do not depend on torch's RNG.  Recorded, B=2 at 128x128:
  eval mode:  SSD outputs (locations, classifications), identity features
              (bottleneck 12 output, conv2 output), input gradient and per-parameter
              gradient summaries of a fixed projection of all four
  train mode: the same outputs with batch statistics, the running statistics after the
              step, input gradient and gradient summaries
and eval-mode outputs at 256x256 (B=1).  The reference's ResNet18 / FeatureExtractModel
cannot be constructed, so no ResNet fixture exists (parity unpinned).
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.det_init import det_input, det_module_state, det_uniform  # noqa: E402

REF = "/root/reference"


def proj(name, shape):
    return torch.from_numpy(det_uniform("proj/" + name, int(np.prod(shape)))).reshape(shape)


def sample_idx(name, numel, k=16):
    u = det_uniform("sample/" + name, k)
    return np.floor((u + 1.0) * 0.5 * numel).astype(np.int64).clip(0, numel - 1)


def run(model, x, tag, rec):
    feats = {}
    hooks = [model.bottlenecks[12].register_forward_hook(lambda m, i, o: feats.__setitem__("f0", o)),
             model.conv2.register_forward_hook(lambda m, i, o: feats.__setitem__("f1", o))]
    loc, cls = model(x)
    for h in hooks:
        h.remove()
    outs = {"loc": loc, "cls": cls, "f0": feats["f0"], "f1": feats["f1"]}
    loss = 0
    for k, v in outs.items():
        rec["%s:%s" % (tag, k)] = v.detach().numpy()
        loss = loss + (v * proj("mnv2/%s/%s" % (tag, k), tuple(v.shape))).sum()
    if x.requires_grad:
        loss.backward()
        rec["%s:dx" % tag] = x.grad.numpy()
        for k, p in model.named_parameters():
            g = p.grad.detach().double().reshape(-1).numpy()
            idx = sample_idx("mnv2/%s/%s" % (tag, k), g.size)
            rec["%s:gsum:%s" % (tag, k)] = np.concatenate([[np.sqrt((g * g).sum()), g.sum()], g[idx]])


def main():
    sys.path.insert(0, REF)
    import MobileNetV2 as MN
    torch.manual_seed(0)
    model = MN.MobileNetV2().double()
    st = det_module_state(model, "mnv2/")
    model.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    rec = {"keys": np.array(list(model.state_dict().keys()))}
    x = torch.from_numpy(det_input("mnv2/x128", (2, 3, 128, 128))).requires_grad_(True)
    rec["in:x128"] = x.detach().numpy()
    model.eval()
    run(model, x, "eval", rec)
    x256 = torch.from_numpy(det_input("mnv2/x256", (1, 3, 256, 256)))
    rec["in:x256"] = x256.numpy()
    with torch.no_grad():
        run(model, x256, "eval256", rec)
    model.zero_grad()
    model.train()
    x2 = x.detach().clone().requires_grad_(True)
    run(model, x2, "train", rec)
    for k, v in model.state_dict().items():
        if k.endswith("running_mean") or k.endswith("running_var"):
            rec["train:state:" + k] = v.numpy()
    store = {k: (np.asarray(v).astype(np.float32) if (np.asarray(v).dtype == np.float64 and np.asarray(v).size > 4096
                                                    and ":gsum:" not in k and not k.startswith("in:")) else np.asarray(v))
             for k, v in rec.items()}
    np.savez_compressed(os.path.join(HERE, "features_golden.npz"), **store)
    print("features fixtures:", len(store))


if __name__ == "__main__":
    main()
