"""Counter-based deterministic values for weights, inputs and projections.

TEST INFRASTRUCTURE (oracle/): only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this package. The product (tp-gan_amd/) never does.

The reference initialises weights through torch's RNG (`ModificationLayer.py:26-52`,
`weight_initialization`, which is broken as written — SURVEY.md R1).  Parity fixtures
must not depend on RNG call order, so every tensor used in a fixture is derived from
its *name* through a splitmix64 counter hash:

    u[i] = uniform[-1, 1) from splitmix64(fnv1a64(name) ^ seed*phi + (i+1)*phi)

Weights are scaled to variance 1/fan_in with fan_in = shape[1]*prod(shape[2:]) (torch's
own fan-in convention for Conv2d, ConvTranspose2d and Linear); biases are 0.1*u.
The product carries an identical implementation (`tp-gan_amd/tpgan_init.py`) so that a
model built by the product and one built by the reference load the same numbers.
"""
import numpy as np

_PHI = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(s: str) -> np.uint64:
    h = 0xCBF29CE484222325
    for b in s.encode("utf-8"):
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return np.uint64(h)


def det_uniform(name: str, n: int, seed: int = 0) -> np.ndarray:
    """float64 array of n values in [-1, 1), a pure function of (name, seed, index)."""
    with np.errstate(over="ignore"):
        key = fnv1a64(name) ^ (np.uint64(seed) * _PHI)
        x = key + (np.arange(1, n + 1, dtype=np.uint64) * _PHI)
        x ^= x >> np.uint64(30)
        x *= _M1
        x ^= x >> np.uint64(27)
        x *= _M2
        x ^= x >> np.uint64(31)
    return (x >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) * 2.0 - 1.0


def det_param(name: str, shape, seed: int = 0) -> np.ndarray:
    """Deterministic parameter value for a state_dict entry `name` of `shape`."""
    shape = tuple(int(s) for s in shape)
    n = int(np.prod(shape)) if shape else 1
    u = det_uniform(name, n, seed).reshape(shape)
    if name.endswith(".bias") or len(shape) == 1:
        return 0.1 * u
    fan_in = int(np.prod(shape[1:]))
    return u * np.sqrt(3.0 / fan_in)


def det_input(name: str, shape, seed: int = 0) -> np.ndarray:
    """Synthetic input in U[-1, 1) (the [-1,1] normalisation of DataAndDataset.py:220)."""
    shape = tuple(int(s) for s in shape)
    return det_uniform("input/" + name, int(np.prod(shape)), seed).reshape(shape)


def det_state_dict(named_shapes, prefix: str, seed: int = 0):
    """{key: ndarray} for an iterable of (key, shape) using name prefix + key."""
    return {k: det_param(prefix + k, s, seed) for k, s in named_shapes}


def det_bn(name: str, c: int, seed: int = 0):
    """Deterministic, well-conditioned BatchNorm2d state for `name` (a state_dict prefix):
    weight 1 + 0.25u, bias 0.1u, running_mean 0.1u, running_var in [1, 1.5)."""
    return {"weight": 1.0 + 0.25 * det_uniform(name + "weight", c, seed),
            "bias": 0.1 * det_uniform(name + "bias", c, seed),
            "running_mean": 0.1 * det_uniform(name + "running_mean", c, seed),
            "running_var": 1.25 + 0.25 * det_uniform(name + "running_var", c, seed)}


def det_module_state(module, prefix: str, seed: int = 0):
    """state_dict of `module` (torch) with det_param weights and det_bn BatchNorm states,
    as float64 numpy arrays keyed like module.state_dict() (num_batches_tracked = 0)."""
    import torch.nn as nn
    out = {}
    bn_prefixes = {n + "." if n else "": m for n, m in module.named_modules()
                   if isinstance(m, (nn.BatchNorm1d, nn.BatchNorm2d))}
    for k, v in module.state_dict().items():
        pre, leaf = (k.rsplit(".", 1) + [""])[:2] if "." in k else ("", k)
        pre = pre + "." if pre else ""
        if pre in bn_prefixes:
            if leaf == "num_batches_tracked":
                out[k] = np.zeros((), dtype=np.int64)
            else:
                out[k] = det_bn(prefix + pre, v.shape[0], seed)[leaf]
        else:
            out[k] = det_param(prefix + k, v.shape, seed)
    return out
