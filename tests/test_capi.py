"""CPU: the C-ABI library (tp-gan_amd/libtpgan_hip.so) loads without a GPU, exports every
function include/tpgan.h declares, and its host-side planner (workspace sizing and
descriptor validation, no device work) behaves."""
import ctypes
import os
import re

import pytest

import tpgan_lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "tpgan.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tpg_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(L.LIB_PATH):
        pytest.skip("libtpgan_hip.so not built")
    lib = ctypes.CDLL(L.LIB_PATH)
    for name, (res, args) in L.EXPORTS.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def test_header_matches_binding():
    assert header_functions() == sorted(L.EXPORTS), "tpgan_lib.EXPORTS must bind exactly the header's functions"


def test_exports(lib):
    for name in header_functions():
        assert hasattr(lib, name), name
    assert lib.tpg_version().decode().startswith("tpgan_hip")


def _desc(n, cin, h, w, cout, k, s, p, transposed=False, op=0, reflect=False, dtype=L.TPG_BF16):
    d = L.ConvDesc()
    d.n, d.in_c, d.in_h, d.in_w, d.out_c = n, cin, h, w, cout
    if transposed:
        d.out_h = (h - 1) * s - 2 * p + k + op
        d.out_w = (w - 1) * s - 2 * p + k + op
    elif reflect:
        d.out_h, d.out_w = h, w
    else:
        d.out_h = (h + 2 * p - k) // s + 1
        d.out_w = (w + 2 * p - k) // s + 1
    d.kh = d.kw = k
    d.stride_h = d.stride_w = s
    if reflect:
        d.pad_t, d.pad_b, d.pad_l, d.pad_r = 1, 0, 1, 0
        d.pad_mode = L.PAD_REFLECT
    else:
        d.pad_t = d.pad_b = d.pad_l = d.pad_r = p
    d.transposed = 1 if transposed else 0
    d.dtype = dtype
    d.act = L.ACT_LEAKY
    d.slope = 0.01
    d.res_scale = 1.0
    return d


# every conv shape class of G + D at bs32
SHAPES = [
    (32, 206, 128, 128, 206, 5, 1, 2, False, 0, False),
    (32, 75, 128, 128, 75, 7, 1, 3, False, 0, False),
    (32, 3, 128, 128, 64, 7, 1, 3, False, 0, False),
    (32, 64, 128, 128, 64, 5, 2, 2, False, 0, False),
    (32, 576, 8, 8, 576, 2, 1, 0, False, 0, True),
    (32, 576, 8, 8, 512, 3, 2, 1, True, 1, False),
    (32, 64, 8, 8, 32, 3, 4, 0, True, 1, False),
    (32, 320, 1, 1, 64, 8, 1, 0, True, 0, False),
    (32, 512, 8, 8, 512, 8, 1, 0, False, 0, False),
    (32, 512, 4, 4, 1, 3, 1, 1, False, 0, False),
    (32, 3, 40, 40, 64, 3, 1, 1, False, 0, False),
]


@pytest.mark.parametrize("shape", SHAPES, ids=[str(i) for i in range(len(SHAPES))])
@pytest.mark.parametrize("dtype", [L.TPG_F32, L.TPG_BF16])
def test_workspace_sizes(lib, shape, dtype):
    n, cin, h, w, cout, k, s, p, tr, op, refl = shape
    d = _desc(n, cin, h, w, cout, k, s, p, tr, op, refl, dtype)
    for op_ in (L.OP_FWD, L.OP_BWD_DATA, L.OP_BWD_FILTER):
        ws = lib.tpg_conv2d_workspace(ctypes.byref(d), op_)
        assert ws > 0, (shape, op_, lib.tpg_last_error())
    # the packed weights alone need at least the weight tensor in the compute dtype
    esize = 2 if dtype == L.TPG_BF16 else 4
    assert lib.tpg_conv2d_workspace(ctypes.byref(d), L.OP_FWD) >= cin * cout * k * k * esize


def test_bad_descriptors(lib):
    d = _desc(2, 16, 8, 8, 16, 3, 1, 1)
    d.out_h = 9  # inconsistent with the geometry
    assert lib.tpg_conv2d_workspace(ctypes.byref(d), L.OP_FWD) == 0
    assert b"Conv2d output" in lib.tpg_last_error()
    d = _desc(2, 16, 8, 8, 16, 3, 1, 1)
    d.dtype = 7
    assert lib.tpg_conv2d_workspace(ctypes.byref(d), L.OP_FWD) == 0
    assert b"dtype" in lib.tpg_last_error()
    d = _desc(2, 16, 8, 8, 16, 9, 1, 4)  # 81 taps > 64
    assert lib.tpg_conv2d_workspace(ctypes.byref(d), L.OP_FWD) == 0
    d = _desc(2, 16, 4, 4, 16, 3, 2, 1, transposed=True, op=1)
    d.pad_mode = L.PAD_REFLECT
    assert lib.tpg_conv2d_workspace(ctypes.byref(d), L.OP_FWD) == 0
    assert b"reflect" in lib.tpg_last_error()
    # a kernel larger than the padded input: C's truncating division gives a "consistent"
    # 0- or 1-pixel output that torch rejects (the 0-pixel case divided by zero in the planner)
    for k, s in ((3, 2), (3, 3)):
        d = _desc(2, 16, 1, 1, 16, k, s, 0)
        assert lib.tpg_conv2d_workspace(ctypes.byref(d), L.OP_FWD) == 0
        assert b"larger than the padded input" in lib.tpg_last_error() or b"empty" in lib.tpg_last_error()


def test_null_tensor_rejected_without_device_work(lib):
    d = _desc(2, 16, 8, 8, 16, 3, 1, 1)
    z = L.TpgTensor()
    rc = lib.tpg_conv2d_fwd(ctypes.byref(d), z, z, None, z, z, None, 0, None)
    assert rc < 0 and b"NULL" in lib.tpg_last_error()


def test_planner_sanitizer_sweep():
    """The planner (descriptor validation, plans, workspace and pre-pack sizing) rebuilt with
    host AddressSanitizer + UBSan and driven over TP-GAN's layer shapes, a seeded random walk of
    geometries and malformed descriptors (tools/planner_asan.cpp).  The sweep first found a
    divide-by-zero on a 0-pixel Conv2d output, now rejected by check_desc."""
    import shutil
    import subprocess
    src = os.path.join(REPO, "tp-gan_amd")
    objs = [os.path.join(src, "build", f) for f in os.listdir(os.path.join(src, "build"))
            if f.endswith(".o")] if os.path.isdir(os.path.join(src, "build")) else []
    if not shutil.which("/opt/rocm/bin/hipcc") or len(objs) < 8:
        pytest.skip("needs hipcc and the built kernel objects (make -C tp-gan_amd)")
    r = subprocess.run(["make", "-s", "-C", src, "asan"], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(src, "build", "asan", "planner_asan"), "20000"], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ok" in r.stdout and "ERROR" not in r.stderr, r.stdout + r.stderr[-4000:]
