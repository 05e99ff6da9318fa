"""bench.py with tpgan_ops module switches set first (for same-box kernel-trace A/Bs under
rocprofv3, which must launch python3 on a script directly):

    python tools/bench_variant.py ACT_LINK=0 tpgan_train.IDENTITY_STREAM=0 -- --steps 10 --no-cpu-baseline
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tp-gan_amd")]


def main():
    argv = sys.argv[1:]
    sets = argv[:argv.index("--")] if "--" in argv else argv
    rest = argv[argv.index("--") + 1:] if "--" in argv else []
    import importlib
    for kv in sets:  # SWITCH=v (a tpgan_ops switch), module.SWITCH=v or module.SWITCH:key=v
        k, v = kv.split("=")
        k, _, key = k.partition(":")
        mod, _, name = k.rpartition(".")
        getattr(importlib.import_module(mod or "tpgan_ops"), name)[key or "enabled"] = (
            float(v) if "." in v else bool(int(v)))
    sys.argv = [os.path.join(REPO, "bench.py")] + rest
    import bench
    bench.main()


if __name__ == "__main__":
    main()
