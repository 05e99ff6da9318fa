"""Diagnostic runner (not product, not a test): tools/bench_variant.py with a native crash
handler installed first (tools/crashtrace.c: faulting address + backtrace of library offsets
on SIGSEGV / SIGBUS / SIGABRT) and the load addresses of the HIP runtime printed, for locating
the round-5 identity side-stream crashes in hipGraphLaunch / hipStreamEndCapture.

    python tools/crash_probe.py <bench_variant args> -- <bench.py args>
"""
import ctypes
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    so = os.path.join(HERE, "crashtrace.so")
    if not os.path.exists(so):
        subprocess.run(["gcc", "-O1", "-g", "-shared", "-fPIC", "-o", so, os.path.join(HERE, "crashtrace.c")],
                       check=True)
    ctypes.CDLL(so).crashtrace_install()
    sys.path.insert(0, HERE)
    import bench_variant
    import torch
    torch.cuda.init()
    ctypes.CDLL(so).crashtrace_install()  # (again, after the runtime initialised)
    with open("/proc/self/maps") as f:  # (where the stripped runtime libraries are mapped)
        for line in f:
            if ("libamdhip64" in line or "libhsa-runtime" in line) and " r-xp " in line:
                print("crashtrace map:", line.strip(), file=sys.stderr, flush=True)
    bench_variant.main()


if __name__ == "__main__":
    main()
