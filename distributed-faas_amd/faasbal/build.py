"""Build libfaasbal.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
SOURCES = ["faasbal_kernels.hip", "faasbal_api.hip"]
OUT = os.path.join(HERE, "libfaasbal.so")
ARCH = os.environ.get("FAASBAL_ARCH", "gfx950")


def build_lib(verbose=False, out=None, defines=()):
    """Compile libfaasbal.so (or a diagnostic variant with extra -D defines)."""
    OUT_ = out or OUT
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    hdrs = [os.path.join(CSRC, "faasbal_kernels.h"), os.path.join(REPO, "include", "faasbal.h")]
    stamp = OUT_ + ".defines"
    want = " ".join(sorted(defines))
    if os.path.exists(OUT_) and os.path.exists(stamp) and open(stamp).read() == want:
        t = os.path.getmtime(OUT_)
        if all(os.path.getmtime(p) < t for p in srcs + hdrs):
            return OUT_
    cmd = ["hipcc", "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-unused-value",
           *["-D" + d for d in defines],
           "-I" + os.path.join(REPO, "include"), "-I" + CSRC, *srcs, "-o", OUT_ + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(OUT_ + ".tmp", OUT_)
    with open(stamp, "w") as f:  # the -D set this library was built with (up-to-date check)
        f.write(want)
    return OUT_


if __name__ == "__main__":
    print(build_lib(verbose=True))
