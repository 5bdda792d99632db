"""Build libhdgnn.so in-tree for gfx950 (hipcc, no torch extension machinery).

    python hd-gnn_amd/hdgnn/build.py
"""
import os
import subprocess
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"


def build(verbose=False, out=None, force=False):
    srcs = [os.path.join(CSRC, f) for f in ("hdgnn.hip", "wide.hip")]
    out = out or os.path.join(CSRC, "libhdgnn.so")
    deps = srcs + [os.path.join(CSRC, "hdgnn_internal.h"), os.path.join(ROOT, "include", "hdgnn.h")]
    extra = os.environ.get("HDG_HIPCC_FLAGS", "").split()   # experiments (A/B builds)
    # the effective flags are stamped next to the library: a build with other flags (an A/B
    # experiment, or the default after one) is never mistaken for an up-to-date one
    stamp, flags = out + ".flags", " ".join(extra)
    same_flags = os.path.exists(stamp) and open(stamp).read() == flags
    if (not force and same_flags and os.path.exists(out)
            and all(os.path.getmtime(out) >= os.path.getmtime(d) for d in deps)):
        return out
    cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I" + os.path.join(ROOT, "include"), "-o", out + ".tmp"] + srcs
    cmd[1:1] = extra
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(flags)
    return out


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv))
