"""Build libgeobpe.so (gfx950) in-tree with hipcc."""
from __future__ import annotations

import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
OUT = os.path.join(HERE, "libgeobpe.so")
SOURCES = [os.path.join(CSRC, "geobpe.hip")]
DEPS = SOURCES + [os.path.join(CSRC, "keyjson.h"), os.path.join(CSRC, "device.h"), os.path.join(CSRC, "kernels.h"), os.path.join(CSRC, "bin_dense.h"), os.path.join(CSRC, "merge.h"), os.path.join(CSRC, "featurize.h"), os.path.join(CSRC, "rmsd.h"), os.path.join(CSRC, "glue.h"), os.path.join(CSRC, "tail.h"), os.path.join(CSRC, "mid.h"), os.path.join(CSRC, "exchange.h"),
                  os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "geobpe.h")]
ARCH = os.environ.get("GEOBPE_ARCH", "gfx950")


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and os.path.exists(OUT):
        t = os.path.getmtime(OUT)
        if all(os.path.getmtime(d) <= t for d in DEPS if os.path.exists(d)):
            return OUT
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-O3", "-fPIC", "-shared", "-std=c++17",
           "-ffp-contract=off", "-Wall", "-Wno-unused-result", "-Wno-unused-value",
           "-Wno-unused-function", *SOURCES, "-o", OUT + ".tmp"]
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed:\n{r.stderr[-4000:]}")
    os.replace(OUT + ".tmp", OUT)
    return OUT


KEY_SRC = os.path.join(CSRC, "rmsdkey.c")
KEY_CPP = os.path.join(CSRC, "frepr.cpp")
KEY_OUT = os.path.join(HERE, "_rmsdkey.so")


def build_keys(force: bool = False, verbose: bool = False) -> str:
    """The RMSD mode's pair-key builder (csrc/rmsdkey.c), a CPython extension built with gcc."""
    import sysconfig
    if not force and os.path.exists(KEY_OUT) and all(os.path.getmtime(f) <= os.path.getmtime(KEY_OUT)
                                                     for f in (KEY_SRC, KEY_CPP)):
        return KEY_OUT
    obj = KEY_OUT + ".frepr.o"
    cmds = [[shutil.which("g++") or "g++", "-O2", "-fPIC", "-std=c++17", "-Wall", "-c", KEY_CPP, "-o", obj],
            [shutil.which("gcc") or "gcc", "-O2", "-shared", "-fPIC", "-Wall", f"-I{sysconfig.get_paths()['include']}",
             KEY_SRC, obj, "-lstdc++", "-o", KEY_OUT + ".tmp"]]
    for cmd in cmds:
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"{cmd[0]} failed:\n{r.stderr[-4000:]}")
    os.replace(KEY_OUT + ".tmp", KEY_OUT)
    os.remove(obj)
    return KEY_OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
    print(build_keys(force=True, verbose=True))
