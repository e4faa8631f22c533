"""Build the native routing library in-tree: shadow_amd/libshadow_routing.so (gfx950).

hipcc compiles the HIP kernels + C ABI (routing.hip) and the host-side GML ingest
(gml.cpp) into one shared object with a plain C ABI (include/shadow_routing.h).
-ffp-contract=off: Rust never contracts `1 - x*y` (mod.rs:328) into an FMA, so neither may we.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libshadow_routing.so")
# the test build: the same sources with the fault-injection hooks (SRG_OPT_TEST_FAULT) compiled in;
# loaded only by tests/fault_hooks_run.py (SRG_LIB_PATH), never by the product
LIB_TEST = os.path.join(HERE, "libshadow_routing_testhooks.so")
SOURCES = [os.path.join(CSRC, "routing.hip"), os.path.join(CSRC, "gml.cpp"), os.path.join(CSRC, "comm.hip"),
           os.path.join(CSRC, "routing_info.cpp")]
DEPS = SOURCES + [os.path.join(CSRC, "kernels.hip.h"), os.path.join(CSRC, "tight_sparse.hip.h"), os.path.join(CSRC, "comm.h"), os.path.join(CSRC, "sparse.hip.h"), os.path.join(CSRC, "sparse_ds.hip.h"), os.path.join(CSRC, "events.hip.h"), os.path.join(CSRC, "edge_codec.h"), os.path.join(CSRC, "xchg.hip.h"), os.path.join(CSRC, "internal.h"), os.path.join(CSRC, "guards.h"), os.path.join(ROOT, "include", "shadow_routing.h")]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("SRG_OFFLOAD_ARCH", "gfx950")


def needs_build():
    for lib in (LIB, LIB_TEST):
        if not os.path.exists(lib):
            return True
        t = os.path.getmtime(lib)
        if any(os.path.getmtime(d) > t for d in DEPS):
            return True
    return False


def _compile(src, obj, defs, verbose):
    cmd = [HIPCC, "-c", "-fPIC", "-O3", "-std=c++17", "-ffp-contract=off", "-Wall",
           "-Wno-unused-function", "-I", os.path.join(ROOT, "include")] + defs
    if src.endswith(".hip"):
        cmd += ["-x", "hip", "--offload-arch=" + ARCH]
    cmd += [src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    return subprocess.Popen(cmd)


def _link(lib, objs, verbose):
    cmd = [HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", lib] + objs + ["-ldl", "-lpthread", "-lhsa-runtime64"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)


def build(force=False, verbose=True):
    if not force and not needs_build():
        return LIB
    objs, jobs = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, os.path.basename(src) + ".o")
        jobs.append(_compile(src, obj, [], verbose))
        objs.append(obj)
    # the test build's routing.hip object (the other sources have no hooks)
    obj_th = os.path.join(CSRC, "routing_testhooks.hip.o")
    jobs.append(_compile(SOURCES[0], obj_th, ["-DSRG_TEST_HOOKS"], verbose))
    for j in jobs:  # (compiled side by side: the two routing.hip objects dominate)
        if j.wait() != 0:
            raise subprocess.CalledProcessError(j.returncode, j.args)
    _link(LIB, objs, verbose)
    _link(LIB_TEST, [obj_th] + objs[1:], verbose)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
