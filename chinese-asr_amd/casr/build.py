"""Build ``libcasr_hip.so`` (the C-ABI library, include/casr.h) in-tree for gfx950 with hipcc.

The shared object is written next to this file so it travels with the repository snapshot to
the GPU box (it is git-ignored, not gpurun-ignored).  Variant "s16x1" builds the same sources with
-DCASR_S16_ONE=1 into ``libcasr_hip_s16x1.so``: the opt-in s16x1 perf arithmetic
(CASR_PREC_S16X1, include/casr.h), loaded only by an Engine asked for it."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(REPO, "include")
LIB = os.path.join(HERE, "libcasr_hip.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
# variant -> (library, object directory, extra hipcc flags)
VARIANTS = {None: ("libcasr_hip.so", "_obj", []),
            "s16x1": ("libcasr_hip_s16x1.so", "_obj_s16x1", ["-DCASR_S16_ONE=1"])}


def lib_path(variant=None):
    return os.path.join(HERE, VARIANTS[variant][0])


def sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))


def headers():
    hs = [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    return hs + [os.path.join(INCLUDE, "casr.h")]


def is_stale(variant=None):
    lib = lib_path(variant)
    if not os.path.exists(lib):
        return True
    t = os.path.getmtime(lib)
    return any(os.path.getmtime(p) > t for p in sources() + headers())


def build(force=False, verbose=False, variant=None):
    """Compile every .hip source into one shared library (one hipcc per source, in
    parallel, then link)."""
    lib = lib_path(variant)
    if not force and not is_stale(variant):
        return lib
    objdir = os.path.join(HERE, VARIANTS[variant][1])
    os.makedirs(objdir, exist_ok=True)
    common = [HIPCC, "-O3", "-std=c++17", f"--offload-arch={ARCH}", "-fPIC", "-Wall",
              "-Wno-unused-result", f"-I{INCLUDE}", f"-I{CSRC}"]
    # CASR_EXTRA_FLAGS: diagnostic builds only (ablation macros such as -DCASR_DG_DIAG=1; never the
    # shipped library)
    common += VARIANTS[variant][2] + os.environ.get("CASR_EXTRA_FLAGS", "").split()
    procs, objs = [], []
    for src in sources():
        obj = os.path.join(objdir, os.path.basename(src)[:-4] + ".o")
        objs.append(obj)
        cmd = common + ["-c", src, "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((src, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    for src, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {src}:\n{out.decode(errors='replace')}")
    tmp = lib + ".tmp"
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout.decode(errors='replace')}")
    os.replace(tmp, lib)
    return lib


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    print(build(force="--force" in sys.argv, verbose=True, variant="s16x1"))
