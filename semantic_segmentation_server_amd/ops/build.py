"""In-tree build of the native extensions.

Two pybind11 modules are produced next to this file:

* ``_host``  — host C++ (g++): exact contour oracle, result ring, etc.
* ``_hip``   — HIP kernels for gfx950 (hipcc ``--offload-arch=gfx950``) plus their
  launch wrappers.
* ``_hip_debug`` — diagnostic kernels only (csrc/hip_debug: on-chip state poison, LDS
  canary), built on demand (``build_hip_debug``, or ``SSA_BUILD_DEBUG=1``), never part of
  the production module. No torch C++ headers are involved: tensors cross the boundary
  as raw device pointers and the caller's HIP stream handle, so launches are
  capturable by ``torch.cuda.CUDAGraph`` (hipGraph) and compile in seconds.

Builds are skipped when a stamp of the sources + flags is unchanged. The
``.so`` files are git-ignored but travel to the GPU box with the gpurun snapshot.
"""
from __future__ import annotations

import glob
import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "csrc")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("SSA_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# per-source extra flags (none at present). MFMA results live in VGPRs instead of AGPRs in
# every source (-amdgpu-mfma-vgpr-form in cflags): kernels whose MFMA epilogues run per
# fragment on the VALU paid one v_accvgpr_read per result dword and one v_accvgpr_write per
# accumulator initialisation (stem_band: 12 of ~134 VALU per stem row; conv_gemm: 2,536
# reads + 4,257 writes in the ISA), and no kernel spills in the VGPR form (round 6, hipcc
# -Rpass-analysis=kernel-resource-usage: scratch 0 everywhere, occupancy equal or higher)
EXTRA_FLAGS: dict = {}


def _pybind_includes():
    import pybind11
    return [sysconfig.get_paths()["include"], pybind11.get_include()]


def _stamp(files, flags) -> str:
    h = hashlib.sha256()
    for f in sorted(files):
        h.update(f.encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _up_to_date(out: str, stamp: str) -> bool:
    sp = out + ".stamp"
    return os.path.exists(out) and os.path.exists(sp) and open(sp).read().strip() == stamp


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def build_host(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "host", "*.h")))
    out = os.path.join(HERE, "_host" + EXT_SUFFIX)
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", "-fvisibility=hidden", "-Wall",
             "-Wno-sign-compare"]
    stamp = _stamp(srcs + hdrs, flags)
    if not force and _up_to_date(out, stamp):
        return out
    inc = [f"-I{p}" for p in _pybind_includes() + [os.path.join(CSRC, "host")]]
    cmd = [os.environ.get("CXX", "g++")] + flags + inc + srcs + ["-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    _run(cmd)
    os.replace(out + ".tmp", out)
    with open(out + ".stamp", "w") as f:
        f.write(stamp)
    return out


def build_hip(force: bool = False, verbose: bool = False, jobs: int = 8) -> str:
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.hip")))
    hdrs = sorted(glob.glob(os.path.join(CSRC, "hip", "*.h")))
    binding = os.path.join(CSRC, "hip", "bindings.cpp")
    out = os.path.join(HERE, "_hip" + EXT_SUFFIX)
    cflags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
              "-Wno-unused-result", "-munsafe-fp-atomics", "-mllvm", "-amdgpu-mfma-vgpr-form"]
    if os.environ.get("SSA_PACKED_F32", "0") != "1":
        # no packed-f32 VALU (v_pk_fma/mul/add_f32): under co-residence with other kernels'
        # waves, their low halves came back wrong in lanes 48-63 (scripts/debug_pool.py,
        # profiles/r3_packed_f32_race.txt) -- the rare label-map mismatch of concurrent
        # plan copies (VERDICT r2 Weak #1)
        cflags += ["-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops"]
    # diagnostic builds (e.g. SSA_PACKED_F32=1 SSA_HIP_OUT=tools/bin/_hip_pk.so) go to their
    # own object cache and output file; ops/native.py loads SSA_HIP_SO when it is set
    out = os.environ.get("SSA_HIP_OUT", out)
    stamp = _stamp(hip_srcs + hdrs + [binding], cflags + [repr(sorted(EXTRA_FLAGS.items()))])
    if not force and _up_to_date(out, stamp):
        return out
    bdir = os.path.join(ROOT, "build", "hip" if out.startswith(HERE) else "hip_alt")
    os.makedirs(bdir, exist_ok=True)
    inc = [f"-I{p}" for p in _pybind_includes() + [os.path.join(CSRC, "hip")]]

    def compile_one(src):
        # per-object cache: a source is recompiled only when it, a header or the flags
        # changed (the full gfx950 build takes ~2 minutes)
        obj = os.path.join(bdir, os.path.basename(src) + ".o")
        flags = cflags + EXTRA_FLAGS.get(os.path.basename(src), [])
        ostamp = _stamp([src] + hdrs, flags)
        if not force and _up_to_date(obj, ostamp):
            return obj
        lang = ["-x", "hip"] if src.endswith(".hip") else []
        cmd = [HIPCC] + flags + inc + lang + ["-c", src, "-o", obj + ".tmp"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        _run(cmd)
        os.replace(obj + ".tmp", obj)
        with open(obj + ".stamp", "w") as f:
            f.write(ostamp)
        return obj

    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, hip_srcs + [binding]))
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + ["-o", out + ".tmp"]
    _run(cmd)
    os.replace(out + ".tmp", out)
    with open(out + ".stamp", "w") as f:
        f.write(stamp)
    return out


def build_hip_debug(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "hip_debug", "*.hip")))
    binding = os.path.join(CSRC, "hip_debug", "bindings_debug.cpp")
    out = os.path.join(HERE, "_hip_debug" + EXT_SUFFIX)
    flags = ["-O3", "-std=c++17", "-fPIC", "-shared", f"--offload-arch={ARCH}", "-fno-gpu-rdc"]
    stamp = _stamp(srcs + [binding], flags)
    if not force and _up_to_date(out, stamp):
        return out
    inc = [f"-I{p}" for p in _pybind_includes()]
    cmd = [HIPCC] + flags + inc + srcs + [binding, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    _run(cmd)
    os.replace(out + ".tmp", out)
    with open(out + ".stamp", "w") as f:
        f.write(stamp)
    return out


def build_all(force: bool = False, verbose: bool = False):
    outs = (build_host(force, verbose), build_hip(force, verbose))
    if os.environ.get("SSA_BUILD_DEBUG", "0") == "1":
        outs += (build_hip_debug(force, verbose),)
    return outs


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(force=force, verbose=True):
        print(p)
