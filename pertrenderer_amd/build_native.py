"""Build libpertrender.so (gfx950) in-tree with hipcc, and the C++ autograd layer over it
(_pr_torch*.so, csrc/pr_torch.cpp: a torch extension of plain host C++).

    python -m pertrenderer_amd.build_native [--force]

Both shared libraries land next to this file so they travel with the repository snapshot to
the GPU box (they are git-ignored, not gpurun-ignored).
"""
import argparse
import concurrent.futures
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "libpertrender.so")
SOURCES = ["pr_capi.hip", "pr_blend.hip", "pr_rast.hip", "pr_pose.hip", "pr_shade.hip", "pr_softblend.hip",
           "pr_normals.hip", "pr_detsum.hip"]
HEADERS = ["pr_common.h", os.path.join("..", "..", "include", "pertrender.h")]
ARCH = os.environ.get("PR_OFFLOAD_ARCH", "gfx950")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-munsafe-fp-atomics",
         f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", "hipcc"):
        if c and (os.path.exists(c) or c == "hipcc"):
            return c
    raise RuntimeError("hipcc not found")


def source_sha():
    """sha256 (16 hex digits) of the native sources and headers: ties a committed rocprofv3 / PMC
    record under profiles/ (its "source_sha") to the code a run loads."""
    import hashlib
    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        h.update(os.path.basename(f).encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _stale():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(CSRC, s) for s in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=True, out=None, defines=()):
    """Compile SOURCES and link the shared library.  `out`/`defines` build a
    diagnostic variant (e.g. -DPR_RAST_PROFILE) beside the product library."""
    lib = out or LIB
    if out is None and not defines and not force and not _stale():
        return LIB
    hipcc = _hipcc()
    tag = "" if out is None else "_" + os.path.basename(out).replace(".", "_")
    objs, cmds = [], []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.replace(".hip", tag + ".o"))
        cmds.append([hipcc] + FLAGS + [f"-D{d}" for d in defines] + ["-c", os.path.join(CSRC, src), "-o", obj])
        objs.append(obj)
    # one hipcc per translation unit, in parallel (bounded: each holds ~1-2 GB while compiling)
    jobs = max(1, min(len(cmds), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1)), 8))
    with concurrent.futures.ThreadPoolExecutor(jobs) as pool:
        for cmd, rc in zip(cmds, pool.map(lambda c: subprocess.call(c), cmds)):
            if verbose:
                print(" ".join(cmd), flush=True)
            if rc != 0:
                raise subprocess.CalledProcessError(rc, cmd)
    tmp = lib + ".tmp"
    cmd = [hipcc, "-shared", f"--offload-arch={ARCH}", "-o", tmp] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(tmp, lib)
    for o in objs:
        os.remove(o)
    return lib


TORCH_EXT_SRC = os.path.join(CSRC, "pr_torch.cpp")


def torch_ext_path():
    import sysconfig
    return os.path.join(HERE, "_pr_torch" + sysconfig.get_config_var("EXT_SUFFIX"))


def build_torch_ext(force=False, verbose=True):
    """g++ of csrc/pr_torch.cpp against the installed torch (headers, libtorch, libc10_hip) and the
    HIP runtime headers: no device code, so no hipcc.  Rebuilt when the source or the ABI header is
    newer than the module."""
    import sysconfig
    import torch
    from torch.utils import cpp_extension as ce
    out = torch_ext_path()
    deps = [TORCH_EXT_SRC, os.path.join(ROOT, "include", "pertrender.h")]
    if not force and os.path.exists(out) and all(os.path.getmtime(d) <= os.path.getmtime(out) for d in deps):
        return out
    rocm = os.environ.get("ROCM_PATH", "/opt/rocm")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = (["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-w", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
            "-DTORCH_EXTENSION_NAME=_pr_torch", "-DTORCH_API_INCLUDE_EXTENSION_H", "-D__HIP_PLATFORM_AMD__=1",
            "-DUSE_ROCM=1", f"-I{os.path.join(ROOT, 'include')}", f"-I{rocm}/include",
            f"-I{sysconfig.get_paths()['include']}"]
           + [f"-I{p}" for p in ce.include_paths()]
           + [TORCH_EXT_SRC, "-o", out + ".tmp"]
           + [f"-L{p}" for p in ce.library_paths()] + [f"-L{rocm}/lib"]
           + ["-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lamdhip64"])
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--out", help="diagnostic variant path (default: the product library)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="preprocessor define")
    args = ap.parse_args()
    print(build(force=args.force, out=args.out, defines=args.defines))
    if args.out is None and not args.defines:
        print(build_torch_ext(force=args.force))
    sys.exit(0)
