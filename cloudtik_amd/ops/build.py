"""In-tree native build driver for cloudtik_amd (gfx950 only).

Every native target is compiled HERE, into the source tree, so the built ``.so``
travels with the repository snapshot to the GPU box:

* ``cloudtik_amd/ops/_C*.so``          -- CDNA4 HIP op library + PyTorch bindings
* ``cloudtik_amd/native/bin/cloudtik-state-server``  -- C++ RESP state server (see native/)
* ``cloudtik_amd/native/_native*.so``  -- C++ runtime helpers (pinned loader, ...)

Kernels (``*.hip``) are compiled by ``hipcc --offload-arch=gfx950``; they expose plain
``extern "C"`` launchers and include no PyTorch headers, so each compiles in seconds.
Only the thin binding translation units include ``torch/extension.h``.  Objects are
cached by a content hash of the source + every header + the flags, and compiled in a
process pool.

Usage:  ``python -m cloudtik_amd.ops.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys
import sysconfig

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("CLOUDTIK_AMD_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"

HIP_FLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
    "-Wno-unused-result", "-Wno-unused-command-line-argument",
]


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    try:
        inc = ce.include_paths(device_type="cuda")
        lib = ce.library_paths(device_type="cuda")
    except TypeError:  # older signature
        inc = ce.include_paths(cuda=True)
        lib = ce.library_paths(cuda=True)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _hash(paths, flags):
    h = hashlib.sha1()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def source_digest(d=None):
    """{file name: sha1} of every source and header of the op library (path-independent, so
    the GPU box, which sees the tree under another root, computes the same digest)."""
    d = d or CSRC
    out = {}
    for f in sorted(os.listdir(d)):
        if f.endswith((".hip", ".cpp", ".h", ".hpp", ".cuh")):
            with open(os.path.join(d, f), "rb") as fh:
                out[f] = hashlib.sha1(fh.read()).hexdigest()
    return out


def manifest_path():
    return os.path.join(HERE, "_C" + EXT_SUFFIX) + ".objs"


def stale_sources():
    """Sources whose content differs from what the in-tree library was linked from (empty:
    current), or None when the library has no manifest (built by an older build driver)."""
    import json
    try:
        with open(manifest_path()) as f:
            m = json.load(f)
    except (OSError, ValueError):
        return None
    built, now = m.get("sources", {}), source_digest()
    return sorted(f for f in set(built) | set(now) if built.get(f) != now.get(f))


def _headers(d):
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith((".h", ".hpp", ".cuh")))


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n" + " ".join(cmd) + "\n" + r.stdout)
    return r.stdout


def _compile(src, obj, flags, compiler):
    os.makedirs(os.path.dirname(obj), exist_ok=True)
    _run([compiler, *flags, "-c", src, "-o", obj])
    return obj


def build_ops(force=False, jobs=None, verbose=True):
    """Build cloudtik_amd/ops/_C<EXT_SUFFIX>.  Returns the .so path."""
    inc, lib, abi = _torch_paths()
    hipcc = os.path.join(ROCM, "bin", "hipcc")
    headers = _headers(CSRC)
    py_inc = sysconfig.get_paths()["include"]
    torch_defs = [
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM=1", "-D__HIP_PLATFORM_AMD__=1",
    ]
    bind_flags = ["-O2", "-fPIC", "-std=c++17", *torch_defs,
                  *[f"-I{p}" for p in inc], f"-I{py_inc}", f"-I{ROCM}/include", "-w"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))
    tasks, objs = [], []
    for f in srcs:
        src = os.path.join(CSRC, f)
        if f.endswith(".hip"):
            flags, comp = HIP_FLAGS + [f"-I{CSRC}"], hipcc
        else:
            flags, comp = bind_flags + [f"-I{CSRC}"], "g++"
        key = _hash([src, *headers], flags + [comp])
        obj = os.path.join(BUILD, "obj", f"{f}.{key}.o")
        objs.append(obj)
        if force or not os.path.exists(obj):
            tasks.append((src, obj, flags, comp))
    out = os.path.join(HERE, "_C" + EXT_SUFFIX)
    if tasks:
        if verbose:
            print(f"[cloudtik_amd.build] compiling {len(tasks)} translation unit(s) for {ARCH}", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            futs = [ex.submit(_compile, *t) for t in tasks]
            for fu in cf.as_completed(futs):
                o = fu.result()
                if verbose:
                    print("  built", os.path.basename(o), flush=True)
    # the object set of the last link, next to the library: a source reverted to content built
    # earlier maps to an OLDER cached object, which an mtime comparison would not relink
    import json
    manifest = manifest_path()
    try:
        with open(manifest) as f:
            linked = json.load(f).get("objs")
    except (OSError, ValueError):
        linked = None
    stale = linked != [os.path.basename(o) for o in objs]
    if tasks or force or stale or not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(o) for o in objs):
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", out + ".tmp",
                *[f"-L{p}" for p in lib], "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
                "-ltorch_hip", "-ltorch_python",
                # PyTorch's own hipBLASLt (bindings_lt.cpp shares its handle and workspace;
                # /opt/rocm's copy would be a second, incompatible instance)
                *[os.path.join(p, "libhipblaslt.so") for p in lib if os.path.exists(os.path.join(p, "libhipblaslt.so"))],
                *[f"-Wl,-rpath,{p}" for p in lib if "torch" in p]]
        _run(link)
        os.replace(out + ".tmp", out)
        with open(manifest, "w") as f:
            json.dump({"objs": [os.path.basename(o) for o in objs], "sources": source_digest()}, f, indent=0)
        if verbose:
            print("[cloudtik_amd.build] linked", out, flush=True)
    return out


def build_all(force=False, jobs=None, verbose=True):
    outs = [build_ops(force=force, jobs=jobs, verbose=verbose)]
    try:
        from cloudtik_amd.native import build as native_build
    except ImportError:
        native_build = None
    if native_build is not None:
        outs.extend(native_build.build(force=force, verbose=verbose))
    return outs


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args(argv)
    for o in build_all(force=a.force, jobs=a.jobs):
        print(o)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(PKG))
    main()
