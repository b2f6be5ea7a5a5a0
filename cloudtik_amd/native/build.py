"""Build the native control-plane / runtime components in-tree (host C++, no GPU code):

* ``bin/cloudtik-state-server``  -- RESP state server (state_server/state_server.cpp)
* ``bin/libcloudtik_criteo.so``   -- Criteo TSV parser / dictionary encoder (criteo/criteo.cpp)

Called from ``cloudtik_amd.ops.build.build_all`` and ``__graft_entry__.build``.
"""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
BIN = os.path.join(HERE, "bin")

TARGETS = {
    "cloudtik-state-server": [os.path.join(HERE, "state_server", "state_server.cpp")],
    # shared libraries (ctypes) end in .so
    "libcloudtik_criteo.so": [os.path.join(HERE, "criteo", "criteo.cpp")],
}


def build(force: bool = False, verbose: bool = True, sanitize: bool = False):
    os.makedirs(BIN, exist_ok=True)
    outs = []
    for name, srcs in TARGETS.items():
        if sanitize and name.endswith(".so"):
            continue            # sanitizer builds are for the executables (a .so would need ASan preloaded)
        out = os.path.join(BIN, name + ("-asan" if sanitize else ""))
        newest = max(os.path.getmtime(s) for s in srcs)
        if force or not os.path.exists(out) or os.path.getmtime(out) < newest:
            flags = ["-O2", "-g", "-std=c++17", "-Wall", "-Wextra", "-Wno-unused-parameter", "-pthread"]
            if sanitize:
                flags = ["-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                         "-fno-sanitize-recover=undefined", "-pthread"]
            if name.endswith(".so"):
                flags += ["-shared", "-fPIC"]
            cmd = ["g++", *flags, *srcs, "-o", out + ".tmp"]
            r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            if r.returncode != 0:
                raise RuntimeError("native build failed:\n" + " ".join(cmd) + "\n" + r.stdout)
            os.replace(out + ".tmp", out)
            if verbose:
                print("[cloudtik_amd.native] built", out, flush=True)
        outs.append(out)
    return outs


def state_server_path(sanitize: bool = False) -> str:
    p = os.path.join(BIN, "cloudtik-state-server" + ("-asan" if sanitize else ""))
    if not os.path.exists(p):
        build(verbose=False, sanitize=sanitize)
    return p


if __name__ == "__main__":
    for o in build(force=True):
        print(o)
