"""Criteo click-log preprocessing for DLRM (reference: the quickstart's Cython build of
DLRM ``data_utils.loadDataset`` driven by cython_criteo.py).

The parser is native C++ (``native/criteo/criteo.cpp``, loaded with ctypes): the TSV is
memory-mapped, split at line boundaries and parsed by all cores straight into int32 NumPy
arrays; categorical columns are then dictionary-encoded to contiguous ids in
first-appearance order (one column per thread).  Output matches data_utils'
``.npz`` layout: ``X_int`` [N, 13], ``X_cat`` [N, 26], ``y`` [N], ``counts`` [26].

    python -m cloudtik_amd.data.criteo --raw-data-file day_0 --processed-data-file day_0.npz \\
        --max-ind-range 10000000
"""
from __future__ import annotations

import argparse
import ctypes
import os
from typing import Dict, Optional

import numpy as np

N_INT, N_CAT = 13, 26
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        from cloudtik_amd.native.build import BIN, build
        path = os.path.join(BIN, "libcloudtik_criteo.so")
        if not os.path.exists(path):
            build(verbose=False)
        lib = ctypes.CDLL(path)
        lib.ct_criteo_count_lines.argtypes = [ctypes.c_char_p, ctypes.c_int]
        lib.ct_criteo_count_lines.restype = ctypes.c_long
        i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        lib.ct_criteo_parse.argtypes = [ctypes.c_char_p, ctypes.c_long, ctypes.c_longlong, ctypes.c_int, i32p, i32p,
                                        i32p]
        lib.ct_criteo_parse.restype = ctypes.c_long
        lib.ct_criteo_dict_encode.argtypes = [i32p, ctypes.c_long, i32p, ctypes.c_int]
        lib.ct_criteo_dict_encode.restype = None
        _LIB = lib
    return _LIB


def parse_criteo(path: str, max_ind_range: int = -1, dict_encode: bool = True,
                 threads: Optional[int] = None) -> Dict[str, np.ndarray]:
    threads = threads or min(32, os.cpu_count() or 1)
    lib = _lib()
    bpath = os.fsencode(path)
    n = lib.ct_criteo_count_lines(bpath, threads)
    if n < 0:
        raise FileNotFoundError(path)
    y = np.zeros(n, np.int32)
    x_int = np.zeros((n, N_INT), np.int32)
    x_cat = np.zeros((n, N_CAT), np.int32)
    got = lib.ct_criteo_parse(bpath, n, int(max_ind_range), threads, y, x_int, x_cat)
    if got < 0:
        raise RuntimeError(f"criteo parse failed ({got})")
    out = {"X_int": x_int[:got], "X_cat": x_cat[:got], "y": y[:got]}
    if dict_encode:
        counts = np.zeros(N_CAT, np.int32)
        xc = np.ascontiguousarray(out["X_cat"])
        lib.ct_criteo_dict_encode(xc, got, counts, threads)
        out["X_cat"], out["counts"] = xc, counts
    return out


def parse_criteo_reference(path: str, max_ind_range: int = -1) -> Dict[str, np.ndarray]:
    """Line-by-line Python definition (data_utils semantics) for tests."""
    ys, xi, xc = [], [], []
    with open(path) as f:
        for line in f:
            line = line.rstrip("\n")
            if not line:
                continue
            parts = line.split("\t")
            parts += [""] * (1 + N_INT + N_CAT - len(parts))
            ys.append(int(parts[0] or 0))
            xi.append([int(v) if v else 0 for v in parts[1:1 + N_INT]])
            cats = [int(v, 16) if v else 0 for v in parts[1 + N_INT:1 + N_INT + N_CAT]]
            if max_ind_range > 0:
                cats = [c % max_ind_range for c in cats]
            xc.append(cats)
    x_cat = np.array(xc, np.int64).reshape(-1, N_CAT)
    counts = np.zeros(N_CAT, np.int32)
    enc = np.zeros_like(x_cat, dtype=np.int32)
    for j in range(N_CAT):
        d = {}
        for r, v in enumerate(x_cat[:, j]):
            enc[r, j] = d.setdefault(int(v), len(d))
        counts[j] = len(d)
    return {"X_int": np.array(xi, np.int32).reshape(-1, N_INT), "X_cat": enc, "y": np.array(ys, np.int32),
            "counts": counts}


def write_synthetic_criteo(path: str, rows: int, seed: int = 0, missing: float = 0.1):
    """A Criteo-format TSV with random values (and missing fields) for tests / benchmarks."""
    rng = np.random.default_rng(seed)
    with open(path, "w") as f:
        for _ in range(rows):
            ints = rng.integers(-2, 5000, N_INT)
            cats = rng.integers(0, 1 << 32, N_CAT)
            fi = ["" if rng.random() < missing else str(v) for v in ints]
            fc = ["" if rng.random() < missing else format(int(v), "08x") for v in cats]
            f.write("\t".join([str(int(rng.random() < 0.25))] + fi + fc) + "\n")


def dense_transform(x_int: np.ndarray) -> np.ndarray:
    """log(1 + max(x, 0)) as float32 (DLRM's dense feature transform)."""
    return np.log1p(np.maximum(x_int, 0).astype(np.float32))


def main(argv=None):
    ap = argparse.ArgumentParser(description="Preprocess a Criteo click log (native parser)")
    ap.add_argument("--raw-data-file", required=True)
    ap.add_argument("--processed-data-file", required=True)
    ap.add_argument("--max-ind-range", type=int, default=-1)
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args(argv)
    d = parse_criteo(a.raw_data_file, a.max_ind_range, threads=a.threads or None)
    np.savez(a.processed_data_file, **d)
    print(f"{a.processed_data_file}: {len(d['y'])} rows, counts={d['counts'].tolist()}")


if __name__ == "__main__":
    main()
