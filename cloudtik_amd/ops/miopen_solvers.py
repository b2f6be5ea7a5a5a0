"""MIOpen solver database for this framework's convolution shapes, installed robustly.

MIOpen's immediate mode (what ``F.conv2d`` uses unless ``cudnn.benchmark`` is on) picks a
solver per problem from the user find-db.  Without a record it runs a solver search at the
first call of every new shape (about 60 s of warm-up for ResNet-50 on a fresh MI355X), and its
record-less fallback can land on ``ConvDirectNaive*`` kernels that take 25-200 ms per call.
``ops/miopen_db`` ships the records searched on MI355X for the ResNet-50 NHWC bf16 training
shapes; this module makes MIOpen see them in every environment:

* the shipped files go to a writable per-user directory (first that works of
  ``$CLOUDTIK_AMD_CACHE``, ``$XDG_CACHE_HOME``, ``~/.cache``, ``$TMPDIR``, ``/tmp``,
  ``/dev/shm``), and ``MIOPEN_USER_DB_PATH`` points there;
* if ``MIOPEN_USER_DB_PATH`` is already set by the environment, the shipped records are
  MERGED into the files there (the shipped solver list wins for the shipped problem keys;
  every other record is kept) instead of being skipped;
* file names are ``<arch><CU count, hex>.HIP.<MIOpen version>.{ufdb,udb}.txt``; besides the
  shipped name, a copy is written under the CU count the KFD topology reports, so a part with
  another CU count still finds the records;
* nothing fails silently: ``status()`` says what was installed where (bench.py prints it),
  and a failure is logged as a warning with its reason.

Set ``CLOUDTIK_AMD_MIOPEN_DB=0`` to leave MIOpen alone.
"""
from __future__ import annotations

import glob
import hashlib
import logging
import os
import re
import tempfile
from typing import Dict, List, Optional

logger = logging.getLogger(__name__)

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "miopen_db")
_NAME = re.compile(r"^(gfx[0-9a-f]+?)([0-9a-f]{2,3})\.(HIP\..+)\.(ufdb|udb)\.txt$")
_STATUS: Dict[str, object] = {"installed": False, "reason": "not run"}


def shipped_files() -> List[str]:
    if not os.path.isdir(SRC):
        return []
    return sorted(f for f in os.listdir(SRC) if f.endswith((".udb.txt", ".ufdb.txt")))


def _kfd_cu_counts() -> List[int]:
    """CU counts of the gfx950 GPU nodes in the KFD topology (no HIP initialisation)."""
    out = set()
    for p in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
        try:
            props = dict(line.split() for line in open(p) if len(line.split()) == 2)
        except (OSError, ValueError):
            continue
        simd, per_cu = int(props.get("simd_count", 0)), int(props.get("simd_per_cu", 0) or 0)
        if simd and per_cu and props.get("gfx_target_version", "").startswith("905"):
            out.add(simd // per_cu)
    return sorted(out)


def _candidate_dirs() -> List[str]:
    bases = [os.environ.get("CLOUDTIK_AMD_CACHE"), os.environ.get("XDG_CACHE_HOME"),
             os.path.join(os.path.expanduser("~"), ".cache"), os.environ.get("TMPDIR"), tempfile.gettempdir(),
             "/tmp", "/dev/shm"]
    seen, out = set(), []
    for b in bases:
        if b and b not in seen:
            seen.add(b)
            out.append(b)
    return out


def _read_records(path: str) -> "Dict[str, str]":
    recs: Dict[str, str] = {}
    try:
        with open(path) as f:
            for line in f:
                line = line.rstrip("\n")
                if "=" in line:
                    k, v = line.split("=", 1)
                    recs[k] = v
    except FileNotFoundError:
        pass
    return recs


def _write_atomic(path: str, recs: "Dict[str, str]"):
    d = os.path.dirname(path)
    fd, tmp = tempfile.mkstemp(prefix=".ct_miopen_", dir=d)
    with os.fdopen(fd, "w") as f:
        for k, v in recs.items():
            f.write(f"{k}={v}\n")
    os.replace(tmp, path)       # concurrent ranks never see a partial file


def _target_names(fname: str, cu_counts: List[int]) -> List[str]:
    names = [fname]
    m = _NAME.match(fname)
    if m:
        for cu in cu_counts:
            alt = f"{m.group(1)}{cu:x}.{m.group(3)}.{m.group(4)}.txt"
            if alt not in names:
                names.append(alt)
    return names


def _install_into(dst: str, files: List[str], merge: bool) -> List[str]:
    os.makedirs(dst, exist_ok=True)
    cus = _kfd_cu_counts()
    written = []
    for f in files:
        ours = _read_records(os.path.join(SRC, f))
        for name in _target_names(f, cus):
            path = os.path.join(dst, name)
            if merge:
                recs = _read_records(path)
                if all(recs.get(k) == v for k, v in ours.items()):
                    written.append(path)
                    continue
                recs.update(ours)
            else:
                if os.path.exists(path) and _read_records(path) == ours:
                    written.append(path)
                    continue
                recs = ours
            _write_atomic(path, recs)
            written.append(path)
    return written


def install() -> Dict[str, object]:
    """Install the shipped records (idempotent; cheap when already installed)."""
    global _STATUS
    if os.environ.get("CLOUDTIK_AMD_MIOPEN_DB", "1") == "0":
        _STATUS = {"installed": False, "reason": "disabled (CLOUDTIK_AMD_MIOPEN_DB=0)"}
        return _STATUS
    files = shipped_files()
    if not files:
        _STATUS = {"installed": False, "reason": f"no shipped db under {SRC}"}
        logger.warning("cloudtik_amd: %s", _STATUS["reason"])
        return _STATUS
    preset = os.environ.get("MIOPEN_USER_DB_PATH")
    errors = []
    if preset:
        try:
            written = _install_into(preset, files, merge=True)
            _STATUS = {"installed": True, "path": preset, "mode": "merged into preset MIOPEN_USER_DB_PATH",
                       "files": [os.path.basename(w) for w in written]}
            return _STATUS
        except OSError as e:
            errors.append(f"{preset}: {e}")
    h = hashlib.sha1()
    for f in files:
        with open(os.path.join(SRC, f), "rb") as fh:
            h.update(f.encode() + fh.read())
    for base in _candidate_dirs():
        dst = os.path.join(base, "cloudtik_amd", "miopen_db", h.hexdigest()[:12])
        try:
            written = _install_into(dst, files, merge=False)
        except OSError as e:
            errors.append(f"{dst}: {e}")
            continue
        if preset:
            logger.warning("cloudtik_amd: preset MIOPEN_USER_DB_PATH=%s is not writable; using %s", preset, dst)
        os.environ["MIOPEN_USER_DB_PATH"] = dst
        _STATUS = {"installed": True, "path": dst, "mode": "private copy",
                   "files": [os.path.basename(w) for w in written]}
        if errors:
            _STATUS["skipped"] = errors
        return _STATUS
    _STATUS = {"installed": False, "reason": "no writable directory", "errors": errors}
    logger.warning("cloudtik_amd: MIOpen find-db NOT installed (%s); convolutions fall back to MIOpen's "
                   "record-less solver choice", "; ".join(errors))
    return _STATUS


def status() -> Dict[str, object]:
    return dict(_STATUS, env_MIOPEN_USER_DB_PATH=os.environ.get("MIOPEN_USER_DB_PATH"),
                env_MIOPEN_FIND_MODE=os.environ.get("MIOPEN_FIND_MODE"))


def miopen_version() -> Optional[str]:
    """The MIOpen build the shipped records are keyed to (from the file names)."""
    for f in shipped_files():
        m = _NAME.match(f)
        if m:
            return m.group(3)[len("HIP."):]
    return None
