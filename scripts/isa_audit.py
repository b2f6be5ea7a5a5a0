#!/usr/bin/env python3
"""Static audit of the gfx950 assembly hipcc emits for the in-tree HIP kernels.

Two checks, both for problems that hipcc does not catch on its own:

1. ``readlane-vmem``: an SGPR written by ``v_readfirstlane_b32`` / ``v_readlane_b32`` and read as
   the scalar base (``saddr``) or offset of a vector-memory instruction fewer than 5 wait states
   later.  A VALU write of an SGPR followed by a VMEM read of it is a hardware hazard.  The
   compiler pads it for the instructions it schedules, but not around inline asm.  Two kernels
   hit it in round 6: the four-wave GEMM, and the streamed conv kernel's weight DMA
   (`profiles/r6/SUMMARY.md`, "Inline-asm hazard audit").
2. ``loop-drain`` (only for kernels matching ``--drain``): an ``s_waitcnt vmcnt(0)`` inside a loop.
   In a loop that prefetches rows ahead this waits for every outstanding load, the prefetched ones
   included.  The usual cause is a branch around the loads: the compiler's wait-count merge at the
   join cannot count them.  This is what held the LayerNorm backward at one row in flight
   (`csrc/layernorm.hip`, the comment on ``load``).

    python scripts/isa_audit.py cloudtik_amd/ops/csrc/gemm_nt.hip [...] [--drain REGEX]

Exit status 1 if any finding is reported.  ``audit_source()`` is the library entry the tests use.
"""
from __future__ import annotations

import argparse
import hashlib
import os
import re
import subprocess
import sys
import tempfile
from typing import Dict, List, Optional, Tuple

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cloudtik_amd", "ops", "csrc")

_READLANE = re.compile(r"^\s*v_readfirstlane_b32\s+(s\d+)|^\s*v_readlane_b32\s+(s\d+)")
_SNOP = re.compile(r"^\s*s_nop\s+(\d+)")
_VMEM = re.compile(r"^\s*(global_|buffer_|scratch_)\S*")
_SRANGE = re.compile(r"s\[(\d+):(\d+)\]")
_SREG = re.compile(r"(?<![\w\[:])s(\d+)\b")
_LABEL = re.compile(r"^(\.LBB\d+_\d+):")
_BRANCH = re.compile(r"^\s*s_(?:cbranch_\w+|branch)\s+(\.LBB\d+_\d+)")
_KERNEL = re.compile(r"^(_Z[^:\s]+):", re.M)


def compile_asm(src: str, cache_dir: Optional[str] = None) -> str:
    """gfx950 device assembly of ``src`` (cached by the source's and common.h's content)."""
    h = hashlib.sha256()
    for p in (src, os.path.join(CSRC, "common.h")):
        if os.path.exists(p):
            with open(p, "rb") as f:
                h.update(f.read())
    cache_dir = cache_dir or os.path.join(tempfile.gettempdir(), "cloudtik_isa_audit")
    os.makedirs(cache_dir, exist_ok=True)
    out = os.path.join(cache_dir, f"{os.path.basename(src)}.{h.hexdigest()[:16]}.s")
    if not os.path.exists(out):
        tmp = out + f".{os.getpid()}.tmp"
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}", "--cuda-device-only",
                        "-S", src, "-o", tmp], check=True, capture_output=True)
        os.replace(tmp, out)
    with open(out) as f:
        return f.read()


def split_kernels(asm: str) -> Dict[str, List[str]]:
    out = {}
    for m in _KERNEL.finditer(asm):
        end = asm.find(".Lfunc_end", m.end())
        out[m.group(1)] = asm[m.end():end if end > 0 else len(asm)].split("\n")
    return out


def _sregs_read(line: str) -> set:
    """SGPR numbers an instruction line names after its mnemonic (destinations included: only
    VMEM lines are asked, whose destinations are vector registers)."""
    body = line.split(None, 1)[1] if len(line.split(None, 1)) > 1 else ""
    body = body.split(";")[0]
    regs = set()
    for a, b in _SRANGE.findall(body):
        regs.update(range(int(a), int(b) + 1))
    regs.update(int(x) for x in _SREG.findall(_SRANGE.sub("", body)))
    return regs


def readlane_vmem_hazards(lines: List[str], need: int = 5) -> List[Tuple[int, str, str]]:
    """(line index, writer, reader) for every VMEM read of a readlane-written SGPR fewer than
    ``need`` wait states after the write.  Straight-line scan: a label resets nothing (the
    hazard needs the wait states on every path, and the fall-through path is one of them)."""
    found = []
    pending: Dict[int, Tuple[int, str]] = {}       # sgpr -> (wait states since the write, writer)
    for i, raw in enumerate(lines):
        line = raw.strip()
        if not line or line.startswith((";", ".")) or line.endswith(":"):
            continue
        m = _SNOP.match(line)
        states = int(m.group(1)) + 1 if m else 1
        if _VMEM.match(line):
            for r in _sregs_read(line) & set(pending):
                found.append((i, pending[r][1], line))
        for r in list(pending):
            w, who = pending[r]
            w += states
            if w >= need:
                del pending[r]
            else:
                pending[r] = (w, who)
        m = _READLANE.match(line)
        if m:
            pending[int((m.group(1) or m.group(2))[1:])] = (0, line)
    return found


def loop_drains(lines: List[str]) -> List[Tuple[str, int]]:
    """(loop header label, line index) of every ``s_waitcnt vmcnt(0)`` between a loop header
    and its last back-edge branch."""
    labels = {}
    for i, raw in enumerate(lines):
        m = _LABEL.match(raw.strip())
        if m:
            labels[m.group(1)] = i
    spans = {}
    for i, raw in enumerate(lines):
        m = _BRANCH.match(raw)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            spans[m.group(1)] = (labels[m.group(1)], i)     # the last back-edge wins
    out = []
    for head, (a, b) in spans.items():
        for i in range(a, b):
            if re.match(r"^\s*s_waitcnt\s+vmcnt\(0\)", lines[i]):
                out.append((head, i))
    return out


def audit_source(src: str, drain: Optional[str] = None) -> Dict[str, list]:
    """{kernel: [finding, ...]} for one HIP source (kernels with no finding are left out)."""
    res: Dict[str, list] = {}
    for name, lines in split_kernels(compile_asm(src)).items():
        f = [("readlane-vmem", i, f"{w.strip()} -> {r.strip()}") for i, w, r in readlane_vmem_hazards(lines)]
        if drain and re.search(drain, name):
            f += [("loop-drain", i, f"s_waitcnt vmcnt(0) in the loop at {h}") for h, i in loop_drains(lines)]
        if f:
            res[name] = f
    return res


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("sources", nargs="*", help="HIP sources (default: every csrc/*.hip)")
    ap.add_argument("--drain", default=None, help="regex of kernel names to check for loop drains")
    a = ap.parse_args(argv)
    srcs = a.sources or sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".hip"))
    bad = 0
    for s in srcs:
        res = audit_source(s, a.drain)
        for k, fs in res.items():
            for kind, i, msg in fs:
                print(f"{os.path.basename(s)}: {kind}: {k[:80]} line {i}: {msg}")
                bad += 1
        print(f"{os.path.basename(s)}: {len(res)} kernel(s) with findings", file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
