"""Per-kernel register / spill / occupancy table of one HIP source (compiler remarks).

    python scripts/kres.py cloudtik_amd/ops/csrc/attention.hip [name-substring]
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "--offload-device-only",
           "-Icloudtik_amd/ops/csrc", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
    err = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r"remark:\s+Function Name: (\S+)", line) or re.search(r"Name: (_Z\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, rx in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("spill", r"VGPRs Spill: (\d+)"),
                        ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                        ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)")):
            m = re.search(rx, line)
            if m:
                cur[key] = int(m.group(1))
    demangle = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                              text=True).stdout.splitlines()
    for r, d in zip(rows, demangle):
        if pat in d:
            print(f"{r.get('vgpr', '?'):>4} v {r.get('agpr', '?'):>3} a spill {r.get('spill', '?'):>3} "
                  f"scr {r.get('scratch', '?'):>4} occ {r.get('occ', '?')} lds {r.get('lds', '?'):>6}  {d[:140]}")


if __name__ == "__main__":
    main()
