"""Where the GPU's clock / power / temperature live on this box (bench.py GpuTelemetry)."""
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

from cloudtik_amd.core.node.metrics import amd_gpu_cards, gpu_clock_snapshot, pci_device_dir  # noqa: E402

p = torch.cuda.get_device_properties(0)
print("props", {k: getattr(p, k, None) for k in ("name", "pci_bus_id", "pci_device_id", "pci_domain_id")})
print("cards", amd_gpu_cards())
print("drm", sorted(glob.glob("/sys/class/drm/*"))[:20])
d = pci_device_dir(getattr(p, "pci_domain_id", 0), p.pci_bus_id, p.pci_device_id)
print("dir", d)
if d:
    print("files", sorted(os.listdir(d))[:200])
    print("hwmon", [(h, sorted(os.listdir(h))) for h in glob.glob(os.path.join(d, "hwmon", "hwmon*"))])
    print(json.dumps(gpu_clock_snapshot(d)))
