"""Why bench.py's torch.profiler kernel audit saw fewer kernels per ResNet-50 step than rocprofv3
(187-216 vs 568): count the same step's kernels three ways -- prof.events(), the exported
Chrome trace by stream, and kineto's raw kernel activities."""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402

args = bench.parse(["--model", "resnet50", "--steps", "1", "--warmup", "3"])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
step, close, info = bench.build_resnet(args, 0, 1, dev, "resnet50")
for _ in range(3):
    step()
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()
ev = [e for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
path = os.path.join(tempfile.mkdtemp(), "t.json")
prof.export_chrome_trace(path)
tr = json.load(open(path))
kern = [e for e in tr.get("traceEvents", []) if e.get("cat") == "kernel"]
by_stream = {}
for e in kern:
    s = (e.get("args") or {}).get("stream")
    by_stream[s] = by_stream.get(s, 0) + 1
print(json.dumps({"events_cuda": len(ev), "trace_kernels": len(kern), "by_stream": by_stream,
                  "trace_cats": sorted({e.get("cat") for e in tr.get("traceEvents", []) if e.get("cat")})}))
close()
