"""C3 drop-in leg alone (bench.py C3.dropin_leg) in a fresh process, for sweeping the context's lane
count / HIP queue count / coalescing policy set through the environment before HIP starts:
  ZGPU_CTX_LANES, GPU_MAX_HW_QUEUES, ZGPU_TRACE=1 (per-batch phases on stderr, tools/co_trace.py).
Usage: python tools/dropin_sweep.py [max_calls] [window_us]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from zarrs_amd import Context  # noqa: E402

mc = int(sys.argv[1]) if len(sys.argv) > 1 else 4
win = int(sys.argv[2]) if len(sys.argv) > 2 else 200
args = types.SimpleNamespace(ctx=Context(0), dropin_calls=mc, dropin_sweep="", cpu_seconds=1, no_cpu=True,
                             dropin_window_us=win)
W = bench.C3(args, 0, 1, torch.device("cuda", 0))
args.ctx.set_coalescing(window_us=win, max_calls=mc)
r = W.dropin_leg()
r.pop("note", None)
print(json.dumps({"lanes": os.environ.get("ZGPU_CTX_LANES", "8"), "hwq": os.environ.get("GPU_MAX_HW_QUEUES"),
                  "max_calls": mc, "window_us": win, **r}), flush=True)
