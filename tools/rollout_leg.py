"""The default bench line's C3_rollout_k200 secondary leg alone (bench.secondary_lines), repeated:
    python tools/rollout_leg.py [reps]        (CP_LIB_PATH selects the library)
Prints one JSON line per repetition."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

bench.SECONDARY = bench.SECONDARY[:1]
dev = torch.device("cuda:0")
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    out = bench.secondary_lines(dev, 3)
    print(json.dumps({"lib": os.environ.get("CP_LIB_PATH", "default"), **out["C3_rollout_k200"]}), flush=True)
