"""Device time of vg_type_mean (k_type_sums + k_type_gather) against the
program-graph size: python tools/type_mean_probe.py (HIP events, 50 launches
per size after 5 warm-up launches)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

from vgan import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    vt = torch.randint(0, 7, (12111,), generator=g).to(dev)
    for n_local in (1, 64, 512, 1891, 8192, 32768):
        lx = torch.randn(n_local, 17, generator=g).to(dev)
        lt = torch.randint(0, 6, (n_local,), generator=g).to(dev)
        out = torch.empty(12111, 17, device=dev)
        for _ in range(5):
            ops.type_mean(lx, lt, vt, 7, out=out)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(50):
            ops.type_mean(lx, lt, vt, 7, out=out)
        b.record()
        torch.cuda.synchronize()
        print(json.dumps({"n_local": n_local, "us_per_call": round(a.elapsed_time(b) * 1000 / 50, 2)}), flush=True)


if __name__ == "__main__":
    main()
