"""configs[3] through the drop-in: bench.stress_model_leg alone -- the
VoxelGNNGenerator forward (eval, no grad) on the 8 x 50k stress batch with
the ring (the GraphNorm reading its input for the statistics: the default),
the ring with the partials from its loaders, and the register gather.

    python tools/stress_model_probe.py [--reps 7]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=7)
    args = ap.parse_args()
    import bench

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    print(json.dumps(bench.stress_model_leg(dev, reps=args.reps)), flush=True)
