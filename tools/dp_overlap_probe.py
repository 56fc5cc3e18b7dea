"""Cost of the data-parallel step's recorded collectives on one GPU: a
one-rank RCCL group with the trainer's GradSync forced on (the collectives
are identities, but recorded and launched like N > 1), replayed steps timed
three ways, alternated twice:

  none      no collectives (the N = 1 step)
  overlap   the generator's decoder bucket all-reduced on a side stream while
            the encoders' backward runs (a parallel branch in the captured
            graph; runtime['overlap_allreduce'], the default)
  serial    the generator's whole gradient in one all-reduce after its backward

    python tools/dp_overlap_probe.py [--steps 30]     # JSON lines
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    from vgan.config import Configuration
    from vgan.dist import GradSync

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 4, 32, dev)
    trainers = {}
    for mode in ("none", "overlap", "serial"):
        tr = bench.build_trainer(cfg, "f32")
        if mode != "none":
            tr.sync = GradSync(force=True)
            tr.configuration.runtime["overlap_allreduce"] = mode == "overlap"
        trainers[mode] = tr
    cfg.runtime["overlap_allreduce"] = True
    for rep in (1, 2):
        for mode, tr in trainers.items():
            # overlap_allreduce is read from the (shared) configuration at capture time
            tr.configuration.runtime["overlap_allreduce"] = mode == "overlap"
            bench.run_steps(tr, pool, 2 * len(pool))  # capture + warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            bench.run_steps(tr, pool, args.steps)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            print(json.dumps({"mode": mode, "rep": rep, "ms_per_step": round(ms, 3),
                              "overlap_ready": bool(tr._overlap_ready())}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
