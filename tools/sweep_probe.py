"""The configs[4] stream sweep per batch, by configuration: loader collating
threads (GraphLoader workers), the f16 forward as one native call
(vg_hgen_sweep) or launched from Python, f16 / f32.

  loader   the loader alone (collate + upload, no forward), per worker count
  staged   the forward alone over batches uploaded beforehand (host + device)
  device   one batch's forward replayed from a captured graph
  stream   the bench's leg: loader and forward together

    python tools/sweep_probe.py [--graphs 3200]     # JSON lines
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=3200)
    ap.add_argument("--workers", default="1,2,3")
    args = ap.parse_args()
    from vgan import infer
    from vgan.config import Configuration
    from vgan.infer import InferenceSweep, geometric_taus
    from vgan.loader import GraphLoader
    from vgan.models import VoxelGNNGenerator
    from vgan.store import write_store
    from vgan.synth import SyntheticDataset

    dev = torch.device("cuda", 0)
    store = write_store(os.path.join(tempfile.mkdtemp(prefix="vgan_sweep_"), "store"),
                        SyntheticDataset(args.graphs, seed=2024))
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    G = VoxelGNNGenerator(cfg, 17, 12)
    taus = geometric_taus(1.0, 0.1, 10)
    workers = [int(w) for w in args.workers.split(",")]

    def loader(w, idx=None):
        return GraphLoader(store, idx, batch_size=32, shuffle=False, device=dev, prefetch=4,
                           prepare=(cfg.NUM_CLASSES, ()), workers=w)

    def timed(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nb = fn()
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) / nb * 1e3, 3)

    plan = [list(range(i, i + 32)) for i in range(0, 32 * 50, 32)]
    for th in (1, 4):  # the host collate alone (page-locked buffers), on this thread
        for idx in plan[:3]:
            store.collate(idx, pin=True, threads=th, prepare=(cfg.NUM_CLASSES, ()))
        t0 = time.perf_counter()
        for idx in plan:
            store.collate(idx, pin=True, threads=th, prepare=(cfg.NUM_CLASSES, ()))
        print(json.dumps({"leg": "collate", "threads": th,
                          "ms_per_batch": round((time.perf_counter() - t0) / len(plan) * 1e3, 3)}), flush=True)
    for w in workers:
        sum(1 for _ in loader(w, list(range(4 * 32))))
        print(json.dumps({"leg": "loader", "workers": w, "ms_per_batch": timed(lambda: sum(1 for _ in loader(w)))}),
              flush=True)
    staged = list(loader(1))
    for dt, native in (("f16", True), ("f16", False), ("f32", False)):
        infer._NATIVE = native
        sw = InferenceSweep(G, taus, dtype=dt)
        sw.run_stream(loader(1, list(range(4 * 32))))
        with sw._eval():
            for b in staged[:3]:
                sw.run_batch(*b)

            def run_staged():
                for b in staged:
                    sw.run_batch(*b)
                return len(staged)

            st_ms = timed(run_staged)
            t0 = time.perf_counter()
            for b in staged:
                sw.run_batch(*b)
            host_ms = round((time.perf_counter() - t0) / len(staged) * 1e3, 3)
            torch.cuda.synchronize()
        sw2 = InferenceSweep(G, taus, graphed=True, dtype=dt)
        sw2.run_batch(*staged[0])
        torch.cuda.synchronize()
        a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(20):
            sw2.run_batch(*staged[0])
        e.record()
        torch.cuda.synchronize()
        dev_ms = round(a.elapsed_time(e) / 20, 3)
        del sw2
        rec = {"leg": "forward", "dtype": dt, "native": native, "staged_ms_per_batch": st_ms,
               "staged_host_ms_per_batch": host_ms, "device_ms_per_batch": dev_ms}
        for w in workers:
            rec[f"stream_ms_per_batch_w{w}"] = timed(lambda: sw.run_stream(loader(w))["batches"])
        print(json.dumps(rec), flush=True)
        del sw


if __name__ == "__main__":
    main()
