"""Where the fresh-batch step loses time against the replayed step.

    python tools/fresh_probe.py [--steps 40] [--warmup 5]

Variants of bench.py's fresh-batch leg (a NEW batch every step through
Trainer._train_batch -> step_fresh), each timed between device syncs:

  loader    GraphLoader prefetching 3 batches on its thread, per-batch
            structures built on the device
  prepared  the same with prepare=NUM_CLASSES (bench.py's leg: the host
            collate also builds type-mean, CSR / ELL, the critic's stacked
            graph, one upload)
  staged    the prepared batches collated and uploaded before the timed
            region (each batch still new to the trainer: capture inside it)
  sync      staged, with a device synchronisation after every step (the
            device time of a step without host work overlapping it)
  quiet     staged, the host waiting for the device after the labels, the
            critic replays and the generator iteration (no host activity
            while they run)
  switch    prepared, with the default 5 ms GIL switch interval (the loader
            lowers it to 0.1 ms while prefetching, vgan/loader.py)

Each line also carries the host time per step phase (Trainer.phase_hook:
prepare / labels / capture / replays / gen / release), medians in ms.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

TIMELINE = os.environ.get("FRESH_TIMELINE", "0") == "1"  # events at the phase marks (device lag per phase)


def run(variant, cfg, bench, dev, steps, warmup, batch=32):
    from vgan.loader import GraphLoader
    from vgan.store import write_store
    from vgan.synth import SyntheticDataset

    n = warmup + steps
    tmp = tempfile.mkdtemp(prefix="vgan_probe_")
    ds = SyntheticDataset(n * batch, seed=4321)
    store = write_store(os.path.join(tmp, "store"), ds)
    prep = None if variant == "loader" else cfg.NUM_CLASSES
    loader = GraphLoader(store, batch_size=batch, shuffle=True, device=dev, prefetch=3, seed=4321, prepare=prep)
    torch.manual_seed(cfg.SEED)
    tr = bench.build_trainer(cfg, "f32")
    cfg.runtime["train_step"] = "auto"
    import vgan.loader as vl
    old = vl._SWITCH_INTERVAL
    if variant == "switch":
        vl._SWITCH_INTERVAL = 5e-3
    if variant in ("staged", "sync", "quiet"):
        batches = list(loader)
        torch.cuda.synchronize()
        it = iter(batches)
    else:
        it = iter(loader)
    for _ in range(warmup):
        tr._train_batch(*next(it))
    torch.cuda.synchronize()
    phases = {}
    last = [0.0]

    timeline = []  # (phase, host time at its end, event recorded there)

    def mark(name):
        t = time.perf_counter()
        phases.setdefault(name, []).append((t - last[0]) * 1e3)
        last[0] = t
        if TIMELINE:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            timeline.append((name, t, ev))
        if variant == "quiet" and name in ("labels", "replays", "gen"):
            torch.cuda.synchronize()  # the host idles while those phases run

    tr.phase_hook = mark
    time.sleep(0.05)  # a >= 40 ms idle gap: tools/prof_summary.py --after-gap keeps what follows
    ref = torch.cuda.Event(enable_timing=True)
    ref.record()  # the device is idle: it reaches ref at ~host time t_ref
    t_ref = time.perf_counter()
    per = []
    t0 = time.perf_counter()
    for _ in range(steps):
        a = time.perf_counter()
        last[0] = a
        tr._train_batch(*next(it))
        if variant == "sync":  # no host / device overlap: each step's device time alone
            torch.cuda.synchronize()
        per.append((time.perf_counter() - a) * 1e3)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps * 1e3
    vl._SWITCH_INTERVAL = old
    del it, loader
    shutil.rmtree(tmp, ignore_errors=True)
    tr.phase_hook = None
    lag = {}
    if TIMELINE:
        # device time at which each phase-end marker executed, minus the host
        # time it was enqueued: ~0 = the device had caught up with the host
        # there (it idled before); large = work was queued ahead of it
        for name, t, ev in timeline:
            dev_ms = ref.elapsed_time(ev)
            lag.setdefault(name, []).append(dev_ms - (t - t_ref) * 1e3)
        lag = {k: {"median": round(sorted(v)[len(v) // 2], 3), "min": round(min(v), 3)} for k, v in lag.items()}
        # device time between consecutive markers = the device time of the work
        # enqueued in that phase, when the device never idled (lag stays > 0)
        dd = {}
        for (n0, _, e0), (n1, _, e1) in zip(timeline, timeline[1:]):
            dd.setdefault(n1, []).append(e0.elapsed_time(e1))
        lag["device_ms_per_phase"] = {k: round(sorted(v)[len(v) // 2], 3) for k, v in dd.items()}
    per.sort()
    med = {k: round(sorted(v)[len(v) // 2], 3) for k, v in phases.items()}
    return {"variant": variant, "ms_per_step": round(el, 3), "host_call_ms_median": round(per[len(per) // 2], 3),
            "host_call_ms_max": round(per[-1], 3), "phase_ms_median": med,
            **({"device_lag_ms": lag} if TIMELINE else {})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--variants", default="prepared,loader,staged,switch,prepared")
    args = ap.parse_args()
    import bench
    from vgan.config import Configuration

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    for v in args.variants.split(","):
        print(json.dumps(run(v, cfg, bench, dev, args.steps, args.warmup)), flush=True)


if __name__ == "__main__":
    main()
