"""Per-phase device time of the hipGraph-captured step (batch 32, fp32).

    python tools/phase_times.py [--reps 20]

Replays each captured graph of one batch on its own between HIP events:
the stacked critic-label G forward, one critic iteration, the generator
iteration.  Prints one JSON line (ms per replay of each phase and their sum
for a full step)."""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def time_graph(g, reps: int) -> float:
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    st.record()
    for _ in range(reps):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    return st.elapsed_time(en) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dump", default="", help="directory: write each phase graph as a DOT file (debug mode)")
    ap.add_argument("--gaps", action="store_true",
                    help="end with one replay of each phase 100 ms apart (split a rocprofv3 trace by phase)")
    args = ap.parse_args()
    from vgan.config import Configuration

    if args.dump:  # every captured graph keeps its node list for debug_dump
        os.makedirs(args.dump, exist_ok=True)
        _orig_init = torch.cuda.CUDAGraph.__init__

        def _init(self, *a, **k):
            _orig_init(self, *a, **k)
            self.enable_debug_mode()

        torch.cuda.CUDAGraph.__init__ = _init

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg)
    loc, vox = pool[0]
    tr.step_graphed(loc, vox)
    torch.cuda.synchronize()
    graphs = vox.derived(tr._graph_key)
    if args.dump:
        for name, g in (("labels", graphs["labels"]), ("critic", graphs["critic"][0]), ("gen", graphs["gen"])):
            if g is not None:
                g.debug_dump(os.path.join(args.dump, f"{name}.dot"))
    res = {}
    if graphs["labels"] is not None:
        res["labels_ms"] = time_graph(graphs["labels"], args.reps)
    res["critic_ms"] = time_graph(graphs["critic"][0], args.reps)
    res["gen_ms"] = time_graph(graphs["gen"], args.reps)
    res["step_sum_ms"] = res.get("labels_ms", 0.0) + cfg.N_CRITIC * res["critic_ms"] + res["gen_ms"]
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(args.reps):
        tr.step_graphed(loc, vox)
    en.record()
    torch.cuda.synchronize()
    res["step_ms"] = st.elapsed_time(en) / args.reps
    if args.gaps:  # for a rocprofv3 kernel trace: one replay per phase, 100 ms apart
        import time

        for name in ("labels", "critic", "gen"):
            g = graphs["critic"][0] if name == "critic" else graphs[name]
            if g is None:
                continue
            torch.cuda.synchronize()
            time.sleep(0.1)
            g.replay()
        torch.cuda.synchronize()
    print(json.dumps({k: round(v, 4) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
