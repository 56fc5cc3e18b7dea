"""Is the replayed step bound by the host's submission of graph nodes?

    python tools/replay_host_probe.py [--steps 20] [--precision f32]

Captures the step graphs of one batch, then replays whole steps and records,
per step, the host time spent inside the replay calls (no synchronisation in
between) next to the device time of the same steps (HIP events).  If hipGraph
launch submits every kernel node from the host, a step whose host submission
time approaches its device time leaves the GPU idle wherever the host falls
behind (the 20-130 us idle gaps of the rocprofv3 step summary).  Also times
the replay of one graph alone, host and device, per node.  One JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--precision", default="f32")
    args = ap.parse_args()
    from vgan.config import Configuration

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg, args.precision)
    loc, vox = pool[0]
    for _ in range(3):
        tr.step_graphed(loc, vox)
    torch.cuda.synchronize()
    graphs = vox.derived(tr._graph_key)
    seq = ([graphs["labels"]] if graphs["labels"] is not None else []) + list(graphs["critic"]) + [graphs["gen"]]

    host, dev_ms = [], []
    for _ in range(args.steps):
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        st.record()
        t0 = time.perf_counter()
        for g in seq:
            g.replay()
        t1 = time.perf_counter()
        en.record()
        torch.cuda.synchronize()
        host.append((t1 - t0) * 1e3)
        dev_ms.append(st.elapsed_time(en))
    # back-to-back steps with no sync: the rate the bench sees
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for g in seq:
            g.replay()
    t_submit = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_total = time.perf_counter() - t0
    # one critic graph alone: host submission vs device time
    g = graphs["critic"][0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        g.replay()
    h1 = (time.perf_counter() - t0) / 10 * 1e3
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(10):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    d1 = st.elapsed_time(en) / 10
    host.sort()
    dev_ms.sort()
    print(json.dumps({"precision": args.precision, "graphs_per_step": len(seq),
                      "step_host_submit_ms_median": round(host[len(host) // 2], 3),
                      "step_device_ms_median": round(dev_ms[len(dev_ms) // 2], 3),
                      "back_to_back_submit_ms_per_step": round(t_submit / args.steps * 1e3, 3),
                      "back_to_back_total_ms_per_step": round(t_total / args.steps * 1e3, 3),
                      "critic_graph_host_ms": round(h1, 3), "critic_graph_device_ms": round(d1, 3)}))


if __name__ == "__main__":
    main()
