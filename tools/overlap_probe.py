"""Do two captured step graphs overlap when replayed on two streams?

    python tools/overlap_probe.py

Captures the stacked critic-label G forward and one critic iteration as two
hipGraphs with SEPARATE memory pools, then times (HIP events, R replays)
  serial      labels; critic        on one stream
  concurrent  labels || critic      on two streams, joined per replay
Values are meaningless (the critic reads labels while they are rewritten);
only the device time is of interest.  Prints one JSON line (us per pair)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def timed(fn, reps):
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from vgan.config import Configuration

    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg)
    loc, vox = pool[0]
    bench.run_steps(tr, pool, 2)  # lazy init + the trainer's own capture
    torch.cuda.synchronize()
    acc = torch.zeros(2, dtype=torch.float32, device=dev)
    pa, pb, pc = (torch.cuda.graph_pool_handle() for _ in range(3))
    gl = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gl, pool=pa):
        labels = tr._critic_labels(loc, vox)
    gc = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gc, pool=pb):
        tr._critic_body(loc, vox, acc, True, labels, 0)
    gc2 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gc2, pool=pc):
        tr._critic_body(loc, vox, acc, True, labels, 1)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    reps = 20

    def serial():
        gl.replay()
        gc.replay()

    def conc(ga, gb):
        def f():
            s1.wait_stream(main_s)
            s2.wait_stream(main_s)
            with torch.cuda.stream(s1):
                ga.replay()
            with torch.cuda.stream(s2):
                gb.replay()
            main_s.wait_stream(s1)
            main_s.wait_stream(s2)
        return f

    res = {}
    for _ in range(2):  # second round is the reported one
        res = {
            "labels_us": timed(gl.replay, reps),
            "critic_us": timed(gc.replay, reps),
            "serial_labels_critic_us": timed(serial, reps),
            "concurrent_labels_critic_us": timed(conc(gl, gc), reps),
            "serial_critic_critic_us": timed(lambda: (gc.replay(), gc2.replay()), reps),
            "concurrent_critic_critic_us": timed(conc(gc, gc2), reps),
        }
    print(json.dumps({k: round(v, 1) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
