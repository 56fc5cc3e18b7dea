"""Device time of the same launches issued eagerly and replayed from a hipGraph.

The fresh-batch step (Trainer.step_fresh) runs the stacked critic-label
forward and the generator iteration eagerly, the replayed step
(step_graphed) from graphs.  Here both forms run with the host far ahead of
the device (a torch.cuda._sleep kernel first), so the device time between
two events is the device's own cost of the launches -- any difference is
per-launch device overhead of eager dispatch, not host speed.  One JSON line.
"""
from __future__ import annotations

import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))


def timed(fn, reps=10, sleep_cycles=20_000_000):
    """device ms of fn() with the host ahead: sleep kernel, event, fn, event"""
    out = []
    for _ in range(reps):
        torch.cuda.synchronize()
        torch.cuda._sleep(sleep_cycles)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    out.sort()
    return round(out[len(out) // 2], 4)


def main():
    import bench
    from vgan.config import Configuration
    from vgan.data import prepared

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Configuration()
    cfg.DEVICE = str(dev)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    pool = bench.make_pool(cfg, 0, 1, 1, 32, dev)
    tr = bench.build_trainer(cfg, "f32")
    loc, vox = pool[0]
    prepared(loc, vox, cfg.NUM_CLASSES)
    for _ in range(2):
        tr.step(loc, vox)
    graphs = tr.capture(loc, vox)
    torch.cuda.synchronize()

    def eager_labels():
        tr._critic_labels(loc, vox)

    def eager_gen():
        tr._gen_iteration(loc, vox)
        tr.adam_g.step(counted=True)

    # the critic iteration as step_fresh records it (raw capture into the fresh
    # pool, executable graph instantiated / updated in place, vg_graph_launch)
    from vgan._lib import LIB, check, stream_handle

    with torch.no_grad():
        hard_all, soft_all = tr._critic_labels(loc, vox)
    slot = (hard_all[0:1].clone(), soft_all[0:1].clone())
    acc = torch.zeros(cfg.N_CRITIC + 1, device=dev)
    execs = []
    for _ in range(3):  # the first instantiates, the next two update in place (ping-pong)
        g_c, _ = tr._fresh_record(lambda: tr._critic_body(loc, vox, acc, True, slot, 0, False))
        execs.append(tr._fresh_exec("critic", g_c))
        tr._fresh_done("critic", torch.cuda.current_stream())
    st = stream_handle(dev)

    def fresh_critic(ex):
        return lambda: check(LIB.vg_graph_launch(ex, st), "vg_graph_launch")

    res = {
        "critic_fresh_instantiated_ms": timed(fresh_critic(execs[0])),
        "critic_fresh_updated_ms": timed(fresh_critic(execs[2])),
        "labels_eager_ms": timed(eager_labels),
        "labels_graph_ms": timed(lambda: graphs["labels"].replay()),
        "gen_eager_ms": timed(eager_gen),
        "gen_graph_ms": timed(lambda: graphs["gen"].replay()),
        "critic_graph_ms": timed(lambda: graphs["critic"][0].replay()),
    }
    # the tiny-kernel floor both ways: 200 dependent one-element adds
    x = torch.zeros(1, device=dev)

    def adds():
        for _ in range(200):
            x.add_(1.0)

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        adds()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        adds()
    res["tiny_add_eager_us"] = round(timed(adds) * 1e3 / 200, 3)
    res["tiny_add_graph_us"] = round(timed(g.replay) * 1e3 / 200, 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
