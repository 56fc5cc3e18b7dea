"""Do independent branches of a captured hipGraph run concurrently here?

    python tools/graph_concurrency.py

Captures 2 x K small dependent kernels (a) on one stream and (b) as two
forked branches of K each (side stream joined at the end), replays both and
prints the per-replay device times (us)."""
import json

import torch


def chain(t, k):
    for _ in range(k):
        t.mul_(1.0001).add_(0.5)


def main():
    dev = torch.device("cuda", 0)
    k = 30
    a = torch.randn(200_000, device=dev)
    b = torch.randn(200_000, device=dev)
    side = torch.cuda.Stream(dev)
    res = {}
    for name in ("serial", "forked"):
        g = torch.cuda.CUDAGraph()
        chain(a, 1)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            if name == "serial":
                chain(a, k)
                chain(b, k)
            else:
                cur = torch.cuda.current_stream(dev)
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    chain(b, k)
                chain(a, k)
                cur.wait_stream(side)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        res[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / 20, 1)
    res["kernels_per_replay"] = 4 * k
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
