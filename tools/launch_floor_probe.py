"""Device time per kernel of a hipGraph of K dependent tiny kernels (one
element each, and one 13 MB streaming read/write each): the floor a
latency-bound kernel of the step pays per launch on this box.  One JSON line."""
import json

import torch


def per_kernel(fn, k=200, reps=10):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(k):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * k)


def main():
    dev = torch.device("cuda", 0)
    x1 = torch.zeros(1, device=dev)
    xb = torch.zeros(13107 * 64 * 4, device=dev)  # 13 MB, the size of a critic activation
    yb = torch.zeros_like(xb)
    res = {"tiny_add_us": per_kernel(lambda: x1.add_(1.0)),
           "copy_13MB_us": per_kernel(lambda: yb.copy_(xb)),
           "add_13MB_inplace_us": per_kernel(lambda: xb.add_(1.0))}
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
