"""How long does dropping a recorded torch CUDAGraph take, and does it wait for
the device?  Records graphs of `--nodes` small kernels into one shared pool
(as Trainer.step_fresh does) and times `del` of a two-step-old graph with the
device idle and with ~`--busy-ms` of queued work.

    python tools/graph_destroy_probe.py [--nodes 300] [--busy-ms 20]
"""
import argparse
import queue
import threading
import time

import torch


def record(pool, side, x, nodes, keep):
    g = torch.cuda.CUDAGraph(keep_graph=keep)
    with torch.cuda.stream(side):
        g.capture_begin(pool=pool, capture_error_mode="thread_local")
        y = x
        for _ in range(nodes):
            y = y * 1.0001 + 1e-6
        g.capture_end()
    return g


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=300)
    ap.add_argument("--busy-ms", type=float, default=20.0)
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    x = torch.randn(4096, device=dev)
    big = torch.randn(8192, 8192, device=dev)
    pool = torch.cuda.graph_pool_handle()
    side = torch.cuda.Stream(dev)
    cur = torch.cuda.current_stream(dev)
    # one matmul's duration, to size the busy queue
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        big @ big
    torch.cuda.synchronize()
    mm = (time.perf_counter() - t0) / 5
    n_busy = max(1, int(args.busy_ms / 1e3 / mm))
    for keep in (True, False):
        for busy in (False, True):
            times = []
            graphs = []
            for r in range(args.reps + 2):
                side.wait_stream(cur)
                g = record(pool, side, x, args.nodes, keep)
                cur.wait_stream(side)
                if keep:
                    g.instantiate()
                g.replay()
                graphs.append(g)
                if len(graphs) > 2:
                    old = graphs.pop(0)
                    torch.cuda.synchronize()
                    if busy:
                        for _ in range(n_busy):
                            big @ big
                    t0 = time.perf_counter()
                    del old
                    times.append(time.perf_counter() - t0)
                    torch.cuda.synchronize()
            times.sort()
            print(f"keep_graph={keep} device {'busy ~%.0f ms' % (n_busy * mm * 1e3) if busy else 'idle':>12}: "
                  f"del of a {args.nodes}-node graph median {times[len(times) // 2] * 1e3:.3f} ms")
            del graphs
    # a background thread resetting old graphs: does the main thread still wait?
    q = queue.SimpleQueue()

    def reaper():
        while True:
            g = q.get()
            if g is None:
                return
            g.reset()

    th = threading.Thread(target=reaper, daemon=True)
    th.start()
    for busy in (False, True):
        times, launch = [], []
        graphs = []
        for r in range(args.reps + 2):
            side.wait_stream(cur)
            g = record(pool, side, x, args.nodes, True)
            cur.wait_stream(side)
            g.instantiate()
            g.replay()
            graphs.append(g)
            if len(graphs) > 2:
                old = graphs.pop(0)
                torch.cuda.synchronize()
                if busy:
                    for _ in range(n_busy):
                        big @ big
                t0 = time.perf_counter()
                q.put(old)
                del old
                t1 = time.perf_counter()
                for _ in range(200):  # main-thread launches while the reaper works
                    x.mul_(1.0)
                t2 = time.perf_counter()
                times.append(t1 - t0)
                launch.append(t2 - t1)
                torch.cuda.synchronize()
        times.sort()
        launch.sort()
        print(f"background reset, device {'busy' if busy else 'idle'}: hand-off {times[len(times) // 2] * 1e3:.3f} ms, "
              f"then 200 launches {launch[len(launch) // 2] * 1e3:.3f} ms")
        del graphs
    q.put(None)
    th.join()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
