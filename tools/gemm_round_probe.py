"""Is a <= 64-column GEMM paying a second workgroup round?  vg_gemm
(k_gemm16: 64-row tiles, 16-wave workgroups, two per CU) timed in a replayed
hipGraph of 50 launches against the row count, across the 512-workgroup
(= 2 x 256 CUs) boundary at 32,768 rows.  python tools/gemm_round_probe.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd"))

import torch  # noqa: E402

from vgan._lib import LIB, check, ptr, stream_handle  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    M = K = 64
    for rows in (16384, 24576, 32000, 32768, 33000, 34000, 38100, 49152, 65536, 98304):
        A = torch.randn(rows, K, device=dev)
        W = torch.randn(M, K, device=dev)
        C = torch.empty(rows, M, device=dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            st = stream_handle(dev)
            for _ in range(3):
                check(LIB.vg_gemm(ptr(A), K, ptr(W), K, 1, None, 0, None, 0, ptr(C), M, rows, M, K, st), "vg_gemm")
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=side):
                st = stream_handle(dev)
                for _ in range(50):
                    check(LIB.vg_gemm(ptr(A), K, ptr(W), K, 1, None, 0, None, 0, ptr(C), M, rows, M, K, st),
                          "vg_gemm")
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(side):
            a.record()
            for _ in range(5):
                g.replay()
            b.record()
        torch.cuda.synchronize()
        print(json.dumps({"rows": rows, "workgroups": (rows + 63) // 64,
                          "us_per_gemm": round(a.elapsed_time(b) * 1000 / 250, 2)}), flush=True)


if __name__ == "__main__":
    main()
