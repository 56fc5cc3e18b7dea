import torch, time
dev = "cuda"
N = 12700
shapes = [(N, 128, 128), (N, 268, 128), (N, 524, 128), (N, 64, 64), (N, 36, 64), (N, 128, 64), (N, 16, 8)]
def bench(fn, reps=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3
for lib in ("hipblaslt", "rocblas"):
    try:
        torch.backends.cuda.preferred_blas_library("cublaslt" if lib == "hipblaslt" else "cublas")
    except Exception as ex:
        print("lib switch failed", ex); continue
    print("==", lib, torch.backends.cuda.preferred_blas_library())
    for (n, k, m) in shapes:
        x = torch.randn(n, k, device=dev); w = torch.randn(m, k, device=dev); gy = torch.randn(n, m, device=dev)
        b = torch.randn(m, device=dev)
        t_f = bench(lambda: torch.nn.functional.linear(x, w, b))
        t_dx = bench(lambda: gy @ w)
        t_dw = bench(lambda: gy.t() @ x)
        t_dw2 = bench(lambda: torch.mm(x.t(), gy).t())
        h = torch.randn(n, m, device=dev); v = torch.randn(m, device=dev)
        t_mv = bench(lambda: torch.mv(h, v))
        t_mv2 = bench(lambda: (h * v).sum(1))
        print(f"N={n} K={k} M={m}: fwd {t_f:7.1f} dX {t_dx:7.1f} dW {t_dw:7.1f} dW' {t_dw2:7.1f}  mv {t_mv:7.1f} mulsum {t_mv2:7.1f} us")
