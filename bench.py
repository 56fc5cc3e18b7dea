"""Benchmark: voxel-graphs/sec of the full G+D training step on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N ...

``--gpus N`` (N > 1) without a torch.distributed environment starts the N
ranks itself (``torch.distributed.run`` in a child process, before anything
touches the GPU) and relays rank 0's line; under torchrun each rank reads
RANK / LOCAL_RANK / WORLD_SIZE from the environment.

Workload (BASELINE.json configs[1]): 6-type synthetic dataset, batch = 32
voxel graphs per GPU, fp32, the full step of trainer.py:466-495 (5 critic
iterations with WGAN-GP + 1 generator iteration, Adam steps included, sklearn
metrics excluded as SURVEY.md 8d specifies).  Each rank cycles over its own
pool of pre-staged batches (inputs resident in HBM when the timed region
starts); with N ranks every rank trains its own 32-building batch and the flat
gradients are averaged over RCCL (weak scaling).

Rank 0 prints ONE JSON line.  ``roofline`` is for the dominant message-passing
kernel, vg_gat_fwd: algorithmic bytes per launch / its average duration from
HIP events recorded on the launch stream around every launch of K instrumented
steps of the same workload run right after the timed region (the timed
region itself is uninstrumented).  ``roofline_stress`` is the same kernel on
config #4 (8 x 50k-node buildings, E' ~ 8.6M) where HBM, not latency, bounds it.
``cpu_baseline`` times the CPU oracle (restatement of the reference step,
pinned bit-for-bit to the reference by tests/golden) on one batch-32 step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd")
for _p in (ROOT, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "voxel-graphs/sec (full G+D step)"


def log(msg: str) -> None:
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def agg_bytes(n: int, e: int, c: int, elem: int = 4) -> int:
    """Algorithmic (compulsory) bytes of one aggregation launch, SURVEY.md 8(d)
    strictly: read h [N,C] and write out [N,C] (``elem`` bytes each), read
    a_src / a_dst [N] f32, col [E'] and row_ptr [N+1] int32.  Outputs the
    implementation chooses to write besides ``out`` (alpha for the backward,
    the GraphNorm partials) are not counted."""
    return 2 * n * c * elem + 4 * (2 * n + e + (n + 1))


L2_PEAK_GBS = 34500.0  # MI355X_MICROARCH.md: L2 (8 x 4 MiB) aggregate
L2_GATHER_GBS = 18800.0  # MI355X_MICROARCH.md: rows gathered from the XCD's L2, measured ceiling (16.8-18.8 TB/s)


def agg_gather_bytes(n: int, e: int, c: int, elem: int = 4) -> int:
    """Bytes the aggregation moves between L2 and the CUs: every edge's whole
    source row (E' * C), its column index and a_src entry, the output row and
    the per-row operands.  The HBM compulsory bytes (agg_bytes) count each
    source row once; the gather reads it once per edge (~6.2x at batch 32,
    ~21.6x on the stress graph), from L2 / the Infinity Cache."""
    return e * c * elem + 4 * 2 * e + n * c * elem + 4 * (2 * n + (n + 1))


def agg_extra_bytes(n: int, e: int) -> int:
    """alpha [E'] f32, written for the backward (not in agg_bytes)."""
    return 4 * e


def step_aggregate_calls(tr, csr):
    """(CSR, channels) of every vg_gat_aggregate_fwd launch in one full step:
    the stacked critic-label G forward (N_CRITIC copies), N_CRITIC critic
    iterations (D over the real / fake / mix stack), the generator
    iteration's G forward and its D forward."""
    n_critic = tr.configuration.N_CRITIC
    gw = tr.generator.encoder.widths[1:]
    dw = tr.discriminator.encoder.widths[1:]
    calls = []
    if tr._stacked_labels():
        calls += [(csr.stacked(n_critic), c) for c in gw]
    calls += [(csr.stacked(3), c) for _ in range(n_critic) for c in dw]
    calls += [(csr, c) for c in gw] + [(csr, c) for c in dw]
    return calls


def gnp_bytes(csr, c: int) -> int:
    """Bytes of the GraphNorm block partials vg_gat_aggregate_fwd_gnp writes
    (count, mean, M2 per column and workgroup; slot 1 of a straddling block is
    not counted)."""
    from vgan._lib import LIB

    g = int(LIB.vg_gat_gnp_rows(csr.num_nodes, c))
    return 4 * 3 * c * (-(-csr.num_nodes // g))


def aggregate_roofline(tr, csr, device, reps: int = 20, gnp: bool = False):
    """Average device duration of the scatter kernel (vg_gat_aggregate_fwd)
    over the step's own mix of launches: one launch per call of a step, on the
    step's CSRs and channel counts, captured in a hipGraph and replayed
    ``reps`` times between HIP events on the replay stream (back-to-back
    launches, as inside the step's own graphs).  gnp: the variant the step
    runs (vg_gat_aggregate_fwd_gnp: the following GraphNorm's column partials
    in the epilogue; its bytes add the partials written)."""
    from vgan import ops
    from vgan._lib import ptr, stream_handle

    calls = step_aggregate_calls(tr, csr)
    gen = torch.Generator(device=device)
    gen.manual_seed(1234)
    bufs = {}
    for c_csr, c in calls:
        key = (c_csr.num_nodes, c)
        if key not in bufs:
            n = c_csr.num_nodes
            bufs[key] = [torch.randn(n, c, device=device, generator=gen),
                         0.3 * torch.randn(n, device=device, generator=gen),
                         0.3 * torch.randn(n, device=device, generator=gen),
                         torch.randn(c, device=device, generator=gen),
                         torch.empty(n, c, device=device),
                         torch.empty(c_csr.num_edges, device=device),
                         ops.gnp_buffer(c_csr, c, device)[0] if gnp else None]
    if gnp and any(b[-1] is None for b in bufs.values()):
        return None

    def launch_all():
        st = stream_handle(device)
        for c_csr, c in calls:
            h, a_s, a_d, b, out, alpha, part = bufs[(c_csr.num_nodes, c)]
            ops.aggregate_fwd_raw(c_csr, c, ptr(h), ptr(a_s), ptr(a_d), ptr(b), 0.2, ptr(out), ptr(alpha), st, part)

    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        launch_all()
    torch.cuda.current_stream(device).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        launch_all()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    total_ms = st.elapsed_time(en)
    launches = reps * len(calls)
    nbytes = reps * sum(agg_bytes(c_csr.num_nodes, c_csr.num_edges, c) for c_csr, c in calls)
    gbytes = reps * sum(agg_gather_bytes(c_csr.num_nodes, c_csr.num_edges, c) for c_csr, c in calls)
    extra = reps * sum(agg_extra_bytes(c_csr.num_nodes, c_csr.num_edges) + (gnp_bytes(c_csr, c) if gnp else 0)
                       for c_csr, c in calls)
    return {"launches": launches, "launches_per_step": len(calls), "avg_us": total_ms * 1e3 / launches,
            "avg_bytes": nbytes / launches, "achieved_gbs": nbytes / (total_ms * 1e-3) / 1e9,
            "avg_extra_written_bytes": extra / launches, "gather_gbs": gbytes / (total_ms * 1e-3) / 1e9,
            "avg_gather_bytes": gbytes / launches}


F32_MFMA_PEAK_TFLOPS = 157.3  # MI355X_MICROARCH.md: dense f32-input MFMA (v_mfma_f32_32x32x2_f32)


def step_gemm_calls(tr, n: int):
    """The step's k_gemm16 products (one f32 step at n voxel rows): every
    GATConv projection with its attention projections (vg_gat_lin_att) and
    every GATConv input gradient dX = dH W (vg_gemm NN; the step forms most
    of them with vg_gemm_gn_bwd, the same tiles plus the GraphNorm partials).
    (kind, rows, cin, cout) per launch, in step order."""
    cfg = tr.configuration
    k = cfg.N_CRITIC
    dw = [(conv.in_channels, conv.out_channels) for conv, _ in tr.critic.blocks]
    G = tr.generator
    gw = [(getattr(G.encoder, f"module_{4 * b}").in_channels, getattr(G.encoder, f"module_{4 * b}").out_channels)
          for b in range(G.encoder.num_blocks)]
    calls = [("att", k * n, ci, co) for ci, co in gw]  # stacked critic-label forward
    for _ in range(k):  # critic iterations: passes A (3 copies), B, C, D (3 copies)
        calls += [("att", 3 * n, ci, co) for ci, co in dw]
        calls += [("nn", n, co, ci) for ci, co in reversed(dw[1:])]
        calls += [("att", n, ci, co) for ci, co in dw]
        calls += [("nn", 3 * n, co, ci) for ci, co in reversed(dw[1:])]
    calls += [("att", n, ci, co) for ci, co in gw + dw]  # generator iteration: G and D forward
    calls += [("nn", n, co, ci) for ci, co in reversed(dw[1:])] + [("nn", n, co, ci) for ci, co in reversed(gw[1:])]
    return calls


def gemm_family_roofline(tr, n: int, device, reps: int = 20):
    """The dense-product family (k_gemm16) as the step launches it: the shapes
    of step_gemm_calls, captured in one hipGraph and replayed between HIP
    events.  FLOPs 2 * rows * cin * cout; compulsory bytes the operand rows,
    the output rows, the weight (and a_src / a_dst for the projections)."""
    from vgan._lib import check, dense, ptr, stream_handle

    calls = step_gemm_calls(tr, n)
    gen = torch.Generator(device=device)
    gen.manual_seed(4321)
    bufs = {}
    for kind, rows, ci, co in calls:
        key = (kind, rows, ci, co)
        if key in bufs:
            continue
        if kind == "att":
            bufs[key] = (torch.randn(rows, ci, device=device, generator=gen),
                         torch.randn(co, ci, device=device, generator=gen),
                         torch.randn(co, device=device, generator=gen), torch.randn(co, device=device, generator=gen),
                         torch.empty(rows, co, device=device), torch.empty(rows, device=device),
                         torch.empty(rows, device=device))
        else:  # dX [rows, co_in] = dH [rows, ci] W [ci, co_in] with (ci, co) = (c, cin)
            bufs[key] = (torch.randn(rows, ci, device=device, generator=gen),
                         torch.randn(ci, co, device=device, generator=gen), torch.empty(rows, co, device=device))

    def launch_all():
        st = stream_handle(device)
        for kind, rows, ci, co in calls:
            b = bufs[(kind, rows, ci, co)]
            if kind == "att":
                x, w, vs, vd, h, a_s, a_d = b
                check(dense("vg_gat_lin_att")(ptr(x), ci, ptr(w), rows, ci, co, ptr(vs), ptr(vd), ptr(h), ptr(a_s),
                                              ptr(a_d), st), "vg_gat_lin_att")
            else:
                a, w, out = b
                check(dense("vg_gemm")(ptr(a), ci, ptr(w), co, 0, None, 0, None, 0, ptr(out), co, rows, co, ci, st),
                      "vg_gemm")

    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        launch_all()
    torch.cuda.current_stream(device).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        launch_all()
    g.replay()
    torch.cuda.synchronize()
    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st.record()
    for _ in range(reps):
        g.replay()
    en.record()
    torch.cuda.synchronize()
    sec = st.elapsed_time(en) * 1e-3
    flops = reps * sum(2.0 * rows * ci * co for _, rows, ci, co in calls)
    nbytes = reps * sum(4.0 * (rows * ci + rows * co + ci * co + (2 * rows if kind == "att" else 0))
                        for kind, rows, ci, co in calls)
    launches = reps * len(calls)
    return {"kernel": "k_gemm16 family (vg_gat_lin_att projections + dX products at the step's shapes)",
            "launches_per_step": len(calls), "avg_launch_us": round(sec * 1e6 / launches, 3),
            "achieved_tflops": round(flops / sec / 1e12, 3),
            "frac_of_f32_mfma": round(flops / sec / 1e12 / F32_MFMA_PEAK_TFLOPS, 5),
            "f32_mfma_peak_tflops": F32_MFMA_PEAK_TFLOPS,
            "achieved_gbs": round(nbytes / sec / 1e9, 2), "frac_of_hbm": round(nbytes / sec / 1e9 / HBM_PEAK_GBS, 5),
            "avg_flops": int(flops / launches), "avg_compulsory_bytes": int(nbytes / launches),
            "timing": "hipGraph-replayed between HIP events on the replay stream (f32 operands)"}


def load_pmc_traffic(name: str = "r06_pmc_aggregate_gnp.json"):
    """Per-launch HBM-side bytes of the scatter kernel from the committed
    rocprofv3 PMC summary of the variant the step runs (tools/pmc_roofline.sh
    --gnp), or (None, None) when this round has not measured it: an older
    round's summary describes other kernels and is not reported."""
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None, None
    with open(path) as f:
        d = json.load(f)
    return d.get("traffic_bytes_per_launch"), os.path.relpath(path, ROOT)


# rocprofv3 kernel-trace summaries the roofline fractions are priced on
# (tools/roofline_trace.sh, tools/stress_trace.sh); the live HIP-event figures
# of the same launches are reported beside them
ROOFLINE_TRACE = "r06_roofline_kernel_trace_gnp.txt"
STRESS_TRACE = "r06_stress_ring_kernel_trace.txt"


def load_trace_mean(name: str):
    """{launches, avg_us, source} from the first line of a committed
    rocprofv3 summary ("... launches traced: L; average duration T us ..."),
    or None when this round has not committed it."""
    import re

    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        m = re.search(r"launches traced: (\d+); average duration ([0-9.]+) us", f.readline())
    if not m:
        return None
    return {"launches": int(m.group(1)), "avg_us": float(m.group(2)), "source": os.path.relpath(path, ROOT)}


def stress_model_leg(device, reps: int = 5):
    """configs[3] through the drop-in: ``VoxelGNNGenerator.forward`` (eval,
    no grad: the fused encoder, 14 GAT blocks) on the 8 x 50k stress batch,
    voxels in lattice-block numbering, with the LDS ring dispatched for the
    64 / 128-channel layers (ops.CSR.ring_on; its GraphNorm statistics from
    their own pass, or from the ring's loaders: ring_gnp) and with it
    switched off (the register gather); median of ``reps`` warm forwards
    between HIP events."""
    from vgan import ops
    from vgan.config import Configuration
    from vgan.graph import GraphBatch
    from vgan.locality import blocked
    from vgan.models import VoxelGNNGenerator
    from vgan.synth import make_stress_building

    items = [make_stress_building(777, i) for i in range(8)]
    loc = GraphBatch.from_data_list([lo for lo, _ in items]).to(device)
    vox = GraphBatch.from_data_list([blocked(v)[0] for _, v in items]).to(device)
    cfg = Configuration()
    cfg.DEVICE = str(device)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    G = VoxelGNNGenerator(cfg, 17, 12).eval()
    n = vox.num_nodes
    z = torch.randn(1, n, cfg.Z_DIM, device=device)
    out = {"workload": f"VoxelGNNGenerator.forward, eval, no grad, 8 x 50k-voxel stress buildings (N={n}), "
                       f"lattice-block numbering, {G.encoder.num_blocks} GAT blocks of widths {G.encoder.widths}"}
    saved = ops._RING, ops._RING_GNP
    try:
        # the ring as dispatched (the GraphNorm forms its statistics from its
        # input), the ring with the partials from its loaders (VGAN_RING_GNP=1),
        # the register gather (with the _gnp partials)
        for label, on, gnp in (("ring", True, False), ("ring_gnp", True, True), ("register", False, True)):
            ops._RING, ops._RING_GNP = on, gnp
            with torch.no_grad():
                for _ in range(2):
                    G(loc, vox, z)
                torch.cuda.synchronize()
                d0 = ops.RING_DISPATCHES
                times = []
                for _ in range(reps):
                    st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    st.record()
                    G(loc, vox, z)
                    en.record()
                    torch.cuda.synchronize()
                    times.append(st.elapsed_time(en))
            ms = sorted(times)[len(times) // 2]
            out[label] = {"ms_per_forward": round(ms, 3), "graphs_per_s": round(8 / (ms * 1e-3), 1),
                          "ring_launches_per_forward": (ops.RING_DISPATCHES - d0) // reps}
            log(f"stress model forward ({label}): {ms:.2f} ms, {out[label]['ring_launches_per_forward']} ring launches")
    finally:
        ops._RING, ops._RING_GNP = saved
    out["speedup"] = round(out["register"]["ms_per_forward"] / out["ring"]["ms_per_forward"], 3)
    return out


def make_pool(cfg, rank: int, world: int, pool: int, batch: int, device):
    from vgan.synth import SyntheticDataset

    ds = SyntheticDataset(6500, seed=777)
    out = []
    for b in range(pool):
        idx = [((b * world + rank) * batch + i) % len(ds) for i in range(batch)]
        loc, vox = ds.batch(idx)
        out.append((loc.to(device), vox.to(device)))
    return out


def build_trainer(cfg, precision: str = "f32"):
    from vgan.models import VoxelGNNDiscriminator, VoxelGNNGenerator
    from vgan.trainer import Trainer

    torch.manual_seed(cfg.SEED)
    G = VoxelGNNGenerator(cfg, 17, 12)
    D = VoxelGNNDiscriminator(cfg, 17, 12)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(og, T_max=cfg.EPOCHS)
    cfg.runtime["precision"] = precision
    return Trainer(G, D, None, og, od, sched, cfg)


GRAPHED = True


def run_steps(tr, pool, k: int, offset: int = 0):
    out = None
    for s in range(k):
        loc, vox = pool[(offset + s) % len(pool)]
        out = tr.step_graphed(loc, vox) if GRAPHED else tr.step(loc, vox)
    return out


def timed_steps(tr, pool, steps: int, warmup: int, world: int, device, profile: bool = False, per_step=None):
    """Warm-up (every pooled batch once: its CSR / type-mean / graphs), then
    ``steps`` timed steps between barrier + synchronize on both sides; the
    max over ranks.  Returns seconds.  ``per_step`` (a list) receives each
    step's milliseconds from HIP events recorded between the steps on the
    replay stream (no host synchronisation inside the timed region)."""
    for (loc, vox) in pool:
        run_steps(tr, [(loc, vox)], 1)
    run_steps(tr, pool, warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    if profile:
        time.sleep(0.05)  # idle gap that tools/prof_summary.py --after-gap keys on
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if per_step is not None else None
    t0 = time.perf_counter()
    if evs:
        evs[0].record()
    for s in range(steps):
        run_steps(tr, pool, 1, offset=s)
        if evs:
            evs[s + 1].record()
        if (s + 1) % 10 == 0:
            log(f"step {s + 1}/{steps}")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if evs:
        per_step.extend(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def stress_roofline(device, channels=(128, 64, 1), reps: int = 20, order: str = "rowmajor", ring_only: bool = False):
    """vg_gat_aggregate_fwd on config #4 (8 x 50k-node buildings), cold MALL;
    for C a multiple of 64 also vg_gat_aggregate_fwd_lds (16-row tiles'
    distinct source rows staged through LDS) and, for C = 64 / 128,
    vg_gat_aggregate_fwd_staged (the persistent kernel staging 64-row tiles
    while the previous tile is aggregated); all bit-identical.  order:
    "rowmajor" (the reference's numbering), "tiled" (4 x 4 (y, x) tiles per
    floor) or "blocked" (4 x 4 x 4 lattice blocks), vgan.locality."""
    from vgan import ops
    from vgan._lib import LIB, check, ptr, stream_handle
    from vgan.synth import make_stress_building
    from vgan.graph import GraphBatch
    from vgan.locality import blocked, tiled

    items = [make_stress_building(777, i)[1] for i in range(8)]
    voxels = items if order == "rowmajor" else [tiled(v, 4)[0] if order == "tiled" else blocked(v)[0] for v in items]
    vox = GraphBatch.from_data_list(voxels).to(device)
    csr = ops.CSR(vox.edge_index, vox.num_nodes)
    n, e = csr.num_nodes, csr.num_edges
    plan = csr.tile_plan()
    tiles = (n + 15) // 16
    uniq = plan[:tiles].clamp_min(0).sum().item()
    splan = csr.stage_plan()
    rplan = csr.ring_plan()
    uc = splan[:csr.stage_tiles()]
    staged_tiles = int((uc > 0).sum().item())
    s_uniq = float(uc.clamp_min(0).sum().item()) / max(1, staged_tiles)
    log(f"tile plans ({order}): 16-row {uniq / tiles:.1f} distinct sources for {e / tiles:.1f} edges, "
        f"64-row {s_uniq:.1f} for {4 * e / tiles:.1f} ({staged_tiles} staged, "
        f"{int((uc < 0).sum().item())} from global memory)")
    scratch = torch.empty(512 * 1024 * 1024 // 4, device=device)  # flush the 256 MB MALL between reps
    res, res_lds, res_st, res_ring, res_ring_gnp = {}, {}, {}, {}, {}
    for c in channels:
        h = torch.randn(n, c, device=device)
        a_s, a_d = 0.3 * torch.randn(n, device=device), 0.3 * torch.randn(n, device=device)
        bias = torch.randn(c, device=device)
        out, alpha = torch.empty(n, c, device=device), torch.empty(e, device=device)

        def run():
            ops.aggregate_fwd_raw(csr, c, ptr(h), ptr(a_s), ptr(a_d), ptr(bias), 0.2, ptr(out), ptr(alpha),
                                  stream_handle(device))

        def run_lds():
            check(LIB.vg_gat_aggregate_fwd_lds(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s), ptr(a_d),
                                               ptr(bias), 0.2, ptr(out), ptr(alpha), ptr(plan), csr._tile_umax,
                                               stream_handle(device)),
                  "vg_gat_aggregate_fwd_lds")

        def run_staged():
            check(LIB.vg_gat_aggregate_fwd_staged(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s),
                                                  ptr(a_d), ptr(bias), 0.2, ptr(out), ptr(alpha), ptr(splan),
                                                  stream_handle(device)),
                  "vg_gat_aggregate_fwd_staged")

        ring_err = torch.zeros(1, dtype=torch.int32, device=device)

        def run_ring():
            check(LIB.vg_gat_aggregate_fwd_ring(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s), ptr(a_d),
                                                ptr(bias), 0.2, ptr(out), ptr(alpha), ptr(rplan), ptr(ring_err),
                                                stream_handle(device)),
                  "vg_gat_aggregate_fwd_ring")

        gnp_r = torch.empty(int(LIB.vg_gat_ring_gnp_floats(n, c)), device=device) if c in (64, 128) else None

        def run_ring_gnp():  # as the drop-in runs it: with the following GraphNorm's column partials
            check(LIB.vg_gat_aggregate_fwd_ring_gnp(ptr(csr.row_ptr), ptr(csr.col), n, c, ptr(h), ptr(a_s),
                                                    ptr(a_d), ptr(bias), 0.2, ptr(out), ptr(alpha), ptr(rplan), n,
                                                    ptr(gnp_r), ptr(ring_err), stream_handle(device)),
                  "vg_gat_aggregate_fwd_ring_gnp")

        def timed(fn):
            for _ in range(3):
                fn()
            times = []
            for _ in range(reps):
                scratch.fill_(1.0)
                st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                st.record()
                fn()
                en.record()
                torch.cuda.synchronize()
                times.append(st.elapsed_time(en))
            return sum(times) / len(times)

        b, gb = agg_bytes(n, e, c), agg_gather_bytes(n, e, c)
        if not ring_only:
            avg = timed(run)
            res[c] = {"avg_us": avg * 1e3, "bytes": b, "achieved_gbs": b / (avg * 1e-3) / 1e9,
                      "gather_gbs": gb / (avg * 1e-3) / 1e9}
            if c % 64 == 0:
                avg = timed(run_lds)
                res_lds[c] = {"avg_us": avg * 1e3, "bytes": b, "achieved_gbs": b / (avg * 1e-3) / 1e9}
        if c in (64, 128):
            if not ring_only:
                avg = timed(run_staged)
                res_st[c] = {"avg_us": avg * 1e3, "bytes": b, "achieved_gbs": b / (avg * 1e-3) / 1e9}
            avg = timed(run_ring)
            if int(ring_err.item()) != 0:
                raise RuntimeError("vg_gat_aggregate_fwd_ring: a hand-over wait expired")
            res_ring[c] = {"avg_us": avg * 1e3, "bytes": b, "achieved_gbs": b / (avg * 1e-3) / 1e9}
            avg = timed(run_ring_gnp)
            if int(ring_err.item()) != 0:
                raise RuntimeError("vg_gat_aggregate_fwd_ring_gnp: a hand-over wait expired")
            res_ring_gnp[c] = {"avg_us": avg * 1e3, "bytes": b, "achieved_gbs": b / (avg * 1e-3) / 1e9}
    del scratch
    return {"nodes": n, "edges": e, "per_channels": res, "per_channels_lds": res_lds, "per_channels_staged": res_st,
            "per_channels_ring": res_ring, "per_channels_ring_gnp": res_ring_gnp,
            "order": order, "distinct_sources_per_tile": round(uniq / tiles, 1), "edges_per_tile": round(e / tiles, 1),
            "staged_plan": {"distinct_sources_per_64_row_tile": round(s_uniq, 1),
                            "edges_per_64_row_tile": round(4 * e / tiles, 1), "staged_tiles": staged_tiles,
                            "global_tiles": int((uc < 0).sum().item())}}


def fresh_batch_leg(cfg, precision: str, steps: int, warmup: int, batch: int, device, rank: int, world: int):
    """What ``Trainer.train()`` delivers: every step on a NEW batch from the
    native data path (GraphStore -> C++ collate into pinned buffers -> async
    upload -> CSR adopted, prefetched on a side thread), the per-batch
    type-matched mean / padded columns built, then the step the trainer picks
    for a batch it has not seen (``Trainer._train_batch`` -> ``step_fresh``:
    the critic iteration recorded once per batch and replayed N_CRITIC times,
    the stacked label forward and the generator iteration eager).  Max over
    ranks."""
    import tempfile

    from vgan.loader import GraphLoader
    from vgan.store import write_store
    from vgan.synth import SyntheticDataset

    n_batches = warmup + steps
    tmp = tempfile.mkdtemp(prefix=f"vgan_fresh_{rank}_")
    ds = SyntheticDataset(n_batches * batch * world, seed=4321)
    store = write_store(os.path.join(tmp, "store"), ds)
    lstats = {}
    loader = GraphLoader(store, batch_size=batch, shuffle=True, device=device, prefetch=3, rank=rank,
                         world_size=world, seed=4321, prepare=cfg.NUM_CLASSES, phase_stats=lstats)
    torch.manual_seed(cfg.SEED + rank)
    tr = build_trainer(cfg, precision)
    cfg.runtime["train_step"] = "auto"
    from vgan.gcscope import gc_frozen

    # host seconds per phase of the timed steps: the loader's pipeline
    # (GraphLoader phase_stats) and step_fresh's own phases (Trainer.phase_hook
    # marks: prepare, labels, capture = recording + executable-graph update,
    # replays, gen, release) -- where a slower host shows up on a fresh box
    phases = {}
    clock = [0.0]

    def mark(name):
        now = time.perf_counter()
        phases[name] = phases.get(name, 0.0) + now - clock[0]
        clock[0] = now

    it = iter(loader)
    with gc_frozen():  # as Trainer._train_each_epoch's batch loop
        for _ in range(warmup):
            loc, vox = next(it)
            tr._train_batch(loc, vox)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        lstats.clear()
        tr.phase_hook = mark
        t0 = time.perf_counter()
        for _ in range(steps):
            clock[0] = time.perf_counter()
            loc, vox = next(it)
            mark("next_batch")
            tr._train_batch(loc, vox)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        tr.phase_hook = None
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    del it, loader, store
    import shutil

    shutil.rmtree(tmp, ignore_errors=True)
    per = lambda sec: round(sec / steps * 1e3, 4)  # noqa: E731
    host = {"enqueue_ms_per_step": per(t_host), "drain_ms": round((elapsed - t_host) * 1e3, 3),
            "step_phases_ms_per_step": {k: per(v) for k, v in phases.items()},
            "loader_ms_per_batch": {k: per(v) for k, v in lstats.items() if k != "batches"},
            "how": "host perf_counter per phase over the timed steps: next_batch = the consumer's wait in the "
                   "loader iterator (queue_wait + upload_wait of loader_ms_per_batch), then step_fresh's phases "
                   "(prepare, labels, capture = critic recording + executable-graph update, replays, gen, "
                   "release); loader collate / upload_issue run on its worker thread; enqueue = host time of "
                   "the loop, drain = the device finishing after it"}
    return {"value": round(batch * world * steps / elapsed, 3), "unit": "graphs/s",
            "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "host_phases": host,
            "execution": "Trainer._train_batch per new batch (step_fresh: critic iteration captured once per batch, "
                         "replayed N_CRITIC times; label forward and generator iteration eager), GraphLoader "
                         "prefetch 3: host collate + host-built per-batch structures, one upload per batch"}


def start_sweep_store(graphs: int = 10000, seed: int = 2024):
    """Write the inference sweep's store of ``graphs`` distinct synthetic
    buildings in a child process (no GPU in it), while the GPU legs run.
    Returns (process, path)."""
    import multiprocessing as mp
    import tempfile

    from vgan.synth import write_synthetic_store

    path = os.path.join(tempfile.mkdtemp(prefix="vgan_sweep_"), "store")
    proc = mp.get_context("spawn").Process(target=write_synthetic_store, args=(path, graphs, seed), daemon=True)
    proc.start()
    return proc, path


# collating threads of the sweep's loader (tools/sweep_probe.py: 2 kept the
# loader under the f16 forward's device time; 3 lost to GIL contention)
SWEEP_WORKERS = int(os.environ.get("VGAN_SWEEP_WORKERS", "2"))


def sweep_leg(device, store_job, batch: int = 32, n_taus: int = 10):
    """BASELINE.json configs[4]: generator-only inference sweep over a STREAM
    of distinct buildings (the store written by ``start_sweep_store``: 10,000
    synthetic buildings, 313 batches of 32), a geometric Gumbel temperature
    schedule 1.0 -> 0.1, f16 (and f32) eval forward, one stacked forward per
    batch over the ``n_taus`` temperature copies.  Each batch comes through
    the native loader (host collate + host-built per-batch structures + one
    upload, prefetched on SWEEP_WORKERS threads); f16: the batch's forward
    captured from the native engine into a hipGraph and launched as one
    (vg_hgen_sweep_graphed, one of two executable graphs updated in place),
    f32: launched from Python (InferenceSweep.run_stream).  The timed region is the whole pass: collate, upload, forward.
    Also the f16 scatter kernel (vg_hgat_fwd) over the sweep's own stacked
    graph and channel schedule, graph-replayed between HIP events."""
    from vgan import data as vdata
    from vgan._lib import LIB, check, ptr, stream_handle
    from vgan.config import Configuration
    from vgan.half import _r8
    from vgan.infer import InferenceSweep, geometric_taus
    from vgan.loader import GraphLoader
    from vgan.models import VoxelGNNGenerator
    from vgan.store import GraphStore

    proc, path = store_job
    t0 = time.perf_counter()
    proc.join()
    if proc.exitcode != 0:
        raise RuntimeError(f"sweep store writer exited with {proc.exitcode}")
    log(f"sweep store ready ({time.perf_counter() - t0:.1f} s wait)")
    store = GraphStore(path)
    cfg = Configuration()
    cfg.DEVICE = str(device)
    cfg.runtime["rng"] = "device"
    torch.manual_seed(cfg.SEED)
    G = VoxelGNNGenerator(cfg, 17, 12)
    taus = geometric_taus(1.0, 0.1, n_taus)

    def loader(indices=None):
        return GraphLoader(store, indices, batch_size=batch, shuffle=False, device=device, prefetch=4,
                           prepare=(cfg.NUM_CLASSES, ()), workers=SWEEP_WORKERS)

    n_batches = -(-len(store) // batch)
    out = {"workload": f"configs[4]: {len(store)} distinct synthetic buildings ({n_batches} batches of {batch}) "
                       f"streamed through the native loader, {n_taus} Gumbel temperatures 1.0->0.1 geometric, eval G "
                       f"forward stacked over the temperatures (InferenceSweep.run_stream; f16: the whole batch -- z and noise "
                       f"draws, forward, Gumbel head, argmax -- captured from the native engine into a hipGraph, one graph launch per batch, vg_hgen_sweep_graphed; f32: launched from "
                       f"Python), {SWEEP_WORKERS} collating loader threads; collate, upload, per-batch structures and "
                       f"forward timed",
           "unit": "samples/s (buildings x temperatures)", "distinct_batches": n_batches,
           "distinct_buildings": len(store)}
    for dt in ("f16", "f32"):
        sw = InferenceSweep(G, taus, dtype=dt)
        sw.run_stream(loader(list(range(4 * batch))))  # warm-up: lazy initialisation, first instantiations
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        res = sw.run_stream(loader())
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        out[dt] = {"value": round(res["samples"] / el, 1), "seconds": round(el, 4), "samples": res["samples"],
                   "batches": res["batches"], "ms_per_batch": round(el / res["batches"] * 1e3, 4)}
        log(f"sweep {dt}: {out[dt]['value']:.0f} samples/s ({el:.3f} s for {res['samples']} samples, "
            f"{res['batches']} distinct batches)")
        del sw
    loc, vox = next(iter(loader(list(range(batch)))))
    # the f16 scatter kernel on the sweep's stacked CSR (n_taus copies)
    csr = vdata.prepared(loc, vox, cfg.NUM_CLASSES).csr.stacked(n_taus)
    rows, e = csr.num_nodes, csr.num_edges
    widths = G.encoder.widths[1:]
    gen = torch.Generator(device=device)
    gen.manual_seed(5)
    bufs = {}
    for c in set(widths):
        ld = _r8(c)
        h = (torch.randn(rows, ld, device=device, generator=gen) * 0.5).half()
        bufs[c] = (h, 0.3 * torch.randn(rows, device=device, generator=gen),
                   0.3 * torch.randn(rows, device=device, generator=gen), torch.randn(c, device=device, generator=gen),
                   torch.empty(rows, ld, dtype=torch.float16, device=device), ld)

    def launch_all():
        st = stream_handle(device)
        for c in widths:
            h, a_s, a_d, bias, o, ld = bufs[c]
            check(LIB.vg_hgat_fwd(ptr(csr.row_ptr), ptr(csr.col), rows, c, ld, ptr(h), ptr(a_s), ptr(a_d),
                                  ptr(bias), 0.2, ptr(o), ld, st), "vg_hgat_fwd")

    side = torch.cuda.Stream(device)
    side.wait_stream(torch.cuda.current_stream(device))
    with torch.cuda.stream(side):
        launch_all()
    torch.cuda.current_stream(device).wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        launch_all()
    g.replay()
    torch.cuda.synchronize()
    reps = 20
    st_ev, en_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st_ev.record()
    for _ in range(reps):
        g.replay()
    en_ev.record()
    torch.cuda.synchronize()
    ms = st_ev.elapsed_time(en_ev)
    nbytes = reps * sum(agg_bytes(rows, e, c, elem=2) for c in widths)
    launches = reps * len(widths)
    gbs = nbytes / (ms * 1e-3) / 1e9
    out["roofline"] = {"kernel": "vg_hgat_fwd (f16 rows: edge softmax + CSR gather-sum + bias)", "bound": "hbm",
                       "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": round(gbs / HBM_PEAK_GBS, 4), "avg_launch_us": round(ms * 1e3 / launches, 3),
                       "avg_algorithmic_bytes": int(nbytes / launches), "rows": rows, "edges": e,
                       "launches_per_forward": len(widths)}
    log(f"sweep vg_hgat_fwd: {ms * 1e3 / launches:.2f} us per launch, {gbs:.0f} GB/s")
    return out


def cpu_baseline(cfg_batch: int, seconds_budget: float):
    """Time the CPU oracle (reference step restatement) on a batch-32 step."""
    from oracle import pyg
    from oracle import reference as R
    from vgan.config import Configuration
    from vgan.synth import SyntheticDataset

    affinity = len(os.sched_getaffinity(0))
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(affinity, cap) if cap > 0 else affinity
    torch.set_num_threads(threads)
    cpu_model = None
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), None)
    except OSError:
        pass
    cfg = Configuration()
    ds = SyntheticDataset(6500, seed=777)
    items = [ds[i] for i in range(cfg_batch)]
    keys_v = ("x", "edge_index", "type", "types_onehot", "site_area", "data_number")
    keys_l = ("x", "type", "data_number")
    local = pyg.Batch.from_data_list([pyg.Data(**{k: getattr(l, k) for k in keys_l}) for l, _ in items])
    voxel = pyg.Batch.from_data_list([pyg.Data(**{k: getattr(v, k) for k in keys_v}) for _, v in items])
    torch.manual_seed(777)
    G, D = R.Generator(cfg), R.Discriminator(cfg)
    og = torch.optim.Adam(G.parameters(), lr=cfg.LEARNING_RATE_GENERATOR, betas=cfg.BETAS)
    od = torch.optim.Adam(D.parameters(), lr=cfg.LEARNING_RATE_DISCRIMINATOR, betas=cfg.BETAS)
    t0 = time.perf_counter()
    R.train_step(G, D, og, od, cfg, local, voxel)  # warm-up: allocator, thread pool
    log(f"cpu baseline warm-up step: {time.perf_counter() - t0:.2f} s")
    times = []
    while True:  # at least 3 timed steps, more while the budget lasts (at most 7)
        t0 = time.perf_counter()
        R.train_step(G, D, og, od, cfg, local, voxel)
        times.append(time.perf_counter() - t0)
        log(f"cpu baseline step {len(times)}: {times[-1]:.2f} s")
        if len(times) >= 3 and (sum(times) >= seconds_budget or len(times) >= 7):
            break
    med = sorted(times)[len(times) // 2]
    return {
        "value": round(cfg_batch / med, 3),
        "unit": "graphs/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "cpu_model": cpu_model,
        "affinity_cpus": affinity,
        "threads_note": (f"torch threads = min(sched_getaffinity {affinity}, OMP_NUM_THREADS {cap}): the pool sets "
                         f"OMP_NUM_THREADS to the per-GPU CPU share of the box" if cap > 0 and cap < affinity else
                         "torch threads = every CPU of sched_getaffinity"),
        "statistic": f"median of {len(times)} timed steps after 1 warm-up step",
        "step_seconds": [round(t, 3) for t in times],
        "sample": f"full G+D steps of batch {cfg_batch} synthetic buildings "
                  f"({voxel.num_nodes} voxel nodes) through the CPU oracle (oracle/reference.py, "
                  f"pinned bit-for-bit to the reference's own trainer.py step), fp32, "
                  f"{med:.2f} s/step (median)",
    }


def _free_port() -> int:
    import socket

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def self_launch(n: int) -> int:
    """``--gpus N`` with no torch.distributed environment: run the N ranks as
    ``python -m torch.distributed.run --nproc-per-node N ... bench.py <same
    arguments>`` in a child process (this process never touches the GPU and
    never execs); the ranks inherit stdout, so rank 0's JSON line is this
    command's output.  Returns the launcher's exit status."""
    import subprocess

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    log(f"--gpus {n}: launching {n} ranks ({' '.join(cmd[1:6])} ...)")
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", os.environ.get("OMP_NUM_THREADS", "8"))
    return subprocess.call(cmd, env=env)


def rehearse(args, rank: int, world: int) -> None:
    """``--rehearse``: the N-rank plumbing without a GPU (CPU container,
    VGAN_DIST_BACKEND=gloo) -- self-launch, process group, barriers around the
    timed region, max over ranks, one line from rank 0.  The "step" is a fixed
    CPU matmul, so the line carries no throughput (value null)."""
    if world > 1:
        dist.init_process_group(os.environ.get("VGAN_DIST_BACKEND", "gloo"), rank=rank, world_size=world)
    a = torch.randn(256, 256)
    for _ in range(args.warmup):
        a = torch.tanh(a @ a)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = torch.tanh(a @ a)
    if world > 1:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    ws = dist.get_world_size() if world > 1 else 1
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "graphs/s", "n_gpus": world, "world_size": ws,
                          "steps": args.steps, "warmup": args.warmup, "rehearsal": True,
                          "elapsed_s_max_over_ranks": round(float(el), 6)}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--pool", type=int, default=4, help="pre-staged batches per rank")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-stress", action="store_true")
    ap.add_argument("--eager", action="store_true", help="no hipGraph capture of the step")
    ap.add_argument("--precision", choices=("f32", "bf16"), default="f32",
                    help="dense-product precision of the main measurement (f32 = configs[1]); the default run adds "
                         "a bf16 line (configs[2]) after it")
    ap.add_argument("--no-bf16", action="store_true", help="skip the extra bf16 (configs[2]) measurement")
    ap.add_argument("--profile", action="store_true",
                    help="for rocprofv3: only warm-up + timed steps (50 ms idle gap before the timed region), "
                         "no instrumented / stress / CPU passes")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the scatter-kernel roofline replays (--steps of them), for rocprofv3 --pmc passes")
    ap.add_argument("--gnp", action="store_true",
                    help="with --roofline-only: the variant the step runs (vg_gat_aggregate_fwd_gnp)")
    ap.add_argument("--stress-only", action="store_true",
                    help="only the configs[3] ring aggregations (blocked numbering, C=128, cold MALL), for "
                         "tools/stress_trace.sh")
    ap.add_argument("--no-fresh", action="store_true", help="skip the fresh-batch (Trainer.train path) leg")
    ap.add_argument("--no-sweep", action="store_true", help="skip the configs[4] inference-sweep leg")
    ap.add_argument("--rehearse", action="store_true",
                    help="the N-rank launch / barrier / max-over-ranks plumbing on the CPU (no GPU, no throughput)")
    args = ap.parse_args()
    global GRAPHED
    GRAPHED = not args.eager

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(self_launch(args.gpus))  # before anything touches the GPU
    rank, world, local = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), int(
        os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.rehearse:
        rehearse(args, rank, world)
        return
    want_sweep = rank == 0 and not args.no_sweep and not args.profile and not args.roofline_only
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    # VGAN_DIST_BACKEND=gloo rehearses the N>1 path (barriers, rank sharding,
    # eager all-reduce + Adam between replays, max-over-ranks timing) with
    # several ranks sharing the GPUs of a smaller box; RCCL ("nccl") is the
    # product backend and refuses two ranks on one GPU.
    backend = os.environ.get("VGAN_DIST_BACKEND", "nccl")
    n_dev = torch.cuda.device_count()
    if local >= n_dev and backend == "nccl":
        raise SystemExit(f"LOCAL_RANK {local} but only {n_dev} GPU(s) visible")
    local_dev = local % n_dev
    torch.cuda.set_device(local_dev)
    device = torch.device("cuda", local_dev)
    bound = None
    if os.environ.get("VGAN_NUMA_BIND", "1") == "1":  # host threads on the GPU's NUMA node (vgan/affinity.py)
        from vgan.affinity import bind_to_device_numa

        bound = bind_to_device_numa(device)
        log(f"host threads bound to the GPU's NUMA node: {len(bound)} CPUs" if bound else
            "host threads not bound (NUMA topology unknown)")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)

    from vgan.config import Configuration

    cfg = Configuration()
    cfg.DEVICE = str(device)
    cfg.runtime["rng"] = "device"
    cfg.runtime["rank"], cfg.runtime["world_size"] = rank, world  # per-rank device RNG streams
    torch.manual_seed(cfg.SEED + rank)
    torch.cuda.manual_seed(cfg.SEED + rank)
    if args.stress_only:  # for rocprofv3: the ring launches of roofline_stress only
        r = stress_roofline(device, channels=(128,), order="blocked", ring_only=True)
        print(json.dumps({"stress_only": True, "ring": r["per_channels_ring"], "ring_gnp": r["per_channels_ring_gnp"]},
                         default=float), flush=True)
        return
    log(f"rank {rank}/{world}: staging {args.pool} batches of {args.batch} buildings")
    pool = make_pool(cfg, rank, world, args.pool, args.batch, device)
    tr = build_trainer(cfg, args.precision)
    n_nodes = sum(v.num_nodes for _, v in pool) / len(pool)
    if args.roofline_only:  # for rocprofv3 --pmc passes: only the scatter-kernel roofline replays
        from vgan import data as vdata

        csr0 = vdata.prepared(pool[0][0], pool[0][1], cfg.NUM_CLASSES).csr
        kern = aggregate_roofline(tr, csr0, device, reps=args.steps, gnp=args.gnp)
        print(json.dumps({"roofline_only": True, **{k: round(v, 3) for k, v in kern.items()}}), flush=True)
        return

    # warm-up (also builds every batch's CSR / type-mean once, as the first step of a batch would)
    per_step = []
    elapsed = timed_steps(tr, pool, args.steps, args.warmup, world, device, profile=args.profile,
                          per_step=None if args.profile else per_step)
    mean_ms = elapsed / args.steps * 1e3
    # SURVEY.md 8(d)'s statistic: the MEDIAN step of the K timed steps (HIP
    # events between the steps on the replay stream, no host sync inside the
    # timed region), max over ranks; the wall-clock mean of the same region
    # beside it
    ms_per_step = mean_ms
    if per_step:
        ms_per_step = sorted(per_step)[len(per_step) // 2]
        if world > 1:
            t = torch.tensor([ms_per_step], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            ms_per_step = float(t.item())
    value = args.batch * world / (ms_per_step * 1e-3)
    log(f"timed ({'hipGraph' if GRAPHED else 'eager'}, {args.precision}): median {ms_per_step:.3f} ms/step "
        f"({value:.1f} graphs/s), mean {mean_ms:.3f} ms/step over {args.steps} steps")
    median = None
    if per_step:
        median = {"ms_per_step": round(ms_per_step, 4), "value": round(value, 3), "steps": args.steps,
                  "mean_ms_per_step": round(mean_ms, 4),
                  "mean_value": round(args.batch * world * args.steps / elapsed, 3),
                  "p10_p90_ms": [round(sorted(per_step)[len(per_step) // 10], 4),
                                 round(sorted(per_step)[(9 * len(per_step)) // 10], 4)],
                  "how": f"value / ms_per_step: the median of the {args.steps} timed steps' HIP-event durations "
                         f"(events between steps on the replay stream, no host sync inside), max over ranks; "
                         f"mean_*: wall clock of the same timed region (barrier + synchronize on both sides) / "
                         f"{args.steps}"}

    if args.profile:
        if rank == 0:
            print(json.dumps({"profile": True, "precision": args.precision, "value": round(value, 3),
                              "ms_per_step": round(ms_per_step, 3), "steps": args.steps}), flush=True)
        if world > 1:
            dist.destroy_process_group()
        return

    # configs[2]: the same step with bf16 dense products (fresh models, same seed)
    bf16 = None
    if args.precision == "f32" and not args.no_bf16:
        del tr
        torch.manual_seed(cfg.SEED + rank)
        tr16 = build_trainer(cfg, "bf16")
        el16 = timed_steps(tr16, pool, args.steps, args.warmup, world, device)
        bf16 = {"value": round(args.batch * world * args.steps / el16, 3), "unit": "graphs/s",
                "ms_per_step": round(el16 / args.steps * 1e3, 3), "dtype": "bf16 operands, f32 accumulate",
                "workload": f"configs[2]: the configs[1] step with every dense product (nn.Linear / GATConv.lin: "
                            f"forward, input and weight gradients) on bf16 operands, f32 accumulation; "
                            f"aggregation, GraphNorm, losses, Adam f32; dp{world}"}
        log(f"timed bf16: {bf16['ms_per_step']:.2f} ms/step, {bf16['value']:.1f} graphs/s")
        tr = tr16
        cfg.runtime["precision"] = "f32"

    # the dominant message-passing kernel's roofline: the step's own mix of
    # vg_gat_aggregate_fwd launches, graph-replayed between HIP events
    from vgan import data as vdata

    csr0 = vdata.prepared(pool[0][0], pool[0][1], cfg.NUM_CLASSES).csr
    kern = aggregate_roofline(tr, csr0, device, reps=max(args.steps, 10))
    log(f"vg_gat_aggregate_fwd: {kern['launches']} launches, avg {kern['avg_us']:.2f} us, "
        f"{kern['achieved_gbs']:.1f} GB/s")
    kern_gnp = aggregate_roofline(tr, csr0, device, reps=max(args.steps, 10), gnp=True)
    if kern_gnp:
        log(f"vg_gat_aggregate_fwd_gnp: avg {kern_gnp['avg_us']:.2f} us, {kern_gnp['achieved_gbs']:.1f} GB/s "
            f"(HBM bytes), {kern_gnp['gather_gbs']:.0f} GB/s L2 gather")
    head = kern_gnp or kern
    traffic, traffic_src = load_pmc_traffic()
    gemms = gemm_family_roofline(tr, csr0.num_nodes, device, reps=max(args.steps, 10)) \
        if args.precision == "f32" and tr.critic is not None else None
    if gemms:
        log(f"k_gemm16 family: {gemms['launches_per_step']} launches, avg {gemms['avg_launch_us']:.2f} us, "
            f"{gemms['achieved_tflops']:.2f} TFLOP/s, {gemms['achieved_gbs']:.0f} GB/s")
    # what Trainer.train() delivers: a new batch from the native loader every step
    fresh = None
    if os.environ.get("VGAN_BENCH_RELEASE", "1") == "1":
        # the replayed legs' trainers, batches and recorded graphs are done
        # with (the fresh leg also runs its loop under vgan.gcscope.gc_frozen,
        # as Trainer.train does: beside them, unfrozen, it took 10.6-11.4 ms)
        del tr, pool, csr0
        import gc

        gc.collect()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    if not args.no_fresh:
        # its own step counts: at ~8.5 ms a step, 20 steps after 5 warm-up
        # ones spread 8.1-10.1 ms between runs on one box (host-bound leg;
        # profiles/r04_fresh_ab.txt); 60 after 10 cost half a second
        fresh = fresh_batch_leg(cfg, args.precision, max(args.steps, 60), max(args.warmup, 10), args.batch, device,
                                rank, world)
        log(f"fresh batches (loader, step_fresh): {fresh['ms_per_step']:.2f} ms/step, {fresh['value']:.1f} graphs/s")

    # configs[4]'s 10,000 distinct buildings are generated in a child process
    # while the stress legs run -- after the host-bound fresh leg, which the
    # writer slowed by ~0.2 ms per step when it ran beside it
    store_job = start_sweep_store() if want_sweep else None
    result = None
    if rank == 0:
        stress_orders = {} if args.no_stress else {o: stress_roofline(device, order=o)
                                                   for o in ("rowmajor", "tiled", "blocked")}
        stress_model = None if args.no_stress else stress_model_leg(device)
        for o, st_ in stress_orders.items():
            for kind, key in (("register", "per_channels"), ("LDS 16-row", "per_channels_lds"),
                              ("staged", "per_channels_staged"), ("ring", "per_channels_ring")):
                for c, r in st_[key].items():
                    log(f"stress ({o}) C={c} ({kind}): {r['avg_us']:.1f} us, {r['achieved_gbs']:.0f} GB/s")
        sweep = None if store_job is None else sweep_leg(device, store_job)
        # the headline fraction priced on the committed rocprofv3 mean of the
        # same replays (tools/roofline_trace.sh --gnp), the live HIP-event
        # figure beside it
        trace = load_trace_mean(ROOFLINE_TRACE)
        roof_us = trace["avg_us"] if trace else head["avg_us"]
        roof_gbs = head["avg_bytes"] / (roof_us * 1e-6) / 1e9
        roof_src = (f"rocprofv3 kernel trace, {trace['source']}: mean of {trace['launches']} launches of the same "
                    f"replays (bench.py --roofline-only --gnp)") if trace else "HIP events of this run (no trace)"
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(args.batch, args.cpu_seconds)
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "graphs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "median": median,
            "world_size": dist.get_world_size() if world > 1 else 1,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.precision,
            "data": "synthetic (seeded 6-type buildings in the reference tensor layout; random-init weights)",
            "config": {
                "workload": ("configs[1]: 6-type dataset, batch=32 voxel graphs per GPU, fp32, full G+D step "
                             "(5 critic WGAN-GP + 1 generator iteration, Adam), HIP message passing")
                if args.precision == "f32" else
                ("configs[2]: 6-type dataset, batch=32 voxel graphs per GPU, bf16 dense products (f32 accumulate), "
                 "full G+D step (5 critic WGAN-GP + 1 generator iteration, Adam), HIP message passing"),
                "global_batch": args.batch * world,
                "avg_voxel_nodes_per_batch": round(n_nodes, 1),
                "parallelism": f"dp{world}",
                "execution": ("hipGraph replay: one stacked no-grad G forward for the N_CRITIC critic labels, "
                              "N_CRITIC critic-engine graphs, one generator-iteration graph") if GRAPHED else "eager",
            },
            "host": {"numa_bound_cpus": len(bound) if bound else None,
                     "note": "host threads on the GPU's NUMA node (vgan.affinity; VGAN_NUMA_BIND=0: unbound)"},
            "roofline": {
                "kernel": "vg_gat_aggregate_fwd_gnp (the scatter kernel as the step runs it: GAT edge softmax + "
                          "CSR gather-sum + bias, with the following GraphNorm's column partials in the epilogue)",
                "bound": "hbm",
                "achieved": round(roof_gbs, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(roof_gbs / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "avg_launch_us": round(roof_us, 3),
                "duration_source": roof_src,
                "live_hip_events": {"avg_launch_us": round(head["avg_us"], 3),
                                    "achieved": round(head["achieved_gbs"], 2),
                                    "frac": round(head["achieved_gbs"] / HBM_PEAK_GBS, 5),
                                    "note": "the same replays timed in this run with HIP events on the replay "
                                            "stream; frac above is priced on the committed rocprofv3 mean"},
                "avg_algorithmic_bytes": int(head["avg_bytes"]),
                "algorithmic_bytes": "SURVEY.md 8(d) compulsory: 2*N*C*4 (h in, out) + 2*N*4 (a_src, a_dst) + "
                                     "E'*4 (col) + (N+1)*4 (row_ptr); alpha and the GraphNorm partials written "
                                     "besides are not counted",
                "avg_extra_written_bytes": int(head["avg_extra_written_bytes"]),
                "launches_timed": head["launches"],
                "launches_per_step": head["launches_per_step"],
                "timing": "the step's own mix of launches (CSRs, channel counts), hipGraph-replayed between HIP "
                          "events on the replay stream",
                "l2_gather": {
                    "what": "the same launches against the L2: every edge's source row, col and a_src entry, "
                            "the output row (agg_gather_bytes); the HBM bytes above count each source row once",
                    "achieved": round(head["gather_gbs"], 1), "unit": "GB/s",
                    "frac_of_l2_peak": round(head["gather_gbs"] / L2_PEAK_GBS, 4), "l2_peak": L2_PEAK_GBS,
                    "frac_of_measured_gather_ceiling": round(head["gather_gbs"] / L2_GATHER_GBS, 4),
                    "measured_gather_ceiling": L2_GATHER_GBS,
                    "avg_gather_bytes": int(head["avg_gather_bytes"]),
                },
                "plain_kernel": {
                    "kernel": "vg_gat_aggregate_fwd (no GraphNorm partials; the eager / inference forward)",
                    "achieved": round(kern["achieved_gbs"], 2),
                    "frac": round(kern["achieved_gbs"] / HBM_PEAK_GBS, 5),
                    "avg_launch_us": round(kern["avg_us"], 3),
                    "avg_algorithmic_bytes": int(kern["avg_bytes"]),
                },
            },
            "cpu_baseline": cpu,
        }
        if gemms:
            result["gemm_family"] = gemms
        if fresh:
            result["fresh_batch_ms_per_step"] = fresh["ms_per_step"]
            result["fresh_batch"] = fresh
        if bf16:
            result["bf16"] = bf16
        if sweep:
            result["inference_sweep"] = sweep
        if stress_orders:
            # configs[3]: the fastest (numbering, kernel) at C = 128 -- the
            # register gather (k_gat_fwd_cp), the 16-row LDS tiles (k_gat_fwd_lds)
            # or the persistent staged kernel (k_gat_fwd_staged); all are
            # reported, DESIGN.md 4.10 / 4.20 explain the pick
            kinds = {"per_channels": "vg_gat_aggregate_fwd (register gather: 16-lane rows, 4 source rows in flight "
                                     "per lane group)",
                     "per_channels_lds": "vg_gat_aggregate_fwd_lds (each 16-row tile's distinct source rows staged "
                                         "through LDS)",
                     "per_channels_staged": "vg_gat_aggregate_fwd_staged (persistent 1024-thread workgroup per CU; "
                                            "each 64-row tile's distinct source rows staged through LDS while the "
                                            "previous tile is aggregated)",
                     "per_channels_ring": "vg_gat_aggregate_fwd_ring (wave-specialised workgroup per CU: 4 loader "
                                          "waves fill a two-slot LDS ring with each 64-row tile's distinct source "
                                          "rows by LDS-DMA, index loads two stages ahead; 12 consumer waves claim "
                                          "(tile, 4-row group) units and aggregate out of LDS; LDS-counter "
                                          "hand-over, no barrier)"}
            kinds["per_channels_ring_gnp"] = ("vg_gat_aggregate_fwd_ring_gnp (the ring as the drop-in dispatches it: "
                                              "with the following GraphNorm's column partials per 64-row tile)")
            cands = [(r[key][128]["avg_us"], o, key) for o, r in stress_orders.items() for key in kinds
                     if 128 in r.get(key, {})]
            _, o_best, k_best = min(cands)
            best = stress_orders[o_best]
            c128 = best[k_best][128]
            names = {"rowmajor": "row-major (the reference's numbering)",
                     "tiled": "4 x 4 (y, x) tiles per floor, vgan.locality.tile_order",
                     "blocked": "4 x 4 x 4 lattice blocks, vgan.locality.block_order"}
            gb = agg_gather_bytes(best["nodes"], best["edges"], 128)
            # priced on the committed rocprofv3 trace of the ring's cold-MALL
            # launches (tools/stress_trace.sh) when the fastest pair is the ring
            st_trace = load_trace_mean(STRESS_TRACE) if k_best == "per_channels_ring" else None
            st_us = st_trace["avg_us"] if st_trace else c128["avg_us"]
            st_gbs = c128["bytes"] / (st_us * 1e-6) / 1e9
            st_src = (f"rocprofv3 kernel trace, {st_trace['source']}: mean of {st_trace['launches']} cold-MALL "
                      f"launches (bench.py --stress-only)") if st_trace else "HIP events of this run"
            result["roofline_stress"] = {
                "workload": f"configs[3]: 8 x 50k-node buildings, N={best['nodes']}, E'={best['edges']}, "
                            f"C=128 fp32, cold MALL, voxels numbered {names[o_best]}",
                "kernel": kinds[k_best],
                "tile_plan": (f"{best['staged_plan']['distinct_sources_per_64_row_tile']} distinct source rows for "
                              f"{best['staged_plan']['edges_per_64_row_tile']} edges per 64-row tile"
                              if k_best in ("per_channels_staged", "per_channels_ring") else
                              f"{best['distinct_sources_per_tile']} distinct source rows for "
                              f"{best['edges_per_tile']} edges per 16-row tile"),
                "bound": "hbm", "achieved": round(st_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(st_gbs / HBM_PEAK_GBS, 4), "avg_launch_us": round(st_us, 2),
                "duration_source": st_src,
                "live_hip_events": {"avg_launch_us": round(c128["avg_us"], 2),
                                    "achieved": round(c128["achieved_gbs"], 1),
                                    "frac": round(c128["achieved_gbs"] / HBM_PEAK_GBS, 4),
                                    "kernel_key": k_best},
                "model_forward": stress_model,
                "algorithmic_bytes": int(c128["bytes"]),
                "edge_gather_bytes": int(gb),
                "by_order": {o: {"distinct_sources_per_16_row_tile": r["distinct_sources_per_tile"],
                                 "staged_plan": r["staged_plan"],
                                 **{key: {str(c): {k: round(v, 2) for k, v in x.items()} for c, x in r[key].items()}
                                    for key in kinds}}
                             for o, r in stress_orders.items()},
            }
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
