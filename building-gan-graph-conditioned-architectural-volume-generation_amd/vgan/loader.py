"""Mini-batch loaders over a ``GraphStore``: the reference's ``GraphDataLoaders``.

``GraphDataLoaders`` (``data.py:166-212``) splits the dataset with
``random_split(dataset, SPLIT_RATIOS)`` and wraps each part in a
``DataLoader(batch_size=BATCH_SIZE, shuffle=True, drop_last=False,
collate_fn=GraphDataset.collate_fn, num_workers=NUM_WORKERS)``.  Here:

* the split and the per-epoch shuffle use the same torch machinery
  (``random_split`` over the store's indices, a ``DataLoader`` over those
  indices for the sampling), so they consume the global CPU RNG exactly as the
  reference does and produce the same building order for the same seed;
* each epoch's index batches are drawn up front on the calling thread; a
  background thread then collates them natively (``GraphStore.collate``, the
  GIL is released inside the C++ collate) into page-locked buffers and issues
  their host-to-device copies on a side stream, ``prefetch`` batches ahead;
* the consumer's stream waits on the copy's event, so a yielded
  ``(local, voxel)`` pair is already device-resident -- the trainer's
  ``.to(DEVICE)`` (``trainer.py:459-460``) is a no-op -- and carries the
  host-built CSR/CSC that ``vgan.data`` adopts without a device build.
"""
from __future__ import annotations

import os
import queue
import sys
import threading
import time
from typing import Iterator, List, Optional, Sequence, Tuple

import torch
from torch.utils.data import DataLoader, random_split

from .graph import GraphBatch
from .store import GraphStore, upload_pair

# GIL switch interval while a prefetch thread runs (seconds; _prefetched)
_SWITCH_INTERVAL = float(os.environ.get("VGAN_LOADER_SWITCH_INTERVAL", "1e-4"))


class _Indices(torch.utils.data.Dataset):
    def __init__(self, indices: Sequence[int]):
        self.indices = list(indices)

    def __len__(self) -> int:
        return len(self.indices)

    def __getitem__(self, i: int) -> int:
        return self.indices[i]


def _as_list(batch) -> List[int]:
    return [int(v) for v in batch]


class GraphLoader:
    """Iterable of ``(local, voxel)`` GraphBatch pairs over ``indices`` of a store."""

    def __init__(self, store: GraphStore, indices: Optional[Sequence[int]] = None, batch_size: int = 1,
                 shuffle: bool = True, drop_last: bool = False, device=None, prefetch: int = 2,
                 threads: int = 4, rank: int = 0, world_size: int = 1, seed: Optional[int] = None,
                 even: bool = True, resident: bool = False, prepare=None, workers: int = 1,
                 phase_stats: Optional[dict] = None):
        """``rank`` / ``world_size``: data-parallel sharding -- every rank draws
        the same epoch plan and takes batches rank, rank + world, ... of it, so
        ranks see disjoint buildings (weak scaling, one batch of
        ``batch_size`` per rank and step).

        With ``world_size > 1`` the shuffle draws from its own generator seeded
        with ``seed + epoch`` -- not the global CPU RNG, which ranks seed
        differently (``SEED + rank``) -- and, for a training loader
        (``even``), the plan is cut to a multiple of ``world_size`` batches
        (every rank runs the same number of steps, so the per-step gradient
        all-reduces pair up).  An evaluation loader (``even=False``) keeps
        every batch: its ranks may get one batch more or less, and the
        trainer reduces the figures over the ranks once per epoch.  One rank
        keeps the reference's global-RNG shuffle (``data.py:177-184``).

        ``prepare`` (the number of classes, or (classes, stacked copy counts)
        -- vgan.store._prepare_spec): every batch also carries the
        per-batch structures vgan.data would build on the device (padded
        columns, the critic's stacked graph, the type-matched mean, the float
        one-hot, the critic's seeds), built by the host collate and uploaded
        with the batch in its one host-to-device copy.

        ``phase_stats`` (a dict): host seconds accumulated per phase of the
        prefetching pipeline -- ``collate`` and ``upload_issue`` on the worker
        threads, ``queue_wait`` (the consumer waiting for a collated batch) and
        ``upload_wait`` (for its copy) on the consumer's -- plus ``batches``.

        ``resident``: the first epoch's batches stay on the device and every
        later epoch yields the same batch objects in the same order (no
        reshuffle) -- an evaluation set kept in HBM, whose per-batch graphs
        the trainer captures once and replays.

        ``workers``: collating threads (batch i on worker i % workers, yielded
        in plan order).  The C++ collate releases the GIL, so two or three
        workers overlap it; the training step keeps one (its ctypes launches
        are host-bound and every extra Python thread competes for the GIL), a
        sweep whose forward is one native call takes more."""
        if not 0 <= rank < world_size:
            raise ValueError("need 0 <= rank < world_size")
        if world_size > 1 and seed is None:
            raise ValueError("data-parallel sharding needs a seed shared by all ranks")
        self.rank, self.world_size = int(rank), int(world_size)
        self.seed = None if seed is None else int(seed)
        self.epoch = 0
        self.store = store
        self.indices = list(range(len(store))) if indices is None else [int(i) for i in indices]
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.device = torch.device(device) if device is not None else None
        self.prefetch = max(1, int(prefetch))
        self.threads = threads
        self.even = bool(even)
        self.resident = bool(resident)
        self._resident_batches: Optional[List[Tuple[GraphBatch, GraphBatch]]] = None
        self.prepare = prepare
        self.workers = max(1, int(workers))
        self.phase_stats = phase_stats

    def __len__(self) -> int:
        n = len(self.indices)
        total = n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size
        if self.even:
            return total // self.world_size
        return len(range(self.rank, total, self.world_size))

    def batches(self, epoch: Optional[int] = None) -> List[List[int]]:
        """This rank's building indices per batch for ``epoch`` (default: the
        loader's epoch counter).  One rank: consumes the CPU RNG like the
        reference's DataLoader (a base seed when the iterator is created, then
        the RandomSampler's seed).  Several ranks: a generator seeded with
        ``seed + epoch``, identical on every rank."""
        gen = None
        if self.seed is not None:
            gen = torch.Generator().manual_seed(self.seed + (self.epoch if epoch is None else int(epoch)))
        dl = DataLoader(_Indices(self.indices), batch_size=self.batch_size, shuffle=self.shuffle,
                        drop_last=self.drop_last, collate_fn=_as_list, num_workers=0, generator=gen)
        plan = list(iter(dl))
        if self.even:
            plan = plan[:len(plan) - len(plan) % self.world_size]
        return plan[self.rank::self.world_size]

    def set_epoch(self, epoch: int) -> None:
        self.epoch = int(epoch)

    def __iter__(self) -> Iterator[Tuple[GraphBatch, GraphBatch]]:
        if self._resident_batches is not None:
            yield from self._resident_batches
            return
        plan = self.batches()
        self.epoch += 1
        dev = self.device
        kept = [] if self.resident else None
        if dev is None or dev.type != "cuda":
            it = (self.store.collate(idx, pin=False, threads=self.threads, prepare=self.prepare) for idx in plan)
        else:
            it = _prefetched(self.store, plan, dev, self.prefetch, self.threads, self.prepare, self.workers,
                             self.phase_stats)
        for pair in it:
            if kept is not None:
                kept.append(pair)
            yield pair
        if kept is not None:
            self._resident_batches = kept


# Prefetchers running at once and the switch interval before the first of
# them: overlapping iterators (a validation loader started while a training
# iterator is suspended) finish in any order, and the interval goes back only
# when the last one ends (reference-counted like vgan.gcscope).
_SWITCH_LOCK = threading.Lock()
_SWITCH_STATE = {"active": 0, "saved": None}


def _switch_enter() -> None:
    with _SWITCH_LOCK:
        if _SWITCH_STATE["active"] == 0:
            _SWITCH_STATE["saved"] = sys.getswitchinterval()
            sys.setswitchinterval(min(_SWITCH_STATE["saved"], _SWITCH_INTERVAL))
        _SWITCH_STATE["active"] += 1


def _switch_exit() -> None:
    with _SWITCH_LOCK:
        _SWITCH_STATE["active"] -= 1
        if _SWITCH_STATE["active"] == 0:
            sys.setswitchinterval(_SWITCH_STATE["saved"])
            _SWITCH_STATE["saved"] = None


def _prefetched(store: GraphStore, plan: List[List[int]], dev: torch.device, depth: int, threads: int,
                prepare=None, workers: int = 1, stats: Optional[dict] = None):
    copy_stream = torch.cuda.Stream(device=dev)
    clock = time.perf_counter
    if stats is not None:
        for k in ("collate", "upload_issue", "queue_wait", "upload_wait", "batches"):
            stats.setdefault(k, 0.0)
        stats_lock = threading.Lock()

    def add(key: str, t0: float) -> float:  # seconds since t0 into stats[key]; returns now
        t1 = clock()
        with stats_lock:  # the caller may clear the dict between steps
            stats[key] = stats.get(key, 0.0) + t1 - t0
        return t1
    nw = max(1, min(int(workers), len(plan) or 1))
    # worker w collates batches w, w + nw, ...; its own queue keeps them in plan order
    qs: List["queue.Queue"] = [queue.Queue(maxsize=max(1, -(-depth // nw))) for _ in range(nw)]
    stop = threading.Event()
    _END = object()

    def worker(w: int):
        q = qs[w]
        try:
            for idx in plan[w::nw]:
                if stop.is_set():
                    return
                t0 = clock() if stats is not None else 0.0
                host = store.collate(idx, pin=True, threads=threads, prepare=prepare)
                if stats is not None:
                    t0 = add("collate", t0)
                with torch.cuda.stream(copy_stream):
                    moved = upload_pair(*host, dev, non_blocking=True)  # one copy of the pair's buffer
                    ev = torch.cuda.Event()
                    ev.record(copy_stream)
                if stats is not None:
                    add("upload_issue", t0)
                q.put((moved, host, ev))  # host buffers stay referenced until the copy is waited on
            q.put(_END)
        except BaseException as exc:  # surfaced on the consumer thread
            q.put(exc)

    ths = [threading.Thread(target=worker, args=(w,), name=f"vgan-loader-{w}", daemon=True) for w in range(nw)]
    # While the worker runs, the interpreter hands the GIL over every 0.1 ms
    # instead of every 5 ms: the consumer (the training step) is host-bound on
    # ctypes launches, each of which releases the GIL, and on return it
    # otherwise waits out whatever Python the worker is running (tensor views,
    # the batch objects) -- 10.1-10.7 vs 8.5 ms per fresh-batch step
    # (tools/fresh_probe.py, profiles/r04_fresh_probe.jsonl).  Restored when
    # the last running prefetcher ends.
    _switch_enter()
    for th in ths:
        th.start()
    try:
        for i in range(len(plan) + 1):
            t0 = clock() if stats is not None else 0.0
            item = qs[i % nw].get()
            if stats is not None:
                t0 = add("queue_wait", t0)
            if item is _END:
                return
            if isinstance(item, BaseException):
                raise item
            moved, host, ev = item
            # The host waits for the upload -- issued `depth` batches earlier,
            # long finished -- instead of the consumer's stream waiting on the
            # copy stream's event: a cross-queue barrier on the device per
            # batch, which took the fresh-batch step to 7.72-8.36 ms against
            # 7.69-7.71 (profiles/r04_loader_wait_ab.txt)
            ev.synchronize()
            if stats is not None:
                add("upload_wait", t0)
                stats["batches"] = stats.get("batches", 0.0) + 1
            for g in moved:  # the consumer stream now owns these allocations
                for t in _tensors(g):
                    t.record_stream(torch.cuda.current_stream(dev))
            del host
            yield moved
    finally:
        _switch_exit()
        stop.set()
        for q, th in zip(qs, ths):
            while th.is_alive():
                try:
                    q.get(timeout=0.1)
                except queue.Empty:
                    pass
            th.join()


def _tensors(g: GraphBatch):
    blob = g.derived("device_blob")
    if blob is not None:  # every tensor of the pair is a view of it
        yield blob
        return
    for key in g.keys():
        v = getattr(g, key)
        if torch.is_tensor(v):
            yield v
    arrays = g.derived("csr_arrays")
    if arrays is not None:
        yield from arrays


class GraphDataLoaders:
    """``train_dataloader`` / ``validation_dataloader`` / ``test_dataloader`` of
    the reference (``data.py:166-212``) over a GraphStore."""

    def __init__(self, configuration, store: GraphStore, device=None, prefetch: int = 2, rank: int = 0,
                 world_size: int = 1, resident_eval: bool = False, prepare: bool = True):
        """``resident_eval``: the validation / test batches are collated once
        and kept on the device (no per-epoch reshuffle), so the trainer replays
        their captured evaluation graphs; the reference reshuffles them every
        epoch (``data.py:186-210``), the default here too."""
        self.configuration = configuration
        self.sanity_checking = bool(getattr(configuration, "SANITY_CHECKING", False))
        self.dataset = store
        indices = list(range(len(store)))[: int(getattr(configuration, "DATA_SLICER", len(store)))]  # data.py:97-98
        if self.sanity_checking:  # data.py:100-102: one building, no validation / test loaders
            indices = [indices[int(getattr(configuration, "DATA_POINT", 0))]]
        # one rank: the reference's split on the global CPU RNG; several ranks:
        # the same split on every rank from a generator seeded with SEED
        seed = int(configuration.SEED) if world_size > 1 else None
        split_gen = torch.Generator().manual_seed(seed) if seed is not None else torch.default_generator
        parts = random_split(indices, configuration.SPLIT_RATIOS, generator=split_gen)
        kw = dict(batch_size=configuration.BATCH_SIZE, shuffle=True, drop_last=False, device=device,
                  prefetch=prefetch, rank=rank, world_size=world_size, seed=seed,
                  prepare=int(configuration.NUM_CLASSES) if prepare else None)
        self.train_dataloader = GraphLoader(store, [indices[i] for i in parts[0].indices], **kw)
        ev = dict(kw, even=False, resident=bool(resident_eval))  # evaluation: every batch, reduced over ranks
        self.validation_dataloader = None if self.sanity_checking else \
            GraphLoader(store, [indices[i] for i in parts[1].indices], **ev)
        self.test_dataloader = None if self.sanity_checking else \
            GraphLoader(store, [indices[i] for i in parts[2].indices], **ev)
