"""Generate ``convert_small.pt``: raw-JSON buildings and what the REFERENCE's
``DataCreatorHelper.process_data`` (building_gan/src/data.py:216-407, run here
through ``oracle.shim``) makes of them.

Run in the build container only (needs /root/reference):

    python tests/golden/make_convert_golden.py

The reference holds no raw JSON data, so the inputs are synthetic buildings in
the reference's JSON schema (the keys ``process_data`` and ``DataCreator.create``
read), exercising: a legacy VOID_OLD (-1) voxel type, integer and float
``site_area`` / ``far``, duplicate and self neighbours, unordered neighbour
lists, global-graph types without a proportion.  The fixture stores the JSON
texts and the attribute tensors of the returned ``LocalGraphData`` /
``VoxelGraphData`` objects (``torch.load(..., weights_only=True)``).
"""
from __future__ import annotations

import json
import os
import random
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, REPO)

from oracle import shim  # noqa: E402

NUM_CLASSES = 7


def json_building(seed: int, floors: int, ny: int, nx: int, int_site: bool):
    rnd = random.Random(seed)
    # voxel graph: a floors x ny x nx lattice, 4-neighbours on a floor + the voxel above / below
    voxels = []
    for f in range(floors):
        for y in range(ny):
            for x in range(nx):
                nbs = [[f, y + dy, x + dx] for dy, dx in ((0, 1), (1, 0), (0, -1), (-1, 0))
                       if 0 <= y + dy < ny and 0 <= x + dx < nx]
                nbs += [[f + df, y, x] for df in (-1, 1) if 0 <= f + df < floors]
                rnd.shuffle(nbs)
                if rnd.random() < 0.1:
                    nbs.append(list(nbs[0]))  # duplicate neighbour
                if rnd.random() < 0.05:
                    nbs.append([f, y, x])  # self neighbour
                t = rnd.randrange(-1, NUM_CLASSES)  # -1 = VOID_OLD
                voxels.append({
                    "location": [f, y, x],
                    "coordinate": [round(f * 3.5, 3), round(y * 4.1 + rnd.random(), 3), round(x * 3.9, 3)],
                    "dimension": [3.5, round(rnd.uniform(3, 5), 4), rnd.choice([4, 4.25, 3.75])],
                    "type": t,
                    "neighbors": nbs,
                })
    # program graph: a few nodes per floor
    nodes = []
    for f in range(floors):
        for k in range(rnd.randrange(2, 5)):
            nodes.append({"floor": f, "type": rnd.randrange(NUM_CLASSES - 1), "type_id": k,
                          "center": [rnd.randrange(40), rnd.randrange(40)]})
    keys = [[n["floor"], n["type"], n["type_id"]] for n in nodes]
    for i, n in enumerate(nodes):
        cand = [keys[j] for j in range(len(nodes)) if j != i and abs(nodes[j]["floor"] - n["floor"]) <= 1]
        n["neighbors"] = rnd.sample(cand, min(len(cand), 3))
    present = sorted({n["type"] for n in nodes})
    props = [rnd.random() for _ in present]
    glob = {
        "far": round(rnd.uniform(0.5, 4.0), 5) if seed % 2 else 2,
        "site_area": rnd.randrange(400, 1600) if int_site else round(rnd.uniform(400, 1600), 3),
        "global_node": [{"type": t, "proportion": p / sum(props)} for t, p in zip(present, props)],
    }
    return glob, {"node": nodes}, {"voxel_node": voxels}


def main():
    shim.install()
    import importlib

    data_mod = importlib.import_module("building_gan.src.data")
    cfg = importlib.import_module("building_gan.src.config").Configuration()
    out = {"buildings": []}
    for seed, (fl, ny, nx, int_site) in enumerate([(3, 4, 5, False), (2, 3, 3, True), (4, 2, 6, False)]):
        g, loc, vox = json_building(100 + seed, fl, ny, nx, int_site)
        number = str(4000 + seed)
        lo, vo = data_mod.DataCreatorHelper.process_data(g, loc, vox, cfg, number)
        rec = {"global_json": json.dumps(g), "local_json": json.dumps(loc), "voxel_json": json.dumps(vox),
               "data_number": number}
        for prefix, obj in (("local.", lo), ("voxel.", vo)):
            for k, v in vars(obj).items():
                if torch.is_tensor(v):
                    rec[prefix + k] = v
                elif k != "data_number":
                    raise TypeError(f"unexpected attribute {k}")
        out["buildings"].append(rec)
    path = os.path.join(HERE, "convert_small.pt")
    torch.save(out, path)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
