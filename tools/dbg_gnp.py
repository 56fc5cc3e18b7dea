import sys, torch
sys.path.insert(0, "building-gan-graph-conditioned-architectural-volume-generation_amd"); sys.path.insert(0, "tests")
from vgan import ops
from vgan._lib import LIB, ptr
from vgan.synth import SyntheticDataset
cuda = torch.device("cuda:0")
loc, vox = SyntheticDataset(8, seed=3).batch(range(2))
csr = ops.CSR(vox.edge_index.to(cuda), vox.num_nodes); csr.ell()
st = csr.stacked(3)
for C in (1, 64):
    n = st.num_nodes
    gnp, g = ops.gnp_buffer(st, C, cuda)
    gnp.fill_(float("nan"))
    h = torch.randn(n, C, device=cuda); a = torch.randn(n, device=cuda); b = torch.randn(C, device=cuda)
    out = torch.empty_like(h); al = torch.empty(st.num_edges, device=cuda)
    ops.aggregate_fwd_raw(st, C, ptr(h), ptr(a), ptr(a), ptr(b), 0.2, ptr(out), ptr(al), st.stream(), gnp)
    torch.cuda.synchronize()
    seg = st.seg_rows; bps = -(-seg // g)
    cnt = gnp.view(-1, 2, C, 3)[:, 0, 0, 0].cpu()
    print("C", C, "n", n, "seg", seg, "G", g, "bps", bps, "blocks expected", 3 * bps, "buffer blocks", cnt.numel())
    print("counts first 3*bps:", cnt[:3 * bps].tolist())
    print("nan positions:", torch.nonzero(torch.isnan(cnt[:3 * bps])).flatten().tolist()[:40])
