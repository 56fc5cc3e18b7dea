"""Kernel resource guards (CPU: hipcc cross-compiles gfx950 here).

Round 6 found kernels of the step and of the configs[4] sweep held back by
what the compiler allocated rather than by their work:

* the merged GAT tangent source pass (k_jvp2_fold_src) and the grouped one
  (k_jvp_src_group) held one 16 KB block_partials image per row shape they
  switch over -- 96 KB of LDS, one workgroup per CU -- until the image came
  from one non-template function (rowgroup.h block_partials_lds);
* the f16 GEMM (k_hgemm) at 184 registers, 2 waves a SIMD, until
  amdgpu_waves_per_eu(4) (half.hip VG_HGEMM_WPE);
* the narrow GAT backward row passes (k_gat_bwd_rows_cp, CPL <= 4) at 3
  waves, 4 with launch bounds.

These tests compile the three sources with -Rpass-analysis=kernel-resource-usage
and hold those properties, so a later change that brings the waste back
fails here rather than as an unexplained step-time regression."""
from __future__ import annotations

import os
import re
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "building-gan-graph-conditioned-architectural-volume-generation_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def _usage(src: str) -> dict:
    """{kernel mangled name: {"vgpr", "agpr", "occ", "lds", "spill"}} of one source."""
    out = subprocess.run([HIPCC, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wno-pass-failed",
                          "-Rpass-analysis=kernel-resource-usage", "-c", os.path.join(CSRC, src), "-o", os.devnull],
                         capture_output=True, text=True, cwd=CSRC)
    assert out.returncode == 0, out.stderr[-2000:]
    res, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = res.setdefault(m.group(1), {})
            continue
        if cur is None:
            continue
        for key, pat in (("vgpr", r"\bVGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"),
                         ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)"),
                         ("spill", r"VGPRs Spill: (\d+)")):
            m = re.search(pat, line)
            if m:
                cur[key] = int(m.group(1))
    return res


@pytest.fixture(scope="module")
def usage():
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not present")
    srcs = ("gat_jvp.hip", "half.hip", "gat_fused.hip")
    with ThreadPoolExecutor(len(srcs)) as ex:
        return dict(zip(srcs, ex.map(_usage, srcs)))


def _named(table: dict, frag: str) -> dict:
    got = {k: v for k, v in table.items() if frag in k}
    assert got, f"no kernel named like {frag!r}"
    return got


def test_merged_source_passes_hold_one_partials_image(usage):
    for frag in ("k_jvp2_fold_src", "k_jvp_src_group"):
        for name, u in _named(usage["gat_jvp.hip"], frag).items():
            assert u["lds"] <= 16384, (name, u)
            assert u["occ"] >= 4, (name, u)


def test_f16_gemm_at_four_waves_without_spills(usage):
    """Every k_hgemm at 4 waves a SIMD; no spills, except the 128-wide
    LayerNorm GEMM's one VGPR (8 B of scratch a lane, in the epilogue's
    transposed statistics), measured faster than the spill-free epilogue
    (profiles/r06_hgemm_ln_probe.txt)."""
    for name, u in _named(usage["half.hip"], "k_hgemm").items():
        allowed = 1 if name.startswith("_ZN12_GLOBAL__N_17k_hgemmILi4ELi1E") else 0
        assert u["occ"] >= 4 and u.get("spill", 0) <= allowed, (name, u)


def test_narrow_gat_backward_rows_at_four_waves_without_spills(usage):
    narrow = {k: v for k, v in _named(usage["gat_fused.hip"], "k_gat_bwd_rows_cp").items()
              if re.search(r"k_gat_bwd_rows_cpILi\d+ELi[124]E", k)}
    assert narrow
    for name, u in narrow.items():
        assert u["occ"] >= 4 and u.get("spill", 0) == 0, (name, u)
