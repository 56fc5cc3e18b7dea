// GraphNorm(+ReLU+Dropout) backward, elementwise part, shared by the
// GraphNorm apply kernels (graphnorm.hip) and the GAT backward row pass that
// computes it in its prologue (gat_fused.hip, vg_gat_bwd_gn): one formula, so
// the fused and the separate paths agree.  torch_geometric 2.6.1 GraphNorm
// (batch=None, models.py:73-75 / 193-195), with stats = [mu | d]:
//
//   d = sqrt(mean((x - ms mu)^2) + eps),  ohat = (x - ms mu) / d,  z = w ohat + b
//   gz = g_y [z > 0] keep,  A = sum gz,  B = sum gz ohat  (the segment's N rows)
//   a = (1 - ms) mu = mean(x - ms mu)
//   g_x  = (w / d)(gz - B ohat / N - (ms / N)(A - B a / d))
//   g_ms = -mu (w / d)(A - B a / d)
#pragma once
#include "rowgroup.h"

namespace vg {

__device__ __forceinline__ float gn_bwd_elem(float xv, float gyv, float kv, bool has_keep, float mu, float sd,
                                             float wc, float bc, float msc, float A, float B, float eps,
                                             float inv_n) {
  (void)eps;  // folded into sd = d by the statistics pass
  const float oh = (xv - mu * msc) / sd;
  const float z = oh * wc + bc;
  float gz = z > 0.f ? gyv : 0.f;
  if (has_keep) gz *= kv;
  const float colsum = A - B * ((1.f - msc) * mu) / sd;  // sum over rows of (gz - B ohat / N)
  return (wc / sd) * (gz - B * oh * inv_n - msc * inv_n * colsum);
}

// mean_scale's gradient of one segment from its column sums A, B
__device__ __forceinline__ float gn_g_ms(float mu, float sd, float wc, float msc, float A, float B) {
  return -mu * (wc / sd) * (A - B * ((1.f - msc) * mu) / sd);
}

// The GraphNorm backward a GAT backward row pass forms in its prologue
// (vg_gn_bwd_in of include/vgan.h, device-side): rows are the S * seg_rows
// stacked rows of the GAT call; inj (element index >= inj_row0 * C) is added.
struct GnRows {
  const float* x;
  const float* keep;
  const float* g_y;
  const float* inj;
  const float* weight;
  const float* bias;
  const float* mean_scale;
  const float* stats;  // [S][2C] mean | d (the GraphNorm denominator)
  const float* sums;   // [S][2C] A | B
  float* g_out;        // g_x, written for the source pass
  float eps;
  int S, seg_rows, inj_row0;
};

// g_x of row i, channels c0 .. c0 + CPL - 1 (rowgroup.h lane layout): x,
// g_y, keep, injection and the column parameters / the segment's statistics
// and sums, all loaded in one round (the parameters are L2 hits)
template <int CPL, bool VEC>
__device__ __forceinline__ void gn_row(const GnRows& g, int C, int i, int c0, Vec<CPL>& out) {
  const int sg = i / g.seg_rows;
  const float* __restrict__ st = g.stats + (size_t)sg * 2 * C;
  const float* __restrict__ sm = g.sums + (size_t)sg * 2 * C;
  Vec<CPL> xr, gr, kr, ir, wv, bv, mv, mu, sd, av, bb;
  load_row<CPL, VEC>(xr, g.x + (size_t)i * C, c0, C);
  load_row<CPL, VEC>(gr, g.g_y + (size_t)i * C, c0, C);
  const bool keep = g.keep != nullptr, inj = g.inj && i >= g.inj_row0;
  if (keep) load_row<CPL, VEC>(kr, g.keep + (size_t)i * C, c0, C);
  if (inj) load_row<CPL, VEC>(ir, g.inj + (size_t)(i - g.inj_row0) * C, c0, C);
  load_row<CPL, VEC>(wv, g.weight, c0, C);
  load_row<CPL, VEC>(bv, g.bias, c0, C);
  load_row<CPL, VEC>(mv, g.mean_scale, c0, C);
  load_row<CPL, VEC>(mu, st, c0, C);
  load_row<CPL, VEC>(sd, st + C, c0, C);
  load_row<CPL, VEC>(av, sm, c0, C);
  load_row<CPL, VEC>(bb, sm + C, c0, C);
  const float inv_n = 1.f / static_cast<float>(g.seg_rows);
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    float r = gn_bwd_elem(xr.v[q], gr.v[q], keep ? kr.v[q] : 1.f, keep, mu.v[q], sd.v[q], wv.v[q], bv.v[q],
                          mv.v[q], av.v[q], bb.v[q], g.eps, inv_n);
    if (inj) r += ir.v[q];
    out.v[q] = c0 + q < C ? r : 0.f;
  }
}

}  // namespace vg
