// GATConv (heads = 1) message passing, fused: attention projections, edge
// logits, segmented softmax, weighted gather-sum and bias in one or two
// kernels; the first-order backward in four.
//
// Forward, per destination row i (torch_geometric 2.6.1 GATConv semantics):
//   a_dst_i = <h_i, att_dst>,  a_src_s = <h_s, att_src>
//   e_k     = leaky_relu(a_src[col_k] + a_dst_i, 0.2)        (self loop last)
//   alpha_k = exp(e_k - max_row e) / (sum_row exp(e - max) + 1e-16)
//   out_i   = sum_k alpha_k h[col_k] + bias
// The reference issues two (h * att).sum(-1) reductions per layer as separate
// ops (rocBLAS gemv at 10-80 us each was the top kernel of the first profile);
// here they are a light per-row pass (C >= 9) or fused into the aggregation
// (C <= 8).
//
// Two decompositions (rowgroup.h):
// * C >= 9, "channel-parallel": L = 8/16/32 lanes x CPL = 2..8 channels per
//   row (pick_fused_shape), so a wave holds 2-8 rows.  A per-row pass forms
//   a_src / a_dst (two group reductions per row); the aggregation pass then
//   takes logits edge-parallel from those [N] vectors (an earlier single-pass
//   variant that formed a_src from each gathered neighbour row paid one
//   cross-lane reduction per EDGE and ran 1.6x slower).
// * C <= 8, "edge-parallel": 8 lanes per row, one edge per lane (up to 3 per
//   lane kept in registers, degree <= 24 covers the dense stress graph); each
//   lane gathers the whole (<= 8-float) neighbour row, so logits need no
//   cross-lane reduction; max / sum / per-channel sums are 3-step shuffles.
//
// Backward (no atomics; deterministic):
//   B1 (destination rows)  ga_k = <g_out_i, h[col_k]>,  t_i = sum alpha ga,
//                          gp_k = alpha_k (ga_k - t_i) lrelu'(pre_k),
//                          g_a_dst_i = sum_k gp_k;  block partials of
//                          sum_i g_out_i (bias) and sum_i g_a_dst_i h_i (att_dst)
//   B2 (source nodes, CSC) g_a_src_j = sum gp,  g_h_j = sum alpha g_out[dst]
//                          + g_a_src_j att_src + g_a_dst_j att_dst;
//                          block partials of sum_j g_a_src_j h_j (att_src)
//   B3 (columns)           fold the block partials into g_bias, g_att_src, g_att_dst.
#include "gnbwd.h"
#include "rowgroup.h"

#ifndef VG_BWD_ROWS_WPE
#define VG_BWD_ROWS_WPE 4  // workgroups per CU the register allocation of k_gat_bwd_rows_cp targets for CPL <= 4
                           // (0: the compiler's choice, 3 at 132-138 VGPRs; 4 fits without a spill: step -0.01 ms,
                           // profiles/r06_occupancy_ab.txt)
#endif

namespace {

using namespace vg;

#ifndef VG_BWD_MAX_BLOCKS
#define VG_BWD_MAX_BLOCKS 4096
#endif
constexpr int kMaxBwdBlocks = VG_BWD_MAX_BLOCKS;  // grid cap of the backward row passes (partials count)
constexpr int kEP = 3;                // edge slots per lane in the edge-parallel kernels
#ifndef VG_FWD_ROWS
#define VG_FWD_ROWS 4
#endif
constexpr int kFwdRows = VG_FWD_ROWS;
#ifndef VG_FWD_PF
#define VG_FWD_PF 0  // 8: measured 7.22 vs 7.03 us per step-mix launch (profiles/r03_rejected_fwd_prefetch.txt)
#endif
constexpr int kFwdPf = VG_FWD_PF;  // source rows gathered before the softmax (k_gat_fwd_cp; <= L)
#ifndef VG_FWD_SLICE_ROWS
#define VG_FWD_SLICE_ROWS 100000
#endif
constexpr int kSliceRows = VG_FWD_SLICE_ROWS;  // aggregate in 64-channel slices from this many rows
#ifndef VG_FWD_SLICE
#define VG_FWD_SLICE 64
#endif
constexpr int kSlice = VG_FWD_SLICE;  // channels per slice: 64 (L 16 x 4) or 32 (L 8 x 4)
static_assert(kSlice == 64 || kSlice == 32, "slice width");
#ifndef VG_FWD_C64_L8
#define VG_FWD_C64_L8 0  // 33..64 channels: 8 lanes x 8 channels per row (A/B knob)
#endif  // neighbour rows in flight per step of the forward gather-sum

template <int CPL>
__device__ __forceinline__ void load_param(Vec<CPL>& r, const float* __restrict__ p, int c0, int C) {
  load_row<CPL, false>(r, p, c0, C);  // parameters live at arbitrary offsets of the flat buffer
}

// GraphNorm column partials (GnpRows, gnp_rows, gnp_block): rowgroup.h

// ===================================================================== forward
// C >= 9, pass A: per-row attention projections a_src_i = <h_i, att_src>,
// a_dst_i = <h_i, att_dst> (two group reductions per ROW, not per edge).
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_gat_att(const float* __restrict__ h, int N, int C,
                                                    const float* __restrict__ att_s,
                                                    const float* __restrict__ att_d,
                                                    float* __restrict__ a_src,
                                                    float* __restrict__ a_dst) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int c0 = g.lane * CPL;
  Vec<CPL> vs, vd, hi;
  load_param<CPL>(vs, att_s, c0, C);
  load_param<CPL>(vd, att_d, c0, C);
  load_row<CPL, VEC>(hi, h + (size_t)g.row * C, c0, C);
  const float as_i = group_sum<L>(dot_row<CPL, VEC>(hi, vs));
  const float ad_i = group_sum<L>(dot_row<CPL, VEC>(hi, vd));
  if (g.lane == 0) {
    a_src[g.row] = as_i;
    a_dst[g.row] = ad_i;
  }
}

// C >= 9, pass B: logits + exact two-pass segment softmax edge-parallel over
// the group's lanes, then the channel-parallel weighted gather-sum (4 rows
// gathered per step, independent loads in flight).
// ELL: the row's sources come from the padded column array ell [N][ew]
// (-1 past the degree, ew <= 4L, vg_csr_ell) at a fixed offset, so their
// loads -- and the a_src gathers behind them -- need not wait for row_ptr,
// which is still read (in parallel) for the degree and the alpha offsets.
// GNP: also the GraphNorm column partials of the output rows (gnp_fold).
template <int L, int CPL, bool VEC, bool ELL = false, bool GNP = false>
__global__ void __launch_bounds__(kBlock) k_gat_fwd_cp(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C,
    const float* __restrict__ h, const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ bias, float slope, float* __restrict__ out,
    float* __restrict__ alpha, int ld = 0, const int32_t* __restrict__ ell = nullptr, int ew = 0,
    float* __restrict__ gnp = nullptr, int seg_rows = 0) {
  // ld > 0: a channel slice -- h / out / bias point at the slice's first
  // channel, rows are ld floats apart, and only the slice at blockIdx.y == 0
  // writes alpha (every slice recomputes the row's softmax)
  const bool wr_alpha = blockIdx.y == 0;
  const int ldc = ld == 0 ? C : ld;  // total columns (the GraphNorm partials' row)
  const int cbase = ld == 0 ? 0 : blockIdx.y * C;
  if (ld == 0) {
    ld = C;
  } else {
    const int cb = blockIdx.y * C;
    h += cb;
    out += cb;
    bias += cb;
  }
  constexpr int T = 4;  // edges per lane kept in registers (rows up to 4L edges)
  GroupIdx g = group_index<L>();
  // GNP: segment-aligned blocks (gnp_rows), and every wave stays to the block
  // barrier: a group past its segment recomputes the segment's last row and
  // stores nothing
  GnpRows gr{0, 0, N};
  if constexpr (GNP) {
    gr = gnp_rows<kBlock / L>(seg_rows);
    g.row = gr.row0 + threadIdx.x / L;
  }
  const bool live = g.row < gr.end;
  if (!GNP && !live) return;
  const int i = live ? g.row : gr.end - 1;
  const int beg = row_ptr[i], end = row_ptr[i + 1];
  const int deg = end - beg;
  const float ad = a_dst[i];

  // edge-parallel logits, kept per lane: edge j lives in lane j % L, slot j / L
  int s_t[T];
  float e_t[T];
  bool v_t[T];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int j = g.lane + t * L;
    if constexpr (ELL) {
      const int sr = j < ew ? ell[(size_t)i * ew + j] : -1;
      v_t[t] = sr >= 0;
      s_t[t] = v_t[t] ? sr : 0;
    } else {
      v_t[t] = beg + j < end;
      s_t[t] = v_t[t] ? col[beg + j] : 0;
    }
  }
  // the first PF source rows are gathered NOW, in flight together with the
  // a_src gathers below: the softmax no longer stands between the column
  // indices and the row loads (one dependent round trip per row instead of
  // two; rows up to PF long -- every row of the training graphs -- are a
  // single round of loads)
  const int c0 = g.lane * CPL;
  constexpr int PF0 = kFwdPf < L ? kFwdPf : L;
  constexpr int PF = PF0 * CPL > 32 ? 32 / CPL : PF0;  // at most 32 prefetch registers per lane
  Vec<CPL> hp[PF > 0 ? PF : 1];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int su = __shfl(s_t[0], g.base + u, 64);
    if (__shfl(static_cast<int>(v_t[0]), g.base + u, 64))
      load_row<CPL, VEC>(hp[u], h + (size_t)su * ld, c0, C);
  }
#pragma unroll
  for (int t = 0; t < T; ++t) {
    e_t[t] = -INFINITY;
    if (v_t[t]) {
      e_t[t] = lrelu(a_src[s_t[t]] + ad, slope);
      m = fmaxf(m, e_t[t]);
    }
  }
  if constexpr (!ELL)
    for (int k = beg + g.lane + T * L; k < end; k += L) m = fmaxf(m, lrelu(a_src[col[k]] + ad, slope));
  m = group_max<L>(m);
  float ssum = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t)
    if (v_t[t]) {
      e_t[t] = expf(e_t[t] - m);  // now holds p = exp(e - max)
      ssum += e_t[t];
    }
  if constexpr (!ELL)
    for (int k = beg + g.lane + T * L; k < end; k += L) ssum += expf(lrelu(a_src[col[k]] + ad, slope) - m);
  const float denom = group_sum<L>(ssum) + kSoftmaxEps;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    if (v_t[t]) {
      e_t[t] = e_t[t] / denom;  // alpha
      if (wr_alpha && live) alpha[beg + g.lane + t * L] = e_t[t];
    }
  }
  if (!ELL && wr_alpha && live)
    for (int k = beg + g.lane + T * L; k < end; k += L)
      alpha[k] = expf(lrelu(a_src[col[k]] + ad, slope) - m) / denom;

  // channel-parallel gather-sum: the prefetched rows, then 4 neighbour rows
  // in flight (same row order, hence bit-identical sums)
  Vec<CPL> acc;
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
  const int dreg = deg < T * L ? deg : T * L;
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < dreg) {
      const float a = __shfl(e_t[0], g.base + u, 64);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, hp[u].v[q], acc.v[q]);
    }
  for (int j0 = PF; j0 < dreg; j0 += kFwdRows) {
    const int nj = dreg - j0 < kFwdRows ? dreg - j0 : kFwdRows;
    Vec<CPL> hv[kFwdRows];
    float a[kFwdRows];
#pragma unroll
    for (int u = 0; u < kFwdRows; ++u)
      if (u < nj) {
        const int j = j0 + u;
        const int t = j / L;
        const int sv = t == 0 ? s_t[0] : t == 1 ? s_t[1] : t == 2 ? s_t[2] : s_t[3];
        const float av = t == 0 ? e_t[0] : t == 1 ? e_t[1] : t == 2 ? e_t[2] : e_t[3];
        const int s = __shfl(sv, g.base + (j & (L - 1)), 64);
        a[u] = __shfl(av, g.base + (j & (L - 1)), 64);
        load_row<CPL, VEC>(hv[u], h + (size_t)s * ld, c0, C);
      }
#pragma unroll
    for (int u = 0; u < kFwdRows; ++u)
      if (u < nj)
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a[u], hv[u].v[q], acc.v[q]);
  }
  for (int j = T * L; !ELL && j < deg; ++j) {  // very long rows: alpha from memory (written above by this group)
    const int s = col[beg + j];
    const float a = expf(lrelu(a_src[s] + ad, slope) - m) / denom;
    Vec<CPL> hv;
    load_row<CPL, VEC>(hv, h + (size_t)s * ld, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, hv.v[q], acc.v[q]);
  }
  Vec<CPL> b;
  load_param<CPL>(b, bias, c0, C);
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] += b.v[q];
  if (live) store_row<CPL, VEC>(acc, out + (size_t)i * ld, c0, C);
  if constexpr (GNP) gnp_block<L, CPL>(acc.v, g.row, gr, C, c0, cbase, ldc, gnp);
}

// C <= 8: 8 lanes per destination row, one edge per lane.
// PRE: a_src / a_dst are inputs (vg_gat_lin_att computed them in the
// projection GEMM's epilogue); otherwise they are formed here and written.
// ELL as in k_gat_fwd_cp (ew <= 8 kEP).
// GNP as in k_gat_fwd_cp (with PRE: the attention projections are inputs).
template <int CMAX, bool PRE = false, bool ELL = false, bool GNP = false>
__global__ void __launch_bounds__(kBlock) k_gat_fwd_ep(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C,
    const float* __restrict__ h, const float* __restrict__ att_s, const float* __restrict__ att_d,
    const float* __restrict__ bias, float slope, float* __restrict__ out, float* __restrict__ alpha,
    float* __restrict__ a_src_io, float* __restrict__ a_dst_io, const int32_t* __restrict__ ell = nullptr,
    int ew = 0, float* __restrict__ gnp = nullptr, int seg_rows = 0) {
  static_assert(!GNP || PRE, "GraphNorm partials with precomputed projections only");
  constexpr int L = 8;
  GroupIdx g = group_index<L>();
  GnpRows gr{0, 0, N};  // GNP: segment-aligned blocks, as in k_gat_fwd_cp
  if constexpr (GNP) {
    gr = gnp_rows<kBlock / L>(seg_rows);
    g.row = gr.row0 + threadIdx.x / L;
  }
  const bool live = g.row < gr.end;
  if (!GNP && !live) return;
  const int i = live ? g.row : gr.end - 1;
  float vs[CMAX];
  float ad = 0.f;
  if constexpr (PRE) {
#pragma unroll
    for (int c = 0; c < CMAX; ++c) vs[c] = 0.f;
    ad = a_dst_io[i];
  } else {
    float as_i = 0.f;
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      const bool ok = c < C;
      vs[c] = ok ? att_s[c] : 0.f;
      const float hv = ok ? h[(size_t)i * C + c] : 0.f;
      ad = fmaf(hv, ok ? att_d[c] : 0.f, ad);
      as_i = fmaf(hv, vs[c], as_i);
    }
    if (g.lane == 0) {
      a_dst_io[i] = ad;
      a_src_io[i] = as_i;
    }
  }
  const int beg = row_ptr[i], end = row_ptr[i + 1];
  float hv[kEP][CMAX];
  float e[kEP];
  bool v[kEP];
  int sv[kEP];
#pragma unroll
  for (int t = 0; t < kEP; ++t) {
    const int j = g.lane + t * L;
    if constexpr (ELL) {
      const int sr = j < ew ? ell[(size_t)i * ew + j] : -1;
      v[t] = sr >= 0;
      sv[t] = v[t] ? sr : 0;
    } else {
      v[t] = beg + j < end;
      sv[t] = v[t] ? col[beg + j] : 0;
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < kEP; ++t) {
    e[t] = -INFINITY;
    if (v[t]) {
      const int s = sv[t];
      float a = PRE ? a_src_io[s] : 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        hv[t][c] = c < C ? h[(size_t)s * C + c] : 0.f;
        if (!PRE) a = fmaf(hv[t][c], vs[c], a);
      }
      e[t] = lrelu(a + ad, slope);
      m = fmaxf(m, e[t]);
    } else {
#pragma unroll
      for (int c = 0; c < CMAX; ++c) hv[t][c] = 0.f;
    }
  }
  // rows longer than 8*kEP: stream the rest (logits only for the max)
  for (int k = beg + g.lane + kEP * L; !ELL && k < end; k += L) {
    const int s = col[k];
    float a = PRE ? a_src_io[s] : 0.f;
    if (!PRE)
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) a = fmaf(h[(size_t)s * C + c], vs[c], a);
    m = fmaxf(m, lrelu(a + ad, slope));
  }
  m = group_max<L>(m);
  float ssum = 0.f;
  float acc[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) acc[c] = 0.f;
#pragma unroll
  for (int t = 0; t < kEP; ++t) {
    if (v[t]) {
      const float p = expf(e[t] - m);
      e[t] = p;
      ssum += p;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) acc[c] = fmaf(p, hv[t][c], acc[c]);
    }
  }
  for (int k = beg + g.lane + kEP * L; !ELL && k < end; k += L) {
    const int s = col[k];
    float a = PRE ? a_src_io[s] : 0.f, hv2[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      hv2[c] = c < C ? h[(size_t)s * C + c] : 0.f;
      if (!PRE) a = fmaf(hv2[c], vs[c], a);
    }
    const float p = expf(lrelu(a + ad, slope) - m);
    ssum += p;
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = fmaf(p, hv2[c], acc[c]);
  }
  const float denom = group_sum<L>(ssum) + kSoftmaxEps;
#pragma unroll
  for (int c = 0; c < CMAX; ++c) acc[c] = group_sum<L>(acc[c]);
  float o = 0.f;
  if (g.lane < C) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < CMAX; ++c)
      if (c == g.lane) v = acc[c];
    o = v / denom + bias[g.lane];
    if (live) out[(size_t)i * C + g.lane] = o;
  }
#pragma unroll
  for (int t = 0; t < kEP; ++t)
    if (v[t] && live) alpha[beg + g.lane + t * L] = e[t] / denom;
  for (int k = beg + g.lane + kEP * L; !ELL && live && k < end; k += L) {
    const int s = col[k];
    float a = PRE ? a_src_io[s] : 0.f;
    if (!PRE)
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) a = fmaf(h[(size_t)s * C + c], vs[c], a);
    alpha[k] = expf(lrelu(a + ad, slope) - m) / denom;
  }
  if constexpr (GNP) {
    const float ov[1] = {o};
    gnp_block<L, 1>(ov, g.row, gr, C, g.lane, 0, C, gnp);
  }
}

// ================================================== backward B1 (destination)
// GN: g_out is not read but formed here -- the GraphNorm(+ReLU+Dropout)
// backward of the layer's output (gnbwd.h, vg_gat_bwd_gn) -- and written to
// gn.g_out for the source pass (one launch and one pass over g_out fewer).
template <int L, int CPL, bool VEC, bool GN = false>
__global__ void __launch_bounds__(kBlock, CPL <= 4 && VG_BWD_ROWS_WPE ? VG_BWD_ROWS_WPE : 1) k_gat_bwd_rows_cp(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C,
    const float* __restrict__ h, const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ alpha, const float* __restrict__ g_out, float slope,
    float* __restrict__ g_pre, float* __restrict__ g_ad, float* __restrict__ part, const GnRows gn = GnRows{}) {
  constexpr int G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  const int base = (threadIdx.x & 63) & ~(L - 1);
  const int c0 = lane * CPL;
  Vec<CPL> pb, pd;  // sum g_out, sum g_a_dst * h
#pragma unroll
  for (int q = 0; q < CPL; ++q) pb.v[q] = pd.v[q] = 0.f;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  for (int i = lb * G + grp; i < N; i += gridDim.x * G) {
    const int beg = row_ptr[i], end = row_ptr[i + 1];
    const int deg = end - beg;
    Vec<CPL> go, hi;
    if constexpr (GN) {
      // every operand of the row's g_out in one round of loads (the column
      // parameters are L2 hits); the store waits for the end of the row, so
      // the neighbour gathers below are not ordered behind it
      gn_row<CPL, VEC>(gn, C, i, c0, go);
    } else {
      load_row<CPL, VEC>(go, g_out + (size_t)i * C, c0, C);
    }
    load_row<CPL, VEC>(hi, h + (size_t)i * C, c0, C);
    const int s_own = lane < deg ? col[beg + lane] : 0;
    const float al_own = lane < deg ? alpha[beg + lane] : 0.f;
    float ga_slot[4] = {0.f, 0.f, 0.f, 0.f};
    float t = 0.f;
    for (int j0 = 0; j0 < deg; j0 += 4) {
      const int nj = deg - j0 < 4 ? deg - j0 : 4;
      Vec<CPL> hv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < nj) {
          const int j = j0 + u;
          const int s = (deg <= L) ? __shfl(s_own, base + j, 64) : col[beg + j];
          load_row<CPL, VEC>(hv[u], h + (size_t)s * C, c0, C);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < nj) {
          const int j = j0 + u;
          const float ga = group_sum<L>(dot_row<CPL, VEC>(go, hv[u]));
          const float al = (deg <= L) ? __shfl(al_own, base + j, 64) : alpha[beg + j];
          t = fmaf(al, ga, t);
          if (lane == (j & (L - 1))) {
            const int slot = j / L;
            if (slot == 0) ga_slot[0] = ga;
            else if (slot == 1) ga_slot[1] = ga;
            else if (slot == 2) ga_slot[2] = ga;
            else if (slot == 3) ga_slot[3] = ga;
          }
        }
    }
    const float adi = a_dst[i];
    float gad = 0.f;
#pragma unroll
    for (int slot = 0; slot < 4; ++slot) {
      const int j = slot * L + lane;
      if (j < deg) {
        const int k = beg + j;
        const float pre = a_src[col[k]] + adi;
        const float gp = alpha[k] * (ga_slot[slot] - t) * (pre > 0.f ? 1.f : slope);
        g_pre[k] = gp;
        gad += gp;
      }
    }
    for (int j = 4 * L; j < deg; ++j) {
      const int k = beg + j;
      Vec<CPL> hv;
      load_row<CPL, VEC>(hv, h + (size_t)col[k] * C, c0, C);
      const float ga = group_sum<L>(dot_row<CPL, VEC>(go, hv));
      if (lane == 0) {
        const float pre = a_src[col[k]] + adi;
        const float gp = alpha[k] * (ga - t) * (pre > 0.f ? 1.f : slope);
        g_pre[k] = gp;
        gad += gp;
      }
    }
    gad = group_sum<L>(gad);
    if (lane == 0) g_ad[i] = gad;
    if constexpr (GN) store_row<CPL, VEC>(go, gn.g_out + (size_t)i * C, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      pb.v[q] += go.v[q];
      pd.v[q] = fmaf(gad, hi.v[q], pd.v[q]);
    }
  }
  Vec<CPL> vals[2] = {pb, pd};
  block_partials<L, CPL>(vals, 2, C, part);
}

template <int CMAX, bool GN = false>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_rows_ep(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C,
    const float* __restrict__ h, const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ alpha, const float* __restrict__ g_out, float slope,
    float* __restrict__ g_pre, float* __restrict__ g_ad, float* __restrict__ part, const GnRows gn = GnRows{}) {
  constexpr int L = 8, G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  float pb[CMAX], pd[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) pb[c] = pd[c] = 0.f;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  for (int i = lb * G + grp; i < N; i += gridDim.x * G) {
    const int beg = row_ptr[i], end = row_ptr[i + 1];
    float go[CMAX];
    if constexpr (GN) {  // every lane forms the whole (<= 8-channel) row; lane c stores it at the end
      Vec<CMAX> gv;
      gn_row<CMAX, false>(gn, C, i, 0, gv);
#pragma unroll
      for (int c = 0; c < CMAX; ++c) go[c] = gv.v[c];
    } else {
#pragma unroll
      for (int c = 0; c < CMAX; ++c) go[c] = c < C ? g_out[(size_t)i * C + c] : 0.f;
    }
    float ga[kEP], al[kEP];
    float t = 0.f;
#pragma unroll
    for (int u = 0; u < kEP; ++u) {
      const int k = beg + lane + u * L;
      ga[u] = 0.f;
      al[u] = 0.f;
      if (k < end) {
        const int s = col[k];
        float d = 0.f;
#pragma unroll
        for (int c = 0; c < CMAX; ++c)
          if (c < C) d = fmaf(go[c], h[(size_t)s * C + c], d);
        ga[u] = d;
        al[u] = alpha[k];
        t = fmaf(al[u], d, t);
      }
    }
    for (int k = beg + lane + kEP * L; k < end; k += L) {
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) d = fmaf(go[c], h[(size_t)col[k] * C + c], d);
      t = fmaf(alpha[k], d, t);
    }
    t = group_sum<L>(t);
    const float adi = a_dst[i];
    float gad = 0.f;
#pragma unroll
    for (int u = 0; u < kEP; ++u) {
      const int k = beg + lane + u * L;
      if (k < end) {
        const float pre = a_src[col[k]] + adi;
        const float gp = al[u] * (ga[u] - t) * (pre > 0.f ? 1.f : slope);
        g_pre[k] = gp;
        gad += gp;
      }
    }
    for (int k = beg + lane + kEP * L; k < end; k += L) {
      float d = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) d = fmaf(go[c], h[(size_t)col[k] * C + c], d);
      const float pre = a_src[col[k]] + adi;
      const float gp = alpha[k] * (d - t) * (pre > 0.f ? 1.f : slope);
      g_pre[k] = gp;
      gad += gp;
    }
    gad = group_sum<L>(gad);
    if constexpr (GN)
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C && lane == c) gn.g_out[(size_t)i * C + c] = go[c];
    if (lane == 0) {
      g_ad[i] = gad;
#pragma unroll
      for (int c = 0; c < CMAX; ++c) {
        pb[c] += go[c];
        pd[c] = fmaf(gad, c < C ? h[(size_t)i * C + c] : 0.f, pd[c]);
      }
    }
  }
  // fold: only lane 0 of each group carries partials
  __shared__ float red[G][2][CMAX];
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < CMAX; ++c) {
      red[grp][0][c] = pb[c];
      red[grp][1][c] = pd[c];
    }
  __syncthreads();
  if (threadIdx.x < 2 * CMAX) {
    const int v = threadIdx.x / CMAX, c = threadIdx.x % CMAX;
    float s = 0.f;
    for (int k = 0; k < G; ++k) s += red[k][v][c];
    if (c < C) part[(size_t)blockIdx.x * 2 * C + v * C + c] = s;
  }
}

// ===================================================== backward B2 (sources)
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_src_cp(
    const int32_t* __restrict__ csc_ptr, const int32_t* __restrict__ csc_slot,
    const int32_t* __restrict__ csc_dst, int N, int C, const float* __restrict__ h,
    const float* __restrict__ att_s, const float* __restrict__ att_d,
    const float* __restrict__ alpha, const float* __restrict__ g_out,
    const float* __restrict__ g_pre, const float* __restrict__ g_ad, const float* __restrict__ inj,
    int inj_row0, float* __restrict__ g_h, float* __restrict__ part) {
  constexpr int G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  const int base = (threadIdx.x & 63) & ~(L - 1);
  const int c0 = lane * CPL;
  Vec<CPL> vs, vd, ps;
  load_param<CPL>(vs, att_s, c0, C);
  load_param<CPL>(vd, att_d, c0, C);
#pragma unroll
  for (int q = 0; q < CPL; ++q) ps.v[q] = 0.f;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  for (int j = lb * G + grp; j < N; j += gridDim.x * G) {
    const int beg = csc_ptr[j], end = csc_ptr[j + 1];
    const int deg = end - beg;
    int d_own = 0;
    float a_own = 0.f, gas = 0.f;
    for (int p = beg + lane; p < end; p += L) {
      const int k = csc_slot[p];
      if (p == beg + lane) {
        d_own = csc_dst[p];
        a_own = alpha[k];
      }
      gas += g_pre[k];
    }
    gas = group_sum<L>(gas);
    Vec<CPL> acc;
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
    for (int e0 = 0; e0 < deg; e0 += 4) {
      const int ne = deg - e0 < 4 ? deg - e0 : 4;
      Vec<CPL> gv[4];
      float a[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < ne) {
          const int e = e0 + u;
          int d;
          if (deg <= L) {
            d = __shfl(d_own, base + e, 64);
            a[u] = __shfl(a_own, base + e, 64);
          } else {
            d = csc_dst[beg + e];
            a[u] = alpha[csc_slot[beg + e]];
          }
          load_row<CPL, VEC>(gv[u], g_out + (size_t)d * C, c0, C);
        }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (u < ne)
#pragma unroll
          for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a[u], gv[u].v[q], acc.v[q]);
    }
    const float gadj = g_ad[j];
    Vec<CPL> hj;
    load_row<CPL, VEC>(hj, h + (size_t)j * C, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      acc.v[q] = fmaf(gas, vs.v[q], fmaf(gadj, vd.v[q], acc.v[q]));
      ps.v[q] = fmaf(gas, hj.v[q], ps.v[q]);
    }
    if (inj && j >= inj_row0) {
      Vec<CPL> iv;
      load_row<CPL, VEC>(iv, inj + (size_t)(j - inj_row0) * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] += iv.v[q];
    }
    store_row<CPL, VEC>(acc, g_h + (size_t)j * C, c0, C);
  }
  Vec<CPL> vals[1] = {ps};
  block_partials<L, CPL>(vals, 1, C, part);
}

template <int CMAX>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_src_ep(
    const int32_t* __restrict__ csc_ptr, const int32_t* __restrict__ csc_slot,
    const int32_t* __restrict__ csc_dst, int N, int C, const float* __restrict__ h,
    const float* __restrict__ att_s, const float* __restrict__ att_d,
    const float* __restrict__ alpha, const float* __restrict__ g_out,
    const float* __restrict__ g_pre, const float* __restrict__ g_ad, const float* __restrict__ inj,
    int inj_row0, float* __restrict__ g_h, float* __restrict__ part) {
  constexpr int L = 8, G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  float ps[CMAX];
#pragma unroll
  for (int c = 0; c < CMAX; ++c) ps[c] = 0.f;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  for (int j = lb * G + grp; j < N; j += gridDim.x * G) {
    const int beg = csc_ptr[j], end = csc_ptr[j + 1];
    float gas = 0.f, acc[CMAX];
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = 0.f;
    for (int p = beg + lane; p < end; p += L) {
      const int k = csc_slot[p];
      const int d = csc_dst[p];
      const float a = alpha[k];
      gas += g_pre[k];
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) acc[c] = fmaf(a, g_out[(size_t)d * C + c], acc[c]);
    }
    gas = group_sum<L>(gas);
#pragma unroll
    for (int c = 0; c < CMAX; ++c) acc[c] = group_sum<L>(acc[c]);
    const float gadj = g_ad[j];
    if (lane < C) {
      float v = 0.f;
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c == lane) v = acc[c];
      if (inj && j >= inj_row0) v += inj[(size_t)(j - inj_row0) * C + lane];
      g_h[(size_t)j * C + lane] = fmaf(gas, att_s[lane], fmaf(gadj, att_d[lane], v));
    }
    if (lane == 0)
#pragma unroll
      for (int c = 0; c < CMAX; ++c)
        if (c < C) ps[c] = fmaf(gas, h[(size_t)j * C + c], ps[c]);
  }
  __shared__ float red[G][CMAX];
  if (lane == 0)
#pragma unroll
    for (int c = 0; c < CMAX; ++c) red[grp][c] = ps[c];
  __syncthreads();
  if (threadIdx.x < CMAX) {
    float s = 0.f;
    for (int k = 0; k < G; ++k) s += red[k][threadIdx.x];
    if ((int)threadIdx.x < C) part[(size_t)blockIdx.x * C + threadIdx.x] = s;
  }
}

// ===================================================== B3: fold the partials
// out[w] = sum_b part[b][w] for w < W (w < split -> out_a, else out_b); one
// 1024-thread block per 64 columns, 16 waves stride over the partial rows,
// LDS fold in a fixed order (deterministic).
// blockIdx.y selects the partial set: 0 -> (part, rows, W, split, out_a, out_b),
// 1 -> (part2, rows2, W2 -> out2).
__global__ void __launch_bounds__(1024) k_fold_cols(const float* __restrict__ part, int rows, int W,
                                                    int split, int acc, float* __restrict__ out_a,
                                                    float* __restrict__ out_b,
                                                    const float* __restrict__ part2 = nullptr,
                                                    int rows2 = 0, int W2 = 0,
                                                    float* __restrict__ out2 = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (blockIdx.y == 1) {
    part = part2;
    rows = rows2;
    W = W2;
    split = W2;
    out_a = out_b = out2;
  }
  const int w = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (w < W) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // loads in flight, fixed combine order
    int r = wave;
    for (; r + 48 < rows; r += 64) {
      a0 += part[(size_t)r * W + w];
      a1 += part[(size_t)(r + 16) * W + w];
      a2 += part[(size_t)(r + 32) * W + w];
      a3 += part[(size_t)(r + 48) * W + w];
    }
    for (; r < rows; r += 16) a0 += part[(size_t)r * W + w];
    s = (a0 + a1) + (a2 + a3);
  }
  __shared__ float red[16][64];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && w < W) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][lane];
    float* o = w < split ? out_a + w : out_b + (w - split);
    *o = acc ? *o + v : v;
  }
}

inline int bwd_grid(int N, int L) {
  const int g = grid_for(N, L);
  return g < kMaxBwdBlocks ? g : kMaxBwdBlocks;
}

}  // namespace

extern "C" int64_t vg_gat_bwd_ws_floats(int32_t num_nodes, int32_t num_edges, int32_t channels) {
  // g_pre [E'] + g_a_dst [N] + partials (B1: 2C per block, B2: C per block)
  return (int64_t)num_edges + num_nodes + (int64_t)kMaxBwdBlocks * 3 * channels;
}

extern "C" int vg_gat_fwd(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                          const float* h, const float* att_src, const float* att_dst,
                          const float* bias, float slope, float* out, float* alpha,
                          float* a_src, float* a_dst, void* stream) {
  if (N <= 0 || !row_ptr || !col || !h || !att_src || !att_dst || !bias || !out || !alpha ||
      !a_src || !a_dst)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (C <= 8) {
    const int grid = grid_for(N, 8);
    if (C <= 1)
      k_gat_fwd_ep<1><<<grid, kBlock, 0, s>>>(row_ptr, col, N, C, h, att_src, att_dst, bias, slope,
                                              out, alpha, a_src, a_dst);
    else if (C <= 2)
      k_gat_fwd_ep<2><<<grid, kBlock, 0, s>>>(row_ptr, col, N, C, h, att_src, att_dst, bias, slope,
                                              out, alpha, a_src, a_dst);
    else if (C <= 4)
      k_gat_fwd_ep<4><<<grid, kBlock, 0, s>>>(row_ptr, col, N, C, h, att_src, att_dst, bias, slope,
                                              out, alpha, a_src, a_dst);
    else
      k_gat_fwd_ep<8><<<grid, kBlock, 0, s>>>(row_ptr, col, N, C, h, att_src, att_dst, bias, slope,
                                              out, alpha, a_src, a_dst);
  } else {
    VG_DISPATCH_FUSED(C, (k_gat_att<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                             h, N, C, att_src, att_dst, a_src, a_dst)));
    VG_DISPATCH_FUSED(C, (k_gat_fwd_cp<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                             row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha)));
  }
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_att(const float* h, int32_t N, int32_t C, const float* att_src,
                          const float* att_dst, float* a_src, float* a_dst, void* stream) {
  if (N <= 0 || C <= 0 || C > 256 || !h || !att_src || !att_dst || !a_src || !a_dst)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (C <= 8)
    k_gat_att<8, 1, false><<<grid_for(N, 8), kBlock, 0, s>>>(h, N, C, att_src, att_dst, a_src,
                                                              a_dst);
  else
    VG_DISPATCH_FUSED(C, (k_gat_att<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                             h, N, C, att_src, att_dst, a_src, a_dst)));
  VG_CHECK_LAUNCH();
  return 0;
}

// the aggregation with (ell != NULL) or without the padded column array; a
// kernel shape takes the ELL path when ew fits its edge slots (4L, or 8 kEP)
// rows per workgroup of the aggregation kernel aggregate_fwd picks for (N, C):
// the granularity of its GraphNorm partials
static int agg_rows_per_block(int32_t N, int32_t C) {
  if (C <= 8) return kBlock / 8;
  if (N >= kSliceRows && C % kSlice == 0 && C > kSlice) return kBlock / (kSlice / 4);
  if (VG_FWD_C64_L8 && C > 32 && C <= 64 && C % 8 == 0) return kBlock / 8;
  Shape sh;
  if (!pick_fused_shape(C, sh)) return 0;
  return kBlock / sh.L;
}

template <bool GNP>
static int aggregate_fwd_launch(const int32_t* row_ptr, const int32_t* col, const int32_t* ell, int32_t ew,
                                 int32_t N, int32_t C, const float* h, const float* a_src, const float* a_dst,
                                 const float* bias, float slope, float* out, float* alpha, float* gnp,
                                 int32_t seg_rows, hipStream_t s) {
  float* as = const_cast<float*>(a_src);  // read-only under PRE
  float* ad = const_cast<float*>(a_dst);
  // GNP: segment-aligned blocks of G rows (gnp_rows), S * ceil(seg_rows / G)
  auto grid_rows = [&](int L) {
    if (!GNP) return grid_for(N, L);
    const int G = kBlock / L;
    return (N / seg_rows) * ((seg_rows + G - 1) / G);
  };
  if (C <= 8) {
    const int grid = grid_rows(8);
    const bool e = ell && ew <= 8 * kEP;
#define VG_EPF(CM)                                                                                           \
  do {                                                                                                       \
    if (e)                                                                                                   \
      k_gat_fwd_ep<CM, true, true, GNP><<<grid, kBlock, 0, s>>>(row_ptr, col, N, C, h, nullptr, nullptr,     \
                                                                bias, slope, out, alpha, as, ad, ell, ew,    \
                                                                gnp, seg_rows);                              \
    else                                                                                                     \
      k_gat_fwd_ep<CM, true, false, GNP><<<grid, kBlock, 0, s>>>(row_ptr, col, N, C, h, nullptr, nullptr,    \
                                                                 bias, slope, out, alpha, as, ad, nullptr,   \
                                                                 0, gnp, seg_rows);                          \
  } while (0)
    if (C <= 1) VG_EPF(1);
    else if (C <= 2) VG_EPF(2);
    else if (C <= 4) VG_EPF(4);
    else VG_EPF(8);
#undef VG_EPF
  } else if (N >= kSliceRows && C % kSlice == 0 && C > kSlice) {
    // large graphs: 64-channel slices, slice-major in dispatch order, so the
    // rows an XCD gathers at a time (a window of ~2 lattice floors) are half
    // or less of the full-width footprint in its 4 MiB L2
    constexpr int Ls = kSlice / 4;
    if (ell && ew <= 4 * Ls)
      k_gat_fwd_cp<Ls, 4, true, true, GNP><<<dim3(grid_rows(Ls), C / kSlice), kBlock, 0, s>>>(
          row_ptr, col, N, kSlice, h, a_src, a_dst, bias, slope, out, alpha, C, ell, ew, gnp, seg_rows);
    else
      k_gat_fwd_cp<Ls, 4, true, false, GNP><<<dim3(grid_rows(Ls), C / kSlice), kBlock, 0, s>>>(
          row_ptr, col, N, kSlice, h, a_src, a_dst, bias, slope, out, alpha, C, nullptr, 0, gnp, seg_rows);
  } else if (VG_FWD_C64_L8 && C > 32 && C <= 64 && C % 8 == 0) {
    k_gat_fwd_cp<8, 8, true, false, GNP><<<grid_rows(8), kBlock, 0, s>>>(
        row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, 0, nullptr, 0, gnp, seg_rows);
  } else {
    Shape sh;
    pick_fused_shape(C, sh);
    if (ell && ew <= 4 * sh.L)
      VG_DISPATCH_FUSED(C, (k_gat_fwd_cp<L_, CPL_, V_, true, GNP><<<grid_rows(L_), kBlock, 0, s>>>(
                               row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, 0, ell, ew, gnp,
                               seg_rows)));
    else
      VG_DISPATCH_FUSED(C, (k_gat_fwd_cp<L_, CPL_, V_, false, GNP><<<grid_rows(L_), kBlock, 0, s>>>(
                               row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, 0, nullptr, 0, gnp,
                               seg_rows)));
  }
  return 0;
}

static int aggregate_fwd(const int32_t* row_ptr, const int32_t* col, const int32_t* ell, int32_t ew, int32_t N,
                         int32_t C, const float* h, const float* a_src, const float* a_dst, const float* bias,
                         float slope, float* out, float* alpha, void* stream, float* gnp = nullptr,
                         int32_t seg_rows = 0) {
  if (N <= 0 || C <= 0 || C > 256 || !row_ptr || !col || !h || !a_src || !a_dst || !bias ||
      !out || !alpha || (ell && ew <= 0) || agg_rows_per_block(N, C) == 0)
    return VG_EINVAL;
  // segments of at least one workgroup's rows, dividing N
  if (gnp && (seg_rows < agg_rows_per_block(N, C) || N % seg_rows != 0)) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int rc = gnp ? aggregate_fwd_launch<true>(row_ptr, col, ell, ew, N, C, h, a_src, a_dst, bias, slope, out,
                                                  alpha, gnp, seg_rows, s)
                     : aggregate_fwd_launch<false>(row_ptr, col, ell, ew, N, C, h, a_src, a_dst, bias, slope,
                                                   out, alpha, nullptr, 0, s);
  if (rc) return rc;
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_aggregate_fwd(const int32_t* row_ptr, const int32_t* col, int32_t N,
                                    int32_t C, const float* h, const float* a_src,
                                    const float* a_dst, const float* bias, float slope, float* out,
                                    float* alpha, void* stream) {
  return aggregate_fwd(row_ptr, col, nullptr, 0, N, C, h, a_src, a_dst, bias, slope, out, alpha, stream);
}

extern "C" int vg_gat_aggregate_fwd_ell(const int32_t* row_ptr, const int32_t* col, const int32_t* ell,
                                        int32_t ell_width, int32_t N, int32_t C, const float* h,
                                        const float* a_src, const float* a_dst, const float* bias, float slope,
                                        float* out, float* alpha, void* stream) {
  if (!ell) return VG_EINVAL;
  return aggregate_fwd(row_ptr, col, ell, ell_width, N, C, h, a_src, a_dst, bias, slope, out, alpha, stream);
}

extern "C" int32_t vg_gat_gnp_rows(int32_t N, int32_t C) { return N > 0 ? agg_rows_per_block(N, C) : 0; }

extern "C" int64_t vg_gat_gnp_floats(int32_t N, int32_t C) {
  const int g = N > 0 ? agg_rows_per_block(N, C) : 0;
  if (g == 0) return 0;
  // segment-aligned blocks: S * ceil(seg_rows / g) <= ceil(N / g) + S, S <= N / g
  return 2 * (((int64_t)N + g - 1) / g) * 2 * C * 3;
}

extern "C" int vg_gat_aggregate_fwd_gnp(const int32_t* row_ptr, const int32_t* col, const int32_t* ell,
                                        int32_t ell_width, int32_t N, int32_t C, const float* h,
                                        const float* a_src, const float* a_dst, const float* bias, float slope,
                                        float* out, float* alpha, int32_t seg_rows, float* gnp, void* stream) {
  if (!gnp) return VG_EINVAL;
  return aggregate_fwd(row_ptr, col, ell, ell ? ell_width : 0, N, C, h, a_src, a_dst, bias, slope, out, alpha,
                       stream, gnp, seg_rows);
}

// ell [N][width] = the row's CSR columns in order, -1 past its degree (the
// caller guarantees width >= the largest degree)
__global__ void k_csr_ell(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int width,
                          int32_t* __restrict__ ell) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)N * width) return;
  const int i = static_cast<int>(t / width), j = static_cast<int>(t % width);
  const int beg = row_ptr[i], deg = row_ptr[i + 1] - beg;
  ell[t] = j < deg ? col[beg + j] : -1;
}

extern "C" int vg_csr_ell(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t width, int32_t* ell,
                          void* stream) {
  if (N <= 0 || width <= 0 || !row_ptr || !col || !ell) return VG_EINVAL;
  const long long total = (long long)N * width;
  k_csr_ell<<<static_cast<int>((total + 255) / 256), 256, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, col, N,
                                                                                                  width, ell);
  VG_CHECK_LAUNCH();
  return 0;
}

static int gat_bwd(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                   const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E, int32_t C,
                   const float* h, const float* att_src, const float* att_dst, const float* a_src,
                   const float* a_dst, const float* alpha, const float* g_out, float slope,
                   float* g_h, float* g_att_src, float* g_att_dst, float* g_bias,
                   int32_t accumulate, const float* inj, int32_t inj_row0, float* workspace,
                   void* stream, vg_fold* defer, int32_t* n_defer, const GnRows* gn = nullptr) {
  if (n_defer) *n_defer = 0;
  const bool pgrads = g_att_src != nullptr;
  if (N <= 0 || E <= 0 || !row_ptr || !col || !csc_ptr || !csc_slot || !csc_dst || !h ||
      !att_src || !att_dst || !a_src || !a_dst || !alpha || !g_out || !g_h || !workspace ||
      (pgrads && (!g_att_dst || !g_bias)) || inj_row0 < 0)
    return VG_EINVAL;
  const size_t gn_lds = 0;
  if (gn && (gn->S <= 0 || gn->seg_rows <= 0 || (long long)gn->S * gn->seg_rows != N ||
             !gn->x || !gn->g_y || !gn->weight || !gn->bias || !gn->mean_scale || !gn->stats || !gn->sums ||
             gn->g_out != g_out || gn->inj_row0 < 0))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* g_pre = workspace;
  float* g_ad = workspace + E;
  float* part1 = g_ad + N;                                // [grid1][2C]
  float* part2 = part1 + (size_t)kMaxBwdBlocks * 2 * C;   // [grid2][C]
  int grid1 = 0, grid2 = 0;
  if (C <= 8) {
    grid1 = grid2 = bwd_grid(N, 8);
#define VG_EP(CM)                                                                                 \
  do {                                                                                            \
    if (gn)                                                                                       \
      k_gat_bwd_rows_ep<CM, true><<<grid1, kBlock, gn_lds, s>>>(row_ptr, col, N, C, h, a_src, a_dst, \
                                                                alpha, g_out, slope, g_pre, g_ad,  \
                                                                part1, *gn);                       \
    else                                                                                          \
      k_gat_bwd_rows_ep<CM><<<grid1, kBlock, 0, s>>>(row_ptr, col, N, C, h, a_src, a_dst, alpha,   \
                                                     g_out, slope, g_pre, g_ad, part1);           \
    k_gat_bwd_src_ep<CM><<<grid2, kBlock, 0, s>>>(csc_ptr, csc_slot, csc_dst, N, C, h, att_src,    \
                                                  att_dst, alpha, g_out, g_pre, g_ad, inj,         \
                                                  inj_row0, g_h, part2);                           \
  } while (0)
    if (C <= 1) VG_EP(1);
    else if (C <= 2) VG_EP(2);
    else if (C <= 4) VG_EP(4);
    else VG_EP(8);
#undef VG_EP
  } else {
    Shape sh;
    if (!pick_fused_shape(C, sh)) return VG_EINVAL;
    grid1 = grid2 = bwd_grid(N, sh.L);
    if (gn)
      VG_DISPATCH_FUSED(C, (k_gat_bwd_rows_cp<L_, CPL_, V_, true><<<grid1, kBlock, gn_lds, s>>>(
                               row_ptr, col, N, C, h, a_src, a_dst, alpha, g_out, slope, g_pre,
                               g_ad, part1, *gn)));
    else
      VG_DISPATCH_FUSED(C, (k_gat_bwd_rows_cp<L_, CPL_, V_><<<grid1, kBlock, 0, s>>>(
                               row_ptr, col, N, C, h, a_src, a_dst, alpha, g_out, slope, g_pre,
                               g_ad, part1)));
    VG_DISPATCH_FUSED(C, (k_gat_bwd_src_cp<L_, CPL_, V_><<<grid2, kBlock, 0, s>>>(
                             csc_ptr, csc_slot, csc_dst, N, C, h, att_src, att_dst, alpha, g_out,
                             g_pre, g_ad, inj, inj_row0, g_h, part2)));
  }
  if (pgrads && defer) {  // described for vg_fold_batch: part1 -> [g_bias | g_att_dst], part2 -> g_att_src
    defer[0] = vg_fold{g_bias, C, C, C, accumulate, 1, {{part1, grid1, 2 * C}, {nullptr, 0, 0}}};
    defer[1] = vg_fold{g_att_dst, C, C, C, accumulate, 1, {{part1 + C, grid1, 2 * C}, {nullptr, 0, 0}}};
    defer[2] = vg_fold{g_att_src, C, C, C, accumulate, 1, {{part2, grid2, C}, {nullptr, 0, 0}}};
    *n_defer = 3;
  } else if (pgrads) {
    // fold: part1 rows -> [g_bias | g_att_dst], part2 rows -> g_att_src
    k_fold_cols<<<dim3(vg_blocks(2 * C, 64), 2), 1024, 0, s>>>(part1, grid1, 2 * C, C, accumulate,
                                                               g_bias, g_att_dst, part2, grid2, C,
                                                               g_att_src);
  }
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_bwd_ex(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                             const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E,
                             int32_t C, const float* h, const float* att_src, const float* att_dst,
                             const float* a_src, const float* a_dst, const float* alpha,
                             const float* g_out, float slope, float* g_h, float* g_att_src,
                             float* g_att_dst, float* g_bias, int32_t accumulate, const float* inj,
                             int32_t inj_row0, float* workspace, void* stream) {
  return gat_bwd(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, att_src, att_dst, a_src,
                 a_dst, alpha, g_out, slope, g_h, g_att_src, g_att_dst, g_bias, accumulate, inj,
                 inj_row0, workspace, stream, nullptr, nullptr);
}

extern "C" int vg_gat_bwd_deferred(const int32_t* row_ptr, const int32_t* col,
                                   const int32_t* csc_ptr, const int32_t* csc_slot,
                                   const int32_t* csc_dst, int32_t N, int32_t E, int32_t C,
                                   const float* h, const float* att_src, const float* att_dst,
                                   const float* a_src, const float* a_dst, const float* alpha,
                                   const float* g_out, float slope, float* g_h, float* g_att_src,
                                   float* g_att_dst, float* g_bias, int32_t accumulate,
                                   const float* inj, int32_t inj_row0, float* workspace,
                                   vg_fold* folds_out, int32_t* n_out, void* stream) {
  if (!folds_out || !n_out) return VG_EINVAL;
  return gat_bwd(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, att_src, att_dst, a_src,
                 a_dst, alpha, g_out, slope, g_h, g_att_src, g_att_dst, g_bias, accumulate, inj,
                 inj_row0, workspace, stream, folds_out, n_out);
}

extern "C" int vg_gat_bwd_gn(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                             const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E, int32_t C,
                             const float* h, const float* att_src, const float* att_dst, const float* a_src,
                             const float* a_dst, const float* alpha, const vg_gn_bwd_in* gn, float* g_out,
                             float slope, float* g_h, float* g_att_src, float* g_att_dst, float* g_bias,
                             int32_t accumulate, const float* inj, int32_t inj_row0, float* workspace,
                             vg_fold* folds_out, int32_t* n_out, void* stream) {
  if (!gn || !g_out || (folds_out != nullptr) != (n_out != nullptr) || gn->inj_offset < 0 ||
      (gn->inj && (gn->inj_offset % (C > 0 ? C : 1) != 0 || gn->inj_offset / (C > 0 ? C : 1) >= (1LL << 31))))
    return VG_EINVAL;
  const GnRows g{gn->x, gn->keep, gn->g_y, gn->inj, gn->weight, gn->bias, gn->mean_scale, gn->stats, gn->sums,
                 g_out, gn->eps, gn->segments, gn->seg_rows,
                 gn->inj ? static_cast<int>(gn->inj_offset / C) : 0};
  return gat_bwd(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, att_src, att_dst, a_src, a_dst, alpha, g_out,
                 slope, g_h, g_att_src, g_att_dst, g_bias, accumulate, inj, inj_row0, workspace, stream, folds_out,
                 n_out, &g);
}

extern "C" int vg_gat_bwd(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                          const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E,
                          int32_t C, const float* h, const float* att_src, const float* att_dst,
                          const float* a_src, const float* a_dst, const float* alpha,
                          const float* g_out, float slope, float* g_h, float* g_att_src,
                          float* g_att_dst, float* g_bias, float* workspace, void* stream) {
  if (!g_att_src || !g_att_dst || !g_bias) return VG_EINVAL;
  return vg_gat_bwd_ex(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, att_src, att_dst,
                       a_src, a_dst, alpha, g_out, slope, g_h, g_att_src, g_att_dst, g_bias, 0,
                       nullptr, 0, workspace, stream);
}
