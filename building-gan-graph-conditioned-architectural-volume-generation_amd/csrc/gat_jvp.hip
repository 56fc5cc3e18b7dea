// GATConv (heads = 1): tangent and second-order terms for the WGAN-GP double
// backward (the critic engine, vgan/critic.py; trainer.py:306-316 with
// create_graph=True).
//
// out = A(h) h + bias with alpha = softmax_row(lrelu(a_src[j] + a_dst[i])),
// a_src = h att_src, a_dst = h att_dst.  Given a tangent u of h and the adjoint
// g (= g_out, from the first backward) this computes
//   J u      = sum_k alpha_k u_j + alpha'_k h_j,      alpha'_k = alpha_k (e'_k - ebar_i)
//              e'_k = lam_k (u_j att_src + u_i att_dst),  lam_k = lrelu'(pre_k),
//              ebar_i = sum alpha e'
// and, for Q = <g, J u>, with per-edge U_k = <g_i, u_j>, H_k = <g_i, h_j>,
// R_k = U_k + e'_k H_k and row means Hbar = sum alpha H, Rbar = sum alpha R:
//   dQ/dpre_k   gz_k  = lam_k alpha_k (R_k - Rbar - (e'_k - ebar) Hbar - ebar (H_k - Hbar))
//   dQ/dpre'_k  gzp_k = lam_k alpha_k (H_k - Hbar)
//   dQ/dh_j     = sum_{k: src j} alpha'_k g_dst + (sum_{src j} gz) att_src + (sum_{row j} gz) att_dst
//   dQ/datt_src = sum_j (sum_{src j} gz) h_j + (sum_{src j} gzp) u_j
//   dQ/datt_dst = sum_i (sum_{row i} gz) h_i + (sum_{row i} gzp) u_i        (dQ/dbias = 0)
// (checked against autograd double backward in float64, tests/critic_ref.py).
//
// Three row passes, deterministic (no atomics): per-node tangent projections,
// destination rows (J u, per-edge gz / gzp / alpha', block partials of
// dQ/datt_dst), source nodes over the CSC (dQ/dh, partials of dQ/datt_src),
// then one fold that ADDS into g_att_src / g_att_dst.
#include "gnjvp.h"
#include "rowgroup.h"

#ifndef VG_JVP_ROWS_WPE
#define VG_JVP_ROWS_WPE 0  // workgroups per CU the register allocation of k_jvp_rows targets for CPL <= 4 (0: the compiler's choice)
#endif

namespace {

using namespace vg;

#ifndef VG_BWD_MAX_BLOCKS
#define VG_BWD_MAX_BLOCKS 4096
#endif
constexpr int kMaxBlocks = VG_BWD_MAX_BLOCKS;

template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_jvp_att(const float* __restrict__ u, int N, int C,
                                                    const float* __restrict__ att_s,
                                                    const float* __restrict__ att_d,
                                                    float* __restrict__ up_src,
                                                    float* __restrict__ up_dst) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int c0 = g.lane * CPL;
  Vec<CPL> vs, vd, ui;
  load_row<CPL, false>(vs, att_s, c0, C);
  load_row<CPL, false>(vd, att_d, c0, C);
  load_row<CPL, VEC>(ui, u + (size_t)g.row * C, c0, C);
  const float s = group_sum<L>(dot_row<CPL, VEC>(ui, vs));
  const float d = group_sum<L>(dot_row<CPL, VEC>(ui, vd));
  if (g.lane == 0) {
    up_src[g.row] = s;
    up_dst[g.row] = d;
  }
}

// The tangent sweep's GraphNorm column sums formed where the GraphNorm's
// input tangent u is produced (GNJ; vg_gat_jvp2_gn_deferred): per column
// [sum u, sum xt u, sum p, sum p u, sum p xt] with xt = x - mu,
// p = g_y [z > 0] keep -- the sums of graphnorm.hip's k_gn_jvp2_partial, which
// re-read x, u, g_y and keep in a launch of its own -- as one row of partials
// per workgroup, part [blocks][5][C] (groups in order: deterministic).
struct GnJvp {
  const float* x;
  const float* keep;
  const float* gy;
  const float* stats;
  const float* w;
  const float* b;
  const float* ms;
  float eps;
  float* part;
};

template <int L, int CPL>
__device__ __forceinline__ void gnj_block_sums(const Vec<CPL> (&v)[5], int C, float* __restrict__ part) {
  constexpr int G = kBlock / L, Wg = L * CPL;
  __shared__ float red[kBlock * CPL];  // G groups x Wg channels
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    __syncthreads();  // the previous sum (or the att_dst partials) is done with red
#pragma unroll
    for (int q = 0; q < CPL; ++q) red[grp * Wg + lane * CPL + q] = v[k].v[q];
    __syncthreads();
    for (int c = threadIdx.x; c < Wg; c += kBlock) {
      float s = 0.f;
      for (int g = 0; g < G; ++g) s += red[g * Wg + c];
      if (c < C) part[((size_t)blockIdx.x * 5 + k) * C + c] = s;
    }
  }
}

// e_u / e_h: per-edge U, H written by the lane that reads them back (no restrict).
template <int L, int CPL, bool VEC, bool GNJ = false>
__global__ void __launch_bounds__(kBlock, CPL <= 4 && VG_JVP_ROWS_WPE ? VG_JVP_ROWS_WPE : 1) k_jvp_rows(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C,
    const float* __restrict__ h, const float* __restrict__ u, const float* __restrict__ gv,
    const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ up_src, const float* __restrict__ up_dst,
    const float* __restrict__ alpha, float slope, float* __restrict__ u_out, float* e_u,
    float* e_h, float* __restrict__ e_gz, float* __restrict__ e_gzp, float* __restrict__ e_alp,
    float* __restrict__ n_gad, float* __restrict__ part, const GnJvp gj = GnJvp{}) {
  constexpr int G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  const int c0 = lane * CPL;
  Vec<CPL> pd;
#pragma unroll
  for (int q = 0; q < CPL; ++q) pd.v[q] = 0.f;
  // GNJ: the lane's columns' GraphNorm operands and its five running sums
  Vec<CPL> gmu, gs, gw, gb, gms, gsum[5];
  if constexpr (GNJ) {
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = c0 + q;
      const bool ok = c < C;
      gmu.v[q] = ok ? gj.stats[c] : 0.f;
      gs.v[q] = ok ? gj.stats[C + c] : 1.f;  // d, the whole denominator
      gw.v[q] = ok ? gj.w[c] : 0.f;
      gb.v[q] = ok ? gj.b[c] : 0.f;
      gms.v[q] = ok ? gj.ms[c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k)
#pragma unroll
      for (int q = 0; q < CPL; ++q) gsum[k].v[q] = 0.f;
  }
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  for (int i = lb * G + grp; i < N; i += gridDim.x * G) {
    const int beg = row_ptr[i], end = row_ptr[i + 1];
    const float adi = a_dst[i], updi = up_dst[i];
    float eb = 0.f;
    for (int k = beg + lane; k < end; k += L) {
      const int j = col[k];
      const float lam = (a_src[j] + adi) > 0.f ? 1.f : slope;
      eb = fmaf(alpha[k], lam * (up_src[j] + updi), eb);
    }
    eb = group_sum<L>(eb);
    Vec<CPL> gi, acc;
    load_row<CPL, VEC>(gi, gv + (size_t)i * C, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
    float hb = 0.f, rb = 0.f;
    for (int k0 = beg; k0 < end; k0 += 4) {
      const int nk = end - k0 < 4 ? end - k0 : 4;
      Vec<CPL> uv[4], hv[4];
      float a[4], ep[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < nk) {
          const int k = k0 + t, j = col[k];
          a[t] = alpha[k];
          const float lam = (a_src[j] + adi) > 0.f ? 1.f : slope;
          ep[t] = lam * (up_src[j] + updi);
          load_row<CPL, VEC>(uv[t], u + (size_t)j * C, c0, C);
          load_row<CPL, VEC>(hv[t], h + (size_t)j * C, c0, C);
        }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < nk) {
          const float U = group_sum<L>(dot_row<CPL, VEC>(gi, uv[t]));
          const float H = group_sum<L>(dot_row<CPL, VEC>(gi, hv[t]));
          const float alp = a[t] * (ep[t] - eb);
#pragma unroll
          for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a[t], uv[t].v[q], fmaf(alp, hv[t].v[q], acc.v[q]));
          hb = fmaf(a[t], H, hb);
          rb = fmaf(a[t], fmaf(ep[t], H, U), rb);
          const int k = k0 + t;
          if (lane == ((k - beg) & (L - 1))) {
            e_u[k] = U;
            e_h[k] = H;
          }
        }
    }
    store_row<CPL, VEC>(acc, u_out + (size_t)i * C, c0, C);
    if constexpr (GNJ) {  // this row's terms of the GraphNorm tangent sums (k_gn_jvp2_partial's formulas)
      Vec<CPL> xv, gyv, kv;
      load_row<CPL, VEC>(xv, gj.x + (size_t)i * C, c0, C);
      load_row<CPL, VEC>(gyv, gj.gy + (size_t)i * C, c0, C);
      if (gj.keep) load_row<CPL, VEC>(kv, gj.keep + (size_t)i * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) {
        const float uv = acc.v[q];
        const float xt = xv.v[q] - gmu.v[q];
        const float z = ((xv.v[q] - gmu.v[q] * gms.v[q]) / gs.v[q]) * gw.v[q] + gb.v[q];
        float pv = z > 0.f ? gyv.v[q] : 0.f;
        if (gj.keep) pv *= kv.v[q];
        gsum[0].v[q] += uv;
        gsum[1].v[q] = fmaf(xt, uv, gsum[1].v[q]);
        gsum[2].v[q] += pv;
        gsum[3].v[q] = fmaf(pv, uv, gsum[3].v[q]);
        gsum[4].v[q] = fmaf(pv, xt, gsum[4].v[q]);
      }
    }
    float gad = 0.f, gpd = 0.f;
    for (int k = beg + lane; k < end; k += L) {
      const int j = col[k];
      const float a = alpha[k];
      const float lam = (a_src[j] + adi) > 0.f ? 1.f : slope;
      const float ep = lam * (up_src[j] + updi);
      const float U = e_u[k], H = e_h[k];
      const float R = fmaf(ep, H, U);
      const float gz = lam * a * (R - rb - (ep - eb) * hb - eb * (H - hb));
      const float gzp = lam * a * (H - hb);
      e_gz[k] = gz;
      e_gzp[k] = gzp;
      e_alp[k] = a * (ep - eb);
      gad += gz;
      gpd += gzp;
    }
    gad = group_sum<L>(gad);
    gpd = group_sum<L>(gpd);
    if (lane == 0) n_gad[i] = gad;
    Vec<CPL> hi, ui;
    load_row<CPL, VEC>(hi, h + (size_t)i * C, c0, C);
    load_row<CPL, VEC>(ui, u + (size_t)i * C, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) pd.v[q] = fmaf(gad, hi.v[q], fmaf(gpd, ui.v[q], pd.v[q]));
  }
  block_partials<L, CPL>(&pd, 1, C, part);
  if constexpr (GNJ) gnj_block_sums<L, CPL>(gsum, C, gj.part);
}

// The source pass as a block body: logical block lb of nb (one launch of
// k_jvp_src, or one item of a grouped launch).
template <int L, int CPL, bool VEC>
__device__ __forceinline__ void jvp_src_body(
    int lb, int nb, const int32_t* __restrict__ csc_ptr, const int32_t* __restrict__ csc_slot,
    const int32_t* __restrict__ csc_dst, int N, int C, const float* __restrict__ h,
    const float* __restrict__ u, const float* __restrict__ gv, const float* __restrict__ att_s,
    const float* __restrict__ att_d, const float* __restrict__ e_gz,
    const float* __restrict__ e_gzp, const float* __restrict__ e_alp,
    const float* __restrict__ n_gad, float* __restrict__ h_inj, float* __restrict__ part) {
  constexpr int G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  const int c0 = lane * CPL;
  Vec<CPL> vs, vd, ps;
  load_row<CPL, false>(vs, att_s, c0, C);
  load_row<CPL, false>(vd, att_d, c0, C);
#pragma unroll
  for (int q = 0; q < CPL; ++q) ps.v[q] = 0.f;
  for (int j = lb * G + grp; j < N; j += nb * G) {
    const int beg = csc_ptr[j], end = csc_ptr[j + 1];
    float gas = 0.f, gps = 0.f;
    for (int p = beg + lane; p < end; p += L) {
      const int k = csc_slot[p];
      gas += e_gz[k];
      gps += e_gzp[k];
    }
    gas = group_sum<L>(gas);
    gps = group_sum<L>(gps);
    Vec<CPL> acc;
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
    for (int p0 = beg; p0 < end; p0 += 4) {
      const int np = end - p0 < 4 ? end - p0 : 4;
      Vec<CPL> gd[4];
      float a[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < np) {
          const int p = p0 + t;
          a[t] = e_alp[csc_slot[p]];
          load_row<CPL, VEC>(gd[t], gv + (size_t)csc_dst[p] * C, c0, C);
        }
#pragma unroll
      for (int t = 0; t < 4; ++t)
        if (t < np)
#pragma unroll
          for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a[t], gd[t].v[q], acc.v[q]);
    }
    const float gadj = n_gad[j];
    Vec<CPL> hj, uj;
    load_row<CPL, VEC>(hj, h + (size_t)j * C, c0, C);
    load_row<CPL, VEC>(uj, u + (size_t)j * C, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      acc.v[q] = fmaf(gas, vs.v[q], fmaf(gadj, vd.v[q], acc.v[q]));
      ps.v[q] = fmaf(gas, hj.v[q], fmaf(gps, uj.v[q], ps.v[q]));
    }
    store_row<CPL, VEC>(acc, h_inj + (size_t)j * C, c0, C);
  }
  block_partials<L, CPL>(&ps, 1, C, part, lb);
}

template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_jvp_src(
    const int32_t* __restrict__ csc_ptr, const int32_t* __restrict__ csc_slot,
    const int32_t* __restrict__ csc_dst, int N, int C, const float* __restrict__ h,
    const float* __restrict__ u, const float* __restrict__ gv, const float* __restrict__ att_s,
    const float* __restrict__ att_d, const float* __restrict__ e_gz,
    const float* __restrict__ e_gzp, const float* __restrict__ e_alp,
    const float* __restrict__ n_gad, float* __restrict__ h_inj, float* __restrict__ part) {
  jvp_src_body<L, CPL, VEC>(xcd_remap(blockIdx.x, gridDim.x), gridDim.x, csc_ptr, csc_slot, csc_dst, N, C, h, u, gv,
                            att_s, att_d, e_gz, e_gzp, e_alp, n_gad, h_inj, part);
}

// Grouped source passes (vg_gat_jvp_src_group): the tangent sweep's dQ/dh
// injections and att_src partials are read only by the later VJP pass and the
// gradient folds, so the critic engine runs every layer's source pass in one
// launch at the end of the sweep.  Blocks [block0[i], block0[i+1]) are item
// i's; shape ids (VEC layouts only): 0 = L8 x 1 (C <= 8), 1 = L8 x 2,
// 2 = L8 x 4, 3 = L16 x 4, 4 = L16 x 8, 5 = L32 x 8.
struct JvpSrcGroup {
  vg_jvp_src d[VG_JVP_GROUP_MAX];
  int block0[VG_JVP_GROUP_MAX + 1];
  int n;
};

__global__ void __launch_bounds__(kBlock) k_jvp_src_group(const JvpSrcGroup g) {
  const int lbg = xcd_remap(blockIdx.x, gridDim.x);
  int i = 0;
  while (i + 1 < g.n && lbg >= g.block0[i + 1]) ++i;
  const vg_jvp_src& d = g.d[i];
  const int lb = lbg - g.block0[i], nb = g.block0[i + 1] - g.block0[i];
#define VG_JS(L_, CPL_)                                                                                   \
  jvp_src_body<L_, CPL_, true>(lb, nb, d.csc_ptr, d.csc_slot, d.csc_dst, d.N, d.C, d.h, d.u, d.g_out,      \
                               d.att_src, d.att_dst, d.e_gz, d.e_gzp, d.e_alp, d.n_gad, d.h_inj, d.part)
  switch (d.shape) {
    case 0: VG_JS(8, 1); break;
    case 1: VG_JS(8, 2); break;
    case 2: VG_JS(8, 4); break;
    case 3: VG_JS(16, 4); break;
    case 4: VG_JS(16, 8); break;
    default: VG_JS(32, 8); break;
  }
#undef VG_JS
}

// The GraphNorm second-order fold (gnjvp.h: one wave per column, blocks
// [0, C): wave 0 works, the others exit) and a described GAT tangent source
// pass (blocks C ..: jvp_src_body) in ONE launch: the source pass's injections
// and att_src partials are read only by the later VJP pass and the folds, so
// it need not be a launch of its own on the tangent sweep's dependent chain
// (vg_graphnorm_jvp2_fold_src).
__global__ void __launch_bounds__(kBlock) k_jvp2_fold_src(const float* __restrict__ part, int chunks, int N, int C,
                                                          const float* __restrict__ w, const float* __restrict__ ms,
                                                          const float* __restrict__ stats, float* __restrict__ sums,
                                                          float* __restrict__ g_w, float* __restrict__ g_ms,
                                                          const vg_jvp_src d) {
  if ((int)blockIdx.x < C) {
    const int lane = threadIdx.x & 63;
    if ((threadIdx.x >> 6) == 0) vg::gn_jvp2_fold_col(part, chunks, N, C, w, ms, stats, sums, g_w, g_ms, blockIdx.x, lane);
    return;
  }
  const int nb = gridDim.x - C;
  const int lb = xcd_remap(blockIdx.x - C, nb);
#define VG_JS(L_, CPL_)                                                                                   \
  jvp_src_body<L_, CPL_, true>(lb, nb, d.csc_ptr, d.csc_slot, d.csc_dst, d.N, d.C, d.h, d.u, d.g_out,      \
                               d.att_src, d.att_dst, d.e_gz, d.e_gzp, d.e_alp, d.n_gad, d.h_inj, d.part)
  switch (d.shape) {
    case 0: VG_JS(8, 1); break;
    case 1: VG_JS(8, 2); break;
    case 2: VG_JS(8, 4); break;
    case 3: VG_JS(16, 4); break;
    case 4: VG_JS(16, 8); break;
    default: VG_JS(32, 8); break;
  }
#undef VG_JS
}

inline int jvp_shape_id(int C, const Shape& sh) {
  if (C <= 8) return 0;
  if (!sh.vec) return -1;
  if (sh.L == 8) return sh.CPL == 2 ? 1 : 2;
  if (sh.L == 16) return sh.CPL == 4 ? 3 : 4;
  return 5;
}

// g_a[c] += sum_b part_a[b][c] (blockIdx.y == 0), g_b[c] += sum_b part_b[b][c] (== 1)
__global__ void __launch_bounds__(1024) k_fold_add2(const float* __restrict__ part_a, int rows_a,
                                                    const float* __restrict__ part_b, int rows_b,
                                                    int C, float* __restrict__ g_a,
                                                    float* __restrict__ g_b) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const float* part = blockIdx.y == 0 ? part_a : part_b;
  const int rows = blockIdx.y == 0 ? rows_a : rows_b;
  float s = 0.f;
  if (c < C) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // loads in flight, fixed combine order
    int r = wave;
    for (; r + 48 < rows; r += 64) {
      a0 += part[(size_t)r * C + c];
      a1 += part[(size_t)(r + 16) * C + c];
      a2 += part[(size_t)(r + 32) * C + c];
      a3 += part[(size_t)(r + 48) * C + c];
    }
    for (; r < rows; r += 16) a0 += part[(size_t)r * C + c];
    s = (a0 + a1) + (a2 + a3);
  }
  __shared__ float red[16][64];
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0 && c < C) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += red[k][lane];
    float* o = blockIdx.y == 0 ? g_a : g_b;
    o[c] += v;
  }
}

inline bool jvp_shape(int C, Shape& sh) {
  if (C <= 0) return false;
  if (C <= 8) {
    sh = {8, 1, true};
    return true;
  }
  return pick_fused_shape(C, sh);
}

#define VG_DISPATCH_JVP(C, KERNEL_CALL)                                                           \
  do {                                                                                            \
    if ((C) <= 8) { constexpr int L_ = 8, CPL_ = 1; constexpr bool V_ = true; KERNEL_CALL; }      \
    else VG_DISPATCH_FUSED(C, KERNEL_CALL);                                                       \
  } while (0)

}  // namespace

extern "C" int64_t vg_gat_jvp2_ws_floats(int32_t num_nodes, int32_t num_edges, int32_t channels) {
  // e_u, e_h, e_gz, e_gzp, e_alp [E'] + up_src, up_dst, n_gad [N] + 2 partial blocks
  return 5 * (int64_t)num_edges + 3 * (int64_t)num_nodes + 2 * (int64_t)kMaxBlocks * channels;
}

extern "C" int vg_gat_jvp2(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                           const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E,
                           int32_t C, const float* h, const float* u, const float* g_out,
                           const float* att_src, const float* att_dst, const float* a_src,
                           const float* a_dst, const float* alpha, float slope, float* u_out,
                           float* h_inj, float* g_att_src, float* g_att_dst, float* workspace,
                           void* stream) {
  return vg_gat_jvp2_ex(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, u, g_out, att_src,
                        att_dst, a_src, a_dst, alpha, slope, u_out, h_inj, g_att_src, g_att_dst,
                        nullptr, nullptr, workspace, stream);
}

extern "C" int vg_gat_jvp2_ex(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                              const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E,
                              int32_t C, const float* h, const float* u, const float* g_out,
                              const float* att_src, const float* att_dst, const float* a_src,
                              const float* a_dst, const float* alpha, float slope, float* u_out,
                              float* h_inj, float* g_att_src, float* g_att_dst,
                              const float* up_src_in, const float* up_dst_in, float* workspace,
                              void* stream) {
  return vg_gat_jvp2_deferred(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, u, g_out,
                              att_src, att_dst, a_src, a_dst, alpha, slope, u_out, h_inj, g_att_src,
                              g_att_dst, up_src_in, up_dst_in, workspace, nullptr, nullptr, stream);
}

// folds_out == NULL: fold immediately (vg_gat_jvp2_ex); else describe the two
// accumulating folds for vg_fold_batch.
static int jvp2(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr, const int32_t* csc_slot,
                const int32_t* csc_dst, int32_t N, int32_t E, int32_t C, const float* h, const float* u,
                const float* g_out, const float* att_src, const float* att_dst, const float* a_src,
                const float* a_dst, const float* alpha, float slope, float* u_out, float* h_inj,
                float* g_att_src, float* g_att_dst, const float* up_src_in, const float* up_dst_in,
                float* workspace, vg_fold* folds_out, int32_t* n_out, vg_jvp_src* src_out, void* stream,
                const vg_gn_jvp* gn = nullptr);

extern "C" int32_t vg_gat_jvp2_blocks(int32_t N, int32_t C) {
  Shape sh;
  if (N <= 0 || !jvp_shape(C, sh)) return 0;
  const int grid = grid_for(N, sh.L);
  return grid > kMaxBlocks ? kMaxBlocks : grid;
}

extern "C" int vg_gat_jvp2_gn_deferred(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                                       const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E,
                                       int32_t C, const float* h, const float* u, const float* g_out,
                                       const float* att_src, const float* att_dst, const float* a_src,
                                       const float* a_dst, const float* alpha, float slope, float* u_out,
                                       float* h_inj, float* g_att_src, float* g_att_dst, const float* up_src_in,
                                       const float* up_dst_in, float* workspace, const vg_gn_jvp* gn,
                                       vg_fold* folds_out, int32_t* n_out, void* stream) {
  if (!gn || !folds_out || !n_out) return VG_EINVAL;
  return jvp2(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, u, g_out, att_src, att_dst, a_src, a_dst,
              alpha, slope, u_out, h_inj, g_att_src, g_att_dst, up_src_in, up_dst_in, workspace, folds_out, n_out,
              nullptr, stream, gn);
}

extern "C" int vg_gat_jvp2_deferred(const int32_t* row_ptr, const int32_t* col,
                                    const int32_t* csc_ptr, const int32_t* csc_slot,
                                    const int32_t* csc_dst, int32_t N, int32_t E, int32_t C,
                                    const float* h, const float* u, const float* g_out,
                                    const float* att_src, const float* att_dst, const float* a_src,
                                    const float* a_dst, const float* alpha, float slope,
                                    float* u_out, float* h_inj, float* g_att_src, float* g_att_dst,
                                    const float* up_src_in, const float* up_dst_in,
                                    float* workspace, vg_fold* folds_out, int32_t* n_out,
                                    void* stream) {
  return jvp2(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, u, g_out, att_src, att_dst, a_src, a_dst,
              alpha, slope, u_out, h_inj, g_att_src, g_att_dst, up_src_in, up_dst_in, workspace, folds_out, n_out,
              nullptr, stream);
}

extern "C" int vg_gat_jvp2_plan(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                                const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t E, int32_t C,
                                const float* h, const float* u, const float* g_out, const float* att_src,
                                const float* att_dst, const float* a_src, const float* a_dst, const float* alpha,
                                float slope, float* u_out, float* h_inj, float* g_att_src, float* g_att_dst,
                                const float* up_src_in, const float* up_dst_in, float* workspace,
                                vg_fold* folds_out, int32_t* n_out, vg_jvp_src* src_out, void* stream) {
  if (!folds_out || !n_out || !src_out) return VG_EINVAL;
  return jvp2(row_ptr, col, csc_ptr, csc_slot, csc_dst, N, E, C, h, u, g_out, att_src, att_dst, a_src, a_dst,
              alpha, slope, u_out, h_inj, g_att_src, g_att_dst, up_src_in, up_dst_in, workspace, folds_out, n_out,
              src_out, stream);
}

extern "C" int vg_gat_jvp_src_group(const vg_jvp_src* items, int32_t n, void* stream) {
  if (n < 0 || n > VG_JVP_GROUP_MAX || (n > 0 && !items)) return VG_EINVAL;
  if (n == 0) return 0;
  JvpSrcGroup g{};
  long long blocks = 0;
  for (int i = 0; i < n; ++i) {
    const vg_jvp_src& d = items[i];
    if (d.shape < 0 || d.shape > 5 || d.blocks <= 0 || d.blocks > kMaxBlocks || d.N <= 0 || d.C <= 0 || !d.csc_ptr ||
        !d.csc_slot || !d.csc_dst || !d.h || !d.u || !d.g_out || !d.att_src || !d.att_dst || !d.e_gz || !d.e_gzp ||
        !d.e_alp || !d.n_gad || !d.h_inj || !d.part)
      return VG_EINVAL;
    g.d[i] = d;
    g.block0[i] = static_cast<int>(blocks);
    blocks += d.blocks;
  }
  g.block0[n] = static_cast<int>(blocks);
  g.n = n;
  k_jvp_src_group<<<static_cast<int>(blocks), kBlock, 0, static_cast<hipStream_t>(stream)>>>(g);
  VG_CHECK_LAUNCH();
  return 0;
}

static int jvp2(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr, const int32_t* csc_slot,
                const int32_t* csc_dst, int32_t N, int32_t E, int32_t C, const float* h, const float* u,
                const float* g_out, const float* att_src, const float* att_dst, const float* a_src,
                const float* a_dst, const float* alpha, float slope, float* u_out, float* h_inj,
                float* g_att_src, float* g_att_dst, const float* up_src_in, const float* up_dst_in,
                float* workspace, vg_fold* folds_out, int32_t* n_out, vg_jvp_src* src_out, void* stream,
                const vg_gn_jvp* gn) {
  if ((folds_out == nullptr) != (n_out == nullptr)) return VG_EINVAL;
  if (gn && (!gn->x || !gn->g_y || !gn->stats || !gn->weight || !gn->bias || !gn->mean_scale || !gn->part))
    return VG_EINVAL;
  if (n_out) *n_out = 0;
  Shape sh;
  if (N <= 0 || E <= 0 || !row_ptr || !col || !csc_ptr || !csc_slot || !csc_dst || !h || !u ||
      !g_out || !att_src || !att_dst || !a_src || !a_dst || !alpha || !u_out || !h_inj ||
      !g_att_src || !g_att_dst || !workspace || !jvp_shape(C, sh))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* e_u = workspace;
  float* e_h = e_u + E;
  float* e_gz = e_h + E;
  float* e_gzp = e_gz + E;
  float* e_alp = e_gzp + E;
  float* up_src_ws = e_alp + E;
  float* up_dst_ws = up_src_ws + N;
  float* n_gad = up_dst_ws + N;
  float* part_r = n_gad + N;
  float* part_s = part_r + (size_t)kMaxBlocks * C;
  int grid = grid_for(N, sh.L);
  if (grid > kMaxBlocks) grid = kMaxBlocks;
  if ((up_src_in == nullptr) != (up_dst_in == nullptr)) return VG_EINVAL;
  const float* up_src = up_src_in ? up_src_in : up_src_ws;
  const float* up_dst = up_dst_in ? up_dst_in : up_dst_ws;
  if (!up_src_in)  // tangent projections not supplied by the tangent GEMM's epilogue
    VG_DISPATCH_JVP(C, (k_jvp_att<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                           u, N, C, att_src, att_dst, up_src_ws, up_dst_ws)));
  if (gn) {
    const GnJvp gj{gn->x, gn->keep, gn->g_y, gn->stats, gn->weight, gn->bias, gn->mean_scale, gn->eps, gn->part};
    VG_DISPATCH_JVP(C, (k_jvp_rows<L_, CPL_, V_, true><<<grid, kBlock, 0, s>>>(
                           row_ptr, col, N, C, h, u, g_out, a_src, a_dst, up_src, up_dst, alpha,
                           slope, u_out, e_u, e_h, e_gz, e_gzp, e_alp, n_gad, part_r, gj)));
  } else {
    VG_DISPATCH_JVP(C, (k_jvp_rows<L_, CPL_, V_><<<grid, kBlock, 0, s>>>(
                           row_ptr, col, N, C, h, u, g_out, a_src, a_dst, up_src, up_dst, alpha,
                           slope, u_out, e_u, e_h, e_gz, e_gzp, e_alp, n_gad, part_r)));
  }
  const int shape_id = jvp_shape_id(C, sh);
  if (src_out && shape_id >= 0) {  // described for vg_gat_jvp_src_group
    *src_out = vg_jvp_src{csc_ptr, csc_slot, csc_dst, h, u, g_out, att_src, att_dst, e_gz, e_gzp, e_alp,
                          n_gad, h_inj, part_s, N, C, grid, shape_id};
  } else {
    if (src_out) src_out->shape = -1;  // ran here
    VG_DISPATCH_JVP(C, (k_jvp_src<L_, CPL_, V_><<<grid, kBlock, 0, s>>>(
                           csc_ptr, csc_slot, csc_dst, N, C, h, u, g_out, att_src, att_dst, e_gz,
                           e_gzp, e_alp, n_gad, h_inj, part_s)));
  }
  if (folds_out) {
    folds_out[0] = vg_fold{g_att_dst, C, C, C, 1, 1, {{part_r, grid, C}, {nullptr, 0, 0}}};
    folds_out[1] = vg_fold{g_att_src, C, C, C, 1, 1, {{part_s, grid, C}, {nullptr, 0, 0}}};
    *n_out = 2;
  } else {
    k_fold_add2<<<dim3(vg_blocks(C, 64), 2), 1024, 0, s>>>(part_r, grid, part_s, grid, C,
                                                           g_att_dst, g_att_src);
  }
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_jvp2_fold_src(int32_t N, int32_t C, const float* weight, const float* mean_scale,
                                          const float* stats, float* ws, float* g_w, float* g_ms,
                                          const vg_jvp_src* src, void* stream) {
  if (N <= 0 || C <= 0 || !weight || !mean_scale || !stats || !ws || !g_w || !g_ms) return VG_EINVAL;
  const bool with_src = src && src->shape >= 0;
  if (with_src && (src->shape > 5 || src->blocks <= 0 || src->blocks > kMaxBlocks || src->N <= 0 || src->C <= 0 ||
                   !src->csc_ptr || !src->csc_slot || !src->csc_dst || !src->h || !src->u || !src->g_out ||
                   !src->att_src || !src->att_dst || !src->e_gz || !src->e_gzp || !src->e_alp || !src->n_gad ||
                   !src->h_inj || !src->part))
    return VG_EINVAL;
  const int chunks = vg::gn_chunks_for(N);
  float* sums = ws + (size_t)vg::kGnChunks * C * 5;  // vg_graphnorm_jvp2's workspace layout
  const vg_jvp_src d = with_src ? *src : vg_jvp_src{};
  k_jvp2_fold_src<<<C + (with_src ? src->blocks : 0), kBlock, 0, static_cast<hipStream_t>(stream)>>>(
      ws, chunks, N, C, weight, mean_scale, stats, sums, g_w, g_ms, d);
  VG_CHECK_LAUNCH();
  return 0;
}
