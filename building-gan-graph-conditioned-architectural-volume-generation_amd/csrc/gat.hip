// Differentiable sparse primitives over the destination CSR / source CSC.
//
// These are the closed set whose adjoints are each other (spmm <-> spmm_t,
// sddmm, gather <-> seg_sum / scatter_src).  The WGAN-GP's create_graph=True
// backward through GATConv is written with them (vgan/ops.py), so every
// derivative order runs on these kernels.  Same row-group decomposition as the
// fused GAT kernels (rowgroup.h).
#include "rowgroup.h"

namespace {

using namespace vg;

// ---- generic weighted row aggregation (spmm / spmm_t) ---------------------
// Y[r] = sum_{p in [ptr[r], ptr[r+1])} w[slot(p)] * X[nbr[p]]
// spmm:   ptr = row_ptr, nbr = col,     slot = identity
// spmm_t: ptr = csc_ptr, nbr = csc_dst, slot = csc_slot
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_aggregate(const int32_t* __restrict__ ptr,
                                                      const int32_t* __restrict__ nbr,
                                                      const int32_t* __restrict__ slot, int N,
                                                      int C, const float* __restrict__ w,
                                                      const float* __restrict__ X,
                                                      float* __restrict__ Y) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int r = g.row;
  const int beg = ptr[r], end = ptr[r + 1];
  const int deg = end - beg;
  int n_own = 0;
  float w_own = 0.f;
  if (g.lane < deg) {
    const int p = beg + g.lane;
    n_own = nbr[p];
    w_own = w[slot ? slot[p] : p];
  }
  const int c0 = g.lane * CPL;
  Vec<CPL> acc;
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
  if (deg <= L) {
#pragma unroll 4
    for (int e = 0; e < deg; ++e) {
      const int n = __shfl(n_own, g.base + e, 64);
      const float a = __shfl(w_own, g.base + e, 64);
      Vec<CPL> xv;
      load_row<CPL, VEC>(xv, X + (size_t)n * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, xv.v[q], acc.v[q]);
    }
  } else {
    for (int p = beg; p < end; ++p) {
      const int n = nbr[p];
      const float a = w[slot ? slot[p] : p];
      Vec<CPL> xv;
      load_row<CPL, VEC>(xv, X + (size_t)n * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, xv.v[q], acc.v[q]);
    }
  }
  store_row<CPL, VEC>(acc, Y + (size_t)r * C, c0, C);
}

// e_k = <A[i], B[col_k]> for the slots k of destination row i
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_sddmm(const int32_t* __restrict__ row_ptr,
                                                  const int32_t* __restrict__ col, int N, int C,
                                                  const float* __restrict__ A,
                                                  const float* __restrict__ B,
                                                  float* __restrict__ e) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int i = g.row;
  const int beg = row_ptr[i], end = row_ptr[i + 1];
  const int c0 = g.lane * CPL;
  Vec<CPL> av;
  load_row<CPL, VEC>(av, A + (size_t)i * C, c0, C);
  for (int k = beg; k < end; ++k) {
    Vec<CPL> bv;
    load_row<CPL, VEC>(bv, B + (size_t)col[k] * C, c0, C);
    float part = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) part = fmaf(av.v[q], bv.v[q], part);
    part = group_sum<L>(part);
    if (g.lane == 0) e[k] = part;
  }
}

// ---- scalar segment helpers (thread per row; rows are short) --------------
__global__ void k_seg_sum(const int32_t* __restrict__ ptr, const int32_t* __restrict__ slot, int N,
                          const float* __restrict__ x, float* __restrict__ s) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  float acc = 0.f;
  for (int p = ptr[r]; p < ptr[r + 1]; ++p) acc += x[slot ? slot[p] : p];
  s[r] = acc;
}

__global__ void k_seg_max(const int32_t* __restrict__ ptr, int N, const float* __restrict__ x,
                          float* __restrict__ m) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  float acc = -INFINITY;
  for (int p = ptr[r]; p < ptr[r + 1]; ++p) acc = fmaxf(acc, x[p]);
  m[r] = acc;
}

__global__ void k_gather(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
                         int N, int by_src, const float* __restrict__ v, float* __restrict__ e) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const float vi = by_src ? 0.f : v[i];
  for (int k = row_ptr[i]; k < row_ptr[i + 1]; ++k) e[k] = by_src ? v[col[k]] : vi;
}

}  // namespace

extern "C" int vg_spmm(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                       const float* w, const float* x, float* y, void* stream) {
  if (N <= 0 || !row_ptr || !col || !w || !x || !y) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  VG_DISPATCH(C, (k_aggregate<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                     row_ptr, col, nullptr, N, C, w, x, y)));
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_spmm_t(const int32_t* csc_ptr, const int32_t* csc_slot, const int32_t* csc_dst,
                         int32_t N, int32_t C, const float* w, const float* g, float* z,
                         void* stream) {
  if (N <= 0 || !csc_ptr || !csc_slot || !csc_dst || !w || !g || !z) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  VG_DISPATCH(C, (k_aggregate<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                     csc_ptr, csc_dst, csc_slot, N, C, w, g, z)));
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_sddmm(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                        const float* a, const float* b, float* e, void* stream) {
  if (N <= 0 || !row_ptr || !col || !a || !b || !e) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  VG_DISPATCH(C, (k_sddmm<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(row_ptr, col, N, C, a,
                                                                            b, e)));
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_seg_sum(const int32_t* row_ptr, int32_t N, const float* x, float* out,
                          void* stream) {
  if (N <= 0 || !row_ptr || !x || !out) return VG_EINVAL;
  k_seg_sum<<<vg_blocks(N, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, nullptr, N,
                                                                              x, out);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_seg_max(const int32_t* row_ptr, int32_t N, const float* x, float* out,
                          void* stream) {
  if (N <= 0 || !row_ptr || !x || !out) return VG_EINVAL;
  k_seg_max<<<vg_blocks(N, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, N, x, out);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gather(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t by_src,
                         const float* v, float* e, void* stream) {
  if (N <= 0 || !row_ptr || !col || !v || !e) return VG_EINVAL;
  k_gather<<<vg_blocks(N, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, col, N,
                                                                             by_src, v, e);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_scatter_src(const int32_t* csc_ptr, const int32_t* csc_slot, int32_t N,
                              const float* x, float* out, void* stream) {
  if (N <= 0 || !csc_ptr || !csc_slot || !x || !out) return VG_EINVAL;
  k_seg_sum<<<vg_blocks(N, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(csc_ptr, csc_slot,
                                                                              N, x, out);
  VG_CHECK_LAUNCH();
  return 0;
}
