// GATConv (heads = 1) message passing over the destination CSR.
//
// Work decomposition (wave64): a destination row is owned by a GROUP of L
// contiguous lanes (L = 8/16/32/64, the smallest power of two >= min(C, 64),
// at least 8), so one wave serves 64/L rows at once and no lane is wasted on the
// tiny-width layers of the generator (C = 1..8).  Each lane owns CPL contiguous
// channels (C <= L*CPL, CPL in {1,2,4}) and loads them with one vector load,
// so a C = 128 fp32 row is one coalesced 512-B access.
//
// Per row, the incoming edges are first processed edge-parallel across the L
// lanes (logit, max, exp-sum: the segmented scatter-max/scatter-add of
// utils/_softmax.py done as in-register group reductions, no atomics), then
// channel-parallel: edge j's source index and weight are broadcast from the
// lane that owns it and every lane accumulates alpha_j * h[src_j] for its
// channels.  Rows are never split across groups, so sums are deterministic.
#include "common.h"

namespace {

constexpr int kBlock = 256;
constexpr float kSoftmaxEps = 1e-16f;

// ---- vector helpers over CPL contiguous floats --------------------------
template <int CPL>
struct Vec {
  float v[CPL];
};

template <int CPL, bool VEC>
__device__ __forceinline__ void load_row(Vec<CPL>& r, const float* __restrict__ base, int c0, int C) {
  if (VEC) {
    if (c0 < C) {
      if constexpr (CPL == 4) {
        const float4 t = *reinterpret_cast<const float4*>(base + c0);
        r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
      } else if constexpr (CPL == 2) {
        const float2 t = *reinterpret_cast<const float2*>(base + c0);
        r.v[0] = t.x; r.v[1] = t.y;
      } else {
        r.v[0] = base[c0];
      }
    } else {
#pragma unroll
      for (int q = 0; q < CPL; ++q) r.v[q] = 0.f;
    }
  } else {
#pragma unroll
    for (int q = 0; q < CPL; ++q) r.v[q] = (c0 + q < C) ? base[c0 + q] : 0.f;
  }
}

template <int CPL, bool VEC>
__device__ __forceinline__ void store_row(const Vec<CPL>& r, float* __restrict__ base, int c0, int C) {
  if (VEC) {
    if (c0 < C) {
      if constexpr (CPL == 4) {
        *reinterpret_cast<float4*>(base + c0) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
      } else if constexpr (CPL == 2) {
        *reinterpret_cast<float2*>(base + c0) = make_float2(r.v[0], r.v[1]);
      } else {
        base[c0] = r.v[0];
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < CPL; ++q)
      if (c0 + q < C) base[c0 + q] = r.v[q];
  }
}

struct GroupIdx {
  int row;   // logical row (destination or source node) owned by the group
  int lane;  // lane inside the group
  int base;  // wave lane id of the group's lane 0
};

template <int L>
__device__ __forceinline__ GroupIdx group_index() {
  constexpr int groups_per_block = kBlock / L;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  GroupIdx g;
  g.row = lb * groups_per_block + threadIdx.x / L;
  g.lane = threadIdx.x & (L - 1);
  g.base = (threadIdx.x & 63) & ~(L - 1);
  return g;
}

// ---- fused forward --------------------------------------------------------
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_gat_fwd(const int32_t* __restrict__ row_ptr,
                                                    const int32_t* __restrict__ col, int N, int C,
                                                    const float* __restrict__ h,
                                                    const float* __restrict__ a_src,
                                                    const float* __restrict__ a_dst,
                                                    const float* __restrict__ bias, float slope,
                                                    float* __restrict__ out,
                                                    float* __restrict__ alpha) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int i = g.row;
  const int beg = row_ptr[i], end = row_ptr[i + 1];
  const int deg = end - beg;
  const float ad = a_dst[i];

  // edge-parallel: logits and segment max (utils/_softmax.py: scatter 'max')
  float m = -INFINITY;
  int s_own = 0;
  float e_own = -INFINITY;
  for (int k = beg + g.lane; k < end; k += L) {
    const int s = col[k];
    const float e = lrelu(a_src[s] + ad, slope);
    if (k == beg + g.lane) {
      s_own = s;
      e_own = e;
    }
    m = fmaxf(m, e);
  }
  m = group_max<L>(m);
  // segment sum of exp(e - max) (scatter 'sum') + 1e-16
  float ssum = 0.f;
  for (int k = beg + g.lane; k < end; k += L) {
    const float e = (k == beg + g.lane) ? e_own : lrelu(a_src[col[k]] + ad, slope);
    ssum += expf(e - m);
  }
  const float denom = group_sum<L>(ssum) + kSoftmaxEps;
  float a_own = 0.f;
  for (int k = beg + g.lane; k < end; k += L) {
    const float e = (k == beg + g.lane) ? e_own : lrelu(a_src[col[k]] + ad, slope);
    const float a = expf(e - m) / denom;
    if (k == beg + g.lane) a_own = a;
    if (alpha) alpha[k] = a;
  }

  // channel-parallel aggregation: out_i = sum_j alpha_j h[src_j] + bias
  const int c0 = g.lane * CPL;
  Vec<CPL> acc;
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
  if (deg <= L) {
#pragma unroll 4
    for (int j = 0; j < deg; ++j) {
      const int s = __shfl(s_own, g.base + j, 64);
      const float a = __shfl(a_own, g.base + j, 64);
      Vec<CPL> hv;
      load_row<CPL, VEC>(hv, h + (size_t)s * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, hv.v[q], acc.v[q]);
    }
  } else {
    for (int k = beg; k < end; ++k) {
      const int s = col[k];
      const float a = expf(lrelu(a_src[s] + ad, slope) - m) / denom;
      Vec<CPL> hv;
      load_row<CPL, VEC>(hv, h + (size_t)s * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, hv.v[q], acc.v[q]);
    }
  }
  if (bias) {
    Vec<CPL> b;
    load_row<CPL, false>(b, bias, c0, C);
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc.v[q] += b.v[q];
  }
  store_row<CPL, VEC>(acc, out + (size_t)i * C, c0, C);
}

// ---- fused first-order backward, pass 1 (destination rows) ---------------
//   ga_k  = <g_out[i], h[src_k]>                (d loss / d alpha_k)
//   t_i   = sum_k alpha_k ga_k
//   gp_k  = alpha_k (ga_k - t_i) * lrelu'(pre_k) (d loss / d pre-activation)
//   g_a_dst[i] = sum_k gp_k
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_rows(const int32_t* __restrict__ row_ptr,
                                                         const int32_t* __restrict__ col, int N,
                                                         int C, const float* __restrict__ h,
                                                         const float* __restrict__ a_src,
                                                         const float* __restrict__ a_dst,
                                                         const float* __restrict__ alpha,
                                                         const float* __restrict__ g_out,
                                                         float slope, float* __restrict__ g_pre,
                                                         float* __restrict__ g_a_dst) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int i = g.row;
  const int beg = row_ptr[i], end = row_ptr[i + 1];
  const int deg = end - beg;
  const int c0 = g.lane * CPL;
  Vec<CPL> go;
  load_row<CPL, VEC>(go, g_out + (size_t)i * C, c0, C);

  // lane (j % L) keeps ga_j of edge j in slot j / L (up to 4 slots)
  float ga_slot[4] = {0.f, 0.f, 0.f, 0.f};
  float t = 0.f;
  for (int j = 0; j < deg; ++j) {
    const int k = beg + j;
    const int s = col[k];
    Vec<CPL> hv;
    load_row<CPL, VEC>(hv, h + (size_t)s * C, c0, C);
    float part = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) part = fmaf(go.v[q], hv.v[q], part);
    const float ga = group_sum<L>(part);
    t = fmaf(alpha[k], ga, t);
    const int slot = j / L;
    if (g.lane == (j & (L - 1))) {
      if (slot == 0) ga_slot[0] = ga;
      else if (slot == 1) ga_slot[1] = ga;
      else if (slot == 2) ga_slot[2] = ga;
      else if (slot == 3) ga_slot[3] = ga;
    }
  }
  const float ad = a_dst[i];
  float gad = 0.f;
#pragma unroll
  for (int slot = 0; slot < 4; ++slot) {
    const int j = slot * L + g.lane;
    if (j < deg) {
      const int k = beg + j;
      const float pre = a_src[col[k]] + ad;
      const float gp = alpha[k] * (ga_slot[slot] - t) * (pre > 0.f ? 1.f : slope);
      g_pre[k] = gp;
      gad += gp;
    }
  }
  // rows longer than 4L: recompute ga for the remaining edges
  for (int j = 4 * L; j < deg; ++j) {
    const int k = beg + j;
    const int s = col[k];
    Vec<CPL> hv;
    load_row<CPL, VEC>(hv, h + (size_t)s * C, c0, C);
    float part = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) part = fmaf(go.v[q], hv.v[q], part);
    const float ga = group_sum<L>(part);
    if (g.lane == 0) {
      const float pre = a_src[s] + ad;
      const float gp = alpha[k] * (ga - t) * (pre > 0.f ? 1.f : slope);
      g_pre[k] = gp;
      gad += gp;
    }
  }
  gad = group_sum<L>(gad);
  if (g.lane == 0) g_a_dst[i] = gad;
}

// ---- pass 2 (source nodes, over the CSC) ----------------------------------
//   g_h[j]     = sum_{k: src_k = j} alpha_k g_out[dst_k]
//   g_a_src[j] = sum_{k: src_k = j} gp_k
template <int L, int CPL, bool VEC>
__global__ void __launch_bounds__(kBlock) k_gat_bwd_src(const int32_t* __restrict__ csc_ptr,
                                                        const int32_t* __restrict__ csc_slot,
                                                        const int32_t* __restrict__ csc_dst,
                                                        int N, int C,
                                                        const float* __restrict__ alpha,
                                                        const float* __restrict__ g_out,
                                                        const float* __restrict__ g_pre,
                                                        float* __restrict__ g_h,
                                                        float* __restrict__ g_a_src) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int j = g.row;
  const int beg = csc_ptr[j], end = csc_ptr[j + 1];
  const int deg = end - beg;
  int d_own = 0;
  float a_own = 0.f, gas = 0.f;
  for (int p = beg + g.lane; p < end; p += L) {
    const int k = csc_slot[p];
    if (p == beg + g.lane) {
      d_own = csc_dst[p];
      a_own = alpha[k];
    }
    gas += g_pre[k];
  }
  gas = group_sum<L>(gas);
  if (g.lane == 0) g_a_src[j] = gas;
  const int c0 = g.lane * CPL;
  Vec<CPL> acc;
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
  if (deg <= L) {
#pragma unroll 4
    for (int e = 0; e < deg; ++e) {
      const int d = __shfl(d_own, g.base + e, 64);
      const float a = __shfl(a_own, g.base + e, 64);
      Vec<CPL> gv;
      load_row<CPL, VEC>(gv, g_out + (size_t)d * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, gv.v[q], acc.v[q]);
    }
  } else {
    for (int p = beg; p < end; ++p) {
      const int d = csc_dst[p];
      const float a = alpha[csc_slot[p]];
      Vec<CPL> gv;
      load_row<CPL, VEC>(gv, g_out + (size_t)d * C, c0, C);
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, gv.v[q], acc.v[q]);
    }
  }
  store_row<CPL, VEC>(acc, g_h + (size_t)j * C, c0, C);
}

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

// ---- dispatch ---------------------------------------------------------------
struct Shape {
  int L, CPL;
  bool vec;
};

inline bool pick_shape(int C, Shape& sh) {
  if (C <= 0) return false;
  if (C <= 8) sh = {8, 1, true};
  else if (C <= 16) sh = {16, 1, true};
  else if (C <= 32) sh = {32, 1, true};
  else if (C <= 64) sh = {64, 1, true};
  else if (C <= 128) sh = {64, 2, (C % 2) == 0};
  else if (C <= 256) sh = {64, 4, (C % 4) == 0};
  else return false;
  return true;
}

#define VG_DISPATCH(C, KERNEL_CALL)                                    \
  do {                                                                 \
    Shape sh;                                                          \
    if (!pick_shape(C, sh)) return VG_EINVAL;                          \
    if (sh.L == 8) { constexpr int L_ = 8, CPL_ = 1; constexpr bool V_ = true; KERNEL_CALL; } \
    else if (sh.L == 16) { constexpr int L_ = 16, CPL_ = 1; constexpr bool V_ = true; KERNEL_CALL; } \
    else if (sh.L == 32) { constexpr int L_ = 32, CPL_ = 1; constexpr bool V_ = true; KERNEL_CALL; } \
    else if (sh.CPL == 1) { constexpr int L_ = 64, CPL_ = 1; constexpr bool V_ = true; KERNEL_CALL; } \
    else if (sh.CPL == 2 && sh.vec) { constexpr int L_ = 64, CPL_ = 2; constexpr bool V_ = true; KERNEL_CALL; } \
    else if (sh.CPL == 2) { constexpr int L_ = 64, CPL_ = 2; constexpr bool V_ = false; KERNEL_CALL; } \
    else if (sh.vec) { constexpr int L_ = 64, CPL_ = 4; constexpr bool V_ = true; KERNEL_CALL; } \
    else { constexpr int L_ = 64, CPL_ = 4; constexpr bool V_ = false; KERNEL_CALL; } \
  } while (0)

inline int grid_for(int N, int L) { return vg_blocks(N, kBlock / L); }

}  // namespace

extern "C" int vg_gat_fwd(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                          const float* h, const float* a_src, const float* a_dst,
                          const float* bias, float slope, float* out, float* alpha,
                          void* stream) {
  if (N <= 0 || !row_ptr || !col || !h || !a_src || !a_dst || !out) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  VG_DISPATCH(C, (k_gat_fwd<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                     row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha)));
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_bwd(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                          const int32_t* csc_slot, const int32_t* csc_dst, int32_t N, int32_t C,
                          const float* h, const float* a_src, const float* a_dst,
                          const float* alpha, const float* g_out, float slope, float* g_pre,
                          float* g_h, float* g_a_src, float* g_a_dst, void* stream) {
  if (N <= 0 || !row_ptr || !col || !csc_ptr || !csc_slot || !csc_dst || !h || !a_src ||
      !a_dst || !alpha || !g_out || !g_pre || !g_h || !g_a_src || !g_a_dst)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  VG_DISPATCH(C, (k_gat_bwd_rows<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                     row_ptr, col, N, C, h, a_src, a_dst, alpha, g_out, slope, g_pre, g_a_dst)));
  VG_DISPATCH(C, (k_gat_bwd_src<L_, CPL_, V_><<<grid_for(N, L_), kBlock, 0, s>>>(
                     csc_ptr, csc_slot, csc_dst, N, C, alpha, g_out, g_pre, g_h, g_a_src)));
  VG_CHECK_LAUNCH();
  return 0;
}

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
