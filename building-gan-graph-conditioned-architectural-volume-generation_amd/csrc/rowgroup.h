// Row-group helpers shared by the message-passing kernels (wave64).
//
// A ROW (destination node of the CSR, or source node of the CSC) is owned by a
// group of L contiguous lanes (L = 8/16/32/64); each lane owns CPL contiguous
// channels and moves them with one vector load (VEC) when the row stride and
// base pointer allow it.
#pragma once
#include "common.h"

namespace vg {

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
      if constexpr (CPL == 8) {  // VEC with CPL 8 requires C % 8 == 0 (pick_fused_shape)
        const float4 t = *reinterpret_cast<const float4*>(base + c0);
        const float4 u = *reinterpret_cast<const float4*>(base + c0 + 4);
        r.v[0] = t.x; r.v[1] = t.y; r.v[2] = t.z; r.v[3] = t.w;
        r.v[4] = u.x; r.v[5] = u.y; r.v[6] = u.z; r.v[7] = u.w;
      } else if constexpr (CPL == 4) {
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
      if constexpr (CPL == 8) {
        *reinterpret_cast<float4*>(base + c0) = make_float4(r.v[0], r.v[1], r.v[2], r.v[3]);
        *reinterpret_cast<float4*>(base + c0 + 4) = make_float4(r.v[4], r.v[5], r.v[6], r.v[7]);
      } else if constexpr (CPL == 4) {
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


template <int CPL, bool VEC>
__device__ __forceinline__ float dot_row(const Vec<CPL>& a, const Vec<CPL>& b) {
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) s = fmaf(a.v[q], b.v[q], s);
  return s;
}

// ---- shape dispatch -------------------------------------------------------
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
    ::vg::Shape sh;                                                    \
    if (!::vg::pick_shape(C, sh)) return VG_EINVAL;                    \
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

// Shapes of the fused GAT kernels: narrow lane groups with wide per-lane
// vectors, so a wave keeps 4-8 destination rows (and their independent
// latency chains) in flight and the per-edge group reductions are short.
//   C in  9..16 : L  8 x 2      17..32 : L  8 x 4      33..64 : L 16 x 4
//        65..128: L 16 x 8     129..256: L 32 x 8
inline bool pick_fused_shape(int C, Shape& sh) {
  if (C <= 8 || C > 256) return false;
  if (C <= 16) sh = {8, 2, (C % 2) == 0};
  else if (C <= 32) sh = {8, 4, (C % 4) == 0};
  else if (C <= 64) sh = {16, 4, (C % 4) == 0};
  else if (C <= 128) sh = {16, 8, (C % 8) == 0};
  else sh = {32, 8, (C % 8) == 0};
  return true;
}

#define VG_DISPATCH_FUSED(C, KERNEL_CALL)                                                        \
  do {                                                                                           \
    ::vg::Shape sh;                                                                              \
    if (!::vg::pick_fused_shape(C, sh)) return VG_EINVAL;                                        \
    if (sh.L == 8 && sh.CPL == 2) {                                                              \
      if (sh.vec) { constexpr int L_ = 8, CPL_ = 2; constexpr bool V_ = true; KERNEL_CALL; }     \
      else { constexpr int L_ = 8, CPL_ = 2; constexpr bool V_ = false; KERNEL_CALL; }           \
    } else if (sh.L == 8) {                                                                      \
      if (sh.vec) { constexpr int L_ = 8, CPL_ = 4; constexpr bool V_ = true; KERNEL_CALL; }     \
      else { constexpr int L_ = 8, CPL_ = 4; constexpr bool V_ = false; KERNEL_CALL; }           \
    } else if (sh.L == 16 && sh.CPL == 4) {                                                      \
      if (sh.vec) { constexpr int L_ = 16, CPL_ = 4; constexpr bool V_ = true; KERNEL_CALL; }    \
      else { constexpr int L_ = 16, CPL_ = 4; constexpr bool V_ = false; KERNEL_CALL; }          \
    } else if (sh.L == 16) {                                                                     \
      if (sh.vec) { constexpr int L_ = 16, CPL_ = 8; constexpr bool V_ = true; KERNEL_CALL; }    \
      else { constexpr int L_ = 16, CPL_ = 8; constexpr bool V_ = false; KERNEL_CALL; }          \
    } else {                                                                                     \
      if (sh.vec) { constexpr int L_ = 32, CPL_ = 8; constexpr bool V_ = true; KERNEL_CALL; }    \
      else { constexpr int L_ = 32, CPL_ = 8; constexpr bool V_ = false; KERNEL_CALL; }          \
    }                                                                                            \
  } while (0)

// ---- block partials ---------------------------------------------------------
// Every group accumulates per-channel partials in registers over the rows it
// visits (grid-stride); the block folds its groups through LDS and writes one
// row of `part` ([gridDim.x][W]).  W <= 3 * 256.
// The LDS image of block_partials: ONE buffer per kernel, whatever row shapes
// the kernel instantiates (a static __shared__ array inside the template gave
// every instantiation its own 16 KB: the grouped / merged source passes, which
// switch over six shapes, took 96 KB of LDS and ran one workgroup per CU).
__device__ __forceinline__ float* block_partials_lds() {
  __shared__ float red[kBlock * 8 * 2];  // (256/L) groups x L*CPL channels (CPL <= 8) x up to 2 vectors
  return red;
}

template <int L, int CPL>
__device__ void block_partials(const Vec<CPL>* vals, int nvec, int C, float* __restrict__ part,
                               int bid = -1) {
  if (bid < 0) bid = blockIdx.x;  // the partial row (grouped launches pass their own block index)
  constexpr int G = kBlock / L;
  float* red = block_partials_lds();
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  const int Wg = L * CPL;
  for (int v = 0; v < nvec; ++v)
#pragma unroll
    for (int q = 0; q < CPL; ++q) red[(grp * nvec + v) * Wg + lane * CPL + q] = vals[v].v[q];
  __syncthreads();
  for (int w = threadIdx.x; w < nvec * Wg; w += kBlock) {
    const int v = w / Wg, c = w % Wg;
    float s = 0.f;
    for (int k = 0; k < G; ++k) s += red[(k * nvec + v) * Wg + c];
    if (c < C) part[(size_t)bid * nvec * C + v * C + c] = s;
  }
}

// GraphNorm column partials of the rows a workgroup aggregated: the forward
// statistics of the GraphNorm that follows every GATConv (models.py:73-75,
// 193-195; graphnorm.hip's k_stats_partial re-read the whole output for them).
// Per column (count, mean, M2) of the block's rows.  Each wave takes its own
// rows' two-pass statistics from the values still in registers (sum by
// xor-shuffles across the wave's L-lane row groups -- every lane ends with the
// total -- the wave mean, then the squared deviations the same way); the four
// waves' (count, mean, M2) meet in LDS behind ONE barrier and are merged in
// wave order with Chan's formula (deterministic).  (The first form took the
// block's two passes through LDS: three barriers, ~1 us per launch more.)
// Blocks are SEGMENT-ALIGNED (gnp_rows): a stacked forward over S copies
// (seg_rows rows each) gives every copy ceil(seg_rows / G) blocks of its own,
// the last one short, so each copy's partials -- and the statistics folded
// from them -- are bit for bit those of a separate forward over that copy.
// (Blocks dealt over the stacked rows straddled copies at offsets that
// depended on the copy: the critic engine's stacked real / fake / mix forward
// then normalised with statistics ~1e-7 off the three separate forwards of
// autograd's double backward, enough to flip bf16 operand roundings.)
// gnp [blocks][2][ldc][3], column cb + c, slot 0 (slot 1 unused).  v: this
// lane's CPL columns c0.. of its row (lanes past C hold anything: their
// columns are not written).
// (A first form folded each column serially over the block's rows with
// Welford updates in one wave: +4 us per launch, slower than the separate
// statistics pass it replaced.)
struct GnpRows {
  int lb, row0, end;  // logical block, its first row, the end of its segment
};

template <int G>
__device__ __forceinline__ GnpRows gnp_rows(int seg_rows) {
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int bps = (seg_rows + G - 1) / G;
  const int seg = lb / bps;
  return {lb, seg * seg_rows + (lb - seg * bps) * G, (seg + 1) * seg_rows};
}

template <int L, int CPL>
__device__ __forceinline__ void gnp_block(const float (&v)[CPL], int row, const GnpRows& gr, int C, int c0,
                                          int cb, int ldc, float* __restrict__ gnp) {
  constexpr int W = L * CPL, RW = 64 / L, NW = kBlock / 64;  // columns, rows per wave, waves
  __shared__ float red[NW][2][W];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool in0 = row < gr.end;
  const int nw = max(0, min(RW, gr.end - (gr.row0 + wave * RW)));  // this wave's rows in the segment
  const float inv = nw > 0 ? 1.f / static_cast<float>(nw) : 0.f;
  float s[CPL], mean[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) s[q] = in0 ? v[q] : 0.f;
#pragma unroll
  for (int off = L; off < 64; off <<= 1)
#pragma unroll
    for (int q = 0; q < CPL; ++q) s[q] += __shfl_xor(s[q], off, 64);
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    mean[q] = s[q] * inv;
    const float d = in0 ? v[q] - mean[q] : 0.f;
    s[q] = d * d;
  }
#pragma unroll
  for (int off = L; off < 64; off <<= 1)
#pragma unroll
    for (int q = 0; q < CPL; ++q) s[q] += __shfl_xor(s[q], off, 64);
  if (lane < L)
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      red[wave][0][c0 + q] = mean[q];
      red[wave][1][c0 + q] = s[q];
    }
  __syncthreads();
  const int c = threadIdx.x;
  if (c < C) {
    const int n_blk = min(gr.end, gr.row0 + kBlock / L) - gr.row0;
    float n = static_cast<float>(min(RW, n_blk)), mu = red[0][0][c], m2 = red[0][1][c];
#pragma unroll
    for (int w = 1; w < NW; ++w) {  // Chan's merge, wave order
      const int k = min(RW, n_blk - w * RW);
      if (k <= 0) break;
      const float nb = static_cast<float>(k), nt = n + nb;
      const float delta = red[w][0][c] - mu, fb = nb / nt;
      mu += delta * fb;
      m2 += red[w][1][c] + delta * delta * n * fb;
      n = nt;
    }
    float* p = gnp + ((size_t)gr.lb * 2 * ldc + cb + c) * 3;
    p[0] = n;
    p[1] = mu;
    p[2] = m2;
  }
}

}  // namespace vg
