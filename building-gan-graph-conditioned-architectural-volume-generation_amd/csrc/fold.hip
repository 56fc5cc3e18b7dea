// Deferred parameter-gradient folds: one launch for every split-K / per-block
// partial set of a whole backward.
//
// The weight-gradient GEMMs (vg_gemm_tn) and the GAT backward / second-order
// kernels (vg_gat_bwd_ex, vg_gat_jvp2_ex) reduce their parameter gradients in
// two steps: per-workgroup partial rows, then a fold launch over those rows.
// The folded values are needed only by the optimizer step, so the *_deferred
// entry points skip the fold and describe it instead (vg_fold: destination,
// shape, up to two partial sources); vg_fold_batch then runs every fold of a
// critic iteration or of the generator backward in ONE launch -- about 24
// launches fewer per critic iteration.  The descriptors travel by value in the
// kernel arguments (no host-to-device copy, capturable in a hipGraph).
//
// Summation order is fixed (deterministic): per source, 16 waves stride the
// partial rows with sixteen accumulators combined pairwise, the waves are added
// in order, and the destination becomes (out + source 0) + source 1.
#include "common.h"

namespace {

#ifndef VG_FOLD_SHORT_ROWS
#define VG_FOLD_SHORT_ROWS 256
#endif
constexpr int kShortRows = VG_FOLD_SHORT_ROWS;
#ifndef VG_FOLD_PACK
#define VG_FOLD_PACK 1  // narrow long folds with packed (row, column) lanes (0: the round-4 mapping, A/B)
#endif

struct FoldBatch {
  int32_t n;
  int32_t block0[VG_FOLD_MAX + 1];  // first workgroup of fold i; block0[n] = grid size
  int32_t waves[VG_FOLD_MAX];       // waves per 64-column group: 16, or 4 for short folds
  int32_t cw[VG_FOLD_MAX];          // narrow long folds: lanes per partial row (pow2 >= width, <= 32); else 0
  vg_fold f[VG_FOLD_MAX];
};

// Sixteen rows in flight per wave and iteration (the GAT / LayerNorm partial
// sets have up to a few thousand rows: a short dependent loop, not one round
// trip per four rows); fixed combination order.  `stride` = waves per column
// group.
__device__ __forceinline__ float fold_rows_sum(const float* __restrict__ part, int rows, int ld,
                                               long long w, int sub, int stride) {
  constexpr int U = 16;
  float a[U];
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = 0.f;
  int r = sub;
  for (; r + stride * (U - 1) < rows; r += stride * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] += part[(size_t)(r + stride * u) * ld + w];
  }
  for (; r < rows; r += stride) a[0] += part[(size_t)r * ld + w];
#pragma unroll
  for (int h = U / 2; h > 0; h >>= 1)
#pragma unroll
    for (int u = 0; u < h; ++u) a[u] += a[u + h];
  return a[0];
}

// Narrow long folds (width <= 32: the GAT parameter partials of the
// 1-32-channel layers, one partial row per 32-row workgroup of a 38k-row
// backward): the lanes of a wave are packed (row, column) -- 64 / cw rows per
// load instruction instead of one row on `width` of 64 lanes -- so a wave
// strides 16x fewer rows at C = 4 and the long pole of the fold launch takes
// fewer dependent round trips.  Rows sub, sub + stride, ... in registers, the
// row-sub lanes combined by a fixed xor tree: deterministic.
__device__ __forceinline__ float fold_rows_packed(const float* __restrict__ part, int rows, int ld, int col,
                                                  int width, int row0, int stride, int cw) {
  constexpr int U = 16;
  float a[U];
#pragma unroll
  for (int u = 0; u < U; ++u) a[u] = 0.f;
  if (col < width) {
    int r = row0;
    for (; r + stride * (U - 1) < rows; r += stride * U) {
#pragma unroll
      for (int u = 0; u < U; ++u) a[u] += part[(size_t)(r + stride * u) * ld + col];
    }
    for (; r < rows; r += stride) a[0] += part[(size_t)r * ld + col];
  }
#pragma unroll
  for (int h = U / 2; h > 0; h >>= 1)
#pragma unroll
    for (int u = 0; u < h; ++u) a[u] += a[u + h];
  float v = a[0];
  for (int off = cw; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// A workgroup (16 waves) folds 64 columns with 16 waves striding the rows, or
// -- short folds (<= kShortRows partial rows: the split-K weight-gradient
// partials, ~40-256 chunks) -- 256 columns, four waves per 64-column group.
// The generator backward folds ~274k columns: at 16 waves per 64 columns its
// grid ran 8+ rounds of 1024-thread workgroups, each one round trip long.
__global__ void __launch_bounds__(1024) k_fold_batch(const FoldBatch b) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int d = 0;
  while (d + 1 < b.n && (int)blockIdx.x >= b.block0[d + 1]) ++d;
  const vg_fold& f = b.f[d];
  if (b.cw[d] > 0) {  // narrow long fold: one workgroup, packed lanes
    const int cw = b.cw[d], rpl = 64 / cw;
    const int col = lane & (cw - 1);
    __shared__ float redn[2][16][32];
    for (int si = 0; si < f.nsrc; ++si) {
      const float v = fold_rows_packed(f.src[si].part, f.src[si].rows, f.src[si].ld, col, f.width,
                                       wave * rpl + lane / cw, 16 * rpl, cw);
      if (lane < cw) redn[si][wave][lane] = v;
    }
    __syncthreads();
    if (wave == 0 && lane < f.width) {
      float* o = f.out + (lane / f.k) * f.ldo + (lane % f.k);
      float v = f.accumulate ? *o : 0.f;
      for (int si = 0; si < f.nsrc; ++si) {
        float s = 0.f;
        for (int k = 0; k < 16; ++k) s += redn[si][k][lane];
        v = f.accumulate || si > 0 ? v + s : s;
      }
      *o = v;
    }
    return;
  }
  const int wpg = b.waves[d];               // waves per column group
  const int grp = wave / wpg, sub = wave % wpg;
  const long long w = ((long long)(blockIdx.x - b.block0[d]) * (16 / wpg) + grp) * 64 + lane;
  __shared__ float red[2][16][64];
  for (int si = 0; si < f.nsrc; ++si)
    red[si][wave][lane] = w < f.width ? fold_rows_sum(f.src[si].part, f.src[si].rows, f.src[si].ld, w, sub, wpg)
                                      : 0.f;
  __syncthreads();
  if (sub == 0 && w < f.width) {
    float* o = f.out + (w / f.k) * f.ldo + (w % f.k);
    float v = f.accumulate ? *o : 0.f;
    for (int si = 0; si < f.nsrc; ++si) {
      float s = 0.f;
      for (int k = 0; k < wpg; ++k) s += red[si][wave + k][lane];
      v = f.accumulate || si > 0 ? v + s : s;
    }
    *o = v;
  }
}

}  // namespace

extern "C" int vg_fold_batch(const vg_fold* folds, int32_t n, void* stream) {
  if (n < 0 || n > VG_FOLD_MAX || (n > 0 && !folds)) return VG_EINVAL;
  if (n == 0) return 0;
  FoldBatch b;
  b.n = n;
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    const vg_fold& f = folds[i];
    if (!f.out || f.width <= 0 || f.k <= 0 || f.ldo < f.k || f.nsrc < 1 || f.nsrc > 2) return VG_EINVAL;
    for (int s = 0; s < f.nsrc; ++s)
      if (!f.src[s].part || f.src[s].rows < 0 || f.src[s].ld < f.width) return VG_EINVAL;
    int rows = 0;
    for (int s = 0; s < f.nsrc; ++s) rows = f.src[s].rows > rows ? f.src[s].rows : rows;
    b.f[i] = f;
    b.waves[i] = rows <= kShortRows ? 4 : 16;
    b.block0[i] = blocks;
    int cw = 0;
    if (VG_FOLD_PACK && rows > kShortRows && f.width <= 32) {
      cw = 1;
      while (cw < f.width) cw <<= 1;
    }
    b.cw[i] = cw;
    blocks += cw ? 1 : (f.width + 64 * (16 / b.waves[i]) - 1) / (64 * (16 / b.waves[i]));
  }
  b.block0[n] = blocks;
  k_fold_batch<<<blocks, 1024, 0, static_cast<hipStream_t>(stream)>>>(b);
  VG_CHECK_LAUNCH();
  return 0;
}
