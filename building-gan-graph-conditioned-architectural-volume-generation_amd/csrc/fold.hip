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
  // split folds (vg_fold_batch_split, first level): chunks of kChunkRows
  // partial rows of src 0 (then src 1), chunk c's column sums into
  // ws[ws_off[i] + c * width ...]; 0 chunks: an ordinary fold
  int32_t chunks0[VG_FOLD_MAX], chunks[VG_FOLD_MAX], ws_off[VG_FOLD_MAX];
  float* ws;
  vg_fold f[VG_FOLD_MAX];
};
#ifndef VG_FOLD_SPLIT_ROWS
#define VG_FOLD_SPLIT_ROWS 768  // vg_fold_batch_split: folds with more partial rows go two-level
#endif
#ifndef VG_FOLD_CHUNK_ROWS
#define VG_FOLD_CHUNK_ROWS 256  // partial rows per first-level chunk (64 / 128 / 256 / 384 / 512 measured)
#endif
constexpr int kChunkRows = VG_FOLD_CHUNK_ROWS;

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
  int d = 0, hi = b.n - 1;  // the fold owning this workgroup: the last d with block0[d] <= blockIdx.x
  while (d < hi) {          // (binary search: up to VG_FOLD_MAX dependent argument loads otherwise)
    const int mid = (d + hi + 1) >> 1;
    if ((int)blockIdx.x >= b.block0[mid]) d = mid; else hi = mid - 1;
  }
  const vg_fold& f = b.f[d];
  if (b.chunks[d] > 0) {  // first level of a split fold: one chunk of one source, 64 columns
    const int groups = (f.width + 63) / 64;
    const int lb = blockIdx.x - b.block0[d];
    const int chunk = lb / groups, grp = lb % groups;
    const int si = chunk < b.chunks0[d] ? 0 : 1;
    const int r0 = (si == 0 ? chunk : chunk - b.chunks0[d]) * kChunkRows;
    const int rows = min(kChunkRows, f.src[si].rows - r0);
    const long long w = (long long)grp * 64 + lane;
    __shared__ float redc[16][64];
    redc[wave][lane] = w < f.width && rows > 0
                           ? fold_rows_sum(f.src[si].part + (size_t)r0 * f.src[si].ld, rows, f.src[si].ld, w, wave, 16)
                           : 0.f;
    __syncthreads();
    if (wave == 0 && w < f.width) {
      float v = 0.f;
      for (int k = 0; k < 16; ++k) v += redc[k][lane];
      b.ws[(size_t)b.ws_off[d] + (size_t)chunk * f.width + w] = v;
    }
    return;
  }
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

// validate fold i; its partial rows (the longer source)
static int fold_rows_of(const vg_fold& f) {
  if (!f.out || f.width <= 0 || f.k <= 0 || f.ldo < f.k || f.nsrc < 1 || f.nsrc > 2) return -1;
  int rows = 0;
  for (int s = 0; s < f.nsrc; ++s) {
    if (!f.src[s].part || f.src[s].rows < 0 || f.src[s].ld < f.width) return -1;
    rows = f.src[s].rows > rows ? f.src[s].rows : rows;
  }
  return rows;
}

// one launch over folds[0, n); split[i] > 0: fold i's first level (chunk count)
static int launch_batch(const vg_fold* folds, int32_t n, const int* split, const int* chunks0, const int* ws_off,
                        float* ws, void* stream) {
  FoldBatch b;
  b.n = n;
  b.ws = ws;
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    const vg_fold& f = folds[i];
    const int rows = fold_rows_of(f);
    if (rows < 0) return VG_EINVAL;
    b.f[i] = f;
    b.block0[i] = blocks;
    b.chunks[i] = split ? split[i] : 0;
    b.chunks0[i] = split ? chunks0[i] : 0;
    b.ws_off[i] = split ? ws_off[i] : 0;
    b.waves[i] = rows <= kShortRows ? 4 : 16;
    int cw = 0;
    if (b.chunks[i] > 0) {
      b.waves[i] = 16;
      b.cw[i] = 0;
      blocks += (f.width + 63) / 64 * b.chunks[i];
      continue;
    }
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

extern "C" int vg_fold_batch(const vg_fold* folds, int32_t n, void* stream) {
  if (n < 0 || n > VG_FOLD_MAX || (n > 0 && !folds)) return VG_EINVAL;
  if (n == 0) return 0;
  return launch_batch(folds, n, nullptr, nullptr, nullptr, nullptr, stream);
}

extern "C" int64_t vg_fold_split_ws_floats(const vg_fold* folds, int32_t n) {
  if (n < 0 || n > VG_FOLD_MAX || (n > 0 && !folds)) return VG_EINVAL;
  int64_t need = 0;
  for (int i = 0; i < n; ++i) {
    const int rows = fold_rows_of(folds[i]);
    if (rows < 0) return VG_EINVAL;
    if (rows > VG_FOLD_SPLIT_ROWS)
      for (int s = 0; s < folds[i].nsrc; ++s)
        need += (int64_t)((folds[i].src[s].rows + kChunkRows - 1) / kChunkRows) * folds[i].width;
  }
  return need;
}

extern "C" int vg_fold_batch_split(const vg_fold* folds, int32_t n, float* ws, int64_t ws_floats, void* stream) {
  if (n < 0 || n > VG_FOLD_MAX || (n > 0 && !folds) || ws_floats < 0 || ws_floats > (int64_t)1 << 31) return VG_EINVAL;
  if (n == 0) return 0;
  // folds with more than VG_FOLD_SPLIT_ROWS partial rows (while ws lasts) go
  // two-level: their chunks' column sums in the same launch as the short
  // folds, then one fold of those sums into the destination (src 0's chunks,
  // then src 1's: the same (out + src 0) + src 1 order)
  int split[VG_FOLD_MAX], c0[VG_FOLD_MAX], off[VG_FOLD_MAX];
  vg_fold second[VG_FOLD_MAX];
  int n2 = 0;
  int64_t used = 0;
  for (int i = 0; i < n; ++i) {
    const vg_fold& f = folds[i];
    const int rows = fold_rows_of(f);
    if (rows < 0) return VG_EINVAL;
    split[i] = c0[i] = off[i] = 0;
    if (rows <= VG_FOLD_SPLIT_ROWS || !ws) continue;
    const int k0 = (f.src[0].rows + kChunkRows - 1) / kChunkRows;
    const int k1 = f.nsrc > 1 ? (f.src[1].rows + kChunkRows - 1) / kChunkRows : 0;
    const int64_t need = (int64_t)(k0 + k1) * f.width;
    if (used + need > ws_floats) continue;  // no room: an ordinary fold
    split[i] = k0 + k1;
    c0[i] = k0;
    off[i] = static_cast<int>(used);
    vg_fold g = f;
    g.src[0] = vg_fold_src{ws + used, k0, f.width};
    if (f.nsrc > 1) g.src[1] = vg_fold_src{ws + used + (int64_t)k0 * f.width, k1, f.width};
    second[n2++] = g;
    used += need;
  }
  const int rc = launch_batch(folds, n, split, c0, off, ws, stream);
  if (rc || n2 == 0) return rc;
  return launch_batch(second, n2, nullptr, nullptr, nullptr, nullptr, stream);
}
