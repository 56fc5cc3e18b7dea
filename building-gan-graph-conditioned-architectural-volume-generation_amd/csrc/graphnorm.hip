// GraphNorm(batch=None) fused with the ReLU and Dropout that follow it in every
// encoder block (models.py:73-75,83-85,193-195,203-205), with torch_geometric
// 2.6.1 nn/norm/graph_norm.py semantics (requirements.txt:11):
//
// Forward   mu = mean_rows(x);  o = x - ms*mu;  var_o = mean_rows(o^2)
//           d = sqrt(var_o + eps);  y = keep * relu(w * o / d + b)
//           var_o = var(x) + ((1 - ms) mu)^2, so the statistics are the
//           population (mean, var) of x (Welford) and the fold stores
//           stats = [mu | d] per column -- every consumer divides by d.
// Backward  gz = g_y * keep * [z > 0];  A = sum gz;  B = sum gz * ohat
//           (ohat = o / d);  a = (1 - ms) mu  (= mean_rows(o))
//           g_x = (w/d) (gz - B ohat / N - (ms/N)(A - B a / d))
//           g_w = B, g_b = A, g_ms = -mu (w/d) (A - B a / d)
//
// Segments: S independent row blocks of Ns rows each (the discriminator's
// real / fake / mix copies stacked as one [3N, C] tensor) each normalise with
// their own column statistics (stats [S][2C]); parameter gradients sum over
// segments.
//
// Second order (the WGAN-GP critic engine, vgan/critic.py): for a tangent u of
// x and the adjoint g_y of y, with p = g_y * keep * [z > 0], m_u = mean(u),
// c' = u - ms*m_u, K = mean(o c') (so d' = K/d):
//   y'  = keep [z > 0] w (c'/d - o K/d^3)
//   Q   = <g_y, y'> = w (P1/d - P2 K/d^3),  P1 = sum p c',  P2 = sum p o
//   dQ/dw, dQ/dms and dQ/dx in closed form from the column sums
//   (sum u, sum xt u, sum p, sum p u, sum p xt), xt = x - mu   (k_gn_jvp2_*)
//
// The column statistics are a two-level deterministic reduction: R row-chunk
// blocks per 64-column slab produce (count, mean, M2) Welford partials, a
// finalize kernel merges them in a fixed order (Chan's formula), and the
// elementwise kernel applies.  Lanes are packed (col, row-sub) so narrow layers
// (C = 1..32) still use every lane of the wave.
#include "common.h"
#include "gnbwd.h"
#include "gnjvp.h"

#include <algorithm>
#include <initializer_list>

namespace {

constexpr int kBlock = 256;
#ifndef VG_GN_CHUNKS
#define VG_GN_CHUNKS 256
#endif
constexpr int kChunks = VG_GN_CHUNKS;  // max row chunks per column slab
constexpr int kFoldU = kChunks / 64;
static_assert(kChunks == vg::kGnChunks, "gnjvp.h folds the same chunk partials");
#ifndef VG_GN_CHUNK_ROWS
#define VG_GN_CHUNK_ROWS 32
#endif
#ifndef VG_GN_APPLY_MAX
#define VG_GN_APPLY_MAX 2048
#endif
constexpr int kChunkRows = VG_GN_CHUNK_ROWS;       // rows per statistics chunk
constexpr int kApplyMaxBlocks = VG_GN_APPLY_MAX;  // elementwise grid cap  // chunk partials per lane in the one-wave folds

struct Welford {
  float n, mean, m2;
};

__device__ __forceinline__ Welford merge(Welford a, Welford b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float delta = b.mean - a.mean;
  const float fb = b.n / n;
  Welford r;
  r.n = n;
  r.mean = a.mean + delta * fb;
  r.m2 = a.m2 + b.m2 + delta * delta * a.n * fb;
  return r;
}

// lane layout inside a wave for a slab of CW columns (CW pow2 <= 64)
struct Lay {
  int cw, rpw;  // columns per wave-step, rows per wave-step
};

__host__ __device__ inline Lay lay_for(int C) {
  int cw = 1;
  while (cw < C && cw < 64) cw <<= 1;
  return {cw, 64 / cw};
}

// Partials of one (chunk, 64-column slab, segment); counter is unused (the
// former last-block fold: one workgroup folding every partial ran at a single
// CU's bandwidth).
// T = float (rows of C) or _Float16 (rows of ld >= C, the f16 inference path).
template <typename T>
__global__ void __launch_bounds__(kBlock) k_stats_partial(const T* __restrict__ x, int N, int C, int ld,
                                                          float* __restrict__ part,
                                                          float* __restrict__ stats, int* counter) {
  float* const part0 = part;
  const Lay ly = lay_for(C);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + (lane & (ly.cw - 1));
  const int rsub = wave * ly.rpw + lane / ly.cw;
  const int rstep = 4 * ly.rpw;
  const int rows_per_chunk = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  const bool col_ok = c < C && (lane & (ly.cw - 1)) < 64;
  x += (size_t)blockIdx.z * N * ld;  // segment
  part += (size_t)blockIdx.z * gridDim.x * C * 3;
  Welford w = {0.f, 0.f, 0.f};
  if (col_ok) {
    // kB rows per lane in flight at once (a chunk is ~13 rows per lane at
    // batch 32), then the Welford updates in row order (as one row at a time)
    constexpr int kB = 16;
    for (int rb = r0 + rsub; rb < r1; rb += kB * rstep) {
      float v[kB];
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        const int r = rb + j * rstep;
        v[j] = r < r1 ? static_cast<float>(x[(size_t)r * ld + c]) : 0.f;
      }
#pragma unroll
      for (int j = 0; j < kB; ++j) {
        if (rb + j * rstep >= r1) break;
        w.n += 1.f;
        const float d = v[j] - w.mean;
        w.mean += d / w.n;
        w.m2 += d * (v[j] - w.mean);
      }
    }
  }
  // merge lanes of the same column inside the wave (xor over the row-sub bits)
  for (int off = ly.cw; off < 64; off <<= 1) {
    Welford o;
    o.n = __shfl_xor(w.n, off, 64);
    o.mean = __shfl_xor(w.mean, off, 64);
    o.m2 = __shfl_xor(w.m2, off, 64);
    w = merge(w, o);
  }
  __shared__ Welford sw[4][64];
  if (lane < ly.cw) sw[wave][lane] = w;
  __syncthreads();
  if (wave == 0 && lane < ly.cw && c < C) {
    Welford acc = sw[0][lane];
    for (int k = 1; k < 4; ++k) acc = merge(acc, sw[k][lane]);
    float* p = part + ((size_t)blockIdx.x * C + c) * 3;
    p[0] = acc.n;
    p[1] = acc.mean;
    p[2] = acc.m2;
  }
  (void)counter;
  (void)part0;
  (void)stats;
}

// Fold of the chunk partials: ONE WAVE PER COLUMN, every segment; lane l takes
// chunks l, l+64, l+128, l+192 (kChunks <= 256: four loads in flight per lane,
// one round trip per segment), then a fixed xor-butterfly across the wave --
// deterministic, and spread over C/4 workgroups.  A single workgroup folding
// all partials (the first version) ran at one CU's bandwidth, ~8-10 us.
// Waves per fold workgroup (VG_FOLD_WAVES, default 1): the folds' loads gather
// one column's partials across rows of partials, 64 lines per instruction, so
// a fold is bound by its CU's address unit; one wave per workgroup spreads the
// columns over C CUs instead of C / 4.
#ifndef VG_FOLD_WAVES
#define VG_FOLD_WAVES 1
#endif
constexpr int kFoldWaves = VG_FOLD_WAVES;
__device__ __forceinline__ int fold_col() { return blockIdx.x * kFoldWaves + (threadIdx.x >> 6); }

__device__ __forceinline__ Welford wave_merge(Welford w) {
  for (int off = 1; off < 64; off <<= 1) {
    Welford o;
    o.n = __shfl_xor(w.n, off, 64);
    o.mean = __shfl_xor(w.mean, off, 64);
    o.m2 = __shfl_xor(w.m2, off, 64);
    w = merge(w, o);
  }
  return w;
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int off = 1; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// The GraphNorm denominator from the column's population (mean, M2):
// d = sqrt(mean((x - ms mu)^2) + eps) = sqrt(var + ((1 - ms) mu)^2 + eps)
__device__ __forceinline__ float gn_denom(Welford a, float msc, float eps) {
  const float var = fmaxf(a.m2 / a.n, 0.f);
  const float sh = (1.f - msc) * a.mean;
  return sqrtf(fmaf(sh, sh, var) + eps);
}

// One wave per (column, segment): grid (C / 4, S).
__global__ void __launch_bounds__(kBlock) k_stats_final(const float* __restrict__ part, int chunks,
                                                        int C, int S, const float* __restrict__ ms, float eps,
                                                        float* __restrict__ stats) {
  const int c = fold_col(), lane = threadIdx.x & 63;
  const int sg = blockIdx.y;
  if (c >= C || sg >= S) return;
  const float msc = ms[c];
  const float* pp = part + (size_t)sg * chunks * C * 3;
  float v[kFoldU][3];
#pragma unroll
  for (int u = 0; u < kFoldU; ++u) {
    const int k = lane + 64 * u;
#pragma unroll
    for (int q = 0; q < 3; ++q) v[u][q] = k < chunks ? pp[((size_t)k * C + c) * 3 + q] : 0.f;
  }
  Welford acc = {0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < kFoldU; ++u) acc = merge(acc, Welford{v[u][0], v[u][1], v[u][2]});
  acc = wave_merge(acc);
  if (lane == 0) {
    stats[(size_t)sg * 2 * C + c] = acc.mean;
    stats[(size_t)sg * 2 * C + C + c] = gn_denom(acc, msc, eps);
  }
}

// The same fold over the block partials the GAT aggregation wrote in its
// epilogue (vg_gat_aggregate_fwd_gnp): gnp [blocks][2][C][3], slot 0, for
// SEGMENT-ALIGNED blocks of G rows -- segment sg owns blocks sg * B ..
// sg * B + B - 1, B = ceil(N / G) -- so a segment folds exactly what a separate
// forward over it would.  One wave per (column, segment); lane l merges the
// segment's blocks l, l + 64, ... in order (16 in flight: one round trip at
// batch 32), then the xor butterfly: deterministic.
__global__ void __launch_bounds__(kBlock) k_stats_final_gnp(const float* __restrict__ gnp, int G, int N, int C,
                                                            int S, const float* __restrict__ ms, float eps,
                                                            float* __restrict__ stats) {
  const int c = fold_col(), lane = threadIdx.x & 63;
  const int sg = blockIdx.y;
  if (c >= C || sg >= S) return;
  const float msc = ms[c];
  const int nb = (N + G - 1) / G;
  const int b0 = sg * nb, b1 = b0 + nb - 1;  // inclusive
  constexpr int U = 16;
  Welford acc = {0.f, 0.f, 0.f};
  for (int bb = b0 + lane; bb <= b1; bb += 64 * U) {
    float v[U][3];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = bb + 64 * u;
      if (b <= b1) {
        const float* p = gnp + ((size_t)b * 2 * C + c) * 3;
        v[u][0] = p[0];
        v[u][1] = p[1];
        v[u][2] = p[2];
      } else {
        v[u][0] = v[u][1] = v[u][2] = 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = merge(acc, Welford{v[u][0], v[u][1], v[u][2]});
  }
  acc = wave_merge(acc);
  if (lane == 0) {
    stats[(size_t)sg * 2 * C + c] = acc.mean;
    stats[(size_t)sg * 2 * C + C + c] = gn_denom(acc, msc, eps);
  }
}

// iter != NULL: draw the dropout multiplier in-kernel (vg_keep with p_drop,
// seed, *iter, salt) and apply it; keep_out != NULL also stores it for the
// backward (a no-grad forward -- the critic labels -- skips the store).
__global__ void k_gn_apply(const float* __restrict__ x, long long total, int C, long long seg_elems,
                           const float* __restrict__ w, const float* __restrict__ b,
                           const float* __restrict__ ms, const float* __restrict__ keep,
                           float eps, const float* __restrict__ stats, float* __restrict__ y,
                           float p_drop, unsigned long long seed, const long long* __restrict__ iter,
                           unsigned int salt, float* __restrict__ keep_out) {
  const bool draw = iter != nullptr;
  const long long it = draw ? *iter : 0;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % C);
    const float* st = stats + 2 * C * (t / seg_elems);
    const float mu = st[c], sd = st[C + c];
    const float o = x[t] - mu * ms[c];
    const float z = (o / sd) * w[c] + b[c];
    float r = z > 0.f ? z : 0.f;
    if (draw) {
      const float k = vg_keep(t, salt, it, seed, p_drop);
      if (keep_out) keep_out[t] = k;
      r *= k;
    } else if (keep) {
      r *= keep[t];
    }
    y[t] = r;
  }
}

// f16 rows (inference): y = relu(GraphNorm(x)) over ld-strided rows, two
// channels per thread; columns C .. wcols-1 (wcols = C rounded up to 8) are
// written as 0, so y may be a column slice of a wider row (ldy).
__global__ void k_gn_apply_h(const _Float16* __restrict__ x, long long pairs, int C, int ld, int wcols,
                             long long seg_rows, const float* __restrict__ w, const float* __restrict__ b,
                             const float* __restrict__ ms, float eps, const float* __restrict__ stats,
                             _Float16* __restrict__ y, int ldy) {
  const int hp = wcols / 2;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < pairs;
       t += (long long)gridDim.x * blockDim.x) {
    const long long row = t / hp;
    const int c = 2 * static_cast<int>(t % hp);
    const float* st = stats + 2 * C * (row / seg_rows);
    const _Float16* xp = x + row * ld + c;
    float r[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int cc = c + q;
      if (cc < C) {
        const float z = ((static_cast<float>(xp[q]) - st[cc] * ms[cc]) / st[C + cc]) * w[cc] + b[cc];
        r[q] = z > 0.f ? z : 0.f;
      } else {
        r[q] = 0.f;
      }
    }
    _Float16* yp = y + row * ldy + c;
    yp[0] = static_cast<_Float16>(r[0]);
    yp[1] = static_cast<_Float16>(r[1]);
  }
}

// backward: column partial sums of gz and gz*xhat (plain sums, chunk order)
__global__ void __launch_bounds__(kBlock) k_gn_bwd_partial(
    const float* __restrict__ x, const float* __restrict__ gy, int N, int C,
    const float* __restrict__ w, const float* __restrict__ b, const float* __restrict__ ms,
    const float* __restrict__ keep, float eps, const float* __restrict__ stats,
    float* __restrict__ part, float* __restrict__ sums, float* __restrict__ g_w,
    float* __restrict__ g_b, float* __restrict__ g_ms, int accumulate, int* counter) {
  const float* const stats0 = stats;
  float* const part0 = part;
  const Lay ly = lay_for(C);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + (lane & (ly.cw - 1));
  const int rsub = wave * ly.rpw + lane / ly.cw;
  const int rstep = 4 * ly.rpw;
  const int rows_per_chunk = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  const size_t so = (size_t)blockIdx.z * N * C;  // segment
  x += so;
  gy += so;
  if (keep) keep += so;
  stats += (size_t)blockIdx.z * 2 * C;
  part += (size_t)blockIdx.z * gridDim.x * C * 2;
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    const float mu = stats[c], s = stats[C + c], wc = w[c], bc = b[c], msc = ms[c];
#pragma unroll 4
    for (int r = r0 + rsub; r < r1; r += rstep) {
      const size_t t = (size_t)r * C + c;
      const float xh = (x[t] - mu * msc) / s;
      const float z = xh * wc + bc;
      float gz = z > 0.f ? gy[t] : 0.f;
      if (keep) gz *= keep[t];
      sa += gz;
      sb = fmaf(gz, xh, sb);
    }
  }
  for (int off = ly.cw; off < 64; off <<= 1) {
    sa += __shfl_xor(sa, off, 64);
    sb += __shfl_xor(sb, off, 64);
  }
  __shared__ float s2[4][64][2];
  if (lane < ly.cw) {
    s2[wave][lane][0] = sa;
    s2[wave][lane][1] = sb;
  }
  __syncthreads();
  if (wave == 0 && lane < ly.cw && c < C) {
    float a = 0.f, bb = 0.f;
    for (int k = 0; k < 4; ++k) {
      a += s2[k][lane][0];
      bb += s2[k][lane][1];
    }
    float* p = part + ((size_t)blockIdx.x * C + c) * 2;
    p[0] = a;
    p[1] = bb;
  }
  (void)counter;
  (void)part0;
  (void)stats0;
  (void)sums;
  (void)g_w;
  (void)g_b;
  (void)g_ms;
  (void)accumulate;
}

// one wave per column: per-segment sums A, B (-> sums[sg][2C]) and the
// parameter gradients summed over segments in order
__global__ void __launch_bounds__(kBlock) k_gn_bwd_final(
    const float* __restrict__ part, int chunks, int C, int S, const float* __restrict__ w,
    const float* __restrict__ ms, float eps, const float* __restrict__ stats,
    float* __restrict__ sums, float* __restrict__ g_w, float* __restrict__ g_b,
    float* __restrict__ g_ms, int accumulate) {
  const int c = fold_col(), lane = threadIdx.x & 63;
  if (c >= C) return;
  float tw = 0.f, tb = 0.f, tm = 0.f;
  constexpr int kSegs = 4;  // segments whose partials are in flight together
  for (int s0 = 0; s0 < S; s0 += kSegs) {
    float va[kSegs][kFoldU], vb[kSegs][kFoldU];
#pragma unroll
    for (int j = 0; j < kSegs; ++j) {
      const float* pp = part + (size_t)(s0 + j) * chunks * C * 2;
#pragma unroll
      for (int u = 0; u < kFoldU; ++u) {
        const int k = lane + 64 * u;
        const bool ok = s0 + j < S && k < chunks;
        va[j][u] = ok ? pp[((size_t)k * C + c) * 2] : 0.f;
        vb[j][u] = ok ? pp[((size_t)k * C + c) * 2 + 1] : 0.f;
      }
    }
#pragma unroll
    for (int j = 0; j < kSegs; ++j) {
      const int sg = s0 + j;
      if (sg >= S) break;
      float a = 0.f, bb = 0.f;
#pragma unroll
      for (int u = 0; u < kFoldU; ++u) {
        a += va[j][u];
        bb += vb[j][u];
      }
      a = wave_sum(a);
      bb = wave_sum(bb);
      const float* st = stats + (size_t)sg * 2 * C;
      if (lane == 0) {
        sums[(size_t)sg * 2 * C + c] = a;
        sums[(size_t)sg * 2 * C + C + c] = bb;
      }
      tw += bb;
      tb += a;
      tm += vg::gn_g_ms(st[c], st[C + c], w[c], ms[c], a, bb);
    }
  }
  if (lane == 0 && g_w) {
    g_w[c] = accumulate ? g_w[c] + tw : tw;
    g_b[c] = accumulate ? g_b[c] + tb : tb;
    g_ms[c] = accumulate ? g_ms[c] + tm : tm;
  }
}

// One group of up to kSegs segments of k_gn_bwd_final_tiles' fold.
template <int kSegs, int kU>
__device__ __forceinline__ void bwd_tiles_group(const float* __restrict__ tpart, int N, int C, int S, int s0,
                                                int c, int lane, const float* __restrict__ w,
                                                const float* __restrict__ ms,
                                                const float* __restrict__ stats, float* __restrict__ sums,
                                                const float* __restrict__ g3[3], float g0[3],
                                                float& tw, float& tb, float& tm) {
  constexpr int kTile = 64;
  float va[kSegs][kU], vb[kSegs][kU], mu[kSegs], sd[kSegs];
  int t0[kSegs], t1[kSegs];
#pragma unroll
  for (int j = 0; j < kSegs; ++j) {
    const int sg = min(s0 + j, S - 1);
    const long long r0 = (long long)sg * N;
    t0[j] = static_cast<int>(r0 / kTile);
    t1[j] = static_cast<int>((r0 + N - 1) / kTile);
    mu[j] = stats[(size_t)sg * 2 * C + c];
    sd[j] = stats[(size_t)sg * 2 * C + C + c];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int t = t0[j] + lane + 64 * u;
      const int tc = min(t, t1[j]);
      const int slot = (long long)tc * kTile >= r0 ? 0 : 1;  // first row in this segment, or in the previous one
      const float2 v = *reinterpret_cast<const float2*>(tpart + ((size_t)(2 * tc + slot) * C + c) * 2);
      va[j][u] = v.x;
      vb[j][u] = v.y;
    }
  }
  // the per-column operands and (first group) the accumulated gradients, in
  // flight with the partials
  const float wc = w[c], msc = ms[c];
  if (g3) {
#pragma unroll
    for (int q = 0; q < 3; ++q) g0[q] = g3[q][c];
  }
#pragma unroll
  for (int j = 0; j < kSegs; ++j) {
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const bool ok = s0 + j < S && t0[j] + lane + 64 * u <= t1[j];
      va[j][u] = ok ? va[j][u] : 0.f;
      vb[j][u] = ok ? vb[j][u] : 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < kSegs; ++j) {
    const int sg = s0 + j;
    if (sg >= S) break;
    float a = 0.f, bb = 0.f;
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      a += va[j][u];
      bb += vb[j][u];
    }
    const long long r0 = (long long)sg * N;
    for (int t = t0[j] + lane + 64 * kU; t <= t1[j]; t += 64) {  // segments of more than 16k rows
      const int slot = (long long)t * kTile >= r0 ? 0 : 1;
      const float* p = tpart + ((size_t)(2 * t + slot) * C + c) * 2;
      a += p[0];
      bb += p[1];
    }
    a = wave_sum(a);
    bb = wave_sum(bb);
    if (lane == 0) {
      sums[(size_t)sg * 2 * C + c] = a;
      sums[(size_t)sg * 2 * C + C + c] = bb;
    }
    tw += bb;
    tb += a;
    tm += vg::gn_g_ms(mu[j], sd[j], wc, msc, a, bb);
  }
}

// The same fold over the partials that the producing GEMM wrote in its
// epilogue (vg_gemm_gn_bwd): tpart[tile][slot][C][2] for 64-row tiles of the
// S * N stacked rows, slot 0 = the segment of the tile's first row, slot 1 =
// the next segment (a tile straddles at most two: N >= 64).  One wave per
// column; segment sg sums its tiles in tile order (deterministic).
//
// Every load of the fold is issued before the first wait: the partials at
// clamped (always valid) addresses, zeroed afterwards when out of range, the
// per-column operands and the accumulated gradients unconditionally, and no
// loop around the common S <= 4 case (a loop header made the compiler drain
// the loads issued before it).  The guarded form (`ok ? p[0] : 0`) compiled to
// a branch per load and a vmcnt(0) per segment group, then a round trip each
// for the statistics and the gradients' read-modify-write: ~6 dependent round
// trips per launch.  Same values, same summation order (bit-identical).
__global__ void __launch_bounds__(kBlock) k_gn_bwd_final_tiles(
    const float* __restrict__ tpart, int N, int C, int S, const float* __restrict__ w,
    const float* __restrict__ ms, float eps, const float* __restrict__ stats, float* __restrict__ sums,
    float* __restrict__ g_w, float* __restrict__ g_b, float* __restrict__ g_ms, int accumulate) {
  constexpr int kSegs = 4, kU = 4;  // segments in flight together, tiles per lane and segment
  const int c = fold_col(), lane = threadIdx.x & 63;
  if (c >= C) return;
  const bool acc = g_w && accumulate;
  const float* g3[3] = {acc ? g_w : w, acc ? g_b : w, acc ? g_ms : w};
  float g0[3] = {0.f, 0.f, 0.f};
  float tw = 0.f, tb = 0.f, tm = 0.f;
  if (S <= kSegs) {
    bwd_tiles_group<kSegs, kU>(tpart, N, C, S, 0, c, lane, w, ms, stats, sums, g3, g0, tw, tb, tm);
  } else {
    for (int s0 = 0; s0 < S; s0 += kSegs)
      bwd_tiles_group<kSegs, kU>(tpart, N, C, S, s0, c, lane, w, ms, stats, sums, s0 == 0 ? g3 : nullptr, g0,
                                 tw, tb, tm);
  }
  if (lane == 0 && g_w) {
    g_w[c] = acc ? g0[0] + tw : tw;
    g_b[c] = acc ? g0[1] + tb : tb;
    g_ms[c] = acc ? g0[2] + tm : tm;
  }
  (void)eps;
}

// g_x (+ inj for elements t >= inj_off: the second-order adjoint of the
// critic engine's mix copy)
__global__ void k_gn_bwd_apply(const float* __restrict__ x, const float* __restrict__ gy,
                               long long total, int N, int C, const float* __restrict__ w,
                               const float* __restrict__ b, const float* __restrict__ ms,
                               const float* __restrict__ keep, float eps,
                               const float* __restrict__ stats, const float* __restrict__ sums,
                               const float* __restrict__ inj, long long inj_off,
                               float* __restrict__ gx) {
  const float inv_n = 1.f / static_cast<float>(N);
  const long long seg_elems = (long long)N * C;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % C);
    const long long sg = t / seg_elems;
    const float* st = stats + 2 * C * sg;
    const float* sm = sums + 2 * C * sg;
    float g = vg::gn_bwd_elem(x[t], gy[t], keep ? keep[t] : 1.f, keep != nullptr, st[c], st[C + c], w[c], b[c],
                              ms[c], sm[c], sm[C + c], eps, inv_n);
    if (inj && t >= inj_off) g += inj[t - inj_off];
    gx[t] = g;
  }
}


// ---------------------------------------------------------- second order
// column sums for the tangent / second-order pass: [sum u, sum xt u, sum p,
// sum p u, sum p xt] per column (plain sums, chunk order)
__global__ void __launch_bounds__(kBlock) k_gn_jvp2_partial(
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ gy, int N,
    int C, const float* __restrict__ w, const float* __restrict__ b, const float* __restrict__ ms,
    const float* __restrict__ keep, float eps, const float* __restrict__ stats,
    float* __restrict__ part, float* __restrict__ sums, float* __restrict__ g_w,
    float* __restrict__ g_ms, int* counter) {
  const Lay ly = lay_for(C);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + (lane & (ly.cw - 1));
  const int rsub = wave * ly.rpw + lane / ly.cw;
  const int rstep = 4 * ly.rpw;
  const int rows_per_chunk = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    const float mu = stats[c], s = stats[C + c], wc = w[c], bc = b[c], msc = ms[c];
#pragma unroll 4
    for (int r = r0 + rsub; r < r1; r += rstep) {
      const size_t t = (size_t)r * C + c;
      const float xv = x[t], uv = u[t];
      const float xt = xv - mu;
      const float z = ((xv - mu * msc) / s) * wc + bc;
      float p = z > 0.f ? gy[t] : 0.f;
      if (keep) p *= keep[t];
      v[0] += uv;
      v[1] = fmaf(xt, uv, v[1]);
      v[2] += p;
      v[3] = fmaf(p, uv, v[3]);
      v[4] = fmaf(p, xt, v[4]);
    }
  }
#pragma unroll
  for (int q = 0; q < 5; ++q)
    for (int off = ly.cw; off < 64; off <<= 1) v[q] += __shfl_xor(v[q], off, 64);
  __shared__ float s5[4][64][5];
  if (lane < ly.cw)
#pragma unroll
    for (int q = 0; q < 5; ++q) s5[wave][lane][q] = v[q];
  __syncthreads();
  if (wave == 0 && lane < ly.cw && c < C) {
    float* pp = part + ((size_t)blockIdx.x * C + c) * 5;
#pragma unroll
    for (int q = 0; q < 5; ++q) pp[q] = (s5[0][lane][q] + s5[1][lane][q]) + (s5[2][lane][q] + s5[3][lane][q]);
  }
  (void)counter;
  (void)sums;
  (void)g_w;
  (void)g_ms;
}

// The same sums over float4 quads (C % 4 == 0, 16-B aligned rows): 16 lanes
// x 4 columns per row, 4 rows per wave, 16 per block step; the 4 row lanes
// of a column meet by xor shuffles, the 4 waves through LDS in order.
__global__ void __launch_bounds__(kBlock) k_gn_jvp2_partial4(
    const float* __restrict__ x, const float* __restrict__ u, const float* __restrict__ gy, int N,
    int C, const float* __restrict__ w, const float* __restrict__ b, const float* __restrict__ ms,
    const float* __restrict__ keep, float eps, const float* __restrict__ stats,
    float* __restrict__ part) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c0 = blockIdx.y * 64 + 4 * (lane & 15);
  const int rsub = wave * 4 + (lane >> 4);
  const int rows_per_chunk = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  float v[5][4];
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int q = 0; q < 4; ++q) v[k][q] = 0.f;
  if (c0 < C) {
    float mu[4], sd[4], wc[4], bc[4], msc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      mu[q] = stats[c0 + q];
      sd[q] = stats[C + c0 + q];
      wc[q] = w[c0 + q];
      bc[q] = b[c0 + q];
      msc[q] = ms[c0 + q];
    }
#pragma unroll 2
    for (int r = r0 + rsub; r < r1; r += 16) {
      const size_t t = (size_t)r * C + c0;
      const float4 xv = *reinterpret_cast<const float4*>(x + t);
      const float4 uv = *reinterpret_cast<const float4*>(u + t);
      const float4 gv = *reinterpret_cast<const float4*>(gy + t);
      const float4 kv = keep ? *reinterpret_cast<const float4*>(keep + t) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float xa[4] = {xv.x, xv.y, xv.z, xv.w}, ua[4] = {uv.x, uv.y, uv.z, uv.w};
      const float ga[4] = {gv.x, gv.y, gv.z, gv.w}, ka[4] = {kv.x, kv.y, kv.z, kv.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float xt = xa[q] - mu[q];
        const float z = ((xa[q] - mu[q] * msc[q]) / sd[q]) * wc[q] + bc[q];
        float p = z > 0.f ? ga[q] : 0.f;
        if (keep) p *= ka[q];
        v[0][q] += ua[q];
        v[1][q] = fmaf(xt, ua[q], v[1][q]);
        v[2][q] += p;
        v[3][q] = fmaf(p, ua[q], v[3][q]);
        v[4][q] = fmaf(p, xt, v[4][q]);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 5; ++k)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[k][q] += __shfl_xor(v[k][q], 16, 64);
      v[k][q] += __shfl_xor(v[k][q], 32, 64);
    }
  __shared__ float s5[4][64][5];
  if (lane < 16)
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int k = 0; k < 5; ++k) s5[wave][4 * lane + q][k] = v[k][q];
  __syncthreads();
  const int c = blockIdx.y * 64 + threadIdx.x;
  if (threadIdx.x < 64 && c < C) {
    float* pp = part + ((size_t)blockIdx.x * C + c) * 5;
#pragma unroll
    for (int k = 0; k < 5; ++k)
      pp[k] = (s5[0][threadIdx.x][k] + s5[1][threadIdx.x][k]) + (s5[2][threadIdx.x][k] + s5[3][threadIdx.x][k]);
  }
}

// one wave per column: the five sums, then the column terms (gnjvp.h)
__global__ void __launch_bounds__(kBlock) k_gn_jvp2_final(
    const float* __restrict__ part, int chunks, int N, int C, const float* __restrict__ w,
    const float* __restrict__ ms, float eps, const float* __restrict__ stats,
    float* __restrict__ sums, float* __restrict__ g_w, float* __restrict__ g_ms) {
  const int c = fold_col(), lane = threadIdx.x & 63;
  if (c >= C) return;
  vg::gn_jvp2_fold_col(part, chunks, N, C, w, ms, stats, sums, g_w, g_ms, c, lane);
  (void)eps;
}

// The same fold over the rows of partials the GAT tangent pass wrote
// (vg_gat_jvp2_gn_deferred: part [blocks][5][C]); one wave per column, lane l
// sums blocks l, l + 64, ... in order (16 in flight), then the butterfly.
__global__ void __launch_bounds__(kBlock) k_gn_jvp2_final_blk(
    const float* __restrict__ part, int blocks, int N, int C, const float* __restrict__ w,
    const float* __restrict__ ms, float eps, const float* __restrict__ stats,
    float* __restrict__ sums, float* __restrict__ g_w, float* __restrict__ g_ms) {
  const int c = fold_col(), lane = threadIdx.x & 63;
  if (c >= C) return;
  constexpr int U = 16;
  // the per-column operands and the gradients are loaded with the partials
  // (one round trip, not three: k_gn_bwd_final_tiles' note); the partials at
  // clamped addresses, zeroed when out of range (same sums, same order)
  const float mu = stats[c], sd = stats[C + c], msc = ms[c], wc = w[c];
  const float gw0 = g_w[c], gm0 = g_ms[c];
  float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  for (int b0 = lane; b0 < blocks; b0 += 64 * U) {
    float t[U][5];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int b = min(b0 + 64 * u, blocks - 1);
#pragma unroll
      for (int q = 0; q < 5; ++q) t[u][q] = part[((size_t)b * 5 + q) * C + c];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < 5; ++q) v[q] += b0 + 64 * u < blocks ? t[u][q] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) v[q] = wave_sum(v[q]);
  if (lane != 0) return;
  float dgw, dgms;
  vg::gn_jvp2_cols(v, 1.f / static_cast<float>(N), mu, sd, msc, wc, sums + (size_t)c * 5, dgw, dgms);
  g_w[c] = gw0 + dgw;
  g_ms[c] = gm0 + dgms;
  (void)eps;
}

// u_out = y' = keep [z>0] w (c'/d - o K/d^3);  x_inj = dQ/dx with
// dd/dx = (o - ms a)/(N d), dK/dx = (c' - ms (1 - ms) m_u)/N, dP2/dx = p - ms Sp/N
__global__ void k_gn_jvp2_apply(const float* __restrict__ x, const float* __restrict__ u,
                                const float* __restrict__ gy, long long total, int N, int C,
                                const float* __restrict__ w, const float* __restrict__ b,
                                const float* __restrict__ ms, const float* __restrict__ keep,
                                float eps, const float* __restrict__ stats,
                                const float* __restrict__ sums, float* __restrict__ u_out,
                                float* __restrict__ x_inj) {
  const float inv_n = 1.f / static_cast<float>(N);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % C);
    const float mu = stats[c], d = stats[C + c];
    const float wc = w[c], msc = ms[c];
    const float* sm = sums + (size_t)c * 5;
    const float mup = sm[0], K = sm[1], Sp = sm[2], P1 = sm[3], P2 = sm[4];
    const float xv = x[t], uv = u[t];
    const float o = xv - msc * mu, cp = uv - msc * mup;
    const float z = (o / d) * wc + b[c];
    float mk = z > 0.f ? 1.f : 0.f;
    if (keep) mk *= keep[t];
    const float id = 1.f / d, id2 = id * id, id3 = id2 * id;
    u_out[t] = mk * wc * (cp * id - o * K * id3);
    const float p = gy[t] * mk;
    const float a = (1.f - msc) * mu;
    const float ddx = (o - msc * a) * inv_n * id;
    const float dKx = (cp - msc * (1.f - msc) * mup) * inv_n;
    const float dP2x = p - msc * Sp * inv_n;
    const float g = -P1 * ddx * id2 - (dP2x * K + P2 * dKx) * id3 + 3.f * P2 * K * ddx * id3 * id;
    x_inj[t] = wc * g;
  }
  (void)eps;
}

// ------------------------------------------------ quad elementwise passes
// The scalar passes above index elements with 64-bit t, so every element pays
// a 64-bit `t % C` and `t / seg_elems` (software division) and, in the
// forward, one Philox call for its dropout draw.  The quad forms take four
// consecutive elements of one row per thread (C % 4 == 0, 16-B aligned
// operands, < 2^31 elements; the host checks and otherwise launches the
// scalar forms): 32-bit index math once per quad, float4 loads/stores, one
// Philox block for all four draws (the same values vg_keep gives each
// element), and the per-column operands (weight, bias, mean_scale, every
// segment's statistics and column sums) staged once per workgroup in LDS and
// read as float4 -- per-lane scalar loads of them at a 4-column lane stride
// touched 4x the cache lines of the scalar form and made the quad backward
// slower than the scalar one (7.05 vs 5.91 us; 5.38 with the LDS image).
// Per-element arithmetic is the scalar forms', expression for expression.
// The second-order pass keeps its scalar form (its quad form was slower).
struct F4 {
  float v[4];
};
__device__ __forceinline__ F4 ld4(const float* __restrict__ p) {
  const float4 t = *reinterpret_cast<const float4*>(p);
  return F4{{t.x, t.y, t.z, t.w}};
}
__device__ __forceinline__ void st4(float* __restrict__ p, const F4& a) {
  *reinterpret_cast<float4*>(p) = make_float4(a.v[0], a.v[1], a.v[2], a.v[3]);
}
// LDS image of the per-column operands: w | b | ms | extra[n_extra]
__device__ __forceinline__ void stage_cols(float* sh, const float* __restrict__ w,
                                           const float* __restrict__ b,
                                           const float* __restrict__ ms, int C,
                                           const float* __restrict__ e0, int n0,
                                           const float* __restrict__ e1, int n1) {
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    sh[i] = w[i];
    sh[C + i] = b[i];
    sh[2 * C + i] = ms[i];
  }
  for (int i = threadIdx.x; i < n0; i += blockDim.x) sh[3 * C + i] = e0[i];
  for (int i = threadIdx.x; i < n1; i += blockDim.x) sh[3 * C + n0 + i] = e1[i];
  __syncthreads();
}

__global__ void k_gn_apply4(const float* __restrict__ x, int quads, int N, int C, int S,
                            const float* __restrict__ w, const float* __restrict__ b,
                            const float* __restrict__ ms, const float* __restrict__ keep,
                            float eps, const float* __restrict__ stats, float* __restrict__ y,
                            float p_drop, unsigned long long seed, const long long* __restrict__ iter,
                            unsigned int salt, float* __restrict__ keep_out) {
  extern __shared__ float4 sh4[];
  float* sh = reinterpret_cast<float*>(sh4);
  // the first quad's x / keep are in flight while the column operands are
  // staged (one memory round trip instead of two: the usual single pass)
  const int q0 = blockIdx.x * blockDim.x + threadIdx.x;
  F4 xp = {{0.f, 0.f, 0.f, 0.f}}, kp = {{1.f, 1.f, 1.f, 1.f}};
  if (q0 < quads) {
    xp = ld4(x + 4 * q0);
    if (!iter && keep) kp = ld4(keep + 4 * q0);
  }
  const bool draw = iter != nullptr;
  const long long it = draw ? *iter : 0;
  stage_cols(sh, w, b, ms, C, stats, 2 * C * S, nullptr, 0);
  for (int q = q0; q < quads; q += gridDim.x * blockDim.x) {
    const int t0 = q * 4;
    const int row = t0 / C;
    const int c0 = t0 - row * C;
    const float* st = sh + 3 * C + 2 * C * (row / N);
    const bool first = q == q0;
    const F4 xv = first ? xp : ld4(x + t0);
    F4 k4 = {{1.f, 1.f, 1.f, 1.f}};
    if (draw) {
      const float4 k = vg_keep4_raw(q, salt, it, seed, p_drop);
      k4 = F4{{k.x, k.y, k.z, k.w}};
      if (keep_out) st4(keep_out + t0, k4);
    } else if (keep) {
      k4 = first ? kp : ld4(keep + t0);
    }
    const F4 wv = ld4(sh + c0), bv = ld4(sh + C + c0), mv = ld4(sh + 2 * C + c0);
    const F4 muv = ld4(st + c0), sdv = ld4(st + C + c0);
    F4 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float o = xv.v[j] - muv.v[j] * mv.v[j];
      const float z = (o / sdv.v[j]) * wv.v[j] + bv.v[j];
      r.v[j] = z > 0.f ? z : 0.f;
      if (draw || keep) r.v[j] *= k4.v[j];
    }
    st4(y + t0, r);
  }
}

// The statistics fold and the apply in ONE launch (vg_graphnorm_fwd_gnp on
// narrow layers, where a segment's block partials fit in LDS): every
// workgroup owns kFuseQ quads per thread of one contiguous range and puts
// their x (and keep, or draws their dropout multipliers) in flight; stages the
// slot-0 partials of the segment(s) the range touches into LDS with coalesced
// 16-B loads (a column's partials are 12 C bytes apart in HBM: gathered
// straight from global memory, every lane's load is its own cache line and the
// L1 address path, not bandwidth, bounds the fold); folds them per column in
// exactly k_stats_final_gnp's order (lane l merges blocks l, l + 64, ...
// ascending, then the xor butterfly), so the same bits; and applies as
// k_gn_apply4.  The workgroup holding a segment's first quad stores that
// segment's [mu | d] for the backward.  One dependent launch and the
// statistics' write + read fewer per GraphNorm, for each workgroup reading its
// segment's partials from L2.
constexpr int kFuseThreads = 512;
constexpr int kFuseQ = 2;      // quads per thread
constexpr int kFuseLd = 8;     // float4 partial loads per thread in flight
__global__ void __launch_bounds__(kFuseThreads) k_gn_apply4_gnp(
    const float* __restrict__ x, int quads, int N, int C, const float* __restrict__ w,
    const float* __restrict__ b, const float* __restrict__ ms, const float* __restrict__ keep, float eps,
    const float* __restrict__ gnp, int G, float* __restrict__ stats, float* __restrict__ y, float p_drop,
    unsigned long long seed, const long long* __restrict__ iter, unsigned int salt, float* __restrict__ keep_out,
    int nseg) {
  extern __shared__ float4 sh4[];
  float* sh = reinterpret_cast<float*>(sh4);
  float* pl = sh + 3 * C + 2 * C * nseg;  // the staged partials [nb][C][3]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, waves = kFuseThreads / 64;
  const int q_begin = blockIdx.x * kFuseThreads * kFuseQ;
  const int q_end = min(quads, q_begin + kFuseThreads * kFuseQ);
  const int sg_lo = (4 * q_begin / C) / N, sg_hi = ((4 * q_end - 1) / C) / N;
  const bool draw = iter != nullptr;
  const long long it = draw ? *iter : 0;
  // this thread's quads: x and keep in flight, dropout drawn, during the fold
  F4 xv[kFuseQ], kv[kFuseQ];
#pragma unroll
  for (int j = 0; j < kFuseQ; ++j) {
    const int q = q_begin + threadIdx.x + j * kFuseThreads;
    xv[j] = F4{{0.f, 0.f, 0.f, 0.f}};
    kv[j] = F4{{1.f, 1.f, 1.f, 1.f}};
    if (q < q_end) {
      xv[j] = ld4(x + 4 * q);
      if (draw) {
        const float4 k = vg_keep4_raw(q, salt, it, seed, p_drop);
        kv[j] = F4{{k.x, k.y, k.z, k.w}};
      } else if (keep) {
        kv[j] = ld4(keep + 4 * q);
      }
    }
  }
  for (int i = threadIdx.x; i < C; i += kFuseThreads) {
    sh[i] = w[i];
    sh[C + i] = b[i];
    sh[2 * C + i] = ms[i];
  }
  const int nb = (N + G - 1) / G;
  const int row4 = 3 * C / 4;  // float4s per block's slot-0 partials
  const int total4 = nb * row4;
  for (int sg = sg_lo; sg <= sg_hi; ++sg) {
    const float* src = gnp + (size_t)sg * nb * 2 * C * 3;
    if (sg > sg_lo) __syncthreads();  // the previous segment's fold has read pl
    for (int i0 = threadIdx.x; i0 < total4; i0 += kFuseThreads * kFuseLd) {
      float4 v[kFuseLd];
#pragma unroll
      for (int u = 0; u < kFuseLd; ++u) {
        const int i = i0 + u * kFuseThreads;
        const int r = i / row4;
        v[u] = i < total4 ? *reinterpret_cast<const float4*>(src + (size_t)r * 2 * C * 3 + 4 * (i - r * row4))
                          : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < kFuseLd; ++u) {
        const int i = i0 + u * kFuseThreads;
        if (i < total4) sh4[(3 * C + 2 * C * nseg) / 4 + i] = v[u];
      }
    }
    __syncthreads();
    float* st = sh + 3 * C + 2 * C * (sg - sg_lo);
    for (int c = wave; c < C; c += waves) {
      Welford acc = {0.f, 0.f, 0.f};
      for (int bk = lane; bk < nb; bk += 64) {
        const float* p = pl + (bk * C + c) * 3;
        acc = merge(acc, Welford{p[0], p[1], p[2]});
      }
      acc = wave_merge(acc);
      if (lane == 0) {
        st[c] = acc.mean;
        st[C + c] = gn_denom(acc, sh[2 * C + c], eps);
      }
    }
  }
  __syncthreads();
  // [mu | d] of every segment whose first quad is in this range
  for (int sg = sg_lo; sg <= sg_hi; ++sg) {
    const long long first = (long long)sg * N * C / 4;
    if (first >= q_begin && first < q_end)
      for (int i = threadIdx.x; i < 2 * C; i += kFuseThreads)
        stats[(size_t)sg * 2 * C + i] = sh[3 * C + 2 * C * (sg - sg_lo) + i];
  }
#pragma unroll
  for (int j = 0; j < kFuseQ; ++j) {
    const int q = q_begin + threadIdx.x + j * kFuseThreads;
    if (q >= q_end) break;
    const int t0 = q * 4;
    const int row = t0 / C;
    const int c0 = t0 - row * C;
    const float* st = sh + 3 * C + 2 * C * (row / N - sg_lo);
    if (draw && keep_out) st4(keep_out + t0, kv[j]);
    const F4 wv = ld4(sh + c0), bv = ld4(sh + C + c0), mv = ld4(sh + 2 * C + c0);
    const F4 muv = ld4(st + c0), sdv = ld4(st + C + c0);
    F4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float o = xv[j].v[i] - muv.v[i] * mv.v[i];
      const float z = (o / sdv.v[i]) * wv.v[i] + bv.v[i];
      r.v[i] = z > 0.f ? z : 0.f;
      if (draw || keep) r.v[i] *= kv[j].v[i];
    }
    st4(y + t0, r);
  }
}

__global__ void k_gn_bwd_apply4(const float* __restrict__ x, const float* __restrict__ gy, int quads,
                                int N, int C, int S, const float* __restrict__ w,
                                const float* __restrict__ b, const float* __restrict__ ms,
                                const float* __restrict__ keep, float eps,
                                const float* __restrict__ stats, const float* __restrict__ sums,
                                const float* __restrict__ inj, int inj_off,
                                float* __restrict__ gx) {
  extern __shared__ float4 sh4[];
  float* sh = reinterpret_cast<float*>(sh4);
  const F4 one = {{1.f, 1.f, 1.f, 1.f}}, zero = {{0.f, 0.f, 0.f, 0.f}};
  // the first quad's operands in flight while the column operands are staged
  const int q0 = blockIdx.x * blockDim.x + threadIdx.x;
  F4 xp = zero, gp = zero, kp = one, ip = zero;
  if (q0 < quads) {
    const int t0 = 4 * q0;
    xp = ld4(x + t0);
    gp = ld4(gy + t0);
    if (keep) kp = ld4(keep + t0);
    if (inj && t0 >= inj_off) ip = ld4(inj + (t0 - inj_off));
  }
  stage_cols(sh, w, b, ms, C, stats, 2 * C * S, sums, 2 * C * S);
  const float inv_n = 1.f / static_cast<float>(N);
  for (int q = q0; q < quads; q += gridDim.x * blockDim.x) {
    const int t0 = q * 4;
    const int row = t0 / C;
    const int c0 = t0 - row * C;
    const int sg = row / N;
    const float* st = sh + 3 * C + 2 * C * sg;
    const float* sm = sh + 3 * C + 2 * C * S + 2 * C * sg;
    const bool first = q == q0;
    const F4 xv = first ? xp : ld4(x + t0), gv = first ? gp : ld4(gy + t0);
    const F4 kv = first ? kp : (keep ? ld4(keep + t0) : one);
    const bool has_inj = inj && t0 >= inj_off;
    const F4 iv = first ? ip : (has_inj ? ld4(inj + (t0 - inj_off)) : zero);
    const F4 wv = ld4(sh + c0), bv = ld4(sh + C + c0), mv = ld4(sh + 2 * C + c0);
    const F4 muv = ld4(st + c0), sdv = ld4(st + C + c0), Av = ld4(sm + c0), Bv = ld4(sm + C + c0);
    F4 out;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float g = vg::gn_bwd_elem(xv.v[j], gv.v[j], kv.v[j], keep != nullptr, muv.v[j], sdv.v[j], wv.v[j], bv.v[j],
                                mv.v[j], Av.v[j], Bv.v[j], eps, inv_n);
      if (has_inj) g += iv.v[j];
      out.v[j] = g;
    }
    st4(gx + t0, out);
  }
}

}  // namespace

static inline int chunks_for(int N) {
  const int c = (N + kChunkRows - 1) / kChunkRows;
  return c < 1 ? 1 : (c > kChunks ? kChunks : c);
}

// elementwise passes: about one element per thread (every grid-stride
// iteration is another dependent memory round trip)
static inline int apply_blocks(long long total) {
  int blocks = vg_blocks(total, 256);
  return blocks > kApplyMaxBlocks ? kApplyMaxBlocks : blocks;
}

// quad forms: C % 4 == 0, fewer than 2^31 elements, every [rows, C] operand
// 16-B aligned (operands may be row slices of larger buffers)
constexpr int kQuadLdsFloats = 8192;  // LDS image cap of the quad forms (32 KB)
static inline bool quad_ok(long long total, int C, int lds_floats,
                           std::initializer_list<const void*> ptrs) {
  if (C % 4 != 0 || total >= (1LL << 31) || lds_floats > kQuadLdsFloats) return false;
  for (const void* p : ptrs)
    if (p && (reinterpret_cast<uintptr_t>(p) & 15) != 0) return false;
  return true;
}

// k_gn_apply4_gnp (statistics fold + apply in one launch) when one segment's
// block partials are at most VG_GN_FUSE_BYTES (0: never; the A/B build): every
// workgroup reads them, so only the narrow layers qualify (batch 32: C <= 16)
#ifndef VG_GN_FUSE_BYTES
#define VG_GN_FUSE_BYTES 49152
#endif
constexpr long long kFuseLdsBytes = 160 * 1024;
static inline bool gn_fuse_ok(int N, int C, int G) {
  const long long nb = (N + (long long)G - 1) / G;
  return G > 0 && nb * C * 12 <= (long long)VG_GN_FUSE_BYTES;
}

extern "C" int32_t vg_graphnorm_fwd_gnp_fused(int32_t N, int32_t C, int32_t gnp_rows) {
  return gn_fuse_ok(N, C, gnp_rows) && C % 4 == 0 ? 1 : 0;
}

extern "C" int64_t vg_graphnorm_seg_ws_floats(int32_t segments, int32_t rows_per_segment,
                                              int32_t channels) {
  (void)rows_per_segment;
  return (int64_t)segments * kChunks * channels * 5 + 5 * (int64_t)segments * channels;
}

extern "C" int64_t vg_graphnorm_ws_floats(int32_t num_nodes, int32_t channels) {
  return vg_graphnorm_seg_ws_floats(1, num_nodes, channels);
}

// gnp != NULL: the column statistics from the GAT aggregation's block
// partials (G rows per block) instead of a pass over x
static int gn_fwd(const float* x, int32_t S, int32_t N, int32_t C, const float* weight,
                  const float* bias, const float* mean_scale, const float* keep, float eps, float* y,
                  float* stats, float* ws, float p_drop, uint64_t seed, const int64_t* iter,
                  uint32_t salt, float* keep_out, int32_t* sync, void* stream, const float* gnp = nullptr,
                  int32_t gnp_rows = 0) {
  if (S <= 0 || N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !y || !stats || (!ws && !gnp) ||
      (gnp && (gnp_rows <= 0 || gnp_rows > N)))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const long long total = (long long)S * N * C;
  if (gnp && gn_fuse_ok(N, C, gnp_rows) && quad_ok(total, C, 0, {x, keep, y, keep_out})) {
    const int quads = static_cast<int>(total / 4);
    const int per_wg = kFuseThreads * kFuseQ;
    const int nseg = per_wg * 4 / C / N + 2;  // segments one workgroup's range can touch
    const long long nb = (N + gnp_rows - 1) / gnp_rows;
    const long long lds_f = 3 * C + 2 * C * nseg + nb * C * 3;
    if (lds_f * 4 <= kFuseLdsBytes) {
      static bool attr = false;  // beyond the default 64 KB of dynamic LDS
      if (!attr) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gn_apply4_gnp),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)kFuseLdsBytes);
        attr = true;
      }
      k_gn_apply4_gnp<<<vg_blocks(quads, per_wg), kFuseThreads, lds_f * 4, s>>>(
          x, quads, N, C, weight, bias, mean_scale, keep, eps, gnp, gnp_rows, stats, y, p_drop,
          (unsigned long long)seed, reinterpret_cast<const long long*>(iter), salt, keep_out, nseg);
      VG_CHECK_LAUNCH();
      return 0;
    }
  }
  if (gnp) {
    k_stats_final_gnp<<<dim3(vg_blocks(C, kFoldWaves), S), 64 * kFoldWaves, 0, s>>>(gnp, gnp_rows, N, C, S, mean_scale,
                                                                                 eps, stats);
  } else {
    const int chunks = chunks_for(N);
    dim3 grid(chunks, (C + 63) / 64, S);
    k_stats_partial<float><<<grid, kBlock, 0, s>>>(x, N, C, C, ws, stats, nullptr);
    k_stats_final<<<dim3(vg_blocks(C, kFoldWaves), S), 64 * kFoldWaves, 0, s>>>(ws, chunks, C, S, mean_scale, eps,
                                                                             stats);
  }
  (void)sync;  // former last-block-fold counter: accepted, unused
  const int lds_f = 3 * C + 2 * C * S;
  if (quad_ok(total, C, lds_f, {x, keep, y, keep_out}))
    k_gn_apply4<<<apply_blocks(total / 4), 256, lds_f * 4, s>>>(
        x, static_cast<int>(total / 4), N, C, S, weight, bias, mean_scale, keep, eps, stats, y, p_drop,
        (unsigned long long)seed, reinterpret_cast<const long long*>(iter), salt, keep_out);
  else
    k_gn_apply<<<apply_blocks(total), 256, 0, s>>>(x, total, C, (long long)N * C, weight, bias,
                                                   mean_scale, keep, eps, stats, y, p_drop,
                                                   (unsigned long long)seed,
                                                   reinterpret_cast<const long long*>(iter), salt,
                                                   keep_out);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_fwd_h(const uint16_t* x, int32_t ld, int32_t S, int32_t N, int32_t C,
                                  const float* weight, const float* bias, const float* mean_scale, float eps,
                                  uint16_t* y, int32_t ldy, float* stats, float* ws, void* stream) {
  const int wcols = (C + 7) / 8 * 8;
  if (S <= 0 || N <= 0 || C <= 0 || ld < wcols || ld % 8 || ldy < wcols || ldy % 8 || !x || !weight || !bias ||
      !mean_scale || !y || !stats || !ws)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const _Float16* X = reinterpret_cast<const _Float16*>(x);
  const int chunks = chunks_for(N);
  dim3 grid(chunks, (C + 63) / 64, S);
  k_stats_partial<_Float16><<<grid, kBlock, 0, s>>>(X, N, C, ld, ws, stats, nullptr);
  k_stats_final<<<dim3(vg_blocks(C, kFoldWaves), S), 64 * kFoldWaves, 0, s>>>(ws, chunks, C, S, mean_scale, eps,
                                                                             stats);
  const long long pairs = (long long)S * N * (wcols / 2);
  k_gn_apply_h<<<apply_blocks(pairs), 256, 0, s>>>(X, pairs, C, ld, wcols, (long long)N, weight, bias,
                                                   mean_scale, eps, stats, reinterpret_cast<_Float16*>(y), ldy);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_fwd_h_gnp(const uint16_t* x, int32_t ld, int32_t S, int32_t N, int32_t C,
                                      const float* weight, const float* bias, const float* mean_scale, float eps,
                                      uint16_t* y, int32_t ldy, float* stats, const float* gnp, int32_t gnp_rows,
                                      void* stream) {
  const int wcols = (C + 7) / 8 * 8;
  if (S <= 0 || N <= 0 || C <= 0 || ld < wcols || ld % 8 || ldy < wcols || ldy % 8 || !x || !weight || !bias ||
      !mean_scale || !y || !stats || !gnp || gnp_rows <= 0 || gnp_rows > N)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  k_stats_final_gnp<<<dim3(vg_blocks(C, kFoldWaves), S), 64 * kFoldWaves, 0, s>>>(gnp, gnp_rows, N, C, S, mean_scale,
                                                                               eps, stats);
  const long long pairs = (long long)S * N * (wcols / 2);
  k_gn_apply_h<<<apply_blocks(pairs), 256, 0, s>>>(reinterpret_cast<const _Float16*>(x), pairs, C, ld, wcols,
                                                   (long long)N, weight, bias, mean_scale, eps, stats,
                                                   reinterpret_cast<_Float16*>(y), ldy);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_fwd_seg(const float* x, int32_t S, int32_t N, int32_t C,
                                    const float* weight, const float* bias,
                                    const float* mean_scale, const float* keep, float eps,
                                    float* y, float* stats, float* ws, int32_t* sync,
                                    void* stream) {
  return gn_fwd(x, S, N, C, weight, bias, mean_scale, keep, eps, y, stats, ws, 0.f, 0, nullptr, 0,
                nullptr, sync, stream);
}

extern "C" int vg_graphnorm_fwd_drop(const float* x, int32_t S, int32_t N, int32_t C,
                                     const float* weight, const float* bias,
                                     const float* mean_scale, float p_drop, uint64_t seed,
                                     const int64_t* iter, uint32_t salt, float eps, float* y,
                                     float* keep_out, float* stats, float* ws, int32_t* sync,
                                     void* stream) {
  if (!iter || !(p_drop >= 0.f && p_drop < 1.f)) return VG_EINVAL;  // keep_out NULL: apply, do not store
  return gn_fwd(x, S, N, C, weight, bias, mean_scale, nullptr, eps, y, stats, ws, p_drop, seed,
                iter, salt, keep_out, sync, stream);
}

extern "C" int vg_graphnorm_fwd_gnp(const float* x, int32_t S, int32_t N, int32_t C, const float* weight,
                                    const float* bias, const float* mean_scale, const float* keep, float p_drop,
                                    uint64_t seed, const int64_t* iter, uint32_t salt, float eps, float* y,
                                    float* keep_out, float* stats, const float* gnp, int32_t gnp_rows,
                                    void* stream) {
  if (!gnp || (iter && !(p_drop >= 0.f && p_drop < 1.f)) || (iter && keep)) return VG_EINVAL;
  return gn_fwd(x, S, N, C, weight, bias, mean_scale, keep, eps, y, stats, nullptr, iter ? p_drop : 0.f,
                iter ? seed : 0, iter, iter ? salt : 0, iter ? keep_out : nullptr, nullptr, stream, gnp, gnp_rows);
}

extern "C" int vg_graphnorm_stats(const float* x, int32_t S, int32_t N, int32_t C, const float* mean_scale,
                                  float eps, float* stats, float* ws, void* stream) {
  if (S <= 0 || N <= 0 || C <= 0 || !x || !mean_scale || !stats || !ws) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int chunks = chunks_for(N);
  k_stats_partial<float><<<dim3(chunks, (C + 63) / 64, S), kBlock, 0, s>>>(x, N, C, C, ws, stats, nullptr);
  k_stats_final<<<dim3(vg_blocks(C, kFoldWaves), S), 64 * kFoldWaves, 0, s>>>(ws, chunks, C, S, mean_scale, eps,
                                                                           stats);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_stats_gnp(int32_t S, int32_t N, int32_t C, const float* gnp, int32_t gnp_rows,
                                      const float* mean_scale, float eps, float* stats, void* stream) {
  if (S <= 0 || N <= 0 || C <= 0 || !gnp || !mean_scale || !stats || gnp_rows <= 0 || gnp_rows > N)
    return VG_EINVAL;
  k_stats_final_gnp<<<dim3(vg_blocks(C, kFoldWaves), S), 64 * kFoldWaves, 0, static_cast<hipStream_t>(stream)>>>(
      gnp, gnp_rows, N, C, S, mean_scale, eps, stats);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_fwd(const float* x, int32_t N, int32_t C, const float* weight,
                                const float* bias, const float* mean_scale, const float* keep,
                                float eps, float* y, float* stats, float* ws, void* stream) {
  return vg_graphnorm_fwd_seg(x, 1, N, C, weight, bias, mean_scale, keep, eps, y, stats, ws,
                              nullptr, stream);
}

static void gn_bwd_apply_launch(const float* x, int32_t S, int32_t N, int32_t C, const float* weight,
                                const float* bias, const float* mean_scale, const float* keep, float eps,
                                const float* stats, const float* sums, const float* g_y, float* g_x,
                                const float* inj, int64_t inj_offset, hipStream_t s);

extern "C" int vg_graphnorm_bwd_seg(const float* x, int32_t S, int32_t N, int32_t C,
                                    const float* weight, const float* bias,
                                    const float* mean_scale, const float* keep, float eps,
                                    const float* stats, const float* g_y, float* g_x, float* g_w,
                                    float* g_b, float* g_ms, int32_t accumulate, const float* inj,
                                    int64_t inj_offset, float* ws, int32_t* sync, void* stream) {
  if (S <= 0 || N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !g_y ||
      !ws || (g_w && (!g_b || !g_ms)) || inj_offset < 0)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int chunks = chunks_for(N);
  float* part = ws;
  float* sums = ws + (size_t)S * kChunks * C * 5;
  dim3 grid(chunks, (C + 63) / 64, S);
  k_gn_bwd_partial<<<grid, kBlock, 0, s>>>(x, g_y, N, C, weight, bias, mean_scale, keep, eps,
                                           stats, part, sums, g_w, g_b, g_ms, accumulate, nullptr);
  (void)sync;
  k_gn_bwd_final<<<vg_blocks(C, kFoldWaves), 64 * kFoldWaves, 0, s>>>(part, chunks, C, S, weight, mean_scale, eps,
                                                              stats, sums, g_w, g_b, g_ms, accumulate);
  if (g_x)  // g_x NULL: the column sums only (vg_gat_bwd_gn applies them)
    gn_bwd_apply_launch(x, S, N, C, weight, bias, mean_scale, keep, eps, stats, sums, g_y, g_x, inj, inj_offset, s);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t vg_graphnorm_bwd_sums_offset(int32_t segments, int32_t channels) {
  return (int64_t)segments * kChunks * channels * 5;
}

extern "C" int64_t vg_gemm_gn_tpart_floats(int32_t rows, int32_t channels) {
  return ((int64_t)rows + 63) / 64 * 2 * 2 * (int64_t)(channels > 0 ? channels : 1);
}

extern "C" int vg_graphnorm_bwd_seg_tiles(const float* x, int32_t S, int32_t N, int32_t C,
                                          const float* weight, const float* bias,
                                          const float* mean_scale, const float* keep, float eps,
                                          const float* stats, const float* g_y, const float* tpart,
                                          float* g_x, float* g_w, float* g_b, float* g_ms,
                                          int32_t accumulate, const float* inj, int64_t inj_offset,
                                          float* ws, void* stream) {
  if (S <= 0 || N < 64 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !g_y || !tpart ||
      !ws || (g_w && (!g_b || !g_ms)) || inj_offset < 0)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* sums = ws + (size_t)S * kChunks * C * 5;
  k_gn_bwd_final_tiles<<<vg_blocks(C, kFoldWaves), 64 * kFoldWaves, 0, s>>>(tpart, N, C, S, weight, mean_scale, eps,
                                                                    stats, sums, g_w, g_b, g_ms, accumulate);
  if (g_x)
    gn_bwd_apply_launch(x, S, N, C, weight, bias, mean_scale, keep, eps, stats, sums, g_y, g_x, inj, inj_offset, s);
  VG_CHECK_LAUNCH();
  return 0;
}

static void gn_bwd_apply_launch(const float* x, int32_t S, int32_t N, int32_t C, const float* weight,
                                const float* bias, const float* mean_scale, const float* keep, float eps,
                                const float* stats, const float* sums, const float* g_y, float* g_x,
                                const float* inj, int64_t inj_offset, hipStream_t s) {
  const long long total = (long long)S * N * C;
  const int lds_f = 3 * C + 4 * C * S;
  // the quad form narrows inj_offset to int: only when it fits (as total does)
  if (quad_ok(total, C, lds_f, {x, g_y, keep, g_x, inj}) &&
      (!inj || (inj_offset % 4 == 0 && inj_offset < (1LL << 31))))
    k_gn_bwd_apply4<<<apply_blocks(total / 4), 256, lds_f * 4, s>>>(
        x, g_y, static_cast<int>(total / 4), N, C, S, weight, bias, mean_scale, keep, eps, stats, sums,
        inj, inj ? static_cast<int>(inj_offset) : 0, g_x);
  else
    k_gn_bwd_apply<<<apply_blocks(total), 256, 0, s>>>(x, g_y, total, N, C, weight, bias,
                                                       mean_scale, keep, eps, stats, sums, inj,
                                                       (long long)inj_offset, g_x);
}

extern "C" int vg_graphnorm_bwd(const float* x, int32_t N, int32_t C, const float* weight,
                                const float* bias, const float* mean_scale, const float* keep,
                                float eps, const float* stats, const float* g_y, float* g_x,
                                float* g_w, float* g_b, float* g_ms, float* ws, void* stream) {
  if (!g_w || !g_b || !g_ms) return VG_EINVAL;
  return vg_graphnorm_bwd_seg(x, 1, N, C, weight, bias, mean_scale, keep, eps, stats, g_y, g_x,
                              g_w, g_b, g_ms, 0, nullptr, 0, ws, nullptr, stream);
}

extern "C" int vg_graphnorm_jvp2_part(const float* x, int32_t N, int32_t C, const float* weight,
                                      const float* bias, const float* mean_scale, const float* keep, float eps,
                                      const float* stats, const float* u, const float* g_y, float* u_out,
                                      float* x_inj, float* g_w, float* g_ms, const float* part, int32_t blocks,
                                      float* ws, void* stream) {
  if (N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !u || !g_y || !u_out || !x_inj ||
      !g_w || !g_ms || !part || blocks <= 0 || !ws)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  float* sums = ws + (size_t)kChunks * C * 5;  // the same workspace layout as vg_graphnorm_jvp2
  k_gn_jvp2_final_blk<<<vg_blocks(C, kFoldWaves), 64 * kFoldWaves, 0, s>>>(part, blocks, N, C, weight, mean_scale, eps,
                                                                   stats, sums, g_w, g_ms);
  const long long total = (long long)N * C;
  k_gn_jvp2_apply<<<apply_blocks(total), 256, 0, s>>>(x, u, g_y, total, N, C, weight, bias, mean_scale, keep, eps,
                                                      stats, sums, u_out, x_inj);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_jvp2(const float* x, int32_t N, int32_t C, const float* weight,
                                 const float* bias, const float* mean_scale, const float* keep,
                                 float eps, const float* stats, const float* u, const float* g_y,
                                 float* u_out, float* x_inj, float* g_w, float* g_ms, float* ws,
                                 int32_t* sync, void* stream) {
  if (N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !u || !g_y ||
      !u_out || !x_inj || !g_w || !g_ms || !ws)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int chunks = chunks_for(N);
  float* part = ws;
  float* sums = ws + (size_t)kChunks * C * 5;
  dim3 grid(chunks, (C + 63) / 64);
  if (quad_ok((long long)N * C, C, 0, {x, u, g_y, keep}))
    k_gn_jvp2_partial4<<<grid, kBlock, 0, s>>>(x, u, g_y, N, C, weight, bias, mean_scale, keep, eps, stats, part);
  else
    k_gn_jvp2_partial<<<grid, kBlock, 0, s>>>(x, u, g_y, N, C, weight, bias, mean_scale, keep, eps,
                                              stats, part, sums, g_w, g_ms, nullptr);
  (void)sync;
  k_gn_jvp2_final<<<vg_blocks(C, kFoldWaves), 64 * kFoldWaves, 0, s>>>(part, chunks, N, C, weight, mean_scale, eps,
                                                               stats, sums, g_w, g_ms);
  const long long total = (long long)N * C;
  // scalar form: the quad form (LDS-staged [C][5] sums) measured 5.6-5.7 us
  // per launch against 5.3 here
  k_gn_jvp2_apply<<<apply_blocks(total), 256, 0, s>>>(x, u, g_y, total, N, C, weight, bias,
                                                      mean_scale, keep, eps, stats, sums, u_out,
                                                      x_inj);
  VG_CHECK_LAUNCH();
  return 0;
}

// vg_graphnorm_jvp2 in three launches the caller sequences (include/vgan.h):
// the column-sum partials, the fold (vg_graphnorm_jvp2_fold_src, gat_jvp.hip,
// optionally beside a GAT tangent source pass), the elementwise pass.  The
// same kernels and workspace layout as vg_graphnorm_jvp2: bit-identical.
extern "C" int vg_graphnorm_jvp2_sums(const float* x, int32_t N, int32_t C, const float* weight, const float* bias,
                                      const float* mean_scale, const float* keep, float eps, const float* stats,
                                      const float* u, const float* g_y, float* ws, void* stream) {
  if (N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !u || !g_y || !ws) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int chunks = chunks_for(N);
  dim3 grid(chunks, (C + 63) / 64);
  if (quad_ok((long long)N * C, C, 0, {x, u, g_y, keep}))
    k_gn_jvp2_partial4<<<grid, kBlock, 0, s>>>(x, u, g_y, N, C, weight, bias, mean_scale, keep, eps, stats, ws);
  else
    k_gn_jvp2_partial<<<grid, kBlock, 0, s>>>(x, u, g_y, N, C, weight, bias, mean_scale, keep, eps, stats, ws,
                                              nullptr, nullptr, nullptr, nullptr);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_jvp2_apply(const float* x, int32_t N, int32_t C, const float* weight, const float* bias,
                                       const float* mean_scale, const float* keep, float eps, const float* stats,
                                       const float* u, const float* g_y, float* u_out, float* x_inj, const float* ws,
                                       void* stream) {
  if (N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !u || !g_y || !u_out || !x_inj || !ws)
    return VG_EINVAL;
  const long long total = (long long)N * C;
  k_gn_jvp2_apply<<<apply_blocks(total), 256, 0, static_cast<hipStream_t>(stream)>>>(
      x, u, g_y, total, N, C, weight, bias, mean_scale, keep, eps, stats, ws + (size_t)kChunks * C * 5, u_out, x_inj);
  VG_CHECK_LAUNCH();
  return 0;
}
