// GraphNorm(batch=None) fused with the ReLU and Dropout that follow it in every
// encoder block (models.py:73-75,83-85,193-195,203-205).
//
// Forward   mu, sigma = population column mean / std over all N rows
//           y = keep * relu(w * (x - ms*mu) / (sigma + eps) + b)
// Backward  gz = g_y * keep * [z > 0];  A = sum gz;  B = sum gz * xhat
//           g_x = (w/s)(gz - ms*A/N) - (w*B/(N*s*sigma)) (x - mu)   (0 if sigma == 0,
//           matching torch's std backward mask), g_w = B, g_b = A, g_ms = -mu*w*A/s
//
// The column statistics are a two-level deterministic reduction: R row-chunk
// blocks per 64-column slab produce (count, mean, M2) Welford partials, a
// finalize kernel merges them in a fixed order (Chan's formula), and the
// elementwise kernel applies.  Lanes are packed (col, row-sub) so narrow layers
// (C = 1..32) still use every lane of the wave.
#include "common.h"

namespace {

constexpr int kBlock = 256;
constexpr int kChunks = 64;  // row chunks per column slab

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

__global__ void __launch_bounds__(kBlock) k_stats_partial(const float* __restrict__ x, int N, int C,
                                                          float* __restrict__ part) {
  const Lay ly = lay_for(C);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + (lane & (ly.cw - 1));
  const int rsub = wave * ly.rpw + lane / ly.cw;
  const int rstep = 4 * ly.rpw;
  const int rows_per_chunk = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  const bool col_ok = c < C && (lane & (ly.cw - 1)) < 64;
  Welford w = {0.f, 0.f, 0.f};
  if (col_ok) {
    for (int r = r0 + rsub; r < r1; r += rstep) {
      const float v = x[(size_t)r * C + c];
      w.n += 1.f;
      const float d = v - w.mean;
      w.mean += d / w.n;
      w.m2 += d * (v - w.mean);
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
}

// Merge the per-chunk Welford partials: one 256-thread block per 64 columns,
// wave w merges chunks w, w+4, ... (fixed order), then the 4 waves in LDS.
__global__ void __launch_bounds__(256) k_stats_final(const float* __restrict__ part, int chunks,
                                                     int C, float* __restrict__ stats) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  Welford acc = {0.f, 0.f, 0.f};
  if (c < C)
    for (int k = wave; k < chunks; k += 4) {
      const float* p = part + ((size_t)k * C + c) * 3;
      acc = merge(acc, Welford{p[0], p[1], p[2]});
    }
  __shared__ Welford sw[4][64];
  sw[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < C) {
    Welford r = merge(merge(sw[0][lane], sw[1][lane]), merge(sw[2][lane], sw[3][lane]));
    stats[c] = r.mean;
    stats[C + c] = sqrtf(fmaxf(r.m2 / r.n, 0.f));
  }
}

__global__ void k_gn_apply(const float* __restrict__ x, long long total, int C,
                           const float* __restrict__ w, const float* __restrict__ b,
                           const float* __restrict__ ms, const float* __restrict__ keep,
                           float eps, const float* __restrict__ stats, float* __restrict__ y) {
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % C);
    const float mu = stats[c], sd = stats[C + c];
    const float o = x[t] - mu * ms[c];
    const float z = (o / (sd + eps)) * w[c] + b[c];
    float r = z > 0.f ? z : 0.f;
    if (keep) r *= keep[t];
    y[t] = r;
  }
}

// backward: column partial sums of gz and gz*xhat (plain sums, chunk order)
__global__ void __launch_bounds__(kBlock) k_gn_bwd_partial(
    const float* __restrict__ x, const float* __restrict__ gy, int N, int C,
    const float* __restrict__ w, const float* __restrict__ b, const float* __restrict__ ms,
    const float* __restrict__ keep, float eps, const float* __restrict__ stats,
    float* __restrict__ part) {
  const Lay ly = lay_for(C);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + (lane & (ly.cw - 1));
  const int rsub = wave * ly.rpw + lane / ly.cw;
  const int rstep = 4 * ly.rpw;
  const int rows_per_chunk = (N + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows_per_chunk;
  const int r1 = min(N, r0 + rows_per_chunk);
  float sa = 0.f, sb = 0.f;
  if (c < C) {
    const float mu = stats[c], s = stats[C + c] + eps, wc = w[c], bc = b[c], msc = ms[c];
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
}

__global__ void __launch_bounds__(256) k_gn_bwd_final(
    const float* __restrict__ part, int chunks, int C, const float* __restrict__ w,
    const float* __restrict__ ms, float eps, const float* __restrict__ stats,
    float* __restrict__ sums, float* __restrict__ g_w, float* __restrict__ g_b,
    float* __restrict__ g_ms) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float a = 0.f, bb = 0.f;
  if (c < C)
    for (int k = wave; k < chunks; k += 4) {
      a += part[((size_t)k * C + c) * 2];
      bb += part[((size_t)k * C + c) * 2 + 1];
    }
  __shared__ float red[4][64][2];
  red[wave][lane][0] = a;
  red[wave][lane][1] = bb;
  __syncthreads();
  if (wave == 0 && c < C) {
    a = (red[0][lane][0] + red[1][lane][0]) + (red[2][lane][0] + red[3][lane][0]);
    bb = (red[0][lane][1] + red[1][lane][1]) + (red[2][lane][1] + red[3][lane][1]);
    sums[c] = a;
    sums[C + c] = bb;
    g_w[c] = bb;
    g_b[c] = a;
    g_ms[c] = -stats[c] * w[c] * a / (stats[C + c] + eps);
  }
}

__global__ void k_gn_bwd_apply(const float* __restrict__ x, const float* __restrict__ gy,
                               long long total, int N, int C, const float* __restrict__ w,
                               const float* __restrict__ b, const float* __restrict__ ms,
                               const float* __restrict__ keep, float eps,
                               const float* __restrict__ stats, const float* __restrict__ sums,
                               float* __restrict__ gx) {
  const float inv_n = 1.f / static_cast<float>(N);
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int c = static_cast<int>(t % C);
    const float mu = stats[c], sd = stats[C + c], s = sd + eps;
    const float wc = w[c], msc = ms[c];
    const float xv = x[t];
    const float xh = (xv - mu * msc) / s;
    const float z = xh * wc + b[c];
    float gz = z > 0.f ? gy[t] : 0.f;
    if (keep) gz *= keep[t];
    const float A = sums[c], B = sums[C + c];
    float g = (wc / s) * (gz - msc * A * inv_n);
    if (sd > 0.f) g -= (wc * B * inv_n / (s * sd)) * (xv - mu);
    gx[t] = g;
  }
}

}  // namespace

extern "C" int64_t vg_graphnorm_ws_floats(int32_t num_nodes, int32_t channels) {
  (void)num_nodes;
  return (int64_t)kChunks * channels * 3 + 2 * (int64_t)channels;
}

static inline int chunks_for(int N) { return N < kChunks * 16 ? (N + 15) / 16 : kChunks; }

extern "C" int vg_graphnorm_fwd(const float* x, int32_t N, int32_t C, const float* weight,
                                const float* bias, const float* mean_scale, const float* keep,
                                float eps, float* y, float* stats, float* ws, void* stream) {
  if (N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !y || !stats || !ws)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int chunks = chunks_for(N);
  dim3 grid(chunks, (C + 63) / 64);
  k_stats_partial<<<grid, kBlock, 0, s>>>(x, N, C, ws);
  k_stats_final<<<vg_blocks(C, 64), 256, 0, s>>>(ws, chunks, C, stats);
  const long long total = (long long)N * C;
  int blocks = vg_blocks(total, 256);
  if (blocks > 2048) blocks = 2048;
  k_gn_apply<<<blocks, 256, 0, s>>>(x, total, C, weight, bias, mean_scale, keep, eps, stats, y);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_graphnorm_bwd(const float* x, int32_t N, int32_t C, const float* weight,
                                const float* bias, const float* mean_scale, const float* keep,
                                float eps, const float* stats, const float* g_y, float* g_x,
                                float* g_w, float* g_b, float* g_ms, float* ws, void* stream) {
  if (N <= 0 || C <= 0 || !x || !weight || !bias || !mean_scale || !stats || !g_y || !g_x ||
      !g_w || !g_b || !g_ms || !ws)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int chunks = chunks_for(N);
  float* part = ws;
  float* sums = ws + (size_t)kChunks * C * 3;
  dim3 grid(chunks, (C + 63) / 64);
  k_gn_bwd_partial<<<grid, kBlock, 0, s>>>(x, g_y, N, C, weight, bias, mean_scale, keep, eps,
                                           stats, part);
  k_gn_bwd_final<<<vg_blocks(C, 64), 256, 0, s>>>(part, chunks, C, weight, mean_scale, eps,
                                                  stats, sums, g_w, g_b, g_ms);
  const long long total = (long long)N * C;
  int blocks = vg_blocks(total, 256);
  if (blocks > 2048) blocks = 2048;
  k_gn_bwd_apply<<<blocks, 256, 0, s>>>(x, g_y, total, N, C, weight, bias, mean_scale, keep, eps,
                                        stats, sums, g_x);
  VG_CHECK_LAUNCH();
  return 0;
}
