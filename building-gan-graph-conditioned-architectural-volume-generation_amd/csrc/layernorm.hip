// nn.LayerNorm(C) followed by LeakyReLU(slope) in one pass -- the
// [Linear -> LayerNorm -> LeakyReLU(0.2)] blocks of the generator's MLPs
// (models.py:33-47 matched_features_encoder, :49-66 mlp_encoder, :92-113
// decoder).  torch runs LayerNorm and the activation as separate kernels
// (three more in the backward); here:
//
//   forward   one row per group of L lanes:  mu, rstd = 1/sqrt(var + eps)
//             (biased variance, as torch), z = (x - mu) rstd gamma + beta,
//             y = lrelu(z); mu / rstd saved for the backward
//   backward  gz = g_y lrelu'(z);  g_x = rstd (gz gamma - mean(gz gamma)
//             - xhat mean(gz gamma xhat));  block partials of sum gz xhat
//             (g_gamma) and sum gz (g_beta), folded in a fixed order
//
// Row statistics are two-pass in registers (the whole row is held by the
// group: C <= 8 L = 512 floats).
#include "rowgroup.h"

namespace {

using namespace vg;

#ifndef VG_LN_MAX_BLOCKS
#define VG_LN_MAX_BLOCKS 512
#endif
constexpr int kMaxBlocks = VG_LN_MAX_BLOCKS;

template <int L, int CPL>
__global__ void __launch_bounds__(kBlock) k_ln_act_fwd(const float* __restrict__ x, int N, int C,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps,
                                                       float slope, float* __restrict__ y,
                                                       float* __restrict__ mean,
                                                       float* __restrict__ rstd) {
  const GroupIdx g = group_index<L>();
  if (g.row >= N) return;
  const int c0 = g.lane * CPL;
  Vec<CPL> v, ga, be;
  load_row<CPL, false>(v, x + (size_t)g.row * C, c0, C);
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) s += v.v[q];
  const float mu = group_sum<L>(s) / static_cast<float>(C);
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q)
    if (c0 + q < C) {
      const float d = v.v[q] - mu;
      ss = fmaf(d, d, ss);
    }
  const float var = group_sum<L>(ss) / static_cast<float>(C);
  const float rs = rsqrtf(var + eps);
  load_row<CPL, false>(ga, gamma, c0, C);
  load_row<CPL, false>(be, beta, c0, C);
  Vec<CPL> o;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const float z = fmaf((v.v[q] - mu) * rs, ga.v[q], be.v[q]);
    o.v[q] = z > 0.f ? z : z * slope;
  }
  store_row<CPL, false>(o, y + (size_t)g.row * C, c0, C);
  if (g.lane == 0 && mean) {
    mean[g.row] = mu;
    rstd[g.row] = rs;
  }
}

template <int L, int CPL, bool VEC = false>  // VEC: row vectors as float4 (C % CPL == 0, 16-B aligned rows)
__global__ void __launch_bounds__(kBlock) k_ln_act_bwd(const float* __restrict__ x, int N, int C,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float slope,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gy,
                                                       float* __restrict__ gx,
                                                       float* __restrict__ part) {
  constexpr int G = kBlock / L;
  const int grp = threadIdx.x / L, lane = threadIdx.x & (L - 1);
  const int c0 = lane * CPL;
  Vec<CPL> ga, be, pg, pb;
  load_row<CPL, false>(ga, gamma, c0, C);
  load_row<CPL, false>(be, beta, c0, C);
#pragma unroll
  for (int q = 0; q < CPL; ++q) pg.v[q] = pb.v[q] = 0.f;
  const float inv_c = 1.f / static_cast<float>(C);
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  for (int i = lb * G + grp; i < N; i += gridDim.x * G) {
    const float mu = mean[i], rs = rstd[i];
    Vec<CPL> v, g;
    load_row<CPL, VEC>(v, x + (size_t)i * C, c0, C);
    load_row<CPL, VEC>(g, gy + (size_t)i * C, c0, C);
    float s1 = 0.f, s2 = 0.f;
    Vec<CPL> xh, gz;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      xh.v[q] = (v.v[q] - mu) * rs;
      const float z = fmaf(xh.v[q], ga.v[q], be.v[q]);
      gz.v[q] = (c0 + q < C) ? (z > 0.f ? g.v[q] : g.v[q] * slope) : 0.f;
      const float a = gz.v[q] * ga.v[q];
      s1 += a;
      s2 = fmaf(a, xh.v[q], s2);
      pg.v[q] = fmaf(gz.v[q], xh.v[q], pg.v[q]);
      pb.v[q] += gz.v[q];
    }
    const float m1 = group_sum<L>(s1) * inv_c, m2 = group_sum<L>(s2) * inv_c;
    Vec<CPL> o;
#pragma unroll
    for (int q = 0; q < CPL; ++q) o.v[q] = rs * (gz.v[q] * ga.v[q] - m1 - xh.v[q] * m2);
    store_row<CPL, VEC>(o, gx + (size_t)i * C, c0, C);
  }
  Vec<CPL> vals[2] = {pg, pb};
  block_partials<L, CPL>(vals, 2, C, part);
}

// g_gamma[c] / g_beta[c] (= or +=) sum over partial rows, fixed order
__global__ void __launch_bounds__(1024) k_ln_fold(const float* __restrict__ part, int rows, int C,
                                                  int acc, float* __restrict__ g_gamma,
                                                  float* __restrict__ g_beta) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int w = blockIdx.x * 64 + lane;
  const int W = 2 * C;
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
    float* o = w < C ? g_gamma + w : g_beta + (w - C);
    *o = acc ? *o + v : v;
  }
}

// rows of up to 64 / 128 / 256 / 512 channels: L lanes x CPL channels
inline bool ln_shape(int C, int& L, int& CPL) {
  if (C <= 0 || C > 512) return false;
  if (C <= 64) { L = 16; CPL = 4; }
  else if (C <= 128) { L = 32; CPL = 4; }
  else if (C <= 256) { L = 64; CPL = 4; }
  else { L = 64; CPL = 8; }
  return true;
}

// float4 row vectors in k_ln_act_bwd: whole lane vectors in or out of C, aligned rows
inline bool ln_vec(int C, int cpl, const float* x, const float* gy, const float* gx) {
  auto al = [](const float* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return C % cpl == 0 && C % 4 == 0 && al(x) && al(gy) && al(gx);
}

#define VG_LN_DISPATCH(C, CALL)                                                  \
  do {                                                                           \
    int l_, c_;                                                                  \
    if (!ln_shape(C, l_, c_)) return VG_EINVAL;                                  \
    if (l_ == 16) { constexpr int L_ = 16, CPL_ = 4; CALL; }                     \
    else if (l_ == 32) { constexpr int L_ = 32, CPL_ = 4; CALL; }                \
    else if (c_ == 4) { constexpr int L_ = 64, CPL_ = 4; CALL; }                 \
    else { constexpr int L_ = 64, CPL_ = 8; CALL; }                              \
  } while (0)

}  // namespace

extern "C" int vg_ln_act_fwd(const float* x, int32_t N, int32_t C, const float* gamma,
                             const float* beta, float eps, float slope, float* y, float* mean,
                             float* rstd, void* stream) {
  if (N <= 0 || !x || !gamma || !beta || !y || (mean == nullptr) != (rstd == nullptr))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  VG_LN_DISPATCH(C, (k_ln_act_fwd<L_, CPL_><<<grid_for(N, L_), kBlock, 0, s>>>(
                        x, N, C, gamma, beta, eps, slope, y, mean, rstd)));
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t vg_ln_act_bwd_ws_floats(int32_t C) { return (int64_t)kMaxBlocks * 2 * C; }

extern "C" int vg_ln_act_bwd(const float* x, int32_t N, int32_t C, const float* gamma,
                             const float* beta, float slope, const float* mean, const float* rstd,
                             const float* g_y, float* g_x, float* g_gamma, float* g_beta,
                             int32_t accumulate, float* workspace, void* stream) {
  if (N <= 0 || !x || !gamma || !beta || !mean || !rstd || !g_y || !g_x || !g_gamma || !g_beta ||
      !workspace)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int grid = 0;
  VG_LN_DISPATCH(C, (grid = grid_for(N, L_) < kMaxBlocks ? grid_for(N, L_) : kMaxBlocks,
                     (ln_vec(C, CPL_, x, g_y, g_x)
                          ? k_ln_act_bwd<L_, CPL_, true><<<grid, kBlock, 0, s>>>(x, N, C, gamma, beta, slope, mean,
                                                                                rstd, g_y, g_x, workspace)
                          : k_ln_act_bwd<L_, CPL_><<<grid, kBlock, 0, s>>>(x, N, C, gamma, beta, slope, mean, rstd,
                                                                          g_y, g_x, workspace))));
  k_ln_fold<<<vg_blocks(2 * C, 64), 1024, 0, s>>>(workspace, grid, C, accumulate, g_gamma, g_beta);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_ln_act_bwd_deferred(const float* x, int32_t N, int32_t C, const float* gamma,
                                      const float* beta, float slope, const float* mean,
                                      const float* rstd, const float* g_y, float* g_x,
                                      float* g_gamma, float* g_beta, int32_t accumulate,
                                      float* workspace, vg_fold* folds_out, int32_t* n_out,
                                      void* stream) {
  if (N <= 0 || !x || !gamma || !beta || !mean || !rstd || !g_y || !g_x || !g_gamma || !g_beta ||
      !workspace || !folds_out || !n_out)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int grid = 0;
  VG_LN_DISPATCH(C, (grid = grid_for(N, L_) < kMaxBlocks ? grid_for(N, L_) : kMaxBlocks,
                     (ln_vec(C, CPL_, x, g_y, g_x)
                          ? k_ln_act_bwd<L_, CPL_, true><<<grid, kBlock, 0, s>>>(x, N, C, gamma, beta, slope, mean,
                                                                                rstd, g_y, g_x, workspace)
                          : k_ln_act_bwd<L_, CPL_><<<grid, kBlock, 0, s>>>(x, N, C, gamma, beta, slope, mean, rstd,
                                                                          g_y, g_x, workspace))));
  // partial rows [grid][2C] = [gamma | beta]: two folds for vg_fold_batch
  folds_out[0] = vg_fold{g_gamma, C, C, C, accumulate, 1, {{workspace, grid, 2 * C}, {nullptr, 0, 0}}};
  folds_out[1] = vg_fold{g_beta, C, C, C, accumulate, 1, {{workspace + C, grid, 2 * C}, {nullptr, 0, 0}}};
  *n_out = 2;
  VG_CHECK_LAUNCH();
  return 0;
}
