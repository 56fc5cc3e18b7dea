// Small kernels of the explicit WGAN-GP critic engine (vgan/critic.py).
//
// vg_critic_input  builds the stacked discriminator input of one critic
//                  iteration: rows [0,N) real, [N,2N) fake, [2N,3N) the
//                  gradient-penalty interpolate (trainer.py:298-301, 319-320):
//                  X[c*N + n] = [ matched_voxel_x[n] | label_c[n] ],
//                  label_mix = eps*real + (1-eps)*soft  (rounded as torch does:
//                  two products then one add, no fused multiply-add); with
//                  copies = 4 the rows [3N,4N) are zeroed (the engine's
//                  tangent rows, whose label columns vg_gp_head fills).
// vg_gp_head       from g = dD(mix)/dlabel [N,K] and the stacked scores:
//                  gp = lambda * mean_n (|g_n| - 1)^2            (trainer.py:313-316)
//                  loss = mean(D(fake)) - mean(D(real)) + gp       (trainer.py:326-328)
//                  u0 = dgp/dg = (2 lambda / N) (|g_n| - 1)/|g_n| g_n   (the seed of the
//                  engine's tangent pass; 0 where |g_n| = 0, as torch's norm backward).
//                  Row-parallel; per-block sums folded in block order by the
//                  last block to finish (deterministic).
#include "common.h"

namespace {

// iter != NULL: eps[n] is not read but drawn here -- the uniform vg_rng_fill
// (kind 1) writes for element n under the same (seed, *iter, salt): lane n % 4
// of the Philox block n / 4, bit for bit -- one launch fewer per iteration.
__global__ void k_critic_input(const float* __restrict__ mvx, int N, int F,
                               const float* __restrict__ real, const float* __restrict__ hard,
                               const float* __restrict__ soft, const float* __restrict__ eps,
                               int K, int copies, float* __restrict__ X, unsigned long long seed = 0,
                               const long long* __restrict__ iter = nullptr, unsigned int salt = 0) {
  const long long it = iter ? *iter : 0;
  const int W = F + K;
  const long long total = (long long)copies * N * W;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const long long r = t / W;
    const int c = static_cast<int>(t - r * W);
    const int cp = static_cast<int>(r / N);
    const long long n = r - (long long)cp * N;
    float v;
    if (cp == 3) {
      v = 0.f;
    } else if (c < F) {
      v = mvx[n * F + c];
    } else {
      const long long e = n * K + (c - F);
      if (cp == 0) v = real[e];
      else if (cp == 1) v = hard[e];
      else {
        float a;
        if (iter) {
          const uint4 r = vg_keep_block(n >> 2, salt, it, seed);
          const int l = static_cast<int>(n & 3);
          a = static_cast<float>((l == 0 ? r.x : l == 1 ? r.y : l == 2 ? r.z : r.w) >> 8) * (1.0f / 16777216.0f);
        } else {
          a = eps[n];
        }
        v = __fadd_rn(__fmul_rn(a, real[e]), __fmul_rn(__fsub_rn(1.f, a), soft[e]));
      }
    }
    X[t] = v;
  }
}

// One row per thread over ceil(N/256) blocks (the row's KMAX <= 8 classes in
// registers: the former runtime-indexed row buffer lived in scratch); per-block
// partial sums of (gp, real, fake) -- wave xor trees, then the four waves in
// order -- go to `part`; the last block folds them in block order.  The
// hand-off uses the single-lane release / acquire form (vg_last_block).  The
// former 1024-thread form (LDS tree with ten barriers, every thread fencing)
// took 20.8 us per call.
template <int KMAX>
__global__ void __launch_bounds__(256) k_gp_head(const float* __restrict__ g, int N, int K,
                                                 const float* __restrict__ scores, float lambda,
                                                 float* __restrict__ u0, int ldu,
                                                 float* __restrict__ part, int* counter,
                                                 float* __restrict__ out) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const float coef = 2.f * lambda / static_cast<float>(N);
  float gp = 0.f, sr = 0.f, sf = 0.f;
  const int n = blockIdx.x * 256 + t;
  if (n < N) {
    const float* gr = g + (size_t)n * K;
    float v[KMAX];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      v[k] = k < K ? gr[k] : 0.f;
      ss = fmaf(v[k], v[k], ss);
    }
    const float nrm = sqrtf(ss);
    const float d = nrm - 1.f;
    gp = d * d;
    const float f = nrm > 0.f ? coef * d / nrm : 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
      if (k < K) u0[(size_t)n * ldu + k] = f * v[k];
    sr = scores[n];
    sf = scores[N + n];
  }
  for (int off = 32; off > 0; off >>= 1) {
    gp += __shfl_xor(gp, off, 64);
    sr += __shfl_xor(sr, off, 64);
    sf += __shfl_xor(sf, off, 64);
  }
  __shared__ float red[4][3];
  if (lane == 0) {
    red[wave][0] = gp;
    red[wave][1] = sr;
    red[wave][2] = sf;
  }
  __syncthreads();
  if (t < 3) part[blockIdx.x * 3 + t] = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
  if (vg_last_block(counter) && t == 0) {
    float a = 0.f, b = 0.f, c = 0.f;
    for (int k = 0; k < (int)gridDim.x; ++k) {
      a += part[k * 3];
      b += part[k * 3 + 1];
      c += part[k * 3 + 2];
    }
    const float fn = static_cast<float>(N);
    const float gpv = a / fn * lambda;
    out[0] = (c / fn - b / fn) + gpv;
    out[1] = gpv;
  }
}

}  // namespace

extern "C" int vg_critic_input(const float* mvx, int32_t N, int32_t F, const float* real,
                               const float* hard, const float* soft, const float* eps, int32_t K,
                               int32_t copies, float* X, void* stream) {
  if (N <= 0 || F < 0 || K <= 0 || (F > 0 && !mvx) || !real || !hard || !soft || !eps || !X ||
      (copies != 3 && copies != 4))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int blocks = vg_blocks((long long)copies * N * (F + K), 256);
  if (blocks > 4096) blocks = 4096;
  k_critic_input<<<blocks, 256, 0, s>>>(mvx, N, F, real, hard, soft, eps, K, copies, X);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_critic_input_drawn(const float* mvx, int32_t N, int32_t F, const float* real,
                                     const float* hard, const float* soft, uint64_t seed, const int64_t* iter,
                                     uint32_t salt, int32_t K, int32_t copies, float* X, void* stream) {
  if (N <= 0 || F < 0 || K <= 0 || (F > 0 && !mvx) || !real || !hard || !soft || !iter || !X ||
      (copies != 3 && copies != 4))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int blocks = vg_blocks((long long)copies * N * (F + K), 256);
  if (blocks > 4096) blocks = 4096;
  k_critic_input<<<blocks, 256, 0, s>>>(mvx, N, F, real, hard, soft, nullptr, K, copies, X,
                                        (unsigned long long)seed, reinterpret_cast<const long long*>(iter), salt);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t vg_gp_head_ws_floats(int32_t N) { return 3 * (int64_t)vg_blocks(N, 256); }

extern "C" int vg_gp_head(const float* g, int32_t N, int32_t K, const float* scores, float lambda,
                          float* u0, int32_t ldu, float* out, float* workspace, int32_t* sync,
                          void* stream) {
  if (N <= 0 || K <= 0 || ldu < K || !g || !scores || !u0 || !out || !workspace || !sync)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // classes live in registers: instantiations for K <= 8 (the path's
  // NUM_CLASSES = 7), 16 and 32; wider rows are refused (vgan.h)
  const int blocks = vg_blocks(N, 256);
  if (K <= 8)
    k_gp_head<8><<<blocks, 256, 0, s>>>(g, N, K, scores, lambda, u0, ldu, workspace, sync, out);
  else if (K <= 16)
    k_gp_head<16><<<blocks, 256, 0, s>>>(g, N, K, scores, lambda, u0, ldu, workspace, sync, out);
  else if (K <= 32)
    k_gp_head<32><<<blocks, 256, 0, s>>>(g, N, K, scores, lambda, u0, ldu, workspace, sync, out);
  else
    return VG_EINVAL;
  VG_CHECK_LAUNCH();
  return 0;
}
