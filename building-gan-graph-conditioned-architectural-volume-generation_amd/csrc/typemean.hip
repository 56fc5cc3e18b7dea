// Program -> voxel "cross-graph pointer": type-matched mean pooling.
//
// Reference (models.py:122-129 and :230-237): for every type t present among
// the voxels, if any program node has type t, every voxel of type t receives
// the mean feature row of ALL program nodes of type t in the mini-batch;
// otherwise zeros.  That loop costs ~7 iterations x (2 boolean masks, a
// `.sum() > 0` host sync, a masked mean, a masked write) per forward.
//
// Here: one 1024-thread workgroup reduces the program nodes into per-type sums
// and counts (16 waves, each accumulating rows into its own LDS slice -- no
// atomics, fixed order -> deterministic), then a grid-wide gather writes the
// pooled rows straight into the caller's (possibly wider, concatenated)
// feature matrix.  No host synchronisation, capturable.
#include "common.h"

namespace {

constexpr int kWaves = 16;
constexpr int kMaxTypes = 16;
constexpr int kMaxFeat = 63;  // lane kMaxFeat.. counts rows

__global__ void __launch_bounds__(1024) k_type_sums(const float* __restrict__ lx,
                                                    const int64_t* __restrict__ lt, int n_local,
                                                    int F, int n_types,
                                                    float* __restrict__ table) {
  __shared__ float acc[kWaves][kMaxTypes][kMaxFeat + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int t = 0; t < n_types; ++t) acc[wave][t][lane] = 0.f;
  __syncthreads();
  for (int r = wave; r < n_local; r += kWaves) {
    const int64_t t = lt[r];
    if (t < 0 || t >= n_types) continue;
    if (lane < F) acc[wave][t][lane] += lx[(size_t)r * F + lane];
    else if (lane == kMaxFeat) acc[wave][t][kMaxFeat] += 1.f;
  }
  __syncthreads();
  // table[t][f] = mean (f < F), table[t][F] = count
  for (int idx = threadIdx.x; idx < n_types * 64; idx += blockDim.x) {
    const int t = idx / 64, f = idx % 64;
    if (f >= F && f != kMaxFeat) continue;
    float s = 0.f;
    for (int w = 0; w < kWaves; ++w) s += acc[w][t][f];
    if (f == kMaxFeat) {
      table[t * (F + 1) + F] = s;
    } else {
      float cnt = 0.f;
      for (int w = 0; w < kWaves; ++w) cnt += acc[w][t][kMaxFeat];
      table[t * (F + 1) + f] = cnt > 0.f ? s / cnt : 0.f;
    }
  }
}

__global__ void k_type_gather(const int64_t* __restrict__ vt, int n_voxel, int F, int n_types,
                              const float* __restrict__ table, float* __restrict__ out,
                              int stride, int col0) {
  const long long total = (long long)n_voxel * F;
  for (long long idx = blockIdx.x * (long long)blockDim.x + threadIdx.x; idx < total;
       idx += (long long)gridDim.x * blockDim.x) {
    const int v = static_cast<int>(idx / F), f = static_cast<int>(idx % F);
    const int64_t t = vt[v];
    float val = 0.f;
    if (t >= 0 && t < n_types && table[t * (F + 1) + F] > 0.f) val = table[t * (F + 1) + f];
    out[(size_t)v * stride + col0 + f] = val;
  }
}

}  // namespace

extern "C" int vg_type_mean(const float* local_x, const int64_t* local_type, int32_t n_local,
                            int32_t feat, const int64_t* voxel_type, int32_t n_voxel,
                            int32_t n_types, float* out, int32_t out_stride, int32_t out_col0,
                            float* workspace, void* stream) {
  if (n_local < 0 || n_voxel <= 0 || feat <= 0 || feat > kMaxFeat || n_types <= 0 ||
      n_types > kMaxTypes || !voxel_type || !out || !workspace || out_stride < out_col0 + feat ||
      (n_local > 0 && (!local_x || !local_type)))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  k_type_sums<<<1, 1024, 0, s>>>(local_x, local_type, n_local, feat, n_types, workspace);
  const long long total = (long long)n_voxel * feat;
  int blocks = vg_blocks(total, 256);
  if (blocks > 2048) blocks = 2048;
  k_type_gather<<<blocks, 256, 0, s>>>(voxel_type, n_voxel, feat, n_types, workspace, out,
                                       out_stride, out_col0);
  VG_CHECK_LAUNCH();
  return 0;
}
