// GraphNorm(+ReLU+Dropout) second-order column fold, shared by the
// stand-alone fold launch (graphnorm.hip, k_gn_jvp2_final) and the launch that
// runs it beside a GAT tangent source pass (gat_jvp.hip, k_jvp2_fold_src):
// one formula, so the two launches agree bit for bit.
//
// Column terms from the five column sums v = [sum u, sum xt u, sum p, sum p u,
// sum p xt] (xt = x - mu) of the statistics-chunk partials, with stats =
// [mu | d] (graphnorm.hip's header for the derivation):
//   m_u = mean u, a = (1 - ms) mu = mean o, K = mean(o c') = mean(o u) - ms m_u a,
//   P1 = sum p c' = sum p u - ms m_u Sp, P2 = sum p o = sum p xt + a Sp;
//   Q / w = P1/d - P2 K/d^3  ->  g_w += Q / w;
//   g_ms += w d(Q/w)/dms with dd/dms = -a mu/d, dK/dms = -2 a m_u,
//           dP1/dms = -m_u Sp, dP2/dms = -mu Sp.
// sums <- [m_u, K, Sp, P1, P2] for the elementwise pass.
#pragma once
#include "common.h"

#ifndef VG_GN_CHUNKS
#define VG_GN_CHUNKS 256
#endif
#ifndef VG_GN_CHUNK_ROWS
#define VG_GN_CHUNK_ROWS 32
#endif

namespace vg {

constexpr int kGnChunks = VG_GN_CHUNKS;         // max row chunks per column slab
constexpr int kGnChunkRows = VG_GN_CHUNK_ROWS;  // rows per statistics chunk

__host__ __device__ inline int gn_chunks_for(int N) {
  const int c = (N + kGnChunkRows - 1) / kGnChunkRows;
  return c < 1 ? 1 : (c > kGnChunks ? kGnChunks : c);
}

__device__ __forceinline__ void gn_jvp2_cols(const float v[5], float inv_n, float mu, float d, float msc, float wc,
                                             float* __restrict__ sm, float& dgw, float& dgms) {
  const float mup = v[0] * inv_n, Sp = v[2];
  const float a = (1.f - msc) * mu;
  const float K = (v[1] + a * v[0]) * inv_n - msc * mup * a;
  const float P1 = v[3] - msc * mup * Sp;
  const float P2 = v[4] + a * Sp;
  const float id = 1.f / d, id2 = id * id, id3 = id2 * id;
  const float dd = -a * mu * id, dK = -2.f * a * mup;
  sm[0] = mup;
  sm[1] = K;
  sm[2] = Sp;
  sm[3] = P1;
  sm[4] = P2;
  dgw = P1 * id - P2 * K * id3;
  dgms = wc * (-mup * Sp * id - P1 * dd * id2 + mu * Sp * K * id3 - P2 * dK * id3 + 3.f * P2 * K * dd * id3 * id);
}

// One wave folds column c: lane l sums chunks l, l + 64, ... (four loads in
// flight per lane), the xor butterfly, then lane 0 forms the column terms and
// adds the weight / mean_scale gradients.  part [chunks][C][5].
__device__ __forceinline__ void gn_jvp2_fold_col(const float* __restrict__ part, int chunks, int N, int C,
                                                 const float* __restrict__ w, const float* __restrict__ ms,
                                                 const float* __restrict__ stats, float* __restrict__ sums,
                                                 float* __restrict__ g_w, float* __restrict__ g_ms, int c,
                                                 int lane) {
  constexpr int kU = kGnChunks / 64;
  float v[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
  float t[kU][5];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const int k = lane + 64 * u;
#pragma unroll
    for (int q = 0; q < 5; ++q) t[u][q] = k < chunks ? part[((size_t)k * C + c) * 5 + q] : 0.f;
  }
#pragma unroll
  for (int q = 0; q < 5; ++q) {
#pragma unroll
    for (int u = 0; u < kU; ++u) v[q] += t[u][q];
    for (int off = 1; off < 64; off <<= 1) v[q] += __shfl_xor(v[q], off, 64);
  }
  if (lane != 0) return;
  float dgw, dgms;
  gn_jvp2_cols(v, 1.f / static_cast<float>(N), stats[c], stats[C + c], ms[c], w[c], sums + (size_t)c * 5, dgw, dgms);
  g_w[c] += dgw;
  g_ms[c] += dgms;
}

}  // namespace vg
