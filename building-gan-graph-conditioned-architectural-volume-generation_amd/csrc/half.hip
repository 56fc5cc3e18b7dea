// f16 inference path of the generator forward (BASELINE.json configs[4]:
// "Generator-only inference sweep ... fp16").  Activations are IEEE binary16
// rows with a padded leading dimension (ld % 8 == 0, pad columns held at 0),
// every kernel accumulates in f32, and parameters other than the GEMM weights
// stay f32.
//
//   vg_hgemm        y = epilogue(A W^T) on the f16 MFMA (v_mfma_f32_32x32x16_f16):
//                   bias + activation, LayerNorm + LeakyReLU (models.py:22-31
//                   MLP blocks), or the GATConv projection with the attention
//                   projections a_src / a_dst in the epilogue (models.py:72,82)
//   vg_hgat_fwd     GATConv edge softmax + CSR gather-sum + bias on f16 rows
//                   (the scatter kernel, gat_fused.hip's k_gat_fwd_cp on half
//                   the bytes)
//
// GraphNorm + ReLU over f16 rows is vg_graphnorm_fwd_h (graphnorm.hip).
//
// GEMM layout: one wave owns 32 output rows and every output column (M <= 128,
// NT = ceil(M/32) 32x32 accumulator tiles).  Lane l holds A[row l&31][k+8(l>>5)
// .. +7] and W[col l&31][same k] as 16-byte loads (rows padded to 8 halves), so
// no LDS staging is needed; W (<= 135 KB) stays in L1/L2.  The LayerNorm and
// attention epilogues reduce a row across the 32 lanes of its half-wave.
#include "common.h"
#include "rowgroup.h"

typedef _Float16 h8_t __attribute__((ext_vector_type(8)));
typedef float f16x_t __attribute__((ext_vector_type(16)));

namespace {

using vg::kBlock;

constexpr int kEpiBias = 0, kEpiLN = 1, kEpiAtt = 2;

__device__ __forceinline__ h8_t load_h8(const _Float16* p, bool ok) {
  if (!ok) return h8_t{0, 0, 0, 0, 0, 0, 0, 0};
  return *reinterpret_cast<const h8_t*>(p);
}

// The GraphNorm + ReLU of the previous GAT block applied to the A operand as
// it is loaded (vg_hgat_lin_att_gn): its column operands and every segment's
// [mu | d] staged in LDS, the expression of k_gn_apply_h element for element
// (the same f16 values reach the MFMA), pad columns 0.
constexpr int kGnaMaxSeg = 16;
constexpr int kGnaFloats = 3 * 128 + 2 * 128 * kGnaMaxSeg;
struct HGnA {
  const float *w, *b, *ms, *stats;
  int C, S, seg_rows;
};

__device__ __forceinline__ h8_t gn_a(h8_t a, int k0, const float* __restrict__ g, const float* __restrict__ st,
                                     int C) {
  h8_t o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + j;
    float z = 0.f;
    if (k < C) {
      z = ((static_cast<float>(a[j]) - st[k] * g[256 + k]) / st[C + k]) * g[k] + g[128 + k];
      z = z > 0.f ? z : 0.f;
    }
    o[j] = static_cast<_Float16>(z);
  }
  return o;
}

__device__ __forceinline__ float half_sum32(float v) {  // sum over the 32 lanes of a half-wave
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Sums of 16 values across the 32 lanes of a half-wave, transposed: each
// xor step hands half of the lane's remaining values to its partner and keeps
// the other half (16 -> 8 -> 4 -> 2 -> 1), so 16 shuffles reduce all 16
// instead of 5 each (80).  Returns the total of value index
// i = 8 b4 + 4 b3 + 2 b2 + b1 (bits of the lane id r), held by lanes 2i and
// 2i + 1.  Summation order differs from half_sum32 (f32 rounding).
__device__ __forceinline__ float half_sum32x16(const float (&v)[16], int r) {
  float a[8];
  {
    const bool b = (r & 16) != 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float keep = b ? v[k + 8] : v[k], give = b ? v[k] : v[k + 8];
      a[k] = keep + __shfl_xor(give, 16, 64);
    }
  }
  float c[4];
  {
    const bool b = (r & 8) != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float keep = b ? a[k + 4] : a[k], give = b ? a[k] : a[k + 4];
      c[k] = keep + __shfl_xor(give, 8, 64);
    }
  }
  float d[2];
  {
    const bool b = (r & 4) != 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float keep = b ? c[k + 2] : c[k], give = b ? c[k] : c[k + 2];
      d[k] = keep + __shfl_xor(give, 4, 64);
    }
  }
  const bool b1 = (r & 2) != 0;
  float e = (b1 ? d[1] : d[0]) + __shfl_xor(b1 ? d[0] : d[1], 2, 64);
  return e + __shfl_xor(e, 1, 64);
}

// The inverse: lanes 2i, 2i + 1 hold the value of index i (half_sum32x16's
// layout); every lane of the half-wave gets all 16 (15 shuffles).
__device__ __forceinline__ void half_gather32x16(float x, int r, float (&out)[16]) {
  float a1[2], a2[4], a3[8];
  {
    const bool b = (r & 2) != 0;
    const float o = __shfl_xor(x, 2, 64);
    a1[0] = b ? o : x;
    a1[1] = b ? x : o;
  }
  {
    const bool b = (r & 4) != 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const float o = __shfl_xor(a1[k], 4, 64);
      a2[k] = b ? o : a1[k];
      a2[k + 2] = b ? a1[k] : o;
    }
  }
  {
    const bool b = (r & 8) != 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float o = __shfl_xor(a2[k], 8, 64);
      a3[k] = b ? o : a2[k];
      a3[k + 4] = b ? a2[k] : o;
    }
  }
  {
    const bool b = (r & 16) != 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float o = __shfl_xor(a3[k], 16, 64);
      out[k] = b ? o : a3[k];
      out[k + 8] = b ? a3[k] : o;
    }
  }
}

#ifndef VG_HGEMM_XRED
#define VG_HGEMM_XRED 1  // the attention epilogue's row sums by half_sum32x16 (0: half_sum32 per row)
#endif
#ifndef VG_HGEMM_XRED_LN
#define VG_HGEMM_XRED_LN 1  // the LayerNorm epilogue's mean / variance the same way, gathered back
#endif

__device__ __forceinline__ float act_apply(float v, int act, float slope) {
  if (act == 1) return v > 0.f ? v : 0.f;
  if (act == 2) return v > 0.f ? v : v * slope;
  return v;
}

// Waves per SIMD the register allocation targets (0: the compiler's choice).
// Left to itself hipcc kept the accumulators in AGPRs beside 120 VGPRs, 184
// registers a lane: 2 waves a SIMD, two workgroups a CU, so the sweep's
// 1,024-workgroup LayerNorm GEMMs ran in two rounds.  At 4 every k_hgemm
// instantiation fits 128 registers without a spill: the 131k-row LayerNorm
// GEMMs 30.8 -> 26.1 us (K = 128), 41.4 -> 32.7 (K = 272), 59.6 -> 46.8
// (K = 528) (tools/hgemm_ln_probe.py, profiles/r06_hgemm_ln_probe.txt).
#ifndef VG_HGEMM_WPE
#define VG_HGEMM_WPE 4
#endif
template <int NT, int EPI, bool OUTF32, bool GNA = false>
__global__ void __launch_bounds__(256)
#if VG_HGEMM_WPE
__attribute__((amdgpu_waves_per_eu(VG_HGEMM_WPE)))
#endif
k_hgemm(
    const _Float16* __restrict__ A, int lda, const _Float16* __restrict__ W, int ldw, int N, int M, int K,
    const float* __restrict__ bias, int act, float slope, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, const float* __restrict__ att_s,
    const float* __restrict__ att_d, float* __restrict__ a_s, float* __restrict__ a_d, void* __restrict__ out,
    int ldo, const HGnA gna = HGnA{}) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = (xcd_remap(blockIdx.x, gridDim.x) * 4 + wave) * 32;
  const bool live = row0 < N;  // every wave joins the W staging (block barriers)
  const int r = lane & 31, hh = lane >> 5;
  const _Float16* ap = A + (size_t)min(row0 + r, N - 1) * lda + 8 * hh;
  bool wok[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) wok[t] = 32 * t + r < M;
  f16x_t acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] = 0.f;

  // W is staged through LDS in chunks of 32 k (two MFMA steps), shared by the
  // block's 4 waves; rows padded to 40 halves (conflict-free 16-byte reads).
  // A fragments come straight from global memory (each row is read once).
  constexpr int kWLoads = NT * 32 * 4 / 256;  // 16-byte W pieces per thread per chunk
  __shared__ h8_t Ws[2][NT * 32][5];
  h8_t wreg[kWLoads > 0 ? kWLoads : 1];
  auto load_w = [&](int k0) {
#pragma unroll
    for (int q = 0; q < kWLoads; ++q) {
      const int idx = threadIdx.x + 256 * q;
      const int c = idx >> 2, j = idx & 3;
      wreg[q] = load_h8(W + (size_t)c * ldw + k0 + 8 * j, c < M && k0 + 8 * j < K);
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int q = 0; q < kWLoads; ++q) {
      const int idx = threadIdx.x + 256 * q;
      Ws[buf][idx >> 2][idx & 3] = wreg[q];
    }
  };
  if constexpr (NT == 1) {  // 128 pieces: the first 128 threads
    if (threadIdx.x < 128) {
      const int c = threadIdx.x >> 2, j = threadIdx.x & 3;
      Ws[0][c][j] = load_h8(W + (size_t)c * ldw + 8 * j, c < M && 8 * j < K);
    }
  } else {
    load_w(0);
    store_w(0);
  }
  __shared__ float gsh[GNA ? kGnaFloats : 1];
  const float* gst = gsh;  // this lane's row's segment statistics (GNA)
  if constexpr (GNA) {
    for (int i = threadIdx.x; i < gna.C; i += 256) {
      gsh[i] = gna.w[i];
      gsh[128 + i] = gna.b[i];
      gsh[256 + i] = gna.ms[i];
    }
    for (int i = threadIdx.x; i < 2 * gna.C * gna.S; i += 256) gsh[384 + i] = gna.stats[i];
    gst = gsh + 384 + 2 * gna.C * (min(row0 + r, N - 1) / gna.seg_rows);
  }
  __syncthreads();
  const int nchunks = (K + 31) / 32;
  h8_t a0 = load_h8(ap, 8 * hh < K), a1 = load_h8(ap + 16, 16 + 8 * hh < K);
  for (int kc = 0; kc < nchunks; ++kc) {
    const int buf = kc & 1;
    const int kn = 32 * (kc + 1);
    const bool more = kc + 1 < nchunks;
    h8_t w1 = h8_t{0, 0, 0, 0, 0, 0, 0, 0};
    if (more) {
      if constexpr (NT == 1) {
        if (threadIdx.x < 128) {
          const int c = threadIdx.x >> 2, j = threadIdx.x & 3;
          w1 = load_h8(W + (size_t)c * ldw + kn + 8 * j, c < M && kn + 8 * j < K);
        }
      } else {
        load_w(kn);
      }
    }
    const h8_t an0 = load_h8(ap + kn, more && kn + 8 * hh < K);
    const h8_t an1 = load_h8(ap + kn + 16, more && kn + 16 + 8 * hh < K);
    if constexpr (GNA) {
      a0 = gn_a(a0, 32 * kc + 8 * hh, gsh, gst, gna.C);
      a1 = gn_a(a1, 32 * kc + 16 + 8 * hh, gsh, gst, gna.C);
    }
    if (live) {
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0, Ws[buf][32 * t + r][hh],
                                                                                   acc[t], 0, 0, 0);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a1, Ws[buf][32 * t + r][2 + hh],
                                                                                   acc[t], 0, 0, 0);
    }
    if (more) {
      if constexpr (NT == 1) {
        if (threadIdx.x < 128) Ws[buf ^ 1][threadIdx.x >> 2][threadIdx.x & 3] = w1;
      } else {
        store_w(buf ^ 1);
      }
    }
    __syncthreads();
    a0 = an0;
    a1 = an1;
  }
  if (!live) return;

  // acc[t][i]: column 32t + r, row (i&3) + 8(i>>2) + 4hh
  float cb[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) cb[t] = (bias && wok[t]) ? bias[32 * t + r] : 0.f;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[t][i] += cb[t];

  if constexpr (EPI == kEpiLN) {
    const float inv_m = 1.f / (float)M;
    float g[NT], be[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      g[t] = wok[t] ? gamma[32 * t + r] : 0.f;
      be[t] = wok[t] ? beta[32 * t + r] : 0.f;
    }
    if constexpr (VG_HGEMM_XRED_LN) {
      // two-pass statistics of the 16 rows: transposed sums, gathered back;
      // one 16-float array (the sums, then each row's mean, then its
      // reciprocal deviation), the accumulators centred in place
      float v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v[i] = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) v[i] += wok[t] ? acc[t][i] : 0.f;
      }
      half_gather32x16(half_sum32x16(v, r) * inv_m, r, v);
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t][i] -= v[i];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        v[i] = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) v[i] += wok[t] ? acc[t][i] * acc[t][i] : 0.f;
      }
      half_gather32x16(rsqrtf(half_sum32x16(v, r) * inv_m + eps), r, v);
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const float y = acc[t][i] * v[i] * g[t] + be[t];
          acc[t][i] = y > 0.f ? y : y * slope;
        }
    } else
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float s = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) s += wok[t] ? acc[t][i] : 0.f;
      const float mean = half_sum32(s) * inv_m;
      float q = 0.f;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float d = acc[t][i] - mean;
        q += wok[t] ? d * d : 0.f;
      }
      const float rstd = rsqrtf(half_sum32(q) * inv_m + eps);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const float v = (acc[t][i] - mean) * rstd * g[t] + be[t];
        acc[t][i] = v > 0.f ? v : v * slope;
      }
    }
  } else if constexpr (EPI == kEpiAtt) {
    float vs[NT], vd[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      vs[t] = wok[t] ? att_s[32 * t + r] : 0.f;
      vd[t] = wok[t] ? att_d[32 * t + r] : 0.f;
    }
    if constexpr (VG_HGEMM_XRED) {
      float ps[16], pd[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        ps[i] = 0.f;
        pd[i] = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          ps[i] = fmaf(acc[t][i], vs[t], ps[i]);
          pd[i] = fmaf(acc[t][i], vd[t], pd[i]);
        }
      }
      const float ss = half_sum32x16(ps, r), sd = half_sum32x16(pd, r);
      const int i = 8 * ((r >> 4) & 1) + 4 * ((r >> 3) & 1) + 2 * ((r >> 2) & 1) + ((r >> 1) & 1);
      const int row = row0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if ((r & 1) == 0 && row < N) {
        a_s[row] = ss;
        a_d[row] = sd;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float ps = 0.f, pd = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          ps = fmaf(acc[t][i], vs[t], ps);
          pd = fmaf(acc[t][i], vd[t], pd);
        }
        ps = half_sum32(ps);
        pd = half_sum32(pd);
        const int row = row0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
        if (r == 0 && row < N) {
          a_s[row] = ps;
          a_d[row] = pd;
        }
      }
    }
  } else {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[t][i] = act_apply(acc[t][i], act, slope);
  }

  // store: columns < M; f16 rows also get their pad columns (M .. M rounded
  // up to 8) as 0 -- ldo is only the row stride (out may be a column slice)
  const int wcols = OUTF32 ? M : (M + 7) / 8 * 8;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int col = 32 * t + r;
    if (col >= wcols) continue;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int row = row0 + (i & 3) + 8 * (i >> 2) + 4 * hh;
      if (row >= N) continue;
      const float v = col < M ? acc[t][i] : 0.f;
      if constexpr (OUTF32)
        static_cast<float*>(out)[(size_t)row * ldo + col] = v;
      else
        static_cast<_Float16*>(out)[(size_t)row * ldo + col] = (_Float16)v;
    }
  }
}

// ---- GATConv aggregation over f16 rows (Cp = padded channels, C real) -------
template <int CPL>
struct alignas(2 * CPL) HVec {
  _Float16 v[CPL];
};

template <int CPL>
__device__ __forceinline__ void load_hrow(float* dst, const _Float16* __restrict__ base) {
  HVec<CPL> t = *reinterpret_cast<const HVec<CPL>*>(base);
#pragma unroll
  for (int q = 0; q < CPL; ++q) dst[q] = (float)t.v[q];
}

// GNP: also the following GraphNorm's column partials over the rows' f16
// outputs (vg::gnp_block: segment-aligned blocks of kBlock / L rows, the
// statistics vg_graphnorm_fwd_h would form from the stored halves), so the
// GraphNorm folds them (vg_graphnorm_fwd_h_gnp) instead of re-reading the
// output; every group stays to the block barrier (a group past its segment
// recomputes the segment's last row and stores nothing).
template <int L, int CPL, bool GNP = false>
__global__ void __launch_bounds__(kBlock) k_hgat_fwd(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C, int ld,
    const _Float16* __restrict__ h, const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ bias, float slope, _Float16* __restrict__ out, int ldo, float* __restrict__ gnp = nullptr,
    int seg_rows = 0) {
  constexpr int T = 4;  // edges per lane kept in registers
  vg::GroupIdx g = vg::group_index<L>();
  vg::GnpRows gr{0, 0, N};
  if constexpr (GNP) {
    gr = vg::gnp_rows<kBlock / L>(seg_rows);
    g.row = gr.row0 + threadIdx.x / L;
  }
  const bool live = g.row < gr.end;
  if (!GNP && !live) return;
  const int i = live ? g.row : gr.end - 1;
  const int beg = row_ptr[i], end = row_ptr[i + 1];
  const int deg = end - beg;
  const float ad = a_dst[i];
  int s_t[T];
  float e_t[T];
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    const int k = beg + g.lane + t * L;
    s_t[t] = 0;
    e_t[t] = -INFINITY;
    if (k < end) {
      s_t[t] = col[k];
      e_t[t] = lrelu(a_src[s_t[t]] + ad, slope);
      m = fmaxf(m, e_t[t]);
    }
  }
  for (int k = beg + g.lane + T * L; k < end; k += L) m = fmaxf(m, lrelu(a_src[col[k]] + ad, slope));
  m = group_max<L>(m);
  float ssum = 0.f;
#pragma unroll
  for (int t = 0; t < T; ++t)
    if (beg + g.lane + t * L < end) {
      e_t[t] = expf(e_t[t] - m);
      ssum += e_t[t];
    }
  for (int k = beg + g.lane + T * L; k < end; k += L) ssum += expf(lrelu(a_src[col[k]] + ad, slope) - m);
  const float inv = 1.f / (group_sum<L>(ssum) + vg::kSoftmaxEps);

  const int c0 = g.lane * CPL;
  float acc[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc[q] = 0.f;
  const int dreg = deg < T * L ? deg : T * L;
  for (int j0 = 0; j0 < dreg; j0 += 4) {
    const int nj = dreg - j0 < 4 ? dreg - j0 : 4;
    float hv[4][CPL];
    float a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < nj) {
        const int j = j0 + u;
        const int t = j / L;
        const int sv = t == 0 ? s_t[0] : t == 1 ? s_t[1] : t == 2 ? s_t[2] : s_t[3];
        const float av = t == 0 ? e_t[0] : t == 1 ? e_t[1] : t == 2 ? e_t[2] : e_t[3];
        const int s = __shfl(sv, g.base + (j & (L - 1)), 64);
        a[u] = __shfl(av, g.base + (j & (L - 1)), 64) * inv;
        load_hrow<CPL>(hv[u], h + (size_t)s * ld + c0);
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < nj)
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc[q] = fmaf(a[u], hv[u][q], acc[q]);
  }
  for (int j = T * L; j < deg; ++j) {  // very long rows
    const int s = col[beg + j];
    const float a = expf(lrelu(a_src[s] + ad, slope) - m) * inv;
    float hv[CPL];
    load_hrow<CPL>(hv, h + (size_t)s * ld + c0);
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc[q] = fmaf(a, hv[q], acc[q]);
  }
  HVec<CPL> o;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = c0 + q;
    o.v[q] = (_Float16)(c < C ? acc[q] + bias[c] : 0.f);
  }
  if (live) *reinterpret_cast<HVec<CPL>*>(out + (size_t)i * ldo + c0) = o;
  if constexpr (GNP) {
    float v[CPL];
#pragma unroll
    for (int q = 0; q < CPL; ++q) v[q] = static_cast<float>(o.v[q]);
    vg::gnp_block<L, CPL>(v, g.row, gr, C, c0, 0, C, gnp);
  }
}

}  // namespace

extern "C" int vg_hgemm(const uint16_t* a, int32_t lda, const uint16_t* w, int32_t ldw, int32_t n, int32_t m,
                        int32_t k, const float* bias, int32_t act, float slope, void* out, int32_t ldo,
                        int32_t out_f32, void* stream) {
  if (n <= 0 || m <= 0 || m > 128 || k <= 0 || k % 8 || lda % 8 || ldw % 8 || lda < k || ldw < k || !a || !w ||
      !out || act < 0 || act > 2 || (out_f32 ? ldo < m : (ldo % 8 || ldo < (m + 7) / 8 * 8)))
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const _Float16* A = reinterpret_cast<const _Float16*>(a);
  const _Float16* W = reinterpret_cast<const _Float16*>(w);
  const int grid = (n + 127) / 128;
  const int nt = (m + 31) / 32;
#define VG_HG(NT_, F32_)                                                                                   \
  k_hgemm<NT_, kEpiBias, F32_><<<grid, 256, 0, s>>>(A, lda, W, ldw, n, m, k, bias, act, slope, nullptr, \
                                                    nullptr, 0.f, nullptr, nullptr, nullptr, nullptr, out, ldo)
  if (out_f32) {
    if (nt == 1) VG_HG(1, true); else if (nt == 2) VG_HG(2, true); else VG_HG(4, true);
  } else {
    if (nt == 1) VG_HG(1, false); else if (nt == 2) VG_HG(2, false); else VG_HG(4, false);
  }
#undef VG_HG
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_hgemm_ln_act(const uint16_t* a, int32_t lda, const uint16_t* w, int32_t ldw, int32_t n,
                               int32_t m, int32_t k, const float* bias, const float* gamma, const float* beta,
                               float eps, float slope, uint16_t* out, int32_t ldo, void* stream) {
  if (n <= 0 || m <= 0 || m > 128 || k <= 0 || k % 8 || lda % 8 || ldw % 8 || ldo % 8 || lda < k || ldw < k ||
      ldo < (m + 7) / 8 * 8 || !a || !w || !gamma || !beta || !out)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const _Float16* A = reinterpret_cast<const _Float16*>(a);
  const _Float16* W = reinterpret_cast<const _Float16*>(w);
  const int grid = (n + 127) / 128;
  const int nt = (m + 31) / 32;
#define VG_HG(NT_)                                                                                          \
  k_hgemm<NT_, kEpiLN, false><<<grid, 256, 0, s>>>(A, lda, W, ldw, n, m, k, bias, 0, slope, gamma, beta, eps, \
                                                   nullptr, nullptr, nullptr, nullptr, out, ldo)
  if (nt == 1) VG_HG(1); else if (nt == 2) VG_HG(2); else VG_HG(4);
#undef VG_HG
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_hgat_lin_att(const uint16_t* x, int32_t ldx, const uint16_t* w, int32_t ldw, int32_t n,
                               int32_t cin, int32_t cout, const float* att_src, const float* att_dst,
                               uint16_t* h, int32_t ldh, float* a_src, float* a_dst, void* stream) {
  if (n <= 0 || cout <= 0 || cout > 128 || cin <= 0 || cin % 8 || ldx % 8 || ldw % 8 || ldh % 8 || ldx < cin ||
      ldw < cin || ldh < (cout + 7) / 8 * 8 || !x || !w || !att_src || !att_dst || !h ||
      !a_src || !a_dst)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const _Float16* A = reinterpret_cast<const _Float16*>(x);
  const _Float16* W = reinterpret_cast<const _Float16*>(w);
  const int grid = (n + 127) / 128;
  const int nt = (cout + 31) / 32;
#define VG_HG(NT_)                                                                                       \
  k_hgemm<NT_, kEpiAtt, false><<<grid, 256, 0, s>>>(A, ldx, W, ldw, n, cout, cin, nullptr, 0, 0.f, nullptr, \
                                                    nullptr, 0.f, att_src, att_dst, a_src, a_dst, h, ldh)
  if (nt == 1) VG_HG(1); else if (nt == 2) VG_HG(2); else VG_HG(4);
#undef VG_HG
  VG_CHECK_LAUNCH();
  return 0;
}


extern "C" int32_t vg_hgat_gna_max_segments(void) { return kGnaMaxSeg; }

extern "C" int vg_hgat_lin_att_gn(const uint16_t* x, int32_t ldx, const uint16_t* w, int32_t ldw, int32_t n,
                                  int32_t cin, int32_t cout, const float* att_src, const float* att_dst, uint16_t* h,
                                  int32_t ldh, float* a_src, float* a_dst, const float* gn_weight,
                                  const float* gn_bias, const float* gn_mean_scale, const float* stats,
                                  int32_t segments, int32_t seg_rows, int32_t gn_channels, void* stream) {
  if (n <= 0 || cout <= 0 || cout > 128 || cin <= 0 || cin % 8 || cin > 128 || ldx % 8 || ldw % 8 || ldh % 8 ||
      ldx < cin || ldw < cin || ldh < (cout + 7) / 8 * 8 || !x || !w || !att_src || !att_dst || !h || !a_src ||
      !a_dst || !gn_weight || !gn_bias || !gn_mean_scale || !stats || segments <= 0 || segments > kGnaMaxSeg ||
      seg_rows <= 0 || (int64_t)segments * seg_rows != n || gn_channels <= 0 || gn_channels > cin ||
      (gn_channels + 7) / 8 * 8 != cin)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const _Float16* A = reinterpret_cast<const _Float16*>(x);
  const _Float16* W = reinterpret_cast<const _Float16*>(w);
  const HGnA g{gn_weight, gn_bias, gn_mean_scale, stats, gn_channels, segments, seg_rows};
  const int grid = (n + 127) / 128;
  const int nt = (cout + 31) / 32;
#define VG_HG(NT_)                                                                                             \
  k_hgemm<NT_, kEpiAtt, false, true><<<grid, 256, 0, s>>>(A, ldx, W, ldw, n, cout, cin, nullptr, 0, 0.f, nullptr, \
                                                          nullptr, 0.f, att_src, att_dst, a_src, a_dst, h, ldh, g)
  if (nt == 1) VG_HG(1); else if (nt == 2) VG_HG(2); else VG_HG(4);
#undef VG_HG
  VG_CHECK_LAUNCH();
  return 0;
}

// lanes per destination row of the f16 aggregation, by row width ld (halves).
// The first form gave every row 8-16 lanes of 2-16 B each: a 16-32-B row took
// 8 load instructions with most of the wave's lanes idle on the ~6-edge
// softmax, and the wide rows moved 8-16 B a lane.  Measured at the sweep's
// shapes (131k rows, tools/hgat_probe.py, profiles/r06_hgat_lanes_probe.txt),
// us per launch, first form -> now: ld 8 (2 lanes x 8 B) 8.4-8.6 -> 5.5-5.8;
// ld 16 (4 x 8 B) 9.0 -> 6.9; ld 32 (2 x 32 B) 11.3 -> 9.2; ld 64 (4 x 32 B)
// 23.0 -> 15.5; ld 128 (8 x 32 B) 45.7 -> 33.9.  A/B builds: VG_HGAT_L<ld>.
#ifndef VG_HGAT_L8
#define VG_HGAT_L8 2
#endif
#ifndef VG_HGAT_L16
#define VG_HGAT_L16 4
#endif
#ifndef VG_HGAT_L32
#define VG_HGAT_L32 2
#endif
#ifndef VG_HGAT_L64
#define VG_HGAT_L64 4
#endif
#ifndef VG_HGAT_L128
#define VG_HGAT_L128 8
#endif
constexpr int kHNarrowL = VG_HGAT_L8, kHNarrowL16 = VG_HGAT_L16;
constexpr int kHL32 = VG_HGAT_L32, kHL64 = VG_HGAT_L64, kHL128 = VG_HGAT_L128;

// lanes per row the aggregation uses for a row of ld halves (0: unsupported)
static int hgat_lanes(int ld) {
  switch (ld) {
    case 8: return kHNarrowL;
    case 16: return kHNarrowL16;
    case 32: return kHL32;
    case 64: return kHL64;
    case 128: return kHL128;
    default: return 0;
  }
}

static int hgat_launch(const int32_t* row_ptr, const int32_t* col, int n, int c, int ld, const _Float16* H,
                       const float* a_src, const float* a_dst, const float* bias, float slope, _Float16* O, int ldo,
                       float* gnp, int seg_rows, hipStream_t s) {
  // gnp: segment-aligned blocks, S * ceil(seg_rows / G)
  auto grid = [&](int L) {
    if (!gnp) return vg::grid_for(n, L);
    const int G = kBlock / L;
    return (n / seg_rows) * ((seg_rows + G - 1) / G);
  };
#define VG_HA(L_, CPL_)                                                                                            \
  do {                                                                                                             \
    if (gnp)                                                                                                       \
      k_hgat_fwd<L_, CPL_, true><<<grid(L_), kBlock, 0, s>>>(row_ptr, col, n, c, ld, H, a_src, a_dst, bias, slope, \
                                                             O, ldo, gnp, seg_rows);                               \
    else                                                                                                           \
      k_hgat_fwd<L_, CPL_><<<grid(L_), kBlock, 0, s>>>(row_ptr, col, n, c, ld, H, a_src, a_dst, bias, slope, O,    \
                                                       ldo);                                                       \
  } while (0)
  if (ld == 8) VG_HA(kHNarrowL, 8 / kHNarrowL);
  else if (ld == 16) VG_HA(kHNarrowL16, 16 / kHNarrowL16);
  else if (ld == 32) VG_HA(kHL32, 32 / kHL32);
  else if (ld == 64) VG_HA(kHL64, 64 / kHL64);
  else if (ld == 128) VG_HA(kHL128, 128 / kHL128);
  else return VG_EINVAL;
#undef VG_HA
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_hgat_fwd(const int32_t* row_ptr, const int32_t* col, int32_t n, int32_t c, int32_t ld,
                           const uint16_t* h, const float* a_src, const float* a_dst, const float* bias, float slope,
                           uint16_t* out, int32_t ldo, void* stream) {
  if (n <= 0 || c <= 0 || ld % 8 || ldo % 8 || ldo < ld || ld < c || ld > 128 || !row_ptr || !col || !h || !a_src ||
      !a_dst || !bias || !out)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const _Float16* H = reinterpret_cast<const _Float16*>(h);
  _Float16* O = reinterpret_cast<_Float16*>(out);
  return hgat_launch(row_ptr, col, n, c, ld, H, a_src, a_dst, bias, slope, O, ldo, nullptr, 0, s);
}

// VG_HGAT_GNP=0 (A/B build): no partials (rows 0), the sweep takes the
// GraphNorm's own statistics pass
#ifndef VG_HGAT_GNP
#define VG_HGAT_GNP 1
#endif
extern "C" int32_t vg_hgat_gnp_rows(int32_t n, int32_t ld) {
  const int L = hgat_lanes(ld);
  return VG_HGAT_GNP && n > 0 && L > 0 ? kBlock / L : 0;
}

extern "C" int64_t vg_hgat_gnp_floats(int32_t n, int32_t ld) {
  const int g = vg_hgat_gnp_rows(n, ld);
  if (g == 0) return 0;
  // segment-aligned blocks: S * ceil(seg_rows / g) <= ceil(n / g) + S, S <= n / g
  return 2 * (((int64_t)n + g - 1) / g) * 2 * (int64_t)ld * 3;
}

extern "C" int vg_hgat_fwd_gnp(const int32_t* row_ptr, const int32_t* col, int32_t n, int32_t c, int32_t ld,
                               const uint16_t* h, const float* a_src, const float* a_dst, const float* bias,
                               float slope, uint16_t* out, int32_t ldo, int32_t seg_rows, float* gnp, void* stream) {
  if (n <= 0 || c <= 0 || ld % 8 || ldo % 8 || ldo < ld || ld < c || ld > 128 || !row_ptr || !col || !h || !a_src ||
      !a_dst || !bias || !out || !gnp || seg_rows < vg_hgat_gnp_rows(n, ld) || n % seg_rows)
    return VG_EINVAL;
  return hgat_launch(row_ptr, col, n, c, ld, reinterpret_cast<const _Float16*>(h), a_src, a_dst, bias, slope,
                     reinterpret_cast<_Float16*>(out), ldo, gnp, seg_rows, static_cast<hipStream_t>(stream));
}
