// Row-local chains of narrow linear layers in ONE launch: the discriminator's
// decoder (models.py:273-279 / reference models.py:212-222: Linear 64 -> 32 ->
// 16 -> 8 -> 1 with ReLU between) in the critic engine's four passes
// (vgan/critic.py): the forward (pass A), the adjoint chains g_in = (g_out W)
// [z > 0] (passes B and D) and the tangent chain u_out = (u W^T) [z > 0]
// (pass C).  Each layer was one vg_gemm launch of 8-38k rows x <= 64
// columns, i.e. a dependent ~7 us launch moving a few MB; here a workgroup
// carries 64 rows through the whole chain: every layer's weights staged once
// in LDS in [out][in] order, the rows as LDS images between layers, 4 lanes
// per row (chain_layer_p), each layer's output stored for the backward.  f32
// FMAs in k order; the MFMA GEMMs sum in another order (f32 rounding).
#include "common.h"

namespace {

constexpr int kChainMax = 4;    // layers per launch

struct ChainLayer {
  const float* w;     // wt 0: [out][in] (y = x W^T); wt 1: [in][out] (y = x W)
  const float* bias;  // [out] or NULL
  const float* aux;   // act 3: mask source [rows][ld_aux] (y = aux > 0 ? y : 0)
  float* out;         // [rows][ld_out] or NULL
  int ld_aux, ld_out, wt, act;
};

struct ChainDesc {
  ChainLayer l[kChainMax];
  const float* x;
  int ldx, rows;
  int bf16;  // products on bf16-rounded operands (the *_bf16 GEMMs' arithmetic: exact products, f32 sums)
};

__device__ __forceinline__ float bf16_round(float v) { return static_cast<float>(static_cast<__bf16>(v)); }

// P lanes per row (consecutive threads of one wave): lane p computes outputs
// j = p, p + P, ... of every layer from the whole input row, read from the
// block's LDS row image (img_pitch: the wave's 64 / P rows on distinct
// banks, the P lanes of a row a broadcast); outputs go back to the image
// for the next layer.  One thread per row (P = 1, the first form) left each
// wave a serial chain of ~2.7k FMAs + LDS reads: 25.8 us for the tangent
// chain at 12.7k rows against 16.9 us for three GEMMs.
constexpr int kP = 4;
constexpr int kRowsPerBlock = 256 / kP;

// row image pitch: W + 4 for float4 rows (the wave's 16 rows 4 banks apart:
// conflict-free float4 reads, the row's 4 lanes a broadcast), else W + 1
constexpr int img_pitch(int w) { return w % 4 == 0 ? w + 4 : w + 1; }

template <int IN, int OUT>
__device__ __forceinline__ void chain_layer_p(const float* xs, float* ys, const float* Ws, const ChainLayer& L,
                                              int row, bool live, int p, bool bf16) {
  constexpr int PITCH_IN = img_pitch(IN), PITCH_OUT = img_pitch(OUT);
  constexpr int J = (OUT + kP - 1) / kP;  // outputs per lane
  const int rl = threadIdx.x / kP;
  float x[IN];
  if constexpr (IN % 4 == 0) {
    const float4* xr = reinterpret_cast<const float4*>(xs + rl * PITCH_IN);
#pragma unroll
    for (int k4 = 0; k4 < IN / 4; ++k4) {
      const float4 v = xr[k4];
      x[4 * k4] = v.x;
      x[4 * k4 + 1] = v.y;
      x[4 * k4 + 2] = v.z;
      x[4 * k4 + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < IN; ++k) x[k] = xs[rl * PITCH_IN + k];
  }
  if (bf16)
#pragma unroll
    for (int k = 0; k < IN; ++k) x[k] = bf16_round(x[k]);
#pragma unroll
  for (int jj = 0; jj < J; ++jj) {
    const int j = p + kP * jj;
    float acc = 0.f;
    if (j < OUT) {
      if constexpr (IN % 4 == 0) {
        const float4* wr = reinterpret_cast<const float4*>(Ws + j * IN);
#pragma unroll
        for (int k4 = 0; k4 < IN / 4; ++k4) {
          const float4 w = wr[k4];
          acc = fmaf(x[4 * k4], w.x, acc);
          acc = fmaf(x[4 * k4 + 1], w.y, acc);
          acc = fmaf(x[4 * k4 + 2], w.z, acc);
          acc = fmaf(x[4 * k4 + 3], w.w, acc);
        }
      } else {
#pragma unroll
        for (int k = 0; k < IN; ++k) acc = fmaf(x[k], Ws[j * IN + k], acc);
      }
      if (L.bias) acc += L.bias[j];
      if (L.act == 1) acc = acc > 0.f ? acc : 0.f;
      else if (L.act == 3) acc = L.aux[(size_t)row * L.ld_aux + j] > 0.f ? acc : 0.f;
      if (L.out && live) L.out[(size_t)row * L.ld_out + j] = acc;
      ys[rl * PITCH_OUT + j] = acc;
    }
  }
}

// Staging loads all issue before the first LDS store (a compile-time count per
// thread, in registers): a load -> wait -> store loop runs its loads one after
// another.
template <int IN, int OUT>
__device__ __forceinline__ void stage_layer(float* Ws, const ChainLayer& L, bool bf16) {
  constexpr int NE = (IN * OUT + 255) / 256;
  float r[NE];
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = threadIdx.x + 256 * u;
    const int j = e / IN, k = e - j * IN;
    r[u] = e < IN * OUT ? (L.wt ? L.w[(size_t)k * OUT + j] : L.w[(size_t)j * IN + k]) : 0.f;
  }
#pragma unroll
  for (int u = 0; u < NE; ++u) {
    const int e = threadIdx.x + 256 * u;
    if (e < IN * OUT) Ws[e] = bf16 ? bf16_round(r[u]) : r[u];
  }
}

constexpr int cmax1(int v) { return v > 0 ? v : 1; }
constexpr int cmaxw(int a, int b) { return a > b ? a : b; }

// W0 -> W1 -> ... ; a zero width ends the chain (2 to 4 layers)
template <int W0, int W1, int W2, int W3, int W4>
__global__ void __launch_bounds__(256) k_chain(const ChainDesc d) {
  constexpr int S0 = W0 * W1, S1 = W1 * W2, S2 = W2 * W3, S3 = W3 * W4;
  constexpr int WMAX = cmaxw(cmaxw(W0, W1), cmaxw(cmaxw(W2, W3), W4));
  __shared__ __attribute__((aligned(16))) float Ws[cmax1(S0 + S1 + S2 + S3)];
  __shared__ __attribute__((aligned(16))) float img[2][kRowsPerBlock * (WMAX + 4)];  // row images: in / out
  const bool bf = d.bf16 != 0;
  stage_layer<W0, W1>(Ws, d.l[0], bf);
  if constexpr (W2 > 0) stage_layer<W1, W2>(Ws + S0, d.l[1], bf);
  if constexpr (W3 > 0) stage_layer<W2, W3>(Ws + S0 + S1, d.l[2], bf);
  if constexpr (W4 > 0) stage_layer<W3, W4>(Ws + S0 + S1 + S2, d.l[3], bf);
  const int row0 = blockIdx.x * kRowsPerBlock;
  // the block's input rows, coalesced, into the image (loads first, as above)
  {
    constexpr int NX = (kRowsPerBlock * W0 + 255) / 256;
    float r[NX];
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int rr = e / W0, k = e - rr * W0;
      const int row = min(row0 + rr, d.rows - 1);
      r[u] = e < kRowsPerBlock * W0 ? d.x[(size_t)row * d.ldx + k] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < NX; ++u) {
      const int e = threadIdx.x + 256 * u;
      const int rr = e / W0, k = e - rr * W0;
      if (e < kRowsPerBlock * W0) img[0][rr * img_pitch(W0) + k] = r[u];
    }
  }
  __syncthreads();
  const int p = threadIdx.x % kP;
  const int rowr = row0 + threadIdx.x / kP;
  const bool live = rowr < d.rows;
  const int row = live ? rowr : d.rows - 1;
  chain_layer_p<W0, W1>(img[0], img[1], Ws, d.l[0], row, live, p, bf);
  if constexpr (W2 > 0) {
    __syncthreads();
    chain_layer_p<W1, W2>(img[1], img[0], Ws + S0, d.l[1], row, live, p, bf);
    if constexpr (W3 > 0) {
      __syncthreads();
      chain_layer_p<W2, W3>(img[0], img[1], Ws + S0 + S1, d.l[2], row, live, p, bf);
      if constexpr (W4 > 0) {
        __syncthreads();
        chain_layer_p<W3, W4>(img[1], img[0], Ws + S0 + S1 + S2, d.l[3], row, live, p, bf);
      }
    }
  }
}

}  // namespace

// The width chains instantiated: the critic's decoder at DISCRIMINATOR_HIDDEN_DIM
// 64 (forward, tangent, adjoint); other widths return VG_EINVAL (per-layer GEMMs).
static int linear_chain(const float* x, int32_t ldx, int32_t rows, const int32_t* widths, int32_t nlayers,
                        const vg_chain_layer* layers, void* stream, int bf16) {
  if (rows <= 0 || !x || !widths || !layers || nlayers < 2 || nlayers > kChainMax) return VG_EINVAL;
  ChainDesc d{};
  d.bf16 = bf16;
  d.x = x;
  d.ldx = ldx;
  d.rows = rows;
  int w[kChainMax + 1] = {0, 0, 0, 0, 0};
  for (int i = 0; i <= nlayers; ++i) w[i] = widths[i];
  if (ldx < w[0] || ((w[0] % 4 == 0) && ((ldx % 4) || (reinterpret_cast<uintptr_t>(x) & 15)))) return VG_EINVAL;
  for (int i = 0; i < nlayers; ++i) {
    const vg_chain_layer& s = layers[i];
    const int o = w[i + 1];
    if (!s.weight || (s.act != 0 && s.act != 1 && s.act != 3) || (s.act == 3 && (!s.aux || s.ld_aux < o)) ||
        (s.out && s.ld_out < o))
      return VG_EINVAL;
    // float4 rows where the width allows: 16-B aligned rows
    if (o % 4 == 0 && ((s.out && ((s.ld_out % 4) || (reinterpret_cast<uintptr_t>(s.out) & 15))) ||
                       (s.act == 3 && ((s.ld_aux % 4) || (reinterpret_cast<uintptr_t>(s.aux) & 15)))))
      return VG_EINVAL;
    d.l[i] = ChainLayer{s.weight, s.bias, s.aux, s.out, s.ld_aux, s.ld_out, s.w_trans, s.act};
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int grid = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  if (nlayers == 4 && w[0] == 64 && w[1] == 32 && w[2] == 16 && w[3] == 8 && w[4] == 1)
    k_chain<64, 32, 16, 8, 1><<<grid, 256, 0, st>>>(d);
  else if (nlayers == 3 && w[0] == 64 && w[1] == 32 && w[2] == 16 && w[3] == 8)
    k_chain<64, 32, 16, 8, 0><<<grid, 256, 0, st>>>(d);
  else if (nlayers == 3 && w[0] == 1 && w[1] == 8 && w[2] == 16 && w[3] == 32)
    k_chain<1, 8, 16, 32, 0><<<grid, 256, 0, st>>>(d);
  else
    return VG_EINVAL;
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_linear_chain(const float* x, int32_t ldx, int32_t rows, const int32_t* widths, int32_t nlayers,
                               const vg_chain_layer* layers, void* stream) {
  return linear_chain(x, ldx, rows, widths, nlayers, layers, stream, 0);
}

extern "C" int vg_linear_chain_bf16(const float* x, int32_t ldx, int32_t rows, const int32_t* widths,
                                    int32_t nlayers, const vg_chain_layer* layers, void* stream) {
  return linear_chain(x, ldx, rows, widths, nlayers, layers, stream, 1);
}
