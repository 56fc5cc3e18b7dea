// Row-local chains of narrow linear layers in ONE launch: the discriminator's
// decoder (models.py:273-279 / reference models.py:212-222: Linear 64 -> 32 ->
// 16 -> 8 -> 1 with ReLU between) in the critic engine's four passes
// (vgan/critic.py): the forward (pass A), the adjoint chains g_in = (g_out W)
// [z > 0] (passes B and D) and the tangent chain u_out = (u W^T) [z > 0]
// (pass C).  Each layer was one vg_gemm launch of 8-38k rows x <= 64
// columns, i.e. a dependent ~7 us launch moving a few MB; here one thread
// owns one row through the whole chain: the row in registers, every layer's
// weights staged once per workgroup in LDS in [out][in] order (read as
// broadcast float4), each layer's output stored for the backward.  f32 FMAs in
// k order; the MFMA GEMMs sum in another order (f32 rounding differences).
#include "common.h"

namespace {

constexpr int kChainMax = 4;    // layers per launch
constexpr int kChainBlock = 64;  // rows (threads) per workgroup: 600 workgroups at 38k rows

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
};

template <int IN, int OUT>
__device__ __forceinline__ void chain_layer(const float (&x)[IN], float (&y)[OUT], const float* Ws,
                                            const ChainLayer& L, int row, bool live) {
#pragma unroll
  for (int j = 0; j < OUT; ++j) {
    float acc = 0.f;
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
    y[j] = acc;
  }
  if (L.bias)
#pragma unroll
    for (int j = 0; j < OUT; ++j) y[j] += L.bias[j];
  if (L.act == 1) {
#pragma unroll
    for (int j = 0; j < OUT; ++j) y[j] = y[j] > 0.f ? y[j] : 0.f;
  } else if (L.act == 3) {
    const float* a = L.aux + (size_t)row * L.ld_aux;
    if constexpr (OUT % 4 == 0) {
#pragma unroll
      for (int j4 = 0; j4 < OUT / 4; ++j4) {
        const float4 m = reinterpret_cast<const float4*>(a)[j4];
        y[4 * j4] = m.x > 0.f ? y[4 * j4] : 0.f;
        y[4 * j4 + 1] = m.y > 0.f ? y[4 * j4 + 1] : 0.f;
        y[4 * j4 + 2] = m.z > 0.f ? y[4 * j4 + 2] : 0.f;
        y[4 * j4 + 3] = m.w > 0.f ? y[4 * j4 + 3] : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < OUT; ++j) y[j] = a[j] > 0.f ? y[j] : 0.f;
    }
  }
  if (L.out && live) {
    float* o = L.out + (size_t)row * L.ld_out;
    if constexpr (OUT % 4 == 0) {
#pragma unroll
      for (int j4 = 0; j4 < OUT / 4; ++j4)
        reinterpret_cast<float4*>(o)[j4] = make_float4(y[4 * j4], y[4 * j4 + 1], y[4 * j4 + 2], y[4 * j4 + 3]);
    } else {
#pragma unroll
      for (int j = 0; j < OUT; ++j) o[j] = y[j];
    }
  }
}

template <int IN, int OUT>
__device__ __forceinline__ void stage_layer(float* Ws, const ChainLayer& L) {
  for (int e = threadIdx.x; e < IN * OUT; e += blockDim.x) {
    const int j = e / IN, k = e - j * IN;
    Ws[e] = L.wt ? L.w[(size_t)k * OUT + j] : L.w[(size_t)j * IN + k];
  }
}

constexpr int cmax1(int v) { return v > 0 ? v : 1; }

// W0 -> W1 -> ... ; a zero width ends the chain (2 to 4 layers)
template <int W0, int W1, int W2, int W3, int W4>
__global__ void __launch_bounds__(kChainBlock) k_chain(const ChainDesc d) {
  constexpr int S0 = W0 * W1, S1 = W1 * W2, S2 = W2 * W3, S3 = W3 * W4;
  __shared__ __attribute__((aligned(16))) float Ws[cmax1(S0 + S1 + S2 + S3)];
  stage_layer<W0, W1>(Ws, d.l[0]);
  if constexpr (W2 > 0) stage_layer<W1, W2>(Ws + S0, d.l[1]);
  if constexpr (W3 > 0) stage_layer<W2, W3>(Ws + S0 + S1, d.l[2]);
  if constexpr (W4 > 0) stage_layer<W3, W4>(Ws + S0 + S1 + S2, d.l[3]);
  const int row0 = blockIdx.x * kChainBlock + threadIdx.x;
  const bool live = row0 < d.rows;
  const int row = live ? row0 : d.rows - 1;
  float x0[W0];
  const float* xr = d.x + (size_t)row * d.ldx;
  if constexpr (W0 % 4 == 0) {
#pragma unroll
    for (int k4 = 0; k4 < W0 / 4; ++k4) {
      const float4 v = reinterpret_cast<const float4*>(xr)[k4];
      x0[4 * k4] = v.x;
      x0[4 * k4 + 1] = v.y;
      x0[4 * k4 + 2] = v.z;
      x0[4 * k4 + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int k = 0; k < W0; ++k) x0[k] = xr[k];
  }
  __syncthreads();  // the staged weights
  float x1[W1];
  chain_layer<W0, W1>(x0, x1, Ws, d.l[0], row, live);
  if constexpr (W2 > 0) {
    float x2[W2];
    chain_layer<W1, W2>(x1, x2, Ws + S0, d.l[1], row, live);
    if constexpr (W3 > 0) {
      float x3[W3];
      chain_layer<W2, W3>(x2, x3, Ws + S0 + S1, d.l[2], row, live);
      if constexpr (W4 > 0) {
        float x4[W4];
        chain_layer<W3, W4>(x3, x4, Ws + S0 + S1 + S2, d.l[3], row, live);
      }
    }
  }
}

}  // namespace

// The width chains instantiated: the critic's decoder at DISCRIMINATOR_HIDDEN_DIM
// 64 (forward, tangent, adjoint); other widths return VG_EINVAL (per-layer GEMMs).
extern "C" int vg_linear_chain(const float* x, int32_t ldx, int32_t rows, const int32_t* widths, int32_t nlayers,
                               const vg_chain_layer* layers, void* stream) {
  if (rows <= 0 || !x || !widths || !layers || nlayers < 2 || nlayers > kChainMax) return VG_EINVAL;
  ChainDesc d{};
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
  const int grid = (rows + kChainBlock - 1) / kChainBlock;
  if (nlayers == 4 && w[0] == 64 && w[1] == 32 && w[2] == 16 && w[3] == 8 && w[4] == 1)
    k_chain<64, 32, 16, 8, 1><<<grid, kChainBlock, 0, st>>>(d);
  else if (nlayers == 3 && w[0] == 64 && w[1] == 32 && w[2] == 16 && w[3] == 8)
    k_chain<64, 32, 16, 8, 0><<<grid, kChainBlock, 0, st>>>(d);
  else if (nlayers == 3 && w[0] == 1 && w[1] == 8 && w[2] == 16 && w[3] == 32)
    k_chain<1, 8, 16, 32, 0><<<grid, kChainBlock, 0, st>>>(d);
  else
    return VG_EINVAL;
  VG_CHECK_LAUNCH();
  return 0;
}
