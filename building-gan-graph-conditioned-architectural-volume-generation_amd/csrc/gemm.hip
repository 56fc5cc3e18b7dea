// Dense per-node GEMMs of the MLPs on the f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// The path's dense layers are tall-skinny: N ~ 12.7k node rows against
// K, M <= 524 x 128 weights.  Library GEMMs paid 19 us minimum per call and
// 77-692 us for the weight gradient (a handful of output tiles with the whole
// K = N reduction in one workgroup; profiles/r01_*).  Two kernels cover all
// three products of nn.Linear:
//
//   k_gemm      C[N, M] = A[N, K] . op(B) (+ bias[M]) (+ activation)
//               forward  (A = X, B = W [M, K], op = transpose)
//               dX       (A = dY, B = W [M, K] read as [K', M'] = no transpose)
//               ACT 3 multiplies by [aux > 0] (aux [N, M]): the ReLU mask of a
//               layer folded into the GEMM that produces its adjoint/tangent
//   k_gemm_tn   C[M, K] = A[N, M]^T . B[N, K] split over N (~768 workgroups),
//               plus db[M] = sum_n A[n, :]; partials folded in chunk order,
//               written or accumulated into C (row stride ldc).
//               weight / bias gradient (A = dY, B = X)
//
// f32 in, f32 accumulate: the MFMA is an exact fmaf chain (no TF32 on gfx950),
// so results differ from a CPU GEMM only by summation order.
//
// bf16 mode (the *_bf16 entry points; BASELINE configs[2]): the same kernels
// with template flag BF round both operands to bf16 (round-to-nearest-even,
// v_cvt_pk_bf16_f32) as they are staged into LDS and multiply them on
// v_mfma_f32_32x32x16_bf16 with f32 accumulation -- torch.autocast's
// treatment of a matmul, except that outputs, epilogues (bias, activation,
// LayerNorm, attention projections) and bias gradients stay f32.  A K-tile of
// 32 is 2 bf16 MFMAs instead of 16 f32 MFMAs.  The global loads are the f32
// path's (coalesced, one float per thread and step); the values are rounded
// as they are written to LDS, whose rows hold 32 bf16 padded to 40 (80 B: the
// 8-element fragment of a lane is one aligned 16-byte read).
//
// Tiling: 256-thread workgroup = 4 waves, 64 x 64 output tile, each wave one
// 32 x 32 MFMA tile; K staged through LDS 32 at a time.  LDS rows are padded
// to 33 floats so the MFMA operand reads (32 lanes down a column) and the
// transposing stores are bank-conflict free.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int TM = 64, TN = 64, TK = 32, LDP = TK + 1;
constexpr int LDH = TK + 8;  // bf16 LDS row pitch (elements)

__device__ __forceinline__ bf16x4 to_bf4(const float (&v)[4]) {
  bf16x4 r;
  r[0] = static_cast<__bf16>(v[0]);
  r[1] = static_cast<__bf16>(v[1]);
  r[2] = static_cast<__bf16>(v[2]);
  r[3] = static_cast<__bf16>(v[3]);
  return r;
}

__device__ __forceinline__ f32x16 mfma_bf(const __bf16* a, const __bf16* b, f32x16 acc) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(a),
                                                 *reinterpret_cast<const bf16x8*>(b), acc, 0, 0, 0);
}
#ifndef VG_LN16
#define VG_LN16 1  // f32 k_gemm_ln16 (16 waves of 16 x 16 MFMA tiles); 0: k_gemm_ln (A/B)
#endif
#ifndef VG_LN_TM32
#define VG_LN_TM32 1
#endif
#ifndef VG_TN_GROUPS
#define VG_TN_GROUPS 2
#endif
constexpr int kTnGroups = VG_TN_GROUPS;  // row groups (of 4 waves) per split-K workgroup

template <int ACT>
__device__ __forceinline__ float act_fn(float v, float aux) {
  if constexpr (ACT == 1) return v > 0.f ? v : 0.f;
  else if constexpr (ACT == 2) return v > 0.f ? v : 0.2f * v;
  else if constexpr (ACT == 3) return aux > 0.f ? v : 0.f;
  else if constexpr (ACT == 4) return v + aux;  // a second adjoint summed in (torch's add_ after the GEMM)
  else return v;
}

// Fragment-ordered operand images for the 16 x 16 x 4 f32 MFMA (k_gemm_ln16).
// The MFMA lane (row r = lane % 16, k-group g = lane / 16) consumes k = g, g + 4,
// ..., g + 28 of a 32-wide K-tile, one per MFMA.  Row r of the image keeps its
// 32 values as slot 8 (k % 4) + k / 4 -- a lane's 8 values contiguous --
// XOR-swizzled in 4-float units by r % 8 with a 48-float pitch, so the lane
// reads them as two ds_read_b128, conflict-free across the instruction's lane
// groups (MI355X_MICROARCH.md LDS table), instead of eight ds_read_b32: half
// the LDS cycles per MFMA.  The MFMAs see the same operands in the same order
// (bit-identical results).
#ifndef VG_FRAG128
#define VG_FRAG128 1  // 0: the row-major images with 33-float pitch (A/B knob)
#endif
constexpr int FP = 48;
__device__ __forceinline__ int frag_pos(int r, int k) { return r * FP + ((8 * (k & 3) + (k >> 2)) ^ (4 * (r & 7))); }
__device__ __forceinline__ int frag_at(int r, int g, int h) { return r * FP + ((8 * g + 4 * h) ^ (4 * (r & 7))); }

// Logical (row tile, column tile) of this workgroup, XCD-aware: the hardware
// deals workgroups round-robin over the 8 XCDs in dispatch order (x fastest),
// so linear id b runs on XCD b % 8; every XCD gets one contiguous range of
// row tiles -- the same row ranges the message-passing kernels (xcd_remap)
// give it, so the rows a GEMM writes are read back through the same L2.
// Speed only, never correctness.
__device__ __forceinline__ void tile_xy(int& tx, int& ty) {
  const int gy = gridDim.y;
  const int hw = blockIdx.x + gridDim.x * blockIdx.y;
  const int logical = xcd_remap(hw, gridDim.x * gy);
  tx = logical / gy;
  ty = logical % gy;
}

// GraphNorm-backward partials in the epilogue of the GEMM that produces the
// layer's output gradient g_y (vg_gemm_gn_bwd): x, keep [rows, M] (the
// GraphNorm input and dropout multiplier), stats [S][2M] of segments of
// seg_rows rows, tpart [row tile][2 slots][M][2] (sum gz, sum gz * xhat).
struct GnpDesc {
  const float* x;
  const float* keep;
  const float* stats;
  const float* w;
  const float* b;
  const float* ms;
  float eps;
  int seg_rows;
  float* tpart;
};

// GraphNorm + ReLU + Dropout applied to the A operand as it is loaded
// (vg_gat_lin_att_gn: the GraphNorm that ends a GATConv block feeding the next
// block's projection, models.py:73-77): A holds the GraphNorm INPUT x [rows, K]
// (lda = K); every element becomes y = keep * relu(w (x - ms mu)/d + b)
// with the statistics of its row's segment -- the formula and operation order
// of k_gn_apply4 -- and y (and a drawn keep) are stored for the backward when
// y != NULL.  keep: multipliers read (iter == NULL) or drawn in-kernel
// (iter != NULL: vg_keep, the same draws as vg_graphnorm_fwd_drop).
struct GnaDesc {
  const float* stats;  // [S][2K]
  const float* w;
  const float* b;
  const float* ms;
  const float* keep;   // multipliers [rows, K] or NULL (iter == NULL)
  float eps, p_drop;
  int seg_rows;
  unsigned int salt;
  unsigned long long seed;
  const long long* iter;
  float* y;         // [rows, K] or NULL
  float* keep_out;  // [rows, K] or NULL (drawn multipliers)
};

constexpr int kGnaMaxK = 128;  // GraphNorm channels the operand transform stages in LDS

// Four consecutive columns k .. k+3 of row n (k % 4 == 0, K % 4 == 0): one
// Philox block draws all four multipliers (vg_keep4_raw: the values vg_keep
// gives each element), float4 stores of y / keep.  gp = the block's staged
// column operands [w | b | ms | mu0 | d0 | mu1 | d1] (segment
// slots 0 / 1: the tile's first row's segment and the next).
__device__ __forceinline__ float4 gna_quad(const GnaDesc& ga, const float* gp, float4 x, int n, int k, int K,
                                           int bound, long long it) {
  const int sl = n >= bound ? 5 * K : 3 * K;
  const size_t t = (size_t)n * K + k;
  float4 kv = make_float4(1.f, 1.f, 1.f, 1.f);
  if (ga.iter) {
    kv = vg_keep4_raw((long long)(t >> 2), ga.salt, it, ga.seed, ga.p_drop);
    if (ga.keep_out) *reinterpret_cast<float4*>(ga.keep_out + t) = kv;
  } else if (ga.keep) {
    kv = *reinterpret_cast<const float4*>(ga.keep + t);
  }
  const bool mul = ga.iter || ga.keep;
  float xv[4] = {x.x, x.y, x.z, x.w}, kk[4] = {kv.x, kv.y, kv.z, kv.w}, r[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float o = xv[j] - gp[sl + k + j] * gp[2 * K + k + j];
    const float z = (o / gp[sl + K + k + j]) * gp[k + j] + gp[K + k + j];
    r[j] = z > 0.f ? z : 0.f;
    if (mul) r[j] *= kk[j];
  }
  const float4 y = make_float4(r[0], r[1], r[2], r[3]);
  if (ga.y) *reinterpret_cast<float4*>(ga.y + t) = y;
  return y;
}

// C = A . op(B) (+bias) (+act).  BT: B is [M, K] (op = B^T); else B is [K, M].
// Software pipelined: the next K-tile is loaded into registers while the MFMAs
// of the current one run; LDS is double-buffered (one barrier per K-tile).
// ATT (BT, ACT 0, M <= 64): also a_src[n] = <C[n,:], att_s>, a_dst[n] =
// <C[n,:], att_d> -- GATConv's attention projections as the epilogue of its
// own projection GEMM (the output tile is staged through LDS once).
// QA (bf16 operands only): A -- and B^T -- loaded as float4 quads (2 per
// thread per K-tile) and stored to the bf16 images 8 bytes at a time,
// instead of 8 scalars and 2-byte stores per thread (quad_ab).
template <bool BT, int ACT, bool ATT = false, bool BF = false, bool GNP = false, bool QA = false>
__global__ void __launch_bounds__(256) k_gemm(const float* __restrict__ A, int lda,
                                              const float* __restrict__ B, int ldb,
                                              const float* __restrict__ bias,
                                              const float* __restrict__ aux, int ldaux,
                                              float* __restrict__ C, int ldc, int N, int M, int K,
                                              const float* __restrict__ att_s = nullptr,
                                              const float* __restrict__ att_d = nullptr,
                                              float* __restrict__ a_src = nullptr,
                                              float* __restrict__ a_dst = nullptr,
                                              const GnpDesc gn = GnpDesc{}) {
  __shared__ __attribute__((aligned(16))) float smem[2 * TM * LDP + 2 * TN * LDP];
  float(*As)[TM][LDP] = reinterpret_cast<float(*)[TM][LDP]>(smem);
  float(*Bs)[TN][LDP] = reinterpret_cast<float(*)[TN][LDP]>(smem + 2 * TM * LDP);  // Bs[j][k] = op(B)[k][j]
  constexpr int PER = (TM * TK) / 256;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  int tx, ty;
  tile_xy(tx, ty);
  const int n0 = tx * TM, m0 = ty * TN;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  // GNP: the epilogue's GraphNorm operands are loaded here, so their latency
  // hides behind the K loop: the tile's 16 rows of x / keep per lane, the two
  // segments' statistics and the column's parameters
  float gx_[GNP ? 16 : 1], gk_[GNP ? 16 : 1];
  float gmu[2] = {0.f, 0.f}, gsd[2] = {1.f, 1.f}, gw_ = 0.f, gb_ = 0.f, gms_ = 0.f;
  int gbound = 0;
  if constexpr (GNP) {
    const int mc = m0 + wc * 32 + (lane & 31);
    const int seg0 = n0 / gn.seg_rows;
    gbound = (seg0 + 1) * gn.seg_rows;  // first row of the next segment
    if (mc < M) {
      gw_ = gn.w[mc];
      gb_ = gn.b[mc];
      gms_ = gn.ms[mc];
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (q == 0 || gbound < N) {
          const float* st = gn.stats + (size_t)(seg0 + q) * 2 * M;
          gmu[q] = st[mc];
          gsd[q] = st[M + mc];
        }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n = n0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const bool ok = n < N && mc < M;
      gx_[r] = ok ? gn.x[(size_t)n * M + mc] : 0.f;
      gk_[r] = ok && gn.keep ? gn.keep[(size_t)n * M + mc] : 1.f;
    }
  }
  float ra[PER], rb[PER];
  // BF && !BT: B in quads of 4 k per thread (lanes along m: coalesced), one
  // 8-byte LDS store per quad instead of four transposing 2-byte stores
  constexpr int QB = (TN * TK / 4) / 256;
  float qb[QB][4];
  static_assert(!QA || BF, "quad staging for the bf16 images");
  constexpr int QN = (TM * TK / 4) / 256, QPR = TK / 4;  // quads per thread / per tile row
  float4 rqa[QA ? QN : 1], rqb[QA ? QN : 1];
  auto load = [&](int k0) {
    if constexpr (QA) {
#pragma unroll
      for (int u = 0; u < QN; ++u) {
        const int g = t + 256 * u;
        const int row = g / QPR, k = k0 + 4 * (g % QPR);
        const int n = n0 + row;
        rqa[u] = (n < N && k < K) ? *reinterpret_cast<const float4*>(A + (size_t)n * lda + k)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        if (BT) {
          const int m = m0 + row;
          rqb[u] = (m < M && k < K) ? *reinterpret_cast<const float4*>(B + (size_t)m * ldb + k)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      const int row = e / TK, kc = e % TK;
      const int n = n0 + row, k = k0 + kc;
      if constexpr (!QA) ra[q] = (n < N && k < K) ? A[(size_t)n * lda + k] : 0.f;
      if (BT) {
        const int m = m0 + row;
        if constexpr (!QA) rb[q] = (m < M && k < K) ? B[(size_t)m * ldb + k] : 0.f;
      } else if (!BF) {
        const int kr = e / TN, j = e % TN;
        const int m = m0 + j, kk = k0 + kr;
        rb[q] = (m < M && kk < K) ? B[(size_t)kk * ldb + m] : 0.f;
      }
    }
    if constexpr (BF && !BT) {
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int g = t + 256 * q;
        const int m = m0 + (g & 63), kq = (g >> 6) * 4;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int kk = k0 + kq + i;
          qb[q][i] = (m < M && kk < K) ? B[(size_t)kk * ldb + m] : 0.f;
        }
      }
    }
  };
  // BF: the same coalesced global loads, staged as bf16 -- Ah[buf][n][k],
  // Bh[buf][m][k] = op(B)[k][m] -- and multiplied 16 k at a time
  __bf16(*Ah)[TM][LDH] = reinterpret_cast<__bf16(*)[TM][LDH]>(smem);
  __bf16(*Bh)[TN][LDH] = reinterpret_cast<__bf16(*)[TN][LDH]>(smem + 2 * TM * LDP);
  load(0);
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += TK) {
    if constexpr (QA) {
#pragma unroll
      for (int u = 0; u < QN; ++u) {
        const int g = t + 256 * u;
        const int row = g / QPR, kq = 4 * (g % QPR);
        const float va[4] = {rqa[u].x, rqa[u].y, rqa[u].z, rqa[u].w};
        *reinterpret_cast<bf16x4*>(&Ah[buf][row][kq]) = to_bf4(va);
        if (BT) {
          const float vb[4] = {rqb[u].x, rqb[u].y, rqb[u].z, rqb[u].w};
          *reinterpret_cast<bf16x4*>(&Bh[buf][row][kq]) = to_bf4(vb);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      if constexpr (QA) {
      } else if constexpr (BF) {
        Ah[buf][e / TK][e % TK] = static_cast<__bf16>(ra[q]);
        if (BT) Bh[buf][e / TK][e % TK] = static_cast<__bf16>(rb[q]);
      } else {
        As[buf][e / TK][e % TK] = ra[q];
        if (BT) Bs[buf][e / TK][e % TK] = rb[q];
        else Bs[buf][e % TN][e / TN] = rb[q];
      }
    }
    if constexpr (BF && !BT) {
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const int g = t + 256 * q;
        *reinterpret_cast<bf16x4*>(&Bh[buf][g & 63][(g >> 6) * 4]) = to_bf4(qb[q]);
      }
    }
    __syncthreads();
    if (k0 + TK < K) load(k0 + TK);
    if constexpr (BF) {
      const int h8 = 8 * (lane >> 5);
#pragma unroll
      for (int s16 = 0; s16 < TK; s16 += 16)
        acc = mfma_bf(&Ah[buf][wr * 32 + (lane & 31)][s16 + h8], &Bh[buf][wc * 32 + (lane & 31)][s16 + h8], acc);
    } else {
      const float* ar = &As[buf][wr * 32 + (lane & 31)][lane >> 5];
      const float* br = &Bs[buf][wc * 32 + (lane & 31)][lane >> 5];
#pragma unroll
      for (int kk = 0; kk < TK; kk += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[kk], br[kk], acc, 0, 0, 0);
    }
    buf ^= 1;
  }
  const int m = m0 + wc * 32 + (lane & 31);
  const float bv = (bias && m < M) ? bias[m] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = n0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (n < N && m < M) {
      const float av = ACT >= 3 ? aux[(size_t)n * ldaux + m] : 0.f;
      C[(size_t)n * ldc + m] = act_fn<ACT>(acc[r] + bv, av);
    }
  }
  if constexpr (GNP) {
    // column partials of gz = g_y [z > 0] keep and gz * xhat over the tile's
    // rows, per segment slot (0: the segment of row n0, 1: the next one);
    // g_y = acc (ACT 0, no bias).  Row order in-lane, then the lane pair
    // holding the other 16 rows, then the two row waves: deterministic.
    float pa[2] = {0.f, 0.f}, pb[2] = {0.f, 0.f};
    if (m < M) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (n < N) {
          const int sl = n >= gbound;
          const float xh = (gx_[r] - (sl ? gmu[1] : gmu[0]) * gms_) / (sl ? gsd[1] : gsd[0]);
          const float gz = xh * gw_ + gb_ > 0.f ? acc[r] * gk_[r] : 0.f;
          if (sl) {
            pa[1] += gz;
            pb[1] = fmaf(gz, xh, pb[1]);
          } else {
            pa[0] += gz;
            pb[0] = fmaf(gz, xh, pb[0]);
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      pa[q] += __shfl_xor(pa[q], 32, 64);
      pb[q] += __shfl_xor(pb[q], 32, 64);
    }
    __syncthreads();  // every wave is done with the last K-tile's LDS images
    float* red = smem;  // [wr][64 columns][4]
    if (lane < 32) {
      float* rp = red + ((wr * 64) + wc * 32 + lane) * 4;
      rp[0] = pa[0];
      rp[1] = pb[0];
      rp[2] = pa[1];
      rp[3] = pb[1];
    }
    __syncthreads();
    if (wr == 0 && lane < 32 && m < M) {
      const float* r0p = red + (wc * 32 + lane) * 4;
      const float* r1p = red + (64 + wc * 32 + lane) * 4;
      float* tp = gn.tpart + (size_t)tx * 2 * M * 2;
      tp[(size_t)m * 2] = r0p[0] + r1p[0];
      tp[(size_t)m * 2 + 1] = r0p[1] + r1p[1];
      tp[(size_t)(M + m) * 2] = r0p[2] + r1p[2];
      tp[(size_t)(M + m) * 2 + 1] = r0p[3] + r1p[3];
    }
  }
  if constexpr (ATT) {
    // stage the 64 x 64 tile in LDS (reusing As), then 4 threads per row dot
    // 16 columns each with att_s / att_d and combine by two shuffles
    float(*Ct)[TN + 1] = reinterpret_cast<float(*)[TN + 1]>(&As[0][0][0]);
    __syncthreads();  // every wave is done with the last K-tile's As
#pragma unroll
    for (int r = 0; r < 16; ++r)
      Ct[wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)][wc * 32 + (lane & 31)] = acc[r] + bv;
    __syncthreads();
    const int row = t >> 2, q = t & 3;
    float ss = 0.f, sd = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = q * 16 + j;
      if (c < M) {
        const float v = Ct[row][c];
        ss = fmaf(v, att_s[c], ss);
        sd = fmaf(v, att_d[c], sd);
      }
    }
    ss += __shfl_xor(ss, 1, 64);
    sd += __shfl_xor(sd, 1, 64);
    ss += __shfl_xor(ss, 2, 64);
    sd += __shfl_xor(sd, 2, 64);
    if (q == 0 && n0 + row < N) {
      a_src[n0 + row] = ss;
      a_dst[n0 + row] = sd;
    }
  }
}

// The plain f32 products (no ATT / GNP epilogue) with 16 waves per 64 x 64
// tile, one 16 x 16 v_mfma_f32_16x16x4_f32 sub-tile each, instead of 4 waves
// with a 32 x 32 tile.  The step's products are skinny (K, M <= 128 over
// 13k-66k rows): k_gemm put 1.5-2.4 waves on a SIMD and its waves spent
// 50-67 % of their cycles parked on loads (rocprofv3 SQ_WAIT_ANY); the same
// work in 4x the waves hides that latency.  Same LDS images, double
// buffering and XCD-aware tile order as k_gemm; same f32 MFMA rate.
typedef float f32x4 __attribute__((ext_vector_type(4)));

// ATT, GNP as in k_gemm (the attention projections / the GraphNorm-backward
// tile partials in the epilogue).  BF: bf16 operands through
// v_mfma_f32_16x16x32_bf16 -- the f32 LDS images are converted when read
// (lane l: row l & 15, k = 8 (l >> 4) + j).
// GNA: GraphNorm + ReLU + Dropout applied to A as it loads (GnaDesc; one
// column tile: every A element is loaded, transformed and stored once).
// QA: A and B loaded as float4 quads by threads 0..511 (one quad per K-tile;
// K % 4 == 0, leading dimensions % 4 == 0, 16-B aligned operands, quad_ab)
// instead of 2 scalars each by every thread; GNA loads A as quads.
template <bool BT, int ACT, bool ATT = false, bool BF = false, bool GNP = false, bool GNA = false, bool QA = false,
          int NW = 16>
__device__ __forceinline__ void gemm16_body(const float* __restrict__ A, int lda,
                                                 const float* __restrict__ B, int ldb,
                                                 const float* __restrict__ bias,
                                                 const float* __restrict__ aux, int ldaux,
                                                 float* __restrict__ C, int ldc, int N, int M, int K,
                                                 const float* __restrict__ att_s = nullptr,
                                                 const float* __restrict__ att_d = nullptr,
                                                 float* __restrict__ a_src = nullptr,
                                                 float* __restrict__ a_dst = nullptr,
                                                 const GnpDesc gn = GnpDesc{}, const GnaDesc ga = GnaDesc{}) {
  constexpr int LDQ = BF ? TK + 4 : LDP;  // BF: 16-B aligned rows for the 8-float reads
  __shared__ __attribute__((aligned(16))) float smem[2 * TM * LDQ + 2 * TN * LDQ];
  float(*As)[TM][LDQ] = reinterpret_cast<float(*)[TM][LDQ]>(smem);
  float(*Bs)[TN][LDQ] = reinterpret_cast<float(*)[TN][LDQ]>(smem + 2 * TM * LDQ);  // Bs[j][k] = op(B)[k][j]
  // NW = 16: 4 x 4 waves, one 16 x 16 sub-tile each; NW = 8: 4 x 2 waves,
  // two side-by-side 16 x 16 sub-tiles each (NS), the A fragment shared
  static_assert(NW == 16 || NW == 8, "16 or 8 waves");
  constexpr int NT = 64 * NW, NS = 16 / NW;
  constexpr int PER = (TM * TK) / NT;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = NW == 16 ? wave >> 2 : wave >> 1;
  const int wc0 = NW == 16 ? wave & 3 : (wave & 1) * 2;  // the first sub-tile column
  int tx, ty;
  tile_xy(tx, ty);
  const int n0 = tx * TM, m0 = ty * TN;
  int mcs[NS];  // this lane's output column per sub-tile
#pragma unroll
  for (int s_ = 0; s_ < NS; ++s_) mcs[s_] = m0 + (wc0 + s_) * 16 + (lane & 15);
  f32x4 accs[NS];
#pragma unroll
  for (int s_ = 0; s_ < NS; ++s_) accs[s_] = f32x4{0.f, 0.f, 0.f, 0.f};
  // GNP: the epilogue's GraphNorm operands (the lane's 4 rows of x / keep, the
  // two segments' statistics, the column's parameters) loaded before the K loop
  float gx_[NS][GNP ? 4 : 1], gk_[NS][GNP ? 4 : 1];
  float gmu[NS][2], gsd[NS][2], gw_[NS], gb_[NS], gms_[NS];
  int gbound = 0;
  if constexpr (GNP) {
    const int seg0 = n0 / gn.seg_rows;
    gbound = (seg0 + 1) * gn.seg_rows;
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      const int mc = mcs[s_];
      gmu[s_][0] = gmu[s_][1] = 0.f;
      gsd[s_][0] = gsd[s_][1] = 1.f;
      gw_[s_] = gb_[s_] = gms_[s_] = 0.f;
      if (mc < M) {
        gw_[s_] = gn.w[mc];
        gb_[s_] = gn.b[mc];
        gms_[s_] = gn.ms[mc];
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (q == 0 || gbound < N) {
            const float* st = gn.stats + (size_t)(seg0 + q) * 2 * M;
            gmu[s_][q] = st[mc];
            gsd[s_][q] = st[M + mc];
          }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wr * 16 + 4 * (lane >> 4) + r;
        const bool ok = n < N && mc < M;
        gx_[s_][r] = ok ? gn.x[(size_t)n * M + mc] : 0.f;
        gk_[s_][r] = ok && gn.keep ? gn.keep[(size_t)n * M + mc] : 1.f;
      }
    }
  }
  float ra[PER], rb[PER];
  const long long g_it = (GNA && ga.iter) ? *ga.iter : 0;
  __shared__ float gpar[GNA ? 7 * kGnaMaxK : 1];
  int gbnd = 0;
  if constexpr (GNA) {
    const int seg0 = n0 / ga.seg_rows;
    gbnd = (seg0 + 1) * ga.seg_rows;
    const bool two = gbnd < N;
    for (int k = t; k < K; k += NT) {
      gpar[k] = ga.w[k];
      gpar[K + k] = ga.b[k];
      gpar[2 * K + k] = ga.ms[k];
      const float* st = ga.stats + (size_t)seg0 * 2 * K;
      gpar[3 * K + k] = st[k];
      gpar[4 * K + k] = st[K + k];
      gpar[5 * K + k] = two ? st[2 * K + k] : 0.f;
      gpar[6 * K + k] = two ? st[3 * K + k] : 1.f;
    }
  }
  // GNA: A as float4 quads, threads 0..511 (one row quad each per K-tile)
  float4 rq = make_float4(0.f, 0.f, 0.f, 0.f);
  constexpr int QPR = TK / 4;  // quads per tile row
  constexpr bool QUAD = GNA || QA;
  float4 rbq = make_float4(0.f, 0.f, 0.f, 0.f);  // QA: B as quads too (along k for BT, along m otherwise)
  auto load = [&](int k0) {
    if constexpr (QUAD) {
      if (t < TM * QPR) {
        const int n = n0 + t / QPR, k = k0 + 4 * (t % QPR);
        rq = (n < N && k < K) ? *reinterpret_cast<const float4*>(A + (size_t)n * lda + k)
                              : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if constexpr (QA) {
      if (t < TN * QPR) {
        if (BT) {
          const int m = m0 + t / QPR, k = k0 + 4 * (t % QPR);
          rbq = (m < M && k < K) ? *reinterpret_cast<const float4*>(B + (size_t)m * ldb + k)
                                 : make_float4(0.f, 0.f, 0.f, 0.f);
        } else {
          const int kk = k0 + t / (TN / 4), m = m0 + 4 * (t % (TN / 4));
          rbq = (m < M && kk < K) ? *reinterpret_cast<const float4*>(B + (size_t)kk * ldb + m)
                                  : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + NT * q;
      const int row = e / TK, kc = e % TK;
      const int n = n0 + row, k = k0 + kc;
      if constexpr (!QUAD) ra[q] = (n < N && k < K) ? A[(size_t)n * lda + k] : 0.f;
      if constexpr (!QA) {
        if (BT) {
          const int m = m0 + row;
          rb[q] = (m < M && k < K) ? B[(size_t)m * ldb + k] : 0.f;
        } else {
          const int kr = e / TN, j = e % TN;
          const int m = m0 + j, kk = k0 + kr;
          rb[q] = (m < M && kk < K) ? B[(size_t)kk * ldb + m] : 0.f;
        }
      }
    }
  };
  load(0);
  if constexpr (GNA) __syncthreads();  // the staged column operands
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += TK) {
    if constexpr (QUAD) {  // GNA: the loaded x quad of this K-tile -> y (stored once: one column tile)
      if (t < TM * QPR) {
        const int row = t / QPR, kq = 4 * (t % QPR);
        const int n = n0 + row, k = k0 + kq;
        if constexpr (GNA)
          if (n < N && k < K) rq = gna_quad(ga, gpar, rq, n, k, K, gbnd, g_it);
        As[buf][row][kq] = rq.x;
        As[buf][row][kq + 1] = rq.y;
        As[buf][row][kq + 2] = rq.z;
        As[buf][row][kq + 3] = rq.w;
      }
    }
    if constexpr (QA) {
      if (t < TN * QPR) {
        if (BT) {
          const int row = t / QPR, kq = 4 * (t % QPR);
          Bs[buf][row][kq] = rbq.x;
          Bs[buf][row][kq + 1] = rbq.y;
          Bs[buf][row][kq + 2] = rbq.z;
          Bs[buf][row][kq + 3] = rbq.w;
        } else {
          const int kr = t / (TN / 4), j4 = 4 * (t % (TN / 4));
          Bs[buf][j4][kr] = rbq.x;
          Bs[buf][j4 + 1][kr] = rbq.y;
          Bs[buf][j4 + 2][kr] = rbq.z;
          Bs[buf][j4 + 3][kr] = rbq.w;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + NT * q;
      if constexpr (!QUAD) As[buf][e / TK][e % TK] = ra[q];
      if constexpr (!QA) {
        if (BT) Bs[buf][e / TK][e % TK] = rb[q];
        else Bs[buf][e % TN][e / TN] = rb[q];
      }
    }
    __syncthreads();
    if (k0 + TK < K) load(k0 + TK);
    if constexpr (BF) {
      const float4* ap = reinterpret_cast<const float4*>(&As[buf][wr * 16 + (lane & 15)][8 * (lane >> 4)]);
      const float4 a0 = ap[0], a1 = ap[1];
      bf16x8 ha;
      ha[0] = static_cast<__bf16>(a0.x); ha[1] = static_cast<__bf16>(a0.y);
      ha[2] = static_cast<__bf16>(a0.z); ha[3] = static_cast<__bf16>(a0.w);
      ha[4] = static_cast<__bf16>(a1.x); ha[5] = static_cast<__bf16>(a1.y);
      ha[6] = static_cast<__bf16>(a1.z); ha[7] = static_cast<__bf16>(a1.w);
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) {
        const float4* bp = reinterpret_cast<const float4*>(&Bs[buf][(wc0 + s_) * 16 + (lane & 15)][8 * (lane >> 4)]);
        const float4 b0 = bp[0], b1 = bp[1];
        bf16x8 hb;
        hb[0] = static_cast<__bf16>(b0.x); hb[1] = static_cast<__bf16>(b0.y);
        hb[2] = static_cast<__bf16>(b0.z); hb[3] = static_cast<__bf16>(b0.w);
        hb[4] = static_cast<__bf16>(b1.x); hb[5] = static_cast<__bf16>(b1.y);
        hb[6] = static_cast<__bf16>(b1.z); hb[7] = static_cast<__bf16>(b1.w);
        accs[s_] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ha, hb, accs[s_], 0, 0, 0);
      }
    } else {
      const float* ar = &As[buf][wr * 16 + (lane & 15)][lane >> 4];
#pragma unroll
      for (int kk = 0; kk < TK; kk += 4) {
        const float av = ar[kk];
#pragma unroll
        for (int s_ = 0; s_ < NS; ++s_)
          accs[s_] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Bs[buf][(wc0 + s_) * 16 + (lane & 15)][(lane >> 4) + kk],
                                                          accs[s_], 0, 0, 0);
      }
    }
    buf ^= 1;
  }
  float bvs[NS];
#pragma unroll
  for (int s_ = 0; s_ < NS; ++s_) {
    const int mc = mcs[s_];
    const f32x4 acc = accs[s_];
    const float bv = (bias && mc < M) ? bias[mc] : 0.f;
    bvs[s_] = bv;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wr * 16 + 4 * (lane >> 4) + r;
      if (n < N && mc < M) {
        const float av = ACT >= 3 ? aux[(size_t)n * ldaux + mc] : 0.f;
        C[(size_t)n * ldc + mc] = act_fn<ACT>(acc[r] + bv, av);
      }
    }
  }
  if constexpr (GNP) {
    // column partials of gz = g_y [z > 0] keep and gz * xhat per segment slot:
    // the lane's 4 rows in order, the 4 lanes of the column (xor 16, 32),
    // then the 4 row waves of the column through LDS in order: deterministic
    float pa[NS][2], pb[NS][2];
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_) {
      const int mc = mcs[s_];
      const f32x4 acc = accs[s_];
      pa[s_][0] = pa[s_][1] = pb[s_][0] = pb[s_][1] = 0.f;
      if (mc < M) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = n0 + wr * 16 + 4 * (lane >> 4) + r;
          if (n < N) {
            const int sl = n >= gbound;
            const float xh = (gx_[s_][r] - (sl ? gmu[s_][1] : gmu[s_][0]) * gms_[s_]) / (sl ? gsd[s_][1] : gsd[s_][0]);
            const float gz = xh * gw_[s_] + gb_[s_] > 0.f ? acc[r] * gk_[s_][r] : 0.f;
            if (sl) {
              pa[s_][1] += gz;
              pb[s_][1] = fmaf(gz, xh, pb[s_][1]);
            } else {
              pa[s_][0] += gz;
              pb[s_][0] = fmaf(gz, xh, pb[s_][0]);
            }
          }
        }
      }
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        pa[s_][q] += __shfl_xor(pa[s_][q], 16, 64);
        pb[s_][q] += __shfl_xor(pb[s_][q], 16, 64);
        pa[s_][q] += __shfl_xor(pa[s_][q], 32, 64);
        pb[s_][q] += __shfl_xor(pb[s_][q], 32, 64);
      }
    }
    __syncthreads();  // every wave is done with the last K-tile's LDS images
    float* red = smem;  // [wr][64 columns][4]
    if (lane < 16)
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) {
        float* rp = red + ((wr * 64) + (wc0 + s_) * 16 + lane) * 4;
        rp[0] = pa[s_][0];
        rp[1] = pb[s_][0];
        rp[2] = pa[s_][1];
        rp[3] = pb[s_][1];
      }
    __syncthreads();
    if (wr == 0 && lane < 16)
#pragma unroll
      for (int s_ = 0; s_ < NS; ++s_) {
        const int mc = mcs[s_];
        if (mc >= M) continue;
        float sm[4] = {0.f, 0.f, 0.f, 0.f};
        for (int w = 0; w < 4; ++w) {
          const float* rp = red + ((w * 64) + (wc0 + s_) * 16 + lane) * 4;
#pragma unroll
          for (int q = 0; q < 4; ++q) sm[q] += rp[q];
        }
        float* tp = gn.tpart + (size_t)tx * 2 * M * 2;
        tp[(size_t)mc * 2] = sm[0];
        tp[(size_t)mc * 2 + 1] = sm[1];
        tp[(size_t)(M + mc) * 2] = sm[2];
        tp[(size_t)(M + mc) * 2 + 1] = sm[3];
      }
  }
  if constexpr (ATT) {
    // the 64 x 64 tile staged in LDS, then 16 threads per row dot 4 columns
    // each with att_s / att_d and combine over the 16 lanes
    float(*Ct)[TN + 1] = reinterpret_cast<float(*)[TN + 1]>(smem);
    __syncthreads();  // every wave is done with the last K-tile's images
#pragma unroll
    for (int s_ = 0; s_ < NS; ++s_)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        Ct[wr * 16 + 4 * (lane >> 4) + r][(wc0 + s_) * 16 + (lane & 15)] = accs[s_][r] + bvs[s_];
    __syncthreads();
    const int q = t & 15;
#pragma unroll
    for (int row = t >> 4; row < TM; row += NT / 16) {
      float ss = 0.f, sd = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = q * 4 + j;
        if (c < M) {
          const float v = Ct[row][c];
          ss = fmaf(v, att_s[c], ss);
          sd = fmaf(v, att_d[c], sd);
        }
      }
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        ss += __shfl_xor(ss, o, 64);
        sd += __shfl_xor(sd, o, 64);
      }
      if (q == 0 && n0 + row < N) {
        a_src[n0 + row] = ss;
        a_dst[n0 + row] = sd;
      }
    }
  }
}

template <bool BT, int ACT, bool ATT = false, bool BF = false, bool GNP = false, bool QA = false>
__global__ void __launch_bounds__(1024) k_gemm16(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                 int ldb, const float* __restrict__ bias,
                                                 const float* __restrict__ aux, int ldaux, float* __restrict__ C,
                                                 int ldc, int N, int M, int K,
                                                 const float* __restrict__ att_s = nullptr,
                                                 const float* __restrict__ att_d = nullptr,
                                                 float* __restrict__ a_src = nullptr,
                                                 float* __restrict__ a_dst = nullptr, const GnpDesc gn = GnpDesc{}) {
  gemm16_body<BT, ACT, ATT, BF, GNP, false, QA>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, N, M, K, att_s, att_d,
                                                a_src, a_dst, gn);
}

// 8-wave form (4 x 2 waves, two 16 x 16 sub-tiles each): four workgroups fit a
// CU where two 16-wave ones do, so a product of more than 512 row tiles (the
// critic's 38k stacked rows: 596) runs in one workgroup round instead of two
// (a second round costs a whole workgroup latency, ~1.7 us: DESIGN.md 9.5).
// Bit-identical to k_gemm16: the same sub-tiles, MFMA order and epilogues.
template <bool BT, int ACT, bool ATT = false, bool BF = false, bool GNP = false, bool QA = false>
__global__ void __launch_bounds__(512) k_gemm8w(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                int ldb, const float* __restrict__ bias,
                                                const float* __restrict__ aux, int ldaux, float* __restrict__ C,
                                                int ldc, int N, int M, int K,
                                                const float* __restrict__ att_s = nullptr,
                                                const float* __restrict__ att_d = nullptr,
                                                float* __restrict__ a_src = nullptr,
                                                float* __restrict__ a_dst = nullptr, const GnpDesc gn = GnpDesc{}) {
  gemm16_body<BT, ACT, ATT, BF, GNP, false, QA, 8>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, N, M, K, att_s, att_d,
                                                   a_src, a_dst, gn);
}

// the projection GEMM with the GraphNorm applied to its operand (vg_gat_lin_att_gn):
// held to 64 VGPRs so two 16-wave workgroups share a CU (78 unconstrained:
// the per-element GraphNorm operands and the dropout draw)
__global__ void __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8, 8)))
k_gemm16_gna(const float* __restrict__ A, const float* __restrict__ B, float* __restrict__ C, int N, int M, int K,
             const float* __restrict__ att_s, const float* __restrict__ att_d, float* __restrict__ a_src,
             float* __restrict__ a_dst, const GnaDesc ga) {
  gemm16_body<true, 0, true, false, false, true>(A, K, B, K, nullptr, nullptr, 0, C, M, N, M, K, att_s, att_d,
                                                 a_src, a_dst, GnpDesc{}, ga);
}

// k_gemm_ln's epilogue over the staged tile Ct [TMR][TN * NT + 1] (bias and
// addend included): the attention projections (ATT) or the row statistics,
// then the normalised, activated rows stored coalesced.  NTH threads.
template <int NT, int TMR, bool ATT, int NTH>
__device__ __forceinline__ void ln_tile_epilogue(const float* Ct, float* s_mu, float* s_rs, int t, int n0, int N,
                                                 int M, const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, float eps, float slope,
                                                 float* __restrict__ H, float* __restrict__ Y,
                                                 float* __restrict__ mean, float* __restrict__ rstd,
                                                 const float* __restrict__ att_s, const float* __restrict__ att_d,
                                                 float* __restrict__ a_src, float* __restrict__ a_dst, int ldy) {
  constexpr int TNC = TN * NT;
  constexpr int CT = TNC + 1;
  if constexpr (ATT) {  // attention projections: TPR threads per row, then coalesced H stores
    constexpr int TPR = NTH / TMR;
    constexpr int CPT = TNC / TPR;
    const int row = t / TPR, q = t % TPR;
    const float* cr = Ct + row * CT + q * CPT;
    float ss = 0.f, sd = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int c = q * CPT + i;
      if (c < M) {
        ss = fmaf(cr[i], att_s[c], ss);
        sd = fmaf(cr[i], att_d[c], sd);
      }
    }
#pragma unroll
    for (int off = 1; off < TPR; off <<= 1) {
      ss += __shfl_xor(ss, off, 64);
      sd += __shfl_xor(sd, off, 64);
    }
    if (q == 0 && n0 + row < N) {
      a_src[n0 + row] = ss;
      a_dst[n0 + row] = sd;
    }
    for (int idx = t; idx < TMR * TNC; idx += NTH) {
      const int r = idx / TNC, c = idx % TNC, n = n0 + r;
      if (c < M && n < N) H[(size_t)n * M + c] = Ct[r * CT + c];
    }
    return;
  }
  {  // row statistics: TPR threads per row, two-pass
    constexpr int TPR = NTH / TMR;
    constexpr int CPT = TNC / TPR;
    const int row = t / TPR, q = t % TPR;
    const float* cr = Ct + row * CT + q * CPT;
    float v[CPT];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      v[i] = q * CPT + i < M ? cr[i] : 0.f;
      s += v[i];
    }
#pragma unroll
    for (int off = 1; off < TPR; off <<= 1) s += __shfl_xor(s, off, 64);
    const float mu = s / static_cast<float>(M);
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < CPT; ++i)
      if (q * CPT + i < M) {
        const float d = v[i] - mu;
        ss = fmaf(d, d, ss);
      }
#pragma unroll
    for (int off = 1; off < TPR; off <<= 1) ss += __shfl_xor(ss, off, 64);
    const float rs = rsqrtf(ss / static_cast<float>(M) + eps);
    if (q == 0) {
      s_mu[row] = mu;
      s_rs[row] = rs;
      if (mean && n0 + row < N) {
        mean[n0 + row] = mu;
        rstd[n0 + row] = rs;
      }
    }
  }
  __syncthreads();
  // normalise + activate, lanes along the columns (coalesced row stores)
  for (int idx = t; idx < TMR * TNC; idx += NTH) {
    const int row = idx / TNC, c = idx % TNC, n = n0 + row;
    if (c < M && n < N) {
      const float v = Ct[row * CT + c];
      if (H) H[(size_t)n * M + c] = v;
      const float z = fmaf((v - s_mu[row]) * s_rs[row], gamma[c], beta[c]);
      Y[(size_t)n * ldy + c] = z > 0.f ? z : z * slope;
    }
  }
}

// Y = leaky_relu(LayerNorm(A . B^T + bias; gamma, beta, eps), slope) with the
// LayerNorm in the epilogue: the [Linear -> LayerNorm -> LeakyReLU(0.2)]
// blocks of the generator's MLPs (models.py:33-47, 49-66, 92-113).  A
// workgroup owns 64 rows x 64*NT columns -- every column of the layer
// (M <= 64 NT) -- so each row's statistics are complete in the tile: the tile
// is staged through LDS, four threads per row take two-pass mean / biased
// variance (as torch), then the whole workgroup normalises, activates and
// stores with lanes along the columns (coalesced).  H (nullable) receives the
// pre-LayerNorm activations and mean / rstd (nullable) the row statistics for
// the backward; the no-grad forwards skip both.  Saves the separate LayerNorm
// launch and its read of the GEMM output.
// TMR rows per block: 64 (2 x 2 waves) or 32 (1 x 4 waves; twice the blocks,
// for grids that would leave CUs idle or a long last round).
// ATT: no LayerNorm -- H = A B^T and a_src / a_dst = H . att_s / att_d per row
// (vg_gat_lin_att for 64 < C <= 128; gamma / beta unused, Y unused).
// Multi-source A for k_gemm_ln (vg_gemm_ln_act_ms): the K columns are the
// concatenation of up to kMaxSrc row-major sources, each with its own stride,
// its first column in W, and optionally rows taken modulo rows_mod (a source
// shared by stacked copies); `add` (rows modulo add_rows) is added before the
// LayerNorm.  Passed by value in kernarg.
constexpr int kMaxSrc = 4;
struct MsDesc {
  const float* p[kMaxSrc];
  int ld[kMaxSrc], kend[kMaxSrc], wcol[kMaxSrc], rmod[kMaxSrc];
  int nsrc;
  const float* add;
  int ld_add, add_rows;
};

// QL (bf16 only): operands staged from float4 quads with 8-byte bf16 stores (as k_gemm's QA).
template <int NT, int TMR = TM, bool ATT = false, bool MS = false, bool BF = false, bool QL = false>
__global__ void __launch_bounds__(256) k_gemm_ln(const float* __restrict__ A, int lda,
                                                 const float* __restrict__ B, int ldb,
                                                 const float* __restrict__ bias, int N, int M, int K,
                                                 const float* __restrict__ gamma,
                                                 const float* __restrict__ beta, float eps,
                                                 float slope, float* __restrict__ H,
                                                 float* __restrict__ Y, float* __restrict__ mean,
                                                 float* __restrict__ rstd,
                                                 const float* __restrict__ att_s = nullptr,
                                                 const float* __restrict__ att_d = nullptr,
                                                 float* __restrict__ a_src = nullptr,
                                                 float* __restrict__ a_dst = nullptr, int ldy = 0,
                                                 const MsDesc ms = MsDesc{}) {
  if (ldy == 0) ldy = M;
  constexpr int TNC = TN * NT;
  constexpr int CT = TNC + 1;  // staged tile row pitch
  constexpr int WCOLS = 4 / (TMR / 32);       // waves across the columns
  constexpr int NJ = TNC / (32 * WCOLS);      // 32-column MFMA tiles per wave
  static_assert(NJ >= 1, "TMR = 32 needs 128 columns");
  __shared__ __attribute__((aligned(16))) float smem[2 * TMR * LDP + 2 * TNC * LDP];
  __shared__ float s_mu[TMR], s_rs[TMR];
  float(*As)[TMR][LDP] = reinterpret_cast<float(*)[TMR][LDP]>(smem);
  float(*Bs)[TNC][LDP] = reinterpret_cast<float(*)[TNC][LDP]>(smem + 2 * TMR * LDP);
  constexpr int PA = (TMR * TK) / 256, PB = (TNC * TK) / 256;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave / WCOLS, wc = wave % WCOLS;
  int tx, ty;
  tile_xy(tx, ty);
  const int n0 = tx * TMR;
  f32x16 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  // MS: sources are TK-aligned column blocks, so one source serves the chunk
  auto chunk_src = [&](int k0, const float*& asrc, int& ald, int& acol, int& wcol) {
    asrc = A;
    ald = lda;
    acol = k0;
    wcol = k0;
    if constexpr (MS) {
      int sidx = 0;
#pragma unroll
      for (int i = 0; i < kMaxSrc - 1; ++i)
        if (i < ms.nsrc - 1 && k0 >= ms.kend[i]) sidx = i + 1;
      const int kb = sidx > 0 ? ms.kend[sidx - 1] : 0;
      asrc = ms.p[sidx];
      ald = ms.ld[sidx];
      acol = k0 - kb;
      wcol = ms.wcol[sidx] + (k0 - kb);
    }
  };
  // BF: the same coalesced global loads, staged as bf16 (Ah[buf][n][k], Bh[buf][m][k])
  __bf16(*Ah)[TMR][LDH] = reinterpret_cast<__bf16(*)[TMR][LDH]>(smem);
  __bf16(*Bh)[TNC][LDH] = reinterpret_cast<__bf16(*)[TNC][LDH]>(smem + 2 * TMR * LDP);
  static_assert(!QL || BF, "quad staging for the bf16 images");
  constexpr int QPR = TK / 4, NQA = (TMR * QPR) / 256, NQB = (TNC * QPR) / 256;  // quads per thread
  float ra[QL ? 1 : PA], rb[QL ? 1 : PB];
  float4 qa[QL ? NQA : 1], qb[QL ? NQB : 1];
  auto load = [&](int k0) {
    const float* asrc;
    int ald, acol, wcol;
    chunk_src(k0, asrc, ald, acol, wcol);
    if constexpr (QL) {
#pragma unroll
      for (int u = 0; u < NQA; ++u) {
        const int g = t + 256 * u;
        const int n = n0 + g / QPR, kq = 4 * (g % QPR);
        qa[u] = (n < N && k0 + kq < K) ? *reinterpret_cast<const float4*>(asrc + (size_t)n * ald + acol + kq)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < NQB; ++u) {
        const int g = t + 256 * u;
        const int m = g / QPR, kq = 4 * (g % QPR);
        qb[u] = (m < M && k0 + kq < K) ? *reinterpret_cast<const float4*>(B + (size_t)m * ldb + wcol + kq)
                                       : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
#pragma unroll
      for (int q = 0; q < PA; ++q) {
        const int e = t + 256 * q;
        const int n = n0 + e / TK, kc = e % TK;
        ra[q] = (n < N && k0 + kc < K) ? asrc[(size_t)n * ald + acol + kc] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int e = t + 256 * q;
        const int m = e / TK, kc = e % TK;
        rb[q] = (m < M && k0 + kc < K) ? B[(size_t)m * ldb + wcol + kc] : 0.f;
      }
    }
  };
  load(0);
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += TK) {
    if constexpr (QL) {
#pragma unroll
      for (int u = 0; u < NQA; ++u) {
        const int g = t + 256 * u;
        const float v[4] = {qa[u].x, qa[u].y, qa[u].z, qa[u].w};
        *reinterpret_cast<bf16x4*>(&Ah[buf][g / QPR][4 * (g % QPR)]) = to_bf4(v);
      }
#pragma unroll
      for (int u = 0; u < NQB; ++u) {
        const int g = t + 256 * u;
        const float v[4] = {qb[u].x, qb[u].y, qb[u].z, qb[u].w};
        *reinterpret_cast<bf16x4*>(&Bh[buf][g / QPR][4 * (g % QPR)]) = to_bf4(v);
      }
    } else {
#pragma unroll
      for (int q = 0; q < PA; ++q) {
        const int e = t + 256 * q;
        if constexpr (BF) Ah[buf][e / TK][e % TK] = static_cast<__bf16>(ra[q]);
        else As[buf][e / TK][e % TK] = ra[q];
      }
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int e = t + 256 * q;
        if constexpr (BF) Bh[buf][e / TK][e % TK] = static_cast<__bf16>(rb[q]);
        else Bs[buf][e / TK][e % TK] = rb[q];
      }
    }
    __syncthreads();
    if (k0 + TK < K) load(k0 + TK);
    if constexpr (BF) {
      const int h8 = 8 * (lane >> 5);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int s16 = 0; s16 < TK; s16 += 16)
          acc[j] = mfma_bf(&Ah[buf][wr * 32 + (lane & 31)][s16 + h8],
                           &Bh[buf][j * 32 * WCOLS + wc * 32 + (lane & 31)][s16 + h8], acc[j]);
    } else {
      const float* ar = &As[buf][wr * 32 + (lane & 31)][lane >> 5];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const float* br = &Bs[buf][j * 32 * WCOLS + wc * 32 + (lane & 31)][lane >> 5];
#pragma unroll
        for (int kk = 0; kk < TK; kk += 2)
          acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(ar[kk], br[kk], acc[j], 0, 0, 0);
      }
    }
    buf ^= 1;
  }
  // stage the full-width tile (+ bias) in LDS
  __syncthreads();
  float* Ct = smem;
  const int add0 = MS && ms.add ? n0 % ms.add_rows : 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 32 * WCOLS + wc * 32 + (lane & 31);
    const float bv = (bias && c < M) ? bias[c] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      float v = acc[j][r] + bv;
      if constexpr (MS) {  // addend row (n0 + rl) mod add_rows; rl < TMR <= add_rows
        if (ms.add && n0 + rl < N && c < M) {
          int ar = add0 + rl;
          if (ar >= ms.add_rows) ar -= ms.add_rows;
          v += ms.add[(size_t)ar * ms.ld_add + c];
        }
      }
      Ct[rl * CT + c] = v;
    }
  }
  __syncthreads();
  ln_tile_epilogue<NT, TMR, ATT, 256>(Ct, s_mu, s_rs, t, n0, N, M, gamma, beta, eps, slope, H, Y, mean, rstd, att_s,
                                      att_d, a_src, a_dst, ldy);
}

// k_gemm_ln with 16 waves (f32): 16 x 16 v_mfma_f32_16x16x4f32 sub-tiles,
// TMR / 16 row waves x 16 / (TMR / 16) column waves, NJ sub-tiles per wave
// (as k_gemm16 against k_gemm: 4x the waves to cover the global -> LDS
// latency of these K <= 128 products).  Same arguments and epilogue.
// QL: A and W loaded as float4 quads (every source's ld, column offsets and
// pointer 16-B aligned; quad_ln) instead of scalars, as in k_gemm16's QA.
template <int NT, int TMR = TM, bool ATT = false, bool MS = false, bool QL = false>
__global__ void __launch_bounds__(1024) k_gemm_ln16(const float* __restrict__ A, int lda,
                                                    const float* __restrict__ B, int ldb,
                                                    const float* __restrict__ bias, int N, int M, int K,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float eps,
                                                    float slope, float* __restrict__ H,
                                                    float* __restrict__ Y, float* __restrict__ mean,
                                                    float* __restrict__ rstd,
                                                    const float* __restrict__ att_s = nullptr,
                                                    const float* __restrict__ att_d = nullptr,
                                                    float* __restrict__ a_src = nullptr,
                                                    float* __restrict__ a_dst = nullptr, int ldy = 0,
                                                    const MsDesc ms = MsDesc{}) {
  if (ldy == 0) ldy = M;
  constexpr int TNC = TN * NT;
  constexpr int CT = TNC + 1;
  constexpr int WRW = TMR / 16, WCW = 16 / WRW;  // row / column waves
  constexpr int NJ = TNC / (16 * WCW);           // 16-column sub-tiles per wave
  static_assert(NJ >= 1 && WRW * WCW == 16, "tile shape");
  constexpr bool FR = VG_FRAG128;
  constexpr int PIT = FR ? FP : LDP;  // image row pitch
  __shared__ __attribute__((aligned(16))) float smem[2 * TMR * PIT + 2 * TNC * PIT];
  __shared__ float s_mu[TMR], s_rs[TMR];
  float* As = smem;                   // [2][TMR * PIT]
  float* Bs = smem + 2 * TMR * PIT;   // [2][TNC * PIT]
  auto at = [&](int r, int kc) { return FR ? frag_pos(r, kc) : r * LDP + kc; };
  constexpr int PA = (TMR * TK) / 1024, PB = (TNC * TK) / 1024;
  static_assert(PA >= 1 && PB >= 1, "tile shape");
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave / WCW, wc = wave % WCW;
  int tx, ty;
  tile_xy(tx, ty);
  const int n0 = tx * TMR;
  f32x4 acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto chunk_src = [&](int k0, const float*& asrc, int& ald, int& acol, int& wcol) {
    asrc = A;
    ald = lda;
    acol = k0;
    wcol = k0;
    if constexpr (MS) {
      int sidx = 0;
#pragma unroll
      for (int i = 0; i < kMaxSrc - 1; ++i)
        if (i < ms.nsrc - 1 && k0 >= ms.kend[i]) sidx = i + 1;
      const int kb = sidx > 0 ? ms.kend[sidx - 1] : 0;
      asrc = ms.p[sidx];
      ald = ms.ld[sidx];
      acol = k0 - kb;
      wcol = ms.wcol[sidx] + (k0 - kb);
    }
  };
  float ra[PA], rb[PB];
  constexpr int QPR = TK / 4, NQA = TMR * QPR, NQB = TNC * QPR;  // quads per row / of A / of W per K-tile
  static_assert(!QL || (NQA <= 1024 && NQB <= 1024), "one quad per thread");
  float4 qa = make_float4(0.f, 0.f, 0.f, 0.f), qb = qa;
  auto load = [&](int k0) {
    const float* asrc;
    int ald, acol, wcol;
    chunk_src(k0, asrc, ald, acol, wcol);
    if constexpr (QL) {
      const int kq = 4 * (t % QPR);
      if (t < NQA) {
        const int n = n0 + t / QPR;
        qa = (n < N && k0 + kq < K) ? *reinterpret_cast<const float4*>(asrc + (size_t)n * ald + acol + kq)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      if (t < NQB) {
        const int m = t / QPR;
        qb = (m < M && k0 + kq < K) ? *reinterpret_cast<const float4*>(B + (size_t)m * ldb + wcol + kq)
                                    : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    } else {
#pragma unroll
      for (int q = 0; q < PA; ++q) {
        const int e = t + 1024 * q;
        const int n = n0 + e / TK, kc = e % TK;
        ra[q] = (n < N && k0 + kc < K) ? asrc[(size_t)n * ald + acol + kc] : 0.f;
      }
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int e = t + 1024 * q;
        const int m = e / TK, kc = e % TK;
        rb[q] = (m < M && k0 + kc < K) ? B[(size_t)m * ldb + wcol + kc] : 0.f;
      }
    }
  };
  load(0);
  int buf = 0;
  for (int k0 = 0; k0 < K; k0 += TK) {
    if constexpr (QL) {
      const int kq = 4 * (t % QPR);
      if (t < NQA) {
        float* d = As + buf * TMR * PIT;
        const int r = t / QPR;
        d[at(r, kq)] = qa.x;
        d[at(r, kq + 1)] = qa.y;
        d[at(r, kq + 2)] = qa.z;
        d[at(r, kq + 3)] = qa.w;
      }
      if (t < NQB) {
        float* d = Bs + buf * TNC * PIT;
        const int r = t / QPR;
        d[at(r, kq)] = qb.x;
        d[at(r, kq + 1)] = qb.y;
        d[at(r, kq + 2)] = qb.z;
        d[at(r, kq + 3)] = qb.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < PA; ++q) {
        const int e = t + 1024 * q;
        As[buf * TMR * PIT + at(e / TK, e % TK)] = ra[q];
      }
#pragma unroll
      for (int q = 0; q < PB; ++q) {
        const int e = t + 1024 * q;
        Bs[buf * TNC * PIT + at(e / TK, e % TK)] = rb[q];
      }
    }
    __syncthreads();
    if (k0 + TK < K) load(k0 + TK);
    if constexpr (FR) {
      const float* Ai = As + buf * TMR * PIT;
      const float* Bi = Bs + buf * TNC * PIT;
      const int ra_ = wr * 16 + (lane & 15), g = lane >> 4;
      const float4 a0 = *reinterpret_cast<const float4*>(Ai + frag_at(ra_, g, 0));
      const float4 a1 = *reinterpret_cast<const float4*>(Ai + frag_at(ra_, g, 1));
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int rb_ = j * 16 * WCW + wc * 16 + (lane & 15);
        const float4 b0 = *reinterpret_cast<const float4*>(Bi + frag_at(rb_, g, 0));
        const float4 b1 = *reinterpret_cast<const float4*>(Bi + frag_at(rb_, g, 1));
        const float bv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[i], acc[j], 0, 0, 0);
      }
    } else {
      const float* ar = As + buf * TMR * PIT + (wr * 16 + (lane & 15)) * LDP + (lane >> 4);
#pragma unroll
      for (int kk = 0; kk < TK; kk += 4)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(
              ar[kk], Bs[buf * TNC * PIT + (j * 16 * WCW + wc * 16 + (lane & 15)) * LDP + (lane >> 4) + kk], acc[j], 0,
              0, 0);
    }
    buf ^= 1;
  }
  // stage the full-width tile (+ bias, + addend) in LDS
  __syncthreads();
  float* Ct = smem;
  const int add0 = MS && ms.add ? n0 % ms.add_rows : 0;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    const int c = j * 16 * WCW + wc * 16 + (lane & 15);
    const float bv = (bias && c < M) ? bias[c] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wr * 16 + 4 * (lane >> 4) + r;
      float v = acc[j][r] + bv;
      if constexpr (MS) {  // addend row (n0 + rl) mod add_rows; rl < TMR <= add_rows
        if (ms.add && n0 + rl < N && c < M) {
          int ar2 = add0 + rl;
          if (ar2 >= ms.add_rows) ar2 -= ms.add_rows;
          v += ms.add[(size_t)ar2 * ms.ld_add + c];
        }
      }
      Ct[rl * CT + c] = v;
    }
  }
  __syncthreads();
  ln_tile_epilogue<NT, TMR, ATT, 1024>(Ct, s_mu, s_rs, t, n0, N, M, gamma, beta, eps, slope, H, Y, mean, rstd, att_s,
                                       att_d, a_src, a_dst, ldy);
}

// k_gemm_ln16<2, 32> (M in (64, 128], 32-row tiles, 16 waves, the same
// fragment-ordered images and MFMA sequence -- bit-identical results) as a
// PERSISTENT launch with W resident in LDS: one 1024-thread workgroup per CU
// stages the whole weight image (K <= 32 * KT) once and walks a contiguous
// range of row tiles; each tile's A is loaded into registers while the
// previous tile's MFMAs and LayerNorm epilogue run.  k_gemm_ln16 re-streamed
// W (4x the bytes of A at M = 128) through a 32-wide K-tile pipeline one
// step deep, so every K-tile waited for an L2 round trip: 33-35 % of the f32
// MFMA rate at 63.5k rows.  The A image doubles as the epilogue's staged
// tile (Ct), so W + A fit the LDS at K = 160.
template <int KT, bool MS>
__global__ void __launch_bounds__(1024) k_gemm_ln_wres(const float* __restrict__ A, int lda,
                                                       const float* __restrict__ B, int ldb,
                                                       const float* __restrict__ bias, int N, int M, int K,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float eps, float slope,
                                                       float* __restrict__ H, float* __restrict__ Y,
                                                       float* __restrict__ mean, float* __restrict__ rstd, int ldy,
                                                       const MsDesc ms) {
  constexpr int TMR = 32, NT = 2, TNC = TN * NT, CT = TNC + 1;
  constexpr int WRW = TMR / 16, WCW = 16 / WRW;  // 2 row waves x 8 column waves, one 16 x 16 sub-tile each
  static_assert(TNC / (16 * WCW) == 1, "one sub-tile per wave");
  constexpr int AIMG = TMR * FP, BIMG = TNC * FP;  // floats per 32-wide K-tile image
  extern __shared__ float4 dyn4[];
  float* Ws = reinterpret_cast<float*>(dyn4);  // [KT][BIMG]
  float* As = Ws + KT * BIMG;                  // [KT][AIMG], Ct during the epilogue
  __shared__ float s_mu[TMR], s_rs[TMR];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int wr = wave / WCW, wc = wave % WCW;
  const int kq4 = K / 4;  // quads per row (K % 4 == 0)
  // the tile range of this workgroup (XCD-aware: contiguous tiles per XCD)
  const int tiles = (N + TMR - 1) / TMR;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int t0 = (int)((long long)tiles * lb / gridDim.x), t1 = (int)((long long)tiles * (lb + 1) / gridDim.x);
  auto a_src = [&](int k, const float*& p, int& ld, int& col) {
    p = A;
    ld = lda;
    col = k;
    if constexpr (MS) {
      int sidx = 0;
#pragma unroll
      for (int i = 0; i < kMaxSrc - 1; ++i)
        if (i < ms.nsrc - 1 && k >= ms.kend[i]) sidx = i + 1;
      const int kb = sidx > 0 ? ms.kend[sidx - 1] : 0;
      p = ms.p[sidx];
      ld = ms.ld[sidx];
      col = k - kb;
    }
  };
  auto w_col = [&](int k) {
    if constexpr (MS) {
      int sidx = 0;
#pragma unroll
      for (int i = 0; i < kMaxSrc - 1; ++i)
        if (i < ms.nsrc - 1 && k >= ms.kend[i]) sidx = i + 1;
      const int kb = sidx > 0 ? ms.kend[sidx - 1] : 0;
      return ms.wcol[sidx] + (k - kb);
    }
    return k;
  };
  // W image, once: quads along k of each output column's row of W
  for (int g = t; g < TNC * kq4; g += 1024) {
    const int m = g / kq4, k = 4 * (g % kq4);
    const float4 v = m < M ? *reinterpret_cast<const float4*>(B + (size_t)m * ldb + w_col(k)) : make_float4(0.f, 0.f, 0.f, 0.f);
    float* d = Ws + (k >> 5) * BIMG;
    const int kk = k & 31;
    d[frag_pos(m, kk)] = v.x;
    d[frag_pos(m, kk + 1)] = v.y;
    d[frag_pos(m, kk + 2)] = v.z;
    d[frag_pos(m, kk + 3)] = v.w;
  }
  // the zero columns of a K-tile past K (K % 32 != 0)
  for (int g = t; g < TNC * (KT * 32 - K); g += 1024) {
    const int m = g / (KT * 32 - K), k = K + g % (KT * 32 - K);
    Ws[(k >> 5) * BIMG + frag_pos(m, k & 31)] = 0.f;
  }
  constexpr int QPT = (TMR * KT * 8 + 1023) / 1024;  // A quads per thread and tile (<= 32 * K / 4)
  float4 qa[QPT];
  auto load_a = [&](int tile) {
    const int n0 = tile * TMR;
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
      const int g = t + 1024 * u;
      const int r = g / kq4, k = 4 * (g % kq4);
      qa[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (g < TMR * kq4 && n0 + r < N) {
        const float* p;
        int ld, col;
        a_src(k, p, ld, col);
        qa[u] = *reinterpret_cast<const float4*>(p + (size_t)(n0 + r) * ld + col);
      }
    }
  };
  auto store_a = [&]() {
#pragma unroll
    for (int u = 0; u < QPT; ++u) {
      const int g = t + 1024 * u;
      if (g < TMR * kq4) {
        const int r = g / kq4, k = 4 * (g % kq4);
        float* d = As + (k >> 5) * AIMG;
        const int kk = k & 31;
        d[frag_pos(r, kk)] = qa[u].x;
        d[frag_pos(r, kk + 1)] = qa[u].y;
        d[frag_pos(r, kk + 2)] = qa[u].z;
        d[frag_pos(r, kk + 3)] = qa[u].w;
      }
    }
    for (int g = t; g < TMR * (KT * 32 - K); g += 1024) {
      const int r = g / (KT * 32 - K), k = K + g % (KT * 32 - K);
      As[(k >> 5) * AIMG + frag_pos(r, k & 31)] = 0.f;
    }
  };
  if (t0 < t1) {
    load_a(t0);
    store_a();
  }
  const int c = wc * 16 + (lane & 15);
  const float bv = (bias && c < M) ? bias[c] : 0.f;
  __syncthreads();
  for (int tile = t0; tile < t1; ++tile) {
    const int n0 = tile * TMR;
    if (tile + 1 < t1) load_a(tile + 1);  // in flight under the MFMAs and the epilogue
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const int ra_ = wr * 16 + (lane & 15), g = lane >> 4;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const float* Ai = As + kt * AIMG;
      const float* Bi = Ws + kt * BIMG;
      const float4 a0 = *reinterpret_cast<const float4*>(Ai + frag_at(ra_, g, 0));
      const float4 a1 = *reinterpret_cast<const float4*>(Ai + frag_at(ra_, g, 1));
      const float av[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
      const float4 b0 = *reinterpret_cast<const float4*>(Bi + frag_at(c, g, 0));
      const float4 b1 = *reinterpret_cast<const float4*>(Bi + frag_at(c, g, 1));
      const float bw[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
#pragma unroll
      for (int i = 0; i < 8; ++i) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bw[i], acc, 0, 0, 0);
    }
    __syncthreads();  // every wave is done with the A images: they become Ct
    float* Ct = As;
    const int add0 = MS && ms.add ? n0 % ms.add_rows : 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int rl = wr * 16 + 4 * (lane >> 4) + r;
      float v = acc[r] + bv;
      if constexpr (MS) {
        if (ms.add && n0 + rl < N && c < M) {
          int ar2 = add0 + rl;
          if (ar2 >= ms.add_rows) ar2 -= ms.add_rows;
          v += ms.add[(size_t)ar2 * ms.ld_add + c];
        }
      }
      Ct[rl * CT + c] = v;
    }
    __syncthreads();
    ln_tile_epilogue<NT, TMR, false, 1024>(Ct, s_mu, s_rs, t, n0, N, M, gamma, beta, eps, slope, H, Y, mean, rstd,
                                           nullptr, nullptr, nullptr, nullptr, ldy);
    __syncthreads();  // Ct read out
    if (tile + 1 < t1) store_a();
    __syncthreads();
  }
}

// W images + the A region (the A images, or the staged tile if larger)
template <int KT>
constexpr int wres_lds_bytes() {
  return (KT * TN * 2 * FP + (KT * 32 * FP > 32 * (2 * TN + 1) ? KT * 32 * FP : 32 * (2 * TN + 1))) * 4;
}

// part[chunk][M][K] = A[chunk rows]^T . B[chunk rows];  pdb[chunk][M] = column sums of A.
// `rows` rows of the N reduction per chunk (a multiple of TK), pipelined like k_gemm.
// G row groups of 4 waves per workgroup: group g takes the chunk's K-steps
// g, g+G, ... into its own LDS buffers (two waves per SIMD for G = 2, so one
// group's MFMAs cover the other's loads -- the f32 MFMA alone is 1024 cycles
// per 32-row step), and the groups' accumulators are added in group order at
// the end (deterministic).
// One (row chunk, 64 x 64 output tile) of a split-K product: the body of
// k_gemm_tn (one product per launch) and k_gemm_tn_group (many).
// smem: the kernel's tn_smem_floats<G>() floats (shared by both tile kinds)
template <int G>
constexpr int tn_smem_floats() { return G * 2 * TK * (TM + 1) + G * 2 * TK * (TN + 1); }

template <int G, bool BF>
__device__ __forceinline__ void tn_tile(float* smem, const float* __restrict__ A, int lda, const float* __restrict__ B,
                                        int ldb, int N, int M, int K, int rows, int chunk, int m0, int k0,
                                        float* __restrict__ part, float* __restrict__ pdb, int db_rows) {
  float(*As)[2][TK][TM + 1] = reinterpret_cast<float(*)[2][TK][TM + 1]>(smem);  // As[g][buf][n][m]
  float(*Bs)[2][TK][TN + 1] = reinterpret_cast<float(*)[2][TK][TN + 1]>(smem + G * 2 * TK * (TM + 1));  // [n][k]
  constexpr int PER = (TK * TM) / 256;
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255, lane = t & 63, wave = t >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int nb = chunk * rows, ne = min(N, nb + rows);
  const int steps = ne > nb ? (ne - nb + TK - 1) / TK : 0;
  const int iters = (steps + G - 1) / G;
  const bool do_db = pdb && k0 == 0;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float dbs = 0.f;
  // BF: the same coalesced global loads, staged as bf16 and transposed --
  // Ah[g][buf][m][n], Bh[g][buf][k][n] -- so a lane's 8 consecutive n are one read
  __bf16(*Ah)[2][TM][LDH] = reinterpret_cast<__bf16(*)[2][TM][LDH]>(smem);
  __bf16(*Bh)[2][TN][LDH] = reinterpret_cast<__bf16(*)[2][TN][LDH]>(smem + G * 2 * TK * (TM + 1));
  // BF: thread t takes column t & 63 and a quad of 4 rows n per q (each
  // load coalesced along the columns), so element (q, i) is row
  // 4 * (e / TM) + i of the f32 mapping's row e / TM -- one 8-byte store into
  // the transposed image per quad
  float ra[PER], rb[PER];
  auto load = [&](int st) {
    const int n1 = nb + st * TK;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      const int c = e % TM;
      const int r = BF ? 4 * ((t >> 6) + 4 * (q >> 2)) + (q & 3) : e / TM;
      const int n = n1 + r;
      const bool in = st < steps && n < ne;
      ra[q] = (in && m0 + c < M) ? A[(size_t)n * lda + m0 + c] : 0.f;
      rb[q] = (in && k0 + c < K) ? B[(size_t)n * ldb + k0 + c] : 0.f;
    }
  };
  load(grp);
  int buf = 0;
  for (int it = 0, st = grp; it < iters; ++it, st += G) {
    const int n1 = nb + st * TK;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int e = t + 256 * q;
      const int r = BF ? 4 * ((t >> 6) + 4 * (q >> 2)) + (q & 3) : e / TM;
      if constexpr (!BF) {
        As[grp][buf][r][e % TM] = ra[q];
        Bs[grp][buf][r][e % TM] = rb[q];
      }
      if (do_db && n1 + r < db_rows) dbs += ra[q];  // column (t & 63), row r (0 past ne)
    }
    if constexpr (BF) {  // transposed images: the reduction index n contiguous
#pragma unroll
      for (int q4 = 0; q4 < PER / 4; ++q4) {
        const int c = t & 63, r0 = 4 * ((t >> 6) + 4 * q4);
        const float va[4] = {ra[4 * q4], ra[4 * q4 + 1], ra[4 * q4 + 2], ra[4 * q4 + 3]};
        const float vb[4] = {rb[4 * q4], rb[4 * q4 + 1], rb[4 * q4 + 2], rb[4 * q4 + 3]};
        *reinterpret_cast<bf16x4*>(&Ah[grp][buf][c][r0]) = to_bf4(va);
        *reinterpret_cast<bf16x4*>(&Bh[grp][buf][c][r0]) = to_bf4(vb);
      }
    }
    __syncthreads();
    load(st + G);
    if (st < steps) {
      if constexpr (BF) {
        const int h8 = 8 * (lane >> 5);
#pragma unroll
        for (int s16 = 0; s16 < TK; s16 += 16)
          acc = mfma_bf(&Ah[grp][buf][wr * 32 + (lane & 31)][s16 + h8],
                        &Bh[grp][buf][wc * 32 + (lane & 31)][s16 + h8], acc);
      } else {
#pragma unroll
        for (int kk = 0; kk < TK; kk += 2) {
          const float a = As[grp][buf][kk + (lane >> 5)][wr * 32 + (lane & 31)];
          const float b = Bs[grp][buf][kk + (lane >> 5)][wc * 32 + (lane & 31)];
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
        }
      }
    }
    buf ^= 1;
  }
  float* sh = smem;  // G * 2 * TK * (TM + 1) >= (G - 1) * 4096 floats
  __shared__ float red[G * 4][64];
  __syncthreads();
  if (grp > 0)
#pragma unroll
    for (int r = 0; r < 16; ++r) sh[(((grp - 1) * 4 + wave) * 16 + r) * 64 + lane] = acc[r];
  red[grp * 4 + wave][lane] = dbs;
  __syncthreads();
  if (grp != 0) return;
  for (int g = 1; g < G; ++g)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += sh[(((g - 1) * 4 + wave) * 16 + r) * 64 + lane];
  const int k = k0 + wc * 32 + (lane & 31);
  float* out = part + (size_t)chunk * M * K;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < M && k < K) out[(size_t)m * K + k] = acc[r];
  }
  if (do_db && t < 64 && m0 + t < M) {
    float v = 0.f;
    for (int w = 0; w < G * 4; ++w) v += red[w][t];
    pdb[(size_t)chunk * M + m0 + t] = v;
  }
}

// Narrow products (M, K <= 32, f32 operands): one 32 x 32 output tile per row
// group, whose four waves split each 32-row K-step (8 rows = 4 MFMAs each)
// instead of padding the product to a 64 x 64 tile, which quadrupled the f32
// MFMA work of the narrow GAT / decoder layers (widths 1..32).  The waves'
// accumulators are added in a fixed order at the end (deterministic).
constexpr int TSN = 32;

template <int G>
__device__ __forceinline__ void tn_tile_narrow(float* smem, const float* __restrict__ A, int lda,
                                               const float* __restrict__ B, int ldb, int N, int M, int K, int rows,
                                               int chunk, float* __restrict__ part, float* __restrict__ pdb,
                                               int db_rows) {
  constexpr int PERN = (TK * TSN) / 256;
  float(*As)[2][TK][TSN + 1] = reinterpret_cast<float(*)[2][TK][TSN + 1]>(smem);  // [g][buf][n][m]
  float(*Bs)[2][TK][TSN + 1] = reinterpret_cast<float(*)[2][TK][TSN + 1]>(smem + G * 2 * TK * (TSN + 1));
  const int grp = threadIdx.x >> 8, t = threadIdx.x & 255, lane = t & 63, wave = t >> 6;
  const int nb = chunk * rows, ne = min(N, nb + rows);
  const int steps = ne > nb ? (ne - nb + TK - 1) / TK : 0;
  const int iters = (steps + G - 1) / G;
  const int c = t & (TSN - 1);  // this thread's column in every load
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float dbs = 0.f;
  float ra[PERN], rb[PERN];
  auto load = [&](int st) {
    const int n1 = nb + st * TK;
#pragma unroll
    for (int q = 0; q < PERN; ++q) {
      const int n = n1 + (t + 256 * q) / TSN;
      const bool in = st < steps && n < ne;
      ra[q] = (in && c < M) ? A[(size_t)n * lda + c] : 0.f;
      rb[q] = (in && c < K) ? B[(size_t)n * ldb + c] : 0.f;
    }
  };
  load(grp);
  int buf = 0;
  for (int it = 0, st = grp; it < iters; ++it, st += G) {
    const int n1 = nb + st * TK;
#pragma unroll
    for (int q = 0; q < PERN; ++q) {
      const int r = (t + 256 * q) / TSN;
      As[grp][buf][r][c] = ra[q];
      Bs[grp][buf][r][c] = rb[q];
      if (pdb && n1 + r < db_rows) dbs += ra[q];
    }
    __syncthreads();
    load(st + G);
    if (st < steps) {
#pragma unroll
      for (int kk = 0; kk < 8; kk += 2) {
        const int r = wave * 8 + kk + (lane >> 5);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[grp][buf][r][lane & 31], Bs[grp][buf][r][lane & 31], acc, 0,
                                                   0, 0);
      }
    }
    buf ^= 1;
  }
  __shared__ float redn[G * 8][TSN];
  __syncthreads();  // every wave is done with the last K-step's images
#pragma unroll
  for (int r = 0; r < 16; ++r) smem[((grp * 4 + wave) * 16 + r) * 64 + lane] = acc[r];
  redn[t >> 5 | grp << 3][c] = dbs;
  __syncthreads();
  if (threadIdx.x >= 64) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    float v = 0.f;
    for (int w = 0; w < G * 4; ++w) v += smem[(w * 16 + r) * 64 + lane];
    const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5), k = lane & 31;
    if (m < M && k < K) part[(size_t)chunk * M * K + (size_t)m * K + k] = v;
  }
  if (pdb && lane < M) {
    float v = 0.f;
    for (int w = 0; w < G * 8; ++w) v += redn[w][lane];
    pdb[(size_t)chunk * M + lane] = v;
  }
}

template <int G, bool BF = false>
__global__ void __launch_bounds__(256 * G) k_gemm_tn(const float* __restrict__ A, int lda,
                                                     const float* __restrict__ B, int ldb, int N,
                                                     int M, int K, int rows, float* __restrict__ part,
                                                     float* __restrict__ pdb, int db_rows) {
  // XCD-aware: each XCD takes a contiguous range of row chunks (tile_xy)
  const int gxy = gridDim.x * gridDim.y;
  const int logical = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                                gxy * gridDim.z);
  const int chunk = logical / gxy, rem = logical % gxy;
  __shared__ __attribute__((aligned(16))) float smem[tn_smem_floats<G>()];
  if (!BF && M <= TSN && K <= TSN)
    tn_tile_narrow<G>(smem, A, lda, B, ldb, N, M, K, rows, chunk, part, pdb, db_rows);
  else
    tn_tile<G, BF>(smem, A, lda, B, ldb, N, M, K, rows, chunk, (rem % gridDim.x) * TM, (rem / gridDim.x) * TN, part,
                   pdb, db_rows);
}

// Up to VG_TN_GROUP_MAX planned products in one launch (vg_gemm_tn_group):
// the weight gradients of a whole backward are only read by the optimizer,
// so they need not run where the backward produces their operands.  Blocks
// [block0[p], block0[p + 1]) belong to product p, chunk-major as in
// k_gemm_tn; the XCD remap spans the whole grid, so each XCD takes a
// contiguous range of (product, chunk) blocks.
struct TnGroup {
  vg_tn p[VG_TN_GROUP_MAX];
  int block0[VG_TN_GROUP_MAX + 1];
  int n;
};

// f32 products without LDS staging: the 32x32x2 f32 MFMA takes lane l's A
// operand as A[n + l / 32][m + l % 32] and its B operand as B[n + l / 32]
// [k + l % 32] -- for a weight gradient (reduction over rows n) both are
// plain coalesced row loads, so every wave feeds its MFMAs straight from
// global memory: no LDS images, no barrier per K-step.  Each of the 4 waves
// takes the whole (up to) 64 x 64 tile (2 x 2 accumulators) over every 4th
// 16-row block of the chunk; the waves' sums are added through LDS once at
// the end in a fixed order ((w0 + w2) + (w1 + w3): deterministic).
#ifndef VG_TN_DIRECT
#define VG_TN_DIRECT 1  // f32 grouped products: 1 tn_tile_direct, 0 the LDS-staged tn_tile (A/B)
#endif
#ifndef VG_TN_DU
#define VG_TN_DU 8
#endif
#ifndef VG_TN_PIPE
#define VG_TN_PIPE 1  // software-pipelined tn_tile_direct (0: the round-4 loop, A/B)
#endif
constexpr int kTnDU = VG_TN_DU;  // row pairs (MFMA K-steps) per wave per block of 2 * kTnDU rows

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const float* p, int bytes) {
  // descriptor words provably wave-uniform, or hipcc wraps every buffer op in a waterfall loop
  const unsigned long long a = reinterpret_cast<unsigned long long>(p);
  const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(a));
  const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(a >> 32));
  void* base = reinterpret_cast<void*>((static_cast<unsigned long long>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, __builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// M1 / K1: the tile's second 32-column halves (of M / K) are live.
// BF: bf16 operands, f32 accumulation (v_mfma_f32_32x32x16_bf16 takes lane
// l's A operand as A[n + 8 (l / 32) + j][m + l % 32], j < 8: the same
// coalesced row loads, eight rows per lane, rounded to bf16 in registers).
template <bool M1, bool K1, bool BF>
__device__ __forceinline__ void tn_tile_direct(float* red, const float* __restrict__ A, int lda,
                                               const float* __restrict__ B, int ldb, int N, int M, int K, int rows,
                                               int chunk, int m0, int k0, float* __restrict__ part,
                                               float* __restrict__ pdb, int db_rows) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nb = chunk * rows, ne = min(N, nb + rows);
  const int col = lane & 31, half = lane >> 5;
  const bool do_db = pdb && k0 == 0;
  static_assert(!BF || kTnDU == 8, "a bf16 block is one 16-row MFMA step");
  // row of load p within the block: f32 pairs (2p + half), bf16 eights (8 half + p)
  const int hrow = BF ? 8 * half : half, prow = BF ? 1 : 2;
  f32x16 c00, c01, c10, c11;
#pragma unroll
  for (int r = 0; r < 16; ++r) c00[r] = c01[r] = c10[r] = c11[r] = 0.f;
  float db0 = 0.f, db1 = 0.f;
  // Buffer loads: a 32-bit per-lane offset (the row pair's step in the
  // scalar soffset) and a hardware range check -- rows >= N (the last
  // chunk's tail; a chunk's 16-row blocks never cross into the next chunk,
  // rows % 32 == 0) read as 0 with no mask; a column past M / K gets an
  // offset beyond the buffer (the host keeps N * ld * 4 < 2^30).
  constexpr unsigned kOob = 1u << 30;
  const auto ra = uniform_rsrc(A, N * lda * 4);
  const auto rb = uniform_rsrc(B, N * ldb * 4);
  const unsigned oa0 = m0 + col < M ? (m0 + col) * 4u : kOob, oa1 = m0 + 32 + col < M ? (m0 + 32 + col) * 4u : kOob;
  const unsigned ob0 = k0 + col < K ? (k0 + col) * 4u : kOob, ob1 = k0 + 32 + col < K ? (k0 + 32 + col) * 4u : kOob;
  // Software pipelined: the next 16-row block's loads are issued before the
  // current block's MFMAs (two register sets), so a wave waits for one load
  // round trip per chunk instead of one per block (a critic chunk is ~12
  // blocks per wave: the loop was a chain of dependent round trips).
  float a0[kTnDU], a1[kTnDU], b0[kTnDU], b1[kTnDU];
  auto load_block = [&](int n16, float (&xa0)[kTnDU], float (&xa1)[kTnDU], float (&xb0)[kTnDU],
                        float (&xb1)[kTnDU]) {
    const unsigned ra_n = (unsigned)(n16 + hrow) * lda * 4u, rb_n = (unsigned)(n16 + hrow) * ldb * 4u;
#pragma unroll
    for (int p = 0; p < kTnDU; ++p) {
      const int sa = prow * p * lda * 4, sb = prow * p * ldb * 4;
      xa0[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, ra_n + oa0, sa, 0));
      xb0[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, rb_n + ob0, sb, 0));
      if constexpr (M1) xa1[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, ra_n + oa1, sa, 0));
      else xa1[p] = 0.f;
      if constexpr (K1) xb1[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, rb_n + ob1, sb, 0));
      else xb1[p] = 0.f;
    }
  };
  auto mfma_block = [&](int n16, const float (&xa0)[kTnDU], const float (&xa1)[kTnDU], const float (&xb0)[kTnDU],
                        const float (&xb1)[kTnDU]) {
    if constexpr (BF) {
      bf16x8 ha0, ha1, hb0, hb1;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        ha0[j] = static_cast<__bf16>(xa0[j]);
        hb0[j] = static_cast<__bf16>(xb0[j]);
        ha1[j] = static_cast<__bf16>(xa1[j]);
        hb1[j] = static_cast<__bf16>(xb1[j]);
      }
      c00 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha0, hb0, c00, 0, 0, 0);
      if constexpr (K1) c01 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha0, hb1, c01, 0, 0, 0);
      if constexpr (M1) c10 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha1, hb0, c10, 0, 0, 0);
      if constexpr (M1 && K1) c11 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ha1, hb1, c11, 0, 0, 0);
    } else {
#pragma unroll
      for (int p = 0; p < kTnDU; ++p) {
        c00 = __builtin_amdgcn_mfma_f32_32x32x2f32(xa0[p], xb0[p], c00, 0, 0, 0);
        if constexpr (K1) c01 = __builtin_amdgcn_mfma_f32_32x32x2f32(xa0[p], xb1[p], c01, 0, 0, 0);
        if constexpr (M1) c10 = __builtin_amdgcn_mfma_f32_32x32x2f32(xa1[p], xb0[p], c10, 0, 0, 0);
        if constexpr (M1 && K1) c11 = __builtin_amdgcn_mfma_f32_32x32x2f32(xa1[p], xb1[p], c11, 0, 0, 0);
      }
    }
#pragma unroll
    for (int p = 0; p < kTnDU; ++p)
      if (do_db && n16 + hrow + prow * p < db_rows) {  // the f32 values (as tn_tile)
        db0 += xa0[p];
        db1 += xa1[p];
      }
  };
  constexpr int kStep = 8 * kTnDU;  // 4 waves x 2 kTnDU rows
  int n16 = nb + 2 * kTnDU * wave;
#if VG_TN_PIPE == 0  // A/B: one register set, loads then MFMAs per block
#pragma nounroll
  for (; n16 < ne; n16 += kStep) {
    load_block(n16, a0, a1, b0, b1);
    mfma_block(n16, a0, a1, b0, b1);
  }
#endif
  if (n16 < ne) load_block(n16, a0, a1, b0, b1);
#pragma nounroll
  for (; n16 < ne; n16 += 2 * kStep) {
    float e0[kTnDU], e1[kTnDU], f0[kTnDU], f1[kTnDU];
    const bool more = n16 + kStep < ne;  // wave-uniform
    if (more) load_block(n16 + kStep, e0, e1, f0, f1);
    mfma_block(n16, a0, a1, b0, b1);
    if (!more) break;
    if (n16 + 2 * kStep < ne) load_block(n16 + 2 * kStep, a0, a1, b0, b1);
    mfma_block(n16 + kStep, e0, e1, f0, f1);
  }
  // Cross-wave sum, one accumulator at a time (so the epilogue never holds
  // all 64 accumulators in VGPRs): ((w0 + w2) + (w1 + w3)), deterministic;
  // red holds 2 slots x 16 floats per lane.  Wave 0 writes the partial.
  const int half4 = 4 * half;
  float* out = part + (size_t)chunk * M * K;
  auto reduce_store = [&](f32x16& c, int mo, int ko) {
    if (wave >= 2)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((wave - 2) * 16 + r) * 64 + lane] = c[r];
    __syncthreads();
    if (wave < 2)
#pragma unroll
      for (int r = 0; r < 16; ++r) c[r] += red[(wave * 16 + r) * 64 + lane];
    __syncthreads();
    if (wave == 1)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[r * 64 + lane] = c[r];
    __syncthreads();
    if (wave == 0) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + mo + (r & 3) + 8 * (r >> 2) + half4, k = k0 + ko + col;
        if (m < M && k < K) out[(size_t)m * K + k] = c[r] + red[r * 64 + lane];
      }
    }
    __syncthreads();  // red is free for the next accumulator
  };
  reduce_store(c00, 0, 0);
  if constexpr (K1) reduce_store(c01, 0, 32);
  if constexpr (M1) reduce_store(c10, 32, 0);
  if constexpr (M1 && K1) reduce_store(c11, 32, 32);
  if (do_db) {  // lanes l and l + 32 hold the same column's other rows
    db0 += __shfl_xor(db0, 32, 64);
    db1 += __shfl_xor(db1, 32, 64);
    if (wave >= 2) {
      red[(wave - 2) * 64 + lane] = db0;
      red[(2 + wave - 2) * 64 + lane] = db1;
    }
    __syncthreads();
    if (wave < 2) {
      db0 += red[wave * 64 + lane];
      db1 += red[(2 + wave) * 64 + lane];
    }
    __syncthreads();
    if (wave == 1) {
      red[lane] = db0;
      red[64 + lane] = db1;
    }
    __syncthreads();
    if (wave == 0 && half == 0) {
      if (m0 + col < M) pdb[(size_t)chunk * M + m0 + col] = db0 + red[lane];
      if (m0 + 32 + col < M) pdb[(size_t)chunk * M + m0 + 32 + col] = db1 + red[64 + lane];
    }
  }
}

constexpr int kTnDirectRed = 2 * 16 * 64;  // floats of the cross-wave buffer (8 KB)

// Narrow products (M <= 16 and K <= 16: the critic's and the generator's
// bottleneck layers, 8 x 16, 16 x 8, 1 x 8 ...) on the 16x16x4 f32 MFMA:
// lane l's A operand is A[n + l / 16][l % 16] and its B operand
// B[n + l / 16][l % 16], four rows per instruction, so a 16-wide product
// wastes none of the 32x32x2 form's 3/4 of idle output lanes and takes a
// quarter of its MFMA cycles per row (32 vs 2 x 64 cycles per 4 rows).  Each
// wave takes 32-row blocks (8 MFMA steps, the next block's loads in flight),
// the waves' sums are added through LDS in the fixed order ((w0 + w2) + (w1 +
// w3)).  The sums differ from the 32x32x2 form's only in order.
#ifndef VG_TN_NARROW
#define VG_TN_NARROW 1
#endif
__device__ __forceinline__ void tn_tile_narrow16(float* red, const float* __restrict__ A, int lda,
                                                 const float* __restrict__ B, int ldb, int N, int M, int K, int rows,
                                                 int chunk, float* __restrict__ part, float* __restrict__ pdb,
                                                 int db_rows) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int nb = chunk * rows, ne = min(N, nb + rows);
  const int col = lane & 15, rq = lane >> 4;
  constexpr unsigned kOob = 1u << 30;
  const auto ra = uniform_rsrc(A, N * lda * 4);
  const auto rb = uniform_rsrc(B, N * ldb * 4);
  const unsigned oa = col < M ? col * 4u : kOob, ob = col < K ? col * 4u : kOob;
  f32x4 c = f32x4{0.f, 0.f, 0.f, 0.f};
  float db = 0.f;
  constexpr int kS = 8;  // MFMA steps (4 rows each) per block
  float a0[kS], b0[kS], a1[kS], b1[kS];
  auto load_block = [&](int n32, float (&xa)[kS], float (&xb)[kS]) {
    const unsigned ra_n = (unsigned)(n32 + rq) * lda * 4u, rb_n = (unsigned)(n32 + rq) * ldb * 4u;
#pragma unroll
    for (int p = 0; p < kS; ++p) {
      xa[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ra, ra_n + oa, 4 * p * lda * 4, 0));
      xb[p] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rb, rb_n + ob, 4 * p * ldb * 4, 0));
    }
  };
  auto mfma_block = [&](int n32, const float (&xa)[kS], const float (&xb)[kS]) {
#pragma unroll
    for (int p = 0; p < kS; ++p) c = __builtin_amdgcn_mfma_f32_16x16x4f32(xa[p], xb[p], c, 0, 0, 0);
    if (pdb)
#pragma unroll
      for (int p = 0; p < kS; ++p)
        if (n32 + rq + 4 * p < db_rows) db += xa[p];
  };
  constexpr int kStep = 4 * 32;  // 4 waves x 32 rows
  int n32 = nb + 32 * wave;
  if (n32 < ne) load_block(n32, a0, b0);
#pragma nounroll
  for (; n32 < ne; n32 += 2 * kStep) {
    const bool more = n32 + kStep < ne;  // wave-uniform
    if (more) load_block(n32 + kStep, a1, b1);
    mfma_block(n32, a0, b0);
    if (!more) break;
    if (n32 + 2 * kStep < ne) load_block(n32 + 2 * kStep, a0, b0);
    mfma_block(n32 + kStep, a1, b1);
  }
  // cross-wave sum ((w0 + w2) + (w1 + w3)); lane l holds D[4 (l / 16) + r][l % 16]
  if (wave >= 2)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[((wave - 2) * 4 + r) * 64 + lane] = c[r];
  __syncthreads();
  if (wave < 2)
#pragma unroll
    for (int r = 0; r < 4; ++r) c[r] += red[(wave * 4 + r) * 64 + lane];
  __syncthreads();
  if (wave == 1)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[r * 64 + lane] = c[r];
  __syncthreads();
  if (wave == 0) {
    float* out = part + (size_t)chunk * M * K;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = 4 * rq + r, k = col;
      if (m < M && k < K) out[(size_t)m * K + k] = c[r] + red[r * 64 + lane];
    }
  }
  if (pdb) {  // column sums of A: lanes l, l + 16, l + 32, l + 48 hold one column's rows
    db += __shfl_xor(db, 16, 64);
    db += __shfl_xor(db, 32, 64);
    __syncthreads();
    if (wave >= 2) red[(wave - 2) * 64 + lane] = db;
    __syncthreads();
    if (wave < 2) db += red[wave * 64 + lane];
    __syncthreads();
    if (wave == 1) red[lane] = db;
    __syncthreads();
    if (wave == 0 && rq == 0 && col < M) pdb[(size_t)chunk * M + col] = db + red[lane];
  }
}

template <bool BF>
__global__ void __launch_bounds__(256) k_gemm_tn_group_direct(const TnGroup g) {
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  int p = 0;
  while (p + 1 < g.n && lb >= g.block0[p + 1]) ++p;
  const vg_tn& d = g.p[p];
  const int local = lb - g.block0[p];
  const int gx = (d.M + TM - 1) / TM, gxy = gx * ((d.K + TN - 1) / TN);
  const int chunk = local / gxy, rem = local % gxy;
  __shared__ float red[kTnDirectRed];
  const int m0 = (rem % gx) * TM, k0 = (rem / gx) * TN;
  const bool m1 = m0 + 32 < d.M, k1 = k0 + 32 < d.K;
  if (!BF && VG_TN_NARROW && d.M <= 16 && d.K <= 16)
    tn_tile_narrow16(red, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, d.part, d.pdb, d.db_rows);
  else if (m1 && k1)
    tn_tile_direct<true, true, BF>(red, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, m0, k0, d.part, d.pdb,
                               d.db_rows);
  else if (m1)
    tn_tile_direct<true, false, BF>(red, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, m0, k0, d.part, d.pdb,
                                d.db_rows);
  else if (k1)
    tn_tile_direct<false, true, BF>(red, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, m0, k0, d.part, d.pdb,
                                d.db_rows);
  else
    tn_tile_direct<false, false, BF>(red, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, m0, k0, d.part, d.pdb,
                                 d.db_rows);
}

template <int G, bool BF>
__global__ void __launch_bounds__(256 * G) k_gemm_tn_group(const TnGroup g) {
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  int p = 0;
  while (p + 1 < g.n && lb >= g.block0[p + 1]) ++p;
  const vg_tn& d = g.p[p];
  const int local = lb - g.block0[p];
  const int gx = (d.M + TM - 1) / TM, gxy = gx * ((d.K + TN - 1) / TN);
  const int chunk = local / gxy, rem = local % gxy;
  __shared__ __attribute__((aligned(16))) float smem[tn_smem_floats<G>()];
  if (!BF && d.M <= TSN && d.K <= TSN)
    tn_tile_narrow<G>(smem, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, d.part, d.pdb, d.db_rows);
  else
    tn_tile<G, BF>(smem, d.A, d.lda, d.B, d.ldb, d.N, d.M, d.K, d.rows, chunk, (rem % gx) * TM, (rem / gx) * TN,
                   d.part, d.pdb, d.db_rows);
}

// out[w / K][w % K] (row stride ldo) = sum_c part[c][w], fixed order (+= when acc);
// 1024 threads per 64 outputs, 16 rows in flight.  Blocks from nb1 on fold a
// second, dense set (part2 [rows][W2] -> out2, the bias gradient) in the same
// launch.
__global__ void __launch_bounds__(1024) k_fold_rows(const float* __restrict__ part, int rows,
                                                    long long W, int K, int ldo, int acc,
                                                    float* __restrict__ out, int nb1 = 1 << 30,
                                                    const float* __restrict__ part2 = nullptr,
                                                    int W2 = 0, float* __restrict__ out2 = nullptr) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int bx = blockIdx.x;
  if (bx >= nb1) {
    bx -= nb1;
    part = part2;
    W = K = ldo = W2;
    out = out2;
  }
  const long long w = bx * 64LL + lane;
  float s = 0.f;
  if (w < W) {
    // 4 independent accumulators (loads in flight), combined in a fixed order
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
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
    float* o = out + (w / K) * ldo + (w % K);
    *o = acc ? *o + v : v;
  }
}

}  // namespace

#ifndef VG_QUAD_A
#define VG_QUAD_A 1  // A/B knob: float4 A loads in k_gemm16 where the operand allows
#endif
// both operands as float4 quads: A along k; B along k (bt) or along m
static inline bool quad_ab(const float* A, int lda, const float* B, int ldb, int K, int M, bool bt) {
  return VG_QUAD_A && K % 4 == 0 && lda % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0 &&
         ldb % 4 == 0 && (reinterpret_cast<uintptr_t>(B) & 15) == 0 && (bt || M % 4 == 0);
}

// 8-wave k_gemm16 workgroups (k_gemm8w) when the product has more row tiles
// than two 16-wave workgroups per CU hold: one workgroup round instead of two
#ifndef VG_GEMM8_MIN_TILES
#define VG_GEMM8_MIN_TILES 513  // 0: never (A/B knob)
#endif
static inline bool use_8w(const dim3& grid) {
  return VG_GEMM8_MIN_TILES > 0 && (long long)grid.x * grid.y >= VG_GEMM8_MIN_TILES;
}

template <bool BF>
static int gemm(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t b_trans, const float* bias,
                int32_t act, const float* aux, int32_t ldaux, float* C, int32_t ldc, int32_t N, int32_t M,
                int32_t K, void* stream) {
  if (N < 0 || M <= 0 || K <= 0 || !A || !B || !C || act < 0 || act > 4) return VG_EINVAL;
  if (act >= 3 && !aux) return VG_EINVAL;
  if (N == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  dim3 grid((N + TM - 1) / TM, (M + TN - 1) / TN);
#ifndef VG_GEMM16
// k_gemm16 (16 waves of 16 x 16 MFMA tiles) instead of k_gemm, per product
// kind (A/B bits): 1 plain f32, 2 the attention projections, 4 the
// GraphNorm-backward partials, 8 bf16 operands.  Bit 8 is off: converting the
// f32 LDS images to bf16 at read time measured slower than k_gemm's bf16
// staging (bf16 step 8.46 vs 8.31 ms, profiles/r02_ab_gemm16_att_gnp.txt)
#define VG_GEMM16 7
#endif
#define VG_G(BT, ACT)                                                                                      \
  do {                                                                                                     \
    if ((VG_GEMM16 & (BF ? 8 : 1)) != 0)                                                                   \
      if (quad_ab(A, lda, B, ldb, K, M, BT))                                                               \
        if (use_8w(grid))                                                                                  \
          k_gemm8w<BT, ACT, false, BF, false, true><<<grid, 512, 0, s>>>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, \
                                                                         N, M, K);                           \
        else                                                                                               \
          k_gemm16<BT, ACT, false, BF, false, true><<<grid, 1024, 0, s>>>(A, lda, B, ldb, bias, aux, ldaux, C,  \
                                                                         ldc, N, M, K);                      \
      else if (use_8w(grid))                                                                               \
        k_gemm8w<BT, ACT, false, BF><<<grid, 512, 0, s>>>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, N, M, K); \
      else                                                                                                 \
        k_gemm16<BT, ACT, false, BF><<<grid, 1024, 0, s>>>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, N, M, K); \
    else if (BF && quad_ab(A, lda, B, ldb, K, M, true))                                                    \
      k_gemm<BT, ACT, false, BF, false, BF><<<grid, 256, 0, s>>>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, N, M, \
                                                                 K);                                       \
    else                                                                                                   \
      k_gemm<BT, ACT, false, BF><<<grid, 256, 0, s>>>(A, lda, B, ldb, bias, aux, ldaux, C, ldc, N, M, K); \
  } while (0)
  if (b_trans) {
    if (act == 0) VG_G(true, 0); else if (act == 1) VG_G(true, 1);
    else if (act == 2) VG_G(true, 2); else if (act == 3) VG_G(true, 3); else VG_G(true, 4);
  } else {
    if (act == 0) VG_G(false, 0); else if (act == 1) VG_G(false, 1);
    else if (act == 2) VG_G(false, 2); else if (act == 3) VG_G(false, 3); else VG_G(false, 4);
  }
#undef VG_G
  VG_CHECK_LAUNCH();
  return 0;
}

template <bool BF>
static int gemm_gn_bwd(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M, int32_t K,
                       float* C, int32_t ldc, const float* gn_x, const float* keep, int32_t seg_rows,
                       const float* weight, const float* bias, const float* mean_scale, float eps,
                       const float* stats, float* tpart, void* stream) {
  if (N <= 0 || M <= 0 || K <= 0 || ldc < M || !A || !B || !C || !gn_x || !weight || !bias || !mean_scale ||
      !stats || !tpart || seg_rows < TM || N % seg_rows)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  dim3 grid((N + TM - 1) / TM, (M + TN - 1) / TN);
  const GnpDesc gn{gn_x, keep, stats, weight, bias, mean_scale, eps, seg_rows, tpart};
  if ((VG_GEMM16 & 4) && (!BF || (VG_GEMM16 & 8)))
    if (quad_ab(A, lda, B, ldb, K, M, false))
      if (use_8w(grid))
        k_gemm8w<false, 0, false, BF, true, true><<<grid, 512, 0, s>>>(A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, N,
                                                                       M, K, nullptr, nullptr, nullptr, nullptr, gn);
      else
        k_gemm16<false, 0, false, BF, true, true><<<grid, 1024, 0, s>>>(A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, N,
                                                                       M, K, nullptr, nullptr, nullptr, nullptr, gn);
    else if (use_8w(grid))
      k_gemm8w<false, 0, false, BF, true><<<grid, 512, 0, s>>>(A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, N, M, K,
                                                               nullptr, nullptr, nullptr, nullptr, gn);
    else
      k_gemm16<false, 0, false, BF, true><<<grid, 1024, 0, s>>>(A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, N, M, K,
                                                               nullptr, nullptr, nullptr, nullptr, gn);
  else if (BF && quad_ab(A, lda, B, ldb, K, M, true))
    k_gemm<false, 0, false, BF, true, BF><<<grid, 256, 0, s>>>(A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, N, M, K,
                                                               nullptr, nullptr, nullptr, nullptr, gn);
  else
    k_gemm<false, 0, false, BF, true><<<grid, 256, 0, s>>>(A, lda, B, ldb, nullptr, nullptr, 0, C, ldc, N, M, K,
                                                           nullptr, nullptr, nullptr, nullptr, gn);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gemm_gn_bwd(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                              int32_t K, float* C, int32_t ldc, const float* gn_x, const float* keep,
                              int32_t seg_rows, const float* weight, const float* bias, const float* mean_scale,
                              float eps, const float* stats, float* tpart, void* stream) {
  return gemm_gn_bwd<false>(A, lda, B, ldb, N, M, K, C, ldc, gn_x, keep, seg_rows, weight, bias, mean_scale, eps,
                            stats, tpart, stream);
}

extern "C" int vg_gemm_gn_bwd_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                                   int32_t K, float* C, int32_t ldc, const float* gn_x, const float* keep,
                                   int32_t seg_rows, const float* weight, const float* bias,
                                   const float* mean_scale, float eps, const float* stats, float* tpart,
                                   void* stream) {
  return gemm_gn_bwd<true>(A, lda, B, ldb, N, M, K, C, ldc, gn_x, keep, seg_rows, weight, bias, mean_scale, eps,
                           stats, tpart, stream);
}

extern "C" int vg_gemm(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t b_trans,
                       const float* bias, int32_t act, const float* aux, int32_t ldaux, float* C,
                       int32_t ldc, int32_t N, int32_t M, int32_t K, void* stream) {
  return gemm<false>(A, lda, B, ldb, b_trans, bias, act, aux, ldaux, C, ldc, N, M, K, stream);
}

extern "C" int vg_gemm_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t b_trans,
                            const float* bias, int32_t act, const float* aux, int32_t ldaux, float* C,
                            int32_t ldc, int32_t N, int32_t M, int32_t K, void* stream) {
  return gemm<true>(A, lda, B, ldb, b_trans, bias, act, aux, ldaux, C, ldc, N, M, K, stream);
}

// rows per split-K chunk: aim at ~768 workgroups in total but at most
// 256 chunks per output tile (the fold reads chunks x M x K partials; more chunks
// made the fold, not the product, the long pole), multiples of TK
#ifndef VG_TN_TARGET
#define VG_TN_TARGET 768
#endif
#ifndef VG_TN_GROUP_TARGET
#define VG_TN_GROUP_TARGET 64  // with tn_tile_direct; step A/B over 16..192: profiles/r02_ab_tn_direct.txt
#endif
// (a product planned for vg_gemm_tn_group shares the grid with the other
// products of its backward: VG_TN_GROUP_TARGET workgroups each, and at least
// min(VG_TN_GROUP_TARGET, N / VG_TN_GROUP_MIN_ROWS) chunks whatever its
// tile count.  Every workgroup of a group computes one 64 x 64 tile over its
// chunk, so its time is set by the chunk's rows: the generator's 128 x 524
// input-layer product got 3 chunks of 4,384 rows (5x the rows of any other
// workgroup in its launch) and its 128 x 128 products 16 of 832, and the
// launch waited on them.  The floor on chunks leaves the critic's products
// (N = 52k rows, 64 x 64) at their 64 chunks: more chunks there cost more in
// partials than they spread (profiles/r04_ab_tn_rows.txt).)
#ifndef VG_TN_GROUP_MIN_ROWS
#define VG_TN_GROUP_MIN_ROWS 416
#endif
static inline int tn_rows(int N, int M, int K, int wg_target = VG_TN_TARGET, int min_rows = 0) {
  const int tiles = ((M + TM - 1) / TM) * ((K + TN - 1) / TN);
  int target = wg_target / tiles;
  if (min_rows > 0) target = max(target, min(wg_target, (N + min_rows - 1) / min_rows));
  if (target > 256) target = 256;
  if (target < 1) target = 1;
  int rows = (N + target - 1) / target;
  rows = ((rows + TK - 1) / TK) * TK;
  return rows < TK ? TK : rows;
}

// Rows per chunk of a product planned for vg_gemm_tn_group.  A grouped launch
// lasts as long as its slowest workgroup, so each product's chunk count
// follows its tile's MFMA cost per row: 64 x 64 tiles (four 32x32x2
// accumulators) get 4x, half-wide ones 2x the workgroups of a 32 x 32 tile,
// and the narrow 16x16x4 products (M, K <= 16: a quarter of a 32 x 32 tile's
// MFMA time per row; f32 only: the bf16 products keep the plain rule) a
// quarter -- every workgroup of the launch then carries
// about the same work.  Products of several output tiles (the generator's
// 128-wide layers, already at the VG_TN_GROUP_MIN_ROWS floor) keep the plain
// rule (VG_TN_BALANCE=0: VG_TN_GROUP_TARGET workgroups for every tile, the
// round-4 plan).
#ifndef VG_TN_BALANCE
#define VG_TN_BALANCE 1
#endif
static inline int tn_group_rows(int N, int M, int K, bool bf = false) {
  int target = VG_TN_GROUP_TARGET;
  if (VG_TN_BALANCE && !bf && M <= TM && K <= TN) {  // one output tile (products over several keep the plain rule)
    const int mw = min(M, TM) > 32 ? 2 : 1, kw = min(K, TN) > 32 ? 2 : 1;
    target = VG_TN_NARROW && M <= 16 && K <= 16 ? VG_TN_GROUP_TARGET / 4 : VG_TN_GROUP_TARGET * mw * kw;
  }
  return tn_rows(N, M, K, target, VG_TN_GROUP_MIN_ROWS);
}

extern "C" int64_t vg_gemm_tn_ws_floats(int32_t N, int32_t M, int32_t K) {
  if (N <= 0) return 1;
  // enough for either plan: one launch per product or a grouped product
  const int r = min(min(tn_rows(N, M, K), tn_group_rows(N, M, K)), tn_group_rows(N, M, K, true));
  const int64_t chunks = (N + r - 1) / r;
  return chunks * ((int64_t)M * K + M);
}

template <bool BF = false>
static int gemm_tn(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                   int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows,
                   int32_t accumulate, float* workspace, void* stream, vg_fold* defer = nullptr,
                   int32_t* n_defer = nullptr) {
  if (n_defer) *n_defer = 0;
  if (N < 0 || M <= 0 || K <= 0 || ldc < K || !A || !B || !C || !workspace || db_rows < 0)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (N == 0) {
    if (accumulate) return 0;
    if (ldc != K) return VG_EINVAL;
    (void)hipMemsetAsync(C, 0, sizeof(float) * M * K, s);
    if (db) (void)hipMemsetAsync(db, 0, sizeof(float) * M, s);
    return 0;
  }
  const int rows = tn_rows(N, M, K);
  const int chunks = (N + rows - 1) / rows;
  float* part = workspace;
  float* pdb = workspace + (size_t)chunks * M * K;
  dim3 grid((M + TM - 1) / TM, (K + TN - 1) / TN, chunks);
  k_gemm_tn<kTnGroups, BF><<<grid, 256 * kTnGroups, 0, s>>>(A, lda, B, ldb, N, M, K, rows, part, db ? pdb : nullptr,
                                 db_rows < N ? db_rows : N);
  const long long W = (long long)M * K;
  if (defer) {  // describe the fold(s) for vg_fold_batch instead of launching them
    defer[0] = vg_fold{C, (int32_t)W, K, ldc, accumulate, 1, {{part, chunks, (int32_t)W}, {nullptr, 0, 0}}};
    *n_defer = 1;
    if (db) {
      defer[1] = vg_fold{db, M, M, M, accumulate, 1, {{pdb, chunks, M}, {nullptr, 0, 0}}};
      *n_defer = 2;
    }
    VG_CHECK_LAUNCH();
    return 0;
  }
  const int nb1 = (int)((W + 63) / 64), nb2 = db ? (M + 63) / 64 : 0;
  k_fold_rows<<<nb1 + nb2, 1024, 0, s>>>(part, chunks, W, K, ldc, accumulate, C, nb1, pdb, M, db);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gemm_tn_deferred(const float* A, int32_t lda, const float* B, int32_t ldb,
                                   int32_t N, int32_t M, int32_t K, float* C, int32_t ldc,
                                   float* db, int32_t db_rows, int32_t accumulate,
                                   float* workspace, vg_fold* folds_out, int32_t* n_out,
                                   void* stream) {
  if (!folds_out || !n_out || N <= 0) return VG_EINVAL;
  return gemm_tn(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, accumulate, workspace, stream,
                 folds_out, n_out);
}

extern "C" int vg_gemm_tn_deferred_bf16(const float* A, int32_t lda, const float* B, int32_t ldb,
                                        int32_t N, int32_t M, int32_t K, float* C, int32_t ldc,
                                        float* db, int32_t db_rows, int32_t accumulate,
                                        float* workspace, vg_fold* folds_out, int32_t* n_out,
                                        void* stream) {
  if (!folds_out || !n_out || N <= 0) return VG_EINVAL;
  return gemm_tn<true>(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, accumulate, workspace, stream,
                       folds_out, n_out);
}

template <bool BF>
static int gemm_tn_plan(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M, int32_t K,
                        float* C, int32_t ldc, float* db, int32_t db_rows, int32_t accumulate, float* workspace,
                        vg_tn* prod_out, vg_fold* folds_out, int32_t* n_out) {
  if (n_out) *n_out = 0;
  if (!prod_out || !folds_out || !n_out || N <= 0 || M <= 0 || K <= 0 || ldc < K || !A || !B || !C ||
      !workspace || db_rows < 0)
    return VG_EINVAL;
  const int rows = tn_group_rows(N, M, K, BF);
  const int chunks = (N + rows - 1) / rows;
  float* part = workspace;
  float* pdb = workspace + (size_t)chunks * M * K;
  *prod_out = vg_tn{A, B, part, db ? pdb : nullptr, lda, ldb, N, M, K, rows, chunks, db_rows < N ? db_rows : N,
                    BF ? 1 : 0};
  const int32_t W = M * K;
  folds_out[0] = vg_fold{C, W, K, ldc, accumulate, 1, {{part, chunks, W}, {nullptr, 0, 0}}};
  *n_out = 1;
  if (db) {
    folds_out[1] = vg_fold{db, M, M, M, accumulate, 1, {{pdb, chunks, M}, {nullptr, 0, 0}}};
    *n_out = 2;
  }
  return 0;
}

extern "C" int vg_gemm_tn_plan(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                               int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows, int32_t accumulate,
                               float* workspace, vg_tn* prod_out, vg_fold* folds_out, int32_t* n_out) {
  return gemm_tn_plan<false>(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, accumulate, workspace, prod_out,
                             folds_out, n_out);
}

extern "C" int vg_gemm_tn_plan_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                                    int32_t M, int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows,
                                    int32_t accumulate, float* workspace, vg_tn* prod_out, vg_fold* folds_out,
                                    int32_t* n_out) {
  return gemm_tn_plan<true>(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, accumulate, workspace, prod_out,
                            folds_out, n_out);
}

extern "C" int vg_gemm_tn_group(const vg_tn* prods, int32_t n, void* stream) {
  if (n < 0 || n > VG_TN_GROUP_MAX || (n > 0 && !prods)) return VG_EINVAL;
  if (n == 0) return 0;
  TnGroup g{};
  long long blocks = 0;
  const int bf = prods[0].bf16;
  for (int i = 0; i < n; ++i) {
    const vg_tn& d = prods[i];
    if (d.bf16 != bf || !d.A || !d.B || !d.part || d.N <= 0 || d.M <= 0 || d.K <= 0 || d.rows <= 0 ||
        d.rows % TK || d.chunks != (d.N + d.rows - 1) / d.rows || d.db_rows < 0 || d.db_rows > d.N)
      return VG_EINVAL;
    g.p[i] = d;
    g.block0[i] = static_cast<int>(blocks);
    blocks += (long long)d.chunks * ((d.M + TM - 1) / TM) * ((d.K + TN - 1) / TN);
  }
  if (blocks > (1LL << 30)) return VG_EINVAL;
  g.block0[n] = static_cast<int>(blocks);
  g.n = n;
  hipStream_t s = static_cast<hipStream_t>(stream);
#ifndef VG_TN_DIRECT_BF
#define VG_TN_DIRECT_BF 1  // bf16 grouped products: 1 tn_tile_direct<.., true>, 0 the LDS-staged tn_tile (A/B)
#endif
  bool direct = bf ? VG_TN_DIRECT_BF : VG_TN_DIRECT;  // buffer offsets: every operand under 2^30 bytes
  for (int i = 0; direct && i < n; ++i)
    direct = (long long)prods[i].N * prods[i].lda * 4 < (1LL << 30) && (long long)prods[i].N * prods[i].ldb * 4 < (1LL << 30);
  if (direct && bf)
    k_gemm_tn_group_direct<true><<<static_cast<int>(blocks), 256, 0, s>>>(g);
  else if (direct)
    k_gemm_tn_group_direct<false><<<static_cast<int>(blocks), 256, 0, s>>>(g);
  else if (bf)
    k_gemm_tn_group<kTnGroups, true><<<static_cast<int>(blocks), 256 * kTnGroups, 0, s>>>(g);
  else
    k_gemm_tn_group<kTnGroups, false><<<static_cast<int>(blocks), 256 * kTnGroups, 0, s>>>(g);
  VG_CHECK_LAUNCH();
  return 0;
}

static inline bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// The persistent W-resident form (k_gemm_ln_wres) for f32, 64 < M <= 128,
// K % 4 == 0, K <= 32 * VG_WRES_KT, at least VG_WRES_MIN_ROWS rows (enough
// 32-row tiles per CU to amortise staging W); VG_WRES=0: k_gemm_ln16 (A/B).
#ifndef VG_WRES
#define VG_WRES 1
#endif
// K from which the f32 LayerNorm GEMMs (64 < M <= 128) take 64-row tiles:
// W (M x K) streamed from L2 per tile dominates there
#ifndef VG_LN_TM64_K
#define VG_LN_TM64_K 384
#endif
#ifndef VG_WRES_MIN_ROWS
#define VG_WRES_MIN_ROWS 16384
#endif
static int wres_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                  hipSuccess || n <= 0)
      n = 256;
    cus = n;
  }
  return cus;
}

template <int KT, bool MS>
static void launch_wres(const float* A, int lda, const float* W, int ldw, const float* bias, int N, int M, int K,
                        const float* gamma, const float* beta, float eps, float slope, float* H, float* Y, float* mean,
                        float* rstd, int ldy, const MsDesc& d, hipStream_t s) {
  static bool attr = false;  // dynamic LDS above the 64 KB default, once per instantiation
  constexpr int bytes = wres_lds_bytes<KT>();
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gemm_ln_wres<KT, MS>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    attr = true;
  }
  const int tiles = (N + 31) / 32;
  const int grid = tiles < wres_cus() ? tiles : wres_cus();
  k_gemm_ln_wres<KT, MS><<<grid, 1024, bytes, s>>>(A, lda, W, ldw, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean,
                                                   rstd, ldy, d);
}

// true: launched (K <= 160 in whole 32-wide tiles of the LDS image)
template <bool MS>
static bool try_wres(const float* A, int lda, const float* W, int ldw, const float* bias, int N, int M, int K,
                     const float* gamma, const float* beta, float eps, float slope, float* H, float* Y, float* mean,
                     float* rstd, int ldy, const MsDesc& d, hipStream_t s) {
  if (!VG_WRES || N < VG_WRES_MIN_ROWS || M <= TN || M > 2 * TN || K % 4 || K <= 0) return false;
  switch ((K + 31) / 32) {
    case 1: launch_wres<1, MS>(A, lda, W, ldw, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd, ldy, d, s); return true;
    case 2: launch_wres<2, MS>(A, lda, W, ldw, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd, ldy, d, s); return true;
    case 3: launch_wres<3, MS>(A, lda, W, ldw, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd, ldy, d, s); return true;
    case 4: launch_wres<4, MS>(A, lda, W, ldw, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd, ldy, d, s); return true;
    case 5: launch_wres<5, MS>(A, lda, W, ldw, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd, ldy, d, s); return true;
    default: return false;
  }
}

template <bool BF>
static int gemm_ln_act(const float* A, int32_t lda, const float* W, int32_t N, int32_t M,
                       int32_t K, const float* bias, const float* gamma, const float* beta,
                       float eps, float slope, float* H, float* Y, float* mean, float* rstd,
                       void* stream) {
  if (N < 0 || M <= 0 || M > 2 * TN || K <= 0 || lda < K || !A || !W || !gamma || !beta || !Y ||
      ((mean == nullptr) != (rstd == nullptr)))
    return VG_EINVAL;
  if (N == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const dim3 grid((N + TM - 1) / TM, 1);
  const bool ql = VG_QUAD_A && K % 4 == 0 && lda % 4 == 0 && al16(A) && al16(W);
  if (!BF && ql && try_wres<false>(A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd, M, MsDesc{}, s)) {
  } else if (!BF && VG_LN16) {
    if (M <= TN && ql)
      k_gemm_ln16<1, TM, false, false, true><<<grid, 1024, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps,
                                                                  slope, H, Y, mean, rstd);
    else if (M <= TN)
      k_gemm_ln16<1, TM><<<grid, 1024, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean,
                                              rstd);
    else if (VG_LN_TM32 && ql && K >= VG_LN_TM64_K)  // long K: 64-row tiles stream W half as often
      k_gemm_ln16<2, TM, false, false, true><<<grid, 1024, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps,
                                                                  slope, H, Y, mean, rstd);
    else if (VG_LN_TM32 && ql)
      k_gemm_ln16<2, 32, false, false, true><<<dim3((N + 31) / 32, 1), 1024, 0, s>>>(
          A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd);
    else if (VG_LN_TM32)
      k_gemm_ln16<2, 32><<<dim3((N + 31) / 32, 1), 1024, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps,
                                                                slope, H, Y, mean, rstd);
    else
      k_gemm_ln16<2, TM><<<grid, 1024, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean,
                                              rstd);
  } else if (M <= TN && BF && ql)
    k_gemm_ln<1, TM, false, false, BF, BF><<<grid, 256, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps,
                                                                 slope, H, Y, mean, rstd);
  else if (M <= TN)
    k_gemm_ln<1, TM, false, false, BF><<<grid, 256, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope,
                                                             H, Y, mean, rstd);
  else if (VG_LN_TM32 && BF && ql)
    k_gemm_ln<2, 32, false, false, BF, BF><<<dim3((N + 31) / 32, 1), 256, 0, s>>>(
        A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope, H, Y, mean, rstd);
  else if (VG_LN_TM32)
    k_gemm_ln<2, 32, false, false, BF><<<dim3((N + 31) / 32, 1), 256, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma,
                                                                              beta, eps, slope, H, Y, mean, rstd);
  else
    k_gemm_ln<2, TM, false, false, BF><<<grid, 256, 0, s>>>(A, lda, W, K, bias, N, M, K, gamma, beta, eps, slope,
                                                             H, Y, mean, rstd);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gemm_ln_act(const float* A, int32_t lda, const float* W, int32_t N, int32_t M,
                              int32_t K, const float* bias, const float* gamma, const float* beta,
                              float eps, float slope, float* H, float* Y, float* mean, float* rstd,
                              void* stream) {
  return gemm_ln_act<false>(A, lda, W, N, M, K, bias, gamma, beta, eps, slope, H, Y, mean, rstd, stream);
}

extern "C" int vg_gemm_ln_act_bf16(const float* A, int32_t lda, const float* W, int32_t N, int32_t M,
                                   int32_t K, const float* bias, const float* gamma, const float* beta,
                                   float eps, float slope, float* H, float* Y, float* mean, float* rstd,
                                   void* stream) {
  return gemm_ln_act<true>(A, lda, W, N, M, K, bias, gamma, beta, eps, slope, H, Y, mean, rstd, stream);
}

template <bool BF>
static int gemm_ln_act_ms(const vg_asrc* src, int32_t nsrc, const float* W, int32_t ldw, int32_t N,
                          int32_t M, const float* bias, const float* addend, int32_t ld_add,
                          int32_t add_rows, const float* gamma, const float* beta, float eps, float slope,
                          float* Y, int32_t ldy, void* stream) {
  if (!src || nsrc <= 0 || nsrc > kMaxSrc || !W || N < 0 || M <= TN || M > 2 * TN || !gamma || !beta || !Y ||
      ldy < M || (addend && (ld_add < M || add_rows < 32)))
    return VG_EINVAL;
  MsDesc d{};
  int K = 0;
  for (int i = 0; i < nsrc; ++i) {
    if (!src[i].ptr || src[i].cols <= 0 || src[i].cols % TK || src[i].ld < src[i].cols || src[i].w_col0 < 0 ||
        src[i].w_col0 + src[i].cols > ldw || src[i].rows_mod != 0)
      return VG_EINVAL;
    K += src[i].cols;
    d.p[i] = src[i].ptr;
    d.ld[i] = src[i].ld;
    d.kend[i] = K;
    d.wcol[i] = src[i].w_col0;
    d.rmod[i] = src[i].rows_mod;
  }
  d.nsrc = nsrc;
  d.add = addend;
  d.ld_add = ld_add;
  d.add_rows = add_rows;
  if (N == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  bool ql = VG_QUAD_A && ldw % 4 == 0 && al16(W);
  for (int i = 0; i < nsrc; ++i) ql = ql && src[i].ld % 4 == 0 && src[i].w_col0 % 4 == 0 && al16(src[i].ptr);
  if (!BF && ql && try_wres<true>(nullptr, 0, W, ldw, bias, N, M, K, gamma, beta, eps, slope, nullptr, Y, nullptr,
                                  nullptr, ldy, d, s)) {
  } else if (!BF && VG_LN16 && ql && K >= VG_LN_TM64_K)  // long K: 64-row tiles stream W half as often
    k_gemm_ln16<2, TM, false, true, true><<<dim3((N + TM - 1) / TM, 1), 1024, 0, s>>>(
        nullptr, 0, W, ldw, bias, N, M, K, gamma, beta, eps, slope, nullptr, Y, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, ldy, d);
  else if (!BF && VG_LN16 && ql)
    k_gemm_ln16<2, 32, false, true, true><<<dim3((N + 31) / 32, 1), 1024, 0, s>>>(
        nullptr, 0, W, ldw, bias, N, M, K, gamma, beta, eps, slope, nullptr, Y, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, ldy, d);
  else if (!BF && VG_LN16)
    k_gemm_ln16<2, 32, false, true><<<dim3((N + 31) / 32, 1), 1024, 0, s>>>(
        nullptr, 0, W, ldw, bias, N, M, K, gamma, beta, eps, slope, nullptr, Y, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, ldy, d);
  else if (BF && ql)
    k_gemm_ln<2, 32, false, true, BF, BF><<<dim3((N + 31) / 32, 1), 256, 0, s>>>(
        nullptr, 0, W, ldw, bias, N, M, K, gamma, beta, eps, slope, nullptr, Y, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, ldy, d);
  else
    k_gemm_ln<2, 32, false, true, BF><<<dim3((N + 31) / 32, 1), 256, 0, s>>>(
        nullptr, 0, W, ldw, bias, N, M, K, gamma, beta, eps, slope, nullptr, Y, nullptr, nullptr, nullptr, nullptr,
        nullptr, nullptr, ldy, d);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gemm_ln_act_ms(const vg_asrc* src, int32_t nsrc, const float* W, int32_t ldw, int32_t N,
                                 int32_t M, const float* bias, const float* addend, int32_t ld_add,
                                 int32_t add_rows, const float* gamma, const float* beta, float eps, float slope,
                                 float* Y, int32_t ldy, void* stream) {
  return gemm_ln_act_ms<false>(src, nsrc, W, ldw, N, M, bias, addend, ld_add, add_rows, gamma, beta, eps, slope,
                               Y, ldy, stream);
}

extern "C" int vg_gemm_ln_act_ms_bf16(const vg_asrc* src, int32_t nsrc, const float* W, int32_t ldw, int32_t N,
                                      int32_t M, const float* bias, const float* addend, int32_t ld_add,
                                      int32_t add_rows, const float* gamma, const float* beta, float eps,
                                      float slope, float* Y, int32_t ldy, void* stream) {
  return gemm_ln_act_ms<true>(src, nsrc, W, ldw, N, M, bias, addend, ld_add, add_rows, gamma, beta, eps, slope,
                              Y, ldy, stream);
}

template <bool BF>
static int gat_lin_att(const float* X, int32_t ldx, const float* W, int32_t N,
                       int32_t Cin, int32_t C, const float* att_src, const float* att_dst,
                       float* H, float* a_src, float* a_dst, void* stream) {
  if (N < 0 || Cin <= 0 || C <= 0 || ldx < Cin || !X || !W || !att_src || !att_dst || !H ||
      !a_src || !a_dst)
    return VG_EINVAL;
  if (N == 0) return 0;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (C > 2 * TN) {  // several column tiles: GEMM, then the per-row projection pass
    const int rc = gemm<BF>(X, ldx, W, Cin, 1, nullptr, 0, nullptr, 0, H, C, N, C, Cin, stream);
    if (rc) return rc;
    return vg_gat_att(H, N, C, att_src, att_dst, a_src, a_dst, stream);
  }
  if (C > TN) {  // whole 128-column rows per block, projections in the epilogue
    if (!BF && VG_LN16 && quad_ab(X, ldx, W, Cin, Cin, C, true))
      k_gemm_ln16<2, 32, true, false, true><<<dim3((N + 31) / 32, 1), 1024, 0, s>>>(
          X, ldx, W, Cin, nullptr, N, C, Cin, nullptr, nullptr, 0.f, 0.f, H, nullptr, nullptr, nullptr, att_src,
          att_dst, a_src, a_dst);
    else if (!BF && VG_LN16)
      k_gemm_ln16<2, 32, true><<<dim3((N + 31) / 32, 1), 1024, 0, s>>>(
          X, ldx, W, Cin, nullptr, N, C, Cin, nullptr, nullptr, 0.f, 0.f, H, nullptr, nullptr, nullptr, att_src,
          att_dst, a_src, a_dst);
    else
      k_gemm_ln<2, 32, true, false, BF><<<dim3((N + 31) / 32, 1), 256, 0, s>>>(
          X, ldx, W, Cin, nullptr, N, C, Cin, nullptr, nullptr, 0.f, 0.f, H, nullptr, nullptr, nullptr, att_src,
          att_dst, a_src, a_dst);
    VG_CHECK_LAUNCH();
    return 0;
  }
  if ((VG_GEMM16 & 2) && (!BF || (VG_GEMM16 & 8)))
    if (quad_ab(X, ldx, W, Cin, Cin, C, true))
      if (use_8w(dim3((N + TM - 1) / TM, 1)))
        k_gemm8w<true, 0, true, BF, false, true><<<dim3((N + TM - 1) / TM, 1), 512, 0, s>>>(
            X, ldx, W, Cin, nullptr, nullptr, 0, H, C, N, C, Cin, att_src, att_dst, a_src, a_dst);
      else
        k_gemm16<true, 0, true, BF, false, true><<<dim3((N + TM - 1) / TM, 1), 1024, 0, s>>>(
            X, ldx, W, Cin, nullptr, nullptr, 0, H, C, N, C, Cin, att_src, att_dst, a_src, a_dst);
    else if (use_8w(dim3((N + TM - 1) / TM, 1)))
      k_gemm8w<true, 0, true, BF><<<dim3((N + TM - 1) / TM, 1), 512, 0, s>>>(
          X, ldx, W, Cin, nullptr, nullptr, 0, H, C, N, C, Cin, att_src, att_dst, a_src, a_dst);
    else
      k_gemm16<true, 0, true, BF><<<dim3((N + TM - 1) / TM, 1), 1024, 0, s>>>(
          X, ldx, W, Cin, nullptr, nullptr, 0, H, C, N, C, Cin, att_src, att_dst, a_src, a_dst);
  else if (BF && quad_ab(X, ldx, W, Cin, Cin, C, true))
    k_gemm<true, 0, true, BF, false, BF><<<dim3((N + TM - 1) / TM, 1), 256, 0, s>>>(
        X, ldx, W, Cin, nullptr, nullptr, 0, H, C, N, C, Cin, att_src, att_dst, a_src, a_dst);
  else
    k_gemm<true, 0, true, BF><<<dim3((N + TM - 1) / TM, 1), 256, 0, s>>>(
        X, ldx, W, Cin, nullptr, nullptr, 0, H, C, N, C, Cin, att_src, att_dst, a_src, a_dst);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_lin_att_gn(const float* X, const float* W, int32_t N, int32_t Cin, int32_t C,
                                 const float* att_src, const float* att_dst, float* H, float* a_src, float* a_dst,
                                 const vg_gn_apply* gn, void* stream) {
  // one column tile (C <= 64) on the 16-wave f32 tile; otherwise VG_EINVAL and
  // the caller applies the GraphNorm itself (vg_graphnorm_fwd_gnp)
  if (N <= 0 || Cin <= 0 || C <= 0 || C > TN || !(VG_GEMM16 & 2) || !X || !W || !att_src || !att_dst || !H ||
      !a_src || !a_dst || !gn || !gn->stats || !gn->weight || !gn->bias || !gn->mean_scale || gn->seg_rows <= 0 ||
      N % gn->seg_rows != 0 || gn->seg_rows < TM || Cin > kGnaMaxK || Cin % 4 != 0 ||
      (reinterpret_cast<uintptr_t>(X) & 15) || (reinterpret_cast<uintptr_t>(gn->y) & 15) ||
      (reinterpret_cast<uintptr_t>(gn->keep) & 15) || (reinterpret_cast<uintptr_t>(gn->keep_out) & 15) ||
      (gn->iter && gn->keep) ||
      (gn->iter && !(gn->p_drop >= 0.f && gn->p_drop < 1.f)))
    return VG_EINVAL;
  GnaDesc ga;
  ga.stats = gn->stats;
  ga.w = gn->weight;
  ga.b = gn->bias;
  ga.ms = gn->mean_scale;
  ga.keep = gn->keep;
  ga.eps = gn->eps;
  ga.p_drop = gn->p_drop;
  ga.seg_rows = gn->seg_rows;
  ga.salt = gn->salt;
  ga.seed = gn->seed;
  ga.iter = reinterpret_cast<const long long*>(gn->iter);
  ga.y = gn->y;
  ga.keep_out = gn->iter ? gn->keep_out : nullptr;
  k_gemm16_gna<<<dim3((N + TM - 1) / TM, 1), 1024, 0, static_cast<hipStream_t>(stream)>>>(
      X, W, H, N, C, Cin, att_src, att_dst, a_src, a_dst, ga);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_lin_att(const float* X, int32_t ldx, const float* W, int32_t N,
                              int32_t Cin, int32_t C, const float* att_src, const float* att_dst,
                              float* H, float* a_src, float* a_dst, void* stream) {
  return gat_lin_att<false>(X, ldx, W, N, Cin, C, att_src, att_dst, H, a_src, a_dst, stream);
}

extern "C" int vg_gat_lin_att_bf16(const float* X, int32_t ldx, const float* W, int32_t N,
                                   int32_t Cin, int32_t C, const float* att_src, const float* att_dst,
                                   float* H, float* a_src, float* a_dst, void* stream) {
  return gat_lin_att<true>(X, ldx, W, N, Cin, C, att_src, att_dst, H, a_src, a_dst, stream);
}

extern "C" int vg_gemm_tn(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                          int32_t M, int32_t K, float* C, int32_t ldc, float* db, int32_t accumulate,
                          float* workspace, void* stream) {
  return gemm_tn(A, lda, B, ldb, N, M, K, C, ldc, db, N, accumulate, workspace, stream);
}

extern "C" int vg_gemm_tn_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                               int32_t M, int32_t K, float* C, int32_t ldc, float* db, int32_t accumulate,
                               float* workspace, void* stream) {
  return gemm_tn<true>(A, lda, B, ldb, N, M, K, C, ldc, db, N, accumulate, workspace, stream);
}

extern "C" int vg_gemm_tn_ex(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                             int32_t M, int32_t K, float* C, int32_t ldc, float* db,
                             int32_t db_rows, int32_t accumulate, float* workspace, void* stream) {
  return gemm_tn(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, accumulate, workspace, stream);
}
