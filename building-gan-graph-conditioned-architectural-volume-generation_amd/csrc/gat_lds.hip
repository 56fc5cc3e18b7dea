// GATConv aggregation with the CSR's source rows staged through LDS (large
// graphs: BASELINE configs[3], the scatter / LDS bandwidth stress).
//
// The register-gather kernel (gat_fused.hip, k_gat_fwd_cp) reads h[src] once
// per EDGE: on the configs[3] lattice (degree 21.6) that is E' x 256 B per
// 64-channel slice, served from the XCD L2 at ~14 TB/s, i.e. the kernel is
// bound by the L2 -> CU gather rate, not by HBM.  Consecutive destination
// rows share most of their sources (x +- 1, y +- 1 and the 3 x 3 blocks of the
// floors above and below), so a tile of 16 destination rows touches ~160
// distinct source rows for ~350 edges.
//
// Tile plan (vg_gat_tile_plan, once per CSR -- the graph, not the layer):
// for tile t (rows [16t, 16t + 16)) the sorted distinct sources of its edges,
// usrc[t * 256 + u], their count ucount[t], and for every edge k its slot
// lidx[k] in that list.  Tiles with more than 1024 edges or 256 distinct
// sources get ucount = -1 and gather from global memory as before.
//
// Aggregation (vg_gat_aggregate_fwd_lds): one 256-thread workgroup per (tile,
// 64-channel slice).  It copies the tile's distinct source rows into LDS
// (16 lanes x float4 per row: coalesced 256-B row reads, every row once),
// forms the row softmax exactly as k_gat_fwd_cp does with 16-lane rows
// (C <= 128: the outputs are bit-identical to it; its 32-lane rows for wider
// C sum the denominator in another grouping), then gathers the
// weighted rows from LDS.  Global gather bytes drop from E' rows to the sum of
// distinct rows per tile (~2.2x fewer on configs[3]).
//
// Measured (profiles/r02_rejected_lds_aggregate.txt): 497 us at C = 128 vs
// 334 us for the register gather -- the exposed staging round trip, the tile
// barrier and the 40 KB LDS image (4 waves / SIMD) cost more than the L2
// reads saved.  Not the product default; bench.py reports both kernels.
#include "rowgroup.h"

namespace {

using namespace vg;

constexpr int kRT = 16;   // destination rows per tile (16 lanes x 4 channels each: 256 threads)
constexpr int kU = 256;   // distinct source rows a tile may stage (64 KB of LDS at 64 channels)
constexpr int kE = 1024;  // edges a tile may sort in the plan

// ---------------------------------------------------------------- plan
__global__ void __launch_bounds__(256) k_tile_plan(const int32_t* __restrict__ row_ptr,
                                                   const int32_t* __restrict__ col, int N,
                                                   int32_t* __restrict__ ucount, int32_t* __restrict__ usrc,
                                                   uint16_t* __restrict__ lidx) {
  __shared__ unsigned long long key[kE];  // (source << 32) | edge offset in the tile
  __shared__ int scan[kE];
  const int t = blockIdx.x, tid = threadIdx.x;
  const int r0 = t * kRT, r1 = min(N, r0 + kRT);
  const int e0 = row_ptr[r0], e1 = row_ptr[r1];
  const int ne = e1 - e0;
  if (ne > kE || ne <= 0) {
    if (tid == 0) ucount[t] = ne <= 0 ? 0 : -1;
    return;
  }
  int P = 2;
  while (P < ne) P <<= 1;
  for (int i = tid; i < P; i += 256)
    key[i] = i < ne ? ((unsigned long long)(uint32_t)col[e0 + i] << 32) | (uint32_t)i : ~0ULL;
  __syncthreads();
  // bitonic sort of P keys (ascending)
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += 256) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = key[i], b = key[ixj];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            key[i] = b;
            key[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  // first-of-run flags, then an inclusive scan: the slot of every sorted key
  for (int i = tid; i < P; i += 256)
    scan[i] = (i < ne && (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32))) ? 1 : 0;
  __syncthreads();
  for (int off = 1; off < P; off <<= 1) {
    int v[kE / 256];
#pragma unroll
    for (int q = 0; q < kE / 256; ++q) {
      const int i = tid + 256 * q;
      v[q] = (i < P && i >= off) ? scan[i - off] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kE / 256; ++q) {
      const int i = tid + 256 * q;
      if (i < P) scan[i] += v[q];
    }
    __syncthreads();
  }
  const int U = scan[ne - 1];
  if (U > kU) {
    if (tid == 0) ucount[t] = -1;
    return;
  }
  for (int i = tid; i < ne; i += 256) {
    const int slot = scan[i] - 1;
    const int src = static_cast<int>(key[i] >> 32);
    if (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32)) usrc[(size_t)t * kU + slot] = src;
    lidx[e0 + static_cast<int>(key[i] & 0xffffffffu)] = static_cast<uint16_t>(slot);
  }
  if (tid == 0) ucount[t] = U;
}

// ---------------------------------------------------------- aggregation
// grid (tiles, C / kSl); h / out / bias rows are ld floats apart, the slice at
// blockIdx.y * kSl, kSl = 16 lanes x CPL channels.  Mirrors k_gat_fwd_cp<16, 4,
// true> (T = 4 edge slots per lane, 4 neighbour rows per step, bias in the
// same pass).  CPL = 2 halves the LDS image per workgroup (occupancy) at the
// price of one more softmax pass per row.
template <int CPL>
__global__ void __launch_bounds__(256) k_gat_fwd_lds(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int ld,
    const float* __restrict__ h, const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ bias, float slope, float* __restrict__ out, float* __restrict__ alpha,
    const int32_t* __restrict__ ucount, const int32_t* __restrict__ usrc, const uint16_t* __restrict__ lidx) {
  constexpr int L = 16, T = 4, QS = kU / (256 / L), kSl = L * CPL;  // QS: staged rows per lane group
  using RowT = typename std::conditional<CPL == 4, float4, float2>::type;
  extern __shared__ float4 lds_raw[];
  RowT* rows = reinterpret_cast<RowT*>(lds_raw);  // [umax][16]: the tile's distinct source rows, kSl channels each
  __shared__ int s_us[kU];
  const int cb = blockIdx.y * kSl;
  h += cb;
  out += cb;
  bias += cb;
  const bool wr_alpha = blockIdx.y == 0;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int tid = threadIdx.x, lane = tid & (L - 1), grp = tid / L;
  const int U = ucount[t];
  if (tid < U) s_us[tid] = usrc[(size_t)t * kU + tid];  // the source list: one coalesced load
  __syncthreads();
  // stage: issue every row load now (16 lanes x float4 per row, each distinct
  // row once), keep them in flight through the softmax, store to LDS after it
  static_assert(QS == 16, "the staging macros name 16 rows per lane group");
#define VG_REP16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
  // named registers, not an array: an indexed float4[16] is parked in scratch
#define VG_DECL(q) RowT st##q;
  VG_REP16(VG_DECL)
#undef VG_DECL
#ifndef VG_LDS_EARLY
#define VG_LDS_EARLY 0  // A/B: store the staged rows to LDS right after their loads
#endif
#ifndef VG_LDS_PROBE
#define VG_LDS_PROBE 0  // A/B probe: 1 = stage but gather from global, 2 = no staging (global gather)
#endif
  // No guards: rows past U clamp to row U - 1 (a duplicate load, mostly an L1
  // hit, and an identical store).  A guarded load becomes its own basic block;
  // the compiler then sinks it into the store loop or parks st[] in scratch,
  // and every load waits before the next one issues.
  const int ulast = U > 0 ? U - 1 : 0;
  const float* hl = h + lane * CPL;
#define VG_LD(q) st##q = *reinterpret_cast<const RowT*>(hl + (size_t)s_us[min(grp + (q) * (256 / L), ulast)] * ld);
  if (VG_LDS_PROBE != 2 && U > 0) { VG_REP16(VG_LD) }
#undef VG_LD
#if VG_LDS_EARLY
#define VG_ST(q) rows[min(grp + (q) * (256 / L), ulast) * L + lane] = st##q;
  if (VG_LDS_PROBE != 2 && U > 0) { VG_REP16(VG_ST) }
#undef VG_ST
#endif
  const int i = t * kRT + grp;
  const bool live = i < N;
  const int base = (tid & 63) & ~(L - 1);
  int beg = 0, end = 0;
  float ad = 0.f;
  if (live) {
    beg = row_ptr[i];
    end = row_ptr[i + 1];
    ad = a_dst[i];
  }
  const int deg = end - beg;
  int s_t[T];
  float e_t[T];
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < T; ++q) {
    const int k = beg + lane + q * L;
    s_t[q] = 0;
    e_t[q] = -INFINITY;
    if (k < end) {
      s_t[q] = col[k];
      e_t[q] = lrelu(a_src[s_t[q]] + ad, slope);
      m = fmaxf(m, e_t[q]);
    }
  }
  for (int k = beg + lane + T * L; k < end; k += L) m = fmaxf(m, lrelu(a_src[col[k]] + ad, slope));
  m = group_max<L>(m);
  float ssum = 0.f;
#pragma unroll
  for (int q = 0; q < T; ++q)
    if (beg + lane + q * L < end) {
      e_t[q] = expf(e_t[q] - m);
      ssum += e_t[q];
    }
  for (int k = beg + lane + T * L; k < end; k += L) ssum += expf(lrelu(a_src[col[k]] + ad, slope) - m);
  const float denom = group_sum<L>(ssum) + kSoftmaxEps;
#pragma unroll
  for (int q = 0; q < T; ++q) {
    const int k = beg + lane + q * L;
    if (k < end) {
      e_t[q] = e_t[q] / denom;
      if (wr_alpha) alpha[k] = e_t[q];
    }
  }
  if (wr_alpha)
    for (int k = beg + lane + T * L; k < end; k += L) alpha[k] = expf(lrelu(a_src[col[k]] + ad, slope) - m) / denom;
  // per-edge LDS slots (or, for an unplanned tile, the sources themselves)
  int l_t[T];
#pragma unroll
  for (int q = 0; q < T; ++q) {
    const int k = beg + lane + q * L;
    l_t[q] = (VG_LDS_PROBE == 0 && U >= 0 && k < end) ? static_cast<int>(lidx[k]) : s_t[q];
  }
#if !VG_LDS_EARLY
#define VG_ST(q) rows[min(grp + (q) * (256 / L), ulast) * L + lane] = st##q;
  if (VG_LDS_PROBE != 2 && U > 0) { VG_REP16(VG_ST) }
#undef VG_ST
#endif
  __syncthreads();  // the staged rows are complete
  const int c0 = lane * CPL;
  Vec<CPL> acc;
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] = 0.f;
  const int dreg = deg < T * L ? deg : T * L;
  for (int j0 = 0; j0 < dreg; j0 += 4) {
    const int nj = dreg - j0 < 4 ? dreg - j0 : 4;
    Vec<CPL> hv[4];
    float a[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < nj) {
        const int j = j0 + u;
        const int q = j / L;
        const int lv = q == 0 ? l_t[0] : q == 1 ? l_t[1] : q == 2 ? l_t[2] : l_t[3];
        const float av = q == 0 ? e_t[0] : q == 1 ? e_t[1] : q == 2 ? e_t[2] : e_t[3];
        const int sl = __shfl(lv, base + (j & (L - 1)), 64);
        a[u] = __shfl(av, base + (j & (L - 1)), 64);
        if (VG_LDS_PROBE == 0 && U >= 0) {
          const RowT r = rows[sl * L + lane];
          const float* rf = reinterpret_cast<const float*>(&r);
#pragma unroll
          for (int q = 0; q < CPL; ++q) hv[u].v[q] = rf[q];
        } else {
          load_row<CPL, true>(hv[u], h + (size_t)sl * ld, c0, kSl);
        }
      }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (u < nj)
#pragma unroll
        for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a[u], hv[u].v[q], acc.v[q]);
  }
  for (int j = T * L; j < deg; ++j) {  // very long rows: alpha recomputed, rows from global memory
    const int s = col[beg + j];
    const float a = expf(lrelu(a_src[s] + ad, slope) - m) / denom;
    Vec<CPL> hv;
    load_row<CPL, true>(hv, h + (size_t)s * ld, c0, kSl);
#pragma unroll
    for (int q = 0; q < CPL; ++q) acc.v[q] = fmaf(a, hv.v[q], acc.v[q]);
  }
  if (!live) return;
  Vec<CPL> b;
  load_row<CPL, false>(b, bias, c0, kSl);
#pragma unroll
  for (int q = 0; q < CPL; ++q) acc.v[q] += b.v[q];
  store_row<CPL, true>(acc, out + (size_t)i * ld, c0, kSl);
}

}  // namespace

extern "C" int64_t vg_gat_tile_plan_ints(int32_t num_nodes, int32_t num_edges) {
  const int64_t tiles = ((int64_t)num_nodes + kRT - 1) / kRT;
  // ucount [tiles] + usrc [tiles * 256] (int32) + lidx [E'] (uint16, rounded up to int32s)
  return tiles + tiles * kU + ((int64_t)num_edges + 1) / 2;
}

extern "C" int vg_gat_tile_plan(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t E, int32_t* plan,
                                void* stream) {
  if (N <= 0 || E <= 0 || !row_ptr || !col || !plan) return VG_EINVAL;
  const int tiles = (N + kRT - 1) / kRT;
  int32_t* ucount = plan;
  int32_t* usrc = plan + tiles;
  uint16_t* lidx = reinterpret_cast<uint16_t*>(usrc + (size_t)tiles * kU);
  k_tile_plan<<<tiles, 256, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, col, N, ucount, usrc, lidx);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_aggregate_fwd_lds(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                                        const float* h, const float* a_src, const float* a_dst, const float* bias,
                                        float slope, float* out, float* alpha, const int32_t* plan, int32_t umax,
                                        void* stream) {
#ifndef VG_LDS_SLICE
#define VG_LDS_SLICE 64  // 32: force 32-channel slices (A/B; profiles/r02_rejected_lds_aggregate.txt)
#endif
  // 64-channel slices; 32 when C is not a multiple of 64.  Halving the LDS
  // image with 32-channel slices for occupancy measured slower (589 vs 494 us).
  const int sl = C % 64 == 0 ? VG_LDS_SLICE : 32;
  if (N <= 0 || C <= 0 || C % sl != 0 || !row_ptr || !col || !h || !a_src || !a_dst || !bias || !out || !alpha ||
      !plan || umax < 1 || umax > kU ||
      (reinterpret_cast<uintptr_t>(out) & (sl == 64 ? 15 : 7)) || (reinterpret_cast<uintptr_t>(h) & (sl == 64 ? 15 : 7)))
    return VG_EINVAL;
  const int tiles = (N + kRT - 1) / kRT;
  const int32_t* ucount = plan;
  const int32_t* usrc = plan + tiles;
  const uint16_t* lidx = reinterpret_cast<const uint16_t*>(usrc + (size_t)tiles * kU);
  const size_t lds = (size_t)umax * sl * sizeof(float);  // the largest tile's rows
  if (sl == 64)
    k_gat_fwd_lds<4><<<dim3(tiles, C / 64), 256, lds, static_cast<hipStream_t>(stream)>>>(
        row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, ucount, usrc, lidx);
  else
    k_gat_fwd_lds<2><<<dim3(tiles, C / 32), 256, lds, static_cast<hipStream_t>(stream)>>>(
        row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, ucount, usrc, lidx);
  VG_CHECK_LAUNCH();
  return 0;
}
