// GATConv aggregation for large graphs (BASELINE configs[3], the scatter / LDS
// bandwidth stress): each 64-row tile's distinct source rows staged through
// LDS by a persistent, software-pipelined kernel.
//
// Why: the register gather (gat_fused.hip, k_gat_fwd_cp)
// reads h[src] once per EDGE -- E' x C x 4 bytes, 10.5x the compulsory bytes on
// the stress lattice -- and runs at ~0.8 of the measured L2 -> CU gather
// ceiling.  Only fewer gathered bytes can move it.  The first LDS kernel
// (gat_lds.hip, 16-row tiles, one short-lived workgroup per tile) saved too
// little (3.1 edges per distinct source) and exposed a staging round trip per
// tile.  Here:
//
// * tiles of 64 destination rows.  With the voxels numbered in 4 x 4 x 4
//   lattice blocks (vgan.locality.block_order) a tile's edges (~1,380) come
//   from ~224 distinct source rows: 6.2 edges per staged row;
// * one 1024-thread workgroup per CU (C = 128: the 288-row image is 144 KB
//   of the 160 KB LDS; C = 64: two per CU), persistent over a static list of
//   tiles.  An XCD owns one contiguous range of tiles and its workgroups take
//   them interleaved, so the tiles in flight on an XCD are lattice neighbours
//   whose source rows overlap in its L2;
// * software pipelined: while a tile is aggregated out of LDS, the loads of
//   the NEXT tile's source rows (and its a_src entries, its edges' LDS slots,
//   its row_ptr) are already in flight into registers, and the tile after
//   that has its source list on the way.  After a barrier the registers land
//   in the LDS image.  No dependent global round trip is exposed per tile;
// * one destination row per wave (64 lanes, one edge per lane for the
//   softmax, C / 64 channels per lane for the gather-sum): the row's degree is
//   wave-uniform, each edge's (slot, alpha) is broadcast with readlane, each
//   source row is one conflict-free ds_read_b64 (C = 128) out of LDS.
//
// Arithmetic: bit-identical to k_gat_fwd_cp with 16-lane rows (every C in
// 33..128 there; the 64-channel slices of large graphs): the max is exact, the
// softmax denominator is formed in the same grouping (lane l of a 16-lane
// group sums edges l, l + 16, l + 32, l + 48, ... in order, then the same xor
// tree), alpha = p / denom, and the gather-sum runs over the edges in CSR
// order with one fmaf per channel, bias last.
//
// Tiles the plan cannot stage (more than kSU distinct sources, more than kSE
// edges, or a row longer than 64 edges) are marked -1 and aggregated from
// global memory by the same workgroup with the same arithmetic.
#include "rowgroup.h"

namespace {

using namespace vg;

constexpr int kSRT = 64;    // destination rows per tile
constexpr int kSU = 288;    // distinct source rows a tile may stage
constexpr int kSE = 2048;   // edges a tile may sort in the plan
constexpr int kSDeg = 64;   // longest row of a staged tile (one edge per lane)
constexpr int kSNT = 1024;  // threads per workgroup (plan and aggregation)
constexpr int kRPW = kSRT / (kSNT / 64);  // destination rows per wave and tile (4)

// ---------------------------------------------------------------- plan
// tile t (rows [64 t, 64 t + 64)): ucount[t] distinct sources, sorted, in
// usrc[t * kSU + u]; lidx[k] = the slot of edge k's source in that list.
__global__ void __launch_bounds__(kSNT) k_stage_plan(const int32_t* __restrict__ row_ptr,
                                                     const int32_t* __restrict__ col, int N,
                                                     int32_t* __restrict__ ucount, int32_t* __restrict__ usrc,
                                                     uint16_t* __restrict__ lidx) {
  __shared__ unsigned long long key[kSE];  // (source << 32) | edge offset in the tile
  __shared__ int scan[kSE];
  __shared__ int s_long;
  const int t = blockIdx.x, tid = threadIdx.x;
  const int r0 = t * kSRT, r1 = min(N, r0 + kSRT);
  const int e0 = row_ptr[r0], e1 = row_ptr[r1];
  const int ne = e1 - e0;
  if (tid == 0) s_long = 0;
  __syncthreads();
  if (tid < r1 - r0 && row_ptr[r0 + tid + 1] - row_ptr[r0 + tid] > kSDeg) s_long = 1;
  __syncthreads();
  if (s_long || ne > kSE || ne <= 0) {
    if (tid == 0) ucount[t] = ne <= 0 ? 0 : -1;
    return;
  }
  int P = 2;
  while (P < ne) P <<= 1;
  for (int i = tid; i < P; i += kSNT)
    key[i] = i < ne ? ((unsigned long long)(uint32_t)col[e0 + i] << 32) | (uint32_t)i : ~0ULL;
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {  // bitonic sort, ascending
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < P; i += kSNT) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const unsigned long long a = key[i], b = key[ixj];
          if ((a > b) == ((i & k) == 0)) {
            key[i] = b;
            key[ixj] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < P; i += kSNT)  // first-of-run flags, then an inclusive scan
    scan[i] = (i < ne && (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32))) ? 1 : 0;
  __syncthreads();
  for (int off = 1; off < P; off <<= 1) {
    int v[kSE / kSNT];
#pragma unroll
    for (int q = 0; q < kSE / kSNT; ++q) {
      const int i = tid + kSNT * q;
      v[q] = (i < P && i >= off) ? scan[i - off] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kSE / kSNT; ++q) {
      const int i = tid + kSNT * q;
      if (i < P) scan[i] += v[q];
    }
    __syncthreads();
  }
  const int U = scan[ne - 1];
  if (U > kSU) {
    if (tid == 0) ucount[t] = -1;
    return;
  }
  for (int i = tid; i < ne; i += kSNT) {
    const int slot = scan[i] - 1;
    if (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32)) usrc[(size_t)t * kSU + slot] = static_cast<int>(key[i] >> 32);
    lidx[e0 + static_cast<int>(key[i] & 0xffffffffu)] = static_cast<uint16_t>(slot);
  }
  if (tid == 0) ucount[t] = U;
}

// ---------------------------------------------------------- aggregation
template <int CPL>
struct RowOf;
template <>
struct RowOf<1> {
  using T = float;
  static __device__ __forceinline__ void fma(float a, T v, float* acc) { acc[0] = fmaf(a, v, acc[0]); }
  static __device__ __forceinline__ T make(const float* a) { return a[0]; }
};
template <>
struct RowOf<2> {
  using T = float2;
  static __device__ __forceinline__ void fma(float a, T v, float* acc) {
    acc[0] = fmaf(a, v.x, acc[0]);
    acc[1] = fmaf(a, v.y, acc[1]);
  }
  static __device__ __forceinline__ T make(const float* a) { return make_float2(a[0], a[1]); }
};

__device__ __forceinline__ int rdl(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// Per-tile state a wave keeps in registers: lane j of rp = row_ptr[r0 + j]
// (clamped to N), rpl = row_ptr[min(r0 + 64, N)], lane j of ad = a_dst[r0 + j],
// li[i] = lane j's edge of the wave's i-th row: its LDS slot (staged tile) or
// its source (a tile aggregated from global memory).
struct TileRegs {
  int U;     // distinct sources (-1: from global memory)
  int rp;    // lane-indexed row_ptr
  int rpl;   // row_ptr past the tile
  float ad;  // lane-indexed a_dst
  int li0, li1, li2, li3;  // named, not an array: an indexed int[4] is parked in scratch
  __device__ __forceinline__ int li(int i) const { return i == 0 ? li0 : i == 1 ? li1 : i == 2 ? li2 : li3; }
  __device__ __forceinline__ void set_li(int i, int v) {
    if (i == 0) li0 = v;
    else if (i == 1) li1 = v;
    else if (i == 2) li2 = v;
    else li3 = v;
  }
};
static_assert(kRPW == 4, "TileRegs names four rows per wave");

__device__ __forceinline__ void tile_head(TileRegs& s, int t, int N, const int32_t* __restrict__ row_ptr,
                                          const float* __restrict__ a_dst, const int32_t* __restrict__ ucount,
                                          int lane) {
  const int r0 = t * kSRT;
  s.U = ucount[t];
  s.rp = row_ptr[min(r0 + lane, N)];
  s.rpl = row_ptr[min(r0 + kSRT, N)];
  s.ad = a_dst[min(r0 + lane, N - 1)];
}

// the wave's rows' edge slots (needs s.rp, s.rpl: loaded one step earlier)
__device__ __forceinline__ void tile_edges(TileRegs& s, int wave, int lane, const int32_t* __restrict__ col,
                                           const uint16_t* __restrict__ lidx) {
#pragma unroll
  for (int i = 0; i < kRPW; ++i) {
    const int ri = wave * kRPW + i;
    const int beg = rdl(s.rp, ri);
    const int end = ri == kSRT - 1 ? s.rpl : rdl(s.rp, ri + 1);
    const int k = beg + lane;
    int v = 0;
    if (k < end) v = s.U >= 0 ? static_cast<int>(lidx[k]) : col[k];
    s.set_li(i, v);
  }
}

// Staging of a tile's rows through named registers st0..st8 (Q <= 9 float4
// per thread): an indexed float4[9] is parked in scratch.  Rows past the
// tile's U clamp to row U - 1 (a duplicate load and an identical store):
// unguarded loads stay in flight together.
#define VG_Q9(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8)
#define VG_ST_DECL(q) float4 st##q = make_float4(0.f, 0.f, 0.f, 0.f);
#define VG_ST_LOAD(q)                                                                        \
  if constexpr ((q) < Q) {                                                                   \
    const int f = tid + kSNT * (q);                                                          \
    const int u = min(f / C4, ul_);                                                          \
    st##q = *reinterpret_cast<const float4*>(h + (size_t)s_us[u] * C + (f % C4) * 4);        \
  }
#define VG_ST_STORE(q)                                                                       \
  if constexpr ((q) < Q) {                                                                   \
    const int f = tid + kSNT * (q);                                                          \
    const int u = min(f / C4, ul_);                                                          \
    s_rows[u * C4 + f % C4] = st##q;                                                         \
  }
#define VG_STAGE_LOAD(U_)                      \
  do {                                         \
    const int ul_ = (U_) - 1;                  \
    VG_Q9(VG_ST_LOAD)                          \
    sa = a_src[s_us[min(tid, ul_)]];           \
  } while (0)
#define VG_STAGE_STORE(U_)                     \
  do {                                         \
    const int ul_ = (U_) - 1;                  \
    VG_Q9(VG_ST_STORE)                         \
    if (tid < (U_)) s_as[tid] = sa;            \
  } while (0)

template <int C>
__global__ void __launch_bounds__(kSNT) k_gat_fwd_staged(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, const float* __restrict__ h,
    const float* __restrict__ a_src, const float* __restrict__ a_dst, const float* __restrict__ bias, float slope,
    float* __restrict__ out, float* __restrict__ alpha, const int32_t* __restrict__ ucount,
    const int32_t* __restrict__ usrc, const uint16_t* __restrict__ lidx, int tiles) {
  constexpr int CPL = C / 64, C4 = C / 4;
  constexpr int Q = (kSU * C4 + kSNT - 1) / kSNT;  // staged float4s per thread
  using R = RowOf<CPL>;
  using RowT = typename R::T;
  __shared__ float4 s_rows[kSU * C4];  // the tile's distinct source rows
  __shared__ float s_as[kSU];          // their a_src
  __shared__ int s_us[kSU];            // the NEXT tile's source list
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // static, XCD-aware schedule: XCD x (hardware block b runs on XCD b % 8)
  // owns tiles [tiles x / 8, tiles (x + 1) / 8); its workgroups take them
  // interleaved, so the tiles in flight on one XCD are neighbours
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int tb = static_cast<int>((long long)tiles * xcd / 8);
  const int te = static_cast<int>((long long)tiles * (xcd + 1) / 8);
  auto tile_at = [&](int k) {
    const int t = tb + slot + k * per;
    return t < te ? t : -1;
  };
  int t = tile_at(0);
  if (t < 0) return;
  RowT bv;
  {
    float b[CPL];
#pragma unroll
    for (int q = 0; q < CPL; ++q) b[q] = bias[lane * CPL + q];
    bv = R::make(b);
  }
  const float* bvf = reinterpret_cast<const float*>(&bv);

  static_assert(Q <= 9, "VG_Q9 names nine staging registers");
  VG_Q9(VG_ST_DECL)
  float sa = 0.f;

  // ---- prologue: tile t staged in LDS, tile n's list in s_us
  TileRegs cur, nxt;
  tile_head(cur, t, N, row_ptr, a_dst, ucount, lane);
  if (tid < kSU) s_us[tid] = usrc[(size_t)t * kSU + tid];
  tile_edges(cur, wave, lane, col, lidx);
  __syncthreads();
  if (cur.U > 0) {
    VG_STAGE_LOAD(cur.U);
    VG_STAGE_STORE(cur.U);
  }
  int n = tile_at(1);
  int ul = 0;
  if (n >= 0) {
    tile_head(nxt, n, N, row_ptr, a_dst, ucount, lane);
    if (tid < kSU) ul = usrc[(size_t)n * kSU + tid];
  }
  __syncthreads();
  if (n >= 0 && tid < kSU) s_us[tid] = ul;
  __syncthreads();

  for (int k = 0;; ++k) {
    const int nn = n >= 0 ? tile_at(k + 2) : -1;
    // ---- A: next tile's rows / slots, and the tile after's list, in flight
    TileRegs nn_regs;
    if (n >= 0) {
      tile_edges(nxt, wave, lane, col, lidx);
      if (nxt.U > 0) VG_STAGE_LOAD(nxt.U);
    }
    if (nn >= 0) {
      tile_head(nn_regs, nn, N, row_ptr, a_dst, ucount, lane);
      if (tid < kSU) ul = usrc[(size_t)nn * kSU + tid];
    }
    // ---- B: aggregate tile t
    const int r0 = t * kSRT;
#pragma unroll
    for (int i = 0; i < kRPW; ++i) {
      const int ri = wave * kRPW + i;
      const int r = r0 + ri;
      if (r >= N) break;
      const int beg = rdl(cur.rp, ri);
      const int end = ri == kSRT - 1 ? cur.rpl : rdl(cur.rp, ri + 1);
      const int deg = end - beg;
      const float ad = rdl(cur.ad, ri);
      const int li = cur.li(i);
      const bool v = lane < deg;
      const bool staged = cur.U >= 0;
      float e = -INFINITY;
      if (v) e = lrelu((staged ? s_as[li] : a_src[li]) + ad, slope);
      float m = e;
      if (!staged)
        for (int kk = beg + lane + 64; kk < end; kk += 64) m = fmaxf(m, lrelu(a_src[col[kk]] + ad, slope));
      m = group_max<64>(m);
      const float p = v ? expf(e - m) : 0.f;
      // the denominator in k_gat_fwd_cp<16, ...>'s grouping: lane l of a
      // 16-lane group sums edges l, l + 16, l + 32, l + 48 (then, on long
      // rows, l + 64, l + 80, ...) in order, then the same xor tree
      float s = p;
      s += __shfl(p, (lane + 16) & 63, 64);
      s += __shfl(p, (lane + 32) & 63, 64);
      s += __shfl(p, (lane + 48) & 63, 64);
      if (!staged && lane < 16)
        for (int kk = beg + lane + 64; kk < end; kk += 16) s += expf(lrelu(a_src[col[kk]] + ad, slope) - m);
      s = group_sum<16>(s);
      const float denom = rdl(s, 0) + kSoftmaxEps;
      const float a = v ? p / denom : 0.f;
      if (v) alpha[beg + lane] = a;
      float acc[CPL];
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc[q] = 0.f;
      const int dreg = deg < 64 ? deg : 64;
      if (staged) {
        const RowT* rows = reinterpret_cast<const RowT*>(s_rows);
        for (int j0 = 0; j0 < dreg; j0 += 4) {
          RowT hv[4];
          float aj[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < dreg) {
              aj[u] = rdl(a, j0 + u);
              hv[u] = rows[rdl(li, j0 + u) * 64 + lane];
            }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < dreg) R::fma(aj[u], hv[u], acc);
        }
      } else {
        for (int kk = beg + lane + 64; kk < end; kk += 64)
          alpha[kk] = expf(lrelu(a_src[col[kk]] + ad, slope) - m) / denom;
        for (int j0 = 0; j0 < dreg; j0 += 4) {
          RowT hv[4];
          float aj[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < dreg) {
              aj[u] = rdl(a, j0 + u);
              hv[u] = *reinterpret_cast<const RowT*>(h + (size_t)rdl(li, j0 + u) * C + lane * CPL);
            }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (j0 + u < dreg) R::fma(aj[u], hv[u], acc);
        }
        for (int j = 64; j < deg; ++j) {  // very long rows: alpha recomputed as k_gat_fwd_cp does
          const int sj = col[beg + j];
          const float aa = expf(lrelu(a_src[sj] + ad, slope) - m) / denom;
          R::fma(aa, *reinterpret_cast<const RowT*>(h + (size_t)sj * C + lane * CPL), acc);
        }
      }
#pragma unroll
      for (int q = 0; q < CPL; ++q) acc[q] += bvf[q];
      *reinterpret_cast<RowT*>(out + (size_t)r * C + lane * CPL) = R::make(acc);
    }
    if (n < 0) break;
    // ---- C / D / E: the next tile's registers into LDS
    __syncthreads();
    if (nxt.U > 0) VG_STAGE_STORE(nxt.U);
    if (nn >= 0 && tid < kSU) s_us[tid] = ul;
    __syncthreads();
    t = n;
    n = nn;
    cur = nxt;
    if (nn >= 0) nxt = nn_regs;
  }
}

int g_num_cu = 0;

int num_cu() {
  if (g_num_cu == 0) {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      g_num_cu = v;
    else
      g_num_cu = 256;
  }
  return g_num_cu;
}

}  // namespace

#undef VG_Q9
#undef VG_ST_DECL
#undef VG_ST_LOAD
#undef VG_ST_STORE
#undef VG_STAGE_LOAD
#undef VG_STAGE_STORE

extern "C" int64_t vg_gat_stage_plan_ints(int32_t num_nodes, int32_t num_edges) {
  const int64_t tiles = ((int64_t)num_nodes + kSRT - 1) / kSRT;
  // ucount [tiles] + usrc [tiles * kSU] (int32) + lidx [E'] (uint16, rounded up to int32s)
  return tiles + tiles * kSU + ((int64_t)num_edges + 1) / 2;
}

extern "C" int vg_gat_stage_plan(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t E, int32_t* plan,
                                 void* stream) {
  if (N <= 0 || E <= 0 || !row_ptr || !col || !plan) return VG_EINVAL;
  const int tiles = (N + kSRT - 1) / kSRT;
  int32_t* ucount = plan;
  int32_t* usrc = plan + tiles;
  uint16_t* lidx = reinterpret_cast<uint16_t*>(usrc + (size_t)tiles * kSU);
  k_stage_plan<<<tiles, kSNT, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, col, N, ucount, usrc, lidx);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_aggregate_fwd_staged(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                                           const float* h, const float* a_src, const float* a_dst,
                                           const float* bias, float slope, float* out, float* alpha,
                                           const int32_t* plan, void* stream) {
  if (N <= 0 || (C != 64 && C != 128) || !row_ptr || !col || !h || !a_src || !a_dst || !bias || !out || !alpha ||
      !plan || (reinterpret_cast<uintptr_t>(h) & 15) || (reinterpret_cast<uintptr_t>(out) & 7))
    return VG_EINVAL;
  const int tiles = (N + kSRT - 1) / kSRT;
  const int32_t* ucount = plan;
  const int32_t* usrc = plan + tiles;
  const uint16_t* lidx = reinterpret_cast<const uint16_t*>(usrc + (size_t)tiles * kSU);
  // one workgroup per CU at C = 128 (144 KB of LDS), two at C = 64; a
  // multiple of 8 (the XCD schedule), no more than the tiles need
  const int per_cu = C == 128 ? 1 : 2;
  int grid = num_cu() * per_cu;
  const int need = (tiles + 7) / 8 * 8;
  if (grid > need) grid = need;
  grid = (grid + 7) / 8 * 8;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (C == 128)
    k_gat_fwd_staged<128><<<grid, kSNT, 0, s>>>(row_ptr, col, N, h, a_src, a_dst, bias, slope, out, alpha, ucount,
                                                  usrc, lidx, tiles);
  else
    k_gat_fwd_staged<64><<<grid, kSNT, 0, s>>>(row_ptr, col, N, h, a_src, a_dst, bias, slope, out, alpha, ucount,
                                                 usrc, lidx, tiles);
  VG_CHECK_LAUNCH();
  return 0;
}
