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
template <int RT, int SU, int SE>
__global__ void __launch_bounds__(kSNT) k_stage_plan(const int32_t* __restrict__ row_ptr,
                                                     const int32_t* __restrict__ col, int N,
                                                     int32_t* __restrict__ ucount, int32_t* __restrict__ usrc,
                                                     uint16_t* __restrict__ lidx) {
  __shared__ unsigned long long key[SE];  // (source << 32) | edge offset in the tile
  __shared__ int scan[SE];
  __shared__ int s_long;
  const int t = blockIdx.x, tid = threadIdx.x;
  const int r0 = t * RT, r1 = min(N, r0 + RT);
  const int e0 = row_ptr[r0], e1 = row_ptr[r1];
  const int ne = e1 - e0;
  if (tid == 0) s_long = 0;
  __syncthreads();
  if (tid < r1 - r0 && row_ptr[r0 + tid + 1] - row_ptr[r0 + tid] > kSDeg) s_long = 1;
  __syncthreads();
  if (s_long || ne > SE || ne <= 0) {
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
    int v[SE / kSNT];
#pragma unroll
    for (int q = 0; q < SE / kSNT; ++q) {
      const int i = tid + kSNT * q;
      v[q] = (i < P && i >= off) ? scan[i - off] : 0;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < SE / kSNT; ++q) {
      const int i = tid + kSNT * q;
      if (i < P) scan[i] += v[q];
    }
    __syncthreads();
  }
  const int U = scan[ne - 1];
  if (U > SU) {
    if (tid == 0) ucount[t] = -1;
    return;
  }
  for (int i = tid; i < ne; i += kSNT) {
    const int slot = scan[i] - 1;
    if (i == 0 || (key[i] >> 32) != (key[i - 1] >> 32)) usrc[(size_t)t * SU + slot] = static_cast<int>(key[i] >> 32);
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

// ------------------------------------------------------ wave-specialised ring
// k_gat_fwd_ring: the plan's tiles through an LDS ring filled by LOADER waves
// while CONSUMER waves aggregate the slots already filled, with no workgroup
// barrier after the prologue.  k_gat_fwd_staged had all 16
// waves stage, barrier, aggregate, barrier: its 1024-thread workgroups sat
// parked on those barriers for 47 % of their cycles.  Here, one 16-wave
// workgroup per CU:
//
// * 4 loader waves fill slot (item % NS) -- an item is one 64-channel slice
//   of a tile -- with the tile's distinct source rows by global_load_lds
//   (LDS-DMA: 16 B a lane, four 256-B rows a wave instruction, no VGPR round
//   trip) and, on its first slice, its metadata (row_ptr, a_dst, the edges'
//   LDS slots, the a_src rows); the index loads run two stages ahead (the
//   next tile's body, the head of the one after).  Then they wait for their
//   loads and bump the slot's FULL counter;
// * 12 consumer waves claim (tile, 4-row group) units in order from an LDS
//   counter, wait for FULL, aggregate their group's rows in 16-lane row groups
//   out of LDS and bump the slot's FREE counter once per group; a unit spans
//   the tile's slices, its softmax kept in registers.  A loader refills a slot
//   once FREE says every group is done with it.  Counters only grow
//   (generation = item / NS), so nothing is reset inside a launch; every wait
//   is bounded (on expiry the launch sets *err and ends -- the caller treats
//   the output as invalid);
// * the per-row arithmetic is k_gat_fwd_cp<16, 4>'s (16 lanes x 4 channels,
//   edge j on lane j % 16, slot j / 16; the same max, the same sum order, the
//   same gather order): bit-identical to vg_gat_aggregate_fwd.  Edge j's
//   (slot, alpha) reach the row's 16 lanes by DPP row_newbcast and the
//   softmax's group reductions run on DPP row rotations (no LDS round trip);
// * tiles the plan could not stage (ucount < 0) are aggregated from global
//   memory by the consumers with the same arithmetic.
#ifndef VG_RING_LW
#define VG_RING_LW 4
#endif
#ifndef VG_RING_RT
#define VG_RING_RT 64  // rows per ring tile: 64 (two slots); 48 (two) and 32 (three) measured slower, DESIGN.md 4.41
#endif
#ifndef VG_RING_CW
#define VG_RING_CW (16 - VG_RING_LW)
#endif
constexpr int kRLW = VG_RING_LW, kRCW = VG_RING_CW;  // loader / consumer waves
constexpr int kRNT = (kRLW + kRCW) * 64;            // threads per workgroup
constexpr int kRSpin = 1 << 22;

// A ring's tile geometry: RT rows a tile, up to SU distinct source rows and SE
// edges staged, NS slots of [SU rows x 64 channels | a_src | row_ptr | a_dst |
// edge slots] in LDS (+ the counters).
template <int RT_, int SU_, int SE_, int NS_>
struct RingGeom {
  static constexpr int RT = RT_, SU = SU_, SE = SE_, NS = NS_;
  static constexpr int Groups = RT / 4;                     // 4-row consumer groups per tile
  static constexpr int RowsB = SU * 64 * 4;
  static constexpr int RpB = ((RT + 1) * 4 + 15) / 16 * 16;
  static constexpr int SlotB = RowsB + SU * 4 + RpB + RT * 4 + SE * 2;
  static constexpr int RingB = NS * SlotB + 64;
  static constexpr int RowI = (SU / 4 + kRLW - 1) / kRLW;      // row-staging instructions per loader wave
  static constexpr int AsQ = (SU + kRLW * 64 - 1) / (kRLW * 64);  // a_src entries per loader lane
  static constexpr int LiQ = (SE + kRLW * 64 - 1) / (kRLW * 64);  // edge slots per loader lane
  static_assert(RingB <= 160 * 1024, "ring fits the LDS");
  static_assert(RT <= 64 && kRLW * 64 > RT, "a loader lane per row_ptr entry");
  static_assert(SU % 4 == 0, "four rows a staging instruction");
};
using RingG = RingGeom<VG_RING_RT, VG_RING_RT == 64 ? kSU : VG_RING_RT == 48 ? 240 : 192,
                       VG_RING_RT == 32 ? 1024 : kSE, VG_RING_RT == 32 ? 3 : 2>;

struct RingSlot {
  float4* rows;   // [SU][16]
  float* as;      // [SU]
  int* rp;        // [RT + 1]
  float* ad;      // [RT]
  uint16_t* li;   // [SE]
};

template <class G>
__device__ __forceinline__ RingSlot ring_slot(char* base, int s) {
  char* p = base + s * G::SlotB;
  RingSlot r;
  r.rows = reinterpret_cast<float4*>(p);
  r.as = reinterpret_cast<float*>(p + G::RowsB);
  r.rp = reinterpret_cast<int*>(p + G::RowsB + G::SU * 4);
  r.ad = reinterpret_cast<float*>(p + G::RowsB + G::SU * 4 + G::RpB);
  r.li = reinterpret_cast<uint16_t*>(p + G::RowsB + G::SU * 4 + G::RpB + G::RT * 4);
  return r;
}

// wait until *flag >= target (LDS counter, workgroup scope); false on expiry
#ifndef VG_RING_PROF
#define VG_RING_PROF 0  // per-wave clocks into g_ring_prof (tools/ring_probe.py; A/B builds only): 1 waits,
                        // softmax, gather; 2 consumer waits by slice, loader FREE -> loaded clocks and items
#endif
#if VG_RING_PROF
__device__ unsigned long long g_ring_prof[2048 * 16 * 4];
#endif

__device__ __forceinline__ bool ring_wait(int* flag, int target) {
  for (int it = 0; it < kRSpin; ++it) {
    if (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}

// lane k of each 16-lane DPP row to the whole row (row_newbcast, gfx90a+)
template <int K>
__device__ __forceinline__ int row_bcast16(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xF, 0xF, false);
}

#ifndef VG_RING_GDEPTH
#define VG_RING_GDEPTH 8  // source rows read out of LDS before their FMAs (8 or 4)
#endif
#ifndef VG_RING_DMA_ALL
#define VG_RING_DMA_ALL 0  // 1: the plain ring also issues every DMA instruction (A/B knob)
#endif
#ifndef VG_RING_GNP_NOSTORE
#define VG_RING_GNP_NOSTORE 0  // A/B builds only: the loaders form the GraphNorm partials but do not store them
#endif
#ifndef VG_RING_DPPRED
#define VG_RING_DPPRED 1  // the softmax's group reductions by DPP row rotations (0: group_max / group_sum)
#endif
// group_sum<16> / group_max<16> (rowgroup.h: the xor butterfly over offsets
// 8, 4, 2, 1) by DPP row rotations inside each 16-lane row: after the
// offset-8 step every value has period 8, so rotating by 4 pairs the same
// lanes as xor 4 (and then 2, 1) -- the same additions, commutative, so every
// lane ends with the butterfly's value bit for bit, with no LDS round trip.
template <int R>
__device__ __forceinline__ float row_ror16(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x120 + R, 0xF, 0xF, false));
}
__device__ __forceinline__ float ring_sum16(float v) {
  v += row_ror16<8>(v);
  v += row_ror16<4>(v);
  v += row_ror16<2>(v);
  v += row_ror16<1>(v);
  return v;
}
__device__ __forceinline__ float ring_max16(float v) {
  v = fmaxf(v, row_ror16<8>(v));
  v = fmaxf(v, row_ror16<4>(v));
  v = fmaxf(v, row_ror16<2>(v));
  v = fmaxf(v, row_ror16<1>(v));
  return v;
}

// edges 16 Q .. 16 Q + 15 of the group's row: slot / alpha from lane j % 16,
// eight source rows read out of LDS before their FMAs (in edge order)
template <int Q>
__device__ __forceinline__ void ring_gather_q(const RingSlot& R, int sq, float eq, int dreg, int dmax, int l16,
                                              float (&acc)[4]) {
  const int eqb = __float_as_int(eq);
#define VG_RG_LD(K)                                                                       \
  const int s##K = row_bcast16<(K)>(sq);                                                  \
  const float a##K = __int_as_float(row_bcast16<(K)>(eqb));                               \
  const float4 h##K = 16 * Q + (K) < dreg ? R.rows[s##K * 16 + l16] : make_float4(0.f, 0.f, 0.f, 0.f);
#define VG_RG_FMA(K)                                                                      \
  if (16 * Q + (K) < dreg) {                                                              \
    acc[0] = fmaf(a##K, h##K.x, acc[0]);                                                  \
    acc[1] = fmaf(a##K, h##K.y, acc[1]);                                                  \
    acc[2] = fmaf(a##K, h##K.z, acc[2]);                                                  \
    acc[3] = fmaf(a##K, h##K.w, acc[3]);                                                  \
  }
#if VG_RING_GDEPTH == 8
  if (16 * Q < dmax) {
    VG_RG_LD(0) VG_RG_LD(1) VG_RG_LD(2) VG_RG_LD(3) VG_RG_LD(4) VG_RG_LD(5) VG_RG_LD(6) VG_RG_LD(7)
    VG_RG_FMA(0) VG_RG_FMA(1) VG_RG_FMA(2) VG_RG_FMA(3) VG_RG_FMA(4) VG_RG_FMA(5) VG_RG_FMA(6) VG_RG_FMA(7)
  }
  if (16 * Q + 8 < dmax) {
    VG_RG_LD(8) VG_RG_LD(9) VG_RG_LD(10) VG_RG_LD(11) VG_RG_LD(12) VG_RG_LD(13) VG_RG_LD(14) VG_RG_LD(15)
    VG_RG_FMA(8) VG_RG_FMA(9) VG_RG_FMA(10) VG_RG_FMA(11) VG_RG_FMA(12) VG_RG_FMA(13) VG_RG_FMA(14) VG_RG_FMA(15)
  }
#else  // four rows in flight
  if (16 * Q < dmax) { VG_RG_LD(0) VG_RG_LD(1) VG_RG_LD(2) VG_RG_LD(3) VG_RG_FMA(0) VG_RG_FMA(1) VG_RG_FMA(2) VG_RG_FMA(3) }
  if (16 * Q + 4 < dmax) { VG_RG_LD(4) VG_RG_LD(5) VG_RG_LD(6) VG_RG_LD(7) VG_RG_FMA(4) VG_RG_FMA(5) VG_RG_FMA(6) VG_RG_FMA(7) }
  if (16 * Q + 8 < dmax) { VG_RG_LD(8) VG_RG_LD(9) VG_RG_LD(10) VG_RG_LD(11) VG_RG_FMA(8) VG_RG_FMA(9) VG_RG_FMA(10) VG_RG_FMA(11) }
  if (16 * Q + 12 < dmax) { VG_RG_LD(12) VG_RG_LD(13) VG_RG_LD(14) VG_RG_LD(15) VG_RG_FMA(12) VG_RG_FMA(13) VG_RG_FMA(14) VG_RG_FMA(15) }
#endif
#undef VG_RG_LD
#undef VG_RG_FMA
}

// One tile's indices held by a loader lane between its two phases (and
// across the tile's channel slices): edge slots, the a_src rows, the source
// rows of this wave's LDS-DMA instructions.
template <class G>
struct RingIdx {
  int U, e0, ne, rp, lq[G::LiQ], ua[G::AsQ], sr[G::RowI];
  float ad;
};

// A tile's head (distinct-source count, edge range, the lane's row_ptr and
// a_dst entries): loaded one tile before its body, whose addresses need it.
struct RingHead {
  int U, e0, e1, rp;  // e1 - e0 is formed in the body: no use of a load result here
  float ad;
};

template <class G>
__device__ __forceinline__ void ring_load_head(RingHead& x, int t, int N, int wave, int lane,
                                               const int32_t* __restrict__ row_ptr, const float* __restrict__ a_dst,
                                               const int32_t* __restrict__ ucount) {
  const int lt = wave * 64 + lane;
  const int r0 = t * G::RT;
  x.U = ucount[t];
  x.e0 = row_ptr[r0];
  x.e1 = row_ptr[min(r0 + G::RT, N)];
  x.rp = row_ptr[min(r0 + min(lt, G::RT), N)];
  x.ad = a_dst[min(r0 + min(lt, G::RT - 1), N - 1)];
}

// the body: the edges' LDS slots, the a_src rows, this wave's DMA source rows
template <class G>
__device__ __forceinline__ void ring_load_body(RingIdx<G>& x, const RingHead& hd, int t, int wave, int lane,
                                               const int32_t* __restrict__ usrc, const uint16_t* __restrict__ lidx) {
  const int lt = wave * 64 + lane;
  x.U = hd.U;
  x.e0 = hd.e0;
  x.ne = hd.e1 - hd.e0;
  x.rp = hd.rp;
  x.ad = hd.ad;
  if (x.U > 0) {
    const int32_t* us = usrc + (size_t)t * G::SU;
#pragma unroll
    for (int q = 0; q < G::LiQ; ++q) {
      const int e = lt + q * kRLW * 64;
      x.lq[q] = e < x.ne ? static_cast<int>(lidx[x.e0 + e]) : 0;
    }
#pragma unroll
    for (int q = 0; q < G::AsQ; ++q) x.ua[q] = us[min(lt + q * kRLW * 64, x.U - 1)];
#pragma unroll
    for (int q = 0; q < G::RowI; ++q) x.sr[q] = us[min(4 * (wave + q * kRLW) + (lane >> 4), x.U - 1)];
  }
}

// a consumer group's row state, kept across the tile's channel slices
struct RingRow {
  int s_t[4];
  float e_t[4];
  int beg, deg, dreg, r;
  float ad, m, denom;
};

// GNP: the following GraphNorm's column partials (count, mean, M2) per 64-row
// tile and 64-channel slice, in gat_fused.hip's gnp layout with 64-row blocks
// ([tile][2][C][3], slot 0; vg_graphnorm_stats_gnp / _fwd_gnp fold them with
// gnp_rows = 64), formed by the loader waves from the output rows once a
// slot's FREE counter says its consumers are done (ring_gnp_load / _store).
// The loaders run NS items past their last one for the last items' partials.
// One column partial (count, mean, M2) and Chan's merge of two, in a fixed
// order (a then b); an empty side passes the other through
struct RingWel {
  float n, mu, m2;
};
__device__ __forceinline__ RingWel ring_chan(const RingWel& a, const RingWel& b) {
  if (b.n <= 0.f) return a;
  if (a.n <= 0.f) return b;
  const float nt = a.n + b.n, fb = b.n / nt, delta = b.mu - a.mu;
  return {nt, a.mu + delta * fb, a.m2 + b.m2 + delta * delta * a.n * fb};
}
// the lane 16 / 32 apart's partial by gfx950's v_permlane16_swap /
// v_permlane32_swap (VALU, no LDS round trip; with both operands w each lane
// gets the lower and the upper row's value), merged lower row (block) first,
// so both lanes of a pair hold the same
__device__ __forceinline__ RingWel ring_chan_x16(const RingWel& w) {
  const auto n = __builtin_amdgcn_permlane16_swap(__float_as_uint(w.n), __float_as_uint(w.n), false, false);
  const auto m = __builtin_amdgcn_permlane16_swap(__float_as_uint(w.mu), __float_as_uint(w.mu), false, false);
  const auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(w.m2), __float_as_uint(w.m2), false, false);
  return ring_chan({__uint_as_float(n[0]), __uint_as_float(m[0]), __uint_as_float(q[0])},
                   {__uint_as_float(n[1]), __uint_as_float(m[1]), __uint_as_float(q[1])});
}
__device__ __forceinline__ RingWel ring_chan_x32(const RingWel& w) {
  const auto n = __builtin_amdgcn_permlane32_swap(__float_as_uint(w.n), __float_as_uint(w.n), false, false);
  const auto m = __builtin_amdgcn_permlane32_swap(__float_as_uint(w.mu), __float_as_uint(w.mu), false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(w.m2), __float_as_uint(w.m2), false, false);
  return ring_chan({__uint_as_float(n[0]), __uint_as_float(m[0]), __uint_as_float(q[0])},
                   {__uint_as_float(n[1]), __uint_as_float(m[1]), __uint_as_float(q[1])});
}

// The tile partial of item k - NS (tile t, slice sl; its consumers are done:
// FREE) formed by the 4 loader waves from the output rows the consumers
// wrote (L2-resident, just written): wave w takes columns 16 w .. 16 w + 15,
// lane l column 16 w + l % 16 and rows 16 (l / 16) .. + 15 of the tile -- 16
// loads a lane, in flight with the slot's DMA -- then an exact two-pass
// (mean, M2) over its 16 rows, and the four lanes of a column merged by
// permlane swaps with Chan's formula in a fixed tree (deterministic, the same
// in every lane of the column).  The consumers do nothing extra: in their
// epilogue the partials cost the ring ~20 % (their issue slots).
template <class G>
__device__ __forceinline__ void ring_gnp_load(float (&pv)[16], const float* __restrict__ out, int t, int sl, int N,
                                              int C, int wave, int lane) {
  const int c = sl * 64 + 16 * wave + (lane & 15), r = t * G::RT + 16 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 16; ++i) pv[i] = r + i < N ? out[(size_t)(r + i) * C + c] : 0.f;
}

template <class G>
__device__ __forceinline__ void ring_gnp_store(const float (&pv)[16], int t, int sl, int N, int C, int wave,
                                               int lane, float* __restrict__ gnp) {
  static_assert(G::RT == 64 && kRLW == 4, "four loader waves, 16 rows a lane");
  const int r = t * G::RT + 16 * (lane >> 4);
  const int n = max(0, min(16, N - r));
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) sum += i < n ? pv[i] : 0.f;
  const float mu = n > 0 ? sum / static_cast<float>(n) : 0.f;
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float d = i < n ? pv[i] - mu : 0.f;
    m2 = fmaf(d, d, m2);
  }
  const RingWel w = ring_chan_x32(ring_chan_x16({static_cast<float>(n), mu, m2}));
  if (lane < 16 && (!VG_RING_GNP_NOSTORE || N < 0)) {
    float* p = gnp + ((size_t)t * 2 * C + sl * 64 + 16 * wave + lane) * 3;
    p[0] = w.n;
    p[1] = w.mu;
    p[2] = w.m2;
  }
}

template <class G, bool GNP = false>
__global__ void __launch_bounds__(kRNT) k_gat_fwd_ring(
    const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int N, int C,
    const float* __restrict__ h, const float* __restrict__ a_src, const float* __restrict__ a_dst,
    const float* __restrict__ bias, float slope, float* __restrict__ out, float* __restrict__ alpha,
    const int32_t* __restrict__ ucount, const int32_t* __restrict__ usrc, const uint16_t* __restrict__ lidx,
    int tiles, int* __restrict__ err, float* __restrict__ gnp = nullptr) {
  extern __shared__ float4 ring4[];
  char* base = reinterpret_cast<char*>(ring4);
  int* cnt = reinterpret_cast<int*>(base + G::NS * G::SlotB);  // full[NS], free[NS], the next unit
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int slices = C / 64;
  // static, XCD-aware schedule as k_gat_fwd_staged; item k = (tile k / slices, slice k % slices)
  const int per = gridDim.x >> 3, xcd = blockIdx.x & 7, wslot = blockIdx.x >> 3;
  const int tb = static_cast<int>((long long)tiles * xcd / 8);
  const int te = static_cast<int>((long long)tiles * (xcd + 1) / 8);
  const int my_tiles = tb + wslot < te ? (te - tb - wslot + per - 1) / per : 0;
  const int items = my_tiles * slices;
  if (tid < 2 * G::NS + 1) cnt[tid] = 0;
  __syncthreads();
  if (items == 0) return;
#if VG_RING_PROF
  const unsigned long long t_start = __builtin_readcyclecounter();
  unsigned long long waited = 0, t_soft = 0, t_gath = 0;
  auto prof_out = [&]() {
    if (lane == 0) {
      g_ring_prof[(blockIdx.x * 16 + wave) * 4] = waited;
      g_ring_prof[(blockIdx.x * 16 + wave) * 4 + 1] = __builtin_readcyclecounter() - t_start;
      g_ring_prof[(blockIdx.x * 16 + wave) * 4 + 2] = t_soft;
      g_ring_prof[(blockIdx.x * 16 + wave) * 4 + 3] = t_gath;
    }
  };
#define VG_RING_WAIT(flag, target, code)                         \
  do {                                                           \
    const unsigned long long w0_ = __builtin_readcyclecounter(); \
    if (!ring_wait(flag, target)) {                              \
      if (lane == 0) atomicOr(err, code);                        \
      return;                                                    \
    }                                                            \
    waited += __builtin_readcyclecounter() - w0_;                \
  } while (0)
#else
#define VG_RING_WAIT(flag, target, code)  \
  do {                                    \
    if (!ring_wait(flag, target)) {       \
      if (lane == 0) atomicOr(err, code); \
      return;                             \
    }                                     \
  } while (0)
#endif

  if (wave < kRLW) {  // ------------------------------------------------ loaders
    const int lt = wave * 64 + lane;  // 0 .. 255
    // Index loads run two stages ahead of the DMA and are issued before the
    // FREE wait: the head of tile j + 2 and the body of tile j + 1 during the
    // last slice of tile j, tile j's a_src rows before its first slice.  No
    // load of an item depends on another load of the same item, so a refill
    // after FREE is one round trip (the DMA) -- with the head and body loaded
    // in one step, the body's addresses waited for the head and for the DMA
    // issued before it (hipcc waits vmcnt(0) at the first use of a plain
    // load's result while an LDS-DMA is outstanding).
    RingIdx<G> cur, nxt;
    RingHead hn;
    {
      RingHead h0;
      ring_load_head<G>(h0, tb + wslot, N, wave, lane, row_ptr, a_dst, ucount);
      ring_load_body<G>(cur, h0, tb + wslot, wave, lane, usrc, lidx);
      if (my_tiles > 1) ring_load_head<G>(hn, tb + wslot + per, N, wave, lane, row_ptr, a_dst, ucount);
    }
    float av[G::AsQ];
    // GNP: the loaders run NS items past the last one, so the last items'
    // group partials are merged by the same loop body as the others (a
    // separate tail block after the loop made the whole kernel ~45 % slower:
    // its extra live registers and code reshaped the loop)
    const int kend = GNP ? items + G::NS : items;
    for (int k = 0; k < kend; ++k) {
      const bool real = k < items;
      const int s = k % G::NS, gen = k / G::NS, sl = k % slices;
      const int j = k / slices;
      const int t = tb + wslot + j * per;
      const bool pre = real && sl == slices - 1 && j + 1 < my_tiles;
      if (pre) {
        ring_load_body<G>(nxt, hn, t + per, wave, lane, usrc, lidx);
        if (j + 2 < my_tiles) ring_load_head<G>(hn, t + 2 * per, N, wave, lane, row_ptr, a_dst, ucount);
      }
      if (real && sl == 0 && cur.U > 0)
#pragma unroll
        for (int q = 0; q < G::AsQ; ++q) av[q] = a_src[cur.ua[q]];
      if (k >= G::NS) VG_RING_WAIT(&cnt[G::NS + s], G::Groups * gen, 1);
#if VG_RING_PROF == 2
      const unsigned long long f0_ = __builtin_readcyclecounter();
#endif
      RingSlot R = ring_slot<G>(base, s);
      if (real && sl == 0) {  // the tile's metadata: row_ptr, a_dst, edge slots, a_src (consumers keep them per tile)
        if (lt <= G::RT) R.rp[lt] = cur.rp;
        if (lt < G::RT) R.ad[lt] = cur.ad;
        if (cur.U > 0) {
#pragma unroll
          for (int q = 0; q < G::LiQ; ++q) {
            const int e = lt + q * kRLW * 64;
            if (e < cur.ne) R.li[e] = static_cast<uint16_t>(cur.lq[q]);
          }
#pragma unroll
          for (int q = 0; q < G::AsQ; ++q) {
            const int u = lt + q * kRLW * 64;
            if (u < cur.U) R.as[u] = av[q];
          }
        }
      }
      // this slice's rows by LDS-DMA
      // GNP: every instruction issued (the slots past U get copies of the last
      // source row, unread): with a branch per instruction hipcc laid the
      // GNP kernel's DMA blocks out as jump targets and waited vmcnt(0) at
      // each -- 17 of 18 refill instructions serialised, the kernel 1.9x slower
      if (real && cur.U > 0) {
        const int ni = (cur.U + 3) / 4;
#pragma unroll
        for (int q = 0; q < G::RowI; ++q) {
          const int i = wave + q * kRLW;
          if (GNP || VG_RING_DMA_ALL || i < ni) {
            const float* src = h + (size_t)cur.sr[q] * C + sl * 64 + (lane & 15) * 4;
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src),
                                             (__attribute__((address_space(3))) void*)(R.rows + 4 * i * 16), 16, 0, 0);
          }
        }
      }
      // GNP: item k - NS's output rows (its groups are done: FREE above),
      // loaded under this slot's DMA wait, folded once it is handed over
      float pv[16];
      const bool merge = GNP && k >= G::NS;
      const int kp = k - G::NS, tp = tb + wslot + (kp / slices) * per;
      if constexpr (GNP) {
        if (merge) ring_gnp_load<G>(pv, out, tp, kp % slices, N, C, wave, lane);
      }
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#if VG_RING_PROF == 2
      t_soft += __builtin_readcyclecounter() - f0_;  // FREE -> loaded
      t_gath += 1;
#endif
      if (real && lane == 0) __hip_atomic_fetch_add(&cnt[s], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if constexpr (GNP) {
        if (merge) ring_gnp_store<G>(pv, tp, kp % slices, N, C, wave, lane, gnp);
      }
      if (pre) cur = nxt;
    }
#if VG_RING_PROF
    prof_out();
#endif
    return;
  }

  // -------------------------------------------------------------- consumers
  // units (tile j, 4-row group g) are claimed in order from an LDS counter,
  // so the consumer waves share a tile's 16 groups whatever their count; a
  // unit spans the tile's channel slices (its softmax is kept in registers)
  constexpr int L = 16, T = 4;
  const int l16 = lane & 15, gbase = lane & 48;
  const int units = my_tiles * G::Groups;
  for (;;) {
    int u = 0;
    if (lane == 0) u = __hip_atomic_fetch_add(&cnt[2 * G::NS], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    u = __builtin_amdgcn_readfirstlane(u);
    if (u >= units) break;
    const int j = u / G::Groups, grp = u % G::Groups;
    RingRow w;
    for (int sl = 0; sl < slices; ++sl) {
    const int k = j * slices + sl;
    const int s = k % G::NS, gen = k / G::NS;
    const int t = tb + wslot + j * per;
    // the tile's plan entry and the slice's bias in flight under the FULL wait
    const int U = ucount[t];
    const float4 bv = *reinterpret_cast<const float4*>(bias + sl * 64 + l16 * 4);
#if VG_RING_PROF == 2
    const unsigned long long wb_ = waited;
#endif
    VG_RING_WAIT(&cnt[s], kRLW * (gen + 1), 2);
#if VG_RING_PROF == 2
    (sl == 0 ? t_soft : t_gath) += waited - wb_;  // waits by slice (probe builds)
#endif
    RingSlot R = ring_slot<G>(base, s);
    const int r0 = t * G::RT;
    const bool staged = U >= 0;
    const float* hs = h + sl * 64;
    {
#if VG_RING_PROF == 1
      const unsigned long long p0 = __builtin_readcyclecounter();
#endif
      if (sl == 0) {  // the row's softmax, once per tile (its slices reuse it)
        const int e0 = R.rp[0];
        const int ri = 4 * grp + (lane >> 4);  // this group's row in the tile
        w.r = r0 + ri;
        w.beg = R.rp[ri];
        const int end = R.rp[ri + 1];
        w.deg = end - w.beg;
        w.ad = R.ad[ri];
        bool v_t[T];
        float m = -INFINITY;
#pragma unroll
        for (int q = 0; q < T; ++q) {
          const int jj = l16 + q * L;
          v_t[q] = jj < w.deg;
          w.s_t[q] = v_t[q] ? (staged ? static_cast<int>(R.li[w.beg - e0 + jj]) : col[w.beg + jj]) : 0;
        }
#pragma unroll
        for (int q = 0; q < T; ++q) {
          w.e_t[q] = -INFINITY;
          if (v_t[q]) {
            w.e_t[q] = lrelu((staged ? R.as[w.s_t[q]] : a_src[w.s_t[q]]) + w.ad, slope);
            m = fmaxf(m, w.e_t[q]);
          }
        }
        for (int kk = w.beg + l16 + T * L; kk < end; kk += L) m = fmaxf(m, lrelu(a_src[col[kk]] + w.ad, slope));
        m = VG_RING_DPPRED ? ring_max16(m) : group_max<L>(m);
        float ssum = 0.f;
#pragma unroll
        for (int q = 0; q < T; ++q)
          if (v_t[q]) {
            w.e_t[q] = expf(w.e_t[q] - m);
            ssum += w.e_t[q];
          }
        for (int kk = w.beg + l16 + T * L; kk < end; kk += L) ssum += expf(lrelu(a_src[col[kk]] + w.ad, slope) - m);
        const float denom = (VG_RING_DPPRED ? ring_sum16(ssum) : group_sum<L>(ssum)) + kSoftmaxEps;
        const bool live = w.r < N;
#pragma unroll
        for (int q = 0; q < T; ++q)
          if (v_t[q]) {
            w.e_t[q] = w.e_t[q] / denom;
            if (live) alpha[w.beg + l16 + q * L] = w.e_t[q];
          }
        if (live)
          for (int kk = w.beg + l16 + T * L; kk < end; kk += L)
            alpha[kk] = expf(lrelu(a_src[col[kk]] + w.ad, slope) - m) / denom;
        w.m = m;
        w.denom = denom;
        w.dreg = w.deg < T * L ? w.deg : T * L;
      }
#if VG_RING_PROF == 1
      const unsigned long long p1 = __builtin_readcyclecounter();
      t_soft += p1 - p0;
#endif
      // gather-sum over the edges in CSR order
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      const int dreg = w.dreg;
      if (staged) {
        // edge j's (slot, alpha) broadcast from lane j % 16 of the row's
        // 16-lane group by DPP row_newbcast (no LDS round trip), four source
        // rows read out of LDS in flight, the FMAs in edge order
        int dmax = dreg;
        for (int off = 16; off < 64; off <<= 1) dmax = max(dmax, __shfl_xor(dmax, off, 64));
        dmax = __builtin_amdgcn_readfirstlane(dmax);
        ring_gather_q<0>(R, w.s_t[0], w.e_t[0], dreg, dmax, l16, acc);
        ring_gather_q<1>(R, w.s_t[1], w.e_t[1], dreg, dmax, l16, acc);
        ring_gather_q<2>(R, w.s_t[2], w.e_t[2], dreg, dmax, l16, acc);
        ring_gather_q<3>(R, w.s_t[3], w.e_t[3], dreg, dmax, l16, acc);
      }
      for (int j0 = 0; !staged && j0 < dreg; j0 += 4) {
        const int nj = dreg - j0 < 4 ? dreg - j0 : 4;
        float4 hv[4];
        float a[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u < nj) {
            const int jj = j0 + u;
            const int q = jj / L;
            const int sv = q == 0 ? w.s_t[0] : q == 1 ? w.s_t[1] : q == 2 ? w.s_t[2] : w.s_t[3];
            const float avv = q == 0 ? w.e_t[0] : q == 1 ? w.e_t[1] : q == 2 ? w.e_t[2] : w.e_t[3];
            const int sr = __shfl(sv, gbase + (jj & (L - 1)), 64);
            a[u] = __shfl(avv, gbase + (jj & (L - 1)), 64);
            hv[u] = *reinterpret_cast<const float4*>(hs + (size_t)sr * C + l16 * 4);
          }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (u < nj) {
            acc[0] = fmaf(a[u], hv[u].x, acc[0]);
            acc[1] = fmaf(a[u], hv[u].y, acc[1]);
            acc[2] = fmaf(a[u], hv[u].z, acc[2]);
            acc[3] = fmaf(a[u], hv[u].w, acc[3]);
          }
      }
      for (int jj = T * L; jj < w.deg; ++jj) {  // very long rows (global tiles only): alpha recomputed
        const int sj = col[w.beg + jj];
        const float aa = expf(lrelu(a_src[sj] + w.ad, slope) - w.m) / w.denom;
        const float4 v = *reinterpret_cast<const float4*>(hs + (size_t)sj * C + l16 * 4);
        acc[0] = fmaf(aa, v.x, acc[0]);
        acc[1] = fmaf(aa, v.y, acc[1]);
        acc[2] = fmaf(aa, v.z, acc[2]);
        acc[3] = fmaf(aa, v.w, acc[3]);
      }
      const float4 ov = make_float4(acc[0] + bv.x, acc[1] + bv.y, acc[2] + bv.z, acc[3] + bv.w);
      if (w.r < N) *reinterpret_cast<float4*>(out + (size_t)w.r * C + sl * 64 + l16 * 4) = ov;
#if VG_RING_PROF == 1
      t_gath += __builtin_readcyclecounter() - p1;
#endif
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(&cnt[G::NS + s], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
#if VG_RING_PROF
  prof_out();
#endif
#undef VG_RING_WAIT
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

extern "C" int64_t vg_gat_ring_plan_ints(int32_t num_nodes, int32_t num_edges) {
  const int64_t tiles = ((int64_t)num_nodes + RingG::RT - 1) / RingG::RT;
  return tiles + tiles * RingG::SU + ((int64_t)num_edges + 1) / 2;
}

extern "C" int vg_gat_ring_plan(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t E, int32_t* plan,
                                void* stream) {
  if (N <= 0 || E <= 0 || !row_ptr || !col || !plan) return VG_EINVAL;
  const int tiles = (N + RingG::RT - 1) / RingG::RT;
  int32_t* ucount = plan;
  int32_t* usrc = plan + tiles;
  uint16_t* lidx = reinterpret_cast<uint16_t*>(usrc + (size_t)tiles * RingG::SU);
  k_stage_plan<RingG::RT, RingG::SU, RingG::SE><<<tiles, kSNT, 0, static_cast<hipStream_t>(stream)>>>(
      row_ptr, col, N, ucount, usrc, lidx);
  VG_CHECK_LAUNCH();
  return 0;
}

// one workgroup per CU (the ring takes the LDS), a multiple of 8 (the XCD schedule)
static int ring_grid(int tiles) {
  int grid = num_cu();
  const int need = (tiles + 7) / 8 * 8;
  if (grid > need) grid = need;
  return (grid + 7) / 8 * 8;
}

template <bool GNP>
static int ring_launch(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C, const float* h,
                       const float* a_src, const float* a_dst, const float* bias, float slope, float* out,
                       float* alpha, const int32_t* plan, int32_t* err, float* gnp, void* stream) {
  if (N <= 0 || (C != 64 && C != 128) || !row_ptr || !col || !h || !a_src || !a_dst || !bias || !out || !alpha ||
      !plan || !err || (reinterpret_cast<uintptr_t>(h) & 15) || (reinterpret_cast<uintptr_t>(out) & 15) ||
      (reinterpret_cast<uintptr_t>(bias) & 15) || (GNP && (!gnp || (reinterpret_cast<uintptr_t>(gnp) & 15))))
    return VG_EINVAL;
  const int tiles = (N + RingG::RT - 1) / RingG::RT;
  const int32_t* ucount = plan;
  const int32_t* usrc = plan + tiles;
  const uint16_t* lidx = reinterpret_cast<const uint16_t*>(usrc + (size_t)tiles * RingG::SU);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_gat_fwd_ring<RingG, GNP>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, RingG::RingB);
    attr = true;
  }
  const int grid = ring_grid(tiles);
  k_gat_fwd_ring<RingG, GNP><<<grid, kRNT, RingG::RingB, static_cast<hipStream_t>(stream)>>>(
      row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, ucount, usrc, lidx, tiles, err, gnp);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gat_aggregate_fwd_ring(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                                         const float* h, const float* a_src, const float* a_dst, const float* bias,
                                         float slope, float* out, float* alpha, const int32_t* plan, int32_t* err,
                                         void* stream) {
  return ring_launch<false>(row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, plan, err, nullptr,
                            stream);
}

extern "C" int32_t vg_gat_ring_tile_rows(void) { return RingG::RT; }

extern "C" int64_t vg_gat_ring_gnp_floats(int32_t N, int32_t C) {
  if (N <= 0 || (C != 64 && C != 128)) return 0;
  const int64_t tiles = ((int64_t)N + RingG::RT - 1) / RingG::RT;
  return tiles * 2 * C * 3;  // the tile partials [tiles][2][C][3]
}

extern "C" int vg_gat_aggregate_fwd_ring_gnp(const int32_t* row_ptr, const int32_t* col, int32_t N, int32_t C,
                                             const float* h, const float* a_src, const float* a_dst,
                                             const float* bias, float slope, float* out, float* alpha,
                                             const int32_t* plan, int32_t seg_rows, float* gnp, int32_t* err,
                                             void* stream) {
  // one segment, or segments of whole tiles: a segment's partials are its own tiles'
  if (seg_rows <= 0 || N % seg_rows != 0 || (seg_rows != N && seg_rows % RingG::RT != 0)) return VG_EINVAL;
  return ring_launch<true>(row_ptr, col, N, C, h, a_src, a_dst, bias, slope, out, alpha, plan, err, gnp, stream);
}

#if VG_RING_PROF
// the per-wave (waited, total) clocks of the last ring launch (profiling builds only)
extern "C" int vg_ring_prof_read(unsigned long long* host, int n) {
  return static_cast<int>(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ring_prof), sizeof(unsigned long long) * n));
}
#endif

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
  k_stage_plan<kSRT, kSU, kSE><<<tiles, kSNT, 0, static_cast<hipStream_t>(stream)>>>(row_ptr, col, N, ucount, usrc,
                                                                                     lidx);
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
