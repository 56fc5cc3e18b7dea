// Destination CSR (+ self loops) and source CSC, built once per mini-batch.
//
// torch-geometric rebuilds the self-loop edge list inside every GATConv call
// (remove_self_loops -> add_self_loops, a boolean mask with a host sync and two
// [2, E'] allocations per layer; 20 layers per G+D forward pair).  Here the
// batch's edge_index is turned into the two index structures once and every
// layer of every G/D pass reuses them.
//
// Ordering is deterministic: inside a row the slots are sorted by original edge
// id (the order torch-geometric's scatter visits them), self loop last.
#include "common.h"

namespace {

__global__ void k_degrees(const int64_t* __restrict__ ei, int64_t E, int32_t N,
                          int32_t* __restrict__ indeg, int32_t* __restrict__ outdeg,
                          int32_t* __restrict__ status) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = ei[e], d = ei[E + e];
    if (s < 0 || s >= N || d < 0 || d >= N) {
      status[1] = 1;
      continue;
    }
    if (s == d) continue;  // remove_self_loops
    atomicAdd(&indeg[d], 1);
    atomicAdd(&outdeg[s], 1);
  }
}

// Exclusive scan of (deg[i] + 1) for two arrays at once (blockIdx.x selects),
// one 1024-thread block each: ptr[0] = 0, ptr[i+1] = ptr[i] + deg[i] + 1.
__global__ void __launch_bounds__(1024) k_scan_plus_one(const int32_t* __restrict__ deg_a,
                                                        const int32_t* __restrict__ deg_b,
                                                        int32_t N, int32_t* __restrict__ ptr_a,
                                                        int32_t* __restrict__ ptr_b,
                                                        int32_t* __restrict__ status) {
  const int32_t* deg = blockIdx.x == 0 ? deg_a : deg_b;
  int32_t* ptr = blockIdx.x == 0 ? ptr_a : ptr_b;
  __shared__ int32_t warp_tot[16];
  __shared__ int32_t carry;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) {
    carry = 0;
    ptr[0] = 0;
  }
  __syncthreads();
  for (int32_t base = 0; base < N; base += 1024) {
    const int32_t i = base + t;
    int32_t v = (i < N) ? deg[i] + 1 : 0;
    // inclusive wave scan
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int32_t u = __shfl_up(v, off, 64);
      if (lane >= off) v += u;
    }
    if (lane == 63) warp_tot[w] = v;
    __syncthreads();
    if (w == 0) {
      int32_t s = lane < 16 ? warp_tot[lane] : 0;
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) {
        const int32_t u = __shfl_up(s, off, 64);
        if (lane >= off) s += u;
      }
      if (lane < 16) warp_tot[lane] = s;  // inclusive prefix of wave totals
    }
    __syncthreads();
    const int32_t prefix = carry + (w > 0 ? warp_tot[w - 1] : 0);
    if (i < N) ptr[i + 1] = prefix + v;
    __syncthreads();
    if (t == 1023) carry = prefix + v;
    __syncthreads();
  }
  if (blockIdx.x == 0 && t == 0) status[0] = carry;
}

// Scatter edge ids into their destination rows (arbitrary order inside a row,
// fixed afterwards by k_sort_rows).  The last slot of each row is the self loop.
__global__ void k_fill_rows(const int64_t* __restrict__ ei, int64_t E, int32_t N,
                            const int32_t* __restrict__ row_ptr, int32_t* __restrict__ cursor,
                            int32_t* __restrict__ slot_eid) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < E + N;
       e += (int64_t)gridDim.x * blockDim.x) {
    if (e < E) {
      const int64_t s = ei[e], d = ei[E + e];
      if (s < 0 || s >= N || d < 0 || d >= N || s == d) continue;
      const int32_t pos = row_ptr[d] + atomicAdd(&cursor[d], 1);
      slot_eid[pos] = static_cast<int32_t>(e);
    } else {
      const int32_t i = static_cast<int32_t>(e - E);
      slot_eid[row_ptr[i + 1] - 1] = -1;  // self loop marker (sorts last below)
    }
  }
}

// One thread per row: insertion-sort the row's edge ids, then emit sources.
__global__ void k_sort_rows(const int64_t* __restrict__ ei, int32_t N,
                            const int32_t* __restrict__ row_ptr, int32_t* __restrict__ slot_eid,
                            int32_t* __restrict__ col) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const int32_t beg = row_ptr[i], end = row_ptr[i + 1] - 1;  // exclude self loop
  for (int32_t a = beg + 1; a < end; ++a) {
    const int32_t key = slot_eid[a];
    int32_t b = a - 1;
    while (b >= beg && slot_eid[b] > key) {
      slot_eid[b + 1] = slot_eid[b];
      --b;
    }
    slot_eid[b + 1] = key;
  }
  for (int32_t k = beg; k < end; ++k) col[k] = static_cast<int32_t>(ei[slot_eid[k]]);
  col[end] = i;
}

// Transpose: thread per destination row pushes its slots into source buckets.
__global__ void k_fill_csc(int32_t N, const int32_t* __restrict__ row_ptr,
                           const int32_t* __restrict__ col, const int32_t* __restrict__ csc_ptr,
                           int32_t* __restrict__ cursor, int32_t* __restrict__ csc_slot) {
  const int32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  for (int32_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
    const int32_t j = col[k];
    const int32_t pos = csc_ptr[j] + atomicAdd(&cursor[j], 1);
    csc_slot[pos] = k;
  }
}

// Sort each source bucket by slot (= by destination row, then edge order) and
// record the destination of every entry.
__global__ void k_sort_csc(int32_t N, const int32_t* __restrict__ row_ptr,
                           const int32_t* __restrict__ csc_ptr, int32_t* __restrict__ csc_slot,
                           int32_t* __restrict__ csc_dst) {
  const int32_t j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= N) return;
  const int32_t beg = csc_ptr[j], end = csc_ptr[j + 1];
  for (int32_t a = beg + 1; a < end; ++a) {
    const int32_t key = csc_slot[a];
    int32_t b = a - 1;
    while (b >= beg && csc_slot[b] > key) {
      csc_slot[b + 1] = csc_slot[b];
      --b;
    }
    csc_slot[b + 1] = key;
  }
  for (int32_t a = beg; a < end; ++a) {
    // destination row of slot k: binary search in row_ptr
    const int32_t k = csc_slot[a];
    int32_t lo = 0, hi = N - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if (row_ptr[mid] <= k) lo = mid; else hi = mid - 1;
    }
    csc_dst[a] = lo;
  }
}

}  // namespace

extern "C" int64_t vg_csr_ws_ints(int64_t num_edges, int32_t num_nodes) {
  return 4 * (int64_t)num_nodes + num_edges + num_nodes;
}

extern "C" int vg_csr_build(const int64_t* edge_index, int64_t num_edges, int32_t num_nodes,
                            int32_t* row_ptr, int32_t* col, int32_t* csc_ptr, int32_t* csc_slot,
                            int32_t* csc_dst, int32_t* workspace, int32_t* status, void* stream) {
  if (num_nodes <= 0 || num_edges < 0 || !row_ptr || !col || !csc_ptr || !csc_slot || !csc_dst ||
      !workspace || !status || (num_edges > 0 && !edge_index))
    return VG_EINVAL;
  if (num_edges + num_nodes > INT32_MAX) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int32_t N = num_nodes;
  int32_t* indeg = workspace;
  int32_t* outdeg = workspace + N;
  int32_t* cur_a = workspace + 2 * (int64_t)N;
  int32_t* cur_b = workspace + 3 * (int64_t)N;
  int32_t* slot_eid = workspace + 4 * (int64_t)N;
  (void)hipMemsetAsync(workspace, 0, sizeof(int32_t) * 4 * (size_t)N, s);
  (void)hipMemsetAsync(status, 0, sizeof(int32_t) * 2, s);
  const int bs = 256;
  const int eb = vg_blocks(num_edges + N, bs) > 4096 ? 4096 : vg_blocks(num_edges + N, bs);
  if (num_edges > 0) k_degrees<<<eb, bs, 0, s>>>(edge_index, num_edges, N, indeg, outdeg, status);
  k_scan_plus_one<<<2, 1024, 0, s>>>(indeg, outdeg, N, row_ptr, csc_ptr, status);
  k_fill_rows<<<eb, bs, 0, s>>>(edge_index, num_edges, N, row_ptr, cur_a, slot_eid);
  k_sort_rows<<<vg_blocks(N, bs), bs, 0, s>>>(edge_index, N, row_ptr, slot_eid, col);
  k_fill_csc<<<vg_blocks(N, bs), bs, 0, s>>>(N, row_ptr, col, csc_ptr, cur_b, csc_slot);
  k_sort_csc<<<vg_blocks(N, bs), bs, 0, s>>>(N, row_ptr, csc_ptr, csc_slot, csc_dst);
  VG_CHECK_LAUNCH();
  return 0;
}
