// Shared helpers for the vgan HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/vgan.h"

#define VG_WAVE 64

#define VG_CHECK_LAUNCH()                                   \
  do {                                                      \
    hipError_t _e = hipGetLastError();                      \
    if (_e != hipSuccess) return static_cast<int>(_e);      \
  } while (0)

// Group-of-L-lanes reductions (L a power of two <= 64).  Lanes of one group are
// contiguous inside the wave, so xor-shuffles with offsets < L stay in-group.
template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, VG_WAVE);
  return v;
}

template <int L>
__device__ __forceinline__ float group_max(float v) {
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, VG_WAVE));
  return v;
}

__device__ __forceinline__ float lrelu(float v, float slope) { return v > 0.f ? v : v * slope; }

// XCD-aware block remap (guide T1): the dispatcher deals blocks round-robin over
// the 8 XCDs, so hardware block b runs on XCD b % 8.  Give every XCD one
// contiguous range of logical blocks so that a destination row and its lattice
// neighbours (rows i +- 1, i +- X, i +- XY) are read through the same L2.
// Bijective for any grid size; placement only changes speed, never results.
__device__ __forceinline__ int xcd_remap(int b, int nblocks) {
  const int xcd = b & 7;
  const int slot = b >> 3;
  const int base = nblocks >> 3;  // blocks every XCD gets
  const int rem = nblocks & 7;    // the first `rem` XCDs get one more
  const int start = xcd * base + (xcd < rem ? xcd : rem);
  return start + slot;
}

static inline int vg_blocks(long long work, int per_block) {
  long long b = (work + per_block - 1) / per_block;
  return b < 1 ? 1 : static_cast<int>(b);
}
