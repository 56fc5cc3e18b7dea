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

// Counter-based Philox4x32-10 (Salmon et al., SC'11): stateless, so a kernel
// replayed from a hipGraph draws fresh numbers whenever the counter it reads
// from device memory has advanced.
__device__ __forceinline__ uint4 vg_philox(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// Dropout multiplier of element t: Bernoulli(1 - p) / (1 - p) from lane t % 4
// of the Philox block at counter (t / 4, salt, iteration) under key = seed --
// one Philox call serves four consecutive elements (vg_keep4, the quad
// elementwise kernels); vg_keep draws the same value for a single element.
__device__ __forceinline__ float vg_keep_of(uint32_t r, float p) {
  const float u = static_cast<float>(r >> 8) * (1.0f / 16777216.0f);
  return u < 1.f - p ? 1.f / (1.f - p) : 0.f;
}

__device__ __forceinline__ uint4 vg_keep_block(long long q, uint32_t salt, long long iter, uint64_t seed) {
  return vg_philox(make_uint4(static_cast<uint32_t>(q), static_cast<uint32_t>(q >> 32), salt,
                              static_cast<uint32_t>(iter)),
                   make_uint2(static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32)));
}

__device__ __forceinline__ float4 vg_keep4_raw(long long q, uint32_t salt, long long iter, uint64_t seed,
                                               float p) {
  const uint4 r = vg_keep_block(q, salt, iter, seed);
  return make_float4(vg_keep_of(r.x, p), vg_keep_of(r.y, p), vg_keep_of(r.z, p), vg_keep_of(r.w, p));
}

__device__ __forceinline__ float vg_keep(long long t, uint32_t salt, long long iter, uint64_t seed,
                                         float p) {
  const uint4 r = vg_keep_block(t >> 2, salt, iter, seed);
  const int l = static_cast<int>(t & 3);
  return vg_keep_of(l == 0 ? r.x : l == 1 ? r.y : l == 2 ? r.z : r.w, p);
}

// "Last block folds": every block calls this after writing its partials; it
// returns true in exactly one block -- the last to arrive -- which then sees
// all partials and folds them in a fixed order, so the result is
// deterministic and no separate fold launch is needed.  Hand-off in the
// single-lane form of MI355X_MICROARCH.md (inter-workgroup visibility):
// every wave waits for its stores, a barrier, then ONE lane releases at agent
// scope, waits, and adds to the counter; the block whose add came last
// acquires at agent scope, waits, and the barrier releases its waves to read.
// `counter` is a caller-owned int32 that is 0 on entry and reset to 0 by the
// last block (launches that share a counter must be stream-ordered).
// vg_last_arrival: the same over a group of `arrivals` blocks sharing a
// counter (called uniformly by every thread of each block).
__device__ __forceinline__ bool vg_last_arrival(int* counter, int arrivals) {
  __shared__ int last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int prev = __hip_atomic_fetch_add(counter, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev == arrivals - 1;
    if (last) {
      __hip_atomic_store(counter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
  return last != 0;
}

// the whole grid arrives on one counter
__device__ __forceinline__ bool vg_last_block(int* counter) {
  return vg_last_arrival(counter, static_cast<int>(gridDim.x * gridDim.y * gridDim.z));
}

static inline int vg_blocks(long long work, int per_block) {
  long long b = (work + per_block - 1) / per_block;
  return b < 1 ? 1 : static_cast<int>(b);
}
