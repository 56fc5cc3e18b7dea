// Host-side plumbing shared by the iterations issued from C++
// (critic_engine.hip: vg_critic_loss_and_grad; gen_engine.hip:
// vg_gen_loss_and_grad): a bump allocator over the caller's arena with a
// dry (sizing) mode, the dense products in the model's precision, and the
// FoldCollector of vgan/_lib.py (grouped weight-gradient products, then the
// parameter-gradient folds merged and batched exactly as the Python collector
// merges them).  Host code only: every launch goes through the library's own
// extern "C" entry points.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <utility>
#include <vector>

#include "../../include/vgan.h"

namespace vg_engine {

constexpr int kActNone = 0, kActRelu = 1, kActMask = 3, kActAdd = 4;

struct Ctx {
  bool dry;  // size the arena only: no launches, no plans
  int bf16;
  void* stream;
  float* base;
  int64_t cap, off;

  // 256-byte aligned temporaries (the quad / float4 kernel forms need 16 B)
  float* take(int64_t floats) {
    const int64_t at = off;
    off += (std::max<int64_t>(floats, 1) + 63) / 64 * 64;
    return dry ? nullptr : base + at;
  }

  int gemm(const float* A, int lda, const float* B, int ldb, int bt, float* C, int ldc, int n, int m, int k,
           const float* bias = nullptr, int act = kActNone, const float* aux = nullptr, int ldaux = 0) const {
    if (dry) return 0;
    return bf16 ? vg_gemm_bf16(A, lda, B, ldb, bt, bias, act, aux, ldaux, C, ldc, n, m, k, stream)
                : vg_gemm(A, lda, B, ldb, bt, bias, act, aux, ldaux, C, ldc, n, m, k, stream);
  }

  // vg_linear_chain: 1 launched, 0 no kernel for this width chain (the caller
  // runs its per-layer GEMMs), < 0 error
  int chain(const float* x, int ldx, int rows, const std::vector<int32_t>& widths,
            const std::vector<vg_chain_layer>& layers) const {
    if (dry) return 1;
    const int rc = bf16 ? vg_linear_chain_bf16(x, ldx, rows, widths.data(), (int32_t)layers.size(), layers.data(), stream)
                        : vg_linear_chain(x, ldx, rows, widths.data(), (int32_t)layers.size(), layers.data(), stream);
    if (rc == VG_EINVAL) return 0;
    return rc == 0 ? 1 : (rc > 0 ? -rc : rc);
  }
};

#ifndef VG_CRITIC_FOLD_SPLIT
#define VG_CRITIC_FOLD_SPLIT 1  // long folds in two levels (vg_fold_batch_split); 0: vg_fold_batch (A/B)
#endif

struct Folds {
  std::vector<vg_fold> folds;
  std::vector<vg_tn> prods;  // planned, not yet launched
  float* ws = nullptr;       // the split folds' chunk sums (arena)
  int64_t ws_floats = 0;

  void add(const vg_fold* f, int n) { folds.insert(folds.end(), f, f + n); }

  int tn(const Ctx& cx, const float* A, int lda, const float* B, int ldb, int N, int M, int K, float* C, int ldc,
         float* db, int db_rows, float* w) {
    if (cx.dry) return 0;
    vg_tn p;
    vg_fold f[2];
    int32_t n = 0;
    const int rc = cx.bf16 ? vg_gemm_tn_plan_bf16(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, 1, w, &p, f, &n)
                           : vg_gemm_tn_plan(A, lda, B, ldb, N, M, K, C, ldc, db, db_rows, 1, w, &p, f, &n);
    if (rc) return rc;
    prods.push_back(p);
    add(f, n);
    return 0;
  }

  int launch_products(void* stream) {
    for (int bf = 0; bf < 2; ++bf) {
      std::vector<vg_tn> sel;
      for (const vg_tn& p : prods)
        if ((p.bf16 != 0) == (bf != 0)) sel.push_back(p);
      for (size_t i = 0; i < sel.size(); i += VG_TN_GROUP_MAX) {
        const int n = (int)std::min<size_t>(VG_TN_GROUP_MAX, sel.size() - i);
        const int rc = vg_gemm_tn_group(sel.data() + i, n, stream);
        if (rc) return rc;
      }
    }
    prods.clear();
    return 0;
  }

  int flush(Ctx& cx) {
    if (cx.dry) return 0;
    int rc = launch_products(cx.stream);  // the products first: their partials feed the folds
    if (rc) return rc;
    // folds into one destination merge into a two-source fold (applied in
    // call order); one that cannot merge starts a new batch, so the two never race
    std::vector<std::vector<vg_fold>> batches;
    std::vector<vg_fold> cur;
    std::vector<std::pair<float*, int>> where;
    auto find = [&](float* out) -> int {
      for (auto& w : where)
        if (w.first == out) return w.second;
      return -1;
    };
    for (const vg_fold& f : folds) {
      const int j = find(f.out);
      if (j >= 0) {
        vg_fold& g = cur[j];
        if (g.nsrc == 1 && f.nsrc == 1 && f.accumulate && g.width == f.width && g.k == f.k && g.ldo == f.ldo) {
          g.src[1] = f.src[0];
          g.nsrc = 2;
          continue;
        }
        batches.push_back(cur);
        cur.clear();
        where.clear();
      }
      if ((int)cur.size() == VG_FOLD_MAX) {
        batches.push_back(cur);
        cur.clear();
        where.clear();
      }
      where.emplace_back(f.out, (int)cur.size());
      cur.push_back(f);
    }
    if (!cur.empty()) batches.push_back(cur);
    for (auto& b : batches) {
      const int rc = VG_CRITIC_FOLD_SPLIT ? vg_fold_batch_split(b.data(), (int32_t)b.size(), ws, ws_floats, cx.stream)
                                          : vg_fold_batch(b.data(), (int32_t)b.size(), cx.stream);
      if (rc) return rc;
    }
    folds.clear();
    return 0;
  }
};

}  // namespace vg_engine

#define VG_TRY(expr)          \
  do {                        \
    const int _rc = (expr);   \
    if (_rc) return _rc;      \
  } while (0)
#define VG_RUN(expr)                  \
  do {                                \
    if (!cx.dry) {                    \
      const int _rc = (expr);         \
      if (_rc) return _rc;            \
    }                                 \
  } while (0)
