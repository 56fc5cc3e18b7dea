// One generator iteration issued from C++: vg_gen_loss_and_grad (include/vgan.h).
//
// A restatement of vgan/genstep.py GeneratorEngine.loss_and_grad in its
// default configuration -- the generator half of trainer.py:483-491: G(z) ->
// Gumbel straight-through labels -> D(label_hard) in train mode -> the loss of
// trainer.py:334-385 -> the backward into G's parameters (D's input VJP only,
// the Gumbel backward, G's backward with every fold and weight-gradient
// product deferred to one grouped flush).  The same entry points run in the
// same order with the same arguments, the device-RNG draws under the same
// salts, so loss, labels and gradients are bit-identical to the Python
// engine's (tests/test_gen_engine_gpu.py); the host pays ~1-2 us per launch
// instead of ~10 (a fresh batch's generator iteration runs eagerly,
// Trainer.step_fresh).  The two kernels below are the copies torch.cat and
// Tensor.add_ make in the Python engine.
#include "common.h"
#include "engine.h"

namespace {

using vg_engine::Ctx;
using vg_engine::Folds;
using vg_engine::kActAdd;
using vg_engine::kActMask;
using vg_engine::kActNone;
using vg_engine::kActRelu;
constexpr int64_t kFoldWsFloats = 1 << 20;  // the split folds' chunk sums (the Python collector sizes them exactly)
constexpr int kCatMax = 6;

struct CatSrc {
  const float* p;
  int w, col0;
};
struct CatSrcs {
  CatSrc s[kCatMax];
  int n;
};

// out [rows][total] = the column blocks of srcs side by side (torch.cat(dim=-1))
__global__ void k_cat_cols(CatSrcs src, int rows, int total, float* __restrict__ out) {
  const long long all = (long long)rows * total;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < all; i += (long long)gridDim.x * blockDim.x) {
    const int r = static_cast<int>(i / total), c = static_cast<int>(i - (long long)r * total);
    int j = 0;
#pragma unroll
    for (int q = 1; q < kCatMax; ++q)
      if (q < src.n && c >= src.s[q].col0) j = q;
    out[i] = src.s[j].p[(long long)r * src.s[j].w + (c - src.s[j].col0)];
  }
}

__global__ void k_add_to(float* __restrict__ a, const float* __restrict__ b, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    a[i] = a[i] + b[i];
}

int cat_cols(const Ctx& cx, std::initializer_list<std::pair<const float*, int>> parts, int rows, float* out,
             int total) {
  if (cx.dry) return 0;
  CatSrcs s{};
  int col = 0;
  for (const auto& p : parts) {
    if (s.n == kCatMax || !p.first) return VG_EINVAL;
    s.s[s.n++] = CatSrc{p.first, p.second, col};
    col += p.second;
  }
  if (col != total) return VG_EINVAL;
  const long long all = (long long)rows * total;
  const int blocks = static_cast<int>(std::min<long long>((all + 255) / 256, 4096));
  k_cat_cols<<<blocks, 256, 0, static_cast<hipStream_t>(cx.stream)>>>(s, rows, total, out);
  VG_CHECK_LAUNCH();
  return 0;
}

// _ln_fwd's saved state
struct LnS {
  const vg_gen_ln_layer* L;
  const float* x;
  int ldx;
  float *h, *y, *mean, *rstd;
};

// _gat_fwd's saved state
struct GatS {
  const vg_critic_block* B;
  const float* X;
  int xw, c;
  float *H, *O, *alpha, *a_s, *a_d, *Y, *stats, *keep;
};

int run(Ctx& cx, const vg_gen_model* md, const vg_gen_batch* bt, float* out, float* hard) {
  const int n = bt->n, K = bt->classes, E = bt->g.num_edges;
  const vg_csr_ref& g1 = bt->g;
  Folds folds;
  folds.ws = cx.take(kFoldWsFloats);
  folds.ws_floats = kFoldWsFloats;

  auto ln_fwd = [&](const float* x, int ldx, const vg_gen_ln_layer& L, LnS* S) -> int {
    const int m = L.out, k = L.in;
    if (k != ldx) return VG_EINVAL;
    *S = LnS{&L, x, ldx, cx.take((int64_t)n * m), cx.take((int64_t)n * m), cx.take(n), cx.take(n)};
    if (cx.dry) return 0;
    return cx.bf16 ? vg_gemm_ln_act_bf16(x, ldx, L.weight, n, m, k, L.bias, L.ln_weight, L.ln_bias, L.ln_eps, L.slope,
                                         S->h, S->y, S->mean, S->rstd, cx.stream)
                   : vg_gemm_ln_act(x, ldx, L.weight, n, m, k, L.bias, L.ln_weight, L.ln_bias, L.ln_eps, L.slope, S->h,
                                    S->y, S->mean, S->rstd, cx.stream);
  };
  auto tn = [&](const float* A, int lda, const float* B, int ldb, int N, int M, int Kk, float* C, int ldc,
                float* db) -> int {
    float* ws = cx.take(std::max<int64_t>(1, vg_gemm_tn_ws_floats(N, M, Kk)));
    return folds.tn(cx, A, lda, B, ldb, N, M, Kk, C, ldc, db, N, ws);
  };
  // g_h = d(pre-norm) from g_y; gamma / beta and weight / bias gradients deferred
  auto ln_bwd = [&](const LnS& S, const float* g_y, float** g_h_out) -> int {
    const vg_gen_ln_layer& L = *S.L;
    const int m = L.out, k = L.in;
    float* g_h = cx.take((int64_t)n * m);
    float* ws = cx.take(vg_ln_act_bwd_ws_floats(m));
    *g_h_out = g_h;
    if (!cx.dry) {
      vg_fold f[3];
      int32_t nf = 0;
      VG_TRY(vg_ln_act_bwd_deferred(S.h, n, m, L.ln_weight, L.ln_bias, L.slope, S.mean, S.rstd, g_y, g_h,
                                    L.g_ln_weight, L.g_ln_bias, 1, ws, f, &nf, cx.stream));
      folds.add(f, nf);
    }
    return tn(g_h, m, S.x, S.ldx, n, m, k, L.g_weight, k, L.g_bias);
  };
  // GATConv -> GraphNorm -> ReLU -> Dropout with the mask drawn in-kernel and stored
  auto gat_fwd = [&](const float* x, int xw, const vg_critic_block& B, float p_drop, uint32_t salt, GatS* S) -> int {
    const int c = B.out;
    if (B.in != xw) return VG_EINVAL;
    const int g = vg_gat_gnp_rows(n, c);
    if (g <= 0 || bt->seg_rows < g || n % bt->seg_rows) return VG_EINVAL;  // (the Python engine's unfused path)
    GatS s{&B, x, xw, c};
    s.H = cx.take((int64_t)n * c);
    s.a_s = cx.take(n);
    s.a_d = cx.take(n);
    s.O = cx.take((int64_t)n * c);
    s.alpha = cx.take(E);
    float* gnp = cx.take(vg_gat_gnp_floats(n, c));
    s.Y = cx.take((int64_t)n * c);
    s.stats = cx.take(2LL * c);
    s.keep = cx.take((int64_t)n * c);
    *S = s;
    VG_RUN(cx.bf16 ? vg_gat_lin_att_bf16(x, xw, B.lin_weight, n, xw, c, B.att_src, B.att_dst, s.H, s.a_s, s.a_d,
                                         cx.stream)
                   : vg_gat_lin_att(x, xw, B.lin_weight, n, xw, c, B.att_src, B.att_dst, s.H, s.a_s, s.a_d, cx.stream));
    VG_RUN(vg_gat_aggregate_fwd_gnp(g1.row_ptr, g1.col, g1.ell, g1.ell ? g1.ell_width : 0, n, c, s.H, s.a_s, s.a_d,
                                    B.bias, B.slope, s.O, s.alpha, bt->seg_rows, gnp, cx.stream));
    VG_RUN(vg_graphnorm_fwd_gnp(s.O, 1, n, c, B.gn_weight, B.gn_bias, B.gn_mean_scale, nullptr, p_drop, bt->seed,
                                bt->iter, salt, B.gn_eps, s.Y, s.keep, s.stats, gnp, g, cx.stream));
    return 0;
  };
  // o [n, m] = A Wt, the output gradient of S's GraphNorm; that backward's
  // column partials from the GEMM epilogue (*tp; NULL when m % 4 != 0)
  auto gemm_dy = [&](const float* A, int lda, const float* Wt, int ldw, float* o, int m, int k, const GatS& S,
                     float** tp) -> int {
    if (m % 4 != 0) {
      *tp = nullptr;
      return cx.gemm(A, lda, Wt, ldw, 0, o, m, n, m, k);
    }
    const vg_critic_block& N = *S.B;
    float* t = cx.take(vg_gemm_gn_tpart_floats(n, m));
    *tp = t;
    if (cx.dry) return 0;
    return cx.bf16 ? vg_gemm_gn_bwd_bf16(A, lda, Wt, ldw, n, m, k, o, m, S.O, S.keep, n, N.gn_weight, N.gn_bias,
                                         N.gn_mean_scale, N.gn_eps, S.stats, t, cx.stream)
                   : vg_gemm_gn_bwd(A, lda, Wt, ldw, n, m, k, o, m, S.O, S.keep, n, N.gn_weight, N.gn_bias,
                                    N.gn_mean_scale, N.gn_eps, S.stats, t, cx.stream);
  };
  // GraphNorm(+ReLU+Dropout) and GATConv backward of one block: dH; with
  // pgrads the block's GraphNorm and attention / bias gradients (deferred)
  auto gat_bwd = [&](const GatS& S, const float* g_y, const float* tp, bool pgrads, float** dH_out) -> int {
    const vg_critic_block& B = *S.B;
    const int c = S.c;
    float* dO = cx.take((int64_t)n * c);
    float* dH = cx.take((int64_t)n * c);
    float* ws = cx.take(vg_gat_bwd_ws_floats(n, E, c));
    float* gws = cx.take(vg_graphnorm_seg_ws_floats(1, n, c));
    *dH_out = dH;
    if (cx.dry) return 0;
    float* gw = pgrads ? B.g_gn_weight : nullptr;
    float* gb = pgrads ? B.g_gn_bias : nullptr;
    float* gm = pgrads ? B.g_gn_mean_scale : nullptr;
    if (tp)
      VG_TRY(vg_graphnorm_bwd_seg_tiles(S.O, 1, n, c, B.gn_weight, B.gn_bias, B.gn_mean_scale, S.keep, B.gn_eps, S.stats,
                                        g_y, tp, nullptr, gw, gb, gm, pgrads ? 1 : 0, nullptr, 0, gws, cx.stream));
    else
      VG_TRY(vg_graphnorm_bwd_seg(S.O, 1, n, c, B.gn_weight, B.gn_bias, B.gn_mean_scale, S.keep, B.gn_eps, S.stats, g_y,
                                  nullptr, gw, gb, gm, pgrads ? 1 : 0, nullptr, 0, gws, bt->sync, cx.stream));
    const vg_gn_bwd_in gn{S.O,        S.keep,   g_y, nullptr, B.gn_weight, B.gn_bias, B.gn_mean_scale, S.stats,
                          gws + vg_graphnorm_bwd_sums_offset(1, c), B.gn_eps, 1, n, 0};
    if (pgrads) {
      vg_fold f[3];
      int32_t nf = 0;
      VG_TRY(vg_gat_bwd_gn(g1.row_ptr, g1.col, g1.csc_ptr, g1.csc_slot, g1.csc_dst, n, E, c, S.H, B.att_src, B.att_dst,
                           S.a_s, S.a_d, S.alpha, &gn, dO, B.slope, dH, B.g_att_src, B.g_att_dst, B.g_bias, 1, nullptr,
                           0, ws, f, &nf, cx.stream));
      folds.add(f, nf);
      return 0;
    }
    return vg_gat_bwd_gn(g1.row_ptr, g1.col, g1.csc_ptr, g1.csc_slot, g1.csc_dst, n, E, c, S.H, B.att_src, B.att_dst,
                         S.a_s, S.a_d, S.alpha, &gn, dO, B.slope, dH, nullptr, nullptr, nullptr, 0, nullptr, 0, ws,
                         nullptr, nullptr, cx.stream);
  };

  // ----------------------------------------------------- generator forward
  float* z = cx.take((int64_t)n * bt->z_dim);
  VG_RUN(vg_rng_fill(z, (int64_t)n * bt->z_dim, 0, bt->seed, bt->iter, bt->z_salt, cx.stream));
  std::vector<LnS> mfe_s(md->n_mfe), mlp_s(md->n_mlp), dec_s(md->n_dec);
  const float* x = bt->mx;
  int xw = bt->mx_w;
  for (int i = 0; i < md->n_mfe; ++i) {  // models.py:122-131 matched-features encoder
    VG_TRY(ln_fwd(x, xw, md->mfe[i], &mfe_s[i]));
    x = mfe_s[i].y;
    xw = md->mfe[i].out;
  }
  const float* em = x;
  const int hl = xw;
  const int mlp_w = hl + bt->vx_w + bt->z_dim;
  float* mlp_in = cx.take((int64_t)n * mlp_w);
  VG_TRY(cat_cols(cx, {{em, hl}, {bt->vx, bt->vx_w}, {z, bt->z_dim}}, n, mlp_in, mlp_w));
  x = mlp_in;
  xw = mlp_w;
  for (int i = 0; i < md->n_mlp; ++i) {
    VG_TRY(ln_fwd(x, xw, md->mlp[i], &mlp_s[i]));
    x = mlp_s[i].y;
    xw = md->mlp[i].out;
  }
  const float* xm = x;
  const int hg = xw;
  std::vector<GatS> genc(md->n_gblocks);
  for (int b = 0; b < md->n_gblocks; ++b) {
    VG_TRY(gat_fwd(x, xw, md->gblock[b], md->p_drop_g, bt->g_keep_salt[b], &genc[b]));
    x = genc[b].Y;
    xw = genc[b].c;
  }
  const float* enc = x;
  const int ec = xw;
  const int dec_w = ec + hg + hl + bt->vx_w + bt->z_dim;  // models.py:145
  float* dec_in = cx.take((int64_t)n * dec_w);
  VG_TRY(cat_cols(cx, {{enc, ec}, {xm, hg}, {em, hl}, {bt->vx, bt->vx_w}, {z, bt->z_dim}}, n, dec_in, dec_w));
  x = dec_in;
  xw = dec_w;
  for (int i = 0; i < md->n_dec; ++i) {
    VG_TRY(ln_fwd(x, xw, md->dec[i], &dec_s[i]));
    x = dec_s[i].y;
    xw = md->dec[i].out;
  }
  const vg_critic_linear& last = md->dec_last;
  if (last.in != xw || last.out != K) return VG_EINVAL;
  float* logits = cx.take((int64_t)n * K);
  VG_TRY(cx.gemm(x, xw, last.weight, xw, 1, logits, K, n, K, xw, last.bias));
  const float* a_last = x;
  const int a_last_w = xw;
  float* noise = cx.take((int64_t)n * K);
  VG_RUN(vg_rng_fill(noise, (int64_t)n * K, 2, bt->seed, bt->iter, bt->noise_salt, cx.stream));
  float* soft = cx.take((int64_t)n * K);
  VG_RUN(vg_gumbel_fwd(logits, noise, n, K, md->tau, soft, hard, nullptr, cx.stream));

  // ------------------------------------------------- discriminator forward
  const int F = bt->mvx_w;
  float* X0 = cx.take((int64_t)n * (F + K));
  VG_TRY(cat_cols(cx, {{bt->mvx, F}, {hard, K}}, n, X0, F + K));
  std::vector<float*> d_mlp_out(md->n_dmlp);
  x = X0;
  xw = F + K;
  for (int i = 0; i < md->n_dmlp; ++i) {
    const vg_critic_linear& L = md->dmlp[i];
    if (L.in != xw) return VG_EINVAL;
    float* y = cx.take((int64_t)n * L.out);
    VG_TRY(cx.gemm(x, xw, L.weight, xw, 1, y, L.out, n, L.out, xw, L.bias, kActRelu));
    d_mlp_out[i] = y;
    x = y;
    xw = L.out;
  }
  std::vector<GatS> denc(md->n_dblocks);
  for (int b = 0; b < md->n_dblocks; ++b) {
    VG_TRY(gat_fwd(x, xw, md->dblock[b], md->p_drop_d, bt->d_keep_salt[b], &denc[b]));
    x = denc[b].Y;
    xw = denc[b].c;
  }
  const int nd = md->n_ddec;
  std::vector<float*> dec_out(nd);
  for (int i = 0; i < nd; ++i) dec_out[i] = cx.take((int64_t)n * md->ddec[i].out);
  {
    std::vector<int32_t> w{xw};
    std::vector<vg_chain_layer> layers;
    for (int i = 0; i < nd; ++i) {
      w.push_back(md->ddec[i].out);
      layers.push_back(vg_chain_layer{md->ddec[i].weight, md->ddec[i].bias, nullptr, dec_out[i], 0, md->ddec[i].out, 0,
                                      i == nd - 1 ? kActNone : kActRelu});
    }
    const int rc = cx.chain(x, xw, n, w, layers);
    if (rc < 0) return -rc;
    if (rc == 0)
      for (int i = 0; i < nd; ++i) {
        const vg_critic_linear& L = md->ddec[i];
        VG_TRY(cx.gemm(x, xw, L.weight, xw, 1, dec_out[i], L.out, n, L.out, xw, L.bias,
                       i == nd - 1 ? kActNone : kActRelu));
        x = dec_out[i];
        xw = L.out;
      }
  }
  if (md->ddec[nd - 1].out != 1) return VG_EINVAL;
  const float* d_fake = dec_out[nd - 1];

  // ------------------------------------------------------------- loss head
  const int ng = bt->num_graphs;
  float* far_gen = cx.take(ng);
  float* far_ref = cx.take(ng);
  VG_RUN(vg_far_per_graph(bt->vx, bt->vx_w, hard, K, bt->graph_ptr, ng, bt->site_area, bt->far_col, bt->dy_col,
                          bt->dx_col, md->dim_scale, md->void_class, far_gen, far_ref, cx.stream));
  float* lws = cx.take(vg_gen_loss_ws_floats(n, K));
  VG_RUN(vg_gen_loss_fwd(d_fake, hard, logits, bt->onehot, bt->type, n, K, far_gen, far_ref, ng, md->lambda_adv,
                         md->lambda_label, md->lambda_ratio, md->lambda_void, md->lambda_far, out, lws, cx.stream));
  float* g_d = cx.take(n);
  float* g_hard = cx.take((int64_t)n * K);
  float* g_l = md->lambda_label != 0.f ? cx.take((int64_t)n * K) : nullptr;
  VG_RUN(vg_gen_loss_bwd(bt->one, out, logits, bt->type, n, K, g_d, g_hard, g_l, cx.stream));

  // --------------------------- discriminator input VJP (no parameter grads)
  std::vector<float*> adj(nd);
  for (int i = 0; i < nd - 1; ++i) adj[i] = cx.take((int64_t)n * md->ddec[i].out);
  adj[nd - 1] = g_d;
  {
    std::vector<int32_t> w;
    for (int i = nd - 1; i >= 1; --i) w.push_back(md->ddec[i].out);
    w.push_back(md->ddec[0].out);
    std::vector<vg_chain_layer> layers;
    for (int i = nd - 1; i >= 1; --i) {
      const int in = md->ddec[i].in;
      layers.push_back(vg_chain_layer{md->ddec[i].weight, nullptr, dec_out[i - 1], adj[i - 1], in, in, 1, kActMask});
    }
    const int rc = cx.chain(g_d, 1, n, w, layers);
    if (rc < 0) return -rc;
    if (rc == 0)
      for (int i = nd - 1; i >= 1; --i) {
        const int aw = md->ddec[i].out, m = md->ddec[i].in;
        VG_TRY(cx.gemm(adj[i], aw, md->ddec[i].weight, m, 0, adj[i - 1], m, n, m, aw, nullptr, kActMask, dec_out[i - 1],
                       m));
      }
  }
  const vg_critic_linear& W = md->ddec[0];
  float* dY = cx.take((int64_t)n * W.in);
  float* tp = nullptr;
  VG_TRY(gemm_dy(adj[0], W.out, W.weight, W.in, dY, W.in, W.out, denc[md->n_dblocks - 1], &tp));
  std::vector<float*> adj_m(md->n_dmlp);
  for (int i = 0; i < md->n_dmlp; ++i) adj_m[i] = cx.take((int64_t)n * md->dmlp[i].out);
  for (int b = md->n_dblocks - 1; b >= 0; --b) {
    const GatS& S = denc[b];
    const int c = S.c, cin = S.xw;
    float* dH = nullptr;
    VG_TRY(gat_bwd(S, dY, tp, false, &dH));
    const float* Wl = S.B->lin_weight;
    if (b > 0) {
      dY = cx.take((int64_t)n * cin);
      VG_TRY(gemm_dy(dH, c, Wl, cin, dY, cin, c, denc[b - 1], &tp));
    } else {
      VG_TRY(cx.gemm(dH, c, Wl, cin, 0, adj_m[md->n_dmlp - 1], cin, n, cin, c, nullptr, kActMask,
                     d_mlp_out[md->n_dmlp - 1], cin));
    }
  }
  for (int i = md->n_dmlp - 1; i >= 1; --i) {
    const int o = md->dmlp[i].out, m = md->dmlp[i].in;
    VG_TRY(cx.gemm(adj_m[i], o, md->dmlp[i].weight, m, 0, adj_m[i - 1], m, n, m, o, nullptr, kActMask, d_mlp_out[i - 1],
                   m));
  }
  const vg_critic_linear& W0 = md->dmlp[0];
  // label_hard feeds the loss head and D (models.py:229-239): both adjoints summed in the product's epilogue
  float* g_lab = cx.take((int64_t)n * K);
  VG_TRY(cx.gemm(adj_m[0], W0.out, W0.weight + F, W0.in, 0, g_lab, K, n, K, W0.out, nullptr, kActAdd, g_hard, K));

  // ----------------------------------------------------- Gumbel backward
  float* g_logits = cx.take((int64_t)n * K);
  VG_RUN(vg_gumbel_bwd(soft, g_lab, nullptr, n, K, md->tau, g_logits, cx.stream));
  if (g_l && !cx.dry) {
    const long long all = (long long)n * K;
    k_add_to<<<static_cast<int>(std::min<long long>((all + 255) / 256, 4096)), 256, 0,
               static_cast<hipStream_t>(cx.stream)>>>(g_logits, g_l, all);
    VG_CHECK_LAUNCH();
  }

  // -------------------------------------------------- generator backward
  VG_TRY(tn(g_logits, K, a_last, a_last_w, n, K, a_last_w, last.g_weight, a_last_w, last.g_bias));
  float* g = cx.take((int64_t)n * a_last_w);
  VG_TRY(cx.gemm(g_logits, K, last.weight, a_last_w, 0, g, a_last_w, n, a_last_w, K));
  float* g_h = nullptr;
  for (int i = md->n_dec - 1; i > 0; --i) {
    const LnS& S = dec_s[i];
    const int m = S.L->out, k = S.L->in;
    VG_TRY(ln_bwd(S, g, &g_h));
    g = cx.take((int64_t)n * k);
    VG_TRY(cx.gemm(g_h, m, S.L->weight, k, 0, g, k, n, k, m));
  }
  {
    const LnS& S = dec_s[0];
    VG_TRY(ln_bwd(S, g, &g_h));
  }
  const vg_gen_ln_layer& Ld = md->dec[0];
  const int md_ = Ld.out, kd = Ld.in;
  float* g_enc = cx.take((int64_t)n * ec);
  VG_TRY(gemm_dy(g_h, md_, Ld.weight, kd, g_enc, ec, md_, genc[md->n_gblocks - 1], &tp));
  float* g_xem = cx.take((int64_t)n * (hg + hl));  // [x | em] columns of the decoder input (enc taken above)
  VG_TRY(cx.gemm(g_h, md_, Ld.weight + ec, kd, 0, g_xem, hg + hl, n, hg + hl, md_));
  const float* g_y = g_enc;
  float* g_x = nullptr;
  for (int b = md->n_gblocks - 1; b >= 0; --b) {
    const GatS& S = genc[b];
    const int c = S.c, cin = S.xw;
    float* dH = nullptr;
    VG_TRY(gat_bwd(S, g_y, tp, true, &dH));
    const vg_critic_block& B = *S.B;
    VG_TRY(tn(dH, c, S.X, cin, n, c, cin, B.g_lin_weight, cin, nullptr));
    if (b > 0) {
      float* gy = cx.take((int64_t)n * cin);
      VG_TRY(gemm_dy(dH, c, B.lin_weight, cin, gy, cin, c, genc[b - 1], &tp));
      g_y = gy;
    } else {  // x feeds the encoder and the decoder (models.py:132-145)
      g_x = cx.take((int64_t)n * cin);
      VG_TRY(cx.gemm(dH, c, B.lin_weight, cin, 0, g_x, cin, n, cin, c, nullptr, kActAdd, g_xem, hg + hl));
    }
  }
  g = g_x;
  for (int i = md->n_mlp - 1; i >= 0; --i) {
    const LnS& S = mlp_s[i];
    const int m = S.L->out, k = S.L->in;
    VG_TRY(ln_bwd(S, g, &g_h));
    if (i > 0) {
      g = cx.take((int64_t)n * k);
      VG_TRY(cx.gemm(g_h, m, S.L->weight, k, 0, g, k, n, k, m));
    } else {  // the em columns of [em | voxel.x | z]: em feeds the MLP encoder and the decoder
      g = cx.take((int64_t)n * hl);
      VG_TRY(cx.gemm(g_h, m, S.L->weight, k, 0, g, hl, n, hl, m, nullptr, kActAdd, g_xem ? g_xem + hg : nullptr,
                     hg + hl));
    }
  }
  for (int i = md->n_mfe - 1; i >= 0; --i) {
    const LnS& S = mfe_s[i];
    const int m = S.L->out, k = S.L->in;
    VG_TRY(ln_bwd(S, g, &g_h));
    if (i > 0) {
      g = cx.take((int64_t)n * k);
      VG_TRY(cx.gemm(g_h, m, S.L->weight, k, 0, g, k, n, k, m));
    }
  }
  return folds.flush(cx);
}

bool model_ok(const vg_gen_model* md, const vg_gen_batch* bt) {
  if (!md || !bt) return false;
  auto in_range = [](int v, int hi) { return v >= 1 && v <= hi; };
  if (!in_range(md->n_mfe, VG_GEN_MAX_LAYERS) || !in_range(md->n_mlp, VG_GEN_MAX_LAYERS) ||
      !in_range(md->n_dec, VG_GEN_MAX_LAYERS) || !in_range(md->n_gblocks, VG_GEN_MAX_BLOCKS) ||
      !in_range(md->n_dmlp, VG_GEN_MAX_LAYERS) || !in_range(md->n_dblocks, VG_GEN_MAX_BLOCKS) ||
      !in_range(md->n_ddec, VG_GEN_MAX_LAYERS))
    return false;
  if (bt->n < 64 || bt->classes < 1 || bt->mx_w < 1 || bt->vx_w < 1 || bt->mvx_w < 1 || bt->z_dim < 1 ||
      bt->num_graphs < 1 || bt->g.num_nodes != bt->n || bt->seg_rows != bt->n)
    return false;
  if (md->mfe[0].in != bt->mx_w || md->dmlp[0].in != bt->mvx_w + bt->classes) return false;
  return true;
}

}  // namespace

extern "C" int64_t vg_gen_arena_floats(const vg_gen_model* model, const vg_gen_batch* batch) {
  if (!model_ok(model, batch)) return -1;
  Ctx cx{true, model->bf16, nullptr, nullptr, 0, 0};
  if (run(cx, model, batch, nullptr, nullptr)) return -1;
  return cx.off;
}

extern "C" int vg_gen_loss_and_grad(const vg_gen_model* model, const vg_gen_batch* batch, float* arena,
                                    int64_t arena_floats, float* out, float* hard, void* stream) {
  if (!model_ok(model, batch) || !arena || !out || !hard || !batch->mx || !batch->vx || !batch->mvx ||
      !batch->onehot || !batch->type || !batch->graph_ptr || !batch->site_area || !batch->iter || !batch->one ||
      !batch->g.row_ptr || !batch->g.col || !batch->g.csc_ptr || !batch->g.csc_slot || !batch->g.csc_dst)
    return VG_EINVAL;
  if (reinterpret_cast<uintptr_t>(arena) & 255) return VG_EINVAL;
  const int64_t need = vg_gen_arena_floats(model, batch);
  if (need < 0 || need > arena_floats) return VG_EINVAL;
  Ctx cx{false, model->bf16, stream, arena, arena_floats, 0};
  return run(cx, model, batch, out, hard);
}
