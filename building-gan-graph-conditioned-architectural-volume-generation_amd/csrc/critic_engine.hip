// One critic iteration issued from C++: vg_critic_loss_and_grad (include/vgan.h).
//
// A restatement of vgan/critic.py CriticEngine.loss_and_grad in its default
// configuration -- the WGAN-GP loss of trainer.py:291-332 and its double
// backward (trainer.py:476-479) as four passes over the discriminator's op
// chain (A: stacked real / fake / mix forward; B: input VJP of the mix copy
// and the penalty head; C: tangent sweep with the second-order terms; D:
// stacked VJP of all copies, weight gradients grouped, folds deferred).  The
// same entry points are called in the same order with the same arguments, so
// the results are bit-identical to the Python engine's; only the host-side
// cost per launch changes (Python: marshalling + one torch allocation per
// temporary; here: a bump allocator over the caller's arena).  Host code
// only: every launch goes through the library's own extern "C" entry points.
#include "engine.h"

namespace {

using vg_engine::Ctx;
using vg_engine::Folds;
using vg_engine::kActMask;
using vg_engine::kActNone;
using vg_engine::kActRelu;
constexpr int64_t kFoldWsFloats = 1 << 17;  // the split folds' chunk sums

// per-block state of the forward (critic.py's blk dicts)
struct Blk {
  float *X, *H, *O, *alpha, *a_s, *a_d, *Y, *stats, *keep;
  int xw, c;
};

int run(Ctx& cx, const vg_critic_model* md, const vg_critic_batch* bt, float* out) {
  const int n = bt->n, F = bt->feat, K = bt->classes;
  const int R = 3 * n, W0 = F + K, X4 = 4 * n;
  const int E = bt->g1.num_edges;
  const int nb = md->n_blocks, nd = md->n_dec, nm = md->n_mlp;
  const int mrow = 2 * n, trow = 3 * n;  // first row of the mix copy / of the tangent (pass-B) rows
  const vg_csr_ref& g1 = bt->g1;
  const vg_csr_ref& g3 = bt->g3;
  auto rows = [](float* t, int r0, int width) { return t ? t + (int64_t)r0 * width : nullptr; };
  Folds folds;
  folds.ws = cx.take(kFoldWsFloats);
  folds.ws_floats = kFoldWsFloats;

  // ------------------------------------------------------------ pass A
  float* X0 = cx.take((int64_t)X4 * W0);
  VG_RUN(vg_critic_input_drawn(bt->mvx, n, F, bt->real, bt->hard, bt->soft, bt->seed, bt->iter, bt->eps_salt, K, 4,
                               X0, cx.stream));
  std::vector<float*> mlp_out(nm);
  float* x = X0;
  int xw = W0;
  for (int i = 0; i < nm; ++i) {
    const vg_critic_linear& L = md->mlp[i];
    float* y = cx.take((int64_t)X4 * L.out);
    VG_TRY(cx.gemm(x, xw, L.weight, xw, 1, y, L.out, R, L.out, xw, L.bias, kActRelu));
    mlp_out[i] = y;
    x = y;
    xw = L.out;
  }
  std::vector<Blk> blk(nb);
  for (int b = 0; b < nb; ++b) {
    const vg_critic_block& B = md->block[b];
    const int c = B.out;
    float* H = cx.take((int64_t)R * c);
    float* a_s = cx.take(R);
    float* a_d = cx.take(R);
    VG_RUN(cx.bf16 ? vg_gat_lin_att_bf16(x, xw, B.lin_weight, R, xw, c, B.att_src, B.att_dst, H, a_s, a_d, cx.stream)
                   : vg_gat_lin_att(x, xw, B.lin_weight, R, xw, c, B.att_src, B.att_dst, H, a_s, a_d, cx.stream));
    float* O = cx.take((int64_t)R * c);
    float* alpha = cx.take(3LL * E);
    const int g = vg_gat_gnp_rows(g3.num_nodes, c);
    if (g <= 0 || n < g || g3.num_nodes % n) return VG_EINVAL;  // (the Python engine's unfused path)
    float* gnp = cx.take(vg_gat_gnp_floats(g3.num_nodes, c));
    VG_RUN(vg_gat_aggregate_fwd_gnp(g3.row_ptr, g3.col, g3.ell, g3.ell ? g3.ell_width : 0, g3.num_nodes, c, H, a_s, a_d,
                                    B.bias, B.slope, O, alpha, n, gnp, cx.stream));
    float* Y = cx.take((int64_t)X4 * c);
    float* stats = cx.take(3LL * 2 * c);
    float* keep = cx.take((int64_t)R * c);
    VG_RUN(vg_graphnorm_fwd_gnp(O, 3, n, c, B.gn_weight, B.gn_bias, B.gn_mean_scale, nullptr, md->p_drop, bt->seed,
                                bt->iter, bt->keep_salt[b], B.gn_eps, Y, keep, stats, gnp, g, cx.stream));
    blk[b] = Blk{x, H, O, alpha, a_s, a_d, Y, stats, keep, xw, c};
    x = Y;
    xw = c;
  }
  std::vector<float*> dec_out(nd);
  for (int i = 0; i < nd; ++i) dec_out[i] = cx.take((int64_t)(i == nd - 1 ? R : X4) * md->dec[i].out);
  {
    std::vector<int32_t> w{xw};
    std::vector<vg_chain_layer> layers;
    for (int i = 0; i < nd; ++i) {
      w.push_back(md->dec[i].out);
      layers.push_back(vg_chain_layer{md->dec[i].weight, md->dec[i].bias, nullptr, dec_out[i], 0, md->dec[i].out, 0,
                                      i == nd - 1 ? kActNone : kActRelu});
    }
    const int rc = cx.chain(x, xw, R, w, layers);
    if (rc < 0) return -rc;
    if (rc == 0)
      for (int i = 0; i < nd; ++i) {
        const vg_critic_linear& L = md->dec[i];
        VG_TRY(cx.gemm(x, xw, L.weight, xw, 1, dec_out[i], L.out, R, L.out, xw, L.bias,
                       i == nd - 1 ? kActNone : kActRelu));
        x = dec_out[i];
        xw = L.out;
      }
  }
  float* scores = dec_out[nd - 1];
  if (md->dec[nd - 1].out != 1) return VG_EINVAL;

  // adjoint buffers of pass D (rows [0,3N)) whose rows [3N,4N) pass B fills
  std::vector<float*> adj_dec(nd), adj_H(nb), adj_mlp(nm);
  for (int i = 0; i < nd - 1; ++i) adj_dec[i] = cx.take((int64_t)X4 * md->dec[i].out);
  adj_dec[nd - 1] = const_cast<float*>(bt->seeds4);
  for (int b = 0; b < nb; ++b) adj_H[b] = cx.take((int64_t)X4 * blk[b].c);
  for (int i = 0; i < nm; ++i) adj_mlp[i] = cx.take((int64_t)X4 * md->mlp[i].out);

  // the decoder's adjoint chain adj_dec[nd-1] -> ... -> adj_dec[0] (rows r0..)
  auto adj_chain = [&](int r0, int nrows, int r_aux) -> int {
    std::vector<int32_t> w;
    for (int i = nd - 1; i >= 1; --i) w.push_back(md->dec[i].out);
    w.push_back(md->dec[0].out);
    std::vector<vg_chain_layer> layers;
    for (int i = nd - 1; i >= 1; --i) {
      const int in = md->dec[i].in;
      layers.push_back(vg_chain_layer{md->dec[i].weight, nullptr, rows(dec_out[i - 1], r_aux, in),
                                      rows(adj_dec[i - 1], r0, in), in, in, 1, kActMask});
    }
    return cx.chain(rows(adj_dec[nd - 1], r0, w[0]), w[0], nrows, w, layers);
  };

  // block b's GraphNorm input, keep and statistics: the mix copy (pass B/C) or all three
  struct GnIn {
    const float *x, *keep, *stats;
  };
  auto gn_inputs = [&](int b, bool mix) {
    const Blk& B = blk[b];
    return mix ? GnIn{rows(B.O, mrow, B.c), rows(B.keep, mrow, B.c), B.stats ? B.stats + 2 * 2 * B.c : nullptr}
               : GnIn{B.O, B.keep, B.stats};
  };
  // out [nrows, m] = A Wt, the output gradient of block b's GraphNorm, with that
  // backward's column partials from the GEMM's epilogue (returned)
  auto gemm_dy = [&](const float* A, int lda, const float* Wt, int ldw, float* o, int nrows, int m, int k, int b,
                     bool mix, float** tp_out) -> int {
    const vg_critic_block& N = md->block[b];
    float* tp = cx.take(vg_gemm_gn_tpart_floats(nrows, m));
    const GnIn gi = gn_inputs(b, mix);
    *tp_out = tp;
    if (cx.dry) return 0;
    return cx.bf16 ? vg_gemm_gn_bwd_bf16(A, lda, Wt, ldw, nrows, m, k, o, m, gi.x, gi.keep, n, N.gn_weight, N.gn_bias,
                                         N.gn_mean_scale, N.gn_eps, gi.stats, tp, cx.stream)
                   : vg_gemm_gn_bwd(A, lda, Wt, ldw, nrows, m, k, o, m, gi.x, gi.keep, n, N.gn_weight, N.gn_bias,
                                    N.gn_mean_scale, N.gn_eps, gi.stats, tp, cx.stream);
  };
  // block b's GraphNorm(+ReLU+Dropout) backward, column sums only: the
  // descriptor with which vg_gat_bwd_gn forms g_x in its destination-row pass
  auto gn_bwd = [&](int b, bool mix, const float* tp, const float* g_y, bool pgrads, const float* inj, int64_t inj_off,
                    vg_gn_bwd_in* gn) -> int {
    const vg_critic_block& N = md->block[b];
    const int c = blk[b].c, S = mix ? 1 : 3;
    const GnIn gi = gn_inputs(b, mix);
    float* ws = cx.take(vg_graphnorm_seg_ws_floats(S, n, c));
    *gn = vg_gn_bwd_in{gi.x,
                       gi.keep,
                       g_y,
                       inj,
                       N.gn_weight,
                       N.gn_bias,
                       N.gn_mean_scale,
                       gi.stats,
                       ws ? ws + vg_graphnorm_bwd_sums_offset(S, c) : nullptr,
                       N.gn_eps,
                       S,
                       n,
                       inj ? inj_off : 0};
    if (cx.dry) return 0;
    return vg_graphnorm_bwd_seg_tiles(gi.x, S, n, c, N.gn_weight, N.gn_bias, N.gn_mean_scale, gi.keep, N.gn_eps,
                                      gi.stats, g_y, tp, nullptr, pgrads ? N.g_gn_weight : nullptr,
                                      pgrads ? N.g_gn_bias : nullptr, pgrads ? N.g_gn_mean_scale : nullptr,
                                      pgrads ? 1 : 0, inj, inj_off, ws, cx.stream);
  };
  auto gemm_tn = [&](const float* A, int lda, const float* B, int ldb, int N, int M, int Kk, float* C, int ldc,
                     float* db, int db_rows) -> int {
    float* ws = cx.take(std::max<int64_t>(1, vg_gemm_tn_ws_floats(N, M, Kk)));
    return folds.tn(cx, A, lda, B, ldb, N, M, Kk, C, ldc, db, db_rows, ws);
  };

  // ------------------------------------------------------------ pass B
  {
    const int rc = adj_chain(trow, n, mrow);
    if (rc < 0) return -rc;
    if (rc == 0)
      for (int i = nd - 1; i >= 1; --i) {
        const int aw = md->dec[i].out, m = md->dec[i].in;
        VG_TRY(cx.gemm(rows(adj_dec[i], trow, aw), aw, md->dec[i].weight, m, 0, rows(adj_dec[i - 1], trow, m), m, n, m,
                       aw, nullptr, kActMask, rows(dec_out[i - 1], mrow, m), m));
      }
  }
  float* tp = nullptr;
  const vg_critic_linear& D0 = md->dec[0];
  float* dY = cx.take((int64_t)n * D0.in);
  VG_TRY(gemm_dy(rows(adj_dec[0], trow, D0.out), D0.out, D0.weight, D0.in, dY, n, D0.in, D0.out, nb - 1, true, &tp));
  std::vector<float*> dY_b(nb), dO_b(nb);
  for (int b = nb - 1; b >= 0; --b) {
    const vg_critic_block& B = md->block[b];
    const Blk& S = blk[b];
    const int c = S.c;
    dY_b[b] = dY;
    float* dO = cx.take((int64_t)n * c);
    float* dH = rows(adj_H[b], trow, c);
    float* ws = cx.take(vg_gat_bwd_ws_floats(n, E, c));
    vg_gn_bwd_in gn;
    VG_TRY(gn_bwd(b, true, tp, dY, false, nullptr, 0, &gn));
    VG_RUN(vg_gat_bwd_gn(g1.row_ptr, g1.col, g1.csc_ptr, g1.csc_slot, g1.csc_dst, n, E, c, rows(S.H, mrow, c), B.att_src,
                         B.att_dst, S.a_s ? S.a_s + mrow : nullptr, S.a_d ? S.a_d + mrow : nullptr,
                         S.alpha ? S.alpha + 2LL * E : nullptr, &gn, dO, B.slope, dH, nullptr, nullptr, nullptr, 0,
                         nullptr, 0, ws, nullptr, nullptr, cx.stream));
    dO_b[b] = dO;
    const int cin = S.xw;
    if (b > 0) {
      float* dX = cx.take((int64_t)n * cin);
      VG_TRY(gemm_dy(dH, c, B.lin_weight, cin, dX, n, cin, c, b - 1, true, &tp));
      dY = dX;
    } else {
      VG_TRY(cx.gemm(dH, c, B.lin_weight, cin, 0, rows(adj_mlp[nm - 1], trow, cin), cin, n, cin, c, nullptr, kActMask,
                     rows(mlp_out[nm - 1], mrow, cin), cin));
    }
  }
  for (int i = nm - 1; i >= 1; --i) {
    const int o = md->mlp[i].out, m = md->mlp[i].in;
    VG_TRY(cx.gemm(rows(adj_mlp[i], trow, o), o, md->mlp[i].weight, m, 0, rows(adj_mlp[i - 1], trow, m), m, n, m, o,
                   nullptr, kActMask, rows(mlp_out[i - 1], mrow, m), m));
  }
  const vg_critic_linear& M0 = md->mlp[0];
  const int hd = M0.out;
  float* g = cx.take((int64_t)n * K);
  VG_TRY(cx.gemm(rows(adj_mlp[0], trow, hd), hd, M0.weight + F, W0, 0, g, K, n, K, hd));
  float* gws = cx.take(vg_gp_head_ws_floats(n));
  float* u0 = X0 ? X0 + (int64_t)trow * W0 + F : nullptr;  // dGP/dg into the label columns of X0's tangent rows
  VG_RUN(vg_gp_head(g, n, K, scores, md->lambda_gp, u0, W0, out, gws, bt->gp_counter, cx.stream));

  // ------------------------------------------------------------ pass C
  VG_TRY(cx.gemm(u0, W0, M0.weight + F, W0, 1, rows(mlp_out[0], trow, hd), hd, n, hd, K, nullptr, kActMask,
                 rows(mlp_out[0], mrow, hd), hd));
  int uw = hd;
  for (int i = 1; i < nm; ++i) {
    const int o = md->mlp[i].out;
    VG_TRY(cx.gemm(rows(mlp_out[i - 1], trow, uw), uw, md->mlp[i].weight, uw, 1, rows(mlp_out[i], trow, o), o, n, o, uw,
                   nullptr, kActMask, rows(mlp_out[i], mrow, o), o));
    uw = o;
  }
  float* u_in = rows(mlp_out[nm - 1], trow, uw);
  std::vector<float*> hinj_b(nb), oinj_b(nb);
  for (int b = 0; b < nb; ++b) {
    const vg_critic_block& B = md->block[b];
    const Blk& S = blk[b];
    const int c = S.c, cin = S.xw;
    float* uH = cx.take((int64_t)n * c);
    float* up_s = cx.take(n);
    float* up_d = cx.take(n);
    VG_RUN(cx.bf16 ? vg_gat_lin_att_bf16(u_in, cin, B.lin_weight, n, cin, c, B.att_src, B.att_dst, uH, up_s, up_d,
                                         cx.stream)
                   : vg_gat_lin_att(u_in, cin, B.lin_weight, n, cin, c, B.att_src, B.att_dst, uH, up_s, up_d,
                                    cx.stream));
    float* uO = cx.take((int64_t)n * c);
    float* hinj = cx.take((int64_t)n * c);
    float* ws = cx.take(vg_gat_jvp2_ws_floats(n, E, c));
    const float* gx = rows(S.O, mrow, c);
    const float* gkeep = rows(S.keep, mrow, c);
    const float* gstats = S.stats ? S.stats + 2 * 2 * c : nullptr;
    float* oinj = cx.take((int64_t)n * c);
    float* gws2 = cx.take(vg_graphnorm_seg_ws_floats(1, n, c));
    if (!cx.dry) {
      // the GAT tangent's destination-row pass, its folds deferred
      // (FoldCollector.jvp) and its source pass described: the source pass
      // writes only pass D's injection and att_src partials, so it runs in the
      // GraphNorm fold's launch (vg_graphnorm_jvp2_fold_src) instead of one of
      // its own -- the same kernels and values as vg_gat_jvp2_deferred +
      // vg_graphnorm_jvp2, one launch fewer per block
      vg_fold f[2];
      int32_t nf = 0;
      vg_jvp_src src;
      VG_TRY(vg_gat_jvp2_plan(g1.row_ptr, g1.col, g1.csc_ptr, g1.csc_slot, g1.csc_dst, n, E, c, rows(S.H, mrow, c),
                              uH, dO_b[b], B.att_src, B.att_dst, S.a_s + mrow, S.a_d + mrow, S.alpha + 2LL * E,
                              B.slope, uO, hinj, B.g_att_src, B.g_att_dst, up_s, up_d, ws, f, &nf, &src, cx.stream));
      folds.add(f, nf);
      VG_TRY(vg_graphnorm_jvp2_sums(gx, n, c, B.gn_weight, B.gn_bias, B.gn_mean_scale, gkeep, B.gn_eps, gstats, uO,
                                    dY_b[b], gws2, cx.stream));
      VG_TRY(vg_graphnorm_jvp2_fold_src(n, c, B.gn_weight, B.gn_mean_scale, gstats, gws2, B.g_gn_weight,
                                        B.g_gn_mean_scale, &src, cx.stream));
      VG_TRY(vg_graphnorm_jvp2_apply(gx, n, c, B.gn_weight, B.gn_bias, B.gn_mean_scale, gkeep, B.gn_eps, gstats, uO,
                                     dY_b[b], rows(S.Y, trow, c), oinj, gws2, cx.stream));
    }
    hinj_b[b] = hinj;
    oinj_b[b] = oinj;
    u_in = rows(S.Y, trow, c);
    uw = c;
  }
  {  // the tangent through the decoder's hidden layers
    std::vector<int32_t> w{uw};
    std::vector<vg_chain_layer> layers;
    for (int i = 0; i < nd - 1; ++i) {
      const int o = md->dec[i].out;
      w.push_back(o);
      layers.push_back(vg_chain_layer{md->dec[i].weight, nullptr, rows(dec_out[i], mrow, o), rows(dec_out[i], trow, o),
                                      o, o, 0, kActMask});
    }
    const int rc = cx.chain(u_in, uw, n, w, layers);
    if (rc < 0) return -rc;
    if (rc == 0)
      for (int i = 0; i < nd - 1; ++i) {
        const int o = md->dec[i].out;
        VG_TRY(cx.gemm(u_in, uw, md->dec[i].weight, uw, 1, rows(dec_out[i], trow, o), o, n, o, uw, nullptr, kActMask,
                       rows(dec_out[i], mrow, o), o));
        u_in = rows(dec_out[i], trow, o);
        uw = o;
      }
  }

  // ------------------------------------------------------------ pass D
  // weight gradients over 4N rows: [pass-D adjoint ; pass-B adjoint]^T [activation ; tangent]
  std::vector<float*> dec_in(nd);
  dec_in[0] = nb ? blk[nb - 1].Y : mlp_out[nm - 1];
  for (int i = 1; i < nd; ++i) dec_in[i] = dec_out[i - 1];
  const int chained = adj_chain(0, R, 0);
  if (chained < 0) return -chained;
  for (int i = nd - 1; i >= 0; --i) {
    const vg_critic_linear& L = md->dec[i];
    const int aw = L.out, m = L.in;
    VG_TRY(gemm_tn(adj_dec[i], aw, dec_in[i], m, X4, aw, m, L.g_weight, m, L.g_bias, R));
    if (i > 0) {
      if (!chained)
        VG_TRY(cx.gemm(adj_dec[i], aw, L.weight, m, 0, adj_dec[i - 1], m, R, m, aw, nullptr, kActMask, dec_out[i - 1],
                       m));
    } else {
      dY = cx.take((int64_t)R * m);
      VG_TRY(gemm_dy(adj_dec[0], aw, L.weight, m, dY, R, m, aw, nb - 1, false, &tp));
    }
  }
  for (int b = nb - 1; b >= 0; --b) {
    const vg_critic_block& B = md->block[b];
    const Blk& S = blk[b];
    const int c = S.c, cin = S.xw;
    float* dO = cx.take((int64_t)R * c);
    float* ws = cx.take(vg_gat_bwd_ws_floats(R, 3 * E, c));
    vg_gn_bwd_in gn;
    VG_TRY(gn_bwd(b, false, tp, dY, true, oinj_b[b], (int64_t)mrow * c, &gn));
    if (!cx.dry) {  // folds deferred (FoldCollector.call)
      vg_fold f[3];
      int32_t nf = 0;
      VG_TRY(vg_gat_bwd_gn(g3.row_ptr, g3.col, g3.csc_ptr, g3.csc_slot, g3.csc_dst, R, 3 * E, c, S.H, B.att_src,
                           B.att_dst, S.a_s, S.a_d, S.alpha, &gn, dO, B.slope, adj_H[b], B.g_att_src, B.g_att_dst,
                           B.g_bias, 1, hinj_b[b], mrow, ws, f, &nf, cx.stream));
      folds.add(f, nf);
    }
    VG_TRY(gemm_tn(adj_H[b], c, S.X, cin, X4, c, cin, B.g_lin_weight, cin, nullptr, X4));
    if (b > 0) {
      dY = cx.take((int64_t)R * cin);
      VG_TRY(gemm_dy(adj_H[b], c, B.lin_weight, cin, dY, R, cin, c, b - 1, false, &tp));
    } else {
      VG_TRY(cx.gemm(adj_H[b], c, B.lin_weight, cin, 0, adj_mlp[nm - 1], cin, R, cin, c, nullptr, kActMask,
                     mlp_out[nm - 1], cin));
    }
  }
  for (int i = nm - 1; i >= 0; --i) {
    const vg_critic_linear& L = md->mlp[i];
    const int o = L.out, m = L.in;
    const float* xin = i == 0 ? X0 : mlp_out[i - 1];
    VG_TRY(gemm_tn(adj_mlp[i], o, xin, m, X4, o, m, L.g_weight, m, L.g_bias, R));
    if (i > 0)
      VG_TRY(cx.gemm(adj_mlp[i], o, L.weight, m, 0, adj_mlp[i - 1], m, R, m, o, nullptr, kActMask, mlp_out[i - 1], m));
  }
  return folds.flush(cx);
}

bool model_ok(const vg_critic_model* md, const vg_critic_batch* bt) {
  if (!md || !bt) return false;
  if (md->n_mlp < 1 || md->n_blocks < 1 || md->n_dec < 1 || md->n_mlp > VG_CRITIC_MAX_LAYERS ||
      md->n_blocks > VG_CRITIC_MAX_LAYERS || md->n_dec > VG_CRITIC_MAX_LAYERS)
    return false;
  if (bt->n < 64 || bt->feat < 1 || bt->classes < 1 || bt->g1.num_nodes != bt->n || bt->g3.num_nodes != 3 * bt->n ||
      bt->g3.num_edges != 3 * bt->g1.num_edges)
    return false;
  if (md->mlp[0].in != bt->feat + bt->classes) return false;
  int w = md->mlp[0].in;
  for (int i = 0; i < md->n_mlp; ++i) {
    if (md->mlp[i].in != w) return false;
    w = md->mlp[i].out;
  }
  for (int b = 0; b < md->n_blocks; ++b) {
    if (md->block[b].in != w) return false;
    w = md->block[b].out;
  }
  for (int i = 0; i < md->n_dec; ++i) {
    if (md->dec[i].in != w) return false;
    w = md->dec[i].out;
  }
  return w == 1;
}

}  // namespace

extern "C" int64_t vg_critic_arena_floats(const vg_critic_model* model, const vg_critic_batch* batch) {
  if (!model_ok(model, batch)) return -1;
  Ctx cx{true, model->bf16, nullptr, nullptr, 0, 0};
  if (run(cx, model, batch, nullptr)) return -1;
  return cx.off;
}

extern "C" int vg_critic_loss_and_grad(const vg_critic_model* model, const vg_critic_batch* batch, float* arena,
                                       int64_t arena_floats, float* out, void* stream) {
  if (!model_ok(model, batch) || !arena || !out || !batch->mvx || !batch->real || !batch->hard || !batch->soft ||
      !batch->seeds4 || !batch->iter || !batch->gp_counter)
    return VG_EINVAL;
  if (reinterpret_cast<uintptr_t>(arena) & 255) return VG_EINVAL;
  const int64_t need = vg_critic_arena_floats(model, batch);
  if (need < 0 || need > arena_floats) return VG_EINVAL;
  Ctx cx{false, model->bf16, stream, arena, arena_floats, 0};
  return run(cx, model, batch, out);
}
