/*
 * vgan -- C ABI of the MI355X-native voxel-graph GAN message-passing core.
 *
 * libvgan_hip.so (gfx950) exports exactly these functions.  They replace the
 * torch-geometric 2.6.1 operator calls the reference issues from
 * building_gan/src/models.py (paths below are relative to /root/reference) and
 * the per-step device work of building_gan/src/trainer.py.
 *
 * Conventions (all functions):
 *   - every pointer is a DEVICE pointer unless named host_*; tensors are
 *     contiguous row-major; features f32; CSR indices int32; edge_index int64;
 *   - the caller allocates every output and workspace (query the *_ws_* sizes);
 *     no function allocates, frees or synchronises, so all are capturable in a
 *     hipGraph;
 *   - work is enqueued on `stream` (hipStream_t passed as void*);
 *   - return 0 on success, a hipError_t value on a launch failure, or
 *     VG_EINVAL for an invalid argument (checked on the host before launch).
 *
 * CSR layout ("destination CSR"): row i lists the incoming edges of node i in
 * original edge order with the self loop LAST -- exactly the edge order of
 * GATConv after remove_self_loops + add_self_loops -- so the per-row sums run
 * in the order torch-geometric's scatter would.  The "source CSC" is its
 * transpose: for source node j, the CSR slots k with col[k] == j (ascending k).
 */
#ifndef VGAN_H_
#define VGAN_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VG_EINVAL (-1)
/* vg_graph_exec_update: the recorded graph differs in topology (instantiate it instead). */
#define VG_EGRAPH_TOPOLOGY (-2)

/* ---- graph structure ---------------------------------------------------- */

/* Workspace (int32 elements) needed by vg_csr_build. */
int64_t vg_csr_ws_ints(int64_t num_edges, int32_t num_nodes);

/* Build destination CSR (+1 self loop per node, input self loops dropped) and
 * its source CSC from edge_index [2, E] int64.
 * Replaces: GATConv.forward's remove_self_loops/add_self_loops, run on every
 * call of every layer (models.py:144,242 -> torch_geometric/nn/conv/gat_conv.py)
 * -- here once per mini-batch.
 * Outputs: row_ptr[N+1], col[E+N], csc_ptr[N+1], csc_slot[E+N], csc_dst[E+N]
 * (sized for the worst case; the used length E' is written to status[0]);
 * status[1] != 0 flags an out-of-range node index. */
int vg_csr_build(const int64_t* edge_index, int64_t num_edges, int32_t num_nodes,
                 int32_t* row_ptr, int32_t* col, int32_t* csc_ptr, int32_t* csc_slot,
                 int32_t* csc_dst, int32_t* workspace, int32_t* status, void* stream);

/* ---- GATConv(heads=1) message passing ----------------------------------- */

/* One GATConv(heads=1) message-passing layer after the projection h = x W^T,
 * fused into a single kernel:
 *   a_dst_i = <h_i, att_dst>,  a_src_i = <h_i, att_src>       (written, [N] each)
 *   e_k     = leaky_relu(a_src[col_k] + a_dst_i, slope)
 *   alpha   = segment softmax of e over row i (max-shifted, denominator + 1e-16)
 *   out_i   = sum_k alpha_k * h[col_k] + bias                   (alpha written, [E'])
 * Replaces the (h*att).sum(-1) projections, GATConv.edge_update
 * (utils/_softmax.py scatter max/sum) and propagate/message/aggregate ('add'
 * scatter) + bias of torch_geometric/nn/conv/gat_conv.py as called from
 * models.py:144 (generator, 14 layers) and models.py:242 (discriminator, 6).
 * att_src / att_dst / bias: [C] (any alignment). */
int vg_gat_fwd(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t channels,
               const float* h, const float* att_src, const float* att_dst, const float* bias,
               float slope, float* out, float* alpha, float* a_src, float* a_dst, void* stream);

/* The two halves of vg_gat_fwd, so the projection can live in a GEMM epilogue.
 *
 * vg_gat_att: a_src_i = <h_i, att_src>, a_dst_i = <h_i, att_dst> ([N] each) --
 * the (x * att).sum(-1) pair of torch_geometric/nn/conv/gat_conv.py (GATConv
 * .forward, heads=1) as called from models.py:144,242.
 *
 * vg_gat_lin_att: H = X W^T (X [N, Cin] row stride ldx, W [C, Cin]) AND the
 * projections above in one launch when C <= 64 (the tile's rows are reduced
 * against att_src / att_dst in the GEMM epilogue; C > 64 runs the GEMM then
 * vg_gat_att) -- GATConv.lin followed by the attention projections.
 *
 * vg_gat_aggregate_fwd: given h and the projections, the edge softmax and the
 * weighted CSR gather-sum (+ bias), writing out [N, C] and alpha [E'] --
 * GATConv.edge_update (utils/_softmax.py scatter max / sum) and
 * propagate/message/aggregate ('add' scatter) + bias.  This is the path's
 * "scatter kernel" (SURVEY.md 8a rows A6-A7). */
int vg_gat_att(const float* h, int32_t num_nodes, int32_t channels, const float* att_src,
               const float* att_dst, float* a_src, float* a_dst, void* stream);
int vg_gat_lin_att(const float* x, int32_t ldx, const float* w, int32_t num_nodes,
                   int32_t in_channels, int32_t channels, const float* att_src,
                   const float* att_dst, float* h, float* a_src, float* a_dst, void* stream);
int vg_gat_aggregate_fwd(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes,
                         int32_t channels, const float* h, const float* a_src, const float* a_dst,
                         const float* bias, float slope, float* out, float* alpha, void* stream);

/* Workspace (floats) for vg_gat_bwd. */
int64_t vg_gat_bwd_ws_floats(int32_t num_nodes, int32_t num_edges, int32_t channels);

/* First-order backward of vg_gat_fwd (the autograd path without create_graph):
 * g_h [N,C] (including the att_src/att_dst projection terms), g_att_src,
 * g_att_dst, g_bias [C].  Three passes, no atomics, deterministic. */
int vg_gat_bwd(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
               const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
               int32_t num_edges, int32_t channels, const float* h, const float* att_src,
               const float* att_dst, const float* a_src, const float* a_dst, const float* alpha,
               const float* g_out, float slope, float* g_h, float* g_att_src, float* g_att_dst,
               float* g_bias, float* workspace, void* stream);

/* vg_gat_bwd with options for the critic engine: g_att_src may be NULL (no
 * parameter gradients; g_att_dst / g_bias are then ignored), parameter
 * gradients are written (accumulate = 0) or added (1), and inj [N - inj_row0,
 * C] (nullable) is added to the rows g_h[inj_row0:] (the second-order adjoint
 * of the gradient-penalty copy).  Same workspace as vg_gat_bwd. */
int vg_gat_bwd_ex(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                  const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
                  int32_t num_edges, int32_t channels, const float* h, const float* att_src,
                  const float* att_dst, const float* a_src, const float* a_dst,
                  const float* alpha, const float* g_out, float slope, float* g_h,
                  float* g_att_src, float* g_att_dst, float* g_bias, int32_t accumulate,
                  const float* inj, int32_t inj_row0, float* workspace, void* stream);

/* Workspace (floats) for vg_gat_jvp2. */
int64_t vg_gat_jvp2_ws_floats(int32_t num_nodes, int32_t num_edges, int32_t channels);

/* Tangent and second-order terms of out = GATConv(h) for the gradient
 * penalty's double backward (trainer.py:306-316, create_graph=True): given a
 * tangent u of h and the first-backward adjoint g_out, u_out = J u and, for
 * Q = <g_out, J u>, h_inj = dQ/dh; dQ/datt_src, dQ/datt_dst are ADDED to
 * g_att_src, g_att_dst (dQ/dbias = 0).  Deterministic (no atomics). */
int vg_gat_jvp2(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
                int32_t num_edges, int32_t channels, const float* h, const float* u,
                const float* g_out, const float* att_src, const float* att_dst, const float* a_src,
                const float* a_dst, const float* alpha, float slope, float* u_out, float* h_inj,
                float* g_att_src, float* g_att_dst, float* workspace, void* stream);

/* vg_gat_jvp2 with the tangent projections u att_src / u att_dst supplied
 * (up_src, up_dst [N], e.g. from vg_gat_lin_att on the tangent), saving its
 * first pass; both NULL = compute them (same as vg_gat_jvp2). */
int vg_gat_jvp2_ex(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                   const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
                   int32_t num_edges, int32_t channels, const float* h, const float* u,
                   const float* g_out, const float* att_src, const float* att_dst,
                   const float* a_src, const float* a_dst, const float* alpha, float slope,
                   float* u_out, float* h_inj, float* g_att_src, float* g_att_dst,
                   const float* up_src, const float* up_dst, float* workspace, void* stream);

/* ---- WGAN-GP critic engine helpers (trainer.py:291-332) ------------------ */

/* X [copies*N, F+K]: rows c*N+n = [mvx[n] | label_c[n]] for c = real, fake
 * (hard), mix = eps[n]*real + (1-eps[n])*soft (two products then one add, as
 * torch); copies = 4 also zeroes rows [3N, 4N) (tangent rows). */
int vg_critic_input(const float* mvx, int32_t N, int32_t F, const float* real, const float* hard,
                    const float* soft, const float* eps, int32_t K, int32_t copies, float* X,
                    void* stream);
/* The same with eps drawn in the kernel: eps[n] = the uniform vg_rng_fill
 * (kind 1) draws for element n under (seed, *iter, salt) -- trainer.py:298's
 * torch.rand(N, 1) in device-RNG mode -- so the draw needs no launch of its own. */
int vg_critic_input_drawn(const float* mvx, int32_t N, int32_t F, const float* real, const float* hard,
                          const float* soft, uint64_t seed, const int64_t* iter, uint32_t salt, int32_t K,
                          int32_t copies, float* X, void* stream);

/* From g [N,K] = dD(mix)/dlabel and the stacked scores [3N]:
 * out[1] = gp = lambda mean_n (|g_n|-1)^2, out[0] = mean(fake) - mean(real) + gp,
 * u0 [N,K] (row stride ldu) = dgp/dg.  Deterministic (per-block sums folded in
 * order by the last block).  workspace: vg_gp_head_ws_floats(N); sync: a
 * caller-owned int32 device counter, 0 on entry (left at 0).  A row's classes
 * are held in registers: K <= 32 (VG_EINVAL above; the path's K is 7). */
int64_t vg_gp_head_ws_floats(int32_t N);
int vg_gp_head(const float* g, int32_t N, int32_t K, const float* scores, float lambda, float* u0,
               int32_t ldu, float* out, float* workspace, int32_t* sync, void* stream);

/* Differentiable sparse primitives (their adjoints are each other), used to
 * build the twice-differentiable path the WGAN-GP needs (trainer.py:306-312,
 * create_graph=True):
 *   vg_spmm      Y_i = sum_{k in row i} w_k X[col_k]              [N,C]
 *   vg_spmm_t    Z_j = sum_{k: col_k = j} w_k G[dst_k]            [N,C]
 *   vg_sddmm     e_k = <A[dst_k], B[col_k]>                       [E']
 *   vg_seg_sum   s_i = sum_{k in row i} x_k                       [N]
 *   vg_seg_max   m_i = max_{k in row i} x_k                       [N]
 *   vg_gather    e_k = v[col_k] (by_src=1) or v[dst_k] (by_src=0) [E']
 *   vg_scatter_src  s_j = sum_{k: col_k = j} x_k                  [N]      */
int vg_spmm(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t channels,
            const float* w, const float* x, float* y, void* stream);
int vg_spmm_t(const int32_t* csc_ptr, const int32_t* csc_slot, const int32_t* csc_dst,
              int32_t num_nodes, int32_t channels, const float* w, const float* g, float* z,
              void* stream);
int vg_sddmm(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t channels,
             const float* a, const float* b, float* e, void* stream);
int vg_seg_sum(const int32_t* row_ptr, int32_t num_nodes, const float* x, float* s, void* stream);
int vg_seg_max(const int32_t* row_ptr, int32_t num_nodes, const float* x, float* m, void* stream);
int vg_gather(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t by_src,
              const float* v, float* e, void* stream);
int vg_scatter_src(const int32_t* csc_ptr, const int32_t* csc_slot, int32_t num_nodes,
                   const float* x, float* s, void* stream);

/* ---- GraphNorm(batch=None) + ReLU + Dropout ----------------------------- */

/* Workspace (floats) for vg_graphnorm_fwd / _bwd. */
int64_t vg_graphnorm_ws_floats(int32_t num_nodes, int32_t channels);

/* o = x - mean_scale*mu, d = sqrt(mean_rows(o^2) + eps),
 * y = keep * relu(weight * o / d + bias), with mu the column mean over all N
 * rows.  Replaces GraphNorm(x) (torch_geometric 2.6.1
 * nn/norm/graph_norm.py, batch=None) -> nn.ReLU(True) -> nn.Dropout(0.2) at
 * models.py:73-75,83-85,193-195,203-205.
 * keep (N*C, already scaled by 1/(1-p)) may be NULL (eval / no dropout).
 * stats (2C) receives [mu | d]; every function below that reads stats takes
 * d as the whole denominator (its eps argument is the statistics pass's). */
int vg_graphnorm_fwd(const float* x, int32_t num_nodes, int32_t channels, const float* weight,
                     const float* bias, const float* mean_scale, const float* keep, float eps,
                     float* y, float* stats, float* workspace, void* stream);

/* First-order backward.  g_w / g_b / g_ms are [C]. */
int vg_graphnorm_bwd(const float* x, int32_t num_nodes, int32_t channels, const float* weight,
                     const float* bias, const float* mean_scale, const float* keep, float eps,
                     const float* stats, const float* g_y, float* g_x, float* g_w, float* g_b,
                     float* g_ms, float* workspace, void* stream);

/* Segmented variants: `segments` row blocks of `rows` rows each (x is
 * [segments*rows, C]) normalise independently -- the discriminator's real /
 * fake / mix forwards of one critic iteration (trainer.py:319-320,304) run as
 * one stacked tensor.  stats is [segments][2C].  Workspace from
 * vg_graphnorm_seg_ws_floats (also valid for vg_graphnorm_jvp2 with 1). */
int64_t vg_graphnorm_seg_ws_floats(int32_t segments, int32_t rows, int32_t channels);
int vg_graphnorm_fwd_seg(const float* x, int32_t segments, int32_t rows, int32_t channels,
                         const float* weight, const float* bias, const float* mean_scale,
                         const float* keep, float eps, float* y, float* stats, float* workspace,
                         int32_t* sync, void* stream);
/* vg_graphnorm_fwd_seg with the dropout drawn in-kernel: keep = Bernoulli(1-p)
 * / (1-p) from a counter-based Philox4x32-10 keyed by seed on the counter
 * (element, salt, *iter) -- *iter is read from device memory, so a hipGraph
 * replay draws fresh masks once the caller advances it.  keep_out [S*N, C]
 * receives the multipliers for the backward (NULL: applied, not stored -- a
 * forward with no backward).  Replaces nn.Dropout(0.2)'s two
 * launches (bernoulli_, div_) at models.py:75,85,195,205. */
int vg_graphnorm_fwd_drop(const float* x, int32_t segments, int32_t rows, int32_t channels,
                          const float* weight, const float* bias, const float* mean_scale,
                          float p_drop, uint64_t seed, const int64_t* iter, uint32_t salt,
                          float eps, float* y, float* keep_out, float* stats, float* workspace,
                          int32_t* sync, void* stream);
/* vg_graphnorm_fwd_seg (iter == NULL: keep multipliers or none) or
 * vg_graphnorm_fwd_drop (iter != NULL, keep NULL) with the column statistics
 * folded from the aggregation's partials (vg_gat_aggregate_fwd_gnp over the
 * segments * rows rows with seg_rows = rows; gnp_rows = vg_gat_gnp_rows of
 * that call) instead of a pass over x: one launch fewer, x read once.  The
 * statistics differ from the chunked fold only in f32 rounding. */
int vg_graphnorm_fwd_gnp(const float* x, int32_t segments, int32_t rows, int32_t channels, const float* weight,
                         const float* bias, const float* mean_scale, const float* keep, float p_drop, uint64_t seed,
                         const int64_t* iter, uint32_t salt, float eps, float* y, float* keep_out, float* stats,
                         const float* gnp, int32_t gnp_rows, void* stream);
/* 1 when vg_graphnorm_fwd_gnp over (rows, channels, gnp_rows) runs as ONE
 * launch -- every workgroup folds its segment's partials (the narrow layers:
 * a segment's partials within the build's VG_GN_FUSE_BYTES) and applies;
 * statistics and output bit-identical to the two-launch form -- else 0.
 * Host-only. */
int32_t vg_graphnorm_fwd_gnp_fused(int32_t rows, int32_t channels, int32_t gnp_rows);
/* Backward over the segments; parameter gradients sum over segments and are
 * written (accumulate = 0) or added (1); g_w may be NULL (no parameter
 * gradients: g_b, g_ms are then ignored).  inj (nullable) is added to g_x
 * from flat element inj_offset on (the critic engine's second-order adjoint
 * of the mix copy). */
int vg_graphnorm_bwd_seg(const float* x, int32_t segments, int32_t rows, int32_t channels,
                         const float* weight, const float* bias, const float* mean_scale,
                         const float* keep, float eps, const float* stats, const float* g_y,
                         float* g_x, float* g_w, float* g_b, float* g_ms, int32_t accumulate,
                         const float* inj, int64_t inj_offset, float* workspace, int32_t* sync,
                         void* stream);
/* Tangent and second-order terms of y = GraphNormReLUDropout(x) for the
 * gradient penalty's double backward (trainer.py:306-316 with
 * create_graph=True): u_out = J u and, for Q = <g_y, J u>, x_inj = dQ/dx;
 * dQ/dweight and dQ/dmean_scale are ADDED to g_w, g_ms (dQ/dbias = 0). */
int vg_graphnorm_jvp2(const float* x, int32_t num_nodes, int32_t channels, const float* weight,
                      const float* bias, const float* mean_scale, const float* keep, float eps,
                      const float* stats, const float* u, const float* g_y, float* u_out,
                      float* x_inj, float* g_w, float* g_ms, float* workspace, int32_t* sync,
                      void* stream);

/* ---- program <-> voxel type-matched mean ("cross-graph pointer") -------- */

/* For every voxel v: out[v, col0 : col0+F] = mean of local_x rows whose
 * local_type == voxel_type[v] over the whole mini-batch, or 0 when no program
 * node has that type.  Replaces the host-synchronising loop at
 * models.py:122-129 (generator) and models.py:230-237 (discriminator).
 * out has row stride out_stride (lets the caller write straight into a
 * concatenated feature matrix).  workspace: n_types*(F+1) floats. */
int vg_type_mean(const float* local_x, const int64_t* local_type, int32_t n_local, int32_t feat,
                 const int64_t* voxel_type, int32_t n_voxel, int32_t n_types, float* out,
                 int32_t out_stride, int32_t out_col0, float* workspace, void* stream);

/* ---- Gumbel-softmax type head ------------------------------------------- */

/* soft = softmax((logits - log(noise)) / tau) per row (noise ~ Exp(1));
 * idx = first argmax; hard = (onehot(idx) - soft) + soft (straight-through).
 * Replaces F.gumbel_softmax(logits, tau=1.0) + scatter one-hot + ST at
 * models.py:150-153.  idx may be NULL. */
int vg_gumbel_fwd(const float* logits, const float* noise, int32_t rows, int32_t classes,
                  float tau, float* soft, float* hard, int32_t* idx, void* stream);

/* vg_gumbel_fwd with the temperature read from device memory: row r uses
 * tau[r / seg_rows] (a stacked inference sweep over a tau schedule, one copy of
 * the batch per temperature; a replayed hipGraph follows updates of tau). */
int vg_gumbel_fwd_dev(const float* logits, const float* noise, int32_t rows, int32_t classes,
                      const float* tau, int32_t seg_rows, float* soft, float* hard, int32_t* idx,
                      void* stream);

/* g_logits = soft * (g - sum(soft*g)) / tau with g = g_hard + g_soft (either NULL = 0). */
int vg_gumbel_bwd(const float* soft, const float* g_hard, const float* g_soft, int32_t rows,
                  int32_t classes, float tau, float* g_logits, void* stream);

/* ---- per-building reductions for the generator loss / metrics ----------- */

/* For each building g (rows ptr[g]..ptr[g+1]):
 *   far_ref[g] = x[ptr[g], far_col]
 *   far_gen[g] = sum_{argmax(label_row) != void} (x[:,dy]*dim_scale)*(x[:,dx]*dim_scale)
 *                / site_area[ptr[g]]
 * Replaces the per-graph Python loop at trainer.py:357-378. */
int vg_far_per_graph(const float* x, int32_t x_stride, const float* label, int32_t classes,
                     const int64_t* ptr, int32_t num_graphs, const float* site_area,
                     int32_t far_col, int32_t dy_col, int32_t dx_col, float dim_scale,
                     int32_t void_class, float* far_gen, float* far_ref, void* stream);

/* Generator loss of the WGAN-GP step (trainer.py:334-385; the FAR term carries
 * no gradient, :380), from the critic scores d_fake [N], label_hard / the
 * float one-hot of the true types / logits [N, classes], the true types [N]
 * and the per-building FAR pair [num_graphs] (vg_far_per_graph):
 *   out[0] = (((-mean(d_fake) l_adv + ratio) + CE l_label) + ratio_void) + far
 * and the gradient coefficients the backward needs (out has classes + 3
 * floats).  Deterministic (block partials folded in order). */
int64_t vg_gen_loss_ws_floats(int32_t N, int32_t classes);
int vg_gen_loss_fwd(const float* d_fake, const float* hard, const float* logits,
                    const float* onehot, const int64_t* type, int32_t N, int32_t classes,
                    const float* far_gen, const float* far_ref, int32_t num_graphs, float l_adv,
                    float l_label, float l_ratio, float l_void, float l_far, float* out,
                    float* workspace, void* stream);
/* d loss / d (d_fake, label_hard, logits) scaled by *g_loss (device scalar);
 * any output may be NULL (not wanted). */
int vg_gen_loss_bwd(const float* g_loss, const float* out, const float* logits,
                    const int64_t* type, int32_t N, int32_t classes, float* g_dfake, float* g_hard,
                    float* g_logits, void* stream);

/* Confusion matrices for the metrics (trainer.py:387-443): conf[g][t][p] counts
 * (truth t, prediction argmax(label_row)) per building; conf_all sums them. */
int vg_confusion(const int64_t* truth, const float* label, int32_t classes, const int64_t* ptr,
                 int32_t num_graphs, int32_t* conf, int32_t* conf_all, void* stream);

/* ---- dense layers (nn.Linear of the MLPs and the GATConv projection) ----- */

/* C[N, M] = A[N, K] . op(B) (+ bias[M]) then act (0 none, 1 ReLU, 2 LeakyReLU
 * 0.2, 3 multiply by [aux > 0] with aux [N, M] row stride ldaux -- a ReLU mask
 * applied to an adjoint or tangent; 4 add aux -- a second adjoint of the same
 * tensor summed in, as torch's add_ after the product; aux may be NULL for
 * act 0-2, and must not alias C).
 * b_trans = 1: B is [M, K] (op = transpose; the nn.Linear forward X W^T);
 * b_trans = 0: B is [K, M] (dX = dY W).  f32 MFMA (v_mfma_f32_32x32x2_f32).
 * Replaces the torch.nn.Linear GEMMs at models.py:33-47,49-66,92-113,
 * 177-185,212-220 and GATConv.lin. bias may be NULL. */
int vg_gemm(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t b_trans,
            const float* bias, int32_t act, const float* aux, int32_t ldaux, float* C,
            int32_t ldc, int32_t N, int32_t M, int32_t K, void* stream);

/* Workspace (floats) for vg_gemm_tn. */
int64_t vg_gemm_tn_ws_floats(int32_t N, int32_t M, int32_t K);

/* C[M, K] (row stride ldc) = A[N, M]^T . B[N, K] and db[M] = sum_n A[n, :]
 * (db may be NULL): the weight and bias gradients of nn.Linear, split over N
 * in row chunks, partials folded in chunk order (deterministic); written
 * (accumulate = 0) or added (1). */
int vg_gemm_tn(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
               int32_t K, float* C, int32_t ldc, float* db, int32_t accumulate,
               float* workspace, void* stream);

/* vg_gemm_tn with db summing only the first db_rows rows of A (the critic
 * engine stacks first- and second-order weight-gradient terms as extra rows
 * of one product; only the first-order rows carry a bias gradient). */
int vg_gemm_tn_ex(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                  int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows,
                  int32_t accumulate, float* workspace, void* stream);

/* ---- LayerNorm + LeakyReLU ------------------------------------------------ */

/* Y = leaky_relu(LayerNorm(A W^T + bias; gamma, beta, eps), slope) for M <= 128
 * output features in ONE launch (the LayerNorm in the GEMM epilogue; A [N, K]
 * row stride lda, W [M, K]): the [Linear -> LayerNorm -> LeakyReLU(0.2)]
 * blocks of models.py:33-47,49-66,92-113.  H (nullable) receives A W^T + bias
 * and mean / rstd [N] (nullable together) the row statistics, both for
 * vg_ln_act_bwd. */
int vg_gemm_ln_act(const float* A, int32_t lda, const float* W, int32_t N, int32_t M, int32_t K,
                   const float* bias, const float* gamma, const float* beta, float eps, float slope,
                   float* H, float* Y, float* mean, float* rstd, void* stream);


/* y = leaky_relu(LayerNorm(x; gamma, beta, eps), slope) per row of x [N, C]
 * (C <= 512): the nn.LayerNorm -> nn.LeakyReLU(0.2) pairs of the generator's
 * MLPs (models.py:33-47,49-66,92-113) in one kernel.  mean / rstd [N]
 * (nullable together) are saved for the backward. */
int vg_ln_act_fwd(const float* x, int32_t N, int32_t C, const float* gamma, const float* beta,
                  float eps, float slope, float* y, float* mean, float* rstd, void* stream);

/* Workspace (floats) for vg_ln_act_bwd. */
int64_t vg_ln_act_bwd_ws_floats(int32_t C);

/* Backward: g_x, and g_gamma / g_beta [C] written (accumulate = 0) or added. */
int vg_ln_act_bwd(const float* x, int32_t N, int32_t C, const float* gamma, const float* beta,
                  float slope, const float* mean, const float* rstd, const float* g_y, float* g_x,
                  float* g_gamma, float* g_beta, int32_t accumulate, float* workspace,
                  void* stream);

/* ---- deferred parameter-gradient folds ------------------------------------ */

/* One fold: out[(w / k) * ldo + w % k] = (accumulate ? out : 0)
 *   + sum_r src[0].part[r * src[0].ld + w] (+ the same over src[1])   for w < width,
 * partial rows summed in a fixed order (deterministic). */
typedef struct {
  const float* part;
  int32_t rows;
  int32_t ld;
} vg_fold_src;

typedef struct {
  float* out;
  int32_t width;
  int32_t k;
  int32_t ldo;
  int32_t accumulate;
  int32_t nsrc; /* 1 or 2 */
  vg_fold_src src[2];
} vg_fold;

#define VG_FOLD_MAX 120 /* the descriptors ride in the kernel arguments (~11 KB) */

/* Run up to VG_FOLD_MAX folds (a HOST array, passed to the kernel by value)
 * in one launch.  The parameter gradients of a backward are needed only by
 * the optimizer step, so the *_deferred variants below skip their own fold
 * launch and return its descriptor(s) instead; the caller keeps their
 * workspaces alive until vg_fold_batch is enqueued. */
int vg_fold_batch(const vg_fold* folds, int32_t n, void* stream);

/* vg_fold_batch, with folds of more than 768 partial rows done in two levels
 * (one fold's rows in one workgroup were the batch's long pole): the column
 * sums of each 256-row chunk land in `ws` in the same launch as the short
 * folds, then a second launch folds those sums into the destinations in the
 * same (out + src 0) + src 1 order.  `ws` (device, ws_floats floats) takes
 * vg_fold_split_ws_floats(folds, n); folds that do not fit run in one level. */
int64_t vg_fold_split_ws_floats(const vg_fold* folds, int32_t n);
int vg_fold_batch_split(const vg_fold* folds, int32_t n, float* ws, int64_t ws_floats, void* stream);

/* vg_gemm_tn_ex without its fold: writes up to 2 descriptors (C, then db when
 * non-NULL) to folds_out and their count to *n_out (host memory). */
int vg_gemm_tn_deferred(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                        int32_t M, int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows,
                        int32_t accumulate, float* workspace, vg_fold* folds_out, int32_t* n_out,
                        void* stream);

/* One planned weight-gradient product (split-K over N): part[chunk][M][K] =
 * A[chunk rows]^T B[chunk rows] (A [N,M] row stride lda, B [N,K] stride ldb)
 * and pdb[chunk][M] = column sums of A over rows < db_rows (pdb NULL: none);
 * rows per chunk a multiple of 32; bf16 != 0: bf16 operands (vg_gemm_bf16). */
typedef struct {
  const float* A;
  const float* B;
  float* part;
  float* pdb;
  int32_t lda, ldb, N, M, K, rows, chunks, db_rows, bf16;
} vg_tn;

#define VG_TN_GROUP_MAX 32

/* vg_gemm_tn_deferred that launches nothing: the product itself is described
 * in *prod_out (host memory) for vg_gemm_tn_group, its folds (C, then db when
 * non-NULL) in folds_out / *n_out.  The weight gradients of a backward are
 * read only by the optimizer step, so the trainer runs all products of one
 * backward in a single vg_gemm_tn_group launch (nn.Linear / GATConv.lin
 * weight gradients of models.py, replacing one launch per layer), then their
 * folds in vg_fold_batch.  The caller keeps A, B and workspace alive and
 * unmodified until then. */
int vg_gemm_tn_plan(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                    int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows, int32_t accumulate,
                    float* workspace, vg_tn* prod_out, vg_fold* folds_out, int32_t* n_out);
int vg_gemm_tn_plan_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                         int32_t K, float* C, int32_t ldc, float* db, int32_t db_rows, int32_t accumulate,
                         float* workspace, vg_tn* prod_out, vg_fold* folds_out, int32_t* n_out);

/* Run up to VG_TN_GROUP_MAX planned products (a HOST array, passed to the
 * kernel by value) in one launch; all of one precision.  Each writes only its
 * own part / pdb. */
int vg_gemm_tn_group(const vg_tn* prods, int32_t n, void* stream);

/* vg_gat_bwd_ex without the parameter-gradient fold: up to 3 descriptors
 * (g_bias, g_att_dst, g_att_src); none when g_att_src is NULL. */
int vg_gat_bwd_deferred(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                        const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
                        int32_t num_edges, int32_t channels, const float* h, const float* att_src,
                        const float* att_dst, const float* a_src, const float* a_dst,
                        const float* alpha, const float* g_out, float slope, float* g_h,
                        float* g_att_src, float* g_att_dst, float* g_bias, int32_t accumulate,
                        const float* inj, int32_t inj_row0, float* workspace, vg_fold* folds_out,
                        int32_t* n_out, void* stream);

/* vg_ln_act_bwd without its fold: 2 descriptors (g_gamma, g_beta). */
int vg_ln_act_bwd_deferred(const float* x, int32_t N, int32_t C, const float* gamma,
                           const float* beta, float slope, const float* mean, const float* rstd,
                           const float* g_y, float* g_x, float* g_gamma, float* g_beta,
                           int32_t accumulate, float* workspace, vg_fold* folds_out,
                           int32_t* n_out, void* stream);

/* vg_gat_jvp2_ex without its fold: 2 descriptors (g_att_dst, g_att_src), both
 * accumulating. */
int vg_gat_jvp2_deferred(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                         const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
                         int32_t num_edges, int32_t channels, const float* h, const float* u,
                         const float* g_out, const float* att_src, const float* att_dst,
                         const float* a_src, const float* a_dst, const float* alpha, float slope,
                         float* u_out, float* h_inj, float* g_att_src, float* g_att_dst,
                         const float* up_src, const float* up_dst, float* workspace,
                         vg_fold* folds_out, int32_t* n_out, void* stream);

/* The source-node pass of vg_gat_jvp2 (dQ/dh injections h_inj and the
 * att_src partials), described for a grouped launch.  shape: the pass's lane
 * layout (0-5), or -1 when vg_gat_jvp2_plan ran it already (non-vector
 * layouts). */
typedef struct {
  const int32_t* csc_ptr;
  const int32_t* csc_slot;
  const int32_t* csc_dst;
  const float* h;
  const float* u;
  const float* g_out;
  const float* att_src;
  const float* att_dst;
  const float* e_gz;
  const float* e_gzp;
  const float* e_alp;
  const float* n_gad;
  float* h_inj;
  float* part;
  int32_t N, C, blocks, shape;
} vg_jvp_src;

#define VG_JVP_GROUP_MAX 16

/* vg_gat_jvp2_deferred that launches only the destination-row pass: the
 * source pass goes to *src_out for vg_gat_jvp_src_group.  The tangent sweep
 * of the critic engine (trainer.py:306-316's double backward) reads h_inj only
 * in its later VJP pass, so the engine runs every layer's source pass in one
 * launch at the end of the sweep.  The caller keeps h, u, g_out and the
 * workspace alive and unmodified until then. */
int vg_gat_jvp2_plan(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                     const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes,
                     int32_t num_edges, int32_t channels, const float* h, const float* u,
                     const float* g_out, const float* att_src, const float* att_dst,
                     const float* a_src, const float* a_dst, const float* alpha, float slope,
                     float* u_out, float* h_inj, float* g_att_src, float* g_att_dst,
                     const float* up_src, const float* up_dst, float* workspace,
                     vg_fold* folds_out, int32_t* n_out, vg_jvp_src* src_out, void* stream);

/* Run up to VG_JVP_GROUP_MAX described source passes (a HOST array, by value)
 * in one launch; items with shape -1 are skipped by the caller. */
int vg_gat_jvp_src_group(const vg_jvp_src* items, int32_t n, void* stream);

/* ---- device RNG ------------------------------------------------------------ */

/* n draws into out: kind 0 standard normal (Box-Muller), 1 uniform [0, 1),
 * 2 Exp(1) -- the z / Gumbel noise / interpolation draws of the step
 * (trainer.py:470,484 torch.randn; models.py:150 F.gumbel_softmax; trainer.py:298
 * torch.rand) in device-RNG mode.  Counter-based Philox4x32-10 on (element
 * group, salt, *iter) with key seed, so a captured graph replays fresh draws
 * as *iter advances. */
int vg_rng_fill(float* out, int64_t n, int32_t kind, uint64_t seed, const int64_t* iter, uint32_t salt,
                void* stream);

/* ---- GraphNorm applied in the next projection's operand load --------------- */

/* The GraphNorm(+ReLU+Dropout) that ends a GATConv block, applied to the next
 * block's projection GEMM operand as it loads (models.py:73-77: module_{4b+1..3}
 * then module_{4(b+1)}.lin): stats [segments][2C] from vg_graphnorm_stats_gnp
 * (or any GraphNorm statistics pass), segments of seg_rows rows.  keep: dropout
 * multipliers [rows, C] read (iter == NULL; NULL = eval, no dropout) or drawn
 * in-kernel (iter != NULL: vg_graphnorm_fwd_drop's draws, stored to keep_out
 * when not NULL).  y != NULL receives the GraphNorm output for the backward. */
typedef struct vg_gn_apply {
  const float* stats;
  const float* weight;
  const float* bias;
  const float* mean_scale;
  const float* keep;
  float eps;
  float p_drop;
  int32_t seg_rows;
  uint32_t salt;
  uint64_t seed;
  const int64_t* iter;
  float* y;
  float* keep_out;
} vg_gn_apply;

/* vg_gat_lin_att(X = GraphNorm INPUT [N, Cin], ldx = Cin) with gn applied to
 * every element of X first: one launch and one pass over the activations
 * fewer than vg_graphnorm_fwd_gnp + vg_gat_lin_att.  H, a_src, a_dst and y are
 * bit-identical to that pair.  C <= 64 (one column tile), f32 products; other
 * shapes return VG_EINVAL (apply the GraphNorm separately). */
int vg_gat_lin_att_gn(const float* X, const float* W, int32_t N, int32_t Cin, int32_t C, const float* att_src,
                      const float* att_dst, float* H, float* a_src, float* a_dst, const vg_gn_apply* gn,
                      void* stream);
/* Only the column statistics of vg_graphnorm_fwd_gnp (the fold of the
 * aggregation's partials), for vg_gat_lin_att_gn. */
int vg_graphnorm_stats_gnp(int32_t segments, int32_t rows, int32_t channels, const float* gnp, int32_t gnp_rows,
                           const float* mean_scale, float eps, float* stats, void* stream);
/* The same column statistics from a pass over x [segments * rows, channels]
 * (vg_graphnorm_fwd_seg's statistics: ws of vg_graphnorm_seg_ws_floats), for
 * an aggregation that formed no partials. */
int vg_graphnorm_stats(const float* x, int32_t segments, int32_t rows, int32_t channels, const float* mean_scale,
                       float eps, float* stats, float* ws, void* stream);

/* ---- the tangent sweep's GraphNorm sums in the GAT tangent pass ------------ */

/* The GraphNorm (+ReLU+Dropout) whose input tangent the GAT tangent pass
 * produces (critic engine pass C): x / keep / g_y [N, C] (keep may be NULL),
 * stats [2C], parameters; part [vg_gat_jvp2_blocks(N, C)][5][C] receives the
 * per-workgroup column sums that vg_graphnorm_jvp2's first pass formed by
 * re-reading x, u, g_y and keep. */
typedef struct vg_gn_jvp {
  const float* x;
  const float* keep;
  const float* g_y;
  const float* stats;
  const float* weight;
  const float* bias;
  const float* mean_scale;
  float eps;
  float* part;
} vg_gn_jvp;

int32_t vg_gat_jvp2_blocks(int32_t num_nodes, int32_t channels);
/* vg_gat_jvp2_deferred that also writes gn->part from the tangent rows it
 * produces (u_out = the GraphNorm input tangent). */
int vg_gat_jvp2_gn_deferred(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                            const int32_t* csc_slot, const int32_t* csc_dst, int32_t num_nodes, int32_t num_edges,
                            int32_t channels, const float* h, const float* u, const float* g_out,
                            const float* att_src, const float* att_dst, const float* a_src, const float* a_dst,
                            const float* alpha, float slope, float* u_out, float* h_inj, float* g_att_src,
                            float* g_att_dst, const float* up_src_in, const float* up_dst_in, float* workspace,
                            const vg_gn_jvp* gn, vg_fold* folds_out, int32_t* n_out, void* stream);
/* vg_graphnorm_jvp2 (segments 1) from those partials: the fold and the
 * elementwise pass only.  workspace as for vg_graphnorm_jvp2. */
int vg_graphnorm_jvp2_part(const float* x, int32_t rows, int32_t channels, const float* weight, const float* bias,
                           const float* mean_scale, const float* keep, float eps, const float* stats, const float* u,
                           const float* g_y, float* u_out, float* x_inj, float* g_w, float* g_ms, const float* part,
                           int32_t blocks, float* workspace, void* stream);
/* vg_graphnorm_jvp2 as three launches the caller sequences: _sums (the
 * column-sum partials, into workspace), _fold_src (the fold, g_w / g_ms ADDED;
 * src != NULL with shape >= 0: a GAT tangent source pass described by
 * vg_gat_jvp2_plan runs in the same launch -- its injections and att_src
 * partials are read only by the later VJP pass and the folds, so it leaves
 * the tangent sweep's dependent chain), _apply (u_out, x_inj).  workspace as
 * for vg_graphnorm_jvp2 (segments 1); results bit-identical to it. */
int vg_graphnorm_jvp2_sums(const float* x, int32_t rows, int32_t channels, const float* weight, const float* bias,
                           const float* mean_scale, const float* keep, float eps, const float* stats, const float* u,
                           const float* g_y, float* workspace, void* stream);
int vg_graphnorm_jvp2_fold_src(int32_t rows, int32_t channels, const float* weight, const float* mean_scale,
                               const float* stats, float* workspace, float* g_w, float* g_ms, const vg_jvp_src* src,
                               void* stream);
int vg_graphnorm_jvp2_apply(const float* x, int32_t rows, int32_t channels, const float* weight, const float* bias,
                            const float* mean_scale, const float* keep, float eps, const float* stats, const float* u,
                            const float* g_y, float* u_out, float* x_inj, const float* workspace, void* stream);

/* ---- row-local chains of narrow linear layers ------------------------------ */

/* One layer of vg_linear_chain: y = x W^T (w_trans 0, weight [out][in], an
 * nn.Linear forward) or y = x W (w_trans 1, weight [in][out]: the adjoint of
 * an nn.Linear of weight [in][out]), + bias (NULL: none), then act 0 none,
 * 1 ReLU, 3 mask (y = aux[row][j] > 0 ? y : 0, aux [rows][ld_aux]: ReLU's
 * derivative taken from the layer's forward output); out [rows][ld_out]
 * receives y (NULL: not stored). */
typedef struct vg_chain_layer {
  const float* weight;
  const float* bias;
  const float* aux;
  float* out;
  int32_t ld_aux;
  int32_t ld_out;
  int32_t w_trans;
  int32_t act;
} vg_chain_layer;

/* nlayers (2-4) narrow linear layers applied row by row in ONE launch: the
 * critic's decoder (models.py:273-279) forward 64-32-16-8-1, its tangent
 * 64-32-16-8 and its adjoint 1-8-16-32 (vgan/critic.py passes A-D), each
 * formerly one vg_gemm launch per layer.  widths [nlayers + 1]; rows of x
 * ldx floats apart.  Other width chains return VG_EINVAL (use vg_gemm). */
int vg_linear_chain(const float* x, int32_t ldx, int32_t rows, const int32_t* widths, int32_t nlayers,
                    const vg_chain_layer* layers, void* stream);
/* The same with every product on bf16-rounded operands (inputs and weights
 * rounded to nearest-even, exact products, f32 sums): the arithmetic of the
 * *_bf16 GEMMs it replaces in bf16 mode (configs[2]). */
int vg_linear_chain_bf16(const float* x, int32_t ldx, int32_t rows, const int32_t* widths, int32_t nlayers,
                         const vg_chain_layer* layers, void* stream);

/* ---- multi-source LayerNorm GEMM (no-grad stacked generator forward) ------- */

/* One source of vg_gemm_ln_act_ms's A: `cols` columns (a multiple of 32) of
 * a row-major matrix with row stride `ld`, multiplied by W's columns
 * [w_col0, w_col0 + cols).  rows_mod: reserved, must be 0. */
typedef struct vg_asrc {
  const float* ptr;
  int32_t ld;
  int32_t cols;
  int32_t w_col0;
  int32_t rows_mod;
} vg_asrc;

/* Y = LeakyReLU(LayerNorm([A_0 | A_1 | ...] W_sel^T + bias + addend[n mod
 * add_rows])), 64 < M <= 128: the first [Linear, LayerNorm, LeakyReLU] block of
 * the generator's MLP encoder and decoder over stacked copies without
 * materialising torch.cat (models.py:131,145); the copy-invariant columns are
 * folded into `addend` (nullable, add_rows >= 32).  Y row stride ldy. */
int vg_gemm_ln_act_ms(const vg_asrc* src, int32_t nsrc, const float* W, int32_t ldw, int32_t N,
                      int32_t M, const float* bias, const float* addend, int32_t ld_add,
                      int32_t add_rows, const float* gamma, const float* beta, float eps, float slope,
                      float* Y, int32_t ldy, void* stream);

/* ---- LDS-staged aggregation (large graphs, BASELINE configs[3]) ----------- */

/* The destination CSR's sources padded to a fixed width: ell [N][width] =
 * row i's columns in CSR order, -1 past its degree (width >= the largest
 * degree).  Built once per graph (the critic's stacked copies: the same
 * width). */
int vg_csr_ell(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t width, int32_t* ell,
               void* stream);
/* vg_gat_aggregate_fwd reading each row's sources from ell (vg_csr_ell), so
 * they load without waiting for row_ptr (still read for the degree and the
 * alpha offsets); kernel shapes whose edge slots cannot hold ell_width fall
 * back to row_ptr -> col.  Bit-identical to vg_gat_aggregate_fwd. */
int vg_gat_aggregate_fwd_ell(const int32_t* row_ptr, const int32_t* col, const int32_t* ell, int32_t ell_width,
                             int32_t num_nodes, int32_t channels, const float* h, const float* a_src,
                             const float* a_dst, const float* bias, float slope, float* out, float* alpha,
                             void* stream);
/* GraphNorm statistics fused into the aggregation (the GraphNorm after every
 * GATConv, models.py:73-75,193-195; it re-read `out` for its column
 * statistics).  vg_gat_aggregate_fwd(_ell) (ell may be NULL) that also writes
 * per-workgroup Welford partials (count, mean, M2) of the output columns to
 * gnp [vg_gat_gnp_floats(N, C)]: one per workgroup of vg_gat_gnp_rows(N, C)
 * rows, segments being seg_rows-row blocks of the N rows (N % seg_rows == 0,
 * seg_rows >= vg_gat_gnp_rows).  Workgroups are segment-aligned (every
 * segment has ceil(seg_rows / gnp_rows) of its own), so a segment's partials
 * are those of a separate call over it.  vg_graphnorm_fwd_gnp folds them.
 * out and alpha are bit-identical to vg_gat_aggregate_fwd. */
int32_t vg_gat_gnp_rows(int32_t num_nodes, int32_t channels);
int64_t vg_gat_gnp_floats(int32_t num_nodes, int32_t channels);
int vg_gat_aggregate_fwd_gnp(const int32_t* row_ptr, const int32_t* col, const int32_t* ell, int32_t ell_width,
                             int32_t num_nodes, int32_t channels, const float* h, const float* a_src,
                             const float* a_dst, const float* bias, float slope, float* out, float* alpha,
                             int32_t seg_rows, float* gnp, void* stream);

/* Tile plan of a destination CSR (vg_csr_build's arrays), once per graph: for
 * every tile of 16 destination rows the sorted distinct sources of its edges
 * and each edge's slot among them.  plan: vg_gat_tile_plan_ints(N, E') int32s. */
int64_t vg_gat_tile_plan_ints(int32_t num_nodes, int32_t num_edges);
int vg_gat_tile_plan(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes,
                     int32_t num_edges, int32_t* plan_out, void* stream);

/* vg_gat_aggregate_fwd (GATConv edge softmax + gather-sum + bias,
 * models.py:144) with every tile's distinct source rows copied once into LDS
 * and gathered from there: the same results (bit for bit for C <= 128), ~2.2x
 * fewer gathered bytes on the configs[3] lattice.  C a multiple of 64; h / out 16-B aligned. */
int vg_gat_aggregate_fwd_lds(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes,
                             int32_t channels, const float* h, const float* a_src,
                             const float* a_dst, const float* bias, float slope, float* out,
                             float* alpha, const int32_t* plan, int32_t umax, void* stream);

/* Build stamp: "<hash> <compiler>" -- the first 16 hex digits of the sha256
 * of every source this library was built from (the csrc .hip and .h files and
 * this header, concatenated in sorted path order) and the hipcc version.  The
 * Python binding recomputes the hash from its tree and refuses a library
 * built from other sources. */
const char* vg_build_stamp(void);

/* Staged-tile plan (configs[3]), once per graph: for every tile of 64
 * destination rows the sorted distinct sources of its edges (at most 288) and
 * each edge's slot among them; tiles with more distinct sources, more than
 * 2048 edges or a row longer than 64 edges get count -1 (aggregated from
 * global memory).  plan: vg_gat_stage_plan_ints(N, E') int32s. */
int64_t vg_gat_stage_plan_ints(int32_t num_nodes, int32_t num_edges);
int vg_gat_stage_plan(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t num_edges,
                      int32_t* plan_out, void* stream);

/* vg_gat_aggregate_fwd (GATConv edge softmax + gather-sum + bias,
 * models.py:144) by a persistent, software-pipelined kernel that stages each
 * 64-row tile's distinct source rows in LDS while the previous tile is
 * aggregated out of it (one 1024-thread workgroup per CU).  Bit-identical to
 * vg_gat_aggregate_fwd.  C = 64 or 128; h 16-B and out 8-B aligned; plan from
 * vg_gat_stage_plan over the same CSR.  Pays off with voxels numbered in
 * lattice blocks (vgan.locality.block_order). */
int vg_gat_aggregate_fwd_staged(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t channels,
                                const float* h, const float* a_src, const float* a_dst, const float* bias,
                                float slope, float* out, float* alpha, const int32_t* plan, void* stream);

/* The same aggregation with wave-specialised workgroups (one per CU): 4 loader
 * waves fill a two-slot LDS ring with each tile's metadata and distinct
 * source rows (tiles of vg_gat_ring_tile_rows() = 64 destination rows;
 * LDS-DMA, one 64-channel slice at a time) while 12 consumer waves aggregate
 * the slots already filled out of LDS in 16-lane row groups; the slots are
 * handed over by LDS counters, no workgroup barrier.  Bit-identical to
 * vg_gat_aggregate_fwd.  C = 64 or 128; h, out, bias 16-B aligned; plan from
 * vg_gat_ring_plan over the same CSR (its tile plan: vg_gat_ring_plan_ints(N,
 * E') int32s: ucount[tiles] -- a tile's distinct sources, -1 for a tile left
 * to global memory -- then the sources and the edges' slots).  *err (a zeroed
 * int32) is left nonzero if a hand-over wait expired (the output is then
 * invalid).  The drop-in's aggregation (vgan.ops.aggregate_fwd_raw)
 * dispatches it for graphs of at least VGAN_RING_MIN_ROWS rows whose plan
 * stages most tiles (GATConv, models.py:72 via models.py:144,242). */
int64_t vg_gat_ring_plan_ints(int32_t num_nodes, int32_t num_edges);
int vg_gat_ring_plan(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t num_edges,
                     int32_t* plan_out, void* stream);
int32_t vg_gat_ring_tile_rows(void);
int vg_gat_aggregate_fwd_ring(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t channels,
                              const float* h, const float* a_src, const float* a_dst, const float* bias, float slope,
                              float* out, float* alpha, const int32_t* plan, int32_t* err, void* stream);

/* The ring aggregation with the following GraphNorm's column partials in its
 * epilogue (as vg_gat_aggregate_fwd_gnp, models.py:73-75,193-195): gnp holds
 * vg_gat_ring_gnp_floats(N, C) floats, 16-B aligned -- the partials (count,
 * mean, M2) of every 64-row tile and column in the vg_gat_aggregate_fwd_gnp
 * layout with 64-row blocks, which vg_graphnorm_stats_gnp / vg_graphnorm_fwd_gnp
 * fold with gnp_rows = vg_gat_ring_tile_rows().
 * seg_rows: the GraphNorm segment (a multiple of the tile rows dividing N). */
int64_t vg_gat_ring_gnp_floats(int32_t num_nodes, int32_t channels);
int vg_gat_aggregate_fwd_ring_gnp(const int32_t* row_ptr, const int32_t* col, int32_t num_nodes, int32_t channels,
                                  const float* h, const float* a_src, const float* a_dst, const float* bias,
                                  float slope, float* out, float* alpha, const int32_t* plan, int32_t seg_rows,
                                  float* gnp, int32_t* err, void* stream);

/* ---- GraphNorm backward partials in the producing GEMM -------------------- */

/* C[N,M] = A[N,K] B[K,M] (vg_gemm, b_trans 0, no bias / activation) is the
 * output gradient g_y of a GraphNorm(+ReLU+Dropout) over S = N / seg_rows
 * stacked segments (the critic engine's dX products, vgan/critic.py); the
 * epilogue also forms that backward's column partials -- sum gz and
 * sum gz * xhat, gz = g_y [z > 0] keep -- per 64-row tile and segment slot
 * into tpart (vg_gemm_gn_tpart_floats(N, M) floats), from gn_x / keep
 * [N, M] (keep nullable), stats [S][2M] and the GraphNorm parameters.  This
 * replaces vg_graphnorm_bwd_seg's partial pass (one launch and its re-read of
 * g_y).  seg_rows >= 64 and N a multiple of it (VG_EINVAL otherwise). */
int64_t vg_gemm_gn_tpart_floats(int32_t rows, int32_t channels);
int vg_gemm_gn_bwd(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                   int32_t K, float* C, int32_t ldc, const float* gn_x, const float* keep,
                   int32_t seg_rows, const float* weight, const float* bias, const float* mean_scale,
                   float eps, const float* stats, float* tpart, void* stream);
int vg_gemm_gn_bwd_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                        int32_t M, int32_t K, float* C, int32_t ldc, const float* gn_x,
                        const float* keep, int32_t seg_rows, const float* weight,
                        const float* bias, const float* mean_scale, float eps, const float* stats,
                        float* tpart, void* stream);

/* vg_graphnorm_bwd_seg from the partials vg_gemm_gn_bwd left in tpart (its
 * fold and apply passes only); N = seg_rows >= 64.  g_x NULL (here and in
 * vg_graphnorm_bwd_seg): the column sums only, left in the workspace at
 * vg_graphnorm_bwd_sums_offset floats ([S][2C]: sum gz | sum gz xhat) for
 * vg_gat_bwd_gn, which applies them. */
int vg_graphnorm_bwd_seg_tiles(const float* x, int32_t S, int32_t N, int32_t C, const float* weight,
                               const float* bias, const float* mean_scale, const float* keep,
                               float eps, const float* stats, const float* g_y, const float* tpart,
                               float* g_x, float* g_w, float* g_b, float* g_ms, int32_t accumulate,
                               const float* inj, int64_t inj_offset, float* ws, void* stream);
int64_t vg_graphnorm_bwd_sums_offset(int32_t segments, int32_t channels);

/* The GraphNorm(+ReLU+Dropout) backward whose output g_x is the g_out of the
 * GATConv below it (models.py:72-75 / 192-195: conv -> norm -> relu ->
 * dropout): x, keep, g_y, stats of the S stacked segments of seg_rows rows,
 * sums = the column sums of vg_graphnorm_bwd_seg(_tiles) called with g_x
 * NULL; inj (nullable) is added from flat element inj_offset on (a multiple
 * of the channel count). */
typedef struct {
  const float* x;
  const float* keep;
  const float* g_y;
  const float* inj;
  const float* weight;
  const float* bias;
  const float* mean_scale;
  const float* stats;
  const float* sums;
  float eps;
  int32_t segments, seg_rows;
  int64_t inj_offset;
} vg_gn_bwd_in;

/* vg_gat_bwd_ex / vg_gat_bwd_deferred (folds_out, n_out both NULL: folded
 * here) with g_out formed in the destination-row pass from *gn and written
 * to g_out (for the source pass and the caller): the GraphNorm backward's
 * elementwise launch and its pass over g_x disappear.  num_nodes =
 * segments * seg_rows. */
int vg_gat_bwd_gn(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr, const int32_t* csc_slot,
                  const int32_t* csc_dst, int32_t num_nodes, int32_t num_edges, int32_t channels,
                  const float* h, const float* att_src, const float* att_dst, const float* a_src,
                  const float* a_dst, const float* alpha, const vg_gn_bwd_in* gn, float* g_out, float slope,
                  float* g_h, float* g_att_src, float* g_att_dst, float* g_bias, int32_t accumulate,
                  const float* inj, int32_t inj_row0, float* workspace, vg_fold* folds_out, int32_t* n_out,
                  void* stream);

/* ---- bf16 training (BASELINE.json configs[2]) ---------------------------- */

/* The dense products of the training step with bf16 operands: the same
 * arguments, buffers (f32) and results as the functions without the suffix,
 * except that both operands of every product are rounded to bf16 (round to
 * nearest even) and multiplied on v_mfma_f32_32x32x16_bf16 with f32
 * accumulation -- what torch.autocast(dtype=torch.bfloat16) does to the
 * nn.Linear / GATConv.lin matmuls of models.py (forward, input gradient and
 * weight gradient).  Outputs, epilogues (bias, activation, LayerNorm,
 * attention projections) and bias gradients stay f32, as does every other
 * kernel of the path (aggregation, softmax, GraphNorm, losses, Adam). */
int vg_gemm_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t b_trans,
                 const float* bias, int32_t act, const float* aux, int32_t ldaux, float* C,
                 int32_t ldc, int32_t N, int32_t M, int32_t K, void* stream);
int vg_gemm_tn_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N, int32_t M,
                    int32_t K, float* C, int32_t ldc, float* db, int32_t accumulate,
                    float* workspace, void* stream);
int vg_gemm_tn_deferred_bf16(const float* A, int32_t lda, const float* B, int32_t ldb, int32_t N,
                             int32_t M, int32_t K, float* C, int32_t ldc, float* db,
                             int32_t db_rows, int32_t accumulate, float* workspace,
                             vg_fold* folds_out, int32_t* n_out, void* stream);
int vg_gemm_ln_act_bf16(const float* A, int32_t lda, const float* W, int32_t N, int32_t M, int32_t K,
                        const float* bias, const float* gamma, const float* beta, float eps,
                        float slope, float* H, float* Y, float* mean, float* rstd, void* stream);
int vg_gemm_ln_act_ms_bf16(const vg_asrc* src, int32_t nsrc, const float* W, int32_t ldw, int32_t N,
                           int32_t M, const float* bias, const float* addend, int32_t ld_add,
                           int32_t add_rows, const float* gamma, const float* beta, float eps,
                           float slope, float* Y, int32_t ldy, void* stream);
int vg_gat_lin_att_bf16(const float* x, int32_t ldx, const float* w, int32_t num_nodes,
                        int32_t c_in, int32_t c_out, const float* att_src, const float* att_dst,
                        float* h, float* a_src, float* a_dst, void* stream);

/* ---- optimiser ---------------------------------------------------------- */

/* torch.optim.Adam (single-tensor semantics, weight_decay, no amsgrad) over one
 * flat parameter buffer -- the optimizer.step() of trainer.py:481,495.
 * one_minus_beta1/2, step_size = lr / (1 - beta1^t) and bc2_sqrt =
 * sqrt(1 - beta2^t) are computed by the caller in double precision and rounded
 * to float, exactly as torch passes them to its kernels. */
int vg_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
            float beta2, float one_minus_beta1, float one_minus_beta2, float eps,
            float weight_decay, float step_size, float bc2_sqrt, void* stream);

/* Opens a training iteration in one launch: *rng_iter += 1 (the device RNG's
 * reset), *step += 1 (the count optimizer.step() increments, trainer.py:481,
 * 495) and grad[0, n) = 0 (optimizer.zero_grad(), trainer.py:475, 486).  Every
 * pointer may be NULL; grad 16-B aligned. */
int vg_iter_begin(int64_t* rng_iter, int32_t* step, float* grad, int64_t n, void* stream);

/* vg_adam with the learning rate and the (already incremented) step count
 * read from device memory, so a captured hipGraph replays correct updates. */
int vg_adam_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                double beta1, double beta2, float eps, float weight_decay, const double* lr,
                const int32_t* step, void* stream);

/* ---- f16 inference path (BASELINE.json configs[4]) ----------------------- */

/* Generator forward in IEEE binary16 for the inference sweep.  f16 buffers are
 * passed as uint16_t bit patterns; every row has a leading dimension (ld*) that
 * is a multiple of 8 halves, and a buffer's columns between its width and that
 * width rounded up to 8 hold zeros (written by the producing kernel).  K (or
 * cin) counts the A columns read and must be a multiple of 8: the caller pads
 * A with zero columns and W with zero columns to that width.  Accumulation is
 * f32; biases, LayerNorm / GraphNorm parameters and attention vectors are f32.
 * An f16 output is written over its width rounded up to 8 columns, so it may
 * be a column slice of a wider row buffer (ldo = that buffer's stride). */

/* y = act(A W^T + bias): nn.Linear (models.py:31,145 decoder head); act 0 none,
 * 1 ReLU, 2 LeakyReLU(slope); out_f32 != 0 writes f32 rows (the logits). */
int vg_hgemm(const uint16_t* a, int32_t lda, const uint16_t* w, int32_t ldw, int32_t n, int32_t m,
             int32_t k, const float* bias, int32_t act, float slope, void* out, int32_t ldo,
             int32_t out_f32, void* stream);

/* y = LeakyReLU(LayerNorm(A W^T + bias)) for m <= 128 outputs: one
 * [Linear, LayerNorm, LeakyReLU] block of the MLPs (models.py:22-31). */
int vg_hgemm_ln_act(const uint16_t* a, int32_t lda, const uint16_t* w, int32_t ldw, int32_t n,
                    int32_t m, int32_t k, const float* bias, const float* gamma, const float* beta,
                    float eps, float slope, uint16_t* out, int32_t ldo, void* stream);

/* GATConv.lin plus the attention projections (h . att_src, h . att_dst; f32)
 * in the epilogue: the f16 vg_gat_lin_att (models.py:72,82). */
int vg_hgat_lin_att(const uint16_t* x, int32_t ldx, const uint16_t* w, int32_t ldw, int32_t n,
                    int32_t cin, int32_t cout, const float* att_src, const float* att_dst,
                    uint16_t* h, int32_t ldh, float* a_src, float* a_dst, void* stream);

/* vg_hgat_lin_att whose operand x is the PREVIOUS block's aggregation output
 * (gn_channels columns, padded to cin = gn_channels rounded up to 8): its
 * GraphNorm + ReLU (models.py:73-74, eval) applied as the operand is loaded,
 * with the statistics [segments][2 gn_channels] of vg_graphnorm_stats_gnp over
 * segments x seg_rows = n rows (segments <= 16) -- the f16 values
 * vg_graphnorm_fwd_h_gnp would have stored, without the launch or the
 * [n, cin] write + read. */
/* The most segments (stacked copies) vg_hgat_lin_att_gn stages.  Host-only. */
int32_t vg_hgat_gna_max_segments(void);
int vg_hgat_lin_att_gn(const uint16_t* x, int32_t ldx, const uint16_t* w, int32_t ldw, int32_t n, int32_t cin,
                       int32_t cout, const float* att_src, const float* att_dst, uint16_t* h, int32_t ldh,
                       float* a_src, float* a_dst, const float* gn_weight, const float* gn_bias,
                       const float* gn_mean_scale, const float* stats, int32_t segments, int32_t seg_rows,
                       int32_t gn_channels, void* stream);

/* GATConv edge softmax + CSR gather-sum + bias over f16 rows of ld = c
 * rounded up to 8 channels (8 / 16 / 32 / 64 / 128): the f16
 * vg_gat_aggregate_fwd (torch_geometric GATConv.propagate, models.py:144). */
int vg_hgat_fwd(const int32_t* row_ptr, const int32_t* col, int32_t n, int32_t c, int32_t ld,
                const uint16_t* h, const float* a_src, const float* a_dst, const float* bias,
                float slope, uint16_t* out, int32_t ldo, void* stream);

/* ReLU(GraphNorm(x)) (eval: no dropout) over S stacked segments of n f16 rows
 * (models.py:73-75,83-85); statistics f32 ([S][2C] like vg_graphnorm_fwd_seg,
 * workspace vg_graphnorm_seg_ws_floats(S, N, C) floats). */
int vg_graphnorm_fwd_h(const uint16_t* x, int32_t ld, int32_t S, int32_t N, int32_t C,
                       const float* weight, const float* bias, const float* mean_scale, float eps,
                       uint16_t* y, int32_t ldy, float* stats, float* ws, void* stream);

/* vg_hgat_fwd that also writes the following GraphNorm's column partials of
 * its f16 outputs (vg_gat_aggregate_fwd_gnp's layout and segment-aligned
 * blocks: gnp [blocks][2][C][3], seg_rows the rows of one stacked copy,
 * dividing n, at least vg_hgat_gnp_rows), so vg_graphnorm_fwd_h_gnp need not
 * re-read the output: one launch fewer per block of the f16 sweep
 * (models.py:144 + 73-75). */
int32_t vg_hgat_gnp_rows(int32_t n, int32_t ld);
int64_t vg_hgat_gnp_floats(int32_t n, int32_t ld);
int vg_hgat_fwd_gnp(const int32_t* row_ptr, const int32_t* col, int32_t n, int32_t c, int32_t ld,
                    const uint16_t* h, const float* a_src, const float* a_dst, const float* bias, float slope,
                    uint16_t* out, int32_t ldo, int32_t seg_rows, float* gnp, void* stream);
/* vg_graphnorm_fwd_h with the statistics folded from vg_hgat_fwd_gnp's
 * partials (gnp_rows = vg_hgat_gnp_rows of that call). */
int vg_graphnorm_fwd_h_gnp(const uint16_t* x, int32_t ld, int32_t S, int32_t N, int32_t C,
                           const float* weight, const float* bias, const float* mean_scale, float eps,
                           uint16_t* y, int32_t ldy, float* stats, const float* gnp, int32_t gnp_rows,
                           void* stream);

/* ---- step-graph re-use (host runtime calls, no kernels) ------------------- */

/* Update the executable graph `exec` (a hipGraphExec_t) in place from the
 * recorded graph `graph` (a hipGraph_t of the same launch sequence: other
 * pointers, sizes and grid dimensions): the critic iteration Trainer.step_fresh
 * records per fresh batch (trainer.py:466-481, one iteration body).  0 on
 * success; VG_EGRAPH_TOPOLOGY when the runtime refuses the update (no error
 * state is left behind; instantiate `graph` instead). */
int vg_graph_exec_update(void* exec, void* graph);

/* hipGraphLaunch(exec, stream). */
int vg_graph_launch(void* exec, void* stream);

/* ---- the critic iteration as one native call (host orchestration) -------- */

/* The WGAN-GP critic loss and discriminator gradient of ONE critic iteration
 * -- _compute_discriminator_loss followed by d_loss.backward()
 * (trainer.py:291-332, :476-479) -- issued from C++: the same ~165 launches
 * of the same kernels, in the same order and with the same arguments, as
 * vgan/critic.py's CriticEngine.loss_and_grad in its default configuration
 * (device-drawn dropout and GP eps, GraphNorm partials from the GAT
 * aggregation and the producing GEMMs, grouped weight-gradient products and
 * deferred folds), so results are bit-identical to it.  The Python engine
 * spends ~10 us of interpreter time per launch (argument marshalling, buffer
 * allocation); this one ~1-2 us, which is what a fresh batch's recording
 * (Trainer.step_fresh) and an eager critic iteration pay.
 *
 * Model: the discriminator's parameters and their gradient buffers (views of
 * the flat buffers, fixed for the model's life).  Batch: the prepared batch
 * (vgan.data.prepared: matched voxel features, float one-hot, the single and
 * 3-copy stacked CSR / CSC / padded columns, the adjoint seeds), the labels
 * and the device-RNG draw specs.  Every temporary lives in `arena` (float
 * offsets 256-byte aligned; vg_critic_arena_floats says how many); the
 * caller keeps it alive while any recorded graph may replay launches that
 * reference it, and runs nothing else on it concurrently.  Gradients are
 * ACCUMULATED; out[0] = d_loss, out[1] = the gradient penalty. */
#define VG_CRITIC_MAX_LAYERS 8

typedef struct {
  const float* weight; /* [out][in] */
  const float* bias;   /* [out] */
  float* g_weight;
  float* g_bias;
  int32_t in, out;
} vg_critic_linear;

typedef struct {
  const float* lin_weight; /* GATConv.lin [out][in] */
  const float* att_src;
  const float* att_dst;
  const float* bias;
  float* g_lin_weight;
  float* g_att_src;
  float* g_att_dst;
  float* g_bias;
  const float* gn_weight; /* GraphNorm */
  const float* gn_bias;
  const float* gn_mean_scale;
  float* g_gn_weight;
  float* g_gn_bias;
  float* g_gn_mean_scale;
  float gn_eps, slope;
  int32_t in, out;
} vg_critic_block;

typedef struct {
  int32_t n_mlp, n_blocks, n_dec;
  int32_t bf16; /* dense products on bf16 operands (the *_bf16 entry points) */
  float lambda_gp, p_drop;
  vg_critic_linear mlp[VG_CRITIC_MAX_LAYERS];
  vg_critic_block block[VG_CRITIC_MAX_LAYERS];
  vg_critic_linear dec[VG_CRITIC_MAX_LAYERS];
} vg_critic_model;

typedef struct {
  const int32_t* row_ptr;
  const int32_t* col;
  const int32_t* csc_ptr;
  const int32_t* csc_slot;
  const int32_t* csc_dst;
  const int32_t* ell; /* NULL: none */
  int32_t num_nodes, num_edges, ell_width;
} vg_csr_ref;

typedef struct {
  int32_t n, feat, classes; /* nodes per copy, matched-feature width, K */
  const float* mvx;         /* [n][feat] */
  const float* real;        /* [n][K] float one-hot */
  const float* hard;        /* [n][K] */
  const float* soft;        /* [n][K] */
  const float* seeds4;      /* [4n]: -1/n | 1/n | 0 | 1 */
  vg_csr_ref g1;            /* the batch graph */
  vg_csr_ref g3;            /* its 3-copy block-diagonal stack (real / fake / mix) */
  uint64_t seed;            /* device RNG: seed, iteration counter, salts */
  const int64_t* iter;
  uint32_t eps_salt;
  uint32_t keep_salt[VG_CRITIC_MAX_LAYERS];
  int32_t* gp_counter; /* a zeroed int32 the GP head leaves at 0 */
} vg_critic_batch;

int64_t vg_critic_arena_floats(const vg_critic_model* model, const vg_critic_batch* batch);
int vg_critic_loss_and_grad(const vg_critic_model* model, const vg_critic_batch* batch, float* arena,
                            int64_t arena_floats, float* out, void* stream);

/* ---- one generator iteration issued from C++ ------------------------------ */

/* The generator half of the training step (trainer.py:483-491: G(z) ->
 * Gumbel labels -> D(label_hard) -> _compute_generator_loss, trainer.py:334-385
 * -> backward into G's parameters only) -- vgan/genstep.py
 * GeneratorEngine.loss_and_grad in its default configuration, issued from
 * C++: the same entry points in the same order with the same arguments and
 * the same device-RNG draws (z, G's dropout masks, the Gumbel noise, D's
 * masks), so loss, labels and gradients are bit-identical to the Python
 * engine's; the host pays ~1-2 us per launch instead of ~10 (the generator
 * iteration of a fresh batch runs eagerly).  G's gradients are ACCUMULATED
 * into the g_* buffers; D's g_* fields are not read.  Every temporary lives in
 * `arena` (vg_gen_arena_floats floats, 256-byte aligned), the same contract as
 * vg_critic_loss_and_grad's. */
#define VG_GEN_MAX_LAYERS 8
#define VG_GEN_MAX_BLOCKS 32

/* [Linear -> LayerNorm -> LeakyReLU] (models.py:33-47,49-66,92-113) */
typedef struct {
  const float* weight; /* [out][in] */
  const float* bias;
  const float* ln_weight;
  const float* ln_bias;
  float* g_weight;
  float* g_bias;
  float* g_ln_weight;
  float* g_ln_bias;
  float ln_eps, slope;
  int32_t in, out;
} vg_gen_ln_layer;

typedef struct {
  int32_t n_mfe, n_mlp, n_gblocks, n_dec;   /* G: matched-features encoder, MLP encoder, GAT blocks, decoder */
  int32_t n_dmlp, n_dblocks, n_ddec;        /* D: MLP encoder, GAT blocks, decoder */
  int32_t bf16;                             /* dense products on bf16 operands */
  float tau, p_drop_g, p_drop_d;
  float lambda_adv, lambda_label, lambda_ratio, lambda_void, lambda_far;
  float dim_scale;
  int32_t void_class;
  vg_gen_ln_layer mfe[VG_GEN_MAX_LAYERS];
  vg_gen_ln_layer mlp[VG_GEN_MAX_LAYERS];
  vg_critic_block gblock[VG_GEN_MAX_BLOCKS];
  vg_gen_ln_layer dec[VG_GEN_MAX_LAYERS];
  vg_critic_linear dec_last; /* the decoder's last Linear (logits) */
  vg_critic_linear dmlp[VG_GEN_MAX_LAYERS];
  vg_critic_block dblock[VG_GEN_MAX_BLOCKS];
  vg_critic_linear ddec[VG_GEN_MAX_LAYERS];
} vg_gen_model;

typedef struct {
  int32_t n, classes;             /* voxel nodes, K */
  int32_t mx_w, vx_w, mvx_w, z_dim; /* widths of matched_x, voxel.x, matched_voxel_x, z */
  const float* mx;                /* [n][mx_w] type-matched program features (the generator's) */
  const float* vx;                /* [n][vx_w] voxel features */
  const float* mvx;               /* [n][mvx_w] the discriminator's matched features */
  const float* onehot;            /* [n][K] float one-hot of the true types */
  const int64_t* type;            /* [n] true types */
  const int64_t* graph_ptr;       /* [num_graphs + 1] building row offsets */
  const float* site_area;         /* per node (read at each building's first row) */
  int32_t num_graphs, far_col, dy_col, dx_col;
  vg_csr_ref g;                   /* the batch graph (ell optional) */
  int32_t seg_rows;               /* GraphNorm segment rows of the aggregation partials (= n) */
  int32_t* sync;                  /* vg_graphnorm_bwd_seg's counter */
  const float* one;               /* device 1.0f: the loss's seed */
  uint64_t seed;                  /* device RNG: seed, iteration counter, salts */
  const int64_t* iter;
  uint32_t z_salt, noise_salt;
  uint32_t g_keep_salt[VG_GEN_MAX_BLOCKS];
  uint32_t d_keep_salt[VG_GEN_MAX_BLOCKS];
} vg_gen_batch;

int64_t vg_gen_arena_floats(const vg_gen_model* model, const vg_gen_batch* batch);
/* out [classes + 3]: vg_gen_loss_fwd's (out[0] = the generator loss); hard
 * [n][classes]: label_hard. */
int vg_gen_loss_and_grad(const vg_gen_model* model, const vg_gen_batch* batch, float* arena, int64_t arena_floats,
                         float* out, float* hard, void* stream);

/* ---- the f16 inference-sweep forward as one native call (configs[4]) ----- */

/* One batch of the configs[4] sweep -- InferenceSweep._forward with the f16
 * generator (vgan/half.py HalfGenerator.logits + the Gumbel head + argmax;
 * the eval forward of models.py:119-155 stacked over `copies` temperatures,
 * trainer.py:749-806 sampling) -- issued from C++: the same f16 kernels in
 * the same order with the same arguments, so the labels are bit-identical to
 * the Python path's; the per-launch host cost (~10 us of interpreter time and
 * one torch allocation per temporary there) drops to ~1-2 us, so a sweep of
 * distinct batches is bound by the device instead of the host.
 *
 * Model: the f16 weight images HalfGenerator.refresh builds (rows padded to
 * multiples of 8 halves) and the f32 vectors.  Batch: the prepared batch's
 * voxel features and type-matched program features (f32, one copy), its CSR
 * (one copy: the engine stacks `copies` block-diagonal copies itself), the
 * per-copy temperatures on the device, and the device-RNG draw spec of z and
 * of the Gumbel noise (vg_rng_fill kinds 0 and 2; advance_iter != 0 first
 * adds 1 to *iter, the RNG's reset).  labels [copies * n] int8 (the argmax
 * class of every voxel of every copy); logits [copies * n][classes] f32 is
 * optional (NULL: kept in the arena).  Temporaries live in `arena`
 * (vg_hgen_arena_bytes, 256-byte aligned). */
#define VG_HGEN_MAX_LAYERS 8
#define VG_HGEN_MAX_BLOCKS 32

typedef struct {
  const uint16_t* weight; /* [out][ldw] f16, ldw = in rounded up to 8 (zero pad) */
  int32_t ldw;
  const float* bias;
  const float* gamma; /* LayerNorm (NULL for the decoder head) */
  const float* beta;
  float eps, slope;
  int32_t in, out;
} vg_hgen_linear;

typedef struct {
  const uint16_t* lin_weight; /* GATConv.lin [out][ldw] f16 */
  int32_t ldw;
  const float* att_src;
  const float* att_dst;
  const float* bias;
  float slope;
  const float* gn_weight; /* GraphNorm */
  const float* gn_bias;
  const float* gn_mean_scale;
  float gn_eps;
  int32_t in, out;
} vg_hgen_block;

typedef struct {
  int32_t n_matched, n_mlp, n_blocks, n_dec;
  vg_hgen_linear matched[VG_HGEN_MAX_LAYERS]; /* matched-feature encoder */
  vg_hgen_linear mlp[VG_HGEN_MAX_LAYERS];     /* MLP encoder over [em | voxel.x | z] */
  vg_hgen_block block[VG_HGEN_MAX_BLOCKS];    /* GAT encoder */
  vg_hgen_linear dec[VG_HGEN_MAX_LAYERS];     /* decoder [Linear, LayerNorm, LeakyReLU] blocks */
  vg_hgen_linear head;                        /* decoder head (f32 logits) */
} vg_hgen_model;

typedef struct {
  int32_t n, copies;                    /* voxel nodes per copy, stacked copies (temperatures) */
  int32_t voxel_dim, matched_dim, z_dim, num_edges;
  const float* voxel_x;                 /* [n][voxel_dim] */
  const float* matched_x;               /* [n][matched_dim] */
  const int32_t* row_ptr;               /* [n + 1], self loops included (vgan.ops.CSR) */
  const int32_t* col;                   /* [num_edges] */
  const float* taus;                    /* [copies] */
  uint64_t seed;
  int64_t* iter;
  int32_t advance_iter;
  uint32_t z_salt, noise_salt;
} vg_hgen_batch;

int64_t vg_hgen_arena_bytes(const vg_hgen_model* model, const vg_hgen_batch* batch);
int vg_hgen_sweep(const vg_hgen_model* model, const vg_hgen_batch* batch, void* arena, int64_t arena_bytes,
                  int8_t* labels, float* logits, void* stream);

/* The same forward as ONE hipGraph launch: vg_hgen_sweep's launches captured
 * (thread-local stream capture) into a graph that updates one of two
 * alternating executable graphs in place (re-instantiated only when the
 * update is refused), after the event behind that executable graph's
 * previous launch has completed.  Same results bit for bit.  A handle holds
 * the two executable graphs; vg_hgen_graph_stats reports how many were
 * instantiated and how many updated in place.  A handle belongs to the device
 * current at vg_hgen_graph_create (its capture stream's); vg_hgen_sweep_graphed
 * returns VG_EINVAL when another device is current.  vg_hgen_arena_bytes
 * returns a negative code for invalid arguments. */
void* vg_hgen_graph_create(void);
void vg_hgen_graph_destroy(void* handle);
int vg_hgen_graph_stats(const void* handle, int32_t* instantiations, int32_t* updates);
int vg_hgen_sweep_graphed(void* handle, const vg_hgen_model* model, const vg_hgen_batch* batch, void* arena,
                          int64_t arena_bytes, int8_t* labels, float* logits, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VGAN_H_ */
