// The configs[4] inference-sweep forward of one batch issued from C++:
// vg_hgen_sweep (include/vgan.h).
//
// A restatement of vgan/infer.py InferenceSweep._forward on the f16 generator
// (vgan/half.py HalfGenerator.logits, then the Gumbel head and the argmax):
// the eval forward of models.py:119-155 over `copies` stacked copies of the
// batch, one per Gumbel temperature (trainer.py:749-806 samples with the
// generator in eval mode).  Every dense / GAT / GraphNorm / head launch is the
// library's own extern "C" entry point with the arguments the Python path
// passes, in its order, so the labels are bit-identical to it.  What the
// Python path did with torch ops -- the f16 row buffer's columns (voxel
// features, z, zero pad), the program-feature encoder's input, the broadcast
// of its output over the copies, the block-diagonal stacked CSR, the int8
// labels -- is done by the three small kernels below; their values are the
// same (f32 -> f16 round-to-nearest-even, integer offsets).
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <algorithm>
#include <new>

#include "../../include/vgan.h"
#include "common.h"

namespace {

inline int r8(int c) { return (c + 7) / 8 * 8; }

// f16 row buffer columns from up to three sources: dst[r][col0 + j] =
// half(src[r % src_rows][j]) for j < w, 0 for j in [w, zero_to); sources f32
// (is_f16 = 0) or f16 bit patterns (is_f16 = 1).
struct PackSrc {
  const void* src;
  int ld, w, src_rows, col0, zero_to, is_f16;
};
struct PackDesc {
  PackSrc s[3];
  int ns;
  uint16_t* dst;
  int ldd, rows;
};

__global__ void k_hg_pack(const PackDesc d) {
  const int q = blockIdx.y;
  if (q >= d.ns) return;
  const PackSrc& p = d.s[q];
  const int span = p.zero_to > p.w ? p.zero_to : p.w;
  const long long total = (long long)d.rows * span;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int r = static_cast<int>(t / span), j = static_cast<int>(t - (long long)r * span);
    const int sr = r % p.src_rows;
    uint16_t v = 0;
    if (j < p.w) {
      if (p.is_f16) {
        v = static_cast<const uint16_t*>(p.src)[(size_t)sr * p.ld + j];
      } else {
        const __half h = __float2half_rn(static_cast<const float*>(p.src)[(size_t)sr * p.ld + j]);
        v = __half_as_ushort(h);
      }
    }
    d.dst[(size_t)r * d.ldd + p.col0 + j] = v;
  }
}

// The same packing four columns a thread (one 8-B store) when every source's
// col0 and span and the row stride are multiples of 4 (the sweep's row
// buffer: em at 256, voxel.x at 384, z at 396 of 528): a quarter of the
// integer divisions and stores of k_hg_pack; the same bits.
__global__ void k_hg_pack4(const PackDesc d) {
  const int q = blockIdx.y;
  if (q >= d.ns) return;
  const PackSrc& p = d.s[q];
  const int span4 = (p.zero_to > p.w ? p.zero_to : p.w) / 4;
  const long long total = (long long)d.rows * span4;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < total;
       t += (long long)gridDim.x * blockDim.x) {
    const int r = static_cast<int>(t / span4), j0 = 4 * static_cast<int>(t - (long long)r * span4);
    const int sr = r % p.src_rows;
    uint16_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int j = j0 + k;
      v[k] = 0;
      if (j < p.w) {
        if (p.is_f16) {
          v[k] = static_cast<const uint16_t*>(p.src)[(size_t)sr * p.ld + j];
        } else {
          const __half h = __float2half_rn(static_cast<const float*>(p.src)[(size_t)sr * p.ld + j]);
          v[k] = __half_as_ushort(h);
        }
      }
    }
    *reinterpret_cast<uint2*>(d.dst + (size_t)r * d.ldd + p.col0 + j0) =
        make_uint2(v[0] | (static_cast<uint32_t>(v[1]) << 16), v[2] | (static_cast<uint32_t>(v[3]) << 16));
  }
}

// k_hg_pack4 when the layout allows it, else k_hg_pack (both grids y = sources)
int hg_pack(const PackDesc& d, long long work, hipStream_t s);

// block-diagonal stack of `copies` copies of a destination CSR (vgan.ops
// CSR.stacked: node ids offset by c * n, edge slots by c * e)
__global__ void k_hg_stack_csr(const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col, int n, int e,
                               int copies, int32_t* __restrict__ rp_out, int32_t* __restrict__ col_out) {
  const long long nr = (long long)copies * n + 1, ne = (long long)copies * e;
  for (long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x; t < nr + ne;
       t += (long long)gridDim.x * blockDim.x) {
    if (t < nr) {
      const int c = static_cast<int>(t / n), i = static_cast<int>(t - (long long)c * n);
      rp_out[t] = t == nr - 1 ? static_cast<int32_t>(ne) : row_ptr[i] + c * e;
    } else {
      const long long k = t - nr;
      const int c = static_cast<int>(k / e), j = static_cast<int>(k - (long long)c * e);
      col_out[k] = col[j] + c * n;
    }
  }
}

// RNG.reset() (vgan/rng.py): the device iteration counter + 1; the argmax
// classes as int8 (hard = onehot(idx) - soft + soft has its maximum at idx)
__global__ void k_hg_tail(int64_t* __restrict__ iter, const int32_t* __restrict__ idx, int8_t* __restrict__ out,
                          int rows) {
  if (iter) {  // the counter step, one lane (launched before the draws)
    if (blockIdx.x == 0 && threadIdx.x == 0) *iter += 1;
    return;
  }
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r < rows) out[r] = static_cast<int8_t>(idx[r]);
}

struct Arena {
  bool dry;
  char* base;
  int64_t off = 0;
  template <class T>
  T* take(int64_t count) {
    const int64_t at = off;
    off += (std::max<int64_t>(count * (int64_t)sizeof(T), 1) + 255) / 256 * 256;
    return dry ? nullptr : reinterpret_cast<T*>(base + at);
  }
};

#define VG_RUN(expr)                  \
  do {                                \
    if (!ar.dry) {                    \
      const int _rc = (expr);         \
      if (_rc) return _rc;            \
    }                                 \
  } while (0)

int launched() { return static_cast<int>(hipGetLastError()); }


int blocks_for(long long work) {
  const long long b = (work + 255) / 256;
  return static_cast<int>(std::min<long long>(std::max<long long>(b, 1), 4096));
}

#ifndef VG_HG_PACK4
#define VG_HG_PACK4 1
#endif

int hg_pack(const PackDesc& d, long long work, hipStream_t s) {
  bool quad = VG_HG_PACK4 && d.ldd % 4 == 0 && (reinterpret_cast<uintptr_t>(d.dst) & 7) == 0;
  for (int q = 0; q < d.ns; ++q) {
    const int span = d.s[q].zero_to > d.s[q].w ? d.s[q].zero_to : d.s[q].w;
    quad = quad && d.s[q].col0 % 4 == 0 && span % 4 == 0;
  }
  if (quad)
    k_hg_pack4<<<dim3(blocks_for(work / 4), d.ns), 256, 0, s>>>(d);
  else
    k_hg_pack<<<dim3(blocks_for(work), d.ns), 256, 0, s>>>(d);
  return launched();
}

// HalfGenerator._run_mlp: the blocks over `rows` rows of a (stride lda); the
// last writes into last_out (stride last_ld) when given
int run_mlp(Arena& ar, hipStream_t s, const vg_hgen_linear* L, int nl, const uint16_t* a, int lda, int k_in, int rows,
            uint16_t* last_out, int last_ld, const uint16_t** out_a, int* out_ld) {
  int k = k_in;
  for (int j = 0; j < nl; ++j) {
    if (r8(L[j].in) != r8(k)) return VG_EINVAL;
    uint16_t* out;
    int ldo;
    if (j == nl - 1 && last_out) {
      out = last_out;
      ldo = last_ld;
    } else {
      ldo = r8(L[j].out);
      out = ar.take<uint16_t>((int64_t)rows * ldo);
    }
    VG_RUN(vg_hgemm_ln_act(a, lda, L[j].weight, L[j].ldw, rows, L[j].out, r8(L[j].in), L[j].bias, L[j].gamma,
                           L[j].beta, L[j].eps, L[j].slope, out, ldo, s));
    a = out;
    lda = ldo;
    k = L[j].out;
  }
  *out_a = a;
  *out_ld = lda;
  return 0;
}

int run(Arena& ar, const vg_hgen_model* md, const vg_hgen_batch* bt, int8_t* labels, float* logits_out,
        hipStream_t s) {
  const int n = bt->n, kk = bt->copies, rows = kk * n;
  const int nm = md->n_matched, nl = md->n_mlp, nb = md->n_blocks, nd = md->n_dec;
  if (n <= 0 || kk <= 0 || nm < 1 || nl < 1 || nb < 1 || nd < 1 || nm > VG_HGEN_MAX_LAYERS ||
      nl > VG_HGEN_MAX_LAYERS || nb > VG_HGEN_MAX_BLOCKS || nd > VG_HGEN_MAX_LAYERS || !md->head.weight ||
      bt->num_edges <= 0 || (long long)kk * n > (1LL << 30) || (long long)kk * bt->num_edges > (1LL << 30))
    return VG_EINVAL;
  if (!ar.dry && (!bt->voxel_x || !bt->matched_x || !bt->row_ptr || !bt->col || !bt->taus || !bt->iter || !labels))
    return VG_EINVAL;
  const int hl = md->matched[nm - 1].out, hg = md->mlp[nl - 1].out, enc_c = md->block[nb - 1].out;
  const int vd = bt->voxel_dim, zd = bt->z_dim, fl = bt->matched_dim;
  // row buffer [enc | x | em | voxel.x | z | pad] (models.py:145 order)
  const int o_x = enc_c, o_em = enc_c + hg, o_vx = o_em + hl, o_z = o_vx + vd, width = o_z + zd;
  const int ld = r8(width);

  // RNG.reset(), then z [copies, n, z_dim] (RNG.normal, salt z_salt)
  if (bt->advance_iter) {
    VG_RUN((k_hg_tail<<<1, 64, 0, s>>>(bt->iter, nullptr, nullptr, 0), launched()));
  }
  float* z = ar.take<float>((int64_t)rows * zd);
  VG_RUN(vg_rng_fill(z, (int64_t)rows * zd, 0, bt->seed, bt->iter, bt->z_salt, s));
  uint16_t* buf = ar.take<uint16_t>((int64_t)rows * ld);
  uint16_t* a0 = ar.take<uint16_t>((int64_t)n * r8(fl));
  {
    PackDesc d{};
    d.dst = buf;
    d.ldd = ld;
    d.rows = rows;
    d.s[0] = PackSrc{bt->voxel_x, vd, vd, n, o_vx, vd, 0};
    d.s[1] = PackSrc{z, zd, zd, rows, o_z, ld - o_z, 0};  // z, then the zero pad columns
    d.ns = 2;
    VG_RUN(hg_pack(d, (long long)rows * (ld - o_z), s));
    PackDesc e{};
    e.dst = a0;
    e.ldd = r8(fl);
    e.rows = n;
    e.s[0] = PackSrc{bt->matched_x, fl, fl, n, 0, r8(fl), 0};
    e.ns = 1;
    VG_RUN(hg_pack(e, (long long)n * r8(fl), s));
  }
  // program-feature encoder once on n rows, broadcast into every copy
  const uint16_t* em;
  int ld_em;
  if (const int rc = run_mlp(ar, s, md->matched, nm, a0, r8(fl), fl, n, nullptr, 0, &em, &ld_em)) return rc;
  {
    PackDesc d{};
    d.dst = buf;
    d.ldd = ld;
    d.rows = rows;
    d.s[0] = PackSrc{em, ld_em, hl, n, o_em, hl, 1};
    d.ns = 1;
    VG_RUN(hg_pack(d, (long long)rows * hl, s));
  }
  // MLP encoder: reads [em | voxel.x | z] in place, writes x into its slice
  {
    const uint16_t* xo;
    int ldxo;
    if (const int rc = run_mlp(ar, s, md->mlp, nl, ar.dry ? nullptr : buf + o_em, ld, width - o_em, rows,
                               ar.dry ? nullptr : buf + o_x, ld, &xo, &ldxo))
      return rc;
  }
  // GAT encoder over the stacked block-diagonal graph
  const int32_t* rp = bt->row_ptr;
  const int32_t* cl = bt->col;
  if (kk > 1) {
    int32_t* rps = ar.take<int32_t>((int64_t)rows + 1);
    int32_t* cls = ar.take<int32_t>((int64_t)kk * bt->num_edges);
    VG_RUN((k_hg_stack_csr<<<blocks_for((long long)rows + 1 + (long long)kk * bt->num_edges), 256, 0, s>>>(
                bt->row_ptr, bt->col, n, bt->num_edges, kk, rps, cls),
            launched()));
    rp = rps;
    cl = cls;
  }
  const uint16_t* x = buf + o_x;
  int ldx = ld;
  // a block's GraphNorm + ReLU applied by the next block's projection
  // (vg_hgat_lin_att_gn) when its statistics come from the aggregation's
  // partials; the last block's stored -- half.py's choices
  struct Pend {
    const uint16_t* agg;
    int ld;
    const vg_hgen_block* blk;
    const float* stats;
  } pend{nullptr, 0, nullptr, nullptr};
  for (int b = 0; b < nb; ++b) {
    const vg_hgen_block& B = md->block[b];
    const int cout = B.out, ldh = r8(cout);
    uint16_t* h = ar.take<uint16_t>((int64_t)rows * ldh);
    float* a_s = ar.take<float>(rows);
    float* a_d = ar.take<float>(rows);
    if (pend.agg) {
      const vg_hgen_block& P = *pend.blk;
      VG_RUN(vg_hgat_lin_att_gn(pend.agg, pend.ld, B.lin_weight, B.ldw, rows, r8(B.in), cout, B.att_src, B.att_dst, h,
                                ldh, a_s, a_d, P.gn_weight, P.gn_bias, P.gn_mean_scale, pend.stats, kk, n, P.out, s));
      pend = Pend{nullptr, 0, nullptr, nullptr};
    } else {
      VG_RUN(vg_hgat_lin_att(x, ldx, B.lin_weight, B.ldw, rows, r8(B.in), cout, B.att_src, B.att_dst, h, ldh, a_s,
                             a_d, s));
    }
    uint16_t* agg = ar.take<uint16_t>((int64_t)rows * ldh);
    // the GraphNorm's column partials from the aggregation's epilogue when one
    // copy spans a partial block
    const int g = vg_hgat_gnp_rows(rows, ldh);
    float* gnp = g > 0 && g <= n ? ar.take<float>(vg_hgat_gnp_floats(rows, ldh)) : nullptr;
    if (gnp)
      VG_RUN(vg_hgat_fwd_gnp(rp, cl, rows, cout, ldh, h, a_s, a_d, B.bias, B.slope, agg, ldh, n, gnp, s));
    else
      VG_RUN(vg_hgat_fwd(rp, cl, rows, cout, ldh, h, a_s, a_d, B.bias, B.slope, agg, ldh, s));
    float* stats = ar.take<float>((int64_t)kk * 2 * cout);
    if (gnp && b < nb - 1 && kk <= vg_hgat_gna_max_segments()) {
      VG_RUN(vg_graphnorm_stats_gnp(kk, n, cout, gnp, g, B.gn_mean_scale, B.gn_eps, stats, s));
      pend = Pend{agg, ldh, &B, stats};
      continue;
    }
    uint16_t* y;
    int ldy;
    if (b == nb - 1) {  // the last block writes enc into columns [0, enc_c)
      y = buf;
      ldy = ld;
    } else {
      y = ar.take<uint16_t>((int64_t)rows * ldh);
      ldy = ldh;
    }
    if (gnp) {
      VG_RUN(vg_graphnorm_fwd_h_gnp(agg, ldh, kk, n, cout, B.gn_weight, B.gn_bias, B.gn_mean_scale, B.gn_eps, y, ldy,
                                    stats, gnp, g, s));
    } else {
      float* ws = ar.take<float>(vg_graphnorm_seg_ws_floats(kk, n, cout));
      VG_RUN(vg_graphnorm_fwd_h(agg, ldh, kk, n, cout, B.gn_weight, B.gn_bias, B.gn_mean_scale, B.gn_eps, y, ldy, stats,
                                ws, s));
    }
    x = y;
    ldx = ldy;
  }
  // decoder over the whole row buffer, f32 logits
  const uint16_t* dd;
  int ldd;
  if (const int rc = run_mlp(ar, s, md->dec, nd, buf, ld, width, rows, nullptr, 0, &dd, &ldd)) return rc;
  const vg_hgen_linear& H = md->head;
  const int K = H.out;
  float* logits = ar.take<float>((int64_t)rows * K);  // (sized either way: one arena size per batch shape)
  if (logits_out) logits = logits_out;
  VG_RUN(vg_hgemm(dd, ldd, H.weight, H.ldw, rows, K, r8(H.in), H.bias, 0, 0.f, logits, K, 1, s));
  // Gumbel head at each copy's temperature (RNG.exponential, salt noise_salt)
  float* noise = ar.take<float>((int64_t)rows * K);
  VG_RUN(vg_rng_fill(noise, (int64_t)rows * K, 2, bt->seed, bt->iter, bt->noise_salt, s));
  float* soft = ar.take<float>((int64_t)rows * K);
  float* hard = ar.take<float>((int64_t)rows * K);
  int32_t* idx = ar.take<int32_t>(rows);
  VG_RUN(vg_gumbel_fwd_dev(logits, noise, rows, K, bt->taus, n, soft, hard, idx, s));
  VG_RUN((k_hg_tail<<<(rows + 255) / 256, 256, 0, s>>>(nullptr, idx, labels, rows), launched()));
  return 0;
}

}  // namespace

extern "C" int64_t vg_hgen_arena_bytes(const vg_hgen_model* model, const vg_hgen_batch* batch) {
  if (!model || !batch) return VG_EINVAL;  // negative: an error, never a size
  Arena ar{true, nullptr};
  const int rc = run(ar, model, batch, nullptr, nullptr, nullptr);
  return rc ? (rc < 0 ? rc : -rc) : ar.off;
}

extern "C" int vg_hgen_sweep(const vg_hgen_model* model, const vg_hgen_batch* batch, void* arena, int64_t arena_bytes,
                             int8_t* labels, float* logits, void* stream) {
  if (!model || !batch || !arena) return VG_EINVAL;
  const int64_t need = vg_hgen_arena_bytes(model, batch);
  if (need < 0) return static_cast<int>(need);
  if (arena_bytes < need || (reinterpret_cast<uintptr_t>(arena) & 255)) return VG_EINVAL;
  Arena ar{false, static_cast<char*>(arena)};
  return run(ar, model, batch, labels, logits, static_cast<hipStream_t>(stream));
}

// ---------------------------------------------------------------- graphed
// The same batch forward CAPTURED into a hipGraph (stream capture of run()
// on a private stream -- capturing records, it runs nothing, and the caller's
// stream may be the legacy one, which cannot capture; thread-local mode:
// other host threads' uploads are unaffected) and launched on the caller's
// stream as one graph.  Two executable graphs alternate; each is updated in place
// from the new capture (hipGraphExecUpdate: same launch sequence, new
// pointers and grid sizes) and re-instantiated only when the update is
// refused, and only after the event behind its previous launch -- two
// batches back -- has completed.
#define VG_HIP_RET(expr)                                    \
  do {                                                      \
    const hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return static_cast<int>(_e);      \
  } while (0)

namespace {
struct HgenGraph {
  hipGraphExec_t exec[2] = {nullptr, nullptr};
  hipEvent_t done[2] = {nullptr, nullptr};
  hipStream_t cap = nullptr;
  bool used[2] = {false, false};
  int next = 0;
  int dev = -1;  // the device current at creation: the capture stream's
  int32_t instantiations = 0, updates = 0;
};
}  // namespace

extern "C" void vg_hgen_graph_destroy(void* handle);

extern "C" void* vg_hgen_graph_create(void) {
  HgenGraph* g = new (std::nothrow) HgenGraph();
  if (!g) return nullptr;
  bool ok = hipGetDevice(&g->dev) == hipSuccess && hipStreamCreateWithFlags(&g->cap, hipStreamNonBlocking) == hipSuccess;
  for (int i = 0; ok && i < 2; ++i) ok = hipEventCreateWithFlags(&g->done[i], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    vg_hgen_graph_destroy(g);
    return nullptr;
  }
  return g;
}

extern "C" void vg_hgen_graph_destroy(void* handle) {
  HgenGraph* g = static_cast<HgenGraph*>(handle);
  if (!g) return;
  for (int i = 0; i < 2; ++i) {
    if (g->used[i]) (void)hipEventSynchronize(g->done[i]);
    if (g->exec[i]) (void)hipGraphExecDestroy(g->exec[i]);
    if (g->done[i]) (void)hipEventDestroy(g->done[i]);
  }
  if (g->cap) (void)hipStreamDestroy(g->cap);
  delete g;
}

extern "C" int vg_hgen_graph_stats(const void* handle, int32_t* instantiations, int32_t* updates) {
  const HgenGraph* g = static_cast<const HgenGraph*>(handle);
  if (!g || !instantiations || !updates) return VG_EINVAL;
  *instantiations = g->instantiations;
  *updates = g->updates;
  return 0;
}

extern "C" int vg_hgen_sweep_graphed(void* handle, const vg_hgen_model* model, const vg_hgen_batch* batch,
                                     void* arena, int64_t arena_bytes, int8_t* labels, float* logits,
                                     void* stream) {
  HgenGraph* G = static_cast<HgenGraph*>(handle);
  if (!G || !model || !batch || !arena) return VG_EINVAL;
  int cur = -1;  // captured on the handle's stream, launched on the caller's: one device for both
  if (hipGetDevice(&cur) != hipSuccess || cur != G->dev) return VG_EINVAL;
  const int64_t need = vg_hgen_arena_bytes(model, batch);
  if (need < 0) return static_cast<int>(need);
  if (arena_bytes < need || (reinterpret_cast<uintptr_t>(arena) & 255)) return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int slot = G->next;
  if (G->used[slot]) VG_HIP_RET(hipEventSynchronize(G->done[slot]));
  VG_HIP_RET(hipStreamBeginCapture(G->cap, hipStreamCaptureModeThreadLocal));
  Arena ar{false, static_cast<char*>(arena)};
  const int rc = run(ar, model, batch, labels, logits, G->cap);
  hipGraph_t graph = nullptr;
  const hipError_t ec = hipStreamEndCapture(G->cap, &graph);
  if (rc || ec != hipSuccess || !graph) {
    if (graph) (void)hipGraphDestroy(graph);
    (void)hipGetLastError();
    return rc ? rc : static_cast<int>(ec != hipSuccess ? ec : hipErrorStreamCaptureInvalidated);
  }
  bool updated = false;
  if (G->exec[slot]) {
    hipGraphNode_t err_node = nullptr;
    hipGraphExecUpdateResult res = hipGraphExecUpdateError;
    if (hipGraphExecUpdate(G->exec[slot], graph, &err_node, &res) == hipSuccess && res == hipGraphExecUpdateSuccess) {
      updated = true;
      ++G->updates;
    } else {
      (void)hipGetLastError();
      (void)hipGraphExecDestroy(G->exec[slot]);
      G->exec[slot] = nullptr;
    }
  }
  if (!updated) {
    const hipError_t ei = hipGraphInstantiate(&G->exec[slot], graph, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      G->exec[slot] = nullptr;
      (void)hipGraphDestroy(graph);
      return static_cast<int>(ei);
    }
    ++G->instantiations;
  }
  (void)hipGraphDestroy(graph);
  VG_HIP_RET(hipGraphLaunch(G->exec[slot], s));
  VG_HIP_RET(hipEventRecord(G->done[slot], s));
  G->used[slot] = true;
  G->next ^= 1;
  return 0;
}

#undef VG_HIP_RET
