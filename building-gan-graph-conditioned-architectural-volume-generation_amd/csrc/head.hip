// Gumbel-softmax type head, per-building loss/metric reductions, flat Adam.
#include "common.h"

namespace {

constexpr int kMaxClasses = 32;

// models.py:150-153 -- F.gumbel_softmax(logits, tau=1.0) (hard=False):
//   g = -log(E), E ~ Exp(1);  soft = softmax((logits + g) / tau)
// then label_hard = onehot(argmax soft) - soft.detach() + soft.
// tau_dev != NULL: row r uses tau_dev[r / seg_rows] (per-copy temperatures of a
// stacked inference sweep, read from device memory so a replayed hipGraph
// follows the schedule).
__global__ void k_gumbel_fwd(const float* __restrict__ logits, const float* __restrict__ noise,
                             int rows, int K, float tau, float* __restrict__ soft,
                             float* __restrict__ hard, int32_t* __restrict__ idx,
                             const float* __restrict__ tau_dev = nullptr, int seg_rows = 1) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  if (tau_dev) tau = tau_dev[r / seg_rows];
  float y[kMaxClasses];
  float mx = -INFINITY;
  for (int k = 0; k < K; ++k) {
    const float g = -logf(noise[(size_t)r * K + k]);
    y[k] = (logits[(size_t)r * K + k] + g) / tau;
    mx = fmaxf(mx, y[k]);
  }
  float sum = 0.f;
  for (int k = 0; k < K; ++k) {
    y[k] = expf(y[k] - mx);
    sum += y[k];
  }
  int best = 0;
  float bv = -INFINITY;
  for (int k = 0; k < K; ++k) {
    y[k] = y[k] / sum;
    if (y[k] > bv) {  // strict: first maximum wins (torch.argmax)
      bv = y[k];
      best = k;
    }
  }
  for (int k = 0; k < K; ++k) {
    soft[(size_t)r * K + k] = y[k];
    const float oh = (k == best) ? 1.f : 0.f;
    hard[(size_t)r * K + k] = (oh - y[k]) + y[k];
  }
  if (idx) idx[r] = best;
}

__global__ void k_gumbel_bwd(const float* __restrict__ soft, const float* __restrict__ gh,
                             const float* __restrict__ gs, int rows, int K, float tau,
                             float* __restrict__ gl) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float dot = 0.f;
  for (int k = 0; k < K; ++k) {
    const size_t t = (size_t)r * K + k;
    const float g = (gh ? gh[t] : 0.f) + (gs ? gs[t] : 0.f);
    dot = fmaf(soft[t], g, dot);
  }
  for (int k = 0; k < K; ++k) {
    const size_t t = (size_t)r * K + k;
    const float g = (gh ? gh[t] : 0.f) + (gs ? gs[t] : 0.f);
    gl[t] = soft[t] * (g - dot) / tau;
  }
}

__device__ __forceinline__ int row_argmax(const float* __restrict__ row, int K) {
  int best = 0;
  float bv = row[0];
  for (int k = 1; k < K; ++k)
    if (row[k] > bv) {
      bv = row[k];
      best = k;
    }
  return best;
}

// trainer.py:357-378, one 256-thread block per building
__global__ void __launch_bounds__(256) k_far(const float* __restrict__ x, int xs,
                                             const float* __restrict__ label, int K,
                                             const int64_t* __restrict__ ptr,
                                             const float* __restrict__ site, int far_col,
                                             int dy_col, int dx_col, float scale, int void_class,
                                             float* __restrict__ far_gen,
                                             float* __restrict__ far_ref) {
  const int gi = blockIdx.x;
  const int lo = static_cast<int>(ptr[gi]), hi = static_cast<int>(ptr[gi + 1]);
  float acc = 0.f;
  for (int v = lo + threadIdx.x; v < hi; v += blockDim.x) {
    if (row_argmax(label + (size_t)v * K, K) != void_class)
      acc += (x[(size_t)v * xs + dy_col] * scale) * (x[(size_t)v * xs + dx_col] * scale);
  }
  __shared__ float red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    far_gen[gi] = hi > lo ? red[0] / site[lo] : 0.f;
    far_ref[gi] = hi > lo ? x[(size_t)lo * xs + far_col] : 0.f;
  }
}

// trainer.py:387-443 -- per-building confusion matrices (truth x prediction)
__global__ void __launch_bounds__(256) k_confusion(const int64_t* __restrict__ truth,
                                                   const float* __restrict__ label, int K,
                                                   const int64_t* __restrict__ ptr,
                                                   int32_t* __restrict__ conf,
                                                   int32_t* __restrict__ conf_all) {
  const int gi = blockIdx.x;
  __shared__ int32_t cm[kMaxClasses * kMaxClasses];
  for (int t = threadIdx.x; t < K * K; t += blockDim.x) cm[t] = 0;
  __syncthreads();
  const int lo = static_cast<int>(ptr[gi]), hi = static_cast<int>(ptr[gi + 1]);
  for (int v = lo + threadIdx.x; v < hi; v += blockDim.x) {
    const int64_t t = truth[v];
    const int p = row_argmax(label + (size_t)v * K, K);
    if (t >= 0 && t < K) atomicAdd(&cm[t * K + p], 1);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < K * K; t += blockDim.x) {
    conf[(size_t)gi * K * K + t] = cm[t];
    if (conf_all && cm[t]) atomicAdd(&conf_all[t], cm[t]);
  }
}

// torch.optim.Adam single-tensor update (torch/optim/adam.py, _single_tensor_adam):
//   g += wd * p;  m.lerp_(g, 1 - b1);  v = v*b2 + ((1-b2)*g)*g
//   p += (-step_size * m) / (sqrt(v) / bc2_sqrt + eps)       (addcdiv order)
// (1 - b1), (1 - b2), step_size and bc2_sqrt arrive pre-rounded from double
// exactly as the Python scalars reach the ATen kernels.
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, long long n, float b2, float omb1, float omb2,
                       float eps, float wd, float neg_step, float bc2_sqrt) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (wd != 0.f) gi = gi + wd * p[i];
    const float mi = m[i];
    // at::lerp: |w| < 0.5 ? self + w*(end-self) : end - (end-self)*(1-w)
    const float mn = (fabsf(omb1) < 0.5f) ? mi + omb1 * (gi - mi) : gi - (gi - mi) * (1.f - omb1);
    const float vn = v[i] * b2 + (omb2 * gi) * gi;
    m[i] = mn;
    v[i] = vn;
    const float denom = sqrtf(vn) / bc2_sqrt + eps;
    p[i] = p[i] + (neg_step * mn) / denom;
  }
}

// Same update with the step count and learning rate read from device memory
// (hipGraph replays: host scalars would be frozen into the graph).  Bias
// corrections are formed in double exactly as torch forms them in Python.
__global__ void k_adam_dev(float* __restrict__ p, const float* __restrict__ g,
                           float* __restrict__ m, float* __restrict__ v, long long n, double b1,
                           double b2, float eps, float wd, const double* __restrict__ lr_p,
                           const int32_t* __restrict__ step_p) {
  const double t = static_cast<double>(*step_p);
  const double lr = *lr_p;
  const float neg_step = static_cast<float>(-(lr / (1.0 - pow(b1, t))));
  const float bc2_sqrt = static_cast<float>(sqrt(1.0 - pow(b2, t)));
  const float fb2 = static_cast<float>(b2), omb1 = static_cast<float>(1.0 - b1),
              omb2 = static_cast<float>(1.0 - b2);
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n;
       i += (long long)gridDim.x * blockDim.x) {
    float gi = g[i];
    if (wd != 0.f) gi = gi + wd * p[i];
    const float mi = m[i];
    const float mn = (fabsf(omb1) < 0.5f) ? mi + omb1 * (gi - mi) : gi - (gi - mi) * (1.f - omb1);
    const float vn = v[i] * fb2 + (omb2 * gi) * gi;
    m[i] = mn;
    v[i] = vn;
    const float denom = sqrtf(vn) / bc2_sqrt + eps;
    p[i] = p[i] + (neg_step * mn) / denom;
  }
}

}  // namespace

extern "C" int vg_gumbel_fwd(const float* logits, const float* noise, int32_t rows,
                             int32_t classes, float tau, float* soft, float* hard, int32_t* idx,
                             void* stream) {
  if (rows <= 0 || classes <= 0 || classes > kMaxClasses || !logits || !noise || !soft || !hard)
    return VG_EINVAL;
  k_gumbel_fwd<<<vg_blocks(rows, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      logits, noise, rows, classes, tau, soft, hard, idx);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gumbel_fwd_dev(const float* logits, const float* noise, int32_t rows,
                                 int32_t classes, const float* tau, int32_t seg_rows, float* soft,
                                 float* hard, int32_t* idx, void* stream) {
  if (rows <= 0 || classes <= 0 || classes > kMaxClasses || seg_rows <= 0 || !logits || !noise ||
      !tau || !soft || !hard)
    return VG_EINVAL;
  k_gumbel_fwd<<<vg_blocks(rows, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      logits, noise, rows, classes, 1.f, soft, hard, idx, tau, seg_rows);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_gumbel_bwd(const float* soft, const float* g_hard, const float* g_soft,
                             int32_t rows, int32_t classes, float tau, float* g_logits,
                             void* stream) {
  if (rows <= 0 || classes <= 0 || classes > kMaxClasses || !soft || !g_logits) return VG_EINVAL;
  k_gumbel_bwd<<<vg_blocks(rows, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(
      soft, g_hard, g_soft, rows, classes, tau, g_logits);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_far_per_graph(const float* x, int32_t x_stride, const float* label,
                                int32_t classes, const int64_t* ptr, int32_t num_graphs,
                                const float* site_area, int32_t far_col, int32_t dy_col,
                                int32_t dx_col, float dim_scale, int32_t void_class,
                                float* far_gen, float* far_ref, void* stream) {
  if (num_graphs <= 0 || classes <= 0 || classes > kMaxClasses || !x || !label || !ptr ||
      !site_area || !far_gen || !far_ref)
    return VG_EINVAL;
  k_far<<<num_graphs, 256, 0, static_cast<hipStream_t>(stream)>>>(
      x, x_stride, label, classes, ptr, site_area, far_col, dy_col, dx_col, dim_scale, void_class,
      far_gen, far_ref);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_confusion(const int64_t* truth, const float* label, int32_t classes,
                            const int64_t* ptr, int32_t num_graphs, int32_t* conf,
                            int32_t* conf_all, void* stream) {
  if (num_graphs <= 0 || classes <= 0 || classes > kMaxClasses || !truth || !label || !ptr ||
      !conf)
    return VG_EINVAL;
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (conf_all) (void)hipMemsetAsync(conf_all, 0, sizeof(int32_t) * classes * classes, s);
  k_confusion<<<num_graphs, 256, 0, s>>>(truth, label, classes, ptr, conf, conf_all);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_adam(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                       int64_t n, float beta2, float one_minus_beta1, float one_minus_beta2,
                       float eps, float weight_decay, float step_size, float bc2_sqrt,
                       void* stream) {
  if (n < 0 || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq))) return VG_EINVAL;
  if (n == 0) return 0;
  int blocks = vg_blocks(n, 256);
  if (blocks > 2048) blocks = 2048;
  k_adam<<<blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(
      param, grad, exp_avg, exp_avg_sq, n, beta2, one_minus_beta1, one_minus_beta2, eps,
      weight_decay, -step_size, bc2_sqrt);
  VG_CHECK_LAUNCH();
  return 0;
}

extern "C" int vg_adam_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                           int64_t n, double beta1, double beta2, float eps, float weight_decay,
                           const double* lr, const int32_t* step, void* stream) {
  if (n < 0 || !lr || !step || (n > 0 && (!param || !grad || !exp_avg || !exp_avg_sq)))
    return VG_EINVAL;
  if (n == 0) return 0;
  int blocks = vg_blocks(n, 256);
  if (blocks > 2048) blocks = 2048;
  k_adam_dev<<<blocks, 256, 0, static_cast<hipStream_t>(stream)>>>(
      param, grad, exp_avg, exp_avg_sq, n, beta1, beta2, eps, weight_decay, lr, step);
  VG_CHECK_LAUNCH();
  return 0;
}
