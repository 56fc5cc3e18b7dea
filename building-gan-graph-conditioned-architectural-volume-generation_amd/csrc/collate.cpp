// Host-side mini-batch collate of building graphs (libvgan_host.so).
//
// Replaces GraphDataset.collate_fn (reference data.py:156-163), i.e. two
// torch_geometric Batch.from_data_list calls, for buildings held in a
// GraphStore (vgan/store.py): every node-level array of the selected buildings
// is concatenated, edge_index is shifted by the running node count, and
// ptr / batch describe graph membership.  On top of that the collate emits the
// int32 destination CSR (+ self loops) and its source CSC directly, so the
// device never rebuilds them (vg_csr_build, csr.hip) and the training loop
// takes no host sync per batch.
//
// Ordering is the one csr.hip produces: inside a CSR row the slots follow the
// original edge order (remove_self_loops drops i->i), the self loop is last;
// every CSC bucket is sorted by slot.  Buildings are independent blocks of the
// block-diagonal graph, so each worker thread owns whole buildings and writes
// disjoint output ranges whose offsets a serial prefix pass fixes first.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <unistd.h>
#include <vector>

#include "../../include/vgan_host.h"

namespace {

struct Plan {
  std::vector<int64_t> node_off, edge_off, csr_off;  // [count + 1]
};

// Prefix sums of nodes / raw edges / CSR slots of the selected buildings.
int plan(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc, const int32_t* edst,
         const int64_t* index, int32_t count, int64_t num_buildings, Plan& p) {
  p.node_off.assign(count + 1, 0);
  p.edge_off.assign(count + 1, 0);
  p.csr_off.assign(count + 1, 0);
  for (int32_t b = 0; b < count; ++b) {
    const int64_t g = index[b];
    if (g < 0 || g >= num_buildings) return VGH_EINDEX;
    const int64_t n = node_ptr[g + 1] - node_ptr[g];
    const int64_t e0 = edge_ptr[g], e1 = edge_ptr[g + 1];
    if (n <= 0 || e1 < e0) return VGH_EINVAL;
    int64_t loops = 0;
    if (esrc && edst)
      for (int64_t e = e0; e < e1; ++e) loops += esrc[e] == edst[e];
    p.node_off[b + 1] = p.node_off[b] + n;
    p.edge_off[b + 1] = p.edge_off[b] + (e1 - e0);
    p.csr_off[b + 1] = p.csr_off[b] + (e1 - e0) - loops + n;
  }
  if (p.node_off[count] > INT32_MAX || p.csr_off[count] > INT32_MAX) return VGH_ERANGE;
  return 0;
}

// Threads pay off only past ~64k items of work each.
constexpr int64_t kWorkPerThread = 1 << 16;

// A persistent pool of helper threads (a spawn + join per call cost ~20-50 us
// a thread, a few hundred us per batch with the loader's two graph collates):
// a call hands its building ranges to idle helpers and runs the first range
// itself.  Concurrent calls (several loader workers) share the helpers; a call
// whose ranges no helper took in time runs them itself, so it never waits on
// another call's work.
class Pool {
 public:
  // One pool per PROCESS: a child forked while a helper held mu_ (or after
  // helpers started -- they do not exist in the child) gets a fresh pool on
  // its first call instead of the parent's, whose mutex may be locked forever
  // and whose thread list counts threads the child does not have.  Pools are
  // never destroyed: helpers may outlive static teardown, and a forked child
  // must not touch the parent's.
  static Pool& get() {
    static std::atomic<Pool*> cur{nullptr};
    const pid_t me = getpid();
    Pool* p = cur.load(std::memory_order_acquire);
    while (!p || p->pid_ != me) {
      Pool* fresh = new Pool(me);
      if (cur.compare_exchange_strong(p, fresh, std::memory_order_acq_rel)) return *fresh;
      delete fresh;  // another thread installed one first: p holds it now, re-checked
    }
    return *p;
  }

  // run fn(w) for w in [0, t): w = 0 on the calling thread
  template <class F>
  void run(int32_t t, F& fn) {
    struct Call {
      std::atomic<int32_t> next{1}, done{0};
      int32_t t;
      std::function<void(int32_t)> body;
    };
    auto call = std::make_shared<Call>();
    call->t = t;
    call->body = [&fn](int32_t w) { fn(w); };
    {
      std::lock_guard<std::mutex> lk(mu_);
      grow(t - 1);
      for (int32_t i = 1; i < t; ++i)
        jobs_.push_back([call] {
          const int32_t w = call->next.fetch_add(1);
          if (w < call->t) {
            call->body(w);
            call->done.fetch_add(1);
          }
        });
    }
    cv_.notify_all();
    fn(0);
    // ranges no helper has started: run them here
    for (int32_t w = call->next.fetch_add(1); w < t; w = call->next.fetch_add(1)) {
      fn(w);
      call->done.fetch_add(1);
    }
    while (call->done.load() < t - 1) std::this_thread::yield();
  }

 private:
  void grow(int32_t want) {  // mu_ held
    while ((int32_t)threads_.size() < std::min<int32_t>(want, 32))
      threads_.emplace_back([this] {
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return !jobs_.empty(); });
            job = std::move(jobs_.front());
            jobs_.pop_front();
          }
          job();
        }
      });
  }
  explicit Pool(pid_t pid) : pid_(pid) {}

 public:
  pid_t owner() const { return pid_; }

 private:
  const pid_t pid_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> jobs_;
  std::vector<std::thread> threads_;
};

template <class F>
void parallel_buildings(int32_t count, int32_t threads, int64_t work, F&& fn) {
  const int64_t by_work = std::max<int64_t>(1, work / kWorkPerThread);
  const int32_t t = static_cast<int32_t>(std::max<int64_t>(1, std::min<int64_t>({threads, count, by_work})));
  if (t == 1) {
    for (int32_t b = 0; b < count; ++b) fn(b);
    return;
  }
  auto range = [&](int32_t w) {
    for (int32_t b = w; b < count; b += t) fn(b);
  };
  Pool::get().run(t, range);
}

}  // namespace

extern "C" int64_t vgh_pool_pid(void) { return static_cast<int64_t>(Pool::get().owner()); }

extern "C" int vgh_collate_sizes(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc,
                                 const int32_t* edst, int64_t num_buildings, const int64_t* index,
                                 int32_t count, int64_t* sizes) {
  if (!node_ptr || !edge_ptr || !index || !sizes || count <= 0) return VGH_EINVAL;
  Plan p;
  if (int rc = plan(node_ptr, edge_ptr, esrc, edst, index, count, num_buildings, p)) return rc;
  sizes[0] = p.node_off[count];
  sizes[1] = p.edge_off[count];
  sizes[2] = p.csr_off[count];
  return 0;
}

extern "C" int vgh_collate_max_in_degree(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc,
                                         const int32_t* edst, int64_t num_buildings, const int64_t* index,
                                         int32_t count, int32_t* max_degree) {
  if (!node_ptr || !edge_ptr || !esrc || !edst || !index || !max_degree || count <= 0) return VGH_EINVAL;
  int32_t best = 0;
  std::vector<int32_t> deg;
  for (int32_t b = 0; b < count; ++b) {
    const int64_t g = index[b];
    if (g < 0 || g >= num_buildings) return VGH_EINDEX;
    const int64_t n = node_ptr[g + 1] - node_ptr[g];
    deg.assign(n, 1);  // the self loop
    for (int64_t e = edge_ptr[g]; e < edge_ptr[g + 1]; ++e) {
      if (edst[e] < 0 || edst[e] >= n) return VGH_EEDGE;
      if (esrc[e] != edst[e]) ++deg[edst[e]];
    }
    for (int64_t i = 0; i < n; ++i) best = std::max(best, deg[i]);
  }
  *max_degree = best;
  return 0;
}

extern "C" int vgh_collate_rows(const void* src, int64_t row_bytes, const int64_t* node_ptr,
                                int64_t num_buildings, const int64_t* index, int32_t count, void* dst,
                                int32_t threads) {
  if (!src || !dst || !node_ptr || !index || row_bytes <= 0 || count <= 0) return VGH_EINVAL;
  std::vector<int64_t> off(count + 1, 0);
  for (int32_t b = 0; b < count; ++b) {
    const int64_t g = index[b];
    if (g < 0 || g >= num_buildings) return VGH_EINDEX;
    off[b + 1] = off[b] + (node_ptr[g + 1] - node_ptr[g]);
  }
  const char* s = static_cast<const char*>(src);
  char* d = static_cast<char*>(dst);
  parallel_buildings(count, threads, off[count] * row_bytes / 16, [&](int32_t b) {
    const int64_t g = index[b];
    std::memcpy(d + off[b] * row_bytes, s + node_ptr[g] * row_bytes, (off[b + 1] - off[b]) * row_bytes);
  });
  return 0;
}

extern "C" int vgh_collate_graph(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc,
                                 const int32_t* edst, int64_t num_buildings, const int64_t* index,
                                 int32_t count, int32_t threads, int64_t* ptr, int64_t* batch,
                                 int64_t* edge_index, int32_t* row_ptr, int32_t* col, int32_t* csc_ptr,
                                 int32_t* csc_slot, int32_t* csc_dst) {
  if (!node_ptr || !edge_ptr || !esrc || !edst || !index || count <= 0) return VGH_EINVAL;
  const bool want_csr = row_ptr && col && csc_ptr && csc_slot && csc_dst;
  Plan p;
  if (int rc = plan(node_ptr, edge_ptr, esrc, edst, index, count, num_buildings, p)) return rc;
  const int64_t n_total = p.node_off[count], e_total = p.edge_off[count];

  // node ids of every edge must lie inside its own building
  for (int32_t b = 0; b < count; ++b) {
    const int64_t g = index[b], n = node_ptr[g + 1] - node_ptr[g];
    for (int64_t e = edge_ptr[g]; e < edge_ptr[g + 1]; ++e)
      if (esrc[e] < 0 || esrc[e] >= n || edst[e] < 0 || edst[e] >= n) return VGH_EEDGE;
  }
  if (ptr)
    for (int32_t b = 0; b <= count; ++b) ptr[b] = p.node_off[b];

  parallel_buildings(count, threads, n_total + 4 * p.csr_off[count], [&](int32_t b) {
    const int64_t g = index[b];
    const int32_t n = static_cast<int32_t>(node_ptr[g + 1] - node_ptr[g]);
    const int64_t e0 = edge_ptr[g], ne = edge_ptr[g + 1] - e0;
    const int64_t no = p.node_off[b], eo = p.edge_off[b];
    const int32_t co = static_cast<int32_t>(p.csr_off[b]);
    if (batch)
      for (int32_t i = 0; i < n; ++i) batch[no + i] = b;
    if (edge_index)
      for (int64_t e = 0; e < ne; ++e) {
        edge_index[eo + e] = esrc[e0 + e] + no;
        edge_index[e_total + eo + e] = edst[e0 + e] + no;
      }
    if (!want_csr) return;
    // destination CSR: counting sort by destination, stable in edge order
    std::vector<int32_t> cnt(n + 1, 0), cur(n, 0);
    for (int64_t e = 0; e < ne; ++e)
      if (esrc[e0 + e] != edst[e0 + e]) ++cnt[edst[e0 + e] + 1];
    for (int32_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i] + 1;  // + self loop per row
    for (int32_t i = 0; i < n; ++i) row_ptr[no + i] = co + cnt[i];
    for (int64_t e = 0; e < ne; ++e) {
      const int32_t s = esrc[e0 + e], d = edst[e0 + e];
      if (s == d) continue;
      col[co + cnt[d] + cur[d]++] = static_cast<int32_t>(s + no);
    }
    for (int32_t i = 0; i < n; ++i) col[co + cnt[i + 1] - 1] = static_cast<int32_t>(i + no);
    // source CSC: visiting slots in ascending order keeps every bucket sorted
    std::vector<int32_t> sc(n + 1, 0);
    const int32_t ep = cnt[n];
    for (int32_t k = 0; k < ep; ++k) ++sc[col[co + k] - no + 1];
    for (int32_t j = 0; j < n; ++j) sc[j + 1] += sc[j];
    for (int32_t j = 0; j < n; ++j) csc_ptr[no + j] = co + sc[j];
    std::fill(cur.begin(), cur.end(), 0);
    for (int32_t i = 0; i < n; ++i)
      for (int32_t k = cnt[i]; k < cnt[i + 1]; ++k) {
        const int32_t j = col[co + k] - static_cast<int32_t>(no);
        const int32_t pos = co + sc[j] + cur[j]++;
        csc_slot[pos] = co + k;
        csc_dst[pos] = static_cast<int32_t>(i + no);
      }
  });
  if (want_csr) {
    row_ptr[n_total] = static_cast<int32_t>(p.csr_off[count]);
    csc_ptr[n_total] = static_cast<int32_t>(p.csr_off[count]);
  }
  return 0;
}

// ----------------------------------------------------------------------------
// Per-batch structures of vgan.data.prepared, built on the host beside the
// collate so a new batch reaches the device as ONE upload (vgan/store.py)
// instead of ~25 copies plus ~30 small build launches per step.

extern "C" int vgh_csr_ell(const int32_t* row_ptr, const int32_t* col, int32_t n, int32_t width, int32_t* ell) {
  if (!row_ptr || !col || !ell || n <= 0 || width <= 0) return VGH_EINVAL;
  for (int32_t i = 0; i < n; ++i) {
    const int32_t b = row_ptr[i], d = row_ptr[i + 1] - b;
    if (d > width || d < 0) return VGH_ERANGE;
    int32_t* row = ell + static_cast<int64_t>(i) * width;
    for (int32_t j = 0; j < d; ++j) row[j] = col[b + j];
    for (int32_t j = d; j < width; ++j) row[j] = -1;
  }
  return 0;
}

extern "C" int vgh_csr_stacked(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr,
                               const int32_t* csc_slot, const int32_t* csc_dst, int32_t n, int32_t slots,
                               int32_t copies, int32_t* s_row_ptr, int32_t* s_col, int32_t* s_csc_ptr,
                               int32_t* s_csc_slot, int32_t* s_csc_dst) {
  if (!row_ptr || !col || !csc_ptr || !csc_slot || !csc_dst || !s_row_ptr || !s_col || !s_csc_ptr || !s_csc_slot ||
      !s_csc_dst || n <= 0 || slots <= 0 || copies <= 0)
    return VGH_EINVAL;
  if (static_cast<int64_t>(n) * copies > INT32_MAX || static_cast<int64_t>(slots) * copies > INT32_MAX)
    return VGH_ERANGE;
  for (int32_t c = 0; c < copies; ++c) {
    const int32_t no = c * n, eo = c * slots;
    for (int32_t i = 0; i < n; ++i) {
      s_row_ptr[no + i] = row_ptr[i] + eo;
      s_csc_ptr[no + i] = csc_ptr[i] + eo;
    }
    for (int32_t k = 0; k < slots; ++k) {
      s_col[eo + k] = col[k] + no;
      s_csc_slot[eo + k] = csc_slot[k] + eo;
      s_csc_dst[eo + k] = csc_dst[k] + no;
    }
  }
  s_row_ptr[n * copies] = slots * copies;
  s_csc_ptr[n * copies] = slots * copies;
  return 0;
}

// models.py:122-129 on the host, in vg_type_mean's exact f32 order (typemean.hip:
// 16 partial sums per type, program row r into partial r % 16 in row order,
// the partials then summed in order, the count likewise, mean = sum / count),
// so the result is bit for bit the device kernel's.
extern "C" int vgh_type_mean(const float* local_x, const int64_t* local_type, int32_t n_local, int32_t feat,
                             const int64_t* voxel_type, int32_t n_voxel, int32_t n_types, float* out,
                             int32_t out_stride, int32_t out_col0) {
  constexpr int kParts = 16;
  if (n_local < 0 || n_voxel <= 0 || feat <= 0 || n_types <= 0 || !voxel_type || !out ||
      out_stride < out_col0 + feat || (n_local > 0 && (!local_x || !local_type)))
    return VGH_EINVAL;
  std::vector<float> acc(static_cast<size_t>(kParts) * n_types * feat, 0.f), cnt(kParts * n_types, 0.f);
  for (int32_t r = 0; r < n_local; ++r) {
    const int64_t t = local_type[r];
    if (t < 0 || t >= n_types) continue;
    const int w = r % kParts;
    float* a = acc.data() + (static_cast<size_t>(w) * n_types + t) * feat;
    const float* x = local_x + static_cast<int64_t>(r) * feat;
    for (int32_t f = 0; f < feat; ++f) a[f] += x[f];
    cnt[w * n_types + t] += 1.f;
  }
  std::vector<float> table(static_cast<size_t>(n_types) * feat, 0.f), count(n_types, 0.f);
  for (int32_t t = 0; t < n_types; ++t) {
    float c = 0.f;
    for (int w = 0; w < kParts; ++w) c += cnt[w * n_types + t];
    count[t] = c;
    for (int32_t f = 0; f < feat; ++f) {
      float s = 0.f;
      for (int w = 0; w < kParts; ++w) s += acc[(static_cast<size_t>(w) * n_types + t) * feat + f];
      table[static_cast<size_t>(t) * feat + f] = c > 0.f ? s / c : 0.f;
    }
  }
  for (int32_t v = 0; v < n_voxel; ++v) {
    const int64_t t = voxel_type[v];
    float* o = out + static_cast<int64_t>(v) * out_stride + out_col0;
    const bool hit = t >= 0 && t < n_types && count[t] > 0.f;
    for (int32_t f = 0; f < feat; ++f) o[f] = hit ? table[static_cast<size_t>(t) * feat + f] : 0.f;
  }
  return 0;
}
