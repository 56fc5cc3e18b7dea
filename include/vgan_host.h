/* vgan host data path: mini-batch collate of building graphs (libvgan_host.so).
 *
 * Host C++ (no GPU): replaces the reference's GraphDataset.collate_fn
 * (building_gan/src/data.py:156-163 -> torch_geometric Batch.from_data_list)
 * for buildings held in a GraphStore (vgan/store.py: per-key arrays of all
 * buildings concatenated, with per-building node_ptr / edge_ptr offsets).
 * It also emits the device index structures of csr.hip (vg_csr_build, declared
 * in vgan.h) directly, so a batch reaches the GPU ready to use.
 *
 * Conventions: `index` selects `count` buildings (in batch order) out of
 * `num_buildings`; node_ptr / edge_ptr have num_buildings + 1 entries; esrc /
 * edst hold each edge's building-local source / destination ids (int32).
 * Outputs are caller-allocated; sizes come from vgh_collate_sizes.  `threads`
 * worker threads each own whole buildings.  Return 0 or a VGH_E* code.
 */
#ifndef VGAN_HOST_H_
#define VGAN_HOST_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VGH_EINVAL 1 /* null pointer, count <= 0, empty building */
#define VGH_EINDEX 2 /* index outside [0, num_buildings) */
#define VGH_EEDGE 3  /* an edge endpoint outside its building */
#define VGH_ERANGE 4 /* batch too large for int32 node / slot ids */

/* sizes[0] = nodes, sizes[1] = edges of edge_index, sizes[2] = CSR/CSC slots
 * (edges without self loops + one self loop per node). */
int vgh_collate_sizes(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc,
                      const int32_t* edst, int64_t num_buildings, const int64_t* index, int32_t count,
                      int64_t* sizes);

/* The largest in-degree of the batch's GATConv graph (self loop included,
 * i->i edges dropped as remove_self_loops does): sizes the padded column array. */
int vgh_collate_max_in_degree(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc,
                              const int32_t* edst, int64_t num_buildings, const int64_t* index, int32_t count,
                              int32_t* max_degree);

/* One node-level attribute (x, type, types_onehot, site_area ...; data.py:117-147):
 * the selected buildings' row blocks of `row_bytes` bytes concatenated into dst
 * (torch.cat(..., dim=0) of Batch.from_data_list). */
int vgh_collate_rows(const void* src, int64_t row_bytes, const int64_t* node_ptr, int64_t num_buildings,
                     const int64_t* index, int32_t count, void* dst, int32_t threads);

/* Graph structure of the batch.  Each output may be NULL (skipped; the five
 * CSR/CSC arrays together):
 *   ptr[count + 1], batch[nodes]       Batch.ptr / Batch.batch (int64)
 *   edge_index[2 * edges]              shifted by the running node count (int64)
 *   row_ptr[nodes + 1], col[slots]     destination CSR + self loops (vg_csr_build)
 *   csc_ptr[nodes + 1], csc_slot[slots], csc_dst[slots]   its source CSC */
int vgh_collate_graph(const int64_t* node_ptr, const int64_t* edge_ptr, const int32_t* esrc,
                      const int32_t* edst, int64_t num_buildings, const int64_t* index, int32_t count,
                      int32_t threads, int64_t* ptr, int64_t* batch, int64_t* edge_index, int32_t* row_ptr,
                      int32_t* col, int32_t* csc_ptr, int32_t* csc_slot, int32_t* csc_dst);

/* ---- per-batch structures of vgan.data.prepared, built on the host ---- */

/* ell[n * width]: row i's CSR sources in order, -1 past its degree (vg_csr_ell). */
int vgh_csr_ell(const int32_t* row_ptr, const int32_t* col, int32_t n, int32_t width, int32_t* ell);

/* The block-diagonal CSR/CSC of `copies` copies of a CSR/CSC over n nodes and
 * `slots` slots (node ids and slots offset per copy): vgan.ops.CSR.stacked. */
int vgh_csr_stacked(const int32_t* row_ptr, const int32_t* col, const int32_t* csc_ptr, const int32_t* csc_slot,
                    const int32_t* csc_dst, int32_t n, int32_t slots, int32_t copies, int32_t* s_row_ptr,
                    int32_t* s_col, int32_t* s_csc_ptr, int32_t* s_csc_slot, int32_t* s_csc_dst);

/* The type-matched mean of models.py:122-129 (vg_type_mean, bit for bit): out[v,
 * out_col0 + f] = mean of local_x[:, f] over the program nodes whose type is
 * voxel v's, 0 where no program node has it. */
int vgh_type_mean(const float* local_x, const int64_t* local_type, int32_t n_local, int32_t feat,
                  const int64_t* voxel_type, int32_t n_voxel, int32_t n_types, float* out, int32_t out_stride,
                  int32_t out_col0);

/* The process id that owns the collate helper pool serving the calling
 * process (the pool is created on first use, and afresh in a forked child:
 * never the parent's, whose mutex a helper may have held at the fork).
 * Introspection for tests. */
int64_t vgh_pool_pid(void);

#ifdef __cplusplus
}
#endif

#endif /* VGAN_HOST_H_ */
