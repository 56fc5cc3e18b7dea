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

#ifdef __cplusplus
}
#endif

#endif /* VGAN_HOST_H_ */
