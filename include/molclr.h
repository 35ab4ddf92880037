/*
 * molclr.h — C ABI of the MI355X-native MolCLR pre-training hot path.
 *
 * This is the drop-in boundary: every entry point is `extern "C"`, takes plain
 * device pointers, element counts and an opaque HIP stream (`void*`, a
 * `hipStream_t`), and returns 0 on success or a non-zero status
 * (MOLCLR_ERR_* below, or a positive hipError_t).  `molclr_last_error()` gives
 * a thread-local message for the last failure.  No entry point allocates,
 * synchronises the device, or keeps state between calls: the caller owns
 * every buffer (including the `workspace` scratch, sized by the matching
 * `*_workspace_bytes` query) and all work is stream-ordered, so a caller may
 * capture any sequence of these calls into a HIP graph.
 *
 * Reference interfaces replaced (CameronDiao/MolCLR @ /root/reference):
 *   - PyG 1.6.3 `add_self_loops` + self-loop edge attr, done per layer in
 *       models/ginet_molclr.py:31-37 and models/gcn_molclr.py:64-70
 *       -> molclr_graph_build (once per batch, self loops implicit)
 *   - MoleculeDataset.__getitem__ node-mask views (dataset/dataset.py:111-145)
 *       + the DataLoader's PyG collate    -> molclr_mask_views (on device)
 *   - atom embedding   models/ginet_molclr.py:103, models/gcn_molclr.py:144
 *       -> molclr_atom_embed_fwd / _bwd
 *   - GINEConv edge embedding + message + PyG aggr='add'
 *       models/ginet_molclr.py:39-44        -> molclr_gine_aggregate_fwd / _bwd
 *   - GCNConv message + aggr='add' + bias
 *       models/gcn_molclr.py:72-88          -> molclr_gcn_aggregate_fwd / _bwd
 *   - nn.Linear (GIN MLP ginet_molclr.py:19-23, heads :90-96), GCN `x @ W`
 *       (gcn_molclr.py:76) and their autograd -> molclr_gemm_f32, molclr_colsum_f32
 *   - BatchNorm1d(train/eval) + ReLU + dropout(p=0)
 *       models/ginet_molclr.py:107-111     -> molclr_batchnorm_fwd / _bwd
 *   - global_mean_pool / global_add_pool  ginet_molclr.py:113
 *                                           -> molclr_segment_pool_fwd / _bwd
 *   - F.normalize(dim=1)                  molclr.py:63-64 -> molclr_l2norm_fwd / _bwd
 *   - NTXentLoss.forward (cosine / dot)   utils/nt_xent.py:33-65
 *                                           -> molclr_ntxent_fwd / _bwd
 *   - torch.optim.Adam(weight_decay=L2)   molclr.py:84-87,127 -> molclr_adam_step
 */
#ifndef MOLCLR_H_
#define MOLCLR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* molclr_stream_t; /* a hipStream_t; NULL = legacy default stream */

enum {
  MOLCLR_OK = 0,
  MOLCLR_ERR_ARG = -1,       /* bad shape / pointer / size argument */
  MOLCLR_ERR_WORKSPACE = -2, /* workspace too small */
  MOLCLR_ERR_UNSUPPORTED = -3
};

/* Vocabulary of the reference (models/ginet_molclr.py:9-13). */
#define MOLCLR_NUM_ATOM_TYPE 119     /* 118 elements + mask token 118 */
#define MOLCLR_NUM_CHIRALITY 3
#define MOLCLR_NUM_BOND_TYPE 5       /* 4 bond types + self-loop type 4 */
#define MOLCLR_NUM_BOND_DIR 3
#define MOLCLR_SELF_LOOP_BOND_TYPE 4 /* ginet_molclr.py:35 */
#define MOLCLR_ECOUNT_STRIDE 8       /* per-node counts: 5 bond types, 3 dirs */
#define MOLCLR_NUM_ECOMB 15          /* combined edge-table rows: bt * 3 + bd */
#define MOLCLR_SELF_LOOP_ECOMB 12    /* bond type 4, dir 0 */
#define MOLCLR_NBR_SLOTS 4           /* in-edges held in a node's neighbour slots */
#define MOLCLR_NBR_OVERFLOW 7        /* degree field: > MOLCLR_NBR_SLOTS, use the CSR */
#define MOLCLR_NBR_MAX_NODES (1 << 24)
/* bit of a graph's status word (molclr_graph_build) that the atom embedding
 * sets when an atom type or chirality index lies outside its table */
#define MOLCLR_STATUS_ATOM_RANGE 8

/* ecode (bond_type | bond_dir << 3) -> combined edge-table row */
#define MOLCLR_ECOMB(ecode) ((int)((ecode) & 7u) * 3 + (int)((ecode) >> 3))

const char* molclr_version(void);
const char* molclr_last_error(void);

/* ------------------------------------------------------------------------
 * Graph build (once per batch and view).
 * Inputs are the PyG Batch fields exactly as the reference collates them
 * (dataset/dataset.py:86-147 + PyG collate): edge_index int64 [2,E]
 * (row 0 = source j, row 1 = destination i, flow source_to_target),
 * edge_attr int64 [E,2] (bond type 0..4, bond dir 0..2), batch int64 [N]
 * (ascending, graphs contiguous).
 * Outputs (device, caller-allocated):
 *   rowptr [N+1] i32, col [E] i32, ecode [E] u8 : in-edges of every node
 *       sorted stably by destination (edge order kept inside a row) — the
 *       order in which PyG's scatter-add accumulates them; the self loop PyG
 *       appends at the end of the edge list is implicit (applied last).
 *       ecode = bond_type | bond_dir << 3.
 *   rowptr_t [N+1] i32, col_t [E] i32 : out-edges sorted stably by source
 *       (the accumulation order of index_select's backward).
 *   nbr [N*4] u32, nbr_t [N*4] u32 : neighbour slots, one 16-byte entry per
 *       node so the aggregation reads a row's neighbours with one load and
 *       no rowptr -> col dependency.  Entry i holds the first 4 CSR (nbr) /
 *       CSC (nbr_t) neighbours of i in row order; nbr packs
 *       src | MOLCLR_ECOMB(ecode) << 24.  Bits 29..31 of word 0 hold the
 *       degree, or MOLCLR_NBR_OVERFLOW when it exceeds 4 (the kernels then
 *       walk the CSR/CSC row instead).  Requires N <= MOLCLR_NBR_MAX_NODES.
 *   ecount [N*8] i32 : per destination, counts of in-edge bond types 0..4
 *       and bond dirs 0..2, self loop included.
 *   graph_ptr [G+1] i32 : node range of every graph.
 *   status [1] i32 : bit 0 edge index out of range, bit 1 edge attr out of
 *       range, bit 2 batch not ascending / out of range.  Offending entries
 *       are clamped so no later kernel reads out of bounds.  The encoders'
 *       atom embedding adds bit 3 (MOLCLR_STATUS_ATOM_RANGE) when handed the
 *       word.
 * ------------------------------------------------------------------------ */
size_t molclr_graph_build_workspace_bytes(int64_t num_nodes, int64_t num_edges);
int molclr_graph_build(const int64_t* edge_index, const int64_t* edge_attr,
                       const int64_t* batch, int64_t num_nodes, int64_t num_edges,
                       int64_t num_graphs, int32_t* rowptr, int32_t* col,
                       uint8_t* ecode, int32_t* rowptr_t, int32_t* col_t,
                       uint32_t* nbr, uint32_t* nbr_t,
                       int32_t* ecount, int32_t* graph_ptr, int32_t* status,
                       void* workspace, size_t workspace_bytes, molclr_stream_t stream);

/* molclr_graph_build over `nseg` (<= MOLCLR_MAX_SEGMENTS) PyG batches taken as
 * one: segment s's nodes / edges / graphs follow those of segments 0..s-1
 * (edge_index values stay local to their segment).  The two contrastive
 * views of a step are built as ONE graph this way and run through one
 * encoder pass (molclr_batchnorm_seg_fwd keeps their statistics apart).
 * Workspace: molclr_graph_build_workspace_bytes(total nodes, total edges). */
#define MOLCLR_MAX_SEGMENTS 8
typedef struct molclr_graph_segment {
  const int64_t* edge_index; /* [2, num_edges] */
  const int64_t* edge_attr;  /* [num_edges, 2] */
  const int64_t* batch;      /* [num_nodes] */
  int64_t num_nodes, num_edges, num_graphs;
} molclr_graph_segment;
int molclr_graph_build_multi(int nseg, const molclr_graph_segment* segs, int32_t* rowptr,
                             int32_t* col, uint8_t* ecode, int32_t* rowptr_t, int32_t* col_t,
                             uint32_t* nbr, uint32_t* nbr_t, int32_t* ecount, int32_t* graph_ptr,
                             int32_t* status, void* workspace, size_t workspace_bytes,
                             molclr_stream_t stream);

/* Device-sized graph build: molclr_graph_build_multi over fixed-capacity
 * buffers, for a training step captured once as a HIP graph and replayed for
 * every batch that fits (molclr_amd/graph_step.py; the reference's per-step
 * loop, molclr.py:107-128).  Two calls:
 *   molclr_stage_segments (outside the captured region; one launch): copies
 *     segment s's PyG fields -- x [n_s,2], edge_index [2,e_s], edge_attr
 *     [e_s,2], batch [n_s] -- into its staging buffers dst[s] (edge_index
 *     rows edge_cap apart), x into x_all [num_nodes_cap,2] at row
 *     n_0 + .. + n_{s-1}, fills the remaining rows of x_all with atom (0, 0),
 *     and writes counts [2*nseg] = n_0..n_{nseg-1}, e_0..e_{nseg-1}.
 *   molclr_graph_build_dev (inside it): the build, reading the counts on the
 *     device.  Outputs sized for num_nodes_cap rows / num_edges_cap edges
 *     (workspace: molclr_graph_build_workspace_bytes of those); rows past the
 *     real nodes are padding: no edges, ecount = the self loop only, outside
 *     every graph (graph_ptr[G] = the real node count).  G = sum of num_graphs
 *     is fixed. */
typedef struct molclr_stage_source {
  const int64_t *x, *edge_index, *edge_attr, *batch;
  int64_t num_nodes, num_edges;
} molclr_stage_source;
typedef struct molclr_graph_staged_segment {
  const int64_t* edge_index; /* [2, edge_cap] */
  const int64_t* edge_attr;  /* [edge_cap, 2] */
  const int64_t* batch;      /* [node_cap] */
  int64_t node_cap, edge_cap, num_graphs;
} molclr_graph_staged_segment;
int molclr_stage_segments(int nseg, const molclr_stage_source* src,
                          const molclr_graph_staged_segment* dst, int64_t* x_all,
                          int64_t num_nodes_cap, int64_t num_edges_cap, int64_t* counts,
                          molclr_stream_t stream);
int molclr_graph_build_dev(int nseg, const molclr_graph_staged_segment* segs, const int64_t* counts,
                           int64_t num_nodes_cap, int64_t num_edges_cap, int32_t* rowptr,
                           int32_t* col, uint8_t* ecode, int32_t* rowptr_t, int32_t* col_t,
                           uint32_t* nbr, uint32_t* nbr_t, int32_t* ecount, int32_t* graph_ptr,
                           int32_t* status, void* workspace, size_t workspace_bytes,
                           molclr_stream_t stream);

/* On-device node-mask augmentation + collate: one contrastive view of a batch
 * of molecules, replacing MoleculeDataset.__getitem__'s masking
 * (dataset/dataset.py:111-145) and the DataLoader's PyG collate
 * (Batch.from_data_list).  Per molecule: max(1, floor(N/4)) atoms become
 * [118, 0]; floor(M/4) bonds are dropped with both directed edges; the kept
 * edges stay in store order.  The subsets are uniform, drawn from splitmix64
 * keys of (seed, view, molecule id, item) (restated in oracle/augment_ref.py).
 * Store (device, int64): x [Ntot,2]; atom_ptr [G+1]; edge_index [2,store_edges]
 * with molecule-local atom indices, molecule g's bonds as the directed pairs
 * 2b, 2b+1 for b in [bond_ptr[g], bond_ptr[g+1]); edge_attr [store_edges,2].
 * mol_ids [batch_size] picks the batch.  Outputs (caller-sized: num_nodes =
 * Σ N_g, num_edges = Σ 2 (M_g - floor(M_g/4))): x_out [num_nodes,2],
 * edge_index_out [2,num_edges], edge_attr_out [num_edges,2], batch_out
 * [num_nodes], ptr_out [batch_size+1] -- the Batch fields.  status [1] i32:
 * bit 0 molecule id out of range, bit 1 output sizes do not match the batch,
 * bit 2 store edge index out of its molecule's range (clamped).  view: 0 / 1. */
size_t molclr_mask_views_workspace_bytes(int64_t batch_size);
int molclr_mask_views(const int64_t* store_x, const int64_t* store_atom_ptr,
                      const int64_t* store_edge_index, const int64_t* store_edge_attr,
                      const int64_t* store_bond_ptr, int64_t store_mols, int64_t store_edges,
                      const int64_t* mol_ids, int64_t batch_size, uint64_t seed, int view,
                      int64_t* x_out, int64_t* edge_index_out, int64_t* edge_attr_out,
                      int64_t* batch_out, int64_t* ptr_out, int64_t num_nodes, int64_t num_edges,
                      int32_t* status, void* workspace, size_t workspace_bytes,
                      molclr_stream_t stream);

/* On-device subgraph-removal views (dataset/dataset_subgraph.py:70-177,
 * mode MOLCLR_AUG_SUBGRAPH) and mixed subgraph + atom/bond masking views
 * (dataset/dataset_mix.py:46-217, mode MOLCLR_AUG_MIX) + collate, from the
 * molclr_mask_views store.  Per molecule: the networkx BFS removal
 * (removeSubgraph: from a random centre, floor(p x atoms-in-bonds) atoms,
 * p = 0.25 or uniform [0, 0.2) in mix, the frontier in CPython set order)
 * masks the removed atoms to [118, 0]; bonds survive as G_i.edges keeps them
 * (mix: both atoms remain; subgraph: additionally (start, end) must be
 * networkx's orientation); mix then masks max(0, floor(N/4) - removed) more
 * atoms among the remaining and drops max(0, kept - ceil(3M/4)) surviving
 * bonds.  Two calls because the edge count is data dependent:
 *   plan: ptr_out [B+1] (atom offsets), *num_edges_out (device int64) =
 *         the view's directed-edge count; the plan lives in the workspace;
 *   write: the Batch fields (as molclr_mask_views) sized by that count.
 * num_nodes = Σ atoms, num_bonds = Σ bonds of the batch's molecules.  status
 * bits: 0 molecule id out of range, 1 num_nodes mismatch, 2 edge index out
 * of its molecule (clamped), 3 the frontier emptied before the quota (the
 * subgraph module would not terminate; dataset_mix.py:55-56's guard is
 * applied), 4 a molecule over 256 atoms / 512 bonds (left un-augmented; with
 * molclr_aug_views_plan_big: over its large-molecule caps), 5 a centre atom
 * without bonds (the reference raises). */
enum { MOLCLR_AUG_SUBGRAPH = 0, MOLCLR_AUG_MIX = 1 };
size_t molclr_aug_views_workspace_bytes(int64_t batch_size, int64_t num_nodes, int64_t num_bonds);
int molclr_aug_views_plan(const int64_t* store_atom_ptr, const int64_t* store_edge_index,
                          const int64_t* store_bond_ptr, int64_t store_mols, int64_t store_edges,
                          const int64_t* mol_ids, int64_t batch_size, uint64_t seed, int view,
                          int mode, int64_t num_nodes, int64_t num_bonds, int64_t* ptr_out,
                          int64_t* num_edges_out, int32_t* status, void* workspace,
                          size_t workspace_bytes, molclr_stream_t stream);
/* The plan with molecules beyond the in-LDS caps (256 atoms / 512 bonds)
 * augmented too, the reference's behaviour for every molecule
 * (dataset_subgraph.py:96-177 and dataset_mix.py:86-217 have no size limit):
 * they run the same plan over int32 tables in `big_workspace`, one slot per
 * such molecule of the batch.  big_slots >= the batch's count of such
 * molecules, big_atoms / big_bonds >= their largest atom / bond counts
 * (molecules past these caps pass unchanged, status bit 4).  Results are
 * identical to molclr_aug_views_plan's on every molecule within its caps. */
size_t molclr_aug_views_big_workspace_bytes(int64_t big_slots, int64_t big_atoms,
                                            int64_t big_bonds);
int molclr_aug_views_plan_big(const int64_t* store_atom_ptr, const int64_t* store_edge_index,
                              const int64_t* store_bond_ptr, int64_t store_mols,
                              int64_t store_edges, const int64_t* mol_ids, int64_t batch_size,
                              uint64_t seed, int view, int mode, int64_t num_nodes,
                              int64_t num_bonds, int64_t* ptr_out, int64_t* num_edges_out,
                              int32_t* status, void* workspace, size_t workspace_bytes,
                              int64_t big_slots, int64_t big_atoms, int64_t big_bonds,
                              void* big_workspace, size_t big_workspace_bytes,
                              molclr_stream_t stream);
int molclr_aug_views_write(const int64_t* store_x, const int64_t* store_atom_ptr,
                           const int64_t* store_edge_index, const int64_t* store_edge_attr,
                           const int64_t* store_bond_ptr, int64_t store_mols, int64_t store_edges,
                           const int64_t* mol_ids, int64_t batch_size, const int64_t* ptr,
                           int64_t num_nodes, int64_t num_bonds, int64_t num_edges, int64_t* x_out,
                           int64_t* edge_index_out, int64_t* edge_attr_out, int64_t* batch_out,
                           const void* workspace, size_t workspace_bytes, molclr_stream_t stream);

/* Atom embedding: h[i] = X1[x[i,0]] + X2[x[i,1]]  (ginet_molclr.py:103).
 * x int64 [N,2]; X1 [n1,D], X2 [n2,D]; h [N,D] f32.  A node whose atom type
 * or chirality lies outside [0,n1) / [0,n2) -- where the reference's
 * nn.Embedding raises -- gets a NaN row and sets MOLCLR_STATUS_ATOM_RANGE in
 * *status (nullable: e.g. the batch's graph status word). */
int molclr_atom_embed_fwd(const int64_t* x, const float* X1, const float* X2,
                          float* h, int64_t num_nodes, int64_t dim, int64_t n1,
                          int64_t n2, int32_t* status, molclr_stream_t stream);
/* dX1 [n1,D], dX2 [n2,D] = Σ over nodes of each type of dh (deterministic, fp64
 * accumulation).  accumulate != 0 adds into dX1/dX2 (fused gradient
 * accumulation into a parameter's .grad); the same flag on the other
 * backward entry points below applies to their parameter-gradient outputs. */
size_t molclr_atom_embed_bwd_workspace_bytes(int64_t num_nodes, int64_t dim, int64_t n1,
                                             int64_t n2);
int molclr_atom_embed_bwd(const int64_t* x, const float* dh, float* dX1, float* dX2,
                          int64_t num_nodes, int64_t dim, int64_t n1, int64_t n2, int accumulate,
                          void* workspace, size_t workspace_bytes, molclr_stream_t stream);

/* Combined edge tables of `layers` GINE layers (ginet_molclr.py:24-27,39):
 *   Ec[l][bt*3 + bd][:] = E1_l[bt][:] + E2_l[bd][:]
 * (the edge embedding the reference computes per edge, one fp32 rounding —
 * so using Ec is bit-identical).  E1s / E2s are HOST arrays of `layers`
 * device pointers to [5,D] / [3,D] tables; Ec is [layers, 15, D].
 * layers <= MOLCLR_MAX_LAYERS.  One launch for all layers. */
#define MOLCLR_MAX_LAYERS 16
int molclr_edge_tables_combine(int layers, const float* const* E1s, const float* const* E2s,
                               float* Ec, int64_t dim, molclr_stream_t stream);

/* GINE aggregation (ginet_molclr.py:39-44 + PyG aggr='add'):
 *   out[i] = Σ_{k in in(i), edge order} (x[src_k] + Ec[bt_k*3+bd_k])
 *            + (x[i] + Ec[12])                              (self loop last)
 * Same operation order as the reference CPU path, so results are
 * bit-identical to it.  x, out [N,D] f32; Ec [15,D] (molclr_edge_tables_combine);
 * nbr from molclr_graph_build, with rowptr/col/ecode for rows of degree > 4. */
int molclr_gine_aggregate_fwd(const float* x, const int32_t* rowptr, const int32_t* col,
                              const uint8_t* ecode, const uint32_t* nbr, const float* Ec,
                              float* out, int64_t num_nodes, int64_t dim,
                              molclr_stream_t stream);
/* molclr_gine_aggregate_fwd that also writes the output's row maxima and,
 * when `slot` is not NULL, folds max |out| into it (zeroed by the caller):
 * the row scales of the h3 product that consumes it (molclr_gemm_f32_h3 with
 * a_row_parts = molclr_rowmax_layout(D)), with no pass of its own.  Layout
 * (molclr_rowmax_layout(D), molclr_rowmax_bytes(N, D) bytes): P > 0: P
 * partial arrays rowparts[p][N] (the row max is the max over p); < 0 (D / 4
 * >= 64): one float2 per 64 float4s of the row-major output (the maxima of
 * the pieces of the wave's first row and of the next row). */
int64_t molclr_rowmax_layout(int64_t D);
size_t molclr_rowmax_bytes(int64_t N, int64_t D);
int molclr_gine_aggregate_fwd_rowmax(const float* x, const int32_t* rowptr, const int32_t* col,
                                     const uint8_t* ecode, const uint32_t* nbr, const float* Ec,
                                     float* out, int64_t N, int64_t D, float* rowparts,
                                     float* slot, molclr_stream_t stream);
/* Backward: dx[j] = Σ_{k in out(j), edge order} g[dst_k] + g[j];
 * dE1[t] = Σ_i ecount[i][t] g[i], dE2[d] = Σ_i ecount[i][5+d] g[i].
 * dx may be NULL (first layer input needs no grad); dE1/dE2 may be NULL. */
size_t molclr_gine_aggregate_bwd_workspace_bytes(int64_t num_nodes, int64_t dim);
int molclr_gine_aggregate_bwd(const float* g, const int32_t* rowptr_t, const int32_t* col_t,
                              const uint32_t* nbr_t, const int32_t* ecount, float* dx, float* dE1, float* dE2,
                              int64_t num_nodes, int64_t dim, int accumulate, void* workspace,
                              size_t workspace_bytes, molclr_stream_t stream);

/* GCN aggregation (gcn_molclr.py:72-88; gcn_norm at :74 is computed and
 * discarded by the reference, so it is not computed here):
 *   out[i] = Σ_{k in in(i)} (e_k + xw[src_k]) + (e_self + xw[i]) + bias
 * with scalar e = E1[bt][0] + E2[bd][0] (tables [5,1], [3,1]). */
int molclr_gcn_aggregate_fwd(const float* xw, const int32_t* rowptr, const int32_t* col,
                             const uint8_t* ecode, const uint32_t* nbr, const float* E1,
                             const float* E2,
                             const float* bias, float* out, int64_t num_nodes,
                             int64_t dim, molclr_stream_t stream);
/* Backward: dxw[j] = Σ_{out(j)} g[dst] + g[j]; dE1[t] = Σ_i ecount[i][t]·Σ_d g[i][d];
 * dE2 likewise; dbias = Σ_i g[i].  Any output pointer may be NULL. */
size_t molclr_gcn_aggregate_bwd_workspace_bytes(int64_t num_nodes, int64_t dim);
int molclr_gcn_aggregate_bwd(const float* g, const int32_t* rowptr_t, const int32_t* col_t,
                             const uint32_t* nbr_t, const int32_t* ecount, float* dxw, float* dE1, float* dE2,
                             float* dbias, int64_t num_nodes, int64_t dim, int accumulate,
                             void* workspace, size_t workspace_bytes, molclr_stream_t stream);

/* ------------------------------------------------------------------------
 * FP32 GEMM on the gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32: exact f32 FMA
 * chains, no TF32-style truncation).
 *   C[m,n] = Σ_k A(m,k) B(k,n)  (+ epilogue)
 *   A(m,k) = a_kmajor ? A[k*lda + m] : A[m*lda + k]
 *   B(k,n) = b_kmajor ? B[k*ldb + n] : B[n*ldb + k]
 * so nn.Linear forward (x W^T) is a_kmajor=0, b_kmajor=0; dX = dY W is
 * a_kmajor=0, b_kmajor=1; dW = dY^T X is a_kmajor=1, b_kmajor=1.
 * Epilogues: MOLCLR_EPI_NONE, _BIAS (C += bias[n]), _BIAS_RELU,
 * _RELU_MASK (C *= (aux[m*ldaux+n] > 0), the ReLU backward), optionally
 * OR-ed with MOLCLR_EPI_ACCUMULATE (C = C_old + result).
 * An operand stored with K contiguous needs K and its ld to be multiples of 4.
 * Split-K (for the weight-gradient shape, K = number of nodes) runs when the
 * workspace is large enough: molclr_gemm_f32_workspace_bytes(M,N,K). */
enum { MOLCLR_EPI_NONE = 0, MOLCLR_EPI_BIAS = 1, MOLCLR_EPI_BIAS_RELU = 2,
       MOLCLR_EPI_RELU_MASK = 3,
       MOLCLR_EPI_ACCUMULATE = 16 /* OR-able flag: C += result (gradient accumulation) */ };
size_t molclr_gemm_f32_workspace_bytes(int64_t M, int64_t N, int64_t K);
int molclr_gemm_f32(const float* A, const float* B, float* C, int64_t M, int64_t N,
                    int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor,
                    int b_kmajor, int epilogue_flags, const float* bias, const float* aux,
                    int64_t ldaux, void* workspace, size_t workspace_bytes,
                    molclr_stream_t stream);

/* molclr_gemm_f32 with the implementation chosen per call (tests and
 * benchmarks; molclr_gemm_f32 is impl = -1): -1 = automatic (split-bf16 "p6",
 * or "w6" for a long-K weight gradient), 0 = f32-input MFMA
 * (v_mfma_f32_32x32x2_f32), 64x64 tiles; 5 / 6 = split-bf16 "p6" (each fp32
 * operand split into 3 round-to-nearest bf16 parts, six bf16 MFMA products,
 * fp32 accumulation; fp32-GEMM accuracy), 64x64 / 128x64 tiles. */
int molclr_gemm_f32_impl(const float* A, const float* B, float* C, int64_t M, int64_t N,
                         int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int a_kmajor,
                         int b_kmajor, int epilogue_flags, const float* bias, const float* aux,
                         int64_t ldaux, void* workspace, size_t workspace_bytes,
                         molclr_stream_t stream, int impl);

/* Pre-split weight operand.  A Linear layer's weight is the B operand of the
 * forward (y = x W^T) and data-gradient (dx = dy W) GEMMs of every row tile;
 * splitting it once per optimizer step instead of once per row tile takes
 * half of the split work out of those GEMMs.
 *   molclr_bplanes_make: planes [3][Npad][Kp] bf16 (hi, mid, lo parts, the
 *     same split as the GEMM) of B(k, n) — stored like molclr_gemm_f32's B
 *     (b_kmajor: B[k*ldb + n], else B[n*ldb + k]) — zero-padded to
 *     Npad = N rounded up to 128, Kp = K rounded up to 32.
 *     molclr_bplanes_bytes(N, K) is their size.
 *   molclr_gemm_f32_bplanes: molclr_gemm_f32 with B given as such planes
 *     (same epilogues, split-K workspace from molclr_gemm_f32_workspace_bytes);
 *     a_kmajor needs M and lda multiples of 4, else K and lda. */
size_t molclr_bplanes_bytes(int64_t N, int64_t K);
int molclr_bplanes_make(const float* B, int64_t N, int64_t K, int64_t ldb, int b_kmajor,
                        uint16_t* planes, molclr_stream_t stream);
/* molclr_bplanes_make for `count` weights in one launch per 32 (host arrays of
 * per-weight arguments); the planes of a whole model after an optimizer step. */
int molclr_bplanes_make_batch(int count, const float* const* B, const int64_t* N,
                              const int64_t* K, const int64_t* ldb, const int* b_kmajor,
                              uint16_t* const* planes, molclr_stream_t stream);
int molclr_gemm_f32_bplanes(const float* A, const uint16_t* planes, float* C, int64_t M,
                            int64_t N, int64_t K, int64_t lda, int64_t ldc, int a_kmajor,
                            int epilogue_flags, const float* bias, const float* aux,
                            int64_t ldaux, void* workspace, size_t workspace_bytes,
                            molclr_stream_t stream);
/* molclr_gemm_f32_bplanes with the tile chosen per call (molclr_gemm_f32_bplanes
 * is tile = 0): 0 = automatic (9 for a row-major A whose 128-row tiles number
 * >= 128, else 64x128 for N >= 512, else 64x64), 5 = 64x64, 6 = 128x64,
 * 7 = 64x128, 8 = 128x128, 9 = "q6": 128 x 160 (or 128 / 64 wide) tiles with A
 * streamed through registers, one wave per 32 rows, for K <= 1024 (a K-major A
 * or a longer K falls back to 5 / 7). */
int molclr_gemm_f32_bplanes_tile(const float* A, const uint16_t* planes, float* C, int64_t M,
                                 int64_t N, int64_t K, int64_t lda, int64_t ldc, int a_kmajor,
                                 int epilogue_flags, const float* bias, const float* aux,
                                 int64_t ldaux, void* workspace, size_t workspace_bytes,
                                 molclr_stream_t stream, int tile);

/* Weight and bias gradients of y = x W^T + b (nn.Linear backward):
 *   dW[n_out][n_in] (+)= Σ_r dy[r][o] x[r][i],   db[n_out] (+)= Σ_r dy[r][o]
 * dy [rows, n_out] (row stride ld_dy), x [rows, n_in] (ld_x).  One split-bf16
 * GEMM that also takes the bias column sums from the dy tiles it stages (no
 * separate pass over dy).  db may be NULL; accumulate != 0 adds into dW / db.
 * db needs n_out and ld_dy multiples of 4.  Falls back to molclr_gemm_f32 +
 * molclr_colsum_f32 for shapes the fused kernel does not take. */
size_t molclr_linear_wgrad_workspace_bytes(int64_t rows, int64_t n_out, int64_t n_in);
int molclr_linear_wgrad(const float* dy, const float* x, float* dW, float* db, int64_t rows,
                        int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x, int accumulate,
                        void* workspace, size_t workspace_bytes, molclr_stream_t stream);
/* molclr_linear_wgrad with the K groups per block of the long-K kernel chosen
 * per call (molclr_linear_wgrad is groups = 2): 2 = two 4-wave groups per block,
 * half as many split-K partial tiles; 1 = one group per block. */
int molclr_linear_wgrad_groups(const float* dy, const float* x, float* dW, float* db,
                               int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                               int64_t ld_x, int accumulate, void* workspace,
                               size_t workspace_bytes, molclr_stream_t stream, int groups);

/* "h3" fp32 GEMMs: three fp16 MFMA products per element pair instead of six
 * bf16 ones.  Each operand is scaled by a power of two chosen from its
 * tensor-wide max |x| (scaled max in [2^14, 2^15)) and split into two
 * round-to-nearest fp16 parts, x 2^s = hi + lo + t with |t| <= 2^-22 |x 2^s|;
 * hi_a hi_b + hi_a lo_b + lo_a hi_b accumulates in fp32 and is scaled back
 * exactly.  Same epilogues and shapes as the q6 / w6 kernels they replace
 * (models/ginet_molclr.py:19-23: the GIN MLP forward, data and weight
 * gradients).
 *   A max slot is 64 entries 128 bytes apart (2048 floats, 8 KB) whose max
 *     is the tensor's max |x| (producers spread their atomic maxima over the
 *     entries; atomics on one cache line serialise).
 *   molclr_absmax_f32: slot <- max |x| over a [rows][cols] (ld) matrix
 *     (accumulate != 0: folded into the current slot; else the slot is reset
 *     first).  The max is order-independent, so every producer of the same
 *     tensor gives the same slot value.
 *   molclr_hplanes_make_batch: weights as h3 B operands (molclr_bplanes_make_batch
 *     arguments): [2][Npad][Kp] fp16 planes, then the max |B| slot,
 *     molclr_hplanes_bytes(N, K) bytes each.
 *   molclr_absmax_rows_f32: rowmax[r] = max_c |x[r][c]| and the slot as
 *     molclr_absmax_f32.
 *   molclr_gemm_f32_h3: C = epilogue(A B) for a row-major A [M][K] (lda) and
 *     h3 planes of B; K <= 1024, K and lda multiples of 4.  a_row_parts == 0:
 *     `amax` is A's max slot (one scale for A); P > 0: `amax` holds A's row
 *     maxima as P partial arrays [P][M] (P < 0: as the per-wave pairs of
 *     molclr_rowmax_layout(K) = P) and every row is scaled by its own
 *     (a row of small values, e.g. a node with a small gradient, keeps full
 *     precision).  cmax / crow (each may be NULL): max |C| folded into the
 *     slot cmax (the caller zeroes it) / C's row maxima as
 *     molclr_gemm_row_parts(N) partial arrays (plain stores); amax_out (may
 *     be NULL, zeroed by the caller): max |A| folded in.  A RELU_MASK
 *     epilogue takes its mask from mask_bits (molclr_gemm_f32_bplanes_max's
 *     relu_bits of the same [M][N]) when given, else from aux.
 *   molclr_linear_wgrad_h3: molclr_linear_wgrad given the max slots of dy
 *     and x (n_out, n_in, ld_dy, ld_x multiples of 4; same workspace). */
int molclr_absmax_f32(const float* x, int64_t rows, int64_t cols, int64_t ld, float* slot,
                      int accumulate, molclr_stream_t stream);
size_t molclr_hplanes_bytes(int64_t N, int64_t K);
int molclr_hplanes_make_batch(int count, const float* const* B, const int64_t* N,
                              const int64_t* K, const int64_t* ldb, const int* b_kmajor,
                              uint16_t* const* planes, molclr_stream_t stream);
/* molclr_gemm_f32_bplanes (x6 planes, row-major A, K <= 1024; same kernel and
 * result as its automatic choice) that also folds max |A| of its A rows into
 * the slot amax_out and max |C| into the slot cmax (zeroed by the caller),
 * and writes C's row maxima as molclr_gemm_row_parts(N) partial arrays
 * crow[p][M] (plain stores; the row max is the max over p): the scales of
 * the h3 products that consume A or C, with no pass when the q6 kernel runs.
 * relu_bits: bit (n % 32) of word [n / 32][m] (ceil(N / 32) x M words) =
 * (C[m][n] > 0) -- the ReLU mask of a bias+ReLU product in 1/32 of the bytes.
 * Each output may be NULL. */
int64_t molclr_gemm_row_parts(int64_t N);
int molclr_gemm_f32_bplanes_max(const float* A, const uint16_t* planes, float* C, int64_t M,
                                int64_t N, int64_t K, int64_t lda, int64_t ldc,
                                int epilogue_flags, const float* bias, const float* aux,
                                int64_t ldaux, float* amax_out, float* cmax, float* crow,
                                uint32_t* relu_bits, void* workspace, size_t workspace_bytes,
                                molclr_stream_t stream);
int molclr_absmax_rows_f32(const float* x, int64_t rows, int64_t cols, int64_t ld,
                           float* rowmax, float* slot, int accumulate, molclr_stream_t stream);
int molclr_gemm_f32_h3(const float* A, const float* amax, int a_row_parts, const uint16_t* hplanes,
                       float* C, int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldc,
                       int epilogue_flags, const float* bias, const float* aux, int64_t ldaux,
                       const uint32_t* mask_bits, float* cmax, float* crow, float* amax_out,
                       molclr_stream_t stream);
/* molclr_gemm_f32_h3_bits with the kernel chosen per call (tests): impl 0 =
 * automatic, 1 = k_gemm_pp / k_gemm_q6, 2 = k_gemm_bs, 3 = k_gemm_bs16 (both
 * bs: K in (288, 304], N > 320, C float4-aligned, ReLU mask as bits;
 * MOLCLR_ERR_UNSUPPORTED otherwise).  Kernels 1 and 2 give bit-identical C,
 * bits and maxima; 3 (16 x 16 x 32 MFMAs) sums each product's k in another
 * order, equal to fp32 rounding.  The row maxima (crow) are
 * molclr_gemm_row_parts(N) arrays whatever the kernel. */
int molclr_gemm_f32_h3_impl(const float* A, const float* amax, int a_row_parts,
                            const uint16_t* hplanes, float* C, int64_t M, int64_t N, int64_t K,
                            int64_t lda, int64_t ldc, int epilogue_flags, const float* bias,
                            const float* aux, int64_t ldaux, const uint32_t* mask_bits, float* cmax,
                            float* crow, float* amax_out, uint32_t* relu_bits,
                            molclr_stream_t stream, int impl);
/* molclr_gemm_f32_h3 whose BIAS_RELU product also writes C's ReLU mask as
 * bits (relu_bits: molclr_gemm_f32_bplanes_max's layout, may be NULL): the h3
 * forward's first GIN-MLP product, whose mask the dz1 product reads back. */
int molclr_gemm_f32_h3_bits(const float* A, const float* amax, int a_row_parts,
                            const uint16_t* hplanes, float* C, int64_t M, int64_t N, int64_t K,
                            int64_t lda, int64_t ldc, int epilogue_flags, const float* bias,
                            const float* aux, int64_t ldaux, const uint32_t* mask_bits,
                            float* cmax, float* crow, float* amax_out, uint32_t* relu_bits,
                            molclr_stream_t stream);
/* molclr_linear_wgrad_h3 with the K groups per block chosen per call (the plain
 * call is groups = 2), as molclr_linear_wgrad_groups. */
int molclr_linear_wgrad_h3_groups(const float* dy, const float* dymax, const float* x,
                                  const float* xmax, float* dW, float* db, int64_t rows,
                                  int64_t n_out, int64_t n_in, int64_t ld_dy, int64_t ld_x,
                                  int accumulate, void* workspace, size_t workspace_bytes,
                                  molclr_stream_t stream, int groups);
int molclr_linear_wgrad_h3(const float* dy, const float* dymax, const float* x,
                           const float* xmax, float* dW, float* db, int64_t rows, int64_t n_out,
                           int64_t n_in, int64_t ld_dy, int64_t ld_x, int accumulate,
                           void* workspace, size_t workspace_bytes, molclr_stream_t stream);
/* Two h3 weight gradients (a: dW_a = dy_a^T x_a, b likewise) over the same
 * row count, their ordered split-K reductions in ONE launch: the same results
 * as two molclr_linear_wgrad_h3 calls (rows >= 1024; sizes multiples of 4). */
size_t molclr_linear_wgrad_h3_pair_workspace_bytes(int64_t rows, int64_t n_out_a, int64_t n_in_a,
                                                   int64_t n_out_b, int64_t n_in_b);
int molclr_linear_wgrad_h3_pair(const float* dy_a, const float* dymax_a, const float* x_a,
                                const float* xmax_a, float* dW_a, float* db_a, int64_t n_out_a,
                                int64_t n_in_a, int64_t ld_dy_a, int64_t ld_x_a,
                                const float* dy_b, const float* dymax_b, const float* x_b,
                                const float* xmax_b, float* dW_b, float* db_b, int64_t n_out_b,
                                int64_t n_in_b, int64_t ld_dy_b, int64_t ld_x_b, int64_t rows,
                                int accumulate, void* workspace, size_t workspace_bytes,
                                molclr_stream_t stream);

/* out[n] = Σ_m X[m*ld + n]  (bias gradients), deterministic. */
size_t molclr_colsum_f32_workspace_bytes(int64_t rows, int64_t cols);
int molclr_colsum_f32(const float* X, float* out, int64_t rows, int64_t cols, int64_t ld,
                      int accumulate, void* workspace, size_t workspace_bytes,
                      molclr_stream_t stream);

/* ------------------------------------------------------------------------
 * BatchNorm1d over the rows of z [N,D] (+ ReLU), ginet_molclr.py:107-111.
 * training != 0: batch statistics (biased variance for normalising),
 *   running_mean/var updated in place with `momentum` and the unbiased
 *   variance, exactly as torch.nn.BatchNorm1d, and *num_batches_tracked
 *   (may be NULL) incremented; save_mean / save_invstd [D] receive the
 *   statistics for the backward.
 * training == 0: running statistics are used and nothing is updated.
 * relu != 0 applies max(y, 0) to the output.  y may be NULL: the statistics
 * (save_mean / save_invstd, running stats) are computed and the normalised
 * output is not written. */
size_t molclr_batchnorm_workspace_bytes(int64_t rows, int64_t dim);
int molclr_batchnorm_fwd(const float* z, const float* gamma, const float* beta,
                         float* running_mean, float* running_var,
                         int64_t* num_batches_tracked, float* y,
                         float* save_mean, float* save_invstd, int64_t rows, int64_t dim,
                         double momentum, double eps, int training, int relu,
                         void* workspace, size_t workspace_bytes, molclr_stream_t stream);
/* dy is the gradient w.r.t. the (ReLU'd) output; dz/dgamma/dbeta out. */
int molclr_batchnorm_bwd(const float* dy, const float* z, const float* gamma,
                         const float* beta, const float* save_mean,
                         const float* save_invstd, float* dz, float* dgamma, float* dbeta,
                         int64_t rows, int64_t dim, int relu, int accumulate, void* workspace,
                         size_t workspace_bytes, molclr_stream_t stream);

/* Segmented BatchNorm: the rows are `nseg` consecutive segments of
 * seg_rows[s] rows (host array), each normalised with its own batch statistics
 * -- the reference's two encoder calls per step (molclr.py:57,60) run as ONE
 * pass over both views -- and the running statistics updated once per
 * segment in segment order (num_batches_tracked += nseg).  Every segment's
 * outputs are bit-identical to a molclr_batchnorm_fwd / _bwd call over its
 * rows alone.  save_mean / save_invstd are [nseg, D].  dgamma / dbeta are the
 * sums over the segments (in segment order).  dtype: MOLCLR_DTYPE_F32 or
 * MOLCLR_DTYPE_BF16 storage of z / y / dy / dz (statistics always fp32). */
enum { MOLCLR_DTYPE_F32 = 0, MOLCLR_DTYPE_BF16 = 1 };
size_t molclr_batchnorm_seg_workspace_bytes(int nseg, const int64_t* seg_rows, int64_t dim);
int molclr_batchnorm_seg_fwd(const void* z, const float* gamma, const float* beta,
                             float* running_mean, float* running_var,
                             int64_t* num_batches_tracked, void* y, float* save_mean,
                             float* save_invstd, int nseg, const int64_t* seg_rows, int64_t dim,
                             int dtype, double momentum, double eps, int training, int relu,
                             void* workspace, size_t workspace_bytes, molclr_stream_t stream);
int molclr_batchnorm_seg_bwd(const void* dy, const void* z, const float* gamma,
                             const float* beta, const float* save_mean, const float* save_invstd,
                             void* dz, float* dgamma, float* dbeta, int nseg,
                             const int64_t* seg_rows, int64_t dim, int dtype, int relu,
                             int accumulate, void* workspace, size_t workspace_bytes,
                             molclr_stream_t stream);

/* molclr_batchnorm_seg_bwd (fp32; same dz) that also writes the row maxima of
 * dz as molclr_bn_row_parts(dim) partial arrays rowmax[p][rows] (plain
 * stores; max |dz[r]| = max over p) and folds max |dz| into the slot (may be
 * NULL; the caller zeroes it): the scales of the h3 products that consume dz
 * (molclr_gemm_f32_h3 row-wise, molclr_linear_wgrad_h3). */
int molclr_bn_row_parts(int64_t dim);
/* Device-sized segments (a captured step over padded buffers): the rows of
 * every segment are read from seg_rows_dev [nseg] on the device; z / y / dy /
 * dz hold rows_cap rows, and rows past the segments' sum are padding (y and dz
 * zero there, no statistics).  Same per-segment plan as the host-sized calls,
 * so the real rows' results are bit-identical to theirs.  The backward's
 * rowmax / slot (fp32 only, may be NULL) as molclr_batchnorm_seg_bwd_max. */
size_t molclr_batchnorm_seg_dev_workspace_bytes(int nseg, int64_t rows_cap, int64_t dim);
int molclr_batchnorm_seg_fwd_dev(const void* z, const float* gamma, const float* beta,
                                 float* running_mean, float* running_var,
                                 int64_t* num_batches_tracked, void* y, float* save_mean,
                                 float* save_invstd, int nseg, const int64_t* seg_rows_dev,
                                 int64_t rows_cap, int64_t dim, int dtype, double momentum,
                                 double eps, int training, int relu, void* workspace,
                                 size_t workspace_bytes, molclr_stream_t stream);
int molclr_batchnorm_seg_bwd_dev(const void* dy, const void* z, const float* gamma,
                                 const float* beta, const float* save_mean,
                                 const float* save_invstd, void* dz, float* dgamma, float* dbeta,
                                 int nseg, const int64_t* seg_rows_dev, int64_t rows_cap,
                                 int64_t dim, int dtype, int relu, int accumulate, float* rowmax,
                                 float* slot, void* workspace, size_t workspace_bytes,
                                 molclr_stream_t stream);
int molclr_batchnorm_seg_bwd_max(const float* dy, const float* z, const float* gamma,
                                 const float* beta, const float* save_mean,
                                 const float* save_invstd, float* dz, float* dgamma, float* dbeta,
                                 int nseg, const int64_t* seg_rows, int64_t dim, int relu,
                                 int accumulate, float* rowmax, float* slot, void* workspace,
                                 size_t workspace_bytes, molclr_stream_t stream);

/* Segment pooling over graph_ptr (PyG global_mean_pool / global_add_pool):
 * mode 0 = mean (sum / max(count,1)), 1 = add. */
int molclr_segment_pool_fwd(const float* h, const int32_t* graph_ptr, float* out,
                            int64_t num_graphs, int64_t dim, int mode,
                            molclr_stream_t stream);
int molclr_segment_pool_bwd(const float* dout, const int32_t* graph_ptr, float* dh,
                            int64_t num_nodes, int64_t num_graphs, int64_t dim, int mode,
                            molclr_stream_t stream);
/* global_max_pool (models/ginet_molclr.py:85-86, gcn_molclr.py:125-126: PyG
 * 1.6.3 -> torch_scatter 2.0.6 scatter_max).  out[g][d] = max over the nodes
 * of graph g, argmax[g][d] = that node (the first in node order among equal
 * values; -1 and out = 0 for a graph without nodes).  h is fp32 or bf16
 * (dtype MOLCLR_DTYPE_*), out / dout fp32; the backward writes dout[g][d] to
 * dh[argmax[g][d]][d] and zero elsewhere (dh in h's dtype).  D % 4 == 0. */
int molclr_segment_max_fwd(const void* h, const int32_t* graph_ptr, float* out, int32_t* argmax,
                           int64_t num_graphs, int64_t dim, int dtype, molclr_stream_t stream);
int molclr_segment_max_bwd(const float* dout, const int32_t* argmax, void* dh, int64_t num_nodes,
                           int64_t num_graphs, int64_t dim, int dtype, molclr_stream_t stream);

/* F.normalize(z, dim=1, eps): y = z / max(||z||, eps); norm [rows] saved. */
int molclr_l2norm_fwd(const float* z, float* y, float* norm, int64_t rows, int64_t dim,
                      double eps, molclr_stream_t stream);
int molclr_l2norm_bwd(const float* dy, const float* y, const float* norm, float* dz,
                      int64_t rows, int64_t dim, double eps, molclr_stream_t stream);

/* ------------------------------------------------------------------------
 * NT-Xent (utils/nt_xent.py:47-65), row-sharded so it also serves the
 * data-parallel global batch.
 *   R = [zj ; zi] in the global order (nt_xent.py:48), 2B rows of width C.
 *   cosine != 0: rows are first scaled by 1/max(||r||, 1e-8)
 *       (torch CosineSimilarity, nt_xent.py:40-45); cosine == 0: dot.
 *   loss = (1/2B) Σ_r [ log Σ_{c≠r} exp(S_rc/T) − S_{r,(r+B) mod 2B}/T ].
 * This process owns `nrows` rows of R: `rows` [nrows,C] with global indices
 * row_gidx [nrows]; `cols` [2B,C] is the full (gathered) R.
 * ntxent_prep: rhat = scaled rows of a [n,C] matrix, norm [n] (clamped denominators).
 * ntxent_fwd:  lse_rows [nrows] (needed by every rank's backward) and
 *              loss_rows [nrows] = per-row loss / 2B.
 * ntxent_bwd:  drhat_rows [nrows,C] = dL/d(rhat rows) given the full
 *              lse_cols [2B] and the upstream scalar gradient *grad_loss.
 * ntxent_prep_bwd: chain rule through the row scaling. */
int molclr_ntxent_prep(const float* r, float* rhat, float* norm, int64_t n, int64_t C,
                       int cosine, molclr_stream_t stream);
int molclr_ntxent_prep_bwd(const float* drhat, const float* rhat, const float* norm,
                           float* dr, int64_t n, int64_t C, int cosine,
                           molclr_stream_t stream);
/* The paired step's F.normalize (molclr.py:63-64, eps) and ntxent_prep in one
 * launch, replacing l2norm_fwd + torch.cat([zjs, zis]) + ntxent_prep
 * (GINet.forward_pair's z = [zis; zjs], 2 * batch_local rows):
 *   rhat [2Bl,C] = scaled rows of R = [zjs; zis], y [2Bl,C] the normalised R,
 *   n1 [2Bl] = |R row| (unclamped, as l2norm_fwd's norm), n2 [2Bl] the clamped
 *   cosine denominator (1 for dot similarity).  Bit-identical to the three ops.
 * ntxent_prep_pair_bwd: dz [2Bl,C] in z's row order from drhat. */
int molclr_ntxent_prep_pair(const float* z, float* y, float* rhat, float* n1, float* n2,
                            int64_t batch_local, int64_t C, double eps, int cosine,
                            molclr_stream_t stream);
int molclr_ntxent_prep_pair_bwd(const float* drhat, const float* rhat, const float* n2,
                                const float* y, const float* n1, float* dz, int64_t batch_local,
                                int64_t C, double eps, int cosine, molclr_stream_t stream);
size_t molclr_ntxent_workspace_bytes(int64_t nrows, int64_t ncols, int64_t C);
int molclr_ntxent_fwd(const float* rhat_rows, const int32_t* row_gidx, const float* rhat_cols,
                      int64_t nrows, int64_t ncols, int64_t C, int64_t batch_size,
                      double temperature, float* lse_rows, float* loss_rows,
                      void* workspace, size_t workspace_bytes, molclr_stream_t stream);
int molclr_ntxent_bwd(const float* rhat_rows, const int32_t* row_gidx, const float* rhat_cols,
                      const float* lse_cols, const float* grad_loss, int64_t nrows,
                      int64_t ncols, int64_t C, int64_t batch_size, double temperature,
                      float* drhat_rows, void* workspace, size_t workspace_bytes,
                      molclr_stream_t stream);
/* molclr_ntxent_fwd / _bwd with the formulation chosen per call (tests and
 * benchmarks; -1 = automatic, as the calls above): 0 = fused f32-MFMA kernels
 * (similarity tiles recomputed in registers, online logsumexp, no S buffer);
 * 1 = S = rows cols^T as one split-bf16 GEMM (fp32 accuracy), then the row
 * logsumexp / the symmetric weights W as elementwise passes and dR = W cols as
 * a second GEMM (ncols % 4 == 0); 2 = the h3 form of 1 (S by three fp16
 * MFMAs per product, W^T through an LDS transpose, dR as an h3 weight-gradient
 * product; nrows, ncols, C % 4 == 0, C <= 1024, ncols >= 1024); 3 = the
 * transposed form of 2 (S^T = cols rows^T kept [ncols][nrows], the row
 * logsumexp down its columns, W^T elementwise in S^T's layout: no transpose
 * pass; same shapes as 2).  Automatic: 0
 * below 2^20 elements of S, 1 up to 2^22, 2 from there where its shapes allow.
 * sim (formulations 1, 2, 3; may be NULL): the forward writes row-major S
 * [nrows][ncols] there (1 and 2) or S^T [ncols][nrows] (3), and a backward given the same
 * buffer uses it instead of recomputing S.  molclr_ntxent_sim_bytes: its
 * size, 0 when the formulation chosen for (nrows, ncols, C, impl) keeps no S. */
size_t molclr_ntxent_sim_bytes(int64_t nrows, int64_t ncols, int64_t C, int impl);
int molclr_ntxent_fwd_impl(const float* rhat_rows, const int32_t* row_gidx,
                           const float* rhat_cols, int64_t nrows, int64_t ncols, int64_t C,
                           int64_t batch_size, double temperature, float* lse_rows,
                           float* loss_rows, float* sim, void* workspace, size_t workspace_bytes,
                           molclr_stream_t stream, int impl);
int molclr_ntxent_bwd_impl(const float* rhat_rows, const int32_t* row_gidx,
                           const float* rhat_cols, const float* lse_cols, const float* grad_loss,
                           int64_t nrows, int64_t ncols, int64_t C, int64_t batch_size,
                           double temperature, const float* sim, float* drhat_rows,
                           void* workspace, size_t workspace_bytes, molclr_stream_t stream,
                           int impl);
/* loss = Σ loss_rows (deterministic single-block sum). */
int molclr_sum_f32(const float* x, float* out, int64_t n, molclr_stream_t stream);

/* ------------------------------------------------------------------------
 * Adam with coupled L2 weight decay over one flat fp32 parameter buffer
 * (torch.optim.Adam semantics, molclr.py:84-87,127):
 *   g += wd·p; m = b1·m + (1−b1)·g; v = b2·v + (1−b2)·g²;
 *   p −= lr/(1−b1^t) · m / (sqrt(v)/sqrt(1−b2^t) + eps)
 * lr and step live in device memory so a captured step replays with the
 * current learning rate; *step is incremented by the kernel. */
int molclr_adam_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                     int64_t n, const float* lr, int32_t* step, double beta1, double beta2,
                     double eps, double weight_decay, molclr_stream_t stream);
/* molclr_adam_step with tick = 0 leaves the step counter alone (the update
 * uses *step + 1 as always): molclr_step_tail then advances it, and also
 * copies the loss scalar and ORs the batch's status word into a sticky word
 * (either may be NULL) -- the HIP-graph step's single closing launch. */
int molclr_adam_step_ex(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                        int64_t n, const float* lr, int32_t* step, double beta1, double beta2,
                        double eps, double weight_decay, int tick, molclr_stream_t stream);
int molclr_step_tail(int32_t* step, const float* loss_src, float* loss_dst,
                     const int32_t* status_src, int32_t* status_acc, molclr_stream_t stream);

/* ------------------------------------------------------------------------
 * GIN encoder executor (models/ginet_molclr.py:98-111 as ONE call).
 * Runs the whole node-embedding stack of GINet on the stream — atom
 * embedding, then per layer GINE aggregation -> Linear(D,2D)+ReLU ->
 * Linear(2D,D) -> BatchNorm1d (+ReLU, not on the last layer) — by calling
 * the entry points above in the order molclr_amd's per-op autograd path
 * calls them (identical kernels, identical results), without a host round
 * trip per operation.  The backward call replays the layers in reverse and
 * ADDS every parameter gradient into the given buffers.
 * Parameters are the reference's (state_dict names in the fields); the four
 * *_planes are molclr_bplanes_make images of the MLP weights as GEMM B
 * operands:
 *   mlp0_planes   : B(k,n) = W0[n][k], N = 2D, K = D   (ldb = D,  b_kmajor 0)
 *   mlp0_planes_t : B(k,n) = W0[k][n], N = D,  K = 2D  (ldb = D,  b_kmajor 1)
 *   mlp2_planes   : B(k,n) = W2[n][k], N = D,  K = 2D  (ldb = 2D, b_kmajor 0)
 *   mlp2_planes_t : B(k,n) = W2[k][n], N = 2D, K = D   (ldb = 2D, b_kmajor 1)
 * BatchNorm: training = batch statistics + running-stat update (momentum,
 * num_batches_tracked may be NULL); eval = running statistics (no backward).
 * ------------------------------------------------------------------------ */
typedef struct molclr_gin_encoder {
  int32_t num_layer;  /* 1 .. MOLCLR_MAX_LAYERS */
  int32_t training;
  int64_t dim;        /* emb_dim, multiple of 4 */
  int64_t n_atom;     /* x_embedding1 rows (119) */
  int64_t n_chiral;   /* x_embedding2 rows (3) */
  double momentum, eps;
  const float* x_embedding1;
  const float* x_embedding2;
  const float* mlp0_weight[MOLCLR_MAX_LAYERS];
  const float* mlp0_bias[MOLCLR_MAX_LAYERS];
  const float* mlp2_weight[MOLCLR_MAX_LAYERS];
  const float* mlp2_bias[MOLCLR_MAX_LAYERS];
  const float* edge_embedding1[MOLCLR_MAX_LAYERS];
  const float* edge_embedding2[MOLCLR_MAX_LAYERS];
  const float* bn_weight[MOLCLR_MAX_LAYERS];
  const float* bn_bias[MOLCLR_MAX_LAYERS];
  float* bn_running_mean[MOLCLR_MAX_LAYERS];
  float* bn_running_var[MOLCLR_MAX_LAYERS];
  int64_t* bn_num_batches_tracked[MOLCLR_MAX_LAYERS];
  const uint16_t* mlp0_planes[MOLCLR_MAX_LAYERS];
  const uint16_t* mlp0_planes_t[MOLCLR_MAX_LAYERS];
  const uint16_t* mlp2_planes[MOLCLR_MAX_LAYERS];
  const uint16_t* mlp2_planes_t[MOLCLR_MAX_LAYERS];
  /* MOLCLR_DTYPE_F32: fp32 node features, split-bf16 GEMMs (fp32 accuracy).
   * MOLCLR_DTYPE_BF16 (dim % 8 == 0): bf16 node features and activation
   * gradients, one bf16 MFMA per product with fp32 accumulation (plane 0 of
   * the *_planes images is the bf16 weight), fp32 statistics, tables, and
   * parameter gradients: the c5 configuration / the reference's
   * mixed-precision switch (molclr.py:16-24,93-96,121-123).  h_out / dh_out
   * are then bf16. */
  int32_t dtype;
  /* fp32 storage only, which products run in "h3" (molclr_gemm_f32_h3 /
   * molclr_linear_wgrad_h3, 2 dim <= 1024) instead of split-bf16 "x6":
   * 0 = none; bit 0 = the backward (weight gradients with per-tensor scales,
   * data gradients with row-wise scales; mlp*_planes_t are then
   * molclr_hplanes_make_batch images); bit 1 = the forward products too
   * (mlp0/2_planes h3 images, A scaled row by row; the Python side's default,
   * 3 = both).  The max slots of agg / a1 live in the arena, those of dz /
   * dz1 and all row maxima in the workspace. */
  int32_t fp32_gemm;
  /* nullable: receives MOLCLR_STATUS_ATOM_RANGE (molclr_atom_embed_fwd) */
  int32_t* status;
} molclr_gin_encoder;

/* Gradient buffers, same shapes as the parameters; NULL = not needed. */
typedef struct molclr_gin_encoder_grads {
  float* x_embedding1;
  float* x_embedding2;
  float* mlp0_weight[MOLCLR_MAX_LAYERS];
  float* mlp0_bias[MOLCLR_MAX_LAYERS];
  float* mlp2_weight[MOLCLR_MAX_LAYERS];
  float* mlp2_bias[MOLCLR_MAX_LAYERS];
  float* edge_embedding1[MOLCLR_MAX_LAYERS];
  float* edge_embedding2[MOLCLR_MAX_LAYERS];
  float* bn_weight[MOLCLR_MAX_LAYERS];
  float* bn_bias[MOLCLR_MAX_LAYERS];
  /* Optional (NULL = none): hipEvent_t handles the backward records on its
   * stream once layer l's parameter gradients (its Linear / GCN weights,
   * edge tables and BatchNorm affine) are final, and once the atom-embedding
   * gradients are: a data-parallel caller starts each layer's gradient
   * all-reduce behind its event while the lower layers' backward runs. */
  void* layer_done[MOLCLR_MAX_LAYERS];
  void* embed_done;
} molclr_gin_encoder_grads;

/* The graph of one batch as molclr_graph_build produced it. */
/* num_segments > 1: the graph is molclr_graph_build_multi's union of that many
 * batches with segment_nodes[s] nodes each; the executors keep the
 * BatchNorm statistics of every segment apart (molclr_batchnorm_seg_fwd).
 * num_segments 0 or 1: one batch. */
typedef struct molclr_device_graph {
  int64_t num_nodes, num_edges, num_graphs;
  const int32_t *rowptr, *col, *rowptr_t, *col_t, *ecount, *graph_ptr;
  const uint8_t* ecode;
  const uint32_t *nbr, *nbr_t;
  int32_t num_segments;
  int64_t segment_nodes[MOLCLR_MAX_SEGMENTS];
  /* NULL, or (molclr_graph_build_dev) the segments' node counts on the device:
   * num_nodes is then the capacity, segment_nodes is unused and the rows past
   * the counts' sum are padding */
  const int64_t* segment_nodes_dev;
} molclr_device_graph;

/* Saved activations of one forward (kept for the backward): arena of
 * molclr_gin_encoder_arena_bytes; scratch: molclr_gin_encoder_workspace_bytes. */
size_t molclr_gin_encoder_arena_bytes(int num_layer, int64_t num_nodes, int64_t dim, int dtype);
size_t molclr_gin_encoder_workspace_bytes(int num_layer, int64_t num_nodes, int64_t dim,
                                          int dtype);
/* x int64 [N,2] (atom type, chirality); h_out [N,D] (enc->dtype): the last
 * BatchNorm's output. */
int molclr_gin_encoder_fwd(const molclr_gin_encoder* enc, const int64_t* x,
                           const molclr_device_graph* graph, void* h_out, void* arena,
                           size_t arena_bytes, void* workspace, size_t workspace_bytes,
                           molclr_stream_t stream);
/* dh_out [N,D] (enc->dtype): gradient w.r.t. h_out; grads are accumulated (+=). */
int molclr_gin_encoder_bwd(const molclr_gin_encoder* enc, const molclr_gin_encoder_grads* grads,
                           const int64_t* x, const molclr_device_graph* graph,
                           const void* dh_out, const void* arena, size_t arena_bytes,
                           void* workspace, size_t workspace_bytes, molclr_stream_t stream);

/* GCN encoder executor: GCN's node-embedding stack (models/gcn_molclr.py:140-151:
 * atom embedding, per layer GCNConv -> BatchNorm1d (+ReLU but the last)) in one
 * host call per direction, issuing the same entry points as the per-op path
 * (molclr_amd.ops: gemm_w, molclr_gcn_aggregate_fwd/_bwd, batchnorm, gemm) in
 * its order, so the results are identical.  weight[l] is GCNConv.weight
 * [D_in, D_out] (not transposed, gcn_molclr.py:45); weight_planes[l] its planes
 * as the B operand of x W (molclr_bplanes_make(W, D, D, D, b_kmajor=1)),
 * weight_planes_t[l] as the B operand of dxw W^T (b_kmajor=0). */
typedef struct molclr_gcn_encoder {
  int32_t num_layer;
  int32_t training;
  int64_t dim;
  int64_t n_atom;
  int64_t n_chiral;
  double momentum, eps;
  const float* x_embedding1;
  const float* x_embedding2;
  const float* weight[MOLCLR_MAX_LAYERS];
  const float* bias[MOLCLR_MAX_LAYERS];
  const float* edge_embedding1[MOLCLR_MAX_LAYERS]; /* [5,1] */
  const float* edge_embedding2[MOLCLR_MAX_LAYERS]; /* [3,1] */
  const float* bn_weight[MOLCLR_MAX_LAYERS];
  const float* bn_bias[MOLCLR_MAX_LAYERS];
  float* bn_running_mean[MOLCLR_MAX_LAYERS];
  float* bn_running_var[MOLCLR_MAX_LAYERS];
  int64_t* bn_num_batches_tracked[MOLCLR_MAX_LAYERS];
  const uint16_t* weight_planes[MOLCLR_MAX_LAYERS];
  const uint16_t* weight_planes_t[MOLCLR_MAX_LAYERS];
  /* 0 = split-bf16 x6 products; 1 = the backward in h3 (as molclr_gin_encoder's
   * bit 0: the weight gradient with per-tensor scales, dx = dxw W^T with
   * row-wise scales; weight_planes_t are then molclr_hplanes_make_batch
   * images, dim <= 1024). */
  int32_t fp32_gemm;
  int32_t* status; /* nullable: MOLCLR_STATUS_ATOM_RANGE, as molclr_gin_encoder */
} molclr_gcn_encoder;

typedef struct molclr_gcn_encoder_grads {
  float* x_embedding1;
  float* x_embedding2;
  float* weight[MOLCLR_MAX_LAYERS];
  float* bias[MOLCLR_MAX_LAYERS];
  float* edge_embedding1[MOLCLR_MAX_LAYERS];
  float* edge_embedding2[MOLCLR_MAX_LAYERS];
  float* bn_weight[MOLCLR_MAX_LAYERS];
  float* bn_bias[MOLCLR_MAX_LAYERS];
  void* layer_done[MOLCLR_MAX_LAYERS]; /* as in molclr_gin_encoder_grads */
  void* embed_done;
} molclr_gcn_encoder_grads;

size_t molclr_gcn_encoder_arena_bytes(int num_layer, int64_t num_nodes, int64_t dim);
size_t molclr_gcn_encoder_workspace_bytes(int num_layer, int64_t num_nodes, int64_t dim);
int molclr_gcn_encoder_fwd(const molclr_gcn_encoder* enc, const int64_t* x,
                           const molclr_device_graph* graph, float* h_out, void* arena,
                           size_t arena_bytes, void* workspace, size_t workspace_bytes,
                           molclr_stream_t stream);
int molclr_gcn_encoder_bwd(const molclr_gcn_encoder* enc, const molclr_gcn_encoder_grads* grads,
                           const int64_t* x, const molclr_device_graph* graph,
                           const float* dh_out, const void* arena, size_t arena_bytes,
                           void* workspace, size_t workspace_bytes, molclr_stream_t stream);

/* ------------------------------------------------------------------------
 * bf16 storage (BASELINE config c5: GIN 5 x 512, bf16, batch 1024 / GPU).
 * Node features and activation gradients are bf16 ([N,D] of uint16 bit
 * patterns, round-to-nearest-even); all arithmetic, tables, statistics and
 * parameter gradients are fp32.  Same semantics as the fp32 entry points.
 * ------------------------------------------------------------------------ */
int molclr_atom_embed_fwd_bf16(const int64_t* x, const float* X1, const float* X2, uint16_t* h,
                               int64_t num_nodes, int64_t dim, int64_t n1, int64_t n2,
                               int32_t* status, molclr_stream_t stream);
/* workspace: molclr_atom_embed_bwd_workspace_bytes */
int molclr_atom_embed_bwd_bf16(const int64_t* x, const uint16_t* dh, float* dX1, float* dX2,
                               int64_t num_nodes, int64_t dim, int64_t n1, int64_t n2,
                               int accumulate, void* workspace, size_t workspace_bytes,
                               molclr_stream_t stream);
int molclr_gine_aggregate_fwd_bf16(const uint16_t* x, const int32_t* rowptr, const int32_t* col,
                                   const uint8_t* ecode, const uint32_t* nbr, const float* Ec,
                                   uint16_t* out, int64_t num_nodes, int64_t dim,
                                   molclr_stream_t stream);
/* workspace: molclr_gine_aggregate_bwd_workspace_bytes */
int molclr_gine_aggregate_bwd_bf16(const uint16_t* g, const int32_t* rowptr_t,
                                   const int32_t* col_t, const uint32_t* nbr_t,
                                   const int32_t* ecount, uint16_t* dx, float* dE1, float* dE2,
                                   int64_t num_nodes, int64_t dim, int accumulate, void* workspace,
                                   size_t workspace_bytes, molclr_stream_t stream);
/* h bf16 -> out fp32 [G,D]; dout fp32 -> dh bf16 */
int molclr_segment_pool_fwd_bf16(const uint16_t* h, const int32_t* graph_ptr, float* out,
                                 int64_t num_graphs, int64_t dim, int mode,
                                 molclr_stream_t stream);
int molclr_segment_pool_bwd_bf16(const float* dout, const int32_t* graph_ptr, uint16_t* dh,
                                 int64_t num_nodes, int64_t num_graphs, int64_t dim, int mode,
                                 molclr_stream_t stream);
/* C[M,N] (bf16) = epilogue(Σ_k A[m][k] B(k,n)), A bf16 row-major (lda), B the
 * weight operand as molclr_bplanes_make planes (plane 0 = bf16(B) is read),
 * one v_mfma_f32_32x32x16_bf16 per product, fp32 accumulation.  Epilogues:
 * NONE / BIAS / BIAS_RELU (bias fp32) / RELU_MASK (aux bf16, ldaux % 4 == 0);
 * no accumulate.  K and lda multiples of 8, ldc a multiple of 4. */
int molclr_gemm_bf16(const uint16_t* A, const uint16_t* planes, uint16_t* C, int64_t M, int64_t N,
                     int64_t K, int64_t lda, int64_t ldc, int epilogue, const float* bias,
                     const uint16_t* aux, int64_t ldaux, molclr_stream_t stream);
/* The same with the tile shape chosen per call (tests and benchmarks; -1 =
 * automatic, as molclr_gemm_bf16): output tiles 0 = 128 x 128, 1 = 128 x 256,
 * 2 = 128 x 512, 3 = 64 x 512, 4 = 128 x 256 (8 waves), 5 = 128 x 128 (shallow
 * A prefetch), 6 = 256 x 256 with LDS-DMA staging (K % 64 == 0), 7 = 256 x 256
 * with a four-stage LDS-DMA ring (K % 32 == 0), 8 = 6 as a persistent kernel
 * (one block per CU, epilogue overlapped with the next tile's staging; K % 64
 * == 0); 6, 7 and 8 fall back to 2 for other K.  Every shape gives the same
 * result bits (those of hipBLASLt's bf16
 * GEMM on the epilogue-free products). */
int molclr_gemm_bf16_impl(const uint16_t* A, const uint16_t* planes, uint16_t* C, int64_t M,
                          int64_t N, int64_t K, int64_t lda, int64_t ldc, int epilogue,
                          const float* bias, const uint16_t* aux, int64_t ldaux,
                          molclr_stream_t stream, int impl);
/* molclr_gemm_bf16 (the persistent 256 x 256 kernel; K % 64 == 0) with the
 * ReLU mask as bits -- column-block-major words bits[n / 32][m], bit n % 32 =
 * (C[m][n] > 0), ceil(N / 32) x M words (molclr_gemm_f32_bplanes_max's
 * layout): epilogue MOLCLR_EPI_BIAS_RELU writes them to bits_out (the GIN
 * MLP's first Linear, ginet_molclr.py:19-23), MOLCLR_EPI_RELU_MASK takes its
 * mask from bits_in instead of a bf16 aux matrix (the ReLU backward): 1/16 of
 * the mask bytes.  Results equal the aux form's bit for bit. */
int molclr_gemm_bf16_bits(const uint16_t* A, const uint16_t* planes, uint16_t* C, int64_t M,
                          int64_t N, int64_t K, int64_t lda, int64_t ldc, int epilogue,
                          const float* bias, uint32_t* bits_out, const uint32_t* bits_in,
                          molclr_stream_t stream);
/* Linear weight / bias gradients from bf16 operands into fp32:
 * dW[n_out][n_in] (+)= Σ_r dy[r][o] x[r][i], db (+)= Σ_r dy[r][o] (db may be
 * NULL); n_out, n_in, ld_dy, ld_x multiples of 8.  Split-K partials summed in
 * a fixed order (deterministic). */
size_t molclr_linear_wgrad_bf16_workspace_bytes(int64_t rows, int64_t n_out, int64_t n_in);
int molclr_linear_wgrad_bf16(const uint16_t* dy, const uint16_t* x, float* dW, float* db,
                             int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                             int64_t ld_x, int accumulate, void* workspace,
                             size_t workspace_bytes, molclr_stream_t stream);
/* The same with the kernel chosen per call (-1 = automatic): 0 = 128 x 128,
 * 1 = 256 x 256, 2 = 128 x 256 output tiles with register staging, 3 = 256 x
 * 256 with both operands LDS-DMA staged (64-row K steps); each has its own
 * split-K plan (the workspace query covers all). */
int molclr_linear_wgrad_bf16_impl(const uint16_t* dy, const uint16_t* x, float* dW, float* db,
                                  int64_t rows, int64_t n_out, int64_t n_in, int64_t ld_dy,
                                  int64_t ld_x, int accumulate, void* workspace,
                                  size_t workspace_bytes, molclr_stream_t stream, int impl);

/* ---- Benchmark instrumentation (no reference counterpart) -------------------
 * Opt-in kernel timer.  While a kind is enabled, its launches go through
 * hipExtLaunchKernelGGL with a start/stop event pair recorded by the dispatch
 * itself, so each sample is the kernel's own execution window (the figure
 * rocprofv3 --kernel-trace reports).  Kinds (a bit mask): 1 = k_gine_agg_fwd,
 * 2 = every kernel of molclr_gemm_f32 (main GEMM + split-K reduce), 4 = the
 * NT-Xent similarity kernels, 8 = k_gcn_agg_fwd. */
#define MOLCLR_KTIMER_GINE_AGG 1
#define MOLCLR_KTIMER_GEMM 2
#define MOLCLR_KTIMER_NTXENT 4 /* k_ntxent_fwd_partial / k_ntxent_bwd_partial */
#define MOLCLR_KTIMER_GCN_AGG 8
int molclr_ktimer_start(int kinds_mask);
/* Waits for the recorded launches of `kind`, returns their summed duration
 * and count, and forgets them. */
int molclr_ktimer_read(int kind, double* total_ms, int64_t* launches);
/* Disables timing and discards unread samples. */
int molclr_ktimer_stop(void);

#ifdef __cplusplus
}
#endif
#endif /* MOLCLR_H_ */
