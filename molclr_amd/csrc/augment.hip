// On-device node-mask augmentation + collate.
//
// The reference builds every contrastive view on the host, per molecule, in
// MoleculeDataset.__getitem__ (dataset/dataset.py:111-147): mask
// max(1, floor(0.25 N)) atoms to [118, 0], drop floor(0.25 M) bonds (both
// directed edges 2i, 2i+1), keep the surviving edges in their original order;
// the DataLoader then collates the views with PyG's Batch.from_data_list
// (x / edge_attr concatenated, edge_index offset by the running atom count,
// ascending `batch`, `ptr`).  Here one wave per molecule does the whole thing
// from a molecule store resident in HBM and writes the collated Batch fields
// directly, so a step's input never touches the host.
//
// Random subsets: the reference draws them with Python's unseeded
// random.sample.  Here item i of a molecule is chosen when its 64-bit key
// (a splitmix64 hash of seed, view, kind, molecule id, i) ranks among the k
// smallest (ties by index) -- a uniformly random k-subset, reproducible from
// the seed and the same on every rank count.  oracle/augment_ref.py restates
// the keys bit for bit.
#include "common.h"

namespace {

constexpr int kMolsPerBlock = 4;  // one wave per molecule

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Stream of one (seed, view, kind, molecule): a chain of splitmix64 over the
// four fields, so distinct tuples give unrelated streams (a flat
// seed ^ (2 view + kind) would make view 1 at seed s replay view 0 at s ^ 2).
// kind 0 = atoms, 1 = bonds.
__device__ __forceinline__ uint64_t subset_stream(uint64_t seed, int view, int kind, int64_t id) {
  uint64_t z = splitmix64(seed);
  z = splitmix64(z ^ (uint64_t)view);
  z = splitmix64(z ^ (uint64_t)kind);
  return splitmix64(z ^ (uint64_t)id);
}

// key of item i of one stream
__device__ __forceinline__ uint64_t item_key(uint64_t stream, int64_t i) {
  return splitmix64(stream ^ (uint64_t)i);
}

// i is among the k smallest keys of the n items (ties broken by index)
__device__ __forceinline__ bool chosen(uint64_t stream, int64_t n, int64_t k, int64_t i) {
  if (k <= 0) return false;
  if (k >= n) return true;
  const uint64_t ki = item_key(stream, i);
  int64_t rank = 0;
  for (int64_t j = 0; j < n && rank < k; ++j) {
    const uint64_t kj = item_key(stream, j);
    rank += (kj < ki || (kj == ki && j < i)) ? 1 : 0;
  }
  return rank < k;
}

// per batch slot: ptr (atom offsets, the Batch's ptr) and kept-edge offsets;
// one block, chunked scan (B is at most a few thousand molecules)
__global__ void k_mask_offsets(const int64_t* __restrict__ atom_ptr,
                               const int64_t* __restrict__ bond_ptr,
                               const int64_t* __restrict__ mol_ids, int64_t B, int64_t G,
                               int64_t* __restrict__ ptr_out, int64_t* __restrict__ edge_off,
                               int64_t num_nodes, int64_t num_edges,
                               int32_t* __restrict__ status) {
  __shared__ int64_t sa[1024], se[1024];
  __shared__ int64_t carry_a, carry_e;
  const int t = threadIdx.x;
  if (t == 0) {
    carry_a = 0;
    carry_e = 0;
    *status = 0;
  }
  __syncthreads();
  int bad = 0;
  for (int64_t base = 0; base < B; base += 1024) {
    const int64_t b = base + t;
    int64_t n = 0, e = 0;
    if (b < B) {
      int64_t id = mol_ids[b];
      if (id < 0 || id >= G) {
        bad |= 1;
      } else {
        n = atom_ptr[id + 1] - atom_ptr[id];
        const int64_t m = bond_ptr[id + 1] - bond_ptr[id];
        e = 2 * (m - m / 4);
      }
    }
    sa[t] = n;
    se[t] = e;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {  // inclusive Hillis-Steele
      const int64_t va = t >= off ? sa[t - off] : 0;
      const int64_t ve = t >= off ? se[t - off] : 0;
      __syncthreads();
      sa[t] += va;
      se[t] += ve;
      __syncthreads();
    }
    if (b < B) {
      ptr_out[b] = carry_a + sa[t] - n;
      edge_off[b] = carry_e + se[t] - e;
    }
    __syncthreads();
    if (t == 1023) {
      carry_a += sa[t];
      carry_e += se[t];
    }
    __syncthreads();
  }
  if (t == 0) {
    ptr_out[B] = carry_a;
    edge_off[B] = carry_e;
    if (carry_a != num_nodes || carry_e != num_edges) bad |= 2;
  }
  if (bad) atomicOr(status, bad);
}

__global__ __launch_bounds__(64 * kMolsPerBlock) void k_mask_views(
    const int64_t* __restrict__ sx, const int64_t* __restrict__ atom_ptr,
    const int64_t* __restrict__ sei, const int64_t* __restrict__ sea,
    const int64_t* __restrict__ bond_ptr, int64_t store_edges, const int64_t* __restrict__ mol_ids,
    int64_t B, int64_t G, uint64_t seed, int view, const int64_t* __restrict__ ptr,
    const int64_t* __restrict__ edge_off, int64_t* __restrict__ x_out,
    int64_t* __restrict__ ei_out, int64_t* __restrict__ ea_out, int64_t* __restrict__ batch_out,
    int64_t num_nodes, int64_t num_edges, int32_t* __restrict__ status) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kMolsPerBlock + (threadIdx.x >> 6);
  if (b >= B) return;  // wave-uniform
  const int64_t id = mol_ids[b];
  if (id < 0 || id >= G) return;  // flagged by k_mask_offsets
  const int64_t a0 = atom_ptr[id], n = atom_ptr[id + 1] - a0;
  const int64_t m0 = bond_ptr[id], M = bond_ptr[id + 1] - m0;
  const int64_t aoff = ptr[b], eoff = edge_off[b];
  // ptr / edge_off totals were checked against the output sizes; these guards
  // keep a mismatched call in bounds
  if (aoff + n > num_nodes || eoff + 2 * (M - M / 4) > num_edges) return;
  const int64_t k_atoms = n > 0 ? (n / 4 > 1 ? n / 4 : 1) : 0;  // max(1, floor(0.25 N))
  const int64_t k_bonds = M / 4;                                // floor(0.25 M)
  const uint64_t atom_stream = subset_stream(seed, view, 0, id);
  const uint64_t bond_stream = subset_stream(seed, view, 1, id);

  for (int64_t i = lane; i < n; i += 64) {
    const bool masked = chosen(atom_stream, n, k_atoms, i);
    const int64_t o = aoff + i;
    const int64_t* src = sx + 2 * (a0 + i);
    x_out[2 * o] = masked ? 118 : src[0];  // len(ATOM_LIST): the mask token
    x_out[2 * o + 1] = masked ? 0 : src[1];
    batch_out[o] = b;
  }

  int bad = 0;
  int64_t kept_before = 0;
  for (int64_t base = 0; base < M; base += 64) {  // wave-uniform trip count
    const int64_t m = base + lane;
    const bool live = m < M;
    const bool keep = live && !chosen(bond_stream, M, k_bonds, m);
    const uint64_t bal = __ballot(keep);
    if (keep) {
      const int64_t p = kept_before + __popcll(bal & ((1ull << lane) - 1ull));
#pragma unroll
      for (int d = 0; d < 2; ++d) {  // the directed pair (s, e), (e, s)
        const int64_t se = 2 * (m0 + m) + d;
        const int64_t oe = eoff + 2 * p + d;
        int64_t s = sei[se], t = sei[store_edges + se];
        if (s < 0 || s >= n || t < 0 || t >= n) {
          bad |= 4;
          s = s < 0 ? 0 : (s >= n ? n - 1 : s);
          t = t < 0 ? 0 : (t >= n ? n - 1 : t);
        }
        ei_out[oe] = s + aoff;
        ei_out[num_edges + oe] = t + aoff;
        ea_out[2 * oe] = sea[2 * se];
        ea_out[2 * oe + 1] = sea[2 * se + 1];
      }
    }
    kept_before += __popcll(bal);
  }
  if (bad) atomicOr(status, bad);
}

}  // namespace

MOLCLR_API size_t molclr_mask_views_workspace_bytes(int64_t batch_size) {
  return (size_t)(batch_size + 1) * sizeof(int64_t) + 256;
}

MOLCLR_API int molclr_mask_views(const int64_t* store_x, const int64_t* store_atom_ptr,
                                 const int64_t* store_edge_index, const int64_t* store_edge_attr,
                                 const int64_t* store_bond_ptr, int64_t store_mols,
                                 int64_t store_edges, const int64_t* mol_ids, int64_t batch_size,
                                 uint64_t seed, int view, int64_t* x_out, int64_t* edge_index_out,
                                 int64_t* edge_attr_out, int64_t* batch_out, int64_t* ptr_out,
                                 int64_t num_nodes, int64_t num_edges, int32_t* status,
                                 void* workspace, size_t workspace_bytes,
                                 molclr_stream_t stream) {
  MOLCLR_REQUIRE(batch_size >= 0 && store_mols >= 0 && store_edges >= 0 && num_nodes >= 0 &&
                     num_edges >= 0,
                 "mask_views: negative size");
  MOLCLR_REQUIRE(view == 0 || view == 1, "mask_views: view must be 0 or 1");
  MOLCLR_REQUIRE(ptr_out && status, "mask_views: null pointer");
  MOLCLR_REQUIRE(batch_size == 0 || (store_atom_ptr && store_bond_ptr && mol_ids),
                 "mask_views: null pointer");
  MOLCLR_REQUIRE(num_nodes == 0 || (store_x && x_out && batch_out), "mask_views: null pointer");
  MOLCLR_REQUIRE(num_edges == 0 || (store_edge_index && store_edge_attr && edge_index_out &&
                                    edge_attr_out),
                 "mask_views: null pointer");
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_mask_views_workspace_bytes(batch_size));
  hipStream_t s = molclr::as_stream(stream);
  int64_t* edge_off = static_cast<int64_t*>(workspace);
  hipLaunchKernelGGL(k_mask_offsets, dim3(1), dim3(1024), 0, s, store_atom_ptr, store_bond_ptr,
                     mol_ids, batch_size, store_mols, ptr_out, edge_off, num_nodes, num_edges,
                     status);
  if (batch_size > 0)
    hipLaunchKernelGGL(k_mask_views, dim3((unsigned)molclr::ceil_div(batch_size, kMolsPerBlock)),
                       dim3(64 * kMolsPerBlock), 0, s, store_x, store_atom_ptr, store_edge_index,
                       store_edge_attr, store_bond_ptr, store_edges, mol_ids, batch_size,
                       store_mols, seed, view, static_cast<const int64_t*>(ptr_out),
                       static_cast<const int64_t*>(edge_off), x_out, edge_index_out,
                       edge_attr_out, batch_out, num_nodes, num_edges, status);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
