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

// ---------------------------------------------------------------------------
// Subgraph-removal views (dataset/dataset_subgraph.py:70-177) and the mixed
// subgraph + atom / bond masking views (dataset/dataset_mix.py:46-217).
//
// Per molecule the reference builds a networkx graph from the bonds
// (nx.Graph(edges): nodes in order of first appearance in the bond list,
// each node's neighbours in bond order; the Graph.copy() inside the removal
// then lists a node's earlier-in-node-order neighbours first, in node order,
// and the later ones in bond order), removes a BFS "subgraph" from a
// random centre (removeSubgraph / remove_subgraph), masks the removed atoms
// to [118, 0] and keeps the bonds that survive in G_i.edges.  One wave per
// molecule restates that loop with lane 0 in LDS:
//   temp = [centre]; while len(removed) < num:
//     (mix's guard, applied in both modes: stop when temp is empty -- the
//      subgraph module would loop forever; flagged in status bit 3)
//     neighbors = [i for n in temp for i in G.neighbors(n) if i not in temp]
//     remove the temp nodes in order until num are removed
//     temp = list(set(neighbors))
// The frontier's order is CPython's set iteration order, which decides which
// atoms go when `num` runs out inside a frontier, so the set is emulated
// exactly: open addressing over 8 << k slots, key = hash = the atom index,
// ten consecutive slots probed from i while i + 9 <= mask, then
// i = 5 i + 1 + (perturb >>= 5); growth to the next power of two above
// 4 x used when fill x 5 >= mask x 3, re-inserting in old-slot order; the
// list is the slot order (CPython 3.x setobject.c; oracle/augment_ref.py
// uses Python's own set).
// Bond survival: mix keeps a bond whose two atoms remain; the subgraph module
// tests only `(start, end) in G_i.edges`, and networkx reports an edge from
// the endpoint that comes first in node order, so a surviving bond whose end
// atom appeared in the bond list before its start atom is dropped there too.
// Random draws (the reference: Python's unseeded random; here splitmix64
// streams, restated in oracle/augment_ref.py): the two views' centres are the
// atoms with the smallest / second smallest key of one molecule stream
// (random.sample(range(N), 2): distinct); mix's percent is 0.2 u with u the
// top 53 bits of a per-view key; mix's extra atom / bond masks are the
// k-smallest-key subsets of the remaining atoms / surviving bonds.
// ---------------------------------------------------------------------------
constexpr int kAugMaxAtoms = 256;  // per molecule in the LDS plan; larger: k_aug_plan_big
constexpr int kAugMaxBonds = 512;
constexpr int kSetSlots = 2048;    // the emulated set never exceeds this for <= 256 keys

// The plan's tables: in LDS (int16 indices) for molecules within the caps
// above, or (int32 indices) in a global workspace slot for larger ones.
template <typename I>
struct AugTabs {
  I* adj_off;      // [n + 1]
  I* adj;          // [2 M]
  I* first;        // [n] position in nx node order, -1: not in the bond graph
  I* removed;      // [n]
  I* in_temp;      // [n]
  I* temp;         // [n]
  I* nbr;          // [2 M]
  I* table;        // [set slots]
  I* fill_cursor;  // [n]
};

struct AugLds {
  int16_t adj_off[kAugMaxAtoms + 1];
  int16_t adj[2 * kAugMaxBonds];
  int16_t first[kAugMaxAtoms];
  int16_t removed[kAugMaxAtoms];
  int16_t in_temp[kAugMaxAtoms];
  int16_t temp[kAugMaxAtoms];
  int16_t nbr[2 * kAugMaxBonds];
  int16_t table[kSetSlots];
  int16_t fill_cursor[kAugMaxAtoms];
};

// set slots a molecule of n atoms can need: CPython grows to the power of two
// above 4 x fill (fill <= n), from 8
__host__ __device__ inline int64_t aug_set_slots(int64_t n) {
  int64_t s = 8;
  while (s <= 4 * n) s <<= 1;
  return s;
}
// int32 elements of one global-workspace slot for n atoms / M bonds
__host__ __device__ inline int64_t aug_big_slot_elems(int64_t n, int64_t M) {
  return (n + 1) + 2 * M + 5 * n + 2 * M + aug_set_slots(n) + n + 4;
}

// CPython set(list) of non-negative ints: iteration order into out, returns
// its length.  `scratch` holds the old keys during a resize (it may be `out`:
// out is written only at the end).
template <typename I>
__device__ int pyset_order(const I* items, int n_items, I* table, I* out, I* scratch) {
  int mask = 7, fill = 0;
  for (int t = 0; t <= mask; ++t) table[t] = -1;
  auto insert_clean = [&](int k) {
    uint32_t i = (uint32_t)k & mask, perturb = (uint32_t)k;
    while (true) {
      if (table[i] < 0) {
        table[i] = (I)k;
        return;
      }
      if (i + 9 <= (uint32_t)mask)
        for (uint32_t j = i + 1; j <= i + 9; ++j)
          if (table[j] < 0) {
            table[j] = (I)k;
            return;
          }
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
    }
  };
  for (int q = 0; q < n_items; ++q) {
    const int k = items[q];
    uint32_t i = (uint32_t)k & mask, perturb = (uint32_t)k;
    bool inserted = false;
    for (;;) {
      const uint32_t last = (i + 9 <= (uint32_t)mask) ? i + 9 : i;
      bool done = false;
      for (uint32_t j = i; j <= last; ++j) {
        if (table[j] < 0) {
          table[j] = (I)k;
          inserted = done = true;
          break;
        }
        if (table[j] == k) {
          done = true;
          break;
        }
      }
      if (done) break;
      perturb >>= 5;
      i = (i * 5 + 1 + perturb) & mask;
    }
    if (inserted && ++fill * 5 >= mask * 3) {
      int old = 0;
      for (int t = 0; t <= mask; ++t)
        if (table[t] >= 0) scratch[old++] = table[t];
      int newsize = 8;
      while (newsize <= fill * 4) newsize <<= 1;
      mask = newsize - 1;
      for (int t = 0; t <= mask; ++t) table[t] = -1;
      for (int t = 0; t < old; ++t) insert_clean(scratch[t]);
    }
  }
  int n = 0;
  for (int t = 0; t <= mask; ++t)
    if (table[t] >= 0) out[n++] = table[t];
  return n;
}

// pass 1: per batch slot atom and bond offsets (ptr_out, bond_off), sizes
// checked against the caps (big_caps: the large-molecule slots' atoms / bonds,
// 0 / 0 without a large-molecule pass); zeroes the large-molecule slot counter
__global__ void k_aug_offsets(const int64_t* __restrict__ atom_ptr,
                              const int64_t* __restrict__ bond_ptr,
                              const int64_t* __restrict__ mol_ids, int64_t B, int64_t G,
                              int64_t* __restrict__ ptr_out, int64_t* __restrict__ bond_off,
                              int64_t num_nodes, int32_t* __restrict__ status, int64_t big_atoms,
                              int64_t big_bonds, int32_t* __restrict__ big_counter) {
  __shared__ int64_t sa[1024], se[1024];
  __shared__ int64_t carry_a, carry_e;
  const int t = threadIdx.x;
  if (t == 0) {
    carry_a = 0;
    carry_e = 0;
    *status = 0;
    if (big_counter) *big_counter = 0;
  }
  __syncthreads();
  int bad = 0;
  for (int64_t base = 0; base < B; base += 1024) {
    const int64_t b = base + t;
    int64_t n = 0, m = 0;
    if (b < B) {
      const int64_t id = mol_ids[b];
      if (id < 0 || id >= G) {
        bad |= 1;
      } else {
        n = atom_ptr[id + 1] - atom_ptr[id];
        m = bond_ptr[id + 1] - bond_ptr[id];
        if ((n > kAugMaxAtoms || m > kAugMaxBonds) && (n > big_atoms || m > big_bonds))
          bad |= 16;
      }
    }
    sa[t] = n;
    se[t] = m;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t va = t >= off ? sa[t - off] : 0;
      const int64_t ve = t >= off ? se[t - off] : 0;
      __syncthreads();
      sa[t] += va;
      se[t] += ve;
      __syncthreads();
    }
    if (b < B) {
      ptr_out[b] = carry_a + sa[t] - n;
      bond_off[b] = carry_e + se[t] - m;
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
    bond_off[B] = carry_e;
    if (carry_a != num_nodes) bad |= 2;
  }
  if (bad) atomicOr(status, bad);
}

// One molecule's plan, run by a single lane over the tables L: drop[atom] =
// masked to [118, 0], keep[bond] = the bond survives, cnt[b] = surviving
// bonds.  mode 0: dataset_subgraph (25 %), 1: dataset_mix.
template <typename I>
__device__ void aug_plan_one(const AugTabs<I>& L, const int64_t* __restrict__ sei,
                             int64_t store_edges, int64_t id, int64_t n, int64_t m0, int64_t M,
                             uint64_t seed, int view, int mode, int64_t aoff, int64_t boff, int64_t b,
                             uint8_t* __restrict__ drop, uint8_t* __restrict__ keep,
                             int64_t* __restrict__ cnt, int32_t* __restrict__ status) {
  int bad = 0;
  // bond endpoints (molecule-local, clamped), nx node order, adjacency in bond order
  auto ends = [&](int64_t m, int& s, int& e) {
    int64_t u = sei[2 * (m0 + m)], v = sei[store_edges + 2 * (m0 + m)];
    if (u < 0 || u >= n || v < 0 || v >= n) {
      bad |= 4;
      u = u < 0 ? 0 : (u >= n ? n - 1 : u);
      v = v < 0 ? 0 : (v >= n ? n - 1 : v);
    }
    s = (int)u;
    e = (int)v;
  };
  for (int i = 0; i < n; ++i) {
    L.first[i] = -1;
    L.removed[i] = 0;
    L.in_temp[i] = 0;
    L.adj_off[i] = 0;
  }
  L.adj_off[n] = 0;
  int nodes = 0;
  for (int64_t m = 0; m < M; ++m) {
    int s, e;
    ends(m, s, e);
    if (L.first[s] < 0) L.first[s] = (I)nodes++;
    if (L.first[e] < 0) L.first[e] = (I)nodes++;
    ++L.adj_off[s + 1];
    if (e != s) ++L.adj_off[e + 1];
  }
  for (int i = 0; i < n; ++i) {
    L.adj_off[i + 1] += L.adj_off[i];
    L.fill_cursor[i] = L.adj_off[i];
  }
  // neighbours in bond order; a repeated bond adds no second entry (nx.Graph)
  for (int64_t m = 0; m < M; ++m) {
    int s, e;
    ends(m, s, e);
    bool dup = false;
    for (int q = L.adj_off[s]; q < L.fill_cursor[s]; ++q) dup |= L.adj[q] == e;
    if (dup) continue;
    L.adj[L.fill_cursor[s]++] = (I)e;
    if (e != s) L.adj[L.fill_cursor[e]++] = (I)s;
  }
  // Graph.copy() reorders every neighbour list: the neighbours earlier in node
  // order first (in node order), then the later ones in bond order
  for (int w = 0; w < n; ++w) {
    const int a = L.adj_off[w], d = L.fill_cursor[w] - a;
    int k = 0;
    for (int q = 0; q < d; ++q)  // earlier neighbours, insertion-sorted by node order
      if (L.first[L.adj[a + q]] < L.first[w]) {
        int p = k++;
        while (p > 0 && L.first[L.nbr[p - 1]] > L.first[L.adj[a + q]]) {
          L.nbr[p] = L.nbr[p - 1];
          --p;
        }
        L.nbr[p] = L.adj[a + q];
      }
    for (int q = 0; q < d; ++q)
      if (L.first[L.adj[a + q]] > L.first[w]) L.nbr[k++] = L.adj[a + q];
    for (int q = 0; q < k; ++q) L.adj[a + q] = L.nbr[q];
    L.fill_cursor[w] = (I)(a + k);  // a self-loop drops out of the walk
  }
  // centres: smallest / second smallest key of the molecule's centre stream
  int centre = 0;
  if (n >= 2) {
    const uint64_t cs = subset_stream(seed, 2, 2, id);
    int c0 = -1, c1 = -1;
    uint64_t k0 = 0, k1 = 0;
    for (int i = 0; i < n; ++i) {
      const uint64_t k = item_key(cs, i);
      if (c0 < 0 || k < k0) {
        c1 = c0;
        k1 = k0;
        c0 = i;
        k0 = k;
      } else if (c1 < 0 || k < k1) {
        c1 = i;
        k1 = k;
      }
    }
    centre = view == 0 ? c0 : c1;
  }
  double pct = 0.25;
  if (mode == 1) {
    const uint64_t u = splitmix64(subset_stream(seed, view, 3, id));
    pct = 0.2 * ((double)(u >> 11) * 0x1.0p-53);
  }
  const int num = (int)floor((double)nodes * pct);
  int nrem = 0, nt = 1;
  L.temp[0] = (I)centre;
  if (num > 0 && L.first[centre] < 0) bad |= 32;  // the reference raises (centre not in G)
  while (nrem < num) {
    if (nt < 1) {  // dataset_mix.py:55-56; dataset_subgraph.py would not terminate
      bad |= 8;
      break;
    }
    for (int q = 0; q < nt; ++q) L.in_temp[L.temp[q]] = 1;
    int nn = 0;
    for (int q = 0; q < nt; ++q) {
      const int u = L.temp[q];
      for (int a = L.adj_off[u]; a < L.fill_cursor[u]; ++a) {
        const int v = L.adj[a];
        if (!L.removed[v] && !L.in_temp[v]) L.nbr[nn++] = (I)v;
      }
    }
    for (int q = 0; q < nt; ++q) {
      if (nrem < num) {
        L.removed[L.temp[q]] = 1;
        ++nrem;
      } else {
        break;
      }
    }
    for (int q = 0; q < nt; ++q) L.in_temp[L.temp[q]] = 0;
    nt = pyset_order<I>(L.nbr, nn, L.table, L.temp, L.temp);  // temp is free here: scratch, then out
  }
  // bonds surviving the removal
  int64_t kept = 0;
  for (int64_t m = 0; m < M; ++m) {
    int s, e;
    ends(m, s, e);
    bool k = !L.removed[s] && !L.removed[e];
    if (mode == 0) k = k && L.first[s] <= L.first[e];  // (start, end) in G_i.edges
    keep[boff + m] = k ? 1 : 0;
    kept += k ? 1 : 0;
  }
  for (int i = 0; i < n; ++i) drop[aoff + i] = L.removed[i] ? 1 : 0;
  if (mode == 1) {
    // extra atom masks among the remaining atoms, extra bond masks among the
    // surviving bonds (dataset_mix.py:174-181)
    const int64_t ka = n / 4 - nrem > 0 ? n / 4 - nrem : 0;
    const int64_t kb0 = kept - (3 * M + 3) / 4;
    const int64_t kb = kb0 > 0 ? kb0 : 0;
    const uint64_t as = subset_stream(seed, view, 4, id), bs = subset_stream(seed, view, 5, id);
    const int64_t nremain = n - nrem;
    int64_t pos = 0;
    for (int i = 0; i < n; ++i) {
      if (L.removed[i]) continue;
      if (chosen(as, nremain, ka, pos)) drop[aoff + i] = 1;
      ++pos;
    }
    pos = 0;
    int64_t kept2 = 0;
    for (int64_t m = 0; m < M; ++m) {
      if (!keep[boff + m]) continue;
      if (chosen(bs, kept, kb, pos)) keep[boff + m] = 0;
      else ++kept2;
      ++pos;
    }
    kept = kept2;
  }
  cnt[b] = kept;
  if (bad) atomicOr(status, bad);
}

// a molecule the plan leaves unchanged (flagged: beyond every cap)
__device__ void aug_passthrough(int lane, int64_t n, int64_t M, int64_t aoff, int64_t boff,
                                int64_t b, uint8_t* __restrict__ drop, uint8_t* __restrict__ keep,
                                int64_t* __restrict__ cnt) {
  for (int64_t i = lane; i < n; i += 64) drop[aoff + i] = 0;
  for (int64_t m = lane; m < M; m += 64) keep[boff + m] = 1;
  if (lane == 0) cnt[b] = M;
}

// pass 2: one wave per molecule (lane 0 runs the reference loop in LDS).
// Molecules beyond the LDS caps are left to k_aug_plan_big when `big` is set,
// else they pass unchanged (flagged by k_aug_offsets).
__global__ __launch_bounds__(64) void k_aug_plan(
    const int64_t* __restrict__ atom_ptr, const int64_t* __restrict__ sei,
    const int64_t* __restrict__ bond_ptr, int64_t store_edges, const int64_t* __restrict__ mol_ids,
    int64_t B, int64_t G, uint64_t seed, int view, int mode, const int64_t* __restrict__ ptr,
    const int64_t* __restrict__ bond_off, uint8_t* __restrict__ drop, uint8_t* __restrict__ keep,
    int64_t* __restrict__ cnt, int32_t* __restrict__ status, int big) {
  __shared__ AugLds S;
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t id = mol_ids[b];
  if (id < 0 || id >= G) return;  // flagged by k_aug_offsets
  const int64_t a0 = atom_ptr[id], n = atom_ptr[id + 1] - a0;
  const int64_t m0 = bond_ptr[id], M = bond_ptr[id + 1] - m0;
  const int64_t aoff = ptr[b], boff = bond_off[b];
  if (n > kAugMaxAtoms || M > kAugMaxBonds) {
    if (!big) aug_passthrough(lane, n, M, aoff, boff, b, drop, keep, cnt);
    return;
  }
  if (lane != 0) return;
  const AugTabs<int16_t> L{S.adj_off, S.adj, S.first, S.removed, S.in_temp,
                           S.temp, S.nbr, S.table, S.fill_cursor};
  aug_plan_one<int16_t>(L, sei, store_edges, id, n, m0, M, seed, view, mode, aoff, boff, b, drop,
                        keep, cnt, status);
}

// pass 2, molecules beyond the LDS caps: the same plan over int32 tables in a
// global workspace slot (slots handed out by an atomic counter; a molecule's
// result does not depend on its slot).  Molecules beyond big_atoms /
// big_bonds or past big_slots pass unchanged (status bit 4 from k_aug_offsets,
// or set here).
__global__ __launch_bounds__(64) void k_aug_plan_big(
    const int64_t* __restrict__ atom_ptr, const int64_t* __restrict__ sei,
    const int64_t* __restrict__ bond_ptr, int64_t store_edges, const int64_t* __restrict__ mol_ids,
    int64_t B, int64_t G, uint64_t seed, int view, int mode, const int64_t* __restrict__ ptr,
    const int64_t* __restrict__ bond_off, uint8_t* __restrict__ drop, uint8_t* __restrict__ keep,
    int64_t* __restrict__ cnt, int32_t* __restrict__ status, int64_t big_atoms, int64_t big_bonds,
    int64_t big_slots, int32_t* __restrict__ counter, int32_t* __restrict__ slots) {
  const int64_t b = blockIdx.x;
  const int lane = threadIdx.x;
  const int64_t id = mol_ids[b];
  if (id < 0 || id >= G) return;
  const int64_t a0 = atom_ptr[id], n = atom_ptr[id + 1] - a0;
  const int64_t m0 = bond_ptr[id], M = bond_ptr[id + 1] - m0;
  if (n <= kAugMaxAtoms && M <= kAugMaxBonds) return;  // k_aug_plan's
  const int64_t aoff = ptr[b], boff = bond_off[b];
  if (n > big_atoms || M > big_bonds) {
    aug_passthrough(lane, n, M, aoff, boff, b, drop, keep, cnt);
    return;
  }
  if (lane != 0) return;
  const int slot = atomicAdd(counter, 1);
  if (slot >= big_slots) {
    for (int64_t i = 0; i < n; ++i) drop[aoff + i] = 0;
    for (int64_t m = 0; m < M; ++m) keep[boff + m] = 1;
    cnt[b] = M;
    atomicOr(status, 16);
    return;
  }
  int32_t* w = slots + (int64_t)slot * aug_big_slot_elems(big_atoms, big_bonds);
  AugTabs<int32_t> L;
  L.adj_off = w;
  w += big_atoms + 1;
  L.adj = w;
  w += 2 * big_bonds;
  L.first = w;
  w += big_atoms;
  L.removed = w;
  w += big_atoms;
  L.in_temp = w;
  w += big_atoms;
  L.temp = w;
  w += big_atoms;
  L.fill_cursor = w;
  w += big_atoms;
  L.nbr = w;
  w += 2 * big_bonds;
  L.table = w;
  aug_plan_one<int32_t>(L, sei, store_edges, id, n, m0, M, seed, view, mode, aoff, boff, b, drop,
                        keep, cnt, status);
}

// exclusive scan of the surviving-bond counts into edge offsets (2 per bond)
__global__ void k_aug_edge_offsets(const int64_t* __restrict__ cnt, int64_t B,
                                   int64_t* __restrict__ edge_off) {
  __shared__ int64_t se[1024];
  __shared__ int64_t carry;
  const int t = threadIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int64_t base = 0; base < B; base += 1024) {
    const int64_t b = base + t;
    const int64_t e = b < B ? 2 * cnt[b] : 0;
    se[t] = e;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int64_t v = t >= off ? se[t - off] : 0;
      __syncthreads();
      se[t] += v;
      __syncthreads();
    }
    if (b < B) edge_off[b] = carry + se[t] - e;
    __syncthreads();
    if (t == 1023) carry += se[t];
    __syncthreads();
  }
  if (t == 0) edge_off[B] = carry;
}

// pass 3: the collated Batch fields of the planned view
__global__ __launch_bounds__(64 * kMolsPerBlock) void k_aug_write(
    const int64_t* __restrict__ sx, const int64_t* __restrict__ atom_ptr,
    const int64_t* __restrict__ sei, const int64_t* __restrict__ sea,
    const int64_t* __restrict__ bond_ptr, int64_t store_edges, const int64_t* __restrict__ mol_ids,
    int64_t B, int64_t G, const int64_t* __restrict__ ptr, const int64_t* __restrict__ bond_off,
    const int64_t* __restrict__ edge_off, const uint8_t* __restrict__ drop,
    const uint8_t* __restrict__ keep, int64_t* __restrict__ x_out, int64_t* __restrict__ ei_out,
    int64_t* __restrict__ ea_out, int64_t* __restrict__ batch_out, int64_t num_nodes,
    int64_t num_edges) {
  const int lane = threadIdx.x & 63;
  const int64_t b = (int64_t)blockIdx.x * kMolsPerBlock + (threadIdx.x >> 6);
  if (b >= B) return;  // wave-uniform
  const int64_t id = mol_ids[b];
  if (id < 0 || id >= G) return;
  const int64_t a0 = atom_ptr[id], n = atom_ptr[id + 1] - a0;
  const int64_t m0 = bond_ptr[id], M = bond_ptr[id + 1] - m0;
  const int64_t aoff = ptr[b], boff = bond_off[b], eoff = edge_off[b];
  if (aoff + n > num_nodes || edge_off[b + 1] > num_edges) return;
  for (int64_t i = lane; i < n; i += 64) {
    const bool masked = drop[aoff + i] != 0;
    const int64_t o = aoff + i;
    const int64_t* src = sx + 2 * (a0 + i);
    x_out[2 * o] = masked ? 118 : src[0];
    x_out[2 * o + 1] = masked ? 0 : src[1];
    batch_out[o] = b;
  }
  int64_t kept_before = 0;
  for (int64_t base = 0; base < M; base += 64) {
    const int64_t m = base + lane;
    const bool k = m < M && keep[boff + m];
    const uint64_t bal = __ballot(k);
    if (k) {
      const int64_t p = kept_before + __popcll(bal & ((1ull << lane) - 1ull));
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const int64_t se = 2 * (m0 + m) + d;
        const int64_t oe = eoff + 2 * p + d;
        int64_t s = sei[se], t = sei[store_edges + se];
        s = s < 0 ? 0 : (s >= n ? n - 1 : s);
        t = t < 0 ? 0 : (t >= n ? n - 1 : t);
        ei_out[oe] = s + aoff;
        ei_out[num_edges + oe] = t + aoff;
        ea_out[2 * oe] = sea[2 * se];
        ea_out[2 * oe + 1] = sea[2 * se + 1];
      }
    }
    kept_before += __popcll(bal);
  }
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

// ---- subgraph / mix views ----------------------------------------------------
namespace {
struct AugWs {
  int64_t *bond_off, *cnt, *edge_off;
  uint8_t *drop, *keep;
};
AugWs aug_ws(void* w, size_t bytes, int64_t B, int64_t num_nodes, int64_t num_bonds) {
  molclr::Workspace ws(w, bytes);
  AugWs a;
  a.bond_off = ws.take<int64_t>(B + 1);
  a.cnt = ws.take<int64_t>(B > 0 ? B : 1);
  a.edge_off = ws.take<int64_t>(B + 1);
  a.drop = ws.take<uint8_t>(num_nodes > 0 ? num_nodes : 1);
  a.keep = ws.take<uint8_t>(num_bonds > 0 ? num_bonds : 1);
  return a;
}
}  // namespace

MOLCLR_API size_t molclr_aug_views_workspace_bytes(int64_t batch_size, int64_t num_nodes,
                                                   int64_t num_bonds) {
  return (size_t)(3 * batch_size + 3) * sizeof(int64_t) + (size_t)num_nodes + (size_t)num_bonds +
         6 * 256;
}

namespace {
int aug_plan_impl(const int64_t* store_atom_ptr, const int64_t* store_edge_index,
                  const int64_t* store_bond_ptr, int64_t store_mols, int64_t store_edges,
                  const int64_t* mol_ids, int64_t batch_size, uint64_t seed, int view, int mode,
                  int64_t num_nodes, int64_t num_bonds, int64_t* ptr_out, int64_t* num_edges_out,
                  int32_t* status, void* workspace, size_t workspace_bytes, int64_t big_slots,
                  int64_t big_atoms, int64_t big_bonds, void* big_ws, size_t big_ws_bytes,
                  hipStream_t s) {
  MOLCLR_REQUIRE(batch_size >= 0 && store_mols >= 0 && store_edges >= 0 && num_nodes >= 0 &&
                     num_bonds >= 0,
                 "aug_views_plan: negative size");
  MOLCLR_REQUIRE(view == 0 || view == 1, "aug_views_plan: view must be 0 or 1");
  MOLCLR_REQUIRE(mode == MOLCLR_AUG_SUBGRAPH || mode == MOLCLR_AUG_MIX,
                 "aug_views_plan: mode %d (0 subgraph, 1 mix)", mode);
  MOLCLR_REQUIRE(ptr_out && num_edges_out && status, "aug_views_plan: null pointer");
  MOLCLR_REQUIRE(batch_size == 0 || (store_atom_ptr && store_bond_ptr && mol_ids &&
                                     (store_edges == 0 || store_edge_index)),
                 "aug_views_plan: null pointer");
  MOLCLR_REQUIRE(batch_size <= (1ll << 31), "aug_views_plan: batch too large");
  MOLCLR_REQUIRE_WS(workspace_bytes,
                    molclr_aug_views_workspace_bytes(batch_size, num_nodes, num_bonds));
  MOLCLR_REQUIRE(big_slots >= 0 && big_atoms >= 0 && big_bonds >= 0 && big_atoms < (1ll << 30) &&
                     big_bonds < (1ll << 29),
                 "aug_views_plan_big: bad large-molecule caps");
  const bool big = big_slots > 0;
  if (big) {
    MOLCLR_REQUIRE(big_ws != nullptr, "aug_views_plan_big: null workspace");
    MOLCLR_REQUIRE_WS(big_ws_bytes,
                      molclr_aug_views_big_workspace_bytes(big_slots, big_atoms, big_bonds));
  }
  int32_t* counter = big ? static_cast<int32_t*>(big_ws) : nullptr;
  int32_t* slots = big ? static_cast<int32_t*>(big_ws) + 64 : nullptr;  // counter on its own line
  const AugWs a = aug_ws(workspace, workspace_bytes, batch_size, num_nodes, num_bonds);
  hipLaunchKernelGGL(k_aug_offsets, dim3(1), dim3(1024), 0, s, store_atom_ptr, store_bond_ptr,
                     mol_ids, batch_size, store_mols, ptr_out, a.bond_off, num_nodes, status,
                     big ? big_atoms : (int64_t)0, big ? big_bonds : (int64_t)0, counter);
  if (batch_size > 0) {
    hipLaunchKernelGGL(k_aug_plan, dim3((unsigned)batch_size), dim3(64), 0, s, store_atom_ptr,
                       store_edge_index, store_bond_ptr, store_edges, mol_ids, batch_size,
                       store_mols, seed, view, mode, static_cast<const int64_t*>(ptr_out),
                       static_cast<const int64_t*>(a.bond_off), a.drop, a.keep, a.cnt, status,
                       big ? 1 : 0);
    if (big)
      hipLaunchKernelGGL(k_aug_plan_big, dim3((unsigned)batch_size), dim3(64), 0, s,
                         store_atom_ptr, store_edge_index, store_bond_ptr, store_edges, mol_ids,
                         batch_size, store_mols, seed, view, mode,
                         static_cast<const int64_t*>(ptr_out),
                         static_cast<const int64_t*>(a.bond_off), a.drop, a.keep, a.cnt, status,
                         big_atoms, big_bonds, big_slots, counter, slots);
  }
  hipLaunchKernelGGL(k_aug_edge_offsets, dim3(1), dim3(1024), 0, s,
                     static_cast<const int64_t*>(a.cnt), batch_size, a.edge_off);
  if (molclr::copy_async(num_edges_out, a.edge_off + batch_size, sizeof(int64_t), s) != hipSuccess) {
    molclr::set_error("aug_views_plan: copy failed");
    return MOLCLR_ERR_ARG;
  }
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
}  // namespace

MOLCLR_API size_t molclr_aug_views_big_workspace_bytes(int64_t big_slots, int64_t big_atoms,
                                                       int64_t big_bonds) {
  if (big_slots <= 0) return 0;
  return (size_t)(64 + big_slots * aug_big_slot_elems(big_atoms, big_bonds)) * sizeof(int32_t) +
         256;
}

MOLCLR_API int molclr_aug_views_plan(const int64_t* store_atom_ptr, const int64_t* store_edge_index,
                                     const int64_t* store_bond_ptr, int64_t store_mols,
                                     int64_t store_edges, const int64_t* mol_ids,
                                     int64_t batch_size, uint64_t seed, int view, int mode,
                                     int64_t num_nodes, int64_t num_bonds, int64_t* ptr_out,
                                     int64_t* num_edges_out, int32_t* status, void* workspace,
                                     size_t workspace_bytes, molclr_stream_t stream) {
  return aug_plan_impl(store_atom_ptr, store_edge_index, store_bond_ptr, store_mols, store_edges,
                       mol_ids, batch_size, seed, view, mode, num_nodes, num_bonds, ptr_out,
                       num_edges_out, status, workspace, workspace_bytes, 0, 0, 0, nullptr, 0,
                       molclr::as_stream(stream));
}

MOLCLR_API int molclr_aug_views_plan_big(
    const int64_t* store_atom_ptr, const int64_t* store_edge_index, const int64_t* store_bond_ptr,
    int64_t store_mols, int64_t store_edges, const int64_t* mol_ids, int64_t batch_size,
    uint64_t seed, int view, int mode, int64_t num_nodes, int64_t num_bonds, int64_t* ptr_out,
    int64_t* num_edges_out, int32_t* status, void* workspace, size_t workspace_bytes,
    int64_t big_slots, int64_t big_atoms, int64_t big_bonds, void* big_workspace,
    size_t big_workspace_bytes, molclr_stream_t stream) {
  return aug_plan_impl(store_atom_ptr, store_edge_index, store_bond_ptr, store_mols, store_edges,
                       mol_ids, batch_size, seed, view, mode, num_nodes, num_bonds, ptr_out,
                       num_edges_out, status, workspace, workspace_bytes, big_slots, big_atoms,
                       big_bonds, big_workspace, big_workspace_bytes, molclr::as_stream(stream));
}

MOLCLR_API int molclr_aug_views_write(const int64_t* store_x, const int64_t* store_atom_ptr,
                                      const int64_t* store_edge_index,
                                      const int64_t* store_edge_attr, const int64_t* store_bond_ptr,
                                      int64_t store_mols, int64_t store_edges,
                                      const int64_t* mol_ids, int64_t batch_size,
                                      const int64_t* ptr, int64_t num_nodes, int64_t num_bonds,
                                      int64_t num_edges, int64_t* x_out, int64_t* edge_index_out,
                                      int64_t* edge_attr_out, int64_t* batch_out,
                                      const void* workspace, size_t workspace_bytes,
                                      molclr_stream_t stream) {
  MOLCLR_REQUIRE(batch_size >= 0 && num_nodes >= 0 && num_edges >= 0, "aug_views_write: bad size");
  MOLCLR_REQUIRE(num_nodes == 0 || (store_x && x_out && batch_out), "aug_views_write: null pointer");
  MOLCLR_REQUIRE(num_edges == 0 || (store_edge_index && store_edge_attr && edge_index_out &&
                                    edge_attr_out),
                 "aug_views_write: null pointer");
  MOLCLR_REQUIRE(batch_size == 0 || (store_atom_ptr && store_bond_ptr && mol_ids && ptr),
                 "aug_views_write: null pointer");
  MOLCLR_REQUIRE_WS(workspace_bytes,
                    molclr_aug_views_workspace_bytes(batch_size, num_nodes, num_bonds));
  if (batch_size == 0) return MOLCLR_OK;
  const AugWs a = aug_ws(const_cast<void*>(workspace), workspace_bytes, batch_size, num_nodes,
                         num_bonds);
  hipLaunchKernelGGL(k_aug_write, dim3((unsigned)molclr::ceil_div(batch_size, kMolsPerBlock)),
                     dim3(64 * kMolsPerBlock), 0, molclr::as_stream(stream), store_x,
                     store_atom_ptr, store_edge_index, store_edge_attr, store_bond_ptr, store_edges,
                     mol_ids, batch_size, store_mols, ptr, static_cast<const int64_t*>(a.bond_off),
                     static_cast<const int64_t*>(a.edge_off), static_cast<const uint8_t*>(a.drop),
                     static_cast<const uint8_t*>(a.keep), x_out, edge_index_out, edge_attr_out,
                     batch_out, num_nodes, num_edges);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}
