// GIN encoder executor: GINet's node-embedding stack (models/ginet_molclr.py:98-111)
// forward and backward as single calls over the library's own entry points.
//
// The per-op autograd path (molclr_amd/ops.py) pays ~30 us of Python per
// operation — ~4 ms of host time per training step, against ~6 ms of GPU
// time.  This file issues the same entry points, with the same arguments and
// in the same order, from C++: the kernels and their results are identical,
// only the host cost goes.
//
// Arena (saved for the backward), per layer l: agg_l [N,D], a1_l [N,2D],
// z_l [N,D], h_l [N,D] (BatchNorm output, the next layer's input; the last
// layer writes h_out instead), mean_l / invstd_l [D]; then h0 [N,D] (atom
// embedding) and the combined edge tables Ec [L,15,D].
// Workspace: backward scratch dh, dz, dagg [N,D] + dz1 [N,2D], then the
// largest workspace any called entry point asks for.
#include "common.h"

namespace {

// byte offsets; node-feature buffers in the encoder's storage type (fp32 or
// bf16), statistics and edge tables fp32; every buffer 256-byte aligned
struct ArenaLayout {
  size_t agg[MOLCLR_MAX_LAYERS], a1[MOLCLR_MAX_LAYERS], z[MOLCLR_MAX_LAYERS],
      h[MOLCLR_MAX_LAYERS], mean[MOLCLR_MAX_LAYERS], invstd[MOLCLR_MAX_LAYERS];
  size_t bits[MOLCLR_MAX_LAYERS];  // h3: ReLU mask of a1_l as bits [ceil(2D / 32)][N]
  size_t h0, ec, smax, bmax, total;
  ArenaLayout(int L, int64_t N, int64_t D, size_t es) {
    size_t used = 0;
    auto off = [&](size_t bytes) {
      const size_t o = used;
      used += (bytes + 255) / 256 * 256;
      return o;
    };
    for (int l = 0; l < L; ++l) {
      agg[l] = off(N * D * es);
      a1[l] = off(N * 2 * D * es);
      z[l] = off(N * D * es);
      h[l] = off(N * D * es);
      mean[l] = off(MOLCLR_MAX_SEGMENTS * D * sizeof(float));  // [segment][D]
      invstd[l] = off(MOLCLR_MAX_SEGMENTS * D * sizeof(float));
      bits[l] = off((size_t)N * ((2 * D + 31) / 32) * sizeof(uint32_t));
    }
    h0 = off(N * D * es);
    ec = off((size_t)L * MOLCLR_NUM_ECOMB * D * sizeof(float));
    smax = off((size_t)MOLCLR_MAX_LAYERS * 2 * kMaxSlotFloats * sizeof(float));  // h3: max |agg_l|, |a1_l|
    // h3: the backward's max |dz_l|, |dz1_l| (zeroed by the forward with smax)
    bmax = off((size_t)MOLCLR_MAX_LAYERS * 2 * kMaxSlotFloats * sizeof(float));
    total = used;
  }
};

size_t elem_bytes(int dtype) { return dtype == MOLCLR_DTYPE_BF16 ? 2 : 4; }

size_t kernels_ws(int64_t N, int64_t D) {
  size_t m = 0;
  auto mx = [&](size_t v) { m = v > m ? v : m; };
  mx(molclr_gemm_f32_workspace_bytes(2 * D, D, N));  // dW0 = dz1^T agg
  mx(molclr_gemm_f32_workspace_bytes(D, 2 * D, N));  // dW2 = dz^T a1
  mx(molclr_gemm_f32_workspace_bytes(N, 2 * D, D));
  mx(molclr_gemm_f32_workspace_bytes(N, D, 2 * D));
  mx(molclr_colsum_f32_workspace_bytes(N, 2 * D));
  mx(molclr_linear_wgrad_workspace_bytes(N, D, 2 * D));
  mx(molclr_linear_wgrad_workspace_bytes(N, 2 * D, D));
  if (N >= 1024 && D % 4 == 0) mx(molclr_linear_wgrad_h3_pair_workspace_bytes(N, D, 2 * D, 2 * D, D));
  mx(molclr_linear_wgrad_bf16_workspace_bytes(N, D, 2 * D));
  mx(molclr_linear_wgrad_bf16_workspace_bytes(N, 2 * D, D));
  mx(molclr_batchnorm_ws_bound(N, D));
  mx(molclr_gine_aggregate_bwd_workspace_bytes(N, D));
  mx(molclr_atom_embed_bwd_workspace_bytes(N, D, MOLCLR_NUM_ATOM_TYPE, MOLCLR_NUM_CHIRALITY));
  return m;
}

// backward scratch dh, dz, dagg [N,D] + dz1 [N,2D], in the storage type
size_t scratch_bytes(int64_t N, int64_t D, size_t es) { return ((size_t)N * D * 3 + (size_t)N * 2 * D) * es; }

int check_encoder(const molclr_gin_encoder* e, const molclr_device_graph* g) {
  MOLCLR_REQUIRE(e && g, "gin_encoder: null encoder / graph");
  MOLCLR_REQUIRE(e->num_layer >= 1 && e->num_layer <= MOLCLR_MAX_LAYERS,
                 "gin_encoder: num_layer %d", e->num_layer);
  MOLCLR_REQUIRE(e->dim > 0 && e->dim % 4 == 0, "gin_encoder: dim %lld", (long long)e->dim);
  MOLCLR_REQUIRE(e->dtype == MOLCLR_DTYPE_F32 || (e->dtype == MOLCLR_DTYPE_BF16 && e->dim % 8 == 0),
                 "gin_encoder: dtype %d (bf16 needs dim %% 8 == 0)", e->dtype);
  MOLCLR_REQUIRE(e->n_atom == MOLCLR_NUM_ATOM_TYPE && e->n_chiral == MOLCLR_NUM_CHIRALITY,
                 "gin_encoder: embedding tables must be [%d,D] and [%d,D]",
                 MOLCLR_NUM_ATOM_TYPE, MOLCLR_NUM_CHIRALITY);
  for (int l = 0; l < e->num_layer; ++l)
    MOLCLR_REQUIRE(e->mlp0_planes[l] && e->mlp0_planes_t[l] && e->mlp2_planes[l] &&
                       e->mlp2_planes_t[l] && e->bn_weight[l] && e->bn_bias[l],
                   "gin_encoder: layer %d: missing planes or BatchNorm affine", l);
  return MOLCLR_OK;
}

// BatchNorm segments of a graph (the views of a paired forward), checked
// (device-sized graph: the rows of every segment are read on the device,
// g->num_nodes rows in all, the rest padding)
struct SegRows {
  int n;
  const int64_t* rows;
  const int64_t* dev;
  int64_t cap;
};
int graph_segments(const molclr_device_graph* g, const int64_t* N, SegRows& out) {
  if (g->segment_nodes_dev) {
    MOLCLR_REQUIRE(g->num_segments >= 1 && g->num_segments <= MOLCLR_MAX_SEGMENTS,
                   "encoder: %d graph segments", g->num_segments);
    out = {g->num_segments, nullptr, g->segment_nodes_dev, *N};
    return MOLCLR_OK;
  }
  if (g->num_segments <= 1) {
    out = {1, N, nullptr, *N};
    return MOLCLR_OK;
  }
  MOLCLR_REQUIRE(g->num_segments <= MOLCLR_MAX_SEGMENTS, "encoder: %d graph segments",
                 g->num_segments);
  int64_t tot = 0;
  for (int s = 0; s < g->num_segments; ++s) tot += g->segment_nodes[s];
  MOLCLR_REQUIRE(tot == *N, "encoder: segment nodes sum to %lld, graph has %lld", (long long)tot,
                 (long long)*N);
  out = {g->num_segments, g->segment_nodes, nullptr, *N};
  return MOLCLR_OK;
}

// the segmented BatchNorm of a graph, host- or device-sized
int seg_bn_fwd(const SegRows& sg, const void* z, const float* gamma, const float* beta,
               float* rmean, float* rvar, int64_t* nbt, void* y, float* mean, float* invstd,
               int64_t D, int dtype, double momentum, double eps, int training, int relu,
               void* ws, size_t ws_bytes, molclr_stream_t stream) {
  if (sg.dev)
    return molclr_batchnorm_seg_fwd_dev(z, gamma, beta, rmean, rvar, nbt, y, mean, invstd, sg.n,
                                        sg.dev, sg.cap, D, dtype, momentum, eps, training, relu,
                                        ws, ws_bytes, stream);
  return molclr_batchnorm_seg_fwd(z, gamma, beta, rmean, rvar, nbt, y, mean, invstd, sg.n,
                                  sg.rows, D, dtype, momentum, eps, training, relu, ws, ws_bytes,
                                  stream);
}
// rowmax != NULL (fp32): also dz's row maxima and max slot (the h3 scales)
int seg_bn_bwd(const SegRows& sg, const void* dy, const void* z, const float* gamma,
               const float* beta, const float* mean, const float* invstd, void* dz, float* dgamma,
               float* dbeta, int64_t D, int dtype, int relu, int accumulate, float* rowmax,
               float* slot, void* ws, size_t ws_bytes, molclr_stream_t stream) {
  if (sg.dev)
    return molclr_batchnorm_seg_bwd_dev(dy, z, gamma, beta, mean, invstd, dz, dgamma, dbeta, sg.n,
                                        sg.dev, sg.cap, D, dtype, relu, accumulate, rowmax, slot,
                                        ws, ws_bytes, stream);
  if (rowmax)
    return molclr_batchnorm_seg_bwd_max((const float*)dy, (const float*)z, gamma, beta, mean,
                                        invstd, (float*)dz, dgamma, dbeta, sg.n, sg.rows, D, relu,
                                        accumulate, rowmax, slot, ws, ws_bytes, stream);
  return molclr_batchnorm_seg_bwd(dy, z, gamma, beta, mean, invstd, dz, dgamma, dbeta, sg.n,
                                  sg.rows, D, dtype, relu, accumulate, ws, ws_bytes, stream);
}

#define MOLCLR_TRY(expr)      \
  do {                        \
    int rc_ = (expr);         \
    if (rc_) return rc_;      \
  } while (0)

// the grads struct's optional "gradients final" events (layer_done / embed_done)
int record_done(void* ev, molclr_stream_t stream) {
  if (ev && hipEventRecord(static_cast<hipEvent_t>(ev), molclr::as_stream(stream)) != hipSuccess) {
    molclr::set_error("encoder_bwd: hipEventRecord failed");
    return MOLCLR_ERR_ARG;
  }
  return MOLCLR_OK;
}

}  // namespace

MOLCLR_API size_t molclr_gin_encoder_arena_bytes(int L, int64_t N, int64_t D, int dtype) {
  if (L < 1 || L > MOLCLR_MAX_LAYERS) return 0;
  return ArenaLayout(L, N, D, elem_bytes(dtype)).total;
}

// workspace: backward scratch | h3 max slots of dz_l / dz1_l | h3 row maxima
// of agg / dz [N] and of a1 / dz1 [parts][N] | the entry points' workspace
constexpr size_t kSlotBytes = MOLCLR_MAX_LAYERS * 2 * kMaxSlotFloats * sizeof(float);
// row maxima of a [N,D] tensor and of a [N,2D] GEMM output
// (molclr_gemm_row_parts(2D) partial arrays)
// the first region: dz's row-max parts, or agg's in the aggregation's layout
// (h3 forward, molclr_rowmax_layout)
size_t rowmax_first_bytes(int64_t N, int64_t D) {
  const size_t dz = (size_t)molclr_bn_row_parts(D) * N * sizeof(float);
  const size_t agg = molclr_rowmax_bytes(N, D);
  return molclr::align_up(dz > agg ? dz : agg, 256);
}
size_t rowmax_bytes(int64_t N, int64_t D) {
  return molclr::align_up(
      rowmax_first_bytes(N, D) + (size_t)molclr_gemm_row_parts(2 * D) * N * sizeof(float), 256);
}

MOLCLR_API size_t molclr_gin_encoder_workspace_bytes(int L, int64_t N, int64_t D, int dtype) {
  (void)L;
  return molclr::align_up(scratch_bytes(N, D, elem_bytes(dtype)), 256) + kSlotBytes +
         rowmax_bytes(N, D) + kernels_ws(N, D) + 256;
}

MOLCLR_API int molclr_gin_encoder_fwd(const molclr_gin_encoder* e, const int64_t* x,
                                      const molclr_device_graph* g, void* h_out, void* arena,
                                      size_t arena_bytes, void* workspace, size_t workspace_bytes,
                                      molclr_stream_t stream) {
  MOLCLR_TRY(check_encoder(e, g));
  const int L = e->num_layer;
  const int64_t N = g->num_nodes, D = e->dim;
  if (N == 0) return MOLCLR_OK;
  SegRows seg;
  MOLCLR_TRY(graph_segments(g, &g->num_nodes, seg));
  MOLCLR_REQUIRE(x && h_out && arena, "gin_encoder_fwd: null pointer");
  const bool bf = e->dtype == MOLCLR_DTYPE_BF16;
  const size_t es = elem_bytes(e->dtype);
  const ArenaLayout lay(L, N, D, es);
  MOLCLR_REQUIRE_WS(arena_bytes, lay.total);
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gin_encoder_workspace_bytes(L, N, D, e->dtype));
  char* A = (char*)arena;
  auto F = [&](size_t off) { return (float*)(A + off); };
  auto H = [&](size_t off) { return (uint16_t*)(A + off); };
  // h3: row maxima of agg and a1 (workspace row-maxima region)
  float* ragg = (float*)((char*)workspace + molclr::align_up(scratch_bytes(N, D, es), 256) +
                         kSlotBytes);
  float* ra1 = (float*)((char*)ragg + rowmax_first_bytes(N, D));  // after agg's row maxima
  void* kws = (char*)ragg + rowmax_bytes(N, D);
  const size_t kws_bytes = kernels_ws(N, D);
  const bool h3 = !bf && e->fp32_gemm != 0;
  const bool h3f = h3 && (e->fp32_gemm & 2);  // h3 forward products (not the default)
  float* fmax = F(lay.smax);  // h3: [l][0] = max |agg_l|, [l][1] = max |a1_l|

  void* h = A + lay.h0;
  if (bf)
    MOLCLR_TRY(molclr_atom_embed_fwd_bf16(x, e->x_embedding1, e->x_embedding2, (uint16_t*)h, N, D,
                                          e->n_atom, e->n_chiral, e->status, stream));
  else
    MOLCLR_TRY(molclr_atom_embed_fwd(x, e->x_embedding1, e->x_embedding2, (float*)h, N, D,
                                     e->n_atom, e->n_chiral, e->status, stream));
  float* Ec = F(lay.ec);
  // h3: the forward's and the backward's max slots (smax, bmax: adjacent)
  // zeroed by the same launch
  const int64_t nz = h3 ? (int64_t)(lay.bmax - lay.smax) / 4 + (int64_t)L * 2 * kMaxSlotFloats : 0;
  MOLCLR_TRY(molclr::edge_tables_combine_zero(L, e->edge_embedding1, e->edge_embedding2, Ec, D,
                                              h3 ? fmax : nullptr, nz, stream));
  for (int l = 0; l < L; ++l) {
    const bool last = l == L - 1;
    void* y = last ? h_out : A + lay.h[l];
    const float* Ecl = Ec + (size_t)l * MOLCLR_NUM_ECOMB * D;
    if (bf) {
      uint16_t *agg = H(lay.agg[l]), *a1 = H(lay.a1[l]), *z = H(lay.z[l]);
      MOLCLR_TRY(molclr_gine_aggregate_fwd_bf16((const uint16_t*)h, g->rowptr, g->col, g->ecode,
                                                g->nbr, Ecl, agg, N, D, stream));
      // GINEConv.update in bf16: one MFMA per product, fp32 accumulation; the
      // first product also writes a1's ReLU mask as bits for the backward
      if (D % 64 == 0)
        MOLCLR_TRY(molclr_gemm_bf16_bits(agg, e->mlp0_planes[l], a1, N, 2 * D, D, D, 2 * D,
                                         MOLCLR_EPI_BIAS_RELU, e->mlp0_bias[l],
                                         (uint32_t*)(A + lay.bits[l]), nullptr, stream));
      else
        MOLCLR_TRY(molclr_gemm_bf16(agg, e->mlp0_planes[l], a1, N, 2 * D, D, D, 2 * D,
                                    MOLCLR_EPI_BIAS_RELU, e->mlp0_bias[l], nullptr, 0, stream));
      MOLCLR_TRY(molclr_gemm_bf16(a1, e->mlp2_planes[l], z, N, D, 2 * D, 2 * D, D,
                                  MOLCLR_EPI_BIAS, e->mlp2_bias[l], nullptr, 0, stream));
      MOLCLR_TRY(seg_bn_fwd(seg, z, e->bn_weight[l], e->bn_bias[l], e->bn_running_mean[l],
                            e->bn_running_var[l], e->bn_num_batches_tracked[l], y, F(lay.mean[l]),
                            F(lay.invstd[l]), D, MOLCLR_DTYPE_BF16, e->momentum, e->eps,
                            e->training, last ? 0 : 1, kws, kws_bytes, stream));
    } else {
      float *agg = F(lay.agg[l]), *a1 = F(lay.a1[l]), *z = F(lay.z[l]);
      float* sl = fmax + 2 * l * kMaxSlotFloats;
      if (h3f)  // agg's row maxima from the aggregation itself, max |agg| from lin1
        MOLCLR_TRY(molclr_gine_aggregate_fwd_rowmax((const float*)h, g->rowptr, g->col, g->ecode,
                                                    g->nbr, Ecl, agg, N, D, ragg, nullptr,
                                                    stream));
      else
        MOLCLR_TRY(molclr_gine_aggregate_fwd((const float*)h, g->rowptr, g->col, g->ecode, g->nbr,
                                             Ecl, agg, N, D, stream));
      if (h3f) {
        // GINEConv.update in h3 (ops._MLP), A scaled row by row; max |agg| (its
        // A reads), max |a1|, a1's row maxima and its ReLU mask as bits from
        // the first GEMM
        const uint16_t* p0 = e->mlp0_planes[l];
        const uint16_t* p2 = e->mlp2_planes[l];
        MOLCLR_TRY(molclr_gemm_f32_h3_bits(agg, ragg, (int)molclr_rowmax_layout(D), p0, a1, N,
                                           2 * D, D, D, 2 * D, MOLCLR_EPI_BIAS_RELU,
                                           e->mlp0_bias[l], nullptr, 0, nullptr,
                                           sl + kMaxSlotFloats, ra1, sl,
                                           (uint32_t*)(A + lay.bits[l]), stream));
        MOLCLR_TRY(molclr_gemm_f32_h3(a1, ra1, (int)molclr_gemm_row_parts(2 * D), p2, z, N, D,
                                      2 * D, 2 * D, D, MOLCLR_EPI_BIAS, e->mlp2_bias[l], nullptr, 0,
                                      nullptr,
                                      nullptr, nullptr, nullptr, stream));
      } else {
        // GINEConv.update: Linear(D,2D) + ReLU, Linear(2D,D)  (ops.linear_fwd);
        // h3 backward: the first product also yields max |agg| and max |a1|
        if (h3)
          MOLCLR_TRY(molclr_gemm_f32_bplanes_max(agg, e->mlp0_planes[l], a1, N, 2 * D, D, D, 2 * D,
                                                 MOLCLR_EPI_BIAS_RELU, e->mlp0_bias[l], nullptr, 0,
                                                 fmax + 2 * l * kMaxSlotFloats,
                                                 fmax + (2 * l + 1) * kMaxSlotFloats, nullptr,
                                                 (uint32_t*)(A + lay.bits[l]), kws, kws_bytes,
                                                 stream));
        else
          MOLCLR_TRY(molclr_gemm_f32_bplanes(agg, e->mlp0_planes[l], a1, N, 2 * D, D, D, 2 * D, 0,
                                             MOLCLR_EPI_BIAS_RELU, e->mlp0_bias[l], nullptr, 0, kws,
                                             kws_bytes, stream));
        MOLCLR_TRY(molclr_gemm_f32_bplanes(a1, e->mlp2_planes[l], z, N, D, 2 * D, 2 * D, D, 0,
                                           MOLCLR_EPI_BIAS, e->mlp2_bias[l], nullptr, 0, kws,
                                           kws_bytes, stream));
      }
      MOLCLR_TRY(seg_bn_fwd(seg, z, e->bn_weight[l], e->bn_bias[l], e->bn_running_mean[l],
                            e->bn_running_var[l], e->bn_num_batches_tracked[l], y, F(lay.mean[l]),
                            F(lay.invstd[l]), D, MOLCLR_DTYPE_F32, e->momentum, e->eps,
                            e->training, last ? 0 : 1, kws, kws_bytes, stream));
    }
    h = y;
  }
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gin_encoder_bwd(const molclr_gin_encoder* e,
                                      const molclr_gin_encoder_grads* gr, const int64_t* x,
                                      const molclr_device_graph* g, const void* dh_out,
                                      const void* arena, size_t arena_bytes, void* workspace,
                                      size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_TRY(check_encoder(e, g));
  MOLCLR_REQUIRE(gr, "gin_encoder_bwd: null grads");
  MOLCLR_REQUIRE(e->training, "gin_encoder_bwd: backward through eval-mode BatchNorm");
  const int L = e->num_layer;
  const int64_t N = g->num_nodes, D = e->dim;
  if (N == 0) return MOLCLR_OK;
  SegRows seg;
  MOLCLR_TRY(graph_segments(g, &g->num_nodes, seg));
  MOLCLR_REQUIRE(x && dh_out && arena, "gin_encoder_bwd: null pointer");
  const bool bf = e->dtype == MOLCLR_DTYPE_BF16;
  const size_t es = elem_bytes(e->dtype);
  const ArenaLayout lay(L, N, D, es);
  MOLCLR_REQUIRE_WS(arena_bytes, lay.total);
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gin_encoder_workspace_bytes(L, N, D, e->dtype));
  const char* A = (const char*)arena;
  auto F = [&](size_t off) { return (const float*)(A + off); };
  char* S = (char*)workspace;
  void* dh = S;                              // gradient w.r.t. the current layer's output
  void* dz = S + (size_t)N * D * es;         // w.r.t. the BatchNorm input z
  void* dagg = S + 2 * (size_t)N * D * es;   // w.r.t. the aggregation output
  void* dz1 = S + 3 * (size_t)N * D * es;    // w.r.t. the first Linear's pre-activation [N,2D]
  // h3: the arena's backward slots, zeroed by the forward (a second backward
  // of the same forward folds the same maxima again: the same values)
  float* bmax = const_cast<float*>(F(lay.bmax));
  float* rdz = (float*)(S + molclr::align_up(scratch_bytes(N, D, es), 256)) +
               kSlotBytes / sizeof(float);  // h3: row maxima of dz, then of dz1
  float* rdz1 = (float*)((char*)rdz + rowmax_first_bytes(N, D));  // after dz's row maxima
  void* kws = (char*)rdz + rowmax_bytes(N, D);
  const size_t kws_bytes = kernels_ws(N, D);
  const int dt = bf ? MOLCLR_DTYPE_BF16 : MOLCLR_DTYPE_F32;
  const bool h3 = !bf && e->fp32_gemm != 0;
  const float* fmax = F(lay.smax);  // the forward's max |agg_l|, max |a1_l|
  // h3: bmax[l][0] = max |dz_l|, [l][1] = max |dz1_l|

  const void* dy = dh_out;
  for (int l = L - 1; l >= 0; --l) {
    const void* agg = A + lay.agg[l];
    const void* a1 = A + lay.a1[l];
    const void* z = A + lay.z[l];
    const bool last = l == L - 1;
    MOLCLR_REQUIRE(gr->bn_weight[l] && gr->bn_bias[l], "gin_encoder_bwd: BatchNorm grads needed");
    if (h3) {
      // dz's row maxima for the h3 products (its max comes from the dz1
      // product's A reads: a max slot here would cost the BatchNorm backward
      // a block barrier)
      MOLCLR_TRY(seg_bn_bwd(seg, dy, z, e->bn_weight[l], e->bn_bias[l], F(lay.mean[l]),
                            F(lay.invstd[l]), dz, gr->bn_weight[l], gr->bn_bias[l], D,
                            MOLCLR_DTYPE_F32, last ? 0 : 1, 1, rdz, nullptr, kws, kws_bytes,
                            stream));
    } else {
      MOLCLR_TRY(seg_bn_bwd(seg, dy, z, e->bn_weight[l], e->bn_bias[l], F(lay.mean[l]),
                            F(lay.invstd[l]), dz, gr->bn_weight[l], gr->bn_bias[l], D, dt,
                            last ? 0 : 1, 1, nullptr, nullptr, kws, kws_bytes, stream));
    }
    if (bf) {
      const uint16_t *hz = (const uint16_t*)dz, *ha1 = (const uint16_t*)a1;
      // second Linear: dW2, db2 from dz and a1; dz1 = (dz W2) * (a1 > 0)
      if (gr->mlp2_weight[l] || gr->mlp2_bias[l]) {
        MOLCLR_REQUIRE(gr->mlp2_weight[l], "gin_encoder_bwd: bf16 needs the weight gradient");
        MOLCLR_TRY(molclr_linear_wgrad_bf16(hz, ha1, gr->mlp2_weight[l], gr->mlp2_bias[l], N, D,
                                            2 * D, D, 2 * D, 1, kws, kws_bytes, stream));
      }
      if (D % 64 == 0)  // the mask from the forward's bits
        MOLCLR_TRY(molclr_gemm_bf16_bits(hz, e->mlp2_planes_t[l], (uint16_t*)dz1, N, 2 * D, D, D,
                                         2 * D, MOLCLR_EPI_RELU_MASK, nullptr, nullptr,
                                         (const uint32_t*)(A + lay.bits[l]), stream));
      else
        MOLCLR_TRY(molclr_gemm_bf16(hz, e->mlp2_planes_t[l], (uint16_t*)dz1, N, 2 * D, D, D, 2 * D,
                                    MOLCLR_EPI_RELU_MASK, nullptr, ha1, 2 * D, stream));
      if (gr->mlp0_weight[l] || gr->mlp0_bias[l]) {
        MOLCLR_REQUIRE(gr->mlp0_weight[l], "gin_encoder_bwd: bf16 needs the weight gradient");
        MOLCLR_TRY(molclr_linear_wgrad_bf16((const uint16_t*)dz1, (const uint16_t*)agg,
                                            gr->mlp0_weight[l], gr->mlp0_bias[l], N, 2 * D, D,
                                            2 * D, D, 1, kws, kws_bytes, stream));
      }
      MOLCLR_TRY(molclr_gemm_bf16((const uint16_t*)dz1, e->mlp0_planes_t[l], (uint16_t*)dagg, N,
                                  D, 2 * D, 2 * D, D, MOLCLR_EPI_NONE, nullptr, nullptr, 0, stream));
      MOLCLR_TRY(molclr_gine_aggregate_bwd_bf16((const uint16_t*)dagg, g->rowptr_t, g->col_t,
                                                g->nbr_t, g->ecount, (uint16_t*)dh,
                                                gr->edge_embedding1[l], gr->edge_embedding2[l], N,
                                                D, 1, kws, kws_bytes, stream));
    } else if (h3) {
      // ops._MLP's h3 backward: dz1 (ReLU mask of a1), dW2 (+db2), dW1 (+db1),
      // dagg.  The data-gradient products scale A row by row (gradient rows
      // span many binades): dz's row maxima come from the BatchNorm backward,
      // max |dz| from the dz1 product's A reads, dz1's from its epilogue.
      const float *fz = (const float*)dz, *fa1 = (const float*)a1, *fagg = (const float*)agg;
      float* sl = bmax + 2 * l * kMaxSlotFloats;
      const float* fl = fmax + 2 * l * kMaxSlotFloats;
      MOLCLR_REQUIRE(gr->mlp2_weight[l] && gr->mlp2_bias[l] && gr->mlp0_weight[l] &&
                         gr->mlp0_bias[l],
                     "gin_encoder_bwd: h3 needs every MLP gradient");
      // dz1 (its epilogue yields dz1's max and row maxima), then the weight
      // gradients
      MOLCLR_TRY(molclr_gemm_f32_h3(fz, rdz, molclr_bn_row_parts(D), e->mlp2_planes_t[l],
                                    (float*)dz1, N, 2 * D, D, D, 2 * D, MOLCLR_EPI_RELU_MASK,
                                    nullptr, fa1, 2 * D, (const uint32_t*)(A + lay.bits[l]),
                                    sl + kMaxSlotFloats, rdz1, sl, stream));
      if (N >= 1024) {  // both weight gradients, one reduction launch
        MOLCLR_TRY(molclr_linear_wgrad_h3_pair(
            fz, sl, fa1, fl + kMaxSlotFloats, gr->mlp2_weight[l], gr->mlp2_bias[l], D, 2 * D, D,
            2 * D, (const float*)dz1, sl + kMaxSlotFloats, fagg, fl, gr->mlp0_weight[l],
            gr->mlp0_bias[l], 2 * D, D, 2 * D, D, N, 1, kws, kws_bytes, stream));
      } else {
        MOLCLR_TRY(molclr_linear_wgrad_h3(fz, sl, fa1, fl + kMaxSlotFloats, gr->mlp2_weight[l],
                                          gr->mlp2_bias[l], N, D, 2 * D, D, 2 * D, 1, kws,
                                          kws_bytes, stream));
        MOLCLR_TRY(molclr_linear_wgrad_h3((const float*)dz1, sl + kMaxSlotFloats, fagg, fl,
                                          gr->mlp0_weight[l], gr->mlp0_bias[l], N, 2 * D, D, 2 * D,
                                          D, 1, kws, kws_bytes, stream));
      }
      MOLCLR_TRY(molclr_gemm_f32_h3((const float*)dz1, rdz1, (int)molclr_gemm_row_parts(2 * D),
                                    e->mlp0_planes_t[l], (float*)dagg, N, D, 2 * D, 2 * D, D,
                                    MOLCLR_EPI_NONE, nullptr, nullptr, 0, nullptr, nullptr,
                                    nullptr, nullptr, stream));
      MOLCLR_TRY(molclr_gine_aggregate_bwd((const float*)dagg, g->rowptr_t, g->col_t, g->nbr_t,
                                           g->ecount, (float*)dh, gr->edge_embedding1[l],
                                           gr->edge_embedding2[l], N, D, 1, kws, kws_bytes, stream));
    } else {
      const float *fz = (const float*)dz, *fa1 = (const float*)a1;
      // second Linear (ops.linear_bwd order: dW with db, dx with the ReLU mask of a1)
      if (gr->mlp2_weight[l])
        MOLCLR_TRY(molclr_linear_wgrad(fz, fa1, gr->mlp2_weight[l], gr->mlp2_bias[l], N, D, 2 * D,
                                       D, 2 * D, 1, kws, kws_bytes, stream));
      else if (gr->mlp2_bias[l])
        MOLCLR_TRY(molclr_colsum_f32(fz, gr->mlp2_bias[l], N, D, D, 1, kws, kws_bytes, stream));
      MOLCLR_TRY(molclr_gemm_f32_bplanes(fz, e->mlp2_planes_t[l], (float*)dz1, N, 2 * D, D, D,
                                         2 * D, 0, MOLCLR_EPI_RELU_MASK, nullptr, fa1, 2 * D, kws,
                                         kws_bytes, stream));
      // first Linear
      if (gr->mlp0_weight[l])
        MOLCLR_TRY(molclr_linear_wgrad((const float*)dz1, (const float*)agg, gr->mlp0_weight[l],
                                       gr->mlp0_bias[l], N, 2 * D, D, 2 * D, D, 1, kws, kws_bytes,
                                       stream));
      else if (gr->mlp0_bias[l])
        MOLCLR_TRY(molclr_colsum_f32((const float*)dz1, gr->mlp0_bias[l], N, 2 * D, 2 * D, 1, kws,
                                     kws_bytes, stream));
      MOLCLR_TRY(molclr_gemm_f32_bplanes((const float*)dz1, e->mlp0_planes_t[l], (float*)dagg, N,
                                         D, 2 * D, 2 * D, D, 0, MOLCLR_EPI_NONE, nullptr, nullptr,
                                         0, kws, kws_bytes, stream));
      // aggregation: dh of the layer input, edge-table gradients
      MOLCLR_TRY(molclr_gine_aggregate_bwd((const float*)dagg, g->rowptr_t, g->col_t, g->nbr_t,
                                           g->ecount, (float*)dh, gr->edge_embedding1[l],
                                           gr->edge_embedding2[l], N, D, 1, kws, kws_bytes, stream));
    }
    MOLCLR_TRY(record_done(gr->layer_done[l], stream));
    dy = dh;
  }
  if (gr->x_embedding1 || gr->x_embedding2) {
    MOLCLR_REQUIRE(gr->x_embedding1 && gr->x_embedding2,
                   "gin_encoder_bwd: both atom-embedding grads or neither");
    if (bf)
      MOLCLR_TRY(molclr_atom_embed_bwd_bf16(x, (const uint16_t*)dh, gr->x_embedding1,
                                            gr->x_embedding2, N, D, e->n_atom, e->n_chiral, 1, kws,
                                            kws_bytes, stream));
    else
      MOLCLR_TRY(molclr_atom_embed_bwd(x, (const float*)dh, gr->x_embedding1, gr->x_embedding2, N,
                                       D, e->n_atom, e->n_chiral, 1, kws, kws_bytes, stream));
  }
  MOLCLR_TRY(record_done(gr->embed_done, stream));
  return MOLCLR_OK;
}

// ---------------------------------------------------------------------------
// GCN encoder executor (models/gcn_molclr.py:140-151), same scheme: per layer
// xw = x W (scratch), z = gcn_aggregate(xw) + bias (BatchNorm input, saved),
// h = BatchNorm(z) (+ReLU but the last; the next layer's input, saved).
// Arena: per layer z_l, h_l [N,D], mean_l / invstd_l [D]; then h0 [N,D].
// Workspace: xw / dxw, dz, dh [N,D] x 3, then the entry points' largest.
// ---------------------------------------------------------------------------
namespace {

struct GcnArena {
  size_t z[MOLCLR_MAX_LAYERS], h[MOLCLR_MAX_LAYERS], mean[MOLCLR_MAX_LAYERS],
      invstd[MOLCLR_MAX_LAYERS];
  size_t hmax[MOLCLR_MAX_LAYERS];  // h3: max slot of layer l's input (floats, contiguous)
  size_t h0, total;
  GcnArena(int L, int64_t N, int64_t D) {
    size_t used = 0;
    auto off = [&](size_t count) {
      const size_t o = used;
      used += (count + 63) / 64 * 64;
      return o;
    };
    for (int l = 0; l < L; ++l) {
      z[l] = off(N * D);
      h[l] = off(N * D);
      mean[l] = off(MOLCLR_MAX_SEGMENTS * D);  // [segment][D]
      invstd[l] = off(MOLCLR_MAX_SEGMENTS * D);
    }
    const size_t slots = off((size_t)L * kMaxSlotFloats);
    for (int l = 0; l < L; ++l) hmax[l] = slots + (size_t)l * kMaxSlotFloats;
    h0 = off(N * D);
    total = used * sizeof(float);
  }
};

size_t gcn_kernels_ws(int64_t N, int64_t D) {
  size_t m = 0;
  auto mx = [&](size_t v) { m = v > m ? v : m; };
  mx(molclr_gemm_f32_workspace_bytes(N, D, D));  // x W, dxw W^T
  mx(molclr_gemm_f32_workspace_bytes(D, D, N));  // dW = x^T dxw
  mx(molclr_linear_wgrad_workspace_bytes(N, D, D));  // its h3 form
  mx(molclr_batchnorm_ws_bound(N, D));
  mx(molclr_gcn_aggregate_bwd_workspace_bytes(N, D));
  mx(molclr_atom_embed_bwd_workspace_bytes(N, D, MOLCLR_NUM_ATOM_TYPE, MOLCLR_NUM_CHIRALITY));
  return m;
}
size_t gcn_scratch_floats(int64_t N, int64_t D) { return (size_t)N * D * 3; }
// h3 backward: dxw's row maxima [N] and max slot, after the scratch
size_t gcn_h3_bytes(int64_t N) {
  return molclr::align_up((size_t)N * sizeof(float), 256) + kMaxSlotFloats * sizeof(float);
}

int check_gcn(const molclr_gcn_encoder* e, const molclr_device_graph* g) {
  MOLCLR_REQUIRE(e && g, "gcn_encoder: null encoder / graph");
  MOLCLR_REQUIRE(e->num_layer >= 1 && e->num_layer <= MOLCLR_MAX_LAYERS,
                 "gcn_encoder: num_layer %d", e->num_layer);
  MOLCLR_REQUIRE(e->dim > 0 && e->dim % 4 == 0, "gcn_encoder: dim %lld", (long long)e->dim);
  MOLCLR_REQUIRE(e->n_atom == MOLCLR_NUM_ATOM_TYPE && e->n_chiral == MOLCLR_NUM_CHIRALITY,
                 "gcn_encoder: embedding tables must be [%d,D] and [%d,D]",
                 MOLCLR_NUM_ATOM_TYPE, MOLCLR_NUM_CHIRALITY);
  for (int l = 0; l < e->num_layer; ++l)
    MOLCLR_REQUIRE(e->weight_planes[l] && e->weight_planes_t[l] && e->bias[l] &&
                       e->edge_embedding1[l] && e->edge_embedding2[l] && e->bn_weight[l] &&
                       e->bn_bias[l],
                   "gcn_encoder: layer %d: missing planes, bias, edge tables or BatchNorm", l);
  return MOLCLR_OK;
}

}  // namespace

MOLCLR_API size_t molclr_gcn_encoder_arena_bytes(int L, int64_t N, int64_t D) {
  if (L < 1 || L > MOLCLR_MAX_LAYERS) return 0;
  return GcnArena(L, N, D).total;
}

MOLCLR_API size_t molclr_gcn_encoder_workspace_bytes(int L, int64_t N, int64_t D) {
  (void)L;
  return gcn_scratch_floats(N, D) * sizeof(float) + 256 + gcn_h3_bytes(N) + gcn_kernels_ws(N, D) +
         256;
}

MOLCLR_API int molclr_gcn_encoder_fwd(const molclr_gcn_encoder* e, const int64_t* x,
                                      const molclr_device_graph* g, float* h_out, void* arena,
                                      size_t arena_bytes, void* workspace, size_t workspace_bytes,
                                      molclr_stream_t stream) {
  MOLCLR_TRY(check_gcn(e, g));
  const int L = e->num_layer;
  const int64_t N = g->num_nodes, D = e->dim;
  if (N == 0) return MOLCLR_OK;
  SegRows seg;
  MOLCLR_TRY(graph_segments(g, &g->num_nodes, seg));
  MOLCLR_REQUIRE(x && h_out && arena, "gcn_encoder_fwd: null pointer");
  const GcnArena lay(L, N, D);
  MOLCLR_REQUIRE_WS(arena_bytes, lay.total);
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gcn_encoder_workspace_bytes(L, N, D));
  float* A = (float*)arena;
  float* xw = (float*)workspace;
  void* kws = (char*)workspace + molclr::align_up(gcn_scratch_floats(N, D) * sizeof(float), 256);
  const size_t kws_bytes = gcn_kernels_ws(N, D);

  const bool h3 = e->fp32_gemm == 1;
  if (h3 && molclr::zero_async(A + lay.hmax[0], (size_t)L * kMaxSlotFloats * sizeof(float),
                           molclr::as_stream(stream)) != hipSuccess) {
    molclr::set_error("gcn_encoder_fwd: zeroing the max slots failed");
    return MOLCLR_ERR_ARG;
  }
  float* h = A + lay.h0;
  MOLCLR_TRY(molclr_atom_embed_fwd(x, e->x_embedding1, e->x_embedding2, h, N, D, e->n_atom,
                                   e->n_chiral, e->status, stream));
  for (int l = 0; l < L; ++l) {
    float* z = A + lay.z[l];
    const bool last = l == L - 1;
    float* y = last ? h_out : A + lay.h[l];
    // x W, W [in, out] as a K-major B (ops.gemm_w(x, W, N, D, D, D, D, False, True))
    if (h3)  // the same product, also folding max |h| into the layer's slot
      MOLCLR_TRY(molclr_gemm_f32_bplanes_max(h, e->weight_planes[l], xw, N, D, D, D, D,
                                             MOLCLR_EPI_NONE, nullptr, nullptr, 0,
                                             (float*)(A + lay.hmax[l]), nullptr, nullptr, nullptr,
                                             kws, kws_bytes, stream));
    else
      MOLCLR_TRY(molclr_gemm_f32_bplanes(h, e->weight_planes[l], xw, N, D, D, D, D, 0,
                                       MOLCLR_EPI_NONE, nullptr, nullptr, 0, kws, kws_bytes,
                                       stream));
    MOLCLR_TRY(molclr_gcn_aggregate_fwd(xw, g->rowptr, g->col, g->ecode, g->nbr,
                                        e->edge_embedding1[l], e->edge_embedding2[l], e->bias[l],
                                        z, N, D, stream));
    MOLCLR_TRY(seg_bn_fwd(seg, z, e->bn_weight[l], e->bn_bias[l], e->bn_running_mean[l],
                          e->bn_running_var[l], e->bn_num_batches_tracked[l], y, A + lay.mean[l],
                          A + lay.invstd[l], D, MOLCLR_DTYPE_F32, e->momentum, e->eps,
                          e->training, last ? 0 : 1, kws, kws_bytes, stream));
    h = y;
  }
  return MOLCLR_OK;
}

MOLCLR_API int molclr_gcn_encoder_bwd(const molclr_gcn_encoder* e,
                                      const molclr_gcn_encoder_grads* gr, const int64_t* x,
                                      const molclr_device_graph* g, const float* dh_out,
                                      const void* arena, size_t arena_bytes, void* workspace,
                                      size_t workspace_bytes, molclr_stream_t stream) {
  MOLCLR_TRY(check_gcn(e, g));
  MOLCLR_REQUIRE(gr, "gcn_encoder_bwd: null grads");
  MOLCLR_REQUIRE(e->training, "gcn_encoder_bwd: backward through eval-mode BatchNorm");
  const int L = e->num_layer;
  const int64_t N = g->num_nodes, D = e->dim;
  if (N == 0) return MOLCLR_OK;
  SegRows seg;
  MOLCLR_TRY(graph_segments(g, &g->num_nodes, seg));
  MOLCLR_REQUIRE(x && dh_out && arena, "gcn_encoder_bwd: null pointer");
  const GcnArena lay(L, N, D);
  MOLCLR_REQUIRE_WS(arena_bytes, lay.total);
  MOLCLR_REQUIRE_WS(workspace_bytes, molclr_gcn_encoder_workspace_bytes(L, N, D));
  const float* A = (const float*)arena;
  float* S = (float*)workspace;
  float* dxw = S;
  float* dz = S + N * D;
  float* dh = S + 2 * N * D;
  // h3: dxw's row maxima and max slot
  float* rdxw = (float*)((char*)workspace +
                         molclr::align_up(gcn_scratch_floats(N, D) * sizeof(float), 256));
  float* sdxw = (float*)((char*)rdxw + molclr::align_up((size_t)N * sizeof(float), 256));
  void* kws = (char*)rdxw + gcn_h3_bytes(N);
  const size_t kws_bytes = gcn_kernels_ws(N, D);
  const bool h3 = e->fp32_gemm == 1;

  const float* dy = dh_out;
  for (int l = L - 1; l >= 0; --l) {
    const float* z = A + lay.z[l];
    const float* xin = l == 0 ? A + lay.h0 : A + lay.h[l - 1];
    const bool last = l == L - 1;
    MOLCLR_REQUIRE(gr->bn_weight[l] && gr->bn_bias[l], "gcn_encoder_bwd: BatchNorm grads needed");
    MOLCLR_TRY(seg_bn_bwd(seg, dy, z, e->bn_weight[l], e->bn_bias[l], A + lay.mean[l],
                          A + lay.invstd[l], dz, gr->bn_weight[l], gr->bn_bias[l], D,
                          MOLCLR_DTYPE_F32, last ? 0 : 1, 1, nullptr, nullptr, kws, kws_bytes,
                          stream));
    // ops._GCNConv.backward order: aggregation (dxw, edge tables, bias), dW, dx
    MOLCLR_TRY(molclr_gcn_aggregate_bwd(dz, g->rowptr_t, g->col_t, g->nbr_t, g->ecount, dxw,
                                        gr->edge_embedding1[l], gr->edge_embedding2[l],
                                        gr->bias[l], N, D, 1, kws, kws_bytes, stream));
    if (h3) {
      // ops._GCNConv's h3 backward: dxw's row maxima / max, dW = x^T dxw
      // (per-tensor scales), dx = dxw W^T (row-wise)
      MOLCLR_TRY(molclr_absmax_rows_f32(dxw, N, D, D, rdxw, sdxw, 0, stream));
      if (gr->weight[l])
        MOLCLR_TRY(molclr_linear_wgrad_h3(xin, A + lay.hmax[l], dxw, sdxw, gr->weight[l], nullptr,
                                          N, D, D, D, D, 1, kws, kws_bytes, stream));
      MOLCLR_TRY(molclr_gemm_f32_h3(dxw, rdxw, 1, e->weight_planes_t[l], dh, N, D, D, D, D,
                                    MOLCLR_EPI_NONE, nullptr, nullptr, 0, nullptr, nullptr,
                                    nullptr, nullptr, stream));
    } else {
      if (gr->weight[l])  // dW [in, out] = x^T dxw
        MOLCLR_TRY(molclr_gemm_f32(xin, dxw, gr->weight[l], D, D, N, D, D, D, 1, 1,
                                   MOLCLR_EPI_NONE | MOLCLR_EPI_ACCUMULATE, nullptr, nullptr, 0,
                                   kws, kws_bytes, stream));
      // dx = dxw W^T  (ops.gemm_w(dxw, W, N, D, D, D, D, False, False))
      MOLCLR_TRY(molclr_gemm_f32_bplanes(dxw, e->weight_planes_t[l], dh, N, D, D, D, D, 0,
                                         MOLCLR_EPI_NONE, nullptr, nullptr, 0, kws, kws_bytes,
                                         stream));
    }
    MOLCLR_TRY(record_done(gr->layer_done[l], stream));
    dy = dh;
  }
  if (gr->x_embedding1 || gr->x_embedding2) {
    MOLCLR_REQUIRE(gr->x_embedding1 && gr->x_embedding2,
                   "gcn_encoder_bwd: both atom-embedding grads or neither");
    MOLCLR_TRY(molclr_atom_embed_bwd(x, dh, gr->x_embedding1, gr->x_embedding2, N, D, e->n_atom,
                                     e->n_chiral, 1, kws, kws_bytes, stream));
  }
  MOLCLR_TRY(record_done(gr->embed_done, stream));
  return MOLCLR_OK;
}
