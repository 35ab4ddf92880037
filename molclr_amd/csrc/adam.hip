// Adam with coupled L2 weight decay over one flat parameter buffer, and the
// library's error/version plumbing.
//
// Reference: torch.optim.Adam(model.parameters(), init_lr,
// weight_decay=eval(config['weight_decay'])) stepped once per batch
// (molclr.py:84-87,127).  torch's Adam adds weight_decay * param to the
// gradient before the moments (coupled L2, not AdamW).
#include "common.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>

#include <mutex>
#include <vector>

namespace molclr {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

struct TimerRec {
  int kind;
  hipEvent_t e0, e1;
};
static std::mutex g_tmu;
static int g_tmask = 0;
static std::vector<TimerRec> g_trecs;

bool timer_wants(int kind) { return (g_tmask & kind) != 0; }
int& timer_kind_override() {
  thread_local int k = 0;
  return k;
}
void timer_record(int kind, hipEvent_t e0, hipEvent_t e1) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_trecs.push_back({kind, e0, e1});
}
}  // namespace molclr

namespace {

// torch.optim.Adam's multi-tensor (GPU) update, op for op:
//   g' = g + wd p;  m = lerp(m, g', 1 - b1);  v = v b2 + (1 - b2) g'^2;
//   p = p + (-lr / bc1) (m / (sqrt(v) / sqrt(bc2) + eps))
// with bc1 = 1 - b1^t, bc2 = 1 - b2^t, step_size and sqrt(bc2) evaluated in
// double (torch does them in Python floats on the host) and rounded to fp32
// once, as torch's scalar arguments are.  The step count t lives on the device.
// A block of 256 threads takes kAdamPer x 256 float4 (a thread's float4s
// 256 apart: coalesced), all loads issued before the math; thread 0 evaluates
// the step's scalars (two double pow) once for the block and shares them
// through LDS -- per thread, the fp64 pows cost the kernel ~3 us at c2.
constexpr int kAdamPer = 4;
__global__ __launch_bounds__(256) void k_adam_step(float4* __restrict__ p,
                                                   const float4* __restrict__ g,
                                                   float4* __restrict__ m, float4* __restrict__ v,
                                                   int64_t n4, const float* __restrict__ lr_ptr,
                                                   const int32_t* __restrict__ step_ptr, double b1,
                                                   double b2, float eps, float wd) {
  __shared__ float sc[2];
  const int64_t base = (int64_t)blockIdx.x * (256 * kAdamPer) + threadIdx.x;
  float4 pp[kAdamPer], gg[kAdamPer], mm[kAdamPer], vv[kAdamPer];
#pragma unroll
  for (int j = 0; j < kAdamPer; ++j) {
    const int64_t t = base + 256 * j;
    if (t < n4) {
      pp[j] = p[t];
      gg[j] = g[t];
      mm[j] = m[t];
      vv[j] = v[t];
    }
  }
  if (threadIdx.x == 0) {
    const int step = *step_ptr + 1;  // the counter is advanced by k_adam_tick afterwards
    const double bc1 = 1.0 - pow(b1, (double)step);
    const double bc2 = 1.0 - pow(b2, (double)step);
    sc[0] = (float)(-((double)*lr_ptr / bc1));
    sc[1] = (float)sqrt(bc2);
  }
  __syncthreads();
  const float neg_step_size = sc[0], bc2s = sc[1];
  const float w1 = (float)(1.0 - b1), fb2 = (float)b2, w2 = (float)(1.0 - b2);
#pragma unroll
  for (int j = 0; j < kAdamPer; ++j) {
    const int64_t t = base + 256 * j;
    if (t >= n4) continue;
    float4 P = pp[j], G = gg[j], M = mm[j], V = vv[j];
#define MOLCLR_ADAM_LANE(c)                                                   \
  {                                                                           \
    const float gr = G.c + wd * P.c;                                          \
    M.c = fabsf(w1) < 0.5f ? M.c + w1 * (gr - M.c) : gr - (gr - M.c) * (1.f - w1); \
    V.c = V.c * fb2 + w2 * gr * gr;                                           \
    const float den = sqrtf(V.c) / bc2s + eps;                                \
    P.c = P.c + neg_step_size * (M.c / den);                                  \
  }
    MOLCLR_ADAM_LANE(x)
    MOLCLR_ADAM_LANE(y)
    MOLCLR_ADAM_LANE(z)
    MOLCLR_ADAM_LANE(w)
#undef MOLCLR_ADAM_LANE
    p[t] = P;
    m[t] = M;
    v[t] = V;
  }
}

__global__ void k_adam_tick(int32_t* step) { *step += 1; }

// the captured step's last launch: Adam's step counter, the loss copied to
// the caller's buffer, the batch's status word ORed into the sticky word
__global__ void k_step_tail(int32_t* step, const float* loss_src, float* loss_dst,
                            const int32_t* status_src, int32_t* status_acc) {
  *step += 1;
  if (loss_dst) *loss_dst = *loss_src;
  if (status_acc) *status_acc |= *status_src;
}

}  // namespace

MOLCLR_API const char* molclr_version(void) { return "molclr_amd 0.1.0 gfx950"; }
MOLCLR_API const char* molclr_last_error(void) { return molclr::g_err; }

MOLCLR_API int molclr_adam_step(float* param, const float* grad, float* exp_avg,
                                float* exp_avg_sq, int64_t n, const float* lr, int32_t* step,
                                double beta1, double beta2, double eps, double weight_decay,
                                molclr_stream_t stream) {
  return molclr_adam_step_ex(param, grad, exp_avg, exp_avg_sq, n, lr, step, beta1, beta2, eps,
                             weight_decay, 1, stream);
}

MOLCLR_API int molclr_step_tail(int32_t* step, const float* loss_src, float* loss_dst,
                                const int32_t* status_src, int32_t* status_acc,
                                molclr_stream_t stream) {
  MOLCLR_REQUIRE(step && (!loss_dst || loss_src) && (!status_acc || status_src),
                 "step_tail: null pointer");
  hipLaunchKernelGGL(k_step_tail, dim3(1), dim3(1), 0, molclr::as_stream(stream), step, loss_src,
                     loss_dst, status_src, status_acc);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_adam_step_ex(float* param, const float* grad, float* exp_avg,
                                   float* exp_avg_sq, int64_t n, const float* lr, int32_t* step,
                                   double beta1, double beta2, double eps, double weight_decay,
                                   int tick, molclr_stream_t stream) {
  MOLCLR_REQUIRE(n % 4 == 0, "adam_step: flat buffer length %lld must be a multiple of 4",
                 (long long)n);
  MOLCLR_REQUIRE(lr && step, "adam_step: lr and step must be device pointers");
  hipStream_t s = molclr::as_stream(stream);
  int64_t n4 = n / 4;
  if (n4 > 0)
    hipLaunchKernelGGL(k_adam_step, dim3(molclr::ceil_div(n4, 256 * kAdamPer)), dim3(256), 0, s,
                       (float4*)param, (const float4*)grad, (float4*)exp_avg, (float4*)exp_avg_sq,
                       n4, lr, step, beta1, beta2, (float)eps, (float)weight_decay);
  if (tick) hipLaunchKernelGGL(k_adam_tick, dim3(1), dim3(1), 0, s, step);
  MOLCLR_LAUNCHED();
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ktimer_start(int kinds) {
  std::lock_guard<std::mutex> lk(molclr::g_tmu);
  molclr::g_tmask = kinds;
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ktimer_read(int kind, double* total_ms, int64_t* launches) {
  MOLCLR_REQUIRE(total_ms && launches, "ktimer_read: null output");
  std::lock_guard<std::mutex> lk(molclr::g_tmu);
  double ms = 0.0;
  int64_t n = 0;
  std::vector<molclr::TimerRec> keep;
  for (auto& r : molclr::g_trecs) {
    if (r.kind != kind) {
      keep.push_back(r);
      continue;
    }
    float t = 0.f;
    if (hipEventSynchronize(r.e1) == hipSuccess && hipEventElapsedTime(&t, r.e0, r.e1) == hipSuccess) {
      ms += t;
      ++n;
    }
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  molclr::g_trecs.swap(keep);
  *total_ms = ms;
  *launches = n;
  return MOLCLR_OK;
}

MOLCLR_API int molclr_ktimer_stop(void) {
  std::lock_guard<std::mutex> lk(molclr::g_tmu);
  molclr::g_tmask = 0;
  for (auto& r : molclr::g_trecs) {
    (void)hipEventDestroy(r.e0);
    (void)hipEventDestroy(r.e1);
  }
  molclr::g_trecs.clear();
  return MOLCLR_OK;
}
