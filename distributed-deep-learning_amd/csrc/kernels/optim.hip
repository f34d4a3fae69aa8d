// Fused optimizer updates on a flat parameter shard (one launch per shard range).
//
// TF1 ApplyAdam (mnist_sync/parameter_server.py:21,26-27), written in
// TF's own update form [TF-semantics]:
//   m += (g - m) * (1 - beta1);  v += (g*g - v) * (1 - beta2);
//   w -= lr_t * m / (sqrt(v) + eps),  lr_t = lr * sqrt(1 - beta2^t) / (1 - beta1^t)
// lr_t is computed on the host per PS step counter.  `scale` folds a 1/W gradient mean
// (or 1.0 for the reference's sum) into the same pass.  HBM-bound: 5 streams of fp32;
// 16-byte vector path (+ scalar tail) when every operand is 16-B aligned.
#include "common.h"
#include "api.h"

namespace ddl {


// 16-B body over n4 = n / 4 float4 elements; the n % 4 tail element(s) by the first lanes.
__global__ void __launch_bounds__(256)
adam_vec_kernel(float4* __restrict__ w, const float4* __restrict__ g, float4* __restrict__ m,
                float4* __restrict__ v, int64_t n, float lr_t, float c1, float c2, float eps,
                float scale) {
  const int64_t n4 = n >> 2;
  const int64_t gid = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  for (int64_t i = gid; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 W = w[i], G = g[i], M = m[i], V = v[i];
    adam1(W.x, G.x * scale, M.x, V.x, lr_t, c1, c2, eps);
    adam1(W.y, G.y * scale, M.y, V.y, lr_t, c1, c2, eps);
    adam1(W.z, G.z * scale, M.z, V.z, lr_t, c1, c2, eps);
    adam1(W.w, G.w * scale, M.w, V.w, lr_t, c1, c2, eps);
    w[i] = W; m[i] = M; v[i] = V;
  }
  if (gid < (n & 3)) {
    const int64_t e = 4 * n4 + gid;
    float* wf = reinterpret_cast<float*>(w);
    float* mf = reinterpret_cast<float*>(m);
    float* vf = reinterpret_cast<float*>(v);
    float W = wf[e], M = mf[e], V = vf[e];
    adam1(W, reinterpret_cast<const float*>(g)[e] * scale, M, V, lr_t, c1, c2, eps);
    wf[e] = W; mf[e] = M; vf[e] = V;
  }
}
__global__ void __launch_bounds__(256)
adam_scalar_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                   float* __restrict__ v, int64_t n, float lr_t, float c1, float c2, float eps,
                   float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float W = w[i], M = m[i], V = v[i];
    adam1(W, g[i] * scale, M, V, lr_t, c1, c2, eps);
    w[i] = W; m[i] = M; v[i] = V;
  }
}

__global__ void __launch_bounds__(256)
momentum_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                int64_t n, float lr, float mu, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float ww = w[i], mm = m[i];
    momentum1(ww, g[i], mm, lr, mu, scale);
    m[i] = mm;
    w[i] = ww;
  }
}

__global__ void __launch_bounds__(256) scale_kernel(float* __restrict__ p, int64_t n, float a) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] *= a;
}
static int grid_for(int64_t n, int max_grid = 2048) {
  int64_t b = (n + 255) / 256;
  if (b > max_grid) b = max_grid;  // (2048: 8 blocks per CU) grid-stride beyond
  return b < 1 ? 1 : (int)b;
}

void launch_adam(float* w, const float* g, float* m, float* v, int64_t n, float lr_t, float b1,
                 float b2, float eps, float scale, hipStream_t st) {
  launch_adam_c(w, g, m, v, n, lr_t, 1.f - b1, 1.f - b2, eps, scale, st);
}

void launch_adam_c(float* w, const float* g, float* m, float* v, int64_t n, float lr_t, float c1,
                   float c2, float eps, float scale, hipStream_t st, int max_grid) {
  if (n <= 0) return;
  const uintptr_t al = (uintptr_t)w | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v;
  if ((al & 15) == 0) {
    DDL_LAUNCH(adam_vec_kernel, dim3(grid_for((n + 3) / 4, max_grid)), dim3(256), 0, st,
               (float4*)w, (const float4*)g, (float4*)m, (float4*)v, n, lr_t, c1, c2, eps, scale);
  } else {
    DDL_LAUNCH(adam_scalar_kernel, dim3(grid_for(n, max_grid)), dim3(256), 0, st, w, g, m, v, n,
                       lr_t, c1, c2, eps, scale);
  }
}

void launch_momentum(float* w, const float* g, float* m, int64_t n, float lr, float mu,
                     float scale, hipStream_t st) {
  if (n <= 0) return;
  DDL_LAUNCH(momentum_kernel, dim3(grid_for(n)), dim3(256), 0, st, w, g, m, n, lr, mu,
                     scale);
}

void launch_scale(float* p, int64_t n, float a, hipStream_t st) {
  if (n <= 0) return;
  DDL_LAUNCH(scale_kernel, dim3(grid_for(n)), dim3(256), 0, st, p, n, a);
}
}  // namespace ddl
