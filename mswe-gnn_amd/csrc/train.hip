// Autograd through the model's layers on gfx950: the training forward (saving
// what the backward needs) and the backward of
//   SWEGNN.forward  models/gnn.py:387-445   (msw_swegnn_train_*)
//   make_mlp        models/models.py:121-146 (msw_mlp_train_*: encoders gnn.py:204-215, decoder :239-240)
//   _pooling        models/gnn.py:242-257     (msw_pool_mean_*: mean pooling, learnable=False)
// as the reference trains it (training_step, training/train.py:125-145).  The reference
// recomputes s_ij from the active edges of every hop; s_ij depends on the hop only through
// the mask, so by linearity of the backward ONE MLP backward of ds = sum_k [active_k] ds_k
// gives the same parameter and input gradients.
//
// Kernels (all deterministic: fixed summation orders, CSR pulls, split-K partials reduced in
// order -- no atomics):
//   k_gemm        C = A B on v_mfma_f32_16x16x4_f32, generic strides (the three shapes of a
//                 linear layer: X W^T forward, dY W backward, dY^T X weight gradient with
//                 split-K over the rows), epilogues bias / activation / addend / partials
//   k_gather_cat  the edge-MLP input rows [x_s[row], x_s[col], x_d[row], x_d[col], e]
//   k_normalize   s = h / ||h||, NaN -> 0 (gnn.py:424-426)
//   k_hop_agg     per destination: sum of active messages in CSR (reference edge) order
//   k_edge_bwd / k_node_bwd   the hop's transpose: per edge ds and the message gradient,
//                 per node the pull over in-edges (CSR by col) and out-edges (CSR by row)
//   k_act_bwd, k_colsum, k_scatter_inputs, k_sum_splits
#include <cmath>
#include <cstring>
#include <string>
#include <type_traits>

#include "../../include/mswegnn.h"
#include "engine.h"

namespace {

using msw::set_error;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kBM = 64, kBN = 64, kBK = 16, kGemmThreads = 256;
constexpr int kMaxSplits = 256;
constexpr int kMaxHops = 8;

__device__ __forceinline__ float act_fwd(int act, float x, float a) {
  switch (act) {
    case MSW_ACT_PRELU: return x > 0.f ? x : a * x;
    case MSW_ACT_RELU: return x > 0.f ? x : 0.f;
    case MSW_ACT_LEAKYRELU: return x > 0.f ? x : 0.1f * x;
    case MSW_ACT_ELU: return x > 0.f ? x : expm1f(x);
    case MSW_ACT_SWISH: return x / (1.f + expf(-x));
    case MSW_ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    case MSW_ACT_TANH: return tanhf(x);
    default: return x;
  }
}
// d act / d x at the pre-activation x
__device__ __forceinline__ float act_grad(int act, float x, float a) {
  switch (act) {
    case MSW_ACT_PRELU: return x > 0.f ? 1.f : a;
    case MSW_ACT_RELU: return x > 0.f ? 1.f : 0.f;
    case MSW_ACT_LEAKYRELU: return x > 0.f ? 1.f : 0.1f;
    case MSW_ACT_ELU: return x > 0.f ? 1.f : expf(x);
    case MSW_ACT_SWISH: {
      const float sg = 1.f / (1.f + expf(-x));
      return sg * (1.f + x * (1.f - sg));
    }
    case MSW_ACT_SIGMOID: {
      const float sg = 1.f / (1.f + expf(-x));
      return sg * (1.f - sg);
    }
    case MSW_ACT_TANH: {
      const float t = tanhf(x);
      return 1.f - t * t;
    }
    default: return 1.f;
  }
}

// ------------------------------------------------------------------------------------ GEMM
// C(m, n) = sum_k A(m, k) B(k, n), A(m, k) = A[m lam + k lak], B(k, n) = B[k lbk + n lbn].
// 64 x 64 output tile per 256-thread workgroup, 16-deep K slices staged in LDS (k-major, so
// the MFMA fragments are read along m / n across lanes); each wave owns a 32 x 32 quarter as
// 2 x 2 tiles of v_mfma_f32_16x16x4_f32 (A: lane l gives A(i = l & 15, k = l >> 4); B: lane l
// gives B(k = l >> 4, j = l & 15); D: lane l holds D(4 (l >> 4) + r, l & 15)).  Split-K
// (part != null, the weight gradients dY^T X): F64 -- the fp32 operands multiplied on
// v_mfma_f64_16x16x4_f64 (exact products, fp64 sums; D: lane l holds D((l >> 4) + 4 r, l & 15)),
// workgroup z writes K slice z as doubles into part[z][M][N]; k_sum_splits adds the slices in
// order in fp64.  A weight / bias gradient sums every edge or node of a layer, often with heavy
// cancellation (a PReLU slope's gradient sums every element): fp64 accumulation leaves only the
// final rounding, closer to exact arithmetic than torch's own fp32 reductions.
struct GemmArgs {
  int M, N, K;
  const float* A; long lam, lak;
  const float* B; long lbk, lbn;
  float* C; long ldc;
  const float* addend; long ldd;  // C = addend + AB (nullable)
  const float* bias;              // + bias[n] (nullable)
  float* pre; long ldp;           // pre-activation store (nullable)
  int act; const float* slope;    // activation of the stored C (device scalar slope)
  float* part; int kchunk;        // split-K partials
  int bones;                      // B(k, N - 1) = 1: an implicit ones column (bias gradient)
};

template <bool F64>
__global__ __launch_bounds__(kGemmThreads) void k_gemm(GemmArgs a) {
  using acc_t = typename std::conditional<F64, f64x4, f32x4>::type;
  __shared__ float As[kBK][kBM + 4];
  __shared__ float Bs[kBK][kBN + 4];
  constexpr int UA = (kBM * kBK) / kGemmThreads, UB = (kBN * kBK) / kGemmThreads;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int m0 = blockIdx.x * kBM, n0 = blockIdx.y * kBN;
  const int kb = a.part ? blockIdx.z * a.kchunk : 0;
  const int ke = a.part ? min(a.K, kb + a.kchunk) : a.K;
  const int wm = (w & 1) * 32, wn = (w >> 1) * 32;
  acc_t acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = acc_t{0, 0, 0, 0};
  const bool a_mfast = a.lam == 1 && a.lak != 1;  // A stored m-contiguous (transposed operand)
  const bool b_kfast = a.lbk == 1 && a.lbn != 1;  // B stored k-contiguous
  // per thread: its UA + UB tile elements (fixed positions), the next slice's values in
  // registers while the current slice is multiplied out of LDS (global latency hidden)
  int am[UA], ak[UA], bn[UB], bk[UB];
#pragma unroll
  for (int u = 0; u < UA; ++u) {
    const int idx = tid + u * kGemmThreads;
    am[u] = a_mfast ? idx % kBM : idx / kBK;
    ak[u] = a_mfast ? idx / kBM : idx % kBK;
  }
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    const int idx = tid + u * kGemmThreads;
    bn[u] = b_kfast ? idx / kBK : idx % kBN;
    bk[u] = b_kfast ? idx % kBK : idx / kBN;
  }
  float ra[UA], rb[UB];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < UA; ++u) {
      const int m = m0 + am[u], k = k0 + ak[u];
      ra[u] = (m < a.M && k < ke) ? a.A[(long)m * a.lam + (long)k * a.lak] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int n = n0 + bn[u], k = k0 + bk[u];
      rb[u] = (n < a.N && k < ke) ? ((a.bones && n == a.N - 1) ? 1.f : a.B[(long)k * a.lbk + (long)n * a.lbn]) : 0.f;
    }
  };
  if (kb < ke) fetch(kb);
  for (int k0 = kb; k0 < ke; k0 += kBK) {
#pragma unroll
    for (int u = 0; u < UA; ++u) As[ak[u]][am[u]] = ra[u];
#pragma unroll
    for (int u = 0; u < UB; ++u) Bs[bk[u]][bn[u]] = rb[u];
    __syncthreads();
    if (k0 + kBK < ke) fetch(k0 + kBK);
#pragma unroll
    for (int k4 = 0; k4 < kBK; k4 += 4) {
      const int kr = k4 + (lane >> 4);
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = As[kr][wm + 16 * i + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Bs[kr][wn + 16 * j + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          if constexpr (F64)
            acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)av[i], (double)bv[j], acc[i][j], 0, 0, 0);
          else
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
        }
    }
    __syncthreads();
  }
  const float sl = a.slope ? *a.slope : 0.f;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + (F64 ? (lane >> 4) + 4 * r : 4 * (lane >> 4) + r);
        const int n = n0 + wn + 16 * j + (lane & 15);
        if (m >= a.M || n >= a.N) continue;
        if constexpr (F64) {  // split-K weight gradients only
          reinterpret_cast<double*>(a.part)[((long)blockIdx.z * a.M + m) * a.N + n] = acc[i][j][r];
          continue;
        } else {
        float v = acc[i][j][r];
        if (a.part) {
          a.part[((long)blockIdx.z * a.M + m) * a.N + n] = v;
          continue;
        }
        if (a.addend) v = a.addend[(long)m * a.ldd + n] + v;
        if (a.bias) v = v + a.bias[n];
        if (a.pre) a.pre[(long)m * a.ldp + n] = v;
        a.C[(long)m * a.ldc + n] = act_fwd(a.act, v, sl);
        }
      }
}

// out[i] = sum_{s < splits} part[s][i], i < count (fp64 partials, summed in fp64).  A
// 256-thread workgroup owns 64 outputs; row group p (of 4) adds splits p, p + 4, ... in order,
// then the 4 partials are added in order through LDS (fixed order: deterministic)
__global__ __launch_bounds__(256) void k_sum_splits(const double* __restrict__ part, int splits, long count,
                                                    float* __restrict__ out) {
  __shared__ double red[4][64];
  const int c = threadIdx.x & 63, p = threadIdx.x >> 6;
  for (long i0 = blockIdx.x * 64L; i0 < count; i0 += gridDim.x * 64L) {
    const long i = i0 + c;
    double v = 0.0;
    if (i < count) {
#pragma unroll 8
      for (int s = p; s < splits; s += 4) v += part[(long)s * count + i];
    }
    red[p][c] = v;
    __syncthreads();
    if (p == 0 && i < count) out[i] = (float)(((red[0][c] + red[1][c]) + red[2][c]) + red[3][c]);
    __syncthreads();
  }
}

// k_sum_splits over [M][N1] partials whose last column is the bias gradient: columns < N1 - 1
// go to dW [M][N1 - 1], the last to db [M]
__global__ __launch_bounds__(256) void k_sum_splits_wb(const double* __restrict__ part, int splits, int M, int N1,
                                                       float* __restrict__ dW, float* __restrict__ db) {
  __shared__ double red[4][64];
  const int c = threadIdx.x & 63, p = threadIdx.x >> 6;
  const long count = (long)M * N1;
  for (long i0 = blockIdx.x * 64L; i0 < count; i0 += gridDim.x * 64L) {
    const long i = i0 + c;
    double v = 0.0;
    if (i < count) {
#pragma unroll 8
      for (int s = p; s < splits; s += 4) v += part[(long)s * count + i];
    }
    red[p][c] = v;
    __syncthreads();
    if (p == 0 && i < count) {
      const float t = (float)(((red[0][c] + red[1][c]) + red[2][c]) + red[3][c]);
      const long m = i / N1;
      const int n = (int)(i - m * N1);
      if (n < N1 - 1) dW[m * (N1 - 1) + n] = t;
      else db[m] = t;
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------------ elementwise
// X0[e] = [x_s[row], x_s[col], x_d[row], x_d[col], edge_attr[e]]  (gnn.py:414-420)
__global__ void k_gather_cat(const int* __restrict__ row, const int* __restrict__ col, const float* __restrict__ xs,
                             const float* __restrict__ xd, const float* __restrict__ ea, int F, int ef, long E,
                             float* __restrict__ X0) {
  const int w0 = 4 * F + ef;
  const long total = E * w0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long e = i / w0;
    const int c = (int)(i - e * w0);
    float v;
    if (c < F) v = xs[(long)row[e] * F + c];
    else if (c < 2 * F) v = xs[(long)col[e] * F + c - F];
    else if (c < 3 * F) v = xd[(long)row[e] * F + c - 2 * F];
    else if (c < 4 * F) v = xd[(long)col[e] * F + c - 3 * F];
    else v = ea[e * ef + c - 4 * F];
    X0[i] = v;
  }
}

// s = h / ||h||_2, NaN -> 0 (gnn.py:424-426); one thread per edge
__global__ void k_normalize(const float* __restrict__ h, int F, long E, int normalize, float* __restrict__ s,
                            float* __restrict__ nrm) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < E; e += (long)gridDim.x * blockDim.x) {
    const float* he = h + e * F;
    float* se = s + e * F;
    if (!normalize) {
      for (int f = 0; f < F; ++f) se[f] = he[f];
      nrm[e] = 1.f;
      continue;
    }
    float q = 0.f;
    for (int f = 0; f < F; ++f) q += he[f] * he[f];
    const float n = sqrtf(q);
    nrm[e] = n;
    for (int f = 0; f < F; ++f) {
      const float v = he[f] / n;
      se[f] = isnan(v) ? 0.f : v;
    }
  }
}

// nz[n] = (sum_f out[n][f]) != 0  (gnn.py:408)
__global__ void k_node_nz(const float* __restrict__ out, int F, long N, int* __restrict__ nz) {
  for (long n = blockIdx.x * (long)blockDim.x + threadIdx.x; n < N; n += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int f = 0; f < F; ++f) v += out[n * F + f];
    nz[n] = v != 0.f ? 1 : 0;
  }
}

// agg[c][f] = sum over active in-edges e of c (reference order) of the message
// (out[c] - out[row]) s (upwind: clamped at 0) or s out[row] (gnn.py:410-438)
__global__ void k_hop_agg(const int* __restrict__ in_ptr, const int* __restrict__ in_edge,
                          const int* __restrict__ row, const float* __restrict__ out, const float* __restrict__ s,
                          const int* __restrict__ nz, int F, long N, int grad, int upwind, float* __restrict__ agg) {
  const long total = N * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long c = i / F;
    const int f = (int)(i - c * F);
    const float oc = out[c * F + f];
    const int zc = nz[c];
    float acc = 0.f;
    for (int q = in_ptr[c]; q < in_ptr[c + 1]; ++q) {
      const int e = in_edge[q], r = row[e];
      if (!(zc | nz[r])) continue;
      float m;
      if (grad) {
        float d = oc - out[(long)r * F + f];
        if (upwind && d < 0.f) d = 0.f;
        m = d * s[(long)e * F + f];
      } else {
        m = s[(long)e * F + f] * out[(long)r * F + f];
      }
      acc += m;
    }
    agg[i] = acc;
  }
}

// The hop's transpose, per edge: dm = dagg[col] on active edges; ds += dm * gradient term;
// t = dm * s * (upwind: [diff > 0]) -- the message's derivative w.r.t. out
__global__ void k_edge_bwd(const int* __restrict__ row, const int* __restrict__ col, const float* __restrict__ out,
                           const float* __restrict__ s, const int* __restrict__ nz, const float* __restrict__ dagg,
                           int F, long E, int grad, int upwind, float* __restrict__ ds, float* __restrict__ t) {
  const long total = E * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long e = i / F;
    const int f = (int)(i - e * F);
    const int r = row[e], c = col[e];
    if (!(nz[r] | nz[c])) {
      t[i] = 0.f;
      continue;
    }
    const float dm = dagg[(long)c * F + f], se = s[i];
    if (grad) {
      const float d = out[(long)c * F + f] - out[(long)r * F + f];
      const bool pass = !upwind || d >= 0.f;  // hydraulic_gradient[hg < 0] = 0 (gnn.py:431-432)
      ds[i] += dm * (pass ? d : 0.f);
      t[i] = pass ? dm * se : 0.f;
    } else {
      ds[i] += dm * out[(long)r * F + f];
      t[i] = dm * se;
    }
  }
}

// Gn[c] = G[c] + sum_{e in in(c)} t_e - sum_{e in out(c)} t_e   (with_gradient)
//       = G[c] + sum_{e in out(c)} t_e                         (s * out[row])
__global__ void k_node_bwd(const int* __restrict__ in_ptr, const int* __restrict__ in_edge,
                           const int* __restrict__ out_ptr, const int* __restrict__ out_edge,
                           const float* __restrict__ G, const float* __restrict__ t, int F, long N, int grad,
                           float* __restrict__ Gn) {
  const long total = N * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / F;
    const int f = (int)(i - n * F);
    float a = 0.f, b = 0.f;
    if (grad)
      for (int q = in_ptr[n]; q < in_ptr[n + 1]; ++q) a += t[(long)in_edge[q] * F + f];
    for (int q = out_ptr[n]; q < out_ptr[n + 1]; ++q) b += t[(long)out_edge[q] * F + f];
    Gn[i] = grad ? G[i] + (a - b) : G[i] + b;
  }
}

// dh = (ds - s (s . ds)) / ||h|| (0 where the norm is 0: s was set to 0 there)
__global__ void k_normalize_bwd(const float* __restrict__ s, const float* __restrict__ nrm,
                                const float* __restrict__ ds, int F, long E, int normalize, float* __restrict__ dh) {
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < E; e += (long)gridDim.x * blockDim.x) {
    const float* se = s + e * F;
    const float* de = ds + e * F;
    float* out = dh + e * F;
    if (!normalize) {
      for (int f = 0; f < F; ++f) out[f] = de[f];
      continue;
    }
    const float n = nrm[e];
    if (!(n > 0.f)) {
      for (int f = 0; f < F; ++f) out[f] = 0.f;
      continue;
    }
    float dot = 0.f;
    for (int f = 0; f < F; ++f) dot += se[f] * de[f];
    for (int f = 0; f < F; ++f) out[f] = (de[f] - se[f] * dot) / n;
  }
}

// dpre = dy * act'(pre); PReLU slope: per-block partial of sum(pre <= 0 ? pre * dy : 0)
// (torch's prelu backward), fp64 products and sums, written to spart[blockIdx.x]
__global__ __launch_bounds__(256) void k_act_bwd(const float* __restrict__ pre, const float* __restrict__ dy, long count,
                                                 int act, const float* __restrict__ slope, float* __restrict__ dpre,
                                                 double* __restrict__ spart) {
  __shared__ double red[256];
  const float a = slope ? *slope : 0.f;
  double sacc = 0.0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < count; i += (long)gridDim.x * blockDim.x) {
    const float x = pre[i], g = dy[i];
    dpre[i] = g * act_grad(act, x, a);
    if (act == MSW_ACT_PRELU && !(x > 0.f)) sacc += (double)x * (double)g;
  }
  red[threadIdx.x] = sacc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0 && spart) spart[blockIdx.x] = red[0];
}

// column sums of X [R][W] over row slice blockIdx.x -> part[blockIdx.x][W] (fp64): thread t
// sums column t % W over rows t / W, t / W + P, ... (P = 256 / W row lanes), then the P
// partials are added in order through LDS (deterministic)
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ X, long R, int W, long rchunk,
                                                double* __restrict__ part) {
  __shared__ double red[256];
  const long r0 = blockIdx.x * rchunk, r1 = min(R, r0 + rchunk);
  for (int c0 = 0; c0 < W; c0 += 256) {
    const int wc = min(256, W - c0);
    const int P = 256 / wc;
    const int c = threadIdx.x % wc, rl = threadIdx.x / wc;
    double v = 0.0;
    if (rl < P)
      for (long r = r0 + rl; r < r1; r += P) v += X[r * W + c0 + c];
    red[threadIdx.x] = v;
    __syncthreads();
    if ((int)threadIdx.x < wc) {
      double sacc = 0.0;
      for (int p = 0; p < P; ++p) sacc += red[p * wc + threadIdx.x];
      part[(long)blockIdx.x * W + c0 + threadIdx.x] = sacc;
    }
    __syncthreads();
  }
}

// input gradients from dX0 [E][4F + ef]: x_s / x_d rows pull their out-edge (row) and in-edge
// (col) slices (CSR orders), dxd accumulates onto the filter-0 term already there
__global__ void k_scatter_inputs(const int* __restrict__ in_ptr, const int* __restrict__ in_edge,
                                 const int* __restrict__ out_ptr, const int* __restrict__ out_edge,
                                 const float* __restrict__ dX0, int F, int ef, long N, float* __restrict__ dxs,
                                 float* __restrict__ dxd) {
  const int w0 = 4 * F + ef;
  const long total = N * F;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / F;
    const int f = (int)(i - n * F);
    float as = 0.f, ad = 0.f, bs = 0.f, bd = 0.f;
    for (int q = out_ptr[n]; q < out_ptr[n + 1]; ++q) {
      const float* r = dX0 + (long)out_edge[q] * w0;
      as += r[f];
      ad += r[2 * F + f];
    }
    for (int q = in_ptr[n]; q < in_ptr[n + 1]; ++q) {
      const float* r = dX0 + (long)in_edge[q] * w0;
      bs += r[F + f];
      bd += r[3 * F + f];
    }
    if (dxs) dxs[i] = as + bs;
    if (dxd) dxd[i] = dxd[i] + (ad + bd);
  }
}

__global__ void k_copy_cols(const float* __restrict__ src, long rows, int src_ld, int c0, int w,
                            float* __restrict__ dst) {
  const long total = rows * w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / w;
    dst[i] = src[r * src_ld + c0 + (i - r * w)];
  }
}

// Mean pooling (gnn.py:242-257, learnable=False): out[c] = sum of x[fine] over c's children in
// pooling-edge order / max(#children, 1) -- a pull over the CSR by coarse node, no atomics;
// backward dx[f] = sum over f's pooling edges of dout[c] / max(#children of c, 1).
__global__ void k_pool_fwd(const int* __restrict__ cptr, const int* __restrict__ cedge, const int* __restrict__ fine,
                           const float* __restrict__ x, int F, long N, float* __restrict__ out) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < N * F; i += (long)gridDim.x * blockDim.x) {
    const long c = i / F;
    const int f = (int)(i - c * F);
    const int b = cptr[c], e = cptr[c + 1];
    float acc = 0.f;
    for (int q = b; q < e; ++q) acc += x[(long)fine[cedge[q]] * F + f];
    const int cnt = e - b;
    out[i] = acc / (float)(cnt > 1 ? cnt : 1);
  }
}
__global__ void k_pool_bwd(const int* __restrict__ fptr, const int* __restrict__ fedge, const int* __restrict__ coarse,
                           const int* __restrict__ cptr, const float* __restrict__ dout, int F, long N,
                           float* __restrict__ dx) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < N * F; i += (long)gridDim.x * blockDim.x) {
    const long n = i / F;
    const int f = (int)(i - n * F);
    float acc = 0.f;
    for (int q = fptr[n]; q < fptr[n + 1]; ++q) {
      const int c = coarse[fedge[q]];
      const int cnt = cptr[c + 1] - cptr[c];
      acc += dout[(long)c * F + f] / (float)(cnt > 1 ? cnt : 1);
    }
    dx[i] = acc;
  }
}

__global__ void k_add(const float* __restrict__ a, const float* __restrict__ b, long n, float* __restrict__ c) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    c[i] = a[i] + b[i];
}

// ---------------------------------------------------------------------------------- host
inline int blocks_for(long n, int threads = 256) {
  long b = (n + threads - 1) / threads;
  return (int)std::max<long>(1, std::min<long>(b, 16384));
}

// split-K partial slices a weight gradient over R rows uses (weight_grad) -- also bounds the
// column-sum slices of mlp_backward (ceil(R / max(256, R / kMaxSplits)) <= this)
inline long splits_for(long R) { return std::min<long>(kMaxSplits, std::max<long>(1, R / (8 * kBK))); }

struct Layout {  // float offsets into the saved / scratch buffers
  long X0, pre[4], post[4], s, nrm, outk, agg, nz, saved;
  long G0, G1, dagg, t, ds, dA, dB, part, spart, scratch;
  int L, w[5], wmax;
};

bool layout_of(const msw_swegnn_train_desc* d, Layout& y) {
  if (!d || d->n_layers < 1 || d->n_layers > 4 || d->F < 1 || d->K < 1 || d->K > kMaxHops || d->num_nodes < 0 ||
      d->num_edges < 0 || d->edge_features < 0)
    return false;
  const long E = d->num_edges, N = d->num_nodes, F = d->F;
  y.L = d->n_layers;
  y.wmax = 0;
  for (int l = 0; l <= y.L; ++l) {
    y.w[l] = d->width[l];
    if (y.w[l] <= 0) return false;
    y.wmax = std::max(y.wmax, y.w[l]);
  }
  if (y.w[0] != 4 * F + d->edge_features || y.w[y.L] != F) return false;
  auto al = [](long n) { return (n + 63) / 64 * 64; };
  long o = 0;
  y.X0 = o; o += al(E * y.w[0]);
  for (int l = 0; l < y.L; ++l) { y.pre[l] = o; o += al(E * y.w[l + 1]); }
  for (int l = 0; l < y.L; ++l) { y.post[l] = o; o += al(E * y.w[l + 1]); }
  y.s = o; o += al(E * F);
  y.nrm = o; o += al(E);
  y.outk = o; o += al((long)(d->K + 1) * N * F);
  y.agg = o; o += al((long)d->K * N * F);
  y.nz = o; o += al((long)d->K * N);
  y.saved = o;
  o = 0;
  y.G0 = o; o += al(N * F);
  y.G1 = o; o += al(N * F);
  y.dagg = o; o += al(N * F);
  y.t = o; o += al(E * F);
  y.ds = o; o += al(E * F);
  y.dA = o; o += al(E * y.wmax);
  y.dB = o; o += al(E * y.wmax);
  y.part = o; o += al(2L * splits_for(std::max(E, N)) * y.wmax * (y.wmax + 1));  // fp64 partials
  y.spart = o; o += al(kMaxSplits * 4L);
  y.scratch = o;
  return true;
}

struct MlpRun {
  long R;
  int L;
  const int* w;    // widths [L + 1]
  const int* act;  // [L]
  const float* const* W;
  const float* const* b;
  const float* const* slope;
};

struct MlpLayout {  // float offsets: saved = pre[0..L-1], post[0..L-2]; scratch = A, B, partials
  long pre[4], post[4], saved;
  long A, B, part, spart, scratch;
  int L, w[5], wmax;
};

bool mlp_layout_of(const msw_mlp_train_desc* d, MlpLayout& y) {
  if (!d || d->n_layers < 1 || d->n_layers > 4 || d->rows < 0) return false;
  const long R = d->rows;
  y.L = d->n_layers;
  y.wmax = 0;
  for (int l = 0; l <= y.L; ++l) {
    y.w[l] = d->width[l];
    if (y.w[l] <= 0) return false;
    y.wmax = std::max(y.wmax, y.w[l]);
  }
  for (int l = 0; l < y.L; ++l)
    if (!d->weight[l]) return false;
  auto al = [](long n) { return (n + 63) / 64 * 64; };
  long o = 0;
  for (int l = 0; l < y.L; ++l) { y.pre[l] = o; o += al(R * y.w[l + 1]); }
  for (int l = 0; l + 1 < y.L; ++l) { y.post[l] = o; o += al(R * y.w[l + 1]); }
  y.saved = o;
  o = 0;
  y.A = o; o += al(R * y.wmax);
  y.B = o; o += al(R * y.wmax);
  y.part = o; o += al(2L * splits_for(R) * y.wmax * (y.wmax + 1));  // fp64 partials
  y.spart = o; o += al(kMaxSplits * 4L);
  y.scratch = o;
  return true;
}

MlpRun mlp_of(const msw_swegnn_train_desc* d, const Layout& y, long rows) {
  return MlpRun{rows, y.L, y.w, d->act, d->weight, d->bias, d->slope};
}

hipError_t gemm(const GemmArgs& a0, hipStream_t st, int splits = 1) {
  GemmArgs a = a0;
  dim3 grid((a.M + kBM - 1) / kBM, (a.N + kBN - 1) / kBN, 1);
  if (a.part) {
    splits = std::max(1, std::min(splits, kMaxSplits));
    a.kchunk = ((a.K + splits - 1) / splits + kBK - 1) / kBK * kBK;
    grid.z = (a.K + a.kchunk - 1) / a.kchunk;
    if (grid.z == 0) grid.z = 1;
  }
  if (a.part)
    hipLaunchKernelGGL(k_gemm<true>, grid, dim3(kGemmThreads), 0, st, a);
  else
    hipLaunchKernelGGL(k_gemm<false>, grid, dim3(kGemmThreads), 0, st, a);
  return hipGetLastError();
}

// dW [M][N] = sum_rows A(row, m) B(row, n): split-K over the rows, partials summed in order
// db (nullable) [M] = sum_rows A(row, m): the same GEMM against an implicit ones column of B
// (part: [splits][M][N (+ 1)] doubles)
hipError_t weight_grad(const float* A, int lda, const float* B, int ldb, long R, int M, int N, float* part,
                       float* dW, hipStream_t st, float* db = nullptr) {
  GemmArgs g{};
  g.M = M; g.N = db ? N + 1 : N; g.K = (int)R;
  g.A = A; g.lam = 1; g.lak = lda;
  g.B = B; g.lbk = ldb; g.lbn = 1;
  g.part = part;
  g.bones = db ? 1 : 0;
  const int splits = (int)splits_for(R);
  hipError_t e = gemm(g, st, splits);
  if (e != hipSuccess) return e;
  const int kchunk = ((g.K + splits - 1) / splits + kBK - 1) / kBK * kBK;
  const int used = std::max(1, (g.K + kchunk - 1) / kchunk);
  const double* p64 = reinterpret_cast<const double*>(part);
  if (db)
    hipLaunchKernelGGL(k_sum_splits_wb, dim3(blocks_for((long)M * g.N, 64)), dim3(256), 0, st, p64, used, M, g.N, dW,
                       db);
  else
    hipLaunchKernelGGL(k_sum_splits, dim3(blocks_for((long)M * N, 64)), dim3(256), 0, st, p64, used, (long)M * N,
                       dW);
  return hipGetLastError();
}

// One make_mlp stack (models/models.py:121-146: Linear + activation after every layer) over R
// rows: the forward saves every layer's pre-activation (and output: the next layer's input),
// the backward walks the layers in reverse -- activation / PReLU-slope, bias (column sums),
// weight (split-K) and input gradients.  Shared by the SWEGNN edge MLP and msw_mlp_train_*.

hipError_t mlp_forward(const MlpRun& m, const float* X, float* const* pre, float* const* post, hipStream_t st) {
  const float* in = X;
  for (int l = 0; l < m.L; ++l) {
    GemmArgs g{};
    g.M = (int)m.R; g.N = m.w[l + 1]; g.K = m.w[l];
    g.A = in; g.lam = m.w[l]; g.lak = 1;
    g.B = m.W[l]; g.lbk = 1; g.lbn = m.w[l];  // B(k, n) = W[n][k]
    g.C = post[l]; g.ldc = m.w[l + 1];
    g.bias = m.b[l];
    g.pre = pre[l]; g.ldp = m.w[l + 1];
    g.act = m.act[l]; g.slope = m.slope[l];
    hipError_t e = gemm(g, st);
    if (e != hipSuccess) return e;
    in = post[l];
  }
  return hipSuccess;
}

// dY [R][w_L] (read-only; may be bufA) -> dX [R][w_0] (null: not needed; may be bufA);
// bufA / bufB: [R][max width] each; part: split partials; spart: [kMaxSplits]
hipError_t mlp_backward(const MlpRun& m, const float* X, const float* const* pre, const float* const* post,
                        const float* dY, float* dX, float* const* dW, float* const* db, float* const* dslope,
                        float* bufA, float* bufB, float* part, float* spart, hipStream_t st) {
  const long R = m.R;
  const long rchunk = std::max<long>(256, (R + kMaxSplits - 1) / kMaxSplits);
  const int nrs = (int)((R + rchunk - 1) / rchunk);
  const float* dcur = dY;
  float* dpre = bufB;
  double* sp64 = reinterpret_cast<double*>(spart);
  double* p64 = reinterpret_cast<double*>(part);
  for (int l = m.L - 1; l >= 0; --l) {
    const int wi = m.w[l], wo = m.w[l + 1];
    const int ab = blocks_for(R * wo) < kMaxSplits ? blocks_for(R * wo) : kMaxSplits;
    hipLaunchKernelGGL(k_act_bwd, dim3(ab), dim3(256), 0, st, pre[l], dcur, R * wo, m.act[l], m.slope[l], dpre, sp64);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    if (dslope[l]) hipLaunchKernelGGL(k_sum_splits, dim3(1), dim3(256), 0, st, sp64, ab, 1L, dslope[l]);
    // the bias gradient rides on the weight-gradient GEMM as an extra ones column of X where
    // that column fits the last 64-wide output tile; else its own column sums
    const bool fuse_db = db[l] && dW[l] && wi % kBN != 0;
    if (db[l] && !fuse_db) {
      hipLaunchKernelGGL(k_colsum, dim3(nrs), dim3(256), 0, st, dpre, R, wo, rchunk, p64);
      hipLaunchKernelGGL(k_sum_splits, dim3(blocks_for(wo, 64)), dim3(256), 0, st, p64, nrs, (long)wo, db[l]);
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const float* Xl = l == 0 ? X : post[l - 1];
    if (dW[l] && (e = weight_grad(dpre, wo, Xl, wi, R, wo, wi, part, dW[l], st, fuse_db ? db[l] : nullptr)) != hipSuccess)
      return e;
    float* tgt = l == 0 ? dX : bufA;
    if (tgt) {
      GemmArgs g{};  // d X_l = dpre W_l
      g.M = (int)R; g.N = wi; g.K = wo;
      g.A = dpre; g.lam = wo; g.lak = 1;
      g.B = m.W[l]; g.lbk = wi; g.lbn = 1;
      g.C = tgt; g.ldc = wi;
      if ((e = gemm(g, st)) != hipSuccess) return e;
    }
    dcur = bufA;
  }
  return hipSuccess;
}

#define TRY(x)                                                                     \
  do {                                                                             \
    hipError_t _e = (x);                                                           \
    if (_e != hipSuccess) return set_error(MSW_ERR_HIP, hipGetErrorString(_e));    \
  } while (0)

}  // namespace

extern "C" {

int msw_swegnn_train_workspace(const msw_swegnn_train_desc* d, int64_t* saved_floats, int64_t* scratch_floats) {
  Layout y;
  if (!layout_of(d, y)) return set_error(MSW_ERR_INVALID, "inconsistent SWEGNN training descriptor");
  if (saved_floats) *saved_floats = y.saved;
  if (scratch_floats) *scratch_floats = y.scratch;
  return MSW_OK;
}

int msw_swegnn_train_forward(const msw_swegnn_train_desc* d, const float* xs, const float* xd, const float* ea,
                             float* saved, float* out, void* stream) {
  Layout y;
  if (!layout_of(d, y)) return set_error(MSW_ERR_INVALID, "inconsistent SWEGNN training descriptor");
  if (!xs || !xd || !saved || !out || (d->edge_features > 0 && !ea)) return set_error(MSW_ERR_INVALID, "null argument");
  if (d->with_filter_matrix)
    for (int k = 0; k <= d->K; ++k)
      if (!d->filter[k]) return set_error(MSW_ERR_INVALID, "filter matrix missing");
  hipStream_t st = (hipStream_t)stream;
  const long E = d->num_edges, N = d->num_nodes;
  const int F = d->F;
  float* X0 = saved + y.X0;
  if (E > 0) {
    hipLaunchKernelGGL(k_gather_cat, dim3(blocks_for(E * y.w[0])), dim3(256), 0, st, d->row, d->col, xs, xd, ea, F,
                       d->edge_features, E, X0);
    TRY(hipGetLastError());
    float* pre[4];
    float* post[4];
    for (int l = 0; l < y.L; ++l) {
      pre[l] = saved + y.pre[l];
      post[l] = saved + y.post[l];
    }
    TRY(mlp_forward(mlp_of(d, y, E), X0, pre, post, st));
    hipLaunchKernelGGL(k_normalize, dim3(blocks_for(E)), dim3(256), 0, st, saved + y.post[y.L - 1], F, E, d->normalize,
                       saved + y.s, saved + y.nrm);
    TRY(hipGetLastError());
  }
  // out_0 = filter_matrix[0] x_d (gnn.py:401-404)
  float* o0 = saved + y.outk;
  if (d->with_filter_matrix) {
    GemmArgs g{};
    g.M = (int)N; g.N = F; g.K = F;
    g.A = xd; g.lam = F; g.lak = 1;
    g.B = d->filter[0]; g.lbk = 1; g.lbn = F;
    g.C = o0; g.ldc = F;
    TRY(gemm(g, st));
  } else {
    TRY(hipMemcpyAsync(o0, xd, sizeof(float) * N * F, hipMemcpyDeviceToDevice, st));
  }
  for (int k = 0; k < d->K; ++k) {
    const float* ok = saved + y.outk + (long)k * N * F;
    float* on = k + 1 == d->K ? out : saved + y.outk + (long)(k + 1) * N * F;  // out_K is not needed later
    float* agg = saved + y.agg + (long)k * N * F;
    int* nz = reinterpret_cast<int*>(saved + y.nz + (long)k * N);
    hipLaunchKernelGGL(k_node_nz, dim3(blocks_for(N)), dim3(256), 0, st, ok, F, N, nz);
    hipLaunchKernelGGL(k_hop_agg, dim3(blocks_for(N * F)), dim3(256), 0, st, d->in_ptr, d->in_edge, d->row, ok,
                       saved + y.s, nz, F, N, d->with_gradient, d->upwind_mode, agg);
    TRY(hipGetLastError());
    if (d->with_filter_matrix) {  // out_{k+1} = out_k + filter_matrix[k+1](agg)
      GemmArgs g{};
      g.M = (int)N; g.N = F; g.K = F;
      g.A = agg; g.lam = F; g.lak = 1;
      g.B = d->filter[k + 1]; g.lbk = 1; g.lbn = F;
      g.C = on; g.ldc = F;
      g.addend = ok; g.ldd = F;
      TRY(gemm(g, st));
    } else {
      hipLaunchKernelGGL(k_add, dim3(blocks_for(N * F)), dim3(256), 0, st, ok, agg, N * F, on);
      TRY(hipGetLastError());
    }
  }
  return MSW_OK;
}

int msw_swegnn_train_backward(const msw_swegnn_train_desc* d, const float* xs, const float* xd, const float* ea,
                              const float* saved, const float* grad_out, const msw_swegnn_grads* gr, float* scratch,
                              void* stream) {
  (void)xs;
  (void)ea;
  Layout y;
  if (!layout_of(d, y)) return set_error(MSW_ERR_INVALID, "inconsistent SWEGNN training descriptor");
  if (!xd || !saved || !grad_out || !gr || !scratch) return set_error(MSW_ERR_INVALID, "null argument");
  if (!gr->d_x_d) return set_error(MSW_ERR_INVALID, "d_x_d is required (it accumulates the filter-0 term)");
  hipStream_t st = (hipStream_t)stream;
  const long E = d->num_edges, N = d->num_nodes;
  const int F = d->F;
  const float* G = grad_out;  // read-only: the first hop's transpose writes G1
  float* Gbuf[2] = {scratch + y.G0, scratch + y.G1};
  int gi = 0;
  float* dagg = scratch + y.dagg;
  float* t = scratch + y.t;
  float* ds = scratch + y.ds;
  float* part = scratch + y.part;
  if (E > 0) TRY(hipMemsetAsync(ds, 0, sizeof(float) * E * F, st));
  for (int k = d->K - 1; k >= 0; --k) {
    const float* ok = saved + y.outk + (long)k * N * F;
    const float* agg = saved + y.agg + (long)k * N * F;
    const int* nz = reinterpret_cast<const int*>(saved + y.nz + (long)k * N);
    if (d->with_filter_matrix) {
      if (gr->d_filter[k + 1]) TRY(weight_grad(G, F, agg, F, N, F, F, part, gr->d_filter[k + 1], st));
      GemmArgs g{};  // dagg = G W_{k+1}
      g.M = (int)N; g.N = F; g.K = F;
      g.A = G; g.lam = F; g.lak = 1;
      g.B = d->filter[k + 1]; g.lbk = F; g.lbn = 1;
      g.C = dagg; g.ldc = F;
      TRY(gemm(g, st));
    }
    const float* dg = d->with_filter_matrix ? dagg : G;  // no filter: dagg = G
    if (E > 0) {
      hipLaunchKernelGGL(k_edge_bwd, dim3(blocks_for(E * F)), dim3(256), 0, st, d->row, d->col, ok, saved + y.s, nz,
                         dg, F, E, d->with_gradient, d->upwind_mode, ds, t);
      TRY(hipGetLastError());
    }
    float* Gn = Gbuf[gi];
    gi ^= 1;
    hipLaunchKernelGGL(k_node_bwd, dim3(blocks_for(N * F)), dim3(256), 0, st, d->in_ptr, d->in_edge, d->out_ptr,
                       d->out_edge, G, t, F, N, d->with_gradient, Gn);
    TRY(hipGetLastError());
    G = Gn;
  }
  // out_0 = W_0 x_d
  if (d->with_filter_matrix) {
    if (gr->d_filter[0]) TRY(weight_grad(G, F, xd, F, N, F, F, part, gr->d_filter[0], st));
    GemmArgs g{};
    g.M = (int)N; g.N = F; g.K = F;
    g.A = G; g.lam = F; g.lak = 1;
    g.B = d->filter[0]; g.lbk = F; g.lbn = 1;
    g.C = gr->d_x_d; g.ldc = F;
    TRY(gemm(g, st));
  } else {
    TRY(hipMemcpyAsync(gr->d_x_d, G, sizeof(float) * N * F, hipMemcpyDeviceToDevice, st));
  }
  if (E == 0) {
    if (gr->d_x_s) TRY(hipMemsetAsync(gr->d_x_s, 0, sizeof(float) * N * F, st));
    for (int l = 0; l < y.L; ++l) {
      if (gr->d_weight[l]) TRY(hipMemsetAsync(gr->d_weight[l], 0, sizeof(float) * y.w[l] * y.w[l + 1], st));
      if (gr->d_bias[l]) TRY(hipMemsetAsync(gr->d_bias[l], 0, sizeof(float) * y.w[l + 1], st));
      if (gr->d_slope[l]) TRY(hipMemsetAsync(gr->d_slope[l], 0, sizeof(float), st));
    }
    return MSW_OK;
  }
  // s = normalize(h): ds -> dh
  float* dcur = scratch + y.dA;
  float* dpre = scratch + y.dB;
  hipLaunchKernelGGL(k_normalize_bwd, dim3(blocks_for(E)), dim3(256), 0, st, saved + y.s, saved + y.nrm, ds, F, E,
                     d->normalize, dcur);
  TRY(hipGetLastError());
  {
    const float* pre[4];
    const float* post[4];
    for (int l = 0; l < y.L; ++l) {
      pre[l] = saved + y.pre[l];
      post[l] = saved + y.post[l];
    }
    float* dW[4] = {gr->d_weight[0], gr->d_weight[1], gr->d_weight[2], gr->d_weight[3]};
    float* db[4] = {gr->d_bias[0], gr->d_bias[1], gr->d_bias[2], gr->d_bias[3]};
    float* dsl[4] = {gr->d_slope[0], gr->d_slope[1], gr->d_slope[2], gr->d_slope[3]};
    TRY(mlp_backward(mlp_of(d, y, E), saved + y.X0, pre, post, dcur, dcur, dW, db, dsl, dcur, dpre, part,
                     scratch + y.spart, st));
  }
  // dcur = dX0 [E][4F + ef]
  hipLaunchKernelGGL(k_scatter_inputs, dim3(blocks_for(N * F)), dim3(256), 0, st, d->in_ptr, d->in_edge, d->out_ptr,
                     d->out_edge, dcur, F, d->edge_features, N, gr->d_x_s, gr->d_x_d);
  TRY(hipGetLastError());
  if (d->edge_features > 0 && gr->d_edge_attr) {
    hipLaunchKernelGGL(k_copy_cols, dim3(blocks_for(E * d->edge_features)), dim3(256), 0, st, dcur, E, y.w[0], 4 * F,
                       d->edge_features, gr->d_edge_attr);
    TRY(hipGetLastError());
  }
  return MSW_OK;
}

int msw_mlp_train_workspace(const msw_mlp_train_desc* d, int64_t* saved_floats, int64_t* scratch_floats) {
  MlpLayout y;
  if (!mlp_layout_of(d, y)) return set_error(MSW_ERR_INVALID, "inconsistent MLP training descriptor");
  if (saved_floats) *saved_floats = y.saved;
  if (scratch_floats) *scratch_floats = y.scratch;
  return MSW_OK;
}

int msw_mlp_train_forward(const msw_mlp_train_desc* d, const float* x, float* saved, float* out, void* stream) {
  MlpLayout y;
  if (!mlp_layout_of(d, y)) return set_error(MSW_ERR_INVALID, "inconsistent MLP training descriptor");
  if (d->rows == 0) return MSW_OK;
  if (!x || !saved || !out) return set_error(MSW_ERR_INVALID, "null argument");
  float* pre[4];
  float* post[4];
  for (int l = 0; l < y.L; ++l) {
    pre[l] = saved + y.pre[l];
    post[l] = l + 1 < y.L ? saved + y.post[l] : out;
  }
  TRY(mlp_forward(MlpRun{d->rows, y.L, y.w, d->act, d->weight, d->bias, d->slope}, x, pre, post,
                  (hipStream_t)stream));
  return MSW_OK;
}

int msw_mlp_train_backward(const msw_mlp_train_desc* d, const float* x, const float* saved, const float* grad_out,
                           const msw_mlp_grads* gr, float* scratch, void* stream) {
  MlpLayout y;
  if (!mlp_layout_of(d, y)) return set_error(MSW_ERR_INVALID, "inconsistent MLP training descriptor");
  if (!gr) return set_error(MSW_ERR_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  float* dW[4] = {gr->d_weight[0], gr->d_weight[1], gr->d_weight[2], gr->d_weight[3]};
  float* db[4] = {gr->d_bias[0], gr->d_bias[1], gr->d_bias[2], gr->d_bias[3]};
  float* dsl[4] = {gr->d_slope[0], gr->d_slope[1], gr->d_slope[2], gr->d_slope[3]};
  if (d->rows == 0) {  // no rows: every gradient is zero
    for (int l = 0; l < y.L; ++l) {
      if (dW[l]) TRY(hipMemsetAsync(dW[l], 0, sizeof(float) * y.w[l] * y.w[l + 1], st));
      if (db[l]) TRY(hipMemsetAsync(db[l], 0, sizeof(float) * y.w[l + 1], st));
      if (dsl[l]) TRY(hipMemsetAsync(dsl[l], 0, sizeof(float), st));
    }
    return MSW_OK;
  }
  if (!x || !saved || !grad_out || !scratch) return set_error(MSW_ERR_INVALID, "null argument");
  const float* pre[4];
  const float* post[4];
  for (int l = 0; l < y.L; ++l) {
    pre[l] = saved + y.pre[l];
    post[l] = l + 1 < y.L ? saved + y.post[l] : nullptr;  // the output is not needed
  }
  TRY(mlp_backward(MlpRun{d->rows, y.L, y.w, d->act, d->weight, d->bias, d->slope}, x, pre, post, grad_out,
                   gr->d_x, dW, db, dsl, scratch + y.A, scratch + y.B, scratch + y.part, scratch + y.spart, st));
  return MSW_OK;
}

int msw_pool_mean_forward(int64_t num_nodes, int32_t F, const int32_t* fine, const int32_t* cptr,
                          const int32_t* cedge, const float* x, float* out, void* stream) {
  if (num_nodes < 0 || F < 1) return set_error(MSW_ERR_INVALID, "bad pooling sizes");
  if (num_nodes == 0) return MSW_OK;
  if (!fine || !cptr || !cedge || !x || !out) return set_error(MSW_ERR_INVALID, "null argument");
  hipLaunchKernelGGL(k_pool_fwd, dim3(blocks_for(num_nodes * F)), dim3(256), 0, (hipStream_t)stream, cptr, cedge,
                     fine, x, F, (long)num_nodes, out);
  TRY(hipGetLastError());
  return MSW_OK;
}

int msw_pool_mean_backward(int64_t num_nodes, int32_t F, const int32_t* coarse, const int32_t* cptr,
                           const int32_t* fptr, const int32_t* fedge, const float* grad_out, float* grad_x,
                           void* stream) {
  if (num_nodes < 0 || F < 1) return set_error(MSW_ERR_INVALID, "bad pooling sizes");
  if (num_nodes == 0) return MSW_OK;
  if (!coarse || !cptr || !fptr || !fedge || !grad_out || !grad_x) return set_error(MSW_ERR_INVALID, "null argument");
  hipLaunchKernelGGL(k_pool_bwd, dim3(blocks_for(num_nodes * F)), dim3(256), 0, (hipStream_t)stream, fptr, fedge,
                     coarse, cptr, grad_out, F, (long)num_nodes, grad_x);
  TRY(hipGetLastError());
  return MSW_OK;
}

}  // extern "C"
