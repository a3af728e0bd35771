// On-device rollout evaluation: the reference's test-time metrics over the
// finest scale of each simulation, computed where the rollout already lives instead of
// shipping [N, 2, T] to the host.
//   get_rollout_loss (RMSE / MAE, all nodes or only_where_water)  utils/miscellaneous.py:177-199,
//                                                                  training/loss.py:8-35
//   confusion matrix -> CSI / F1 at water-depth thresholds        utils/miscellaneous.py:123-169
//   stored water volume sum(area * h) per step, the core of the mass-conservation metric
//   get_mass_conservation_loss / conservation_loss      utils/miscellaneous.py:116-121,
//                                                         training/loss.py:120-169
// The kernels produce per-(simulation, step) sums in fp64 and exact integer counts; the host
// side (mswegnn/metrics.py) forms the reference's ratios.  No floating-point atomics: each
// workgroup writes its partial sums (waves combined in a fixed order), a second kernel adds the
// workgroups' partials in order -- the metrics are bit-reproducible run to run.  (The
// integer confusion counts use integer atomics: exact in any order.)
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../../include/mswegnn.h"
#include "engine.h"

namespace {

constexpr int kThreads = 256;
constexpr int kTChunk = 32;    // time steps per workgroup (blockIdx.y)
constexpr int kMaxThr = 4;
constexpr int kSums = 10;

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One thread = one fine-scale row of simulation g, all steps of the block's time chunk.
// sums[g][t][10]: sum|dh|, sum|dv|, sum dh^2, sum dv^2, the same four over the rows where
// dh != 0 or dv != 0 (mask_on_water), that row count, sum area * h_pred (0 without area).
// counts[g][t][k][4]: TP, TN, FP, FN of (pred_h > thr_k) vs (real_h > thr_k).
struct MetricArgs {
  const float* pred;
  const float* real;
  const float* area;            // [rows] by graph row, or null
  int T;
  int row0, nrows;  // fine-scale rows [row0, row0 + nrows) of this simulation
  int nthr;
  float thr[kMaxThr];
  double* part;                 // this simulation's [nblocks][T][kSums] workgroup partials
  unsigned long long* counts;   // this simulation's [T][nthr][4]
};

// Grid-stride over 256-row blocks (at most kMaxParts workgroups per simulation, so the partials
// do not grow with the mesh): each thread adds its rows' terms in row-block order, then the
// workgroup's waves are combined in a fixed order -- deterministic for a given grid.
constexpr int kMaxParts = 512;
__global__ __launch_bounds__(kThreads) void k_metrics(MetricArgs a) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __shared__ double wsum[kThreads / 64][kSums];
  const int t0 = blockIdx.y * kTChunk;
  for (int t = t0; t < t0 + kTChunk && t < a.T; ++t) {
    double acc[kSums];
#pragma unroll
    for (int k = 0; k < kSums; ++k) acc[k] = 0.0;
    for (int rb = blockIdx.x; rb * kThreads < a.nrows; rb += gridDim.x) {  // uniform per workgroup
      const int i = rb * kThreads + threadIdx.x;
      const bool valid = i < a.nrows;
      const size_t n = (size_t)a.row0 + (valid ? i : 0);
      float dh = 0.f, dv = 0.f, ph = 0.f, rh = 0.f;
      if (valid) {
        ph = a.pred[(n * 2 + 0) * a.T + t];
        rh = a.real[(n * 2 + 0) * a.T + t];
        dh = ph - rh;
        dv = a.pred[(n * 2 + 1) * a.T + t] - a.real[(n * 2 + 1) * a.T + t];
      }
      const double ar = valid && a.area ? (double)a.area[n] : 0.0;
      const bool wet = valid && (dh != 0.f || dv != 0.f);
      const double ah = fabs((double)dh), av = fabs((double)dv);
      const double qh = (double)dh * dh, qv = (double)dv * dv;
      acc[0] += ah;
      acc[1] += av;
      acc[2] += qh;
      acc[3] += qv;
      acc[4] += wet ? ah : 0.0;
      acc[5] += wet ? av : 0.0;
      acc[6] += wet ? qh : 0.0;
      acc[7] += wet ? qv : 0.0;
      acc[8] += wet ? 1.0 : 0.0;
      acc[9] += ar * (double)ph;
      for (int k = 0; k < a.nthr; ++k) {
        const bool p = ph > a.thr[k], r = rh > a.thr[k];
        const unsigned long long tp = __popcll(__ballot(valid && p && r));
        const unsigned long long tn = __popcll(__ballot(valid && !p && !r));
        const unsigned long long fp = __popcll(__ballot(valid && p && !r));
        const unsigned long long fn = __popcll(__ballot(valid && !p && r));
        if (lane == 0) {
          unsigned long long* c = a.counts + ((size_t)t * a.nthr + k) * 4;
          atomicAdd(c + 0, tp);
          atomicAdd(c + 1, tn);
          atomicAdd(c + 2, fp);
          atomicAdd(c + 3, fn);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < kSums; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0) {
#pragma unroll
      for (int k = 0; k < kSums; ++k) wsum[w][k] = acc[k];
    }
    __syncthreads();
    if (threadIdx.x < kSums) {  // the waves' sums in a fixed order
      double b = 0.0;
#pragma unroll
      for (int q = 0; q < kThreads / 64; ++q) b += wsum[q][threadIdx.x];
      a.part[((size_t)blockIdx.x * a.T + t) * kSums + threadIdx.x] = b;
    }
    __syncthreads();
  }
}

// sums[t][k] = sum over the workgroups b = 0, 1, ... (in order) of part[b][t][k]
__global__ __launch_bounds__(kThreads) void k_metrics_reduce(const double* __restrict__ part, int nblocks, long count,
                                                             double* __restrict__ sums) {
  const long i = blockIdx.x * (long)kThreads + threadIdx.x;
  if (i >= count) return;
  double v = 0.0;
  for (int b = 0; b < nblocks; ++b) v += part[(size_t)b * count + i];
  sums[i] = v;
}

}  // namespace

extern "C" int msw_rollout_metrics(const float* pred, const float* real, int32_t T,
                                   const int64_t* fine_ranges, int32_t num_sims,
                                   const float* thresholds, int32_t n_thr, const float* area, double* sums,
                                   uint64_t* counts, void* stream) {
  if (!pred || !real || !fine_ranges || !sums || (n_thr > 0 && (!thresholds || !counts)))
    return msw::set_error(MSW_ERR_INVALID, "null argument");
  if (T < 0 || num_sims < 0 || n_thr < 0 || n_thr > kMaxThr)
    return msw::set_error(MSW_ERR_INVALID, "T, num_sims or n_thr out of range (n_thr <= 4)");
  if (T == 0) return MSW_OK;
  hipStream_t st = (hipStream_t)stream;
  // one stream-ordered scratch for every simulation's workgroup partials, sized for the largest
  // (kMaxParts workgroups at most: bounded whatever the mesh)
  const long count = (long)T * kSums;
  int nb_max = 0;
  for (int g = 0; g < num_sims; ++g) {
    const long nr = fine_ranges[2 * g + 1] - fine_ranges[2 * g];
    if (nr < 0) return msw::set_error(MSW_ERR_INVALID, "fine range end < start");
    nb_max = std::max(nb_max, (int)std::min<long>(kMaxParts, (nr + kThreads - 1) / kThreads));
  }
  double* part = nullptr;
  if (nb_max > 0) {
    const hipError_t e = hipMallocAsync((void**)&part, (size_t)nb_max * count * sizeof(double), st);
    if (e != hipSuccess) return msw::set_error(MSW_ERR_HIP, hipGetErrorString(e));
  }
  hipError_t e = hipSuccess;
  for (int g = 0; g < num_sims && e == hipSuccess; ++g) {
    MetricArgs a{};
    a.pred = pred;
    a.real = real;
    a.area = area;
    a.T = T;
    a.row0 = (int)fine_ranges[2 * g];
    a.nrows = (int)(fine_ranges[2 * g + 1] - fine_ranges[2 * g]);
    a.nthr = n_thr;
    for (int k = 0; k < n_thr; ++k) a.thr[k] = thresholds[k];
    double* out = sums + (size_t)g * T * kSums;
    a.counts = reinterpret_cast<unsigned long long*>(counts) + (size_t)g * T * (n_thr > 0 ? n_thr : 1) * 4;
    if (a.nrows == 0) {  // no fine rows: zero sums (the caller zeroes the counts)
      e = hipMemsetAsync(out, 0, (size_t)count * sizeof(double), st);
      continue;
    }
    const int nb = (int)std::min<long>(kMaxParts, ((long)a.nrows + kThreads - 1) / kThreads);
    a.part = part;
    hipLaunchKernelGGL(k_metrics, dim3(nb, (T + kTChunk - 1) / kTChunk), dim3(kThreads), 0, st, a);
    hipLaunchKernelGGL(k_metrics_reduce, dim3((unsigned)((count + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                       (const double*)part, nb, count, out);
    e = hipGetLastError();
  }
  const hipError_t f = part ? hipFreeAsync(part, st) : hipSuccess;
  if (e != hipSuccess) return msw::set_error(MSW_ERR_HIP, hipGetErrorString(e));
  if (f != hipSuccess) return msw::set_error(MSW_ERR_HIP, hipGetErrorString(f));
  return MSW_OK;
}
