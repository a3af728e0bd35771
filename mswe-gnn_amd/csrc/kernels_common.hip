// Non-templated kernels: rollout state initialisation and device-side I/O records.
#include "kernels_impl.h"

namespace msw {

// x (graph numbering) -> internal rollout state + BC of step 0
// (rollout_test training/train.py:87-90, apply_boundary_condition dataset.py:486-497)
__global__ __launch_bounds__(kBlock) void k_init_state(InitArgs a) {
  const int n = blockIdx.x * kBlock + threadIdx.x;
  if (n == 0) a.io->step = -1;
  if (n >= a.N) return;
  const int ext = a.perm ? a.perm[n] : n;
  if (ext < 0) return;  // padding row of the 16-aligned internal numbering
  float* xr = a.X + (size_t)n * a.nnf;
  const float* src = a.x0 + (size_t)ext * a.nnf;
  for (int k = 0; k < a.nnf; ++k) xr[k] = src[k];
  const int b = a.bc_slot ? a.bc_slot[n] : -1;
  if (b >= 0) {
    const int nstat = a.nnf - a.dyn;
    for (int tau = 0; tau < a.p; ++tau)
      xr[nstat + (a.io->type_bc - 1) + 2 * tau] = a.io->bc[((size_t)b * a.p + tau) * a.io->bc_tstride];
  }
}

__global__ void k_set_slots(SlotArgs a) {
  const int i = threadIdx.x;
  if (i < a.n) a.slot[a.row[i]] = a.val[i];
}

__global__ void k_set_io(RolloutIO* dst, RolloutIO v) {
  if (threadIdx.x == 0) *dst = v;
}

// Halo exchange row moves: dst[drow(i)] = src[srow(i)] for i < n, rows of `width` floats
// (multiple of 4); a null index array is the identity (contiguous staging buffer).
__global__ __launch_bounds__(kBlock) void k_copy_rows(const float* __restrict__ src, const int* __restrict__ srows,
                                                      float* __restrict__ dst, const int* __restrict__ drows,
                                                      int n, int width) {
  const int w4 = width / 4;
  const long i = (long)blockIdx.x * kBlock + threadIdx.x;
  if (i >= (long)n * w4) return;
  const int r = (int)(i / w4), c = (int)(i % w4) * 4;
  const size_t s = (size_t)(srows ? srows[r] : r) * width + c;
  const size_t d = (size_t)(drows ? drows[r] : r) * width + c;
  *reinterpret_cast<float4*>(dst + d) = *reinterpret_cast<const float4*>(src + s);
}

hipError_t launch_copy_rows(const float* src, const int* srows, float* dst, const int* drows, int n, int width,
                            hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const long total = (long)n * (width / 4);
  hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, st, src, srows,
                     dst, drows, n, width);
  return hipGetLastError();
}

hipError_t launch_init_state(const InitArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_init_state, dim3(cdiv(a.N > 0 ? a.N : 1, kBlock)), dim3(kBlock), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_set_slots(const SlotArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_set_slots, dim3(1), dim3(kSlotBatch), 0, st, a);
  return hipGetLastError();
}
hipError_t launch_set_io(RolloutIO* dst, const RolloutIO& v, hipStream_t st) {
  hipLaunchKernelGGL(k_set_io, dim3(1), dim3(64), 0, st, dst, v);
  return hipGetLastError();
}

}  // namespace msw
