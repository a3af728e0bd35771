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
