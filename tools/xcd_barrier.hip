// Microbenchmark (verdict r2 item 3): what does a barrier among G <= 32 co-resident
// workgroups on ONE XCD cost on MI355X, against the kernel boundary it would replace?
//
// Each phase every participating workgroup reads the 1-KB record its neighbour wrote in the
// previous phase (a dependent cross-CU hand-off, like a hop gathering the previous hop's rows),
// checks it, and writes its own.  Participants are workgroups b with b % 8 == 0 of a grid of
// 8 G workgroups: workgroups b and b + 8 share an XCD (MI355X_MICROARCH.md, dispatch), so all
// G sit on one XCD, as the engine's XCD packing places the coarse scales (kernels_impl.h).
//
// Variants (per phase, P phases per launch; per-phase cost = slope over P):
//   launch   one kernel launch per phase, P launches captured in one hipGraph
//   acquire  one launch; barrier = lane-0 agent release fence + relaxed agent counter add,
//            relaxed poll, agent acquire fence, workgroup barrier; plain record loads/stores
//   sc1      one launch; records stored and loaded with agent-scope relaxed atomics (sc1,
//            L2-served, no L1), every storing wave waits vmcnt(0) before the workgroup
//            barrier, lane 0 adds to the counter and polls it -- no fences
// Every spin is bounded (an expired spin sets an error flag and leaves).
//
//   hipcc --offload-arch=gfx950 -O3 tools/xcd_barrier.hip -o tools/_bin/xcd_barrier
//   tools/_bin/xcd_barrier  -> one JSON line per (variant, G)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                 \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
      exit(2);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kThreads = 256;   // one 1-KB record (256 floats) per workgroup
constexpr int kSpin = 1 << 22;  // bounded polls

struct Args {
  float* rec;         // [2][G][256] ping-pong records
  unsigned* ctr;      // barrier counter (monotonic)
  int* err;           // [0] wrong values, [1] expired spins
  unsigned* xcc;      // [G] XCC id of each participant
  int G, phases, phase0;
};

__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xf;
}

// one phase of work: read the neighbour's record of phase p-1, check, write own record of p
template <bool SC1>
__device__ __forceinline__ void phase_work(const Args& a, int b, int p) {
  const int t = threadIdx.x;
  float v = 0.f;
  if (p > 0) {
    const float* src = a.rec + ((size_t)((p - 1) & 1) * a.G + (b + 1) % a.G) * kThreads + t;
    v = SC1 ? __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *src;
    if (v != (float)(p - 1)) atomicAdd(&a.err[0], 1);
  }
  float* dst = a.rec + ((size_t)(p & 1) * a.G + b) * kThreads + t;
  if (SC1) __hip_atomic_store(dst, (float)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *dst = (float)p;
}

template <int MODE>  // 1 acquire, 2 sc1
__device__ __forceinline__ void grid_barrier(const Args& a, unsigned target) {
  if (MODE == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (MODE == 1) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(a.ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int n = 0;
    while (__hip_atomic_load(a.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++n < kSpin)
      __builtin_amdgcn_s_sleep(1);
    if (n >= kSpin) atomicAdd(&a.err[1], 1);
    if (MODE == 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
  __syncthreads();
}

// MODE 0: one phase per launch (phase = a.phase0); 1 / 2: all phases in one launch
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_phases(Args a) {
  if (blockIdx.x % 8) return;  // participants: one XCD
  const int b = blockIdx.x / 8;
  if (threadIdx.x == 0 && a.phase0 == 0) a.xcc[b] = xcc_id();
  if (MODE == 0) {
    phase_work<false>(a, b, a.phase0);
    return;
  }
  for (int p = 0; p < a.phases; ++p) {
    phase_work<MODE == 2>(a, b, p);
    grid_barrier<MODE>(a, (unsigned)(p + 1) * a.G);
  }
}

static float time_mode(int mode, int G, int P, Args a, hipStream_t st) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipMemsetAsync(a.ctr, 0, sizeof(unsigned), st));
    hipGraphExec_t exec = nullptr;
    if (mode == 0) {  // P dependent launches in one graph
      hipGraph_t g;
      CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      for (int p = 0; p < P; ++p) {
        Args ap = a;
        ap.phase0 = p;
        hipLaunchKernelGGL(k_phases<0>, dim3(8 * G), dim3(kThreads), 0, st, ap);
      }
      CHECK(hipStreamEndCapture(st, &g));
      CHECK(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0));
      CHECK(hipGraphDestroy(g));
      CHECK(hipGraphLaunch(exec, st));  // warm
      CHECK(hipStreamSynchronize(st));
    }
    CHECK(hipEventRecord(e0, st));
    if (mode == 0) {
      CHECK(hipGraphLaunch(exec, st));
    } else {
      a.phases = P;
      a.phase0 = 0;
      if (mode == 1) hipLaunchKernelGGL(k_phases<1>, dim3(8 * G), dim3(kThreads), 0, st, a);
      else hipLaunchKernelGGL(k_phases<2>, dim3(8 * G), dim3(kThreads), 0, st, a);
    }
    CHECK(hipEventRecord(e1, st));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
    if (exec) CHECK(hipGraphExecDestroy(exec));
  }
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return best * 1e3f;  // us
}

int main() {
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Args a{};
  CHECK(hipMalloc(&a.rec, sizeof(float) * 2 * 32 * kThreads));
  CHECK(hipMalloc(&a.ctr, 256));
  CHECK(hipMalloc(&a.err, sizeof(int) * 2));
  CHECK(hipMalloc(&a.xcc, sizeof(unsigned) * 32));
  const char* names[3] = {"launch", "acquire", "sc1"};
  for (int G : {8, 16, 32}) {
    a.G = G;
    for (int mode = 0; mode < 3; ++mode) {
      CHECK(hipMemset(a.err, 0, sizeof(int) * 2));
      CHECK(hipMemset(a.rec, 0, sizeof(float) * 2 * 32 * kThreads));
      const int P1 = 8, P2 = 72;
      const float t1 = time_mode(mode, G, P1, a, st), t2 = time_mode(mode, G, P2, a, st);
      int err[2];
      std::vector<unsigned> x(G);
      CHECK(hipMemcpy(err, a.err, sizeof(err), hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(x.data(), a.xcc, sizeof(unsigned) * G, hipMemcpyDeviceToHost));
      bool one_xcd = true;
      for (int b = 1; b < G; ++b) one_xcd = one_xcd && x[b] == x[0];
      printf("{\"variant\": \"%s\", \"G\": %d, \"per_phase_us\": %.3f, \"t_%d_phases_us\": %.2f, "
             "\"t_%d_phases_us\": %.2f, \"wrong_values\": %d, \"expired_spins\": %d, \"one_xcd\": %s}\n",
             names[mode], G, (t2 - t1) / (P2 - P1), P1, t1, P2, t2, err[0], err[1], one_xcd ? "true" : "false");
      fflush(stdout);
      if (err[1]) return 3;  // a barrier did not complete: stop
    }
  }
  return 0;
}
