// Modes 0 / 1 (round 5): is a / b == fma(fma(-q0, b, a), y, q0) with y = 1 / b, q0 = a * y (all
// IEEE fp32, RN) for every input the normalisation sees?  (Markstein: with y = RN(1/b) one fma
// correction step gives RN(a/b) outside the subnormal range.)  It is not: rejected.
// Mode 2 (round 6): the engine's fast division (kernels/k_base.h normalize_s: the compiler's own
// sequence with the reciprocal shared and the v_div_scale / v_div_fmas / v_div_fixup identities
// dropped, taken only where div_fast_ok) against a / b, on random pairs inside the fast range and
// on its boundaries.  Counts bitwise mismatches on the GPU.
//   hipcc --offload-arch=gfx950 -O3 tools/div_check.hip -o /tmp/div_check && /tmp/div_check
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ float fin(uint32_t u) {  // a finite float from random bits
  float f = __uint_as_float(u);
  return isfinite(f) ? f : __uint_as_float(u & 0xbf7fffffu);
}
__device__ __forceinline__ float div_shared(float n, float d, float r) {
#pragma clang fp contract(off)
  float q = n * r;
  float x = __builtin_fmaf(-d, q, n);
  q = __builtin_fmaf(x, r, q);
  x = __builtin_fmaf(-d, q, n);
  return __builtin_fmaf(x, r, q);
}
__device__ __forceinline__ float div_recip(float d) {
  const float r0 = __builtin_amdgcn_rcpf(d);
  return __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
}
__global__ void k_check(uint64_t seed, int mode, unsigned long long* bad, unsigned long long* sub, float* ex) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float a = fin(mix(seed * 0x9e3779b97f4a7c15ULL + 2 * i));
  float b = fin(mix(seed * 0x9e3779b97f4a7c15ULL + 2 * i + 1));
  if (mode == 1) {  // the normalisation's case: |a| <= b, b > 0 normal
    b = fabsf(b);
    if (b < 1e-30f || b > 1e30f) b = 1.f + (float)(i & 1023) * 0.37f;
    a = fmodf(a, b);
  }
  if (mode == 2) {  // the fast range: b in [2^-40, 2^40], |a| in [2^-80, b]; boundaries for i % 8 < 2
    const uint32_t u = mix(seed * 0x51ed2701ULL + i);
    b = ldexpf(1.f + (u & 0xffff) / 65536.f, (int)(u >> 16) % 81 - 40);
    if ((i & 7) == 0) b = (u & 1) ? 0x1p-40f : 0x1p40f;
    b = fminf(fmaxf(b, 0x1p-40f), 0x1p40f);
    const float m = ldexpf(1.f + (mix(i * 7 + seed) & 0xffff) / 65536.f, -(int)(mix(i + 3 * seed) % 120));
    a = fminf(m * b, b);
    if ((i & 7) == 1) a = 0x1p-80f;
    if (fabsf(a) < 0x1p-80f) a = 0x1p-80f;
    if (u & 2) a = -a;
    const float q = a / b;
    const float q2 = div_shared(a, b, div_recip(b));
    if (__float_as_uint(q) != __float_as_uint(q2)) {
      atomicAdd(bad, 1ull);
      ex[0] = a; ex[1] = b; ex[2] = q; ex[3] = q2;
    }
    return;
  }
  if (b == 0.f) return;
  const float q = a / b;
  const float y = 1.f / b;
  const float q0 = a * y;
  const float r = fmaf(-q0, b, a);
  const float q1 = fmaf(r, y, q0);
  const bool same = __float_as_uint(q) == __float_as_uint(q1) || (q != q && q1 != q1);
  if (!same) {
    const bool subn = fabsf(q) < 1.17549435e-38f;
    atomicAdd(subn ? sub : bad, 1ull);
    if (!subn) { ex[0] = a; ex[1] = b; ex[2] = q; ex[3] = q1; }
  }
}
int main() {
  unsigned long long *bad, *sub;
  float* ex;
  hipMalloc(&bad, 8); hipMalloc(&sub, 8); hipMalloc(&ex, 16);
  for (int mode = 0; mode < 3; ++mode) {
    hipMemset(bad, 0, 8); hipMemset(sub, 0, 8); hipMemset(ex, 0, 16);
    const int blocks = 1 << 20, rounds = 16;
    for (int s = 0; s < rounds; ++s) hipLaunchKernelGGL(k_check, dim3(blocks), dim3(256), 0, 0, (uint64_t)(s + 1 + 100 * mode), mode, bad, sub, ex);
    unsigned long long hb = 0, hs = 0; float he[4];
    hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(&hs, sub, 8, hipMemcpyDeviceToHost);
    hipMemcpy(he, ex, 16, hipMemcpyDeviceToHost);
    printf("mode %d (%s): %.3g pairs, mismatches normal range %llu, subnormal quotients %llu; example %a / %a = %a vs %a\n",
           mode, mode == 2 ? "fast division range, shared reciprocal" : mode ? "|a| <= b" : "any finite", (double)blocks * 256 * rounds, hb, hs, he[0], he[1], he[2], he[3]);
  }
  return 0;
}
