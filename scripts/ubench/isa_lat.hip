// Dependent-chain latency of a few gfx950 instruction patterns the chain kernels use, one
// wave alone on the GPU (s_memtime around 64 dependent copies).  Diagnostic only:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/isa_lat scripts/ubench/isa_lat.hip && /tmp/isa_lat
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__device__ __forceinline__ unsigned long long now() {
  unsigned long long t;
  asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__global__ void lat(unsigned long long* out, unsigned* sink, unsigned seed) {
  unsigned v = threadIdx.x + seed, w = seed * 3u;
  unsigned long long s64 = 0x123456789abcdefull ^ seed;
  unsigned long long t0, t1;
  int k = 0;
  // 0: v_add_u32 dependent chain
  t0 = now();
  asm volatile(REP64("v_add_u32 %0, %0, %1\n") : "+v"(v) : "v"(w));
  t1 = now(); out[k++] = t1 - t0;
  // 1: 64-bit shift (v_lshrrev_b64) dependent chain
  unsigned long long x64 = ((unsigned long long)v << 32) | w;
  t0 = now();
  asm volatile(REP64("v_lshrrev_b64 %0, 1, %0\n") : "+v"(x64));
  t1 = now(); out[k++] = t1 - t0;
  // 2: v_bfe_u32 chain
  t0 = now();
  asm volatile(REP64("v_bfe_u32 %0, %0, 1, 16\n") : "+v"(v));
  t1 = now(); out[k++] = t1 - t0;
  // 3: DPP row_shr add chain (with the 2-state DPP hazard nop)
  t0 = now();
  asm volatile(REP64("s_nop 1\n v_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n") : "+v"(v));
  t1 = now(); out[k++] = t1 - t0;
  // 4: ds_bpermute round trips
  unsigned a = (threadIdx.x ^ 1) << 2;
  t0 = now();
  for (int i = 0; i < 64; ++i) {
    v = __builtin_amdgcn_ds_bpermute((int)a, (int)v);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v));
  }
  t1 = now(); out[k++] = t1 - t0;
  // 5: ds_read_b32 round trips (LDS pointer chase)
  __shared__ unsigned lds[256];
  lds[threadIdx.x] = (threadIdx.x + 1) & 63;
  __syncthreads();
  unsigned p = threadIdx.x & 63;
  t0 = now();
  for (int i = 0; i < 64; ++i) {
    p = lds[p];
    asm volatile("" : "+v"(p));
  }
  t1 = now(); out[k++] = t1 - t0;
  // 6: ballot -> SALU -> VALU: v_cmp to SGPR pair, s_and, v_cndmask
  t0 = now();
  for (int i = 0; i < 64; ++i) {
    unsigned long long b;
    asm volatile("v_cmp_gt_u32 %0, %1, 7\n s_and_b64 %0, %0, %0\n v_cndmask_b32 %1, 0, %1, %0"
                 : "=s"(b), "+v"(v));
  }
  t1 = now(); out[k++] = t1 - t0;
  // 7: v_mad_u64_u32 chain
  unsigned long long m64 = v;
  t0 = now();
  asm volatile(REP64("v_mad_u64_u32 %0, s[0:1], %1, %1, %0\n") : "+v"(m64) : "v"(w) : "s0", "s1");
  t1 = now(); out[k++] = t1 - t0;
  // 8: v_readfirstlane -> s_add -> v_add chain (VALU -> SALU -> VALU)
  t0 = now();
  for (int i = 0; i < 64; ++i) {
    unsigned s;
    asm volatile("v_readfirstlane_b32 %0, %1\n s_add_u32 %0, %0, 1\n v_add_u32 %1, %0, %1" : "=s"(s), "+v"(v));
  }
  t1 = now(); out[k++] = t1 - t0;
  // 9: v_cndmask with VCC from v_cmp (VALU -> VCC -> VALU)
  t0 = now();
  asm volatile(REP64("v_cmp_gt_u32 vcc, %0, 7\n v_cndmask_b32 %0, 0, %0, vcc\n") : "+v"(v) :: "vcc");
  t1 = now(); out[k++] = t1 - t0;
  // 10: global load (L2-resident line) round trips
  t0 = now();
  for (int i = 0; i < 16; ++i) {
    v = __hip_atomic_load(sink + (v & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  t1 = now(); out[k++] = (t1 - t0) * 4;
  // 11: global atomic CAS round trips (agent scope)
  t0 = now();
  for (int i = 0; i < 16; ++i) {
    unsigned o = v & 1u;
    __hip_atomic_compare_exchange_strong(sink + 32 + threadIdx.x, &o, v, __ATOMIC_RELAXED,
                                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    v += o;
  }
  t1 = now(); out[k++] = (t1 - t0) * 4;
  // 12: permlane16_swap chain
  t0 = now();
  for (int i = 0; i < 64; ++i) {
    auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = r[0] + 1u;
  }
  t1 = now(); out[k++] = t1 - t0;
  // 13: v_readlane (uniform lane) -> VALU use
  t0 = now();
  for (int i = 0; i < 64; ++i) v = __builtin_amdgcn_readlane(v, 5) + threadIdx.x;
  t1 = now(); out[k++] = t1 - t0;
  sink[200 + threadIdx.x] = v + (unsigned)x64 + (unsigned)m64 + p + (unsigned)s64;
}

int main() {
  unsigned long long* out;
  unsigned* sink;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&sink, 4096);
  hipMemset(sink, 0, 4096);
  const char* names[] = {"v_add_u32", "v_lshrrev_b64", "v_bfe_u32", "dpp add (+s_nop 1)", "ds_bpermute trip",
                         "ds_read_b32 trip", "v_cmp->s_and->v_cndmask", "v_mad_u64_u32", "readfirstlane->s_add->v_add",
                         "v_cmp vcc->v_cndmask", "global load (L2) trip", "global CAS (agent) trip",
                         "permlane16_swap (+v_add)", "readlane->v_add"};
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(lat, dim3(1), dim3(64), 0, 0, out, sink, 7u + rep);
    hipDeviceSynchronize();
  }
  unsigned long long h[64];
  hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  printf("s_memtime ticks per dependent op (64 ops per row; trips x4 for the 16-op global rows)\n");
  for (int i = 0; i < 14; ++i) printf("%-30s %8.2f\n", names[i], h[i] / 64.0);
  return 0;
}
