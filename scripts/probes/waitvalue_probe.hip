// waitvalue_probe.hip -- can a flag that a running kernel raises early start a copy-engine transfer
// while that kernel still holds every CU?  Diagnostic for the N > 1 exchange.
// "busy" is held like merson_pair (512 threads, ~150 KiB LDS, 256 VGPRs: one workgroup per CU);
// its workgroup 0 raises a flag right at its start.  A second stream waits for the flag
// (hipStreamWaitValue32/64), then runs an 8-byte copy-engine copy and an event: if the wait is a
// command-processor packet, the event lands right after busy starts; if it is a kernel, it lands
// when busy ends (no CU slot before).  Flag memory: uncached device, coarse device, pinned host.
//   hipcc --offload-arch=gfx950 -O3 waitvalue_probe.hip -o waitvalue_probe && ./waitvalue_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(512) void busy(const double* __restrict__ in, double* __restrict__ out, long n_per_wg,
                                            int reps, unsigned int* f32, unsigned long long* f64, unsigned long long v)
{
  extern __shared__ double lds[];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (f32) __hip_atomic_store(f32, (unsigned int)v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    if (f64) __hip_atomic_store(f64, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const long base = blockIdx.x * n_per_wg;
  double s = 0.0;
  for (int r = 0; r < reps; ++r)
    for (long i = threadIdx.x; i < n_per_wg; i += 512) s += in[base + i] * 1.0000001;
  asm volatile("" ::: "v255");
  lds[threadIdx.x] = s;
  __syncthreads();
  out[blockIdx.x * 512 + threadIdx.x] = lds[(threadIdx.x + 1) & 511];
}

static double ms(hipEvent_t a, hipEvent_t b)
{
  float t = 0;
  (void)hipEventElapsedTime(&t, a, b);
  return t;
}

int main()
{
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t lds_bytes = 150 * 1024;
  CHK(hipFuncSetAttribute((const void*)busy, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
  const int nwg = ncu;
  const long n_per_wg = 1L << 16;
  double *in, *out, *cs, *cd;
  CHK(hipMalloc(&in, sizeof(double) * n_per_wg * nwg));
  CHK(hipMemset(in, 0, sizeof(double) * n_per_wg * nwg));
  CHK(hipMalloc(&out, sizeof(double) * 512 * nwg));
  CHK(hipMalloc(&cs, 1 << 20));
  CHK(hipMalloc(&cd, 1 << 20));
  void* mem[3];
  CHK(hipExtMallocWithFlags(&mem[0], 4096, hipDeviceMallocUncached));
  CHK(hipMalloc(&mem[1], 4096));
  CHK(hipHostMalloc(&mem[2], 4096, hipHostMallocMapped | hipHostMallocCoherent));
  const char* mname[3] = {"uncached device", "coarse device", "pinned host"};
  hipStream_t sA, sC;
  CHK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
  CHK(hipStreamCreateWithFlags(&sC, hipStreamNonBlocking));
  hipEvent_t a0, a1, c1;
  CHK(hipEventCreate(&a0)); CHK(hipEventCreate(&a1)); CHK(hipEventCreate(&c1));
  const int reps = 16;
  for (int w = 0; w < 3; ++w) busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps, nullptr, nullptr, 0);
  CHK(hipDeviceSynchronize());
  unsigned long long v = 0;
  for (int m = 0; m < 3; ++m) {
    for (int wide = 0; wide < 2; ++wide) {
      for (int rep = 0; rep < 3; ++rep) {
        ++v;
        void* dp = mem[m];
        if (m == 2) CHK(hipHostGetDevicePointer(&dp, mem[m], 0));
        unsigned int* f32 = wide ? nullptr : (unsigned int*)dp;
        unsigned long long* f64 = wide ? (unsigned long long*)dp : nullptr;
        CHK(hipEventRecord(a0, sA));
        busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps, f32, f64, v);
        CHK(hipEventRecord(a1, sA));
        if (wide) CHK(hipStreamWaitValue64(sC, mem[m], v, hipStreamWaitValueGte, ~0ULL));
        else CHK(hipStreamWaitValue32(sC, mem[m], (unsigned int)v, hipStreamWaitValueGte, ~0u));
        CHK(hipMemcpyAsync(cd, cs, 8, hipMemcpyDeviceToDeviceNoCU, sC));
        CHK(hipEventRecord(c1, sC));
        CHK(hipDeviceSynchronize());
        printf("%-16s wait%d: busy %.3f ms, copy after the wait done at %.3f ms\n", mname[m], wide ? 64 : 32,
               ms(a0, a1), ms(a0, c1));
      }
    }
  }
  // the cost of two satisfied waits between two short kernels: two hipStreamWaitValue64 against one
  // hipStreamBatchMemOp of two waits (the exchange's flags from below and from above)
  {
    unsigned long long* fl;
    CHK(hipExtMallocWithFlags((void**)&fl, 64, hipDeviceMallocUncached));
    unsigned long long ones[2] = {5, 5};
    CHK(hipMemcpy(fl, ones, 16, hipMemcpyHostToDevice));
    hipEvent_t b0, b1;
    CHK(hipEventCreate(&b0)); CHK(hipEventCreate(&b1));
    for (int how = 0; how < 3; ++how)
      for (int rep = 0; rep < 4; ++rep) {
        CHK(hipEventRecord(b0, sA));
        for (int it = 0; it < 20; ++it) {
          busy<<<64, 512, lds_bytes, sA>>>(in, out, 64, 1, nullptr, nullptr, 0);
          if (how == 1) {
            CHK(hipStreamWaitValue64(sA, fl, 5, hipStreamWaitValueGte, ~0ULL));
            CHK(hipStreamWaitValue64(sA, fl + 1, 5, hipStreamWaitValueGte, ~0ULL));
          } else if (how == 2) {
            hipStreamBatchMemOpParams op[2];
            memset(op, 0, sizeof(op));
            for (int i = 0; i < 2; ++i) {
              op[i].operation = hipStreamMemOpWaitValue64;
              op[i].waitValue.address = (hipDeviceptr_t)(fl + i);
              op[i].waitValue.value64 = 5;
              op[i].waitValue.flags = hipStreamWaitValueGte;
            }
            CHK(hipStreamBatchMemOp(sA, 2, op, 0));
          }
        }
        CHK(hipEventRecord(b1, sA));
        CHK(hipDeviceSynchronize());
        printf("20 short kernels %-26s: %.1f us per kernel\n", how == 0 ? "back to back" : how == 1 ? "+ two WaitValue64" :
               "+ one BatchMemOp of two waits", 1000.0 * ms(b0, b1) / 20);
      }
  }
  printf("done\n");
  return 0;
}
