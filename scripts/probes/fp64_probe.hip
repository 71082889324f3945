// fp64_probe.hip -- FP64 vector issue on MI355X (diagnostic, not part of libpft): throughput of
// v_add_f64 / v_mul_f64 / correctly rounded division / sqrt chains per SIMD, as a function of
// independent chains per wave (ILP) and waves per SIMD (occupancy).  Every CU gets W waves per
// SIMD (workgroups of 64 W threads pinned one per CU by their LDS); each lane runs C independent
// chains of N dependent operations.  Prints the SIMD cycles per wave instruction (4.0 = the FP64
// pipe never idles) from the kernel time and the clock measured in-kernel (s_memtime).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off fp64_probe.hip -o fp64_probe && ./fp64_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)
#pragma clang fp contract(off)

enum { ADD = 0, MUL = 1, DIV = 2, SQRT = 3, DIVC = 4 };

template <int OP, int C>
__global__ void chains(double* out, int n, double a, double b, unsigned long long* clk)
{
  __shared__ double pin[16384];   // 128 KiB: one workgroup per CU
  double v[C];
#pragma unroll
  for (int c = 0; c < C; ++c) v[c] = 1.0 + 1e-3 * (threadIdx.x + c);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 16
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (OP == ADD) v[c] = v[c] + a;
      else if (OP == MUL) v[c] = v[c] * b;
      else if (OP == DIV) v[c] = a / v[c];          // a per-lane divisor: the full sequence
      else if (OP == DIVC) v[c] = v[c] / b;         // a uniform divisor
      else v[c] = sqrt(v[c] + a);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < C; ++c) s += v[c];
  if (s == 12345.678) pin[threadIdx.x] = s;         // never: keeps the LDS allocation
  out[blockIdx.x * blockDim.x + threadIdx.x] = s + pin[0] * 0.0;
  if (threadIdx.x == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = r1 - r0; }
}

template <int OP, int C>
static void run(const char* name, int waves, int ncu, double* out, unsigned long long* clk)
{
  const int n = 16384;
  const int threads = 64 * 4 * waves;                // W waves on each of the 4 SIMDs
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  chains<OP, C><<<ncu, threads>>>(out, 16, 0.5, 0.999, clk);   // warm
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(e0));
  chains<OP, C><<<ncu, threads>>>(out, n, 0.5, 0.999, clk);
  CHK(hipEventRecord(e1));
  CHK(hipEventSynchronize(e1));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, e0, e1));
  unsigned long long hc[2];
  CHK(hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost));
  const double ghz = (double)hc[0] / ((double)hc[1] / 100e6) / 1e9;   // s_memrealtime: 100 MHz
  // per SIMD: waves * C * n operations issued, in (ms * ghz) cycles
  const double cyc = ms * 1e-3 * ghz * 1e9 / ((double)waves * C * n);
  printf("%-5s waves/SIMD %d  chains %d : %7.3f ms  clock %.2f GHz  %6.2f SIMD cycles per wave-op\n", name, waves,
         C, ms, ghz, cyc);
  CHK(hipEventDestroy(e0));
  CHK(hipEventDestroy(e1));
}

template <int OP>
static void sweep(const char* name, int ncu, double* out, unsigned long long* clk)
{
  for (int w = 1; w <= 4; w *= 2) {
    run<OP, 1>(name, w, ncu, out, clk);
    run<OP, 2>(name, w, ncu, out, clk);
    run<OP, 4>(name, w, ncu, out, clk);
  }
}

int main()
{
  int dev = 0, ncu = 0;
  CHK(hipGetDevice(&dev));
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  double* out;
  unsigned long long* clk;
  CHK(hipMalloc(&out, (size_t)ncu * 1024 * sizeof(double)));
  CHK(hipMalloc(&clk, 2 * sizeof(unsigned long long)));
  printf("CUs %d\n", ncu);
  sweep<ADD>("add", ncu, out, clk);
  sweep<MUL>("mul", ncu, out, clk);
  sweep<DIV>("div", ncu, out, clk);
  sweep<DIVC>("divc", ncu, out, clk);
  sweep<SQRT>("sqrt", ncu, out, clk);
  return 0;
}
