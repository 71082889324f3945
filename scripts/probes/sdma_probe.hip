// sdma_probe.hip -- can the halo planes move on the copy engines (SDMA) while a pair-kernel-like
// launch holds every CU?  Diagnostic for the N > 1 transport.
// The "busy" kernel is held like merson_pair: 512 threads, ~150 KiB of dynamic LDS and 256 VGPRs
// (one workgroup per CU, no slot left for any other kernel), and streams ~1.2 GB through HBM.
// Measured, each against busy alone:
//   - 4 copies of 2 planes of a 400 x 400 field (2.56 MB each) as hipMemcpyDeviceToDeviceNoCU and
//     as hipMemcpyDeviceToDevice, alone and beside busy (completion time from busy's start)
//   - the same followed by a flag (hipStreamWriteValue64, or an 8-byte NoCU copy) that a third
//     stream waits on (hipStreamWaitValue64) before an event
//   - hipMemcpy2DAsync with the NoCU kind (one call for 2 fields at a field stride)
//   hipcc --offload-arch=gfx950 -O3 sdma_probe.hip -o sdma_probe && ./sdma_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(512) void busy(const double* __restrict__ in, double* __restrict__ out, long n_per_wg, int reps)
{
  extern __shared__ double lds[];
  const long base = blockIdx.x * n_per_wg;
  double s = 0.0;
  for (int r = 0; r < reps; ++r)
    for (long i = threadIdx.x; i < n_per_wg; i += 512) s += in[base + i] * 1.0000001;
  asm volatile("" ::: "v255");   // hold 256 VGPRs: 2 waves per SIMD
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
  int occ = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)busy, 512, lds_bytes));
  const int nwg = ncu * occ;
  const long n_per_wg = 1L << 16;  // 512 KB per workgroup and rep
  printf("CUs %d, busy occupancy %d/CU -> %d workgroups\n", ncu, occ, nwg);
  double *in, *out;
  CHK(hipMalloc(&in, sizeof(double) * n_per_wg * nwg));
  CHK(hipMemset(in, 0, sizeof(double) * n_per_wg * nwg));
  CHK(hipMalloc(&out, sizeof(double) * 512 * nwg));
  // a slab-like buffer: 3 fields at a field stride, 404 planes of 400 x 400
  const long plane = 400L * 400, fs = 404L * plane;
  double *src, *dst;
  CHK(hipMalloc(&src, sizeof(double) * 3 * fs));
  CHK(hipMalloc(&dst, sizeof(double) * 3 * fs));
  CHK(hipMemset(src, 0x3c, sizeof(double) * 3 * fs));
  CHK(hipMemset(dst, 0, sizeof(double) * 3 * fs));
  unsigned long long* flag;
  CHK(hipExtMallocWithFlags((void**)&flag, 64, hipDeviceMallocUncached));
  CHK(hipMemset(flag, 0, 64));
  unsigned long long* seqdev;   // device words holding 1..1024: an 8-byte copy raises the flag
  CHK(hipMalloc(&seqdev, 8 * 1024));
  {
    unsigned long long h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = i + 1;
    CHK(hipMemcpy(seqdev, h, sizeof(h), hipMemcpyHostToDevice));
  }
  hipStream_t sA, sB, sC;
  int prio_lo = 0, prio_hi = 0;
  CHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  CHK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
  CHK(hipStreamCreateWithPriority(&sB, hipStreamNonBlocking, prio_hi));
  CHK(hipStreamCreateWithFlags(&sC, hipStreamNonBlocking));
  hipEvent_t a0, a1, b1, c1;
  CHK(hipEventCreate(&a0)); CHK(hipEventCreate(&a1)); CHK(hipEventCreate(&b1)); CHK(hipEventCreate(&c1));

  // 4 copies: fields 0,1 x (planes 1-2 -> planes n3+1..n3+2 ; planes n3-1..n3 -> planes -1..0)
  auto copies = [&](hipStream_t st, hipMemcpyKind kind) -> hipError_t {
    for (int f = 0; f < 2; ++f) {
      hipError_t e = hipMemcpyAsync(dst + f * fs + 402 * plane, src + f * fs + 2 * plane, 2 * plane * 8, kind, st);
      if (e != hipSuccess) return e;
      e = hipMemcpyAsync(dst + f * fs, src + f * fs + 400 * plane, 2 * plane * 8, kind, st);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  };
  const int reps = 16;
  unsigned long long seq = 0;
  for (int w = 0; w < 3; ++w) {
    busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps);
    CHK(copies(sB, hipMemcpyDeviceToDeviceNoCU));
    CHK(copies(sB, hipMemcpyDeviceToDevice));
  }
  CHK(hipDeviceSynchronize());
  for (int rep = 0; rep < 3; ++rep) {
    CHK(hipEventRecord(a0, sA));
    busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps);
    CHK(hipEventRecord(a1, sA));
    CHK(hipDeviceSynchronize());
    printf("busy alone: %.3f ms (%.0f GB/s)\n", ms(a0, a1), 8.0 * n_per_wg * nwg * reps / ms(a0, a1) / 1e6);
  }
  for (int kind = 0; kind < 2; ++kind) {
    const hipMemcpyKind k = kind ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToDeviceNoCU;
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(a0, sB));
      CHK(copies(sB, k));
      CHK(hipEventRecord(b1, sB));
      CHK(hipDeviceSynchronize());
      printf("%-6s copies alone: %.3f ms (%.1f GB/s)\n", kind ? "D2D" : "NoCU", ms(a0, b1), 4 * 2 * plane * 8 / ms(a0, b1) / 1e6);
    }
  }
  // beside busy: the copies become ready right after busy starts
  for (int kind = 0; kind < 2; ++kind) {
    const hipMemcpyKind k = kind ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToDeviceNoCU;
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(a0, sA));
      busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps);
      CHK(hipEventRecord(a1, sA));
      CHK(hipStreamWaitEvent(sB, a0, 0));
      CHK(copies(sB, k));
      CHK(hipEventRecord(b1, sB));
      CHK(hipDeviceSynchronize());
      printf("%-6s beside busy: busy %.3f ms, copies done at %.3f ms\n", kind ? "D2D" : "NoCU", ms(a0, a1), ms(a0, b1));
    }
  }
  // flags: NoCU copies, then a flag on sB; sC waits for it, then records c1
  for (int how = 0; how < 2; ++how) {
    for (int rep = 0; rep < 3; ++rep) {
      ++seq;
      CHK(hipEventRecord(a0, sA));
      busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps);
      CHK(hipEventRecord(a1, sA));
      CHK(hipStreamWaitEvent(sB, a0, 0));
      CHK(copies(sB, hipMemcpyDeviceToDeviceNoCU));
      if (how == 0) CHK(hipStreamWriteValue64(sB, flag, seq, 0));
      else CHK(hipMemcpyAsync(flag, seqdev + (seq - 1), 8, hipMemcpyDeviceToDeviceNoCU, sB));
      CHK(hipEventRecord(b1, sB));
      CHK(hipStreamWaitValue64(sC, flag, seq, hipStreamWaitValueGte, ~0ULL));
      CHK(hipEventRecord(c1, sC));
      CHK(hipDeviceSynchronize());
      printf("flag by %-14s: busy %.3f ms, copies+flag done at %.3f ms, waiter released at %.3f ms\n",
             how ? "NoCU 8-B copy" : "WriteValue64", ms(a0, a1), ms(a0, b1), ms(a0, c1));
    }
  }
  // 2D copy with the NoCU kind: 2 fields at stride fs in one call
  {
    CHK(hipMemset(dst, 0, sizeof(double) * 3 * fs));
    hipError_t e = hipMemcpy2DAsync(dst + 402 * plane, fs * 8, src + 2 * plane, fs * 8, 2 * plane * 8, 2,
                                    hipMemcpyDeviceToDeviceNoCU, sB);
    printf("hipMemcpy2DAsync NoCU: %s\n", hipGetErrorString(e));
    CHK(hipDeviceSynchronize());
    double h[2];
    CHK(hipMemcpy(&h[0], dst + 402 * plane + 5, 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&h[1], dst + fs + 403 * plane + 7, 8, hipMemcpyDeviceToHost));
    double want;
    memset(&want, 0x3c, 8);
    printf("  2D result %s\n", (h[0] == want && h[1] == want) ? "correct" : "WRONG");
    for (int rep = 0; rep < 3; ++rep) {
      CHK(hipEventRecord(a0, sA));
      busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps);
      CHK(hipEventRecord(a1, sA));
      CHK(hipStreamWaitEvent(sB, a0, 0));
      CHK(hipMemcpy2DAsync(dst + 402 * plane, fs * 8, src + 2 * plane, fs * 8, 2 * plane * 8, 2, hipMemcpyDeviceToDeviceNoCU, sB));
      CHK(hipMemcpy2DAsync(dst, fs * 8, src + 400 * plane, fs * 8, 2 * plane * 8, 2, hipMemcpyDeviceToDeviceNoCU, sB));
      CHK(hipEventRecord(b1, sB));
      CHK(hipDeviceSynchronize());
      printf("2D NoCU beside busy: busy %.3f ms, copies done at %.3f ms\n", ms(a0, a1), ms(a0, b1));
    }
  }
  // correctness of the 1D NoCU copies (the fill ordered on the copy's own stream)
  {
    CHK(hipMemsetAsync(dst, 0, sizeof(double) * 3 * fs, sB));
    CHK(copies(sB, hipMemcpyDeviceToDeviceNoCU));
    CHK(hipDeviceSynchronize());
    double h[4];
    CHK(hipMemcpy(&h[0], dst + 402 * plane, 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&h[1], dst + fs + 403 * plane + plane - 1, 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&h[2], dst, 8, hipMemcpyDeviceToHost));
    CHK(hipMemcpy(&h[3], dst + fs + 2 * plane - 1, 8, hipMemcpyDeviceToHost));
    double want;
    memset(&want, 0x3c, 8);
    printf("1D NoCU result %s (%a %a %a %a, want %a)\n", (h[0] == want && h[1] == want && h[2] == want && h[3] == want) ? "correct" : "WRONG",
           h[0], h[1], h[2], h[3], want);
  }
  // the four copies on four streams (one SDMA queue each?), and eight half-copies on eight streams
  {
    hipStream_t ss[8];
    for (int i = 0; i < 8; ++i) CHK(hipStreamCreateWithFlags(&ss[i], hipStreamNonBlocking));
    hipEvent_t e8[8];
    for (int i = 0; i < 8; ++i) CHK(hipEventCreate(&e8[i]));
    for (int nst = 2; nst <= 8; nst *= 2) {
      const int pieces = nst < 4 ? 4 : nst;           // 4 copies, or 8 halves
      const long len = (pieces == 8 ? plane : 2 * plane);
      for (int besides = 0; besides < 2; ++besides)
        for (int rep = 0; rep < 3; ++rep) {
          CHK(hipEventRecord(a0, sA));
          if (besides) busy<<<nwg, 512, lds_bytes, sA>>>(in, out, n_per_wg, reps);
          CHK(hipEventRecord(a1, sA));
          for (int c = 0; c < pieces; ++c) {
            hipStream_t st = ss[c % nst];
            CHK(hipStreamWaitEvent(st, a0, 0));
            const int f = (c / (pieces / 2)) & 1, half = c % (pieces / 2);
            CHK(hipMemcpyAsync(dst + f * fs + 402 * plane + half * len, src + f * fs + 2 * plane + half * len, len * 8,
                               hipMemcpyDeviceToDeviceNoCU, st));
          }
          for (int i = 0; i < nst; ++i) CHK(hipEventRecord(e8[i], ss[i]));
          CHK(hipDeviceSynchronize());
          double last = 0;
          for (int i = 0; i < nst; ++i) last = ms(a0, e8[i]) > last ? ms(a0, e8[i]) : last;
          printf("NoCU %d pieces on %d streams %s: busy %.3f ms, copies done at %.3f ms (%.1f GB/s)\n", pieces, nst,
                 besides ? "beside busy" : "alone", ms(a0, a1), last, pieces * len * 8 / last / 1e6);
        }
    }
  }
  printf("done\n");
  return 0;
}
