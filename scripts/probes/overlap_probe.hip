// overlap_probe.hip -- does a small kernel on a second stream (the RCCL halo exchange) get CU
// slots while a stage kernel that fills every slot runs?  And what does reserving one CU per
// XCD (hipExtStreamCreateWithCUMask on the compute stream) cost the big kernel?  Diagnostic.
// The "exchange" is a real RCCL grouped send/recv (to itself, 1-rank communicator) of one
// 400 x 400 plane of 3 fields; the big kernel is held at 240 VGPRs (2 waves per SIMD), like stage 5.
//   hipcc --offload-arch=gfx950 -O3 overlap_probe.hip -o overlap_probe -lrccl && ./overlap_probe
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void busy(const double* __restrict__ in, double* __restrict__ out, long n_per_wg)
{
  __shared__ double lds[4096];   // 32 KB: a few workgroups per CU, like the stage kernels
  const long base = blockIdx.x * n_per_wg;
  double s = 0.0;
  for (long i = threadIdx.x; i < n_per_wg; i += 256) s += in[base + i];
  asm volatile("" ::: "v239");   // hold 240 VGPRs: 2 waves per SIMD, no room beside it
  lds[threadIdx.x] = s;
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = lds[(threadIdx.x + 1) & 255];
}

__global__ void tiny(double* p) { p[blockIdx.x * 64 + threadIdx.x] += 1.0; }

int main()
{
  int ncu = 0;
  CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  int occ = 0;
  CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, (const void*)busy, 256, 0));
  const int nwg = ncu * occ;
  const long n_per_wg = 1L << 17;   // 1 MB per workgroup
  double *in, *out, *t;
  CHK(hipMalloc(&in, sizeof(double) * n_per_wg * 2 * nwg));   // the two-round variants
  CHK(hipMemset(in, 0, sizeof(double) * n_per_wg * 2 * nwg));
  CHK(hipMalloc(&out, sizeof(double) * 256 * 2 * nwg));
  CHK(hipMalloc(&t, sizeof(double) * 64 * 64));
  printf("CUs %d, busy occupancy %d/CU -> %d workgroups, %.0f MB\n", ncu, occ, nwg, 8.0 * n_per_wg * nwg / 1e6);
  int prio_lo = 0, prio_hi = 0;
  CHK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  hipStream_t sA, sB, sH;
  CHK(hipStreamCreateWithFlags(&sA, hipStreamNonBlocking));
  CHK(hipStreamCreateWithFlags(&sB, hipStreamNonBlocking));
  CHK(hipStreamCreateWithPriority(&sH, hipStreamNonBlocking, prio_hi));
  printf("stream priorities: least %d greatest %d\n", prio_lo, prio_hi);
  ncclUniqueId id;
  ncclComm_t comm;
  if (ncclGetUniqueId(&id) != ncclSuccess || ncclCommInitRank(&comm, 1, id, 0) != ncclSuccess) { printf("rccl init failed\n"); return 1; }
  const size_t plane = 400 * 400 * 3;
  double *sb, *rb;
  CHK(hipMalloc(&sb, plane * 8)); CHK(hipMalloc(&rb, plane * 8));
  auto exchange = [&](hipStream_t st) {
    ncclGroupStart();
    ncclSend(sb, plane, ncclFloat64, 0, comm, st);
    ncclRecv(rb, plane, ncclFloat64, 0, comm, st);
    ncclGroupEnd();
  };
  hipEvent_t a0, a1, b0, b1;
  CHK(hipEventCreate(&a0)); CHK(hipEventCreate(&a1)); CHK(hipEventCreate(&b0)); CHK(hipEventCreate(&b1));
  for (int w = 0; w < 3; ++w) exchange(sB);
  CHK(hipDeviceSynchronize());
  CHK(hipEventRecord(b0, sB)); exchange(sB); CHK(hipEventRecord(b1, sB));
  CHK(hipDeviceSynchronize());
  float tx = 0; CHK(hipEventElapsedTime(&tx, b0, b1));
  printf("exchange alone: %.3f ms\n", tx);
  struct V { int nwg; int hi; int order; const char* what; };
  const V vs[] = {{nwg, 0, 0, "full one round, normal prio, busy first"},
                  {nwg - 16, 0, 0, "16 slots free, normal prio, busy first"},
                  {nwg - 128, 0, 0, "128 slots free, normal prio, busy first"},
                  {nwg / 2, 0, 0, "half the slots free, normal prio, busy first"},
                  {2 * nwg, 0, 0, "two rounds, normal prio, busy first"},
                  {nwg, 1, 0, "full one round, HIGH prio, busy first"},
                  {2 * nwg, 1, 0, "two rounds, HIGH prio, busy first"},
                  {nwg, 1, 1, "full one round, HIGH prio, exchange enqueued first behind an event"}};
  hipEvent_t gate;
  CHK(hipEventCreateWithFlags(&gate, hipEventDisableTiming));
  for (const V& v : vs) {
    if (v.nwg > 2 * nwg) return 2;
    hipStream_t sx = v.hi ? sH : sB;
    for (int rep = 0; rep < 3; ++rep) {
      busy<<<v.nwg, 256, 0, sA>>>(in, out, n_per_wg);
      CHK(hipDeviceSynchronize());
      if (v.order == 0) {
        CHK(hipEventRecord(a0, sA));
        busy<<<v.nwg, 256, 0, sA>>>(in, out, n_per_wg);
        CHK(hipEventRecord(a1, sA));
        exchange(sx);
        CHK(hipEventRecord(b1, sx));
      } else {
        // the solver's pattern: a small "boundary" kernel, then the exchange (waiting for it) and
        // the big interior kernel become ready at the same moment
        CHK(hipEventRecord(a0, sA));
        tiny<<<8, 64, 0, sA>>>(t);
        CHK(hipEventRecord(gate, sA));
        CHK(hipStreamWaitEvent(sx, gate, 0));
        exchange(sx);
        CHK(hipEventRecord(b1, sx));
        busy<<<v.nwg, 256, 0, sA>>>(in, out, n_per_wg);
        CHK(hipEventRecord(a1, sA));
      }
      CHK(hipDeviceSynchronize());
      float ta = 0, tb = 0;
      CHK(hipEventElapsedTime(&ta, a0, a1));
      CHK(hipEventElapsedTime(&tb, a0, b1));
      printf("%-70s busy %.3f ms, exchange done at %.3f ms\n", v.what, ta, tb);
    }
  }
  return 0;
}
