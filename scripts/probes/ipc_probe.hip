// ipc_probe.hip -- can two processes on one GPU (or on two GPUs of a node) exchange halo planes
// through IPC-mapped device memory and order their streams with memory flags?  Diagnostic for the
// "ipc" transport of pft_comm.hip.
//   hipcc --offload-arch=gfx950 -O3 ipc_probe.hip -o ipc_probe
//   ./ipc_probe 0 DIR & ./ipc_probe 1 DIR & wait     (DIR: an empty directory for the handles)
// Each rank allocates a buffer (data + 64 flag words) and exports it; rank r opens rank 1-r's.
// Test 1: a kernel writes a pattern into the peer's buffer, then a system-scope release store of
//         the peer's flag; the peer's stream waits on its own flag (hipStreamWaitValue64) and a
//         kernel checks the pattern.
// Test 2: ping-pong of N flag hops (kernel signal -> stream wait), per-hop latency.
// Test 3: the same with hipStreamWriteValue64 to the peer's flag instead of a kernel.
// Test 4: an interprocess event handle can be created.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("rank %d: %s: %s\n", rank, #x, hipGetErrorString(e)); fflush(stdout); return 1; } } while (0)

static int rank;

__global__ void put_pattern(double* peer, long n, double base, unsigned long long* peer_flag, unsigned long long v,
                            unsigned int* done, unsigned int nblocks)
{
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    peer[i] = base + (double)i;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned int prev = atomicAdd(done, 1u);
    if (prev == nblocks - 1) {
      *done = 0;
      __threadfence_system();
      __hip_atomic_store(peer_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void check_pattern(const double* mine, long n, double base, unsigned int* bad)
{
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    if (mine[i] != base + (double)i) atomicAdd(bad, 1u);
}

__global__ void signal1(unsigned long long* peer_flag, unsigned long long v)
{
  __threadfence_system();
  __hip_atomic_store(peer_flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now()
{
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + 1e-9 * t.tv_nsec;
}

static int wait_file(const char* p, double tmax)
{
  const double t0 = now();
  struct stat st;
  while (stat(p, &st) != 0 || st.st_size == 0) {
    if (now() - t0 > tmax) return 1;
    usleep(1000);
  }
  return 0;
}

int main(int argc, char** argv)
{
  if (argc < 3) return 2;
  rank = atoi(argv[1]);
  const char* dir = argv[2];
  const int dev = argc > 3 ? atoi(argv[3]) : 0;
  const int peer = 1 - rank;
  CHK(hipSetDevice(dev));
  int can_wait = -1;
  CHK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, dev));
  printf("rank %d: device %d CanUseStreamWaitValue = %d\n", rank, dev, can_wait);

  const long n = 1L << 20;   // 8 MB of data
  const size_t bytes = sizeof(double) * n + 64 * 8;
  char* buf;
  CHK(hipMalloc(&buf, bytes));
  CHK(hipMemset(buf, 0, bytes));
  unsigned long long* flags = (unsigned long long*)(buf + sizeof(double) * n);
  unsigned int *done, *bad;
  CHK(hipMalloc(&done, 64));
  CHK(hipMemset(done, 0, 64));
  CHK(hipMalloc(&bad, 64));
  CHK(hipMemset(bad, 0, 64));
  CHK(hipDeviceSynchronize());

  hipIpcMemHandle_t h;
  CHK(hipIpcGetMemHandle(&h, buf));
  char path[512], tmp[512];
  snprintf(tmp, sizeof tmp, "%s/h%d.tmp", dir, rank);
  snprintf(path, sizeof path, "%s/h%d", dir, rank);
  FILE* f = fopen(tmp, "wb");
  fwrite(&h, sizeof h, 1, f);
  fclose(f);
  rename(tmp, path);
  snprintf(path, sizeof path, "%s/h%d", dir, peer);
  if (wait_file(path, 30.0)) { printf("rank %d: no peer handle\n", rank); return 1; }
  hipIpcMemHandle_t ph;
  f = fopen(path, "rb");
  if (fread(&ph, sizeof ph, 1, f) != 1) { printf("rank %d: short handle\n", rank); return 1; }
  fclose(f);
  char* pbuf = nullptr;
  CHK(hipIpcOpenMemHandle((void**)&pbuf, ph, hipIpcMemLazyEnablePeerAccess));
  unsigned long long* pflags = (unsigned long long*)(pbuf + sizeof(double) * n);
  printf("rank %d: opened peer buffer\n", rank);
  fflush(stdout);

  hipStream_t st;
  CHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));

  // test 1: data + flag (flag word 0)
  double t0 = now();
  hipLaunchKernelGGL(put_pattern, dim3(256), dim3(256), 0, st, (double*)pbuf, n, 1000.0 * (rank + 1), pflags, 1ULL,
                     done, 256u);
  CHK(hipGetLastError());
  CHK(hipStreamWaitValue64(st, flags, 1ULL, hipStreamWaitValueGte, ~0ULL));
  hipLaunchKernelGGL(check_pattern, dim3(256), dim3(256), 0, st, (const double*)buf, n, 1000.0 * (peer + 1), bad);
  CHK(hipStreamSynchronize(st));
  unsigned int hbad = 0;
  CHK(hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost));
  printf("rank %d: test1 data via peer write + flag: %s (%u bad) %.3f ms\n", rank, hbad ? "FAIL" : "ok", hbad,
         1e3 * (now() - t0));
  fflush(stdout);

  // test 2: ping-pong of flag hops through kernels (flag word 1), rank 0 starts
  const int N = 2000;
  t0 = now();
  for (int i = 1; i <= N; ++i) {
    if (rank == 0) {
      hipLaunchKernelGGL(signal1, dim3(1), dim3(1), 0, st, pflags + 1, (unsigned long long)i);
      CHK(hipStreamWaitValue64(st, flags + 1, (unsigned long long)i, hipStreamWaitValueGte, ~0ULL));
    } else {
      CHK(hipStreamWaitValue64(st, flags + 1, (unsigned long long)i, hipStreamWaitValueGte, ~0ULL));
      hipLaunchKernelGGL(signal1, dim3(1), dim3(1), 0, st, pflags + 1, (unsigned long long)i);
    }
  }
  const double tq = now() - t0;
  CHK(hipStreamSynchronize(st));
  double dt = now() - t0;
  printf("rank %d: test2 kernel-signal ping-pong: %d round trips in %.3f ms = %.2f us per round trip (enqueue %.3f ms)\n",
         rank, N, 1e3 * dt, 1e6 * dt / N, 1e3 * tq);
  fflush(stdout);

  // test 3: hipStreamWriteValue64 to the peer's flag (flag word 2)
  t0 = now();
  hipError_t e3 = hipSuccess;
  for (int i = 1; i <= N && e3 == hipSuccess; ++i) {
    if (rank == 0) {
      e3 = hipStreamWriteValue64(st, pflags + 2, (unsigned long long)i, 0);
      if (e3 == hipSuccess) e3 = hipStreamWaitValue64(st, flags + 2, (unsigned long long)i, hipStreamWaitValueGte, ~0ULL);
    } else {
      e3 = hipStreamWaitValue64(st, flags + 2, (unsigned long long)i, hipStreamWaitValueGte, ~0ULL);
      if (e3 == hipSuccess) e3 = hipStreamWriteValue64(st, pflags + 2, (unsigned long long)i, 0);
    }
  }
  if (e3 != hipSuccess) {
    printf("rank %d: test3 WriteValue64 to the peer: %s (skipped)\n", rank, hipGetErrorString(e3));
    // unblock the peer
    hipLaunchKernelGGL(signal1, dim3(1), dim3(1), 0, st, pflags + 2, (unsigned long long)N);
  }
  CHK(hipStreamSynchronize(st));
  dt = now() - t0;
  if (e3 == hipSuccess)
    printf("rank %d: test3 WriteValue64 ping-pong: %.2f us per round trip\n", rank, 1e6 * dt / N);
  fflush(stdout);

  // test 4: interprocess event
  hipEvent_t ev;
  hipError_t e4 = hipEventCreateWithFlags(&ev, hipEventInterprocess | hipEventDisableTiming);
  hipIpcEventHandle_t eh;
  if (e4 == hipSuccess) e4 = hipIpcGetEventHandle(&eh, ev);
  printf("rank %d: test4 interprocess event handle: %s\n", rank, hipGetErrorString(e4));

  // local reference: one kernel hop inside one process (signal own flag, wait on it)
  t0 = now();
  for (int i = 1; i <= N; ++i) {
    hipLaunchKernelGGL(signal1, dim3(1), dim3(1), 0, st, flags + 3, (unsigned long long)i);
    CHK(hipStreamWaitValue64(st, flags + 3, (unsigned long long)i, hipStreamWaitValueGte, ~0ULL));
  }
  CHK(hipStreamSynchronize(st));
  dt = now() - t0;
  printf("rank %d: local kernel-signal + wait: %.2f us per pair\n", rank, 1e6 * dt / N);

  // final handshake so neither side unmaps while the other still writes
  hipLaunchKernelGGL(signal1, dim3(1), dim3(1), 0, st, pflags + 4, 1ULL);
  CHK(hipStreamWaitValue64(st, flags + 4, 1ULL, hipStreamWaitValueGte, ~0ULL));
  CHK(hipStreamSynchronize(st));
  CHK(hipIpcCloseMemHandle(pbuf));
  CHK(hipFree(buf));
  printf("rank %d: done\n", rank);
  return 0;
}
