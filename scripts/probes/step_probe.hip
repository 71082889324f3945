// Small-slab step structure on one MI355X (f4, configs[0] 100^3): what does a dependent kernel
// boundary cost, against a grid-wide barrier inside one persistent launch, and against a host
// round trip that a persistent launch waits for?  Each "phase" reads and writes one double pair per
// thread over G workgroups of 256 threads (about the footprint of one 100^3 stage: 512 x 256 pairs
// = 262 144 pairs).
//   chain  : K dependent launches on one stream (hipEvent over the whole chain) -> us per launch
//   coop   : one hipLaunchCooperativeKernel, K phases separated by cooperative_groups grid sync
//   bar    : one cooperative launch, K phases separated by a counter barrier (agent-scope
//            release/acquire atomics, one arrival per workgroup, bounded spin)
//   host   : one cooperative launch; per round, workgroup 0 publishes a word to pinned host
//            memory, the host answers in another pinned word, workgroup 0 polls it, then the
//            counter barrier releases every workgroup (the persistent step's host hand-off)
// Every spin is bounded (the kernel gives up and flags an error; the host checks the flag).
// hipcc --offload-arch=gfx950 -O3 -o step_probe step_probe.hip
#include <hip/hip_cooperative_groups.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

namespace cg = cooperative_groups;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));         \
      return 1;                                                                                 \
    }                                                                                           \
  } while (0)

typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void phase_work(const dbl2* __restrict__ in, dbl2* __restrict__ out, int p)
{
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  dbl2 v = in[i];
  v.x = v.x * 1.0000001 + (double)p;
  v.y = v.y * 0.9999999 - (double)p;
  out[i] = v;
}

__global__ __launch_bounds__(256) void k_phase(const dbl2* in, dbl2* out, int p) { phase_work(in, out, p); }

__global__ __launch_bounds__(256) void k_coop(dbl2* a, dbl2* b, int K)
{
  cg::grid_group g = cg::this_grid();
  for (int p = 0; p < K; ++p) {
    phase_work((p & 1) ? b : a, (p & 1) ? a : b, p);
    g.sync();
  }
}

#define SPIN_MAX (1L << 22)

// generation barrier: cnt counts arrivals of this generation; the last arrival resets it and bumps
// gen.  Returns false when the spin bound ran out (err set).
__device__ __forceinline__ bool bar_sync(unsigned* cnt, unsigned* gen, unsigned nb, unsigned* err)
{
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    const unsigned g0 = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // release: this workgroup's stores are visible agent-wide before it is counted
    if (__hip_atomic_fetch_add(cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == nb - 1) {
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      long it = 0;
      while (__hip_atomic_load(gen, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == g0) {
        if (++it > SPIN_MAX) {
          atomicOr(err, 1u);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  __syncthreads();
  return ok;
}

__global__ __launch_bounds__(256) void k_bar(dbl2* a, dbl2* b, int K, unsigned* cnt, unsigned* gen, unsigned* err)
{
  for (int p = 0; p < K; ++p) {
    phase_work((p & 1) ? b : a, (p & 1) ? a : b, p);
    if (!bar_sync(cnt, gen, gridDim.x, err)) return;
  }
}

// host round trip per phase: wg 0 publishes p + 1 to pub, waits for ans == p + 1, then barrier
__global__ __launch_bounds__(256) void k_host(dbl2* a, dbl2* b, int K, unsigned* cnt, unsigned* gen, unsigned* err,
                                              unsigned long long* pub, const unsigned long long* ans)
{
  for (int p = 0; p < K; ++p) {
    phase_work((p & 1) ? b : a, (p & 1) ? a : b, p);
    if (!bar_sync(cnt, gen, gridDim.x, err)) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      __hip_atomic_store(pub, (unsigned long long)(p + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      long it = 0;
      while (__hip_atomic_load(ans, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < (unsigned long long)(p + 1)) {
        if (++it > SPIN_MAX) {
          atomicOr(err, 2u);
          break;
        }
      }
    }
    if (!bar_sync(cnt, gen, gridDim.x, err)) return;
  }
}

static double now_us()
{
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main()
{
  int dev = 0, ncu = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int coop = 0;
  CK(hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev));
  int occ_coop = 0, occ_bar = 0;
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_coop, (const void*)k_coop, 256, 0));
  CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_bar, (const void*)k_bar, 256, 0));
  printf("CUs %d, cooperative launch %d, occupancy coop %d bar %d\n", ncu, coop, occ_coop, occ_bar);
  const int GMAX = 2048;
  dbl2 *a, *b;
  CK(hipMalloc((void**)&a, (size_t)GMAX * 256 * sizeof(dbl2)));
  CK(hipMalloc((void**)&b, (size_t)GMAX * 256 * sizeof(dbl2)));
  CK(hipMemset(a, 0, (size_t)GMAX * 256 * sizeof(dbl2)));
  CK(hipMemset(b, 0, (size_t)GMAX * 256 * sizeof(dbl2)));
  unsigned *cnt, *gen, *err;
  CK(hipMalloc((void**)&cnt, 256));
  CK(hipMalloc((void**)&gen, 256));
  CK(hipMalloc((void**)&err, 256));
  CK(hipMemset(cnt, 0, 256));
  CK(hipMemset(gen, 0, 256));
  CK(hipMemset(err, 0, 256));
  unsigned long long *pub, *ans;
  CK(hipHostMalloc((void**)&pub, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&ans, 64, hipHostMallocMapped | hipHostMallocCoherent));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int K = 400;
  for (int G : {256, 512, 1024}) {
    // warm the clock and the code
    for (int r = 0; r < 3000; ++r) k_phase<<<G, 256, 0, st>>>(a, b, r);
    CK(hipStreamSynchronize(st));
    float ms = 0;
    // chain
    CK(hipEventRecord(e0, st));
    for (int p = 0; p < K; ++p) k_phase<<<G, 256, 0, st>>>((p & 1) ? b : a, (p & 1) ? a : b, p);
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("G %5d  chain  %7.2f us per launch\n", G, 1000.0 * ms / K);
    const bool fits = G <= ncu * std::min(occ_coop, occ_bar);
    if (!coop || !fits) {
      printf("G %5d  (does not fit co-resident: skipped coop/bar/host)\n", G);
      continue;
    }
    // cooperative groups grid sync
    {
      int KK = K;
      void* args[] = {&a, &b, &KK};
      CK(hipEventRecord(e0, st));
      CK(hipLaunchCooperativeKernel((const void*)k_coop, dim3(G), dim3(256), args, 0, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("G %5d  coop   %7.2f us per phase\n", G, 1000.0 * ms / K);
    }
    // counter barrier
    {
      int KK = K;
      void* args[] = {&a, &b, &KK, &cnt, &gen, &err};
      CK(hipEventRecord(e0, st));
      CK(hipLaunchCooperativeKernel((const void*)k_bar, dim3(G), dim3(256), args, 0, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned herr = 0;
      CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      printf("G %5d  bar    %7.2f us per phase (err %u)\n", G, 1000.0 * ms / K, herr);
    }
    // host round trip
    {
      *pub = 0;
      *ans = 0;
      int KK = K;
      void* args[] = {&a, &b, &KK, &cnt, &gen, &err, &pub, &ans};
      const double t0 = now_us();
      CK(hipLaunchCooperativeKernel((const void*)k_host, dim3(G), dim3(256), args, 0, st));
      bool to = false;
      std::vector<double> rt;
      double tl = now_us();
      for (int p = 1; p <= K && !to; ++p) {
        const double ts = now_us();
        while (__atomic_load_n(pub, __ATOMIC_ACQUIRE) < (unsigned long long)p) {
          if (now_us() - ts > 2e6) { to = true; break; }
        }
        const double tn = now_us();
        if (p > 1) rt.push_back(tn - tl);
        tl = tn;
        __atomic_store_n(ans, (unsigned long long)p, __ATOMIC_RELEASE);
      }
      CK(hipStreamSynchronize(st));
      const double tt = now_us() - t0;
      unsigned herr = 0;
      CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
      std::sort(rt.begin(), rt.end());
      if (!rt.empty())
        printf("G %5d  host   %7.2f us per phase median (p10 %.2f p90 %.2f), whole %.1f us (err %u%s)\n", G,
               rt[rt.size() / 2], rt[rt.size() / 10], rt[rt.size() * 9 / 10], tt / K, herr, to ? ", TIMEOUT" : "");
      if (herr || to) return 1;
    }
  }
  printf("ok\n");
  return 0;
}
