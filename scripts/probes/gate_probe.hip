// Host -> GPU hand-over latency on one MI355X (f4, the small-slab step): how long after the host
// writes a decision to pinned memory does a kernel on the stream start?  Round trip measured on the
// host: write the word, spin until the kernel's store into another pinned word is visible.
//   launch : the host launches the kernel on an idle stream after its write (today's path)
//   cpwait : the kernel is enqueued behind hipStreamWaitValue64 on the pinned word (command
//            processor polls host memory), the host only writes the word
//   poll   : the kernel is already running and one thread polls the pinned word
// hipcc --offload-arch=gfx950 -O2 -o gate_probe gate_probe.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

__global__ void mark(unsigned long long* done, unsigned long long v)
{
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// reads the decision word like a gated stage kernel would (every workgroup), then marks
__global__ void mark_read(const unsigned long long* gate, unsigned long long* done, unsigned long long v,
                          unsigned long long* sink)
{
  const unsigned long long g = __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0 && g != v) sink[blockIdx.x] = g;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// bounded poll (exit condition every wave reaches): gives up after ~2^26 reads
__global__ void poll_mark(const unsigned long long* gate, unsigned long long* done, unsigned long long v)
{
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (long it = 0; it < (1L << 26); ++it)
    if (__hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) >= v) break;
  __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// the gate: one workgroup polls the host's pinned decision word and copies it into device memory
// for the launches behind it on the stream
__global__ void gate_kernel(const unsigned long long* pin, unsigned long long* dev, unsigned long long v)
{
  if (threadIdx.x != 0) return;
  unsigned long long g = 0;
  for (long it = 0; it < (1L << 26); ++it)
    if ((g = __hip_atomic_load(pin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) >= v) break;
  __hip_atomic_store(dev, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every workgroup reads a device-memory word (as gated stage kernels would), then marks
__global__ void mark_dev(const unsigned long long* dev, unsigned long long* done, unsigned long long v,
                         unsigned long long* sink)
{
  const unsigned long long g = dev[0];
  if (threadIdx.x == 0 && g != v) sink[blockIdx.x] = g;
  __syncthreads();
  if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(done, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us()
{
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static const unsigned long long* gate_w(unsigned long long* p) { return p; }

static bool spin(volatile unsigned long long* w, unsigned long long v)
{
  const double t0 = now_us();
  while (__atomic_load_n(w, __ATOMIC_ACQUIRE) != v)
    if (now_us() - t0 > 2e6) return false;
  return true;
}

static void report(const char* name, std::vector<double>& v)
{
  std::sort(v.begin(), v.end());
  printf("%-24s median %7.2f us  p10 %7.2f  p90 %7.2f  (n=%zu)\n", name, v[v.size() / 2], v[v.size() / 10],
         v[v.size() * 9 / 10], v.size());
}

int main()
{
  unsigned long long *gate, *done, *sink;
  CK(hipHostMalloc((void**)&gate, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&done, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipMalloc((void**)&sink, 4096 * 8));
  *gate = 0;
  *done = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int N = 300;
  unsigned long long seq = 0;
  // warm up
  for (int i = 0; i < 50; ++i) {
    mark<<<1, 64, 0, st>>>(done, ++seq);
    CK(hipStreamSynchronize(st));
  }
  for (int grid : {1, 512}) {
    std::vector<double> la, cw, cr, po;
    for (int i = 0; i < N; ++i) {
      // launch
      ++seq;
      const double t0 = now_us();
      __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
      mark_read<<<grid, 256, 0, st>>>(gate, done, seq, sink);
      if (!spin(done, seq)) { fprintf(stderr, "launch: timeout\n"); return 1; }
      la.push_back(now_us() - t0);
      CK(hipStreamSynchronize(st));
      // cpwait (+ every workgroup reading the pinned word)
      ++seq;
      CK(hipStreamWaitValue64(st, gate, seq, hipStreamWaitValueGte, ~0ULL));
      mark_read<<<grid, 256, 0, st>>>(gate, done, seq, sink);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      const double t1 = now_us();
      __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
      if (!spin(done, seq)) { fprintf(stderr, "cpwait: timeout\n"); return 1; }
      cw.push_back(now_us() - t1);
      CK(hipStreamSynchronize(st));
      // cpwait, plain mark
      ++seq;
      CK(hipStreamWaitValue64(st, gate, seq, hipStreamWaitValueGte, ~0ULL));
      mark<<<grid, 256, 0, st>>>(done, seq);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      const double t2 = now_us();
      __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
      if (!spin(done, seq)) { fprintf(stderr, "cpwait2: timeout\n"); return 1; }
      cr.push_back(now_us() - t2);
      CK(hipStreamSynchronize(st));
      // poll (one workgroup)
      if (grid == 1) {
        ++seq;
        poll_mark<<<1, 64, 0, st>>>(gate, done, seq);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
        const double t3 = now_us();
        __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
        if (!spin(done, seq)) { fprintf(stderr, "poll: timeout\n"); return 1; }
        po.push_back(now_us() - t3);
        CK(hipStreamSynchronize(st));
      }
    }
    printf("grid %d workgroups\n", grid);
    report("launch+read", la);
    report("cpwait+read", cw);
    report("cpwait", cr);
    if (!po.empty()) report("poll", po);
  }
  // gate kernel + a 512-workgroup launch reading the copy in device memory
  {
    unsigned long long* dev;
    CK(hipMalloc((void**)&dev, 64));
    std::vector<double> g1, g2;
    for (int i = 0; i < N; ++i) {
      ++seq;
      gate_kernel<<<1, 64, 0, st>>>(gate_w(gate), dev, seq);
      mark_dev<<<512, 256, 0, st>>>(dev, done, seq, sink);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      const double t0 = now_us();
      __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
      if (!spin(done, seq)) { fprintf(stderr, "gate: timeout\n"); return 1; }
      g1.push_back(now_us() - t0);
      CK(hipStreamSynchronize(st));
      // cpwait, then the gate (which finds the word already written), then the launch
      ++seq;
      CK(hipStreamWaitValue64(st, gate, seq, hipStreamWaitValueGte, ~0ULL));
      gate_kernel<<<1, 64, 0, st>>>(gate_w(gate), dev, seq);
      mark_dev<<<512, 256, 0, st>>>(dev, done, seq, sink);
      std::this_thread::sleep_for(std::chrono::microseconds(200));
      const double t1 = now_us();
      __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
      if (!spin(done, seq)) { fprintf(stderr, "cpwait+gate: timeout\n"); return 1; }
      g2.push_back(now_us() - t1);
      CK(hipStreamSynchronize(st));
    }
    report("gate+512 reading dev", g1);
    report("cpwait+gate+512", g2);
  }
  // the host-side cost of the stream wait itself
  {
    std::vector<double> enq;
    for (int i = 0; i < N; ++i) {
      ++seq;
      const double t0 = now_us();
      CK(hipStreamWaitValue64(st, gate, seq, hipStreamWaitValueGte, ~0ULL));
      enq.push_back(now_us() - t0);
      __atomic_store_n(gate, seq, __ATOMIC_RELEASE);
      CK(hipStreamSynchronize(st));
    }
    report("enqueue wait (host)", enq);
  }
  CK(hipStreamSynchronize(st));
  printf("ok\n");
  return 0;
}
