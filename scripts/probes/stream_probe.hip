// stream_probe.hip -- HBM ceiling of the stage kernels' access pattern on MI355X (diagnostic,
// not part of libpft).  R read arrays + W write arrays of the 400^3 slab layout (3 fields are
// 3 arrays each), dbl2 per lane:
//   flat  : grid-stride over the whole array
//   zmarch: the stage kernels' geometry (64x8 tiles of 2-cell pairs, kz-plane z-march, one
//           resident round of workgroups), no halo, no LDS
//   zhalo : zmarch + the halo ring loads (one 16-B pair per thread for t < NH) + LDS + barrier
//   hipcc --offload-arch=gfx950 -O3 stream_probe.hip -o stream_probe && ./stream_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
typedef double dbl2 __attribute__((ext_vector_type(2)));
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
constexpr int MAXA = 12;
struct Arrs { const double* in[MAXA]; double* out[MAXA]; };

template <int R, int W>
__global__ __launch_bounds__(256) void flat(Arrs a, long n2)
{
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n2; i += (long)gridDim.x * 256) {
    dbl2 s = {0, 0};
#pragma unroll
    for (int r = 0; r < R; ++r) s += reinterpret_cast<const dbl2*>(a.in[r])[i];
#pragma unroll
    for (int w = 0; w < W; ++w) reinterpret_cast<dbl2*>(a.out[w])[i] = s + (double)w;
  }
}

template <int R, int W, bool HALO>
__global__ __launch_bounds__(256) void zmarch(Arrs a, int n1, int n2, int n3, int kz, int ntile)
{
  __shared__ dbl2 lds[2][R][10 * 34];
  const int ntx = (n1 + 63) / 64;
  const int tile = blockIdx.x % ntile, chunk = blockIdx.x / ntile;
  const int x0 = (tile % ntx) * 64, y0 = (tile / ntx) * 8;
  const int tx = threadIdx.x % 32, ty = threadIdx.x / 32;
  const int i0 = x0 + 2 * tx, j = y0 + ty;
  const bool act = i0 < n1 && j < n2;
  const long plane = (long)n1 * n2;
  const long po = (long)(j < n2 ? j : n2 - 1) * n1 + (i0 < n1 ? i0 : n1 - 2);
  const int hj = y0 - 1 + (threadIdx.x / 34) % 10;
  const int hi = x0 - 2 + 2 * (threadIdx.x % 34);
  const bool hact = HALO && threadIdx.x < 68;   // two halo rows of 34 pairs (approximate ring)
  const long hp = (long)(hj < 0 ? 0 : hj >= n2 ? n2 - 1 : hj) * n1 + (hi < 0 ? 0 : hi >= n1 ? n1 - 2 : hi);
  const int kb = chunk * kz, ke = min(kb + kz, n3);
  int cur = 0;
  for (int k = kb; k < ke; ++k) {
    const long o = (long)(k + 1) * plane + po;
    dbl2 s = {0, 0};
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const dbl2 v = *reinterpret_cast<const dbl2*>(a.in[r] + o);
      s += v;
      if (HALO) lds[cur][r][threadIdx.x] = v;
    }
    if (hact) {
#pragma unroll
      for (int r = 0; r < R; ++r) lds[cur][r][256 + threadIdx.x % 68] = *reinterpret_cast<const dbl2*>(a.in[r] + (long)(k + 1) * plane + hp);
    }
    if (HALO) {
      __syncthreads();
#pragma unroll
      for (int r = 0; r < R; ++r) s += lds[cur][r][(threadIdx.x + 1) % 324];
      cur ^= 1;
    }
    if (act) {
#pragma unroll
      for (int w = 0; w < W; ++w) *reinterpret_cast<dbl2*>(a.out[w] + o) = s + (double)w;
    }
  }
}

int main(int argc, char** argv)
{
  const int n1 = argc > 2 ? atoi(argv[1]) : 200, n2 = argc > 2 ? atoi(argv[2]) : 200, n3 = 400;
  printf("n1=%d n2=%d n3=%d\n", n1, n2, n3);
  const long plane = (long)n1 * n2, fs = (n3 + 2) * plane;
  std::vector<double*> buf(2 * MAXA);
  for (auto& b : buf) { CHK(hipMalloc(&b, fs * 8)); CHK(hipMemset(b, 0, fs * 8)); }
  Arrs a;
  for (int r = 0; r < MAXA; ++r) { a.in[r] = buf[r]; a.out[r] = buf[MAXA + r]; }
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
  int ncu = 0; CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto run = [&](const char* name, int R, int W, auto launch) {
    for (int it = 0; it < 3; ++it) launch();
    hipEventRecord(e0);
    const int reps = 20;
    for (int it = 0; it < reps; ++it) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    ms /= reps;
    const double bytes = (double)(R + W) * n3 * plane * 8;
    printf("%-8s R=%d W=%d  %.4f ms  %.0f GB/s\n", name, R, W, ms, bytes / (ms * 1e-3) / 1e9);
  };
  const int ntile = ((n1 + 63) / 64) * ((n2 + 7) / 8);
#define CASE(R, W)                                                                                   \
  run("flat", R, W, [&] { flat<R, W><<<ncu * 8, 256>>>(a, n3 * plane / 2); });                      \
  for (int nch : {5, 8, 10}) {                                                                       \
    const int kz = (n3 + nch - 1) / nch;                                                             \
    char nm[32]; snprintf(nm, 32, "zm%d", nch);                                                      \
    run(nm, R, W, [&] { zmarch<R, W, false><<<ntile * nch, 256>>>(a, n1, n2, n3, kz, ntile); });     \
    snprintf(nm, 32, "zh%d", nch);                                                                   \
    run(nm, R, W, [&] { zmarch<R, W, true><<<ntile * nch, 256>>>(a, n1, n2, n3, kz, ntile); });      \
  }
  CASE(1, 1) CASE(3, 2) CASE(5, 2) CASE(7, 2) CASE(9, 3)
  return 0;
}
