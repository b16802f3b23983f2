// Launch-cost audit (VERDICT r5 "next" item 1a): what one dependent launch
// costs on one stream, unprofiled, timed with HIP events over chains of K
// back-to-back launches (per launch = elapsed / K).  Run it plain and under
// `rocprofv3 --kernel-trace --stats` to compare the profiler's per-kernel time
// with the unprofiled per-launch wall time.
//   hipcc -O3 --offload-arch=gfx950 launch_probe.hip -o launch_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

struct Arg160 { double v[20]; };                  // PcgState-sized (k_set_state)
template <int B> struct ArgB { char b[B]; };      // kernel-argument size sweep

__global__ void k_empty() {}
__global__ void k_state(Arg160 a, Arg160* dst) {  // one thread stores a 160-B struct
  if (threadIdx.x == 0 && blockIdx.x == 0) *dst = a;
}
__global__ void k_rw(double* p) {  // one thread: dependent load + store
  if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = p[0] + 1.0;
}
template <int B>
__global__ void k_argsz(ArgB<B> a, char* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = a.b[B - 1];
}
__global__ void k_lds(double* p) {  // one thread, 52 KB static LDS (the march's footprint)
  __shared__ double s[6600];
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    s[threadIdx.x] = p[0];
    p[1] = s[0];
  }
}
__global__ void k_stream(const double* __restrict__ a, double* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) b[i] = a[i] * 1.0000001;
}
__global__ void k_touch(double* __restrict__ a, size_t n) {  // small grid-stride pass (~125 K nodes)
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, s = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += s) a[i] += 1.0;
}

static hipEvent_t e0, e1, e2;
template <class F>
static float chain(F f, int K, hipStream_t st) {
  f();  // warm
  hipStreamSynchronize(st);
  hipEventRecord(e0, st);
  for (int k = 0; k < K; ++k) f();
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / K;  // us per launch
}

int main(int argc, char** argv) {
  const int K = 2000;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  Arg160 a{};
  Arg160* dst;
  double* p;
  char* out;
  CK(hipMalloc(&dst, sizeof(Arg160)));
  CK(hipMalloc(&p, 1 << 20));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(p, 0, 1 << 20));
  const size_t nbig = (size_t)1 << 24;  // 128 MB per array
  double *A, *B, *S;
  CK(hipMalloc(&A, nbig * 8));
  CK(hipMalloc(&B, nbig * 8));
  CK(hipMalloc(&S, 1 << 24));
  CK(hipMemset(A, 0, nbig * 8));
  CK(hipMemset(S, 0, 1 << 24));
  double* hpin;
  CK(hipHostMalloc(&hpin, 4096));
  CK(hipDeviceSynchronize());

  printf("# per-launch wall time, chains of %d launches on one stream, HIP events (us)\n", K);
  printf("empty 1x64              %.2f\n", chain([&] { k_empty<<<1, 64, 0, st>>>(); }, K, st));
  printf("empty 256x256           %.2f\n", chain([&] { k_empty<<<256, 256, 0, st>>>(); }, K, st));
  printf("empty 1024x256          %.2f\n", chain([&] { k_empty<<<1024, 256, 0, st>>>(); }, K, st));
  printf("set_state 1x64 (160 B)  %.2f\n", chain([&] { k_state<<<1, 64, 0, st>>>(a, dst); }, K, st));
  printf("load+store 1x64         %.2f\n", chain([&] { k_rw<<<1, 64, 0, st>>>(p); }, K, st));
  printf("52 KB LDS 1x512         %.2f\n", chain([&] { k_lds<<<1, 512, 0, st>>>(p); }, K, st));
  printf("argsz 64 B              %.2f\n", chain([&] { k_argsz<64><<<1, 64, 0, st>>>(ArgB<64>{}, out); }, K, st));
  printf("argsz 512 B             %.2f\n", chain([&] { k_argsz<512><<<1, 64, 0, st>>>(ArgB<512>{}, out); }, K, st));
  printf("argsz 1536 B            %.2f\n", chain([&] { k_argsz<1536><<<1, 64, 0, st>>>(ArgB<1536>{}, out); }, K, st));
  printf("argsz 3072 B            %.2f\n", chain([&] { k_argsz<3072><<<1, 64, 0, st>>>(ArgB<3072>{}, out); }, K, st));
  // a 125 K-node pass (1 MB r+w): a share/8 coarse level's streaming launch
  printf("touch 125K 512x256      %.2f\n", chain([&] { k_touch<<<512, 256, 0, st>>>(S, 125000); }, K, st));
  printf("touch 1M 2048x256       %.2f\n", chain([&] { k_touch<<<2048, 256, 0, st>>>(S, 1000000); }, K, st));
  // polls: an event record / a 160-B D2H copy between launches
  printf("set_state + event       %.2f\n", chain([&] {
    k_state<<<1, 64, 0, st>>>(a, dst);
    hipEventRecord(e2, st);
  }, K, st));
  printf("set_state + D2H 160 B   %.2f\n", chain([&] {
    k_state<<<1, 64, 0, st>>>(a, dst);
    hipMemcpyAsync(hpin, dst, sizeof(Arg160), hipMemcpyDeviceToHost, st);
  }, K, st));
  printf("memset 8 B              %.2f\n", chain([&] { hipMemsetAsync(out, 0, 8, st); }, K, st));

  // dirty bytes: a streaming kernel writing W bytes, then ONE trivial launch; the
  // trivial launch's wall time = (pair time) - (streaming kernel alone)
  printf("# trivial launch behind a kernel that leaves W bytes written (us, pair - alone)\n");
  for (size_t mb : {1, 4, 16, 64, 128}) {
    const size_t n = mb * (1 << 20) / 8;
    const int grid = 2048;
    float alone = chain([&] { k_stream<<<grid, 256, 0, st>>>(A, B, n); }, 200, st);
    float pair = chain([&] {
      k_stream<<<grid, 256, 0, st>>>(A, B, n);
      k_rw<<<1, 64, 0, st>>>(p);
    }, 200, st);
    printf("W = %4zu MB: stream %.2f, +trivial %.2f\n", mb, alone, pair - alone);
  }
  CK(hipDeviceSynchronize());
  return 0;
}
