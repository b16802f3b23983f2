// Hardware probe: HBM copy bandwidth (double2 streaming), FP64 FMA rate, DPP wave shift check.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

__global__ void copy2(const double2* __restrict__ a, double2* __restrict__ b, size_t n){
  size_t i = blockIdx.x*(size_t)blockDim.x + threadIdx.x; size_t s = (size_t)gridDim.x*blockDim.x;
  for(; i<n; i+=s) b[i]=a[i];
}
__global__ void fma64(double* out, int iters){
  double a=threadIdx.x*1e-3, b=1.0000001, c=1e-9, d=0.5, e=0.25, f=0.125, g=0.1, h=0.2;
  for(int k=0;k<iters;k++){ a=fma(a,b,c); d=fma(d,b,c); e=fma(e,b,c); f=fma(f,b,c); g=fma(g,b,c); h=fma(h,b,c);}
  out[blockIdx.x*blockDim.x+threadIdx.x]=a+d+e+f+g+h;
}
__global__ void dpp_test(double* out){
  int l = threadIdx.x;
  double v = (double)l + 0.5;
  // wave_shr:1 on both 32-bit halves (dpp_ctrl 0x138), bound_ctrl to get 0 for lane0
  int lo = __double2loint(v), hi = __double2hiint(v);
  int lo2 = __builtin_amdgcn_update_dpp(0, lo, 0x138, 0xF, 0xF, false);
  int hi2 = __builtin_amdgcn_update_dpp(0, hi, 0x138, 0xF, 0xF, false);
  out[l] = __hiloint2double(hi2, lo2);
  int lo3 = __builtin_amdgcn_update_dpp(0, lo, 0x130, 0xF, 0xF, false); // wave_shl:1
  int hi3 = __builtin_amdgcn_update_dpp(0, hi, 0x130, 0xF, 0xF, false);
  out[64+l] = __hiloint2double(hi3, lo3);
}
int main(){
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p,0));
  printf("device %s gcn %s CUs %d clock %d kHz mem %zu GB l2 %d\n", p.name, p.gcnArchName, p.multiProcessorCount, p.clockRate, p.totalGlobalMem>>30, p.l2CacheSize);
  size_t n = (size_t)1<<27; // 2^27 double2 = 2 GiB
  double2 *a,*b; CK(hipMalloc(&a,n*16)); CK(hipMalloc(&b,n*16));
  CK(hipMemset(a,0,n*16)); CK(hipMemset(b,0,n*16));
  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for(int grid : {2048, 8192, 65536}){
    copy2<<<grid,256>>>(a,b,n); CK(hipDeviceSynchronize());
    hipEventRecord(e0); for(int r=0;r<10;r++) copy2<<<grid,256>>>(a,b,n); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms,e0,e1); printf("copy2 grid %d: %.1f GB/s\n", grid, 10.0*2*n*16/ (ms*1e-3)/1e9);
  }
  double* o; CK(hipMalloc(&o, 1<<24));
  int blocks=256*8, iters=4096;
  fma64<<<blocks,256>>>(o,iters); CK(hipDeviceSynchronize());
  hipEventRecord(e0); fma64<<<blocks,256>>>(o,iters); hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms,e0,e1); printf("fp64 fma: %.1f TFLOP/s\n", 2.0*6*iters*(double)blocks*256/(ms*1e-3)/1e12);
  dpp_test<<<1,64>>>(o); CK(hipDeviceSynchronize());
  std::vector<double> h(128); CK(hipMemcpy(h.data(),o,128*8,hipMemcpyDeviceToHost));
  printf("wave_shr: "); for(int i=0;i<6;i++) printf("%g ",h[i]); printf("... %g\n", h[63]);
  printf("wave_shl: "); for(int i=0;i<4;i++) printf("%g ",h[64+i]); printf("... %g %g\n", h[126], h[127]);
  // fp64 atomic add rate check
  return 0;
}
