// Standalone experiment (not product code): ceilings for the C4 query on one MI355X.
// V0 stream read; V1 specialised LDS hash (probe + LDS atomics) = the product algorithm without
// interpretation; V2 dense LDS array by key (no probe); V3 V1 without MIN/MAX atomics.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1);} } while (0)
typedef long long i64x2 __attribute__((ext_vector_type(2)));
__device__ inline uint64_t sm64(uint64_t x){uint64_t z=x+0x9E3779B97F4A7C15ull;z=(z^(z>>30))*0xBF58476D1CE4E5B9ull;z=(z^(z>>27))*0x94D049BB133111EBull;return z^(z>>31);}
__global__ void gen(int64_t* k, int64_t* a, int64_t* b, int64_t n){for(int64_t i=blockIdx.x*(int64_t)blockDim.x+threadIdx.x;i<n;i+=(int64_t)gridDim.x*blockDim.x){k[i]=sm64(42^(0*0x9E3779B97F4A7C15ull)^i)%1024;a[i]=sm64(42^(1*0x9E3779B97F4A7C15ull)^i)%(1<<20);b[i]=sm64(42^(2*0x9E3779B97F4A7C15ull)^i)%(1<<20);}}
__global__ void __launch_bounds__(512) v0(const int64_t* k,const int64_t* a,const int64_t* b,int64_t n,unsigned long long* out){
  unsigned long long acc=0; int lane=threadIdx.x&63; int64_t w=(blockIdx.x*(int64_t)blockDim.x+threadIdx.x)>>6, nw=((int64_t)gridDim.x*blockDim.x)>>6;
  for(int64_t base=w*256;base<n;base+=nw*256){int64_t r0=base+2*lane;
    i64x2 k0=*(const i64x2*)(k+r0),k1=*(const i64x2*)(k+r0+128),a0=*(const i64x2*)(a+r0),a1=*(const i64x2*)(a+r0+128),b0=*(const i64x2*)(b+r0),b1=*(const i64x2*)(b+r0+128);
    acc^=k0.x^k0.y^k1.x^k1.y^a0.x^a0.y^a1.x^a1.y^b0.x^b0.y^b1.x^b1.y;}
  if(acc==12345) out[0]=acc;}
template<int MODE>
__global__ void __launch_bounds__(512) v1(const int64_t* __restrict__ k,const int64_t* __restrict__ a,const int64_t* __restrict__ b,int64_t n,int64_t thr,unsigned long long* out){
  constexpr int S=2048; __shared__ long long keys[S]; __shared__ unsigned cnt[S]; __shared__ long long sum[S],mn[S],mx[S];
  for(int i=threadIdx.x;i<S;i+=blockDim.x){keys[i]=INT64_MIN;cnt[i]=0;sum[i]=0;mn[i]=INT64_MAX;mx[i]=INT64_MIN;}
  __syncthreads();
  int lane=threadIdx.x&63; int64_t w=(blockIdx.x*(int64_t)blockDim.x+threadIdx.x)>>6, nw=((int64_t)gridDim.x*blockDim.x)>>6;
  for(int64_t base=w*256;base<n;base+=nw*256){int64_t r0=base+2*lane;
    i64x2 k0=*(const i64x2*)(k+r0),k1=*(const i64x2*)(k+r0+128),a0=*(const i64x2*)(a+r0),a1=*(const i64x2*)(a+r0+128),b0=*(const i64x2*)(b+r0),b1=*(const i64x2*)(b+r0+128);
    long long kk[4]={k0.x,k0.y,k1.x,k1.y}, aa[4]={a0.x,a0.y,a1.x,a1.y}, bb[4]={b0.x,b0.y,b1.x,b1.y};
    #pragma unroll
    for(int r=0;r<4;++r){ if(!(aa[r]>thr)) continue; int s;
      if(MODE==2){ s=(int)kk[r]; }
      else { uint32_t x=(uint32_t)kk[r]^(uint32_t)(kk[r]>>32)*0x85EBCA6Bu; uint32_t h=(x*0x9E3779B1u)>>21;
        while(true){ long long c=keys[h]; if(c==kk[r]) break; if(c==INT64_MIN){ long long o=(long long)atomicCAS((unsigned long long*)&keys[h],(unsigned long long)INT64_MIN,(unsigned long long)kk[r]); if(o==INT64_MIN||o==kk[r]) break;} h=(h+1)&(S-1);} s=h; }
      atomicAdd(&cnt[s],1u); atomicAdd((unsigned long long*)&sum[s],(unsigned long long)(aa[r]+bb[r]));
      if(MODE!=3){ atomicMin(&mn[s],aa[r]); atomicMax(&mx[s],bb[r]); } }
  }
  __syncthreads();
  for(int i=threadIdx.x;i<S;i+=blockDim.x) if(cnt[i]){ long long key= MODE==2? i: keys[i]; atomicAdd(&out[key&1023],(unsigned long long)sum[i]); atomicAdd(&out[1024+(key&1023)],cnt[i]); atomicMin((long long*)&out[2048+(key&1023)],mn[i]); atomicMax((long long*)&out[3072+(key&1023)],mx[i]);}
}
int main(){ int64_t n=1000000000; int64_t *k,*a,*b; unsigned long long* out;
  CHECK(hipMalloc(&k,n*8));CHECK(hipMalloc(&a,n*8));CHECK(hipMalloc(&b,n*8));CHECK(hipMalloc(&out,4096*8));
  hipLaunchKernelGGL(gen,dim3(16384),dim3(256),0,0,k,a,b,n); CHECK(hipDeviceSynchronize());
  hipEvent_t e0,e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[]={"v0 stream","v1 lds-hash","v2 dense-lds","v3 hash no minmax"};
  for(int rep=0;rep<2;++rep) for(int v=0;v<4;++v){ for(int grid : {512, 1024}) { hipMemset(out,0,4096*8); hipEventRecord(e0);
    if(v==0) hipLaunchKernelGGL(v0,dim3(grid),dim3(512),0,0,k,a,b,n,out);
    if(v==1) hipLaunchKernelGGL(v1<1>,dim3(grid),dim3(512),0,0,k,a,b,n,1<<19,out);
    if(v==2) hipLaunchKernelGGL(v1<2>,dim3(grid),dim3(512),0,0,k,a,b,n,1<<19,out);
    if(v==3) hipLaunchKernelGGL(v1<3>,dim3(grid),dim3(512),0,0,k,a,b,n,1<<19,out);
    hipEventRecord(e1); CHECK(hipEventSynchronize(e1)); float ms; hipEventElapsedTime(&ms,e0,e1);
    if(rep) printf("%-20s grid %5d  %.3f ms  %.0f GB/s\n",names[v],grid,ms,24e9/ms/1e6); } }
  return 0; }
