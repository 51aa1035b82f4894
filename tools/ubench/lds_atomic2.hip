// LDS integer vs float atomic throughput (gfx950): cycles per wave-instruction per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void __launch_bounds__(512) k(float* out, int iters) {
  __shared__ unsigned long long s[16384];
  for (int i = threadIdx.x; i < 16384; i += blockDim.x) s[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int addr = (w * 64 + lane) & 16383;
  unsigned int* s32 = reinterpret_cast<unsigned int*>(s);
  float* sf = reinterpret_cast<float*>(s);
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) atomicAdd(&sf[addr], 1.5f);
    if (MODE == 1) atomicAdd(&s32[addr], 3u);
    if (MODE == 2) atomicAdd(&s[addr], 3ull);
    if (MODE == 3) { __hip_atomic_fetch_add(&s32[addr], 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
    addr = (addr + 64 * 8) & 16383;
  }
  __syncthreads();
  long long t1 = clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(t1 - t0) / iters;
  if (threadIdx.x == 1) out[blockIdx.x + gridDim.x] = (float)s[5];
}
int main() {
  float* d; (void)hipMalloc(&d, 4096 * 8);
  float h[512];
  const int iters = 4096;
  const char* names[] = {"ds_add_f32", "ds_add_u32", "ds_add_u64", "ds_add_u32 relaxed wg"};
  for (int mode = 0; mode < 4; ++mode) {
    for (int waves : {1, 8}) {
      hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
      (void)hipEventRecord(a);
      if (mode == 0) k<0><<<256, 64 * waves>>>(d, iters);
      if (mode == 1) k<1><<<256, 64 * waves>>>(d, iters);
      if (mode == 2) k<2><<<256, 64 * waves>>>(d, iters);
      if (mode == 3) k<3><<<256, 64 * waves>>>(d, iters);
      (void)hipEventRecord(b); (void)hipEventSynchronize(b);
      float ms; (void)hipEventElapsedTime(&ms, a, b);
      (void)hipMemcpy(h, d, 4 * 256, hipMemcpyDeviceToHost);
      const double instr = 256.0 * waves * iters;
      printf("%-22s waves/CU %d: %.3f ms, cycles/iter per wave %.1f, wave-instr per CU-us %.1f\n", names[mode], waves,
             ms, h[0], instr / 256.0 / (ms * 1e3));
    }
  }
  return 0;
}
