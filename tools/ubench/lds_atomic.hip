// LDS float-atomic throughput micro-benchmark (gfx950): cycles per wave-instruction for
// ds_add_f32 vs ds_read+v_add+ds_write, by address pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
template <int MODE>
__global__ void __launch_bounds__(512) k(float* out, int iters, int stride) {
  __shared__ float s[32768];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) s[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int addr;
  if (MODE == 0 || MODE == 3) addr = (w * 64 + lane) & 32767;                  // distinct, conflict-free
  else if (MODE == 1) addr = (w * 64 + (lane & 7) * 4 + (lane >> 3) * 32 * stride) & 32767;  // 8 rows x 8 lanes strided 16B
  else addr = (lane & 31);                                                       // 2 lanes / address, all waves same
  float v = 1.0f + lane;
  long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 3) { float x = s[addr]; s[addr] = x + v; }
    else atomicAdd(&s[addr], v);
    addr = (addr + 64 * 8) & 32767;
  }
  __syncthreads();
  long long t1 = clock64();
  if (threadIdx.x == 0) out[blockIdx.x] = (float)(t1 - t0) / iters;
  if (threadIdx.x == 1) out[blockIdx.x + gridDim.x] = s[5];
}
int main() {
  float* d; hipMalloc(&d, 4096 * 8);
  float h[512];
  const int iters = 4096;
  for (int mode = 0; mode < 4; ++mode) {
    for (int waves : {1, 4, 8}) {
      hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
      hipEventRecord(a);
      if (mode == 0) k<0><<<256, 64 * waves>>>(d, iters, 1);
      if (mode == 1) k<1><<<256, 64 * waves>>>(d, iters, 1);
      if (mode == 2) k<2><<<256, 64 * waves>>>(d, iters, 1);
      if (mode == 3) k<3><<<256, 64 * waves>>>(d, iters, 1);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      hipMemcpy(h, d, 4 * 256, hipMemcpyDeviceToHost);
      const double instr = 256.0 * waves * iters;
      printf("mode %d (%s) waves/CU %d: %.3f ms, clock-cycles/iter per wave %.1f, wave-instr per CU-us %.1f\n", mode,
             mode == 0 ? "ds_add conflict-free" : mode == 1 ? "ds_add 8x8 strided" : mode == 2 ? "ds_add 2 lanes/addr" : "read+add+write",
             waves, ms, h[0], instr / 256.0 / (ms * 1e3));
    }
  }
  return 0;
}
