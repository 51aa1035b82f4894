// Cycles per MFMA, back-to-back on one SIMD (one wave per workgroup, 4 independent accumulators):
// v_mfma_f32_16x16x16_f16 vs v_mfma_f32_16x16x32_f16.  hipcc --offload-arch=gfx950 -O3 mfma_rate.hip -o mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
using f4 = float __attribute__((ext_vector_type(4)));
using h4 = _Float16 __attribute__((ext_vector_type(4)));
using h8 = _Float16 __attribute__((ext_vector_type(8)));
constexpr int kIters = 4096;

template <int K>
__global__ void __launch_bounds__(64) rate(const float* in, float* out, long long* cyc) {
  f4 c0 = {in[0], 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  h8 a8, b8;
  h4 a4, b4;
  for (int j = 0; j < 8; ++j) { a8[j] = (_Float16)in[threadIdx.x + j]; b8[j] = (_Float16)in[j + 1]; }
  for (int j = 0; j < 4; ++j) { a4[j] = a8[j]; b4[j] = b8[j]; }
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kIters; ++i) {
    if constexpr (K == 32) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, b8, c3, 0, 0, 0);
    } else {
      c0 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, b4, c3, 0, 0, 0);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  const f4 s = c0 + c1 + c2 + c3;
  out[threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *in, *out;
  long long* cyc;
  (void)hipMalloc(&in, 256 * 4);
  (void)hipMalloc(&out, 256 * 4);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemset(in, 0, 256 * 4);
  long long h = 0;
  for (int rep = 0; rep < 2; ++rep) {
    rate<16><<<1, 64>>>(in, out, cyc);
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    if (rep) printf("16x16x16 f16: %.2f cycles per MFMA\n", double(h) / (4.0 * kIters));
    rate<32><<<1, 64>>>(in, out, cyc);
    (void)hipMemcpy(&h, cyc, 8, hipMemcpyDeviceToHost);
    if (rep) printf("16x16x32 f16: %.2f cycles per MFMA\n", double(h) / (4.0 * kIters));
  }
  return 0;
}
