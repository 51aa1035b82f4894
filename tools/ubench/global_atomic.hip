// Global fp32 atomic-add throughput on gfx950 for the MSDA backward's window flush: 128-byte rows
// (32 floats) added with
//   mode 0: 8 lanes per row, float4 per lane, 4 atomic instructions (component k: 8 dwords 16 B apart)
//   mode 1: 8 lanes per row, lane j owns channels j, j+8, j+16, j+24 (each instruction: 8 contiguous dwords)
//   mode 2: 32 lanes per row, one dword per lane (each instruction: 2 rows x 128 contiguous bytes)
//   mode 3: plain float4 stores in the mode-0 layout (reference: no atomics)
// Rows are spread over a 2 GB buffer with the flush's access pattern (each row hit by a few workgroups).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ void __launch_bounds__(256) flush(float* __restrict__ g, long rows_total, int rows_per_block) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long base = static_cast<long>(blockIdx.x) * rows_per_block;
  if (MODE == 0 || MODE == 3) {
    const int j = lane & 7, grp = (threadIdx.x >> 3);
    for (int r = grp; r < rows_per_block; r += 32) {
      float* dst = g + ((base + r) % rows_total) * 32 + 4 * j;
      if (MODE == 0) {
        atomicAdd(dst + 0, 1.f); atomicAdd(dst + 1, 1.f); atomicAdd(dst + 2, 1.f); atomicAdd(dst + 3, 1.f);
      } else {
        float4 v = *reinterpret_cast<float4*>(dst);
        v.x += 1.f;
        *reinterpret_cast<float4*>(dst) = v;
      }
    }
  } else if (MODE == 1) {
    const int j = lane & 7, grp = (threadIdx.x >> 3);
    for (int r = grp; r < rows_per_block; r += 32) {
      float* dst = g + ((base + r) % rows_total) * 32 + j;
      atomicAdd(dst + 0, 1.f); atomicAdd(dst + 8, 1.f); atomicAdd(dst + 16, 1.f); atomicAdd(dst + 24, 1.f);
    }
  } else {
    const int c = lane & 31, half = lane >> 5;
    for (int r = wave * 2 + half; r < rows_per_block; r += 8) {
      float* dst = g + ((base + r) % rows_total) * 32 + c;
      atomicAdd(dst, 1.f);
    }
  }
}

template <int MODE>
float run(float* g, long rows_total, int blocks, int rpb) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  flush<MODE><<<blocks, 256>>>(g, rows_total, rpb);
  hipEventRecord(a);
  for (int i = 0; i < 5; ++i) flush<MODE><<<blocks, 256>>>(g, rows_total, rpb);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const long rows_total = 16L * 21504 * 8;  // grad_value rows of config 2 (n, s, m)
  float* g;
  hipMalloc(&g, rows_total * 128);
  hipMemset(g, 0, rows_total * 128);
  const int rpb = 2048, blocks = 8192;       // ~ the flush: 8192 workgroups x ~2k window rows
  const double bytes = static_cast<double>(blocks) * rpb * 128;
  float t0 = run<0>(g, rows_total, blocks, rpb), t1 = run<1>(g, rows_total, blocks, rpb);
  float t2 = run<2>(g, rows_total, blocks, rpb), t3 = run<3>(g, rows_total, blocks, rpb);
  printf("{\"bytes_GB\": %.3f, \"float4x4_atomics_ms\": %.3f, \"strided8_atomics_ms\": %.3f, "
         "\"contig32_atomics_ms\": %.3f, \"plain_rmw_ms\": %.3f}\n", bytes / 1e9, t0, t1, t2, t3);
  hipFree(g);
  return 0;
}
