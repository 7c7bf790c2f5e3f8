// Per-CU store throughput: each 512-thread workgroup writes a 256 x 256 bf16 tile (128 KiB) per item with 16-B
// stores, in one of two shapes: (0) "frag": a wave instruction covers 16 rows x 64 B; (1) "rows": 2 rows x 512 B.
// Prints the cycles (s_memtime) from the first store to vmcnt(0), median over workgroups, for 1..256 workgroups.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>

__global__ __launch_bounds__(512, 1) void store_tile(uint4* out, int64_t ld16, int shape, int items,
                                                     unsigned long long* cyc) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  uint4 v = make_uint4(tid, blockIdx.x, 7, 9);
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < items; ++it) {
    const int64_t tile = (int64_t)blockIdx.x * items + it;
    const int64_t r0 = tile * 256;                       // tiles stacked along rows
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      int64_t row, c16;
      if (shape == 0) {            // wave w: rows (w>>2)*128 + s*16/2.. : 16 rows x 4 lanes x 16 B
        row = (wave >> 2) * 128 + (s >> 1) * 16 + (lane & 15);
        c16 = ((wave & 3) * 2 + (s & 1)) * 4 + (lane >> 4);   // 16-B column chunk 0..31
      } else {                      // 2 rows x 32 lanes x 16 B
        row = wave * 32 + s * 2 + (lane >> 5);
        c16 = lane & 31;
      }
      out[(r0 + row) * ld16 + c16] = v;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int maxwg = 256, items = 8;
  const int64_t ld16 = 32;                                 // 256 bf16 per row = 32 x 16 B
  uint4* out;
  unsigned long long* cyc;
  hipMalloc(&out, (size_t)maxwg * items * 256 * ld16 * 16);
  hipMalloc(&cyc, maxwg * 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int shape = 0; shape < 2; ++shape)
    for (int nwg : {1, 8, 32, 128, 256}) {
      for (int rep = 0; rep < 3; ++rep) {
        hipEventRecord(e0);
        store_tile<<<nwg, 512>>>(out, ld16, shape, items, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> h(nwg);
      hipMemcpy(h.data(), cyc, nwg * 8, hipMemcpyDeviceToHost);
      std::sort(h.begin(), h.end());
      const double bytes = (double)nwg * items * 128 * 1024;
      printf("shape=%s wgs=%3d  med %8llu cyc per %d tiles = %6.0f cyc/tile = %5.1f B/clk/CU   wall %.1f us  %.2f TB/s\n",
             shape ? "rows" : "frag", nwg, h[nwg / 2], items, (double)h[nwg / 2] / items,
             items * 131072.0 / h[nwg / 2], ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    }
  return 0;
}
