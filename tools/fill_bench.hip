// Per-CU fill rate from an L2-resident buffer on gfx950 (diagnostic, not part of
// the library): every workgroup streams the same 256 KB window (read by all
// workgroups of an XCD, so it sits in L2) in 32 KB blocks, ITER times, by
//   mode 0: LDS-DMA (buffer_load_dwordx4 ... lds, 1 KB per wave instruction)
//   mode 1: global_load_dwordx4 into VGPRs, then ds_write_b128
//   mode 2: global_load_dwordx4 into VGPRs only (summed so the loads stay live)
// with 8 waves per workgroup, one workgroup per CU (LDS sized to force it).
// Prints bytes per cycle per CU at the measured clock-free rate (GB/s / CU).
// Build: hipcc -O3 --offload-arch=gfx950 tools/fill_bench.hip -o /tmp/fill_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef __attribute__((address_space(3))) void* lds_t;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff) {
  unsigned keep;
  asm volatile(
      "s_nop 4\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds), "s"(r)
      : "memory");
}

template <int MODE>
__global__ void __launch_bounds__(512, 1) fill_kernel(const char* __restrict__ src, int iters, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char smem[4][32768];  // 128 KB: one workgroup per CU
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(src), (short)0, 262144, 0x00020000);
  uint4 accv = make_uint4(0, 0, 0, 0);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int blk = 0; blk < 8; ++blk) {  // 8 x 32 KB = the 256 KB window
      const int slot = blk & 3;
#pragma unroll
      for (int u = 0; u < 4; ++u) {  // 32 KB = 32 pieces of 1 KB, 4 per wave
        const int piece = u * 8 + w;
        unsigned off = (unsigned)(blk * 32768 + piece * 1024 + lane * 16);
        asm volatile("" : "+v"(off));  // opaque: no hoisting of the loads out of the iteration loop
        if (MODE == 0) {
          dma16(r, (unsigned)(unsigned long long)(lds_t)(&smem[slot][piece * 1024]), off);
        } else {
          typedef __attribute__((ext_vector_type(4))) unsigned u4;
          const u4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
          if (MODE == 1) {
            unsigned lo = (unsigned)(unsigned long long)(lds_t)(&smem[slot][piece * 1024 + lane * 16]);
            asm volatile("ds_write_b128 %0, %1" ::"v"(lo), "v"(v) : "memory");
          } else {
            accv.x ^= v.x; accv.y ^= v.y; accv.z ^= v.z; accv.w ^= v.w;
          }
        }
      }
      if (MODE == 0 && slot == 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // two blocks in flight
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (MODE == 2 && (accv.x | accv.y | accv.z | accv.w) == 0x12345678u) out[0] = 1;
  if (MODE != 2 && threadIdx.x == 0 && smem[1][5] == 123) out[1] = 1;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  char* src;
  unsigned* out;
  hipMalloc(&src, 262144);
  hipMalloc(&out, 64);
  hipMemset(src, 1, 262144);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(fill_kernel<0>, dim3(cus), dim3(512), 0, 0, src, iters, out);
      if (mode == 1) hipLaunchKernelGGL(fill_kernel<1>, dim3(cus), dim3(512), 0, 0, src, iters, out);
      if (mode == 2) hipLaunchKernelGGL(fill_kernel<2>, dim3(cus), dim3(512), 0, 0, src, iters, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double bytes_cu = 262144.0 * iters;
      if (rep == 1)
        printf("mode %d (%s): %.3f ms, %.1f GB/s per CU, %.1f B/cycle/CU at 2.4 GHz, %.2f TB/s over %d CUs\n", mode,
               mode == 0 ? "LDS-DMA" : mode == 1 ? "global_load + ds_write" : "global_load only", ms,
               bytes_cu / ms / 1e6, bytes_cu / (ms * 1e-3) / 2.4e9, bytes_cu * cus / ms / 1e9, cus);
    }
  }
  return 0;
}
