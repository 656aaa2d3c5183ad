// LDS-DMA and barrier helpers shared by the big-tile conv kernels (conv_tile.hip,
// conv_wtile.hip).
#pragma once
#include "common.h"

__device__ __forceinline__ void tile_lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// LDS-DMA of one 16-B chunk per lane into lds_dst + 16 * lane (lds_dst wave-uniform);
// M0 saved/restored in the same statement (it is compiler-reserved)
__device__ __forceinline__ void ct_glds16(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

// the same with an SGPR base + per-lane 32-bit byte offset (no 64-bit address math)
__device__ __forceinline__ void ct_glds16_s(const void* sbase, unsigned voff, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_dst)
               : "memory");
}

// LDS-DMA of one dword per lane into lds_dst + 4 * lane (lds_dst wave-uniform)
__device__ __forceinline__ void ct_glds4(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}

__device__ __forceinline__ unsigned ct_lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) void*)p;
}


// The same two DMAs without a "memory" clobber, for DMAs issued between the MFMAs of a k-loop:
// with the clobber hipcc drains every LDS read in flight (lgkmcnt(0)) in front of each one.
// Only for DMAs into a buffer that no code reads before the next tile_lds_barrier() (an asm
// volatile with a memory clobber: volatile asm statements keep their order).
__device__ __forceinline__ void ct_glds16_nc(const void* gsrc, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst));
}
__device__ __forceinline__ void ct_glds16_s_nc(const void* sbase, unsigned voff, unsigned lds_dst) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds_dst));
}
